#!/bin/bash
# HBM traffic per launch of cfg4's block-CG kernels (block DIA SpMV, r pass,
# deferred p pass, flush), as MI355X_MICROARCH.md "HBM" prescribes: separate
# FETCH_SIZE and WRITE_SIZE rocprofv3 --pmc passes, KiB, the read side
# calibrated on tools/dia_bench's "values only" stream of known size. Each
# pass its own run under its own time limit; stop at the first failure.
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_cfg4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BIN=$GRAFT_REPO_ROOT/tools/dia_bench
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $OUT/micro_$c -o run -- $BIN 216 3 > $OUT/micro_$c.log 2>&1
  rc=$?; echo "micro $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/cfg4_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/cfg_time.py cfg4 28 > $OUT/cfg4_$c.log 2>&1
  rc=$?; echo "cfg4 $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 $GRAFT_REPO_ROOT/tools/pmc_cfg4_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
