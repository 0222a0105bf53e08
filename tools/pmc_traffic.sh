#!/bin/bash
# HBM traffic of the dominant kernel (bench.py roofline.traffic), collected as
# MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes (they do not fit one TCC pass), unit KiB, and the
# read side calibrated on a kernel with the same access widths and a known
# byte count: tools/dia_bench's "values only" probe streams exactly the
# diagonal-offset image's value array (8 B/lane, 512 B per slot column, the
# same width as the SpMV's value loads and its contiguous x runs).
# One pass per rocprofv3 run, each under its own time limit; stop at the first
# failure. Summary -> gpurun_out/pmc_traffic/summary.json (tools/pmc_summarize.py).
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BIN=$GRAFT_REPO_ROOT/tools/dia_bench
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $OUT/micro_$c -o run -- $BIN 216 3 > $OUT/micro_$c.log 2>&1
  rc=$?; echo "micro $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $OUT/bench_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --quick --steps 64 --warmup 0 > $OUT/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summarize.py $OUT > $OUT/summary.json && cat $OUT/summary.json
