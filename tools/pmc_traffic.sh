#!/bin/bash
# HBM traffic of the metric CG's SpMV kernels (bench.py roofline.traffic and
# spmv_general.traffic), collected as MI355X_MICROARCH.md "HBM" prescribes:
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes (they do not
# fit one TCC pass), unit KiB, and the read side calibrated on a kernel with
# the same access widths and a known byte count: tools/dia_bench's "values
# only" probe streams exactly the diagonal-offset image's value array (16 B
# per lane). The profiled program is tools/spmv_legs.py (both kernels, 64
# CG iterations each). One pass per rocprofv3 run, each under its own time
# limit; stop at the first failure. Summary -> gpurun_out/pmc_traffic/summary.json.
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BIN=$GRAFT_REPO_ROOT/tools/dia_bench
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $OUT/micro_$c -o run -- $BIN 216 3 > $OUT/micro_$c.log 2>&1
  rc=$?; echo "micro $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/bench_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/spmv_legs.py 64 > $OUT/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summarize.py $OUT > $OUT/summary.json && cat $OUT/summary.json
