#!/bin/bash
# Paired-row SELL-128 image: the whole GPU suite, then the metric CG SpMV
# legs (DIA, pair, SELL-64) timed with HIP events. Stop at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_full.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest_full.log | head -30; tail -3 $OUT/pytest_full.log; exit 1; }
tail -2 $OUT/pytest_full.log
timeout -k 10 300 python tools/spmv_legs.py 200 > $OUT/spmv_legs.log 2>&1 || { tail -5 $OUT/spmv_legs.log; exit 1; }
cat $OUT/spmv_legs.log
