#!/bin/bash
# Session start on a fresh box: the whole GPU suite, smoke(), then the
# shifted-window block DIA SpMV probe (tools/dia_blk_bench, DIA_BLK_SHIFT).
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_full.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest_full.log | head -20; tail -3 $OUT/pytest_full.log; exit 1; }
tail -2 $OUT/pytest_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
DIA_BLK_SHIFT=1 timeout -k 10 180 ./tools/dia_blk_bench 3163 20 > $OUT/dia_shift.log 2>&1 || { tail -5 $OUT/dia_shift.log; exit 1; }
cat $OUT/dia_shift.log
