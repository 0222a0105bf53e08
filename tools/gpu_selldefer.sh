#!/bin/bash
# SELL-64 SpMV (the general-CSR path, KRY_SPMV_DIA=0 leg of tools/spmv_legs.py
# on the metric matrix): epilogue deferred behind the next slice's gathers
# (default) against at the end of each slice (KRY_SELL_DEFER=0), after the
# SpMV bitwise tests. (KRY_SELL_DEFER was a temporary A/B switch, removed after
# the measurement in profiles/r03_sell_defer.txt.)
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/selldefer; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_solvers.py tests/test_gpu_precond.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 1 0 1; do
  KRY_SELL_DEFER=$v timeout -k 10 300 python3 tools/spmv_legs.py 200 > $OUT/v$v.log 2>&1 || { tail -5 $OUT/v$v.log; exit 1; }
  echo "defer=$v $(grep general $OUT/v$v.log)"
done
