#!/bin/bash
# Software-pipelined SELL-64 SpMV (k = 1): the SpMV / DIA-vs-SELL solver
# tests, then the general-CSR leg of tools/spmv_legs.py on the metric matrix
# with the pipelined kernel (default) and the plain one (KRY_SELL_PIPE=0).
# (Both the variant and its switch were removed after the measurement in
# profiles/r03_sell_pipe.txt.)
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/sellpipe; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_dia.py tests/test_gpu_solvers.py > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 1 0 1; do
  KRY_SELL_PIPE=$v timeout -k 10 300 python3 tools/spmv_legs.py 200 > $OUT/v$v.log 2>&1 || { tail -5 $OUT/v$v.log; exit 1; }
  echo "pipe=$v $(grep general $OUT/v$v.log)"
done
