#!/bin/bash
# Deferred yk updates on the block CG path: the block-CG parity tests, then
# cfg4 A/B (KRY_CG_YDEFER = 0 / 3 / 7), alternating. Stop at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/ydefer; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dia.py tests/test_gpu_fullsize_golden.py tests/test_gpu_solvers.py tests/test_gpu_distributed.py > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for d in 0 3 7; do
    KRY_CG_YDEFER=$d timeout -k 10 200 python bench.py --workload cfg4 --quick > $OUT/d${d}_$i.log 2>&1 || { tail -5 $OUT/d${d}_$i.log; exit 1; }
    python3 -c "import json; b=json.loads(open('$OUT/d${d}_$i.log').read().strip().splitlines()[-1]); print('ydefer=$d run $i', round(b['value']/8,1), 'it/s', round(b['ms_per_step'],4), 'ms/it, spmv', round(b['roofline']['spmv_ms'],4))"
  done
done
