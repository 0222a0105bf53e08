#!/bin/bash
# Upload path after the parallel-filled staging buffers: image-building and
# SpMV parity tests, then kry_csr_create's phases (tools/upload_time.py).
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/upload; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_dia.py tests/test_gpu_solvers.py tests/test_gpu_precond.py > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 500 python tools/upload_time.py > $OUT/upload.log 2>&1 || { tail -20 $OUT/upload.log; exit 1; }
grep -E 'call|kry_csr_create' $OUT/upload.log
