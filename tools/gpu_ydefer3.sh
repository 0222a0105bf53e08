#!/bin/bash
# Default deferral decision (vectors > 128 MB only): the CG/DIA parity tests,
# then metric and cfg4 bench lines with the defaults.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/ydefer3; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dia.py tests/test_gpu_fullsize_golden.py tests/test_gpu_faults.py tests/test_gpu_distributed.py > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --quick > $OUT/m_$i.log 2>&1 || { tail -5 $OUT/m_$i.log; exit 1; }
  python3 -c "import json; b=json.loads(open('$OUT/m_$i.log').read().strip().splitlines()[-1]); print('metric run $i', round(b['value'],1), 'it/s', round(b['ms_per_step'],4), 'ms/it, spmv', round(b['roofline']['spmv_ms'],4))"
  timeout -k 10 200 python bench.py --workload cfg4 --quick > $OUT/c_$i.log 2>&1 || { tail -5 $OUT/c_$i.log; exit 1; }
  python3 -c "import json; b=json.loads(open('$OUT/c_$i.log').read().strip().splitlines()[-1]); print('cfg4 run $i', round(b['value']/8,1), 'it/s', round(b['ms_per_step'],4), 'ms/it')"
done
