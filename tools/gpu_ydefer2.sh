#!/bin/bash
# Deferred yk updates (block path and the one-launch k = 1 update): the whole
# GPU suite, then metric and cfg4 A/B (KRY_CG_YDEFER = 0 / 7), alternating.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/ydefer2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for d in 0 7; do
    KRY_CG_YDEFER=$d timeout -k 10 200 python bench.py --quick > $OUT/m${d}_$i.log 2>&1 || { tail -5 $OUT/m${d}_$i.log; exit 1; }
    python3 -c "import json; b=json.loads(open('$OUT/m${d}_$i.log').read().strip().splitlines()[-1]); print('metric ydefer=$d run $i', round(b['value'],1), 'it/s', round(b['ms_per_step'],4), 'ms/it, spmv', round(b['roofline']['spmv_ms'],4))"
    KRY_CG_YDEFER=$d timeout -k 10 200 python bench.py --workload cfg4 --quick > $OUT/c${d}_$i.log 2>&1 || { tail -5 $OUT/c${d}_$i.log; exit 1; }
    python3 -c "import json; b=json.loads(open('$OUT/c${d}_$i.log').read().strip().splitlines()[-1]); print('cfg4 ydefer=$d run $i', round(b['value']/8,1), 'it/s', round(b['ms_per_step'],4), 'ms/it')"
  done
done
