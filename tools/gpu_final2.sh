#!/bin/bash
# Final tree check: the whole GPU suite (incl. the deferred-y fault test),
# smoke(), then the default bench line. Stop at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/final2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 -c "import json; b=json.loads([l for l in open('$OUT/bench.log') if l.startswith('{')][-1]); print('metric', round(b['value'],1), 'spmv', round(b['spmv_ms'],4), 'frac', round(b['roofline']['frac'],3), 'general', round(b['spmv_general']['frac'],3), 'cfg4', round(b['cfg4_sharded']['it_per_s'],1), 'gmres', round(b['gmres']['it_per_s'],1), round(b['gmres_metric']['it_per_s'],1))"
