#!/bin/bash
# Whole GPU suite (as the driver runs it at round end), smoke(), then the
# default bench line. Each step with its own limit; stop at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_full.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest_full.log | head -20; tail -3 $OUT/pytest_full.log; exit 1; }
tail -2 $OUT/pytest_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_full.log 2>&1 || { tail -20 $OUT/bench_full.log; exit 1; }
tail -c 400 $OUT/bench_full.log
