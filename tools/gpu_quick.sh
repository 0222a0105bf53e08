#!/bin/bash
# Focused GPU pass: the named test files (-s, so printed headroom is logged),
# then tools/dia_bench. Each step under its own time limit; stop at the first
# failure.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu ${TESTS} > $OUT/pytest_quick.log 2>&1 || { tail -40 $OUT/pytest_quick.log; exit 1; }
grep -E "passed|failed|history max rel|cfg5_minres:" $OUT/pytest_quick.log | tail -20
if [ -n "$DIA" ]; then
  timeout -k 10 120 ./tools/dia_bench 216 20 > $OUT/dia_bench.log 2>&1 || { echo dia_bench failed; cat $OUT/dia_bench.log; exit 1; }
  cat $OUT/dia_bench.log
fi
