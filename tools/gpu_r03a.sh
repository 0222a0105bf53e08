#!/bin/bash
# Round-3 check: the changed GPU tests, the new bench line, and the
# rocprofv3 --configs run that used to crash at exit. Each GPU step has its
# own time limit; stop at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT/prof_cfg
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu ${TESTS} > $OUT/pytest_r03a.log 2>&1 || { tail -40 $OUT/pytest_r03a.log; exit 1; }
grep -E "passed|failed|restart|history max rel" $OUT/pytest_r03a.log | tail -8
timeout -k 10 400 python bench.py --no-cpu > $OUT/bench_r03a.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_r03a.log; exit 1; }
tail -c 3000 $OUT/bench_r03a.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --configs --no-cpu --quick > $OUT/prof_cfg/stdout.log 2>&1
rc=$?; echo "rocprof --configs exit $rc"; exit $rc
