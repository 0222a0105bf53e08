#!/bin/bash
# Round-3 measurement pass: parity tests touched by the self-noise bound, the
# default bench line (CPU baseline included), its rocprofv3 kernel-trace
# summary, and the MFMA counter pass. Each GPU step has its own limit; stop
# at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT/prof_r03
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_solvers.py tests/test_gpu_fullsize_golden.py > $OUT/pytest_r03d.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest_r03d.log | head -30; exit 1; }
grep -E "passed|failed|history max rel|cycles" $OUT/pytest_r03d.log | tail -12
timeout -k 10 600 python bench.py > $OUT/bench_r03d.log 2>&1 || { tail -20 $OUT/bench_r03d.log; exit 1; }
tail -c 600 $OUT/bench_r03d.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r03 -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof_r03/stdout.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash $GRAFT_REPO_ROOT/tools/pmc_mfma.sh
