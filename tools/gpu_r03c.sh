#!/bin/bash
# Round-3: DIA tests (fused-p block CG), full-size parity, the cfg4 headline,
# then the PMC traffic passes. Each GPU step has its own limit; stop at the
# first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dia.py tests/test_gpu_fullsize_golden.py > $OUT/pytest_r03c.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest_r03c.log | head -30; tail -5 $OUT/pytest_r03c.log; exit 1; }
grep -E "passed|failed|history max rel|cycles" $OUT/pytest_r03c.log | tail -12
timeout -k 10 300 python bench.py --workload cfg4 --quick > $OUT/bench_cfg4.log 2>&1 || { tail -20 $OUT/bench_cfg4.log; exit 1; }
tail -c 1500 $OUT/bench_cfg4.log
[ -n "$PMC" ] && bash tools/pmc_traffic.sh
exit 0
