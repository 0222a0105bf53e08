set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 120 ./tools/dia_bench 216 20 > $OUT/dia_bench.log 2>&1 || { echo dia_bench failed; cat $OUT/dia_bench.log; exit 1; }
cat $OUT/dia_bench.log
PROFILE=1 PMC=1 BENCH_ARGS="--configs" PYTEST_ARGS="-x --timeout 300 --timeout-method thread" bash tools/gpu_check.sh
