#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the script stops at the first failure.
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT/prof
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -q -m gpu ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
echo "pytest exit $?" >> $OUT/pytest_gpu.log
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log | tail -20; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -c 3000 $OUT/bench.log
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py ${BENCH_ARGS} --no-cpu > $OUT/prof/bench_stdout.log 2>&1
  rc=$?; echo "rocprof exit $rc"; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$PMC" ]; then
  $GRAFT_REPO_ROOT/tools/pmc_traffic.sh || exit 1
fi
if [ -n "$TORCHRUN" ]; then
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --quick --steps 64 --warmup 8 > $OUT/bench_torchrun.log 2>&1 || { echo "torchrun bench failed"; tail -20 $OUT/bench_torchrun.log; exit 1; }
  tail -1 $OUT/bench_torchrun.log
fi
