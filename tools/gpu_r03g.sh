#!/bin/bash
# Round-3 end-of-session measurement pass: the whole GPU suite and smoke(),
# the default bench line (CPU baseline included), --configs (cfg2, cfg4,
# cfg5), the rocprofv3 kernel-trace summary of the bench, and the torchrun
# 1-rank launch path. Each GPU step has its own limit; stop at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03g; mkdir -p $OUT/prof
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; tail -3 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -c 200 $OUT/bench.log; echo
timeout -k 10 600 python bench.py --configs --no-cpu > $OUT/bench_configs.log 2>&1 || { tail -20 $OUT/bench_configs.log; exit 1; }
echo configs ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof/stdout.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --quick --steps 64 --warmup 8 > $OUT/bench_torchrun.log 2>&1 || { echo "torchrun bench failed"; tail -20 $OUT/bench_torchrun.log; exit 1; }
echo torchrun ok
