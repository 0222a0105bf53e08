#!/bin/bash
# Round-3 second-session measurement pass (after the paired-row SELL-128
# image): the default bench line (CPU baseline included), its rocprofv3
# kernel-trace summary, PMC traffic of the metric SpMV kernels (DIA, pair,
# SELL-64), and the driver's torchrun launch path at one rank. Each GPU step
# has its own limit; stop at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03f; mkdir -p $OUT/prof
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -c 300 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof/stdout.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
$GRAFT_REPO_ROOT/tools/pmc_traffic.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
cp $GRAFT_REPO_ROOT/gpurun_out/pmc_traffic/summary.json $OUT/pmc_summary.json
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --quick --steps 64 --warmup 8 > $OUT/bench_torchrun.log 2>&1 || { echo "torchrun bench failed"; tail -20 $OUT/bench_torchrun.log; exit 1; }
tail -1 $OUT/bench_torchrun.log
