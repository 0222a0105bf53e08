#!/bin/bash
# End-of-round measurement pass: bench line, --configs legs, rocprofv3
# kernel-trace summary of the bench, PMC traffic of the CG SpMV, and the
# driver's torchrun launch path at one rank. Each GPU step has its own time
# limit; the script stops at the first failure.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT/prof
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 400 python bench.py --configs --no-cpu > $OUT/bench_configs.log 2>&1 || { echo "bench --configs failed"; tail -20 $OUT/bench_configs.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof/bench_stdout.log 2>&1
rc=$?; echo "rocprof exit $rc"; [ $rc -ne 0 ] && exit $rc
$GRAFT_REPO_ROOT/tools/pmc_traffic.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --quick --steps 64 --warmup 8 > $OUT/bench_torchrun.log 2>&1 || { echo "torchrun bench failed"; tail -20 $OUT/bench_torchrun.log; exit 1; }
tail -1 $OUT/bench_torchrun.log
