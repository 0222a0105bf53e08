#!/bin/bash
# The cfg4 headline line (--workload cfg4) plain and through the driver's
# torchrun launch path at one rank (RCCL allreduce per iteration).
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/cfg4line; mkdir -p $OUT
timeout -k 10 300 python bench.py --workload cfg4 --quick > $OUT/plain.log 2>&1 || { tail -20 $OUT/plain.log; exit 1; }
tail -1 $OUT/plain.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --workload cfg4 --quick > $OUT/torchrun.log 2>&1 || { tail -20 $OUT/torchrun.log; exit 1; }
tail -1 $OUT/torchrun.log
