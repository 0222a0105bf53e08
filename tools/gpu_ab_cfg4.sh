#!/bin/bash
# A/B on one box: cfg4 block CG with and without a two-stage partial
# reduction (KRY_YP_STAGE), alternating, then the kernel trace once.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab_cfg4; mkdir -p $OUT
for i in 1 2; do
  for s in 1 0; do
    KRY_YP_STAGE=$s timeout -k 10 200 python bench.py --workload cfg4 --quick > $OUT/s${s}_$i.log 2>&1 || { tail -5 $OUT/s${s}_$i.log; exit 1; }
    python3 -c "import json,sys; b=json.loads(open('$OUT/s${s}_$i.log').read().strip().splitlines()[-1]); print('yp_stage=$s run $i', round(b['value']/8,1), 'it/s', round(b['ms_per_step'],4), 'ms', round(b['roofline']['spmv_ms'],4))"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/cfg_time.py cfg4 40 > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
