#!/bin/bash
# A/B timing of one switch: `CFGS="gmres_metric gmres_cfg3" VAR=KRY_MGS_QR VALS="1 0" bash tools/gpu_ab.sh`,
# then the same configs from _ab_head/ (a build of the previous commit) when present.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out; mkdir -p $OUT
for c in $CFGS; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 180 python -u tools/cfg_time.py $c > $OUT/ab_${c}_${v}.log 2>&1 || { echo "$c $VAR=$v failed"; tail -20 $OUT/ab_${c}_${v}.log; exit 1; }
    echo "$VAR=$v $(tail -1 $OUT/ab_${c}_${v}.log)"
  done
  if [ -d _ab_head ]; then
    (cd _ab_head && timeout -k 10 180 python -u tools/cfg_time.py $c > ../$OUT/ab_${c}_head.log 2>&1) || { echo "$c head failed"; tail -20 $OUT/ab_${c}_head.log; exit 1; }
    echo "head $(tail -1 $OUT/ab_${c}_head.log)"
  fi
done
