#!/bin/bash
# GMRES(30) cycle time on cfg3 for MGS grid settings (tuning helper).
cd $GRAFT_REPO_ROOT
for cfg in "1024 1024" "512 2048" "2048 512"; do
  set -- $cfg
  KRY_MGS_GRID=$1 KRY_MGS_PER=$2 timeout -k 10 120 python3 tools/gmres_probe.py 4 > gpurun_out/mgs_$1.log 2>&1 || exit 1
  echo "grid cap $1 per $2: $(tail -1 gpurun_out/mgs_$1.log)"
done
