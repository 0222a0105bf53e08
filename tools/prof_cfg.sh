#!/bin/bash
# Kernel trace of one secondary config (tools/cfg_time.py CFG STEPS) under
# rocprofv3 --kernel-trace --stats; output gpurun_out/prof_CFG/.
#   [PROF_TAG=t] tools/prof_cfg.sh CFG [STEPS]   (PROF_TAG: a suffix for the output directory)
CFG=$1; STEPS=${2:-20}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$CFG${PROF_TAG:+_$PROF_TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/cfg_time.py $CFG $STEPS > $OUT/run.log 2>&1
rc=$?; tail -3 $OUT/run.log; exit $rc
