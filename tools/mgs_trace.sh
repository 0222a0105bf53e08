#!/bin/bash
# Phase split of the register-resident MGS kernels (KRY_MGS_TRACE) on
# tools/cfg_time.py CFG, with the lookahead off and on:
#   tools/mgs_trace.sh gmres_cfg3
cd "$GRAFT_REPO_ROOT" || exit 1
for la in 0 1; do
  out=$(KRY_MGS_TRACE=1 KRY_MGS_LOOKAHEAD=$la timeout -k 10 240 python3 tools/cfg_time.py "$@" 2>&1); rc=$?
  [ $rc -ne 0 ] && { echo "$out" | tail -8; exit $rc; }
  echo "KRY_MGS_LOOKAHEAD=$la"; echo "$out" | grep -E "mgs trace" | tail -2; echo "$out" | tail -1 | cut -c1-120
done
