#!/bin/bash
# Phase split of the register-resident MGS kernel (KRY_MGS_TRACE) on
# tools/cfg_time.py CFG under one environment switch with two values:
#   tools/mgs_trace.sh VAR A B gmres_cfg3
cd "$GRAFT_REPO_ROOT" || exit 1
VAR=$1; A=$2; B=$3; shift 3
for val in "$A" "$B"; do
  out=$(env KRY_MGS_TRACE=1 "$VAR=$val" timeout -k 10 240 python3 tools/cfg_time.py "$@" 2>&1); rc=$?
  [ $rc -ne 0 ] && { echo "$out" | tail -8; exit $rc; }
  echo "$VAR=$val"; echo "$out" | grep -E "mgs trace" | tail -2; echo "$out" | tail -1 | cut -c1-120
done
