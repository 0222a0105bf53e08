#!/bin/bash
# A/B of a persistent CG loop switch on cfg2 (round 5), alternating processes;
# tools/cfg_time.py cfg2, and one phase trace of each. VAR (default
# KRY_CGP_DIA): 1 (default) against 0, e.g. the DIA form against the compact
# SELL-64 form, or KRY_CGP_WR: DIA values held in registers against re-read.
#   tools/cgp_ab.sh [VAR]
cd "$GRAFT_REPO_ROOT" || exit 1
V=${1:-KRY_CGP_DIA}
for rep in 1 2 3; do
  for d in 1 0; do
    out=$(env $V=$d timeout -k 10 240 python3 tools/cfg_time.py cfg2 2000 2>&1); rc=$?
    [ $rc -ne 0 ] && { echo "$out" | tail -5; exit $rc; }
    echo "$V=$d $(echo "$out" | tail -1 | cut -c1-80)"
  done
done
for d in 1 0; do
  out=$(env $V=$d KRY_CGP_TRACE=1 timeout -k 10 240 python3 tools/cfg_time.py cfg2 1000 2>&1); rc=$?
  [ $rc -ne 0 ] && { echo "$out" | tail -5; exit $rc; }
  echo "$V=$d $(echo "$out" | grep 'cgp trace' | tail -1)"
done
