#!/bin/bash
# A/B of the persistent CG loop's SpMV image on cfg2 (round 5): the DIA form
# (default) against the compact SELL-64 form (KRY_CGP_DIA=0), alternating
# processes; tools/cfg_time.py cfg2, and one phase trace of each.
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2 3; do
  for d in 1 0; do
    out=$(KRY_CGP_DIA=$d timeout -k 10 240 python3 tools/cfg_time.py cfg2 2000 2>&1); rc=$?
    [ $rc -ne 0 ] && { echo "$out" | tail -5; exit $rc; }
    echo "KRY_CGP_DIA=$d $(echo "$out" | tail -1 | cut -c1-80)"
  done
done
for d in 1 0; do
  out=$(KRY_CGP_DIA=$d KRY_CGP_TRACE=1 timeout -k 10 240 python3 tools/cfg_time.py cfg2 1000 2>&1); rc=$?
  [ $rc -ne 0 ] && { echo "$out" | tail -5; exit $rc; }
  echo "KRY_CGP_DIA=$d $(echo "$out" | grep 'cgp trace' | tail -1)"
done
