#!/bin/bash
# A/B of the in-launch exchange poll (round 5): the persistent MGS and CG
# kernels with the 16-B granule-pair poll (default) against the round-4 poll
# (KRY_XCHG_LEGACY=1: two 8-B loads, every pair re-read), alternating on one
# box, each configuration in its own process under its own limit; stop at
# the first failure. metric GMRES(30), cfg3 GMRES(30), cfg2 CG.
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for mode in 0 1; do
    for cfg in gmres_metric gmres_cfg3 "cfg2 2000"; do
      out=$(KRY_XCHG_LEGACY=$mode timeout -k 10 240 python3 tools/cfg_time.py $cfg 2>&1)
      rc=$?
      [ $rc -ne 0 ] && { echo "$out" | tail -5; exit $rc; }
      echo "legacy=$mode rep=$rep $(echo "$out" | tail -1 | cut -c1-160)"
    done
  done
done
