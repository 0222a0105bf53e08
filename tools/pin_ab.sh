#!/bin/bash
# A/B of the pinned-in-place host transfers (round 5): tools/e2e_time.py
# phases with KRY_HOST_PIN=1 (default) and 0, alternating processes.
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for pin in 1 0; do
    KRY_HOST_PIN=$pin timeout -k 10 240 python3 -u tools/e2e_time.py phases || exit $?
  done
done
