#!/bin/bash
# A/B of one environment switch on one box, alternating processes:
#   tools/env_ab.sh VAR A B CFG [ARGS]   (tools/cfg_time.py CFG ARGS with VAR=A, then VAR=B; 3 rounds)
# prints each run's rate and, for GMRES legs, the SpMV and MGS ms per launch.
cd "$GRAFT_REPO_ROOT" || exit 1
VAR=$1; A=$2; B=$3; shift 3
for rep in 1 2 3; do
  for val in "$A" "$B"; do
    out=$(env "$VAR=$val" timeout -k 10 240 python3 tools/cfg_time.py "$@" 2>&1); rc=$?
    [ $rc -ne 0 ] && { echo "$out" | tail -8; exit $rc; }
    echo "$VAR=$val $(echo "$out" | tail -1 | python3 -c '
import ast, sys
line = sys.stdin.read().strip()
name, _, rest = line.partition(" ")
try:
    d = ast.literal_eval(rest)
except Exception:
    print(line[:160]); sys.exit()
out = {"it_per_s": round(d.get("it_per_s", 0), 1)}
for k in ("spmv", "mgs"):
    if k in d:
        out[k + "_ms"] = round(d[k]["ms_per_launch"], 4)
print(name, out)')"
  done
done
