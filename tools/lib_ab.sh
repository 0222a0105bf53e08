#!/bin/bash
# A/B of two library builds on one box, alternating processes: the in-tree
# library against KRYLOV_LIB=$1 (a build of another commit), on
# tools/cfg_time.py $2 [$3].
#   tools/lib_ab.sh build_ab/libkrylov_hip_COMMIT.so cfg2 2000
cd "$GRAFT_REPO_ROOT" || exit 1
OTHER=$1; shift
for rep in 1 2 3; do
  for lib in tree other; do
    if [ $lib = tree ]; then
      out=$(timeout -k 10 240 python3 tools/cfg_time.py "$@" 2>&1); rc=$?
    else
      out=$(KRYLOV_LIB=$OTHER timeout -k 10 240 python3 tools/cfg_time.py "$@" 2>&1); rc=$?
    fi
    [ $rc -ne 0 ] && { echo "$out" | tail -5; exit $rc; }
    echo "$lib $(echo "$out" | tail -1 | cut -c1-90)"
  done
done
