#!/bin/bash
# Which --configs leg makes the process crash at exit under rocprofv3
# --kernel-trace (profiles/README.md, round 2)? One leg per profiled run, in
# the order given by LEGS; stop at the first crash (nothing more on the GPU
# after it). /proc/self/maps at exit goes to gpurun_out/exit_maps_<leg>.txt.
OUT=$GRAFT_REPO_ROOT/gpurun_out/exit_bisect; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for leg in ${LEGS:-cfg2 cfg4 cfg5}; do
  KRY_EXIT_MAPS=$OUT/maps_$leg.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$leg -o run -- python3 $GRAFT_REPO_ROOT/tools/cfg_time.py $leg 20 > $OUT/$leg.log 2>&1
  rc=$?; echo "$leg rc=$rc"
  if [ $rc -ne 0 ]; then grep -A30 "Aborted at" $OUT/$leg.log | head -40; exit $rc; fi
done
