#!/bin/bash
# Round-3 refresh after the column-blocked quad loads: the default bench line
# and its rocprofv3 kernel-trace summary. Each step has its own limit.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT/prof_r03e
timeout -k 10 600 python bench.py > $OUT/bench_r03e.log 2>&1 || { tail -20 $OUT/bench_r03e.log; exit 1; }
tail -c 300 $OUT/bench_r03e.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r03e -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof_r03e/stdout.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; exit $rc
