#!/bin/bash
# The counter names this box's rocprofv3 offers (gfx950), for choosing PMC passes.
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_list
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 -L > $OUT/list.txt 2>&1
rc=$?; echo "list rc=$rc"; grep -c . $OUT/list.txt; exit $rc
