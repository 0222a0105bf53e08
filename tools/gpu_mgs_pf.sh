#!/bin/bash
# cfg3 GMRES(30): per-pass cost of the register-resident MGS kernel with the
# next basis vector prefetched (default) and without (KRY_MGS_NOPF=1: timing
# experiment only, wrong results; the switch was a temporary template flag of
# gm_mgsp_kernel, removed after the measurement in profiles/r03_mgs_prefetch.txt).
OUT=$GRAFT_REPO_ROOT/gpurun_out/mgspf; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  KRY_MGS_NOPF=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/pf$v -o gm -- python3 $GRAFT_REPO_ROOT/tools/gm_steps.py cfg3 2 > $OUT/pf$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "nopf $v rc=$rc"; tail -3 $OUT/pf$v.log; exit $rc; }
  echo "== KRY_MGS_NOPF=$v"; python3 $GRAFT_REPO_ROOT/tools/gm_steps_summary.py $(ls $OUT/pf$v/gm_kernel_trace.csv $OUT/pf$v/*/gm_kernel_trace.csv 2>/dev/null | head -1) 2 | grep -E "fit|spmv mean|j= 0|j=29"
done
