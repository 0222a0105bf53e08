#!/bin/bash
# Counter passes over tools/gmres_probe.py (one small group per rocprofv3 run,
# each under its own time limit; stop at the first failure).
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_gmres
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "FETCH_SIZE" "SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/gmres_probe.py 1 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
