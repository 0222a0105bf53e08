#!/bin/bash
# PMC passes over the SpMV microbenchmark (one small counter group per
# rocprofv3 run; stop at the first failing pass).
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
BIN=$GRAFT_REPO_ROOT/tools/spmv_bench
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TA_TA_BUSY GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES" \
           "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ" "TCC_HIT TCC_MISS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 5 60 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $BIN 216 3 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
