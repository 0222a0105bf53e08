#!/bin/bash
# Counter passes over tools/dia_blk_probe (the library's block DIA SpMV, the
# slot-major probe with and without shuffled values and x loads, the copy
# floor; cfg4's Poisson 3163^2 at k = 8), one small group per rocprofv3 run
# under its own limit; stop at the first failing pass.
# tools/pmc_dia_blk_summary.py -> per-kernel means per dispatch.
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_dia_blk
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BIN=$GRAFT_REPO_ROOT/tools/dia_blk_probe
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU" \
           "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TD_TD_BUSY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $BIN 3163 5 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_dia_blk_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
