#!/bin/bash
# Counter passes over any program, one small group per rocprofv3 run under its
# own limit (the gfx950 per-block slot limits: 8 SQ, 4 TCP, 2 TA, 2 TD, 2
# GRBM, FETCH_SIZE and WRITE_SIZE alone); stop at the first failing pass.
# tools/pmc_summary.py -> per-kernel means per dispatch.
#
#   tools/pmc_passes.sh NAME [BYTES] -- PROGRAM ARGS...
#
# BYTES (optional) is the kernel's algorithmic bytes per dispatch, for the
# traffic ratio. PMC_TRAFFIC_ONLY=1 runs only the L2 hit/miss, FETCH_SIZE and
# WRITE_SIZE passes. Output: gpurun_out/pmc_NAME/summary.json.
NAME=$1; shift
BYTES=0
if [ "$1" != "--" ]; then BYTES=$1; shift; fi
[ "$1" == "--" ] && shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
GROUPS_ALL=( "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU" \
           "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TD_TD_BUSY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE")
[ -n "$PMC_TRAFFIC_ONLY" ] && GROUPS_ALL=("TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE")
for grp in "${GROUPS_ALL[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT $BYTES > $OUT/summary.json && cat $OUT/summary.json
