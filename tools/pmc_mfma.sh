#!/bin/bash
# MFMA utilisation of the GMRES(30) Arnoldi step on the metric matrix and of
# block CG on cfg4 (north_star: "MFMA utilisation (block orthogonalisation)
# reported"). The counter list of this box goes to mfma/counters.txt; every
# SQ counter whose name mentions MFMA (at most 6) plus SQ_BUSY_CYCLES and
# GRBM_GUI_ACTIVE is collected in one --pmc pass per program. Each pass under
# its own time limit; stop at the first failure.
OUT=$GRAFT_REPO_ROOT/gpurun_out/mfma; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
C=$(grep -o "SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*" $OUT/counters.txt | sort -u | head -6 | tr '\n' ' ')
echo "MFMA counters: $C"
[ -z "$C" ] && { echo "no MFMA counter listed"; exit 1; }
for prog in gmres_metric cfg4; do
  timeout -s KILL 240 rocprofv3 --pmc $C SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/$prog -o run -- python3 $GRAFT_REPO_ROOT/tools/cfg_time.py $prog > $OUT/$prog.log 2>&1
  rc=$?; echo "$prog rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$prog.log; exit $rc; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_mfma_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
