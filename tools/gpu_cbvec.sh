#!/bin/bash
# Column-blocked SpMV: 16-B quad loads (default) against one load per entry
# (KRY_CB_VEC=0) on cfg3 GMRES(30), after the column-blocked bitwise tests.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/cbvec; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_fullsize_golden.py tests/test_gpu_solvers.py -k "column_blocked or compact or cfg3 or gmres" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for v in 1 0 1; do
  KRY_CB_VEC=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$v -o run -- python3 $GRAFT_REPO_ROOT/tools/cfg_time.py gmres_cfg3 > $OUT/v$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "vec $v rc=$rc"; tail -3 $OUT/v$v.log; exit $rc; }
  python3 - $OUT/v$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if 'spmv_cb' in row['Name']:
        print('vec', sys.argv[2], row['Calls'], 'calls', round(float(row['AverageNs'])/1e3, 1), 'us', row['Name'][:60])
PY
  grep "^gmres_cfg3" $OUT/v$v.log | cut -c1-100
done
