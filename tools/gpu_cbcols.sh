#!/bin/bash
# cfg3 column-blocked SpMV vs the column-block width (KRY_CB_COLS): the x
# window each pass keeps L2-resident against the per-(block, row) offset
# bytes that grow with the block count. Kernel trace per setting.
OUT=$GRAFT_REPO_ROOT/gpurun_out/cbcols; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in 262144 131072 65536 524288; do
  KRY_CB_COLS=$c timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c$c -o run -- python3 $GRAFT_REPO_ROOT/tools/cfg_time.py gmres_cfg3 > $OUT/c$c.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "cols $c rc=$rc"; tail -3 $OUT/c$c.log; exit $rc; }
  python3 - $OUT/c$c/run_kernel_stats.csv $c <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if 'spmv_cb' in row['Name'] and 'EpiStoreDotV' in row['Name']:
        print('cols', sys.argv[2], row['Calls'], 'calls', round(float(row['AverageNs'])/1e3, 1), 'us', row['Name'][:40])
PY
  grep "^gmres_cfg3" $OUT/c$c.log | cut -c1-120
done
