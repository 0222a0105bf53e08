#!/bin/bash
# HBM traffic of the metric GMRES(30) cycle's streamed MGS kernel
# (gm_mgsl_kernel) and its SpMV: FETCH_SIZE / WRITE_SIZE passes over
# tools/cfg_time.py gmres_metric (one warm-up cycle + one timed cycle), read
# side calibrated on tools/dia_bench's value stream. One pass per run.
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_mgsl
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BIN=$GRAFT_REPO_ROOT/tools/dia_bench
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $OUT/micro_$c -o run -- $BIN 216 3 > $OUT/micro_$c.log 2>&1
  rc=$?; echo "micro $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/gm_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/cfg_time.py gmres_metric > $OUT/gm_$c.log 2>&1
  rc=$?; echo "gmres $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 - "$OUT" <<'PY'
import csv, os, sys, json
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "tools"))
from pmc_summarize import dia_slots, find, per_kernel
out = sys.argv[1]
f = lambda w, c: per_kernel(os.path.join(out, f"{w}_{c}", "run_counter_collection.csv"), c)
mf, bf, bw = f("micro", "FETCH_SIZE"), f("gm", "FETCH_SIZE"), f("gm", "WRITE_SIZE")
cal, _ = find(mf, "dia_probe<16, 4>")
scale = 8.0 * dia_slots(out) / cal
res = {"read_scale": scale}
for k, (v, cnt) in bf.items():
    if "mgsl" in k or "spmv_dia_kernel" in k:
        w = bw.get(k, (0, 0))[0]
        res[k[:90]] = {"dispatches": cnt, "fetch_bytes_mean": v * scale, "write_bytes_mean": w}
print(json.dumps(res, indent=1))
PY
