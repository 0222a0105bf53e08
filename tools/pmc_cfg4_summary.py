"""Summarise tools/pmc_cfg4.sh: per-kernel mean HBM bytes per dispatch of
cfg4's block-CG kernels (FETCH_SIZE x read-side calibration + WRITE_SIZE),
next to each kernel's compulsory bytes (n = 10,004,569, k = 8: one vector
= 640.3 MB; the block DIA image's values 400.1 MB)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summarize import dia_slots, find, per_kernel  # noqa: E402

out = sys.argv[1]
f = lambda w, c: per_kernel(os.path.join(out, f"{w}_{c}", "run_counter_collection.csv"), c)
mf, bf, bw = f("micro", "FETCH_SIZE"), f("cfg4", "FETCH_SIZE"), f("cfg4", "WRITE_SIZE")
cal_fetch, _ = find(mf, "dia_probe<16, 4>")
scale = 8.0 * dia_slots(out) / cal_fetch
vec = 10_004_569 * 8 * 8
vals = 50_016_768 * 8
compulsory = {
    "spmv_dia_blk_kernel": ("values + p read, Ap written", vals + vec, vec),
    "OpCgR": ("r, Ap read; r written", 2 * vec, vec),
    "cg_pdefer_kernel": ("r, p_i read, p_i+1 written (+ y and 6 older p in, y out once per 7 steps)",
                         2 * vec + (7 * vec) / 7, vec + vec / 7),
}
res = {"read_scale_from_calibration": scale, "kernels": {}}
parts = {"spmv_dia_blk_kernel": ("spmv_dia_blk_kernel", "EpiApDot"), "OpCgR": ("OpCgR",),
         "cg_pdefer_kernel": ("cg_pdefer_kernel",)}
for key, (what, rd, wr) in compulsory.items():
    fetch, name = find(bf, *parts[key])
    write, _ = find(bw, *parts[key])
    res["kernels"][key] = {"kernel": name, "fetch_bytes": fetch * scale, "write_bytes": write,
                           "compulsory_read": rd, "compulsory_write": wr, "compulsory": what,
                           "traffic_over_compulsory": (fetch * scale + write) / (rd + wr)}
res["program"] = "tools/cfg_time.py cfg4 28 (block CG, Poisson 3163^2, 8 RHS, KRY_CG_YDEFER default 7)"
print(json.dumps(res, indent=1))
