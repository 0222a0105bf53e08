"""Summarise tools/pmc_dia_blk.sh: per kernel of tools/dia_blk_probe (the
library's block DIA SpMV, the slot-major probe variants and the copy floor), the mean of every counter per dispatch, and derived rates:
VMEM instructions per slice, TA busy share, L2 hit rate, HBM bytes (FETCH_SIZE
x 2, the gfx950 correction for 16-B streaming reads, MI355X_MICROARCH.md
"HBM"; WRITE_SIZE as is) against the kernel's compulsory bytes."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N, K, SLOTS = 10_004_569, 8, 50_016_768
SLICES = (N + 127) // 128
COMPULSORY = SLOTS * 8 + SLOTS / 128 * 20 + 2 * N * K * 8


def main(out):
    acc = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(out, "p*", "run_counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for kern, cs in acc.items():
        short = kern.split("(")[0][:90] if "slot_major" not in kern else kern[:kern.index(">") + 1]
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"kernel": kern[:200], "dispatches": max(len(v) for v in cs.values()), "counters": m}
        if "SQ_INSTS_VMEM_RD" in m and "SQ_WAVES" in m:
            d["vmem_rd_per_wave"] = m["SQ_INSTS_VMEM_RD"] / max(m["SQ_WAVES"], 1)
            d["vmem_wr_per_wave"] = m.get("SQ_INSTS_VMEM_WR", 0) / max(m["SQ_WAVES"], 1)
        if "TA_TA_BUSY_sum" in m and "GRBM_GUI_ACTIVE" in m:
            # TA_BUSY summed over the TA instances (one per CU) against the GPU's active cycles (summed over XCDs)
            d["ta_busy_per_cu_share"] = m["TA_TA_BUSY_sum"] / 256 / (m["GRBM_GUI_ACTIVE"] / 8)
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            d["l2_hit_rate"] = m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m["TCC_MISS_sum"], 1)
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            d["hbm_bytes"] = 2 * 1024 * m["FETCH_SIZE"] + 1024 * m["WRITE_SIZE"]
            d["over_compulsory"] = d["hbm_bytes"] / COMPULSORY
        if "SQ_WAVE_CYCLES" in m:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    d[c.lower() + "_share"] = m[c] / max(m["SQ_WAVE_CYCLES"], 1)
        res[short] = d
    print(json.dumps({"compulsory_bytes": COMPULSORY, "slices": SLICES, "kernels": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
