"""Summarise tools/pmc_passes.sh: per kernel, the mean of every counter per
dispatch and derived rates (VMEM instructions per wave, TA busy share, L2 hit
rate, L1->L2 read requests and their mean latency, HBM bytes: FETCH_SIZE in
KiB, x2 for the gfx950 correction of 16-B streaming reads as
MI355X_MICROARCH.md "HBM" prescribes, reported beside the raw figure since a
kernel of 8-B random gathers is not covered by that calibration; WRITE_SIZE
as is).

    python3 tools/pmc_summary.py OUT_DIR [BYTES_PER_DISPATCH]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(out, compulsory):
    acc = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(out, "p*", "run_counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for kern, cs in acc.items():
        short = kern.replace("(anonymous namespace)::", "").split("(")[0][:90]
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"kernel": kern[:200], "dispatches": max(len(v) for v in cs.values()), "counters": m}
        if "SQ_INSTS_VMEM_RD" in m and "SQ_WAVES" in m:
            d["vmem_rd_per_wave"] = m["SQ_INSTS_VMEM_RD"] / max(m["SQ_WAVES"], 1)
            d["vmem_wr_per_wave"] = m.get("SQ_INSTS_VMEM_WR", 0) / max(m["SQ_WAVES"], 1)
        if "TA_TA_BUSY_sum" in m and "GRBM_GUI_ACTIVE" in m:
            # summed over the TA instances (one per CU) against the active cycles (summed over XCDs)
            d["ta_busy_per_cu_share"] = m["TA_TA_BUSY_sum"] / 256 / (m["GRBM_GUI_ACTIVE"] / 8)
            if "SQ_INSTS_VMEM_RD" in m:
                d["ta_cycles_per_vmem"] = m["TA_TA_BUSY_sum"] / max(m["SQ_INSTS_VMEM_RD"] + m.get("SQ_INSTS_VMEM_WR", 0), 1)
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            d["l2_hit_rate"] = m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m["TCC_MISS_sum"], 1)
        if "TCP_TCC_READ_REQ_sum" in m:
            d["l2_read_requests"] = m["TCP_TCC_READ_REQ_sum"]
            if "TCP_TCC_READ_REQ_LATENCY_sum" in m:
                d["l2_read_latency_cycles"] = m["TCP_TCC_READ_REQ_LATENCY_sum"] / max(m["TCP_TCC_READ_REQ_sum"], 1)
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            d["hbm_read_bytes_raw"] = 1024 * m["FETCH_SIZE"]
            d["hbm_bytes_corrected"] = 2 * 1024 * m["FETCH_SIZE"] + 1024 * m["WRITE_SIZE"]
            d["hbm_bytes_raw"] = 1024 * m["FETCH_SIZE"] + 1024 * m["WRITE_SIZE"]
            if compulsory:
                d["over_compulsory_corrected"] = d["hbm_bytes_corrected"] / compulsory
                d["over_compulsory_raw"] = d["hbm_bytes_raw"] / compulsory
        if "SQ_WAVE_CYCLES" in m:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    d[c.lower() + "_share"] = m[c] / max(m["SQ_WAVE_CYCLES"], 1)
        res[short] = d
    print(json.dumps({"compulsory_bytes": compulsory or None, "kernels": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
