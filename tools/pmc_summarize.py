"""Summarise tools/pmc_traffic.sh output into per-launch HBM traffic.

Reads <dir>/{micro,bench}_{FETCH_SIZE,WRITE_SIZE}/run_counter_collection.csv,
averages the counters per kernel name (KiB per dispatch -> bytes), derives
the read-side scale from the calibration kernel (tools/dia_bench's
"values only" probe: known bytes = 8 * dia_slots of the 216^3 diagonal-offset
image) and reports the CG SpMV kernel's corrected traffic per launch next to
its algorithmic bytes.
"""
import csv
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def find(d, *parts):
    hits = [k for k in d if all(p in k for p in parts)]
    if len(hits) != 1:
        raise SystemExit(f"kernel match for {parts}: {hits}")
    return d[hits[0]][0], hits[0]


def dia_slots(out):
    """dia_slots as printed by tools/dia_bench's first line."""
    with open(os.path.join(out, "micro_FETCH_SIZE.log")) as f:
        for line in f:
            for tok in line.split():
                if tok.startswith("dia_slots="):
                    return int(tok.split("=")[1])
    raise SystemExit("dia_bench header not found")


def main(out):
    import bench
    from krylov_amd import problems

    A = problems.stencil15_3d(216)
    n, nnz = A.shape[0], int(A.nnz)
    slots = dia_slots(out)
    f = lambda w, c: per_kernel(os.path.join(out, f"{w}_{c}", "run_counter_collection.csv"), c)
    mf, bf, bw = f("micro", "FETCH_SIZE"), f("bench", "FETCH_SIZE"), f("bench", "WRITE_SIZE")
    cal_fetch, _ = find(mf, "dia_probe<16, 4>")
    scale = 8.0 * slots / cal_fetch
    alg = bench.spmv_S(n, nnz)
    kernels = {}
    for key, parts in (("dia", ("spmv_dia_kernel", "EpiApDot")), ("pair", ("spmv_pair_kernel", "EpiApDot")),
                       ("sell", ("spmv_sell_kernel", "EpiApDot"))):
        if not any(all(p in k for p in parts) for k in bf):
            continue
        fetch, name = find(bf, *parts)
        write, _ = find(bw, *parts)
        traffic = fetch * scale + write
        kernels[key] = {
            "kernel": name,
            "fetch_raw_bytes": fetch,
            "write_bytes": write,
            "traffic_bytes_per_launch": traffic,
            "traffic_over_algorithmic_S": traffic / alg,
        }
    res = {
        "read_scale_from_calibration": scale,
        "calibration": "dia_probe<16,4> (tools/dia_bench 'values only'): the diagonal-offset image's 16 B/lane (two "
                       "rows' values) nontemporal value stream, 8 B x dia_slots known bytes, FETCH_SIZE x 1024 measured",
        "kernels": kernels,
        "algorithmic_bytes_per_launch": alg,
        "dia_slots": slots,
        "n": n,
        "nnz": nnz,
        "program": "tools/spmv_legs.py 64 (64 metric CG iterations on each image: DIA, paired-row SELL-128, "
                   "compact SELL-64)",
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
