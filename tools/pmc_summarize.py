"""Summarise tools/pmc_traffic.sh output into per-launch HBM traffic.

Reads <dir>/{micro,bench}_{FETCH_SIZE,WRITE_SIZE}/run_counter_collection.csv,
averages the counters per kernel name (KiB per dispatch -> bytes), derives
the read-side scale from the calibration kernel (known bytes = 10 * nslots of
the 216^3 compact SELL-64 image) and reports the CG SpMV kernel's corrected
traffic per launch next to its algorithmic bytes.
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


def main(out):
    import bench
    from krylov_amd import _lib, problems

    A = problems.stencil15_3d(216)
    n, nnz = A.shape[0], int(A.nnz)
    nslices, nslots, nirr = _lib.csr_layout(A.indptr)
    f = lambda w, c: per_kernel(os.path.join(out, f"{w}_{c}", "run_counter_collection.csv"), c)
    mf, mw, bf, bw = f("micro", "FETCH_SIZE"), f("micro", "WRITE_SIZE"), f("bench", "FETCH_SIZE"), f("bench", "WRITE_SIZE")
    cal_fetch, _ = find(mf, "sell_stream_calib<unsigned short>")
    scale = 10.0 * nslots / cal_fetch
    fetch, name = find(bf, "spmv_sell_kernel", "true", "EpiApDot")
    write, _ = find(bw, "spmv_sell_kernel", "true", "EpiApDot")
    alg = bench.spmv_S(n, nnz)
    res = {
        "kernel": name,
        "fetch_raw_bytes": fetch,
        "write_bytes": write,
        "read_scale_from_calibration": scale,
        "calibration": "sell_stream_calib<uint16>: the compact image's 2 + 8 B/lane nontemporal matrix stream, "
                       "10 B x nslots known bytes, FETCH_SIZE x 1024 measured",
        "traffic_bytes_per_launch": fetch * scale + write,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (fetch * scale + write) / alg,
        "nslots": nslots,
        "n": n,
        "nnz": nnz,
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
