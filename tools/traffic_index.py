"""Build profiles/r06_traffic_index.json: HBM traffic per launch of every
bench.py leg's kernels, from the rocprofv3 --pmc passes of tools/pmc_legs.sh
(development tool; the passes run on the GPU box, their summaries are copied
to profiles/r06_pmc_legs/LEG.json with the build stamp in
profiles/r06_pmc_legs/build_id).

Read bytes are FETCH_SIZE KiB x 1024 x 2 (MI355X_MICROARCH.md "HBM": on
gfx950 FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read);
write bytes WRITE_SIZE KiB x 1024. Every entry carries the library build it
was measured on (kry_build_id); bench.py (leg_traffic) uses an entry only
when that equals the loaded library's, and prints traffic: null otherwise.

    python3 tools/traffic_index.py
"""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")
SRC = os.path.join(P, "r06_pmc_legs")
OUT = os.path.join(P, "r06_traffic_index.json")

METRIC = (10_077_696, 149_770_936)
CFG2 = (1_000_000, 4_996_000)
CFG3 = (2_000_000, 39_999_788)
CFG4 = (10_004_569, 50_010_193)
CFG5 = (8_000_000, 55_760_000)

# leg of the index -> (summary file, (n, nnz), {key: (kernel-name prefix, note)})
LEGS = {
    "metric_cg": ("metric", METRIC, {"spmv": ("void kry::spmv_dia_kernel<double, double, 16, kry::SrcPlain", None),
                                     "update": ("cg_upd_kernel", None)}),
    "spmv_general": ("general", METRIC, {"spmv": ("void kry::spmv_pair_kernel", None)}),
    "spmv_unstructured": ("unstructured", METRIC, {"spmv": ("void kry::spmv_rs1_kernel", None)}),
    "gmres": ("gmres_cfg3", CFG3, {"spmv": ("void kry::spmv_cbp_kernel", None),
                                   "mgs": ("gm_mgsp", "mean over the launches of the MGS kernel of a GMRES(30) cycle")}),
    "bicgstab_cfg3": ("bicgstab_cfg3", CFG3, {"spmv": ("void kry::spmv_cbp_kernel", None)}),
    "gmres_metric": ("gmres_metric", METRIC, {"spmv": ("void kry::spmv_dia_kernel", None),
                                              "mgs": ("gm_mgsl", "mean over the launches of a GMRES(30) cycle")}),
    "cfg4": ("cfg4", CFG4, {"spmv": ("void kry::spmv_dia_blk_kernel", None),
                            "ppass": ("cg_pdefer_kernel", None)}),
    "cfg5": ("cfg5", CFG5, {"spmv": ("void kry::spmv_dia_kernel", None), "update": ("mr_upd_kernel", None)}),
}


def kernel_bytes(summary, prefix):
    """(bytes per dispatch, dispatches) of the one kernel whose name starts
    with `prefix` (after 'void (anonymous namespace)::' is dropped)."""
    hits = []
    for name, d in summary["kernels"].items():
        full = d["kernel"].replace("(anonymous namespace)::", "")
        short = full.replace("void ", "", 1)
        if full.startswith(prefix) or short.startswith(prefix):
            c = d["counters"]
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                hits.append((2 * 1024 * c["FETCH_SIZE"] + 1024 * c["WRITE_SIZE"], d["dispatches"], full))
    if not hits:
        raise KeyError(prefix)
    hits.sort(key=lambda h: -h[1])  # the kernel with most dispatches (the leg's own)
    return hits[0]


def main():
    with open(os.path.join(SRC, "build_id")) as f:
        build = f.read().strip()
    idx = {"build": build}
    for leg, (fname, (n, nnz), keys) in LEGS.items():
        path = os.path.join(SRC, f"{fname}.json")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            summ = json.load(f)
        for key, (prefix, note) in keys.items():
            try:
                b, disp, full = kernel_bytes(summ, prefix)
            except KeyError:
                continue
            e = {"n": n, "nnz": nnz, "bytes": float(b), "dispatches": disp, "kernel": full[:120],
                 "src": f"profiles/r06_pmc_legs/{fname}.json", "build": build}
            if note:
                e["note"] = note
            idx.setdefault(leg, {})[key] = e
    # cfg2: the persistent loop's bytes per iteration (its launches run whole chunks)
    path = os.path.join(SRC, "cfg2.json")
    if os.path.exists(path):
        with open(path) as f:
            summ = json.load(f)
        b, disp, full = kernel_bytes(summ, "cg_persist_kernel")
        iters = 210  # tools/cfg_time.py cfg2: 10 warm-up + 200 timed iterations
        idx["cfg2"] = {"iteration": {"n": CFG2[0], "nnz": CFG2[1], "bytes": b * disp / iters, "kernel": full[:120],
                                     "src": "profiles/r06_pmc_legs/cfg2.json", "build": build,
                                     "note": f"per iteration: {disp} launches over {iters} iterations"}}
    with open(OUT, "w") as f:
        json.dump(idx, f, indent=1)
    for leg, ks in idx.items():
        if leg != "build":
            print(leg, {k: round(v["bytes"] / 1e9, 4) for k, v in ks.items()})


if __name__ == "__main__":
    main()
