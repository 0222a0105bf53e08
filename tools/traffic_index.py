"""Build profiles/r05_traffic_index.json: HBM traffic per launch for every
bench.py leg that has a committed rocprofv3 --pmc summary (development tool).

Each summary was taken with FETCH_SIZE and WRITE_SIZE in separate passes
(MI355X_MICROARCH.md, HBM / rocprofv3 section). Read bytes are FETCH_SIZE
KiB x 1024 x the calibrated read scale, as the guide's gfx950 correction
prescribes (x1.997 measured on a 16-B stream of known size); write bytes are
WRITE_SIZE KiB x 1024. bench.py (leg_traffic) copies these into the compact
line's `traffic` fields when the leg runs on the same (n, nnz).

    python3 tools/traffic_index.py
"""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")

METRIC = (10_077_696, 149_770_936)
CFG2 = (1_000_000, 4_996_000)
CFG3 = (2_000_000, 39_999_788)
CFG4 = (10_004_569, 50_010_193)
CFG5 = (8_000_000, 55_760_000)


def load(name):
    with open(os.path.join(P, name)) as f:
        return json.load(f)


def entry(nnz_pair, nbytes, src, note=None):
    e = {"n": nnz_pair[0], "nnz": nnz_pair[1], "bytes": float(nbytes), "src": f"profiles/{src}"}
    if note:
        e["note"] = note
    return e


def kernel_row(d, prefix):
    for k, v in d["kernels"].items():
        if k.startswith(prefix):
            return v
    raise KeyError(prefix)


def main():
    idx = {}
    tr = load("r03b_pmc_traffic.json")
    idx["metric_cg"] = {"spmv": entry(METRIC, tr["kernels"]["dia"]["traffic_bytes_per_launch"], "r03b_pmc_traffic.json")}
    idx["spmv_general"] = {"spmv": entry(METRIC, tr["kernels"]["pair"]["traffic_bytes_per_launch"],
                                         "r03b_pmc_traffic.json")}
    cb = load("r04_pmc_cb.json")["kernels"]
    # corrected = FETCH x2 + WRITE, per dispatch; the permuted metric takes 3 dispatches per SpMV
    idx["spmv_unstructured"] = {"spmv": entry(METRIC, cb["metric_permuted"]["hbm_bytes_corrected"] * 3,
                                              "r04_pmc_cb.json", "3 dispatches per SpMV")}
    idx["gmres"] = {"spmv": entry(CFG3, cb["cfg3"]["hbm_bytes_corrected"], "r04_pmc_cb.json")}
    idx["bicgstab_cfg3"] = {"spmv": entry(CFG3, cb["cfg3"]["hbm_bytes_corrected"], "r04_pmc_cb.json")}
    mg = load("r03_pmc_mgsl.json")
    mgsl = next(v for k, v in mg.items() if "gm_mgsl_kernel" in k)
    sd = next(v for k, v in mg.items() if "EpiStoreDot" in k)
    idx["gmres_metric"] = {"mgs": entry(METRIC, mgsl["fetch_bytes_mean"] + mgsl["write_bytes_mean"], "r03_pmc_mgsl.json"),
                           "spmv": entry(METRIC, sd["fetch_bytes_mean"] + sd["write_bytes_mean"], "r03_pmc_mgsl.json")}
    db = load("r05_pmc_dia_blk.json")
    idx["cfg4"] = {"spmv": entry(CFG4, kernel_row(db, "void kry::spmv_dia_blk_kernel")["hbm_bytes"],
                                 "r05_pmc_dia_blk.json")}
    c5 = load("r04_pmc_cfg5.json")
    idx["cfg5"] = {"spmv": entry(CFG5, kernel_row(c5, "void kry::spmv_dia_kernel<double, float, 8, kry::SrcPlain<double>, "
                                                  "kry::EpiLanczos")["hbm_bytes_corrected"], "r04_pmc_cfg5.json"),
                   "update": entry(CFG5, c5["kernels"]["void "]["hbm_bytes_corrected"], "r04_pmc_cfg5.json",
                                   "mr_upd_kernel (its name is truncated to 'void ' in the summary)")}
    c2 = load("r05_pmc_cfg2_wr.json")
    idx["cfg2"] = {"iteration": entry(CFG2, c2["read_bytes_per_iteration"] + c2["write_bytes_per_iteration"],
                                      "r05_pmc_cfg2_wr.json", "per iteration of the persistent loop")}
    extra = os.path.join(P, "r05_traffic_extra.json")  # newer passes override the ones above
    if os.path.exists(extra):
        with open(extra) as f:
            for leg, kernels in json.load(f).items():
                idx.setdefault(leg, {}).update(kernels)
    with open(os.path.join(P, "r05_traffic_index.json"), "w") as f:
        json.dump(idx, f, indent=1)
    for leg, ks in idx.items():
        for k, e in ks.items():
            print(f"{leg:20s} {k:10s} {e['bytes'] / 1e9:8.3f} GB  {e['src']}")


if __name__ == "__main__":
    main()
