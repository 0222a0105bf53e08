"""Gather ceilings of the column-blocked SpMV (tools/gather_ceiling.hip) on
the matrices whose single-RHS SpMV takes it: cfg3 (random nonsymmetric,
n = 2e6, 19 random columns per row) and the metric matrix under a random
symmetric permutation (bench.py's spmv_unstructured). Writes
profiles/r04_gather_ceiling.json, which bench.py reads for the gather view of
those legs' rooflines.

    python3 tools/gather_ceiling.py [out.json]
"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from krylov_amd import problems  # noqa: E402


def run(lib, A, reps=20):
    ip = np.ascontiguousarray(A.indptr, dtype=np.int32)
    ix = np.ascontiguousarray(A.indices, dtype=np.int32)
    dv = np.ascontiguousarray(A.data, dtype=np.float64)
    res = np.zeros(32)
    rc = lib.gc_run(ctypes.c_int64(A.shape[0]), ctypes.c_int64(A.nnz), ip.ctypes.data_as(ctypes.c_void_p),
                    ix.ctypes.data_as(ctypes.c_void_p), dv.ctypes.data_as(ctypes.c_void_p), reps,
                    res.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
    nnz = int(A.nnz)
    g = lambda ms: nnz / (ms * 1e-3) / 1e9  # noqa: E731
    gather_ms = nnz / (res[3] * 1e9) * 1e3  # every gather at the L2-window rate
    overlap_ms, serial_ms = max(gather_ms, res[6]), gather_ms + res[6]
    return {
        "n": int(A.shape[0]), "nnz": nnz, "col_blocks": int(res[4]), "cols_per_block": int(res[5]),
        "library_spmv_ms": res[0], "library_g_per_s": g(res[0]),
        "grid_stride_gather_only_ms": res[1], "grid_stride_image_and_gather_ms": res[2],
        "window_2mb_g_per_s": res[3], "gathers_at_window_rate_ms": gather_ms,
        "image_stream_ms": res[6],
        "ceiling_overlap_ms": overlap_ms, "ceiling_serial_ms": serial_ms,
        "ceiling_g_per_s": g(overlap_ms),
        "what": "max(nnz gathers at the L2-resident random-gather rate (2 MB window), the 12-B column + value "
                "stream alone): gathers and stream perfectly overlapped (tools/gather_ceiling.hip); serial sum "
                "beside it as ceiling_serial_ms",
        "library_frac_of_ceiling": overlap_ms / res[0],
        "library_frac_of_serial": serial_ms / res[0],
        "candidate_contiguous_ms": res[7], "candidate_contiguous_mismatches": int(res[8]),
        "cbx_variants": {name: {"ms": res[9 + 2 * i], "mismatches": int(res[10 + 2 * i])}
                         for i, name in enumerate(CBX)},
        "window_g_per_s_by_mb": dict(zip(["2", "3", "4", "5", "8", "all_x"], [float(v) for v in res[25:31]])),
        "roff_bytes": int(res[4]) * int(A.shape[0]) * 2,
    }


# spmv_cbx<OWN, QPT, PF> at a grid (tools/gather_ceiling.hip, gc_run's variant table)
CBX = ["own16_q1_grid1024", "own16_q1_pf_grid1024", "own16_q2_grid768", "own16_q1_grid1024_no_row_offsets",
       "own8_q1_pf_grid1280", "own8_q2_pf_grid768", "own16_q1_pf_grid1024_no_row_offsets", "own16_q1_pf_grid768"]

def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "r04_gather_ceiling.json")
    which = sys.argv[2].split(",") if len(sys.argv) > 2 else ["cfg3", "metric_permuted"]
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "libgather_ceiling.so"))
    result = {}
    if "cfg3" in which:
        result["cfg3"] = run(lib, problems.random_nonsym(2_000_000))
        print("cfg3", json.dumps(result["cfg3"]), flush=True)
    if "metric_permuted" in which:
        B = problems.permuted_sym(problems.stencil15_3d(216), 0)
        result["metric_permuted"] = run(lib, B)
        print("metric_permuted", json.dumps(result["metric_permuted"]), flush=True)
        # column-block widths (KRY_CB_COLS, read when the image is built)
        for cols in (os.environ.get("GC_COLS_SWEEP") or "").split(","):
            if cols:
                os.environ["KRY_CB_COLS"] = cols
                r = run(lib, B)
                result[f"metric_permuted_cols{cols}"] = r
                print(f"metric_permuted cols={cols}", json.dumps(r), flush=True)
        os.environ.pop("KRY_CB_COLS", None)
    with open(out, "w") as f:
        json.dump(result, f, indent=1)


if __name__ == "__main__":
    main()
