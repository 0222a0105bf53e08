"""bench.py's roofline arithmetic (host logic, no device): the bytes each
image must move per SpMV launch, the roofline object built from them, and
block CG's iteration bytes with and without the deferred yk updates."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

N, NNZ = 10_077_696, 149_770_936


def _layout(**kw):
    lay = {"slices": (N + 63) // 64, "slots": 150_285_696, "irregular": 0, "compact": True, "col_blocks": 0,
           "dia": False, "dia_slots": 0, "pair": False, "pair_slots": 0}
    lay.update(kw)
    return lay


def test_image_bytes_dia_metric():
    kern, b, form = bench.image_bytes_k1(_layout(dia=True, dia_slots=150_423_552), N, NNZ)
    assert kern == "spmv_dia_kernel"
    assert b == pytest.approx(150_423_552 * 8 + 150_423_552 / 128 * 20 + 2 * N * 8)
    assert b == pytest.approx(1_388_135_232)  # the bench line's figure for the metric
    # fp32 values (cfg5): 4 B per slot
    _, b4, f4 = bench.image_bytes_k1(_layout(dia=True, dia_slots=1000 * 128), 1000, 7000, vectors=3, vb=4)
    assert b4 == pytest.approx(1000 * 128 * 4 + 1000 * 20 + 3 * 1000 * 8) and "dia_slots*4" in f4


def test_image_bytes_column_blocked_launch_count():
    kern, b, _ = bench.image_bytes_k1(_layout(col_blocks=16), N, NNZ)
    ng = (N + 255) // 256
    assert kern == "spmv_cbp_kernel (3 launches over row-group ranges)"  # 39,366 groups, 16,384 per launch
    assert b == 12 * NNZ + 16 * N * 2 + (16 * ng + 1) * 8 + 2 * N * 8
    kern2, _, _ = bench.image_bytes_k1(_layout(col_blocks=8), 2_000_000, 39_999_788)
    assert kern2 == "spmv_cbp_kernel"  # cfg3: one launch


def test_image_bytes_pair_and_sell():
    _, b, _ = bench.image_bytes_k1(_layout(pair=True, pair_slots=150_400_000), N, NNZ)
    assert b == pytest.approx(150_400_000 * 10 + 150_400_000 / 128 * 4 + (N + 127) // 128 * 12 + 2 * N * 8)
    kern, b, _ = bench.image_bytes_k1(_layout(), N, NNZ)
    assert kern.startswith("spmv_sell_kernel (compact)")
    lay = _layout(compact=False)
    _, b, _ = bench.image_bytes_k1(lay, N, NNZ)
    assert b == lay["slots"] * 12 + lay["slices"] * 12 + 2 * N * 8


def test_hbm_roofline_fraction():
    r = bench.hbm_roofline("k", 8e9, 2e-3, "f", 10)
    assert r["achieved"] == pytest.approx(4000.0) and r["frac"] == pytest.approx(0.5)
    assert r["peak"] == bench.HBM_PEAK_GBS == 8000.0 and r["unit"] == "GB/s" and r["bound"] == "hbm"


@pytest.mark.parametrize("D", [0, 7, 31])
def test_cfg4_iteration_bytes(D):
    from krylov_amd import _lib

    n, k = 10_004_569, 8
    ds = 50_016_768
    res = {"n": n, "rhs": k, "layout": _layout(dia=True, dia_slots=ds), "elapsed": 1.3e-3 * 40,
           "prof": {_lib.PROF_SPMV: (40, 40 * 0.44)}, "ydefer": (D, 0)}
    spmv, it = bench.cfg4_rooflines(res, 40)
    vec = n * k * 8
    sb = ds * 8 + ds / 128 * 20 + 2 * vec
    assert spmv["bytes_per_launch"] == pytest.approx(sb)
    assert spmv["ms_per_launch"] == pytest.approx(0.44)
    flush = (D + 1) / D * vec if D else 2 * vec  # y in and out + the D - 1 older p, once per D steps
    assert it["bytes_per_iteration"] == pytest.approx(sb + 6 * vec + flush)
    assert it["ydefer"] == D
    assert it["frac"] == pytest.approx(it["bytes_per_iteration"] / 1.3e-3 / 1e9 / 8000.0)
