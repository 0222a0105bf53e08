"""Operator images built on the device (round 5, device_build.hip).

kry_csr_create uploads an int32 CSR once and builds the SELL-64 image (and
its compact uint16 form) and the SELL-128 diagonal-offset image with
kernels. The host builders (host_image.cpp: sell_plan, sell_fill,
compact_fill, dia_build; KRY_DEVICE_BUILD=0) are the definition: every
buffer of the device-built image must equal theirs byte for byte
(kry_csr_compare), and the SpMV over it stays bitwise SciPy's csr_matvec
(the reference's A @ x, _helpers.py:44-48). Cases: stencils (DIA), fp32
values, irregular slices (kept as CSR), unsorted rows (no DIA), slices with
more offsets than the DIA kernel keeps (the host builder decides), empty
rows and a ragged last slice, and invalid input rejected as on the host.
"""
import ctypes

import numpy as np
import pytest
import scipy.sparse

pytestmark = pytest.mark.gpu


def _compare(a, b):
    from krylov_amd import _lib

    out = np.zeros(2, dtype=np.int64)
    _lib.check(_lib.lib.kry_csr_compare(a.handle, b.handle, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
    return int(out[0]), int(out[1])


def _banded(n, offsets, seed, drop=0.0, dtype=np.float64):
    rng = np.random.default_rng(seed)
    diags, offs = [], []
    for o in offsets:
        d = rng.standard_normal(n - abs(o))
        if drop:
            d[rng.random(d.shape[0]) < drop] = 0.0
        diags.append(d)
        offs.append(o)
    A = scipy.sparse.diags(diags, offs, shape=(n, n), format="csr", dtype=dtype)
    A.eliminate_zeros()
    A.sort_indices()
    return A


def _cases():
    from krylov_amd import problems

    rng = np.random.default_rng(3)
    lens = rng.integers(0, 6, 9001)
    lens[5000:5003] = 900  # irregular slices: a few very long rows
    lens[100:300] = 0  # empty rows
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    cols = np.sort(rng.integers(0, 9001, ip[-1]).astype(np.int32))
    rows = np.repeat(np.arange(9001), lens)
    order = np.lexsort((cols, rows))
    irr = scipy.sparse.csr_matrix((rng.standard_normal(ip[-1]), cols[order], ip), shape=(9001, 9001))
    uns = problems.poisson2d(200).tocsr().copy()
    for r in range(0, uns.shape[0], 7):  # reverse some rows: unsorted, no DIA
        a, b = uns.indptr[r], uns.indptr[r + 1]
        uns.indices[a:b] = uns.indices[a:b][::-1].copy()
        uns.data[a:b] = uns.data[a:b][::-1].copy()
    W, _ = problems.shifted_lap3d_weighted(30)
    return {
        "stencil15": problems.stencil15_3d(40),
        "poisson_ragged": problems.poisson2d(301),
        "fp32_weighted": W,
        "irregular": irr,
        "unsorted": uns,
        "wide_offsets": _banded(40_000, list(range(-40, 41)), 5),  # 81 offsets per slice: beyond the kernel's 64
        "holes": _banded(70_001, [-300, -2, 0, 1, 5, 300], 6, drop=0.3),
    }


@pytest.mark.parametrize("name", ["stencil15", "poisson_ragged", "fp32_weighted", "irregular", "unsorted",
                                  "wide_offsets", "holes"])
def test_device_built_image_equals_host(name, monkeypatch):
    import krylov_amd

    A = _cases()[name]
    dev = krylov_amd.CsrOperator(A)
    monkeypatch.setenv("KRY_DEVICE_BUILD", "0")
    host = krylov_amd.CsrOperator(A)
    lay = dev.layout()
    assert lay == host.layout()
    if name in ("stencil15", "poisson_ragged", "fp32_weighted", "holes", "wide_offsets"):
        assert lay["dia"]
    if name == "unsorted":
        assert not lay["dia"]
    if name == "irregular":
        assert lay["irregular"] > 0
    assert _compare(dev, host) == (0, 0)
    x = np.random.default_rng(1).standard_normal(A.shape[0]).astype(A.dtype)
    np.testing.assert_array_equal(np.asarray(dev @ x).view(np.uint8), np.asarray(A @ x).view(np.uint8))
    X = np.random.default_rng(2).standard_normal((A.shape[0], 4)).astype(A.dtype)
    np.testing.assert_array_equal(np.asarray(dev @ X).view(np.uint8), np.asarray(A @ X).view(np.uint8))


def test_device_built_metric_image_equals_host(monkeypatch):
    """The BASELINE metric matrix (15-point 216^3): the device build gives the
    host builders' SELL-64, compact and DIA images byte for byte."""
    import krylov_amd
    from krylov_amd import problems

    A = problems.stencil15_3d(216)
    dev = krylov_amd.CsrOperator(A)
    monkeypatch.setenv("KRY_DEVICE_BUILD", "0")
    host = krylov_amd.CsrOperator(A)
    assert dev.layout()["dia"] and dev.layout() == host.layout()
    assert _compare(dev, host) == (0, 0)


@pytest.mark.parametrize("defect", ["col_negative", "col_too_large", "indptr_decreasing"])
def test_device_build_rejects_invalid_csr(defect):
    """Validation on the device: the same ValueError (KRY_EINVAL) as the host
    check, nothing left allocated."""
    import krylov_amd
    from krylov_amd import problems

    A = problems.poisson2d(100).tocsr().copy()
    if defect == "col_negative":
        A.indices[777] = -1
    elif defect == "col_too_large":
        A.indices[778] = A.shape[0]
    else:
        A.indptr[5000] = A.indptr[5001] + 1
    before = krylov_amd.memory_stats()["bytes_in_use"]
    with pytest.raises(ValueError):
        krylov_amd.CsrOperator(A)
    assert krylov_amd.memory_stats()["bytes_in_use"] == before
