"""The diagonal-offset image (SELL-64/DIA, kry_csr::dia_*) on the MI355X.

Structured matrices (stencils, bands) are stored as per-slice offset lists
with lane masks and no per-entry column index. The single-RHS SpMV over that
image must stay bitwise SciPy csr_matvec: every row summed from 0 in stored
order, holes skipped (never multiplied, so an inf or NaN that only a hole
would reach cannot leak in), explicit zeros still multiplied.
"""
import numpy as np
import pytest
import scipy.sparse

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))


def _structured():
    from krylov_amd import problems

    W, _ = problems.shifted_lap3d_weighted(24)
    return {
        "stencil15_40": problems.stencil15_3d(40),
        "poisson2d_300": problems.poisson2d(300),
        "poisson2d_61": problems.poisson2d(61),  # n = 3721: slices straddle the grid lines
        "shifted_lap3d_f32": W,
    }


@pytest.mark.parametrize("name", ["stencil15_40", "poisson2d_300", "poisson2d_61", "shifted_lap3d_f32"])
def test_dia_spmv_bitwise(name, monkeypatch):
    import krylov_amd

    A = _structured()[name]
    op = krylov_amd.CsrOperator(A)
    lay = op.layout()
    assert lay["dia"]
    assert lay["dia_slots"] <= lay["slots"] * 1.25
    rng = np.random.default_rng(1)
    x = rng.standard_normal(A.shape[0]).astype(A.dtype) * 10.0 ** rng.integers(-20, 20, A.shape[0])
    y = op @ x
    _bits_equal(y, A @ x)
    monkeypatch.setenv("KRY_SPMV_DIA", "0")
    op0 = krylov_amd.CsrOperator(A)
    assert not op0.layout()["dia"]
    _bits_equal(op0 @ x, y)


def test_dia_holes_are_never_read():
    """Row 5 lacks the -1 offset its slice holds; x[4] = NaN is reached by
    rows 3 and 4 only, so y[5] stays finite and bitwise; an explicit zero at
    offset +1 of row 8 multiplies x[9] = inf into NaN, as SciPy does."""
    import krylov_amd

    n = 200
    rows, cols, vals = [], [], []
    for r in range(n):
        for off, v in ((-1, -1.0), (0, 4.0), (1, -2.0)):
            c = r + off
            if 0 <= c < n and not (r == 5 and off == -1):  # (5, 4) absent: a hole
                rows.append(r)
                cols.append(c)
                vals.append(0.0 if (r == 8 and off == 1) else v)  # (8, 9) an explicit zero
    indptr = np.searchsorted(np.asarray(rows), np.arange(n + 1)).astype(np.int32)
    A = scipy.sparse.csr_matrix((np.asarray(vals), np.asarray(cols, dtype=np.int32), indptr), shape=(n, n))
    assert A.nnz == len(vals) and A.has_sorted_indices
    op = krylov_amd.CsrOperator(A)
    assert op.layout()["dia"]
    x = np.arange(1.0, n + 1.0)
    x[4] = np.nan
    x[9] = np.inf
    y = op @ x
    ref = A @ x
    assert np.isfinite(y[5]) and np.isnan(y[3]) and np.isnan(y[4]) and np.isnan(y[8])
    np.testing.assert_array_equal(y, ref)
    fin = np.isfinite(ref)
    _bits_equal(y[fin], ref[fin])


def test_dia_not_built_for_unsorted_duplicate_or_scattered():
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(50).tocsr()
    # unsorted row 70: swap its first two entries
    U = P.copy()
    a = U.indptr[70]
    U.indices[a], U.indices[a + 1] = U.indices[a + 1], U.indices[a]
    U.data[a], U.data[a + 1] = U.data[a + 1], U.data[a]
    assert not krylov_amd.CsrOperator(U).layout()["dia"]
    x = np.random.default_rng(2).standard_normal(P.shape[0])
    _bits_equal(krylov_amd.CsrOperator(U) @ x, U @ x)
    # a duplicate entry (summed as stored)
    D = scipy.sparse.csr_matrix((np.r_[1.5, P.data], np.r_[0, P.indices].astype(np.int32),
                                 np.r_[0, P.indptr[1:] + 1].astype(np.int32)), shape=P.shape)
    assert D.indices[0] == D.indices[1] == 0  # row 0 holds column 0 twice
    assert not krylov_amd.CsrOperator(D).layout()["dia"]
    _bits_equal(krylov_amd.CsrOperator(D) @ x, D @ x)
    # scattered columns: no shared offsets
    R = problems.random_nonsym(20_000, seed=4)
    assert not krylov_amd.CsrOperator(R).layout()["dia"]


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000])
def test_dia_ragged_sizes(n):
    import krylov_amd

    r = np.arange(n)
    rows = np.concatenate([r[3:], r, r[:-1]])
    cols = np.concatenate([r[:-3], r, r[1:]]) if n > 3 else np.concatenate([r[:0], r, r[1:]])
    vals = np.concatenate([np.full(max(n - 3, 0), 0.5), np.full(n, 3.0), np.full(max(n - 1, 0), -1.0)])
    A = scipy.sparse.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    A.sort_indices()
    assert A.nnz == vals.size
    op = krylov_amd.CsrOperator(A)
    assert op.layout()["dia"]
    x = np.random.default_rng(n).standard_normal(n)
    _bits_equal(op @ x, A @ x)


def test_dia_cg_matches_oracle():
    """The CG SpMV on the DIA image inside a whole solve: the reference's
    iteration count and history (15-point stencil 24^3)."""
    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref

    S = problems.stencil15_3d(24)
    A = krylov_amd.CsrOperator(S)
    assert A.layout()["dia"]
    b = np.ones(S.shape[0])
    _, info = krylov_amd.cg(A, b, tol=1e-10)
    _, ref = krylov_ref.cg(S, b, tol=1e-10)
    assert info.numsteps == ref.numsteps
    np.testing.assert_allclose(np.asarray(info.resnorms)[:-1], np.asarray(ref.resnorms)[:-1], rtol=1e-10)
