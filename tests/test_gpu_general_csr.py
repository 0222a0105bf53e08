"""General CSR at the metric size: matrices that are not diagonal-structured.

The metric matrix (15-point 216^3, 149.8 M nonzeros) runs on the DIA image.
Two general-CSR paths take the same nonzeros at the same scale:

- with the DIA image off (KRY_SPMV_DIA=0) the paired-row SELL-128 image
  (spmv_pair_kernel): slot columns whose rows have adjacent columns;
- under a random symmetric permutation P A P^T (problems.permuted_sym, the
  bench's spmv_unstructured leg) the columns are scattered over all 10 M, and
  the column-blocked image takes it: 39,366 row groups, more than one launch
  of spmv_cbp_kernel holds, so the SpMV runs as 3 launches over group ranges.

Each SpMV must equal SciPy's csr_matvec (the reference's `A @ x`,
_helpers.py:44-48) bit for bit, and a CG on the permuted matrix must follow
the oracle's history (reference cg.py:155-234) to the parity tolerance.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def metric():
    from krylov_amd import problems

    return problems.stencil15_3d(216)


@pytest.fixture(scope="module")
def permuted(metric):
    from krylov_amd import problems

    return problems.permuted_sym(metric, 0)


def _x(n, seed):
    return np.random.default_rng(seed).uniform(-1.0, 1.0, n) * np.exp2(np.random.default_rng(seed + 1).integers(-20, 20, n))


def _bitwise(a, b):
    np.testing.assert_array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


def test_pair_image_metric_bitwise(metric, monkeypatch):
    import krylov_amd

    monkeypatch.setenv("KRY_SPMV_DIA", "0")
    op = krylov_amd.CsrOperator(metric)
    lay = op.layout()
    assert not lay["dia"] and lay["pair"] and lay["col_blocks"] == 0
    x = _x(metric.shape[0], 3)
    _bitwise(op @ x, metric @ x)


def test_permuted_metric_column_blocked_bitwise(permuted):
    import krylov_amd

    op = krylov_amd.CsrOperator(permuted)
    lay = op.layout()
    assert not lay["dia"] and lay["col_blocks"] > 0
    assert (permuted.shape[0] + 255) // 256 > 1024 * 16  # more than one launch of group ranges
    for seed in (5, 7):
        x = _x(permuted.shape[0], seed)
        _bitwise(op @ x, permuted @ x)


def test_permuted_metric_cg_matches_oracle(permuted):
    """CG on the permuted matrix (the CG SpMV epilogue's <p, Ap> block
    partials of all 3 launches feed alpha): 12 steps against the oracle."""
    import krylov_amd
    from oracle import krylov_ref

    b = np.ones(permuted.shape[0])
    op = krylov_amd.CsrOperator(permuted)
    _, info = krylov_amd.cg(op, b, tol=0.0, atol=0.0, maxiter=12)
    _, ref = krylov_ref.cg(permuted, b, tol=0.0, atol=0.0, maxiter=12)
    assert info.numsteps == ref.numsteps == 12
    got, want = np.asarray(info.resnorms), np.asarray(ref.resnorms)
    np.testing.assert_allclose(got[:-1], want[:-1], rtol=1e-10)
