"""General CSR at the metric size: matrices that are not diagonal-structured.

The metric matrix (15-point 216^3, 149.8 M nonzeros) runs on the DIA image.
Two general-CSR paths take the same nonzeros at the same scale:

- with the DIA image off (KRY_SPMV_DIA=0) the paired-row SELL-128 image
  (spmv_pair_kernel): slot columns whose rows have adjacent columns;
- under a random symmetric permutation P A P^T (problems.permuted_sym, the
  bench's spmv_unstructured leg) the columns are scattered over all 10 M.
  Since round 5 the upload renumbers it (reverse Cuthill-McKee) and the
  rank-sorted SELL-128 image takes it; with KRY_RENUMBER=0 the
  column-blocked image does: 39,366 row groups, more than one launch of
  spmv_cbp_kernel holds, so the SpMV runs as 3 launches over group ranges.

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


def test_permuted_metric_column_blocked_bitwise(permuted, monkeypatch):
    import krylov_amd

    monkeypatch.setenv("KRY_RENUMBER", "0")
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


@pytest.fixture(scope="module")
def permuted_op(permuted):
    import krylov_amd

    return krylov_amd.CsrOperator(permuted)


def test_permuted_metric_renumbered_bitwise(permuted, permuted_op):
    """The default upload renumbers the permuted metric (reverse
    Cuthill-McKee) onto the rank-sorted image; y = A x in the caller's
    numbering is SciPy's bit for bit."""
    lay = permuted_op.layout()
    assert lay["renumbered"] and lay["rs"] and lay["col_blocks"] == 0
    for seed in (5, 7):
        x = _x(permuted.shape[0], seed)
        _bitwise(permuted_op @ x, permuted @ x)


def test_permuted_metric_cg_to_convergence(permuted, permuted_op):
    """CG to tol 1e-8 on the renumbered permuted metric against the reference's
    own CG on the same (permuted) matrix (tests/golden/permuted.npz,
    tests/golden/make_permuted.py): the same step count and success, the
    history within 1e-10 rel or 2x the reference's own summation-order noise
    on this matrix (tests/golden/selfnoise.npz "perm_cg": its CG under 1 / 2 /
    4 / N OpenBLAS threads, pairwise, extended and fsum inner products; the
    permuted-order SpMV makes this CG far more order-sensitive than the
    metric's: 2.1e-4 at the last steps against 3e-9), the final explicit
    residual within 64 eps (||b|| + ||A||_1 ||x||), and x's size-independent
    summaries equal to the metric solution's."""
    import os

    import krylov_amd
    from tests import gpu_helpers as H

    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    F = np.load(os.path.join(gold, "permuted.npz"))
    M = np.load(os.path.join(gold, "fullsize.npz"))
    b = np.ones(permuted.shape[0])
    x, info = krylov_amd.cg(permuted_op, b, tol=1e-8)
    ref = F["perm_cg_resnorms"]
    got = np.asarray(info.resnorms)
    assert info.success and info.numsteps == int(F["perm_cg_numsteps"]) == int(M["metric_cg_numsteps"])
    tol = np.maximum(1e-10, H.NOISE_FACTOR * H.selfnoise_envelope("perm_cg", ref))
    dev = np.abs(got[:-1] - ref[:-1]) / np.abs(ref[:-1])
    print(f"\npermuted metric CG (renumbered): {info.numsteps} steps, history max rel {dev.max():.2e} "
          f"({(dev / tol).max():.2f} of the tolerance)")
    assert np.all(dev <= tol)
    eps = np.finfo(np.float64).eps
    bound = 64 * eps * (np.linalg.norm(b) + float(abs(permuted).sum(axis=0).max()) * F["perm_cg_xstats"][1])
    assert abs(got[-1] - ref[-1]) <= bound
    xa = np.abs(x)
    np.testing.assert_allclose([xa.sum(), np.linalg.norm(x), xa.max()], F["perm_cg_xstats"], rtol=1e-8)
