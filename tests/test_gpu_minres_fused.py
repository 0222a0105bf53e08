"""The one-launch MINRES step tail (mr_upd_kernel): alpha, the Lanczos
orthogonalisation, the QR update and the z / W / yk / p update in one launch
after the SpMV (one RHS, no preconditioners, float64 vectors).

Its inner products are summed in other fixed orders than the separate
kernels' (KRY_MR_UPD=0), so the two agree to rounding; both follow the
reference's iteration (oracle / fixtures) to 1e-10.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _state(A, b, inner=None):
    import krylov_amd
    from krylov_amd import _helpers
    from krylov_amd.minres import _MinresState

    st = _MinresState(_helpers.Problem(krylov_amd.CsrOperator(A) if not hasattr(A, "handle") else A, b, None, inner))
    st.start()
    st.set_criterion(np.zeros(1))
    return st


@pytest.mark.parametrize("weighted", [False, True])
def test_fused_tail_matches_separate_kernels_and_oracle(weighted, monkeypatch):
    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref

    W, w = problems.shifted_lap3d_weighted(40)  # n = 64,000 (fp32 matrix; float64 vectors under the weighted inner)
    A = W.astype(np.float64) if not weighted else W
    b = np.ones(A.shape[0], dtype=np.float64 if not weighted else np.float32)
    inner = krylov_amd.WeightedInner(w) if weighted else None
    st = _state(A, b, inner)
    h1, inv1 = st.run(60)
    assert st.update_path() == (True, 0) and not inv1
    monkeypatch.setenv("KRY_MR_UPD", "0")
    st0 = _state(A, b, inner)
    h0, _ = st0.run(60)
    assert st0.update_path() == (False, 0)
    np.testing.assert_allclose(h1[:, 0], h0[:, 0], rtol=1e-11)
    rkw = {"inner": (lambda x, y: np.dot(x.T, w * y))} if weighted else {}
    _, ref = krylov_ref.minres(A, b, tol=0.0, maxiter=60, **rkw)
    # the weighted case runs on a float32 matrix and right-hand side: the
    # north_star's fp32 contract (1e-4 rel) against the oracle
    np.testing.assert_allclose(h1[:, 0], np.asarray(ref.resnorms, dtype=np.float64)[1:61],
                               rtol=1e-4 if weighted else 1e-10)


def test_fused_tail_solution_and_explicit_residual(monkeypatch):
    """A whole solve to 1e-9 on the fused tail: the reference's step count,
    history and solution (x = x0 + yk with yk updated inside the launch)."""
    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref

    P = problems.poisson2d(120)
    b = np.random.default_rng(21).standard_normal(P.shape[0])
    _, got = krylov_amd.minres(krylov_amd.CsrOperator(P), b, tol=1e-9)
    _, ref = krylov_ref.minres(P, b, tol=1e-9)
    assert got.numsteps == ref.numsteps
    np.testing.assert_allclose(np.asarray(got.resnorms)[:-1], np.asarray(ref.resnorms)[:-1], rtol=1e-10)
    np.testing.assert_allclose(got.xk, ref.xk, rtol=0, atol=1e-9 * np.abs(ref.xk).max())


@pytest.mark.parametrize("fault_step", [0, 5])
def test_fused_tail_timeout_falls_back(fault_step, monkeypatch):
    """A block that never joins the exchange at `fault_step`: nothing was
    written, the rest of the chunk runs with the separate kernels, and the
    history and iterate equal a clean solve's to rounding."""
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(150)
    b = np.random.default_rng(22).standard_normal(P.shape[0])
    A = krylov_amd.CsrOperator(P)
    _, clean = krylov_amd.minres(A, b, tol=1e-9, maxiter=300)
    monkeypatch.setenv("KRY_MRU_FAULT", str(fault_step))
    _, faulted = krylov_amd.minres(A, b, tol=1e-9, maxiter=300)
    assert faulted.numsteps == clean.numsteps
    np.testing.assert_allclose(np.asarray(faulted.resnorms)[:-1], np.asarray(clean.resnorms)[:-1], rtol=1e-10)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=0, atol=1e-10 * np.abs(clean.xk).max())
    st = _state(A, b)
    h, _ = st.run(8)
    assert len(h) == 8 and st.update_path() == (True, 1)


@pytest.mark.parametrize("late", [1, 3, 4, 6])
def test_fused_tail_late_block_all_or_nothing(late, monkeypatch):
    """A block that joins the exchange late, about when the others' spin runs
    out (KRY_MRU_FAULT_LATE): every block commits or every block aborts
    (decide_exchange), so whichever way the race goes the history and iterate
    equal a clean solve's; a split decision would leave a partly updated step
    behind the rerun."""
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(150)
    b = np.random.default_rng(23).standard_normal(P.shape[0])
    A = krylov_amd.CsrOperator(P)
    _, clean = krylov_amd.minres(A, b, tol=1e-9, maxiter=300)
    monkeypatch.setenv("KRY_MRU_FAULT", "3")
    monkeypatch.setenv("KRY_MRU_FAULT_LATE", str(late))
    _, faulted = krylov_amd.minres(A, b, tol=1e-9, maxiter=300)
    assert faulted.numsteps == clean.numsteps
    np.testing.assert_allclose(np.asarray(faulted.resnorms)[:-1], np.asarray(clean.resnorms)[:-1], rtol=1e-10)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=0, atol=1e-10 * np.abs(clean.xk).max())
