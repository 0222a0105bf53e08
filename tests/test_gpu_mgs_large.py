"""The streamed persistent MGS kernel (gm_mgsl_kernel): all MGS passes of an
Arnoldi step in one launch with w held in registers and the basis streamed,
for n·k beyond the register-resident kernel's ~2.1 M doubles (up to ~10.5 M:
the BASELINE metric's GMRES(30), tests/test_gpu_fullsize_golden.py).

Its passes sum the inner products in a different grouping from the
launch-per-pass kernels, so the two paths agree to rounding; both follow the
reference's iteration (oracle) to 1e-10.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def poisson1800():
    from krylov_amd import problems

    return problems.poisson2d(1800)  # n = 3.24 M


def _state_path(A, b, sweeps):
    from krylov_amd import _helpers
    from krylov_amd.gmres import _GmresState

    st = _GmresState(_helpers.Problem(A, b, None, None), 30, sweeps)
    st.start()
    st.set_criterion(np.zeros(1 if b.ndim == 1 else b.shape[1]))
    hist, _ = st.run(4)
    assert len(hist) == 4
    return st.path()


@pytest.mark.parametrize("ortho", ["mgs", "mgs2"])
def test_streamed_mgs_matches_launch_per_pass_and_oracle(poisson1800, ortho, monkeypatch):
    import krylov_amd
    from oracle import krylov_ref

    P = poisson1800
    b = np.random.default_rng(11).standard_normal(P.shape[0])
    A = krylov_amd.CsrOperator(P)
    assert _state_path(A, b, 1 if ortho == "mgs" else 2) == (True, 0)
    _, got = krylov_amd.gmres(A, b, ortho=ortho, maxiter=30, tol=0.0)
    monkeypatch.setenv("KRY_MGS_PERSIST", "0")
    A0 = krylov_amd.CsrOperator(P)
    assert _state_path(A0, b, 1 if ortho == "mgs" else 2) == (False, 0)
    _, lpp = krylov_amd.gmres(A0, b, ortho=ortho, maxiter=30, tol=0.0)
    g, l = np.asarray(got.resnorms), np.asarray(lpp.resnorms)
    assert got.numsteps == lpp.numsteps == 30
    np.testing.assert_allclose(g[:-1], l[:-1], rtol=1e-12)
    np.testing.assert_allclose(got.xk, lpp.xk, rtol=0, atol=1e-11 * np.abs(lpp.xk).max())
    if ortho == "mgs":
        _, ref = krylov_ref.gmres(P, b, maxiter=30, tol=0.0)
        np.testing.assert_allclose(g[:-1], np.asarray(ref.resnorms)[:-1], rtol=1e-10)


def test_streamed_mgs_block_columns(monkeypatch):
    """k = 4 columns (n·k = 4 M): the counter-barrier exchange of the
    streamed kernel against the launch-per-pass path."""
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(1000)
    B = np.random.default_rng(5).standard_normal((P.shape[0], 4))
    A = krylov_amd.CsrOperator(P)
    assert _state_path(A, B, 1) == (True, 0)
    _, got = krylov_amd.gmres(A, B, maxiter=20, tol=0.0)
    monkeypatch.setenv("KRY_MGS_PERSIST", "0")
    _, lpp = krylov_amd.gmres(krylov_amd.CsrOperator(P), B, maxiter=20, tol=0.0)
    np.testing.assert_allclose(np.asarray(got.resnorms)[:-1], np.asarray(lpp.resnorms)[:-1], rtol=1e-12)
    np.testing.assert_allclose(got.xk, lpp.xk, rtol=0, atol=1e-11 * np.abs(lpp.xk).max())


def test_streamed_mgs_timeout_falls_back(poisson1800, monkeypatch):
    """A block that never joins step 2's exchange (KRY_MGS_FAULT): the step
    is rerun launch per pass and the solve matches the clean one."""
    import krylov_amd

    P = poisson1800
    b = np.ones(P.shape[0])
    A = krylov_amd.CsrOperator(P)
    _, clean = krylov_amd.gmres(A, b, maxiter=30, tol=1e-9)
    monkeypatch.setenv("KRY_MGS_FAULT", "2")
    _, faulted = krylov_amd.gmres(A, b, maxiter=30, tol=1e-9)
    assert faulted.numsteps == clean.numsteps
    f, c = np.asarray(faulted.resnorms), np.asarray(clean.resnorms)
    np.testing.assert_allclose(f[:-1], c[:-1], rtol=1e-11)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=0, atol=1e-10 * np.abs(clean.xk).max())
    assert _state_path(A, b, 1) == (False, 1)


def test_mgs_partner_two_passes_ahead_is_bitwise(monkeypatch):
    """gm_mgsp3_kernel (k = 1: the partner of pass p + 1 copied into LDS two
    passes ahead, buffer_load ... lds) performs gm_mgsp_kernel's passes and
    sums in the same order: the GMRES history, Hessenberg and iterate are
    bitwise those of KRY_MGS_PF2=0, for mgs and mgs2, and at a size whose
    last block is ragged (the copies' out-of-range rows read 0)."""
    import krylov_amd
    from krylov_amd import problems

    for n, ortho in ((200_000, "mgs"), (200_000, "mgs2"), (123_457, "mgs")):
        R = problems.random_nonsym(n)
        b = np.random.default_rng(3).standard_normal(n)
        monkeypatch.setenv("KRY_MGS_PF2", "1")
        A1 = krylov_amd.CsrOperator(R)
        assert _state_path(A1, b, 1 if ortho == "mgs" else 2) == (True, 0)
        _, i1 = krylov_amd.gmres(A1, b, ortho=ortho, maxiter=30, tol=0.0)
        monkeypatch.setenv("KRY_MGS_PF2", "0")
        _, i0 = krylov_amd.gmres(krylov_amd.CsrOperator(R), b, ortho=ortho, maxiter=30, tol=0.0)
        np.testing.assert_array_equal(np.asarray(i1.resnorms).view(np.uint8), np.asarray(i0.resnorms).view(np.uint8))
        np.testing.assert_array_equal(np.asarray(i1.xk).view(np.uint8), np.asarray(i0.xk).view(np.uint8))
