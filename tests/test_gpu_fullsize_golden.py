"""BASELINE-size parity against the REFERENCE itself.

tests/golden/fullsize.npz holds what ju-liu/krylov's own cg / gmres / minres
returned here on the BASELINE configurations (tests/golden/make_fullsize.py;
the matrices are pinned by the SHA-256s in tests/golden/problems.json):
numsteps, success, the whole residual-norm history and, for the solution,
sum|x|, ||x||, max|x| and 4096 sampled entries. The device path must give:

* the same numsteps and success flag (bit-exact iteration counts);
* every recurrence residual norm within 1e-10 rel (fp64) / 1e-4 rel (fp32),
  the north_star tolerances, except where the reference's OWN history moves
  by more than that when only the summation order of its inner product
  changes (tests/golden/selfnoise.npz: OpenBLAS 1/2/4/8 threads, pairwise,
  extended precision, fsum; the metric CG's last entries move by up to 3e-9
  rel, 1e-8 x ||r0|| below the start): there entry i may deviate by
  2 x that measured envelope (tests/gpu_helpers.selfnoise_envelope); the
  last entry is the explicit residual ||b - A x||, a cancellation-dominated
  quantity, compared with an absolute bound of 64 eps (||b|| + ||A||_1 ||x||)
  (SURVEY.md §8(c));
* the solution's summaries and samples within the drift that bound implies.

The observed worst deviations are printed (pytest -s) so the headroom under
each tolerance is on record in the GPU test log.
"""
import os

import numpy as np
import pytest

from tests import gpu_helpers as H

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

HERE = os.path.dirname(os.path.abspath(__file__))
EPS = np.finfo(np.float64).eps


@pytest.fixture(scope="module")
def full():
    return np.load(os.path.join(HERE, "golden", "fullsize.npz"))


def _sample(n, m):
    return np.sort(np.random.default_rng(12345).choice(n, m, replace=False))


def _check(info, F, prefix, A, b, rtol, xtol, noise_case=None):
    assert info.numsteps == int(F[f"{prefix}_numsteps"])
    assert bool(info.success) == bool(F[f"{prefix}_success"])
    ref = F[f"{prefix}_resnorms"]
    got = np.asarray(info.resnorms, dtype=np.float64)
    assert got.shape == ref.shape
    dev = np.abs(got[:-1] - ref[:-1]) / np.abs(ref[:-1])
    rel = np.max(dev)
    # rtol, or twice the reference's own summation-order noise at that entry
    tol = np.full(dev.shape, rtol)
    if noise_case is not None:
        tol = np.maximum(tol, H.NOISE_FACTOR * H.selfnoise_envelope(noise_case, ref))
    budget = np.max(dev / tol)
    x = np.asarray(info.xk, dtype=np.float64)
    xa = np.abs(x)
    stats = np.array([xa.sum(axis=0), np.sqrt((xa * xa).sum(axis=0)), xa.max(axis=0)])
    rstats = F[f"{prefix}_xstats"]
    normA1 = float(abs(A).sum(axis=0).max())
    bnorm = np.linalg.norm(np.asarray(b, dtype=np.float64), axis=0)
    bound = 64 * EPS * (bnorm + normA1 * rstats[1])
    fin = np.max(np.abs(got[-1] - ref[-1]) / bound)
    xs = x[_sample(x.shape[0], int(F["nsample"]))]
    xdev = np.max(np.abs(xs - F[f"{prefix}_xsample"]) / rstats[2])
    sdev = np.max(np.abs(stats - rstats) / rstats)
    print(f"\n{prefix}: numsteps {info.numsteps}, history max rel {rel:.2e} ({budget:.2f} of the per-entry "
          f"tolerance: {rtol:.0e} rel{' or 2x the reference self-noise' if noise_case else ''}), final "
          f"{fin:.2e} of the explicit-residual bound, x samples {xdev:.2e} of max|x|, x summaries {sdev:.2e} rel")
    assert budget <= 1.0
    assert fin <= 1.0
    assert xdev <= xtol and sdev <= xtol


@pytest.fixture(scope="module")
def stencil216():
    from krylov_amd import problems

    return problems.stencil15_3d(216)


def test_metric_cg_to_convergence(full, stencil216):
    """BASELINE metric (15-point 216^3, b = ones) solved to tol=1e-8, as
    measured in SURVEY §6: 363 steps."""
    import krylov_amd

    b = np.ones(stencil216.shape[0])
    _, info = krylov_amd.cg(krylov_amd.CsrOperator(stencil216), b, tol=1e-8)
    _check(info, full, "metric_cg", stencil216, b, 1e-10, 1e-8, noise_case="metric_cg")


def test_metric_gmres30(full, stencil216):
    """north_star: GMRES(30) on the metric matrix within 1e-10 rel of the
    reference residual history."""
    import krylov_amd

    b = np.ones(stencil216.shape[0])
    _, info = krylov_amd.gmres(krylov_amd.CsrOperator(stencil216), b, maxiter=30, tol=0.0)
    _check(info, full, "metric_gmres30", stencil216, b, 1e-10, 1e-9)


def test_cfg2_cg_to_convergence(full):
    """cfg2 (Poisson 1000^2) to tol=1e-8: 1853 steps on the persistent loop."""
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(1000)
    b = np.ones(P.shape[0])
    _, info = krylov_amd.cg(krylov_amd.CsrOperator(P), b, tol=1e-8)
    _check(info, full, "cfg2_cg", P, b, 1e-10, 1e-8, noise_case="cfg2_cg")


def test_cfg3_gmres30(full):
    import krylov_amd
    from krylov_amd import problems

    R = problems.random_nonsym(2_000_000)
    b = np.ones(R.shape[0])
    _, info = krylov_amd.gmres(krylov_amd.CsrOperator(R), b, maxiter=30, tol=0.0)
    _check(info, full, "cfg3_gmres30", R, b, 1e-10, 1e-9)


def test_cfg4_block_cg(full):
    """cfg4's per-GPU shard: 8 right-hand sides on Poisson 3163^2, 40 steps."""
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(3163)
    B = np.random.default_rng(0).standard_normal((P.shape[0], 8))
    _, info = krylov_amd.cg(krylov_amd.CsrOperator(P), B, tol=0.0, maxiter=40)
    _check(info, full, "cfg4_blockcg", P, B, 1e-10, 1e-9)


def test_cfg5_minres_weighted_fp32(full):
    """cfg5: fp32 shifted 3-D Laplacian 200^3, W-weighted inner, 100 steps."""
    import krylov_amd
    from krylov_amd import problems

    W, w = problems.shifted_lap3d_weighted(200)
    b = np.ones(W.shape[0], dtype=np.float32)
    _, info = krylov_amd.minres(krylov_amd.CsrOperator(W), b, inner=krylov_amd.WeightedInner(w), tol=0.0,
                                maxiter=100)
    # fp32 contract: 1e-4 rel over the whole history, the explicit final entry included
    ref = full["cfg5_minres_resnorms"]
    got = np.asarray(info.resnorms, dtype=np.float64)
    assert info.numsteps == int(full["cfg5_minres_numsteps"]) and got.shape == ref.shape
    rel = np.max(np.abs(got - ref) / np.abs(ref))
    xs = np.asarray(info.xk)[_sample(W.shape[0], int(full["nsample"]))]
    xdev = np.max(np.abs(xs.astype(np.float64) - full["cfg5_minres_xsample"]) / full["cfg5_minres_xstats"][2])
    print(f"\ncfg5_minres: history max rel {rel:.2e} (tol 1e-4), x samples {xdev:.2e} of max|x|")
    assert rel <= 1e-4
    assert xdev <= 1e-4


def _check_restart(F, prefix, A, b, max_cycles, xtol):
    """x0-chained GMRES(30) (krylov_amd.gmres_restarted, the chaining of
    make_fullsize.restart_chain) against the reference's own chained run:
    the same cycles with the same step counts and success flags, every entry
    of the chained history within 1e-10 rel (each cycle starts from the
    explicit residual ||b - A x_c||; the very last entry of a converged run is
    the explicit residual at convergence, compared with the absolute bound
    64 eps (||b|| + ||A||_1 ||x||)), and the iterate's samples / summaries."""
    import krylov_amd

    x, infos = krylov_amd.gmres_restarted(krylov_amd.CsrOperator(A), b, restart=30, tol=1e-8, max_cycles=max_cycles)
    steps = np.array([i.numsteps for i in infos])
    succ = np.array([bool(i.success) for i in infos])
    np.testing.assert_array_equal(steps, F[f"{prefix}_cycle_steps"])
    np.testing.assert_array_equal(succ, F[f"{prefix}_cycle_success"])
    hist = np.concatenate([np.asarray(i.resnorms, dtype=np.float64) for i in infos])
    ref = F[f"{prefix}_hist"]
    assert hist.shape == ref.shape
    last_explicit = bool(succ[-1])
    body = slice(0, len(ref) - 1) if last_explicit else slice(0, len(ref))
    rel = np.max(np.abs(hist[body] - ref[body]) / np.abs(ref[body]))
    rstats = F[f"{prefix}_xstats"]
    fin = 0.0
    if last_explicit:
        normA1 = float(abs(A).sum(axis=0).max())
        bound = 64 * EPS * (np.linalg.norm(b) + normA1 * rstats[1])
        fin = abs(hist[-1] - ref[-1]) / bound
    xa = np.abs(np.asarray(x, dtype=np.float64))
    stats = np.array([xa.sum(), np.sqrt((xa * xa).sum()), xa.max()])
    xs = np.asarray(x)[_sample(len(b), int(F["nsample"]))]
    xdev = np.max(np.abs(xs - F[f"{prefix}_xsample"]) / rstats[2])
    sdev = np.max(np.abs(stats - rstats) / rstats)
    print(f"\n{prefix}: {len(infos)} cycles {steps.tolist()}, chained history max rel {rel:.2e}, final explicit "
          f"{fin:.2e} of its bound, x samples {xdev:.2e} of max|x|, x summaries {sdev:.2e} rel")
    assert rel <= 1e-10
    assert fin <= 1.0
    assert xdev <= xtol and sdev <= xtol


def test_metric_gmres30_restarted(full, stencil216):
    """north_star: GMRES(30) on the metric matrix, restarted through x0 as the
    reference is driven (10 cycles of the 1e-8 chaining: 300 Arnoldi steps,
    residual 3175 -> 337), against the reference's own chained history."""
    b = np.ones(stencil216.shape[0])
    _check_restart(full, "metric_gmres30_restart", stencil216, b, 10, 1e-9)


def test_cfg3_gmres30_restarted_to_convergence(full):
    """cfg3: GMRES restart=30 converging to 1e-8 relative (2 cycles, 30 + 26
    steps), against the reference's own chained run."""
    from krylov_amd import problems

    R = problems.random_nonsym(2_000_000)
    _check_restart(full, "cfg3_gmres30_restart", R, np.ones(R.shape[0]), 20, 1e-9)
