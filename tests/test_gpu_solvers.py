"""Solver parity on the MI355X against fixtures produced by the reference
(tests/golden/solvers.npz) and the oracle, plus the reference's own solver
tests restated for the device path (tests/test_cg.py, test_gmres.py,
test_minres.py, test_solvers.py of ju-liu/krylov)."""
import numpy as np
import pytest
import scipy.sparse

from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu

REAL_SPD_CASES = [
    H.spd_dense((5,)),
    H.spd_dense((5, 1)),
    H.spd_dense((5, 3)),
    H.spd_rhs_0((5,)),
    H.spd_rhs_0sol0(),
    H.symmetric_indefinite(),
]


@pytest.mark.parametrize("A_b", REAL_SPD_CASES)
def test_cg_reference_cases(A_b):
    import krylov_amd

    A, b = A_b
    calls = 0

    def callback(x, r):
        nonlocal calls
        calls += 1

    sol, info = krylov_amd.cg(A, b, tol=1.0e-7, callback=callback)
    assert calls == info.numsteps + 1
    assert info.success
    H.assert_consistent(A, b, info, sol, 1.0e-7)


@pytest.mark.parametrize("A_b", REAL_SPD_CASES)
def test_minres_reference_cases(A_b):
    import krylov_amd

    A, b = A_b
    calls = 0

    def callback(x, r):
        nonlocal calls
        calls += 1

    sol, info = krylov_amd.minres(A, b, tol=1.0e-7, callback=callback)
    assert calls == info.numsteps + 1
    assert info.success
    H.assert_consistent(A, b, info, sol, 1.0e-7)


@pytest.mark.parametrize("A_b", REAL_SPD_CASES + [H.real_unsymmetric()])
@pytest.mark.parametrize("ortho", ["mgs", "mgs2"])
def test_gmres_reference_cases(A_b, ortho):
    import krylov_amd

    A, b = A_b
    calls = 0

    def callback(x, r):
        nonlocal calls
        calls += 1

    sol, info = krylov_amd.gmres(A, b, tol=1.0e-7, ortho=ortho, callback=callback)
    assert calls == info.numsteps + 1
    assert info.success
    H.assert_consistent(A, b, info, sol, 1.0e-7)


@pytest.mark.parametrize("name", ["cg", "gmres", "minres"])
@pytest.mark.parametrize("shape", [(100,), (100, 1)])
def test_readme_goldens(name, shape):
    # tests/test_solvers.py:123-144 known answers
    import krylov_amd

    refs = {
        "cg": [1004.1873775173957, 1000.0003174916551, 999.9999999997555],
        "gmres": [1004.1873724888546, 1000.0003124630923, 999.999994971191],
        "minres": [1004.187372488912, 1000.0003124632159, 999.9999949713145],
    }[name]
    A = np.diag([1.0e-3] + list(range(2, 101)))
    b = np.ones(shape)
    sol, _ = getattr(krylov_amd, name)(A, b)
    assert sol.shape == b.shape
    tol = 1.0e-11
    assert abs(np.sum(np.abs(sol)) - refs[0]) < tol * refs[0]
    assert abs(np.sqrt(np.dot(sol.T, sol)).item() - refs[1]) < tol * refs[1]
    assert abs(np.max(np.abs(sol)) - refs[2]) < tol * refs[2]


@pytest.mark.parametrize("name", ["cg", "gmres", "minres"])
@pytest.mark.parametrize("shape", ["1d", "nx1"])
def test_diag100_histories(golden, name, shape):
    import krylov_amd

    A = np.diag([1.0e-3] + list(range(2, 101)))
    b = np.ones(100) if shape == "1d" else np.ones((100, 1))
    sol, info = getattr(krylov_amd, name)(A, b)
    H.assert_parity(info, golden["solvers"], f"diag100_{name}_{shape}", rtol=1e-9, xtol=1e-10)


@pytest.mark.parametrize("name", ["cg", "minres", "gmres"])
def test_weighted_inner_goldens(name):
    # tests/test_solvers.py:147-196 with inner = np.dot(x.T, w * y)
    import krylov_amd

    n = 100
    A = np.diag([1.0e-3] + list(range(2, n + 1)))
    w = 10 / np.arange(1, n + 1)
    for b in (np.ones(n), np.ones((n, 1))):
        sol, _ = getattr(krylov_amd, name)(A, b, inner=krylov_amd.WeightedInner(w))
        sol = sol.reshape(-1)
        assert abs(np.sum(np.abs(sol)) - 1004.1873775173957) < 1e-9 * 1004.1873775173957
        assert abs(np.sqrt(np.dot(sol, sol)) - 1000.0003174916551) < 1e-9 * 1000.0003174916551
        assert abs(np.max(np.abs(sol)) - 999.9999999997555) < 1e-9 * 999.9999999997555


@pytest.mark.parametrize("name", ["cg", "minres", "gmres"])
@pytest.mark.parametrize("b_shape", [(5,), (5, 1), (5, 3)])
def test_explicit_residual(name, b_shape):
    import krylov_amd

    a = np.linspace(1.0, 2.0, b_shape[0])
    a[-1] = 1e-2
    _, info = getattr(krylov_amd, name)(np.diag(a), np.ones(b_shape), tol=1.0e-7)
    assert np.all(info.resnorms[-1] < 1.0e-7)


@pytest.mark.parametrize("name", ["cg", "minres", "gmres"])
def test_exact_solution_as_initial_guess(name):
    import krylov_amd

    A = np.diag([1.0e-3] + list(range(2, 11)))
    b = np.ones(10)
    x0 = np.linalg.solve(A, b)
    sol, info = getattr(krylov_amd, name)(A, b, x0=x0)
    assert len(info.resnorms) == 1
    if name == "gmres":
        assert info.xk is x0


@pytest.mark.parametrize("name", ["cg", "minres", "gmres"])
def test_scipy_sparse_and_csr_operator(name):
    import krylov_amd

    n = 5
    a = np.linspace(1.0, 2.0, n)
    a[-1] = 1e-2
    for A in (scipy.sparse.spdiags(a, [0], n, n), krylov_amd.CsrOperator(scipy.sparse.spdiags(a, [0], n, n))):
        _, info = getattr(krylov_amd, name)(A, np.ones(n), tol=1.0e-12)
        assert info.resnorms[-1] <= 1.0e-12


def test_cg_poisson_histories(golden):
    import krylov_amd
    from krylov_amd import problems

    d = golden["solvers"]
    P = krylov_amd.CsrOperator(problems.poisson2d(64))
    n = P.shape[0]
    H.assert_parity(krylov_amd.cg(P, np.ones(n), tol=1e-8)[1], d, "cg_poisson64_1d")
    H.assert_parity(krylov_amd.cg(P, d["poisson64_B"], tol=1e-8)[1], d, "cg_poisson64_blk8")
    H.assert_parity(krylov_amd.cg(P, np.ones(n), x0=d["poisson64_x0"], tol=1e-6, maxiter=150)[1], d, "cg_poisson64_x0")
    S = problems.stencil15_3d(24)
    H.assert_parity(krylov_amd.cg(S, np.ones(S.shape[0]), tol=1e-8)[1], d, "cg_st15_24")


def test_gmres_random_histories(golden):
    import krylov_amd
    from krylov_amd import problems

    d = golden["solvers"]
    R = krylov_amd.CsrOperator(problems.random_nonsym(5000))
    for ortho in ("mgs", "mgs2"):
        info = krylov_amd.gmres(R, np.ones(5000), ortho=ortho, maxiter=30, tol=0.0)[1]
        H.assert_parity(info, d, f"gmres_rand5k_{ortho}", rtol=1e-10, xtol=1e-9)
    info = krylov_amd.gmres(R, d["rand5k_B3"], maxiter=20, tol=0.0)[1]
    H.assert_parity(info, d, "gmres_rand5k_blk3", rtol=1e-10, xtol=1e-9)


def test_minres_histories(golden):
    import krylov_amd
    from krylov_amd import problems

    d = golden["solvers"]
    P = problems.poisson2d(64)
    H.assert_parity(krylov_amd.minres(P, np.ones(P.shape[0]), tol=1e-8)[1], d, "minres_poisson64")


def test_minres_fp32_weighted(golden):
    """cfg5 pattern at 20^3: float32 operator, float64 weights (the reference
    then runs its Lanczos vectors in float64), 50 fixed iterations; fp32
    parity bar 1e-4 relative."""
    import krylov_amd
    from krylov_amd import problems

    d = golden["solvers"]
    W, w = problems.shifted_lap3d_weighted(20)
    info = krylov_amd.minres(W, np.ones(W.shape[0], dtype=np.float32), inner=krylov_amd.WeightedInner(w),
                             tol=0.0, maxiter=50)[1]
    assert info.xk.dtype == np.float32
    H.assert_parity(info, d, "minres_w20_f32", rtol=1e-4, xtol=1e-4, final_atol=1e-4 * d["minres_w20_f32_resnorms"][0])


def test_cg_weighted_histories(golden):
    """641 weighted-CG iterations on the shifted 20^3 Laplacian. This history
    is chaotic in the summation order of the inner products: the reference's
    own history moves by up to 8.7% relative late in the run when only its
    inner product's summation order changes (correctly rounded fsum; 5.6%
    pairwise, 2.0% extended precision), and by 5e-8 at step 100
    (tests/golden/selfnoise.npz, make_selfnoise.py). The device is held to
    that measured envelope: identical step count and success, every entry
    within max(1e-10, 2 x the reference's own deviation up to that step), the
    final explicit residual and the solution to the solve tolerance."""
    import krylov_amd
    from krylov_amd import problems

    d = golden["solvers"]
    W, w = problems.shifted_lap3d_weighted(20)
    info = krylov_amd.cg(W.astype(np.float64), np.ones(W.shape[0]), inner=krylov_amd.WeightedInner(w), tol=1e-8)[1]
    ref = d["cg_w20_weighted_resnorms"]
    H.assert_parity(info, d, "cg_w20_weighted", rtol=1e-10, xtol=1e-6, noise=H.selfnoise_envelope("cg_w20_weighted", ref),
                    final_atol=1e-8 * ref[0])


def test_cg_weighted_spd_histories(golden):
    """Weighted CG pinned at the 1e-10 contract (round 4): the unshifted 20^3
    Laplacian row-scaled by 1/w is positive definite in <x, y>_W, and the
    reference's history on it moves by <= 1.3e-12 when only the summation order
    of its inner product changes (selfnoise.npz, make_golden.make_weighted_spd), unlike the
    indefinite case above. 87 steps; same step count and success, every
    entry within 1e-10 relative, the solution to 1e-8."""
    import krylov_amd
    from krylov_amd import problems

    d = golden["solvers"]
    W, w = problems.shifted_lap3d_weighted(20, sigma=0.0)
    info = krylov_amd.cg(W.astype(np.float64), np.ones(W.shape[0]), inner=krylov_amd.WeightedInner(w), tol=1e-8)[1]
    ref = d["cg_w20spd_weighted_resnorms"]
    assert int(d["cg_w20spd_weighted_numsteps"]) == 87
    H.assert_parity(info, d, "cg_w20spd_weighted", rtol=1e-10, xtol=1e-8, final_atol=1e-8 * ref[0])


def _restart_dev(hist, ref):
    """Per-entry relative deviation of a chained restart history."""
    return np.abs(hist - ref) / np.abs(ref)


def test_restarted_gmres_matches_reference_chaining(golden):
    """GMRES(30) restarted by x0-chaining to 1e-8 relative, against what the
    reference itself recorded for the same chaining (tests/golden/make_golden.py,
    gmres_restart_*: gmres(R, b, x0=x, maxiter=30, tol=1e-8 ||b|| / ||b - R x||)
    until success): the same number of cycles, the whole chained history within
    1e-10 rel (each cycle's first entry is the explicit ||b - A x_c||), and the
    final iterate."""
    import krylov_amd
    from krylov_amd import problems

    d = golden["solvers"]
    R = problems.random_nonsym(5000)
    b = np.ones(5000)
    x, infos = krylov_amd.gmres_restarted(R, b, restart=30, tol=1e-8, max_cycles=20)
    hist = np.concatenate([np.asarray(i.resnorms, dtype=np.float64) for i in infos])
    ref = d["gmres_restart_hist"]
    assert len(infos) == int(d["gmres_restart_cycles"])
    assert infos[-1].success and not any(i.success for i in infos[:-1])
    assert all(i.numsteps == 30 for i in infos[:-1])
    assert hist.shape == ref.shape
    # every entry but the last within 1e-10 rel (the cycles' first entries are
    # explicit residuals ||b - A x_c|| too, at 1e-8..1e-3 of ||b||: measured
    # <= 1e-12 rel); the last one, the explicit residual at convergence
    # (~1e-8 ||b||), is cancellation-dominated and compared with the absolute
    # bound of the other parity tests, 64 eps (||b|| + ||A||_1 ||x||)
    rel = _restart_dev(hist[:-1], ref[:-1])
    normA1 = float(abs(R).sum(axis=0).max())
    bound = 64 * np.finfo(float).eps * (np.linalg.norm(b) + normA1 * np.linalg.norm(d["gmres_restart_x"]))
    fin = abs(hist[-1] - ref[-1]) / bound
    print(f"\nrestart rand5k: {len(infos)} cycles, history max rel {np.max(rel):.2e}, final explicit residual "
          f"{fin:.2e} of its bound")
    assert np.max(rel) <= 1e-10, (np.max(rel), int(np.argmax(rel)))
    assert fin <= 1.0
    xr = d["gmres_restart_x"]
    np.testing.assert_allclose(x, xr, rtol=1e-9, atol=1e-9 * np.max(np.abs(xr)))
    assert np.linalg.norm(b - R @ x) <= 1e-8 * np.linalg.norm(b)


def test_device_matches_oracle_on_metric_shape_small():
    """Same generator as the metric (15-pt stencil) at 32^3: device vs oracle."""
    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref as K

    S = problems.stencil15_3d(32)
    b = np.ones(S.shape[0])
    _, ref = K.cg(S, b, tol=1e-10)
    _, got = krylov_amd.cg(S, b, tol=1e-10)
    assert got.numsteps == ref.numsteps
    r, g = np.asarray(ref.resnorms), np.asarray(got.resnorms)
    assert np.all(np.abs(g[:-1] - r[:-1]) <= 1e-10 * np.abs(r[:-1]))


@pytest.mark.parametrize("name", ["diag_1d", "diag_blk3", "pvar16_M"])
def test_return_arnoldi(name):
    """cg(return_arnoldi=True) returns the reference's Lanczos relation
    [V, H, P] (cg.py:140-148, 218-258; tests/test_solvers.py:41-50)."""
    import os

    import scipy.sparse as sp

    import krylov_amd
    from krylov_amd import problems

    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "arnoldi.npz"))
    a = np.linspace(1.0, 2.0, 5)
    a[-1] = 1e-2
    kw = {}
    if name == "diag_1d":
        A, b = np.diag(a), np.ones(5)
    elif name == "diag_blk3":
        A, b = np.diag(a), np.ones((5, 3))
    else:
        P = problems.poisson2d(16)
        dg = P.diagonal() + np.random.default_rng(3).uniform(0.0, 1.0, P.shape[0])
        A = (P + sp.diags(dg - P.diagonal())).tocsr()
        b = np.ones(A.shape[0])
        kw["M"] = sp.diags(1.0 / dg).tocsr()
    _, info = krylov_amd.cg(A, b, tol=1.0e-7, return_arnoldi=True, **kw)
    p = f"arnoldi_{name}"
    if name.startswith("diag"):
        assert np.all(info.resnorms[-1] < 1.0e-7)  # the reference test's own check
    assert info.success == bool(d[p + "_success"])
    assert info.numsteps == int(d[p + "_numsteps"])
    V, H, Pb = info.arnoldi
    # Lanczos vectors r_k / ||r_k|| are compared where r_k is above round-off:
    # once CG has converged to machine precision (the 5 x 5 diagonal case
    # reaches r_5 ~ 1e-17), r_k is rounding noise in both runs
    res = np.asarray(d[p + "_resnorms"]).reshape(len(V), -1)
    live = np.all(res > 1e-12 * res[0], axis=1)
    for got, ref in ((np.array(V), d[p + "_V"]), (np.array(Pb), d[p + "_P"])):
        assert got.shape == ref.shape
        np.testing.assert_allclose(got[live], ref[live], rtol=1e-8, atol=1e-10 * np.abs(ref).max())
    Hg, Hr = np.asarray(H), d[p + "_H"]
    assert Hg.shape == Hr.shape
    np.testing.assert_allclose(Hg, Hr, rtol=1e-8, atol=1e-8 * np.abs(Hr).max())


@pytest.mark.parametrize("k", [1, 4])
@pytest.mark.parametrize("ortho", ["mgs", "mgs2"])
def test_gmres_persistent_mgs_matches_pass_kernels(monkeypatch, k, ortho):
    """The persistent MGS kernel (w in registers, one launch per Arnoldi step,
    granule all-gather for k = 1, counter barrier for k > 1) against the
    one-launch-per-pass MGS kernels (KRY_MGS_PERSIST=0): the same step count
    and histories to round-off (the two reduce the inner products in
    different fixed orders), and the oracle."""
    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref

    R = problems.random_nonsym(200_000)
    A = krylov_amd.CsrOperator(R)
    b = np.ones(R.shape[0]) if k == 1 else np.random.default_rng(7).standard_normal((R.shape[0], k))
    _, fast = krylov_amd.gmres(A, b, ortho=ortho, maxiter=30, tol=1e-9)
    monkeypatch.setenv("KRY_MGS_PERSIST", "0")
    _, slow = krylov_amd.gmres(A, b, ortho=ortho, maxiter=30, tol=1e-9)
    assert fast.numsteps == slow.numsteps
    f, s = np.asarray(fast.resnorms), np.asarray(slow.resnorms)
    np.testing.assert_allclose(f[:-1], s[:-1], rtol=1e-11)
    np.testing.assert_allclose(fast.xk, slow.xk, rtol=1e-9, atol=1e-12)
    if k == 1 and ortho == "mgs":
        _, ref = krylov_ref.gmres(R, b, maxiter=30, tol=1e-9)
        assert ref.numsteps == fast.numsteps
        np.testing.assert_allclose(f[:-1], np.asarray(ref.resnorms)[:-1], rtol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["wr", "dia", "sell"])
@pytest.mark.parametrize("m,dtype", [(30, np.float64), (300, np.float64), (600, np.float64), (1000, np.float64),
                                     (300, np.float32), (1000, np.float32)])
def test_cg_persistent_matches_pass_kernels(monkeypatch, m, dtype, form):
    """The persistent small-n CG loop (one launch per chunk, two in-launch
    all-gathers per iteration, KRY_CG_PERSIST=2 makes it mandatory) against
    the launch-per-pass path (KRY_CG_PERSIST=0) and the oracle: same step
    count, histories to round-off (the dot products are summed in different
    fixed orders), same iterate. m = 30 is one partly filled block, m = 1000
    the largest size it takes (4 slices per wave), m = 600 two slices per
    wave: the SpMV of an even number of slices per wave reads the DIA image
    with its values held in registers for the chunk ("wr", the default for a
    5-point matrix), or re-read every iteration ("dia", KRY_CGP_WR=0), and
    with KRY_CGP_DIA=0 the compact SELL-64 image ("sell")."""
    import krylov_amd

    monkeypatch.setenv("KRY_CGP_DIA", "0" if form == "sell" else "1")
    monkeypatch.setenv("KRY_CGP_WR", "0" if form == "dia" else "1")
    from krylov_amd import problems
    from oracle import krylov_ref

    R = problems.poisson2d(m).astype(dtype)
    A = krylov_amd.CsrOperator(R)
    b = np.random.default_rng(3).standard_normal(R.shape[0]).astype(dtype)
    tol = 1e-9 if dtype == np.float64 else 1e-4
    rt = 1e-10 if dtype == np.float64 else 1e-4
    monkeypatch.setenv("KRY_CG_PERSIST", "2")
    _, fast = krylov_amd.cg(A, b, tol=tol, maxiter=400)
    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    _, slow = krylov_amd.cg(A, b, tol=tol, maxiter=400)
    assert fast.numsteps == slow.numsteps
    f, s = np.asarray(fast.resnorms), np.asarray(slow.resnorms)
    np.testing.assert_allclose(f[:-1], s[:-1], rtol=rt)
    np.testing.assert_allclose(fast.xk, slow.xk, rtol=rt, atol=rt * np.abs(slow.xk).max())
    if m <= 300:
        _, ref = krylov_ref.cg(R, b, tol=tol, maxiter=400)
        assert ref.numsteps == fast.numsteps
        np.testing.assert_allclose(f[:-1], np.asarray(ref.resnorms)[:-1], rtol=rt)


@pytest.mark.gpu
@pytest.mark.parametrize("m", [200, 600, 1000])
def test_cg_persistent_chunk_boundaries(monkeypatch, m):
    """maxiter cut mid-chunk and a callback (one step per launch): the state
    the persistent loop leaves (y, r, p, scalars) carries across launches.
    m = 600 and 1000 take the register-resident DIA form, which stores p only
    at the end of a launch."""
    import krylov_amd
    from krylov_amd import problems

    R = problems.poisson2d(m)
    A = krylov_amd.CsrOperator(R)
    b = np.random.default_rng(4).standard_normal(R.shape[0])
    out = {}
    for mode in ("2", "0"):
        monkeypatch.setenv("KRY_CG_PERSIST", mode)
        seen = []
        _, info = krylov_amd.cg(A, b, tol=0.0, maxiter=45)
        _, info_cb = krylov_amd.cg(A, b, tol=0.0, maxiter=10, callback=lambda x, r: seen.append(float(np.linalg.norm(r))))
        out[mode] = (info, info_cb, seen)
    f, s = out["2"], out["0"]
    assert f[0].numsteps == s[0].numsteps == 45
    np.testing.assert_allclose(f[0].resnorms, s[0].resnorms, rtol=1e-10)
    np.testing.assert_allclose(f[0].xk, s[0].xk, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(f[1].resnorms, s[1].resnorms, rtol=1e-10)
    np.testing.assert_allclose(f[2], s[2], rtol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["wide_columns", "f32_matrix_f64_vectors"])
def test_cg_persistent_image_variants(monkeypatch, variant):
    """The persistent CG loop on the full SELL image (column spans beyond the
    compact image's 65534: couplings 80,000 rows apart) and on a float32
    matrix under float64 vectors: against the launch-per-pass path and the
    oracle."""
    import scipy.sparse as sp

    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref

    R = problems.poisson2d(300).tocsr()
    n = R.shape[0]
    if variant == "wide_columns":
        i = np.arange(0, n - 80_000, 7)
        C = sp.coo_matrix((np.full(i.size, -0.25), (i, i + 80_000)), shape=(n, n))
        R = (R + C + C.T + sp.identity(n) * 0.5).tocsr()
        R.sort_indices()
    else:
        R = R.astype(np.float32)
    A = krylov_amd.CsrOperator(R)
    lay = A.layout()
    assert lay["irregular"] == 0 and lay["col_blocks"] == 0
    assert lay["compact"] == (variant != "wide_columns")
    b = np.random.default_rng(5).standard_normal(n)
    monkeypatch.setenv("KRY_CG_PERSIST", "2")
    _, fast = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    _, slow = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    assert fast.numsteps == slow.numsteps
    np.testing.assert_allclose(np.asarray(fast.resnorms)[:-1], np.asarray(slow.resnorms)[:-1], rtol=1e-10)
    _, ref = krylov_ref.cg(R, b, tol=1e-9, maxiter=500)
    assert ref.numsteps == fast.numsteps
    np.testing.assert_allclose(np.asarray(fast.resnorms)[:-1], np.asarray(ref.resnorms)[:-1], rtol=1e-10)


@pytest.mark.gpu
def test_cg_preferred_chunk(monkeypatch):
    """kry_cg_preferred_chunk: 256 iterations per call on the persistent
    small-n loop, 32 on the launch-per-pass path (KRY_CG_PERSIST=0, or a
    weighted inner product)."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState

    R = problems.poisson2d(100)
    A = krylov_amd.CsrOperator(R)
    b = np.ones(R.shape[0])

    def chunk(inner=None):
        st = _CGState(_helpers.Problem(A, b, None, inner))
        st.start()
        return st.preferred_chunk()

    assert chunk() == 256
    assert chunk(krylov_amd.WeightedInner(np.full(R.shape[0], 2.0))) == 32
    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    assert chunk() == 32


@pytest.mark.parametrize("case", ["Mr", "block3", "householder", "x0", "Ml", "weighted", "callback"])
def test_restarted_gmres_variants_match_oracle_chaining(case):
    """gmres_restarted with a right preconditioner, with a 3-column block
    (per-column tol = 1e-8 ||b_c|| / ||b_c - A x_c||), with Householder
    Arnoldi, from a nonzero x0 (the first cycle's x_in), with a left
    preconditioner (criterion 1e-8 ||Ml b|| / ||Ml (b - A x_c)||), with a
    WeightedInner (both norms in <., .>_w, device kry_dot) and with a callback
    (the host download of each cycle's x_in), against the same x0-chaining of
    the oracle (restart 15), and, for every case but the callback, against the
    reference's own chain (tests/golden/make_restart_variants.py) at 1e-10."""
    import krylov_amd
    from oracle import krylov_ref as K
    from tests import solver_cases

    q = solver_cases.inputs()
    R = q["R"]
    kw, okw = {}, {}
    b = np.ones(R.shape[0])
    xo = None
    norm = lambda v: np.linalg.norm(v, axis=0)  # noqa: E731
    calls, ocalls = [], []
    if case == "Mr":
        kw = okw = {"Mr": q["RMj"]}
    elif case == "block3":
        b = np.random.default_rng(21).standard_normal((R.shape[0], 3))
    elif case == "householder":
        kw = okw = {"ortho": "householder"}
    elif case == "x0":
        xo = np.random.default_rng(22).standard_normal(R.shape[0])
        kw = {"x0": xo.copy()}
    elif case == "Ml":
        kw = okw = {"Ml": q["RMj"]}
        norm = lambda v: np.linalg.norm(q["RMj"] @ v, axis=0)  # noqa: E731
    elif case == "weighted":
        w = np.random.default_rng(23).uniform(0.5, 2.0, R.shape[0])
        kw = okw = {"inner": krylov_amd.WeightedInner(w)}
        norm = lambda v: np.sqrt(v @ (w * v))  # noqa: E731
    else:
        kw = {"callback": lambda x, r: calls.append((np.array(x, copy=True), np.array(r, dtype=np.float64)))}
        okw = {"callback": lambda x, r: ocalls.append((np.array(x, copy=True), np.array(r, dtype=np.float64)))}
    x, infos = krylov_amd.gmres_restarted(R, b, restart=15, tol=1e-8, max_cycles=12, **kw)
    # the oracle, chained the same way
    xo = np.zeros_like(b) if xo is None else xo
    bnorm = norm(b)
    hist, steps = [], []
    for _ in range(12):
        _, info = K.gmres(R, b, x0=xo, maxiter=15, tol=1e-8 * bnorm / np.maximum(norm(b - R @ xo), 1e-300), **okw)
        hist.extend(np.asarray(info.resnorms, dtype=np.float64))
        steps.append(info.numsteps)
        xo = info.xk
        if info.success:
            break
    assert [i.numsteps for i in infos] == steps
    got = np.concatenate([np.asarray(i.resnorms, dtype=np.float64) for i in infos])
    ref = np.array(hist)
    assert got.shape == ref.shape
    np.testing.assert_allclose(got[:-1], ref[:-1], rtol=1e-9)
    if case != "callback":
        # the reference's own chain (tests/golden/restart_variants.npz, made by
        # running the reference: parity pinned, not only the oracle's)
        import os

        d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "restart_variants.npz"))
        assert [i.numsteps for i in infos] == d[f"{case}_steps"].tolist()
        rref = d[f"{case}_hist"]
        assert got.shape == rref.shape
        # 1e-10 rel, with the cancellation floor of a residual recomputed from
        # x at each cycle's start (the explicit-residual bound's form,
        # 64 eps ||b||): the weighted chain's late entries differ from the
        # reference's by 1.2e-15 absolute (1.6e-10 rel at 7e-6)
        floor = 64 * np.finfo(float).eps * np.max(np.atleast_1d(bnorm))
        np.testing.assert_allclose(got[:-1], rref[:-1], rtol=1e-10, atol=floor)
        xr = d[f"{case}_x"]
        np.testing.assert_allclose(x, xr, rtol=0, atol=1e-9 * np.abs(xr).max())
        print(f"\nrestart {case}: {len(infos)} cycles, history max rel vs the reference "
              f"{np.max(np.abs(got[:-1] - rref[:-1]) / np.abs(rref[:-1])):.2e}")
    if case == "callback":
        assert len(calls) == len(ocalls) > 0
        for (gx, gr), (ox, orr) in zip(calls, ocalls):
            # the residual b - A x_c comes from cancellation against b (= ones): an absolute bound
            np.testing.assert_allclose(gr, orr, rtol=1e-8, atol=1e-12)
            np.testing.assert_allclose(gx, ox, rtol=1e-8, atol=1e-10 * max(np.abs(ox).max(), 1.0))
    np.testing.assert_allclose(x, xo, rtol=1e-8, atol=1e-10 * np.abs(xo).max())


@pytest.mark.gpu
def test_restarted_gmres_zero_cycles_returns_x0():
    """max_cycles = 0 runs no cycle: the iterate is x0 (zeros without one),
    with no Info, not None."""
    import krylov_amd
    from tests import solver_cases

    R = solver_cases.inputs()["R"]
    b = np.ones(R.shape[0])
    x, infos = krylov_amd.gmres_restarted(R, b, max_cycles=0)
    assert infos == [] and x.shape == b.shape and not np.any(x)
    x0 = np.linspace(0.0, 1.0, R.shape[0])
    x, infos = krylov_amd.gmres_restarted(R, b, x0=x0, max_cycles=0)
    assert infos == [] and np.array_equal(x, x0) and x is not x0
