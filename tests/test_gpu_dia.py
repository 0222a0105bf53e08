"""The diagonal-offset image (SELL-128/DIA, kry_csr::dia_*) on the MI355X.

Structured matrices (stencils, bands) are stored as per-slice offset lists
with lane masks and no per-entry column index; each lane owns two rows and
loads its two x entries as one pair, so a hole's x entry may be loaded (at
worst one element outside x, inside the allocation slack) but is never used. The single-RHS SpMV over that
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
    assert lay["dia_slots"] <= lay["slots"] * 1.25 + 128 * 32
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


@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1000, 1001])
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


def _convdiff(m, seed=0):
    """Nonsymmetric banded operator (2-D convection-diffusion, 5-point,
    upwinded, random per-row coefficients): DIA-eligible, not symmetric."""
    rng = np.random.default_rng(seed)
    n = m * m
    main = 4.0 + rng.uniform(0.0, 1.0, n)
    east = -1.0 - rng.uniform(0.0, 0.5, n)
    west = -1.0 + rng.uniform(0.0, 0.5, n)
    east[np.arange(n) % m == m - 1] = 0.0
    west[np.arange(n) % m == 0] = 0.0
    A = scipy.sparse.diags([main, east[:-1], west[1:], np.full(n - m, -0.7), np.full(n - m, -1.2)],
                           [0, 1, -1, m, -m], format="csr")
    A.eliminate_zeros()
    A.sort_indices()
    A.indices = A.indices.astype(np.int32)
    A.indptr = A.indptr.astype(np.int32)
    return A


@pytest.mark.parametrize("solver", ["cg", "gmres", "minres", "gmres_prec", "minres_weighted", "cg_prec"])
def test_dia_solvers_match_sell_and_oracle(solver, monkeypatch):
    """Every SpMV epilogue the solvers use over the DIA image (CG Ap/<p,Ap>,
    residual, GMRES's fused normalisation source and basis store, Lanczos,
    preconditioner stores and norms, x = x0 + Mr y) inside whole solves: the
    reference's iteration count and history (oracle) with the DIA image and
    with the SELL image. The two images' SpMVs are bitwise equal; the block
    partials of the fused inner products follow each image's grid, so the
    two histories agree to rounding, not bit for bit."""
    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref

    m = 45  # n = 2025: 15 full 128-row slices and a ragged one
    if solver.startswith("cg") or solver.startswith("minres"):
        A = problems.poisson2d(m).tocsr()
    else:
        A = _convdiff(m)
    n = A.shape[0]
    b = np.random.default_rng(7).standard_normal(n)
    kw, rkw = {}, {}
    if solver.endswith("prec"):
        d = A.diagonal()
        kw["M"] = scipy.sparse.diags(1.0 / np.abs(d)).tocsr()
        if solver.startswith("gmres"):
            kw["Ml"] = scipy.sparse.diags(1.0 / np.sqrt(np.abs(d))).tocsr()
            kw["Mr"] = scipy.sparse.diags(1.0 / np.sqrt(np.abs(d))).tocsr()
        rkw = dict(kw)
    if solver == "minres_weighted":
        w = np.random.default_rng(3).uniform(1.0, 2.0, n)
        A = (scipy.sparse.diags(1.0 / w) @ A).tocsr()
        A.sort_indices()
        kw["inner"] = krylov_amd.WeightedInner(w)
        rkw["inner"] = lambda x, y: np.dot(x.T, w * y)
    name = solver.split("_")[0]
    # GMRES: one 40-step cycle; weighted MINRES: its Lanczos history is
    # chaotic in the inner products' summation order past ~60 steps (as the
    # weighted CG fixture's, DESIGN.md "Oracle and parity"), so 40 steps
    extra = {"maxiter": 40} if name == "gmres" or solver == "minres_weighted" else {}
    _, ref = getattr(krylov_ref, name)(A, b, tol=1e-9, **rkw, **extra)
    fn = getattr(krylov_amd, name)
    op = krylov_amd.CsrOperator(A)
    assert op.layout()["dia"]
    _, on = fn(op, b, tol=1e-9, **kw, **extra)
    monkeypatch.setenv("KRY_SPMV_DIA", "0")
    krylov_amd.clear_operator_cache()  # preconditioners are re-uploaded without the image too
    op0 = krylov_amd.CsrOperator(A)
    assert not op0.layout()["dia"]
    _, off = fn(op0, b, tol=1e-9, **kw, **extra)
    krylov_amd.clear_operator_cache()
    r = np.asarray(ref.resnorms)
    for got in (on, off):
        assert got.numsteps == ref.numsteps
        np.testing.assert_allclose(np.asarray(got.resnorms)[:-1], r[:-1], rtol=1e-10, atol=0)
    np.testing.assert_allclose(np.asarray(on.resnorms), np.asarray(off.resnorms), rtol=1e-12, atol=1e-14 * r[0])


@pytest.mark.parametrize("k", [2, 3, 4, 8])
@pytest.mark.parametrize("name", ["stencil15_40", "poisson2d_61", "shifted_lap3d_f32"])
def test_dia_block_spmv_bitwise(name, k, monkeypatch):
    """Block right-hand sides (n x k row-major, k padded to a power of two)
    over the DIA image: bitwise SciPy csr_matvecs, and equal to the
    lane-group SELL kernel (KRY_SPMV_DIA_BLK=0)."""
    import krylov_amd

    A = _structured()[name]
    op = krylov_amd.CsrOperator(A)
    assert op.layout()["dia"]
    rng = np.random.default_rng(k)
    X = (rng.standard_normal((A.shape[0], k)) * 10.0 ** rng.integers(-20, 20, (A.shape[0], 1))).astype(A.dtype)
    Y = op @ X
    _bits_equal(Y, A @ X)


def test_dia_block_cg_matches_lane_group_and_oracle(golden, monkeypatch):
    """Block CG (8 columns, Poisson 64^2 fixture of the reference): the DIA
    block SpMV against the lane-group SELL kernel and the reference history."""
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(64)
    B = golden["solvers"]["poisson64_B"]
    ref = golden["solvers"]["cg_poisson64_blk8_resnorms"]
    _, on = krylov_amd.cg(krylov_amd.CsrOperator(P), B, tol=1e-8)
    monkeypatch.setenv("KRY_SPMV_DIA_BLK", "0")
    _, off = krylov_amd.cg(krylov_amd.CsrOperator(P), B, tol=1e-8)
    for got in (on, off):
        assert got.numsteps == int(golden["solvers"]["cg_poisson64_blk8_numsteps"])
        np.testing.assert_allclose(np.asarray(got.resnorms)[:-1], ref[:-1], rtol=1e-10)


@pytest.mark.parametrize("D", [1, 3, 7, 15, 31])
@pytest.mark.parametrize("case", ["poisson2d_300_f64", "lap3d_f32", "poisson_weighted", "banded_general", "Ml"])
def test_block_cg_deferred_y_bitwise(case, D, monkeypatch):
    """Block CG with yk += alpha p deferred and applied D steps at a time
    (cg_pdefer_kernel, p cycling through D + 1 buffers indexed by the global
    step across chunks; the updates pending at a chunk's end applied when the
    host reads y, cg_ydefer_flush) against one update per step (KRY_CG_YDEFER=0): the same
    roundings in the same order, so the history, the iterate and the step
    count are bitwise equal, for chunks of 1, 7, 32, 1 and 19 steps (ends
    that fall before, on and after a flush), a solve stopping in the middle
    of a chunk (tol), a weighted inner product, a general (non-DIA)
    matrix and a left preconditioner Ml (cg.py:180,207: r and p carry Ml; the
    deferral only needs p_i, so it stays on)."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState

    inner = None
    Ml = None
    k = 4
    if case == "poisson2d_300_f64":
        A = problems.poisson2d(300)
        k = 8
    elif case == "lap3d_f32":
        A, _ = problems.shifted_lap3d_weighted(24)
    elif case == "banded_general":
        n = 20_000
        rng = np.random.default_rng(9)
        offs = [-301, -17, -1, 0, 1, 17, 301]
        diags = [rng.uniform(-1.0, 0.0, n - abs(o)) for o in offs]
        A = scipy.sparse.diags(diags, offs, format="csr")
        A = (A + A.T).tocsr()
        A = A + scipy.sparse.diags(np.asarray(abs(A).sum(axis=1)).ravel() + 1.0)
        A = A.tocsr()
        A.sort_indices()
        k = 2
    elif case == "Ml":
        A = problems.poisson2d(200)
        Ml = scipy.sparse.diags(1.0 / A.diagonal() * np.random.default_rng(6).uniform(0.5, 1.5, A.shape[0])).tocsr()
    else:
        A = problems.poisson2d(200)
        inner = krylov_amd.WeightedInner(np.random.default_rng(4).uniform(1.0, 2.0, A.shape[0]))
    dt = np.float32 if A.dtype == np.float32 else np.float64
    B = np.random.default_rng(k).standard_normal((A.shape[0], k)).astype(dt)
    B[:, -1] *= 1e-2  # columns converge at different steps
    op = krylov_amd.CsrOperator(A)

    def solve(d):
        monkeypatch.setenv("KRY_CG_YDEFER", str(d))
        st = _CGState(_helpers.Problem(op, B, None, inner, Ml=Ml))
        st.start()
        st.set_criterion(np.zeros(k))
        hs = [st.run(n) for n in (1, 7, 32, 1, 19)]
        assert st.defer_info()[0] == d
        h, x = np.concatenate(hs), st.get(0)
        _, info = krylov_amd.cg(op, B, Ml=Ml, inner=inner, tol=1e-6)
        return h, x, info

    h1, x1, info1 = solve(D)
    h0, x0, info0 = solve(0)
    _bits_equal(h1, h0)
    _bits_equal(x1, x0)
    assert info1.numsteps == info0.numsteps and info1.success == info0.success
    _bits_equal(np.asarray(info1.resnorms), np.asarray(info0.resnorms))
    _bits_equal(info1.xk, info0.xk)


@pytest.mark.parametrize("path", ["upd", "passes", "upd_general"])
def test_single_rhs_cg_deferred_y_bitwise(path, monkeypatch):
    """One right-hand side with yk deferred 7 steps at a time: the one-launch
    update kernel skipping y (cg_upd_kernel<..., DEF>, OpCgYSteps on every
    7th step) and the separate passes (KRY_CG_UPD=0: cg_pdefer_kernel at
    k = 1), on the DIA image and on a general matrix (paired image), against
    KRY_CG_YDEFER=0: histories, iterates and step counts bitwise equal, for
    chunks ending before, on and after a flush and a solve stopping
    mid-chunk."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState

    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    if path == "passes":
        monkeypatch.setenv("KRY_CG_UPD", "0")
    if path == "upd_general":
        monkeypatch.setenv("KRY_SPMV_DIA", "0")
    A = problems.stencil15_3d(40)
    op = krylov_amd.CsrOperator(A)
    assert op.layout()["pair"] == (path == "upd_general")
    b = np.random.default_rng(2).standard_normal(A.shape[0])

    def solve(d):
        monkeypatch.setenv("KRY_CG_YDEFER", str(d))
        st = _CGState(_helpers.Problem(op, b, None, None))
        st.start()
        st.set_criterion(np.zeros(1))
        hs = [st.run(n) for n in (1, 7, 32, 1, 19, 6)]
        upd = st.update_path()
        h, x = np.concatenate(hs), st.get(0)
        _, info = krylov_amd.cg(op, b, tol=1e-7)
        return h, x, info, upd

    h1, x1, info1, upd1 = solve(7)
    h0, x0, info0, upd0 = solve(0)
    assert upd1[0] == upd0[0] == (0 if path == "passes" else 1)
    _bits_equal(h1, h0)
    _bits_equal(x1, x0)
    assert info1.numsteps == info0.numsteps and info1.success == info0.success
    _bits_equal(np.asarray(info1.resnorms), np.asarray(info0.resnorms))
    _bits_equal(info1.xk, info0.xk)


def test_block_cg_default_ring_depth(monkeypatch):
    """The deferral policy without an override: an n x k block above 128 MB
    (Poisson 1500^2 x 8 columns, 144 MB) defers yk 15 steps at a time, its
    ring of 15 p buffers and 15 x k alphas reported by kry_cg_defer_info;
    a block below 128 MB does not defer."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState

    monkeypatch.delenv("KRY_CG_YDEFER", raising=False)
    for m, want in ((1500, 15), (1000, 0)):
        P = problems.poisson2d(m)
        B = np.random.default_rng(m).standard_normal((P.shape[0], 8))
        st = _CGState(_helpers.Problem(krylov_amd.CsrOperator(P), B, None, None))
        st.start()
        st.set_criterion(np.zeros(8))
        assert len(st.run(2)) == 2
        D, nbytes = st.defer_info()
        assert D == want
        vb = (P.shape[0] * 8 + 15) // 16 * 16 * 8
        assert nbytes == (D * vb + D * 8 * 8 if D else 0)


def _hip_free_bytes():
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
    return free.value


def test_block_cg_ring_depth_follows_free_memory(monkeypatch):
    """The default ring is sized by what is free when the solver starts
    (kry_cg_start: a quarter of it, and at most 10 GB): with a balloon
    allocated next to the solver so that about 2.5 GB stay free, the 144 MB
    block gets D = 3 (3 x 144 MB fit 625 MB, 7 x 144 MB do not) and still
    iterates bitwise as one update per step."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState
    from krylov_amd.device import DeviceVector

    monkeypatch.delenv("KRY_CG_YDEFER", raising=False)
    P = problems.poisson2d(1500)
    B = np.random.default_rng(7).standard_normal((P.shape[0], 8))
    A = krylov_amd.CsrOperator(P)

    def solve(start=True):
        st = _CGState(_helpers.Problem(A, B, None, None))
        if start:
            st.start()
            st.set_criterion(np.zeros(8))
        return st

    st = solve(start=False)
    krylov_amd.empty_cache()
    keep = int(2.5 * 2**30)
    free = _hip_free_bytes()
    assert free > keep + 2**30
    balloon = DeviceVector(A.ctx, (free - keep) // 8, 1, np.float64)
    try:
        st.start()
        st.set_criterion(np.zeros(8))
        h = st.run(12)
        D, _ = st.defer_info()
        assert D == 3
    finally:
        del balloon
        krylov_amd.empty_cache()
    monkeypatch.setenv("KRY_CG_YDEFER", "0")
    st0 = solve()
    h0 = st0.run(12)
    assert st0.defer_info()[0] == 0
    _bits_equal(np.asarray(h), np.asarray(h0))
