"""Kernel-level parity on the MI355X: SpMV bitwise vs SciPy csr_matvec(s),
lartg bitwise vs LAPACK, dot/axpy vs the NumPy expressions they replace."""
import numpy as np
import pytest
import scipy.sparse

pytestmark = pytest.mark.gpu


def _golden_csr(d, key):
    n = d[f"{key}_indptr"].shape[0] - 1
    A = scipy.sparse.csr_matrix((d[f"{key}_data"], d[f"{key}_indices"], d[f"{key}_indptr"]), shape=(n, n))
    A.indices = d[f"{key}_indices"]
    A.indptr = d[f"{key}_indptr"]
    return A


@pytest.mark.parametrize("compact", ["1", "0"])
@pytest.mark.parametrize("key", ["f64_i32", "f64_i64", "f32_i32", "f32_i64"])
def test_spmv_bitwise_adversarial(golden, key, compact, monkeypatch):
    """Unsorted indices, duplicates, explicit zeros, empty rows, a 3000-nnz row
    (an irregular slice), magnitudes 1e+-20: bitwise SciPy, with the column
    indices stored as int32 and as compact uint16 deltas."""
    import krylov_amd

    monkeypatch.setenv("KRY_SELL_COMPACT", compact)
    d = golden["spmv"]
    A = krylov_amd.CsrOperator(_golden_csr(d, key))
    assert A.layout()["compact"] == (compact == "1")  # indices fit int32: CsrOperator passes int32
    y = A @ d[f"{key}_x"]
    np.testing.assert_array_equal(y.view(np.uint8), d[f"{key}_y"].view(np.uint8))
    Y = A @ d[f"{key}_X"]  # row-major block, csr_matvecs semantics
    np.testing.assert_array_equal(Y.view(np.uint8), d[f"{key}_Y"].view(np.uint8))


@pytest.mark.parametrize("k", [1, 2, 3, 4, 8, 16, 64])
def test_spmv_block_widths(k):
    import krylov_amd
    from krylov_amd import problems

    A = problems.random_nonsym(3000, seed=3)
    X = np.random.default_rng(k).standard_normal((3000, k))
    got = krylov_amd.CsrOperator(A) @ X
    np.testing.assert_array_equal(got, A @ X)


@pytest.mark.parametrize("key", ["f64_i64", "f32_i64"])
def test_spmv_int64_image_through_abi(golden, key):
    """int64 indices handed straight to kry_csr_create keep an int64 image
    (never compact) and stay bitwise."""
    import ctypes

    from krylov_amd import _lib
    from krylov_amd.device import DeviceVector, get_context

    d = golden["spmv"]
    ctx = get_context()
    ip, ix = d[f"{key}_indptr"].astype(np.int64), d[f"{key}_indices"].astype(np.int64)
    dv = np.ascontiguousarray(d[f"{key}_data"])
    n = ip.shape[0] - 1
    h = ctypes.c_void_p()
    _lib.check(_lib.lib.kry_csr_create(ctx.handle, n, ix.shape[0], _lib.ptr(ip), _lib.ptr(ix), _lib.ptr(dv),
                                       _lib.dtype_code(dv.dtype), _lib.KRY_I64, ctypes.byref(h)))
    try:
        info = np.zeros(7, dtype=np.int64)
        _lib.check(_lib.lib.kry_csr_info_n(h, info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), 7))
        assert info[3] == 0
        # the version-100 entry point writes its five values and nothing past them
        info5 = np.full(8, -7, dtype=np.int64)
        _lib.check(_lib.lib.kry_csr_info(h, info5.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        np.testing.assert_array_equal(info5[:5], info[:5])
        assert np.all(info5[5:] == -7)
        x = DeviceVector.from_host(ctx, d[f"{key}_x"])
        y = DeviceVector(ctx, n, 1, dv.dtype)
        _lib.check(_lib.lib.kry_spmv(ctx.handle, h, x.handle, y.handle))
        got = y.to_host().reshape(-1)
        np.testing.assert_array_equal(got.view(np.uint8), d[f"{key}_y"].view(np.uint8))
    finally:
        _lib.lib.kry_csr_destroy(h)


def test_compact_image_selection():
    """Stencils and bands get the compact image; a random sparsity pattern
    (slot columns spanning more than 65534 columns) keeps int32 indices; the
    two images give the same bits."""
    import krylov_amd
    from krylov_amd import problems

    S = problems.stencil15_3d(40)
    assert krylov_amd.CsrOperator(S).layout()["compact"]
    R = problems.random_nonsym(200_000, seed=1)
    assert not krylov_amd.CsrOperator(R).layout()["compact"]
    x = np.random.default_rng(0).standard_normal(S.shape[0])
    np.testing.assert_array_equal(krylov_amd.CsrOperator(S) @ x, S @ x)


def test_compact_boundary_spread(monkeypatch):
    """Slot columns spanning exactly 65534 columns are compact, 65535 are not."""
    import krylov_amd

    n = 70_000
    for span, expect in ((65534, True), (65535, False)):
        rows = np.arange(64)
        cols = np.where(rows == 0, span, 0).astype(np.int32)  # slot column 0 spans [0, span]
        A = scipy.sparse.csr_matrix((np.arange(1.0, 65.0), (rows, cols)), shape=(n, n))
        op = krylov_amd.CsrOperator(A)
        assert op.layout()["compact"] == expect
        x = np.random.default_rng(span).standard_normal(n)
        np.testing.assert_array_equal(op @ x, A @ x)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sell64_k1_regular_compact_bitwise(monkeypatch, dtype):
    """SELL-64 at k = 1 on a compact image of regular slices (no DIA image):
    rows of 0-16 banded entries, an empty slice, a 16-wide slice, a partial
    last slice; bitwise SciPy csr_matvec. (The solvers on this path:
    tests/test_gpu_dia.py with KRY_SPMV_DIA=0 and KRY_SPMV_PAIR=0.)"""
    import krylov_amd

    monkeypatch.setenv("KRY_SPMV_DIA", "0")
    monkeypatch.setenv("KRY_SPMV_PAIR", "0")
    rng = np.random.default_rng(7)
    n = 64 * 37 + 5
    lens = rng.integers(0, 17, n)
    lens[64:128] = 0  # an empty slice
    lens[128:192] = 16  # a full-width slice
    rows, cols = [], []
    for i in range(n):
        c = np.unique(rng.integers(max(0, i - 400), min(n, i + 400), lens[i]))
        rows.append(np.full(c.shape[0], i))
        cols.append(c)
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    vals = rng.standard_normal(rows.shape[0]).astype(dtype)
    A = scipy.sparse.csr_matrix((vals, (rows, cols)), shape=(n, n))
    A.sort_indices()
    op = krylov_amd.CsrOperator(A)
    lay = op.layout()
    assert lay["compact"] and not lay["dia"] and lay["irregular"] == 0 and lay["col_blocks"] == 0
    assert not lay["pair"]
    x = rng.standard_normal(n).astype(dtype)
    np.testing.assert_array_equal(np.asarray(op @ x).view(np.uint8), (A @ x).view(np.uint8))


def _pair_adversarial(dtype, seed=11):
    """A general CSR for the paired-row SELL-128 image: n not a multiple of
    128 or of 2, rows of 0-20 entries, an empty slice, unsorted rows,
    duplicate and explicit-zero entries, values and x spanning 1e+-20
    (1e+-8 in float32, where products stay finite); even
    rows 2l and odd rows 2l + 1 share their offsets in some slices (one 16-B
    x load serves both) and not in others (the second load)."""
    rng = np.random.default_rng(seed)
    n = 128 * 29 + 67
    lens = rng.integers(0, 21, n)
    lens[128:256] = 0  # an empty slice
    rows, cols = [], []
    for i in range(n):
        if (i // 128) % 3 == 0:  # stencil-like: pairs of rows share offsets
            offs = np.sort(rng.choice(np.arange(-900, 900), lens[i - (i & 1)], replace=False))
            c = np.clip(i + offs, 0, n - 1)[: lens[i]]
        else:
            c = rng.integers(max(0, i - 3000), min(n, i + 3000), lens[i])
            if i % 5 == 0:
                c = np.sort(c)
        if i % 7 == 0 and c.shape[0] > 1:
            c[-1] = c[0]  # a duplicate (kept, added twice as csr_matvec does)
        rows.append(np.full(c.shape[0], i))
        cols.append(c)
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    e = 20 if dtype == np.float64 else 8
    vals = (rng.standard_normal(rows.shape[0]) * 10.0 ** rng.integers(-e, e, rows.shape[0])).astype(dtype)
    vals[::17] = 0.0  # explicit zeros
    indptr = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=n))]).astype(np.int32)
    A = scipy.sparse.csr_matrix((vals, cols.astype(np.int32), indptr), shape=(n, n))  # stored order kept
    x = (rng.standard_normal(n) * 10.0 ** rng.integers(-e, e, n)).astype(dtype)
    return A, x


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_pair_image_bitwise_adversarial(dtype):
    """The paired-row SELL-128 kernel (general CSR, k = 1): bitwise SciPy
    csr_matvec on unsorted rows, duplicates, explicit zeros, empty and
    partial slices, paired and unpaired x loads; block RHS on the same
    operator stay on SELL-64 and bitwise csr_matvecs."""
    import krylov_amd

    A, x = _pair_adversarial(dtype)
    assert not A.has_sorted_indices
    op = krylov_amd.CsrOperator(A)
    lay = op.layout()
    assert lay["pair"] and not lay["dia"] and lay["col_blocks"] == 0
    assert lay["pair_slots"] % 128 == 0 and lay["pair_slots"] <= 1.25 * lay["slots"] + 4 * 128 * 20
    np.testing.assert_array_equal(np.asarray(op @ x).view(np.uint8), (A @ x).view(np.uint8))
    X = np.stack([x, x[::-1].copy()], axis=1)
    np.testing.assert_array_equal(np.asarray(op @ X).view(np.uint8), (A @ X).view(np.uint8))


def test_pair_image_unreferenced_nan_never_added():
    """x entries no row references hold NaN: the paired 16-B load reads the
    neighbour of a column without using it, and padding slots are dropped by
    a select, so y stays finite and bitwise."""
    import krylov_amd

    A, x = _pair_adversarial(np.float64, seed=5)
    used = np.zeros(A.shape[0], dtype=bool)
    used[A.indices] = True
    x = x.copy()
    x[~used] = np.nan
    assert (~used).sum() > 0
    op = krylov_amd.CsrOperator(A)
    assert op.layout()["pair"]
    y = op @ x
    ref = A @ x
    assert np.isfinite(ref).all()
    np.testing.assert_array_equal(y.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_pair_image_int64_through_abi(dtype):
    """int64 indices handed straight to kry_csr_create get the paired image
    too (the deltas are relative; n < 2^31) and stay bitwise."""
    import ctypes

    from krylov_amd import _lib
    from krylov_amd.device import DeviceVector, get_context

    A, x = _pair_adversarial(dtype, seed=3)
    ctx = get_context()
    ip, ix = A.indptr.astype(np.int64), A.indices.astype(np.int64)
    dv = np.ascontiguousarray(A.data)
    n = A.shape[0]
    h = ctypes.c_void_p()
    _lib.check(_lib.lib.kry_csr_create(ctx.handle, n, ix.shape[0], _lib.ptr(ip), _lib.ptr(ix), _lib.ptr(dv),
                                       _lib.dtype_code(dv.dtype), _lib.KRY_I64, ctypes.byref(h)))
    try:
        info = np.zeros(9, dtype=np.int64)
        _lib.check(_lib.lib.kry_csr_info_n(h, info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), 9))
        assert info[7] == 1 and info[3] == 0
        xv = DeviceVector.from_host(ctx, x)
        y = DeviceVector(ctx, n, 1, dv.dtype)
        _lib.check(_lib.lib.kry_spmv(ctx.handle, h, xv.handle, y.handle))
        got = y.to_host().reshape(-1)
        np.testing.assert_array_equal(got.view(np.uint8), (A @ x).view(np.uint8))
    finally:
        _lib.lib.kry_csr_destroy(h)


def test_pair_image_selection(monkeypatch):
    """Stencils keep the DIA image, cfg3-like scattered matrices the
    column-blocked one, random patterns whose slot columns span more than
    65534 columns keep SELL-64; KRY_SPMV_PAIR=0 disables the paired image
    and both images give the same bits."""
    import krylov_amd
    from krylov_amd import problems

    S = problems.stencil15_3d(24)
    lay = krylov_amd.CsrOperator(S).layout()
    assert lay["dia"] and not lay["pair"]
    R = problems.random_nonsym(200_000, seed=1)
    assert not krylov_amd.CsrOperator(R).layout()["pair"]
    monkeypatch.setenv("KRY_SPMV_DIA", "0")
    x = np.random.default_rng(0).standard_normal(S.shape[0])
    op = krylov_amd.CsrOperator(S)
    assert op.layout()["pair"]
    y = op @ x
    monkeypatch.setenv("KRY_SPMV_PAIR", "0")
    op0 = krylov_amd.CsrOperator(S)
    assert not op0.layout()["pair"]
    np.testing.assert_array_equal(op0 @ x, y)
    np.testing.assert_array_equal(y, S @ x)


def _scattered_csr(n, lens, seed, sort=True, dtype=np.float64):
    """CSR with lens[i] uniform random columns in row i (scattered sparsity)."""
    rng = np.random.default_rng(seed)
    lens = np.asarray(lens, dtype=np.int64)
    indptr = np.concatenate([[0], np.cumsum(lens)])
    rows = np.repeat(np.arange(n), lens)
    cols = rng.integers(0, n, indptr[-1])
    if sort:
        order = np.lexsort((cols, rows))
        cols = cols[order]
    vals = rng.standard_normal(indptr[-1]).astype(dtype)
    A = scipy.sparse.csr_matrix((vals, cols.astype(np.int32), indptr.astype(np.int32)), shape=(n, n))
    return A


def test_column_blocked_cfg3_bitwise(monkeypatch):
    """cfg3's scattered matrix gets the column-blocked image (8 blocks of
    262144 columns); it and the SELL image both give SciPy's bits."""
    import krylov_amd
    from krylov_amd import problems

    R = problems.random_nonsym(2_000_000)
    x = np.random.default_rng(5).standard_normal(R.shape[0])
    ref = R @ x
    A = krylov_amd.CsrOperator(R)
    assert A.layout()["col_blocks"] == 8
    np.testing.assert_array_equal(A @ x, ref)
    monkeypatch.setenv("KRY_SPMV_CB", "0")
    A0 = krylov_amd.CsrOperator(R)
    assert A0.layout()["col_blocks"] == 0
    np.testing.assert_array_equal(A0 @ x, ref)


def test_column_blocked_long_segments_and_empty_rows():
    """Segments longer than one LDS chunk (rows of 150 entries in the first
    groups), empty rows, a ragged last group, float32 data."""
    import krylov_amd

    n = 1_200_003
    lens = np.full(n, 6)
    lens[:700] = 150
    lens[1000:1300] = 0
    for dt in (np.float64, np.float32):
        A = _scattered_csr(n, lens, seed=11, dtype=dt)
        op = krylov_amd.CsrOperator(A)
        assert op.layout()["col_blocks"] == 5
        x = np.random.default_rng(3).standard_normal(n).astype(dt)
        np.testing.assert_array_equal(op @ x, A @ x)
        x64 = np.random.default_rng(4).standard_normal(n)
        np.testing.assert_array_equal(op @ x64, A @ x64)  # float32 matrix, float64 vector


def test_column_blocked_multipass_for_large_n():
    """Past 16 groups per persistent block (n > 4,194,304) the column-blocked
    SpMV runs one launch per column block, with running sums in HBM."""
    import krylov_amd

    n = 4_300_001
    A = _scattered_csr(n, np.full(n, 4), seed=13)
    op = krylov_amd.CsrOperator(A)
    assert op.layout()["col_blocks"] == 16
    x = np.random.default_rng(6).standard_normal(n)
    np.testing.assert_array_equal(op @ x, A @ x)


def test_column_blocked_not_built_for_unsorted_rows():
    import krylov_amd

    n = 1_200_000
    A = _scattered_csr(n, np.full(n, 6), seed=2, sort=False)
    op = krylov_amd.CsrOperator(A)
    assert op.layout()["col_blocks"] == 0
    x = np.random.default_rng(1).standard_normal(n)
    np.testing.assert_array_equal(op @ x, A @ x)


def test_spmv_mixed_f32_matrix_f64_vector():
    import krylov_amd
    from krylov_amd import problems

    W, _ = problems.shifted_lap3d_weighted(12)
    x = np.random.default_rng(0).standard_normal(W.shape[0])
    got = krylov_amd.CsrOperator(W) @ x  # float32 matrix, float64 vector
    np.testing.assert_array_equal(got, W @ x)  # SciPy upcasts the data


def test_spmv_empty_and_tiny():
    import krylov_amd

    A = scipy.sparse.csr_matrix((7, 7))
    np.testing.assert_array_equal(krylov_amd.CsrOperator(A) @ np.ones(7), np.zeros(7))
    A1 = scipy.sparse.csr_matrix(np.array([[2.0]]))
    np.testing.assert_array_equal(krylov_amd.CsrOperator(A1) @ np.array([3.0]), [6.0])


def test_lartg_bitwise(golden):
    import krylov_amd

    d = golden["lartg"]
    c, s, r = krylov_amd.lartg(d["fg"][:, 0].copy(), d["fg"][:, 1].copy())
    np.testing.assert_array_equal(np.stack([c, s, r], 1).view(np.uint64), d["d"].view(np.uint64))
    c, s, r = krylov_amd.lartg(d["fg32"][:, 0].copy(), d["fg32"][:, 1].copy())
    np.testing.assert_array_equal(np.stack([c, s, r], 1).view(np.uint32), d["s"].view(np.uint32))
    G, rr = krylov_amd.givens(d["fg"].T.copy())
    np.testing.assert_array_equal(G, d["givens_G"])
    np.testing.assert_array_equal(rr, d["givens_r"])


@pytest.mark.parametrize("a,b", [(0.0, 0.0), (1.0, 0.0), (0.0, 1.0), (1e8, 1e-8), (1e-8, 1e8), (3.0, -4.0)])
def test_givens_reference_properties(a, b):
    # tests/test_givens.py:11-25 (real factors)
    import krylov_amd

    x = np.array([a, b])
    G, _ = krylov_amd.givens(x)
    assert np.linalg.norm(np.eye(2) - G.T @ G, 2) <= 1e-14
    y = G @ x
    ref = np.linalg.norm(x, 2)
    assert abs(ref - abs(y[0])) <= 1e-14 * ref
    assert abs(y[1]) <= 1e-14 * ref


def test_dot_and_axpy():
    import ctypes

    from krylov_amd import _lib
    from krylov_amd.device import DeviceVector, get_context

    ctx = get_context()
    rng = np.random.default_rng(0)
    for n, k in [(1, 1), (1001, 1), (100003, 1), (5003, 4)]:
        x, y = rng.standard_normal((n, k)), rng.standard_normal((n, k))
        w = rng.uniform(1, 2, n)
        xv, yv = DeviceVector.from_host(ctx, x), DeviceVector.from_host(ctx, y)
        wv = DeviceVector.from_host(ctx, w[:, None])
        out = np.zeros(k)
        _lib.check(_lib.lib.kry_dot(ctx.handle, xv.handle, yv.handle, None, _lib.dptr(out)))
        np.testing.assert_allclose(out, np.einsum("ij,ij->j", x, y), rtol=1e-12, atol=1e-12)
        _lib.check(_lib.lib.kry_dot(ctx.handle, xv.handle, yv.handle, wv.handle, _lib.dptr(out)))
        np.testing.assert_allclose(out, np.einsum("ij,ij->j", x, w[:, None] * y), rtol=1e-12, atol=1e-12)
        alpha = rng.standard_normal(k)
        _lib.check(_lib.lib.kry_axpy(ctx.handle, _lib.dptr(alpha), xv.handle, yv.handle))
        got = yv.to_host()
        np.testing.assert_array_equal(got, y + alpha * x)  # bitwise: y += alpha * x


def test_dot_is_deterministic():
    from krylov_amd import _lib
    from krylov_amd.device import DeviceVector, get_context

    ctx = get_context()
    x = np.random.default_rng(1).standard_normal((1_000_003, 1))
    xv = DeviceVector.from_host(ctx, x)
    vals = set()
    for _ in range(5):
        out = np.zeros(1)
        _lib.check(_lib.lib.kry_dot(ctx.handle, xv.handle, xv.handle, None, _lib.dptr(out)))
        vals.add(out[0])
    assert len(vals) == 1


@pytest.mark.slow
def test_spmv_metric_matrix_bitwise():
    """Full BASELINE size (15-pt 216^3, nnz = 149,770,936): bitwise SciPy."""
    import krylov_amd
    from krylov_amd import problems

    A = problems.stencil15_3d(216)
    x = np.random.default_rng(0).standard_normal(A.shape[0])
    got = krylov_amd.CsrOperator(A) @ x
    np.testing.assert_array_equal(got, A @ x)


def test_operator_upload_cache():
    """a scipy matrix passed again is not re-uploaded;
    an in-place change of its values is detected and re-uploaded."""
    import krylov_amd
    from krylov_amd import problems

    krylov_amd.clear_operator_cache()
    A = problems.poisson2d(40)
    b = np.ones(A.shape[0])
    op1 = krylov_amd.as_device_operator(A)
    assert krylov_amd.as_device_operator(A) is op1
    _, i1 = krylov_amd.cg(A, b, tol=1e-10)
    assert krylov_amd.as_device_operator(A) is op1
    A.data *= 2.0  # in place: the fingerprint changes
    op2 = krylov_amd.as_device_operator(A)
    assert op2 is not op1
    _, i2 = krylov_amd.cg(A, b, tol=1e-10)
    assert i2.numsteps == i1.numsteps
    np.testing.assert_allclose(np.asarray(i2.resnorms[:-1]), np.asarray(i1.resnorms[:-1]), rtol=1e-10)
    B = A.copy()
    assert krylov_amd.as_device_operator(B) is not op2  # another object: its own upload
    krylov_amd.clear_operator_cache()


@pytest.mark.parametrize("m,k", [(1, 1), (5, 3), (30, 1), (64, 4), (90, 2)])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_multi_solve_triangular(m, k, dtype):
    """gmres.py:24-38 on the device against scipy.linalg.solve_triangular per
    column (the reference's own loop); zero right-hand sides give zeros."""
    import scipy.linalg

    import krylov_amd

    rng = np.random.default_rng(m * 10 + k)
    R = np.triu(rng.standard_normal((m, m, k)).transpose(2, 0, 1)).transpose(1, 2, 0).astype(dtype)
    for c in range(k):
        R[np.arange(m), np.arange(m), c] += np.sign(R[np.arange(m), np.arange(m), c]) * 3.0
    y = rng.standard_normal((m, k)).astype(dtype)
    if k > 1:
        y[:, 1] = 0.0
    got = krylov_amd.multi_solve_triangular(R, y)
    ref = np.array([np.zeros(m) if np.all(y[:, c] == 0) else scipy.linalg.solve_triangular(R[:, :, c], y[:, c])
                    for c in range(k)]).T
    assert got.shape == ref.shape and got.dtype == ref.dtype
    tol = 1e-12 if dtype == np.float64 else 1e-4
    np.testing.assert_allclose(got, ref, rtol=tol, atol=tol * np.abs(ref).max())
    if k > 1:
        assert np.all(got[:, 1] == 0.0)


def test_multi_solve_triangular_errors():
    import krylov_amd

    R = np.triu(np.ones((4, 4, 1)).transpose(2, 0, 1)).transpose(1, 2, 0)
    y = np.ones((4, 1))
    bad = R.copy()
    bad[2, 2, 0] = 0.0
    with pytest.raises(np.linalg.LinAlgError):
        krylov_amd.multi_solve_triangular(bad, y)
    nan = R.copy()
    nan[0, 3, 0] = np.nan
    with pytest.raises(ValueError):
        krylov_amd.multi_solve_triangular(nan, y)
    np.testing.assert_array_equal(krylov_amd.multi_solve_triangular(bad, np.zeros((4, 1))), np.zeros((4, 1)))


def test_host_transfers_pinned_in_place_and_fallback():
    """Large host <-> device copies go through the caller's pages pinned in
    place (host_xfer: hipHostRegister for the copy, then unregistered).
    Round trips are bitwise for a pageable array, a view that starts inside
    a page, an array that is already page-locked (hipHostMalloc:
    registration fails, the plain copy runs), and a read-only array; the
    same host array can be copied again afterwards (it was unregistered)."""
    import ctypes

    import krylov_amd
    from krylov_amd.device import DeviceVector

    ctx = krylov_amd.CsrOperator(scipy.sparse.identity(8, format="csr")).ctx
    n = 1_000_003  # 8 MB: above the 4 MB pinning threshold
    rng = np.random.default_rng(5)
    base = rng.standard_normal(n + 3)
    # page-locked host memory from the HIP runtime the library itself uses
    hip = ctypes.CDLL("libamdhip64.so.7")  # the soname the library links (not torch's bundled copy)
    hp = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(n * 8), ctypes.c_uint(0)) == 0
    pinned = np.ctypeslib.as_array(ctypes.cast(hp, ctypes.POINTER(ctypes.c_double)), shape=(n,))
    pinned[:] = rng.standard_normal(n)
    ro = rng.standard_normal(n)
    ro.setflags(write=False)
    for src in (base[:n].copy(), base[3:], pinned, ro):
        v = DeviceVector(ctx, n, 1, np.float64)
        v.upload(src.reshape(n, 1))
        out = np.empty((n, 1))
        v.to_host(out)
        np.testing.assert_array_equal(out[:, 0].view(np.uint64), np.ascontiguousarray(src).view(np.uint64))
        v.upload(src.reshape(n, 1))  # again: the pages were unregistered after the first copy
        back = np.full((n, 1), np.nan)
        v.to_host(back)
        np.testing.assert_array_equal(back.view(np.uint64), out.view(np.uint64))
    del pinned
    hip.hipHostFree(hp)


def test_host_transfers_concurrent_same_and_overlapping_arrays():
    """Threads copying the same host array (the devices=[...] driver uploads
    one CSR to every device at once) share one page-lock; a range overlapping
    one in flight waits for its release. Four contexts on device 0, each
    driven by its own thread, upload and download the same array and two
    overlapping views of it, several times: every round trip is bitwise."""
    import threading

    from krylov_amd.device import Context, DeviceVector

    n = 2_000_000  # 16 MB
    src = np.random.default_rng(9).standard_normal(n + 8)
    views = [src[:n], src[:n], src[4:n + 4], src[8:n + 8]]
    errs = []

    def work(t):
        try:
            ctx = Context(0)
            for _ in range(5):
                v = DeviceVector(ctx, n, 1, np.float64)
                v.upload(views[t].reshape(n, 1))
                out = np.empty((n, 1))
                v.to_host(out)
                assert np.array_equal(out[:, 0].view(np.uint64), views[t].view(np.uint64))
                v.close()
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
