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


@pytest.mark.parametrize("key", ["f64_i32", "f64_i64", "f32_i32", "f32_i64"])
def test_spmv_bitwise_adversarial(golden, key):
    """Unsorted indices, duplicates, explicit zeros, empty rows, a 3000-nnz row
    (longer than one LDS tile), magnitudes 1e+-20: bitwise SciPy."""
    import krylov_amd

    d = golden["spmv"]
    A = krylov_amd.CsrOperator(_golden_csr(d, key))
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
