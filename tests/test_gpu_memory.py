"""The caching device allocator (abi_core.hip, kry_mem_stats / kry_mem_release):
a second solve on the same operator reuses the first solve's freed blocks
instead of hipMalloc'ing new ones, gives bitwise the same results, and
empty_cache() returns the cached blocks to the runtime."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_repeated_solves_reuse_blocks_bitwise():
    import krylov_amd
    from krylov_amd import problems

    M = problems.stencil15_3d(24)
    A = krylov_amd.CsrOperator(M)
    b = np.ones(M.shape[0])
    x1, i1 = krylov_amd.cg(A, b, tol=1e-8)
    s1 = krylov_amd.memory_stats()
    assert s1["enabled"] == 1
    assert s1["bytes_cached"] > 0  # the first solve's state went back to the pool
    x2, i2 = krylov_amd.cg(A, b, tol=1e-8)
    s2 = krylov_amd.memory_stats()
    assert s2["device_mallocs"] == s1["device_mallocs"]  # every buffer of the second solve was a reuse
    assert s2["reuses"] > s1["reuses"]
    assert i1.numsteps == i2.numsteps
    assert np.array_equal(np.asarray(i1.resnorms), np.asarray(i2.resnorms))
    assert np.array_equal(x1, x2)
    # GMRES after CG: other sizes (the basis) are fresh, the shared ones reused
    x3, i3 = krylov_amd.gmres(A, b, tol=1e-8, maxiter=40)
    x4, i4 = krylov_amd.gmres(A, b, tol=1e-8, maxiter=40)
    assert np.array_equal(np.asarray(i3.resnorms), np.asarray(i4.resnorms))
    assert np.array_equal(x3, x4)


def test_reused_block_is_not_read_stale():
    """A reused block holds the previous owner's bytes: every solver must
    initialise what it reads (a wrong answer here means a missing memset)."""
    import krylov_amd
    from krylov_amd import problems

    M = problems.poisson2d(64)
    A = krylov_amd.CsrOperator(M)
    rng = np.random.default_rng(1)
    b1 = rng.standard_normal(M.shape[0]) * 1e6
    krylov_amd.minres(A, b1, tol=1e-10)
    krylov_amd.gmres(A, b1, tol=1e-10, maxiter=50)
    b = np.ones(M.shape[0])
    krylov_amd.empty_cache()
    ref = [krylov_amd.cg(A, b, tol=1e-8)[1], krylov_amd.gmres(A, b, tol=1e-8, maxiter=50)[1],
           krylov_amd.minres(A, b, tol=1e-8)[1]]
    # now with the pool warm from solves on a different right-hand side
    krylov_amd.cg(A, b1, tol=1e-10)
    krylov_amd.gmres(A, b1, tol=1e-10, maxiter=50)
    krylov_amd.minres(A, b1, tol=1e-10)
    again = [krylov_amd.cg(A, b, tol=1e-8)[1], krylov_amd.gmres(A, b, tol=1e-8, maxiter=50)[1],
             krylov_amd.minres(A, b, tol=1e-8)[1]]
    for r, a in zip(ref, again):
        assert r.numsteps == a.numsteps
        assert np.array_equal(np.asarray(r.resnorms), np.asarray(a.resnorms))
        assert np.array_equal(r.xk, a.xk)


def test_empty_cache_releases_blocks():
    import krylov_amd
    from krylov_amd import problems

    M = problems.poisson2d(32)
    A = krylov_amd.CsrOperator(M)
    krylov_amd.cg(A, np.ones(M.shape[0]), tol=1e-6)
    assert krylov_amd.memory_stats()["bytes_cached"] > 0
    krylov_amd.empty_cache()
    assert krylov_amd.memory_stats()["bytes_cached"] == 0
    # and the library keeps working after a release
    _, info = krylov_amd.cg(A, np.ones(M.shape[0]), tol=1e-6)
    assert info.success


def test_block_freed_with_work_in_flight_is_not_reused_early():
    """A vector freed while SpMVs that read it are still queued on one stream,
    and a block of the same size then taken on another context's stream: the
    allocator retires the freed block only after a device sync, so the queued
    SpMVs still read the old bytes (bitwise csr_matvec of the old x)."""
    import krylov_amd
    from krylov_amd import problems
    from krylov_amd.device import Context, DeviceVector, get_context

    M = problems.poisson2d(300)
    n = M.shape[0]
    ctx = get_context(0)
    A = krylov_amd.CsrOperator(M)
    x_host = np.linspace(1.0, 2.0, n).reshape(n, 1)
    ctx.synchronize()
    krylov_amd.empty_cache()  # no free block of x's size: z below can only take x's
    x = DeviceVector.from_host(ctx, x_host)
    y = DeviceVector(ctx, n, 1, np.float64)
    for _ in range(64):
        A.matvec_device(x, y)
    before = krylov_amd.memory_stats()
    x.close()  # the SpMVs above may still be queued
    other = Context(0)  # a second stream on the same device
    z = DeviceVector(other, n, 1, np.float64)
    z.upload(np.full((n, 1), -7.0))
    after = krylov_amd.memory_stats()
    assert after["reuses"] > before["reuses"]
    assert after["retire_syncs"] > before["retire_syncs"]
    assert np.array_equal(y.to_host()[:, 0], M @ x_host[:, 0])
    assert np.array_equal(z.to_host(), np.full((n, 1), -7.0))
