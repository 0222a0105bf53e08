"""Timeout path of the persistent kernels (fault injection).

The persistent CG loop and the persistent MGS kernel exchange partial sums
between blocks inside one launch, so they need every block resident. A block
that never becomes resident (CUs held by another stream or process) makes the
others' bounded spins time out. These tests force that with
KRY_CGP_FAULT / KRY_MGS_FAULT (the last block drops out at a given step, and
the spin bound shrinks to milliseconds) and check that the solve still
returns the reference's iterations: the kernel leaves the chunk-start state
(CG) or the step's input (GMRES) untouched, and the host reruns the work on
the launch-per-pass path, which needs no co-residency.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fault_step", [0, 3])
def test_cg_persistent_timeout_falls_back(monkeypatch, fault_step):
    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref

    R = problems.poisson2d(300)  # 88 blocks of 1024 threads
    A = krylov_amd.CsrOperator(R)
    b = np.random.default_rng(11).standard_normal(R.shape[0])
    _, clean = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    monkeypatch.setenv("KRY_CGP_FAULT", str(fault_step))
    _, faulted = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    assert faulted.numsteps == clean.numsteps
    f, c = np.asarray(faulted.resnorms), np.asarray(clean.resnorms)
    np.testing.assert_allclose(f[:-1], c[:-1], rtol=1e-10)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=1e-10, atol=1e-12 * np.abs(clean.xk).max())
    _, ref = krylov_ref.cg(R, b, tol=1e-9, maxiter=500)
    assert ref.numsteps == faulted.numsteps
    np.testing.assert_allclose(f[:-1], np.asarray(ref.resnorms)[:-1], rtol=1e-10)


def test_cg_timeout_after_committed_chunks(monkeypatch):
    """Clean persistent chunks first (their state swapped in), then a chunk
    that times out and is rerun launch per pass: the whole history equals a
    launch-per-pass solve's to round-off."""
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState
    import krylov_amd

    R = problems.poisson2d(200)
    A = krylov_amd.CsrOperator(R)
    b = np.random.default_rng(12).standard_normal(R.shape[0])

    def state():
        st = _CGState(_helpers.Problem(A, b, None, None))
        st.start()
        st.set_criterion(np.zeros(1))
        return st

    st = state()
    h1 = st.run(7)
    h2 = st.run(5)
    assert st.path() == (True, 0)
    monkeypatch.setenv("KRY_CGP_FAULT", "2")
    h3 = st.run(40)
    assert st.path() == (False, 1)
    h4 = st.run(9)  # stays launch per pass
    assert st.path() == (False, 1)
    got = np.concatenate([h1, h2, h3, h4])[:, 0]
    x_got = st.get(0)[:, 0]
    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    monkeypatch.delenv("KRY_CGP_FAULT")
    ref = state()
    want = ref.run(61)[:, 0]
    assert ref.path() == (False, 0)
    np.testing.assert_allclose(got, want, rtol=1e-10)
    np.testing.assert_allclose(x_got, ref.get(0)[:, 0], rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("ortho", ["mgs", "mgs2"])
def test_gmres_persistent_mgs_timeout_falls_back(monkeypatch, ortho):
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.gmres import _GmresState
    from oracle import krylov_ref

    R = problems.random_nonsym(200_000)
    A = krylov_amd.CsrOperator(R)
    b = np.ones(R.shape[0])
    _, clean = krylov_amd.gmres(A, b, ortho=ortho, maxiter=30, tol=1e-9)
    monkeypatch.setenv("KRY_MGS_FAULT", "2")
    _, faulted = krylov_amd.gmres(A, b, ortho=ortho, maxiter=30, tol=1e-9)
    assert faulted.numsteps == clean.numsteps
    f, c = np.asarray(faulted.resnorms), np.asarray(clean.resnorms)
    np.testing.assert_allclose(f[:-1], c[:-1], rtol=1e-11)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=1e-9, atol=1e-12)
    if ortho == "mgs":
        _, ref = krylov_ref.gmres(R, b, maxiter=30, tol=1e-9)
        assert ref.numsteps == faulted.numsteps
        np.testing.assert_allclose(f[:-1], np.asarray(ref.resnorms)[:-1], rtol=1e-10)
    # the state reports the switch
    st = _GmresState(_helpers.Problem(A, b, None, None), 30, 1 if ortho == "mgs" else 2)
    st.start()
    st.set_criterion(np.zeros(1))
    hist, _ = st.run(6)
    assert len(hist) == 6
    assert st.path() == (False, 1)


@pytest.mark.parametrize("fault_step", [0, 4])
def test_cg_update_kernel_timeout_falls_back(monkeypatch, fault_step):
    """The one-launch update of the launch-per-pass form (cg_upd_kernel,
    n beyond the persistent loop; forced here with KRY_CG_PERSIST=0): a block
    that never joins the exchange at step `fault_step` of the first chunk.
    Nothing was written, the rest of the chunk is rerun with separate passes
    from that step's SpMV, and the solve keeps the reference's iteration."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState
    from oracle import krylov_ref

    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    R = problems.poisson2d(300)
    A = krylov_amd.CsrOperator(R)
    b = np.random.default_rng(13).standard_normal(R.shape[0])
    _, clean = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    monkeypatch.setenv("KRY_CGU_FAULT", str(fault_step))
    _, faulted = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    assert faulted.numsteps == clean.numsteps
    f, c = np.asarray(faulted.resnorms), np.asarray(clean.resnorms)
    np.testing.assert_allclose(f[:-1], c[:-1], rtol=1e-10)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=1e-10, atol=1e-12 * np.abs(clean.xk).max())
    _, ref = krylov_ref.cg(R, b, tol=1e-9, maxiter=500)
    assert ref.numsteps == faulted.numsteps
    np.testing.assert_allclose(f[:-1], np.asarray(ref.resnorms)[:-1], rtol=1e-10)
    # the state reports the switch: used in the faulted chunk, then off
    st = _CGState(_helpers.Problem(A, b, None, None))
    st.start()
    st.set_criterion(np.zeros(1))
    assert len(st.run(8)) == 8
    assert st.update_path() == (True, 1)
    assert len(st.run(8)) == 8
    assert st.update_path() == (False, 1)


@pytest.mark.parametrize("late", [1, 3, 4, 6])
def test_cg_update_kernel_late_block_all_or_nothing(monkeypatch, late):
    """The last block joins the exchange late, about when the others' spin
    runs out (KRY_CGU_FAULT_LATE): the blocks agree on commit or abort
    (decide_exchange), so whichever way the race goes no block stores y / p /
    r after another gave up, and the solve equals a clean one."""
    import krylov_amd
    from krylov_amd import problems

    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    R = problems.poisson2d(300)
    A = krylov_amd.CsrOperator(R)
    b = np.random.default_rng(15).standard_normal(R.shape[0])
    _, clean = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    monkeypatch.setenv("KRY_CGU_FAULT", "2")
    monkeypatch.setenv("KRY_CGU_FAULT_LATE", str(late))
    _, faulted = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    assert faulted.numsteps == clean.numsteps
    f, c = np.asarray(faulted.resnorms), np.asarray(clean.resnorms)
    np.testing.assert_allclose(f[:-1], c[:-1], rtol=1e-10)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=1e-10, atol=1e-12 * np.abs(clean.xk).max())


def test_cg_update_kernel_timeout_under_communicator_is_an_error(monkeypatch):
    """Under a communicator a rank must not rerun part of a chunk alone (its
    allreduces would pair with other iterations of the other ranks): a
    timed-out exchange of the one-launch update raises instead, after posting
    the fault to every rank (1-rank RCCL communicator; the update kernel
    forced with KRY_CG_PERSIST=0; tests/test_gpu_shard_ranks.py covers the
    other solvers and the receiving side)."""
    from krylov_amd import distributed, problems
    import krylov_amd

    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    P = krylov_amd.CsrOperator(problems.poisson2d(300))
    b = np.random.default_rng(16).standard_normal((P.shape[0], 1))
    comm = distributed.ShardComm(0, 1, distributed.ShardComm.unique_id())
    try:
        monkeypatch.setenv("KRY_CGU_FAULT", "1")
        with pytest.raises(RuntimeError, match="every rank of the communicator stopped"):
            distributed.cg(P, b, comm, tol=1e-9, maxiter=100)
        monkeypatch.delenv("KRY_CGU_FAULT")
        _, info = distributed.cg(P, b, comm, tol=1e-9, maxiter=100)
        _, ref = krylov_amd.cg(P, b, tol=1e-9, maxiter=100)
        np.testing.assert_array_equal(np.asarray(info.resnorms), np.asarray(ref.resnorms))
    finally:
        comm.close()


def test_cg_update_kernel_matches_separate_passes(monkeypatch):
    """n = 2.0 M (Poisson 1414^2, above the persistent loop's 1 M): the
    one-launch update against the alpha / r / yp passes (KRY_CG_UPD=0) and
    the oracle's first 40 steps."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState
    from oracle import krylov_ref

    P = problems.poisson2d(1414)
    A = krylov_amd.CsrOperator(P)
    b = np.random.default_rng(14).standard_normal(P.shape[0])
    st = _CGState(_helpers.Problem(A, b, None, None))
    st.start()
    st.set_criterion(np.zeros(1))
    h1 = st.run(40)[:, 0]
    assert st.update_path() == (True, 0)
    monkeypatch.setenv("KRY_CG_UPD", "0")
    st0 = _CGState(_helpers.Problem(A, b, None, None))
    st0.start()
    st0.set_criterion(np.zeros(1))
    h0 = st0.run(40)[:, 0]
    assert st0.update_path() == (False, 0)
    np.testing.assert_allclose(h1, h0, rtol=1e-12)
    _, ref = krylov_ref.cg(P, b, tol=0.0, atol=0.0, maxiter=40)
    np.testing.assert_allclose(h1, np.asarray(ref.resnorms)[1:41], rtol=1e-10)


@pytest.mark.parametrize("fault_step", [0, 5])
def test_streamed_mgs_timeout_at_final_exchange(monkeypatch, fault_step):
    """The streamed persistent MGS kernel (gm_mgsl_kernel, chosen above 2 M
    unknowns: 15-point stencil 140^3, n = 2.74 M) timing out at its final,
    normalising exchange (KRY_MGS_FAULT_FINAL): the other blocks have already
    written their segments of V_{k+1} and block 0 its h entries. The host
    reruns the step from its SpMV on the per-pass kernels, which rewrite both,
    so the history and iterate equal a clean solve's."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.gmres import _GmresState

    S = problems.stencil15_3d(140)
    A = krylov_amd.CsrOperator(S)
    b = np.random.default_rng(17).standard_normal(S.shape[0])
    _, clean = krylov_amd.gmres(A, b, maxiter=20, tol=0.0)
    st = _GmresState(_helpers.Problem(A, b, None, None), 20, 1)
    st.start()
    st.set_criterion(np.zeros(1))
    st.run(3)
    assert st.path() == (True, 0)  # the persistent (streamed) MGS serves this size
    monkeypatch.setenv("KRY_MGS_FAULT", str(fault_step))
    monkeypatch.setenv("KRY_MGS_FAULT_FINAL", "1")
    _, faulted = krylov_amd.gmres(A, b, maxiter=20, tol=0.0)
    assert faulted.numsteps == clean.numsteps == 20
    np.testing.assert_allclose(np.asarray(faulted.resnorms)[:-1], np.asarray(clean.resnorms)[:-1], rtol=1e-11)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=1e-9, atol=1e-12 * np.abs(clean.xk).max())
    st = _GmresState(_helpers.Problem(A, b, None, None), 20, 1)
    st.start()
    st.set_criterion(np.zeros(1))
    hist, _ = st.run(8)
    assert len(hist) == 8 and st.path() == (False, 1)


def test_exchange_timeout_is_time_bounded(monkeypatch):
    """The exchanges give up after a fixed time (wall_clock64 ticks, 100 MHz:
    1 ms under fault injection, 20 ms in production), not after a poll count.
    A block that never joins costs about that bound once, then the chunk runs
    on the per-pass kernels: the faulted solve takes ~1 ms longer than the
    clean one (well under the 2^20-poll stall of round 2)."""
    import time

    import krylov_amd
    from krylov_amd import problems

    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    R = problems.poisson2d(300)
    A = krylov_amd.CsrOperator(R)
    b = np.random.default_rng(18).standard_normal(R.shape[0])

    def timed():
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=64)
            ts.append(time.perf_counter() - t0)
        return min(ts)

    clean = timed()
    monkeypatch.setenv("KRY_CGU_FAULT", "0")
    faulted = timed()
    print(f"\nclean {1e3 * clean:.2f} ms, faulted {1e3 * faulted:.2f} ms (extra {1e3 * (faulted - clean):.2f} ms)")
    assert faulted - clean < 0.1


@pytest.mark.parametrize("fault_step", [3, 6, 7])
def test_cg_update_kernel_dropout_with_deferred_y(monkeypatch, fault_step):
    """The one-launch update with yk deferred 7 steps (KRY_CG_YDEFER=7): a
    timed-out exchange at a step before, on and after a flush point leaves
    the pending updates to the chunk's end flush, which also moves p back
    into place for the launch-per-pass rerun; the faulted solve equals the
    clean deferred one to 1e-10 (the rerun's separate passes sum the inner
    products in another order, as in the per-step fallback test above), and
    the clean one equals the per-step form bit for bit."""
    import krylov_amd
    from krylov_amd import problems

    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    monkeypatch.setenv("KRY_CG_YDEFER", "7")
    R = problems.poisson2d(300)
    A = krylov_amd.CsrOperator(R)
    b = np.random.default_rng(17).standard_normal(R.shape[0])
    _, clean = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    monkeypatch.setenv("KRY_CGU_FAULT", str(fault_step))
    _, faulted = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    monkeypatch.delenv("KRY_CGU_FAULT")
    monkeypatch.setenv("KRY_CG_YDEFER", "0")
    _, plain = krylov_amd.cg(A, b, tol=1e-9, maxiter=500)
    assert plain.numsteps == clean.numsteps == faulted.numsteps
    np.testing.assert_array_equal(np.asarray(plain.resnorms).view(np.uint8), np.asarray(clean.resnorms).view(np.uint8))
    np.testing.assert_array_equal(plain.xk.view(np.uint8), clean.xk.view(np.uint8))
    f, c = np.asarray(faulted.resnorms), np.asarray(clean.resnorms)
    np.testing.assert_allclose(f[:-1], c[:-1], rtol=1e-10)
    np.testing.assert_allclose(faulted.xk, clean.xk, rtol=1e-10, atol=1e-12 * np.abs(clean.xk).max())
