"""The sharded device path as rank r > 0 of W, on one GPU.

A GPU box here has one GPU, so a real W-rank run cannot execute. What can:
``ShardComm.solo(r, W)`` is a 1-rank RCCL communicator (its allreduce is the
identity) with the layout of rank r of W. The solvers then attach at column
offset r * kpad of W * kpad global slots and run every per-step collective,
the zero-padded global vector, the global stop rule (``cg_global_check`` /
``gm_global_check`` / ``mr_global_check``) and ``shard.drive``'s outer loop
exactly as rank r would. The other ranks' slots stay exactly 0 (nobody posts
them), and 0 <= their criterion, so this rank's columns must reproduce the
unsharded device solve of the same columns BIT FOR BIT: history, step count
and iterate (reference rule: cg.py:156,162, gmres.py:193, minres.py:162).

Paths covered, each asserted from the solver state: CG k = 1 on the
one-launch update (cg_upd_kernel), block CG k = 8 on the DIA block SpMV with
deferred yk (cg_pdefer_kernel), GMRES k = 1 on the streamed persistent MGS
(gm_mgsl_kernel) and k = 4 on gm_mgsp_kernel, MINRES k = 1 on the one-launch
step tail (mr_upd_kernel).

Then the failure protocol (include/krylov_hip.h, "fault count"): a rank whose
in-launch exchange times out posts a fault in the step's allreduce instead of
its norms, every rank stops before that step, the faulting rank raises
KRY_EDEVICE and the others KRY_ECOMM. Here the local side runs with the
existing fault switches and the receiving side with KRY_COMM_PEER_FAULT (a
fault arriving in the allreduce as if from a peer); after either, the same
communicator runs a clean solve bit for bit, so no collective was left
unpaired.
"""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (a.shape, b.shape, a.dtype, b.dtype)
    np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8))


def _check_rank(info, ref, rank, world, kc):
    """This rank's slots of every global history row == the unsharded
    history; every other slot exactly 0."""
    H = np.asarray(info.resnorms, dtype=np.float64)
    R = np.asarray(ref.resnorms, dtype=np.float64).reshape(len(ref.resnorms), kc)
    assert info.numsteps == ref.numsteps and info.success == ref.success
    assert H.shape == (R.shape[0], world * kc)
    mine = slice(rank * kc, (rank + 1) * kc)
    _bits(H[:, mine], R)
    others = np.delete(H, np.arange(rank * kc, (rank + 1) * kc), axis=1)
    assert others.size == 0 or np.all(others == 0.0)
    _bits(info.xk, ref.xk)


def _mod(name):
    """The module krylov_amd.<name> (the package attribute of that name is the
    solver function)."""
    return importlib.import_module(f"krylov_amd.{name}")


class _Record:
    """Keeps every solver state a driver creates (to read its path after)."""

    def __init__(self, monkeypatch, module, name):
        base = getattr(module, name)
        made = self.made = []

        class Rec(base):
            def __init__(self, *a, **k):
                super().__init__(*a, **k)
                made.append(self)

        monkeypatch.setattr(module, name, Rec)


@pytest.mark.parametrize("rank,world", [(1, 2), (3, 4)])
def test_rank_cg_single_rhs_update_kernel(monkeypatch, rank, world):
    import krylov_amd
    from krylov_amd import distributed, problems

    cgmod = _mod("cg")

    monkeypatch.setenv("KRY_CG_PERSIST", "0")  # the unsharded solve takes cg_upd_kernel too
    A = krylov_amd.CsrOperator(problems.poisson2d(150))
    B = np.random.default_rng(30 + rank).standard_normal((A.shape[0], 1))
    rec = _Record(monkeypatch, distributed, "_CGState")
    comm = distributed.ShardComm.solo(rank, world)
    try:
        _, info = distributed.cg(A, B, comm, tol=1e-8, maxiter=2000)
    finally:
        comm.close()
    assert rec.made[0].update_path()[0] == 1 and rec.made[0].path() == (False, 0)
    rec2 = _Record(monkeypatch, cgmod, "_CGState")
    _, ref = krylov_amd.cg(A, B, tol=1e-8, maxiter=2000)
    assert rec2.made[0].update_path()[0] == 1
    assert info.success and info.numsteps > 100  # ~450 steps
    _check_rank(info, ref, rank, world, 1)


@pytest.mark.parametrize("rank,world", [(1, 2), (3, 4)])
def test_rank_block_cg_dia_deferred_y(monkeypatch, rank, world):
    """k = 8 on the DIA block SpMV with yk deferred 7 steps (the cfg4 path;
    forced with KRY_CG_YDEFER at a size that fits a quick test)."""
    import krylov_amd
    from krylov_amd import distributed, problems

    cgmod = _mod("cg")

    monkeypatch.setenv("KRY_CG_YDEFER", "7")
    A = krylov_amd.CsrOperator(problems.poisson2d(150))
    assert A.layout()["dia"]
    B = np.random.default_rng(40 + rank).standard_normal((A.shape[0], 8))
    B[:, 3] *= 1e-3  # columns converge at different steps
    rec = _Record(monkeypatch, distributed, "_CGState")
    comm = distributed.ShardComm.solo(rank, world)
    try:
        _, info = distributed.cg(A, B, comm, tol=1e-8, maxiter=2000)
    finally:
        comm.close()
    assert rec.made[0].defer_info()[0] == 7
    rec2 = _Record(monkeypatch, cgmod, "_CGState")
    _, ref = krylov_amd.cg(A, B, tol=1e-8, maxiter=2000)
    assert rec2.made[0].defer_info()[0] == 7
    assert info.success
    _check_rank(info, ref, rank, world, 8)


@pytest.mark.parametrize("rank,world", [(1, 2), (3, 4)])
def test_rank_gmres_streamed_mgs(monkeypatch, rank, world):
    """k = 1 above 2 M unknowns: the streamed persistent MGS kernel."""
    import krylov_amd
    from krylov_amd import distributed, problems

    gmmod = _mod("gmres")

    A = krylov_amd.CsrOperator(problems.stencil15_3d(140))
    B = np.random.default_rng(50 + rank).standard_normal((A.shape[0], 1))
    rec = _Record(monkeypatch, gmmod, "_GmresState")
    comm = distributed.ShardComm.solo(rank, world)
    try:
        _, info = distributed.gmres(A, B, comm, maxiter=20, tol=0.0)
    finally:
        comm.close()
    assert rec.made[0].path() == (True, 0)
    _, ref = krylov_amd.gmres(A, B, maxiter=20, tol=0.0)
    assert rec.made[-1].path() == (True, 0)
    assert info.numsteps == 20
    _check_rank(info, ref, rank, world, 1)


@pytest.mark.parametrize("rank,world", [(1, 2), (2, 3)])
def test_rank_gmres_block(golden, monkeypatch, rank, world):
    """3 columns (padded to 4) on the persistent MGS kernel, with a tolerance
    so the global rule waits for the slowest column."""
    import krylov_amd
    from krylov_amd import distributed, problems

    gmmod = _mod("gmres")

    d = golden["solvers"]
    A = krylov_amd.CsrOperator(problems.random_nonsym(5000))
    B = d["rand5k_B3"]
    rec = _Record(monkeypatch, gmmod, "_GmresState")
    comm = distributed.ShardComm.solo(rank, world)
    try:
        _, info = distributed.gmres(A, B, comm, maxiter=60, tol=1e-6)
    finally:
        comm.close()
    assert rec.made[0].path()[0]
    _, ref = krylov_amd.gmres(A, B, maxiter=60, tol=1e-6)
    assert info.success
    _check_rank(info, ref, rank, world, 3)


@pytest.mark.parametrize("rank,world", [(1, 2), (3, 4)])
def test_rank_minres_step_tail(monkeypatch, rank, world):
    import krylov_amd
    from krylov_amd import distributed, problems

    mrmod = _mod("minres")

    A = krylov_amd.CsrOperator(problems.poisson2d(150))
    B = np.random.default_rng(60 + rank).standard_normal((A.shape[0], 1))
    rec = _Record(monkeypatch, mrmod, "_MinresState")
    comm = distributed.ShardComm.solo(rank, world)
    try:
        _, info = distributed.minres(A, B, comm, tol=1e-8, maxiter=2000)
    finally:
        comm.close()
    assert rec.made[0].update_path()[0]
    _, ref = krylov_amd.minres(A, B, tol=1e-8, maxiter=2000)
    assert rec.made[-1].update_path()[0]
    assert info.success
    _check_rank(info, ref, rank, world, 1)


# ------------------------------------------------------------ failure protocol
def _solve(kind, A, B, comm):
    from krylov_amd import distributed

    if kind == "cg":
        return distributed.cg(A, B, comm, tol=1e-9, maxiter=100)
    if kind == "gmres":
        return distributed.gmres(A, B, comm, maxiter=12, tol=0.0)
    return distributed.minres(A, B, comm, tol=1e-9, maxiter=100)


@pytest.mark.parametrize("kind,switch", [("cg", "KRY_CGU_FAULT"), ("gmres", "KRY_MGS_FAULT"),
                                         ("minres", "KRY_MRU_FAULT")])
def test_local_exchange_timeout_stops_every_rank(monkeypatch, kind, switch):
    """This rank's in-launch exchange times out at step 2: it posts the fault
    and raises; the communicator is left with every collective paired (the
    next solve on it is the clean one, bit for bit)."""
    import krylov_amd
    from krylov_amd import distributed, problems

    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    A = krylov_amd.CsrOperator(problems.stencil15_3d(140) if kind == "gmres" else problems.poisson2d(300))
    B = np.random.default_rng(70).standard_normal((A.shape[0], 1))
    comm = distributed.ShardComm.solo(1, 2)
    try:
        _, clean = _solve(kind, A, B, comm)
        monkeypatch.setenv(switch, "2")
        with pytest.raises(RuntimeError, match="every rank of the communicator stopped"):
            _solve(kind, A, B, comm)
        monkeypatch.delenv(switch)
        _, again = _solve(kind, A, B, comm)
    finally:
        comm.close()
    _bits(np.asarray(again.resnorms), np.asarray(clean.resnorms))
    _bits(again.xk, clean.xk)


@pytest.mark.parametrize("kind", ["cg", "block_cg", "gmres", "minres"])
def test_peer_fault_stops_this_rank(monkeypatch, kind):
    """A fault count arriving in step 2's allreduce (as a peer whose exchange
    timed out would post it): this rank stops before step 2 and raises
    KRY_ECOMM; the same communicator then solves cleanly."""
    import krylov_amd
    from krylov_amd import distributed, problems

    A = krylov_amd.CsrOperator(problems.poisson2d(200))
    k = 8 if kind == "block_cg" else 1
    B = np.random.default_rng(71).standard_normal((A.shape[0], k))
    solver = "cg" if kind == "block_cg" else kind
    comm = distributed.ShardComm.solo(0, 3)
    try:
        _, clean = _solve(solver, A, B, comm)
        monkeypatch.setenv("KRY_COMM_PEER_FAULT", "2")
        with pytest.raises(RuntimeError, match="another rank's in-launch exchange failed at step 2"):
            _solve(solver, A, B, comm)
        monkeypatch.delenv("KRY_COMM_PEER_FAULT")
        _, again = _solve(solver, A, B, comm)
    finally:
        comm.close()
    _bits(np.asarray(again.resnorms), np.asarray(clean.resnorms))
    _bits(again.xk, clean.xk)
