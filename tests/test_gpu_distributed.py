"""The RCCL-sharded CG path on a GPU box with one GPU: a 1-rank RCCL
communicator is a valid communicator, so the whole sharded code path (zero-
padded residual-norm allreduce every iteration, global stop rule, global
history) runs and must reproduce the unsharded device block solve exactly,
and the reference fixture to the parity tolerance."""
import numpy as np
import pytest

from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu


def test_sharded_cg_single_rank_matches_block_cg(golden):
    import krylov_amd
    from krylov_amd import distributed, problems

    d = golden["solvers"]
    P = krylov_amd.CsrOperator(problems.poisson2d(64))
    B = d["poisson64_B"]
    comm = distributed.ShardComm(0, 1, distributed.ShardComm.unique_id())
    sol, info = distributed.cg(P, B, comm, tol=1e-8)
    _, ref = krylov_amd.cg(P, B, tol=1e-8)
    assert info.success and info.numsteps == ref.numsteps
    np.testing.assert_array_equal(np.asarray(info.resnorms), np.asarray(ref.resnorms))
    np.testing.assert_array_equal(info.xk, ref.xk)
    H.assert_parity(info, d, "cg_poisson64_blk8")
    comm.close()


def test_sharded_cg_odd_columns():
    """3 local columns (padded to 4 on the device) stay inert in the stop rule."""
    import krylov_amd
    from krylov_amd import distributed, problems

    P = problems.poisson2d(32)
    B = np.random.default_rng(1).standard_normal((P.shape[0], 3))
    comm = distributed.ShardComm(0, 1, distributed.ShardComm.unique_id())
    _, info = distributed.cg(P, B, comm, tol=1e-9)
    _, ref = krylov_amd.cg(P, B, tol=1e-9)
    assert info.numsteps == ref.numsteps
    np.testing.assert_array_equal(np.asarray(info.resnorms), np.asarray(ref.resnorms))
    comm.close()


def test_sharded_gmres_single_rank_matches_block_gmres(golden):
    """RCCL path of distributed.gmres (per-step allreduce of the residual norms
    and the non-invariant count): bitwise the unsharded device block solve,
    and the reference's block-GMRES fixture to the parity tolerance."""
    import krylov_amd
    from krylov_amd import distributed, problems

    d = golden["solvers"]
    R = krylov_amd.CsrOperator(problems.random_nonsym(5000))
    B = d["rand5k_B3"]
    comm = distributed.ShardComm(0, 1, distributed.ShardComm.unique_id())
    _, info = distributed.gmres(R, B, comm, maxiter=20, tol=0.0)
    _, ref = krylov_amd.gmres(R, B, maxiter=20, tol=0.0)
    assert info.numsteps == ref.numsteps == 20
    np.testing.assert_array_equal(np.asarray(info.resnorms), np.asarray(ref.resnorms))
    np.testing.assert_array_equal(info.xk, ref.xk)
    H.assert_parity(info, d, "gmres_rand5k_blk3")
    # with a tolerance: the global stop rule waits for the slowest column
    _, info = distributed.gmres(R, B, comm, maxiter=60, tol=1e-6)
    _, ref = krylov_amd.gmres(R, B, maxiter=60, tol=1e-6)
    assert info.success and info.numsteps == ref.numsteps
    np.testing.assert_array_equal(np.asarray(info.resnorms), np.asarray(ref.resnorms))
    comm.close()


def test_sharded_minres_single_rank_matches_block_minres(golden):
    import krylov_amd
    from krylov_amd import distributed, problems

    d = golden["solvers"]
    P = krylov_amd.CsrOperator(problems.poisson2d(64))
    B = d["poisson64_B"]
    comm = distributed.ShardComm(0, 1, distributed.ShardComm.unique_id())
    _, info = distributed.minres(P, B, comm, tol=1e-8)
    _, ref = krylov_amd.minres(P, B, tol=1e-8)
    assert info.success and info.numsteps == ref.numsteps
    np.testing.assert_array_equal(np.asarray(info.resnorms), np.asarray(ref.resnorms))
    np.testing.assert_array_equal(info.xk, ref.xk)
    comm.close()
