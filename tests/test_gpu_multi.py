"""Several GPUs of one process from the reference signature (round 5):
``krylov_amd.cg / gmres / minres(A, B, devices=[...])`` (krylov_amd.multi).

The pool's boxes have one GPU, so the path is exercised at devices=[0]: one
communicator from ncclCommInitAll (kry_comm_create_all), one host thread
driving the sharded loop (krylov_amd.distributed + shard.drive, one RCCL
allreduce per step) - which must give the unsharded block solve bit for bit
(the per-column recurrences are independent; the global stop rule over a
1-rank allreduce is the local one). Uneven column splits over several ranks
run on the CPU over gloo (tests/test_sharding_cpu.py, cg_uneven), and the
rank > 0 slot arithmetic on one GPU in tests/test_gpu_shard_ranks.py.
Reference: cg.py:16-28 (fully blocked b), _helpers.py:107-108, the stop
rule cg.py:156,162.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(a, b):
    np.testing.assert_array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))


@pytest.mark.parametrize("method", ["cg", "gmres", "minres"])
def test_devices_single_gpu_equals_block_solve(method):
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(96)
    B = np.random.default_rng(8).standard_normal((P.shape[0], 8))
    kw = dict(tol=1e-8, maxiter=400) if method != "gmres" else dict(tol=0.0, maxiter=25)
    x1, i1 = getattr(krylov_amd, method)(P, B, **kw)
    x2, i2 = getattr(krylov_amd, method)(P, B, devices=[0], **kw)
    assert i1.numsteps == i2.numsteps and bool(i1.success) == bool(i2.success)
    _bits(np.array(i2.resnorms), np.array(i1.resnorms))
    _bits(i2.xk, i1.xk)
    assert i2.xk.shape == B.shape
    if i1.success:
        _bits(x2, x1)


def test_devices_vector_rhs_and_x0(monkeypatch):
    """A 1-D b keeps scalar history entries; x0 is split like b. (One column
    on one device would take the persistent small-n CG loop, which sums its
    inner products in another order and cannot carry the per-step allreduce:
    KRY_CG_PERSIST=0 puts the plain solve on the same launch-per-pass path.)"""
    import krylov_amd
    from krylov_amd import problems

    monkeypatch.setenv("KRY_CG_PERSIST", "0")
    P = problems.poisson2d(64)
    b = np.ones(P.shape[0])
    x0 = np.linspace(-1.0, 1.0, P.shape[0])
    x1, i1 = krylov_amd.cg(P, b, x0=x0, tol=1e-9)
    x2, i2 = krylov_amd.cg(P, b, x0=x0, tol=1e-9, devices=[0])
    assert i2.numsteps == i1.numsteps and np.ndim(i2.resnorms[0]) == 0
    _bits(np.array(i2.resnorms), np.array(i1.resnorms))
    _bits(x2, x1)


def test_devices_argument_errors():
    import krylov_amd
    from krylov_amd import problems

    P = problems.poisson2d(16)
    B = np.ones((P.shape[0], 2))
    with pytest.raises(ValueError):
        krylov_amd.cg(P, B, devices=[0, 0])
    with pytest.raises(NotImplementedError):
        krylov_amd.cg(P, B, devices=[0], return_arnoldi=True)
    with pytest.raises(ValueError):  # a preconditioner list must match the devices
        krylov_amd.gmres(P, B, devices=[0], M=[krylov_amd.CsrOperator(P, device=0)] * 2)
    with pytest.raises(ValueError):
        krylov_amd.cg(krylov_amd.CsrOperator(P), B, devices=[0])
    ops = [krylov_amd.CsrOperator(P, device=0)]
    _, info = krylov_amd.cg(ops, B, devices=[0], tol=1e-8)
    assert info.success


def test_devices_abort_on_failure_and_aborted_comm_refuses():
    """A device thread that fails aborts every communicator (kry_comm_abort),
    so no other device waits forever in a collective it will not get; the
    first error is raised. An aborted communicator refuses later collectives
    with KRY_ECOMM (RuntimeError) and still closes."""
    import krylov_amd
    from krylov_amd import distributed, problems

    P = problems.poisson2d(32)
    B = np.ones((P.shape[0], 2))
    with pytest.raises(TypeError):
        krylov_amd.cg(P, B, devices=[0], maxiter="many")
    (comm,) = distributed.ShardComm.all_devices([0])
    comm.abort()
    with pytest.raises(RuntimeError):
        comm.allreduce(np.ones(3))
    comm.close()
    _, info = krylov_amd.cg(P, B, devices=[0], tol=1e-8)  # a fresh communicator works
    assert info.success
