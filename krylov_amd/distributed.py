"""Right-hand-side sharding across GPUs.

The reference is "fully blocked": a block ``b`` of shape (n, K) runs K
independent CG recurrences whose only coupling is the stop rule
``np.all(resnorms[-1] <= criterion)`` over all columns (cg.py:156,162). Here
the K columns are split into equal contiguous blocks, one per process/GPU;
each GPU runs the whole fused CG loop on its block against a replicated copy
of A, and every iteration performs exactly one ``ncclAllReduce`` (RCCL over
xGMI) of the zero-padded residual-norm vector so that every rank applies the
global stop rule and records the global history. The result equals the
unsharded block solve (same per-column recurrences, same stop step).

One process per GPU. The RCCL unique id is exchanged either over a
``torch.distributed`` process group the caller already has (any backend:
control plane only, ``ShardComm.from_torch``) or without PyTorch, through a
file every rank of the node can see (``ShardComm.from_file``). The rank
bookkeeping and the outer loop are ``krylov_amd.shard`` (pure NumPy, the code
the gloo CPU tests run); this module binds them to the device states.
"""
import ctypes

import numpy as np

from . import _helpers, _lib
from ._helpers import Info, Problem
from ._lib import check, lib
from .cg import _CGState
from .device import get_context
from .shard import ShardLayout, drive, file_rendezvous


class ShardComm:
    """An RCCL communicator over ``world`` ranks, one GPU each."""

    def __init__(self, rank, world, unique_id, device=None, ctx=None):
        self.ctx = get_context(device) if ctx is None else ctx
        self.rank = int(rank)
        self.world = int(world)
        idb = np.frombuffer(bytes(unique_id), dtype=np.uint8).copy()
        assert idb.size == 128
        h = ctypes.c_void_p()
        check(lib.kry_comm_create(self.ctx.handle, self.world, self.rank, _lib.ptr(idb), ctypes.byref(h)))
        self.handle = h
        self._fin = _lib.own(self, lib.kry_comm_destroy, h)

    @staticmethod
    def unique_id():
        buf = np.zeros(128, dtype=np.uint8)
        check(lib.kry_comm_unique_id(_lib.ptr(buf)))
        return buf.tobytes()

    @classmethod
    def from_torch(cls, group=None, device=None):
        """Create the communicator, exchanging the unique id through an
        initialised ``torch.distributed`` process group (any backend)."""
        import torch
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        idt = torch.zeros(128, dtype=torch.int64)
        if rank == 0:
            idt = torch.from_numpy(np.frombuffer(cls.unique_id(), dtype=np.uint8).astype(np.int64))
        dist.broadcast(idt, src=0, group=group)
        uid = idt.numpy().astype(np.uint8).tobytes()
        return cls(rank, world, uid, device=device)

    @classmethod
    def solo(cls, rank, world, device=None, ctx=None):
        """Rank ``rank`` of ``world`` rehearsed on ONE GPU: a 1-rank RCCL
        communicator (its allreduce is the identity) with the layout of rank
        ``rank`` of ``world``. The solvers then attach at column offset
        ``rank * kpad`` of ``world * kpad`` global slots and run every
        per-step collective and global check of that rank; the other ranks'
        slots of each global vector stay exactly 0 (no one posts them), so
        this rank's slots must equal the unsharded solve of its columns bit
        for bit. Used to execute the rank > 0 device code without a node.
        ``ctx``: a context of its own (e.g. one per host thread, several
        ranks rehearsed concurrently on one GPU)."""
        if not (0 <= int(rank) < int(world)):
            raise ValueError(f"bad rank {rank} of {world}")
        c = cls(0, 1, cls.unique_id(), device=device, ctx=ctx)
        c.rank, c.world = int(rank), int(world)
        return c

    @classmethod
    def all_devices(cls, devices):
        """One communicator per device of THIS process (kry_comm_create_all,
        ncclCommInitAll): the single-process multi-GPU path, rank i on
        devices[i], each driven by its own host thread."""
        devices = [int(d) for d in devices]
        ctxs = [get_context(d) for d in devices]
        arr = (ctypes.c_void_p * len(devices))(*[c.handle.value for c in ctxs])
        outs = (ctypes.c_void_p * len(devices))()
        check(lib.kry_comm_create_all(arr, len(devices), outs))
        comms = []
        for i, c in enumerate(ctxs):
            obj = cls.__new__(cls)
            obj.ctx, obj.rank, obj.world = c, i, len(devices)
            obj.handle = ctypes.c_void_p(outs[i])
            obj._fin = _lib.own(obj, lib.kry_comm_destroy, obj.handle)
            comms.append(obj)
        return comms

    @classmethod
    def from_file(cls, path, rank, world, device=None, timeout=120.0):
        """Create the communicator without PyTorch: rank 0 writes the unique id
        to ``path`` (a fresh file name on a file system every rank sees, e.g.
        under /dev/shm), the others read it (``shard.file_rendezvous``)."""
        uid = file_rendezvous(path, int(rank), cls.unique_id, timeout=timeout)
        return cls(rank, world, uid, device=device)

    def allreduce(self, values):
        """Sum a small float64 vector over ranks (setup-time exchanges)."""
        v = np.ascontiguousarray(values, dtype=np.float64).copy()
        check(lib.kry_comm_allreduce(self.handle, _lib.dptr(v), v.size))
        return v

    def abort(self):
        """Abort the communicator (kry_comm_abort): a collective pending on it
        in another thread, and every later one, fails with KRY_ECOMM instead
        of waiting for a rank that will not come. ``close()`` still releases
        it."""
        check(lib.kry_comm_abort(self.handle))

    def close(self):
        self._fin()


def _block(B):
    B = np.asarray(B)
    return B[:, None] if B.ndim == 1 else B


class _Engine:
    """A device solver state in the shape ``shard.drive`` expects."""

    def __init__(self, st, run_fn, total, start_fn, norm2_fn):
        self.st, self._run, self.total = st, run_fn, total
        self._start, self._norm2 = start_fn, norm2_fn

    def start_norms(self):
        return self._start()

    def set_criterion(self, crit_full):
        self.st.set_criterion(crit_full)

    def run(self, steps):
        return self._run(steps)

    def residual_norm2(self):
        return self._norm2()


def _run_global(lib_run, h, steps, total):
    out = np.zeros((max(steps, 1), total))
    done = ctypes.c_int32()
    inv = ctypes.c_int32()
    check(lib_run(h, int(steps), ctypes.byref(done), _lib.dptr(out), ctypes.byref(inv)))
    return out[: done.value], bool(inv.value)


def gather_columns(comm, lay, prob, local):
    """This rank's (n, kpad) host block -> the global (n, K) block of the real
    columns, in rank order: a zero-padded allreduce (sum) over the
    communicator, i.e. an all-gather (x + 0 is x). Every rank must call it,
    since it is a collective. Used only for callbacks, which see the whole
    iterate as the unsharded solve would give it."""
    a = np.zeros((prob.n, lay.total))
    a[:, lay.off:lay.off + prob.kpad] = np.asarray(local, dtype=np.float64).reshape(prob.n, prob.kpad)
    g = comm.allreduce(a.reshape(-1)).reshape(prob.n, lay.total)[:, lay.real]
    return np.ascontiguousarray(g).astype(prob.r0_dtype, copy=False)


def _hook(callback, first, step):
    """The drive() hook that calls ``callback`` as the reference does:
    ``first(resnorm)`` and ``step(resnorm)`` return its arguments (after the
    collective gathers, which every rank runs; ``callback`` is called on
    every rank that passed one)."""
    if callback is None:
        return None

    def hook(k, resnorm):
        args = first(resnorm) if k == 0 else step(resnorm)
        callback(*args)

    return hook


def _problem(A, B, x0, inner, comm, M=None, Ml=None, Mr=None):
    return Problem(A, _block(B), x0, inner, M=M, Ml=Ml, Mr=Mr, device=comm.ctx.device)


def cg(A, B, comm, x0=None, tol=1e-5, atol=1.0e-15, maxiter=None, callback=None, kcs=None, M=None, Ml=None,
       inner=None):
    """Block CG on this rank's RHS columns ``B`` (n, k_local), k_local equal
    on every rank, with the reference's global stop rule. ``M``/``Ml`` and
    ``inner`` (None or WeightedInner) as in ``krylov_amd.cg``: applied on this
    rank's device to its own columns (every rank holds all n rows, so the
    preconditioners and weights are per-column operations). ``callback(xk,
    Ml_rk)`` as in cg.py:119-120,202-204, with the GLOBAL (n, K) iterate and
    residual (gathered every step: a debugging aid, not a fast path).

    Returns ``(xk_local or None, Info)``; ``Info.resnorms`` holds the GLOBAL
    history (each entry an array over all world * k_local columns, in rank
    order), identical on every rank.
    """
    prob = _problem(A, B, x0, inner, comm, M=M, Ml=Ml)
    lay = ShardLayout(prob.kc, prob.kpad, comm.rank, comm.world, kcs)
    maxiter = prob.A.shape[0] if maxiter is None else maxiter
    st = _CGState(prob)
    check(lib.kry_cg_attach_comm(st.h, comm.handle, lay.off, lay.total))
    eng = _Engine(st, lambda steps: (st.run(steps, ncols=lay.total), False), lay.total,
                  lambda: np.sqrt(st.start().astype(prob.inner_dtype)).astype(np.float64), st.residual_norm2)

    def args(_rn):
        return gather_columns(comm, lay, prob, st.get(0)), gather_columns(comm, lay, prob, st.get(1))

    def first(_rn):
        x0g = gather_columns(comm, lay, prob, prob.pad(prob.x0)) if prob.x0 is not None else \
            np.zeros((prob.n, lay.real.size), dtype=prob.r0_dtype)
        return x0g, gather_columns(comm, lay, prob, st.get(1))

    success, k, resnorms = drive(eng, lay, comm.allreduce, tol, atol, maxiter, prob.inner_dtype, _helpers.CHUNK,
                                 hook=_hook(callback, first, args))
    xk = prob.unpad_vec(st.get(0), prob.r0_dtype)
    ops = {"A": 1 + k, "M": 2 + k, "Ml": 2 + k, "Mr": 1 + k, "inner": 2 + 2 * k, "axpy": 2 + 2 * k}
    return xk if success else None, Info(success, xk, k, resnorms, num_operations=ops,
                                         renumbered=prob.A.renumbered)


def gmres(A, B, comm, x0=None, tol=1e-5, atol=1.0e-15, maxiter=None, ortho="mgs", kcs=None, M=None, Ml=None,
          Mr=None, inner=None, callback=None):
    """GMRES (MGS) on this rank's RHS columns ``B`` (n, k_local), k_local
    equal on every rank. Every Arnoldi step performs one RCCL allreduce of the
    residual norms and a non-invariant count, so all ranks apply the
    reference's stop rule (gmres.py:193) and invariance test (arnoldi.py:187)
    to ALL columns and stop at the same step as the unsharded block solve.
    ``M``/``Ml``/``Mr``, ``inner`` and ``callback(xk, resnorm)`` as in
    ``krylov_amd.gmres`` (the callback sees the gathered global iterate).
    Returns ``(xk_local or None, Info)`` with the global history."""
    from .gmres import _GmresState, _sweeps

    if not ortho.startswith("mgs"):
        raise NotImplementedError("the sharded path runs MGS Arnoldi (Householder is single right-hand side)")
    sweeps = _sweeps(ortho, inner, M, B)
    prob = _problem(A, B, x0, inner, comm, M=M, Ml=Ml, Mr=Mr)
    maxiter = prob.A.shape[0] if maxiter is None else maxiter
    lay = ShardLayout(prob.kc, prob.kpad, comm.rank, comm.world, kcs)
    st = _GmresState(prob, maxiter, sweeps)
    check(lib.kry_gmres_attach_comm(st.h, comm.handle, lay.off, lay.total))

    def norm2():
        st.solution()  # the explicit residual of x0 + V R^-1 y (gmres.py:197-199)
        return st.residual_norm2()

    def first(_rn):
        # callback(x0, Ml (b - A x0)) (gmres.py:143-144), on this rank's columns, then gathered
        x0h = prob.x0_or_zeros()
        x0l = prob.pad(x0h)
        mr = prob.pad(prob.apply_host("Ml", prob.b - prob.A @ x0h))
        return gather_columns(comm, lay, prob, x0l), gather_columns(comm, lay, prob, mr)

    def step(rn):
        st.solution()
        return gather_columns(comm, lay, prob, prob.pad(st.xk())), np.array(rn)

    eng = _Engine(st, lambda steps: _run_global(lib.kry_gmres_run, st.h, steps, lay.total), lay.total, st.start,
                  norm2)
    success, k, resnorms = drive(eng, lay, comm.allreduce, tol, atol, maxiter, prob.inner_dtype, _helpers.CHUNK,
                                 hook=_hook(callback, first, step))
    if k == 0:
        xk = prob.zeros_like_b() if prob.x0 is None else prob.x0
    else:
        st.solution()
        xk = st.xk()
    ops = {"A": 1 + k, "M": 2 + k, "Ml": 2 + k, "Mr": 1 + k, "inner": 2 + k + k * (k + 1) / 2,
           "axpy": 4 + 2 * k + k * (k + 1) / 2}
    return xk if success else None, Info(success, xk, k, resnorms, num_operations=ops,
                                         renumbered=prob.A.renumbered)


def minres(A, B, comm, x0=None, inner=None, tol=1e-5, atol=1.0e-15, maxiter=None, kcs=None, M=None, Ml=None,
           Mr=None, callback=None):
    """MINRES on this rank's RHS columns ``B`` (n, k_local), k_local equal on
    every rank; one RCCL allreduce per iteration for the global stop rule
    (minres.py:162) and the Lanczos invariance test over all columns.
    ``M``/``Ml``/``Mr`` and ``callback(xk, resnorm)`` as in
    ``krylov_amd.minres`` (the callback sees the gathered global iterate).
    Returns ``(xk_local or None, Info)`` with the global history."""
    from .minres import _MinresState

    prob = _problem(A, B, x0, inner, comm, M=M, Ml=Ml, Mr=Mr)
    maxiter = prob.A.shape[0] if maxiter is None else maxiter
    lay = ShardLayout(prob.kc, prob.kpad, comm.rank, comm.world, kcs)
    st = _MinresState(prob)
    check(lib.kry_minres_attach_comm(st.h, comm.handle, lay.off, lay.total))

    def first(rn):
        x0h = prob.x0_or_zeros()
        return gather_columns(comm, lay, prob, prob.pad(x0h)), np.array(rn)

    def step(rn):
        return gather_columns(comm, lay, prob, prob.pad(st.xk())), np.array(rn)

    eng = _Engine(st, lambda steps: _run_global(lib.kry_minres_run, st.h, steps, lay.total), lay.total, st.start,
                  st.residual_norm2)
    success, k, resnorms = drive(eng, lay, comm.allreduce, tol, atol, maxiter, prob.inner_dtype, _helpers.CHUNK,
                                 hook=_hook(callback, first, step))
    xk = st.xk()
    ops = {"A": 1 + k, "M": 2 + k, "Ml": 2 + k, "Mr": 1 + k, "inner": 2 + 2 * k, "axpy": 4 + 8 * k}
    return xk if success else None, Info(success, xk, k, resnorms, num_operations=ops,
                                         renumbered=prob.A.renumbered)
