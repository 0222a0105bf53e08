"""Several GPUs from the reference signature, in ONE process (round 5).

``krylov_amd.cg(A, B, devices=[0, 1, ...])`` (likewise ``gmres`` and
``minres``) splits the columns of a block right-hand side over the listed
devices and returns the gathered global iterate, as the single-device block
solve would: SURVEY §8(e), "B = (n, 64): 8 RHS per GPU, one RCCL allreduce of
the residual norms per iteration, xk gathered into X[:, 8g:8g+8]".

* One communicator per device from one ``ncclCommInitAll``
  (``kry_comm_create_all``); each device gets its own context (stream),
  operator replica and solver state, and is driven by its own host thread
  (ctypes releases the GIL inside every C-ABI call, so the devices' chunk
  launches and their per-step allreduces overlap).
* K columns over D devices: ``ceil(K / D)`` device columns each, a short last
  device padded with zero columns that are not real columns of the layout
  (never in the history, +inf in the stop rule: ``shard.ShardLayout``'s
  ``kcs``), at most one device per column.
* The per-rank loop is ``krylov_amd.distributed``'s (``shard.drive``), so
  every device applies the reference's global stop rule over ALL columns
  (cg.py:156,162; gmres.py:193; minres.py:162) and the invariance test over
  all columns (arnoldi.py:187, 270-272): the same step count and history as
  the unsharded block solve.

``A``: a scipy.sparse matrix or dense array (uploaded once per device, the
uploads in parallel threads), or a list of ``CsrOperator``, one per device
in ``devices`` order. ``M``/``Ml``/``Mr`` likewise (a host matrix is
uploaded to every device; each device applies it to its own columns with the
single-device kernels), and ``inner`` (None or WeightedInner). ``callback``
is called once per step, from the first device's thread, with the gathered
global iterate, exactly as the single-device solve calls it (cg.py:119-120,
202-204; gmres.py:143-144, 226-228; minres.py:160-161, 230-232); every step
then gathers x over the devices, so it is a debugging aid, not a fast path.
If one device's thread fails, every communicator is aborted
(kry_comm_abort), so the others stop at their next collective instead of
waiting for it, and that first error is raised.
"""
import threading

import numpy as np

from . import distributed
from .distributed import ShardComm


def _operators(A, devices):
    from .sparse import CsrOperator

    if isinstance(A, (list, tuple)):
        if len(A) != len(devices) or not all(isinstance(a, CsrOperator) for a in A):
            raise ValueError("A as a list: one CsrOperator per device, in devices order")
        for a, d in zip(A, devices):
            if a.device != d:
                raise ValueError(f"operator on device {a.device} listed for device {d}")
        return list(A)
    if isinstance(A, CsrOperator):
        raise ValueError("devices=[...]: pass the host matrix (uploaded to every device) or one CsrOperator per "
                         "device")
    ops = [None] * len(devices)
    errs = []

    def up(i, d):
        try:
            ops[i] = CsrOperator(A, device=d)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    th = [threading.Thread(target=up, args=(i, d)) for i, d in enumerate(devices)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return ops


def _per_device(name, op, devices):
    """A preconditioner for each device: None, a host matrix (each device's
    Problem uploads it), or one CsrOperator per device in devices order."""
    from .sparse import CsrOperator

    if isinstance(op, (list, tuple)):
        if len(op) != len(devices) or not all(isinstance(a, CsrOperator) and a.device == d
                                               for a, d in zip(op, devices)):
            raise ValueError(f"{name} as a list: one CsrOperator per device, in devices order")
        return list(op)
    if isinstance(op, CsrOperator) and (len(devices) > 1 or op.device != devices[0]):
        raise ValueError(f"devices=[...]: pass {name} as a host matrix (uploaded to every device) or one "
                         "CsrOperator per device")
    return [op] * len(devices)


def solve(method, A, B, devices, x0=None, **kw):
    """The sharded solve of ``method`` ("cg", "gmres", "minres") over
    ``devices``: returns ``(xk or None, Info)`` with ``Info.xk`` the gathered
    global iterate and ``Info.resnorms`` the global history."""
    callback = kw.pop("callback", None)
    devices = [int(d) for d in devices]
    if len(set(devices)) != len(devices) or not devices:
        raise ValueError(f"devices must be distinct device ids, got {devices}")
    B = np.asarray(B)
    vec = B.ndim == 1
    B2 = B[:, None] if vec else B.reshape(B.shape[0], -1)
    K = B2.shape[1]
    D = min(len(devices), K)
    devices = devices[:D]
    per = -(-K // D)
    kcs = [max(0, min(per, K - g * per)) for g in range(D)]
    if min(kcs) < 1:  # fewer columns than per * (D - 1) + 1: use fewer devices
        D = -(-K // per)
        devices, kcs = devices[:D], kcs[:D]
    X0 = None if x0 is None else np.asarray(x0).reshape(B2.shape)

    def local(a, g):
        blk = a[:, g * per:g * per + kcs[g]]
        if kcs[g] < per:
            blk = np.concatenate([blk, np.zeros((a.shape[0], per - kcs[g]), dtype=a.dtype)], axis=1)
        return np.ascontiguousarray(blk)

    ops = _operators(A, devices)
    precs = {name: _per_device(name, kw.pop(name), devices) for name in ("M", "Ml", "Mr") if kw.get(name) is not None}
    for name in ("M", "Ml", "Mr"):
        kw.pop(name, None)
    user_cb = None
    if callback is not None:
        def user_cb(x, second):
            # the single-device call's shapes: b's shape for vectors, the
            # reference's per-column array (a 0-d one for a 1-D b) for norms
            x = x.reshape(B.shape)
            second = np.asarray(second)
            second = second.reshape(B.shape) if second.size == x.size else (
                np.array(second.reshape(-1)[0]) if vec else second.reshape(B.shape[1:]))
            callback(x, second)

        def noop(*_a):
            pass
    comms = ShardComm.all_devices(devices)
    fn = getattr(distributed, method)
    out = [None] * D
    errs = [None] * D

    abort_lock = threading.Lock()
    aborted = []

    def run(g):
        try:
            cb = None if user_cb is None else (user_cb if g == 0 else noop)
            pg = {name: lst[g] for name, lst in precs.items()}
            out[g] = fn(ops[g], local(B2, g), comms[g], x0=None if X0 is None else local(X0, g), kcs=kcs,
                        callback=cb, **pg, **kw)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs[g] = e
            # the other devices may be waiting in a collective this one will
            # never join: abort every communicator so they fail too
            with abort_lock:
                if not aborted:
                    aborted.append(g)
                    for c in comms:
                        try:
                            c.abort()
                        except RuntimeError:
                            pass

    th = [threading.Thread(target=run, args=(g,), name=f"krylov_amd-dev{d}") for g, d in enumerate(devices)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in comms:
        c.close()
    if aborted:  # the device that failed first, not the peers it stopped
        raise errs[aborted[0]]
    info = out[0][1]
    xk = np.concatenate([np.asarray(out[g][1].xk).reshape(B2.shape[0], -1)[:, :kcs[g]] for g in range(D)], axis=1)
    xk = xk.reshape(B.shape)
    info = info._replace(xk=xk)
    if vec:  # a 1-D b: scalar history entries, as the single-device driver's
        info = info._replace(resnorms=[np.asarray(r).reshape(-1)[0] for r in info.resnorms])
    return (xk if info.success else None), info
