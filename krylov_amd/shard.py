"""Host side of right-hand-side sharding: the rank
bookkeeping and the reference's outer loop over a column block split across
ranks. Pure NumPy: no device calls and no communication library of its own,
so the same code runs over RCCL on GPUs (``krylov_amd.distributed``) and over
gloo in the CPU tests (``tests/test_sharding_cpu.py``).

The reference is fully blocked: K columns run K independent recurrences,
coupled only by ``np.all(resnorms[-1] <= criterion)`` over ALL columns
(``cg.py:156,162``, ``gmres.py:193``, ``minres.py:162``) and, for the
Arnoldi/Lanczos methods, the invariance test ``np.all(h[k+1] <= 1e-14)``
(``arnoldi.py:187``, ``arnoldi.py:270-272``). Each rank holds ``kc`` real
columns padded to ``kpad`` on its device; the global vector of a per-column
quantity has ``world * kpad`` slots, rank r owning ``[r kpad, (r+1) kpad)``,
and a zero-padded allreduce (sum) is an all-gather of it.

Per step the device applies the global stop rule itself after one allreduce
(``cg_global_check`` / ``gm_global_check`` / ``mr_global_check``); the host
part here is everything around it: the initial norms, the criterion over the
real columns (padded slots never block the rule: +inf), the explicit
residual recheck, the step count and the global history.
"""
import os
import time

import numpy as np


class ShardLayout:
    """Where this rank's columns sit in the global per-column vectors."""

    def __init__(self, kc, kpad, rank, world, kcs=None):
        """``kc`` device columns per rank (padded to ``kpad``); ``kcs``: the
        real columns of each rank when they differ (an uneven split of K
        columns: every rank holds kc device columns, rank r's first kcs[r]
        real and the rest zero columns that never enter the history or the
        stop rule); default kc on every rank."""
        if not (0 <= rank < world) or kc < 1 or kpad < kc:
            raise ValueError(f"bad shard layout kc={kc} kpad={kpad} rank={rank} world={world}")
        kcs = [int(kc)] * int(world) if kcs is None else [int(c) for c in kcs]
        if len(kcs) != world or any(c < 1 or c > kc for c in kcs):
            raise ValueError(f"bad per-rank column counts {kcs} for kc={kc}, world={world}")
        self.kc, self.kpad, self.rank, self.world = int(kc), int(kpad), int(rank), int(world)
        self.kcs = kcs
        self.total = self.kpad * self.world
        self.off = self.kpad * self.rank
        # global slot of every real column, in rank order (the reference's
        # column order of the unsharded block)
        self.real = np.concatenate([np.arange(r * self.kpad, r * self.kpad + kcs[r]) for r in range(self.world)])

    def glob(self, local_vals, allreduce):
        """This rank's kpad values -> the global vector (zero-padded sum over
        ranks, i.e. an all-gather)."""
        v = np.zeros(self.total)
        v[self.off:self.off + self.kpad] = np.asarray(local_vals, dtype=np.float64)[: self.kpad]
        return np.asarray(allreduce(v), dtype=np.float64)

    def criterion_full(self, criterion):
        """The per-real-column criterion on the global slots; padded slots get
        +inf so they never hold the stop rule back."""
        full = np.full(self.total, np.inf)
        full[self.real] = np.broadcast_to(np.asarray(criterion, dtype=np.float64), self.real.shape)
        return full


def drive(engine, layout, allreduce, tol, atol, maxiter, inner_dtype, chunk=32, hook=None):
    """The reference's outer loop over a sharded block (cg.py:150-234,
    gmres.py:179-234, minres.py:160-236 with the global stop rule).

    ``hook(k, resnorm)``, if given, runs where the reference calls its
    callback: once after the initial norms (k = 0; cg.py:119-120,
    gmres.py:143-144, minres.py:160-161) and after every step (cg.py:202-204,
    gmres.py:226-228, minres.py:230-232), with the global norms of the real
    columns; the chunk is then one step, as on one device.

    ``engine`` is this rank's solver state:
      start_norms()      -> local kpad initial residual norms (float64)
      set_criterion(v)   -> the global criterion vector (layout.total)
      run(steps)         -> (rows, invariant): the global history rows
                            (done x layout.total) of a chunk that stops itself
                            after the first step meeting the global rule
      residual_norm2()   -> local kpad squared explicit residual norms
    Returns ``(success, numsteps, resnorms)`` with the global history over the
    real columns, identical on every rank."""
    real = layout.real

    def cast(v):
        return np.asarray(v, dtype=np.float64).astype(inner_dtype).astype(np.float64)

    rn0 = layout.glob(engine.start_norms(), allreduce)
    resnorms = [cast(rn0[real])]
    criterion = np.maximum(tol * resnorms[0], atol)
    engine.set_criterion(layout.criterion_full(criterion))
    if hook is not None:
        hook(0, resnorms[0])
        chunk = 1
    k = 0
    success = False
    while True:
        if np.all(resnorms[-1] <= criterion):
            sq = layout.glob(engine.residual_norm2(), allreduce)
            resnorms[-1] = np.sqrt(sq[real].astype(inner_dtype)).astype(np.float64)
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        # an invariant step is not a stop by itself (the reference's drivers
        # do not test it either: its residual meets the rule, or the next
        # Arnoldi/Lanczos step raises)
        rows, _ = engine.run(min(chunk, maxiter - k))
        if len(rows) == 0:
            raise RuntimeError("sharded solve: a chunk made no progress")
        for row in rows:
            resnorms.append(cast(np.asarray(row)[real]))
            k += 1
        if hook is not None:
            hook(k, resnorms[-1])
    return success, k, resnorms


# ------------------------------------------------------------ rendezvous
def file_rendezvous(path, rank, payload_fn, timeout=120.0, poll=0.02):
    """Torch-free exchange of the communicator's unique id: rank 0 writes
    ``payload_fn()`` (bytes) to ``path`` atomically (temporary file + rename),
    every other rank polls until it appears. ``path`` must be on a file system
    all ranks see (one node: /tmp or /dev/shm) and fresh for every job."""
    if rank == 0:
        data = bytes(payload_fn())
        tmp = f"{path}.tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(data)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
        return data
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as f:
                data = f.read()
            if data:
                return data
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rank {rank}: no communicator id at {path} after {timeout:.0f} s")
        time.sleep(poll)
