"""Preconditioned CG driver (reference ``cg.py:16-259``) over the device loop.

The loop structure, stop rule, explicit-residual recheck and ``Info`` record
are the reference's; every iteration's arithmetic (SpMV, inner products, the
x/r/p updates and the scalar recurrences) runs on the GPU through
``kry_cg_run`` in chunks of up to ``kry_cg_preferred_chunk`` iterations (32;
256 on the persistent small-n loop) with one host sync per chunk. The device stops a chunk right after the first iteration whose
residual norms satisfy the criterion, so the host sees exactly the
iterations the reference performs.
"""
import ctypes
import time

import numpy as np

from . import _helpers, _lib
from ._helpers import Info, Problem
from .device import HostOut
from ._lib import check, lib


# host-clock split of the last cg() call on the device path: the whole call
# and the part spent inside the chunked device loop (kry_cg_run calls); the
# difference is the call's fixed cost at the host-array boundary (bench.py
# end_to_end)
last_timing = {}


class _CGState:
    def __init__(self, prob):
        self.prob = prob
        h = ctypes.c_void_p()
        check(lib.kry_cg_create(prob.ctx.handle, prob.A.handle, prob.kpad, _lib.dtype_code(prob.dtype), ctypes.byref(h)))
        self.h = h
        self._fin = _lib.own(self, lib.kry_cg_destroy, h)
        if prob.ops["Mr"] is not None:
            raise TypeError("cg has no right preconditioner Mr")
        if prob.has_precond():
            check(lib.kry_cg_set_preconditioners(h, *prob.op_handles("M", "Ml")))

    def start(self):
        p = self.prob
        rho = np.zeros(p.kpad)
        check(lib.kry_cg_start(self.h, p.b_dev.handle, p.x0_dev.handle if p.x0_dev else None,
                               p.w_dev.handle if p.w_dev else None, _lib.dptr(rho)))
        return rho

    def set_criterion(self, crit):
        crit = np.ascontiguousarray(crit, dtype=np.float64)
        check(lib.kry_cg_set_criterion(self.h, _lib.dptr(crit)))

    def run(self, steps, ncols=None):
        ncols = self.prob.kpad if ncols is None else ncols
        out = np.zeros((max(steps, 1), ncols))
        done = ctypes.c_int32()
        check(lib.kry_cg_run(self.h, int(steps), ctypes.byref(done), _lib.dptr(out)))
        return out[: done.value]

    def preferred_chunk(self):
        """Iterations per run call (after start): 256 on the persistent
        small-n loop, 32 on the launch-per-pass path."""
        n = ctypes.c_int32()
        check(lib.kry_cg_preferred_chunk(self.h, ctypes.byref(n)))
        return n.value

    def path(self):
        """(persistent, fallbacks): whether the last run chunk was one
        persistent launch, and how many chunks were rerun launch per pass
        after an in-launch exchange timed out (kry_cg_path)."""
        info = (ctypes.c_int32 * 2)()
        check(lib.kry_cg_path(self.h, info))
        return bool(info[0]), int(info[1])

    def update_path(self):
        """(path, fallbacks) of the launch-per-pass form (kry_cg_update_path):
        path 1 (== True) = the one-launch update (k = 1), 0 (== False) =
        separate passes."""
        info = (ctypes.c_int32 * 2)()
        check(lib.kry_cg_update_path(self.h, info))
        return int(info[0]), int(info[1])

    def defer_info(self):
        """(D, bytes): yk updates applied D steps at a time (0 = every step)
        and the device memory its ring buffers hold (kry_cg_defer_info)."""
        d, nb = ctypes.c_int32(), ctypes.c_int64()
        check(lib.kry_cg_defer_info(self.h, ctypes.byref(d), ctypes.byref(nb)))
        return int(d.value), int(nb.value)

    def residual_norm2(self):
        out = np.zeros(self.prob.kpad)
        check(lib.kry_cg_residual(self.h, _lib.dptr(out)))
        return out

    def get(self, which, out=None):
        p = self.prob
        if out is None:
            out = np.empty((p.n, p.kpad), dtype=p.dtype)
        assert out.shape == (p.n, p.kpad) and out.dtype == p.dtype and out.flags.c_contiguous
        check(lib.kry_cg_get(self.h, which, _lib.ptr(out)))
        return out

    def scalars(self):
        """[rho, rho_prev, alpha, omega] rows (kpad values each)."""
        out = np.zeros((4, self.prob.kpad))
        check(lib.kry_cg_scalars(self.h, _lib.dptr(out)))
        return out


def _norm_from_sq(prob, sq):
    return np.sqrt(np.asarray(sq[: prob.kc]).astype(prob.inner_dtype))


def cg(A, b, M=None, Ml=None, inner=None, x0=None, tol=1e-5, atol=1.0e-15, maxiter=None,
       return_arnoldi=False, callback=None, *, devices=None):
    """Preconditioned CG, reference signature (``cg.py:16-28``).

    ``A``: ``krylov_amd.CsrOperator``, scipy.sparse matrix or dense ndarray
    (uploaded once as CSR). ``inner``: ``None`` or ``WeightedInner``.
    ``M``/``Ml``: ``None``/``Identity`` or an operator of the same kinds as
    ``A`` (applied on the device as SpMVs, cg.py:70-90, 180, 207).
    ``devices=[...]``: split the columns of a block ``b`` over these GPUs of
    this process (``krylov_amd.multi``: one RCCL allreduce per iteration, the
    global iterate gathered), the same steps and history as one device.
    """
    if devices is not None:
        if return_arnoldi:
            raise NotImplementedError("devices=[...] does not return the Lanczos relation")
        from .multi import solve

        return solve("cg", A, b, devices, x0=x0, tol=tol, atol=atol, maxiter=maxiter, callback=callback, M=M,
                     Ml=Ml, inner=inner)
    t_call = time.perf_counter()
    t_run = 0.0
    prob = Problem(A, b, x0, inner, M=M, Ml=Ml)
    t_prob = time.perf_counter()
    N = prob.A.shape[0]
    maxiter = N if maxiter is None else maxiter

    st = _CGState(prob)
    x_out = HostOut((prob.n, prob.kpad), prob.dtype)  # pages faulted in while the device iterates
    rho0 = st.start()
    t_start = time.perf_counter()
    chunk = st.preferred_chunk()
    rn0 = _norm_from_sq(prob, rho0)
    if callback is not None:
        callback(prob.x0_or_zeros(), prob.unpad_vec(st.get(1), prob.r0_dtype))
    resnorms = [prob.colvals(rn0)]
    criterion = np.maximum(tol * resnorms[0], atol)
    st.set_criterion(prob.pad_cols(criterion, np.inf))
    lanczos = _Lanczos(prob, st, resnorms[0], maxiter) if return_arnoldi else None

    k = 0
    success = False
    while True:
        if np.all(resnorms[-1] <= criterion):
            # the reference's explicit residual recheck (cg.py:156-164)
            resnorms[-1] = prob.colvals(_norm_from_sq(prob, st.residual_norm2()))
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        steps = 1 if (callback is not None or lanczos is not None) else min(chunk, maxiter - k)
        t0 = time.perf_counter()
        hist = st.run(steps)
        t_run += time.perf_counter() - t0
        for row in hist:
            resnorms.append(prob.colvals(row))
            if lanczos is not None:
                lanczos.step(k, resnorms[-1])
            k += 1
        if callback is not None and len(hist):
            callback(prob.unpad_vec(st.get(0), prob.r0_dtype), prob.unpad_vec(st.get(1), prob.r0_dtype))

    t_loop = time.perf_counter()
    xk = prob.unpad_vec(st.get(0, out=x_out.take()), prob.r0_dtype)
    t_get = time.perf_counter()
    num_operations = {
        "A": 1 + k,
        "M": 2 + k,
        "Ml": 2 + k,
        "Mr": 1 + k,
        "inner": 2 + 2 * k,
        "axpy": 2 + 2 * k,
    }
    arnoldi = lanczos.result(k) if lanczos is not None else None
    t_end = time.perf_counter()
    last_timing.update(call_ms=1e3 * (t_end - t_call), chunks_ms=1e3 * t_run, problem_ms=1e3 * (t_prob - t_call),
                       setup_start_ms=1e3 * (t_start - t_prob), loop_host_ms=1e3 * (t_loop - t_start - t_run),
                       get_ms=1e3 * (t_get - t_loop), finish_ms=1e3 * (t_end - t_get))
    return xk if success else None, Info(success, xk, k, resnorms, num_operations=num_operations, arnoldi=arnoldi,
                                         renumbered=prob.A.renumbered)


class _Lanczos:
    """The Lanczos relation CG returns with ``return_arnoldi`` (cg.py:140-148,
    218-233): V_k = (-1)^k M Ml r_k / ||.||, P_k the same with Ml r_k, and the
    tridiagonal H built from alpha, omega and the rho ratios read back from the
    device after every step (one step per run in this mode)."""

    def __init__(self, prob, st, norm0, maxiter):
        self.prob, self.st = prob, st
        nz = np.where(np.asarray(norm0) > 0.0, norm0, 1.0)
        self.V = [self._vec(2) / nz]
        self.P = [self._vec(1) / nz]
        self.H = np.zeros([maxiter + 1, maxiter] + list(prob.tail), dtype=float)
        self.alpha_old = 0
        self.omega = None

    def _vec(self, which):
        return self.prob.unpad_vec(self.st.get(which), self.prob.r0_dtype)

    def _sc(self, row):
        return self.prob.colvals(row)

    def step(self, k, norm):
        rho, rho_prev, alpha, omega_next = (self._sc(r) for r in self.st.scalars())
        sign = (-1) ** (k + 1)
        self.V.append(sign * self._vec(2) / norm)
        self.P.append(sign * self._vec(1) / norm)
        H = self.H
        H[k, k] = 1.0 / alpha
        if k > 0:
            H[k - 1, k] = H[k, k - 1]
            H[k, k] += self.omega / self.alpha_old
        H[k + 1, k] = np.sqrt(rho / rho_prev) / alpha
        self.alpha_old = alpha
        self.omega = omega_next  # the omega of the next iteration's p update (cg.py:177)

    def result(self, k):
        return [self.V, self.H[: k + 1, :k], self.P]
