"""Preconditioned MINRES driver (reference ``minres.py:28-253``) over the
device loop: Lanczos (arnoldi.py:203-281), the two-rotation QR update, the
three-term direction recurrence and the x update run on the GPU
(``kry_minres_*``), in chunks with one host sync per chunk.
"""
import ctypes

import numpy as np

from . import _helpers, _lib
from ._helpers import Info, Problem
from .device import HostOut
from ._lib import check, lib


class _MinresState:
    def __init__(self, prob):
        self.prob = prob
        h = ctypes.c_void_p()
        check(lib.kry_minres_create(prob.ctx.handle, prob.A.handle, prob.kpad, _lib.dtype_code(prob.dtype),
                                    ctypes.byref(h)))
        self.h = h
        self._fin = _lib.own(self, lib.kry_minres_destroy, h)
        if prob.has_precond():
            check(lib.kry_minres_set_preconditioners(h, *prob.op_handles("M", "Ml", "Mr")))

    def start(self):
        p = self.prob
        out = np.zeros(p.kpad)
        check(lib.kry_minres_start(self.h, p.b_dev.handle, p.x0_dev.handle if p.x0_dev else None,
                                   p.w_dev.handle if p.w_dev else None, _lib.dptr(out)))
        return out

    def set_criterion(self, crit):
        crit = np.ascontiguousarray(crit, dtype=np.float64)
        check(lib.kry_minres_set_criterion(self.h, _lib.dptr(crit)))

    def run(self, steps):
        out = np.zeros((max(steps, 1), self.prob.kpad))
        done = ctypes.c_int32()
        inv = ctypes.c_int32()
        check(lib.kry_minres_run(self.h, int(steps), ctypes.byref(done), _lib.dptr(out), ctypes.byref(inv)))
        return out[: done.value], bool(inv.value)

    def update_path(self):
        """(one_launch_tail, fallbacks) of the last run chunk
        (kry_minres_update_path)."""
        info = (ctypes.c_int32 * 2)()
        check(lib.kry_minres_update_path(self.h, info))
        return bool(info[0]), int(info[1])

    def residual_norm2(self):
        out = np.zeros(self.prob.kpad)
        check(lib.kry_minres_residual(self.h, _lib.dptr(out)))
        return out

    def xk(self, out=None):
        p = self.prob
        if out is None:
            out = np.empty((p.n, p.kpad), dtype=p.dtype)
        assert out.shape == (p.n, p.kpad) and out.dtype == p.dtype and out.flags.c_contiguous
        check(lib.kry_minres_get(self.h, 0, _lib.ptr(out)))
        return p.unpad_vec(out, p.r0_dtype)


def lanczos(A, v, maxiter, M=None, inner=None):
    """The device Lanczos process of ``minres`` on its own (``ArnoldiLanczos``,
    ``arnoldi.py:203-281``): up to ``maxiter`` steps from ``v``, stopping at an
    invariant subspace. Returns ``(V, H, P, is_invariant)`` with the bases as
    lists of vectors and the (steps + 1) x steps tridiagonal H (steps x steps
    after an invariant step), as tests/test_arnoldi.py assembles them."""
    v = np.asarray(v)
    if v.ndim != 1:
        raise ValueError("lanczos takes one start vector")
    prob = Problem(A, v, None, inner, M=M)
    st = _MinresState(prob)
    st.start()
    st.set_criterion(prob.pad_cols(np.full(prob.kc, -1.0), np.inf))  # never "converged"

    def vec(which):
        out = np.empty((prob.n, prob.kpad), dtype=prob.dtype)
        check(lib.kry_minres_get(st.h, which, _lib.ptr(out)))
        return out[:, 0].copy()

    V, P, cols = [vec(2)], [vec(1)], []
    prev_h2 = 0.0
    invariant = False
    for _ in range(maxiter):
        hist, invariant = st.run(1)
        if len(hist) == 0:
            break
        h = np.empty((3, prob.kpad))
        check(lib.kry_minres_get(st.h, 3, _lib.dptr(h)))
        cols.append(np.array([prev_h2, h[1, 0], h[2, 0]]))
        prev_h2 = h[2, 0]
        if invariant:
            break
        V.append(vec(2))
        P.append(vec(1))
    k = len(cols)
    H = np.zeros((k + 1, k))
    for i, hv in enumerate(cols):
        if i == 0:
            H[:2, 0] = hv[1:]
        else:
            H[i - 1:i + 2, i] = hv
    if invariant:
        H = H[:k]
    return V, H.astype(prob.dtype), P, invariant


def minres(A, b, M=None, Ml=None, Mr=None, inner=None, x0=None, tol=1e-5, atol=1.0e-15, maxiter=None,
           callback=None, *, devices=None):
    """Preconditioned MINRES, reference signature (``minres.py:28-40``).
    ``devices=[...]``: the columns of a block ``b`` over several GPUs of this
    process (``krylov_amd.multi``)."""
    if devices is not None:
        from .multi import solve

        return solve("minres", A, b, devices, x0=x0, inner=inner, tol=tol, atol=atol, maxiter=maxiter,
                     callback=callback, M=M, Ml=Ml, Mr=Mr)
    prob = Problem(A, b, x0, inner, M=M, Ml=Ml, Mr=Mr)
    N = prob.A.shape[0]
    maxiter = N if maxiter is None else maxiter

    st = _MinresState(prob)
    host_out = HostOut((prob.n, prob.kpad), prob.dtype)  # pages faulted in while the device iterates
    rn0 = st.start()
    first = prob.colvals(rn0)
    if callback is not None:
        callback(prob.x0_or_zeros(), np.array(first))
    resnorms = [first]
    criterion = np.maximum(tol * resnorms[0], atol)
    st.set_criterion(prob.pad_cols(criterion, np.inf))

    k = 0
    success = False
    while True:
        if np.all(resnorms[-1] <= criterion):
            sq = st.residual_norm2()
            resnorms[-1] = prob.colvals(np.sqrt(np.asarray(sq[: prob.kc]).astype(prob.inner_dtype)))
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        steps = 1 if callback is not None else min(_helpers.CHUNK, maxiter - k)
        hist, _ = st.run(steps)
        for row in hist:
            resnorms.append(prob.colvals(row))
            k += 1
        if callback is not None and len(hist):
            callback(st.xk(), np.array(resnorms[-1]))

    xk = st.xk(out=host_out.take())
    num_operations = {
        "A": 1 + k,
        "M": 2 + k,
        "Ml": 2 + k,
        "Mr": 1 + k,
        "inner": 2 + 2 * k,
        "axpy": 4 + 8 * k,
    }
    return xk if success else None, Info(success, xk, k, resnorms, num_operations=num_operations, renumbered=prob.A.renumbered)
