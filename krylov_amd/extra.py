"""The reference's other Krylov solvers on the device:
``bicgstab`` (bicgstab.py:24-144), ``cgs`` (cgs.py:24-117), ``cgr``
(cgr.py:16-100) and ``gcr`` (gcr.py:18-97).

They share the SpMV + inner product + AXPY loop shape of CG. The host runs
the reference's control flow; the arithmetic of an iteration is enqueued on
the device with no host round trip (``kry_prog_*``, a device-resident scalar
chain): every SpMV is the device SpMV, every inner product reduces into a
device register, every scalar line of the reference (``beta = rho * alpha /
where(...)``, ...) evaluates on registers in float64 as the host evaluated
it, every AXPY-type line is one lincomb launch reading its coefficients from
registers, and the convergence tests run on the device and stop the chunk.
A chunk of iterations costs one host sync (callbacks: one iteration per
chunk). Signatures, control flow and quirks follow the reference line by
line (e.g. bicgstab's mid-step convergence test on the explicit residual of
the *previous* iterate, bicgstab.py:123-127, stops the chunk in the middle
of a step and replaces the last history entry, as there).
"""
import ctypes

import numpy as np

from . import _helpers, _lib
from ._helpers import Info, Problem
from ._lib import check, lib
from .device import DeviceVector, HostOut

LC_AXPY, LC_NEST_ADD, LC_NEST_SUB, LC_DIV, LC_SUB, LC_ADD, LC_COPY, LC_SCALE = range(8)
SOP_COPY, SOP_DIVG, SOP_MULDIVG, SOP_SQRT, SOP_GUARD, SOP_SET = range(6)
class _Dev:
    """Device vectors of one solve (n x kpad blocks) and the primitives."""

    def __init__(self, prob):
        if prob.kpad > 64:
            raise NotImplementedError("at most 64 right-hand-side columns on bicgstab / cgs / cgr / gcr")
        self.prob = prob
        self.ctx = prob.ctx
        # the chain's vectors live in the operator's numbering (a renumbered
        # A: b and the weights moved in once; uploads and downloads move rows)
        self.renumbered = prob.A.renumbered
        self.b = self._to_op(prob.b_dev)
        self.w = None if prob.w_dev is None else self._to_op(prob.w_dev)
        self.out = HostOut((prob.n, prob.kpad), prob.dtype)  # the returned iterate's pages, faulted in meanwhile

    def _to_op(self, v):
        if not self.renumbered:
            return v
        t = DeviceVector(self.ctx, v.n, v.k, v.dtype)
        self.prob.A.permute(v, t, True)
        return t

    def _from_op(self, v):
        if not self.renumbered:
            return v
        t = DeviceVector(self.ctx, v.n, v.k, v.dtype)
        self.prob.A.permute(v, t, False)
        return t

    def zeros(self):
        v = DeviceVector(self.ctx, self.prob.n, self.prob.kpad, self.prob.dtype)
        return v

    def upload(self, a):
        v = self.zeros()
        v.upload(self.prob.pad(np.asarray(a).astype(self.prob.dtype, copy=False)))
        return self._to_op(v)

    def host(self, v):
        return self.prob.unpad_vec(self._from_op(v).to_host(), self.prob.r0_dtype)

    def host_final(self, v):
        """The returned iterate, into the array allocated at the start."""
        return self.prob.unpad_vec(self._from_op(v).to_host(out=self.out.take()), self.prob.r0_dtype)

    def matvec(self, op, x):
        """op @ x into a new vector; op None = the reference's Identity (x itself)."""
        if op is None:
            return x
        y = self.zeros()
        op.matvec_op(x, y)
        return y

    def A(self, x):
        return self.matvec(self.prob.A, x)

    def op(self, name, x):
        return self.matvec(self.prob.ops[name], x)

    def dot(self, x, y):
        """The reference's inner(x, y) per column (kpad float64 values)."""
        out = np.zeros(self.prob.kpad)
        check(lib.kry_dot(self.ctx.handle, x.handle, y.handle, self.w.handle if self.w else None, _lib.dptr(out)))
        return out

    def lc(self, form, x, y=None, w=None, a=None, b=None, out=None):
        z = self.zeros() if out is None else out
        kp = self.prob.kpad
        aa = None if a is None else np.ascontiguousarray(np.broadcast_to(np.asarray(a, dtype=np.float64), (kp,)))
        bb = None if b is None else np.ascontiguousarray(np.broadcast_to(np.asarray(b, dtype=np.float64), (kp,)))
        check(lib.kry_vec_lincomb(self.ctx.handle, form, z.handle, x.handle, None if y is None else y.handle,
                                  None if w is None else w.handle, None if aa is None else _lib.dptr(aa),
                                  None if bb is None else _lib.dptr(bb)))
        return z

    def copy(self, x):
        return self.lc(LC_COPY, x)

    def residual(self, x):
        """b - A @ x."""
        return self.lc(LC_SUB, self.b, self.A(x))

    def cols(self, v):
        """kpad per-column values -> the reference's scalar / (k,) array."""
        return self.prob.colvals(v)


class _Chain:
    """A device register file of named per-column float64 scalars and the
    chunk control of one solve (``kry_prog``); every method enqueues work for
    chunk step ``st`` without a host sync."""

    def __init__(self, D, names, cap=_helpers.CHUNK):
        self.D = D
        self.r = {nm: i for i, nm in enumerate(names)}
        self.kp = D.prob.kpad
        self.cap = cap
        h = ctypes.c_void_p()
        check(lib.kry_prog_create(D.ctx.handle, len(names), self.kp, cap, ctypes.byref(h)))
        self.h = h
        self._fin = _lib.own(self, lib.kry_prog_destroy, h)
        self.r32 = 4 if D.prob.inner_dtype == np.float32 else 0

    def set(self, name, vals):
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(vals, dtype=np.float64), (self.kp,)))
        check(lib.kry_prog_set(self.h, -1 if name is None else self.r[name], _lib.dptr(v)))

    def get(self, name):
        out = np.zeros(self.kp)
        check(lib.kry_prog_get(self.h, self.r[name], _lib.dptr(out)))
        return out

    def begin(self):
        check(lib.kry_prog_begin(self.h))

    def end(self, steps):
        """(rows of the steps that ran, midstep row or None)."""
        rows = np.zeros((steps + 1, self.kp))
        done, mid = ctypes.c_int32(), ctypes.c_int32()
        check(lib.kry_prog_end(self.h, int(steps), ctypes.byref(done), ctypes.byref(mid), _lib.dptr(rows)))
        d = done.value
        return rows[:d], (rows[d] if mid.value else None)

    def sc(self, op, d, st, a=None, b=None, c=None, e=None, value=0.0):
        ix = [self.r[x] if x is not None else 0 for x in (d, a, b, c, e)]
        check(lib.kry_prog_scalar(self.h, op, *ix, float(value), st))

    def dot(self, x, y, d, st):
        w = self.D.w
        check(lib.kry_prog_dot(self.h, x.handle, y.handle, w.handle if w else None, self.r[d], st))

    def lc(self, form, z, x, st, y=None, w=None, a=None, sa=1.0, b=None, sb=1.0):
        check(lib.kry_prog_lincomb(self.h, form, z.handle, x.handle, None if y is None else y.handle,
                                   None if w is None else w.handle, -1 if a is None else self.r[a], sa,
                                   -1 if b is None else self.r[b], sb, st))
        return z

    def spmv(self, op, x, y, st):
        check(lib.kry_prog_spmv(self.h, op.handle, x.handle, y.handle, st))
        return y

    def apply(self, name, x, out, st):
        """op @ x into `out` (the reference's Identity: x itself)."""
        op = self.D.prob.ops[name]
        return x if op is None else self.spmv(op, x, out, st)

    def norm(self, v, tmp, d, st, M=None):
        """d = sqrt(<v, M v>) (M None: <v, v>)."""
        mv = v if M is None else self.apply(M, v, tmp, st)
        self.dot(v, mv, d, st)
        self.sc(SOP_SQRT, d, st, a=d)

    def check(self, d, st, mode=0):
        check(lib.kry_prog_check(self.h, self.r[d], mode | (self.r32 if mode == 0 else 0), st))


def _chunks(D, callback):
    """Iterations per chunk: one with a callback (it sees every iterate)."""
    return 1 if callback is not None else _helpers.CHUNK


def _real(v):
    v = np.asarray(v)
    if np.any(np.asarray(v).imag != 0.0):
        raise ValueError("inner product <x, x> gave nonzero imaginary part")
    return v.real


def _guard(d):
    return np.where(d != 0.0, d, 1.0)


def _start(D, x0):
    """x and r0 as the reference sets them up (x0 None: x = 0, r0 = b copy)."""
    prob = D.prob
    if x0 is None:
        x = D.zeros()
        r0 = D.copy(D.b)
    else:
        x = D.upload(x0)
        r0 = D.residual(x)
    return x, r0


def bicgstab(A, b, Ml=None, Mr=None, x0=None, inner=None, tol=1e-5, atol=1.0e-15, maxiter=None, callback=None):
    """BiCGSTAB, reference signature and iteration (bicgstab.py:24-144)."""
    prob = Problem(A, b, x0, inner, Ml=Ml, Mr=Mr)
    D = _Dev(prob)

    def norm(v):  # bicgstab.py:47-51
        return np.sqrt(_real(D.dot(v, D.op("Ml", v))))

    x, r0 = _start(D, x0)
    r0_ = r0
    r = D.copy(r0)
    if callback is not None:
        callback(D.host(x), D.host(r))
    resnorms = [D.cols(norm(r0))]
    C = _Chain(D, ["rho", "rho_old", "alpha", "omega", "beta", "r0v", "tt", "ts", "nh", "nr"])
    for nm in ("rho", "alpha", "omega"):
        C.set(nm, 1.0)
    p, v = D.zeros(), D.zeros()
    s_, h, t, rx = D.zeros(), D.zeros(), D.zeros(), D.zeros()
    ml = prob.ops["Ml"] is not None
    mr = prob.ops["Mr"] is not None
    t1, t2, t3, t4, t5 = ([D.zeros() for _ in range(5)] if (ml or mr) else [None] * 5)
    criterion = np.maximum(tol * resnorms[0], atol)
    C.set(None, prob.pad_cols(criterion, np.inf))

    def step(st):
        C.sc(SOP_COPY, "rho_old", st, a="rho")
        C.dot(r0_, r, "rho", st)  # rho = inner(r0_, r)
        C.sc(SOP_MULDIVG, "beta", st, a="rho", b="alpha", c="rho_old", e="omega")
        C.lc(LC_NEST_SUB, p, r, st, y=p, w=v, a="beta", b="omega")  # p = r + beta (p - omega v)
        y = C.apply("Mr", C.apply("Ml", p, t1, st), t2, st)
        C.spmv(prob.A, y, v, st)  # v = A y
        C.dot(r0_, v, "r0v", st)
        C.sc(SOP_DIVG, "alpha", st, a="rho", b="r0v")
        C.lc(LC_AXPY, s_, r, st, y=v, a="alpha", sa=-1.0)  # s = r - alpha v
        C.lc(LC_AXPY, h, x, st, y=y, a="alpha")  # h = x + alpha y
        # resnorm_h = _norm(Ml (b - A x)) of the previous iterate x (bicgstab.py:123)
        C.spmv(prob.A, x, rx, st)
        C.lc(LC_SUB, rx, D.b, st, y=rx)
        C.norm(C.apply("Ml", rx, t3, st), t4, "nh", st, M="Ml" if ml else None)
        C.check("nh", st, mode=1)
        ml_s = C.apply("Ml", s_, t3, st)
        z = C.apply("Mr", ml_s, t5, st)
        C.spmv(prob.A, z, t, st)
        ml_t = C.apply("Ml", t, t4, st)
        C.dot(ml_t, ml_t, "tt", st)
        C.dot(ml_t, ml_s, "ts", st)
        C.sc(SOP_DIVG, "omega", st, a="ts", b="tt")
        C.lc(LC_AXPY, x, h, st, y=z, a="omega")  # x = h + omega z
        C.lc(LC_AXPY, r, s_, st, y=t, a="omega", sa=-1.0)  # r = s - omega t
        C.norm(r, t1 if ml else None, "nr", st, M="Ml" if ml else None)
        C.check("nr", st)

    k = 0
    success = False
    while True:
        if np.all(resnorms[-1] <= criterion):
            resnorms[-1] = D.cols(norm(D.residual(x)))
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        steps = _chunks(D, callback) if maxiter is None else min(_chunks(D, callback), maxiter - k)
        C.begin()
        for st in range(steps):
            step(st)
        rows, mid = C.end(steps)
        for row in rows:
            if callback is not None:
                callback(D.host(x), D.host(r))
            resnorms.append(D.cols(row))
            k += 1
        if mid is not None:  # bicgstab.py:124-127
            resnorms[-1] = D.cols(mid)
            success = True
            break
    xk = D.host_final(x)
    return xk if success else None, Info(success, xk, k, resnorms, renumbered=prob.A.renumbered)


def cgs(A, b, M=None, x0=None, inner=None, tol=1e-5, atol=1.0e-15, maxiter=None, callback=None):
    """CGS, reference signature and iteration (cgs.py:24-117)."""
    prob = Problem(A, b, x0, inner, M=M)
    D = _Dev(prob)
    mm = prob.ops["M"] is not None

    def norm(v):  # cgs.py:44-48
        return np.sqrt(_real(D.dot(v, D.op("M", v))))

    x, r0 = _start(D, x0)
    rp = r0
    r = D.copy(r0)
    if callback:
        callback(D.host(x), D.host(r))
    resnorms = [D.cols(norm(r))]
    C = _Chain(D, ["rho", "rho_old", "beta", "s", "alpha", "nr"])
    C.set("rho", 1.0)
    p, q, u, v, uq, au = (D.zeros() for _ in range(6))
    t1, t2 = (D.zeros(), D.zeros()) if mm else (None, None)
    criterion = np.maximum(tol * resnorms[0], atol)
    C.set(None, prob.pad_cols(criterion, np.inf))

    def step(st):
        C.sc(SOP_COPY, "rho_old", st, a="rho")
        C.dot(rp, r, "rho", st)
        C.sc(SOP_DIVG, "beta", st, a="rho", b="rho_old")
        C.lc(LC_AXPY, u, r, st, y=q, a="beta")  # u = r + beta q
        C.lc(LC_NEST_ADD, p, u, st, y=q, w=p, a="beta", b="beta")  # p = u + beta (q + beta p)
        C.spmv(prob.A, C.apply("M", p, t1, st), v, st)  # v = A M p
        C.dot(rp, v, "s", st)
        C.sc(SOP_DIVG, "alpha", st, a="rho", b="s")
        C.lc(LC_AXPY, q, u, st, y=v, a="alpha", sa=-1.0)  # q = u - alpha v
        C.lc(LC_ADD, uq, u, st, y=q)
        u_ = C.apply("M", uq, t2, st)  # u_ = M (u + q)
        C.lc(LC_AXPY, x, x, st, y=u_, a="alpha")
        C.spmv(prob.A, u_, au, st)
        C.lc(LC_AXPY, r, r, st, y=au, a="alpha", sa=-1.0)
        C.norm(r, t1 if mm else None, "nr", st, M="M" if mm else None)
        C.check("nr", st)

    k = 0
    success = False
    while True:
        if np.all(resnorms[-1] <= criterion):
            resnorms[-1] = D.cols(norm(D.residual(x)))
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        steps = _chunks(D, callback) if maxiter is None else min(_chunks(D, callback), maxiter - k)
        C.begin()
        for st in range(steps):
            step(st)
        rows, _ = C.end(steps)
        for row in rows:
            if callback:
                callback(D.host(x), D.host(r))
            resnorms.append(D.cols(row))
            k += 1
    xk = D.host_final(x)
    return xk if success else None, Info(success, xk, k, resnorms, renumbered=prob.A.renumbered)


def cgr(A, b, M=None, x0=None, inner=None, tol=1e-5, atol=1.0e-15, maxiter=None, callback=None):
    """Conjugate residual, reference signature and iteration (cgr.py:16-100)."""
    prob = Problem(A, b, x0, inner, M=M)
    D = _Dev(prob)
    if x0 is None:
        x = D.zeros()
        r = D.copy(D.b)
    else:
        x = D.upload(x0)
        r = D.residual(x)
    r = D.op("M", r)

    def norm(v):  # cgr.py:47-51 (no M)
        return np.sqrt(_real(D.dot(v, v)))

    Ar = D.A(r)
    C = _Chain(D, ["rAr", "rAr_old", "ApMAp", "alpha", "beta", "nr"])
    C.set("rAr", D.dot(r, Ar))
    resnorms = [D.cols(norm(r))]
    if callback is not None:
        callback(D.host(x), D.host(r))
    p = D.copy(r)
    Ap = D.copy(Ar)
    mAp = D.zeros() if prob.ops["M"] is not None else None
    criterion = np.maximum(tol * resnorms[0], atol)
    C.set(None, prob.pad_cols(criterion, np.inf))

    def step(st):
        MAp = C.apply("M", Ap, mAp, st)
        C.dot(Ap, MAp, "ApMAp", st)
        C.sc(SOP_DIVG, "alpha", st, a="rAr", b="ApMAp")
        C.lc(LC_AXPY, x, x, st, y=p, a="alpha")
        C.lc(LC_AXPY, r, r, st, y=MAp, a="alpha", sa=-1.0)
        C.spmv(prob.A, r, Ar, st)
        C.sc(SOP_COPY, "rAr_old", st, a="rAr")
        C.dot(r, Ar, "rAr", st)
        C.sc(SOP_DIVG, "beta", st, a="rAr", b="rAr_old")
        C.lc(LC_AXPY, p, r, st, y=p, a="beta")  # p = r + beta p
        C.lc(LC_AXPY, Ap, Ar, st, y=Ap, a="beta")  # Ap = Ar + beta Ap
        C.norm(r, None, "nr", st)
        C.check("nr", st)

    k = 0
    success = False
    while True:
        if np.all(resnorms[-1] <= criterion):
            resnorms[-1] = D.cols(norm(D.residual(x)))
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        steps = _chunks(D, callback) if maxiter is None else min(_chunks(D, callback), maxiter - k)
        C.begin()
        for st in range(steps):
            step(st)
        rows, _ = C.end(steps)
        for row in rows:
            if callback is not None:
                callback(D.host(x), D.host(r))
            resnorms.append(D.cols(row))
            k += 1
    xk = D.host_final(x)
    return xk if success else None, Info(success, xk, k, resnorms, renumbered=prob.A.renumbered)


# gcr's basis grows by two n x k vectors per step; a chunk enqueued before its
# stop test allocates them all up front, so chunks are cut to this many bytes
# of new basis (at n = 1e7 fp64: 12 steps instead of 32)
_GCR_CHUNK_BYTES = 2 << 30


def gcr(A, b, x0=None, inner=None, tol=1e-5, atol=1.0e-15, maxiter=None, callback=None):
    """Generalised conjugate residual with MGS (gcr.py:18-97)."""
    prob = Problem(A, b, x0, inner)
    D = _Dev(prob)
    if x0 is None:
        x = D.zeros()
        r = D.copy(D.b)
    else:
        x = D.upload(x0)
        r = D.residual(x)

    def norm(v):
        return np.sqrt(_real(D.dot(v, v)))

    if callback is not None:
        callback(D.host(x), D.host(r))
    resnorms = [D.cols(norm(r))]
    C = _Chain(D, ["alpha", "beta", "gb", "gamma", "nr"])
    s, v = [], []
    criterion = np.maximum(tol * resnorms[0], atol)
    C.set(None, prob.pad_cols(criterion, np.inf))

    def step(st, kk):
        s.append(C.lc(LC_COPY, D.zeros(), r, st))
        v.append(C.spmv(prob.A, s[-1], D.zeros(), st))
        for i in range(kk):  # modified Gram-Schmidt (gcr.py:76-81)
            C.dot(v[-1], v[i], "alpha", st)
            C.lc(LC_AXPY, v[-1], v[-1], st, y=v[i], a="alpha", sa=-1.0)
            C.lc(LC_AXPY, s[-1], s[-1], st, y=s[i], a="alpha", sa=-1.0)
        C.norm(v[-1], None, "beta", st)
        C.sc(SOP_GUARD, "gb", st, a="beta")
        C.lc(LC_DIV, v[-1], v[-1], st, a="gb")
        C.lc(LC_DIV, s[-1], s[-1], st, a="gb")
        C.dot(D.b, v[-1], "gamma", st)
        C.lc(LC_AXPY, x, x, st, y=s[-1], a="gamma")
        C.lc(LC_AXPY, r, r, st, y=v[-1], a="gamma", sa=-1.0)
        C.norm(r, None, "nr", st)
        C.check("nr", st)

    k = 0
    success = False
    while True:
        if np.all(resnorms[-1] <= criterion):
            resnorms[-1] = D.cols(norm(D.residual(x)))
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        steps = _chunks(D, callback) if maxiter is None else min(_chunks(D, callback), maxiter - k)
        # each step appends two basis vectors before the chunk's stop is known:
        # enqueue at most _GCR_CHUNK_BYTES of them ahead of the convergence test
        steps = max(1, min(steps, _GCR_CHUNK_BYTES // max(1, 2 * prob.n * prob.kpad * prob.dtype.itemsize)))
        C.begin()
        for st in range(steps):
            step(st, k + st)
        rows, _ = C.end(steps)
        del s[k + len(rows):], v[k + len(rows):]  # vectors of steps the chunk's stop skipped
        for row in rows:
            if callback is not None:
                callback(D.host(x), D.host(r))
            resnorms.append(D.cols(row))
            k += 1
    xk = D.host_final(x)
    return xk if success else None, Info(success, xk, k, resnorms, renumbered=prob.A.renumbered)
