"""The reference's other Krylov solvers on the device:
``bicgstab`` (bicgstab.py:24-144), ``cgs`` (cgs.py:24-117), ``cgr``
(cgr.py:16-100) and ``gcr`` (gcr.py:18-97).

They share the SpMV + inner product + AXPY loop shape of CG, so they run as
host-driven loops over device vectors: every SpMV is the device SpMV
(``kry_spmv``), every AXPY-type line is one ``kry_vec_lincomb`` launch that
evaluates the reference's NumPy expression tree, and every inner product is a
device reduction (``kry_dot``) whose per-column value returns to the host,
where the scalar recurrences are evaluated with the reference's own NumPy
expressions. Vectors stay in HBM for the whole solve; only inner products (and
callback arguments) cross PCIe. Signatures, control flow and quirks follow
the reference line by line (e.g. bicgstab's mid-step convergence test on the
explicit residual of the *previous* iterate, bicgstab.py:123-127).
"""
import numpy as np

from . import _lib
from ._helpers import Info, Problem
from ._lib import check, lib
from .device import DeviceVector

LC_AXPY, LC_NEST_ADD, LC_NEST_SUB, LC_DIV, LC_SUB, LC_ADD, LC_COPY, LC_SCALE = range(8)


class _Dev:
    """Device vectors of one solve (n x kpad blocks) and the primitives."""

    def __init__(self, prob):
        if prob.kpad > 64:
            raise NotImplementedError("at most 64 right-hand-side columns on the host-driven solvers")
        self.prob = prob
        self.ctx = prob.ctx
        self.w = prob.w_dev

    def zeros(self):
        v = DeviceVector(self.ctx, self.prob.n, self.prob.kpad, self.prob.dtype)
        return v

    def upload(self, a):
        v = self.zeros()
        v.upload(self.prob.pad(np.asarray(a).astype(self.prob.dtype, copy=False)))
        return v

    def host(self, v):
        return self.prob.unpad_vec(v.to_host(), self.prob.r0_dtype)

    def matvec(self, op, x):
        """op @ x into a new vector; op None = the reference's Identity (x itself)."""
        if op is None:
            return x
        y = self.zeros()
        op.matvec_device(x, y)
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
        return self.lc(LC_SUB, self.prob.b_dev, self.A(x))

    def cols(self, v):
        """kpad per-column values -> the reference's scalar / (k,) array."""
        return self.prob.colvals(v)


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
        r0 = D.copy(prob.b_dev)
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
    rho, alpha, omega = 1.0, 1.0, 1.0
    p, v = D.zeros(), D.zeros()
    criterion = np.maximum(tol * resnorms[0], atol)
    crit_p = prob.pad_cols(criterion, np.inf)
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
        rho_old = rho
        rho = D.dot(r0_, r)
        rho_old_omega = rho_old * omega
        beta = rho * alpha / _guard(rho_old_omega)
        p = D.lc(LC_NEST_SUB, r, p, v, a=beta, b=omega)  # p = r + beta * (p - omega * v)
        y = D.op("Mr", D.op("Ml", p))
        v = D.A(y)
        r0v = D.dot(r0_, v)
        alpha = rho / _guard(r0v)
        s = D.lc(LC_AXPY, r, v, a=-alpha)  # s = r - alpha * v
        h = D.lc(LC_AXPY, x, y, a=alpha)  # h = x + alpha * y
        resnorm_h = norm(D.op("Ml", D.residual(x)))  # of x, not h (bicgstab.py:123)
        if np.all(resnorm_h <= crit_p):
            resnorms[-1] = D.cols(resnorm_h)
            success = True
            break
        Ml_s = D.op("Ml", s)
        z = D.op("Mr", Ml_s)
        t = D.A(z)
        Ml_t = D.op("Ml", t)
        tt = D.dot(Ml_t, Ml_t)
        omega = D.dot(Ml_t, Ml_s) / _guard(tt)
        x = D.lc(LC_AXPY, h, z, a=omega)
        r = D.lc(LC_AXPY, s, t, a=-omega)
        if callback is not None:
            callback(D.host(x), D.host(r))
        resnorms.append(D.cols(norm(r)))
        k += 1
    xk = D.host(x)
    return xk if success else None, Info(success, xk, k, resnorms)


def cgs(A, b, M=None, x0=None, inner=None, tol=1e-5, atol=1.0e-15, maxiter=None, callback=None):
    """CGS, reference signature and iteration (cgs.py:24-117)."""
    prob = Problem(A, b, x0, inner, M=M)
    D = _Dev(prob)

    def norm(v):  # cgs.py:44-48
        return np.sqrt(_real(D.dot(v, D.op("M", v))))

    x, r0 = _start(D, x0)
    rp = r0
    r = D.copy(r0)
    if callback:
        callback(D.host(x), D.host(r))
    resnorms = [D.cols(norm(r))]
    rho = 1.0
    p, q = D.zeros(), D.zeros()
    criterion = np.maximum(tol * resnorms[0], atol)
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
        rho_old = rho
        rho = D.dot(rp, r)
        beta = rho / _guard(rho_old)
        u = D.lc(LC_AXPY, r, q, a=beta)  # u = r + beta * q
        p = D.lc(LC_NEST_ADD, u, q, p, a=beta, b=beta)  # p = u + beta * (q + beta * p)
        v = D.A(D.op("M", p))
        s = D.dot(rp, v)
        alpha = rho / _guard(s)
        q = D.lc(LC_AXPY, u, v, a=-alpha)  # q = u - alpha * v
        u_ = D.op("M", D.lc(LC_ADD, u, q))
        D.lc(LC_AXPY, x, u_, a=alpha, out=x)  # x += alpha * u_
        D.lc(LC_AXPY, r, D.A(u_), a=-alpha, out=r)  # r -= alpha * (A @ u_)
        if callback:
            callback(D.host(x), D.host(r))
        resnorms.append(D.cols(norm(r)))
        k += 1
    xk = D.host(x)
    return xk if success else None, Info(success, xk, k, resnorms)


def cgr(A, b, M=None, x0=None, inner=None, tol=1e-5, atol=1.0e-15, maxiter=None, callback=None):
    """Conjugate residual, reference signature and iteration (cgr.py:16-100)."""
    prob = Problem(A, b, x0, inner, M=M)
    D = _Dev(prob)
    if x0 is None:
        x = D.zeros()
        r = D.copy(prob.b_dev)
    else:
        x = D.upload(x0)
        r = D.residual(x)
    r = D.op("M", r)

    def norm(v):  # cgr.py:47-51 (no M)
        return np.sqrt(_real(D.dot(v, v)))

    Ar = D.A(r)
    rAr = D.dot(r, Ar)
    resnorms = [D.cols(norm(r))]
    if callback is not None:
        callback(D.host(x), D.host(r))
    p = D.copy(r)
    Ap = D.copy(Ar)
    criterion = np.maximum(tol * resnorms[0], atol)
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
        MAp = D.op("M", Ap)
        ApMAp = D.dot(Ap, MAp)
        alpha = rAr / _guard(ApMAp)
        D.lc(LC_AXPY, x, p, a=alpha, out=x)
        D.lc(LC_AXPY, r, MAp, a=-alpha, out=r)
        Ar = D.A(r)
        rAr_old = rAr
        rAr = D.dot(r, Ar)
        beta = rAr / _guard(rAr_old)
        p = D.lc(LC_AXPY, r, p, a=beta)
        Ap = D.lc(LC_AXPY, Ar, Ap, a=beta)
        if callback is not None:
            callback(D.host(x), D.host(r))
        resnorms.append(D.cols(norm(r)))
        k += 1
    xk = D.host(x)
    return xk if success else None, Info(success, xk, k, resnorms)


def gcr(A, b, x0=None, inner=None, tol=1e-5, atol=1.0e-15, maxiter=None, callback=None):
    """Generalised conjugate residual with MGS (gcr.py:18-97)."""
    prob = Problem(A, b, x0, inner)
    D = _Dev(prob)
    if x0 is None:
        x = D.zeros()
        r = D.copy(prob.b_dev)
    else:
        x = D.upload(x0)
        r = D.residual(x)

    def norm(v):
        return np.sqrt(_real(D.dot(v, v)))

    if callback is not None:
        callback(D.host(x), D.host(r))
    resnorms = [D.cols(norm(r))]
    s, v = [], []
    criterion = np.maximum(tol * resnorms[0], atol)
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
        s.append(D.copy(r))
        v.append(D.A(s[-1]))
        for i in range(k):  # modified Gram-Schmidt (gcr.py:76-81)
            alpha = D.dot(v[-1], v[i])
            D.lc(LC_AXPY, v[-1], v[i], a=-alpha, out=v[-1])
            D.lc(LC_AXPY, s[-1], s[i], a=-alpha, out=s[-1])
        beta = norm(v[-1])
        D.lc(LC_DIV, v[-1], a=_guard(beta), out=v[-1])
        D.lc(LC_DIV, s[-1], a=_guard(beta), out=s[-1])
        gamma = D.dot(prob.b_dev, v[-1])
        D.lc(LC_AXPY, x, s[-1], a=gamma, out=x)
        D.lc(LC_AXPY, r, v[-1], a=-gamma, out=r)
        if callback is not None:
            callback(D.host(x), D.host(r))
        resnorms.append(D.cols(norm(r)))
        k += 1
    xk = D.host(x)
    return xk if success else None, Info(success, xk, k, resnorms)
