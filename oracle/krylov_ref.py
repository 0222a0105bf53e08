"""ORACLE — CPU restatement of the reference Krylov iterations (TEST INFRASTRUCTURE).

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it. The MI355X path (``krylov_amd``) never calls into ``oracle/``.

It restates, for real dtypes, the iteration of ``ju-liu/krylov`` 0.0.3
(``/root/reference/src/krylov``), including the preconditioners M, Ml, Mr
(``None`` = identity; otherwise anything with ``@``, e.g. scipy.sparse),
applied in the reference's order and with its identity aliasing:

* ``cg``      — ``cg.py:16-259`` (loop ``cg.py:155-234``)
* ``gmres``   — ``gmres.py:41-251`` with ``ArnoldiMGS`` ``arnoldi.py:107-200``
* ``minres``  — ``minres.py:28-253`` with ``ArnoldiLanczos`` ``arnoldi.py:203-281``
* ``givens``  — ``givens.py:5-47`` (LAPACK ``?lartg`` per column)
* ``Info``    — ``_helpers.py:93-98``

Arithmetic is delegated exactly where the reference delegates it: SpMV to
SciPy ``csr_matvec``/``csr_matvecs`` (``A @ x``), 1-D inner products to
``np.dot`` (OpenBLAS), block inner products to ``np.einsum`` (sequential per
column), rotations to LAPACK ``dlartg``. Parity pinned: every function here is
checked against fixtures produced by the reference itself
(``tests/golden/make_golden.py`` → ``tests/golden/solvers.npz``) in
``tests/test_oracle.py``.
"""
from collections import namedtuple

import numpy as np
import scipy.linalg
from scipy.linalg import lapack

Info = namedtuple(
    "IterInfo",
    ["success", "xk", "numsteps", "resnorms", "num_operations", "arnoldi"],
    defaults=(None, None),
)


class InvariantError(Exception):
    """Stands for ``krylov.errors.ArgumentError`` (errors.py:1-9)."""


def default_inner(shape):
    """_helpers.py:101-110: np.dot for vectors, einsum over axis 0 otherwise."""
    if len(shape) == 1:
        return lambda x, y: np.dot(x.conj(), y)
    return lambda x, y: np.einsum("i...,i...->...", x.conj(), y)


def _safe(d):
    """The reference's zero-division guard ``np.where(d != 0, d, 1.0)``."""
    return np.where(d != 0, d, 1.0)


def _real_norm2(v):
    if np.any(v.imag != 0.0):
        raise ValueError("inner product <x, M x> gave nonzero imaginary part")
    return v.real


class _Prod:
    """Product(Ml, A, Mr) (_helpers.py:39-48): applies right to left."""

    def __init__(self, Ml, A, Mr):
        self.Ml, self.A, self.Mr = Ml, A, Mr
        self.shape = A.shape

    def __matmul__(self, x):
        return _apply(self.Ml, self.A @ _apply(self.Mr, x))


def _apply(op, x):
    """``op @ x``; the reference's Identity returns x itself (_helpers.py:26-36)."""
    return x if op is None else op @ x


def givens(X):
    """givens.py:5-47 — one LAPACK lartg call per trailing column."""
    assert X.shape[0] == 2
    flat = X.reshape(2, -1)
    lartg = lapack.get_lapack_funcs("lartg", (flat,))
    cs, rs = [], []
    for col in range(flat.shape[1]):
        c, s, r = lartg(*flat[:, col])
        cs.append(np.array([[c, s], [-np.conj(s), c]]))
        rs.append(r)
    G = np.moveaxis(np.array(cs), 0, -1).reshape(2, 2, *X.shape[1:])
    return G, np.array(rs)


def _rot(G, v):
    """multi_matmul (gmres.py:19-21, minres.py:23-25)."""
    return np.einsum("ij...,j...->i...", G, v)


def cg(A, b, inner=None, x0=None, tol=1e-5, atol=1e-15, maxiter=None, callback=None, M=None, Ml=None):
    """Restates cg.py:16-259 (no Lanczos return)."""
    b = np.asarray(b)
    assert A.shape[0] == A.shape[1] == b.shape[0]
    inner = default_inner(b.shape) if inner is None else inner
    maxiter = A.shape[0] if maxiter is None else maxiter
    x0 = np.zeros_like(b) if x0 is None else x0

    def residual(z):  # cg.py:71-95
        r = b - A @ z
        Ml_r = _apply(Ml, r)
        M_Ml_r = _apply(M, Ml_r)
        return M_Ml_r, Ml_r, _real_norm2(inner(Ml_r, M_Ml_r))

    M_Ml_r0, Ml_r0, rho = residual(x0)
    if callback is not None:
        callback(x0, Ml_r0)
    resnorms = [np.sqrt(rho)]
    y = np.zeros(x0.shape, dtype=M_Ml_r0.dtype)
    rho_prev, rho_cur = None, rho
    Ml_rk = Ml_r0.copy()
    M_Ml_rk = M_Ml_r0.copy()
    p = M_Ml_rk.copy()  # cg.py:138
    xk = None
    k = 0
    success = False
    criterion = np.maximum(tol * resnorms[0], atol)
    while True:
        if np.all(resnorms[-1] <= criterion):  # cg.py:156-164
            xk = x0 + y if xk is None else xk
            resnorms[-1] = np.sqrt(residual(xk)[2])
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        if k > 0:  # cg.py:175-178
            p = M_Ml_rk + (rho_cur / _safe(rho_prev)) * p
        Ap = _apply(Ml, A @ p)  # Product(Ml, A) (cg.py:110, 180)
        alpha = rho_cur / _safe(inner(p, Ap))  # cg.py:183-185
        y += alpha * p
        xk = None
        Ml_rk -= alpha * Ap
        if callback is not None:
            xk = x0 + y
            callback(xk, Ml_rk)
        M_Ml_rk = _apply(M, Ml_rk)  # cg.py:205-209
        rr = _real_norm2(inner(Ml_rk, M_Ml_rk))
        rho_prev, rho_cur = rho_cur, rr
        resnorms.append(np.sqrt(rr))
        k += 1
    xk = x0 + y if xk is None else xk
    ops = {"A": 1 + k, "M": 2 + k, "Ml": 2 + k, "Mr": 1 + k, "inner": 2 + 2 * k, "axpy": 2 + 2 * k}
    return (xk if success else None), Info(success, xk, k, resnorms, num_operations=ops)


def _trisolve_columns(R, y):
    """multi_solve_triangular (gmres.py:24-38): per-column solve, zero rhs -> 0."""
    k = R.shape[0]
    Rc = R.reshape(k, k, -1)
    yc = y.reshape(k, -1)
    cols = []
    for c in range(Rc.shape[2]):
        if np.all(yc[:, c] == 0.0):
            cols.append(np.zeros(k))
        else:
            cols.append(scipy.linalg.solve_triangular(Rc[:, :, c], yc[:, c]))
    return np.array(cols).T.reshape([k] + list(R.shape[2:]))


class _House:
    """householder.py:6-65 (real case): H x = alpha ||x|| e_1."""

    def __init__(self, x):
        v = x.copy()
        gamma = v[0].copy()
        v[0] = 1
        sigma2 = np.dot(v[1:].conj(), v[1:]) if v.ndim == 1 else np.einsum("i...,i...->...", v[1:].conj(), v[1:])
        xnorm = np.sqrt(np.abs(gamma) ** 2 + sigma2)
        if sigma2 == 0:
            beta = 0
            xnorm = np.abs(gamma)
            alpha = 1 if gamma == 0 else gamma / xnorm
        else:
            beta = 2
            if gamma == 0:
                v[0] = -np.sqrt(sigma2)
                alpha = 1
            else:
                v[0] = gamma + gamma / np.abs(gamma) * xnorm
                alpha = -gamma / np.abs(gamma)
        self.v = v / np.sqrt(np.abs(v[0]) ** 2 + sigma2)
        self.alpha = alpha
        self.beta = beta
        self.inner = default_inner(x.shape)

    def __matmul__(self, x):
        if self.beta == 0:
            return x
        return x - self.beta * self.v * self.inner(self.v, x)


class _ArnoldiHouseholder:
    """arnoldi.py:33-104."""

    def __init__(self, A, v):
        self.A = A
        self.v = v
        self.iter = 0
        self.is_invariant = False
        self.houses = [_House(v)]
        vnorm = np.linalg.norm(v, 2)
        self.V = [v / np.where(vnorm != 0.0, vnorm, 1.0)]

    def __next__(self):
        if self.is_invariant:
            raise InvariantError("Krylov subspace was found to be invariant in the previous iteration.")
        k = self.iter
        Av = self.A @ self.V[k]
        for j in range(k + 1):
            Av[j:] = self.houses[j] @ Av[j:]
            Av[j] *= np.conj(self.houses[j].alpha)
        N = self.v.shape[0]
        if k < N - 1:
            house = _House(Av[k + 1:])
            self.houses.append(house)
            Av[k + 1:] = (house @ Av[k + 1:]) * np.conj(house.alpha)
            h = Av[: k + 2]
            h[-1] = np.abs(h[-1])
            if h[-1] <= 1.0e-14:
                self.is_invariant = True
                v = None
            else:
                vnew = np.zeros_like(self.v)
                vnew[k + 1] = 1
                for j in range(k + 1, -1, -1):
                    vnew[j:] = self.houses[j] @ vnew[j:]
                v = vnew * self.houses[-1].alpha
                self.V.append(v)
        else:
            h = np.zeros([len(Av) + 1] + list(self.v.shape[1:]), Av.dtype)
            h[:-1] = Av
            self.is_invariant = True
            v = None
        self.iter += 1
        return v, h


def _ident(v):
    return v


def gmres(A, b, inner=None, ortho="mgs", x0=None, tol=1e-5, atol=1e-15, maxiter=None, callback=None, M=None,
          Ml=None, Mr=None, shard=None):
    """Restates gmres.py:41-251 with Arnoldi MGS (arnoldi.py:107-200) or
    Householder (arnoldi.py:33-104).

    ``shard`` (test hook for the RHS-sharded path): a callable
    mapping this rank's per-column values to the global column vector (all
    ranks, in rank order). The history, the stop rule and the invariance test
    then act on all columns, as krylov_amd.distributed.gmres does."""
    glob = _ident if shard is None else shard
    b = np.asarray(b)
    assert A.shape[0] == A.shape[1] == b.shape[0]
    house = ortho == "householder"
    assert house or ortho.startswith("mgs")
    sweeps = 1 if ortho in ("mgs", "householder") else int(ortho[3:])
    inner = default_inner(b.shape) if inner is None else inner
    maxiter = A.shape[0] if maxiter is None else maxiter
    x0 = np.zeros_like(b) if x0 is None else np.asarray(x0)

    def resid(z):  # gmres.py:105-118
        Ml_r = _apply(Ml, b - A @ z)
        M_Ml_r = _apply(M, Ml_r)
        return M_Ml_r, Ml_r, np.sqrt(_real_norm2(inner(Ml_r, M_Ml_r)))

    def resnorm_of(z):
        return glob(resid(z)[2])

    M_Ml_r0, Ml_r0, r0norm = resid(x0)
    r0 = M_Ml_r0
    resnorms = [glob(r0norm)]
    if callback is not None:
        callback(x0, Ml_r0)

    hdtype = np.result_type(A.dtype, r0.dtype)
    # ArnoldiMGS.__init__ with Mv = M_Ml_r0 (arnoldi.py:136-150): P = Ml r0, V = M Ml r0
    P = [Ml_r0 / np.where(r0norm != 0.0, r0norm, 1.0)]
    V = [M_Ml_r0 / np.where(r0norm != 0.0, r0norm, 1.0)]
    if house:  # ArnoldiHouseholder(Ml_A_Mr, Ml_r0) (gmres.py:158-161)
        op = _Prod(Ml, A, Mr)
        hh = _ArnoldiHouseholder(op, Ml_r0)
        V = hh.V
    invariant = False
    steps = 0
    R = np.zeros([maxiter + 1, maxiter] + list(b.shape[1:]), dtype=r0.dtype)
    y = np.zeros([maxiter + 1] + list(b.shape[1:]), dtype=r0.dtype)
    y[0] = r0norm
    G = []

    def solution(yv):
        if yv is None:
            return x0
        if steps > 0:
            coef = _trisolve_columns(R[:steps, :steps], yv)
            acc = sum(c * v for c, v in zip(coef, V))
            return x0 + _apply(Mr, acc)
        return x0

    yk = None
    xk = None
    k = 0
    success = False
    criterion = np.maximum(tol * resnorms[0], atol)
    while True:
        if np.all(resnorms[-1] <= criterion):
            xk = solution(yk) if xk is None else xk
            resnorms[-1] = resnorm_of(xk)
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        # --- Arnoldi MGS step (arnoldi.py:167-200) ---
        if invariant:
            raise InvariantError("Krylov subspace was found to be invariant in the previous iteration.")
        if house:
            _, h = next(hh)
            steps += 1
            if hh.is_invariant:
                invariant = True
            # --- Givens QR update (gmres.py:206-221) ---
            R[: k + 2, k] = h[: k + 2]
            for i in range(k):
                R[i : i + 2, k] = _rot(G[i], R[i : i + 2, k])
            g, rr = givens(R[k : k + 2, k])
            G.append(g)
            R[k, k] = rr
            R[k + 1, k] = 0.0
            y[k : k + 2] = _rot(G[k], y[k : k + 2])
            yk = y[: k + 1]
            xk = None
            rn = np.array(np.abs(y[k + 1]))
            if callback is not None:
                xk = solution(yk)
                callback(xk, rn)
            resnorms.append(rn[()])
            k += 1
            continue
        w = _apply(Ml, A @ _apply(Mr, V[steps]))  # Product(Ml, A, Mr)
        h = np.zeros([steps + 2] + list(b.shape[1:]), dtype=hdtype)
        for _ in range(sweeps):
            for j in range(steps + 1):
                a = inner(V[j], w)
                h[j] += a
                w -= a * P[j]
        Mw = _apply(M, w)
        h[steps + 1] = np.sqrt(inner(w, Mw))
        if np.all(glob(h[steps + 1]) <= 1.0e-14):
            invariant = True
        else:
            hk = np.where(h[steps + 1] != 0.0, h[steps + 1], 1.0)
            P.append(w / hk)
            V.append(Mw / hk)
        steps += 1
        # --- Givens QR update (gmres.py:206-221) ---
        R[: k + 2, k] = h[: k + 2]
        for i in range(k):
            R[i : i + 2, k] = _rot(G[i], R[i : i + 2, k])
        g, rr = givens(R[k : k + 2, k])
        G.append(g)
        R[k, k] = rr
        R[k + 1, k] = 0.0
        y[k : k + 2] = _rot(G[k], y[k : k + 2])
        yk = y[: k + 1]
        xk = None
        rn = np.array(np.abs(y[k + 1]))
        if callback is not None:
            xk = solution(yk)
            callback(xk, rn)
        resnorms.append(glob(rn[()]))
        k += 1
    if xk is None:
        xk = solution(y[:steps])
    ops = {"A": 1 + k, "M": 2 + k, "Ml": 2 + k, "Mr": 1 + k,
           "inner": 2 + k + k * (k + 1) / 2, "axpy": 4 + 2 * k + k * (k + 1) / 2}
    return (xk if success else None), Info(success, xk, k, resnorms, num_operations=ops)


def minres(A, b, inner=None, x0=None, tol=1e-5, atol=1e-15, maxiter=None, callback=None, M=None, Ml=None, Mr=None,
           shard=None):
    """Restates minres.py:28-253 with Lanczos (arnoldi.py:203-281).
    ``shard``: the RHS-sharding test hook, as in ``gmres``.

    Precision follows the reference under NumPy-2 promotion: the Lanczos
    scalars ``h`` are kept in the vector dtype, while ``R``, the rotations, ``y``
    and therefore ``z``/``W`` are float64 (minres.py:195,219).
    """
    b = np.asarray(b)
    assert A.shape[0] == A.shape[1] == b.shape[0]
    inner = default_inner(b.shape) if inner is None else inner
    maxiter = A.shape[0] if maxiter is None else maxiter
    x0 = np.zeros_like(b) if x0 is None else x0

    glob = _ident if shard is None else shard

    def resnorm_of(z):  # minres.py:105-118
        Ml_r = _apply(Ml, b - A @ z)
        return glob(np.sqrt(_real_norm2(inner(Ml_r, _apply(M, Ml_r)))))

    r = b - A @ x0
    Ml_r = _apply(Ml, r)
    M_Ml_r = _apply(M, Ml_r)
    rnorm = np.sqrt(_real_norm2(inner(Ml_r, _apply(M, Ml_r))))
    dtype = M_Ml_r.dtype
    hdtype = np.result_type(A.dtype, M_Ml_r.dtype)
    # Lanczos state (arnoldi.py:203-235): p = Ml r, v = M Ml r
    lz_h = np.zeros([3] + list(b.shape[1:]), dtype=hdtype)
    lz_scale = np.where(rnorm != 0.0, rnorm, 1.0)
    lz_v = M_Ml_r / lz_scale
    lz_p = Ml_r / lz_scale
    lz_pold = None
    lz_iter = 0
    invariant = False

    W = [np.zeros(b.shape, dtype=dtype), np.zeros(b.shape, dtype=dtype)]
    y = np.array([rnorm, np.zeros_like(rnorm)])
    G = [None, None]
    yk = np.zeros(b.shape, dtype=dtype)
    xk = None
    rn = np.array(rnorm)
    if callback is not None:
        callback(x0, rn)
    resnorms = [glob(rn[()])]
    k = 0
    success = False
    criterion = np.maximum(tol * resnorms[0], atol)
    while True:
        if np.all(resnorms[-1] <= criterion):
            xk = x0 + _apply(Mr, yk) if xk is None else xk
            resnorms[-1] = resnorm_of(xk)
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        v = lz_v
        # --- Lanczos step (arnoldi.py:237-281) ---
        if invariant:
            raise InvariantError("Krylov subspace was found to be invariant in the previous iteration.")
        w = _apply(Ml, A @ _apply(Mr, lz_v))  # Product(Ml, A, Mr)
        if lz_iter > 0:
            lz_h[0] = lz_h[2]
            w -= lz_h[0] * lz_pold
        a = inner(lz_v, w)
        lz_h[1] = a
        w -= a * lz_p
        Mw = _apply(M, w)
        lz_h[2] = np.sqrt(inner(w, Mw))
        if np.all(glob(lz_h[2]) <= 1.0e-14):
            invariant = True
            lz_v = lz_p = None
        else:
            s = np.where(lz_h[2] != 0.0, lz_h[2], 1.0)
            lz_pold = lz_p
            lz_p = w / s
            lz_v = Mw / s
        lz_iter += 1
        h = lz_h.real
        # --- QR update (minres.py:193-224) ---
        Rv = np.zeros([4] + list(b.shape[1:]), dtype=float)
        Rv[1] = h[0]
        if G[1] is not None:
            Rv[:2] = _rot(G[1], Rv[:2])
        Rv[2] = h[1]
        Rv[3] = h[2]
        if G[0] is not None:
            Rv[1:3] = _rot(G[0], Rv[1:3])
        G[1] = G[0]
        G[0], rr = givens(Rv[2:4])
        Rv[2] = rr
        Rv[3] = 0.0
        y = _rot(G[0], y)
        z = (v - Rv[0] * W[0] - Rv[1] * W[1]) / np.where(Rv[2] != 0.0, Rv[2], 1.0)
        W[0], W[1] = W[1], z
        yk += y[0] * z
        xk = None
        y = np.array([y[1], np.zeros_like(y[1])])
        rn = np.array(np.abs(y[0]))
        if callback is not None:
            xk = x0 + _apply(Mr, yk)
            callback(xk, rn)
        resnorms.append(glob(rn[()]))
        k += 1
    if xk is None:
        xk = x0 + _apply(Mr, yk)
    ops = {"A": 1 + k, "M": 2 + k, "Ml": 2 + k, "Mr": 1 + k, "inner": 2 + 2 * k, "axpy": 4 + 8 * k}
    return (xk if success else None), Info(success, xk, k, resnorms, num_operations=ops)


# --------------------------------------------------------------------------
# The reference's other Krylov solvers, restated.


def _start_xr(A, b, x0, copy_x0):
    if x0 is None:
        return np.zeros_like(b), b.copy()
    x = np.array(x0) if copy_x0 else np.asarray(x0)
    return x, b - A @ x


def bicgstab(A, b, Ml=None, Mr=None, x0=None, inner=None, tol=1e-5, atol=1e-15, maxiter=None, callback=None):
    """Restates bicgstab.py:24-144 (including the mid-step test on the
    explicit residual of x, bicgstab.py:123-127)."""
    b = np.asarray(b)
    inner = default_inner(b.shape) if inner is None else inner

    def _norm(x):
        return np.sqrt(_real_norm2(inner(x, _apply(Ml, x))))

    x, r0 = _start_xr(A, b, x0, copy_x0=False)
    r0_ = r0
    r = r0.copy()
    if callback is not None:
        callback(x, r)
    resnorms = [_norm(r0)]
    rho = 1.0
    alpha = 1.0
    omega = 1.0
    p = np.zeros_like(b)
    v = np.zeros_like(b)
    k = 0
    success = False
    criterion = np.maximum(tol * resnorms[0], atol)
    while True:
        if np.all(resnorms[-1] <= criterion):
            resnorms[-1] = _norm(b - A @ x)
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        rho_old = rho
        rho = inner(r0_, r)
        rho_old_omega = rho_old * omega
        beta = rho * alpha / np.where(rho_old_omega != 0.0, rho_old_omega, 1.0)
        p = r + beta * (p - omega * v)
        y = _apply(Mr, _apply(Ml, p))
        v = A @ y
        r0v = inner(r0_, v)
        alpha = rho / np.where(r0v != 0.0, r0v, 1.0)
        s = r - alpha * v
        h = x + alpha * y
        resnorm_h = _norm(_apply(Ml, b - A @ x))
        if np.all(resnorm_h <= criterion):
            resnorms[-1] = resnorm_h
            success = True
            break
        Ml_s = _apply(Ml, s)
        z = _apply(Mr, Ml_s)
        t = A @ z
        Ml_t = _apply(Ml, t)
        tt = inner(Ml_t, Ml_t)
        omega = inner(Ml_t, Ml_s) / np.where(tt != 0.0, tt, 1.0)
        x = h + omega * z
        r = s - omega * t
        if callback is not None:
            callback(x, r)
        resnorms.append(_norm(r))
        k += 1
    return x if success else None, Info(success, x, k, resnorms)


def cgs(A, b, M=None, x0=None, inner=None, tol=1e-5, atol=1e-15, maxiter=None, callback=None):
    """Restates cgs.py:24-117."""
    b = np.asarray(b)
    inner = default_inner(b.shape) if inner is None else inner

    def _norm(x):
        return np.sqrt(_real_norm2(inner(x, _apply(M, x))))

    x, r0 = _start_xr(A, b, x0, copy_x0=True)
    rp = r0
    r = r0.copy()
    if callback:
        callback(x, r)
    resnorms = [_norm(r)]
    rho = 1.0
    p = np.zeros_like(b)
    q = np.zeros_like(b)
    k = 0
    success = False
    criterion = np.maximum(tol * resnorms[0], atol)
    while True:
        if np.all(resnorms[-1] <= criterion):
            resnorms[-1] = _norm(b - A @ x)
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        rho_old = rho
        rho = inner(rp, r)
        beta = rho / np.where(rho_old != 0.0, rho_old, 1.0)
        u = r + beta * q
        p = u + beta * (q + beta * p)
        v = A @ _apply(M, p)
        s = inner(rp, v)
        alpha = rho / np.where(s != 0.0, s, 1.0)
        q = u - alpha * v
        u_ = _apply(M, u + q)
        x += alpha * u_
        r -= alpha * (A @ u_)
        if callback:
            callback(x, r)
        resnorms.append(_norm(r))
        k += 1
    return x if success else None, Info(success, x, k, resnorms)


def cgr(A, b, M=None, x0=None, inner=None, tol=1e-5, atol=1e-15, maxiter=None, callback=None):
    """Restates cgr.py:16-100."""
    b = np.asarray(b)
    if x0 is None:
        x = np.zeros_like(b)
        r = b.copy()
    else:
        x = np.array(x0)
        r = b - A @ x0
    r = _apply(M, r)
    inner = default_inner(b.shape) if inner is None else inner

    def _norm(x):
        return np.sqrt(_real_norm2(inner(x, x)))

    Ar = A @ r
    rAr = inner(r, Ar)
    resnorms = [_norm(r)]
    if callback is not None:
        callback(x, r)
    p = r.copy()
    Ap = Ar.copy()
    k = 0
    success = False
    criterion = np.maximum(tol * resnorms[0], atol)
    while True:
        if np.all(resnorms[-1] <= criterion):
            resnorms[-1] = _norm(b - A @ x)
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        MAp = _apply(M, Ap)
        ApMAp = inner(Ap, MAp)
        alpha = rAr / np.where(ApMAp != 0.0, ApMAp, 1.0)
        x += alpha * p
        r -= alpha * MAp
        Ar = A @ r
        rAr_old = rAr
        rAr = inner(r, Ar)
        beta = rAr / np.where(rAr_old != 0.0, rAr_old, 1.0)
        p = r + beta * p
        Ap = Ar + beta * Ap
        if callback is not None:
            callback(x, r)
        resnorms.append(_norm(r))
        k += 1
    return x if success else None, Info(success, x, k, resnorms)


def gcr(A, b, x0=None, inner=None, tol=1e-5, atol=1e-15, maxiter=None, callback=None):
    """Restates gcr.py:18-97."""
    b = np.asarray(b)
    if x0 is None:
        x = np.zeros_like(b)
        r = b.copy()
    else:
        x = np.array(x0)
        r = b - A @ x0
    inner = default_inner(b.shape) if inner is None else inner

    def _norm(x):
        return np.sqrt(_real_norm2(inner(x, x)))

    if callback is not None:
        callback(x, r)
    resnorms = [_norm(r)]
    s = []
    v = []
    k = 0
    success = False
    criterion = np.maximum(tol * resnorms[0], atol)
    while True:
        if np.all(resnorms[-1] <= criterion):
            resnorms[-1] = _norm(b - A @ x)
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        s.append(r.copy())
        v.append(A @ s[-1])
        for i in range(k):
            alpha = inner(v[-1], v[i])
            v[-1] -= alpha * v[i]
            s[-1] -= alpha * s[i]
        beta = _norm(v[-1])
        v[-1] /= np.where(beta != 0.0, beta, 1.0)
        s[-1] /= np.where(beta != 0.0, beta, 1.0)
        gamma = inner(b, v[-1])
        x += gamma * s[-1]
        r -= gamma * v[-1]
        if callback is not None:
            callback(x, r)
        resnorms.append(_norm(r))
        k += 1
    return x if success else None, Info(success, x, k, resnorms)
