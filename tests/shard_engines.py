"""Host solver engines for the sharded driver (TEST INFRASTRUCTURE).

``krylov_amd.shard.drive`` runs the reference's outer loop over a column
block split across ranks; on GPUs its engine is the device solver state with
an RCCL communicator attached (``krylov_amd.distributed``). These are the same
engines restated on the host over any ``allreduce`` (gloo in the CPU tests),
so the product's rank bookkeeping, global criterion, explicit-residual
recheck and history assembly run without a GPU.

Per step an engine does what the device chunk does: the local recurrence
(cg.py:175-209 / arnoldi.py:167-200 + gmres.py:206-221 / arnoldi.py:237-281 +
minres.py:193-228, via the oracle's helpers), ONE allreduce of the
zero-padded residual norms plus the number of non-invariant columns, and the
global stop rule ``np.all(row <= criterion)`` that ``cg_global_check`` /
``gm_global_check`` / ``mr_global_check`` apply on the device; a chunk ends
after the first step that meets it.
"""
import numpy as np

from oracle import krylov_ref as K


def _einsum_inner(x, y):
    return np.einsum("i...,i...->...", x.conj(), y)


class _Base:
    def __init__(self, A, B, layout, allreduce):
        self.A, self.B, self.lay, self.allreduce = A, np.asarray(B, dtype=np.float64), layout, allreduce
        assert self.B.ndim == 2 and self.B.shape[1] == layout.kc == layout.kpad
        self.crit = None

    def set_criterion(self, crit_full):
        self.crit = np.asarray(crit_full, dtype=np.float64)

    def _exchange(self, local_norms, non_invariant):
        """One allreduce per step: global norms + non-invariant count."""
        v = np.zeros(self.lay.total + 1)
        v[self.lay.off:self.lay.off + self.lay.kpad] = local_norms
        v[-1] = float(non_invariant)
        g = np.asarray(self.allreduce(v), dtype=np.float64)
        return g[:-1], g[-1] == 0.0

    def run(self, steps):
        rows, invariant = [], False
        for _ in range(steps):
            row, invariant = self.step()
            rows.append(row)
            if np.all(row <= self.crit):
                break
        return np.array(rows).reshape(len(rows), self.lay.total), invariant


class HostCG(_Base):
    """cg.py:155-234 on this rank's columns (M = Ml = I, x0 = 0)."""

    def start_norms(self):
        self.y = np.zeros_like(self.B)
        self.r = self.B - self.A @ self.y
        self.rho = _einsum_inner(self.r, self.r)
        self.rho_prev = None
        self.p = self.r.copy()
        self.k = 0
        return np.sqrt(self.rho)

    def step(self):
        if self.k > 0:
            self.p = self.r + (self.rho / K._safe(self.rho_prev)) * self.p
        Ap = self.A @ self.p
        alpha = self.rho / K._safe(_einsum_inner(self.p, Ap))
        self.y += alpha * self.p
        self.r -= alpha * Ap
        self.rho_prev, self.rho = self.rho, _einsum_inner(self.r, self.r)
        self.k += 1
        row, _ = self._exchange(np.sqrt(self.rho), 0)
        return row, False

    def residual_norm2(self):
        rr = self.B - self.A @ self.y
        return _einsum_inner(rr, rr)

    def xk(self):
        return self.y.copy()


class HostGMRES(_Base):
    """ArnoldiMGS (arnoldi.py:167-200) + the Givens QR update
    (gmres.py:206-221) on this rank's columns (x0 = 0, no preconditioner)."""

    def __init__(self, A, B, layout, allreduce, maxiter):
        super().__init__(A, B, layout, allreduce)
        self.maxiter = maxiter

    def start_norms(self):
        kl = self.B.shape[1]
        r0 = self.B - self.A @ np.zeros_like(self.B)
        rn = np.sqrt(_einsum_inner(r0, r0))
        self.V = [r0 / np.where(rn != 0.0, rn, 1.0)]
        self.R = np.zeros((self.maxiter + 1, self.maxiter, kl))
        self.yv = np.zeros((self.maxiter + 1, kl))
        self.yv[0] = rn
        self.G = []
        self.k = 0
        return rn

    def step(self):
        k = self.k
        w = self.A @ self.V[k]
        h = np.zeros((k + 2, w.shape[1]))
        for j in range(k + 1):
            a = _einsum_inner(self.V[j], w)
            h[j] += a
            w -= a * self.V[j]
        h[k + 1] = np.sqrt(_einsum_inner(w, w))
        self.R[: k + 2, k] = h
        for i in range(k):
            self.R[i:i + 2, k] = K._rot(self.G[i], self.R[i:i + 2, k])
        g, rr = K.givens(self.R[k:k + 2, k])
        self.G.append(g)
        self.R[k, k] = rr
        self.R[k + 1, k] = 0.0
        self.yv[k:k + 2] = K._rot(g, self.yv[k:k + 2])
        row, invariant = self._exchange(np.abs(self.yv[k + 1]), int(np.sum(h[k + 1] > 1.0e-14)))
        if not invariant:
            self.V.append(w / np.where(h[k + 1] != 0.0, h[k + 1], 1.0))
        self.k += 1
        return row, invariant

    def xk(self):
        k = self.k
        if k == 0:
            return np.zeros_like(self.B)
        coef = K._trisolve_columns(self.R[:k, :k], self.yv[:k])
        return sum(c * v for c, v in zip(coef, self.V))

    def residual_norm2(self):
        rr = self.B - self.A @ self.xk()
        return _einsum_inner(rr, rr)


class HostMINRES(_Base):
    """ArnoldiLanczos (arnoldi.py:237-281) + the MINRES QR update
    (minres.py:193-228) on this rank's columns (x0 = 0, no preconditioner)."""

    def start_norms(self):
        r = self.B - self.A @ np.zeros_like(self.B)
        rn = np.sqrt(_einsum_inner(r, r))
        s = np.where(rn != 0.0, rn, 1.0)
        self.v = r / s
        self.p = r / s
        self.pold = None
        self.h = np.zeros((3, self.B.shape[1]))
        self.W = [np.zeros_like(self.B), np.zeros_like(self.B)]
        self.yy = np.array([rn, np.zeros_like(rn)])
        self.G = [None, None]
        self.yk = np.zeros_like(self.B)
        self.k = 0
        return rn

    def step(self):
        v = self.v
        w = self.A @ self.v
        if self.k > 0:
            self.h[0] = self.h[2]
            w -= self.h[0] * self.pold
        a = _einsum_inner(self.v, w)
        self.h[1] = a
        w -= a * self.p
        self.h[2] = np.sqrt(_einsum_inner(w, w))
        Rv = np.zeros((4, self.B.shape[1]))
        Rv[1] = self.h[0]
        if self.G[1] is not None:
            Rv[:2] = K._rot(self.G[1], Rv[:2])
        Rv[2] = self.h[1]
        Rv[3] = self.h[2]
        if self.G[0] is not None:
            Rv[1:3] = K._rot(self.G[0], Rv[1:3])
        self.G[1] = self.G[0]
        self.G[0], rr = K.givens(Rv[2:4])
        Rv[2] = rr
        Rv[3] = 0.0
        self.yy = K._rot(self.G[0], self.yy)
        z = (v - Rv[0] * self.W[0] - Rv[1] * self.W[1]) / np.where(Rv[2] != 0.0, Rv[2], 1.0)
        self.W[0], self.W[1] = self.W[1], z
        self.yk += self.yy[0] * z
        self.yy = np.array([self.yy[1], np.zeros_like(self.yy[1])])
        row, invariant = self._exchange(np.abs(self.yy[0]), int(np.sum(self.h[2] > 1.0e-14)))
        if not invariant:
            s = np.where(self.h[2] != 0.0, self.h[2], 1.0)
            self.pold = self.p
            self.p = w / s
            self.v = w / s
        self.k += 1
        return row, invariant

    def residual_norm2(self):
        rr = self.B - self.A @ self.yk
        return _einsum_inner(rr, rr)

    def xk(self):
        return self.yk.copy()
