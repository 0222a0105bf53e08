"""Operator / inner-product plumbing shared by the drivers.

Mirrors the reference's ``_helpers.py`` (Identity 26-36, aslinearoperator
83-90, Info 93-98, get_default_inner 101-110) and adds the pieces the device
path needs: ``WeightedInner`` (the only custom inner product the GPU path
recognises) and ``Problem`` (shape/dtype bookkeeping between numpy inputs and
the n x k device blocks).
"""
from collections import namedtuple

import numpy as np

from .sparse import _next_pow2, as_device_operator

# the reference's record (_helpers.py:93-98) plus ``renumbered``: True when
# the operator's device image runs in a bandwidth-reducing renumbering (RCM,
# CsrOperator.layout()["renumbered"]), so the solve's summation order differs
# from the reference's and its history matches only to the reference's own
# order spread (INTEGRATION.md "Renumbering"; KRY_RENUMBER=0 turns it off).
Info = namedtuple(
    "IterInfo",
    ["success", "xk", "numsteps", "resnorms", "num_operations", "arnoldi", "renumbered"],
    defaults=(None, None, None),
)


class Identity:
    """The identity operator (returns its argument, like the reference)."""

    dtype = np.dtype("u1")

    @staticmethod
    def __matmul__(x):
        return x

    @staticmethod
    def rmatvec(x):
        return x


def aslinearoperator(A):
    if not hasattr(A, "__matmul__"):
        raise ValueError(f"Unknown linear operator A = {A}")
    return A


def get_default_inner(b_shape):
    """Host form of the default inner product (_helpers.py:101-110)."""

    def inner_dot(x, y):
        return np.dot(x.conj(), y)

    def inner_einsum(x, y):
        return np.einsum("i...,i...->...", x.conj(), y)

    return inner_dot if len(b_shape) == 1 else inner_einsum


class WeightedInner:
    """Inner product ``<x, y>_w = sum_i x_i (w_i y_i)`` per column.

    Callable on host arrays exactly like the reference's custom inner of
    tests/test_solvers.py:157-161 (``np.dot(x.T, w * y)``); the device path
    evaluates the same per-term products in float64 with its own reduction.
    """

    def __init__(self, w):
        w = np.asarray(w)
        if w.ndim != 1:
            raise ValueError("weights must be a 1-D array")
        if np.iscomplexobj(w):
            raise TypeError("complex weights are not supported")
        self.w = np.ascontiguousarray(w, dtype=np.float64)

    def __call__(self, x, y):
        if y.ndim == 1:
            return np.dot(x.T, self.w * y)
        wy = self.w.reshape((-1,) + (1,) * (y.ndim - 1)) * y
        return np.einsum("i...,i...->...", x.conj(), wy)


def _is_identity(M):
    return M is None or isinstance(M, Identity)


class Problem:
    """Shapes and dtypes of one solve, mapped onto an n x kpad device block.

    ``kpad`` is the column count rounded up to a power of two; padded columns
    carry b = 0, x0 = 0 and are inert (zero residual, always converged).
    """

    def __init__(self, A, b, x0, inner, M=None, Ml=None, Mr=None, device=None):
        b = np.asarray(b)
        if len(A.shape) != 2 or A.shape[0] != A.shape[1] or A.shape[1] != b.shape[0]:
            raise AssertionError("A must be square with A.shape[1] == b.shape[0]")
        for name, op in (("M", M), ("Ml", Ml), ("Mr", Mr)):
            if not _is_identity(op) and len(getattr(op, "shape", ())) != 2:
                raise NotImplementedError(
                    f"preconditioner {name} must be None, Identity, a krylov_amd.CsrOperator, a scipy.sparse "
                    f"matrix or a dense array on the MI355X path (got {type(op).__name__})"
                )
        if np.iscomplexobj(b) or (x0 is not None and np.iscomplexobj(x0)):
            raise TypeError("complex right-hand sides are outside the MI355X path")
        if inner is None:
            self.weights = None
        elif isinstance(inner, WeightedInner):
            if inner.w.shape[0] != b.shape[0]:
                raise ValueError("inner-product weights have the wrong length")
            self.weights = inner.w
        else:
            raise TypeError(
                "the MI355X path supports inner=None or krylov_amd.WeightedInner(w); "
                f"got {type(inner).__name__}"
            )
        self.A = as_device_operator(A, device=device)
        self.ctx = self.A.ctx
        # preconditioners as device operators (None = identity)
        self.ops = {}
        for name, op in (("M", M), ("Ml", Ml), ("Mr", Mr)):
            if _is_identity(op):
                self.ops[name] = None
                continue
            dop = as_device_operator(op, device=self.ctx.device, like=self.A, ctx=self.ctx)
            if dop.shape != self.A.shape:
                raise ValueError(f"preconditioner {name} has shape {dop.shape}, the operator {self.A.shape}")
            self.ops[name] = dop
        self.b = b
        self.n = b.shape[0]
        self.tail = b.shape[1:]
        self.kc = int(np.prod(self.tail)) if len(self.tail) else 1
        self.kpad = _next_pow2(self.kc)
        if self.kpad > 256:
            raise NotImplementedError("at most 256 right-hand-side columns per device")
        x0a = None if x0 is None else np.asarray(x0)
        # dtype of the reference's residual b - A x0 and of the device vectors
        rtypes = [self.A.dtype, b.dtype] + ([x0a.dtype] if x0a is not None else [])
        rtypes += [op.dtype for op in self.ops.values() if op is not None]
        r0 = np.result_type(*rtypes)
        if r0 not in (np.float32, np.float64):
            r0 = np.dtype(np.float64)
        self.r0_dtype = np.dtype(r0)
        vt = np.result_type(r0, np.float64) if self.weights is not None else r0
        self.dtype = np.dtype(vt)
        # dtype in which the reference's inner products (and norms) come out
        self.inner_dtype = np.dtype(np.float64) if self.weights is not None else self.dtype
        self.x0 = x0a
        from .device import DeviceVector

        self.b_dev = DeviceVector.from_host(self.ctx, self.pad(b), dtype=self.dtype)
        self.x0_dev = None if x0a is None else DeviceVector.from_host(self.ctx, self.pad(x0a), dtype=self.dtype)
        self.w_dev = None
        if self.weights is not None:
            self.w_dev = DeviceVector.from_host(self.ctx, self.weights.reshape(-1, 1), dtype=np.float64)

    # --- host <-> device block layout ---------------------------------------
    def pad(self, a):
        a2 = np.asarray(a).reshape(self.n, self.kc)
        if self.kpad != self.kc:
            a2 = np.concatenate([a2, np.zeros((self.n, self.kpad - self.kc), dtype=a2.dtype)], axis=1)
        return a2

    def unpad_vec(self, a2, dtype=None):
        out = np.ascontiguousarray(a2[:, : self.kc]).reshape(self.b.shape)
        return out if dtype is None else out.astype(dtype, copy=False)

    def pad_cols(self, v, fill):
        v = np.asarray(v, dtype=np.float64).reshape(self.kc)
        out = np.full(self.kpad, fill, dtype=np.float64)
        out[: self.kc] = v
        return out

    def colvals(self, row):
        """kpad device values -> the reference's per-step scalar/array."""
        v = np.asarray(row[: self.kc], dtype=np.float64).astype(self.inner_dtype)
        if len(self.tail) == 0:
            return v[0]
        return v.reshape(self.tail)

    def op_handles(self, *names):
        """ctypes handles of the named preconditioners (None = identity)."""
        return [None if self.ops[nm] is None else self.ops[nm].handle for nm in names]

    def has_precond(self):
        return any(op is not None for op in self.ops.values())

    def apply_host(self, name, x):
        """op @ x for a preconditioner (identity: x itself, as the reference's
        Identity returns the same object)."""
        op = self.ops[name]
        return x if op is None else op @ x

    def zeros_like_b(self):
        return np.zeros_like(self.b)

    def x0_or_zeros(self):
        """x0, or the reference's ``zeros_like(b)`` (cg.py:57, gmres.py:120,
        minres.py:82) built on first use and then the same object: an 80 MB
        fill at the metric size that a solve without callback never reads."""
        if self.x0 is not None:
            return self.x0
        if getattr(self, "_zeros", None) is None:
            self._zeros = np.zeros_like(self.b)
        return self._zeros


CHUNK = 32
