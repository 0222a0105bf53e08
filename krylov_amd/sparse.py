"""``CsrOperator``: a device-resident CSR matrix behind the reference's
operator protocol (``.shape``, ``.dtype``, ``__matmul__``; _helpers.py:14-24,
tests/test_solvers.py:229-237).

The matrix is uploaded once. ``A @ x`` runs the gfx950 SpMV kernel (bitwise
SciPy ``csr_matvec``/``csr_matvecs``); the solvers use the device copy
directly and never move A again.
"""
import ctypes
import weakref

import numpy as np
import scipy.sparse

from . import _lib
from ._lib import check, lib
from .device import DeviceVector, get_context


def _next_pow2(k):
    p = 1
    while p < k:
        p *= 2
    return p


class CsrOperator:
    """A device-resident CSR matrix. ``like``: build it with another
    operator's bandwidth-reducing renumbering (a preconditioner of a
    renumbered operator, kry_csr_create_like); the device picks the
    renumbering on its own otherwise (reverse Cuthill-McKee for scattered
    matrices with a narrow level structure). Vectors always cross in the
    caller's numbering. ``ctx``: a ``device.Context`` to build it on instead
    of the device's shared one (its own stream; e.g. two solves driven
    concurrently on one GPU)."""

    def __init__(self, A, device=None, like=None, ctx=None):
        if isinstance(A, CsrOperator):
            raise TypeError("already a CsrOperator")
        if scipy.sparse.issparse(A):
            csr = A.tocsr() if A.format != "csr" else A
        elif isinstance(A, np.ndarray):
            if A.ndim != 2:
                raise ValueError("A must be 2-D")
            csr = scipy.sparse.csr_matrix(A)
        else:
            raise TypeError(
                f"cannot place {type(A).__name__} on the device: pass a scipy.sparse matrix, a dense "
                "ndarray, or a krylov_amd.CsrOperator (host-callback operators are not supported)"
            )
        if csr.shape[0] != csr.shape[1]:
            raise ValueError("A must be square")
        if np.iscomplexobj(csr.data):
            raise TypeError("complex matrices are outside the MI355X path (float32/float64 only)")
        dt = np.dtype(csr.dtype)
        if dt not in (np.float32, np.float64):
            dt = np.dtype(np.float64)
        self.ctx = get_context(device) if ctx is None else ctx
        self.shape = csr.shape
        self.dtype = dt
        self.n = csr.shape[0]
        self.nnz = int(csr.nnz)
        itype = np.int32 if (self.nnz < 2**31 and self.n < 2**31) else np.int64
        indptr = np.ascontiguousarray(csr.indptr, dtype=itype)
        indices = np.ascontiguousarray(csr.indices, dtype=itype)
        data = np.ascontiguousarray(csr.data, dtype=dt)
        self.index_dtype = np.dtype(itype)
        h = ctypes.c_void_p()
        if like is not None and like.renumbered:
            if like.ctx is not self.ctx or like.n != self.n:
                raise ValueError("like: an operator of the same size on the same device")
            check(
                lib.kry_csr_create_like(
                    self.ctx.handle, like.handle, self.n, self.nnz, _lib.ptr(indptr), _lib.ptr(indices),
                    _lib.ptr(data), _lib.dtype_code(dt), _lib.itype_code(itype), ctypes.byref(h),
                )
            )
        else:
            check(
                lib.kry_csr_create(
                    self.ctx.handle, self.n, self.nnz, _lib.ptr(indptr), _lib.ptr(indices),
                    _lib.ptr(data), _lib.dtype_code(dt), _lib.itype_code(itype), ctypes.byref(h),
                )
            )
        self.handle = h
        self._fin = _lib.own(self, lib.kry_csr_destroy, h)
        self.renumbered = self.layout()["renumbered"]

    @property
    def device(self):
        return self.ctx.device

    def layout(self):
        """The device image: {"slices", "slots", "irregular", "compact",
        "col_blocks", "dia", "dia_slots", "pair", "pair_slots", "rs",
        "rs_slots", "renumbered", "rcm_levels"} (kry_csr_info_n)."""
        info = np.zeros(13, dtype=np.int64)
        check(lib.kry_csr_info_n(self.handle, info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), 13))
        return {"slices": int(info[0]), "slots": int(info[1]), "irregular": int(info[2]), "compact": bool(info[3]),
                "col_blocks": int(info[4]), "dia": bool(info[5]), "dia_slots": int(info[6]), "pair": bool(info[7]),
                "pair_slots": int(info[8]), "rs": bool(info[9]), "rs_slots": int(info[10]),
                "renumbered": bool(info[11]), "rcm_levels": int(info[12])}

    def matvec_device(self, x, y):
        """y = A x for DeviceVectors in the caller's numbering (no host traffic)."""
        check(lib.kry_spmv(self.ctx.handle, self.handle, x.handle, y.handle))

    def matvec_op(self, x, y):
        """y = A x for DeviceVectors already in the operator's numbering
        (kry_spmv_op; the same as matvec_device when not renumbered)."""
        check(lib.kry_spmv_op(self.ctx.handle, self.handle, x.handle, y.handle))

    def permute(self, src, dst, to_operator):
        """dst = src with its rows moved into (to_operator) or out of the
        operator's numbering (kry_csr_permute; a copy when not renumbered)."""
        check(lib.kry_csr_permute(self.ctx.handle, self.handle, src.handle, dst.handle, 1 if to_operator else 0))

    def __matmul__(self, x):
        x = np.asarray(x)
        if x.shape[0] != self.n:
            raise ValueError("dimension mismatch")
        dt = np.result_type(self.dtype, x.dtype)
        if dt not in (np.float32, np.float64):
            raise TypeError(f"unsupported vector dtype {x.dtype}")
        x2 = np.ascontiguousarray(x.reshape(self.n, -1), dtype=dt)
        k = x2.shape[1]
        kp = _next_pow2(k)
        if kp != k:
            x2 = np.concatenate([x2, np.zeros((self.n, kp - k), dtype=dt)], axis=1)
        xv = DeviceVector(self.ctx, self.n, kp, dt)
        xv.upload(x2)
        yv = DeviceVector(self.ctx, self.n, kp, dt)
        self.matvec_device(xv, yv)
        y = yv.to_host()[:, :k]
        return np.ascontiguousarray(y).reshape(x.shape)

    matvec = __matmul__

    def close(self):
        self._fin()

    def __repr__(self):
        return f"CsrOperator(n={self.n}, nnz={self.nnz}, dtype={self.dtype}, device={self.device})"


# --------------------------------------------------------------- upload cache
# a scipy/dense matrix handed to krylov_amd.cg/gmres/...
# again (the reference's tests and users call the solvers repeatedly on one A)
# is not uploaded and re-imaged again. The cache is keyed by the object and
# verified by a content fingerprint (xxh3 over indptr/indices/data, shape,
# dtype), so an in-place change of the matrix is re-uploaded. It holds at most
# _CACHE_MAX entries and drops an entry when its matrix is garbage-collected.
_CACHE_MAX = 4
_cache = {}  # (device, id(A), id(like) or None) -> (weakref(A), fingerprint, CsrOperator, weakref(like) or None)


def _fingerprint(A):
    import xxhash

    h = xxhash.xxh3_64()
    if scipy.sparse.issparse(A):
        csr = A if A.format == "csr" else None
        if csr is None:
            return None  # other formats are converted on every call
        for arr in (csr.indptr, csr.indices, csr.data):
            h.update(np.ascontiguousarray(arr).view(np.uint8).data)
        return (csr.shape, str(csr.dtype), str(csr.indices.dtype), csr.nnz, h.intdigest())
    if isinstance(A, np.ndarray):
        h.update(np.ascontiguousarray(A).view(np.uint8).data)
        return (A.shape, str(A.dtype), h.intdigest())
    return None


def clear_operator_cache():
    """Release every cached device copy of a host matrix, and return the
    device blocks freed so far to the runtime (kry_mem_release)."""
    _cache.clear()
    _lib.empty_cache()


def as_device_operator(A, device=None, like=None, ctx=None):
    """Return ``A`` as a CsrOperator (uploading scipy/dense inputs once).
    ``like``: the operator a preconditioner serves; when it is renumbered the
    preconditioner is built with its renumbering (a CsrOperator given as a
    preconditioner must already carry it). ``ctx``: the context to upload on
    (default: the device's shared one; another context is not cached)."""
    import os

    lk = like if (like is not None and like.renumbered) else None
    if isinstance(A, CsrOperator):
        if ctx is not None and A.ctx is not ctx:
            raise ValueError("the operator lives on another context than the solve")
        return A
    if ctx is not None and ctx is not get_context(ctx.device):
        return CsrOperator(A, like=lk, ctx=ctx)
    if os.environ.get("KRYLOV_CSR_CACHE", "1") == "0":
        return CsrOperator(A, device=device, like=lk)
    dev = get_context(device).device
    fp = _fingerprint(A)
    if fp is None:
        return CsrOperator(A, device=device, like=lk)
    key = (dev, id(A), None if lk is None else id(lk))
    hit = _cache.get(key)
    # the entry also holds a weakref to the operator it was built like: a new
    # operator that reuses a dead one's id() must not get a preconditioner
    # carrying the dead one's permutation
    if (hit is not None and hit[0]() is A and hit[1] == fp
            and (hit[3] is None if lk is None else (hit[3] is not None and hit[3]() is lk))):
        return hit[2]
    op = CsrOperator(A, device=dev, like=lk)
    try:
        ref = weakref.ref(A, lambda _r, key=key: _cache.pop(key, None))
        lref = None if lk is None else weakref.ref(lk, lambda _r, key=key: _cache.pop(key, None))
    except TypeError:
        return op
    _cache.pop(key, None)
    while len(_cache) >= _CACHE_MAX:
        _cache.pop(next(iter(_cache)))
    _cache[key] = (ref, fp, op, lref)
    return op
