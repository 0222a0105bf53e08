"""Device contexts and device-resident vectors (thin owners of C-ABI handles)."""
import ctypes
import os
import threading

import numpy as np

from . import _lib
from ._lib import check, lib

_contexts = {}
_ctx_lock = threading.Lock()


class Context:
    """One GPU + one HIP stream (``kry_ctx``)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib.kry_ctx_create(int(device), ctypes.byref(h)))
        self.device = int(device)
        self.handle = h
        self._fin = _lib.own(self, lib.kry_ctx_destroy, h, context=True)

    def synchronize(self):
        check(lib.kry_ctx_synchronize(self.handle))

    # HIP-event timing on the context stream --------------------------------
    def timer_start(self):
        check(lib.kry_timer_start(self.handle))

    def timer_stop(self):
        ms = ctypes.c_double()
        check(lib.kry_timer_stop(self.handle, ctypes.byref(ms)))
        return ms.value

    def profile(self, enable=True, kernels=None, every=1):
        """HIP-event timing of the solvers' launches: every kernel id, or
        only the ids in ``kernels`` (e.g. ``[_lib.PROF_SPMV]``), one launch
        in ``every``."""
        if kernels is None and every == 1:
            check(lib.kry_profile_enable(self.handle, 1 if enable else 0))
        else:
            ids = range(4) if kernels is None else kernels
            mask = sum(1 << int(i) for i in ids) if enable else 0
            check(lib.kry_profile_select(self.handle, mask, int(every)))

    def profile_read(self, kernel_id=_lib.PROF_SPMV):
        cnt = ctypes.c_int64()
        ms = ctypes.c_double()
        check(lib.kry_profile_read(self.handle, kernel_id, ctypes.byref(cnt), ctypes.byref(ms)))
        return cnt.value, ms.value


def default_device():
    """``KRYLOV_DEVICE`` if set, else the launcher's LOCAL_RANK, else 0."""
    for var in ("KRYLOV_DEVICE", "LOCAL_RANK"):
        if os.environ.get(var, "") != "":
            return int(os.environ[var])
    return 0


def get_context(device=None):
    device = default_device() if device is None else int(device)
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = Context(device)
            _contexts[device] = ctx
        return ctx


class HostOut:
    """The host array a solve's iterate is downloaded into, allocated when the
    solve starts, with its pages faulted in by a helper thread while the device
    iterates. A fresh numpy array of 80 MB (the metric's x) otherwise pays its
    pages' first-touch zeroing inside the download: 3.8 ms against the 1.45 ms
    of the copy itself (tools/xfer_bench.hip, profiles/r04_xfer_probe.txt).
    Below MIN_BYTES (8 MiB) the array is plain. ``take()`` joins the helper and
    returns the array; the download then overwrites every element."""

    MIN_BYTES = 8 << 20

    def __init__(self, shape, dtype):
        self.a = np.empty(shape, dtype=dtype)
        self._t = None
        if self.a.nbytes >= self.MIN_BYTES:
            self._t = threading.Thread(target=self.a.fill, args=(0,), name="krylov_amd-prefault", daemon=True)
            self._t.start()

    def take(self):
        if self._t is not None:
            self._t.join()
            self._t = None
        return self.a


class DeviceVector:
    """An n x k row-major block in HBM (``kry_vec``)."""

    def __init__(self, ctx, n, k, dtype):
        self.ctx = ctx
        self.n = int(n)
        self.k = int(k)
        self.dtype = np.dtype(dtype)
        h = ctypes.c_void_p()
        check(lib.kry_vec_create(ctx.handle, self.n, self.k, _lib.dtype_code(self.dtype), ctypes.byref(h)))
        self.handle = h
        self._fin = _lib.own(self, lib.kry_vec_destroy, h)

    @classmethod
    def from_host(cls, ctx, a, dtype=None):
        a = np.asarray(a)
        dtype = a.dtype if dtype is None else np.dtype(dtype)
        a2 = np.ascontiguousarray(a.reshape(a.shape[0], -1), dtype=dtype)
        v = cls(ctx, a2.shape[0], a2.shape[1], dtype)
        v.upload(a2)
        return v

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.size == self.n * self.k
        check(lib.kry_vec_upload(self.handle, _lib.ptr(a)))

    def to_host(self, out=None):
        """The vector as an (n, k) host array: a new one, or ``out`` (a
        C-contiguous array of that shape and dtype, e.g. ``HostOut.take()``)."""
        if out is None:
            out = np.empty((self.n, self.k), dtype=self.dtype)
        assert out.shape == (self.n, self.k) and out.dtype == self.dtype and out.flags.c_contiguous
        check(lib.kry_vec_download(self.handle, _lib.ptr(out)))
        return out

    def close(self):
        self._fin()
