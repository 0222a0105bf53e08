"""Device Householder reflector (reference ``householder.py:6-81``).

``Householder(x)`` builds H with ``H x = alpha ||x|| e_1``, ``|alpha| = 1``
(Golub & Van Loan 5.1.1, real case) on the GPU with the kernels of
Householder Arnoldi (``kry_householder``); ``H @ y`` evaluates the
reference's ``y - beta * v * <v, y>`` on the device (``kry_dot``,
``kry_vec_lincomb``). Quasi-1-D vectors ((n,) or (n, 1)), float32/float64.
"""
import numpy as np

from . import _lib
from ._lib import check, lib
from .device import DeviceVector, get_context

_LC_AXPY, _LC_SCALE = 0, 7


class Householder:
    def __init__(self, x, device=None):
        x = np.asarray(x)
        assert len(x.shape) == 1 or (len(x.shape) == 2 and x.shape[1] == 1), (
            "Householder only works for quasi-1D vectors for now. " f"Input vector has shape {x.shape}."
        )
        if np.iscomplexobj(x):
            raise TypeError("complex Householder reflectors are outside the MI355X path")
        dt = x.dtype if x.dtype in (np.float32, np.float64) else np.dtype(np.float64)
        self.ctx = get_context(device)
        self.shape = x.shape
        self.dtype = np.dtype(dt)
        xv = DeviceVector.from_host(self.ctx, x.reshape(-1, 1), dt)
        self._v = DeviceVector(self.ctx, x.shape[0], 1, dt)
        out = np.zeros(3)
        check(lib.kry_householder(self.ctx.handle, xv.handle, self._v.handle, _lib.dptr(out)))
        self.beta = dt.type(out[0]) if out[0] != 0 else 0
        self.alpha = dt.type(out[1])
        self.xnorm = dt.type(out[2])
        self.v = self._v.to_host().reshape(x.shape)

    def __matmul__(self, x):
        x = np.asarray(x)
        if x.shape != self.v.shape:
            raise ValueError(f"Shape mismatch! (v.shape = {self.v.shape} != {x.shape} = x.shape)")
        if self.beta == 0:
            return x
        dt = np.result_type(self.dtype, x.dtype)
        xv = DeviceVector.from_host(self.ctx, x.reshape(-1, 1), self.dtype)
        ip = np.zeros(1)
        check(lib.kry_dot(self.ctx.handle, self._v.handle, xv.handle, None, _lib.dptr(ip)))
        bv = DeviceVector(self.ctx, x.shape[0], 1, self.dtype)
        beta = np.array([float(self.beta)])
        check(lib.kry_vec_lincomb(self.ctx.handle, _LC_SCALE, bv.handle, self._v.handle, None, None,
                                  _lib.dptr(beta), None))
        # x - (beta v) <v, x>  ==  x + (-<v, x>) (beta v), exactly
        neg = np.array([-float(self.dtype.type(ip[0]))])
        out = DeviceVector(self.ctx, x.shape[0], 1, self.dtype)
        check(lib.kry_vec_lincomb(self.ctx.handle, _LC_AXPY, out.handle, xv.handle, bv.handle, None,
                                  _lib.dptr(neg), None))
        return out.to_host().reshape(x.shape).astype(dt, copy=False)

    def matrix(self):
        """Dense I - beta v v^T, built on the host from the device reflector
        (a test utility, as in the reference)."""
        n = self.v.shape[0]
        eye = np.zeros([n, n] + list(self.v.shape[1:]))
        idx = np.arange(n)
        eye[idx, idx] = 1.0
        return eye - self.beta * np.einsum("i...,j...->ij...", self.v, self.v)
