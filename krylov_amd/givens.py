"""Device Givens rotations (reference ``givens.py:5-47``).

``givens(X)`` computes, per trailing column of a (2, ...) array, LAPACK
>= 3.10 ``?lartg`` on the GPU (bitwise scipy.linalg.lapack ``dlartg`` /
``slartg``) and returns ``G = [[c, s], [-s, c]]`` of shape (2, 2, ...) and
``r`` — the same contract as the reference.
"""
import numpy as np

from . import _lib
from ._lib import check, lib
from .device import get_context


def lartg(f, g, device=None):
    """Batched lartg on device: returns (c, s, r) arrays."""
    f = np.ascontiguousarray(f)
    g = np.ascontiguousarray(g, dtype=f.dtype)
    if f.dtype not in (np.float32, np.float64):
        raise TypeError("lartg supports float32/float64")
    c = np.empty_like(f)
    s = np.empty_like(f)
    r = np.empty_like(f)
    ctx = get_context(device)
    check(lib.kry_lartg(ctx.handle, f.size, _lib.dtype_code(f.dtype), _lib.ptr(f), _lib.ptr(g), _lib.ptr(c),
                        _lib.ptr(s), _lib.ptr(r)))
    return c, s, r


def givens(X):
    X = np.asarray(X)
    assert X.shape[0] == 2
    flat = X.reshape(2, -1)
    if np.iscomplexobj(flat):
        raise TypeError("complex Givens rotations are outside the MI355X path")
    dt = flat.dtype if flat.dtype in (np.float32, np.float64) else np.float64
    c, s, r = lartg(np.ascontiguousarray(flat[0], dtype=dt), np.ascontiguousarray(flat[1], dtype=dt))
    G = np.array([[c, s], [-s, c]])  # (2, 2, ncols)
    return G.reshape(2, 2, *X.shape[1:]), r
