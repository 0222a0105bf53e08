"""The C-ABI library loads, exports every symbol include/krylov_hip.h declares,
and its host-only logic (tile partition, error mapping) is right. CPU only:
no kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _declared_symbols():
    with open(os.path.join(REPO, "include", "krylov_hip.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kry_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from krylov_amd import _lib

    declared = _declared_symbols()
    assert len(declared) > 30
    for name in declared:
        assert hasattr(_lib.lib, name), name
    # and the ctypes binding covers exactly the header
    assert sorted(_lib.EXPORTED) == declared


def test_library_is_gfx950_code_object():
    from krylov_amd import _lib

    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_version_and_device_count_without_gpu():
    from krylov_amd import _lib

    assert _lib.lib.kry_version() >= 100
    n = _lib.device_count()
    assert n >= 0


def test_no_device_fails_loudly():
    from krylov_amd import _lib

    if _lib.device_count() > 0:
        pytest.skip("a GPU is present")
    from krylov_amd.device import Context

    with pytest.raises(RuntimeError, match="no HIP device"):
        Context(0)


def _partition(indptr, tile_nnz, tile_rows):
    from krylov_amd import _lib

    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    n = indptr.shape[0] - 1
    cnt = ctypes.c_int64()
    _lib.check(_lib.lib.kry_csr_partition(n, _lib.ptr(indptr), _lib.KRY_I64, tile_nnz, tile_rows,
                                           ctypes.byref(cnt), None))
    rs = np.zeros(cnt.value + 1, dtype=np.int64)
    _lib.check(_lib.lib.kry_csr_partition(n, _lib.ptr(indptr), _lib.KRY_I64, tile_nnz, tile_rows,
                                           ctypes.byref(cnt), rs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
    return rs


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_partition_invariants(seed):
    rng = np.random.default_rng(seed)
    n = 5000
    lens = rng.integers(0, 40, n)
    lens[rng.choice(n, 5, replace=False)] = rng.integers(2049, 9000, 5)  # long rows
    indptr = np.concatenate([[0], np.cumsum(lens)])
    rs = _partition(indptr, 2048, 256)
    assert rs[0] == 0 and rs[-1] == n
    assert np.all(np.diff(rs) >= 1)
    for a, b in zip(rs[:-1], rs[1:]):
        nnz = indptr[b] - indptr[a]
        if b - a == 1 and nnz > 2048:
            continue  # a long row alone in its tile
        assert nnz <= 2048 and b - a <= 256
    # maximality: a tile could not have taken its next row
    for a, b in zip(rs[:-2], rs[1:-1]):
        if b - a == 1 and indptr[b] - indptr[a] > 2048:
            continue
        assert b - a == 256 or indptr[b + 1] - indptr[a] > 2048


def test_partition_int32_matches_int64():
    from krylov_amd import _lib, problems

    A = problems.poisson2d(40)
    cnt32 = ctypes.c_int64()
    ip32 = np.ascontiguousarray(A.indptr, dtype=np.int32)
    _lib.check(_lib.lib.kry_csr_partition(A.shape[0], _lib.ptr(ip32), _lib.KRY_I32, 2048, 256,
                                           ctypes.byref(cnt32), None))
    rs = _partition(A.indptr, 2048, 256)
    assert cnt32.value == len(rs) - 1


def test_error_mapping():
    from krylov_amd import _lib
    from krylov_amd.errors import ArgumentError

    with pytest.raises(ValueError):
        _lib.check(_lib.lib.kry_csr_partition(-1, None, _lib.KRY_I32, 1, 1, None, None))
    with pytest.raises(ArgumentError):
        _lib.check(_lib.KRY_EINVARIANT)
    with pytest.raises(np.linalg.LinAlgError):
        _lib.check(_lib.KRY_ESINGULAR)
    with pytest.raises(MemoryError):
        _lib.check(_lib.KRY_ENOMEM)
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.KRY_EUNSUPPORTED)


def test_weighted_inner_matches_reference_form():
    from krylov_amd import WeightedInner

    rng = np.random.default_rng(0)
    n = 50
    w = 10 / np.arange(1, n + 1)
    x, y = rng.standard_normal(n), rng.standard_normal(n)
    assert WeightedInner(w)(x, y) == np.dot(x.T, w * y)  # tests/test_solvers.py:157-161
    X, Y = rng.standard_normal((n, 3)), rng.standard_normal((n, 3))
    got = WeightedInner(w)(X, Y)
    for c in range(3):
        np.testing.assert_allclose(got[c], np.dot(X[:, c], w * Y[:, c]), rtol=1e-14)


def test_unsupported_inputs_are_rejected_before_any_device_work():
    import krylov_amd

    with pytest.raises(TypeError):
        krylov_amd.cg(np.eye(3), np.ones(3), inner=lambda x, y: np.dot(x, y))
    with pytest.raises(NotImplementedError):
        krylov_amd.cg(np.eye(3), np.ones(3), M=np.eye(3))
    with pytest.raises(TypeError):
        krylov_amd.cg(np.eye(3), np.ones(3, dtype=complex))
    with pytest.raises(NotImplementedError):
        krylov_amd.gmres(np.eye(3), np.ones(3), ortho="householder")
