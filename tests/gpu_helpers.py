"""Small systems and the consistency check used by the reference's own test
suite (tests/linear_problems.py, tests/helpers.py:4-23), restated for the
real-valued problems the MI355X path covers."""
import os

import numpy as np
import scipy.sparse

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# The device sums its inner products in one more valid order; its deviation
# from the fixture is allowed twice the envelope of the reference's own
# deviation under 5 other orders (tests/golden/make_selfnoise.py).
NOISE_FACTOR = 2.0


def selfnoise_envelope(case, ref):
    """Per history entry (all but the final explicit one): the spread of the
    reference's own history when only the summation order of its inner
    product changes (tests/golden/selfnoise.npz: OpenBLAS 1 / 2 / 4 / 8
    threads, pairwise, extended precision, fsum, and for small cases 40
    random orders), as the largest relative difference between any two of
    those histories and the fixture ``ref``, carried forward as a running
    maximum along the history (rounding differences propagate through the
    recurrence)."""
    d = np.load(os.path.join(GOLD, "selfnoise.npz"))
    hs = [d[k] for k in sorted(d.files) if k.startswith(case + "_")]
    assert hs and all(h.shape == ref.shape for h in hs), case
    H = np.array([ref[:-1]] + [h[:-1] for h in hs])
    spread = (H.max(axis=0) - H.min(axis=0)) / np.abs(ref[:-1])
    return np.maximum.accumulate(spread)


def _spd_diag(n):
    a = np.linspace(1.0, 2.0, n)
    a[-1] = 1e-2
    return a


def spd_dense(shape):
    return np.diag(_spd_diag(shape[0])), np.ones(shape)


def spd_sparse(shape):
    n = shape[0]
    return scipy.sparse.spdiags(_spd_diag(n), [0], n, n), np.ones(shape)


def spd_rhs_0(shape):
    return np.diag(_spd_diag(shape[0])), np.zeros(shape)


def spd_rhs_0sol0():
    A = np.diag(_spd_diag(5))
    rng = np.random.RandomState(0)
    cols = [np.zeros(5), rng.rand(5), rng.rand(5)]
    sol = np.linalg.solve(A, cols[1])
    return A, np.column_stack([np.zeros(5), sol, np.zeros(5)])


def symmetric_indefinite():
    a = np.linspace(1.0, 2.0, 5)
    a[-1] = -1.0
    return np.diag(a), np.ones(5)


def real_unsymmetric():
    a = np.arange(1, 6, dtype=float)
    a[-1] = -10.0
    A = np.diag(a)
    A[0, -1] = 10.0
    return A, np.ones(5)


def assert_consistent(A, b, info, sol, tol):
    res = b - A @ info.xk
    resnorm = np.sqrt(np.einsum("i...,i...->...", res, res.conj()))
    bnorm = np.sqrt(np.einsum("i...,i...->...", b, b.conj()))
    if info.success:
        assert sol.shape == b.shape
        assert np.all(resnorm < tol * (1.0 + bnorm))
        assert np.may_share_memory(sol, info.xk)
    assert np.issubdtype(np.asarray(info.resnorms).dtype, np.floating)
    assert np.all(np.abs(resnorm - info.resnorms[-1]) <= 1.0e-12 * (1 + resnorm))
    assert np.asarray(info.resnorms).shape == (info.numsteps + 1, *b.shape[1:])


def assert_parity(info, d, prefix, rtol=1e-10, xtol=1e-9, final_atol=None, noise=None, floor=0.0):
    """Device run vs the reference fixture: identical step count and success,
    updated-residual history within rtol, final explicit residual within an
    absolute round-off bound, solution within xtol.

    noise: for a history the reference's own summation-order noise moves by
    more than rtol, the per-entry envelope of that noise (selfnoise_envelope):
    entry i may deviate by max(rtol, NOISE_FACTOR * noise[i]) rel."""
    assert info.numsteps == int(d[prefix + "_numsteps"])
    assert info.success == bool(d[prefix + "_success"])
    got = np.asarray(info.resnorms, dtype=np.float64)
    ref = d[prefix + "_resnorms"]
    assert got.shape == ref.shape
    # floor: an absolute allowance of floor * ||r_0|| for methods whose
    # updated residual loses relative accuracy as it decreases (eps ||r_0|| / ||r_k||)
    diff = np.maximum(np.abs(got[:-1] - ref[:-1]) - floor * np.max(np.abs(ref[0])), 0.0)
    rel = diff / np.maximum(np.abs(ref[:-1]), 1e-300)
    tol = rtol if noise is None else np.maximum(rtol, NOISE_FACTOR * noise)
    assert np.all(rel <= tol), (np.max(rel / tol), int(np.argmax(rel / tol)))
    if final_atol is None:
        final_atol = 1e-12 * np.max(np.abs(ref[0])) + 1e-300
    assert np.all(np.abs(got[-1] - ref[-1]) <= final_atol)
    xr = d[prefix + "_xk"]
    np.testing.assert_allclose(info.xk, xr, rtol=xtol, atol=xtol * np.max(np.abs(xr)))
    ops = info.num_operations
    if ops is None:
        assert np.all(np.isnan(d[prefix + "_ops"]))
    else:
        np.testing.assert_array_equal([ops[k] for k in ("A", "M", "Ml", "Mr", "inner", "axpy")], d[prefix + "_ops"])
