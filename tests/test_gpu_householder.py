"""tests/test_householder.py of the reference restated for the device
reflector (real factors; complex ones are outside the MI355X path)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_FACTORS = [0.0, 1.0, 1e8, 1e-8]


@pytest.mark.parametrize("a", _FACTORS)
@pytest.mark.parametrize("b", _FACTORS)
@pytest.mark.parametrize("shape", [(10,), (10, 1), (1,)])
def test_house(a, b, shape):
    import krylov_amd

    x = np.full(shape, b, dtype=np.float64)
    x[0] = a
    n = shape[0]
    H = krylov_amd.Householder(x)
    y = H @ x
    cols = []
    for k in range(n):
        e = np.zeros(shape)
        e[k] = 1.0
        cols.append(H @ e)
        assert cols[-1].shape == e.shape
    HI = np.moveaxis(np.array(cols), 0, 1)
    Hm = H.matrix()
    assert np.max(np.abs(HI - Hm)) <= 1e-14                      # matrix() = H applied to I
    HmT = np.moveaxis(Hm, 0, 1)
    assert np.max(Hm - HmT) <= 1e-14                             # symmetric
    eye = np.zeros([n, n] + list(x.shape[1:]))
    eye[np.arange(n), np.arange(n)] = 1.0
    assert np.max(np.abs(eye - np.einsum("ij...,jk...->ik...", HmT, Hm))) <= 1e-14  # orthogonal
    xn = np.linalg.norm(x, 2)
    assert np.abs(xn - np.abs(y[0])) <= 1e-14 * xn                # |y0| = ||x||
    assert np.abs(1 - np.abs(H.alpha)) <= 1e-14                   # |alpha| = 1
    assert np.abs(y[0] - H.alpha * H.xnorm) <= 1e-14 * xn         # y0 = alpha ||x||
    if y.shape[0] > 1:
        assert np.linalg.norm(y[1:], 2) <= 1e-14 * xn             # y = y0 e_1


def test_house_matches_oracle():
    """The device reflector equals the oracle's restatement (householder.py)."""
    import krylov_amd
    from oracle import krylov_ref

    x = np.random.default_rng(4).standard_normal(5000)
    H = krylov_amd.Householder(x)
    R = krylov_ref._House(x.copy())
    np.testing.assert_allclose(H.v, R.v, rtol=1e-12, atol=1e-15)
    assert float(H.alpha) == float(R.alpha) and float(H.beta) == float(R.beta)
    y = np.random.default_rng(5).standard_normal(5000)
    np.testing.assert_allclose(H @ y, R @ y, rtol=1e-12, atol=1e-13)
