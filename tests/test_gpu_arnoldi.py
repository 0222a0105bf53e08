"""The reference's Arnoldi backward-stability tests (tests/test_arnoldi.py
of ju-liu/krylov: MGS 84-106, Householder 38-63, checks 166-263) restated for
the device Arnoldi process of GMRES (krylov_amd.arnoldi): real matrices, the
Euclidean and the diagonally B-weighted inner product, M = None or B.

Bounds (Drkosova, Greenbaum, Rozloznik, Strakos 1995, as the reference uses
them): Arnoldi residual || M A V_k - V_{k+1} H || <= k N^1.5 eps ||A|| (2.3);
loss of orthogonality || I - <V, P> || <= k^1.5 N eps (Householder, 2.4) or
k^2 N eps sigma_max / sigma_min of [v, M A V_k] (MGS, 2.5); projection
|| <P, M A V> - H || within 10 (ortho * ||A|| + arnoldi * sqrt||<V,V>||)."""
import numpy as np
import pytest
import scipy.linalg
import scipy.sparse.linalg

pytestmark = pytest.mark.gpu

N = 10
_BDIAG = np.linspace(1.0, 5.0, N)


def _spd():
    a = np.linspace(1.0, 2.0, N)
    a[-1] = 1e-2
    return np.diag(a)


def _symm_indef():
    a = np.linspace(1.0, 2.0, N)
    a[-1] = -1.0
    return np.diag(a)


def _nonsymm():
    a = np.arange(1.0, N + 1.0)
    a[-1] = -10.0
    A = np.diag(a)
    A[0, -1] = 10.0
    return A


def _e0():
    x = np.zeros(N)
    x[0] = 1.0
    return x


def _check(A, v, V, H, P, maxiter, ortho, Bm, weighted):
    eps = np.finfo(np.float64).eps
    An = np.linalg.norm(A, 2)
    W = np.diag(_BDIAG) if weighted else np.eye(N)

    def ip(x, y):
        return x.T @ (W @ y)

    k = H.shape[1]
    assert k <= maxiter
    invariant = H.shape[0] == k
    assert len(V) == H.shape[0]
    Mv = v if Bm is None else Bm @ v
    assert np.linalg.norm(P[0] - v / np.sqrt(ip(v, Mv))) <= 1e-14
    assert np.all(np.tril(H, -2) == 0.0)
    assert np.all(np.diag(H[1:, :]) >= 0.0)
    Vm, Pm = np.column_stack(V), np.column_stack(P)
    AV = A @ (Vm if invariant else Vm[:, :-1])
    MAV = AV if Bm is None else Bm @ AV
    res = MAV - Vm @ H
    arnoldi_res = np.linalg.norm(ip(res, res), 2)
    assert arnoldi_res <= k * N**1.5 * eps * An
    ortho_res = np.linalg.norm(np.eye(Vm.shape[1]) - ip(Vm, Pm), 2)
    if ortho == "householder":
        ortho_tol = k**1.5 * N * eps
    else:
        sv = scipy.linalg.svd(np.column_stack([Vm[:, [0]], MAV[:, :-1] if invariant else MAV]), compute_uv=False)
        ortho_tol = np.inf if sv[-1] == 0 else k**2 * N * eps * sv[0] / sv[-1]
    # MGS (at k = N) and Lanczos cannot detect an invariant space reliably
    if (ortho != "mgs" or N != k) and ortho != "lanczos":
        assert ortho_res <= ortho_tol
    proj = np.linalg.norm(ip(Pm, MAV) - H, 2)
    assert proj <= max(10 * (ortho_res * An + arnoldi_res * np.sqrt(np.linalg.norm(ip(Vm, Vm), 2))), eps)


@pytest.mark.parametrize("A", [_spd(), _symm_indef(), _nonsymm()], ids=["spd", "symm_indef", "nonsymm"])
@pytest.mark.parametrize("v", [np.ones(N), _e0()], ids=["ones", "e0"])
@pytest.mark.parametrize("maxiter", [1, 5, 9, 10])
@pytest.mark.parametrize("use_m", [False, True])
@pytest.mark.parametrize("weighted", [False, True])
def test_arnoldi_mgs(A, v, maxiter, use_m, weighted):
    import krylov_amd

    Bm = np.diag(_BDIAG) if use_m else None
    inner = krylov_amd.WeightedInner(_BDIAG) if weighted else None
    V, H, P, _ = krylov_amd.arnoldi(A, v, maxiter, ortho="mgs", M=Bm, inner=inner)
    _check(A, v, V, H, P, maxiter, "mgs", Bm, weighted)


@pytest.mark.parametrize("A", [_spd(), _symm_indef(), _nonsymm()], ids=["spd", "symm_indef", "nonsymm"])
@pytest.mark.parametrize("v", [np.ones(N), _e0()], ids=["ones", "e0"])
@pytest.mark.parametrize("maxiter", [1, 5, 9, 10])
def test_arnoldi_householder(A, v, maxiter):
    import krylov_amd

    V, H, P, _ = krylov_amd.arnoldi(A, v, maxiter, ortho="householder")
    _check(A, v, V, H, V, maxiter, "householder", None, False)


def test_arnoldi_matches_oracle_relation():
    """The device H equals the oracle's Arnoldi coefficients to round-off on a
    larger random problem (persistent MGS path, n = 5000)."""
    import krylov_amd
    from krylov_amd import problems
    from oracle import krylov_ref

    R = problems.random_nonsym(5000)
    v = np.ones(R.shape[0])
    V, H, P, inv = krylov_amd.arnoldi(R, v, 20)
    assert not inv and len(V) == 21 and H.shape == (21, 20)
    _, info = krylov_ref.gmres(R, v, maxiter=20, tol=0.0)
    _, g = krylov_amd.gmres(R, v, maxiter=20, tol=0.0)
    np.testing.assert_allclose(np.asarray(g.resnorms), np.asarray(info.resnorms), rtol=1e-10)
    Vm = np.column_stack(V)
    res = R @ Vm[:, :-1] - Vm @ H
    assert np.linalg.norm(res) <= 20 * 5000**1.5 * np.finfo(float).eps * scipy.sparse.linalg.norm(R, 1)


@pytest.mark.parametrize("A", [_spd(), _symm_indef()], ids=["spd", "symm_indef"])
@pytest.mark.parametrize("v", [np.ones(N), _e0()], ids=["ones", "e0"])
@pytest.mark.parametrize("maxiter", [1, 5, 9, 10])
@pytest.mark.parametrize("use_m", [False, True])
@pytest.mark.parametrize("weighted", [False, True])
def test_arnoldi_lanczos(A, v, maxiter, use_m, weighted):
    """tests/test_arnoldi.py:125-163 on the MINRES device Lanczos process."""
    import krylov_amd

    Bm = np.diag(_BDIAG) if use_m else None
    inner = krylov_amd.WeightedInner(_BDIAG) if weighted else None
    V, H, P, _ = krylov_amd.lanczos(A, v, maxiter, M=Bm, inner=inner)
    _check(A, v, V, H, P, maxiter, "lanczos", Bm, weighted)
