"""Preconditioned solves (M, Ml, Mr as device CSR operators) against the
reference's own results (tests/golden/precond.npz, tests/solver_cases.py)
and the reference's preconditioner tests (tests/test_solvers.py:90-120)."""
import os

import numpy as np
import pytest

from tests import gpu_helpers as H
from tests import solver_cases

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def fixtures():
    return np.load(os.path.join(HERE, "golden", "precond.npz"))


@pytest.mark.parametrize("case", solver_cases.CASES, ids=lambda c: c[0])
def test_preconditioned_parity(fixtures, case):
    import krylov_amd

    solver, A, b, kw = solver_cases.build(case)
    _, info = getattr(krylov_amd, solver)(A, b, **kw)
    # bicgstab / cgs / cgr / gcr form their residuals by cancellation
    # (r = s - omega t, ...): their attainable relative accuracy at step k is
    # ~eps ||r_0|| / ||r_k||, hence an absolute floor of 1e-14 ||r_0||
    floor = 1e-14 if solver in ("bicgstab", "cgs", "cgr", "gcr") else 0.0
    H.assert_parity(info, fixtures, case[0], floor=floor)


@pytest.mark.parametrize("case", solver_cases.CASES[:4], ids=lambda c: c[0])
def test_preconditioners_as_device_operators(fixtures, case):
    """The same with every operator uploaded once as a CsrOperator."""
    import krylov_amd

    solver, A, b, kw = solver_cases.build(case, wrap=krylov_amd.CsrOperator)
    _, info = getattr(krylov_amd, solver)(A, b, **kw)
    H.assert_parity(info, fixtures, case[0])


def _diag_problem():
    a = np.linspace(1.0, 2.0, 5)
    A = np.diag(a)
    A[0, 0] = 1e-2
    return A, np.ones(5), np.diag(a)


@pytest.mark.parametrize("solver", ["cg", "minres", "gmres"])
def test_m(solver):
    import krylov_amd

    A, b, M = _diag_problem()
    _, info = getattr(krylov_amd, solver)(A, b, M=M, tol=1.0e-12)
    assert info.resnorms[-1] <= 1.0e-12


@pytest.mark.parametrize("solver", ["cg", "minres", "gmres"])
def test_ml(solver):
    import krylov_amd

    A, b, M = _diag_problem()
    _, info = getattr(krylov_amd, solver)(A, b, Ml=M, tol=1.0e-12)
    assert info.resnorms[-1] <= 1.0e-12


@pytest.mark.parametrize("solver", ["minres", "gmres"])
def test_mr(solver):
    import krylov_amd

    A, b, M = _diag_problem()
    _, info = getattr(krylov_amd, solver)(A, b, Mr=M, tol=1.0e-12)
    assert info.resnorms[-1] <= 1.0e-12


def test_preconditioned_matches_oracle_block_and_callback():
    """Block right-hand side with Ml and M, against the oracle; the callback
    sees Ml r (cg.py:201-203)."""
    import krylov_amd
    from oracle import krylov_ref as K

    q = solver_cases.inputs()
    A, B, Mj, S = q["Pvar"], q["B3"], q["Mj"], q["S"]
    seen = []
    _, got = krylov_amd.cg(A, B, M=Mj, Ml=S, tol=0.0, maxiter=15, callback=lambda x, r: seen.append(r.copy()))
    ref_seen = []
    _, ref = K.cg(A, B, M=Mj, Ml=S, tol=0.0, maxiter=15, callback=lambda x, r: ref_seen.append(r.copy()))
    assert got.numsteps == ref.numsteps == 15
    np.testing.assert_allclose(np.asarray(got.resnorms), np.asarray(ref.resnorms), rtol=1e-10)
    assert len(seen) == len(ref_seen) == 16
    for a, b in zip(seen, ref_seen):
        np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-12 * np.abs(b).max())
