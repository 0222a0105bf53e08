"""Solver cases (preconditioners M/Ml/Mr, Householder Arnoldi, and the other
solvers bicgstab/cgs/cgr/gcr) shared by the fixture generator
(tests/golden/make_golden.py -> tests/golden/precond.npz), the oracle tests
and the GPU parity tests. Inputs are rebuilt identically from seeds."""
import numpy as np
import scipy.sparse as sp

from krylov_amd import problems


def inputs():
    """A variable-coefficient SPD matrix with its Jacobi and symmetric-scaling
    diagonals, a random nonsymmetric matrix with |Jacobi| (SPD) and Jacobi
    diagonals, and a 3-column right-hand side."""
    P = problems.poisson2d(32)
    n = P.shape[0]
    shift = np.random.default_rng(7).uniform(0.0, 2.0, n)
    Pvar = (P + sp.diags(shift)).tocsr()
    d = Pvar.diagonal()
    R = problems.random_nonsym(3000, seed=4)
    dr = R.diagonal()
    # the reference's Householder test problem (tests/test_solvers.py:12-26) in real arithmetic
    a = np.linspace(1.0, 2.0, 5)
    a[-1] = 1e-3
    small5 = np.diag(a)
    small5[-1, 0] = 10.0
    small5[0, -1] = -10.0
    return {
        "x0R": np.random.default_rng(10).standard_normal(R.shape[0]),
        "small5": small5,
        "diag10": np.diag(np.arange(1.0, 11.0)),
        "b10": np.random.default_rng(9).standard_normal(10),
        "Pvar": Pvar,
        "Mj": sp.diags(1.0 / d).tocsr(),
        "S": sp.diags(1.0 / np.sqrt(d)).tocsr(),
        "R": R,
        "RMabs": sp.diags(1.0 / np.abs(dr)).tocsr(),
        "RMj": sp.diags(1.0 / dr).tocsr(),
        "B3": np.random.default_rng(8).standard_normal((n, 3)),
    }


# (fixture prefix, solver, operator, right-hand side, keyword arguments);
# string values of M / Ml / Mr name entries of inputs()
CASES = [
    ("cg_M", "cg", "Pvar", "ones", dict(M="Mj", tol=1e-8)),
    ("cg_Ml", "cg", "Pvar", "ones", dict(Ml="Mj", tol=0.0, maxiter=25)),
    ("cg_M_Ml", "cg", "Pvar", "ones", dict(M="Mj", Ml="S", tol=0.0, maxiter=25)),
    ("cg_M_blk3", "cg", "Pvar", "B3", dict(M="Mj", tol=1e-8)),
    ("gmres_M", "gmres", "R", "ones", dict(M="RMabs", tol=0.0, maxiter=30)),
    ("gmres_Ml", "gmres", "R", "ones", dict(Ml="RMj", tol=0.0, maxiter=30)),
    ("gmres_Mr", "gmres", "R", "ones", dict(Mr="RMj", tol=0.0, maxiter=30)),
    ("gmres_all", "gmres", "R", "ones", dict(M="RMabs", Ml="RMj", Mr="RMj", tol=0.0, maxiter=30)),
    ("gmres_M_mgs2", "gmres", "R", "ones", dict(M="RMabs", ortho="mgs2", tol=0.0, maxiter=20)),
    ("minres_M", "minres", "Pvar", "ones", dict(M="Mj", tol=1e-8)),
    ("minres_MlMr", "minres", "Pvar", "ones", dict(Ml="S", Mr="S", tol=1e-8)),
    ("minres_all", "minres", "Pvar", "ones", dict(M="Mj", Ml="S", Mr="S", tol=0.0, maxiter=40)),
    # Householder Arnoldi (arnoldi.py:33-104)
    ("gmres_hh", "gmres", "R", "ones", dict(ortho="householder", tol=0.0, maxiter=30)),
    ("gmres_hh_MlMr", "gmres", "R", "ones", dict(ortho="householder", Ml="RMj", Mr="RMj", tol=0.0, maxiter=20)),
    ("gmres_hh_small5", "gmres", "small5", "ones", dict(ortho="householder", tol=1e-12)),
    ("gmres_hh_small5_nx1", "gmres", "small5", "ones_nx1", dict(ortho="householder", tol=1e-12)),
    ("gmres_hh_diag10", "gmres", "diag10", "b10", dict(ortho="householder", tol=1e-15, atol=0.0)),
    # the other solvers (bicgstab.py, cgs.py, cgr.py, gcr.py)
    ("bicgstab_R", "bicgstab", "R", "ones", dict(tol=0.0, maxiter=20)),
    ("bicgstab_R_MlMr", "bicgstab", "R", "ones", dict(Ml="RMj", Mr="RMj", tol=0.0, maxiter=15)),
    ("bicgstab_Pvar", "bicgstab", "Pvar", "ones", dict(tol=1e-8)),
    ("bicgstab_R_x0", "bicgstab", "R", "ones", dict(x0="x0R", tol=0.0, maxiter=10)),
    ("cgs_R", "cgs", "R", "ones", dict(tol=0.0, maxiter=12)),
    ("cgs_Pvar_M", "cgs", "Pvar", "ones", dict(M="Mj", tol=1e-8)),
    ("cgr_Pvar", "cgr", "Pvar", "ones", dict(tol=1e-8)),
    ("cgr_Pvar_M", "cgr", "Pvar", "ones", dict(M="Mj", tol=1e-8)),
    ("cgr_Pvar_blk3", "cgr", "Pvar", "B3", dict(tol=1e-8)),
    ("gcr_R", "gcr", "R", "ones", dict(tol=0.0, maxiter=25)),
    ("gcr_Pvar_blk3", "gcr", "Pvar", "B3", dict(tol=1e-8)),
    ("gcr_R_x0", "gcr", "R", "ones", dict(x0="x0R", tol=0.0, maxiter=10)),
]


def build(case, q=None, wrap=None):
    """-> (solver name, A, b, kwargs) with the named matrices substituted;
    `wrap` maps each operator (e.g. to a device operator) if given."""
    q = inputs() if q is None else q
    prefix, solver, a, b, kw = case
    A = q[a]
    if b == "ones":
        bb = np.ones(A.shape[0])
    elif b == "ones_nx1":
        bb = np.ones((A.shape[0], 1))
    else:
        bb = q[b]
    out = {}
    for key, val in kw.items():
        if key in ("M", "Ml", "Mr"):
            val = q[val] if wrap is None else wrap(q[val])
        elif key == "x0":
            val = q[val]
        out[key] = val
    return solver, (A if wrap is None else wrap(A)), bb, out
