"""Generate the committed golden fixtures by running the REFERENCE itself.

Run only in the build container (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (``ju-liu/krylov`` 0.0.3, ``/root/reference/src``) is imported
read-only. It calls two names NumPy 2 removed (``np.find_common_type`` at
``_helpers.py:42`` / ``arnoldi.py:126,209`` and ``np.Infinity`` in
``utils.py``); they are re-added on the numpy module object before the import
(SURVEY.md §8(c)). Nothing in the reference tree is modified and no reference
source is copied: only inputs and outputs are stored.

Outputs (``tests/golden/``):
  spmv.npz        SciPy csr_matvec / csr_matvecs on adversarial CSR (bitwise)
  lartg.npz       scipy dlartg / slartg and krylov.givens on edge-case pairs
  solvers.npz     cg / gmres / minres histories and solutions on small problems
  precond.npz     the same with preconditioners M, Ml, Mr (make_precond)
  arnoldi.npz     cg(return_arnoldi=True) Lanczos relations (make_arnoldi)
  problems.json   SHA-256 of the generated BASELINE matrices
"""
import contextlib
import io
import json
import os
import sys

import numpy as np
import scipy.sparse
from scipy.linalg import lapack

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def _load_problems():
    """krylov_amd/problems.py by path: the generators are plain NumPy/SciPy, and
    importing the package would load libkrylov_hip.so (not needed here, and
    mid-rebuild while a long fixture run is going)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("_kry_problems", os.path.join(REPO, "krylov_amd", "problems.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


problems = _load_problems()


def _import_reference():
    if not hasattr(np, "find_common_type"):

        def find_common_type(array_types, scalar_types):
            assert list(scalar_types) == []
            return np.result_type(*array_types)

        np.find_common_type = find_common_type
    if not hasattr(np, "Infinity"):
        np.Infinity = np.inf
    sys.path.insert(0, "/root/reference/src")
    import krylov

    assert krylov.__file__.startswith("/root/reference/"), krylov.__file__
    return krylov


def adversarial_csr(n, seed, dtype, itype):
    """CSR with unsorted indices, duplicates, explicit zeros, empty rows, one
    long row and magnitudes spanning 1e-20..1e20."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 12, n)
    lens[rng.choice(n, n // 10, replace=False)] = 0
    lens[n // 3] = 3000  # longer than one LDS tile
    lens[n // 3 + 1] = 700
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=indptr[1:])
    nnz = int(indptr[-1])
    indices = rng.integers(0, n, nnz)
    # duplicates inside rows
    dup = rng.random(nnz) < 0.05
    indices[1:][dup[1:]] = indices[:-1][dup[1:]]
    mag = 10.0 ** rng.uniform(-20, 20, nnz)
    data = rng.choice([-1.0, 1.0], nnz) * mag
    data[rng.random(nnz) < 0.03] = 0.0
    A = scipy.sparse.csr_matrix(
        (data.astype(dtype), indices.astype(itype), indptr.astype(itype)),
        shape=(n, n),
    )
    assert not A.has_sorted_indices
    return A


def make_spmv():
    out = {}
    for dname, dt in (("f64", np.float64), ("f32", np.float32)):
        for iname, it in (("i32", np.int32), ("i64", np.int64)):
            A = adversarial_csr(2000, 7, dt, it)
            # scipy may downcast index dtype on construction; force it back
            A.indices = A.indices.astype(it)
            A.indptr = A.indptr.astype(it)
            rng = np.random.default_rng(11)
            x = (rng.standard_normal(2000) * 10.0 ** rng.uniform(-3, 3, 2000)).astype(dt)
            X = (rng.standard_normal((2000, 8))).astype(dt)
            key = f"{dname}_{iname}"
            out[f"{key}_indptr"] = A.indptr
            out[f"{key}_indices"] = A.indices
            out[f"{key}_data"] = A.data
            out[f"{key}_x"] = x
            out[f"{key}_y"] = A @ x
            out[f"{key}_X"] = X
            out[f"{key}_Y"] = A @ X
    np.savez_compressed(os.path.join(HERE, "spmv.npz"), **out)


def make_lartg(krylov):
    vals = [0.0, 1.0, -1.0, 3.0, -4.0, 1e-300, -1e-300, 1e300, -1e300, 5e-324,
            -5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, 1e8, 1e-8,
            1.4916681462400413e-154, 6.703903964971299e153, 1e154, 1e-154]
    rng = np.random.default_rng(3)
    pairs = [(f, g) for f in vals for g in vals]
    for _ in range(200):
        pairs.append(tuple(rng.standard_normal(2) * 10.0 ** rng.integers(-200, 200, 2)))
    fg = np.array(pairs, dtype=np.float64)
    d = np.array([lapack.dlartg(f, g) for f, g in fg])
    fg32 = fg.astype(np.float32)
    fin = np.all(np.isfinite(fg32), axis=1)
    fg32 = fg32[fin]
    s = np.array([lapack.slartg(f, g) for f, g in fg32], dtype=np.float32)
    # krylov.givens on a (2, k) block: G (2,2,k), r (k,)
    X = fg.T.copy()
    G, r = krylov.givens(X)
    np.savez_compressed(
        os.path.join(HERE, "lartg.npz"), fg=fg, d=d, fg32=fg32, s=s, givens_G=G, givens_r=r
    )


def _info_arrays(prefix, sol, info, out):
    out[f"{prefix}_success"] = np.array(info.success)
    out[f"{prefix}_numsteps"] = np.array(info.numsteps)
    out[f"{prefix}_resnorms"] = np.asarray(info.resnorms, dtype=np.float64)
    out[f"{prefix}_xk"] = np.asarray(info.xk)
    out[f"{prefix}_sol_is_none"] = np.array(sol is None)
    ops = info.num_operations
    if ops is None:  # bicgstab / cgs / cgr / gcr report none
        out[f"{prefix}_ops"] = np.full(6, np.nan)
    else:
        out[f"{prefix}_ops"] = np.array([ops[k] for k in ("A", "M", "Ml", "Mr", "inner", "axpy")], dtype=np.float64)


def make_solvers(krylov):
    out = {}
    quiet = contextlib.redirect_stdout(io.StringIO())  # gmres.py:201-205 prints

    # cfg1: README diag-100, default tol, 1-D and (n,1)
    A, b = problems.diag100()
    for shape_name, bb in (("1d", b), ("nx1", b[:, None])):
        for name in ("cg", "gmres", "minres"):
            with quiet:
                sol, info = getattr(krylov, name)(A, bb)
            _info_arrays(f"diag100_{name}_{shape_name}", sol, info, out)

    # CG on Poisson 64^2, 1-D and 8 columns, tol 1e-8
    P = problems.poisson2d(64)
    n = P.shape[0]
    B = np.random.default_rng(0).standard_normal((n, 8))
    out["poisson64_B"] = B
    with quiet:
        sol, info = krylov.cg(P, np.ones(n), tol=1e-8)
    _info_arrays("cg_poisson64_1d", sol, info, out)
    with quiet:
        sol, info = krylov.cg(P, B, tol=1e-8)
    _info_arrays("cg_poisson64_blk8", sol, info, out)
    # CG on the 15-point stencil at 24^3, b = ones
    S = problems.stencil15_3d(24)
    with quiet:
        sol, info = krylov.cg(S, np.ones(S.shape[0]), tol=1e-8)
    _info_arrays("cg_st15_24", sol, info, out)
    # CG with a nonzero x0
    x0 = np.random.default_rng(5).standard_normal(n)
    with quiet:
        sol, info = krylov.cg(P, np.ones(n), x0=x0, tol=1e-6, maxiter=150)
    out["poisson64_x0"] = x0
    _info_arrays("cg_poisson64_x0", sol, info, out)

    # GMRES(30) on random nonsym n=5000, tol=0, mgs / mgs2
    R = problems.random_nonsym(5000)
    bR = np.ones(R.shape[0])
    for ortho in ("mgs", "mgs2"):
        with quiet:
            sol, info = krylov.gmres(R, bR, ortho=ortho, maxiter=30, tol=0.0)
        _info_arrays(f"gmres_rand5k_{ortho}", sol, info, out)
    # restarted GMRES(30) by x0-chaining to 1e-8 relative
    x = np.zeros_like(bR)
    bnorm = np.linalg.norm(bR)
    hist = []
    cycles = 0
    while cycles < 20:
        with quiet:
            sol, info = krylov.gmres(R, bR, x0=x, maxiter=30, tol=1e-8 * bnorm / max(np.linalg.norm(bR - R @ x), 1e-300))
        hist.extend(list(np.asarray(info.resnorms, dtype=np.float64)))
        x = info.xk
        cycles += 1
        if info.success:
            break
    out["gmres_restart_hist"] = np.array(hist)
    out["gmres_restart_x"] = x
    out["gmres_restart_cycles"] = np.array(cycles)
    # GMRES with a block rhs (3 columns)
    B3 = np.random.default_rng(2).standard_normal((R.shape[0], 3))
    out["rand5k_B3"] = B3
    with quiet:
        sol, info = krylov.gmres(R, B3, maxiter=20, tol=0.0)
    _info_arrays("gmres_rand5k_blk3", sol, info, out)

    # MINRES fp64 on Poisson 64^2 and fp32 weighted at 20^3 (50 fixed iters)
    with quiet:
        sol, info = krylov.minres(P, np.ones(n), tol=1e-8)
    _info_arrays("minres_poisson64", sol, info, out)
    W, w = problems.shifted_lap3d_weighted(20)
    bW = np.ones(W.shape[0], dtype=np.float32)

    def inner(x, y):
        return np.dot(x.T, w * y)

    with quiet:
        sol, info = krylov.minres(W, bW, inner=inner, tol=0.0, maxiter=50)
    out["minres_w20_w"] = w
    _info_arrays("minres_w20_f32", sol, info, out)
    # CG with the weighted inner product on the same (fp64) operator
    W64 = W.astype(np.float64)
    with quiet:
        sol, info = krylov.cg(W64, np.ones(W.shape[0]), inner=inner, tol=1e-8)
    _info_arrays("cg_w20_weighted", sol, info, out)
    out.update(make_weighted_spd(krylov))

    np.savez_compressed(os.path.join(HERE, "solvers.npz"), **out)


def make_weighted_spd(krylov):
    """CG with the weighted inner product on a positive definite operator
    (round 4): the 20^3 Laplacian with no shift (sigma = 0), row-scaled by
    1/w, so that A is self-adjoint and positive definite in <x, y>_W. The
    cg_w20_weighted case above runs CG on the shifted, indefinite operator,
    whose 641-step history is chaotic in the summation order; this one
    converges in 87 steps and its history moves by <= 1.3e-12 when only the
    summation order changes, so the weighted path is pinned at 1e-10."""
    out = {}
    W, w = problems.shifted_lap3d_weighted(20, sigma=0.0)

    def inner(x, y):
        return np.dot(x.T, w * y)

    with contextlib.redirect_stdout(io.StringIO()):
        sol, info = krylov.cg(W.astype(np.float64), np.ones(W.shape[0]), inner=inner, tol=1e-8)
    _info_arrays("cg_w20spd_weighted", sol, info, out)
    return out


def make_precond(krylov):
    from tests import solver_cases

    out = {}
    quiet = contextlib.redirect_stdout(io.StringIO())
    q = solver_cases.inputs()
    for case in solver_cases.CASES:
        solver, A, b, kw = solver_cases.build(case, q)
        with quiet:
            sol, info = getattr(krylov, solver)(A, b, **kw)
        _info_arrays(case[0], sol, info, out)
    np.savez_compressed(os.path.join(HERE, "precond.npz"), **out)


def make_arnoldi(krylov):
    """cg(..., return_arnoldi=True): the Lanczos relation [V, H, P]
    (cg.py:140-148, 218-258) on the reference's test problem
    (tests/test_solvers.py:41-50) and on Poisson 16^2 with a Jacobi M."""
    import scipy.sparse as sp

    out = {}
    a = np.linspace(1.0, 2.0, 5)
    a[-1] = 1e-2
    cases = [("diag_1d", np.diag(a), np.ones(5), {}), ("diag_blk3", np.diag(a), np.ones((5, 3)), {})]
    P = problems.poisson2d(16)
    d = P.diagonal() + np.random.default_rng(3).uniform(0.0, 1.0, P.shape[0])
    Pv = (P + sp.diags(d - P.diagonal())).tocsr()
    cases.append(("pvar16_M", Pv, np.ones(Pv.shape[0]), {"M": sp.diags(1.0 / d).tocsr()}))
    for name, A, b, kw in cases:
        _, info = krylov.cg(A, b, tol=1.0e-7, return_arnoldi=True, **kw)
        V, H, Pb = info.arnoldi
        _info_arrays(f"arnoldi_{name}", None if not info.success else info.xk, info, out)
        out[f"arnoldi_{name}_V"] = np.array(V)
        out[f"arnoldi_{name}_H"] = np.asarray(H)
        out[f"arnoldi_{name}_P"] = np.array(Pb)
    np.savez_compressed(os.path.join(HERE, "arnoldi.npz"), **out)


def make_problem_hashes():
    out = {}
    for name, fn in (
        ("stencil15_3d_24", lambda: problems.stencil15_3d(24)),
        ("stencil15_3d_216", lambda: problems.stencil15_3d(216)),
        ("poisson2d_64", lambda: problems.poisson2d(64)),
        ("poisson2d_1000", lambda: problems.poisson2d(1000)),
        ("random_nonsym_5000", lambda: problems.random_nonsym(5000)),
        ("random_nonsym_2000000", lambda: problems.random_nonsym(2_000_000)),
        ("shifted_lap3d_weighted_20", lambda: problems.shifted_lap3d_weighted(20)[0]),
        ("shifted_lap3d_weighted_200", lambda: problems.shifted_lap3d_weighted(200)[0]),
    ):
        A = fn()
        out[name] = {"n": A.shape[0], "nnz": int(A.nnz), "sha256": problems.csr_sha256(A)}
        del A
    with open(os.path.join(HERE, "problems.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    krylov = _import_reference()
    if "--only-weighted-spd" in sys.argv:  # append to the existing solvers.npz
        path = os.path.join(HERE, "solvers.npz")
        out = dict(np.load(path))
        out.update(make_weighted_spd(krylov))
        np.savez_compressed(path, **out)
        sys.exit(0)
    if "--only-precond" in sys.argv:
        make_precond(krylov)
        make_arnoldi(krylov)
        sys.exit(0)
    make_spmv()
    make_lartg(krylov)
    make_solvers(krylov)
    make_precond(krylov)
    make_arnoldi(krylov)
    if "--no-large" not in sys.argv:
        make_problem_hashes()
    print("golden fixtures written to", HERE)
