"""The REFERENCE's own summation-order noise on the full-size CG histories.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_selfnoise.py

The parity contract compares the device history with the one the reference
recorded here (tests/golden/fullsize.npz, solvers.npz). The device sums its
inner products in a different (two-stage tree) order from OpenBLAS's ddot.
This script measures how far the reference's history moves by itself when
only the summation order of its inner product changes, every other line of
``krylov.cg`` (cg.py:16-259) running unchanged:

  blas1      default inner (np.dot, _helpers.py:104-105), OPENBLAS_NUM_THREADS=1
  blas2/4    the same with 2 / 4 OpenBLAS threads (ddot splits the vector into
             one partial sum per thread, so the order changes with the count)
  blasN      the same with the container's default thread count (8): the
             configuration the committed fixtures were recorded under
  pairwise   inner = numpy's pairwise sum of the products (np.add.reduce)
  longdouble inner = dot accumulated in x87 extended precision, rounded once
  fsum       inner = math.fsum of the products: the correctly rounded sum
  permK      (small cases only) inner = numpy's pairwise sum of the products
             taken in a fixed random order (permutation seed K, 0..39)

Each variant is a valid evaluation of the reference's <x, y>; the spread
between them is the reference's own rounding noise. Every variant runs in
its own process (the OpenBLAS thread count is fixed at load time).

Output: tests/golden/selfnoise.npz with, per case, every variant's history
(``{case}_{variant}``). tests/test_gpu_fullsize_golden.py derives its
per-entry tolerance from them.
"""
import contextlib
import io
import math
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

CASES = {
    # name: (generator, tol, inner kind) -- the fixture cases of make_fullsize.py
    # and make_golden.py these histories stand beside
    "metric_cg": ("stencil15_3d(216)", 1e-8, "default"),
    "cfg2_cg": ("poisson2d(1000)", 1e-8, "default"),
    "cg_w20_weighted": ("shifted_lap3d_weighted(20)", 1e-8, "weighted"),
    # round 4: the positive definite weighted case (make_golden.make_weighted_spd)
    "cg_w20spd_weighted": ("shifted_lap3d_weighted(20, sigma=0.0)", 1e-8, "weighted"),
    # round 5: the metric matrix under a random symmetric permutation (the
    # renumbered path's case, tests/golden/permuted.npz): its rows sum in a
    # scattered order, and its history is more sensitive to the inner
    # product's order than the stencil-ordered metric's
    "perm_cg": ("permuted_sym(problems.stencil15_3d(216), 0)", 1e-8, "default"),
}
SMALL_CASES = ("cg_w20_weighted", "cg_w20spd_weighted")
VARIANTS = {
    "blas1": {"OPENBLAS_NUM_THREADS": "1"},
    "blas2": {"OPENBLAS_NUM_THREADS": "2"},
    "blas4": {"OPENBLAS_NUM_THREADS": "4"},
    "blasN": {},
    "pairwise": {},
    "longdouble": {},
    "fsum": {},
}


SMALL_ONLY = tuple(f"perm{k}" for k in range(40))
for _v in SMALL_ONLY:
    VARIANTS[_v] = {}


def _perm_inner(seed, n, w=None):
    perm = np.random.default_rng(seed).permutation(n)
    if w is None:
        return lambda x, y: np.add.reduce((x.conj() * y)[perm])
    return lambda x, y: np.add.reduce((x * (w * y))[perm])


def _inner_for(variant, kind, w, n):
    """The inner product a variant hands to krylov.cg (None = the reference's
    default np.dot)."""
    if variant.startswith("perm"):
        return _perm_inner(int(variant[4:]), n, None if kind == "default" else w)
    if kind == "default":
        if variant.startswith("blas"):
            return None
        if variant == "pairwise":
            return lambda x, y: np.add.reduce(x.conj() * y)
        if variant == "fsum":
            return lambda x, y: np.float64(math.fsum(x.conj() * y))
        return lambda x, y: np.float64(np.dot(x.astype(np.longdouble), y.astype(np.longdouble)))
    # tests/test_solvers.py:157-161 weighted form np.dot(x.T, w * y)
    if variant.startswith("blas"):
        return lambda x, y: np.dot(x.T, w * y)
    if variant == "pairwise":
        return lambda x, y: np.add.reduce(x * (w * y))
    if variant == "fsum":
        return lambda x, y: np.float64(math.fsum(x * (w * y)))
    return lambda x, y: np.float64(np.dot(x.astype(np.longdouble), (w * y).astype(np.longdouble)))


def run_one(case, variant, out_path):
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    from make_golden import _import_reference, problems

    krylov = _import_reference()
    gen, tol, kind = CASES[case]
    made = eval(f"problems.{gen}")  # generator names above are fixed strings
    if kind == "weighted":
        W, w = made
        A = W.astype(np.float64)
    else:
        A, w = made, None
    b = np.ones(A.shape[0])
    t = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        _, info = krylov.cg(A, b, tol=tol, inner=_inner_for(variant, kind, w, A.shape[0]))
    np.save(out_path, np.asarray(info.resnorms, dtype=np.float64))
    print(f"{case} {variant}: {info.numsteps} steps, {time.time() - t:.0f}s", flush=True)


def main():
    """Usage: make_selfnoise.py [--jobs J] [case ...]: the missing variants of
    the named cases (all by default), J processes at a time."""
    args = sys.argv[1:]
    jobs = 1
    if args[:1] == ["--jobs"]:
        jobs, args = int(args[1]), args[2:]
    only = args
    out = {}
    path = os.path.join(HERE, "selfnoise.npz")
    if os.path.exists(path):
        out.update(dict(np.load(path)))
    todo = []
    for case in CASES:
        if only and case not in only:
            continue
        for variant, env in VARIANTS.items():
            if f"{case}_{variant}" in out:  # recorded by an earlier run
                continue
            if variant in SMALL_ONLY and case not in SMALL_CASES:
                continue
            todo.append((case, variant, env))
    for i in range(0, len(todo), jobs):
        procs = []
        for case, variant, env in todo[i:i + jobs]:
            tmp = os.path.join(HERE, f"_selfnoise_tmp_{case}_{variant}.npy")
            e = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", **env)
            procs.append((case, variant, tmp, subprocess.Popen([sys.executable, __file__, "--one", case, variant, tmp],
                                                               env=e)))
        for case, variant, tmp, pr in procs:
            if pr.wait() != 0:
                raise RuntimeError(f"{case} {variant} failed")
            out[f"{case}_{variant}"] = np.load(tmp)
            os.remove(tmp)
        np.savez_compressed(path, **out)
    print("written", path)


if __name__ == "__main__":
    if len(sys.argv) == 5 and sys.argv[1] == "--one":
        run_one(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        main()
