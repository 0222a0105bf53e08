"""Golden history of the reference's CG on the PERMUTED metric matrix
(problems.permuted_sym(stencil15_3d(216), 0): the bench's spmv_unstructured
matrix), to tol 1e-8, b = ones (round 5). The permutation changes the order in
which every row of the SpMV is summed, so the history differs from the metric
fixture (fullsize.npz, metric_cg) beyond the reference's inner-product
self-noise late in the run; the renumbered device path is compared with
this, the reference on the same matrix.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_permuted.py

The reference is imported read-only exactly as in make_golden.py. Output:
tests/golden/permuted.npz (numsteps, success, resnorms, xstats). ~2 minutes on
8 cores.
"""
import contextlib
import io
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from krylov_amd import problems  # noqa: E402
from make_golden import _import_reference  # noqa: E402


def main():
    krylov = _import_reference()
    A = problems.permuted_sym(problems.stencil15_3d(216), 0)
    b = np.ones(A.shape[0])
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        _, info = krylov.cg(A, b, tol=1e-8)
    x = np.asarray(info.xk, dtype=np.float64)
    xa = np.abs(x)
    out = {"perm_cg_success": np.array(info.success), "perm_cg_numsteps": np.array(info.numsteps),
           "perm_cg_resnorms": np.asarray(info.resnorms, dtype=np.float64),
           "perm_cg_xstats": np.array([xa.sum(), np.sqrt((xa * xa).sum()), xa.max()])}
    np.savez_compressed(os.path.join(HERE, "permuted.npz"), **out)
    print(f"perm_cg: {info.numsteps} steps, success {info.success}, {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
