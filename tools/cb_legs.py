"""The column-blocked SpMV (spmv_cbp_kernel) alone, for rocprofv3 --pmc passes
(tools/pmc_passes.sh): REPS launches of y = A x on cfg3 (random nonsymmetric,
n = 2e6) or on the metric matrix under a random symmetric permutation
(bench.py's spmv_unstructured), x uploaded and y downloaded per call (the counters are per kernel).

    python3 tools/cb_legs.py cfg3|permuted [REPS]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import krylov_amd  # noqa: E402
from krylov_amd import problems  # noqa: E402

which = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
A = problems.random_nonsym(2_000_000) if which == "cfg3" else problems.permuted_sym(problems.stencil15_3d(216), 0)
op = krylov_amd.CsrOperator(A)
assert op.layout()["col_blocks"] > 0, op.layout()
y = op @ np.ones(A.shape[0])
for _ in range(reps):
    y = op @ np.ones(A.shape[0])
print(which, op.layout(), float(np.sum(y)), flush=True)
