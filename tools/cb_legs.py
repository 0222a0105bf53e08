"""The SpMV of a scattered matrix alone, for rocprofv3 --pmc passes
(tools/pmc_passes.sh): REPS launches of y = A x on cfg3 (random nonsymmetric,
n = 2e6; the column-blocked spmv_cbp_kernel) or on the metric matrix under a
random symmetric permutation (bench.py's spmv_unstructured): "permuted" as
given (KRY_RENUMBER=0: column-blocked), "permuted_rs" renumbered at upload
(round 5: the rank-sorted spmv_rs1_kernel, plus the two row permutations of
kry_spmv). x uploaded and y downloaded per call (the counters are per kernel).

    python3 tools/cb_legs.py cfg3|permuted|permuted_rs [REPS]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import krylov_amd  # noqa: E402
from krylov_amd import problems  # noqa: E402

which = sys.argv[1]
if which == "permuted":
    os.environ["KRY_RENUMBER"] = "0"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
A = problems.random_nonsym(2_000_000) if which == "cfg3" else problems.permuted_sym(problems.stencil15_3d(216), 0)
op = krylov_amd.CsrOperator(A)
if which == "permuted_rs":
    assert op.layout()["rs"] and op.layout()["renumbered"], op.layout()
else:
    assert op.layout()["col_blocks"] > 0, op.layout()
y = op @ np.ones(A.shape[0])
for _ in range(reps):
    y = op @ np.ones(A.shape[0])
print(which, op.layout(), float(np.sum(y)), flush=True)
