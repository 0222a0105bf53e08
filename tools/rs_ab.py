"""A/B of the rank-sorted SpMV kernels on the renumbered permuted metric
(bench.py's spmv_unstructured matrix): the paired kernel (two rows per lane,
KRY_SPMV_RS1=0) against the one-row-per-lane kernel (KRY_SPMV_RS1=1, eight
slot columns' loads in flight; 2: sixteen), y = A x in the operator's
numbering (kry_spmv_op), HIP-event timed, bitwise compared.

    python3 tools/rs_ab.py [reps]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import krylov_amd  # noqa: E402
from krylov_amd import problems  # noqa: E402
from krylov_amd.device import DeviceVector  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
A = problems.permuted_sym(problems.stencil15_3d(216), 0)
op = krylov_amd.CsrOperator(A)
lay = op.layout()
assert lay["rs"] and lay["renumbered"], lay
n = A.shape[0]
x = DeviceVector.from_host(op.ctx, np.random.default_rng(1).standard_normal((n, 1)))
y = DeviceVector(op.ctx, n, 1, np.float64)
nbytes = 1968960144  # bench.py spmv_unstructured bytes_per_launch (rs image + x + y)
ref = None
for rep in range(2):
    for mode in ("0", "1", "2"):
        os.environ["KRY_SPMV_RS1"] = mode
        op.matvec_op(x, y)
        op.ctx.synchronize()
        got = y.to_host()
        if ref is None:
            ref = got.copy()
        same = np.array_equal(got.view(np.uint64), ref.view(np.uint64))
        op.ctx.timer_start()
        for _ in range(reps):
            op.matvec_op(x, y)
        ms = op.ctx.timer_stop() / reps
        print(f"KRY_SPMV_RS1={mode}: {ms:.4f} ms per SpMV, {nbytes / ms / 1e6:.0f} GB/s of image+vectors, "
              f"bitwise {'same' if same else 'DIFFERENT'}", flush=True)
