"""Wall-clock of CsrOperator(A) (kry_csr_create: host image build + H2D) on
the BASELINE matrices, with KRY_UPLOAD_TRACE=1's per-phase split on stderr.
Usage: python tools/upload_time.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KRY_UPLOAD_TRACE"] = "1"
os.environ["KRYLOV_CSR_CACHE"] = "0"
import krylov_amd  # noqa: E402
from krylov_amd import problems  # noqa: E402
from krylov_amd.device import get_context  # noqa: E402

get_context()
cases = [("metric 15-pt 216^3", lambda: problems.stencil15_3d(216), {}),
         ("metric, KRY_SPMV_DIA=0", lambda: problems.stencil15_3d(216), {"KRY_SPMV_DIA": "0"}),
         ("cfg3 random n=2e6", lambda: problems.random_nonsym(2_000_000, seed=0), {}),
         ("cfg4 Poisson 3163^2", lambda: problems.poisson2d(3163), {})]
for name, make, env in cases:
    A = make()
    for k, v in env.items():
        os.environ[k] = v
    for rep in range(2):
        print(f"== {name} (call {rep + 1})", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        op = krylov_amd.CsrOperator(A)
        get_context().synchronize()
        t1 = time.perf_counter()
        print(f"{name:28s} call {rep + 1}: {1e3 * (t1 - t0):8.1f} ms  layout {op.layout()}", flush=True)
        del op
    for k in env:
        del os.environ[k]
