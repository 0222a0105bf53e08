"""Host round trips between chunks: CG iterations/s on the metric matrix (one
RHS, the one-launch update path) and on cfg4 (8 RHS, deferred yk) when the
host enqueues `chunk` iterations per kry_cg_run (one sync per chunk), as the
drivers do with kry_cg_preferred_chunk (32 on the launch-per-pass path).

    python3 tools/chunk_time.py [metric|cfg4] [steps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import krylov_amd  # noqa: E402
from krylov_amd import problems  # noqa: E402
from krylov_amd.device import get_context  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "metric"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 256
if which == "metric":
    A_host, B = problems.stencil15_3d(216), None
    B = np.ones(A_host.shape[0])
else:
    A_host = problems.poisson2d(3163)
    B = bench.cfg4_rhs(A_host.shape[0], 0)
ctx = get_context()
A = krylov_amd.CsrOperator(A_host)
st, ncols = bench._cg_state(A, B)
print(which, "preferred chunk", st.preferred_chunk(), flush=True)
bench._iterate(st, 64, ncols, 32)
for rep in range(2):
    for chunk in (32, 64, 128, 256):
        ctx.synchronize()
        t0 = time.perf_counter()
        bench._iterate(st, steps, ncols, chunk)
        ctx.synchronize()
        t = time.perf_counter() - t0
        print(f"{which} chunk {chunk:4d}: {steps / t:9.1f} it/s  {1e3 * t / steps:.4f} ms/it", flush=True)
