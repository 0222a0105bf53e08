import sys, time, os
sys.path.insert(0, os.getcwd())
import numpy as np, bench
from krylov_amd import problems, _lib
import krylov_amd
from krylov_amd.device import get_context
A_host = problems.stencil15_3d(216)
ctx = get_context(0)
A = krylov_amd.CsrOperator(A_host)
st, ncols = bench._cg_state(A, np.ones(A.n))
chunk = st.preferred_chunk()
for mode in ["none", "spmv", "all", "none", "spmv", "all"]:
    bench._iterate(st, 20, ncols, chunk); ctx.synchronize()
    if mode == "spmv": ctx.profile(True, kernels=[_lib.PROF_SPMV])
    elif mode == "all": ctx.profile(True)
    t0 = time.perf_counter(); bench._iterate(st, 200, ncols, chunk); ctx.synchronize(); t = time.perf_counter() - t0
    ctx.profile(False)
    print(mode, "%.1f it/s  %.1f us/it" % (200 / t, 1e6 * t / 200), flush=True)
