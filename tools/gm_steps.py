"""GMRES(30) cycles on the metric matrix (15-point 216^3) or cfg3, for a
rocprofv3 kernel trace: the per-launch durations of the persistent MGS kernel
in launch order give its cost per Arnoldi step j (tools/gm_steps_summary.py).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o gm -- python3 tools/gm_steps.py metric 2
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(which="metric", reps=2):
    import krylov_amd
    from krylov_amd import problems

    if which.startswith("metric"):
        M = problems.stencil15_3d(216)
    else:
        M = problems.random_nonsym(2_000_000)
    dt = np.float32 if which.endswith("32") else np.float64  # metric32: the same matrix in fp32
    M = M.astype(dt)
    A = krylov_amd.CsrOperator(M)
    b = np.ones(M.shape[0], dtype=dt)
    krylov_amd.gmres(A, b, tol=0.0, atol=0.0, maxiter=30)  # warm-up
    for _ in range(reps):
        t0 = time.perf_counter()
        krylov_amd.gmres(A, b, tol=0.0, atol=0.0, maxiter=30)
        print(f"{which} gmres(30) cycle {1e3 * (time.perf_counter() - t0):.2f} ms (incl. host)", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "metric", int(sys.argv[2]) if len(sys.argv) > 2 else 2)
