"""One GMRES(30) cycle on the cfg3 matrix (random nonsymmetric, n = 2e6),
repeated; a target for rocprofv3 counter passes (tools/pmc_gmres.sh)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps=3):
    import krylov_amd
    from krylov_amd import problems

    R = problems.random_nonsym(2_000_000)
    A = krylov_amd.CsrOperator(R)
    print("layout", A.layout(), flush=True)
    b = np.ones(R.shape[0])
    for _ in range(reps):
        t0 = time.perf_counter()
        krylov_amd.gmres(A, b, tol=0.0, atol=0.0, maxiter=30)
        print(f"gmres(30) cycle {1e3 * (time.perf_counter() - t0):.2f} ms (incl. host)", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
