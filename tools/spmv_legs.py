"""The metric CG's SpMV kernels in one process, for rocprofv3 --pmc passes
(tools/pmc_traffic.sh): 64 CG iterations on the DIA image (spmv_dia_kernel),
64 with KRY_SPMV_DIA=0 (the paired-row SELL-128 kernel general CSR takes,
spmv_pair_kernel) and 64 with KRY_SPMV_DIA=0 KRY_SPMV_PAIR=0 (the compact
SELL-64 kernel), each on the 216^3 15-point stencil."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from krylov_amd import problems  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
A = problems.stencil15_3d(216)
r = bench.run_cg_bench(A, lambda _r: np.ones(A.shape[0]), steps, 0, bench.Job.single(), roofline_launches=1)
print("dia", r["layout"]["dia"], "spmv_ms", 1e3 * r["spmv_avg_s"], flush=True)
g = bench.run_spmv_general(A, steps)
print("general", g["kernel"].split(" ")[0], "spmv_ms", g["spmv_ms"], flush=True)
os.environ["KRY_SPMV_PAIR"] = "0"
g = bench.run_spmv_general(A, steps)
print("general (KRY_SPMV_PAIR=0)", g["kernel"].split(" ")[0], "spmv_ms", g["spmv_ms"], flush=True)
