"""One bench leg on its own, for a kernel trace or a PMC pass:
`python tools/cfg_time.py metric|general|unstructured|cfg4|cfg5|cfg2|gmres_cfg3|bicgstab_cfg3 [steps]` or
`gmres_metric [m]` (run under `rocprofv3 --kernel-trace --stats` to split an iteration by kernel, or under
tools/pmc_legs.sh for the traffic index)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from krylov_amd import problems  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
if cfg == "cfg4":
    P3 = problems.poisson2d(3163)
    B = np.random.default_rng(0).standard_normal((P3.shape[0], 8))
    print(cfg, bench.run_cg_config(P3, B, steps, 3), flush=True)
elif cfg == "cfg2":
    print(cfg, bench.run_cg_config(problems.poisson2d(1000), np.ones(1_000_000), steps, 10), flush=True)
elif cfg == "cfg5":
    print(cfg, bench.run_minres_cfg5(steps), flush=True)
elif cfg == "gmres_metric":
    m = steps if len(sys.argv) > 2 else 216
    print(cfg, bench.run_gmres(problems.stencil15_3d(m), f"metric {m}^3 GMRES(30)"), flush=True)
elif cfg == "metric":
    A = problems.stencil15_3d(216)
    r = bench.run_cg_bench(A, lambda _r: np.ones(A.shape[0]), 200, 20, bench.Job.single())
    print(cfg, {"it_per_s": 200 / r["elapsed"], "spmv_ms": 1e3 * r["spmv_avg_s"]}, flush=True)
elif cfg == "gmres_cfg3":
    print(cfg, bench.run_gmres(), flush=True)
elif cfg == "general":  # the metric matrix on the paired-row image (KRY_SPMV_DIA=0), bench's spmv_general
    r = bench.run_spmv_general(problems.stencil15_3d(216), steps)
    print(cfg, {"it_per_s": r["cg_it_per_s"], "spmv_ms": r["spmv_ms"]}, flush=True)
elif cfg == "unstructured":  # the permuted metric (renumbered, rank-sorted image), bench's spmv_unstructured
    r = bench.run_spmv_unstructured(problems.stencil15_3d(216), steps)
    print(cfg, {"it_per_s": r["cg_it_per_s"], "spmv_ms": r["ms_per_launch"]}, flush=True)
elif cfg == "bicgstab_cfg3":
    r = bench.run_bicgstab(problems.random_nonsym(2_000_000), steps)
    print(cfg, {"it_per_s": r["it_per_s"], "spmv_ms": r["roofline"]["ms_per_launch"]}, flush=True)
