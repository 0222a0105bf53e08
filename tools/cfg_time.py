"""One secondary BASELINE config on its own, for a kernel trace:
`python tools/cfg_time.py metric|cfg4|cfg5|cfg2|gmres_cfg3 [steps]` or `gmres_metric [m]` (run under
`rocprofv3 --kernel-trace --stats` to split an iteration by kernel)."""
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
