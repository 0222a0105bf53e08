"""Timing probe for the persistent CG loop (Poisson m^2, default cfg2's
1000^2): us per iteration of the persistent loop and of the launch-per-pass
path; `trace` adds the kernel's per-phase wall-clock split (KRY_CGP_TRACE)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from krylov_amd import problems  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
R = problems.poisson2d(m)
if "trace" in sys.argv:
    os.environ["KRY_CG_PERSIST"] = "2"
    os.environ["KRY_CGP_TRACE"] = "1"
    bench.run_cg_config(R, np.ones(R.shape[0]), 96, 32)
    del os.environ["KRY_CGP_TRACE"]
for mode in ("2", "0"):
    os.environ["KRY_CG_PERSIST"] = mode
    r = bench.run_cg_config(R, np.ones(R.shape[0]), 640, 64)
    print(f"persist={mode}: {r['us_per_it']:.2f} us/it", flush=True)
