"""Timing probe for the persistent CG loop on cfg2 (Poisson 1000^2): per
iteration time under KRY_CGP_DBG variants (1 no gathers, 2 no release /
acquire, 4 no SpMV, 8 no release, 16 no acquire, 32 write-through R / P stores; results wrong by design) and the pass path."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import krylov_amd  # noqa: E402
from krylov_amd import problems  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
R = problems.poisson2d(m)
for mode, dbg in [("2", "0"), ("2", "1"), ("0", "0")]:
    os.environ["KRY_CG_PERSIST"] = mode
    os.environ["KRY_CGP_DBG"] = dbg
    r = bench.run_cg_config(R, np.ones(R.shape[0]), 640, 64)
    print(f"persist={mode} dbg={dbg}: {r['us_per_it']:.2f} us/it", flush=True)
