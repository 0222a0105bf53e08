"""Device history of the weighted fp64 CG on the shifted 20^3 Laplacian
(tests/test_gpu_solvers.py::test_cg_weighted_histories) saved for comparison
with the reference's summation-order spread (tests/golden/selfnoise.npz)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import krylov_amd  # noqa: E402
from krylov_amd import problems  # noqa: E402

W, w = problems.shifted_lap3d_weighted(20)
_, info = krylov_amd.cg(W.astype(np.float64), np.ones(W.shape[0]), inner=krylov_amd.WeightedInner(w), tol=1e-8)
out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "w20_device.npy")
np.save(out, np.asarray(info.resnorms, dtype=np.float64))
print("numsteps", info.numsteps, "saved", out)
