"""Debug probe: one-launch CG update vs separate passes, step by step
(x = 0 + y and r after each step, scalars)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import krylov_amd
from krylov_amd import _helpers, problems
from krylov_amd.cg import _CGState

dtype = np.float32 if (len(sys.argv) < 2 or sys.argv[1] == "f32") else np.float64
m = int(sys.argv[2]) if len(sys.argv) > 2 else 300
R = problems.poisson2d(m).astype(dtype)
A = krylov_amd.CsrOperator(R)
b = np.random.default_rng(3).standard_normal(R.shape[0]).astype(dtype)
res = {}
for upd in ("1", "0"):
    os.environ["KRY_CG_UPD"] = upd
    os.environ["KRY_CG_PERSIST"] = "0"
    st = _CGState(_helpers.Problem(A, b, None, None))
    st.start()
    st.set_criterion(np.zeros(st.prob.kpad))
    rows = []
    for i in range(4):
        h = st.run(1)
        rows.append((h[0, 0], st.get(0)[:, 0].copy(), st.get(1)[:, 0].copy(), st.scalars()[:, 0].copy()))
    res[upd] = rows
    print("upd", upd, st.update_path(), [r[0] for r in rows], flush=True)
for i in range(4):
    a, c = res["1"][i], res["0"][i]
    print(i, "hist", a[0], c[0], "x maxdiff", np.abs(a[1] - c[1]).max(), "r maxdiff", np.abs(a[2] - c[2]).max(),
          "scal", a[3], c[3], "nonzero r diff idx", np.flatnonzero(np.abs(a[2] - c[2]) > 1e-3 * np.abs(c[2]).max())[:10])
a, c = res["1"][0], res["0"][0]
bad = np.flatnonzero(a[2] != c[2])
W = 4 if dtype == np.float32 else 2
NV = 8
seg = NV * 512 * W
blk, within = bad // seg, bad % seg
u, tid, v = within // (512 * W), (within % (512 * W)) // W, within % W
print("bad", bad.size, "of", a[2].size)
for name, arr in (("blk", blk), ("u", u), ("tid", tid), ("v", v)):
    vals, cnt = np.unique(arr, return_counts=True)
    print(name, dict(zip(vals.tolist()[:40], cnt.tolist()[:40])))
print("sample", [(int(i), float(a[2][i]), float(c[2][i])) for i in bad[:6]])
