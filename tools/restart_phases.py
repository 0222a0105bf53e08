"""Where the wall time of krylov_amd.gmres_restarted goes on the metric
matrix (10 x0-chained GMRES(30) cycles): each _GmresState method wrapped with
a host timer that synchronises the stream first and last, plus the call's
setup (Problem: b upload, ||b||) and the final download, against the
single-cycle time bench.py reports (run(30) + solution()).

    python3 tools/restart_phases.py [cycles]
"""
import os
import sys
import time
from collections import defaultdict

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import krylov_amd  # noqa: E402
from krylov_amd import problems  # noqa: E402
from krylov_amd.device import get_context  # noqa: E402

gm = sys.modules["krylov_amd.gmres"]
cycles = int(sys.argv[1]) if len(sys.argv) > 1 else 10
A = krylov_amd.CsrOperator(problems.stencil15_3d(216))
b = np.ones(A.n)
ctx = get_context()
tot = defaultdict(float)
cnt = defaultdict(int)


def wrap(cls, name):
    f = getattr(cls, name)

    def g(*a, **k):
        ctx.synchronize()
        t0 = time.perf_counter()
        r = f(*a, **k)
        ctx.synchronize()
        tot[name] += time.perf_counter() - t0
        cnt[name] += 1
        return r

    setattr(cls, name, g)


def call():
    t0 = time.perf_counter()
    _, infos = krylov_amd.gmres_restarted(A, b, restart=30, tol=1e-300, atol=0.0, max_cycles=cycles)
    assert len(infos) == cycles
    return time.perf_counter() - t0


call()
plain = [call() for _ in range(3)]
for name in ("start", "set_criterion", "run", "solution", "xk", "xk_into"):
    wrap(gm._GmresState, name)
tot.clear()
cnt.clear()
t = call()
print(f"plain call: {1e3 * np.median(plain):.2f} ms for {cycles} cycles = {1e3 * np.median(plain) / cycles:.3f} ms/cycle")
print(f"instrumented call: {1e3 * t:.2f} ms")
acc = 0.0
for k in sorted(tot, key=lambda k: -tot[k]):
    acc += tot[k]
    print(f"  {k:14s} {cnt[k]:3d} calls {1e3 * tot[k]:9.2f} ms  ({1e3 * tot[k] / cnt[k]:.3f} ms each)")
print(f"  {'(other)':14s}           {1e3 * (t - acc):9.2f} ms  (Problem, ||b||, allocation, Python)")
