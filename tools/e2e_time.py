"""End-to-end (host-array boundary) timing of the user-facing solvers on the
metric matrix: krylov_amd.cg / gmres called with numpy b, returning numpy x,
against the device-resident iteration rate the bench reports. Splits out the
per-call pieces: Problem (b upload), the solve, the x download, and (round 5)
a cProfile of one call by own time (ctypes calls count in their caller).

    python3 tools/e2e_time.py [steps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(steps=200):
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState

    M = problems.stencil15_3d(216)
    t0 = time.perf_counter()
    A = krylov_amd.CsrOperator(M)
    A.ctx.synchronize()
    print(f"upload+image {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    b = np.ones(M.shape[0])
    krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=8)  # warm-up
    for _ in range(3):
        t0 = time.perf_counter()
        _, info = krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=steps)
        t = time.perf_counter() - t0
        print(f"cg maxiter={steps}: {1e3 * t:.1f} ms, {info.numsteps / t:.0f} it/s end to end", flush=True)
    for _ in range(3):
        t0 = time.perf_counter()
        prob = _helpers.Problem(A, b, None, None)
        t1 = time.perf_counter()
        st = _CGState(prob)
        st.start()
        A.ctx.synchronize()
        t2 = time.perf_counter()
        x = st.get(0)
        t3 = time.perf_counter()
        print(f"  Problem (b upload) {1e3 * (t1 - t0):.1f} ms, state+start {1e3 * (t2 - t1):.1f} ms, "
              f"x download {1e3 * (t3 - t2):.1f} ms", flush=True)
        del st, prob, x
    krylov_amd.gmres(A, b, tol=0.0, atol=0.0, maxiter=30)
    for _ in range(3):
        t0 = time.perf_counter()
        krylov_amd.gmres(A, b, tol=0.0, atol=0.0, maxiter=30)
        t = time.perf_counter() - t0
        print(f"gmres(30): {1e3 * t:.1f} ms, {30 / t:.0f} it/s end to end", flush=True)
    # per-phase host time of both drivers (each state method wrapped in a timer)
    cgmod, gmmod = sys.modules["krylov_amd.cg"], sys.modules["krylov_amd.gmres"]

    acc = {}

    def wrap(cls, name):
        f = getattr(cls, name)

        def g(*a, **k):
            t = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[cls.__name__ + "." + name] = acc.get(cls.__name__ + "." + name, 0.0) + time.perf_counter() - t

        setattr(cls, name, g)

    for cls in (cgmod._CGState, gmmod._GmresState):
        for name in ("__init__", "start", "set_criterion", "run", "get", "solution", "xk", "residual_norm2"):
            if hasattr(cls, name):
                wrap(cls, name)
    ohelp = _helpers.Problem.__init__

    def pinit(self, *a, **k):
        t = time.perf_counter()
        ohelp(self, *a, **k)
        acc["Problem.__init__"] = acc.get("Problem.__init__", 0.0) + time.perf_counter() - t

    _helpers.Problem.__init__ = pinit
    for label, fn in (("cg", lambda: krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=steps)),
                      ("gmres", lambda: krylov_amd.gmres(A, b, tol=0.0, atol=0.0, maxiter=30))):
        acc.clear()
        t0 = time.perf_counter()
        fn()
        t = time.perf_counter() - t0
        print(f"{label} phases (total {1e3 * t:.1f} ms): " +
              ", ".join(f"{k} {1e3 * v:.1f}" for k, v in sorted(acc.items(), key=lambda kv: -kv[1])), flush=True)


def profile_calls(steps_list=(20, 200)):
    import cProfile
    import pstats

    import krylov_amd
    from krylov_amd import problems

    M = problems.stencil15_3d(216)
    A = krylov_amd.CsrOperator(M)
    b = np.ones(M.shape[0])
    for steps in steps_list:
        for _ in range(2):
            krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=steps)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=steps)
            ts.append(time.perf_counter() - t0)
        # the device rate of the same chunks without the host boundary
        prob = krylov_amd._helpers.Problem(A, b, None, None)
        st = sys.modules["krylov_amd.cg"]._CGState(prob)
        st.start()
        st.set_criterion(np.zeros(1))
        A.ctx.synchronize()
        t0 = time.perf_counter()
        k = 0
        while k < steps:
            k += len(st.run(min(st.preferred_chunk(), steps - k)))
        dev = time.perf_counter() - t0
        del st, prob
        print(f"cg maxiter={steps}: calls {', '.join(f'{1e3 * t:.1f}' for t in ts)} ms; chunked device loop "
              f"{1e3 * dev:.1f} ms -> fixed {1e3 * (float(np.median(ts)) - dev):.1f} ms", flush=True)
        pr = cProfile.Profile()
        pr.enable()
        krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=steps)
        pr.disable()
        pstats.Stats(pr, stream=sys.stdout).sort_stats("tottime").print_stats(14)


def phases(steps=200, calls=5):
    """cg()'s sequence restated with a clock between its phases, the
    results kept alive as bench.py's end_to_end leg keeps them."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.cg import _CGState
    from krylov_amd.device import HostOut

    M = problems.stencil15_3d(216)
    cs = []
    for _ in range(3):
        t0 = time.perf_counter()
        A = krylov_amd.CsrOperator(M)
        A.ctx.synchronize()
        cs.append(time.perf_counter() - t0)
    print(f"CsrOperator (kry_csr_create) median of 3: {1e3 * float(np.median(cs)):.1f} ms "
          f"(KRY_HOST_PIN={os.environ.get('KRY_HOST_PIN', '1')})", flush=True)
    b = np.ones(M.shape[0])
    keep, rows = [], []
    for c in range(calls + 1):
        t = [time.perf_counter()]
        prob = _helpers.Problem(A, b, None, None)
        t.append(time.perf_counter())
        st = _CGState(prob)
        t.append(time.perf_counter())
        xo = HostOut((prob.n, prob.kpad), prob.dtype)
        t.append(time.perf_counter())
        st.start()
        t.append(time.perf_counter())
        st.set_criterion(np.zeros(1))
        chunk = st.preferred_chunk()
        k = 0
        while k < steps:
            k += len(st.run(min(chunk, steps - k)))
        t.append(time.perf_counter())
        x = xo.take()
        t.append(time.perf_counter())
        st.get(0, out=x)
        t.append(time.perf_counter())
        del st, prob
        t.append(time.perf_counter())
        keep.append(x)
        if c:
            rows.append(np.diff(t) * 1e3)
    names = ["Problem (b upload)", "_CGState", "HostOut", "start", "chunks", "HostOut.take", "get (x D2H)", "destructors"]
    med = np.median(np.array(rows), axis=0)
    print(f"cg maxiter={steps} phases, median of {calls} (ms): " + ", ".join(f"{n} {v:.2f}" for n, v in zip(names, med))
          + f"; total {med.sum():.2f}, outside the chunks {med.sum() - med[4]:.2f}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "profile":
        profile_calls()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "phases":
        phases(200)
        phases(20)
        sys.exit(0)
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
