"""Benchmark of the BASELINE metric on MI355X.

Workload (BASELINE.json metric): CG on the 3-D 15-point stencil
216^3 (n = 10,077,696, nnz = 149,770,936, fp64, int32 indices), b = ones,
tol = 0 (fixed iteration count). One step = one CG iteration: the SpMV
(+ <p,Ap>) launch, the one-block alpha kernel, the r pass (+ <r,r>) and the
fused rho / y / p pass; no host sync inside a chunk (kry_cg_preferred_chunk:
32 iterations here, 256 on the persistent small-n loop of cfg2).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--quick]

N > 1 (launched by torch.distributed.run): each rank solves its own RHS
column of the same matrix on its own GPU (RHS sharding) with
one RCCL allreduce of the residual-norm vector per iteration for the global
stop rule; value = total RHS-iterations per second (weak scaling).

Also reported (N = 1): the live SpMV roofline (HIP events around one SpMV
launch in 4 of the timed region: two event records per timed launch cost the
stream ~6 us, so timing all of them would slow the measured iteration), GMRES(30) on the cfg3 matrix, the secondary
BASELINE configs (cfg2 CG Poisson 1000^2, cfg4 block CG 8 RHS on Poisson
3163^2, cfg5 weighted fp32 MINRES 200^3), and the CPU baseline: the oracle
(the reference iteration on NumPy/SciPy) on a bounded sample of the metric
workload, rank 0 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SPMV_TIMED_EVERY = 4  # the live SpMV timing samples one launch in 4 of the timed region


def spmv_S(n, nnz, k=1, vb=8, ib=4, mvb=None):
    """S = nnz (vb + ib) + (n + 1) ib + 2 n k vb."""
    mvb = vb if mvb is None else mvb
    return nnz * (mvb + ib) + (n + 1) * ib + 2 * n * k * vb


def cg_iteration_bytes(n, nnz, k=1, vb=8, ib=4):
    """SpMV + fused x/r/rho pass (6 vectors) + p pass (3)."""
    return spmv_S(n, nnz, k, vb, ib) + 9 * n * k * vb


def gmres_cycle_bytes(n, nnz, m=30, vb=8, ib=4):
    """Per m-step cycle: (m + 1) S + (1950 + 37) n vb."""
    return (m + 1) * spmv_S(n, nnz) + (1950 + 37) * n * vb


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if "WORLD_SIZE" in os.environ:  # launched by torch.distributed.run (any N)
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)  # control plane only
        pg = dist
    return world, rank, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def allmax(pg, x):
    if pg is None:
        return x
    import torch

    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def _cg_state(A, B, comm=None, rank=0, world=1):
    """Device CG state on the product path (krylov_amd.cg's engine), with the
    RCCL communicator attached when sharded."""
    from krylov_amd import _helpers, _lib
    from krylov_amd.cg import _CGState

    prob = _helpers.Problem(A, B, None, None)
    st = _CGState(prob)
    ncols = prob.kpad
    if comm is not None:
        _lib.check(_lib.lib.kry_cg_attach_comm(st.h, comm.handle, rank * prob.kpad, world * prob.kpad))
        ncols = world * prob.kpad
    st.start()
    st.set_criterion(np.zeros(ncols))  # tol = atol = 0: never converges -> fixed steps
    return st, ncols


def _iterate(st, k, ncols, chunk=32):
    done = 0
    while done < k:
        s = min(chunk, k - done)
        hist = st.run(s, ncols)
        assert len(hist) == s, "solver stopped early"
        done += s


def run_metric(A_host, steps, warmup, world, rank, local, pg):
    import krylov_amd
    from krylov_amd import _lib, distributed
    from krylov_amd.device import get_context

    ctx = get_context(local)
    A = krylov_amd.CsrOperator(A_host, device=local)
    comm = distributed.ShardComm.from_torch(device=local) if pg is not None else None
    st, ncols = _cg_state(A, np.ones(A.n), comm, rank, world)
    chunk = st.preferred_chunk()
    _iterate(st, warmup, ncols, chunk)
    ctx.synchronize()
    # HIP events around one SpMV launch in 4 (two event records per timed
    # launch cost ~6 us of stream time; every launch of every kernel, 20 us)
    ctx.profile(True, kernels=[_lib.PROF_SPMV], every=SPMV_TIMED_EVERY)
    barrier(pg)
    ctx.synchronize()
    t0 = time.perf_counter()
    _iterate(st, steps, ncols, chunk)
    ctx.synchronize()
    t1 = time.perf_counter()
    barrier(pg)
    elapsed = allmax(pg, t1 - t0)
    cnt, spmv_ms = ctx.profile_read(_lib.PROF_SPMV)
    ctx.profile(False)
    del st
    if comm is not None:
        comm.close()
    layout = A.layout()
    return {"elapsed": elapsed, "spmv_count": cnt, "spmv_ms": spmv_ms, "n": A.n, "nnz": A.nnz, "layout": layout}


def spmv_kernel_desc(layout):
    """The CG SpMV kernel launch_spmv picks for k = 1 on this image, and the
    bytes that image moves per launch (next to SURVEY's algorithmic S)."""
    if layout["dia"]:
        return ("spmv_dia_kernel<double,double,16,SrcPlain,EpiApDot> (SELL-128/DIA diagonal-offset image, two rows "
                "per lane: values only, one offset + two lane masks per slot column; Ap stored + <p,Ap> partials)",
                "the DIA image moves dia_slots*8 + dia_slots/128*20 for the matrix, no index stream")
    if layout["compact"]:
        return ("spmv_sell_kernel<double,double,int,1,16,true,SrcPlain,EpiApDot> (SELL-64 SpMV, compact index "
                "image, Ap stored + <p,Ap> partials)", "the compact image moves nnz*(8+2) for the matrix")
    return ("spmv_sell_kernel<double,double,int,1,16,false,SrcPlain,EpiApDot> (SELL-64 SpMV, int32 indices)",
            "the SELL image moves slots*(8+4) for the matrix")


def run_cg_config(A_host, B, steps, warmup=5):
    """CG iterations/s on one GPU for a secondary config (k = B.shape[1])."""
    import krylov_amd
    from krylov_amd.device import get_context

    ctx = get_context()
    A = krylov_amd.CsrOperator(A_host)
    st, ncols = _cg_state(A, B)
    chunk = st.preferred_chunk()  # as krylov_amd.cg drives this solve
    _iterate(st, warmup, ncols, chunk)
    ctx.synchronize()
    t0 = time.perf_counter()
    _iterate(st, steps, ncols, chunk)
    ctx.synchronize()
    t = time.perf_counter() - t0
    k = 1 if B.ndim == 1 else B.shape[1]
    # algorithmic_gbs: SURVEY §8(d)'s per-iteration bytes of the launch-per-pass
    # CG over the measured time. The persistent small-n loop (cfg2) keeps y and
    # Ap on chip and moves about half of them (profiles/r01_pmc_cfg2.json), so
    # there this figure is an effective rate, not HBM traffic.
    return {"it_per_s": steps / t, "us_per_it": 1e6 * t / steps, "rhs": k, "n": A.n, "nnz": A.nnz,
            "algorithmic_gbs": cg_iteration_bytes(A.n, A.nnz, k) * steps / t / 1e9,
            "persistent_loop": chunk == 256}


def run_gmres(R=None, label="cfg3 random nonsym n=2e6, GMRES(30) mgs, one cycle"):
    """GMRES(30) iterations/s, one 30-step cycle (tol = 0) incl. the final
    x = x0 + V y; median of 3 after one warm-up cycle. Default matrix: cfg3."""
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.device import get_context
    from krylov_amd.gmres import _GmresState

    if R is None:
        R = problems.random_nonsym(2_000_000)
    A = krylov_amd.CsrOperator(R)
    prob = _helpers.Problem(A, np.ones(R.shape[0]), None, None)
    ctx = get_context()
    st = _GmresState(prob, 30, 1)
    times = []
    for rep in range(4):
        st.start()
        st.set_criterion(np.zeros(1))
        ctx.synchronize()
        t0 = time.perf_counter()
        hist, _ = st.run(30)
        st.solution()
        ctx.synchronize()
        t1 = time.perf_counter()
        assert len(hist) == 30
        if rep >= 1:
            times.append(t1 - t0)
    t = float(np.median(times))
    return {"it_per_s": 30.0 / t, "cycle_ms": 1e3 * t, "gbs": gmres_cycle_bytes(R.shape[0], R.nnz) / t / 1e9,
            "n": R.shape[0], "nnz": int(R.nnz), "config": label}


def run_end_to_end(A_host, steps):
    """The reference API at the host-array boundary: krylov_amd.cg(A, b) and
    gmres(A, b, maxiter=30) with numpy b in and numpy x out, on an operator
    uploaded beforehand (CsrOperator). Includes the b upload (H2D), solver
    setup, the per-chunk host syncs and the x download (D2H): the
    PCIe-inclusive rate DESIGN.md (d) quotes. Median of 3 after a warm-up."""
    import krylov_amd

    A = krylov_amd.CsrOperator(A_host)
    b = np.ones(A.n)
    out = {}
    for label, run, iters in (
        ("cg", lambda: krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=steps), steps),
        ("gmres30", lambda: krylov_amd.gmres(A, b, tol=0.0, atol=0.0, maxiter=30), 30),
    ):
        run()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            _, info = run()
            ts.append(time.perf_counter() - t0)
            assert info.numsteps == iters
        t = float(np.median(ts))
        out[f"{label}_it_per_s"] = iters / t
        out[f"{label}_call_ms"] = 1e3 * t
    out["includes"] = ("b upload (H2D), solver state setup, per-chunk host syncs, x download (D2H); the operator "
                       "is uploaded once before (CsrOperator)")
    return out


def run_minres_cfg5(steps=100):
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.device import get_context
    from krylov_amd.minres import _MinresState

    W, w = problems.shifted_lap3d_weighted(200)
    A = krylov_amd.CsrOperator(W)
    prob = _helpers.Problem(A, np.ones(W.shape[0], dtype=np.float32), None, krylov_amd.WeightedInner(w))
    ctx = get_context()
    st = _MinresState(prob)
    st.start()
    st.set_criterion(np.zeros(1))
    st.run(5)
    ctx.synchronize()
    t0 = time.perf_counter()
    done = 0
    while done < steps:
        hist, inv = st.run(min(32, steps - done))
        assert len(hist) == min(32, steps - done) and not inv, "MINRES stopped early"
        done += len(hist)
    ctx.synchronize()
    t = time.perf_counter() - t0
    return {"it_per_s": steps / t, "us_per_it": 1e6 * t / steps, "n": W.shape[0], "nnz": int(W.nnz),
            "config": "cfg5 shifted 3-D Laplacian 200^3, fp32 matrix, f64 weights (vectors f64 as in the reference)"}


PMC_SUMMARY = "r02_pmc_traffic.json"


def pmc_traffic(n, nnz, kernel):
    """HBM bytes per launch of the fused CG SpMV from the committed PMC
    summary (tools/pmc_traffic.sh: FETCH_SIZE and WRITE_SIZE passes, read side
    calibrated on a same-width stream of known size), if it was taken on this
    workload and this kernel. PMC needs its own rocprofv3 runs, so it cannot
    be live here."""
    path = os.path.join(REPO, "profiles", PMC_SUMMARY)
    try:
        with open(path) as f:
            d = json.load(f)
    except OSError:
        return {}
    if d.get("n") != n or d.get("nnz") != nnz or kernel.split("<")[0] not in d.get("kernel", ""):
        return {}
    return {"traffic_bytes_per_launch": d["traffic_bytes_per_launch"],
            "source": "profiles/%s (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, read side x%.3f "
                      "calibrated)" % (PMC_SUMMARY, d["read_scale_from_calibration"])}


def cpu_baseline(A_host, target_s=12.0):
    """The oracle (reference iteration on NumPy/SciPy, oracle/krylov_ref.py)
    timed on this host: CG with tol=0 on the metric matrix, bounded sample."""
    from oracle import krylov_ref

    b = np.ones(A_host.shape[0])
    t0 = time.perf_counter()
    krylov_ref.cg(A_host, b, tol=0.0, atol=0.0, maxiter=2)
    t_cal = time.perf_counter() - t0
    iters = int(max(3, min(60, target_s / max(t_cal / 3.0, 1e-3))))
    t0 = time.perf_counter()
    krylov_ref.cg(A_host, b, tol=0.0, atol=0.0, maxiter=iters)
    t = time.perf_counter() - t0
    threads = os.environ.get("OPENBLAS_NUM_THREADS") or os.environ.get("OMP_NUM_THREADS") or str(os.cpu_count())
    return {
        "value": iters / t,
        "unit": "CG iters/s",
        "cores": int(threads),
        "kind": "port",
        "sample": f"{iters} CG iterations (tol=0) of oracle/krylov_ref.cg on the full 216^3 15-pt matrix "
                  f"(incl. setup residual + final explicit residual); SciPy csr_matvec 1 thread, "
                  f"np.dot OpenBLAS {threads} threads",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--m", type=int, default=216, help="stencil edge (216 = BASELINE metric)")
    ap.add_argument("--quick", action="store_true", help="metric only (no GMRES leg, no CPU baseline)")
    ap.add_argument("--configs", action="store_true", help="also time the secondary BASELINE configs (cfg2, cfg4, cfg5)")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world, rank, local, pg = dist_setup()
    os.environ["KRYLOV_DEVICE"] = str(local)
    if world > 1 and args.gpus != world:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)

    from krylov_amd import problems

    A_host = problems.stencil15_3d(args.m)
    n, nnz = A_host.shape[0], int(A_host.nnz)
    res = run_metric(A_host, args.steps, args.warmup, world, rank, local, pg)
    T = res["elapsed"]
    spmv_avg_s = res["spmv_ms"] / max(res["spmv_count"], 1) / 1e3
    spmv_bytes = spmv_S(n, nnz)
    achieved = spmv_bytes / spmv_avg_s / 1e9
    kname, image_note = spmv_kernel_desc(res["layout"])
    image_bytes = None
    if res["layout"]["dia"]:  # the bytes the DIA image moves per launch (next to the algorithmic S)
        ds = res["layout"]["dia_slots"]
        image_bytes = ds * 8 + ds / 128 * 20 + 2 * n * 8
    traffic = pmc_traffic(n, nnz, kname)
    out = {
        "metric": "CG iters/sec + SpMV GB/s (fp64, n=10M, nnz=150M); GMRES(30) iters/sec",
        "value": world * args.steps / T,
        "unit": "CG iters/s (RHS-iterations/s over all GPUs)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * T / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY App. A generator, b = ones)",
        "config": {
            "workload": f"krylov.cg, 3-D 15-point stencil {args.m}^3, one RHS per GPU, tol=0 fixed iterations",
            "n": n,
            "nnz": nnz,
            "index": "int32",
            "rhs_per_gpu": 1,
            "parallelism": f"rhs-shard x{world}" + (" (one RCCL resnorm allreduce per iteration)" if world > 1 else ""),
        },
        "spmv_gbs": achieved,
        "spmv_ms": 1e3 * spmv_avg_s,
        "cg_iter_gbs_per_gpu": cg_iteration_bytes(n, nnz) * args.steps / T / 1e9,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic.get("traffic_bytes_per_launch"),
            "traffic_source": traffic.get("source"),
            "kernel": kname,
            "bytes_per_launch": spmv_bytes,
            "bytes_formula": "S = nnz*(8+4) + (n+1)*4 + 2*n*8 (SURVEY §8(d), int32-CSR algorithmic bytes; "
                             + image_note + ")",
            "launches_timed": res["spmv_count"],
            "timing": f"HIP events on the solver stream around one SpMV launch in {SPMV_TIMED_EVERY} of the timed "
                      f"region ({args.steps} launches)",
            "image_bytes_per_launch": image_bytes,
            "image_gbs": image_bytes / spmv_avg_s / 1e9 if image_bytes else None,
            "image_frac": image_bytes / spmv_avg_s / 1e9 / HBM_PEAK_GBS if image_bytes else None,
        },
    }
    if world == 1 and not args.quick:
        g = run_gmres()
        out["gmres30_it_per_s"] = g["it_per_s"]
        out["gmres"] = g
        # north_star: GMRES(30) on the same (metric) matrix
        out["gmres_metric"] = run_gmres(A_host, f"metric 15-point {args.m}^3, GMRES(30) mgs, one cycle")
        out["end_to_end"] = run_end_to_end(A_host, args.steps)
    if world == 1 and args.configs:
        extra = {}
        extra["cfg2_cg_poisson1000"] = run_cg_config(problems.poisson2d(1000), np.ones(1_000_000), 200, 10)
        P3 = problems.poisson2d(3163)
        B = np.random.default_rng(0).standard_normal((P3.shape[0], 8))
        extra["cfg4_blockcg_8rhs_per_gpu"] = run_cg_config(P3, B, 20, 3)
        del P3, B
        extra["cfg5_minres_fp32_weighted"] = run_minres_cfg5()
        out["extra"] = extra
    if rank == 0 and world == 1 and not args.no_cpu and not args.quick:
        out["cpu_baseline"] = cpu_baseline(A_host)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
