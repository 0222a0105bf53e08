"""Benchmark of the BASELINE metric on MI355X.

Workload (BASELINE.json metric): CG on the 3-D 15-point stencil
216^3 (n = 10,077,696, nnz = 149,770,936, fp64, int32 indices), b = ones,
tol = 0 (fixed iteration count). One step = one CG iteration (one fused
p-update + SpMV + <p,Ap>, one fused x/r update + <r,r>, two scalar kernels).

  python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 (launched by torch.distributed.run): each rank solves its own RHS
column of the same matrix on its own GPU (RHS sharding) and
every iteration performs one RCCL allreduce of the residual-norm vector for
the global stop test; value = total RHS-iterations per second (weak scaling).

Extra fields: the live SpMV roofline (HIP events around every SpMV launch of
the timed region), GMRES(30) iterations/s on the cfg3 matrix (N = 1), and
the CPU baseline (the oracle: the reference's iteration on NumPy/SciPy) on a
bounded sample of the same workload (rank 0, N = 1 only).
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


def spmv_fused_bytes(n, nnz, vb=8, ib=4):
    """Algorithmic bytes of one fused CG SpMV launch: the matrix once
    (nnz*(vb+ib) + (n+1)*ib), plus r and p_old read (the gather builds
    p = r + omega p_old) and p, Ap written: S + 2 n vb with SURVEY's
    S = nnz(vb+ib) + (n+1) ib + 2 n vb."""
    return nnz * (vb + ib) + (n + 1) * ib + 4 * n * vb


def cg_iteration_bytes(n, nnz, vb=8, ib=4):
    """Algorithmic bytes of one CG iteration as implemented: fused SpMV
    (above) + update pass (read y, r, p, Ap; write y, r = 6 n vb)."""
    return spmv_fused_bytes(n, nnz, vb, ib) + 6 * n * vb


def gmres_cycle_bytes(n, nnz, m=30, vb=8, ib=4):
    """Per 30-step cycle: 31 S + (1950 + 37) n vb."""
    S = nnz * (vb + ib) + (n + 1) * ib + 2 * n * vb
    return (m + 1) * S + (1950 + 37) * n * vb


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
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


def make_comm(pg, ctx, world, rank):
    import ctypes

    from krylov_amd import _lib

    idbuf = np.zeros(128, dtype=np.uint8)
    if rank == 0:
        _lib.check(_lib.lib.kry_comm_unique_id(_lib.ptr(idbuf)))
    import torch

    t = torch.from_numpy(idbuf.astype(np.int64))
    pg.broadcast(t, src=0)
    idbuf = t.numpy().astype(np.uint8)
    h = ctypes.c_void_p()
    _lib.check(_lib.lib.kry_comm_create(ctx.handle, world, rank, _lib.ptr(idbuf), ctypes.byref(h)))
    return h


def run_cg(A_host, steps, warmup, world, rank, local, pg):
    import ctypes

    import krylov_amd
    from krylov_amd import _helpers, _lib
    from krylov_amd.cg import _CGState
    from krylov_amd.device import get_context

    ctx = get_context(local)
    A = krylov_amd.CsrOperator(A_host, device=local)
    n = A.n
    b = np.ones(n)
    prob = _helpers.Problem(A, b, None, None)
    st = _CGState(prob)
    comm = None
    if world > 1:
        comm = make_comm(pg, ctx, world, rank)
        _lib.check(_lib.lib.kry_cg_attach_comm(st.h, comm, rank, world))
    st.start()
    # tol = 0, atol = 0: never converges -> exactly the requested iterations
    st.set_criterion(np.zeros(world if comm else 1))
    ncols = world if comm else 1
    chunk = _helpers.CHUNK

    def iterate(k):
        done = 0
        while done < k:
            s = min(chunk, k - done)
            hist = st.run(s, ncols)
            assert len(hist) == s, "solver stopped early"
            done += s
        return hist

    iterate(warmup)
    ctx.synchronize()
    ctx.profile(True)
    barrier(pg)
    ctx.synchronize()
    t0 = time.perf_counter()
    hist = iterate(steps)
    ctx.synchronize()
    t1 = time.perf_counter()
    barrier(pg)
    elapsed = allmax(pg, t1 - t0)
    cnt, spmv_ms = ctx.profile_read(_lib.PROF_SPMV)
    ucnt, upd_ms = ctx.profile_read(_lib.PROF_UPDATE)
    ctx.profile(False)
    if comm is not None:
        _lib.check(_lib.lib.kry_comm_destroy(comm))
    return {
        "elapsed": elapsed,
        "spmv_count": cnt,
        "spmv_ms": spmv_ms,
        "update_count": ucnt,
        "update_ms": upd_ms,
        "last_resnorm": float(np.max(hist[-1])),
        "n": n,
        "nnz": A.nnz,
    }


def run_gmres(steps_warm=1):
    import krylov_amd
    from krylov_amd import _helpers, problems
    from krylov_amd.device import get_context
    from krylov_amd.gmres import _GmresState

    R = problems.random_nonsym(2_000_000)
    A = krylov_amd.CsrOperator(R)
    b = np.ones(R.shape[0])
    prob = _helpers.Problem(A, b, None, None)
    ctx = get_context()
    st = _GmresState(prob, 30, 1)
    times = []
    for rep in range(steps_warm + 3):
        st.start()
        st.set_criterion(np.zeros(1))
        ctx.synchronize()
        t0 = time.perf_counter()
        hist, _ = st.run(30)
        st.solution()
        ctx.synchronize()
        t1 = time.perf_counter()
        assert len(hist) == 30
        if rep >= steps_warm:
            times.append(t1 - t0)
    t = float(np.median(times))
    return {"gmres30_it_per_s": 30.0 / t, "gmres30_cycle_ms": 1e3 * t,
            "gmres30_gbs": gmres_cycle_bytes(R.shape[0], R.nnz) / t / 1e9, "n": R.shape[0], "nnz": int(R.nnz)}


def cpu_baseline(A_host, target_s=12.0):
    """The oracle (reference iteration on NumPy/SciPy, oracle/krylov_ref.py)
    timed on this host: CG with tol=0 on the same matrix, bounded sample."""
    from oracle import krylov_ref

    b = np.ones(A_host.shape[0])
    # calibrate: 2 iterations, then size the sample to ~target_s
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
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gmres", action="store_true")
    args = ap.parse_args()

    world, rank, local, pg = dist_setup()
    if world != args.gpus and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    os.environ["KRYLOV_DEVICE"] = str(local)

    from krylov_amd import problems

    A_host = problems.stencil15_3d(args.m)
    n, nnz = A_host.shape[0], int(A_host.nnz)
    res = run_cg(A_host, args.steps, args.warmup, world, rank, local, pg)
    T = res["elapsed"]
    value = world * args.steps / T
    spmv_avg_s = res["spmv_ms"] / max(res["spmv_count"], 1) / 1e3
    spmv_bytes = spmv_fused_bytes(n, nnz)
    achieved = spmv_bytes / spmv_avg_s / 1e9
    out = {
        "metric": "CG iters/sec + SpMV GB/s (fp64, n=10M, nnz=150M); GMRES(30) iters/sec",
        "value": value,
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
            "parallelism": f"rhs-shard x{world}" + (" (RCCL resnorm allreduce/iter)" if world > 1 else ""),
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
            "traffic": None,
            "kernel": "spmv_stream_kernel<double,double,int,SrcCgP,EpiCgAp> (fused p-update + SpMV + <p,Ap>)",
            "bytes_per_launch": spmv_bytes,
            "launches_timed": res["spmv_count"],
        },
    }
    if world == 1 and not args.no_gmres:
        out["gmres"] = run_gmres()
        out["gmres30_it_per_s"] = out["gmres"]["gmres30_it_per_s"]
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(A_host)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
