"""Benchmark of the BASELINE metric on MI355X.

Workload (BASELINE.json metric): CG on the 3-D 15-point stencil
216^3 (n = 10,077,696, nnz = 149,770,936, fp64, int32 indices), b = ones,
tol = 0 (fixed iteration count). One step = one CG iteration: the SpMV
(+ <p,Ap>) launch and the one-launch update (alpha, r, rho, omega, y, p); no
host sync inside a chunk (kry_cg_preferred_chunk: 32 iterations here, 256 on
the persistent small-n loop of cfg2).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--quick] [--configs]
                  [--workload metric|cfg4] [--no-cpu]

N > 1 (launched by torch.distributed.run): each rank solves its own RHS
columns of the same matrix on its own GPU (RHS sharding) with
one RCCL allreduce of the residual-norm vector per iteration for the global
stop rule; value = total RHS-iterations per second (weak scaling). Unless
--quick, every N also times cfg4 (Poisson 3163^2, 8 RHS per GPU, the
BASELINE multi-GPU configuration) the same way ("cfg4_sharded");
--workload cfg4 makes it the headline.

roofline: the CG SpMV kernel's bytes per launch are the bytes its image must
move (the DIA image has no index stream; the compact SELL image 2 B of index
per slot), divided by its average launch time from HIP events on the solver
stream in a dedicated pass after the timed region (every launch of >= 64
iterations); SURVEY's int32-CSR bytes S over the same time is reported
beside it as effective_gbs / frac_vs_csr_S. spmv_general repeats the
measurement on the same matrix with the DIA image disabled (KRY_SPMV_DIA=0):
the compact SELL kernel that arbitrary sorted CSR takes.

Also reported (N = 1): GMRES(30) on the cfg3 matrix and on the metric
matrix, the reference API at the host-array boundary, the secondary BASELINE
configs with --configs (cfg2 CG Poisson 1000^2, cfg4 block CG 8 RHS, cfg5
weighted fp32 MINRES 200^3), and the CPU baseline: the oracle (the reference
iteration on NumPy/SciPy) on a bounded sample of the metric workload, median
of 5, rank 0 only.
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


def spmv_S(n, nnz, k=1, vb=8, ib=4, mvb=None):
    """S = nnz (vb + ib) + (n + 1) ib + 2 n k vb."""
    mvb = vb if mvb is None else mvb
    return nnz * (mvb + ib) + (n + 1) * ib + 2 * n * k * vb


def image_bytes_k1(layout, n, nnz, vectors=2, vb=8):
    """Bytes a k = 1 SpMV must move on the image launch_spmv picks:
    (kernel, bytes, formula). `vectors` n-vectors of 8 B beside the matrix
    (2: x read, y written; GMRES's epilogue also reads V_0: 3); `vb` the
    matrix value bytes (DIA image; 8 on the other images' callers)."""
    v = vectors * n * 8
    vt = f"{vectors}*n*8"
    if layout["dia"]:
        ds = layout["dia_slots"]
        return ("spmv_dia_kernel", ds * vb + ds / 128 * 20 + v,
                f"dia_slots*{vb} + dia_slots/128*20 + {vt}")
    if layout.get("col_blocks", 0):
        nb = layout["col_blocks"]
        ng = (n + 255) // 256
        nl = (ng + 16383) // 16384  # launch_spmv: one launch per 16,384 row groups
        kname = "spmv_cbp_kernel" + (f" ({nl} launches over row-group ranges)" if nl > 1 else "")
        return (kname, nnz * (4 + 8) + nb * n * 2 + (nb * ng + 1) * 8 + v,
                f"nnz*(4+8) (column + value) + col_blocks*n*2 (row offsets) + (col_blocks*ng+1)*8 (segment "
                f"pointers) + {vt}")
    if layout.get("pair"):
        ps = layout["pair_slots"]
        return ("spmv_pair_kernel", ps * (8 + 2) + ps / 128 * 4 + (n + 127) // 128 * 12 + v,
                f"pair_slots*(8+2) + pair_slots/128*4 + slices*12 + {vt}")
    if layout.get("rs"):
        rs = layout["rs_slots"]
        kname = ("spmv_rs_kernel" if os.environ.get("KRY_SPMV_RS1") == "0" else "spmv_rs1_kernel") + (
            " (renumbered)" if layout.get("renumbered") else "")
        return (kname, rs * (8 + 4) + (n + 127) // 128 * 12 + v,
                f"rs_slots*(8+4) (values + column/rank words) + slices*12 + {vt}")
    slots, slices = layout["slots"], layout["slices"]
    if layout["compact"]:
        return ("spmv_sell_kernel (compact)", slots * (8 + 2) + slots / 64 * 4 + slices * 12 + v,
                f"slots*(8+2) + slots/64*4 + slices*12 + {vt}")
    return ("spmv_sell_kernel", slots * (8 + 4) + slices * 12 + v, f"slots*(8+4) + slices*12 + {vt}")


def hbm_roofline(kernel, bytes_per_launch, seconds_per_launch, formula, launches, traffic=None, **extra):
    """A roofline object: algorithmic bytes per launch over the measured
    average launch time, against the 8 TB/s HBM3E spec."""
    gbs = bytes_per_launch / seconds_per_launch / 1e9
    out = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
           "traffic": traffic, "kernel": kernel, "ms_per_launch": 1e3 * seconds_per_launch,
           "bytes_per_launch": bytes_per_launch, "bytes_formula": formula, "launches_timed": launches,
           "timing": "HIP events on the solver stream around every launch of a pass after the timed region"}
    out.update(extra)
    return out


def profiled(ctx, ids, fn):
    """Run fn() with HIP-event timing of every launch of the kernel ids in
    `ids` (ProfScope, krylov_amd/csrc); returns {id: (launches, ms)}."""
    ctx.synchronize()
    ctx.profile(True, kernels=list(ids), every=1)
    try:
        fn()
        ctx.synchronize()
        return {i: ctx.profile_read(i) for i in ids}
    finally:
        ctx.profile(False)


def gather_ceiling(label):
    """The measured random-gather ceiling for a column-blocked image
    (profiles/<GATHER_CEILING>, tools/gather_ceiling.py), if present."""
    try:
        with open(os.path.join(REPO, "profiles", GATHER_CEILING)) as f:
            return json.load(f).get(label)
    except OSError:
        return None


def plan_launch(gpus, env, device_count, launch="auto"):
    """How this process's ranks come about, decided before any GPU work:

    * ``torchrun``: ``WORLD_SIZE`` is set (python -m torch.distributed.run):
      one rank per process, this process drives device LOCAL_RANK, world =
      WORLD_SIZE (a ``--gpus`` that disagrees is noted, WORLD_SIZE wins);
    * ``threads``: ``--gpus N`` > 1 with no launcher: ONE process drives
      devices 0..N-1, one host thread each, over communicators from one
      ncclCommInitAll (krylov_amd.multi's path);
    * ``single``: one GPU (device KRYLOV_DEVICE, default 0).

    ``device_count()`` is called only to check that enough devices are
    visible; too few raise SystemExit (non-zero), never a silent N = 1.
    ``launch="threads"`` takes the threaded path at any N (at N = 1: one
    device, a one-rank ncclCommInitAll communicator attached - the path's
    rehearsal on a one-GPU box)."""
    if gpus < 1:
        raise SystemExit(f"--gpus {gpus}: need at least one GPU")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        rank = int(env.get("RANK", "0"))
        local = int(env.get("LOCAL_RANK", "0"))
        have = device_count()
        if local >= have:
            raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {have} GPU(s) visible")
        note = None if gpus == world else f"--gpus {gpus} but WORLD_SIZE {world}; using WORLD_SIZE"
        return {"mode": "torchrun", "world": world, "rank": rank, "devices": [local], "ranks": [rank], "note": note}
    if gpus > 1 or launch == "threads":
        have = device_count()
        if have < gpus:
            raise SystemExit(f"--gpus {gpus} but only {have} GPU(s) visible")
        return {"mode": "threads", "world": gpus, "rank": 0, "devices": list(range(gpus)),
                "ranks": list(range(gpus)), "note": None}
    dev = int(env.get("KRYLOV_DEVICE", "0") or 0)
    return {"mode": "single", "world": 1, "rank": 0, "devices": [dev], "ranks": [0], "note": None}


class Job:
    """The ranks this process drives (plan_launch) and the control plane
    between processes (torchrun: a gloo group for barriers and the max over
    ranks; the data path is RCCL)."""

    def __init__(self, plan):
        self.mode, self.world, self.rank = plan["mode"], plan["world"], plan["rank"]
        self.devices, self.ranks = plan["devices"], plan["ranks"]
        self.pg = None
        if self.mode == "torchrun":
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)  # control plane only
            self.pg = dist

    @property
    def local(self):
        """The device of this process's first rank."""
        return self.devices[0]

    def run_all(self, fn):
        """fn(i) for every local rank i, concurrently (one host thread per
        device: the C-ABI calls release the GIL); the first error is raised."""
        if len(self.devices) == 1:
            return [fn(0)]
        import threading

        out, errs = [None] * len(self.devices), []

        def run(i):
            try:
                out[i] = fn(i)
            except BaseException as e:  # noqa: BLE001 - re-raised below
                errs.append(e)

        th = [threading.Thread(target=run, args=(i,), name=f"bench-dev{d}") for i, d in enumerate(self.devices)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]
        return out

    def barrier(self):
        if self.pg is not None:
            self.pg.barrier()

    def allmax(self, x):
        if self.pg is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.pg is not None:
            self.pg.destroy_process_group()

    @classmethod
    def single(cls, device=None):
        dev = int(os.environ.get("KRYLOV_DEVICE", "0") or 0) if device is None else int(device)
        return cls({"mode": "single", "world": 1, "rank": 0, "devices": [dev], "ranks": [0]})


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


def comm_ranks(comm):
    """(nranks, rank) as RCCL itself reports them (kry_comm_info)."""
    import ctypes

    from krylov_amd import _lib

    n, r = ctypes.c_int32(), ctypes.c_int32()
    _lib.check(_lib.lib.kry_comm_info(comm.handle, ctypes.byref(n), ctypes.byref(r)))
    return int(n.value), int(r.value)


def run_cg_bench(A_host, rhs_of_rank, steps, warmup, job, repeats=1, roofline_launches=64, prof_ids=None):
    """CG on every local rank's RHS block (rhs_of_rank(rank): n or n x k) of
    A: warmup, then `repeats` timed regions of EXACTLY `steps` iterations,
    each between barrier + device sync on both sides (max over ranks; in one
    process the threads' common wall clock), then a separate pass of
    max(steps, roofline_launches) iterations with HIP events around every
    SpMV launch of the first local rank (the kernel's average launch time;
    event records add stream time, so this pass is not a timed one)."""
    import krylov_amd
    from krylov_amd import _lib, distributed
    from krylov_amd.device import get_context
    from krylov_amd.multi import _operators

    devs = job.devices
    ctxs = [get_context(d) for d in devs]
    ops = _operators(A_host, devs) if len(devs) > 1 else [krylov_amd.CsrOperator(A_host, device=devs[0])]
    if job.mode == "threads":
        comms = distributed.ShardComm.all_devices(devs)
    elif job.mode == "torchrun" and job.world > 1:
        comms = [distributed.ShardComm.from_torch(device=devs[0])]
    else:
        comms = [None]
    rccl = comm_ranks(comms[0]) if comms[0] is not None else None
    sts = [_cg_state(ops[i], rhs_of_rank(job.ranks[i]), comms[i], job.ranks[i], job.world) for i in range(len(devs))]
    ncols = sts[0][1]
    chunk = sts[0][0].preferred_chunk()

    def iterate(k):
        def one(i):
            _iterate(sts[i][0], k, ncols, chunk)
            ctxs[i].synchronize()
        job.run_all(one)

    iterate(warmup)
    elapsed = []
    for _ in range(repeats):
        job.barrier()
        for c in ctxs:
            c.synchronize()
        t0 = time.perf_counter()
        iterate(steps)
        t1 = time.perf_counter()
        job.barrier()
        elapsed.append(job.allmax(t1 - t0))
    ids = [_lib.PROF_SPMV] + [i for i in (prof_ids or []) if i != _lib.PROF_SPMV]
    prof = profiled(ctxs[0], ids, lambda: iterate(max(steps, roofline_launches)))
    cnt, spmv_ms = prof[_lib.PROF_SPMV]
    defer = sts[0][0].defer_info()
    del sts
    for c in comms:
        if c is not None:
            c.close()
    layout = ops[0].layout()
    med = float(np.median(elapsed))
    return {"elapsed": med, "elapsed_all": elapsed, "spmv_count": cnt, "spmv_avg_s": spmv_ms / max(cnt, 1) / 1e3,
            "n": ops[0].n, "nnz": ops[0].nnz, "layout": layout, "rhs": ncols // job.world,
            "persistent_loop": chunk == 256, "prof": prof, "prof_iters": max(steps, roofline_launches),
            "ydefer": defer, "rccl_ranks": None if rccl is None else rccl[0]}


def spmv_kernel_desc(layout, n):
    """The CG SpMV kernel launch_spmv picks for k = 1 on this image, the
    bytes that image must move per launch, and how they are counted."""
    slots, slices = layout["slots"], layout["slices"]
    if layout["dia"]:
        ds = layout["dia_slots"]
        return ("spmv_dia_kernel<double,double,16,SrcPlain,EpiApDot> (SELL-128/DIA diagonal-offset image, two rows "
                "per lane: values only, one offset + two lane masks per slot column; Ap stored + <p,Ap> partials)",
                ds * 8 + ds / 128 * 20 + 2 * n * 8,
                "dia_slots*8 (values) + dia_slots/128*20 (offset + two lane masks per slot column) + 2*n*8 "
                "(p read once, Ap written once); no index stream")
    if layout.get("pair"):
        ps = layout["pair_slots"]
        pslices = (n + 127) // 128
        return ("spmv_pair_kernel<double,double,8,SrcPlain,EpiApDot> (paired-row SELL-128 SpMV for general CSR: "
                "two rows per lane, one 16-B value load, one 4-B load of two uint16 column deltas over a "
                "per-slot-column int32 base and one 16-B x load for adjacent columns per slot column; Ap stored + "
                "<p,Ap> partials)",
                ps * (8 + 2) + ps / 128 * 4 + pslices * 12 + 2 * n * 8,
                "pair_slots*(8+2) (values + uint16 deltas) + pair_slots/128*4 (column bases) + slices*12 (slice "
                "pointer + width) + 2*n*8 (p read once, Ap written once)")
    if layout["compact"]:
        return ("spmv_sell_kernel<double,double,int,1,16,true,SrcPlain,EpiApDot> (SELL-64 SpMV, compact index "
                "image: uint16 column deltas over per-slot-column int32 bases; Ap stored + <p,Ap> partials)",
                slots * (8 + 2) + slots / 64 * 4 + slices * 12 + 2 * n * 8,
                "slots*(8+2) (values + uint16 deltas) + slots/64*4 (column bases) + slices*12 (slice pointer + "
                "width) + 2*n*8 (p read once, Ap written once)")
    return ("spmv_sell_kernel<double,double,int,1,16,false,SrcPlain,EpiApDot> (SELL-64 SpMV, int32 indices)",
            slots * (8 + 4) + slices * 12 + 2 * n * 8,
            "slots*(8+4) + slices*12 + 2*n*8")


def roofline_of(res, n, nnz, traffic=None):
    """roofline object of one CG SpMV measurement (run_cg_bench)."""
    kname, image_bytes, formula = spmv_kernel_desc(res["layout"], n)
    t = res["spmv_avg_s"]
    S = spmv_S(n, nnz)
    traffic = traffic or {}
    return {
        "bound": "hbm",
        "achieved": image_bytes / t / 1e9,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": image_bytes / t / 1e9 / HBM_PEAK_GBS,
        "traffic": traffic.get("traffic_bytes_per_launch"),
        "traffic_source": traffic.get("source"),
        "kernel": kname,
        "spmv_ms": 1e3 * t,
        "ms_per_launch": 1e3 * t,
        "bytes_per_launch": image_bytes,
        "bytes_formula": formula,
        "launches_timed": res["spmv_count"],
        "timing": "HIP events on the solver stream around every SpMV launch of a pass after the timed region",
        "csr_S_bytes": S,
        "effective_gbs": S / t / 1e9,
        "frac_vs_csr_S": S / t / 1e9 / HBM_PEAK_GBS,
        "csr_S_formula": "S = nnz*(8+4) + (n+1)*4 + 2*n*8 (SURVEY §8(d), the int32-CSR algorithmic bytes: an "
                         "effective rate, not HBM traffic, for an image that moves fewer bytes)",
    }


def cfg4_rooflines(res, steps):
    """Block CG (k columns, DIA image): the block SpMV's roofline and the
    iteration's, on the bytes the kernels must move: SpMV (values, the
    per-slot-column descriptors, p read, Ap written), the r pass (r, Ap in;
    r out), the p pass (r, p_i in; p_{i+1} out) and, with yk deferred D steps,
    once per D steps y in and out and the D - 1 older p vectors in (p_i is
    the pass's own; D = 0: the fused y / p pass, r, y, p in and y, p out)."""
    from krylov_amd import _lib

    n, k = res["n"], res["rhs"]
    lay = res["layout"]
    vec = n * k * 8
    ds = lay["dia_slots"]
    sb = ds * 8 + ds / 128 * 20 + 2 * vec
    cnt, ms = res["prof"][_lib.PROF_SPMV]
    spmv = hbm_roofline("spmv_dia_blk_kernel<double,double,2,8,SrcPlain,EpiApDot> (block DIA SpMV, k = %d)" % k,
                        sb, ms / max(cnt, 1) / 1e3,
                        "dia_slots*8 + dia_slots/128*20 + 2*n*k*8 (values, descriptors, p read, Ap written)", cnt)
    D = res["ydefer"][0]
    pass_b = 3 * vec + 3 * vec + ((D + 1) / D * vec if D else 2 * vec)
    it_b = sb + pass_b
    t_it = res["elapsed"] / steps
    return spmv, {"bound": "hbm", "achieved": it_b / t_it / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": it_b / t_it / 1e9 / HBM_PEAK_GBS, "bytes_per_iteration": it_b, "ydefer": D,
                  "bytes_formula": "SpMV (above) + 3*n*k*8 (r pass) + 3*n*k*8 (p pass) + "
                                   + ("(D+1)/D*n*k*8 (yk flush every D steps: y in and out, the D-1 older p in)"
                                      if D else "2*n*k*8 (y in the y/p pass)")}


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
    return {"it_per_s": steps / t, "us_per_it": 1e6 * t / steps, "rhs": k, "n": A.n, "nnz": A.nnz,
            "persistent_loop": chunk == 256, "layout": A.layout()}


def run_cfg2(steps=200, warmup=10):
    """BASELINE cfg2: CG on Poisson 1000^2 (n = 1e6), b = ones, tol = 0. The
    default path is the persistent loop (cg_persist_kernel: a whole chunk of
    iterations in one launch, y, Ap and p's gathers on chip), so the roofline
    is the iteration's: the bytes that loop must move per iteration over the
    measured time per iteration. It is bound by its two grid-wide exchanges
    per iteration (the reference's two dependent inner products), not by HBM:
    frac says how far."""
    from krylov_amd import problems

    P = problems.poisson2d(1000)
    r = run_cg_config(P, np.ones(P.shape[0]), steps, warmup)
    lay, n = r.pop("layout"), r["n"]
    t_it = r["us_per_it"] * 1e-6
    wr = (r["persistent_loop"] and lay["dia"] and os.environ.get("KRY_CGP_DIA", "1") != "0"
          and os.environ.get("KRY_CGP_WR", "1") != "0")
    if wr:
        # register-resident DIA form (round 5): the values are loaded once per
        # 256-iteration chunk, and r and p stored once per chunk; per
        # iteration each block reads its halo's r_t (span = 1000 rows either
        # side; the halo's p stays in LDS) and stores the r rows within span
        # of its edges (its neighbours' halos)
        spw = next(w for w in (1, 2, 4) if -(-lay["slices"] // (16 * w)) <= 256)
        G, span = -(-lay["slices"] // (16 * spw)), 1000
        b = (lay["dia_slots"] * 8 + 2 * n * 8) / 256 + 2 * (G * 2 * span * 8)
        form = ("(dia_slots*8 + 2*n*8)/256 (values in, r and p out once per chunk) + 2*G*2*span*8 (halo r_t read, "
                "edge r rows stored); y, Ap, p and the values stay on chip")
        kern = "cg_persist_kernel (DIA values in registers, x from an LDS halo; one launch per chunk)"
    elif r["persistent_loop"]:
        slots, slices = lay["slots"], lay["slices"]
        b = slots * (8 + 2) + slots / 64 * 4 + slices * 12 + 3 * n * 8
        form = ("slots*(8+2) + slots/64*4 + slices*12 (compact SELL-64 image) + 3*n*8 (p read once, r and p "
                "written; y, Ap and the partials stay on chip)")
        kern = "cg_persist_kernel (one launch per chunk of iterations)"
    else:
        kern, b, form = image_bytes_k1(lay, n, r["nnz"])
        b += 7 * n * 8
        form += " + 7*n*8 (update)"
    r["config"] = "BASELINE cfg2: CG on Poisson 1000^2, b = ones, tol = 0"
    r["roofline"] = {"bound": "hbm", "achieved": b / t_it / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": b / t_it / 1e9 / HBM_PEAK_GBS, "kernel": kern, "bytes_per_iteration": b,
                     "bytes_formula": form, "ms_per_iteration": 1e3 * t_it,
                     "note": "latency-bound: two grid-wide exchanges and one halo exchange per iteration "
                             "(profiles/r05_cgp_wr_ab.txt phase trace)"}
    return r


def run_gmres(R=None, label="cfg3 random nonsym n=2e6, GMRES(30) mgs, one cycle", ceiling_key=None):
    """GMRES(30) iterations/s, one 30-step cycle (tol = 0) incl. the final
    x = x0 + V y; median of 3 after one warm-up cycle. Default matrix: cfg3.
    Then one more cycle with HIP events around every SpMV and MGS launch:
    each kernel's roofline on the bytes it must move, and the cycle's."""
    import krylov_amd
    from krylov_amd import _helpers, _lib, problems
    from krylov_amd.device import get_context
    from krylov_amd.gmres import _GmresState

    if R is None:
        R = problems.random_nonsym(2_000_000)
    A = krylov_amd.CsrOperator(R)
    prob = _helpers.Problem(A, np.ones(R.shape[0]), None, None)
    ctx = get_context()
    st = _GmresState(prob, 30, 1)

    def cycle():
        st.start()
        st.set_criterion(np.zeros(1))
        ctx.synchronize()
        t0 = time.perf_counter()
        hist, _ = st.run(30)
        st.solution()
        ctx.synchronize()
        assert len(hist) == 30
        return time.perf_counter() - t0

    times = [cycle() for _ in range(4)][1:]
    t = float(np.median(times))
    n, nnz = R.shape[0], int(R.nnz)
    prof = profiled(ctx, [_lib.PROF_SPMV, _lib.PROF_MGS], cycle)
    (ns, ms_s), (nm, ms_m) = prof[_lib.PROF_SPMV], prof[_lib.PROF_MGS]
    layout = A.layout()
    kname, sb, sform = image_bytes_k1(layout, n, nnz, vectors=3)
    # MGS of Arnoldi step j: w in, V_0..V_j read once, V_{j+1} out (the first
    # inner product <V_0, w> is the SpMV epilogue's): (j + 3) n 8 B
    mgs_b = sum((j + 3) * n * 8 for j in range(30))
    sol_b = 32 * n * 8  # x = x0 + V y: V_0..V_29 and x0 read, x written
    cyc_b = 30 * sb + mgs_b + sol_b
    spmv_roof = hbm_roofline(kname, sb, ms_s / max(ns, 1) / 1e3, sform + " (w = A V_k stored; V_0 read for <V_0, w>)",
                             ns)
    mgs_roof = hbm_roofline("gm_mgsl_kernel / gm_mgsp_kernel (all MGS passes of a step in one launch)",
                            mgs_b / max(nm, 1), ms_m / max(nm, 1) / 1e3, "mean over steps j = 0..29 of (j + 3)*n*8 (w in, V_0..V_j read "
                            "once, V_{j+1} out)", nm)
    share_s, share_m = ms_s / 1e3 / t, ms_m / 1e3 / t
    out = {"it_per_s": 30.0 / t, "cycle_ms": 1e3 * t, "n": n, "nnz": nnz, "config": label,
           "roofline": spmv_roof if share_s >= share_m else mgs_roof,
           "spmv": spmv_roof, "mgs": mgs_roof,
           "time_share": {"spmv": share_s, "mgs": share_m, "rest": 1.0 - share_s - share_m},
           "cycle_roofline": {"bound": "hbm", "achieved": cyc_b / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": cyc_b / t / 1e9 / HBM_PEAK_GBS, "bytes_per_cycle": cyc_b,
                              "bytes_formula": "30 SpMVs (above) + sum_j (j+3)*n*8 (MGS) + 32*n*8 (x = x0 + V y)"}}
    if kname.startswith("spmv_cb"):
        cal = gather_ceiling(ceiling_key or "cfg3")
        if cal:
            sec = ms_s / max(ns, 1) / 1e3
            out["spmv"]["gather"] = {"bound": "gather", "achieved": nnz / sec / 1e9, "unit": "G gathers/s",
                                     "peak": cal["ceiling_g_per_s"], "frac": nnz / sec / 1e9 / cal["ceiling_g_per_s"],
                                     "peak_source": f"profiles/{GATHER_CEILING}[{ceiling_key or 'cfg3'}]: "
                                                    + cal["what"]}
    return out


def run_gmres_restarted(A_host, cycles=10):
    """krylov_amd.gmres_restarted(A, b, restart=30) on the metric matrix for
    `cycles` x0-chained cycles (tol small enough that none succeeds): the
    whole call (b upload, the chain on the device, the final x download) over
    its cycles, median of 3 after a warm-up."""
    import krylov_amd

    A = krylov_amd.CsrOperator(A_host)
    b = np.ones(A.n)

    def call():
        t0 = time.perf_counter()
        _, infos = krylov_amd.gmres_restarted(A, b, restart=30, tol=1e-300, atol=0.0, max_cycles=cycles)
        t = time.perf_counter() - t0
        assert len(infos) == cycles and all(i.numsteps == 30 for i in infos)
        return t

    call()
    t = float(np.median([call() for _ in range(3)]))
    return {"cycles": cycles, "call_ms": 1e3 * t, "cycle_ms": 1e3 * t / cycles, "it_per_s": 30 * cycles / t,
            "config": f"metric 15-point, krylov_amd.gmres_restarted restart=30, {cycles} x0-chained cycles "
                      "(b upload and x download included; the chain stays on the device)"}


def run_bicgstab(R, iters=30):
    """krylov_amd.bicgstab on the cfg3 matrix (tol = 0, `iters` iterations,
    2 SpMVs and 6 inner products each, the scalars chained on the device):
    the call's rate at the host-array boundary, median of 3 after a warm-up;
    then one call with HIP events around every SpMV (the dominant kernel)."""
    import krylov_amd
    from krylov_amd import _lib

    A = krylov_amd.CsrOperator(R)
    b = np.ones(R.shape[0])
    krylov_amd.bicgstab(A, b, tol=0.0, atol=0.0, maxiter=iters)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        _, info = krylov_amd.bicgstab(A, b, tol=0.0, atol=0.0, maxiter=iters)
        ts.append(time.perf_counter() - t0)
        assert info.numsteps == iters
    t = float(np.median(ts))
    n, nnz = R.shape[0], int(R.nnz)
    prof = profiled(A.ctx, [_lib.PROF_SPMV], lambda: krylov_amd.bicgstab(A, b, tol=0.0, atol=0.0, maxiter=iters))
    cnt, ms = prof[_lib.PROF_SPMV]
    kname, sb, sform = image_bytes_k1(A.layout(), n, nnz)
    roof = hbm_roofline(kname, sb, ms / max(cnt, 1) / 1e3, sform, cnt, spmv_share_of_call=ms / 1e3 / t)
    return {"it_per_s": iters / t, "call_ms": 1e3 * t, "n": n, "nnz": nnz, "roofline": roof,
            "config": f"cfg3 random nonsym n=2e6, krylov_amd.bicgstab tol=0 maxiter={iters} (b upload and x download "
                      "included)"}


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
        ts, keep = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            r = run()
            ts.append(time.perf_counter() - t0)
            assert r[1].numsteps == iters
            keep.append(r)  # the caller's x outlives the call: its release is not the solver's cost
        t0 = time.perf_counter()
        del keep, r
        out[f"{label}_result_free_ms"] = 1e3 * (time.perf_counter() - t0) / 3
        t = float(np.median(ts))
        out[f"{label}_it_per_s"] = iters / t
        out[f"{label}_call_ms"] = 1e3 * t
    # the call's fixed cost: the call minus its own chunked device loop
    # (krylov_amd.cg.last_timing: the host clock around the kry_cg_run calls)
    cgmod = sys.modules["krylov_amd.cg"]
    fixed, parts = [], []
    names = ("problem_ms", "setup_start_ms", "loop_host_ms", "get_ms", "finish_ms")
    for _ in range(5):
        r = krylov_amd.cg(A, b, tol=0.0, atol=0.0, maxiter=steps)
        lt = dict(cgmod.last_timing)
        fixed.append(lt["call_ms"] - lt["chunks_ms"])
        parts.append([lt[nm] for nm in names])
        del r
    out["cg_fixed_ms"] = float(np.median(fixed))
    med = dict(zip(names, np.median(np.array(parts), axis=0)))
    out["cg_fixed_parts_ms"] = {nm: float(v) for nm, v in med.items()}
    # the box's host link, from the two 80 MB copies of the call (b in, x out):
    # the fixed cost net of them is what the library spends itself
    out["h2d_gbs"] = b.nbytes / (med["problem_ms"] * 1e6)
    out["d2h_gbs"] = b.nbytes / (med["get_ms"] * 1e6)
    out["cg_fixed_net_of_copies_ms"] = out["cg_fixed_ms"] - med["problem_ms"] - med["get_ms"]
    out["includes"] = ("b upload (H2D), solver state setup, per-chunk host syncs, x download (D2H); the operator "
                       "is uploaded once before (CsrOperator); cg_fixed_ms = the call minus its own chunked device "
                       "loop (median of 5); the caller's x is released after the timing (result_free_ms)")
    # the operator upload itself (kry_csr_create: one H2D of the CSR arrays,
    # the SELL-64 and DIA images built on the device), median of 3
    del A
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        op = krylov_amd.CsrOperator(A_host)
        op.ctx.synchronize()
        ts.append(time.perf_counter() - t0)
        del op
    out["csr_create_s"] = float(np.median(ts))
    return out


def run_minres_cfg5(steps=100):
    """BASELINE cfg5: MINRES on the shifted, row-scaled 3-D Laplacian 200^3
    (fp32 matrix, W-weighted inner with float64 w, so float64 vectors as in
    the reference), 100 fixed iterations. Then one more pass of 64 with HIP
    events around every SpMV and update launch: each kernel's roofline."""
    import krylov_amd
    from krylov_amd import _helpers, _lib, problems
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

    def iterate(k):
        done = 0
        while done < k:
            hist, inv = st.run(min(32, k - done))
            assert len(hist) == min(32, k - done) and not inv, "MINRES stopped early"
            done += len(hist)

    t0 = time.perf_counter()
    iterate(steps)
    ctx.synchronize()
    t = time.perf_counter() - t0
    prof = profiled(ctx, [_lib.PROF_SPMV, _lib.PROF_UPDATE], lambda: iterate(64))
    (ns, ms_s), (nu, ms_u) = prof[_lib.PROF_SPMV], prof[_lib.PROF_UPDATE]
    n, nnz = W.shape[0], int(W.nnz)
    kname, sb, sform = image_bytes_k1(A.layout(), n, nnz, vectors=3, vb=4)
    ub = 8 * n * 8 + n * 8
    out = {"it_per_s": steps / t, "us_per_it": 1e6 * t / steps, "n": n, "nnz": nnz,
           "config": "BASELINE cfg5: MINRES on the shifted 3-D Laplacian 200^3, fp32 matrix, f64 weights "
                     "(vectors f64 as in the reference), 100 fixed iterations",
           "spmv": hbm_roofline(kname + " (EpiLanczos)", sb, ms_s / max(ns, 1) / 1e3,
                                sform + " (Av = A v - h0 p_old: v read, p_old read, Av written; fp32 values)", ns),
           "update": hbm_roofline("mr_upd_kernel (the step tail in one launch)", ub, ms_u / max(nu, 1) / 1e3,
                                  "8*n*8 (w, p, W0, W1, yk in; z, yk, p_new out) + n*8 (weights)", nu)}
    it_b = sb + ub
    out["roofline"] = out["spmv"] if ms_s >= ms_u else out["update"]
    out["iteration_roofline"] = {"bound": "hbm", "achieved": it_b / (t / steps) / 1e9, "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": it_b / (t / steps) / 1e9 / HBM_PEAK_GBS,
                                 "bytes_per_iteration": it_b, "bytes_formula": "SpMV + update (above)"}
    return out


GATHER_CEILING = "r04_gather_ceiling.json"


def cpu_baseline(A_host, runs=5, target_run_s=3.0):
    """The oracle (reference iteration on NumPy/SciPy, oracle/krylov_ref.py)
    timed on this host: CG with tol=0 on the metric matrix. Each sample is one
    cg call of `iters` iterations minus one call of 0 iterations (its setup
    residual and final explicit residual), both the median of `runs` calls."""
    from oracle import krylov_ref

    b = np.ones(A_host.shape[0])

    def call(m):
        t0 = time.perf_counter()
        krylov_ref.cg(A_host, b, tol=0.0, atol=0.0, maxiter=m)
        return time.perf_counter() - t0

    t_setup = call(0)
    t_cal = call(2) - t_setup
    iters = int(max(3, min(40, target_run_s / max(t_cal / 2.0, 1e-3))))
    t0s = [call(0) for _ in range(runs)]
    tms = [call(iters) for _ in range(runs)]
    per_it = (float(np.median(tms)) - float(np.median(t0s))) / iters
    threads = os.environ.get("OPENBLAS_NUM_THREADS") or os.environ.get("OMP_NUM_THREADS") or str(os.cpu_count())
    return {
        "value": 1.0 / per_it,
        "unit": "CG iters/s",
        "cores": int(threads),
        "kind": "port",
        "sample": f"median of {runs} oracle/krylov_ref.cg calls of {iters} iterations (tol=0) minus the median of "
                  f"{runs} calls of 0 iterations (setup + explicit residual), full 216^3 15-pt matrix; SciPy "
                  f"csr_matvec 1 thread, np.dot OpenBLAS {threads} threads",
        "samples_s": tms,
        "setup_samples_s": t0s,
    }


def cfg4_rhs(n, rank, k=8):
    """cfg4's per-GPU block: 8 standard-normal RHS columns (BASELINE cfg4:
    B = default_rng(0).standard_normal((n, 64)), 8 per GPU; each rank draws
    its own 8 columns from default_rng(rank) instead of slicing a 5 GB host
    array: synthetic data of that shape, timed with tol = 0)."""
    return np.random.default_rng(rank).standard_normal((n, k))


def run_spmv_general(A_host, steps):
    """The same CG SpMV measurement with the DIA image disabled
    (KRY_SPMV_DIA=0 at upload): the kernel a general CSR matrix takes when it
    is not diagonal-structured (the paired-row SELL-128 image since round 3;
    KRY_SPMV_PAIR=0: the compact SELL-64 kernel)."""
    prev = os.environ.get("KRY_SPMV_DIA")
    os.environ["KRY_SPMV_DIA"] = "0"
    try:
        res = run_cg_bench(A_host, lambda _r: np.ones(A_host.shape[0]), steps, 5, Job.single())
    finally:
        if prev is None:
            del os.environ["KRY_SPMV_DIA"]
        else:
            os.environ["KRY_SPMV_DIA"] = prev
    assert not res["layout"]["dia"]
    n, nnz = A_host.shape[0], int(A_host.nnz)
    roof = roofline_of(res, n, nnz)
    roof["cg_it_per_s"] = steps / res["elapsed"]
    roof["n"], roof["nnz"] = n, nnz
    return roof


def run_spmv_unstructured(A_host, steps):
    """The metric matrix under a fixed random symmetric permutation
    (problems.permuted_sym, seed 0: the same nonzeros and values, scattered
    columns): CG's SpMV as general CSR takes it, with the kernel it lands on
    and that kernel's roofline on its image bytes (and, for the column-blocked
    kernels, its gather rate against the measured ceiling)."""
    from krylov_amd import problems

    B = problems.permuted_sym(A_host, 0)
    n, nnz = B.shape[0], int(B.nnz)
    res = run_cg_bench(B, lambda _r: np.ones(n), steps, 5, Job.single(), roofline_launches=steps)
    kname, sb, form = image_bytes_k1(res["layout"], n, nnz)
    roof = hbm_roofline(kname, sb, res["spmv_avg_s"], form, res["spmv_count"],
                        cg_it_per_s=steps / res["elapsed"], matrix="15-point 216^3 under P A P^T, P = "
                        "default_rng(0).permutation(n)", n=n, nnz=nnz)
    cal = gather_ceiling("metric_permuted")
    if cal and kname.startswith("spmv_cb"):
        roof["gather"] = {"bound": "gather", "achieved": nnz / res["spmv_avg_s"] / 1e9, "unit": "G gathers/s",
                          "peak": cal["ceiling_g_per_s"], "frac": nnz / res["spmv_avg_s"] / 1e9 / cal["ceiling_g_per_s"],
                          "peak_source": f"profiles/{GATHER_CEILING}[metric_permuted]: " + cal["what"]}
    return roof


TRAFFIC_INDEX = "r06_traffic_index.json"
FORMULAS = "profiles/bench_formulas.md"


def traffic_index():
    """Per-leg HBM traffic per launch from the committed PMC summaries
    (profiles/<TRAFFIC_INDEX>, built by tools/traffic_index.py from the
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of tools/pmc_legs.sh): {leg:
    {kernel key: {"bytes": B, "src": file, "build": stamp}}}."""
    try:
        with open(os.path.join(REPO, "profiles", TRAFFIC_INDEX)) as f:
            return json.load(f)
    except OSError:
        return {}


def leg_traffic(idx, leg, key, n, nnz):
    """(bytes, source) of one leg's kernel, or (None, None) unless the entry
    was taken on the same matrix (n, nnz) AND on the library build that is
    loaded now (kry_build_id): a PMC of other code is not evidence for this
    one, so the line then says traffic: null."""
    from krylov_amd import _lib

    e = idx.get(leg, {}).get(key) if isinstance(idx.get(leg), dict) else None
    if not e or e.get("n") != n or e.get("nnz") != nnz or e.get("build") != _lib.build_id():
        return None, None
    return e["bytes"], e["src"]


def _r(x, d=4):
    """Round to d significant digits (compact line)."""
    if isinstance(x, float):
        return float(f"{x:.{d}g}")
    return x


def _short(kernel):
    """The kernel's name without template arguments or descriptions."""
    return kernel.split("<")[0].split(" (")[0].strip()


def _kroof(r, traffic=None, src=None):
    """Compact form of one kernel roofline object."""
    out = {"kernel": _short(r["kernel"]), "ms": _r(r["ms_per_launch"]), "bytes": int(r["bytes_per_launch"]),
           "frac": _r(r["frac"], 3), "traffic": int(traffic) if traffic else None}
    if out["traffic"] and src:
        out["traffic_src"] = src.split(" ")[0]
    return out


def compact(full, idx=None):
    """The driver keeps only the tail of bench.py's stdout (about 8 KB), so
    the printed line is this compact form (<= 6 KB): the contract keys, the
    headline roofline and cpu_baseline, and per leg only its rate, its
    dominant kernel (short name), bytes per launch, frac and HBM traffic.
    Kernel template names and byte formulas are in profiles/bench_formulas.md
    (FORMULAS); --full-out PATH writes the verbose line as well."""
    idx = traffic_index() if idx is None else idx
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "repeats", "ms_per_step_min",
            "ms_per_step_max", "launch", "rccl_ranks", "higher_is_better", "scaling", "vs_baseline", "dtype", "data",
            "config")
    out = {k: _r(full[k]) if k.startswith(("value", "ms_per_step")) else full[k] for k in keys if k in full}
    ro = full["roofline"]
    out["roofline"] = {"bound": ro["bound"], "achieved": _r(ro["achieved"]), "peak": ro["peak"], "unit": ro["unit"],
                       "frac": _r(ro["frac"], 3), "traffic": int(ro["traffic"]) if ro.get("traffic") else None,
                       "kernel": _short(ro["kernel"]),
                       "ms_per_launch": _r(ro["ms_per_launch"]), "bytes_per_launch": int(ro["bytes_per_launch"]),
                       "launches_timed": ro.get("launches_timed")}
    if ro.get("traffic_source"):
        out["roofline"]["traffic_src"] = ro["traffic_source"].split(" ")[0]
    it = full.get("iteration_roofline")
    if it:
        out["iteration_roofline"] = {"frac": _r(it["frac"], 3), "bytes": int(it.get("bytes_per_iteration", 0))}
    legs = {}
    c4 = full.get("cfg4_sharded")
    if c4:
        n, nnz = c4["n"], c4["nnz"]
        t, src = leg_traffic(idx, "cfg4", "spmv", n, nnz)
        legs["cfg4_sharded"] = {"it_per_s": _r(c4["it_per_s"]), "rhs_it_per_s": _r(c4["rhs_it_per_s"]),
                                **_kroof(c4["roofline"], t, src), "iter_frac": _r(c4["iteration_roofline"]["frac"], 3),
                                "ydefer": c4["iteration_roofline"].get("ydefer"), "rccl_ranks": c4.get("rccl_ranks")}
    for leg in ("spmv_general", "spmv_unstructured"):
        r = full.get(leg)
        if r:
            n, nnz = r.get("n", 0), r.get("nnz", 0)
            t, src = leg_traffic(idx, leg, "spmv", n, nnz)
            legs[leg] = {"cg_it_per_s": _r(r.get("cg_it_per_s")), **_kroof(r, t, src)}
            if "gather" in r:
                legs[leg]["gather_frac"] = _r(r["gather"]["frac"], 3)
    for leg in ("gmres", "gmres_metric"):
        g = full.get(leg)
        if g:
            n, nnz = g["n"], g["nnz"]
            ts, ss = leg_traffic(idx, leg, "spmv", n, nnz)
            tm, sm = leg_traffic(idx, leg, "mgs", n, nnz)
            legs[leg] = {"it_per_s": _r(g["it_per_s"]), "cycle_ms": _r(g["cycle_ms"]),
                         "spmv": _kroof(g["spmv"], ts, ss), "mgs": _kroof(g["mgs"], tm, sm),
                         "cycle_frac": _r(g["cycle_roofline"]["frac"], 3),
                         "share": {k: _r(v, 3) for k, v in g["time_share"].items()}}
            if "gather" in g["spmv"]:
                legs[leg]["spmv"]["gather_frac"] = _r(g["spmv"]["gather"]["frac"], 3)
    gr = full.get("gmres_metric_restarted")
    if gr:
        legs["gmres_metric_restarted"] = {"it_per_s": _r(gr["it_per_s"]), "cycle_ms": _r(gr["cycle_ms"]),
                                          "vs_single_cycle": _r(gr.get("vs_single_cycle"))}
    b = full.get("bicgstab_cfg3")
    if b:
        t, src = leg_traffic(idx, "bicgstab_cfg3", "spmv", b["n"], b["nnz"])
        legs["bicgstab_cfg3"] = {"it_per_s": _r(b["it_per_s"]), **_kroof(b["roofline"], t, src)}
    e = full.get("end_to_end")
    if e:
        legs["end_to_end"] = {k: ({kk: _r(vv, 3) for kk, vv in v.items()} if isinstance(v, dict) else _r(v))
                              for k, v in e.items() if k != "includes"}
    c2 = full.get("cfg2")
    if c2:
        r = c2["roofline"]
        t, src = leg_traffic(idx, "cfg2", "iteration", c2["n"], c2["nnz"])
        legs["cfg2"] = {"it_per_s": _r(c2["it_per_s"]), "kernel": _short(r["kernel"]),
                        "ms": _r(r["ms_per_iteration"]), "bytes": int(r["bytes_per_iteration"]),
                        "frac": _r(r["frac"], 3), "traffic": int(t) if t else None}
        if src:
            legs["cfg2"]["traffic_src"] = src
    c5 = full.get("cfg5")
    if c5:
        ts, ss = leg_traffic(idx, "cfg5", "spmv", c5["n"], c5["nnz"])
        tu, su = leg_traffic(idx, "cfg5", "update", c5["n"], c5["nnz"])
        legs["cfg5"] = {"it_per_s": _r(c5["it_per_s"]), "spmv": _kroof(c5["spmv"], ts, ss),
                        "update": _kroof(c5["update"], tu, su), "iter_frac": _r(c5["iteration_roofline"]["frac"], 3)}
    if legs:
        out["legs"] = legs
    cb = full.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {k: (_r(cb[k]) if k == "value" else cb[k]) for k in ("value", "unit", "cores", "kind",
                                                                                 "sample")}
    out["formulas"] = FORMULAS
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--m", type=int, default=216, help="stencil edge (216 = BASELINE metric)")
    ap.add_argument("--workload", choices=["metric", "cfg4"], default="metric",
                    help="headline: metric CG (1 RHS per GPU) or cfg4 block CG (8 RHS per GPU, Poisson 3163^2)")
    ap.add_argument("--quick", action="store_true", help="headline only (no other legs, no CPU baseline)")
    ap.add_argument("--configs", action="store_true",
                    help="also time cfg4 as a plain 8-RHS block CG (and cfg2 / cfg5 under --quick; the full run has them)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--full-out", default=None, help="also write the verbose JSON line (formulas, timings) here")
    ap.add_argument("--launch", choices=["auto", "threads"], default="auto",
                    help="auto: torchrun if WORLD_SIZE is set, else threads for --gpus > 1; threads: force the "
                         "one-process threaded path (also at --gpus 1, a rehearsal with a 1-rank communicator)")
    ap.add_argument("--repeats", type=int, default=5,
                    help="timed regions of --steps iterations each; the line reports their median (min and max beside)")
    args = ap.parse_args()

    from krylov_amd import _lib

    plan = plan_launch(args.gpus, os.environ, _lib.device_count, args.launch)
    if plan["note"]:
        print("note: " + plan["note"], file=sys.stderr)
    job = Job(plan)
    world, rank = job.world, job.rank
    os.environ["KRYLOV_DEVICE"] = str(job.local)
    repeats = max(1, args.repeats)

    from krylov_amd import problems

    A_host = problems.stencil15_3d(args.m)
    n, nnz = A_host.shape[0], int(A_host.nnz)
    P3 = None
    cfg4 = None
    if args.workload == "cfg4" or not args.quick:
        P3 = problems.poisson2d(3163)
        cfg4 = run_cg_bench(P3, lambda r: cfg4_rhs(P3.shape[0], r), min(args.steps, 40), min(args.warmup, 5), job,
                            repeats=repeats, roofline_launches=16, prof_ids=[_lib.PROF_UPDATE, _lib.PROF_OTHER])
    if args.workload == "cfg4":
        res, hn, hnnz = cfg4, P3.shape[0], int(P3.nnz)
        workload = (f"krylov.cg block CG, 2-D 5-point Poisson 3163^2, {cfg4['rhs']} RHS per GPU (BASELINE cfg4), "
                    "tol=0 fixed iterations")
        steps_timed = min(args.steps, 40)
    else:
        res = run_cg_bench(A_host, lambda _r: np.ones(n), args.steps, args.warmup, job, repeats=repeats)
        hn, hnnz = n, nnz
        workload = f"krylov.cg, 3-D 15-point stencil {args.m}^3, one RHS per GPU, tol=0 fixed iterations"
        steps_timed = args.steps
    T = res["elapsed"]
    rhs = res["rhs"]
    if args.workload == "cfg4":
        roof, it_roof = cfg4_rooflines(res, steps_timed)
        t, src = leg_traffic(traffic_index(), "cfg4", "spmv", hn, hnnz)
        roof["traffic"], roof["traffic_source"] = t, src
    else:
        t, src = leg_traffic(traffic_index(), "metric_cg", "spmv", hn, hnnz)
        roof = roofline_of(res, hn, hnnz, {"traffic_bytes_per_launch": t, "source": src} if t else None)
        # the iteration: the SpMV's image bytes + the one-launch update
        # (cg_upd_kernel: r, y, p read and written, Ap read = 7 n 8 B)
        it_b = roof["bytes_per_launch"] + 7 * hn * 8
        t_it = T / steps_timed
        it_roof = {"bound": "hbm", "achieved": it_b / t_it / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": it_b / t_it / 1e9 / HBM_PEAK_GBS, "bytes_per_iteration": it_b,
                   "bytes_formula": "SpMV image bytes (roofline.bytes_per_launch) + 7*n*8 (cg_upd_kernel: r, y, p "
                                    "in and out, Ap in)"}
    out = {
        "metric": "CG iters/sec + SpMV GB/s (fp64, n=10M, nnz=150M); GMRES(30) iters/sec",
        "value": world * rhs * steps_timed / T,
        "unit": "CG iters/s (RHS-iterations/s over all GPUs)",
        "n_gpus": world,
        "steps": steps_timed,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * T / steps_timed,
        "repeats": len(res["elapsed_all"]),
        "ms_per_step_min": 1e3 * min(res["elapsed_all"]) / steps_timed,
        "ms_per_step_max": 1e3 * max(res["elapsed_all"]) / steps_timed,
        "launch": job.mode,
        "rccl_ranks": res["rccl_ranks"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY App. A generator, b = ones)" if args.workload == "metric" else
                "synthetic (SURVEY App. A poisson2d generator, standard-normal RHS)",
        "config": {
            "workload": workload,
            "n": hn,
            "nnz": hnnz,
            "index": "int32",
            "rhs_per_gpu": rhs,
            "parallelism": f"rhs-shard x{world}" + (" (one RCCL resnorm allreduce per iteration)" if world > 1 else ""),
            "launch": {"torchrun": "one process per GPU (torch.distributed.run)",
                       "threads": "one process, one host thread per GPU, ncclCommInitAll",
                       "single": "one GPU"}[job.mode],
        },
        "spmv_gbs": roof["achieved"],
        "spmv_ms": roof["ms_per_launch"],
        "roofline": roof,
        "iteration_roofline": it_roof,
    }
    if cfg4 is not None and args.workload != "cfg4":
        c4 = P3.shape[0]
        out["cfg4_sharded"] = {
            "rhs_it_per_s": world * cfg4["rhs"] * min(args.steps, 40) / cfg4["elapsed"],
            "it_per_s": min(args.steps, 40) / cfg4["elapsed"],
            "ms_per_it": 1e3 * cfg4["elapsed"] / min(args.steps, 40),
            "rhs_per_gpu": cfg4["rhs"],
            "n": c4,
            "nnz": int(P3.nnz),
            "spmv_ms": 1e3 * cfg4["spmv_avg_s"],
            "rccl_ranks": cfg4["rccl_ranks"],
            "config": "BASELINE cfg4: Poisson 3163^2 block CG, 8 RHS per GPU"
                      + (f", {world} ranks, one RCCL allreduce per iteration" if world > 1
                         else ", one GPU (no communicator attached at N = 1)"),
        }
        c4_spmv, c4_it = cfg4_rooflines(cfg4, min(args.steps, 40))
        out["cfg4_sharded"]["roofline"] = c4_spmv
        out["cfg4_sharded"]["iteration_roofline"] = c4_it
    del P3
    if world == 1 and not args.quick and args.workload == "metric":
        out["spmv_general"] = run_spmv_general(A_host, args.steps)
        out["spmv_unstructured"] = run_spmv_unstructured(A_host, min(args.steps, 64))
        R3 = problems.random_nonsym(2_000_000)
        g = run_gmres(R3, ceiling_key="cfg3")
        out["gmres30_it_per_s"] = g["it_per_s"]
        out["gmres"] = g
        out["bicgstab_cfg3"] = run_bicgstab(R3)
        del R3
        # north_star: GMRES(30) on the same (metric) matrix
        out["gmres_metric"] = run_gmres(A_host, f"metric 15-point {args.m}^3, GMRES(30) mgs, one cycle")
        out["gmres_metric_restarted"] = run_gmres_restarted(A_host)
        out["gmres_metric_restarted"]["vs_single_cycle"] = (out["gmres_metric_restarted"]["cycle_ms"]
                                                            / out["gmres_metric"]["cycle_ms"])
        out["end_to_end"] = run_end_to_end(A_host, args.steps)
        out["cfg2"] = run_cfg2()
        out["cfg5"] = run_minres_cfg5()
    if world == 1 and args.configs:
        extra = {}
        P3 = problems.poisson2d(3163)
        B = np.random.default_rng(0).standard_normal((P3.shape[0], 8))
        extra["cfg4_blockcg_8rhs_per_gpu"] = run_cg_config(P3, B, 20, 3)
        extra["cfg4_blockcg_8rhs_per_gpu"].pop("layout")
        del P3, B
        if args.quick:
            extra["cfg2"] = run_cfg2()
            extra["cfg5"] = run_minres_cfg5()
        out["extra"] = extra
    if rank == 0 and world == 1 and not args.no_cpu and not args.quick and args.workload == "metric":
        out["cpu_baseline"] = cpu_baseline(A_host)
    if rank == 0:
        if args.full_out:
            with open(args.full_out, "w") as f:
                f.write(json.dumps(out) + "\n")
        print(json.dumps(compact(out)), flush=True)
    job.close()


if __name__ == "__main__":
    main()
