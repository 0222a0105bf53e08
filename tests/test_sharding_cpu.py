"""RHS-column sharding semantics on CPU (world_size 2, gloo).

The sharded path (krylov_amd.distributed.cg on GPUs over RCCL) splits the
reference's block right-hand side into per-rank column blocks and couples
them only through one allreduce of the zero-padded residual-norm vector per
iteration (the global stop rule, cg.py:156,162). This test restates that
decomposition on the host with gloo and checks it reproduces the reference's
own unsharded block-CG fixture bit for bit (per-column recurrences are
independent, so sharding must not change a single bit of the history).
"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sharded_cg_host(A, B_local, allreduce, rank, world, tol, atol=1e-15, maxiter=None):
    """Host restatement of the device loop of krylov_amd.distributed.cg."""
    kl = B_local.shape[1]
    total = kl * world

    def glob(v):
        full = np.zeros(total)
        full[rank * kl:(rank + 1) * kl] = v
        return allreduce(full)

    def inner(x, y):
        return np.einsum("i...,i...->...", x, y)

    x = np.zeros_like(B_local)
    r = B_local - A @ x
    rho = inner(r, r)
    resn = [np.sqrt(glob(rho))]
    crit = np.maximum(tol * resn[0], atol)
    y = np.zeros_like(B_local)
    p = r.copy()
    rho_prev = None
    k = 0
    maxiter = A.shape[0] if maxiter is None else maxiter
    while True:
        if np.all(resn[-1] <= crit):
            rr = B_local - A @ (x + y)
            resn[-1] = np.sqrt(glob(inner(rr, rr)))
            if np.all(resn[-1] <= crit):
                break
        if k == maxiter:
            break
        if k > 0:
            p = r + (rho / np.where(rho_prev != 0, rho_prev, 1.0)) * p
        Ap = A @ p
        alpha = rho / np.where(inner(p, Ap) != 0, inner(p, Ap), 1.0)
        y += alpha * p
        r -= alpha * Ap
        rho_prev, rho = rho, inner(r, r)
        resn.append(np.sqrt(glob(rho)))
        k += 1
    return k, np.array(resn), x + y


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce(v):
        t = torch.from_numpy(np.ascontiguousarray(v))
        dist.all_reduce(t)
        return t.numpy().copy()

    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from krylov_amd import problems

    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "solvers.npz"))
    P = problems.poisson2d(64)
    B = d["poisson64_B"]
    kl = B.shape[1] // world
    k, resn, x = _sharded_cg_host(P, B[:, rank * kl:(rank + 1) * kl].copy(), allreduce, rank, world, tol=1e-8)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), k=k, resn=resn, x=x)
    dist.destroy_process_group()


def test_rhs_sharding_reproduces_block_cg_bitwise(tmp_path):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "solvers.npz"))
    ref_k = int(d["cg_poisson64_blk8_numsteps"])
    ref_res = d["cg_poisson64_blk8_resnorms"]
    xs = []
    for r in range(world):
        o = np.load(tmp_path / f"r{r}.npz")
        assert int(o["k"]) == ref_k
        np.testing.assert_array_equal(o["resn"], ref_res)  # global history on every rank
        xs.append(o["x"])
    np.testing.assert_array_equal(np.concatenate(xs, axis=1), d["cg_poisson64_blk8_xk"])


# ---------------------------------------------------------------- GMRES / MINRES
# krylov_amd.distributed.gmres / .minres couple the ranks through one
# allreduce per step of the residual norms and a non-invariant count. The
# oracle restatements take the same coupling as a `shard` hook; over gloo,
# one column per rank must reproduce the unsharded block solve (same stop
# step; per-column recurrences equal up to the einsum of a (n, 1) vs (n, 3)
# block) and the reference's block-GMRES fixture.


def _solver_worker(rank, world, port, outdir, which):
    import sys

    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from krylov_amd import problems
    from oracle import krylov_ref

    def shard(local):
        local = np.atleast_1d(np.asarray(local, dtype=np.float64))
        full = np.zeros(world * local.size)
        full[rank * local.size:(rank + 1) * local.size] = local
        t = torch.from_numpy(full)
        dist.all_reduce(t)
        return t.numpy().copy()

    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "solvers.npz"))
    out = {}
    if which == "gmres":
        R = problems.random_nonsym(5000)
        B = d["rand5k_B3"]
        Bl = B[:, [rank]].copy()
        _, info = krylov_ref.gmres(R, Bl, maxiter=20, tol=0.0, shard=shard)
        out["fixed_k"], out["fixed_res"], out["fixed_x"] = info.numsteps, np.array(info.resnorms), info.xk
        # columns converge at different steps: the global rule keeps all going
        _, info = krylov_ref.gmres(R, Bl, maxiter=60, tol=1e-6, shard=shard)
        out["tol_k"], out["tol_res"] = info.numsteps, np.array(info.resnorms)
    else:
        P = problems.poisson2d(32)
        B = np.random.default_rng(3).standard_normal((P.shape[0], world))
        B[:, 1] *= 1e-3
        _, info = krylov_ref.minres(P, B[:, [rank]].copy(), tol=1e-8, shard=shard)
        out["tol_k"], out["tol_res"], out["x"] = info.numsteps, np.array(info.resnorms), info.xk
    np.savez(os.path.join(outdir, f"{which}{rank}.npz"), **out)
    dist.destroy_process_group()


def test_rhs_sharding_gmres_global_rules(tmp_path):
    pytest.importorskip("torch")
    import torch.multiprocessing as mp

    from krylov_amd import problems
    from oracle import krylov_ref

    world = 3
    mp.spawn(_solver_worker, args=(world, _free_port(), str(tmp_path), "gmres"), nprocs=world, join=True)
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "solvers.npz"))
    R = problems.random_nonsym(5000)
    B = d["rand5k_B3"]
    _, blk = krylov_ref.gmres(R, B, maxiter=60, tol=1e-6)
    ref_k = int(d["gmres_rand5k_blk3_numsteps"])
    ref_res = np.asarray(d["gmres_rand5k_blk3_resnorms"])
    for r in range(world):
        o = np.load(tmp_path / f"gmres{r}.npz")
        assert int(o["fixed_k"]) == ref_k
        np.testing.assert_allclose(o["fixed_res"], ref_res, rtol=1e-12)  # global history on every rank
        np.testing.assert_allclose(o["fixed_x"][:, 0], d["gmres_rand5k_blk3_xk"][:, r], rtol=1e-9, atol=1e-12)
        assert int(o["tol_k"]) == blk.numsteps  # the slowest column decides the global stop step
        ref = np.asarray(blk.resnorms)
        np.testing.assert_allclose(o["tol_res"][:-1], ref[:-1], rtol=1e-12)
        # the final entry is the explicit residual: compared absolutely
        np.testing.assert_allclose(o["tol_res"][-1], ref[-1], rtol=0, atol=1e-12 * ref[0].max())


def test_rhs_sharding_minres_global_rules(tmp_path):
    pytest.importorskip("torch")
    import torch.multiprocessing as mp

    from krylov_amd import problems
    from oracle import krylov_ref

    world = 2
    mp.spawn(_solver_worker, args=(world, _free_port(), str(tmp_path), "minres"), nprocs=world, join=True)
    P = problems.poisson2d(32)
    B = np.random.default_rng(3).standard_normal((P.shape[0], world))
    B[:, 1] *= 1e-3
    _, blk = krylov_ref.minres(P, B, tol=1e-8)
    for r in range(world):
        o = np.load(tmp_path / f"minres{r}.npz")
        assert int(o["tol_k"]) == blk.numsteps
        ref = np.asarray(blk.resnorms)
        np.testing.assert_allclose(o["tol_res"][:-1], ref[:-1], rtol=1e-12)
        np.testing.assert_allclose(o["tol_res"][-1], ref[-1], rtol=0, atol=1e-12 * ref[0].max())
        np.testing.assert_allclose(o["x"][:, 0], blk.xk[:, r], rtol=1e-10, atol=1e-13)
