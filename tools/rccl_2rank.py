"""A real two-rank RCCL allreduce on the pool's one-GPU box: two processes,
both on device 0, one communicator (krylov_amd.distributed.ShardComm.from_file).
Rank r solves columns [8 r, 8 r + 8) of a 16-column block problem with
krylov_amd.distributed.cg / gmres / minres. The parent then checks:
- at tol = 0 (fixed steps: the halves do not interact but through the
  allreduce), bit for bit, that each rank's iterate equals the one-process
  8-column solve of its half, and that both ranks' global histories equal
  those two solves' histories side by side (every step's allreduce summed
  the other rank's slots in);
- at tol = 1e-8, that both ranks stop at the step of the 16-column block
  solve (the global stop rule over both ranks' columns) with its history to
  1e-12.
If RCCL refuses two ranks on one device, the script says so and exits 3:
RCCL does ("Duplicate GPU detected", gpurun r05t, profiles/r05_rccl_2rank.txt),
so on the pool's one-GPU boxes the real cross-rank sum cannot run; on a node
with two GPUs, KRY_2RANK_DEVICES=0,1 puts the ranks on two devices.

    python3 tools/rccl_2rank.py            (parent: spawns the two ranks)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = (("cg", dict(tol=0.0, atol=0.0, maxiter=60)), ("gmres", dict(tol=0.0, atol=0.0, maxiter=25)),
         ("minres", dict(tol=0.0, atol=0.0, maxiter=60)), ("cg", dict(tol=1e-8, maxiter=400)))


def problem():
    from krylov_amd import problems

    P = problems.poisson2d(96)
    B = np.random.default_rng(8).standard_normal((P.shape[0], 16))
    return P, B


def worker(rank, path, out):
    from krylov_amd import distributed

    P, B = problem()
    devs = [int(d) for d in os.environ.get("KRY_2RANK_DEVICES", "0,0").split(",")]
    comm = distributed.ShardComm.from_file(path, rank, 2, device=devs[rank])
    for c, (method, kw) in enumerate(CASES):
        _, info = getattr(distributed, method)(P, np.ascontiguousarray(B[:, 8 * rank:8 * rank + 8]), comm, **kw)
        np.save(f"{out}_{c}_{rank}_x.npy", np.asarray(info.xk))
        np.save(f"{out}_{c}_{rank}_h.npy", np.array(info.resnorms))
        np.save(f"{out}_{c}_{rank}_n.npy", np.array([info.numsteps, int(bool(info.success))]))
    comm.close()
    print(f"rank {rank}: done", flush=True)


def main():
    tmp = tempfile.mkdtemp(prefix="rccl2_")
    path = f"/dev/shm/krylov_rccl2_{os.getpid()}.id"
    out = os.path.join(tmp, "r")
    procs = [subprocess.Popen([sys.executable, "-u", __file__, "worker", str(r), path, out]) for r in range(2)]
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=180))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    if os.path.exists(path):
        os.remove(path)
    if any(rcs):
        print(f"ranks exited {rcs}: two RCCL ranks on one device did not complete", flush=True)
        sys.exit(3)
    import krylov_amd

    P, B = problem()
    ok = True

    def bits(a, b):
        a, b = np.asarray(a), np.asarray(b)
        return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))

    for c, (method, kw) in enumerate(CASES):
        x = [np.load(f"{out}_{c}_{r}_x.npy") for r in range(2)]
        h = [np.load(f"{out}_{c}_{r}_h.npy") for r in range(2)]
        nm = [np.load(f"{out}_{c}_{r}_n.npy") for r in range(2)]
        if kw["tol"] == 0.0:
            halves = [getattr(krylov_amd, method)(P, np.ascontiguousarray(B[:, 8 * r:8 * r + 8]), **kw)[1]
                      for r in range(2)]
            glob = np.concatenate([np.array(halves[r].resnorms) for r in range(2)], axis=1)
            same_x = all(bits(x[r], halves[r].xk) for r in range(2))
            same_h = all(bits(hh, glob) for hh in h)
            steps = all(int(n[0]) == halves[0].numsteps for n in nm)
            print(f"{method} tol=0: {halves[0].numsteps} steps; 2-rank xk bitwise the halves {same_x}, global "
                  f"histories bitwise {same_h}, steps equal {steps}", flush=True)
            ok = ok and same_x and same_h and steps
        else:
            _, ref = getattr(krylov_amd, method)(P, B, **kw)
            steps = all(int(n[0]) == ref.numsteps and bool(n[1]) == bool(ref.success) for n in nm)
            close = all(np.allclose(hh, np.array(ref.resnorms), rtol=1e-12, atol=0) for hh in h)
            print(f"{method} tol=1e-8: block solve {ref.numsteps} steps, ranks {[int(n[0]) for n in nm]}; "
                  f"histories within 1e-12 {close}", flush=True)
            ok = ok and steps and close
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "worker":
        worker(int(sys.argv[2]), sys.argv[3], sys.argv[4])
    else:
        main()
