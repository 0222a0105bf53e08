"""Preconditioned GMRES driver (reference ``gmres.py:41-251``) over the device
loop: Arnoldi with modified Gram-Schmidt (``ortho="mgs"`` / ``"mgsK"``,
arnoldi.py:107-200), the Givens QR update of the Hessenberg matrix, and the
solution ``x0 + V R^-1 y`` all run on the GPU (``kry_gmres_*``).

Like the reference there is no restart parameter: ``maxiter`` bounds the
Arnoldi basis, and restarted GMRES(m) is ``gmres(..., maxiter=m)`` chained
through ``x0`` (see ``gmres_restarted``).
"""
import ctypes

import numpy as np

from . import _helpers, _lib
from ._helpers import Info, Problem
from .device import HostOut
from ._lib import check, lib


def multi_solve_triangular(A, B, device=None):
    """``multi_solve_triangular`` (reference ``gmres.py:24-38``) on the GPU:
    for every trailing column c, solve the upper-triangular ``A[:, :, c] y =
    B[:, c]`` (``kry_trsv_upper``). All-zero right-hand sides give zeros;
    non-finite input raises ``ValueError`` and a zero diagonal
    ``numpy.linalg.LinAlgError``, as ``scipy.linalg.solve_triangular`` does."""
    from .device import get_context

    A = np.asarray(A)
    B = np.asarray(B)
    m = A.shape[0]
    a = A.reshape(A.shape[0], A.shape[1], -1)
    b = B.reshape(B.shape[0], -1)
    if a.shape[0] != a.shape[1] or b.shape[0] != m or b.shape[1] != a.shape[2]:
        raise ValueError(f"shapes {A.shape} and {B.shape} do not match")
    if np.iscomplexobj(a) or np.iscomplexobj(b):
        raise TypeError("complex systems are outside the MI355X path")
    k = a.shape[2]
    dt = np.result_type(a.dtype, b.dtype, np.float32)
    work = np.float32 if dt == np.float32 else np.float64
    out = np.empty((m, k))
    if m > 0 and k > 0:
        ctx = get_context(device)
        check(lib.kry_trsv_upper(ctx.handle, m, k, _lib.dtype_code(work),
                                 _lib.dptr(np.ascontiguousarray(a, dtype=np.float64)),
                                 _lib.dptr(np.ascontiguousarray(b, dtype=np.float64)), _lib.dptr(out)))
    # the reference stacks per-column results: float32 solves next to float64
    # zero columns promote to float64
    zero_cols = np.all(b == 0.0, axis=0)
    res_dt = work if (work == np.float64 or not zero_cols.any()) else np.float64
    return out.astype(res_dt).reshape([A.shape[0]] + list(A.shape[2:]))


class _GmresState:
    def __init__(self, prob, maxiter, sweeps):
        self.prob = prob
        h = ctypes.c_void_p()
        check(lib.kry_gmres_create(prob.ctx.handle, prob.A.handle, prob.kpad, _lib.dtype_code(prob.dtype),
                                   int(maxiter), int(sweeps), ctypes.byref(h)))
        self.h = h
        self._fin = _lib.own(self, lib.kry_gmres_destroy, h)
        if prob.has_precond():
            check(lib.kry_gmres_set_preconditioners(h, *prob.op_handles("M", "Ml", "Mr")))

    def start(self, x0_dev=None):
        """r0 = b - A x0 on the device; x0 = the problem's own x0 or, for a
        restart chain, ``x0_dev`` (a DeviceVector of the solve's shape)."""
        p = self.prob
        out = np.zeros(p.kpad)
        x0 = x0_dev if x0_dev is not None else p.x0_dev
        check(lib.kry_gmres_start(self.h, p.b_dev.handle, x0.handle if x0 is not None else None,
                                  p.w_dev.handle if p.w_dev else None, _lib.dptr(out)))
        return out

    def set_criterion(self, crit):
        crit = np.ascontiguousarray(crit, dtype=np.float64)
        check(lib.kry_gmres_set_criterion(self.h, _lib.dptr(crit)))

    def run(self, steps):
        out = np.zeros((max(steps, 1), self.prob.kpad))
        done = ctypes.c_int32()
        inv = ctypes.c_int32()
        check(lib.kry_gmres_run(self.h, int(steps), ctypes.byref(done), _lib.dptr(out), ctypes.byref(inv)))
        return out[: done.value], bool(inv.value)

    def solution(self):
        check(lib.kry_gmres_solution(self.h))

    def path(self):
        """(persistent, fallbacks): whether Arnoldi steps run their MGS as one
        persistent launch, and how many chunks finished launch per pass after a
        persistent MGS exchange timed out (kry_gmres_path)."""
        info = (ctypes.c_int32 * 2)()
        check(lib.kry_gmres_path(self.h, info))
        return bool(info[0]), int(info[1])

    def residual_norm2(self):
        out = np.zeros(self.prob.kpad)
        check(lib.kry_gmres_residual(self.h, _lib.dptr(out)))
        return out

    def xk_into(self, vec):
        """xk (after solution()) into a DeviceVector, device to device."""
        check(lib.kry_gmres_xk_device(self.h, vec.handle))

    def xk(self, out=None):
        p = self.prob
        if out is None:
            out = np.empty((p.n, p.kpad), dtype=p.dtype)
        assert out.shape == (p.n, p.kpad) and out.dtype == p.dtype and out.flags.c_contiguous
        check(lib.kry_gmres_get(self.h, 0, _lib.ptr(out)))
        return p.unpad_vec(out, p.r0_dtype)


def arnoldi(A, v, maxiter, ortho="mgs", M=None, inner=None):
    """The device Arnoldi process of ``gmres`` run on its own: ``ArnoldiMGS``
    (``arnoldi.py:107-200``, ``ortho="mgs"`` / ``"mgsK"``) or
    ``ArnoldiHouseholder`` (``arnoldi.py:33-104``) from the start vector ``v``
    for up to ``maxiter`` steps, stopping early at an invariant subspace like
    the reference's ``while arnoldi.iter < maxiter and not
    arnoldi.is_invariant`` loop (tests/test_arnoldi.py).

    Returns ``(V, H, P, is_invariant)``: the basis as a list of vectors
    (``V = M P``), the (steps + 1) x steps Hessenberg matrix (steps x steps
    after an invariant step), and the ``P`` basis (``P is V`` without M)."""
    if ortho.startswith("mgs"):
        sweeps = 1 if len(ortho) == 3 else int(ortho[3:])
    elif ortho == "householder":
        assert inner is None and _helpers._is_identity(M)
        sweeps = 0
    else:
        raise ValueError(f"unknown ortho {ortho!r}")
    v = np.asarray(v)
    if v.ndim != 1:
        raise ValueError("arnoldi takes one start vector")
    prob = Problem(A, v, None, inner, M=M)
    st = _GmresState(prob, maxiter, sweeps)
    st.start()
    st.set_criterion(prob.pad_cols(np.full(prob.kc, -1.0), np.inf))  # never "converged"
    steps = 0
    invariant = False
    while steps < maxiter and not invariant:
        hist, invariant = st.run(min(_helpers.CHUNK, maxiter - steps))
        steps += len(hist)
        if len(hist) == 0:
            break
    nv = steps + (0 if invariant else 1)
    n, kp = prob.n, prob.kpad

    def basis(which):
        out = np.empty((max(nv, 1), n, kp), dtype=prob.dtype)
        check(lib.kry_gmres_get(st.h, which, _lib.ptr(out)))
        return [out[i, :, 0].copy() for i in range(nv)]

    V = basis(1)
    P = basis(2) if (not _helpers._is_identity(M) and sweeps > 0) else V
    mi = max(maxiter, 1)
    Hs = np.empty((maxiter + 1, mi, kp))
    check(lib.kry_gmres_get(st.h, 3, _lib.ptr(Hs)))
    H = Hs[: steps + 1, :steps, 0].astype(prob.dtype)
    if invariant:
        H = H[:steps]
    return V, H, P, invariant


def gmres(A, b, M=None, Ml=None, Mr=None, inner=None, ortho="mgs", x0=None, tol=1e-5, atol=1.0e-15,
          maxiter=None, callback=None, *, devices=None):
    """Preconditioned GMRES, reference signature (``gmres.py:41-54``).

    ``ortho``: "mgs", "mgsK" (K MGS sweeps) or "householder" (Householder
    Arnoldi, arnoldi.py:33-104, one right-hand side, default inner, no M)."""
    if devices is not None:  # several GPUs of this process (krylov_amd.multi)
        from .multi import solve

        return solve("gmres", A, b, devices, x0=x0, tol=tol, atol=atol, maxiter=maxiter, ortho=ortho,
                     callback=callback, M=M, Ml=Ml, Mr=Mr, inner=inner)
    sweeps = _sweeps(ortho, inner, M, b)
    prob = Problem(A, b, x0, inner, M=M, Ml=Ml, Mr=Mr)
    maxiter = prob.A.shape[0] if maxiter is None else maxiter
    st = _GmresState(prob, maxiter, sweeps)
    host_out = HostOut((prob.n, prob.kpad), prob.dtype)  # pages faulted in while the device iterates
    success, xk, k, resnorms = _cycle(prob, st, maxiter, tol, atol, callback, host_out=host_out)
    return xk if success else None, Info(success, xk, k, resnorms, num_operations=_num_operations(k), renumbered=prob.A.renumbered)


def _sweeps(ortho, inner, M, b):
    if ortho.startswith("mgs"):
        return 1 if len(ortho) == 3 else int(ortho[3:])
    if ortho == "householder":
        # gmres.py:158-161 and householder.py:19-22: Euclidean inner product,
        # no M, one (quasi-1-D) right-hand side
        assert inner is None, "ortho='householder' needs the default inner product"
        assert _helpers._is_identity(M), "ortho='householder' does not take M"
        bs = np.shape(b)
        assert len(bs) == 1 or (len(bs) == 2 and bs[1] == 1), (
            "Householder only works for quasi-1D vectors for now. " f"Input vector has shape {bs}."
        )
        return 0
    raise ValueError(f"unknown ortho {ortho!r}")


def _num_operations(k):
    return {
        "A": 1 + k,
        "M": 2 + k,
        "Ml": 2 + k,
        "Mr": 1 + k,
        "inner": 2 + k + k * (k + 1) / 2,
        "axpy": 4 + 2 * k + k * (k + 1) / 2,
    }


def _cycle(prob, st, maxiter, tol, atol, callback, tol_of_r0=None, x_in=None, x_out=None, host_x=True,
           host_out=None):
    """One ``gmres`` call's loop (gmres.py:150-251) on the device state ``st``.

    ``tol_of_r0`` (restarts) maps the device's initial residual norm
    ``||Ml (b - A x0)||`` to this call's ``tol``, so the norm is read once.
    Restarts keep the iterate on the device: ``x_in`` (a DeviceVector) is x0
    instead of the problem's own, ``x_out`` receives xk device to device (it
    may be ``x_in``), and the host copy of xk is made only if ``host_x`` (else
    the returned xk is None), into ``host_out`` (a ``HostOut``) when given.
    Returns ``(success, xk, numsteps, resnorms)``."""
    rn0 = st.start(x_in)
    resnorms = [prob.colvals(rn0)]

    def host_x0():
        if x_in is None:
            return prob.x0_or_zeros()  # _get_xk(None) / k == 0 returns x0 itself (gmres.py:89-99)
        return prob.unpad_vec(x_in.to_host(), prob.r0_dtype)

    if callback is not None:
        # the reference passes Ml_r0 = Ml (b - A x0) here (gmres.py:143-144)
        x0h = host_x0()
        callback(x0h, prob.apply_host("Ml", prob.b - prob.A @ x0h))
    if tol_of_r0 is not None:
        tol = tol_of_r0(resnorms[0])
    criterion = np.maximum(tol * resnorms[0], atol)
    st.set_criterion(prob.pad_cols(criterion, np.inf))

    steps_done = 0
    solved = False  # st holds x0 + V R^-1 y of the steps done so far
    k = 0
    success = False

    def solve():
        nonlocal solved
        if not solved:
            st.solution()
            solved = True

    while True:
        if np.all(resnorms[-1] <= criterion):
            solve()  # with no step done this is x0 (the explicit residual's input)
            resnorms[-1] = prob.colvals(np.sqrt(np.asarray(st.residual_norm2()[: prob.kc]).astype(prob.inner_dtype)))
            if np.all(resnorms[-1] <= criterion):
                success = True
                break
        if k == maxiter:
            break
        steps = 1 if callback is not None else min(_helpers.CHUNK, maxiter - k)
        hist, _ = st.run(steps)
        solved = False
        for row in hist:
            resnorms.append(prob.colvals(row))
            k += 1
            steps_done += 1
        if callback is not None and len(hist):
            solve()
            callback(st.xk(), np.array(resnorms[-1]))

    if x_out is not None:
        solve()
        st.xk_into(x_out)
    if steps_done == 0:
        xk = host_x0() if host_x else None
    else:
        solve()
        xk = st.xk(out=host_out.take() if host_out is not None else None) if host_x else None
    return success, xk, k, resnorms


def gmres_restarted(A, b, restart=30, x0=None, tol=1e-5, atol=1.0e-15, max_cycles=100, ortho="mgs", *, M=None,
                    Ml=None, Mr=None, inner=None, callback=None):
    """Restarted GMRES(restart): the reference's ``gmres`` (``gmres.py:41-54``,
    no restart parameter of its own) chained through ``x0``, one call of
    ``maxiter=restart`` per cycle, exactly as the reference's restart fixture
    drives it (tests/golden/make_golden.py, ``gmres_restart_*``):

        cycle c:  gmres(A, b, x0=x_c, maxiter=restart,
                        tol=tol * ||b|| / max(||b - A x_c||, 1e-300), atol=atol)
                  x_{c+1} = info.xk; stop after the first cycle with success

    so every cycle's criterion is ``tol * ||b||`` (relative to b, not to the
    cycle's start: a different ``tol`` meaning from ``gmres``'s) and the run
    stops when ``||b - A x|| <= tol ||b||``. ``||b - A x_c||`` is the device's
    own initial residual norm of the cycle (the norm of the Euclidean or
    ``WeightedInner`` inner product; with Ml, of ``Ml (b - A x_c)``), and
    ``||b||`` is taken in the same norm (with Ml: ``||Ml b||``), so the
    criterion compares like with like. The preconditioned chains (M, Ml, Mr)
    are parity unpinned: the reference's fixtures chain unpreconditioned
    cycles only (the oracle chaining of tests/test_gpu_solvers.py covers Mr).

    The chain stays on the device: the operator, b and the solver state are
    set up once, each cycle starts from the previous cycle's iterate in device
    memory and leaves its own there, so a cycle moves no vector over PCIe; the
    final iterate is downloaded once. M, Ml, Mr and inner are keyword-only.

    Returns ``(x, infos)``: the last iterate and one ``Info`` per cycle (the
    last cycle's ``xk`` is x; earlier cycles' iterates stay on the device, their
    ``xk`` is None); the chained history is ``sum(info.resnorms for info in
    infos)``.
    """
    from .device import DeviceVector
    from .sparse import as_device_operator

    sweeps = _sweeps(ortho, inner, M, b)
    Aop = as_device_operator(A)
    b = np.asarray(b)
    prob = Problem(Aop, b, x0, inner, M=M, Ml=Ml, Mr=Mr)
    if max_cycles <= 0:  # no cycle: the iterate is x0 (zeros_like(b) without one), as the reference's start
        return (np.array(x0, dtype=prob.r0_dtype, copy=True) if x0 is not None
                else np.zeros(b.shape, dtype=prob.r0_dtype)), []
    # ||b|| (with Ml: ||Ml b||) in the solve's inner product, on the device:
    # the same two-stage reduction as the cycles' ||Ml (b - A x_c)|| (a host
    # norm of an 80 MB b took ~5 ms per call at the metric size)
    bv = prob.b_dev
    if prob.ops["Ml"] is not None:
        bv = DeviceVector(prob.ctx, prob.n, prob.kpad, prob.dtype)
        prob.ops["Ml"].matvec_device(prob.b_dev, bv)
    sq = np.zeros(prob.kpad)
    check(lib.kry_dot(prob.ctx.handle, bv.handle, bv.handle, prob.w_dev.handle if prob.w_dev else None,
                      _lib.dptr(sq)))
    bnorm = prob.colvals(np.sqrt(sq[: prob.kc].astype(prob.inner_dtype)))

    def tol_of_r0(r0):
        return tol * bnorm / np.maximum(r0, 1e-300)

    st = _GmresState(prob, restart, sweeps)
    x_buf = DeviceVector(prob.ctx, prob.n, prob.kpad, prob.dtype)
    host_out = HostOut((prob.n, prob.kpad), prob.dtype)  # the final x's pages, faulted in during the cycles
    x_cur = prob.x0_dev  # None: x0 = 0 on the device, nothing uploaded
    infos = []
    x = None
    for c in range(max_cycles):
        last = c == max_cycles - 1
        success, xk, k, resnorms = _cycle(prob, st, restart, tol, atol, callback, tol_of_r0=tol_of_r0,
                                          x_in=x_cur, x_out=x_buf, host_x=last, host_out=host_out)
        x_cur = x_buf
        if success and xk is None:
            xk = prob.unpad_vec(x_buf.to_host(out=host_out.take()), prob.r0_dtype)
        infos.append(Info(success, xk, k, resnorms, num_operations=_num_operations(k), renumbered=prob.A.renumbered))
        x = xk
        if success:
            break
    return x, infos
