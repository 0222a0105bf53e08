"""ctypes binding of ``libkrylov_hip.so`` (declared in ``include/krylov_hip.h``).

The shared library is the only compute path of this package. If it is missing
the import fails loudly; there is no CPU fallback.
"""
import atexit
import ctypes
import os
import threading
import weakref

import numpy as np

from .errors import exception_for

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkrylov_hip.so")
# KRYLOV_LIB: load another build of the C-ABI instead, e.g. the host-only
# sanitizer builds of the image builders (make -C krylov_amd/csrc sanitize;
# tests/test_host_sanitize.py). Whether the loaded build is host-only is
# decided by probing it for the device entry points (HOST_ONLY below), not by
# the variable: another full GPU build loaded this way binds every entry point
# and keeps the ordered teardown.
if os.environ.get("KRYLOV_LIB"):
    LIB_PATH = os.environ["KRYLOV_LIB"]

KRY_F32, KRY_F64 = 1, 2
KRY_I32, KRY_I64 = 1, 2

KRY_OK = 0
KRY_EINVAL = -1
KRY_ENOMEM = -2
KRY_EDEVICE = -3
KRY_EINVARIANT = -4
KRY_EUNSUPPORTED = -5
KRY_ESINGULAR = -6
KRY_ENONFINITE = -7
KRY_ECOMM = -8

PROF_SPMV, PROF_UPDATE, PROF_MGS, PROF_OTHER = 0, 1, 2, 3

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
        "or `make -C krylov_amd/csrc` (hipcc, gfx950). krylov_amd has no CPU fallback."
    )

lib = ctypes.CDLL(LIB_PATH)
# a build without the device entry points (the host-only sanitizer builds)
HOST_ONLY = not hasattr(lib, "kry_ctx_create")

_vp = ctypes.c_void_p
_pvp = ctypes.POINTER(ctypes.c_void_p)
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_int = ctypes.c_int
_dp = ctypes.POINTER(ctypes.c_double)
_ip32 = ctypes.POINTER(ctypes.c_int32)
_ip64 = ctypes.POINTER(ctypes.c_int64)

# name: argtypes (all return int status except kry_version / kry_last_error)
_SIGNATURES = {
    "kry_device_count": [ctypes.POINTER(_int)],
    "kry_ctx_create": [_int, _pvp],
    "kry_ctx_destroy": [_vp],
    "kry_ctx_synchronize": [_vp],
    "kry_csr_create": [_vp, _i64, _i64, _vp, _vp, _vp, _int, _int, _pvp],
    "kry_csr_destroy": [_vp],
    "kry_csr_create_like": [_vp, _vp, _i64, _i64, _vp, _vp, _vp, _int, _int, _pvp],
    "kry_csr_permute": [_vp, _vp, _vp, _vp, _int],
    "kry_csr_compare": [_vp, _vp, _ip64],
    "kry_spmv_op": [_vp, _vp, _vp, _vp],
    "kry_rcm_plan": [ctypes.c_int64, ctypes.c_int64, _vp, _vp, _int, ctypes.c_int64, _ip64, _vp],
    "kry_rs_plan": [ctypes.c_int64, ctypes.c_int64, _vp, _vp, _int, _ip64, _vp, _vp],
    "kry_rcm_device": [_vp, ctypes.c_int64, ctypes.c_int64, _vp, _vp, ctypes.c_int64, _ip64, _vp],
    "kry_csr_layout": [_i64, _vp, _int, _ip64, _ip64, _ip64],
    "kry_dia_plan": [ctypes.c_int64, ctypes.c_int64, _vp, _vp, _int, _ip64, _vp, _vp, _vp],
    "kry_pair_plan": [ctypes.c_int64, ctypes.c_int64, _vp, _vp, _int, _ip64, _vp, _vp, _vp],
    "kry_cb_plan": [ctypes.c_int64, ctypes.c_int64, _vp, _vp, _int, _ip64, _vp],
    "kry_csr_info": [_vp, _ip64],
    "kry_csr_info_n": [_vp, _ip64, _i32],
    "kry_vec_create": [_vp, _i64, _i32, _int, _pvp],
    "kry_vec_destroy": [_vp],
    "kry_vec_upload": [_vp, _vp],
    "kry_vec_download": [_vp, _vp],
    "kry_spmv": [_vp, _vp, _vp, _vp],
    "kry_dot": [_vp, _vp, _vp, _vp, _dp],
    "kry_axpy": [_vp, _dp, _vp, _vp],
    "kry_lartg": [_vp, _i64, _int, _vp, _vp, _vp, _vp, _vp],
    "kry_cg_create": [_vp, _vp, _i32, _int, _pvp],
    "kry_cg_destroy": [_vp],
    "kry_cg_start": [_vp, _vp, _vp, _vp, _dp],
    "kry_cg_set_criterion": [_vp, _dp],
    "kry_cg_run": [_vp, _i32, _ip32, _dp],
    "kry_cg_preferred_chunk": [_vp, _ip32],
    "kry_cg_path": [_vp, _ip32],
    "kry_cg_update_path": [_vp, _ip32],
    "kry_cg_defer_info": [_vp, _ip32, _ip64],
    "kry_minres_update_path": [_vp, _ip32],
    "kry_cg_residual": [_vp, _dp],
    "kry_cg_get": [_vp, _int, _vp],
    "kry_cg_scalars": [_vp, _dp],
    "kry_vec_lincomb": [_vp, _int, _vp, _vp, _vp, _vp, _dp, _dp],
    "kry_cg_set_preconditioners": [_vp, _vp, _vp],
    "kry_gmres_set_preconditioners": [_vp, _vp, _vp, _vp],
    "kry_minres_set_preconditioners": [_vp, _vp, _vp, _vp],
    "kry_gmres_create": [_vp, _vp, _i32, _int, _i32, _i32, _pvp],
    "kry_gmres_destroy": [_vp],
    "kry_gmres_start": [_vp, _vp, _vp, _vp, _dp],
    "kry_gmres_set_criterion": [_vp, _dp],
    "kry_gmres_run": [_vp, _i32, _ip32, _dp, _ip32],
    "kry_trsv_upper": [_vp, _i32, _i32, ctypes.c_int, _dp, _dp, _dp],
    "kry_householder": [_vp, _vp, _vp, _dp],
    "kry_gmres_solution": [_vp],
    "kry_gmres_residual": [_vp, _dp],
    "kry_gmres_get": [_vp, _int, _vp],
    "kry_gmres_xk_device": [_vp, _vp],
    "kry_gmres_path": [_vp, _ip32],
    "kry_minres_create": [_vp, _vp, _i32, _int, _pvp],
    "kry_minres_destroy": [_vp],
    "kry_minres_start": [_vp, _vp, _vp, _vp, _dp],
    "kry_minres_set_criterion": [_vp, _dp],
    "kry_minres_run": [_vp, _i32, _ip32, _dp, _ip32],
    "kry_minres_residual": [_vp, _dp],
    "kry_minres_get": [_vp, _int, _vp],
    "kry_comm_unique_id": [_vp],
    "kry_comm_create": [_vp, _i32, _i32, _vp, _pvp],
    "kry_comm_destroy": [_vp],
    "kry_comm_abort": [_vp],
    "kry_comm_create_all": [_vp, _i32, _vp],
    "kry_comm_allreduce": [_vp, _dp, _i32],
    "kry_comm_info": [_vp, _vp, _vp],
    "kry_cg_attach_comm": [_vp, _vp, _i32, _i32],
    "kry_gmres_attach_comm": [_vp, _vp, _i32, _i32],
    "kry_minres_attach_comm": [_vp, _vp, _i32, _i32],
    "kry_timer_start": [_vp],
    "kry_timer_stop": [_vp, _dp],
    "kry_profile_enable": [_vp, _int],
    "kry_profile_select": [_vp, ctypes.c_uint32, ctypes.c_int32],
    "kry_profile_read": [_vp, _int, _ip64, _dp],
    "kry_prog_create": [_vp, _i32, _i32, _i32, _pvp],
    "kry_prog_destroy": [_vp],
    "kry_prog_set": [_vp, _i32, _dp],
    "kry_prog_get": [_vp, _i32, _dp],
    "kry_prog_begin": [_vp],
    "kry_prog_end": [_vp, _i32, _ip32, _ip32, _dp],
    "kry_prog_scalar": [_vp, _i32, _i32, _i32, _i32, _i32, _i32, ctypes.c_double, _i32],
    "kry_prog_dot": [_vp, _vp, _vp, _vp, _i32, _i32],
    "kry_prog_lincomb": [_vp, _i32, _vp, _vp, _vp, _vp, _i32, ctypes.c_double, _i32, ctypes.c_double, _i32],
    "kry_prog_spmv": [_vp, _vp, _vp, _vp, _i32],
    "kry_prog_check": [_vp, _i32, _i32, _i32],
    "kry_mem_stats": [_ip64],
    "kry_mem_release": [],
}

for _name, _args in _SIGNATURES.items():
    try:
        _f = getattr(lib, _name)
    except AttributeError:
        if HOST_ONLY:
            continue
        raise
    _f.argtypes = _args
    _f.restype = _int
if not HOST_ONLY:
    lib.kry_version.argtypes = []
    lib.kry_version.restype = _int
    lib.kry_build_id.argtypes = []
    lib.kry_build_id.restype = ctypes.c_char_p
lib.kry_last_error.argtypes = []
lib.kry_last_error.restype = ctypes.c_char_p

EXPORTED = sorted(list(_SIGNATURES) + ["kry_version", "kry_last_error", "kry_build_id"])


def build_id():
    """The loaded library's build stamp (kry_build_id: sha256 of its
    sources, 16 hex digits), or None for the host-only build."""
    if HOST_ONLY:
        return None
    return lib.kry_build_id().decode()


def check(rc):
    """Raise the exception the reference would raise for a C-ABI status."""
    if rc == KRY_OK:
        return
    raise exception_for(rc, (lib.kry_last_error() or b"").decode(errors="replace"))


def dtype_code(dt):
    dt = np.dtype(dt)
    if dt == np.float64:
        return KRY_F64
    if dt == np.float32:
        return KRY_F32
    raise TypeError(f"the MI355X path computes in float32/float64, not {dt}")


def itype_code(dt):
    dt = np.dtype(dt)
    if dt == np.int32:
        return KRY_I32
    if dt == np.int64:
        return KRY_I64
    raise TypeError(f"CSR index arrays must be int32 or int64, not {dt}")


def ptr(a):
    """Data pointer of a C-contiguous numpy array (as a c_void_p)."""
    assert a.flags.c_contiguous
    return ctypes.c_void_p(a.ctypes.data)


def dptr(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def device_count():
    c = _int(0)
    check(lib.kry_device_count(ctypes.byref(c)))
    return c.value


def memory_stats():
    """The caching device allocator's counters (kry_mem_stats)."""
    out = np.zeros(6, dtype=np.int64)
    check(lib.kry_mem_stats(out.ctypes.data_as(_ip64)))
    keys = ("bytes_in_use", "bytes_cached", "reuses", "device_mallocs", "retire_syncs", "enabled")
    return {k: int(v) for k, v in zip(keys, out)}


def empty_cache():
    """Return every cached (freed) device block to the runtime (kry_mem_release)."""
    check(lib.kry_mem_release())


def dia_plan(indptr, indices):
    """Host-only diagonal-offset plan (kry_dia_plan): None if the image would
    not be built, else {"slices", "slots", "max_width", "widths", "offsets",
    "masks"}."""
    indptr = np.ascontiguousarray(indptr)
    indices = np.ascontiguousarray(indices, dtype=indptr.dtype)
    n, nnz = indptr.shape[0] - 1, indices.shape[0]
    info = np.zeros(4, dtype=np.int64)
    ip64 = info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    check(lib.kry_dia_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), ip64, None, None, None))
    if not info[0]:
        return None
    cols = int(info[2]) // 128
    widths = np.zeros(int(info[1]), dtype=np.int32)
    offsets = np.zeros(cols, dtype=np.int32)
    masks = np.zeros(2 * cols, dtype=np.uint64)
    check(lib.kry_dia_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), ip64, ptr(widths),
                           ptr(offsets), ptr(masks)))
    return {"slices": int(info[1]), "slots": int(info[2]), "max_width": int(info[3]), "widths": widths,
            "offsets": offsets, "masks": masks}


def pair_plan(indptr, indices):
    """Host-only paired-row SELL-128 plan (kry_pair_plan): None if the image
    would not be built, else {"slices", "slots", "max_width", "widths",
    "cbase", "deltas"}."""
    indptr = np.ascontiguousarray(indptr)
    indices = np.ascontiguousarray(indices, dtype=indptr.dtype)
    n, nnz = indptr.shape[0] - 1, indices.shape[0]
    info = np.zeros(4, dtype=np.int64)
    ip64 = info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    check(lib.kry_pair_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), ip64, None, None, None))
    if not info[0]:
        return None
    slots = int(info[2])
    widths = np.zeros(int(info[1]), dtype=np.int32)
    cbase = np.zeros(slots // 128, dtype=np.int32)
    deltas = np.zeros(slots, dtype=np.uint16)
    check(lib.kry_pair_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), ip64, ptr(widths),
                            ptr(cbase), ptr(deltas)))
    return {"slices": int(info[1]), "slots": slots, "max_width": int(info[3]), "widths": widths, "cbase": cbase,
            "deltas": deltas}


def cb_plan(indptr, indices):
    """Host-only column-blocked plan (kry_cb_plan): None if the image would
    not be built, else {"nb", "cols", "ng", "gptr"}."""
    indptr = np.ascontiguousarray(indptr)
    indices = np.ascontiguousarray(indices, dtype=indptr.dtype)
    n, nnz = indptr.shape[0] - 1, indices.shape[0]
    info = np.zeros(4, dtype=np.int64)
    ip64 = info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    check(lib.kry_cb_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), ip64, None))
    if not info[0]:
        return None
    nb, ng = int(info[1]), int(info[3])
    gptr = np.zeros(nb * ng + 1, dtype=np.int64)
    check(lib.kry_cb_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), ip64, ptr(gptr)))
    return {"nb": nb, "cols": int(info[2]), "ng": ng, "gptr": gptr}


def rcm_plan(indptr, indices, wlimit=0):
    """Host-only reverse Cuthill-McKee order (kry_rcm_plan): None if refused
    (a BFS level wider than wlimit), else (perm, levels) with new row r = old
    row perm[r]."""
    indptr = np.ascontiguousarray(indptr)
    indices = np.ascontiguousarray(indices, dtype=indptr.dtype)
    n, nnz = indptr.shape[0] - 1, indices.shape[0]
    info = np.zeros(2, dtype=np.int64)
    perm = np.zeros(max(n, 1), dtype=np.int32)
    check(lib.kry_rcm_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), int(wlimit),
                           info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ptr(perm)))
    if not info[0]:
        return None
    return perm[:n], int(info[1])


def rs_plan(indptr, indices):
    """Host-only rank-sorted SELL-128 plan (kry_rs_plan): None if not built,
    else {"slices", "slots", "max_width", "widths", "colrank"}."""
    indptr = np.ascontiguousarray(indptr)
    indices = np.ascontiguousarray(indices, dtype=indptr.dtype)
    n, nnz = indptr.shape[0] - 1, indices.shape[0]
    info = np.zeros(4, dtype=np.int64)
    ip64 = info.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    check(lib.kry_rs_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), ip64, None, None))
    if not info[0]:
        return None
    widths = np.zeros(int(info[1]), dtype=np.int32)
    colrank = np.zeros(int(info[2]), dtype=np.uint32)
    check(lib.kry_rs_plan(n, nnz, ptr(indptr), ptr(indices), itype_code(indptr.dtype), ip64, ptr(widths),
                          ptr(colrank)))
    return {"slices": int(info[1]), "slots": int(info[2]), "max_width": int(info[3]), "widths": widths,
            "colrank": colrank}


def csr_layout(indptr):
    """SELL-64 plan of a CSR row pointer: (nslices, nslots, nirregular)."""
    indptr = np.ascontiguousarray(indptr)
    ns, slots, irr = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    check(lib.kry_csr_layout(indptr.shape[0] - 1, ptr(indptr), itype_code(indptr.dtype), ctypes.byref(ns),
                             ctypes.byref(slots), ctypes.byref(irr)))
    return ns.value, slots.value, irr.value


# ------------------------------------------------------------- teardown
# Every C-ABI handle a Python object owns is released by a weakref.finalize
# created through `own` and marked not to run from weakref's exit hook. At
# interpreter exit `_shutdown` (an atexit hook registered when this module
# loads) releases them in a fixed order while the HIP runtime is still up:
# wait for
# every context's stream, destroy solvers / operators / vectors /
# communicators (newest first), return the allocator's cached blocks to the
# runtime (kry_mem_release), then destroy the contexts. Nothing is left for
# static destructors or a profiler's exit hooks to race with.
_owned = []
_owned_lock = threading.Lock()


def own(obj, destroy, handle, context=False):
    """weakref.finalize(obj, destroy, handle), released in order at exit."""
    fin = weakref.finalize(obj, destroy, handle)
    fin.atexit = False  # _shutdown runs it, in order
    with _owned_lock:
        _owned.append((fin, context))
        if len(_owned) > 4096:  # drop finalizers that already ran
            _owned[:] = [(f, c) for f, c in _owned if f.alive]
    return fin


def _release(fin):
    """Run a finalizer and close its owner: every attribute of the owner that
    holds the released handle becomes None, so a later call through a live
    object (a hook that runs after this one, a daemon thread) passes NULL and
    the library refuses it (KRY_EINVAL, "null argument") instead of touching
    freed memory."""
    info = fin.peek()  # (owner, func, args, kwargs), None once it ran
    fin()
    if info is None:
        return
    owner, handle = info[0], info[2][0]
    for name, val in list(getattr(owner, "__dict__", {}).items()):
        if val is handle:
            setattr(owner, name, None)


def _shutdown():
    if HOST_ONLY:  # a host-only build owns no device objects
        return
    with _owned_lock:
        owned = list(_owned)
        _owned.clear()
    ctxs = [f for f, c in owned if c and f.alive]
    for f in ctxs:  # drain every stream before anything is freed
        info = f.peek()  # (obj, func, args, kwargs)
        if info is not None:
            lib.kry_ctx_synchronize(info[2][0])
    for f, c in reversed(owned):
        if not c:
            _release(f)
    lib.kry_mem_release()
    for f in reversed(ctxs):
        _release(f)
    maps = os.environ.get("KRY_EXIT_MAPS")  # diagnostics: the address map at exit (archive:gpu_exit_bisect.sh)
    if maps:
        with open("/proc/self/maps") as src, open(maps, "w") as dst:
            dst.write(src.read())


atexit.register(_shutdown)
