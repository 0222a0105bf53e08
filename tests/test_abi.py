"""The C-ABI library loads, exports every symbol include/krylov_hip.h declares,
and its host-only logic (SELL-64 layout plan, error mapping) is right. CPU only:
no kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest
import scipy.sparse

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _declared_symbols():
    with open(os.path.join(REPO, "include", "krylov_hip.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kry_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from krylov_amd import _lib

    declared = _declared_symbols()
    assert len(declared) > 30
    for name in declared:
        assert hasattr(_lib.lib, name), name
    # and the ctypes binding covers exactly the header
    assert sorted(_lib.EXPORTED) == declared


def test_library_is_gfx950_code_object():
    from krylov_amd import _lib

    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_version_and_device_count_without_gpu():
    from krylov_amd import _lib

    assert _lib.lib.kry_version() >= 101
    n = _lib.device_count()
    assert n >= 0


def test_memory_stats_without_gpu():
    import krylov_amd

    s = krylov_amd.memory_stats()
    assert set(s) == {"bytes_in_use", "bytes_cached", "reuses", "device_mallocs", "retire_syncs", "enabled"}
    assert s["bytes_in_use"] >= 0 and s["bytes_cached"] >= 0
    krylov_amd.empty_cache()  # nothing cached: a no-op, no device needed
    assert krylov_amd.memory_stats()["bytes_cached"] == 0


def test_no_device_fails_loudly():
    from krylov_amd import _lib

    if _lib.device_count() > 0:
        pytest.skip("a GPU is present")
    from krylov_amd.device import Context

    with pytest.raises(RuntimeError, match="no HIP device"):
        Context(0)


def _layout(indptr):
    from krylov_amd import _lib

    indptr = np.ascontiguousarray(indptr)
    it = _lib.KRY_I32 if indptr.dtype == np.int32 else _lib.KRY_I64
    ns, slots, irr = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    _lib.check(_lib.lib.kry_csr_layout(indptr.shape[0] - 1, _lib.ptr(indptr), it, ctypes.byref(ns),
                                        ctypes.byref(slots), ctypes.byref(irr)))
    return ns.value, slots.value, irr.value


def _layout_py(indptr):
    """Restatement of the SELL-64 plan: slices of 64 rows, width = longest
    row, irregular when 64 * width > 2 * nnz_slice + 1024."""
    n = indptr.shape[0] - 1
    ns = (n + 63) // 64
    slots = irr = 0
    for s in range(ns):
        r0, r1 = 64 * s, min(n, 64 * s + 64)
        lens = np.diff(indptr[r0:r1 + 1])
        w = int(lens.max()) if len(lens) else 0
        if 64 * w > 2 * int(indptr[r1] - indptr[r0]) + 1024:
            irr += 1
        else:
            slots += 64 * w
    return ns, slots, irr


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_sell_layout_matches_restatement(seed):
    rng = np.random.default_rng(seed)
    n = 5000
    lens = rng.integers(0, 40, n)
    lens[rng.choice(n, 5, replace=False)] = rng.integers(2049, 9000, 5)  # long rows
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    got = _layout(indptr)
    assert got == _layout_py(indptr)
    assert got[2] >= 1  # the long rows make their slices irregular
    assert _layout(indptr.astype(np.int32)) == got


def test_sell_layout_of_stencils_is_regular():
    from krylov_amd import problems

    for A in (problems.poisson2d(40), problems.stencil15_3d(12)):
        ns, slots, irr = _layout(A.indptr)
        assert irr == 0
        assert ns == (A.shape[0] + 63) // 64
        assert A.nnz <= slots <= 1.2 * A.nnz
        assert (ns, slots, irr) == _layout_py(A.indptr)


def test_error_mapping():
    from krylov_amd import _lib
    from krylov_amd.errors import ArgumentError

    with pytest.raises(ValueError):
        _lib.check(_lib.lib.kry_csr_layout(-1, None, _lib.KRY_I32, None, None, None))
    with pytest.raises(ArgumentError):
        _lib.check(_lib.KRY_EINVARIANT)
    with pytest.raises(np.linalg.LinAlgError):
        _lib.check(_lib.KRY_ESINGULAR)
    with pytest.raises(MemoryError):
        _lib.check(_lib.KRY_ENOMEM)
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.KRY_EUNSUPPORTED)


def test_weighted_inner_matches_reference_form():
    from krylov_amd import WeightedInner

    rng = np.random.default_rng(0)
    n = 50
    w = 10 / np.arange(1, n + 1)
    x, y = rng.standard_normal(n), rng.standard_normal(n)
    assert WeightedInner(w)(x, y) == np.dot(x.T, w * y)  # tests/test_solvers.py:157-161
    X, Y = rng.standard_normal((n, 3)), rng.standard_normal((n, 3))
    got = WeightedInner(w)(X, Y)
    for c in range(3):
        np.testing.assert_allclose(got[c], np.dot(X[:, c], w * Y[:, c]), rtol=1e-14)


def test_unsupported_inputs_are_rejected_before_any_device_work():
    import krylov_amd

    with pytest.raises(TypeError):
        krylov_amd.cg(np.eye(3), np.ones(3), inner=lambda x, y: np.dot(x, y))
    with pytest.raises(NotImplementedError):
        krylov_amd.cg(np.eye(3), np.ones(3), M=lambda x: x)  # host callbacks cannot run on the device
    with pytest.raises(TypeError):
        krylov_amd.cg(np.eye(3), np.ones(3, dtype=complex))
    with pytest.raises(AssertionError):  # as the reference (gmres.py:159-161)
        krylov_amd.gmres(np.eye(3), np.ones((3, 2)), ortho="householder")
    with pytest.raises(ValueError):
        krylov_amd.gmres(np.eye(3), np.ones(3), ortho="cgs")


def _dia_plan_py(indptr, indices):
    """Restatement of the SELL-128/DIA plan (kry_dia_plan): slices of 128
    rows; each slice's sorted distinct offsets col - row; a row's entries must
    be strictly increasing (so offset order is stored order); the slice is
    refused when 128 * width > 2 * nnz_slice + 2048, and the whole image when
    it holds more than 1.25x the SELL-64 slots plus one slice of padding."""
    n = indptr.shape[0] - 1
    if n == 0:
        return None
    ns = (n + 127) // 128
    widths, offs, masks = [], [], []
    maxw = 0
    for s in range(ns):
        r0, r1 = 128 * s, min(n, 128 * s + 128)
        rows = np.repeat(np.arange(r0, r1), np.diff(indptr[r0:r1 + 1]))
        cols = indptr.dtype.type(0) + indices[indptr[r0]:indptr[r1]].astype(np.int64)
        seg = np.split(cols, np.cumsum(np.diff(indptr[r0:r1 + 1]))[:-1])
        if any(np.any(np.diff(c) <= 0) for c in seg):
            return None
        o = np.unique(cols - rows)
        if 128 * len(o) > 2 * int(indptr[r1] - indptr[r0]) + 2048:
            return None
        m = np.zeros((len(o), 2), dtype=np.uint64)
        for r, c in zip(rows, cols):
            j = np.searchsorted(o, c - r)
            rl = r - r0
            m[j, rl & 1] |= np.uint64(1) << np.uint64(rl >> 1)
        widths.append(len(o))
        offs.extend(o.tolist())
        masks.extend(m.ravel().tolist())
        maxw = max(maxw, len(o))
    slots = 128 * sum(widths)
    sell_slots = _layout_py(indptr)[1]
    if slots * 4 > sell_slots * 5 + 4 * 128 * maxw:
        return None
    return {"slices": ns, "slots": slots, "max_width": maxw, "widths": np.array(widths, dtype=np.int32),
            "offsets": np.array(offs, dtype=np.int32), "masks": np.array(masks, dtype=np.uint64)}


def _banded(n, offsets, seed, drop=0.1):
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for o in offsets:
        r = np.arange(max(0, -o), min(n, n - o))
        keep = rng.random(r.size) >= drop
        rows.append(r[keep])
        cols.append(r[keep] + o)
    A = scipy.sparse.coo_matrix((np.ones(sum(x.size for x in rows)), (np.concatenate(rows), np.concatenate(cols))),
                                shape=(n, n)).tocsr()
    A.sort_indices()
    return A


@pytest.mark.parametrize("case", ["poisson2d_61", "stencil15_12", "banded_holes", "ragged_129", "one_row",
                                  "unsorted", "scattered"])
def test_dia_plan_matches_restatement(case):
    """The host side of the diagonal-offset image (offsets, lane masks,
    widths, and when it is refused) against a NumPy restatement, without a
    device (kry_dia_plan)."""
    from krylov_amd import _lib, problems

    if case == "poisson2d_61":
        A = problems.poisson2d(61)
    elif case == "stencil15_12":
        A = problems.stencil15_3d(12)
    elif case == "banded_holes":
        A = _banded(3000, [-70, -3, -1, 0, 2, 9, 70], 1, drop=0.2)
    elif case == "ragged_129":
        A = _banded(129, [-1, 0, 1], 2, drop=0.0)
    elif case == "one_row":
        A = scipy.sparse.csr_matrix(np.array([[2.0]]))
    elif case == "unsorted":
        A = problems.poisson2d(20).tocsr()
        a = A.indptr[37]
        A.indices[a], A.indices[a + 1] = A.indices[a + 1], A.indices[a]
    else:
        A = problems.random_nonsym(4000, seed=3)
    ip = A.indptr.astype(np.int32)
    ix = A.indices.astype(np.int32)
    got = _lib.dia_plan(ip, ix)
    want = _dia_plan_py(ip, ix)
    if want is None:
        assert got is None
        return
    assert got is not None
    for key in ("slices", "slots", "max_width"):
        assert got[key] == want[key], key
    for key in ("widths", "offsets", "masks"):
        np.testing.assert_array_equal(got[key], want[key])
    assert case not in ("unsorted", "scattered")


def _pair_plan_py(indptr, indices):
    """Restatement of the paired-row SELL-128 plan (kry_pair_plan): slices of
    128 rows, width = the longest row; slot column j holds every row's j-th
    stored entry (stored order, unsorted rows and duplicates as they are) as
    column - base, base = the slot column's smallest column, 0xFFFF where the
    row is shorter; refused when a slot column spans more than 65534
    columns, or when the slots exceed 1.25x the SELL-64 slots plus one slice
    of padding."""
    n = indptr.shape[0] - 1
    if n == 0 or n >= 2**31:
        return None
    ns = (n + 127) // 128
    lens = np.diff(indptr.astype(np.int64))
    widths = np.array([lens[128 * s:128 * s + 128].max() for s in range(ns)], dtype=np.int32)
    maxw = int(widths.max())
    slots = 128 * int(widths.sum())
    sell_slots = _layout_py(indptr)[1]
    if slots == 0 or slots * 4 > sell_slots * 5 + 4 * 128 * maxw:
        return None
    cbase, deltas = [], []
    for s in range(ns):
        r0, r1 = 128 * s, min(n, 128 * s + 128)
        for j in range(widths[s]):
            col = np.full(128, -1, dtype=np.int64)
            for r in range(r0, r1):
                if j < lens[r]:
                    col[r - r0] = indices[indptr[r] + j]
            have = col >= 0
            base = int(col[have].min()) if have.any() else 0
            if have.any() and int(col[have].max()) - base > 65534:
                return None
            d = np.where(have, col - base, 0xFFFF).astype(np.uint16)
            cbase.append(base)
            deltas.append(d)
    return {"slices": ns, "slots": slots, "max_width": maxw, "widths": widths,
            "cbase": np.array(cbase, dtype=np.int32), "deltas": np.concatenate(deltas)}


@pytest.mark.parametrize("case", ["banded_holes", "ragged_129", "one_row", "unsorted_dups", "wide_span",
                                  "uneven", "int64"])
def test_pair_plan_matches_restatement(case):
    """The host side of the paired-row image (widths, bases, deltas, and when
    it is refused) against a NumPy restatement, without a device
    (kry_pair_plan)."""
    from krylov_amd import _lib

    itype = np.int32
    if case == "banded_holes":
        A = _banded(3000, [-70, -3, -1, 0, 2, 9, 70], 1, drop=0.2)
    elif case == "ragged_129":
        A = _banded(129, [-1, 0, 1], 2, drop=0.0)
    elif case == "one_row":
        A = scipy.sparse.csr_matrix(np.array([[2.0]]))
    elif case == "unsorted_dups":
        rng = np.random.default_rng(5)
        n = 700
        lens = rng.integers(0, 9, n)
        ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        rows = np.repeat(np.arange(n), lens)
        ix = np.clip(rows + rng.integers(-40, 40, rows.size), 0, n - 1).astype(np.int32)
        A = scipy.sparse.csr_matrix((np.ones(ix.size), ix, ip), shape=(n, n))
    elif case == "wide_span":  # one slot column spans 65535 columns: refused
        n = 70_000
        A = scipy.sparse.csr_matrix((np.ones(2), ([0, 1], [0, 65535])), shape=(n, n))
    elif case == "uneven":  # one long row in a slice of short ones: past 1.25x, refused
        n = 512
        rows = np.concatenate([np.zeros(400, dtype=int), np.arange(1, n)])
        cols = np.concatenate([np.arange(400), np.arange(1, n)])
        A = scipy.sparse.csr_matrix((np.ones(rows.size), (rows, cols)), shape=(n, n))
    else:
        A = _banded(1000, [-5, 0, 5], 3, drop=0.1)
        itype = np.int64
    ip = A.indptr.astype(itype)
    ix = A.indices.astype(itype)
    got = _lib.pair_plan(ip, ix)
    want = _pair_plan_py(ip, ix)
    if want is None:
        assert got is None
        assert case in ("wide_span", "uneven")
        return
    assert got is not None
    for key in ("slices", "slots", "max_width"):
        assert got[key] == want[key], key
    for key in ("widths", "cbase", "deltas"):
        np.testing.assert_array_equal(got[key], want[key])


def _cb_plan_py(indptr, indices):
    """Restatement of the column-blocked plan (kry_cb_plan): int32 indices;
    x over 8 MB (n >= 2^20); columns cut into blocks of max(2^18, ceil(n / 16))
    columns (at least 2 blocks); refused unless every row is sorted and at
    least a quarter of the entries lie more than half a block from the
    diagonal; segment (block b, 256-row group g) holds the group's entries in
    block b, in row order, its start at gptr[b * ng + g]; a segment over 65535
    entries refuses the image."""
    n = indptr.shape[0] - 1
    if indptr.dtype != np.int32 or n * 8 < (8 << 20):
        return None
    cols = max(1 << 18, (n + 15) // 16)
    nb = (n + cols - 1) // cols
    if nb < 2:
        return None
    ip = indptr.astype(np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(ip))
    ix = indices.astype(np.int64)
    same_row = rows[1:] == rows[:-1]
    if np.any(same_row & (ix[1:] < ix[:-1])):
        return None
    d = ix - rows
    if ix.size == 0 or 4 * int(np.count_nonzero((d > cols // 2) | (d < -(cols // 2)))) < ix.size:
        return None
    ng = (n + 255) // 256
    cnt = np.bincount((ix // cols) * ng + rows // 256, minlength=nb * ng)
    if cnt.max() > 65535:
        return None
    gptr = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    return {"nb": nb, "cols": cols, "ng": ng, "gptr": gptr}


@pytest.mark.parametrize("case", ["scattered", "scattered_wide", "stencil", "unsorted", "small", "int64"])
def test_cb_plan_matches_restatement(case):
    """The host side of the column-blocked image (column blocks, segment
    pointers, and when it is refused) against a NumPy restatement, without a
    device (kry_cb_plan). Sizes are past the builder's threading thresholds,
    so the sanitizer runs (tests/test_host_sanitize.py) see its threads."""
    from krylov_amd import _lib, problems

    n = 1_100_000
    if case in ("scattered", "unsorted", "int64"):
        A = problems.random_nonsym(n, per_row=5, seed=4)
    elif case == "scattered_wide":
        A = problems.random_nonsym(4_500_000, per_row=3, seed=5)
    elif case == "stencil":
        A = problems.poisson2d(1100)  # columns near the diagonal: refused
    else:
        A = problems.random_nonsym(200_000, per_row=5, seed=6)  # x fits the caches: refused
    ip, ix = A.indptr.astype(np.int32), A.indices.astype(np.int32)
    if case == "unsorted":
        ix = ix.copy()
        a = ip[1234]
        ix[a], ix[a + 1] = ix[a + 1], ix[a]
    if case == "int64":
        ip, ix = ip.astype(np.int64), ix.astype(np.int64)
    got = _lib.cb_plan(ip, ix)
    want = _cb_plan_py(ip, ix)
    if want is None:
        assert got is None
        assert case in ("stencil", "unsorted", "small", "int64")
        return
    assert got is not None and case.startswith("scattered")
    for key in ("nb", "cols", "ng"):
        assert got[key] == want[key], key
    np.testing.assert_array_equal(got["gptr"], want["gptr"])


def test_plans_of_large_matrices_match():
    """The threaded paths of the plan builders (more than 2048 slices): the
    DIA plan of a 600^2 Poisson matrix against the restatement, and the
    paired plan of a banded 300k-row matrix checked entry by entry (each
    slot's base + delta is the stored column)."""
    from krylov_amd import _lib, problems

    A = problems.poisson2d(600)
    got = _lib.dia_plan(A.indptr, A.indices)
    want = _dia_plan_py(A.indptr, A.indices)
    assert got is not None and want is not None
    for key in ("slices", "slots", "max_width"):
        assert got[key] == want[key], key
    for key in ("widths", "offsets", "masks"):
        np.testing.assert_array_equal(got[key], want[key])
    B = _banded(300_000, [-700, -3, 0, 2, 9, 700], 7, drop=0.15)
    p = _lib.pair_plan(B.indptr, B.indices)
    assert p is not None
    ip = B.indptr.astype(np.int64)
    lens = np.diff(ip)
    ns = (B.shape[0] + 127) // 128
    np.testing.assert_array_equal(p["widths"], [lens[128 * s:128 * s + 128].max() for s in range(ns)])
    sptr = np.concatenate([[0], 128 * np.cumsum(p["widths"].astype(np.int64))])
    rows = np.repeat(np.arange(B.shape[0]), lens)
    j = np.arange(B.nnz) - ip[rows]  # position in the row
    slot = sptr[rows // 128] + 128 * j + rows % 128
    np.testing.assert_array_equal(p["cbase"][slot // 128].astype(np.int64) + p["deltas"][slot], B.indices)
    assert np.count_nonzero(p["deltas"] != 0xFFFF) == B.nnz


@pytest.mark.parametrize("defect", ["nnz_short", "nnz_long", "indptr_start", "indptr_decreasing", "col_negative",
                                    "col_too_large"])
@pytest.mark.parametrize("plan", ["dia", "pair", "cb"])
def test_plans_reject_malformed_csr(plan, defect):
    """Every host plan entry point (kry_dia_plan / kry_pair_plan /
    kry_cb_plan) checks the CSR arrays before building anything: indptr
    starting at 0, non-decreasing, ending at nnz = len(indices), and every
    column in [0, n). An inconsistent pair is KRY_EINVAL (ValueError), never
    an out-of-bounds read or write (the sanitizer runs of tests/
    test_host_sanitize.py execute these cases too). Sizes are past the
    checker's threading threshold."""
    from krylov_amd import _lib, problems

    A = problems.random_nonsym(1_100_000, per_row=3, seed=9)
    ip, ix = A.indptr.astype(np.int32).copy(), A.indices.astype(np.int32).copy()
    if defect == "nnz_short":
        ix = ix[:-7]
    elif defect == "nnz_long":
        ix = np.concatenate([ix, np.zeros(5, np.int32)])
    elif defect == "indptr_start":
        ip[0] = 1
    elif defect == "indptr_decreasing":
        ip[777_777] = ip[777_778] + 2
    elif defect == "col_negative":
        ix[123_456] = -3
    else:
        ix[1_000_001] = A.shape[0]
    fn = {"dia": _lib.dia_plan, "pair": _lib.pair_plan, "cb": _lib.cb_plan}[plan]
    with pytest.raises(ValueError):
        fn(ip, ix)


def _rcm_py(indptr, indices, wlimit):
    """Restatement of kry_rcm_plan (host_image.hpp rcm_order): George-Liu
    root from the lowest-index node of smallest degree (at most 4 BFS
    sweeps, the last level's smallest (degree, index) node next while the
    level count grows), Cuthill-McKee levels ordered by (smallest parent
    number, degree, index), new components from the lowest unnumbered index,
    reversed. None when a BFS level exceeds wlimit."""
    ip = indptr.astype(np.int64)
    ix = indices.astype(np.int64)
    n = ip.shape[0] - 1
    deg = np.diff(ip)

    def nbrs(v):
        return ix[ip[v]:ip[v + 1]]

    def sweep(root):
        level = np.full(n, -1)
        level[root] = 0
        front, nl = [root], 1
        while True:
            nxt = []
            for u in front:
                for w in nbrs(u):
                    if level[w] == -1:
                        level[w] = nl
                        nxt.append(int(w))
            if not nxt:
                break
            if len(nxt) > wlimit:
                return None
            front, nl = nxt, nl + 1
        return nl, min(front, key=lambda v: (deg[v], v))

    root = int(np.lexsort((np.arange(n), deg))[0])
    r = sweep(root)
    if r is None:
        return None
    ecc, cand = r
    for _ in range(3):
        if cand == root:
            break
        r2 = sweep(cand)
        if r2 is None:
            return None
        if r2[0] <= ecc:
            break
        root, ecc, cand = cand, r2[0], r2[1]
    num = np.full(n, -1)
    cm, scan, levels = [], 0, 0
    while len(cm) < n:
        if not cm:
            start = root
        else:
            while num[scan] != -1:
                scan += 1
            start = scan
        num[start] = len(cm)
        cm.append(start)
        a, b = len(cm) - 1, len(cm)
        levels += 1
        while True:
            key = {}
            for q in range(a, b):
                for w in nbrs(cm[q]):
                    w = int(w)
                    if num[w] == -1:
                        key[w] = min(key.get(w, q), q)
            if not key:
                break
            if len(key) > wlimit:
                return None
            nxt = sorted(key, key=lambda w: (key[w], deg[w], w))
            for w in nxt:
                num[w] = len(cm)
                cm.append(w)
            a, b = b, len(cm)
            levels += 1
    return np.array(cm[::-1], dtype=np.int32), levels


def _sym_perm(A, seed):
    p = np.random.default_rng(seed).permutation(A.shape[0])
    return A[p][:, p].tocsr()


@pytest.mark.parametrize("case", ["grid", "threaded", "components", "unsymmetric", "refused"])
def test_rcm_plan_matches_restatement(case):
    """The host renumbering (kry_rcm_plan: reverse Cuthill-McKee with a
    George-Liu root) against a pure-Python restatement of the same
    definition, node for node: a randomly numbered 2-D grid, one large enough
    for the threaded level passes (n > 2^16), disconnected components with
    isolated nodes, an unsymmetric pattern, and the refusal of a random graph
    whose BFS levels exceed the width limit. The renumbering brings the
    grid's bandwidth back to O(sqrt n)."""
    import scipy.sparse as sp
    from krylov_amd import _lib, problems

    wlimit = 1 << 16
    if case == "grid":
        A = _sym_perm(problems.poisson2d(30), 1)
    elif case == "threaded":
        A = _sym_perm(problems.poisson2d(265), 2)
    elif case == "components":
        A = _sym_perm(sp.block_diag([problems.poisson2d(12), sp.identity(7), problems.poisson2d(9)]).tocsr(), 3)
    elif case == "unsymmetric":
        rng = np.random.default_rng(4)
        L = sp.random(600, 600, density=0.004, random_state=5, format="csr") + sp.identity(600)
        A = _sym_perm(sp.tril(L).tocsr() + sp.diags(rng.uniform(1, 2, 600), 1, shape=(600, 600)), 6)
    else:
        A = problems.random_nonsym(20_000, per_row=6, seed=7)
        wlimit = 500
    A = A.tocsr()
    A.sort_indices()
    ip, ix = A.indptr.astype(np.int32), A.indices.astype(np.int32)
    got = _lib.rcm_plan(ip, ix, wlimit)
    want = _rcm_py(ip, ix, wlimit)
    if case == "refused":
        assert got is None and want is None
        return
    assert got is not None and want is not None
    np.testing.assert_array_equal(got[0], want[0])
    assert got[1] == want[1]
    assert np.array_equal(np.sort(got[0]), np.arange(A.shape[0]))
    if case in ("grid", "threaded"):
        p = got[0]
        B = A[p][:, p].tocoo()
        m = int(round(np.sqrt(A.shape[0])))
        assert np.abs(B.row - B.col).max() <= 2 * m + 2


def _rs_plan_py(indptr, indices):
    """Restatement of kry_rs_plan: slices of 128 rows, width = the longest
    row, slot (j, r) of a slice at 128 * (sptr[s] / 128 + j) + r - 128 s holds
    the j-th entry of row r with every run of 16 stored entries sorted by
    column (ties in stored order), as column | position-in-run << 28;
    padding 0xFFFFFFFF; refused above 1.25x the SELL-64 slots."""
    ip = indptr.astype(np.int64)
    n = ip.shape[0] - 1
    lens = np.diff(ip)
    ns = (n + 127) // 128
    widths = np.array([lens[128 * s:128 * s + 128].max() for s in range(ns)], dtype=np.int64)
    sptr = np.concatenate([[0], 128 * np.cumsum(widths)])
    sell = sum(64 * lens[64 * s:64 * s + 64].max() for s in range((n + 63) // 64))
    if sptr[-1] == 0 or sptr[-1] * 4 > sell * 5 + 4 * 128 * widths.max():
        return None
    cr = np.full(sptr[-1], 0xFFFFFFFF, dtype=np.uint32)
    for r in range(n):
        s = r // 128
        cols = indices[ip[r]:ip[r + 1]].astype(np.int64)
        for c0 in range(0, len(cols), 16):
            run = cols[c0:c0 + 16]
            order = np.argsort(run, kind="stable")
            for j, k in enumerate(order):
                cr[sptr[s] + 128 * (c0 + j) + r - 128 * s] = run[k] | (k << 28)
    return {"slices": ns, "slots": int(sptr[-1]), "widths": widths.astype(np.int32), "colrank": cr}


@pytest.mark.parametrize("case", ["unsorted", "long_rows", "duplicates"])
def test_rs_plan_matches_restatement(case):
    """The rank-sorted SELL-128 image's host side (kry_rs_plan) against a
    NumPy restatement: unsorted rows, rows longer than one 16-entry run, and
    duplicate columns (stable order)."""
    import scipy.sparse as sp
    from krylov_amd import _lib, problems

    if case == "unsorted":
        A = _sym_perm(problems.stencil15_3d(12), 8)  # the permuted columns of each row are unsorted in storage
        ip, ix = A.indptr.astype(np.int32), A.indices.astype(np.int32)
        ix = ix.copy()
        rng = np.random.default_rng(9)
        for r in range(0, A.shape[0], 3):
            seg = ix[ip[r]:ip[r + 1]]
            rng.shuffle(seg)
    elif case == "long_rows":
        A = sp.random(700, 700, density=0.06, random_state=10, format="csr") + sp.identity(700, format="csr")
        ip, ix = A.indptr.astype(np.int32), A.indices.astype(np.int32)
    else:
        ip = np.array([0, 3, 5, 9], dtype=np.int32)
        ix = np.array([2, 0, 2, 1, 1, 0, 2, 0, 1], dtype=np.int32)
    got = _lib.rs_plan(ip, ix)
    want = _rs_plan_py(ip, ix)
    assert got is not None and want is not None
    assert got["slices"] == want["slices"] and got["slots"] == want["slots"]
    np.testing.assert_array_equal(got["widths"], want["widths"])
    np.testing.assert_array_equal(got["colrank"], want["colrank"])


def test_build_id_matches_sources():
    """The loaded library is built from the sources in the tree: its stamp
    (kry_build_id, csrc/Makefile) is the sha256 over them, so a stale .so
    (or a PMC summary stamped with another build, bench.py) is caught."""
    import glob
    import hashlib
    import os

    from krylov_amd import _lib

    if _lib.HOST_ONLY:
        pytest.skip("host-only build")
    csrc = os.path.join(os.path.dirname(_lib.__file__), "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp"))
                   + glob.glob(os.path.join(csrc, "*.cpp")), key=os.path.basename)
    files.append(os.path.join(csrc, "..", "..", "include", "krylov_hip.h"))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    assert _lib.build_id() == h.hexdigest()[:16]
