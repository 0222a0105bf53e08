"""Synthetic CSR problems used by the benchmarks and the parity tests.

These are the generators of SURVEY.md Appendix A, written for speed at the
BASELINE sizes (n = 10M, nnz = 150M builds in a few seconds): every matrix is
assembled directly in canonical CSR form (sorted column indices, no
duplicates, int32 indices) with vectorised numpy, never through COO.

The same functions run here and on the GPU box; ``tests/golden/problems.json``
pins the SHA-256 of the arrays they produce so the two hosts are known to build
identical inputs.
"""
import hashlib

import numpy as np
import scipy.sparse

__all__ = [
    "stencil15_3d",
    "poisson2d",
    "random_nonsym",
    "shifted_lap3d_weighted",
    "csr_sha256",
    "diag100",
]


def _assemble(n, offsets, valid_fns, values, dtype=np.float64):
    """Build CSR from per-offset validity masks.

    ``offsets`` must already be in ascending order so every row comes out with
    sorted column indices. ``valid_fns[t](rows)`` returns the boolean mask of
    rows that own a neighbour at ``rows + offsets[t]``.
    """
    rows = np.arange(n, dtype=np.int64)
    masks = [fn(rows) for fn in valid_fns]
    counts = np.zeros(n, dtype=np.int64)
    for m in masks:
        counts += m
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    nnz = int(indptr[-1])
    indices = np.empty(nnz, dtype=np.int32)
    data = np.empty(nnz, dtype=dtype)
    cursor = indptr[:-1].copy()
    for off, m, val in zip(offsets, masks, values):
        r = rows[m]
        pos = cursor[r]
        indices[pos] = (r + off).astype(np.int32)
        data[pos] = val
        cursor[r] += 1
    if nnz < 2**31:
        indptr = indptr.astype(np.int32)
    return scipy.sparse.csr_matrix((data, indices, indptr), shape=(n, n))


def stencil15_3d(m=216):
    """3-D 15-point stencil on an m^3 grid (metric matrix).

    Lexicographic index ``i + m*j + m*m*k``, Dirichlet boundary. Centre 14,
    the six face neighbours and the eight (+-1,+-1,+-1) corners -1. SPD.
    m=216 gives n=10,077,696 and nnz=149,770,936.
    """
    n = m**3
    mm = m * m

    def coords(r):
        return r % m, (r // m) % m, r // mm

    nbrs = []
    for dk in (-1, 0, 1):
        for dj in (-1, 0, 1):
            for di in (-1, 0, 1):
                nz = (di != 0) + (dj != 0) + (dk != 0)
                if nz in (0, 1, 3):
                    nbrs.append((dk * mm + dj * m + di, di, dj, dk))
    nbrs.sort(key=lambda t: t[0])

    def make_fn(di, dj, dk):
        def fn(r):
            i, j, k = coords(r)
            ok = np.ones(r.shape, dtype=bool)
            for d, c in ((di, i), (dj, j), (dk, k)):
                if d == -1:
                    ok &= c > 0
                elif d == 1:
                    ok &= c < m - 1
            return ok

        return fn

    offsets = [t[0] for t in nbrs]
    fns = [make_fn(*t[1:]) for t in nbrs]
    vals = [14.0 if t[0] == 0 else -1.0 for t in nbrs]
    return _assemble(n, offsets, fns, vals)


def poisson2d(m=1000):
    """5-point Poisson ``kron(I, T(-1,4,-1)) + kron(T(-1,0,-1), I)`` on m^2."""
    n = m * m

    def fx(lo):
        return (lambda r: (r % m) > 0) if lo else (lambda r: (r % m) < m - 1)

    offsets = [-m, -1, 0, 1, m]
    fns = [
        lambda r: r >= m,
        fx(True),
        lambda r: np.ones(r.shape, dtype=bool),
        fx(False),
        lambda r: r < n - m,
    ]
    vals = [-1.0, -1.0, 4.0, -1.0, -1.0]
    return _assemble(n, offsets, fns, vals)


def random_nonsym(n=2_000_000, per_row=19, diag=0.8, seed=0):
    """Random nonsymmetric CSR (cfg3): ``per_row`` U(-1,1)/sqrt(per_row)
    off-diagonals per row at uniformly random columns, duplicates summed,
    plus ``diag * I``; canonical (sorted) CSR."""
    rng = np.random.default_rng(seed)
    rows = np.repeat(np.arange(n, dtype=np.int64), per_row)
    cols = rng.integers(0, n, per_row * n)
    vals = rng.uniform(-1.0, 1.0, per_row * n) / np.sqrt(per_row)
    A = scipy.sparse.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    A = A + diag * scipy.sparse.identity(n, format="csr")
    A = scipy.sparse.csr_matrix(A)
    A.sum_duplicates()
    A.sort_indices()
    if A.indices.dtype != np.int32 and A.nnz < 2**31:
        A.indices = A.indices.astype(np.int32)
        A.indptr = A.indptr.astype(np.int32)
    return A


def shifted_lap3d_weighted(m=200, sigma=0.5, seed=0):
    """Shifted 3-D 7-point Laplacian, row-scaled by 1/w (cfg5).

    Returns ``(A, w)`` with ``A = diag(1/w) K`` in float32 and ``w`` float64,
    ``w = default_rng(seed).uniform(1, 2, n)``. ``A`` is self-adjoint in the
    inner product ``<x, y>_W = x . (w * y)``.
    """
    n = m**3
    mm = m * m
    offsets = [-mm, -m, -1, 0, 1, m, mm]
    fns = [
        lambda r: (r // mm) > 0,
        lambda r: ((r // m) % m) > 0,
        lambda r: (r % m) > 0,
        lambda r: np.ones(r.shape, dtype=bool),
        lambda r: (r % m) < m - 1,
        lambda r: ((r // m) % m) < m - 1,
        lambda r: (r // mm) < m - 1,
    ]
    vals = [-1.0, -1.0, -1.0, 6.0 - sigma, -1.0, -1.0, -1.0]
    K = _assemble(n, offsets, fns, vals)
    w = np.random.default_rng(seed).uniform(1.0, 2.0, n)
    rowlen = np.diff(K.indptr)
    scale = np.repeat(1.0 / w, rowlen)
    A = scipy.sparse.csr_matrix(
        ((K.data * scale).astype(np.float32), K.indices, K.indptr), shape=K.shape
    )
    return A, w


def permuted_sym(A, seed=0):
    """``P A P^T`` for a uniformly random permutation (``default_rng(seed)``):
    the same nonzeros and values, rows and columns relabelled, so a banded or
    stencil matrix becomes one with scattered columns (the general-CSR SpMV
    case). Row i of the result is row p[i] of A with column c renamed
    pinv[c], sorted (canonical CSR, int32 indices kept)."""
    n = A.shape[0]
    p = np.random.default_rng(seed).permutation(n)
    pinv = np.empty(n, dtype=np.int64)
    pinv[p] = np.arange(n, dtype=np.int64)
    ip = A.indptr.astype(np.int64)
    lens = np.diff(ip)[p]
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=indptr[1:])
    nnz = int(indptr[-1])
    # source position of every output slot: row p[i]'s entries, in order
    start = np.repeat(ip[p] - indptr[:-1], lens)
    src = start + np.arange(nnz, dtype=np.int64)
    cols = pinv[A.indices[src]]
    # sort within rows: key = row * n + col (< 2^63 for n < 3e9)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    order = np.argsort(rows * n + cols, kind="stable")
    del rows
    indices = cols[order].astype(A.indices.dtype)
    data = A.data[src[order]]
    it = A.indptr.dtype if nnz < 2**31 else np.int64
    return scipy.sparse.csr_matrix((data, indices, indptr.astype(it)), shape=A.shape)


def diag100(n=100):
    """README / cfg1 problem: ``A = diag([1e-3, 2, ..., n])``, ``b = ones``."""
    return np.diag([1.0e-3] + list(range(2, n + 1))), np.ones(n)


def csr_sha256(A):
    """SHA-256 over (indptr, indices, data) bytes of a CSR matrix."""
    h = hashlib.sha256()
    for arr in (A.indptr, A.indices, A.data):
        h.update(np.ascontiguousarray(arr).tobytes())
    return h.hexdigest()
