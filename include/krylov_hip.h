/*
 * krylov_hip.h — C-ABI of libkrylov_hip.so, the MI355X (gfx950) inner loop of
 * the Krylov solvers cg / gmres / minres.
 *
 * The reference (ju-liu/krylov 0.0.3) is pure Python: its hot path ends in
 * SciPy/OpenBLAS/LAPACK calls made from the solver loops. Each entry point
 * below replaces one of those call sites (cited per function) and is bound
 * from Python through ctypes (krylov_amd/_lib.py; INTEGRATION.md shows the
 * stub). Plain pointers and sizes only; no C++ exceptions cross this boundary.
 *
 * Conventions
 *  - Every function returns an int status: KRY_OK (0) or a negative KRY_E*
 *    code; kry_last_error() returns the message of the calling thread's last
 *    failure.
 *  - Handles are opaque and owned by the caller (create/destroy pairs).
 *  - A vector is an n x k block stored row-major (the reference's "blocked"
 *    right-hand sides, b.shape == (n, k)); k = 1 is a plain vector.
 *  - One kry_ctx = one device + one HIP stream; a context is not thread-safe.
 *  - Host buffers are C-contiguous arrays of the stated dtype.
 *  - Device-resident state: per-iteration scalars never leave the GPU; the
 *    solver "run" calls return the residual-norm history of the steps they
 *    executed (the only mandatory device-to-host traffic).
 */
#ifndef KRYLOV_HIP_H
#define KRYLOV_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kry_ctx kry_ctx;
typedef struct kry_csr kry_csr;
typedef struct kry_vec kry_vec;
typedef struct kry_cg kry_cg;
typedef struct kry_gmres kry_gmres;
typedef struct kry_minres kry_minres;
typedef struct kry_comm kry_comm;
typedef struct kry_prog kry_prog;

/* value / index types */
enum { KRY_F32 = 1, KRY_F64 = 2 };
enum { KRY_I32 = 1, KRY_I64 = 2 };

/* status codes */
enum {
  KRY_OK = 0,
  KRY_EINVAL = -1,       /* bad argument (shape, dtype, null handle)   -> ValueError      */
  KRY_ENOMEM = -2,       /* device allocation failed                   -> MemoryError     */
  KRY_EDEVICE = -3,      /* HIP runtime / no device                    -> RuntimeError    */
  KRY_EINVARIANT = -4,   /* Krylov space invariant (arnoldi.py:168-171) -> ArgumentError  */
  KRY_EUNSUPPORTED = -5, /* outside the device path's scope            -> NotImplementedError */
  KRY_ESINGULAR = -6,    /* singular triangular factor (gmres.py:36)   -> LinAlgError     */
  KRY_ENONFINITE = -7,   /* NaN/inf handed to solve_triangular         -> ValueError      */
  KRY_ECOMM = -8         /* RCCL failure                               -> RuntimeError    */
};

/* ---- library / context ------------------------------------------------ */
int kry_version(void);
const char *kry_last_error(void);
/* The build stamp of this library (kry_version() >= 106): the first 16 hex
 * digits of the sha256 over its HIP/C++ sources, fixed at build time
 * (csrc/Makefile). Measurements taken on one build (profiles/ PMC passes) are
 * stamped with it, so a benchmark can tell whether they describe the code it
 * runs. No reference counterpart. */
const char *kry_build_id(void);
int kry_device_count(int *count);
int kry_ctx_create(int device, kry_ctx **out);
int kry_ctx_destroy(kry_ctx *ctx);
int kry_ctx_synchronize(kry_ctx *ctx);

/* ---- device memory -------------------------------------------------------
 * The library's device buffers come from a caching allocator: blocks freed by
 * a destroyed solver / operator / vector are reused by the next allocation of
 * the same rounded size (after one device synchronisation), instead of a
 * hipMalloc + hipFree pair per reference-API call (the reference allocates
 * its NumPy work arrays per call, cg.py:116-131, arnoldi.py:129-131).
 * KRYLOV_ALLOC_CACHE=0 disables it; KRYLOV_ALLOC_CACHE_MAX_GB caps it (16).
 * stats: out[0..5] = bytes in use, bytes cached, reuses, hipMallocs, device
 * syncs taken to retire freed blocks, enabled (0/1). release: hipFree every
 * cached block (in use blocks are untouched). */
int kry_mem_stats(int64_t *out);
int kry_mem_release(void);

/* ---- CSR operator ------------------------------------------------------
 * Replaces the scipy.sparse matrix the reference multiplies with `A @ x`
 * (_helpers.py:44-48 Product.__matmul__, cg.py:86, gmres.py:106,
 * minres.py:111,121). Uploads once; the library owns the device copy, which
 * it lays out as SELL-64 (slices of 64 rows = one wavefront, column-major
 * within a slice; slices with very uneven rows stay CSR). Indices may be
 * unsorted and contain duplicates; they are honoured in stored order (SciPy
 * csr_matvec semantics). */
int kry_csr_create(kry_ctx *ctx, int64_t n, int64_t nnz, const void *indptr,
                   const void *indices, const void *data, int dtype, int itype,
                   kry_csr **out);
int kry_csr_destroy(kry_csr *A);
/* kry_csr_create with another operator's bandwidth-reducing renumbering
 * (kry_version() >= 104): the image holds P M P^T for `like`'s permutation P
 * (rows' entries in their stored order), so M can precondition solves with
 * `like` (kry_*_set_preconditioners refuses operators renumbered differently).
 * Same as kry_csr_create when `like` is not renumbered. Replaces the
 * preconditioner operands M / Ml / Mr of cg.py:70-110, gmres.py:105-139,
 * minres.py:95-151 for a renumbered A. */
int kry_csr_create_like(kry_ctx *ctx, const kry_csr *like, int64_t n, int64_t nnz, const void *indptr,
                        const void *indices, const void *data, int dtype, int itype, kry_csr **out);
/* Renumbering (kry_version() >= 104). kry_csr_create renumbers a matrix whose
 * columns are scattered (the column-blocked test below) but whose graph has
 * narrow BFS levels (a mesh or stencil stored in a bad order) by reverse
 * Cuthill-McKee; its images then hold P A P^T with every row's entries in
 * stored order, so the SpMV stays bitwise csr_matvec. Every vector still
 * crosses the C-ABI in the caller's numbering: kry_*_start permutes b / x0 /
 * weights in, kry_*_get, kry_gmres_xk_device and kry_spmv permute out. The
 * reference multiplies the caller's matrix as given (_helpers.py:44-48): this
 * is storage order only. kry_csr_permute moves the rows of an n x k block
 * into the operator's numbering (to_operator = 1: dst[r] = src[perm[r]]) or
 * back (0), for callers that keep their own device vectors in the operator's
 * numbering (kry_prog_*). KRY_RENUMBER=0 disables renumbering. */
int kry_csr_permute(kry_ctx *ctx, const kry_csr *A, const kry_vec *src, kry_vec *dst, int to_operator);
/* Byte comparison of two operators' SELL-64 and diagonal-offset images and
 * their sizes (kry_version() >= 104; tests: kry_csr_create builds those images
 * on the device for int32 CSR, KRY_DEVICE_BUILD=0 on the host, and the two
 * must be identical): out[0] = number of differing items, out[1] = bitmask. */
int kry_csr_compare(const kry_csr *A, const kry_csr *B, int64_t *out);
/* kry_spmv with x and y already in the operator's numbering (kry_csr_permute);
 * the same as kry_spmv for an operator that is not renumbered. */
int kry_spmv_op(kry_ctx *ctx, kry_csr *A, kry_vec *x, kry_vec *y);
/* Host-only (no device): the reverse Cuthill-McKee order kry_csr_create
 * would use (int32 indices): info[0..1] = built (0 = a BFS level exceeded
 * wlimit nodes: no narrow level structure), BFS levels of the numbering;
 * when built and perm is non-null: perm[n], new row r = old row perm[r].
 * wlimit <= 0 takes the library's default (max(2^16, n / 32)). */
int kry_rcm_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t wlimit,
                 int64_t *info, int32_t *perm);
/* The same order computed on the device (what kry_csr_create runs; int32
 * CSR from the host, uploaded inside): info[0] = 1 built, 0 refused, -1 gave
 * up (more than 64 components: kry_csr_create then uses the host order),
 * info[1] = levels; perm as kry_rcm_plan's, node for node. */
int kry_rcm_device(kry_ctx *ctx, int64_t n, int64_t nnz, const int32_t *indptr, const int32_t *indices, int64_t wlimit,
                   int64_t *info, int32_t *perm);
/* Host-only: the rank-sorted SELL-128 plan (kry_version() >= 104; the image a
 * matrix takes for single-RHS SpMVs when no DIA, column-blocked or paired
 * image is built): info[0..3] = built, slices, slots, widest slice; when built
 * and the arrays are non-null: widths[slices], colrank[slots] (slot of row r,
 * slot column j of its slice at 128 * (sptr[s] / 128 + j) + r - 128 s: the
 * column in bits 0..27, its position among the run of 16 stored entries it
 * belongs to in bits 28..31, 0xFFFFFFFF = padding). */
int kry_rs_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t *info,
                int32_t *widths, uint32_t *colrank);
/* Host-only (no GPU needed): the SELL-64 plan kry_csr_create will build —
 * slice count, stored slots (nonzeros + padding of regular slices) and the
 * number of irregular slices (64 * width > 2 * slice_nnz + 1024) that the
 * kernel walks in CSR form instead. */
int kry_csr_layout(int64_t n, const void *indptr, int itype, int64_t *nslices,
                   int64_t *nslots, int64_t *nirregular);
/* Host-only: the diagonal-offset (SELL-128/DIA) plan kry_csr_create would
 * build for these CSR arrays (no device needed). info[0..3] = built (0/1),
 * slices, slots, widest slice; when built and the arrays are non-null:
 * widths[slices], offsets[slots / 128] (each slice's sorted offsets col - row),
 * masks[2 * slots / 128] (word q, bit l: row 128 s + 2 l + q has an entry at
 * that offset). Call once with null arrays to size them. */
int kry_dia_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t *info,
                 int32_t *widths, int32_t *offsets, uint64_t *masks);
/* Host-only view of the paired-row SELL-128 plan (no device needed; the
 * image kry_csr_create builds for a general matrix, kry_version() >= 102):
 * info[0..3] = built (0 = refused: a slot column spans more than 65534
 * columns, n >= 2^31, or more than 1.25x the SELL-64 slots), slices, slots,
 * widest slice; when built and the arrays are non-null: widths[slices],
 * cbase[slots / 128] (each slot column's smallest column), deltas[slots]
 * (column - base at slot 128 * (sptr[s] / 128 + j) + row - 128 s, 0xFFFF =
 * padding). Call once with null arrays to size them. */
int kry_pair_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t *info,
                  int32_t *widths, int32_t *cbase, uint16_t *deltas);
/* Host-only view of the column-blocked plan (no device needed; the image
 * kry_csr_create builds for single-RHS SpMVs of a matrix with scattered
 * columns when the diagonal-offset image is not built, kry_version() >= 103):
 * info[0..3] = built (0 = refused: int64 indices, x under 8 MB, rows not
 * sorted, fewer than a quarter of the entries more than half a block from the
 * diagonal, or a segment over 65535 entries), column blocks nb, columns per
 * block, 256-row groups ng; when built and gptr is non-null: gptr[nb * ng + 1],
 * the first entry of segment (block b, group g) at gptr[b * ng + g]. */
int kry_cb_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t *info,
                int64_t *gptr);
/* The device image kry_csr_create built, size-checked: writes the first
 * min(len, KRY_CSR_INFO_LEN) of info[0..8] = slices, slots, irregular slices,
 * compact (1 when the column indices are stored as uint16 deltas over
 * per-slot-column int32 bases: every slot column spans <= 65534 columns,
 * int32 indices and KRY_SELL_COMPACT != 0 in the environment), the number of
 * column blocks of the column-blocked image used by single-RHS SpMVs on
 * scattered sparsity (0 = none; KRY_SPMV_CB=0 disables), dia (1 when the
 * diagonal-offset image serves single-RHS SpMVs: int32 indices, every row
 * strictly sorted, the rows of each 64-row slice sharing a short list of
 * column offsets; KRY_SPMV_DIA=0 disables) and that image's slot count,
 * then (kry_version() >= 102) pair (1 when the paired-row SELL-128 image
 * serves single-RHS SpMVs of a general matrix: no diagonal-offset or
 * column-blocked image, n < 2^31, every 128-row slot column spans <= 65534
 * columns, at most 1.25x the SELL-64 slots; KRY_SPMV_PAIR=0 disables) and
 * that image's slot count. Fields added later go at the end, so a caller
 * built against this header keeps working (kry_version() >= 101). */
/* then (kry_version() >= 104) rs (1 when the rank-sorted SELL-128 image
 * serves single-RHS SpMVs), its slot count, renumbered (1 when the images hold
 * the reverse Cuthill-McKee renumbering P A P^T) and the renumbering's BFS
 * level count. */
#define KRY_CSR_INFO_LEN 13
int kry_csr_info_n(const kry_csr *A, int64_t *info, int32_t len);
/* The version-100 form: info[0..4] only (`info` holds 5 values). */
int kry_csr_info(const kry_csr *A, int64_t *info);

/* ---- vectors (n x k row-major blocks) ---------------------------------- */
int kry_vec_create(kry_ctx *ctx, int64_t n, int32_t k, int dtype, kry_vec **out);
int kry_vec_destroy(kry_vec *v);
int kry_vec_upload(kry_vec *v, const void *host);
int kry_vec_download(kry_vec *v, void *host);

/* ---- primitives --------------------------------------------------------
 * y = A @ x. Replaces SciPy csr_matvec / csr_matvecs (SURVEY §2 kernel
 * table); bitwise equal to them (sequential per-row sum, no FMA). */
int kry_spmv(kry_ctx *ctx, kry_csr *A, kry_vec *x, kry_vec *y);
/* out[c] = sum_i x[i,c] * (w[i] * y[i,c])  (w == NULL: plain). Replaces
 * get_default_inner (_helpers.py:101-110) and the weighted inner of
 * tests/test_solvers.py:157-161. Deterministic two-stage reduction. */
int kry_dot(kry_ctx *ctx, kry_vec *x, kry_vec *y, kry_vec *w, double *out);
/* y = alpha[c] * x + y  (the reference's `y += alpha * x`, e.g. cg.py:196). */
int kry_axpy(kry_ctx *ctx, const double *alpha, kry_vec *x, kry_vec *y);
/* z = one of the reference's vector expressions, per column c (k <= 64),
 * evaluated exactly as its NumPy expression tree; stream-ordered (no sync):
 *   form 0: z = x + a[c] * y             (x += alpha * p, bicgstab.py:120)
 *   form 1: z = x + a[c] * (y + b[c] * w)  (cgs.py:88)
 *   form 2: z = x + a[c] * (y - b[c] * w)  (bicgstab.py:109)
 *   form 3: z = x / a[c]   form 4: z = x - y   form 5: z = x + y
 *   form 6: z = x          form 7: z = a[c] * x
 * z may alias x, y or w. Replaces the AXPY-type lines of the other
 * solvers (bicgstab.py, cgs.py, cgr.py, gcr.py; krylov_amd/extra.py). */
int kry_vec_lincomb(kry_ctx *ctx, int form, kry_vec *z, kry_vec *x, kry_vec *y, kry_vec *w,
                    const double *a, const double *b);
/* ---- device-resident scalar chain of the other solvers --------------------
 * bicgstab.py:24-144, cgs.py:24-117, cgr.py:16-100, gcr.py:18-97 (driven by
 * krylov_amd/extra.py): the per-iteration scalars live in a device register
 * file of nregs rows of k float64 values, so a chunk of iterations is
 * enqueued with no host round trip and read back with one sync.
 * create: nregs registers, k columns (power of two <= 64), history capacity
 *         `cap` steps per chunk.
 * set / get: register r (r = -1 in set: the criterion row, +inf on padded
 *         columns) from / to k host doubles (synchronous).
 * begin: start a chunk (every step runs until a check stops it).
 * scalar: register ops of the reference's scalar lines, float64:
 *         op 0 d = a; 1 d = a / g(b); 2 d = (a * b) / g(c * e); 3 d = sqrt(a);
 *         4 d = g(a); 5 d = value   (g(x) = x != 0 ? x : 1, np.where guard)
 * dot:   register d = inner(x, y) per column (w: weights or NULL).
 * lincomb: kry_vec_lincomb's forms with a = sa * reg[ra], b = sb * reg[rb]
 *         (register -1 = unused; sa, sb = +1 / -1).
 * spmv:  y = A x.
 * check: register r against the criterion: mode 0 appends it to the chunk
 *         history and stops the chunk after this step when every column
 *         meets it; mode 1 (bicgstab's mid-step test on the previous iterate,
 *         bicgstab.py:123-127) stops the chunk AT this step on success and
 *         records its row there; mode | 4: compare the norm rounded to
 *         float32 (the history of a float32 solve).
 * end:   one sync: *done steps ran in full, *midstep = 1 if a mode-1 check
 *         stopped step *done; rows receives done (+ midstep) rows of k.
 * Every launch takes the chunk step it belongs to and does nothing once a
 * check has stopped the chunk before it. */
int kry_prog_create(kry_ctx *ctx, int32_t nregs, int32_t k, int32_t cap, kry_prog **out);
int kry_prog_destroy(kry_prog *p);
int kry_prog_set(kry_prog *p, int32_t r, const double *vals);
int kry_prog_get(kry_prog *p, int32_t r, double *vals);
int kry_prog_begin(kry_prog *p);
int kry_prog_end(kry_prog *p, int32_t steps, int32_t *done, int32_t *midstep, double *rows);
int kry_prog_scalar(kry_prog *p, int32_t op, int32_t d, int32_t a, int32_t b, int32_t c, int32_t e, double value,
                    int32_t step);
int kry_prog_dot(kry_prog *p, kry_vec *x, kry_vec *y, kry_vec *w, int32_t d, int32_t step);
int kry_prog_lincomb(kry_prog *p, int32_t form, kry_vec *z, kry_vec *x, kry_vec *y, kry_vec *w, int32_t ra, double sa,
                     int32_t rb, double sb, int32_t step);
int kry_prog_spmv(kry_prog *p, kry_csr *A, kry_vec *x, kry_vec *y, int32_t step);
int kry_prog_check(kry_prog *p, int32_t r, int32_t mode, int32_t step);

/* Batched LAPACK >= 3.10 ?lartg on device (givens.py:35-40); host arrays of
 * `count` values of `dtype`. Bitwise equal to scipy.linalg.lapack ?lartg. */
int kry_lartg(kry_ctx *ctx, int64_t count, int dtype, const void *f, const void *g,
              void *c, void *s, void *r);

/* ---- CG (cg.py:16-259) ----------------------------------------------------
 * set_preconditioners: M and Ml as device operators (NULL = identity), before
 *        start; the loop then applies Ml (A p) (Product(Ml, A), cg.py:110) and
 *        z = M Ml_r with rho = <Ml_r, z> (cg.py:205-209).
 * start: r0 = Ml (b - A x0), rho0 = <r0, M r0>_w; rho0 (k values) returned.
 * run:   executes up to max_steps iterations of cg.py:175-217 on device; stops
 *        early after the first iteration whose residual norms all satisfy
 *        resnorm <= criterion (the test at cg.py:156). Writes the new residual
 *        norms (steps_done x k) to resnorms.
 * residual: explicit ||M Ml (b - A xk)||_{M^-1} with xk = x0 + yk (cg.py:158-160).
 * get:   download xk (which = 0), the updated residual Ml_r (which = 1) or
 *        M Ml_r (which = 2).
 * scalars: the current [rho, rho_prev, alpha, omega] (4 x k values) of the
 *        recurrence, for the Lanczos relation of return_arnoldi
 *        (cg.py:218-233). */
int kry_cg_create(kry_ctx *ctx, kry_csr *A, int32_t k, int dtype, kry_cg **out);
int kry_cg_destroy(kry_cg *s);
int kry_cg_set_preconditioners(kry_cg *s, kry_csr *M, kry_csr *Ml);
int kry_cg_start(kry_cg *s, kry_vec *b, kry_vec *x0, kry_vec *w, double *rho0);
int kry_cg_set_criterion(kry_cg *s, const double *criterion);
int kry_cg_run(kry_cg *s, int32_t max_steps, int32_t *steps_done, double *resnorms);
/* Iterations per kry_cg_run call this solve is best driven with (after
 * kry_cg_start): 256 when it runs the persistent small-n loop (one launch per
 * call, nothing launched past convergence), 32 otherwise. The driver-side
 * chunking of the reference's loop (cg.py:155-234) is free to use any value. */
int kry_cg_preferred_chunk(kry_cg *s, int32_t *steps);
/* Which path the last kry_cg_run chunk took (host-side bookkeeping, no
 * device work): info[0] = 1 if it ran as the persistent small-n loop (one
 * launch per chunk), 0 if launch per pass; info[1] = chunks that
 * were rerun launch per pass after an in-launch exchange timed out (a block
 * that never became resident). The rerun starts from the chunk-start state,
 * which the persistent loop never overwrites, so the history is that of an
 * uninterrupted solve. Fault injection for tests: KRY_CGP_FAULT=t makes the
 * last block drop out at iteration t of a chunk. */
int kry_cg_path(kry_cg *s, int32_t *info);
/* The same for the one-launch update of the launch-per-pass form (large n,
 * one RHS, no M / Ml, Euclidean inner: alpha, r, rho, omega, y and p of an
 * iteration in one launch after the SpMV): info[0] = 1 if the last
 * kry_cg_run chunk used it; info[1] = chunks whose remaining steps were rerun
 * with separate passes after its exchange timed out (it writes nothing
 * before the exchange completes). KRY_CG_UPD=0 disables it; KRY_CGU_FAULT=t
 * makes the last block drop out at step t of a chunk (tests). */
int kry_cg_update_path(kry_cg *s, int32_t *info);
/* Deferred yk updates (yk += alpha p, cg.py:196, applied D steps at a time;
 * bitwise the per-step updates): *D = the steps per flush this solver uses
 * (0 = one update per step; decided at the first kry_cg_run), *bytes = the
 * device memory its D ring buffers of p and the alpha ring hold until
 * kry_cg_destroy. Default, when an n x k vector exceeds 128 MB: the
 * deepest D of 31, 15, 7, 3 whose ring fits an eighth of the device's total
 * memory, else 0; KRY_CG_YDEFER = D (1..31) overrides; an allocation failure
 * falls back to D = 0. */
int kry_cg_defer_info(kry_cg *s, int32_t *D, int64_t *bytes);
int kry_cg_residual(kry_cg *s, double *resnorm);
int kry_cg_get(kry_cg *s, int which, void *host);
int kry_cg_scalars(kry_cg *s, double *out);

/* ---- GMRES (gmres.py:41-251, ArnoldiMGS arnoldi.py:107-200) --------------
 * set_preconditioners: M, Ml, Mr as device operators (NULL = identity); the
 *         Arnoldi operator is Ml A Mr, M gives the second basis P (V = M P),
 *         and xk = x0 + Mr (sum_i yy_i V_i) (gmres.py:97-99, 139).
 * create: workspace for up to `maxiter` Arnoldi steps with `sweeps` MGS
 *         passes per step ("mgs" = 1, "mgsK" = K), or sweeps = 0 for
 *         Householder Arnoldi (ortho="householder", arnoldi.py:33-104; k = 1,
 *         default inner, no M).
 * start:  r0 = b - A x0, ||r0||, V0 = r0 / ||r0|| (guarded), y[0] = ||r0||.
 * run:    up to max_steps Arnoldi + Givens steps; stops early after a step
 *         whose |y[k+1]| all satisfy the criterion or that found the space
 *         invariant (*invariant = 1). Returns KRY_EINVARIANT if called after
 *         an invariant step (arnoldi.py:168-171).
 * solution: xk = x0 + sum_i yy_i V_i with yy = R^-1 y (gmres.py:89-99),
 *         left on device; residual: explicit ||b - A xk||.
 * get:    which = 0: xk (after solution); 1: the basis V_0..V_m and 2: P_0..P_m
 *         (m = steps, or steps - 1 after an invariant step; n x k each, packed);
 *         3: the Hessenberg matrix H, (maxiter + 1) x maxiter x k (ArnoldiMGS /
 *         ArnoldiHouseholder state, arnoldi.py:33-200). */
int kry_gmres_create(kry_ctx *ctx, kry_csr *A, int32_t k, int dtype, int32_t maxiter,
                     int32_t sweeps, kry_gmres **out);
int kry_gmres_destroy(kry_gmres *s);
int kry_gmres_set_preconditioners(kry_gmres *s, kry_csr *M, kry_csr *Ml, kry_csr *Mr);
int kry_gmres_start(kry_gmres *s, kry_vec *b, kry_vec *x0, kry_vec *w, double *r0norm);
int kry_gmres_set_criterion(kry_gmres *s, const double *criterion);
int kry_gmres_run(kry_gmres *s, int32_t max_steps, int32_t *steps_done,
                  double *resnorms, int32_t *invariant);
int kry_gmres_solution(kry_gmres *s);
int kry_gmres_residual(kry_gmres *s, double *resnorm);
int kry_gmres_get(kry_gmres *s, int which, void *host);
/* xk (after kry_gmres_solution) copied into a device vector of the solver's
 * shape, on the context stream: restarted GMRES(m) chains x0 = xk of the last
 * cycle (gmres.py:41-54 called again with x0) without leaving the device. */
int kry_gmres_xk_device(kry_gmres *s, kry_vec *out);
/* info[0] = 1 while Arnoldi steps run their MGS passes as one persistent
 * launch (gm_mgsp_kernel), 0 launch per pass (not eligible, or switched off
 * after a timeout); info[1] = chunks finished launch per pass after a
 * persistent MGS exchange timed out. The timed-out step is rerun from its
 * SpMV, so the history is that of an uninterrupted solve. Fault injection
 * for tests: KRY_MGS_FAULT=s makes the last block drop out at chunk step s. */
int kry_gmres_path(kry_gmres *s, int32_t *info);
/* multi_solve_triangular (gmres.py:24-38) as a standalone call: per column c
 * of k, out[:, c] = R[:, :, c]^-1 y[:, c] for upper-triangular R (m x m x k,
 * C order) and y (m x k), host float64 arrays; arithmetic in `dtype`
 * (dtrtrs / strtrs). Zero rhs -> 0; KRY_ENONFINITE, KRY_ESINGULAR as LAPACK. */
int kry_trsv_upper(kry_ctx *ctx, int32_t m, int32_t k, int dtype, const double *R, const double *y,
                   double *out);
/* Householder(x) (householder.py:6-53) for one vector (k = 1): v_out = the
 * normalised reflector vector, out3 = [beta, alpha, xnorm] (H x = alpha xnorm
 * e_1); the kernels of Householder Arnoldi, arithmetic in x's dtype. */
int kry_householder(kry_ctx *ctx, kry_vec *x, kry_vec *v_out, double *out3);

/* ---- MINRES (minres.py:28-253, ArnoldiLanczos arnoldi.py:203-281) --------
 * set_preconditioners: M, Ml, Mr as device operators (NULL = identity);
 * Lanczos on Ml A Mr with p / v = M p, xk = x0 + Mr yk (minres.py:95-98).
 * Same run protocol as CG; R, rotations, y, z and W are float64 as in the
 * reference under NumPy-2 promotion (minres.py:195,219). */
int kry_minres_create(kry_ctx *ctx, kry_csr *A, int32_t k, int dtype, kry_minres **out);
int kry_minres_destroy(kry_minres *s);
int kry_minres_set_preconditioners(kry_minres *s, kry_csr *M, kry_csr *Ml, kry_csr *Mr);
int kry_minres_start(kry_minres *s, kry_vec *b, kry_vec *x0, kry_vec *w, double *r0norm);
int kry_minres_set_criterion(kry_minres *s, const double *criterion);
int kry_minres_run(kry_minres *s, int32_t max_steps, int32_t *steps_done,
                   double *resnorms, int32_t *invariant);
/* Whether the last kry_minres_run chunk ran the one-launch step tail (alpha,
 * Lanczos orthogonalisation, QR update and the z / W / yk / p update in one
 * launch after the SpMV: one RHS, no M / Ml / Mr, float64 vectors): info[0];
 * info[1] = chunks whose remaining steps were rerun with the separate kernels
 * after its exchange timed out (it writes nothing before the exchange
 * completes). KRY_MR_UPD=0 disables it; KRY_MRU_FAULT=t drops the last block
 * out at step t of a chunk (tests). */
int kry_minres_update_path(kry_minres *s, int32_t *info);
int kry_minres_residual(kry_minres *s, double *resnorm);
/* get: which = 0: xk; 1: the current Lanczos vector p; 2: v = M p; 3: the last
 * step's [h0, h1, h2] (3 x k; ArnoldiLanczos state, arnoldi.py:203-281). */
int kry_minres_get(kry_minres *s, int which, void *host);

/* ---- multi-GPU: RHS columns sharded one block per GPU ----
 * One RCCL communicator per process/GPU. After attaching, each CG iteration
 * performs exactly one ncclAllReduce(sum, f64, count = total_k + 1) on the
 * zero-padded residual-norm vector so every rank applies the reference's
 * global stop rule np.all(resnorms[-1] <= criterion) (cg.py:156).
 * The last slot of every per-step allreduce (CG, GMRES, MINRES) is a fault
 * count: a rank whose in-launch exchange timed out at a step (a block that
 * never became resident) posts a fault there instead of its norms, so EVERY
 * rank stops the chunk before that step, after the same collectives: the
 * faulting rank's run returns KRY_EDEVICE, every other rank's KRY_ECOMM, and
 * no rank blocks in a later allreduce. KRY_COMM_PEER_FAULT=s makes step s of
 * a run call receive a fault as if a peer had posted it (tests on one GPU). */
int kry_comm_unique_id(void *id128);
int kry_comm_create(kry_ctx *ctx, int32_t nranks, int32_t rank, const void *id128,
                    kry_comm **out);
/* One communicator per context of one process (ncclCommInitAll over the
 * contexts' devices; out[i] is rank i of n), kry_version() >= 104: the
 * single-process multi-GPU path, krylov_amd.cg / gmres / minres(...,
 * devices=[...]), one host thread per device. Replaces the per-process
 * ranks of SURVEY §8(e) when the caller has one process for the node. */
int kry_comm_create_all(kry_ctx **ctxs, int32_t n, kry_comm **out);
int kry_comm_destroy(kry_comm *c);
/* Abort a communicator, from any thread, while a collective on it may be
 * pending (ncclCommAbort; kry_version() >= 105): that and every later
 * collective fail, so a solver waiting on a rank that will not come stops
 * with KRY_ECOMM. kry_comm_destroy still releases the handle. No reference
 * counterpart: the devices=[...] driver aborts every device's communicator
 * when one device's thread fails. */
int kry_comm_abort(kry_comm *c);
/* The communicator as RCCL sees it (kry_version() >= 106): *nranks from
 * ncclCommCount, *rank from ncclCommUserRank; KRY_ECOMM once aborted. */
int kry_comm_info(kry_comm *c, int32_t *nranks, int32_t *rank);
/* in-place sum over ranks of `count` host doubles (setup-time exchanges) */
int kry_comm_allreduce(kry_comm *c, double *host, int32_t count);
int kry_cg_attach_comm(kry_cg *s, kry_comm *c, int32_t col_offset, int32_t total_k);
/* GMRES / MINRES: the same sharding (gmres.py:193 and minres.py:162 stop rules,
 * arnoldi.py:187 / 270-272 invariance over all columns): one
 * ncclAllReduce(sum, f64, count = total_k + 2) per step of the zero-padded
 * residual norms, a count of ranks with a non-invariant column and the fault
 * count. After
 * attaching, set_criterion takes total_k values and each run history row
 * holds total_k values. */
int kry_gmres_attach_comm(kry_gmres *s, kry_comm *c, int32_t col_offset, int32_t total_k);
int kry_minres_attach_comm(kry_minres *s, kry_comm *c, int32_t col_offset, int32_t total_k);

/* ---- timing: HIP events on the context stream --------------------------- */
int kry_timer_start(kry_ctx *ctx);
int kry_timer_stop(kry_ctx *ctx, double *ms);
/* device time of the solvers' launches per kernel id (0 SpMV, 1 update
 * pass, 2 MGS, 3 other), measured with HIP events around the launches when
 * enabled; enable != 0 times every launch of every id, kry_profile_select
 * only the ids whose bit is set in mask and of those one launch in `every`
 * (each timed launch adds two event records to the stream: ~3 us at the
 * metric). Both reset the counts. kry_profile_read: timed launches, total ms. */
int kry_profile_enable(kry_ctx *ctx, int enable);
int kry_profile_select(kry_ctx *ctx, uint32_t mask, int32_t every);
int kry_profile_read(kry_ctx *ctx, int kernel_id, int64_t *count, double *total_ms);

#ifdef __cplusplus
}
#endif
#endif /* KRYLOV_HIP_H */
