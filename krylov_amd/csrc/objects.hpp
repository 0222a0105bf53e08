// Host-side objects behind the opaque C-ABI handles.
#pragma once

#include <utility>
#include <vector>

#include "common.hpp"

struct kry_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t t0 = nullptr, t1 = nullptr;
  // per-kernel HIP-event profiling (bench.py's live roofline measurement)
  unsigned profile = 0;  // bit id: HIP events around launches of kernel id (PROF_*)
  int prof_every = 1;    // ... around one launch in prof_every of each id
  int64_t prof_calls[4] = {0, 0, 0, 0};
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  size_t ev_used = 0;
  int ev_kernel_id = 0;  // which kernel family the pool currently records
  // accumulated {count, ms} per kernel id, folded in at kry_profile_read
  int64_t prof_count[4] = {0, 0, 0, 0};
  double prof_ms[4] = {0, 0, 0, 0};
  std::vector<int> ev_ids;
  // scratch for one-shot reductions and scalar staging (blas.hip, kry_dot)
  double *scratch = nullptr;
  size_t scratch_bytes = 0;
  // pinned host staging for the per-chunk readback (control word + history)
  void *pinned = nullptr;
  size_t pinned_bytes = 0;
};

struct kry_csr {
  kry_ctx *ctx = nullptr;
  int64_t n = 0, nnz = 0;
  int dtype = 0, itype = 0;
  // SELL-64 image (device): slice s covers rows [64 s, 64 s + 64)
  int64_t nslices = 0, nslots = 0, nirregular = 0;
  int max_width = 0;        // widest regular slice (picks the SpMV unroll)
  void *sptr = nullptr;     // int64, nslices + 1 slot offsets
  void *swidth = nullptr;   // int32, slice width, -1 = irregular (CSR walk)
  void *sidx = nullptr;     // itype, nslots (+ pad), -1 = padding
  void *sval = nullptr;     // dtype, nslots (+ pad)
  // compact column image (SELL-64/d16): when every slot column of every
  // regular slice spans <= 65534 columns, sidx is replaced by a per-lane
  // uint16 delta (0xFFFF = padding) over a per-slot-column int32 base
  bool compact = false;
  void *sdelta = nullptr;   // uint16, nslots (+ pad)
  void *scbase = nullptr;   // int32, nslots / 64 (+ pad): base of slot column j of slice s at sptr[s] / 64 + j
  // column-blocked image (scattered sparsity, single-RHS SpMV): the columns
  // are cut into cb_nb blocks of cb_cols (x block L2-resident); segment (b,
  // g) holds 256-row group g's entries with columns in block b, in stored
  // order (bitwise: rows are sorted, so block order is stored order); the
  // SpMV walks the blocks in order with each row's running sum in a register
  // (spmv_cbp_kernel). Built only for int32 indices, sorted rows and scattered
  // columns; the SELL image is kept for k > 1.
  int64_t cb_nb = 0, cb_cols = 0, cb_ng = 0;
  void *cb_gptr = nullptr;  // int64, cb_nb * cb_ng + 1: segment (block b, group g) at [gptr[b ng + g], ...)
  void *cb_roff = nullptr;  // uint16, cb_nb * n (+ pad): row's first entry inside its segment
  void *cb_col = nullptr;   // int32, nnz (+ pad)
  void *cb_val = nullptr;   // dtype, nnz (+ pad)
  // diagonal-offset image (SELL-128/DIA, structured matrices, k = 1): in
  // every slice of 128 rows the columns of each row are row + o_j for a short
  // sorted list of offsets o_j shared by the slice, so slot column j holds the
  // entry at offset o_j of every row (or a masked-off hole). Lane l of the
  // wave owns rows 2l and 2l + 1: per slot column its two values, its two x
  // entries x[row + o_j], x[row + 1 + o_j] and (at the end) its two results
  // are each one 16-byte access (8 bytes for float). Per slot column one
  // int32 offset and two uint64 lane masks (even rows, odd rows), read with
  // scalar loads, replace the 128 per-row indices: the matrix stream is the
  // values alone. Built only for int32 inputs whose every row is strictly
  // sorted, and only when the slot count stays within 1.25x of the SELL
  // image's.
  bool dia = false;
  int64_t dia_nslices = 0;
  int64_t dia_nslots = 0;
  int dia_max_width = 0;
  int dia_span = -1;          // max |offset| over the image; -1 = not computed yet (cg.hip dia_span_of)
  void *dia_sptr = nullptr;   // int64, dia_nslices + 1 (slots; kDiaSlice per slot column)
  void *dia_width = nullptr;  // int32, dia_nslices
  void *dia_off = nullptr;    // int32, dia_nslots / kDiaSlice (+ kDiaPad)
  void *dia_mask = nullptr;   // uint64 x 2 per slot column: bit l of word q = row 2l + q present
  void *dia_val = nullptr;    // dtype, dia_nslots (+ pad), row order within a slot column; holes are 0
  // paired-row SELL-128 image (general matrices, k = 1; spmv_pair_kernel):
  // slice s covers rows [128 s, 128 s + 128); slot column j of the slice
  // holds the j-th stored entry of every row, row r at position r - 128 s,
  // as a value and a uint16 delta over the slot column's int32 base
  // (0xFFFF = padding). Built when neither the DIA nor the column-blocked
  // image serves k = 1, every slot column spans <= 65534 columns and the
  // slots stay within 1.25x the SELL-64 image's.
  bool sp = false;
  int64_t sp_nslices = 0, sp_nslots = 0;
  int sp_max_width = 0;
  void *sp_sptr = nullptr;   // int64, sp_nslices + 1 (slots; kPairSlice per slot column)
  void *sp_width = nullptr;  // int32, sp_nslices
  void *sp_cbase = nullptr;  // int32, sp_nslots / kPairSlice (+ kDiaPad)
  void *sp_delta = nullptr;  // uint16, sp_nslots (+ pad)
  void *sp_val = nullptr;    // dtype, sp_nslots (+ pad)
  // rank-sorted SELL-128 image (round 5; spmv_rs_kernel, host_image.hpp
  // rs_build): the paired-row geometry with int32 columns, each run of
  // kRsChunk stored entries of a row sorted by column, the entry's position
  // in its run in the word's top 4 bits (the kernel sums the run back in
  // stored order). Built for k = 1 when no DIA, column-blocked or paired image
  // is (unsorted rows, wide slot columns: a renumbered matrix).
  bool rs = false;
  int64_t rs_nslices = 0, rs_nslots = 0;
  int rs_max_width = 0;
  void *rs_sptr = nullptr;     // int64, rs_nslices + 1
  void *rs_width = nullptr;    // int32, rs_nslices
  void *rs_colrank = nullptr;  // uint32, rs_nslots (+ pad): column | run position << 28, 0xFFFFFFFF = padding
  void *rs_val = nullptr;      // dtype, rs_nslots (+ pad)
  // bandwidth-reducing renumbering (round 5): every image holds P A P^T
  // (row r of the images is the caller's row perm[r], rows' entries in their
  // stored order), and the solvers work in that numbering; vectors cross the
  // C-ABI in the caller's numbering (kry_*_start permutes b / x0 / weights in,
  // kry_*_get / kry_gmres_xk_device / kry_spmv permute results out).
  bool renumbered = false;
  std::vector<int32_t> perm_host;  // new -> old (preconditioners built "like" this operator reuse it)
  uint64_t perm_hash = 0;          // preconditioners must carry the same renumbering
  int64_t rcm_levels = 0;
  void *perm = nullptr;            // int32, n: new -> old
  void *iperm = nullptr;           // int32, n: old -> new
  // CSR arrays, kept on the device only when irregular slices exist
  void *indptr = nullptr;
  void *indices = nullptr;
  void *data = nullptr;
};

struct kry_vec {
  kry_ctx *ctx = nullptr;
  int64_t n = 0;
  int32_t k = 1;
  int dtype = 0;
  void *d = nullptr;  // n*k elements, allocation padded to 16 elements
  size_t bytes() const { return (size_t)n * k * (dtype == KRY_F64 ? 8 : 4); }
};

namespace kry {

inline size_t dsize(int dtype) { return dtype == KRY_F64 ? 8 : 4; }
inline size_t isize(int itype) { return itype == KRY_I64 ? 8 : 4; }

void *dev_alloc(size_t bytes);
void dev_free(void *p);  // to the caching pool (abi_core.hip)
void mem_stats(int64_t *out);
void mem_release();
double *ctx_scratch(kry_ctx *ctx, size_t bytes);  // grown on demand, owned by the context
// Renumbered operators (kry_csr::renumbered): rows of an n x k block moved
// between the caller's numbering and the operator's. to_op: dst[r] = src[perm[r]]
// (into the operator's numbering); otherwise dst[o] = src[iperm[o]]. Both are
// gathers (no scatter races). Plain copies when A is not renumbered.
void permute_rows(const kry_csr *A, const void *src, void *dst, int k, size_t esize, bool to_op, hipStream_t st);
// The solver-start form: a caller-numbered block into solver storage.
void load_in(const kry_csr *A, const void *src, void *dst, int k, size_t esize, hipStream_t st);
// The get form: solver storage (operator numbering) to a host buffer in the
// caller's numbering (through a temporary device block when renumbered).
void store_out(const kry_csr *A, const void *src, void *host, int k, size_t esize, hipStream_t st);
// A synchronous host <-> device copy; from 4 MB on through the caller's
// pages pinned in place for the copy (hipHostRegister), so the DMA engine
// reads / writes them directly at the link rate instead of a pageable copy
// staged through a bounce buffer by host memcpy (28-56 GB/s by box). Pages
// that cannot be registered take the pageable path. KRY_HOST_PIN=0: always
// pageable.
void host_xfer(void *dst, const void *src, size_t bytes, hipMemcpyKind kind, hipStream_t st);
// true when the environment variable is set to 0 (a default-on switch turned off)
bool env_off(const char *name);
// Device-side image build (device_build.hip; int32 CSR): uploads the CSR
// arrays, validates them, builds SELL-64 (+ compact) and the DIA image.
// Returns 0: nothing built (scattered and renumber_candidates: the
// renumbering path takes over); 1: SELL-64 and DIA built; 2: SELL-64 built,
// no DIA (refused as dia_build refuses); 3: SELL-64 built, the DIA decision
// left to the host builder (a slice beyond the kernel's LDS capacity).
struct DeviceCsrFlags {
  bool strictly_sorted = false, sorted = false, scattered = false;
};
template <typename MV>
int device_image_build(kry_csr *A, const int32_t *ip, const int32_t *ix, const MV *dv, bool renumber_candidates,
                       DeviceCsrFlags *out);
// Reverse Cuthill-McKee on the device over device CSR arrays (renumber.hip):
// 1 built, 0 refused (a level wider than wlimit), -1 gave up (too many
// components: use the host order, host_image.hpp rcm_order, the same order).
int rcm_order_device(kry_ctx *ctx, int64_t n, const int32_t *d_ip, const int32_t *d_ix, int64_t wlimit,
                     std::vector<int32_t> &perm, int64_t *levels);

// Event-timed launch bracket used by the solvers around their SpMV launches.
struct ProfScope {
  kry_ctx *ctx;
  int id;
  hipEvent_t e1 = nullptr;
  ProfScope(kry_ctx *c, int kernel_id);
  ~ProfScope();
};

enum { PROF_SPMV = 0, PROF_UPDATE = 1, PROF_MGS = 2, PROF_OTHER = 3 };

}  // namespace kry
