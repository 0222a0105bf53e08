// Host-side image builders of kry_csr_create (kry_csr::sptr / dia_* /
// cb_* / sp_*) and the host-only plans the C-ABI exposes (kry_csr_layout,
// kry_dia_plan, kry_pair_plan, kry_cb_plan). Plain C++ (no HIP): compiled by
// host_image.cpp, which the library links, and which `make sanitize` builds
// on its own with -fsanitize=address,undefined and -fsanitize=thread
// (tests/test_host_sanitize.py). Templates are instantiated there for
// int32 / int64 indices and float / double values.
#pragma once

#include <stdint.h>

#include <memory>
#include <utility>
#include <vector>

#include "host_common.hpp"

namespace kry {

// ------------------------------------------------- host staging buffers
// Image staging vectors: no zero-initialisation on resize (std::vector's
// value-initialisation writes every page from one thread), filled in
// parallel instead, so the first touch of the pages is spread over threads.
template <class T>
struct NoInit : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInit<U>;
  };
  NoInit() = default;
  template <class U>
  NoInit(const NoInit<U> &) {}
  template <class U, class... A>
  void construct(U *q, A &&...a) {
    if constexpr (sizeof...(A) == 0) ::new ((void *)q) U;
    else ::new ((void *)q) U(std::forward<A>(a)...);
  }
};
template <class T>
using hvec = std::vector<T, NoInit<T>>;


// Releases a staging vector's pages (on a detached thread above 64 MB, once
// its H2D copies have completed).
template <class T>
void release_later(hvec<T> &v);

// Structural check of a square CSR matrix before any image is built from
// it: indptr[0] = 0, indptr non-decreasing, indptr[n] = nnz, and every column
// index in [0, n). Throws Error{KRY_EINVAL} otherwise (the builders index
// host and device arrays with these values; threaded above 2^20 entries).
template <typename I>
void check_csr(int64_t n, int64_t nnz, const I *ip, const I *ix);

// SELL-64 plan: slice s = rows [64 s, 64 s + 64); width = longest row; a
// slice is irregular (CSR walk) when 64 * width > 2 * nnz_slice + 1024.
template <typename I>
void sell_plan(int64_t n, const I *ip, std::vector<int64_t> *sptr, std::vector<int32_t> *width, int64_t *nslices,
               int64_t *nslots, int64_t *nirr);
template <typename I, typename MV>
void sell_fill(int64_t n, const I *ip, const I *ix, const MV *dv, const std::vector<int64_t> &sptr,
               const std::vector<int32_t> &width, hvec<I> &sidx, hvec<MV> &sval);
// uint16 column deltas over per-slot-column bases; false when a slot column
// spans more than 65534 columns
template <typename I>
bool compact_fill(const std::vector<int64_t> &sptr, const std::vector<int32_t> &width, const hvec<I> &sidx,
                  hvec<uint16_t> &sdelta, std::vector<int32_t> &scbase);

template <typename MV>
struct DiaHost {
  std::vector<int64_t> sptr;
  std::vector<int32_t> width;
  std::vector<int32_t> off;
  hvec<uint64_t> mask;
  hvec<MV> val;
  int max_width = 0;
};

template <typename I, typename MV>
bool dia_build(int64_t n, const I *ip, const I *ix, const MV *dv, int64_t sell_slots, DiaHost<MV> &d);

template <typename MV>
struct CbHost {
  int64_t nb = 0, cols = 0, ng = 0;
  std::vector<int64_t> gptr;
  hvec<uint16_t> roff;
  hvec<int32_t> col;
  hvec<MV> val;
};

template <typename I, typename MV>
bool cb_build(int64_t n, const I *ip, const I *ix, const MV *dv, CbHost<MV> &cb);

template <typename MV>
struct PairHost {
  std::vector<int64_t> sptr;
  std::vector<int32_t> width;
  std::vector<int32_t> cbase;
  hvec<uint16_t> delta;
  hvec<MV> val;
  int max_width = 0;
};

template <typename I, typename MV>
bool pair_build(int64_t n, const I *ip, const I *ix, const MV *dv, int64_t sell_slots, PairHost<MV> &p);

// ------------------------------------------- bandwidth-reducing renumbering
// Reverse Cuthill-McKee order of the row pattern (round 5), for matrices whose
// columns are scattered but whose graph has small level sets (a mesh or
// stencil numbered badly). Deterministic, level-synchronous, threaded:
//  - root: George-Liu pseudo-peripheral node, starting from the lowest-index
//    node of smallest degree; in each BFS's last level the smallest-degree
//    (then lowest-index) node is the next candidate, while the level count
//    grows (at most 4 BFS sweeps);
//  - Cuthill-McKee numbering level by level: the nodes of level k + 1 are
//    ordered by (the smallest number among their level-k neighbours, degree,
//    index), which is the sequential algorithm's order with children of one
//    parent taken by increasing degree;
//  - a node not reached (another component, or no in-edge of a
//    non-symmetric pattern) starts a new BFS at the lowest unnumbered index;
//  - reversed: perm[r] = cm[n - 1 - r] (new row r is old row perm[r]).
// Returns false (no renumbering) as soon as a level holds more than `wlimit`
// nodes: the graph has no narrow level structure (a random matrix), and the
// column-blocked image serves it instead.
template <typename I>
bool rcm_order(int64_t n, const I *ip, const I *ix, int64_t wlimit, std::vector<int32_t> &perm, int64_t *levels);

// The scatter test of the column-blocked image, without the sortedness
// requirement: x over 8 MB and at least a quarter of the entries farther
// than half a block (max(2^18, n / 16) columns) from the diagonal.
template <typename I>
bool scattered(int64_t n, const I *ip, const I *ix);

// P A P^T with every row's entries kept in their stored order (old row perm[r]
// becomes row r, column c becomes iperm[c]): the same per-row summation
// order as the input, so an SpMV over it is bitwise the input's, permuted.
template <typename I, typename MV>
void renumber_csr(int64_t n, const I *ip, const I *ix, const MV *dv, const std::vector<int32_t> &perm,
                  hvec<I> &ip2, hvec<I> &ix2, hvec<MV> &dv2);

// Rank-sorted SELL-128 image (kry_csr::rs_*, spmv_rs_kernel; round 5): the
// paired-row slice geometry (slices of 128 rows, lane l owns rows 2l, 2l + 1)
// with int32 columns, and within every run of kRsChunk consecutive stored
// entries of a row the entries sorted by column, so that slot column j of
// neighbouring rows gathers neighbouring x entries (renumbered or unsorted
// rows). Each slot word packs the column (low 28 bits) and the entry's
// position within its run of stored entries (high 4 bits); the kernel sums a
// run's products back in that stored order: bitwise csr_matvec. Padding:
// 0xFFFFFFFF. Needs n < 2^28 - 1; refused above 1.25x the SELL-64 slots.
template <typename MV>
struct RsHost {
  std::vector<int64_t> sptr;
  std::vector<int32_t> width;
  hvec<uint32_t> colrank;
  hvec<MV> val;
  int max_width = 0;
};
template <typename I, typename MV>
bool rs_build(int64_t n, const I *ip, const I *ix, const MV *dv, int64_t sell_slots, RsHost<MV> &r);

}  // namespace kry
