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

}  // namespace kry
