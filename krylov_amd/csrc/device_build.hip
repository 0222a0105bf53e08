// Operator images built on the device (round 5): kry_csr_create uploads the
// caller's CSR arrays once (indptr, indices, values: 1.8 GB at the metric,
// ~33 ms of H2D) and builds the SELL-64 image (with its compact uint16 column
// form) and the SELL-128 diagonal-offset image with kernels, instead of the
// threaded host passes (0.6-0.9 s at the metric, round 4). The images are
// byte for byte the host builders' (host_image.cpp sell_plan / sell_fill /
// compact_fill / dia_build stay the definition and the test oracle:
// kry_csr_compare, tests/test_gpu_device_build.py).
//
//   csr_check_kernel   one thread per row: indptr monotone, columns in
//                      [0, n), rows strictly sorted (DIA), rows sorted (the
//                      column-blocked test), entries far from the diagonal
//   sell_plan_kernel   one wave per 64-row slice: width (longest row) or
//                      irregular (-1), slots
//   sell_fill_kernel   one wave per slice: slot columns of indices and
//                      values, and per slot column the compact base (wave
//                      min) and deltas; a span over 65534 disables compact
//   dia_offsets_kernel one block per 128-row slice: the slice's column
//                      offsets sorted (bitonic, in LDS) and made unique
//   dia_fill_kernel    one block per slice: each entry's slot column by
//                      binary search, its lane-mask bit (LDS atomicOr), its
//                      value
// Slot pointers are exclusive scans of the per-slice slot counts
// (hipcub::DeviceScan). Vector atomics only.
#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "host_image.hpp"
#include "objects.hpp"

namespace kry {
namespace {

constexpr int kDb = 256;
constexpr int kDiaWMax = 64;       // offsets per slice kept between the two DIA passes
constexpr int kDiaLdsEnt = 8192;   // a slice's entries sorted in LDS (more: no DIA image)

enum : unsigned {
  F_INDPTR = 1u,      // indptr decreases
  F_RANGE = 2u,       // a column outside [0, n)
  F_UNSORTED = 4u,    // a row not strictly increasing (no DIA)
  F_UNSORTED_NS = 8u  // a row decreasing somewhere (no column-blocked image)
};

__global__ __launch_bounds__(kDb) void csr_check_kernel(int64_t n, int64_t nnz, const int32_t *__restrict__ ip,
                                                        const int32_t *__restrict__ ix, int64_t half, unsigned *flags,
                                                        unsigned long long *far) {
  unsigned f = 0;
  unsigned long long fa = 0;
  for (int64_t r = (int64_t)blockIdx.x * kDb + threadIdx.x; r < n; r += (int64_t)gridDim.x * kDb) {
    const int32_t e0 = ip[r], e1 = ip[r + 1];
    if (e1 < e0 || e0 < 0 || (int64_t)e1 > nnz) {  // never read outside indices[0, nnz)
      f |= F_INDPTR;
      continue;
    }
    int32_t prev = INT32_MIN;
    for (int32_t e = e0; e < e1; ++e) {
      const int32_t c = ix[e];
      if (c < 0 || (int64_t)c >= n) f |= F_RANGE;
      if (e > e0 && c <= prev) f |= F_UNSORTED;
      if (e > e0 && c < prev) f |= F_UNSORTED_NS;
      prev = c;
      const int64_t d = (int64_t)c - r;
      fa += (d > half || d < -half) ? 1u : 0u;
    }
  }
  if (f) atomicOr(flags, f);
  if (fa) atomicAdd(far, fa);
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

// SELL-64 plan (host_image.cpp sell_plan): one wave per slice
__global__ __launch_bounds__(kDb) void sell_plan_kernel(int64_t n, int64_t ns, const int32_t *__restrict__ ip,
                                                        int *width, long long *slots, unsigned long long *nirr,
                                                        int *maxw) {
  const int lane = threadIdx.x & 63;
  const int64_t s = ((int64_t)blockIdx.x * kDb + threadIdx.x) >> 6;
  if (s >= ns) return;
  const int64_t r = s * kSlice + lane;
  const int len = r < n ? ip[r + 1] - ip[r] : 0;
  const int w = wave_max_i(len);
  if (lane == 0) {
    const int64_t r0 = s * kSlice, r1 = r0 + kSlice < n ? r0 + kSlice : n;
    const int64_t snnz = (int64_t)ip[r1] - (int64_t)ip[r0];
    const bool irregular = (int64_t)kSlice * w > 2 * snnz + 1024 || w > (1 << 30);
    width[s] = irregular ? -1 : w;
    slots[s] = irregular ? 0 : (long long)kSlice * w;
    if (irregular) atomicAdd(nirr, 1ull);
    atomicMax(maxw, irregular ? -1 : w);
  }
}

// SELL-64 fill + compact image (sell_fill / compact_fill): one wave per slice
template <typename MV>
__global__ __launch_bounds__(kDb) void sell_fill_kernel(int64_t n, int64_t ns, const int32_t *__restrict__ ip,
                                                        const int32_t *__restrict__ ix, const MV *__restrict__ dv,
                                                        const long long *__restrict__ sptr, const int *__restrict__ width,
                                                        int32_t *sidx, MV *sval, uint16_t *sdelta, int32_t *scbase,
                                                        unsigned *nocompact) {
  const int lane = threadIdx.x & 63;
  const int64_t s = ((int64_t)blockIdx.x * kDb + threadIdx.x) >> 6;
  if (s >= ns) return;
  const int w = width[s];
  if (w <= 0) return;
  const int64_t base = sptr[s];
  const int64_t r = s * kSlice + lane;
  const int len = r < n ? ip[r + 1] - ip[r] : 0;
  const int64_t e0 = r < n ? ip[r] : 0;
  bool span_ok = true;
  for (int j = 0; j < w; ++j) {
    const bool valid = j < len;
    const int32_t c = valid ? ix[e0 + j] : -1;
    const int64_t q = base + (int64_t)j * kSlice + lane;
    sidx[q] = c;
    sval[q] = valid ? dv[e0 + j] : MV(0);
    int mn = wave_min_i(valid ? c : INT32_MAX);
    const int mx = wave_max_i(valid ? c : -1);
    if (mx < 0) mn = 0;
    if (mx - mn > 65534) span_ok = false;
    if (lane == 0) scbase[base / kSlice + j] = mn;
    sdelta[q] = valid ? (uint16_t)(c - mn) : (uint16_t)0xFFFF;
  }
  if (!span_ok && lane == 0) atomicOr(nocompact, 1u);
}

template <typename T>
__global__ __launch_bounds__(kDb) void fill_kernel(T *a, int64_t count, T v) {
  for (int64_t i = (int64_t)blockIdx.x * kDb + threadIdx.x; i < count; i += (int64_t)gridDim.x * kDb) a[i] = v;
}

// DIA pass 1 (dia_build): one block per 128-row slice; the slice's offsets
// col - row sorted and made unique in LDS
__global__ __launch_bounds__(kDb) void dia_offsets_kernel(int64_t n, int64_t ns, const int32_t *__restrict__ ip,
                                                          const int32_t *__restrict__ ix, int *width, int *offs,
                                                          long long *slots, unsigned *fail, int *maxw) {
  __shared__ int buf[kDiaLdsEnt];
  __shared__ int pre[kDb];
  const int64_t s = blockIdx.x;
  const int t = threadIdx.x;
  const int64_t r0 = s * kDiaSlice, r1 = r0 + kDiaSlice < n ? r0 + kDiaSlice : n;
  const int32_t b0 = ip[r0];
  const int snnz = ip[r1] - b0;
  if (snnz > kDiaLdsEnt) {  // beyond this kernel's LDS: the host builder decides
    if (t == 0) atomicOr(fail, 2u);
    return;
  }
  int m = 1;
  while (m < snnz) m <<= 1;
  for (int i = t; i < m; i += kDb) buf[i] = INT32_MAX;
  __syncthreads();
  for (int64_t r = r0 + t; r < r1; r += kDb)
    for (int32_t e = ip[r]; e < ip[r + 1]; ++e) buf[e - b0] = (int)((int64_t)ix[e] - r);
  __syncthreads();
  for (int k = 2; k <= m; k <<= 1)  // bitonic sort, ascending
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < m; i += kDb) {
        const int p = i ^ j;
        if (p > i) {
          const int a = buf[i], b = buf[p];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            buf[i] = b;
            buf[p] = a;
          }
        }
      }
      __syncthreads();
    }
  // unique: entry i starts a new offset when it differs from i - 1; ranks by
  // a block scan over chunks of kDb
  int total = 0;
  for (int c0 = 0; c0 < snnz; c0 += kDb) {
    const int i = c0 + t;
    const int head = (i < snnz && (i == 0 || buf[i] != buf[i - 1])) ? 1 : 0;
    pre[t] = head;
    __syncthreads();
    for (int d = 1; d < kDb; d <<= 1) {
      const int v = t >= d ? pre[t - d] : 0;
      __syncthreads();
      pre[t] += v;
      __syncthreads();
    }
    const int rank = total + pre[t] - head;
    if (head && rank < kDiaWMax) offs[s * kDiaWMax + rank] = buf[i];
    const int add = pre[kDb - 1];
    __syncthreads();
    total += add;
  }
  if (t == 0) {
    if ((int64_t)total * kDiaSlice > 2 * (int64_t)snnz + 2048) atomicOr(fail, 1u);  // dia_build's refusal
    else if (total > kDiaWMax) atomicOr(fail, 2u);  // fits dia_build, not this kernel: the host builder decides
    width[s] = total;
    slots[s] = (long long)kDiaSlice * total;
    atomicMax(maxw, total);
  }
}

// DIA pass 2: one block per slice: slot column by binary search, lane mask
// bits in LDS, values (holes stay 0 from the fill before)
template <typename MV>
__global__ __launch_bounds__(kDb) void dia_fill_kernel(int64_t n, const int32_t *__restrict__ ip,
                                                       const int32_t *__restrict__ ix, const MV *__restrict__ dv,
                                                       const long long *__restrict__ sptr, const int *__restrict__ width,
                                                       const int *__restrict__ offs, int32_t *doff, uint64_t *dmask,
                                                       MV *dval) {
  __shared__ int o[kDiaWMax];
  __shared__ unsigned long long msk[2 * kDiaWMax];
  const int64_t s = blockIdx.x;
  const int t = threadIdx.x;
  const int w = width[s];
  const int64_t base = sptr[s];
  const int64_t c0 = base / kDiaSlice;
  if (t < w) o[t] = offs[s * kDiaWMax + t];
  if (t < 2 * kDiaWMax) msk[t] = 0ull;
  __syncthreads();
  const int64_t r0 = s * kDiaSlice;
  if (t < kDiaSlice && r0 + t < n) {
    const int64_t r = r0 + t;
    for (int32_t e = ip[r]; e < ip[r + 1]; ++e) {
      const int off = (int)((int64_t)ix[e] - r);
      int lo = 0, hi = w;  // first o[j] >= off (present: the list holds every offset of the slice)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (o[mid] < off) lo = mid + 1;
        else hi = mid;
      }
      atomicOr(&msk[2 * lo + (t & 1)], 1ull << (t >> 1));
      dval[base + (int64_t)lo * kDiaSlice + t] = dv[e];
    }
  }
  __syncthreads();
  if (t < w) {
    doff[c0 + t] = o[t];
    dmask[2 * (c0 + t)] = msk[2 * t];
    dmask[2 * (c0 + t) + 1] = msk[2 * t + 1];
  }
}

int grid_for_n(int64_t items, int per_block) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(1 << 20, (items + per_block - 1) / per_block));
}

// exclusive scan of cnt[0, m) into out[0, m] (out[m] = total)
void exclusive_scan(const long long *cnt, long long *out, int64_t m, hipStream_t st) {
  size_t tb = 0;
  KRY_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, out, (int)(m + 1), st));
  void *tmp = dev_alloc(tb + 16);
  try {
    KRY_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, out, (int)(m + 1), st));
  } catch (...) {
    dev_free(tmp);
    throw;
  }
  dev_free(tmp);
}

struct Tmp {
  void *p = nullptr;
  explicit Tmp(size_t b) : p(dev_alloc(b)) {}
  ~Tmp() { dev_free(p); }
  Tmp(const Tmp &) = delete;
  Tmp &operator=(const Tmp &) = delete;
  template <class T>
  T *as() const {
    return static_cast<T *>(p);
  }
  void *release() {
    void *q = p;
    p = nullptr;
    return q;
  }
};

template <typename T>
T read1(const T *d, hipStream_t st) {
  T v;
  KRY_HIP(hipMemcpyAsync(&v, d, sizeof(T), hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  return v;
}

}  // namespace

template <typename MV>
int device_image_build(kry_csr *A, const int32_t *ip, const int32_t *ix, const MV *dv, bool renumber_candidates,
                       DeviceCsrFlags *out) {
  hipStream_t st = A->ctx->stream;
  const int64_t n = A->n, nnz = A->nnz;
  KRY_REQUIRE(ip[0] == 0 && (int64_t)ip[n] == nnz, KRY_EINVAL, "indptr must start at 0 and end at nnz");
  // the caller's CSR, once
  Tmp dip((size_t)(n + 1) * 4 + 16), dix((size_t)nnz * 4 + 16), ddv((size_t)nnz * sizeof(MV) + 16);
  host_xfer(dip.p, ip, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, st);
  host_xfer(dix.p, ix, (size_t)nnz * 4, hipMemcpyHostToDevice, st);
  host_xfer(ddv.p, dv, (size_t)nnz * sizeof(MV), hipMemcpyHostToDevice, st);
  Tmp small(256);
  KRY_HIP(hipMemsetAsync(small.p, 0, 256, st));
  unsigned *flags = small.as<unsigned>();
  unsigned long long *far = reinterpret_cast<unsigned long long *>(small.as<char>() + 16);
  const int64_t cols = std::max<int64_t>(int64_t(1) << 18, (n + 15) / 16);
  hipLaunchKernelGGL(csr_check_kernel, dim3(grid_for_n(n, kDb)), dim3(kDb), 0, st, n, nnz, dip.as<int32_t>(),
                     dix.as<int32_t>(), cols / 2, flags, far);
  KRY_HIP(hipGetLastError());
  const unsigned f = read1(flags, st);
  const unsigned long long nfar = read1(far, st);
  KRY_REQUIRE(!(f & F_INDPTR), KRY_EINVAL, "indptr must be non-decreasing");
  KRY_REQUIRE(!(f & F_RANGE), KRY_EINVAL, "column index out of range [0, n)");
  out->strictly_sorted = !(f & F_UNSORTED);
  out->sorted = !(f & F_UNSORTED_NS);
  out->scattered = n * 8 >= (int64_t(8) << 20) && nnz > 0 && (int64_t)nfar * 4 >= nnz;
  if (out->scattered && renumber_candidates) return 0;  // the renumbering path (host images)
  // ---- SELL-64 (+ compact)
  const int64_t ns = (n + kSlice - 1) / kSlice;
  Tmp cnt((size_t)(ns + 1) * 8 + 16);
  KRY_HIP(hipMemsetAsync(cnt.p, 0, (size_t)(ns + 1) * 8, st));
  void *swidth = dev_alloc((size_t)ns * 4 + 4);
  A->swidth = swidth;
  unsigned long long *nirr = reinterpret_cast<unsigned long long *>(small.as<char>() + 32);
  int *maxw = reinterpret_cast<int *>(small.as<char>() + 48);
  fill_kernel<int><<<1, 1, 0, st>>>(maxw, 1, -1);
  hipLaunchKernelGGL(sell_plan_kernel, dim3(grid_for_n(ns * 64, kDb)), dim3(kDb), 0, st, n, ns, dip.as<int32_t>(),
                     static_cast<int *>(swidth), cnt.as<long long>(), nirr, maxw);
  A->sptr = dev_alloc((size_t)(ns + 1) * 8);
  exclusive_scan(cnt.as<long long>(), static_cast<long long *>(A->sptr), ns, st);
  A->nslices = ns;
  A->nslots = read1(static_cast<const long long *>(A->sptr) + ns, st);
  A->nirregular = (int64_t)read1(nirr, st);
  A->max_width = read1(maxw, st);
  const int64_t slots = A->nslots;
  Tmp sidx((size_t)(slots + 256) * 4);
  A->sval = dev_alloc((size_t)(slots + 256) * sizeof(MV));
  Tmp sdelta((size_t)(slots + 256) * 2 + 16);
  Tmp scbase((size_t)(slots / kSlice + 16) * 4);
  fill_kernel<int32_t><<<grid_for_n(slots + 256, kDb), kDb, 0, st>>>(sidx.as<int32_t>(), slots + 256, -1);
  fill_kernel<MV><<<grid_for_n(slots + 256, kDb), kDb, 0, st>>>(static_cast<MV *>(A->sval), slots + 256, MV(0));
  fill_kernel<uint16_t><<<grid_for_n(slots + 256, kDb), kDb, 0, st>>>(sdelta.as<uint16_t>(), slots + 256, (uint16_t)0xFFFF);
  KRY_HIP(hipMemsetAsync(scbase.p, 0, (size_t)(slots / kSlice + 16) * 4, st));
  unsigned *nocompact = small.as<unsigned>() + 16;
  if (slots > 0)
    hipLaunchKernelGGL(sell_fill_kernel<MV>, dim3(grid_for_n(ns * 64, kDb)), dim3(kDb), 0, st, n, ns, dip.as<int32_t>(),
                       dix.as<int32_t>(), ddv.as<MV>(), static_cast<const long long *>(A->sptr),
                       static_cast<const int *>(swidth), sidx.as<int32_t>(), static_cast<MV *>(A->sval),
                       sdelta.as<uint16_t>(), scbase.as<int32_t>(), nocompact);
  KRY_HIP(hipGetLastError());
  const char *cenv = getenv("KRY_SELL_COMPACT");
  A->compact = !(cenv && atoi(cenv) == 0) && slots > 0 && read1(nocompact, st) == 0;
  if (A->compact) {
    A->sdelta = sdelta.release();
    A->scbase = scbase.release();
  } else {
    A->sidx = sidx.release();
  }
  // ---- SELL-128 diagonal-offset image
  const char *denv = getenv("KRY_SPMV_DIA");
  bool dia = out->strictly_sorted && !(denv && atoi(denv) == 0) && n > 0;
  bool host_dia = false;
  if (dia) {
    const int64_t dns = (n + kDiaSlice - 1) / kDiaSlice;
    unsigned *dfail = small.as<unsigned>() + 20;
    int *dmaxw = reinterpret_cast<int *>(small.as<char>() + 96);
    Tmp dcnt((size_t)(dns + 1) * 8 + 16), offs((size_t)dns * kDiaWMax * 4 + 16);
    KRY_HIP(hipMemsetAsync(dcnt.p, 0, (size_t)(dns + 1) * 8, st));
    Tmp dwidth((size_t)dns * 4 + 4);
    hipLaunchKernelGGL(dia_offsets_kernel, dim3((unsigned)dns), dim3(kDb), 0, st, n, dns, dip.as<int32_t>(),
                       dix.as<int32_t>(), dwidth.as<int>(), offs.as<int>(), dcnt.as<long long>(), dfail, dmaxw);
    KRY_HIP(hipGetLastError());
    const unsigned df = read1(dfail, st);
    if (df & 1u) dia = false;  // refused, as dia_build would
    if (!(df & 1u) && (df & 2u)) host_dia = true;
    if (df == 0) {
      Tmp dsptr((size_t)(dns + 1) * 8);
      exclusive_scan(dcnt.as<long long>(), dsptr.as<long long>(), dns, st);
      const int64_t dslots = read1(dsptr.as<long long>() + dns, st);
      const int dmw = read1(dmaxw, st);
      // the 128-row slices may hold up to one slice more padding than SELL-64's
      if (!(dslots * 4 > slots * 5 + (int64_t)4 * kDiaSlice * dmw)) {
        const int64_t dcols = dslots / kDiaSlice;
        Tmp doff((size_t)(dcols + kDiaPad) * 4), dmask((size_t)2 * (dcols + kDiaPad) * 8),
            dval((size_t)(dslots + 2 * kDiaSlice) * sizeof(MV));
        KRY_HIP(hipMemsetAsync(doff.p, 0, (size_t)(dcols + kDiaPad) * 4, st));
        KRY_HIP(hipMemsetAsync(dmask.p, 0, (size_t)2 * (dcols + kDiaPad) * 8, st));
        KRY_HIP(hipMemsetAsync(dval.p, 0, (size_t)(dslots + 2 * kDiaSlice) * sizeof(MV), st));
        hipLaunchKernelGGL(dia_fill_kernel<MV>, dim3((unsigned)dns), dim3(kDb), 0, st, n, dip.as<int32_t>(),
                           dix.as<int32_t>(), ddv.as<MV>(), dsptr.as<const long long>(), dwidth.as<const int>(),
                           offs.as<const int>(), doff.as<int32_t>(), dmask.as<uint64_t>(), dval.as<MV>());
        KRY_HIP(hipGetLastError());
        A->dia = true;
        A->dia_nslices = dns;
        A->dia_nslots = dslots;
        A->dia_max_width = dmw;
        A->dia_sptr = dsptr.release();
        A->dia_width = dwidth.release();
        A->dia_off = doff.release();
        A->dia_mask = dmask.release();
        A->dia_val = dval.release();
      }
    }
  }
  if (A->nirregular > 0) {  // the irregular slices walk the CSR arrays: keep them
    A->indptr = dip.release();
    A->indices = dix.release();
    A->data = ddv.release();
  }
  KRY_HIP(hipStreamSynchronize(st));
  return A->dia ? 1 : (host_dia ? 3 : 2);
}

template int device_image_build<double>(kry_csr *, const int32_t *, const int32_t *, const double *, bool,
                                        DeviceCsrFlags *);
template int device_image_build<float>(kry_csr *, const int32_t *, const int32_t *, const float *, bool,
                                       DeviceCsrFlags *);

}  // namespace kry
