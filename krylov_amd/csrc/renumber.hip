// Reverse Cuthill-McKee on the device (round 5): the same order as the host
// definition (host_image.hpp rcm_order, which stays the test oracle and the
// fallback), computed level-synchronously on the GPU so that renumbering a
// 10 M-row matrix costs milliseconds, not the seconds of a host BFS whose
// every edge is a random cache miss.
//
// Per BFS level (the George-Liu sweeps and the Cuthill-McKee pass alike) one
// kernel claims the frontier's unvisited neighbours with a compare-and-swap
// and appends them to the next frontier through one counter; the numbering
// pass also keeps, per claimed node, the smallest number among its parents
// (atomicMin) and orders the level by (that number, degree, index): a
// counting sort by parent number (histogram, scan, scatter), then each
// parent's children (a handful) sorted by (degree, index) by one thread.
// Every order is a total order on node ids, so the result is deterministic
// and equal to the host's, node for node (tests/test_gpu_renumber.py).
// Vector atomics only (device-scope global atomics from vector ALUs).
#include <vector>

#include "common.hpp"
#include "host_image.hpp"
#include "objects.hpp"

namespace kry {
namespace {

constexpr int kRb = 256;

__global__ __launch_bounds__(kRb) void rcm_fill_kernel(int32_t *a, int64_t n, int32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * kRb + threadIdx.x; i < n; i += (int64_t)gridDim.x * kRb) a[i] = v;
}

__global__ void rcm_set_kernel(int32_t *a, int64_t i, int32_t v) { a[i] = v; }

// the lowest-index row of smallest degree, packed (degree << 32 | index)
__global__ __launch_bounds__(kRb) void rcm_min_rows_kernel(const int32_t *__restrict__ ip, int64_t n,
                                                           unsigned long long *best) {
  unsigned long long m = ~0ull;
  for (int64_t v = (int64_t)blockIdx.x * kRb + threadIdx.x; v < n; v += (int64_t)gridDim.x * kRb) {
    const unsigned long long key = ((unsigned long long)(uint32_t)(ip[v + 1] - ip[v]) << 32) | (uint32_t)v;
    m = key < m ? key : m;
  }
  atomicMin(best, m);
}

// frontier expansion, levels only: level[w] = next for unvisited neighbours
__global__ __launch_bounds__(kRb) void rcm_expand_kernel(const int32_t *__restrict__ ip, const int32_t *__restrict__ ix,
                                                         const int32_t *__restrict__ front, int32_t nf, int32_t next,
                                                         int32_t *level, int32_t *out, int32_t *cnt) {
  for (int32_t q = blockIdx.x * kRb + threadIdx.x; q < nf; q += gridDim.x * kRb) {
    const int32_t u = front[q];
    for (int32_t e = ip[u]; e < ip[u + 1]; ++e) {
      const int32_t w = ix[e];
      if (__hip_atomic_load(level + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == -1 &&
          atomicCAS(level + w, -1, next) == -1)
        out[atomicAdd(cnt, 1)] = w;
    }
  }
}

// the smallest (degree, index) of a frontier, packed (degree << 32 | index)
__global__ __launch_bounds__(kRb) void rcm_min_kernel(const int32_t *__restrict__ ip, const int32_t *__restrict__ front,
                                                      int32_t nf, unsigned long long *best) {
  unsigned long long m = ~0ull;
  for (int32_t q = blockIdx.x * kRb + threadIdx.x; q < nf; q += gridDim.x * kRb) {
    const int32_t v = front[q];
    const unsigned long long key = ((unsigned long long)(uint32_t)(ip[v + 1] - ip[v]) << 32) | (uint32_t)v;
    m = key < m ? key : m;
  }
  atomicMin(best, m);
}

// Cuthill-McKee claim: children of the level's parents (numbers [a, b) in
// cm): the smallest parent number per child, first toucher appends it
__global__ __launch_bounds__(kRb) void rcm_claim_kernel(const int32_t *__restrict__ ip, const int32_t *__restrict__ ix,
                                                        const int32_t *__restrict__ cm, int32_t a, int32_t b,
                                                        const int32_t *__restrict__ num, int32_t *key, int32_t *out,
                                                        int32_t *cnt) {
  for (int32_t q = a + blockIdx.x * kRb + threadIdx.x; q < b; q += gridDim.x * kRb) {
    const int32_t u = cm[q];
    for (int32_t e = ip[u]; e < ip[u + 1]; ++e) {
      const int32_t w = ix[e];
      if (num[w] >= 0) continue;  // numbered in an earlier level (num is not written during this kernel)
      if (atomicMin(key + w, q) == INT32_MAX) out[atomicAdd(cnt, 1)] = w;
    }
  }
}

__global__ __launch_bounds__(kRb) void rcm_hist_kernel(const int32_t *__restrict__ list, int32_t m,
                                                       const int32_t *__restrict__ key, int32_t a, int32_t *hist) {
  for (int32_t i = blockIdx.x * kRb + threadIdx.x; i < m; i += gridDim.x * kRb) atomicAdd(hist + key[list[i]] - a, 1);
}

// exclusive scan of hist[0, span) into off[] (one block, chunked)
__global__ __launch_bounds__(1024) void rcm_scan_kernel(const int32_t *__restrict__ hist, int32_t span, int32_t *off) {
  __shared__ int32_t s[1024];
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int32_t c0 = 0; c0 < span; c0 += 1024) {
    const int32_t i = c0 + threadIdx.x;
    const int32_t v = i < span ? hist[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
      const int32_t t = threadIdx.x >= d ? s[threadIdx.x - d] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < span) off[i] = carry + s[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += s[1023];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kRb) void rcm_scatter_kernel(const int32_t *__restrict__ list, int32_t m,
                                                          const int32_t *__restrict__ key, int32_t a, int32_t *pos,
                                                          int32_t *sorted) {
  for (int32_t i = blockIdx.x * kRb + threadIdx.x; i < m; i += gridDim.x * kRb) {
    const int32_t w = list[i];
    sorted[atomicAdd(pos + key[w] - a, 1)] = w;
  }
}

// one thread per parent: its children [start, end) by (degree, index); then
// their numbers b + position, and cm
__global__ __launch_bounds__(kRb) void rcm_bucket_kernel(const int32_t *__restrict__ ip, const int32_t *__restrict__ start,
                                                         const int32_t *__restrict__ hist, int32_t span, int32_t *sorted,
                                                         int32_t b, int32_t *num, int32_t *cm) {
  for (int32_t p = blockIdx.x * kRb + threadIdx.x; p < span; p += gridDim.x * kRb) {
    const int32_t c = hist[p];
    if (c == 0) continue;
    int32_t *v = sorted + start[p];
    for (int32_t i = 1; i < c; ++i) {  // insertion sort (a few children)
      const int32_t x = v[i];
      const int32_t dx = ip[x + 1] - ip[x];
      int32_t j = i - 1;
      while (j >= 0) {
        const int32_t y = v[j];
        const int32_t dy = ip[y + 1] - ip[y];
        if (dy < dx || (dy == dx && y < x)) break;
        v[j + 1] = y;
        --j;
      }
      v[j + 1] = x;
    }
    for (int32_t i = 0; i < c; ++i) {
      num[v[i]] = b + start[p] + i;
      cm[b + start[p] + i] = v[i];
    }
  }
}

__global__ __launch_bounds__(kRb) void rcm_first_unnumbered_kernel(const int32_t *__restrict__ num, int64_t from,
                                                                   int64_t n, unsigned long long *best) {
  unsigned long long m = ~0ull;
  for (int64_t i = from + (int64_t)blockIdx.x * kRb + threadIdx.x; i < n; i += (int64_t)gridDim.x * kRb)
    if (num[i] < 0) {
      m = (unsigned long long)i;
      break;  // the grid-stride order: later i of this thread are larger
    }
  atomicMin(best, m);
}

int grid_of(int64_t m) { return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (m + kRb - 1) / kRb)); }

struct DevBuf {
  void *p = nullptr;
  explicit DevBuf(size_t bytes) : p(dev_alloc(bytes)) {}
  ~DevBuf() { dev_free(p); }
  template <class T>
  T *as() const {
    return static_cast<T *>(p);
  }
};

}  // namespace

// 1: built (perm, levels), 0: refused (a level wider than wlimit), -1: gave
// up (more than kMaxComponents components: the host order takes over).
int rcm_order_device(kry_ctx *ctx, int64_t n, const int32_t *d_ip, const int32_t *d_ix, int64_t wlimit,
                     std::vector<int32_t> &perm, int64_t *levels) {
  constexpr int kMaxComponents = 64;
  hipStream_t st = ctx->stream;
  const size_t nb = (size_t)n * 4 + 64;
  DevBuf level(nb), key(nb), buf0(nb), buf1(nb), cm(nb), hist(nb), off(nb), cur(nb), small(64);
  int32_t *cnt = small.as<int32_t>();
  unsigned long long *best = reinterpret_cast<unsigned long long *>(small.as<char>() + 16);
  auto fill = [&](int32_t *a, int64_t m, int32_t v) {
    hipLaunchKernelGGL(rcm_fill_kernel, dim3(grid_of(m)), dim3(kRb), 0, st, a, m, v);
  };
  auto set = [&](int32_t *a, int64_t i, int32_t v) { hipLaunchKernelGGL(rcm_set_kernel, dim3(1), dim3(1), 0, st, a, i, v); };
  auto read_i32 = [&](const int32_t *d) {
    int32_t v;
    KRY_HIP(hipMemcpyAsync(&v, d, 4, hipMemcpyDeviceToHost, st));
    KRY_HIP(hipStreamSynchronize(st));
    return v;
  };
  auto read_u64 = [&](const unsigned long long *d) {
    unsigned long long v;
    KRY_HIP(hipMemcpyAsync(&v, d, 8, hipMemcpyDeviceToHost, st));
    KRY_HIP(hipStreamSynchronize(st));
    return v;
  };
  auto deg_min_root = [&]() -> int32_t {
    KRY_HIP(hipMemsetAsync(best, 0xFF, 8, st));
    hipLaunchKernelGGL(rcm_min_rows_kernel, dim3(grid_of(n)), dim3(kRb), 0, st, d_ip, n, best);
    return (int32_t)(read_u64(best) & 0xffffffffull);
  };
  // levels-only BFS: level count and the last level's min-(degree, index)
  // node; -1 when a level exceeds wlimit
  auto sweep = [&](int32_t root, int32_t *far_node) -> int64_t {
    fill(level.as<int32_t>(), n, -1);
    set(level.as<int32_t>(), root, 0);
    set(buf0.as<int32_t>(), 0, root);
    int32_t *front = buf0.as<int32_t>(), *nxt = buf1.as<int32_t>();
    int32_t nf = 1;
    int64_t nl = 1;
    for (;;) {
      KRY_HIP(hipMemsetAsync(cnt, 0, 4, st));
      hipLaunchKernelGGL(rcm_expand_kernel, dim3(grid_of(nf)), dim3(kRb), 0, st, d_ip, d_ix, front, nf, (int32_t)nl,
                         level.as<int32_t>(), nxt, cnt);
      const int32_t m = read_i32(cnt);
      if (m == 0) break;
      if (m > wlimit) return -1;
      std::swap(front, nxt);
      nf = m;
      ++nl;
    }
    KRY_HIP(hipMemsetAsync(best, 0xFF, 8, st));
    hipLaunchKernelGGL(rcm_min_kernel, dim3(grid_of(nf)), dim3(kRb), 0, st, d_ip, front, nf, best);
    *far_node = (int32_t)(read_u64(best) & 0xffffffffull);
    return nl;
  };
  int32_t root = deg_min_root();
  int32_t cand = root;
  int64_t ecc = sweep(root, &cand);
  if (ecc < 0) return 0;
  static const int max_sweeps = [] {
    const char *e = getenv("KRY_RCM_SWEEPS");
    return e ? std::max(0, atoi(e)) : 3;
  }();
  for (int it = 0; it < max_sweeps && cand != root; ++it) {
    int32_t c2 = cand;
    const int64_t e2 = sweep(cand, &c2);
    if (e2 < 0) return 0;
    if (e2 <= ecc) break;
    root = cand;
    ecc = e2;
    cand = c2;
  }
  // Cuthill-McKee numbering (num = level buffer reused), key = smallest parent
  int32_t *num = level.as<int32_t>(), *ky = key.as<int32_t>();
  fill(num, n, -1);
  fill(ky, n, INT32_MAX);
  int64_t done = 0, nlev = 0, scan_from = 0;
  int components = 0;
  while (done < n) {
    if (++components > kMaxComponents) return -1;
    int32_t r0 = root;
    if (done > 0) {
      KRY_HIP(hipMemsetAsync(best, 0xFF, 8, st));
      hipLaunchKernelGGL(rcm_first_unnumbered_kernel, dim3(grid_of(n - scan_from)), dim3(kRb), 0, st, num, scan_from, n,
                         best);
      r0 = (int32_t)read_u64(best);
      scan_from = r0;
    }
    set(num, r0, (int32_t)done);
    set(cm.as<int32_t>(), done, r0);
    int32_t a = (int32_t)done, b = (int32_t)done + 1;
    ++nlev;
    for (;;) {
      KRY_HIP(hipMemsetAsync(cnt, 0, 4, st));
      hipLaunchKernelGGL(rcm_claim_kernel, dim3(grid_of(b - a)), dim3(kRb), 0, st, d_ip, d_ix, cm.as<int32_t>(), a, b,
                         num, ky, buf0.as<int32_t>(), cnt);
      const int32_t m = read_i32(cnt);
      if (m == 0) break;
      if (m > wlimit) return 0;
      const int32_t span = b - a;
      KRY_HIP(hipMemsetAsync(hist.p, 0, (size_t)span * 4, st));
      hipLaunchKernelGGL(rcm_hist_kernel, dim3(grid_of(m)), dim3(kRb), 0, st, buf0.as<int32_t>(), m, ky, a,
                         hist.as<int32_t>());
      hipLaunchKernelGGL(rcm_scan_kernel, dim3(1), dim3(1024), 0, st, hist.as<int32_t>(), span, off.as<int32_t>());
      // scatter through a copy of the offsets (cursors); buf1: the sorted children
      KRY_HIP(hipMemcpyAsync(cur.p, off.p, (size_t)span * 4, hipMemcpyDeviceToDevice, st));
      hipLaunchKernelGGL(rcm_scatter_kernel, dim3(grid_of(m)), dim3(kRb), 0, st, buf0.as<int32_t>(), m, ky, a,
                         cur.as<int32_t>(), buf1.as<int32_t>());
      hipLaunchKernelGGL(rcm_bucket_kernel, dim3(grid_of(span)), dim3(kRb), 0, st, d_ip, off.as<int32_t>(),
                         hist.as<int32_t>(), span, buf1.as<int32_t>(), b, num, cm.as<int32_t>());
      KRY_HIP(hipGetLastError());
      a = b;
      b += m;
      ++nlev;
    }
    done = b;
  }
  std::vector<int32_t> h(n);
  KRY_HIP(hipMemcpyAsync(h.data(), cm.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  perm.resize(n);
  for (int64_t r = 0; r < n; ++r) perm[r] = h[n - 1 - r];
  if (levels) *levels = nlev;
  return 1;
}

}  // namespace kry

using namespace kry;

#define KRY_API_BEGIN try {
#define KRY_API_END                  \
  return KRY_OK;                     \
  }                                  \
  catch (const kry::Error &e) {      \
    kry::set_error(e.msg);           \
    return e.code;                   \
  }                                  \
  catch (const std::exception &e) {  \
    kry::set_error(e.what());        \
    return KRY_EDEVICE;              \
  }

extern "C" {

int kry_rcm_device(kry_ctx *ctx, int64_t n, int64_t nnz, const int32_t *indptr, const int32_t *indices, int64_t wlimit,
                   int64_t *info, int32_t *perm) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && indptr && info && n >= 1 && nnz >= 0 && (nnz == 0 || indices), KRY_EINVAL, "bad argument");
  KRY_REQUIRE(n < (int64_t(1) << 31) - 1 && nnz < (int64_t(1) << 31), KRY_EINVAL, "int32 indices only");
  check_csr(n, nnz, indptr, indices);
  KRY_HIP(hipSetDevice(ctx->device));
  const int64_t wl = wlimit > 0 ? wlimit : std::max<int64_t>(int64_t(1) << 16, n / 32);
  void *dip = dev_alloc((size_t)(n + 1) * 4);
  void *dix = dev_alloc((size_t)std::max<int64_t>(nnz, 1) * 4);
  std::vector<int32_t> p;
  int64_t levels = 0;
  int r = 0;
  try {
    KRY_HIP(hipMemcpyAsync(dip, indptr, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, ctx->stream));
    if (nnz) KRY_HIP(hipMemcpyAsync(dix, indices, (size_t)nnz * 4, hipMemcpyHostToDevice, ctx->stream));
    r = rcm_order_device(ctx, n, static_cast<const int32_t *>(dip), static_cast<const int32_t *>(dix), wl, p, &levels);
  } catch (...) {
    dev_free(dip);
    dev_free(dix);
    throw;
  }
  dev_free(dip);
  dev_free(dix);
  info[0] = r;
  info[1] = r == 1 ? levels : 0;
  if (r == 1 && perm) std::copy(p.begin(), p.end(), perm);
  KRY_API_END
}

}  // extern "C"
