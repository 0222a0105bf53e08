// C-ABI: library, context, CSR operator, vectors, primitives, timers.
#include <algorithm>
#include <atomic>
#include <climits>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <chrono>
#include <unordered_map>

#include "device.hpp"
#include "host_image.hpp"

using namespace kry;

namespace kry {

// Every device buffer carries kAllocSlack bytes of readable slack before and
// after it: the diagonal-offset SpMV loads x[j], x[j + 1] as one pair even
// when one of them is a masked-off hole at j = -1 or j + 1 = n (the value is
// never used, the address only has to be mapped).
constexpr size_t kAllocSlack = 256;

// ------------------------------------------------ caching device allocator
// A solve allocates its vectors (and GMRES its m + 1 basis vectors: 2.5 GB
// at the metric) when the solver state is created and frees them when it is
// destroyed, once per reference-API call. hipMalloc / hipFree of buffers
// that size cost milliseconds each and hipFree synchronises the device, so
// freed blocks are kept per (device, rounded size) and handed out again.
// A freed block first goes to a pending list: it may still be read by work
// queued on any stream. It is reused only after one hipDeviceSynchronize
// retires the whole pending list (in practice the device is idle by then:
// the solve's results have been downloaded). On hipMalloc failure every
// cached block is released and the allocation retried once.
// KRYLOV_ALLOC_CACHE=0 restores plain hipMalloc / hipFree.
namespace {

struct BlockKey {
  int device;
  size_t bytes;
  bool operator<(const BlockKey &o) const { return device != o.device ? device < o.device : bytes < o.bytes; }
};

struct DevicePool {
  std::mutex mu;
  std::multimap<BlockKey, char *> free_blocks;           // reusable now
  std::vector<std::pair<BlockKey, char *>> pending;      // freed, maybe still in use by queued work
  std::unordered_map<char *, BlockKey> live;             // handed out (allocation base -> key)
  size_t cached_bytes = 0, live_bytes = 0;
  int64_t hits = 0, misses = 0, syncs = 0;
};

DevicePool &pool() {
  static DevicePool *p = new DevicePool;  // never destroyed: frees may run from static destructors
  return *p;
}

bool cache_enabled() {
  static const bool on = [] {
    const char *e = getenv("KRYLOV_ALLOC_CACHE");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// Bytes the cache may hold (KRYLOV_ALLOC_CACHE_MAX_GB, default 16 of the
// 288 GB: every state of the BASELINE configurations, the metric GMRES(30)
// basis of 2.5 GB included, several times over; other allocators in the
// process see the rest): a larger free goes straight back to the runtime.
size_t cache_cap() {
  static const size_t cap = [] {
    const char *e = getenv("KRYLOV_ALLOC_CACHE_MAX_GB");
    const double gb = e ? atof(e) : 16.0;
    return (size_t)(gb > 0 ? gb * 1e9 : 0);
  }();
  return cap;
}

// 4 KiB granules below 64 KiB (control words, scalars, partials), 64 KiB
// below 2 MiB, 2 MiB above (the HBM page size the runtime maps large buffers
// with): a reused block wastes < 4 KiB / 64 KiB / 2 MiB.
size_t round_alloc(size_t total) {
  const size_t g = total < ((size_t)64 << 10)  ? ((size_t)4 << 10)
                   : total < ((size_t)2 << 20) ? ((size_t)64 << 10)
                                               : ((size_t)2 << 20);
  return (total + g - 1) / g * g;
}

// Caller holds the lock, with `dev` the current device. Moves the device's
// pending blocks to the free list after it has finished all queued work
// (other devices' pending blocks stay: this sync says nothing about them).
void retire_pending(DevicePool &P, int dev) {
  (void)hipDeviceSynchronize();
  ++P.syncs;
  size_t keep = 0;
  for (size_t i = 0; i < P.pending.size(); ++i) {
    if (P.pending[i].first.device == dev) P.free_blocks.emplace(P.pending[i].first, P.pending[i].second);
    else P.pending[keep++] = P.pending[i];
  }
  P.pending.resize(keep);
}

// Caller holds the lock. hipFree of every cached (free or pending) block
// (hipFree waits for the block's device to finish its queued work).
void release_cached(DevicePool &P) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto &b : P.pending) P.free_blocks.emplace(b.first, b.second);
  P.pending.clear();
  for (auto &b : P.free_blocks) {
    (void)hipSetDevice(b.first.device);
    (void)hipFree(b.second);
  }
  (void)hipSetDevice(cur);
  P.free_blocks.clear();
  P.cached_bytes = 0;
}

}  // namespace

void *dev_alloc(size_t bytes) {
  if (bytes == 0) bytes = 16;
  void *p = nullptr;
  if (!cache_enabled()) {
    hipError_t e = hipMalloc(&p, bytes + 2 * kAllocSlack);
    if (e != hipSuccess)
      throw Error{e == hipErrorOutOfMemory ? KRY_ENOMEM : KRY_EDEVICE,
                  std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e)};
    return static_cast<char *>(p) + kAllocSlack;
  }
  int dev = 0;
  KRY_HIP(hipGetDevice(&dev));
  const BlockKey key{dev, round_alloc(bytes + 2 * kAllocSlack)};
  DevicePool &P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  auto take = [&](std::multimap<BlockKey, char *>::iterator it) {
    char *b = it->second;
    P.free_blocks.erase(it);
    P.cached_bytes -= key.bytes;
    P.live.emplace(b, key);
    P.live_bytes += key.bytes;
    ++P.hits;
    return b + kAllocSlack;
  };
  auto it = P.free_blocks.find(key);
  if (it != P.free_blocks.end()) return take(it);
  bool in_pending = false;
  for (auto &b : P.pending) in_pending = in_pending || (b.first.device == dev && b.first.bytes == key.bytes);
  if (in_pending) {
    retire_pending(P, dev);
    it = P.free_blocks.find(key);
    if (it != P.free_blocks.end()) return take(it);
  }
  hipError_t e = hipMalloc(&p, key.bytes);
  if (e == hipErrorOutOfMemory && (P.cached_bytes > 0 || !P.pending.empty())) {
    (void)hipGetLastError();
    release_cached(P);
    e = hipMalloc(&p, key.bytes);
  }
  if (e != hipSuccess)
    throw Error{e == hipErrorOutOfMemory ? KRY_ENOMEM : KRY_EDEVICE,
                std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e)};
  char *b = static_cast<char *>(p);
  P.live.emplace(b, key);
  P.live_bytes += key.bytes;
  ++P.misses;
  return b + kAllocSlack;
}

void dev_free(void *ptr) {
  if (!ptr) return;
  char *b = static_cast<char *>(ptr) - kAllocSlack;
  if (!cache_enabled()) {
    (void)hipFree(b);
    return;
  }
  DevicePool &P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  auto it = P.live.find(b);
  if (it == P.live.end()) {  // not ours (cannot happen through dev_alloc): plain free
    (void)hipFree(b);
    return;
  }
  const BlockKey key = it->second;
  P.live.erase(it);
  P.live_bytes -= key.bytes;
  if (P.cached_bytes + key.bytes > cache_cap()) {  // over the cap: back to the runtime
    (void)hipFree(b);
    return;
  }
  P.pending.emplace_back(key, b);
  P.cached_bytes += key.bytes;
}

// kry_mem_stats / kry_mem_release (C-ABI below)
void mem_stats(int64_t *out) {
  DevicePool &P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  out[0] = (int64_t)P.live_bytes;
  out[1] = (int64_t)P.cached_bytes;
  out[2] = P.hits;
  out[3] = P.misses;
  out[4] = P.syncs;
  out[5] = cache_enabled() ? 1 : 0;
}

void mem_release() {
  DevicePool &P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  release_cached(P);
}

double *ctx_scratch(kry_ctx *ctx, size_t bytes) {
  if (ctx->scratch_bytes < bytes) {
    KRY_HIP(hipStreamSynchronize(ctx->stream));  // the old buffer may still be in use
    dev_free(ctx->scratch);
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
    ctx->scratch = static_cast<double *>(dev_alloc(bytes));
    ctx->scratch_bytes = bytes;
  }
  return ctx->scratch;
}


// ------------------------------------------------ renumbering: row moves
template <int ES>
__global__ __launch_bounds__(kBlock) void permute_rows_kernel(int64_t n, int kshift, const int32_t *__restrict__ idx,
                                                              const char *__restrict__ src, char *__restrict__ dst) {
  typedef typename std::conditional<ES == 8, unsigned long long, unsigned>::type T;
  const int64_t N = n << kshift;
  const int64_t k1 = ((int64_t)1 << kshift) - 1;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i >> kshift;
    const int64_t from = ((int64_t)idx[r] << kshift) | (i & k1);
    reinterpret_cast<T *>(dst)[i] = reinterpret_cast<const T *>(src)[from];
  }
}

void permute_rows(const kry_csr *A, const void *src, void *dst, int k, size_t esize, bool to_op, hipStream_t st) {
  const size_t bytes = (size_t)A->n * k * esize;
  if (!A->renumbered) {
    if (bytes) KRY_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
    return;
  }
  KRY_REQUIRE(src != dst, KRY_EINVAL, "permute_rows: in place");
  int ks = 0;
  while ((1 << ks) < k) ++ks;
  KRY_REQUIRE((1 << ks) == k, KRY_EINVAL, "permute_rows: k must be a power of two");
  const int64_t N = A->n * (int64_t)k;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxGrid, (N + kBlock - 1) / kBlock));
  const int32_t *idx = static_cast<const int32_t *>(to_op ? A->perm : A->iperm);
  if (esize == 8)
    hipLaunchKernelGGL(permute_rows_kernel<8>, dim3(grid), dim3(kBlock), 0, st, A->n, ks, idx,
                       static_cast<const char *>(src), static_cast<char *>(dst));
  else
    hipLaunchKernelGGL(permute_rows_kernel<4>, dim3(grid), dim3(kBlock), 0, st, A->n, ks, idx,
                       static_cast<const char *>(src), static_cast<char *>(dst));
  KRY_HIP(hipGetLastError());
}

void load_in(const kry_csr *A, const void *src, void *dst, int k, size_t esize, hipStream_t st) {
  permute_rows(A, src, dst, k, esize, true, st);
}

bool env_off(const char *name) {
  const char *e = getenv(name);
  return e && atoi(e) == 0;
}

// Ranges of host memory this library has registered for in-flight copies,
// with their users: threads copying the same array (the devices=[...] driver
// uploads one CSR to every device in parallel) share one registration, and a
// range whose PAGES overlap a registered one's waits until that is released
// (hipHostRegister / hipHostUnregister pin and unpin whole pages, so two
// byte-disjoint arrays sharing a page must not register independently), so
// no thread's DMA ever runs on pages another thread has just unregistered.
namespace {
struct HostReg {
  size_t end;         // exact byte range [key, end): what was registered
  uintptr_t pa, pe;   // the pages it pins
  int users;
};
std::mutex host_reg_mu;
std::condition_variable host_reg_cv;
std::map<uintptr_t, HostReg> host_regs;
constexpr uintptr_t kHostPage = 4096;

bool overlaps_other(uintptr_t a, uintptr_t e, uintptr_t pa, uintptr_t pe) {
  for (const auto &kv : host_regs)
    if (kv.second.pa < pe && pa < kv.second.pe && !(kv.first == a && kv.second.end == e)) return true;
  return false;
}
}  // namespace

void host_xfer(void *dst, const void *src, size_t bytes, hipMemcpyKind kind, hipStream_t st) {
  constexpr size_t kPinMin = size_t(4) << 20;
  static const bool pin = !env_off("KRY_HOST_PIN");
  void *host = kind == hipMemcpyHostToDevice ? const_cast<void *>(src) : dst;
  const uintptr_t a = reinterpret_cast<uintptr_t>(host), e = a + bytes;
  const uintptr_t pa = a & ~(kHostPage - 1), pe = (e + kHostPage - 1) & ~(kHostPage - 1);
  bool reg = false;
  if (pin && bytes >= kPinMin) {
    std::unique_lock<std::mutex> lk(host_reg_mu);
    host_reg_cv.wait(lk, [&] { return !overlaps_other(a, e, pa, pe); });
    auto it = host_regs.find(a);
    if (it != host_regs.end() && it->second.end == e) {
      ++it->second.users;
      reg = true;
    } else if (hipHostRegister(host, bytes, hipHostRegisterDefault) == hipSuccess) {
      host_regs[a] = HostReg{e, pa, pe, 1};
      reg = true;
    } else {
      (void)hipGetLastError();  // locked by its owner (e.g. pinned memory), or not lockable: pageable
    }
  }
  auto release = [&] {
    if (!reg) return;
    std::lock_guard<std::mutex> lk(host_reg_mu);
    auto it = host_regs.find(a);
    if (--it->second.users == 0) {
      (void)hipHostUnregister(host);
      host_regs.erase(it);
      host_reg_cv.notify_all();
    }
  };
  try {
    KRY_HIP(hipMemcpyAsync(dst, src, bytes, kind, st));
    KRY_HIP(hipStreamSynchronize(st));
  } catch (...) {
    release();
    throw;
  }
  release();
}

void store_out(const kry_csr *A, const void *src, void *host, int k, size_t esize, hipStream_t st) {
  const size_t bytes = (size_t)A->n * k * esize;
  if (!A->renumbered) {
    host_xfer(host, src, bytes, hipMemcpyDeviceToHost, st);
    return;
  }
  void *tmp = dev_alloc(bytes + 16);
  try {
    permute_rows(A, src, tmp, k, esize, false, st);
    host_xfer(host, tmp, bytes, hipMemcpyDeviceToHost, st);
  } catch (...) {
    dev_free(tmp);
    throw;
  }
  dev_free(tmp);
}

ProfScope::ProfScope(kry_ctx *c, int kernel_id) : ctx(c), id(kernel_id) {
  if (!((ctx->profile >> kernel_id) & 1u)) return;
  if (ctx->prof_calls[kernel_id]++ % ctx->prof_every != 0) return;
  if (ctx->ev_used == ctx->ev_pool.size()) {
    hipEvent_t a, b;
    KRY_HIP(hipEventCreate(&a));
    KRY_HIP(hipEventCreate(&b));
    ctx->ev_pool.emplace_back(a, b);
    ctx->ev_ids.push_back(0);
  }
  auto &pr = ctx->ev_pool[ctx->ev_used];
  ctx->ev_ids[ctx->ev_used] = id;
  KRY_HIP(hipEventRecord(pr.first, ctx->stream));
  e1 = pr.second;
}

ProfScope::~ProfScope() {
  if (!e1) return;
  (void)hipEventRecord(e1, ctx->stream);
  ctx->ev_used++;
}



template <typename V>
struct OpDot {
  const V *x, *y;
  const double *w;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&acc)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V a[W], b[W];
    VIO<V>::load(x, e, N, a);
    VIO<V>::load(y, e, N, b);
#pragma unroll
    for (int v = 0; v < W; ++v)
      if (e + v < N)
        acc[v] += w ? dterm_w((double)a[v], w[(e + v) / k], (double)b[v]) : dterm((double)a[v], (double)b[v]);
  }
};

template <typename V>
struct OpAxpy {
  const V *x;
  V *y;
  const double *alpha;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V a[W], b[W];
    VIO<V>::load(x, e, N, a);
    VIO<V>::load(y, e, N, b);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const V t = (V)alpha[(e + v) & (k - 1)] * a[v];
      b[v] = b[v] + t;
    }
    VIO<V>::store(y, e, N, b);
  }
};

template <typename T>
__global__ void lartg_kernel(int64_t count, const T *f, const T *g, T *c, T *s, T *r) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) lartg<T>(f[i], g[i], c[i], s[i], r[i]);
}

}  // namespace kry

#define KRY_API_BEGIN try {
#define KRY_API_END                                                    \
  return KRY_OK;                                                       \
  }                                                                    \
  catch (const kry::Error &e) {                                        \
    kry::set_error(e.msg);                                             \
    return e.code;                                                     \
  }                                                                    \
  catch (const std::exception &e) {                                    \
    kry::set_error(e.what());                                          \
    return KRY_EDEVICE;                                                \
  }

extern "C" {

// 101: kry_csr_info_n (size-checked image info); kry_csr_info back to its
// version-100 five values. 102: kry_csr_info_n reports the paired-row image.
// 103: the per-step allreduces of the sharded solvers carry a fault count
// (CG total_k + 1, GMRES / MINRES total_k + 2 values); kry_cg_defer_info,
// kry_gmres_xk_device.
int kry_version(void) { return 106; }

#ifndef KRY_BUILD_ID
#define KRY_BUILD_ID "unknown"
#endif
const char *kry_build_id(void) { return KRY_BUILD_ID; }

int kry_device_count(int *count) {
  KRY_API_BEGIN
  KRY_REQUIRE(count, KRY_EINVAL, "null count");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  *count = (e == hipSuccess) ? c : 0;
  KRY_API_END
}

int kry_mem_stats(int64_t *out) {
  KRY_API_BEGIN
  KRY_REQUIRE(out, KRY_EINVAL, "null out");
  kry::mem_stats(out);
  KRY_API_END
}

int kry_mem_release(void) {
  KRY_API_BEGIN
  kry::mem_release();
  KRY_API_END
}

int kry_ctx_create(int device, kry_ctx **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(out, KRY_EINVAL, "null out");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  KRY_REQUIRE(e == hipSuccess && c > 0, KRY_EDEVICE, "no HIP device available");
  KRY_REQUIRE(device >= 0 && device < c, KRY_EINVAL, "device index out of range");
  KRY_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  KRY_HIP(hipGetDeviceProperties(&prop, device));
  KRY_REQUIRE(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0, KRY_EDEVICE,
              std::string("libkrylov_hip is built for gfx950 only; found ") + prop.gcnArchName);
  auto *ctx = new kry_ctx();
  ctx->device = device;
  KRY_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  KRY_HIP(hipEventCreate(&ctx->t0));
  KRY_HIP(hipEventCreate(&ctx->t1));
  *out = ctx;
  KRY_API_END
}

int kry_ctx_destroy(kry_ctx *ctx) {
  KRY_API_BEGIN
  if (!ctx) return KRY_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto &p : ctx->ev_pool) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  (void)hipEventDestroy(ctx->t0);
  (void)hipEventDestroy(ctx->t1);
  dev_free(ctx->scratch);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  KRY_API_END
}

int kry_ctx_synchronize(kry_ctx *ctx) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx, KRY_EINVAL, "null ctx");
  KRY_HIP(hipStreamSynchronize(ctx->stream));
  KRY_API_END
}

int kry_csr_info_n(const kry_csr *A, int64_t *info, int32_t len) {
  KRY_API_BEGIN
  KRY_REQUIRE(A && (info || len == 0) && len >= 0, KRY_EINVAL, "bad argument");
  const int64_t all[KRY_CSR_INFO_LEN] = {A->nslices,   A->nslots,    A->nirregular,        A->compact ? 1 : 0,
                                         A->cb_nb,      A->dia ? 1 : 0, A->dia_nslots,     A->sp ? 1 : 0,
                                         A->sp_nslots,  A->rs ? 1 : 0, A->rs_nslots,     A->renumbered ? 1 : 0,
                                         A->rcm_levels};
  for (int i = 0; i < len && i < KRY_CSR_INFO_LEN; ++i) info[i] = all[i];
  KRY_API_END
}

int kry_csr_info(const kry_csr *A, int64_t *info) { return kry_csr_info_n(A, info, 5); }

}  // extern "C"

namespace {
// KRY_UPLOAD_TRACE=1: wall-clock split of kry_csr_create's phases, to stderr
struct UploadTrace {
  bool on;
  std::chrono::steady_clock::time_point t;
  UploadTrace() {
    const char *e = getenv("KRY_UPLOAD_TRACE");
    on = e && atoi(e) != 0;
    t = std::chrono::steady_clock::now();
  }
  void mark(const char *what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "kry_csr_create %-28s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

// FNV-1a over the permutation: preconditioners must carry their operator's
uint64_t perm_fingerprint(const std::vector<int32_t> &p) {
  uint64_t h = 1469598103934665603ull;
  for (int32_t v : p) {
    h ^= (uint32_t)v;
    h *= 1099511628211ull;
  }
  return h;
}


// like_perm: build P A P^T with another operator's renumbering (a
// preconditioner of a renumbered operator); otherwise renumber when the
// columns are scattered and the graph has narrow levels (KRY_RENUMBER=0
// disables; KRY_RCM_WLIMIT sets the level-width limit, default max(2^16, n / 32)).
template <typename I, typename MV>
void csr_upload(kry_csr *A, const I *ip, const I *ix, const MV *dv, const std::vector<int32_t> *like_perm) {
  hipStream_t st = A->ctx->stream;
  const int64_t n = A->n, nnz = A->nnz;
  UploadTrace tr;
  // the device build (int32 CSR; KRY_DEVICE_BUILD=0: the host builders):
  // 1 = SELL-64 and DIA built on the device, nothing else to do (stencils:
  // the metric); 2 / 3 = SELL-64 built, no DIA / DIA left to the host
  // builder; 0 = nothing built (scattered, the renumbering path below)
  int dres = 0;
  if constexpr (sizeof(I) == 4) {
    if (!like_perm && n > 0 && nnz > 0 && !env_off("KRY_DEVICE_BUILD")) {
      DeviceCsrFlags df;
      dres = device_image_build(A, ip, ix, dv, !env_off("KRY_RENUMBER"), &df);
      tr.mark("device build (H2D + SELL-64 + DIA)");
      if (dres == 1) return;
    }
  }
  if (dres == 0) check_csr(n, nnz, ip, ix);  // validated on the device otherwise
  std::vector<int32_t> own;
  const std::vector<int32_t> *perm = like_perm;
  if (perm) {
    KRY_REQUIRE((int64_t)perm->size() == n, KRY_EINVAL, "renumbering of another size");
  } else if (sizeof(I) == 4 && !env_off("KRY_RENUMBER") && scattered(n, ip, ix)) {
    const char *we = getenv("KRY_RCM_WLIMIT");
    const int64_t wlimit = we ? std::max<int64_t>(1, atoll(we)) : std::max<int64_t>(int64_t(1) << 16, n / 32);
    // on the device (one H2D of indptr / indices; KRY_RCM_DEVICE=0: the host
    // order, the same permutation)
    int r = -1;
    if constexpr (sizeof(I) == 4) {
      if (!env_off("KRY_RCM_DEVICE")) {
        void *dip = dev_alloc((size_t)(n + 1) * 4);
        void *dix = dev_alloc((size_t)std::max<int64_t>(nnz, 1) * 4);
        try {
          host_xfer(dip, ip, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, st);
          if (nnz) host_xfer(dix, ix, (size_t)nnz * 4, hipMemcpyHostToDevice, st);
          r = rcm_order_device(A->ctx, n, static_cast<const int32_t *>(dip), static_cast<const int32_t *>(dix), wlimit,
                               own, &A->rcm_levels);
        } catch (...) {
          dev_free(dip);
          dev_free(dix);
          throw;
        }
        dev_free(dip);
        dev_free(dix);
      }
    }
    if (r < 0) r = rcm_order(n, ip, ix, wlimit, own, &A->rcm_levels) ? 1 : 0;
    if (r == 1) perm = &own;
    tr.mark("RCM order");
  }
  hvec<I> ip2, ix2;
  hvec<MV> dv2;
  if (perm) {
    renumber_csr(n, ip, ix, dv, *perm, ip2, ix2, dv2);
    ip = ip2.data();
    ix = ix2.data();
    dv = dv2.data();
    A->renumbered = true;
    A->perm_host = *perm;
    A->perm_hash = perm_fingerprint(A->perm_host);
    std::vector<int32_t> inv(n);
    for (int64_t r = 0; r < n; ++r) inv[A->perm_host[r]] = (int32_t)r;
    A->perm = dev_alloc((size_t)n * 4 + 4);
    A->iperm = dev_alloc((size_t)n * 4 + 4);
    KRY_HIP(hipMemcpyAsync(A->perm, A->perm_host.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    KRY_HIP(hipMemcpyAsync(A->iperm, inv.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    KRY_HIP(hipStreamSynchronize(st));
    tr.mark("renumbered CSR + perm H2D");
  }
  if (dres < 2) {  // SELL-64 on the host (the device build made it otherwise)
    std::vector<int64_t> sptr;
    std::vector<int32_t> width;
    sell_plan(n, ip, &sptr, &width, &A->nslices, &A->nslots, &A->nirregular);
    A->max_width = 0;
    for (int32_t w : width) A->max_width = std::max(A->max_width, w);
    hvec<I> sidx;
    hvec<MV> sval;
    sell_fill(n, ip, ix, dv, sptr, width, sidx, sval);
    tr.mark("SELL-64 plan + fill");
    A->sptr = dev_alloc(sptr.size() * 8);
    A->swidth = dev_alloc(width.size() * 4 + 4);
    // compact image unless disabled (KRY_SELL_COMPACT=0) or impossible
    const char *cenv = getenv("KRY_SELL_COMPACT");
    hvec<uint16_t> sdelta;
    std::vector<int32_t> scbase;
    A->compact = sizeof(I) == 4 && !(cenv && atoi(cenv) == 0) && A->nslots > 0 &&
                 compact_fill(sptr, width, sidx, sdelta, scbase);
    if (A->compact) {
      A->sdelta = dev_alloc(sdelta.size() * 2);
      A->scbase = dev_alloc(scbase.size() * 4);
      KRY_HIP(hipMemcpyAsync(A->sdelta, sdelta.data(), sdelta.size() * 2, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->scbase, scbase.data(), scbase.size() * 4, hipMemcpyHostToDevice, st));
    } else {
      A->sidx = dev_alloc(sidx.size() * sizeof(I));
      KRY_HIP(hipMemcpyAsync(A->sidx, sidx.data(), sidx.size() * sizeof(I), hipMemcpyHostToDevice, st));
    }
    A->sval = dev_alloc(sval.size() * sizeof(MV));
    KRY_HIP(hipMemcpyAsync(A->sptr, sptr.data(), sptr.size() * 8, hipMemcpyHostToDevice, st));
    if (!width.empty()) KRY_HIP(hipMemcpyAsync(A->swidth, width.data(), width.size() * 4, hipMemcpyHostToDevice, st));
    KRY_HIP(hipMemcpyAsync(A->sval, sval.data(), sval.size() * sizeof(MV), hipMemcpyHostToDevice, st));
    KRY_HIP(hipStreamSynchronize(st));
    release_later(sidx);
    release_later(sval);
    release_later(sdelta);
    tr.mark("compact image + H2D");
  }
  // diagonal-offset image for structured single-RHS SpMVs (KRY_SPMV_DIA=0 disables)
  const char *denv = getenv("KRY_SPMV_DIA");
  if (dres != 2 && !(denv && atoi(denv) == 0)) {
    DiaHost<MV> dh;
    if (dia_build(n, ip, ix, dv, A->nslots, dh)) {
      A->dia = true;
      A->dia_nslices = (int64_t)dh.width.size();
      A->dia_nslots = dh.sptr.back();
      A->dia_max_width = dh.max_width;
      A->dia_sptr = dev_alloc(dh.sptr.size() * 8);
      A->dia_width = dev_alloc(dh.width.size() * 4 + 4);
      A->dia_off = dev_alloc(dh.off.size() * 4);
      A->dia_mask = dev_alloc(dh.mask.size() * 8);
      A->dia_val = dev_alloc(dh.val.size() * sizeof(MV));
      KRY_HIP(hipMemcpyAsync(A->dia_sptr, dh.sptr.data(), dh.sptr.size() * 8, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->dia_width, dh.width.data(), dh.width.size() * 4, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->dia_off, dh.off.data(), dh.off.size() * 4, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->dia_mask, dh.mask.data(), dh.mask.size() * 8, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->dia_val, dh.val.data(), dh.val.size() * sizeof(MV), hipMemcpyHostToDevice, st));
      KRY_HIP(hipStreamSynchronize(st));
      release_later(dh.val);
    }
    tr.mark("DIA image + H2D");
  }
  // column-blocked image for scattered single-RHS SpMVs (KRY_SPMV_CB=0 disables)
  const char *cbenv = getenv("KRY_SPMV_CB");
  if (!A->dia && !A->renumbered && !(cbenv && atoi(cbenv) == 0)) {
    CbHost<MV> cb;
    if (cb_build(n, ip, ix, dv, cb)) {
      A->cb_nb = cb.nb;
      A->cb_cols = cb.cols;
      A->cb_ng = cb.ng;
      A->cb_gptr = dev_alloc(cb.gptr.size() * 8);
      A->cb_roff = dev_alloc(cb.roff.size() * 2);
      A->cb_col = dev_alloc(cb.col.size() * 4);
      A->cb_val = dev_alloc(cb.val.size() * sizeof(MV));
      KRY_HIP(hipMemcpyAsync(A->cb_gptr, cb.gptr.data(), cb.gptr.size() * 8, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->cb_roff, cb.roff.data(), cb.roff.size() * 2, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->cb_col, cb.col.data(), cb.col.size() * 4, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->cb_val, cb.val.data(), cb.val.size() * sizeof(MV), hipMemcpyHostToDevice, st));
      KRY_HIP(hipStreamSynchronize(st));
      release_later(cb.val);
      release_later(cb.col);
      release_later(cb.roff);
    }
    tr.mark("column-blocked image + H2D");
  }
  // paired-row SELL-128 image for general single-RHS SpMVs (KRY_SPMV_PAIR=0 disables)
  const char *penv = getenv("KRY_SPMV_PAIR");
  // (not for a renumbered matrix: its rows are unsorted in the new numbering,
  // and the rank-sorted image's column-sorted runs gather coalesced)
  if (!A->dia && A->cb_nb == 0 && !A->renumbered && !(penv && atoi(penv) == 0)) {
    PairHost<MV> ph;
    if (pair_build(n, ip, ix, dv, A->nslots, ph)) {
      A->sp = true;
      A->sp_nslices = (int64_t)ph.width.size();
      A->sp_nslots = ph.sptr.back();
      A->sp_max_width = ph.max_width;
      A->sp_sptr = dev_alloc(ph.sptr.size() * 8);
      A->sp_width = dev_alloc(ph.width.size() * 4 + 4);
      A->sp_cbase = dev_alloc(ph.cbase.size() * 4);
      A->sp_delta = dev_alloc(ph.delta.size() * 2);
      A->sp_val = dev_alloc(ph.val.size() * sizeof(MV));
      KRY_HIP(hipMemcpyAsync(A->sp_sptr, ph.sptr.data(), ph.sptr.size() * 8, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->sp_width, ph.width.data(), ph.width.size() * 4, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->sp_cbase, ph.cbase.data(), ph.cbase.size() * 4, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->sp_delta, ph.delta.data(), ph.delta.size() * 2, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->sp_val, ph.val.data(), ph.val.size() * sizeof(MV), hipMemcpyHostToDevice, st));
      KRY_HIP(hipStreamSynchronize(st));
      release_later(ph.val);
      release_later(ph.delta);
    }
    tr.mark("paired image + H2D");
  }
  // rank-sorted SELL-128 image: unsorted rows or wide slot columns (KRY_SPMV_RS=0 disables)
  if (!A->dia && A->cb_nb == 0 && !A->sp && !env_off("KRY_SPMV_RS")) {
    RsHost<MV> rh;
    if (rs_build(n, ip, ix, dv, A->nslots, rh)) {
      A->rs = true;
      A->rs_nslices = (int64_t)rh.width.size();
      A->rs_nslots = rh.sptr.back();
      A->rs_max_width = rh.max_width;
      A->rs_sptr = dev_alloc(rh.sptr.size() * 8);
      A->rs_width = dev_alloc(rh.width.size() * 4 + 4);
      A->rs_colrank = dev_alloc(rh.colrank.size() * 4);
      A->rs_val = dev_alloc(rh.val.size() * sizeof(MV));
      KRY_HIP(hipMemcpyAsync(A->rs_sptr, rh.sptr.data(), rh.sptr.size() * 8, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->rs_width, rh.width.data(), rh.width.size() * 4, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->rs_colrank, rh.colrank.data(), rh.colrank.size() * 4, hipMemcpyHostToDevice, st));
      KRY_HIP(hipMemcpyAsync(A->rs_val, rh.val.data(), rh.val.size() * sizeof(MV), hipMemcpyHostToDevice, st));
      KRY_HIP(hipStreamSynchronize(st));
      release_later(rh.colrank);
      release_later(rh.val);
    }
    tr.mark("rank-sorted image + H2D");
  }
  if (A->nirregular > 0 && !A->indptr) {
    A->indptr = dev_alloc((n + 1) * sizeof(I));
    A->indices = dev_alloc((nnz + 1) * sizeof(I));
    A->data = dev_alloc((nnz + 1) * sizeof(MV));
    host_xfer(A->indptr, ip, (n + 1) * sizeof(I), hipMemcpyHostToDevice, st);
    if (nnz) {
      host_xfer(A->indices, ix, nnz * sizeof(I), hipMemcpyHostToDevice, st);
      host_xfer(A->data, dv, nnz * sizeof(MV), hipMemcpyHostToDevice, st);
    }
  }
  KRY_HIP(hipStreamSynchronize(st));  // host staging vectors die at return
  release_later(ix2);
  release_later(dv2);
  tr.mark("CSR copy + final sync");
}
}  // namespace

static void csr_free(kry_csr *A) {
  void *bufs[] = {A->sptr,   A->swidth,   A->sidx,     A->sval,     A->indptr,    A->indices,
                  A->data,   A->sdelta,   A->scbase,   A->cb_gptr,  A->cb_roff,   A->cb_col,
                  A->cb_val, A->dia_sptr, A->dia_width, A->dia_off, A->dia_mask, A->dia_val,
                  A->sp_sptr, A->sp_width, A->sp_cbase, A->sp_delta, A->sp_val,
                  A->rs_sptr, A->rs_width, A->rs_colrank, A->rs_val, A->perm, A->iperm};
  for (void *b : bufs) dev_free(b);
}

extern "C" {

static kry_csr *csr_create(kry_ctx *ctx, int64_t n, int64_t nnz, const void *indptr, const void *indices,
                           const void *data, int dtype, int itype, const kry_csr *like) {
  KRY_REQUIRE(ctx && indptr && (nnz == 0 || (indices && data)), KRY_EINVAL, "null argument");
  KRY_REQUIRE(n >= 0 && nnz >= 0, KRY_EINVAL, "negative size");
  KRY_REQUIRE(dtype == KRY_F32 || dtype == KRY_F64, KRY_EINVAL, "dtype must be f32 or f64");
  KRY_REQUIRE(itype == KRY_I32 || itype == KRY_I64, KRY_EINVAL, "itype must be i32 or i64");
  if (itype == KRY_I32) KRY_REQUIRE(nnz < (int64_t(1) << 31) && n < (int64_t(1) << 31), KRY_EINVAL,
                                    "int32 indices cannot address this matrix");
  KRY_REQUIRE(!like || like->n == n, KRY_EINVAL, "the operator to renumber like has another size");
  KRY_HIP(hipSetDevice(ctx->device));
  auto *A = new kry_csr();
  A->ctx = ctx;
  A->n = n;
  A->nnz = nnz;
  A->dtype = dtype;
  A->itype = itype;
  static const int32_t zi32 = 0;
  static const int64_t zi64 = 0;
  static const double zd = 0;
  const std::vector<int32_t> *lp = like && like->renumbered ? &like->perm_host : nullptr;
  try {
    const void *ix = nnz ? indices : (itype == KRY_I32 ? (const void *)&zi32 : (const void *)&zi64);
    const void *dv = nnz ? data : (const void *)&zd;
    if (itype == KRY_I32 && dtype == KRY_F64)
      csr_upload(A, static_cast<const int32_t *>(indptr), static_cast<const int32_t *>(ix), static_cast<const double *>(dv), lp);
    else if (itype == KRY_I32)
      csr_upload(A, static_cast<const int32_t *>(indptr), static_cast<const int32_t *>(ix), static_cast<const float *>(dv), lp);
    else if (dtype == KRY_F64)
      csr_upload(A, static_cast<const int64_t *>(indptr), static_cast<const int64_t *>(ix), static_cast<const double *>(dv), lp);
    else
      csr_upload(A, static_cast<const int64_t *>(indptr), static_cast<const int64_t *>(ix), static_cast<const float *>(dv), lp);
  } catch (...) {
    csr_free(A);
    delete A;
    throw;
  }
  return A;
}

int kry_csr_create(kry_ctx *ctx, int64_t n, int64_t nnz, const void *indptr, const void *indices,
                   const void *data, int dtype, int itype, kry_csr **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(out, KRY_EINVAL, "null argument");
  *out = csr_create(ctx, n, nnz, indptr, indices, data, dtype, itype, nullptr);
  KRY_API_END
}

int kry_csr_create_like(kry_ctx *ctx, const kry_csr *like, int64_t n, int64_t nnz, const void *indptr,
                        const void *indices, const void *data, int dtype, int itype, kry_csr **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(out && like, KRY_EINVAL, "null argument");
  *out = csr_create(ctx, n, nnz, indptr, indices, data, dtype, itype, like);
  KRY_API_END
}

// Byte comparison of two operators' SELL-64 and DIA images (tests: the
// device-built image against the host builders'): out[0] = the number of
// differing fields / buffers, out[1] = a bitmask of which (bit i = the i-th
// item of the list below).
int kry_csr_compare(const kry_csr *A, const kry_csr *B, int64_t *out) {
  KRY_API_BEGIN
  KRY_REQUIRE(A && B && out, KRY_EINVAL, "null argument");
  KRY_HIP(hipSetDevice(A->ctx->device));
  KRY_HIP(hipDeviceSynchronize());
  int64_t nd = 0, mask = 0;
  int item = 0;
  auto note = [&](bool differ) {
    if (differ) {
      ++nd;
      mask |= int64_t(1) << item;
    }
    ++item;
  };
  const int64_t scal[][2] = {{A->nslices, B->nslices}, {A->nslots, B->nslots}, {A->nirregular, B->nirregular},
                             {A->max_width, B->max_width}, {A->compact, B->compact}, {A->dia, B->dia},
                             {A->dia_nslices, B->dia_nslices}, {A->dia_nslots, B->dia_nslots},
                             {A->dia_max_width, B->dia_max_width}};
  for (auto &p : scal) note(p[0] != p[1]);
  auto buf = [&](const void *a, const void *b, size_t bytes) {
    if (!a || !b) {
      note(a != b);
      return;
    }
    std::vector<char> ha(bytes), hb(bytes);
    if (bytes) {
      KRY_HIP(hipMemcpy(ha.data(), a, bytes, hipMemcpyDeviceToHost));
      KRY_HIP(hipMemcpy(hb.data(), b, bytes, hipMemcpyDeviceToHost));
    }
    note(bytes && std::memcmp(ha.data(), hb.data(), bytes) != 0);
  };
  if (nd == 0) {
    const size_t ds = dsize(A->dtype), is = isize(A->itype);
    buf(A->sptr, B->sptr, (A->nslices + 1) * 8);
    buf(A->swidth, B->swidth, A->nslices * 4);
    buf(A->sval, B->sval, (A->nslots + 256) * ds);
    buf(A->sidx, B->sidx, A->compact ? 0 : (A->nslots + 256) * is);
    buf(A->sdelta, B->sdelta, A->compact ? (A->nslots + 256) * 2 : 0);
    buf(A->scbase, B->scbase, A->compact ? (A->nslots / kSlice + 16) * 4 : 0);
    const int64_t dc = A->dia_nslots / kDiaSlice + kDiaPad;
    buf(A->dia_sptr, B->dia_sptr, A->dia ? (A->dia_nslices + 1) * 8 : 0);
    buf(A->dia_width, B->dia_width, A->dia ? A->dia_nslices * 4 : 0);
    buf(A->dia_off, B->dia_off, A->dia ? dc * 4 : 0);
    buf(A->dia_mask, B->dia_mask, A->dia ? dc * 16 : 0);
    buf(A->dia_val, B->dia_val, A->dia ? (A->dia_nslots + 256) * ds : 0);
    buf(A->indptr, B->indptr, A->nirregular ? (A->n + 1) * is : 0);
    buf(A->indices, B->indices, A->nirregular ? A->nnz * is : 0);
    buf(A->data, B->data, A->nirregular ? A->nnz * ds : 0);
  }
  out[0] = nd;
  out[1] = mask;
  KRY_API_END
}

int kry_csr_permute(kry_ctx *ctx, const kry_csr *A, const kry_vec *src, kry_vec *dst, int to_operator) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && A && src && dst, KRY_EINVAL, "null argument");
  KRY_REQUIRE(src->n == A->n && dst->n == A->n && src->k == dst->k && src->dtype == dst->dtype, KRY_EINVAL,
              "shape mismatch");
  KRY_REQUIRE(src != dst, KRY_EINVAL, "src and dst must differ");
  KRY_HIP(hipSetDevice(ctx->device));
  permute_rows(A, src->d, dst->d, src->k, dsize(src->dtype), to_operator != 0, ctx->stream);
  KRY_API_END
}

int kry_csr_destroy(kry_csr *A) {
  KRY_API_BEGIN
  if (!A) return KRY_OK;
  (void)hipSetDevice(A->ctx->device);
  (void)hipStreamSynchronize(A->ctx->stream);
  csr_free(A);
  delete A;
  KRY_API_END
}

int kry_vec_create(kry_ctx *ctx, int64_t n, int32_t k, int dtype, kry_vec **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && out, KRY_EINVAL, "null argument");
  KRY_REQUIRE(n >= 0 && k >= 1, KRY_EINVAL, "bad vector shape");
  KRY_REQUIRE(dtype == KRY_F32 || dtype == KRY_F64, KRY_EINVAL, "dtype must be f32 or f64");
  KRY_HIP(hipSetDevice(ctx->device));
  auto *v = new kry_vec();
  v->ctx = ctx;
  v->n = n;
  v->k = k;
  v->dtype = dtype;
  const size_t elems = ((size_t)n * k + 15) / 16 * 16;
  try {
    v->d = dev_alloc(elems * dsize(dtype));
    KRY_HIP(hipMemsetAsync(v->d, 0, elems * dsize(dtype), ctx->stream));
  } catch (...) {
    delete v;
    throw;
  }
  *out = v;
  KRY_API_END
}

int kry_vec_destroy(kry_vec *v) {
  KRY_API_BEGIN
  if (!v) return KRY_OK;
  (void)hipSetDevice(v->ctx->device);
  (void)hipStreamSynchronize(v->ctx->stream);
  dev_free(v->d);
  delete v;
  KRY_API_END
}

int kry_vec_upload(kry_vec *v, const void *host) {
  KRY_API_BEGIN
  KRY_REQUIRE(v && host, KRY_EINVAL, "null argument");
  host_xfer(v->d, host, v->bytes(), hipMemcpyHostToDevice, v->ctx->stream);
  KRY_API_END
}

int kry_vec_download(kry_vec *v, void *host) {
  KRY_API_BEGIN
  KRY_REQUIRE(v && host, KRY_EINVAL, "null argument");
  host_xfer(host, v->d, v->bytes(), hipMemcpyDeviceToHost, v->ctx->stream);
  KRY_API_END
}

int kry_spmv(kry_ctx *ctx, kry_csr *A, kry_vec *x, kry_vec *y) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && A && x && y, KRY_EINVAL, "null argument");
  KRY_REQUIRE(x->n == A->n && y->n == A->n && x->k == y->k, KRY_EINVAL, "shape mismatch");
  KRY_REQUIRE(x->dtype == y->dtype, KRY_EINVAL, "dtype mismatch");
  KRY_REQUIRE(is_pow2(x->k) && x->k <= kMaxCols, KRY_EUNSUPPORTED, "k must be a power of two <= 256");
  KRY_HIP(hipSetDevice(ctx->device));
  const int k = x->k;
  // a renumbered operator: x and y in the caller's numbering, moved through
  // two temporaries (y = P^T (P A P^T) P x)
  const size_t vb = (size_t)A->n * k * dsize(x->dtype) + 16;
  void *xt = A->renumbered ? dev_alloc(vb) : nullptr;
  void *yt = A->renumbered ? dev_alloc(vb) : nullptr;
  try {
    if (xt) permute_rows(A, x->d, xt, k, dsize(x->dtype), true, ctx->stream);
    const void *xs = xt ? xt : x->d;
    void *ys = yt ? yt : y->d;
    dispatch_vmi(x->dtype, A->dtype, A->itype, [&](auto v0, auto m0, auto i0) {
      using V = decltype(v0);
      using MV = decltype(m0);
      using I = decltype(i0);
      ProfScope ps(ctx, PROF_SPMV);
      launch_spmv<V, MV, I>(A, k, SrcPlain<V>{static_cast<const V *>(xs), k}, EpiStore<V>{static_cast<V *>(ys), k},
                            nullptr, nullptr, nullptr, 0, ctx->stream);
    });
    if (yt) permute_rows(A, yt, y->d, k, dsize(x->dtype), false, ctx->stream);
  } catch (...) {
    dev_free(xt);
    dev_free(yt);
    throw;
  }
  dev_free(xt);  // the caching pool retires freed blocks only after a device sync
  dev_free(yt);
  KRY_HIP(hipGetLastError());  // stream-ordered: a download or reduction of y waits for it
  KRY_API_END
}

int kry_spmv_op(kry_ctx *ctx, kry_csr *A, kry_vec *x, kry_vec *y) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && A && x && y, KRY_EINVAL, "null argument");
  KRY_REQUIRE(x->n == A->n && y->n == A->n && x->k == y->k, KRY_EINVAL, "shape mismatch");
  KRY_REQUIRE(x->dtype == y->dtype, KRY_EINVAL, "dtype mismatch");
  KRY_REQUIRE(is_pow2(x->k) && x->k <= kMaxCols, KRY_EUNSUPPORTED, "k must be a power of two <= 256");
  KRY_HIP(hipSetDevice(ctx->device));
  const int k = x->k;
  dispatch_vmi(x->dtype, A->dtype, A->itype, [&](auto v0, auto m0, auto i0) {
    using V = decltype(v0);
    using MV = decltype(m0);
    using I = decltype(i0);
    ProfScope ps(ctx, PROF_SPMV);
    launch_spmv<V, MV, I>(A, k, SrcPlain<V>{static_cast<const V *>(x->d), k}, EpiStore<V>{static_cast<V *>(y->d), k},
                          nullptr, nullptr, nullptr, 0, ctx->stream);
  });
  KRY_HIP(hipGetLastError());
  KRY_API_END
}

int kry_dot(kry_ctx *ctx, kry_vec *x, kry_vec *y, kry_vec *w, double *out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && x && y && out, KRY_EINVAL, "null argument");
  KRY_REQUIRE(x->n == y->n && x->k == y->k && x->dtype == y->dtype, KRY_EINVAL, "shape mismatch");
  KRY_REQUIRE(!w || (w->n == x->n && w->k == 1 && w->dtype == KRY_F64), KRY_EINVAL,
              "weights must be an (n,) float64 vector");
  KRY_REQUIRE(is_pow2(x->k) && x->k <= kMaxCols, KRY_EUNSUPPORTED, "k must be a power of two <= 256");
  KRY_HIP(hipSetDevice(ctx->device));
  const int k = x->k;
  const int64_t N = x->n * (int64_t)k;
  double *part = ctx_scratch(ctx, (part_rows(k) + 1) * (size_t)k * 8);
  {
    int P;
    const double *wd = w ? static_cast<const double *>(w->d) : nullptr;
    if (x->dtype == KRY_F64)
      P = launch_elementwise<double>(N, k, OpDot<double>{static_cast<const double *>(x->d), static_cast<const double *>(y->d), wd, k},
                                     part, nullptr, 0, ctx->stream);
    else
      P = launch_elementwise<float>(N, k, OpDot<float>{static_cast<const float *>(x->d), static_cast<const float *>(y->d), wd, k},
                                    part, nullptr, 0, ctx->stream);
    double *res = part + part_rows(k) * k;
    hipLaunchKernelGGL(reduce_to_kernel<0>, dim3(1), dim3(kBlock), 0, ctx->stream, part, P, k, res);
    KRY_HIP(hipGetLastError());
    KRY_HIP(hipMemcpyAsync(out, res, k * 8, hipMemcpyDeviceToHost, ctx->stream));
    KRY_HIP(hipStreamSynchronize(ctx->stream));
  }
  KRY_API_END
}

int kry_axpy(kry_ctx *ctx, const double *alpha, kry_vec *x, kry_vec *y) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && alpha && x && y, KRY_EINVAL, "null argument");
  KRY_REQUIRE(x->n == y->n && x->k == y->k && x->dtype == y->dtype, KRY_EINVAL, "shape mismatch");
  KRY_REQUIRE(is_pow2(x->k) && x->k <= kMaxCols, KRY_EUNSUPPORTED, "k must be a power of two <= 256");
  KRY_HIP(hipSetDevice(ctx->device));
  const int k = x->k;
  const int64_t N = x->n * (int64_t)k;
  double *a = static_cast<double *>(dev_alloc(k * 8));
  try {
    KRY_HIP(hipMemcpyAsync(a, alpha, k * 8, hipMemcpyHostToDevice, ctx->stream));
    if (x->dtype == KRY_F64)
      launch_elementwise<double>(N, k, OpAxpy<double>{static_cast<const double *>(x->d), static_cast<double *>(y->d), a, k},
                                 nullptr, nullptr, 0, ctx->stream);
    else
      launch_elementwise<float>(N, k, OpAxpy<float>{static_cast<const float *>(x->d), static_cast<float *>(y->d), a, k},
                                nullptr, nullptr, 0, ctx->stream);
    KRY_HIP(hipStreamSynchronize(ctx->stream));
  } catch (...) {
    dev_free(a);
    throw;
  }
  dev_free(a);
  KRY_API_END
}

int kry_lartg(kry_ctx *ctx, int64_t count, int dtype, const void *f, const void *g, void *c, void *s,
              void *r) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && f && g && c && s && r && count >= 0, KRY_EINVAL, "null argument");
  KRY_REQUIRE(dtype == KRY_F32 || dtype == KRY_F64, KRY_EINVAL, "bad dtype");
  if (count == 0) return KRY_OK;
  KRY_HIP(hipSetDevice(ctx->device));
  const size_t vs = dsize(dtype), bytes = count * vs;
  char *buf = static_cast<char *>(dev_alloc(5 * bytes));
  try {
    KRY_HIP(hipMemcpyAsync(buf, f, bytes, hipMemcpyHostToDevice, ctx->stream));
    KRY_HIP(hipMemcpyAsync(buf + bytes, g, bytes, hipMemcpyHostToDevice, ctx->stream));
    const int grid = (int)((count + kBlock - 1) / kBlock);
    if (dtype == KRY_F64) {
      double *b = reinterpret_cast<double *>(buf);
      hipLaunchKernelGGL(lartg_kernel<double>, dim3(grid), dim3(kBlock), 0, ctx->stream, count, b, b + count,
                         b + 2 * count, b + 3 * count, b + 4 * count);
    } else {
      float *b = reinterpret_cast<float *>(buf);
      hipLaunchKernelGGL(lartg_kernel<float>, dim3(grid), dim3(kBlock), 0, ctx->stream, count, b, b + count,
                         b + 2 * count, b + 3 * count, b + 4 * count);
    }
    KRY_HIP(hipGetLastError());
    KRY_HIP(hipMemcpyAsync(c, buf + 2 * bytes, bytes, hipMemcpyDeviceToHost, ctx->stream));
    KRY_HIP(hipMemcpyAsync(s, buf + 3 * bytes, bytes, hipMemcpyDeviceToHost, ctx->stream));
    KRY_HIP(hipMemcpyAsync(r, buf + 4 * bytes, bytes, hipMemcpyDeviceToHost, ctx->stream));
    KRY_HIP(hipStreamSynchronize(ctx->stream));
  } catch (...) {
    dev_free(buf);
    throw;
  }
  dev_free(buf);
  KRY_API_END
}

int kry_timer_start(kry_ctx *ctx) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx, KRY_EINVAL, "null ctx");
  KRY_HIP(hipEventRecord(ctx->t0, ctx->stream));
  KRY_API_END
}

int kry_timer_stop(kry_ctx *ctx, double *ms) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && ms, KRY_EINVAL, "null argument");
  KRY_HIP(hipEventRecord(ctx->t1, ctx->stream));
  KRY_HIP(hipEventSynchronize(ctx->t1));
  float f = 0;
  KRY_HIP(hipEventElapsedTime(&f, ctx->t0, ctx->t1));
  *ms = f;
  KRY_API_END
}

int kry_profile_enable(kry_ctx *ctx, int enable) { return kry_profile_select(ctx, enable ? 0xFu : 0u, 1); }

int kry_profile_select(kry_ctx *ctx, uint32_t mask, int32_t every) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && every >= 1, KRY_EINVAL, "bad argument");
  KRY_HIP(hipStreamSynchronize(ctx->stream));
  ctx->profile = mask & 0xFu;
  ctx->prof_every = every;
  for (int i = 0; i < 4; ++i) ctx->prof_calls[i] = 0;
  ctx->ev_used = 0;
  for (int i = 0; i < 4; ++i) {
    ctx->prof_count[i] = 0;
    ctx->prof_ms[i] = 0;
  }
  KRY_API_END
}

int kry_profile_read(kry_ctx *ctx, int kernel_id, int64_t *count, double *total_ms) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && count && total_ms && kernel_id >= 0 && kernel_id < 4, KRY_EINVAL, "bad argument");
  KRY_HIP(hipStreamSynchronize(ctx->stream));
  for (size_t i = 0; i < ctx->ev_used; ++i) {
    float f = 0;
    KRY_HIP(hipEventElapsedTime(&f, ctx->ev_pool[i].first, ctx->ev_pool[i].second));
    ctx->prof_count[ctx->ev_ids[i]] += 1;
    ctx->prof_ms[ctx->ev_ids[i]] += f;
  }
  ctx->ev_used = 0;
  *count = ctx->prof_count[kernel_id];
  *total_ms = ctx->prof_ms[kernel_id];
  KRY_API_END
}

}  // extern "C"
