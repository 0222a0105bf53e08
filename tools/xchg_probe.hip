// In-launch all-gather latency probe (development tool, not product; round 5).
// Times ONE exchange of the persistent kernels alone at the production grids:
// G = one block per CU (256), T = 512 threads (gm_mgsl / gm_mgsp / cg_upd /
// mr_upd) or 1024 (cg_persist). Every round each block reduces one double
// (block_sum, as block_sum1_t0), exchanges it with every other block and
// broadcasts the total to its threads through LDS; the round time minus the
// NONE variant's (block sum + barrier, no exchange) is the exchange's cost.
//
// Variants (the transport of the 256 block partials):
//   FLAT    today's sweep_partials: two 8-B {tag, half} granules per block,
//           wave 0 of every block re-reads all of them per poll
//   FLAT16  the same granule pair read with one 16-B sc1 load per block, and
//           a lane re-polls only granules whose tags have not matched yet
//   R32     32 reader blocks sweep all partials (FLAT16), sum, and publish
//           the total as one granule pair; every other block polls the
//           reader blockIdx % 32 (same XCD under round-robin placement)
//   R8      the same with 8 readers
//   XCD     two-level tree: 8 groups blockIdx % 8, group leader g sweeps its
//           32 members and publishes the group sum; every block sweeps the 8
//           group sums
// Summation orders are fixed per variant (no atomics on values).
// Prefetch mode PF: before the sweep every thread of waves PF_FIRST.. issues
// L 16-B loads of a 1 GB buffer (as the streamed MGS kernel's chunk-0
// prefetch) and consumes them after the exchange; PF_FIRST = 0 puts them on
// the sweeping wave too (in-order vmcnt: the sweep waits behind them).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xchg_probe.hip -o tools/xchg_probe
//   ./tools/xchg_probe            (prints one JSON line per configuration)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef unsigned long long ull;
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

enum { NONE = 0, FLAT = 1, FLAT16 = 2, R32 = 3, R8 = 4, XCD = 5 };
static const char *kName[] = {"none", "flat", "flat16", "r32", "r8", "xcd"};
constexpr unsigned kSpinTicks = 2000000u;  // 20 ms of the 100 MHz clock
constexpr int kPfL = 4;                    // prefetch loads per thread

__device__ __forceinline__ void publish(ull *g, unsigned tag, double v) {
  const ull bits = (ull)__double_as_longlong(v);
  const ull t = (ull)tag << 32;
  __hip_atomic_store(g, t | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, t | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double unpack(ull lo, ull hi) {
  return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
}
// one granule pair, 16 B, agent scope (sc1: past the CU's L1), through a
// wave-uniform buffer descriptor over the whole region and a per-lane offset;
// the memory clobber in the poll loop keeps LLVM from hoisting it
__device__ __forceinline__ __amdgpu_buffer_rsrc_t region_rsrc(const ull *base) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((unsigned long long)hi << 32) | lo), 0, 8192, 0x00020000);
}
__device__ __forceinline__ u4 ld16(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
}
__device__ __forceinline__ bool tags_ok(u4 g, unsigned tag) { return g.y == tag && g.w == tag; }
__device__ __forceinline__ double val16(u4 g) {
  return __longlong_as_double((long long)(((ull)g.z << 32) | (ull)g.x));
}

// wave 0 only. Today's form.
__device__ bool sweep_flat(ull *gr, int G, unsigned tag, double *out, unsigned *err) {
  const int lane = threadIdx.x;
  ull g[4][2];
  const ull t0 = wall_clock64();
  unsigned spins = 0;
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = lane + 64 * i;
      if (b < G) {
        g[i][0] = __hip_atomic_load(gr + 2 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        g[i][1] = __hip_atomic_load(gr + 2 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = ok && (unsigned)(g[i][0] >> 32) == tag && (unsigned)(g[i][1] >> 32) == tag;
      }
    }
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255u) == 0 && wall_clock64() - t0 > kSpinTicks) {
      if (lane == 0) atomicAdd(err, 1u);
      return false;
    }
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < G) s += unpack(g[i][0], g[i][1]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  *out = s;
  return true;
}

// wave 0 only: granule pairs gr[2 * (first + stride * i)], i < cnt <= 256,
// one 16-B load each, unmatched lanes only; fixed-order sum (lane l:
// i = l, l + 64, ..., then the xor butterfly)
__device__ bool sweep16(const ull *gr, int first, int stride, int cnt, unsigned tag, double *out, unsigned *err) {
  const int lane = threadIdx.x;
  u4 g[4];
  bool got[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    got[i] = lane + 64 * i >= cnt;
    g[i] = u4{0, 0, 0, 0};
  }
  const __amdgpu_buffer_rsrc_t rs = region_rsrc(gr);
  const ull t0 = wall_clock64();
  unsigned spins = 0;
  for (;;) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (!got[i]) g[i] = ld16(rs, 16 * (first + stride * (lane + 64 * i)));
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!got[i]) got[i] = tags_ok(g[i], tag);
      ok = ok && got[i];
    }
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255u) == 0 && wall_clock64() - t0 > kSpinTicks) {
      if (lane == 0) atomicAdd(err, 1u);
      return false;
    }
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < cnt) s += val16(g[i]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  *out = s;
  return true;
}

template <int T>
__device__ __forceinline__ double block_sum_t0(double v, double *wsum) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) wsum[wv] = v;
  __syncthreads();
  double s = 0.0;
  if (wv == 0) {
    s = lane < T / 64 ? wsum[lane] : 0.0;
    for (int off = 1; off < T / 64; off <<= 1) s += __shfl_xor(s, off);
  }
  return s;
}

// regions: gran [2 parities][2 * 256], bc [2 parities][2 * 256]
template <int VAR, int T, int PF_FIRST>
__global__ __launch_bounds__(T) void xchg_kernel(int R, ull *gran, ull *bc, const u4 *big, size_t big_n, double *out,
                                                 unsigned *err) {
  __shared__ double wsum[T / 64];
  __shared__ double shv;
  __shared__ int flag;
  extern __shared__ char pad[];  // dynamic LDS: one block per CU
  const int tid = threadIdx.x, G = gridDim.x;
  const int wid = tid >> 6;
  double acc = 0.0;
  u4 pfacc = u4{0, 0, 0, 0};
  for (int r = 0; r < R; ++r) {
    const double v = (double)((blockIdx.x * 7 + tid + r) % 13);
    const double bp = block_sum_t0<T>(v, wsum);
    const unsigned tag = (unsigned)(r + 1);
    ull *gr = gran + (size_t)(r & 1) * 512;
    ull *bq = bc + (size_t)(r & 1) * 512;
    if (VAR != NONE && tid == 0) publish(gr + 2 * blockIdx.x, tag, bp);
    u4 pf[kPfL];
    const bool do_pf = PF_FIRST >= 0 && wid >= PF_FIRST;
    if (do_pf) {
      const size_t base = ((size_t)r * G + blockIdx.x) * T * kPfL;
#pragma unroll
      for (int l = 0; l < kPfL; ++l) pf[l] = big[(base + (size_t)l * T + tid) % big_n];
    }
    if (tid < 64) {
      bool ok = true;
      double s = bp;
      if (VAR == FLAT) {
        ok = sweep_flat(gr, G, tag, &s, err);
      } else if (VAR == FLAT16) {
        ok = sweep16(gr, 0, 1, G, tag, &s, err);
      } else if (VAR == R32 || VAR == R8) {
        constexpr int NR = VAR == R32 ? 32 : 8;
        const int rd = blockIdx.x % NR;
        if ((int)blockIdx.x < NR) {
          ok = sweep16(gr, 0, 1, G, tag, &s, err);
          if (ok && tid == 0) publish(bq + 2 * blockIdx.x, tag, s);
        } else {
          ok = sweep16(bq, rd, 0, 1, tag, &s, err);
        }
      } else if (VAR == XCD) {
        const int grp = blockIdx.x & 7;
        if ((int)blockIdx.x < 8) {
          const int cnt = (G - grp + 7) / 8;
          ok = sweep16(gr, grp, 8, cnt, tag, &s, err);
          if (ok && tid == 0) publish(bq + 2 * grp, tag, s);
        }
        if (ok) ok = sweep16(bq, 0, 1, G < 8 ? G : 8, tag, &s, err);
      }
      if (tid == 0) {
        shv = s;
        flag = ok;
      }
    }
    __syncthreads();
    if (!flag) break;
    acc += shv;
    if (do_pf) {
#pragma unroll
      for (int l = 0; l < kPfL; ++l) pfacc += pf[l];
    }
  }
  out[(size_t)blockIdx.x * T + tid] = acc + (double)(pfacc.x ^ pfacc.y ^ pfacc.z ^ pfacc.w);
  (void)pad;
}

template <int VAR, int T, int PF>
static void run(int G, int R, int reps, ull *gran, ull *bc, const u4 *big, size_t big_n, double *out, unsigned *err,
                double base_us) {
  const size_t lds = 96 * 1024;  // with the static arrays: one block per CU
  CK(hipFuncSetAttribute((const void *)xchg_kernel<VAR, T, PF>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int i = 0; i < reps + 1; ++i) {
    CK(hipMemset(gran, 0, 2 * 512 * 8));
    CK(hipMemset(bc, 0, 2 * 512 * 8));
    CK(hipMemset(err, 0, 4));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((xchg_kernel<VAR, T, PF>), dim3(G), dim3(T), lds, 0, R, gran, bc, big, big_n, out, err);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (i) ms.push_back(t);
  }
  unsigned herr = 0;
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  // check: every thread's acc = sum_r total_r (pf buffer is zero)
  std::vector<double> h((size_t)G * T);
  CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
  double expect = 0.0;
  if (VAR != NONE)
    for (int r = 0; r < R; ++r)
      for (int b = 0; b < G; ++b)
        for (int t = 0; t < T; ++t) expect += (double)((b * 7 + t + r) % 13);
  long bad = 0;
  if (VAR != NONE)
    for (double x : h) bad += x != expect;
  std::sort(ms.begin(), ms.end());
  const double us = 1e3 * ms[ms.size() / 2] / R;
  printf("{\"variant\": \"%s\", \"T\": %d, \"G\": %d, \"pf_first_wave\": %d, \"rounds\": %d, \"us_per_round\": %.3f, "
         "\"exchange_us\": %.3f, \"min_us_per_round\": %.3f, \"timeouts\": %u, \"bad\": %ld}\n",
         kName[VAR], T, G, PF, R, us, us - base_us, 1e3 * ms[0] / R, herr, bad);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int VAR, int T, int PF>
static double base_of(int G, int R, ull *gran, ull *bc, const u4 *big, size_t big_n, double *out, unsigned *err) {
  const size_t lds = 96 * 1024;
  CK(hipFuncSetAttribute((const void *)xchg_kernel<NONE, T, PF>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int i = 0; i < 6; ++i) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((xchg_kernel<NONE, T, PF>), dim3(G), dim3(T), lds, 0, R, gran, bc, big, big_n, out, err);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (i) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double us = 1e3 * ms[ms.size() / 2] / R;
  printf("{\"variant\": \"none\", \"T\": %d, \"G\": %d, \"pf_first_wave\": %d, \"us_per_round\": %.3f}\n", T, G, PF, us);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return us;
}

template <int T, int PF>
static void family(int G, int R, ull *gran, ull *bc, const u4 *big, size_t big_n, double *out, unsigned *err) {
  const double b = base_of<NONE, T, PF>(G, R, gran, bc, big, big_n, out, err);
  run<FLAT, T, PF>(G, R, 5, gran, bc, big, big_n, out, err, b);
  run<FLAT16, T, PF>(G, R, 5, gran, bc, big, big_n, out, err, b);
  run<R32, T, PF>(G, R, 5, gran, bc, big, big_n, out, err, b);
  run<R8, T, PF>(G, R, 5, gran, bc, big, big_n, out, err, b);
  run<XCD, T, PF>(G, R, 5, gran, bc, big, big_n, out, err, b);
}

int main(int argc, char **argv) {
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  const int G = argc > 1 ? atoi(argv[1]) : prop.multiProcessorCount;
  const int R = argc > 2 ? atoi(argv[2]) : 2000;
  if (G < 1 || G > 256) {
    fprintf(stderr, "G must be in [1, 256]\n");
    return 1;
  }
  ull *gran, *bc;
  double *out;
  unsigned *err;
  u4 *big;
  const size_t big_n = (size_t)1 << 26;  // 1 GiB of 16-B granules
  CK(hipMalloc(&gran, 2 * 512 * 8));
  CK(hipMalloc(&bc, 2 * 512 * 8));
  CK(hipMalloc(&out, (size_t)256 * 1024 * 8));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&big, big_n * 16));
  CK(hipMemset(big, 0, big_n * 16));
  printf("{\"device\": \"%s\", \"cus\": %d, \"G\": %d, \"rounds\": %d}\n", prop.name, prop.multiProcessorCount, G, R);
  family<512, -1>(G, R, gran, bc, big, big_n, out, err);   // parked
  family<512, 1>(G, R, gran, bc, big, big_n, out, err);    // prefetch on waves 1..7
  family<512, 0>(G, R, gran, bc, big, big_n, out, err);    // prefetch on every wave (the MGS kernel)
  family<1024, -1>(G, R, gran, bc, big, big_n, out, err);  // cg_persist's block
  CK(hipFree(big));
  CK(hipFree(gran));
  CK(hipFree(bc));
  CK(hipFree(out));
  CK(hipFree(err));
  return 0;
}
