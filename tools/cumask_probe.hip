// CU-masked streams on MI355X (development probe, not product; round 6).
//
// The overlap probe (tools/overlap_probe.hip) found that cfg3's random
// x gathers and its HBM stream serialise on one CU, but run side by side on
// different CUs. This probe asks whether two CU-masked streams can give the
// gathers and the stream their own CUs inside one SpMV's time:
//
//  1. where the blocks of a kernel on a masked stream land (XCC_ID, HW_ID
//     se / sh / cu), for a mask of every 8th CU bit, so the mapping of mask
//     bits to XCDs is on record;
//  2. gathers (40 M random 8-B loads from a 2 MB window) on stream A masked
//     to the complement, concurrently with a 480 MB stream on stream B masked
//     to those CUs, against each alone on the same masks and unmasked.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/cumask_probe.hip -o tools/cumask_probe
//   tools/cumask_probe [every] [reps]    (every: the stream CUs are mask bits i % every == 0)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef int i4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;
constexpr int64_t kWin = 262144;           // 2 MB of fp64
constexpr int64_t kStreamB = 480LL << 20;  // column + value stream
constexpr int64_t kQuads = kStreamB / 16;
constexpr int64_t kGathers = 40000000;

__device__ __forceinline__ uint32_t xs(uint32_t h) {
  h ^= h << 13; h ^= h >> 17; h ^= h << 5;
  return h;
}

__global__ void where(unsigned *out) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    out[blockIdx.x] = (xcc << 16) | ((hw >> 13) & 7) << 8 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 15);
  }
}

// grid-stride gathers: every thread `rounds` rounds of 8
__global__ __launch_bounds__(kBlock) void gathers(const double *__restrict__ x, int rounds, double *out) {
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
  double acc = 0.0;
  for (int r = 0; r < rounds; ++r) {
    double v[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) { h = xs(h); v[g] = x[h % (uint32_t)kWin]; }
#pragma unroll
    for (int g = 0; g < 8; ++g) acc += v[g];
  }
  if (acc == 1234.5678) out[0] = acc;
}

// grid-stride stream, 8 quads in flight per thread
__global__ __launch_bounds__(kBlock) void stream(const i4 *__restrict__ s, double *out) {
  const int64_t nthr = (int64_t)gridDim.x * kBlock;
  int isum = 0;
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < kQuads; q += 8 * nthr) {
    i4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t qq = q + u * nthr;
      v[u] = qq < kQuads ? __builtin_nontemporal_load(s + qq) : i4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) isum += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (isum == 0x7fffabcd) out[0] = isum;
}

int main(int argc, char **argv) {
  const int every = argc > 1 ? atoi(argv[1]) : 8;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const int words = (ncu + 31) / 32;
  std::vector<uint32_t> ma(words, 0), mb(words, 0);
  int na = 0, nb = 0;
  for (int i = 0; i < ncu; ++i) {
    if (i % every == 0) { mb[i / 32] |= 1u << (i % 32); ++nb; }
    else { ma[i / 32] |= 1u << (i % 32); ++na; }
  }
  hipStream_t sa, sb, sfull;
  CK(hipExtStreamCreateWithCUMask(&sa, words, ma.data()));
  CK(hipExtStreamCreateWithCUMask(&sb, words, mb.data()));
  CK(hipStreamCreate(&sfull));
  printf("{\"cus\": %d, \"gather_cus\": %d, \"stream_cus\": %d}\n", ncu, na, nb);

  // 1. placement of a masked launch
  unsigned *pl;
  const int pg = nb * 8;
  CK(hipMalloc(&pl, pg * 4));
  hipLaunchKernelGGL(where, dim3(pg), dim3(64), 0, sb, pl);
  CK(hipStreamSynchronize(sb));
  std::vector<unsigned> h(pg);
  CK(hipMemcpy(h.data(), pl, pg * 4, hipMemcpyDeviceToHost));
  std::map<unsigned, int> cus;
  std::map<unsigned, int> per_xcc;
  for (unsigned v : h) cus[v]++;
  for (auto &kv : cus) per_xcc[kv.first >> 16]++;
  printf("{\"placement\": \"stream-mask blocks on %zu distinct CUs\", \"cus_per_xcc\": {", cus.size());
  bool first = true;
  for (auto &kv : per_xcc) { printf("%s\"%u\": %d", first ? "" : ", ", kv.first, kv.second); first = false; }
  printf("}}\n");

  i4 *s;
  double *x, *out;
  CK(hipMalloc(&s, kStreamB));
  CK(hipMalloc(&x, kWin * 8));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(s, 1, kStreamB));
  CK(hipMemset(x, 0, kWin * 8));
  hipEvent_t e0, e1, ea, eb;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));

  const int64_t gthreads_full = (int64_t)ncu * 4 * kBlock;
  auto run = [&](const char *name, bool g, bool st, hipStream_t gs, int gcus, hipStream_t ss, int scus) {
    float tot = 0.f, best = 1e30f;
    for (int r = 0; r < reps + 2; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, sfull));
      CK(hipStreamWaitEvent(gs, e0, 0));
      CK(hipStreamWaitEvent(ss, e0, 0));
      if (g) {
        const int grid = gcus * 4;
        const int rounds = (int)((kGathers / ((int64_t)grid * kBlock) + 7) / 8);
        hipLaunchKernelGGL(gathers, dim3(grid), dim3(kBlock), 0, gs, x, rounds, out);
      }
      if (st) hipLaunchKernelGGL(stream, dim3(scus * 8), dim3(kBlock), 0, ss, s, out);
      CK(hipEventRecord(ea, gs));
      CK(hipEventRecord(eb, ss));
      CK(hipStreamWaitEvent(sfull, ea, 0));
      CK(hipStreamWaitEvent(sfull, eb, 0));
      CK(hipEventRecord(e1, sfull));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) { tot += ms; best = ms < best ? ms : best; }
    }
    printf("{\"mode\": \"%s\", \"ms_mean\": %.4f, \"ms_min\": %.4f}\n", name, tot / reps, best);
  };
  (void)gthreads_full;
  run("gather_full", true, false, sfull, ncu, sfull, 0);
  run("stream_full", false, true, sfull, 0, sfull, ncu);
  run("gather_maskA", true, false, sa, na, sb, 0);
  run("stream_maskB", false, true, sa, 0, sb, nb);
  run("both_masked", true, true, sa, na, sb, nb);
  run("both_serial_unmasked", true, true, sfull, ncu, sfull, ncu);
  CK(hipFree(pl));
  CK(hipFree(s));
  CK(hipFree(x));
  CK(hipFree(out));
  return 0;
}
