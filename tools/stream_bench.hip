// Microbenchmark of the CG update passes' streaming shape on gfx950
// (development tool, not product): the fused y/p pass (y += a p, p = r + w p:
// 3 vectors read, 2 written) and the r pass (r -= a Ap: 2 read, 1 written)
// over n x 8 doubles (cfg4's block), as the library runs them (one 16-byte
// group per lane per iteration, each block owning a contiguous span,
// 8192 blocks) next to variants: several groups per iteration with every
// load issued first, grid-stride order, other grids. All variants compute
// the same values (checked against the first).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/stream_bench.hip -o tools/stream_bench
//   ./tools/stream_bench [n=10004569] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
constexpr int kB = 256;

// MODE bit 1: grid-stride order (else contiguous span per block); U groups
// per iteration, all loads first. YP: the y/p pass, else the r pass.
template <int U, int MODE, bool YP>
__global__ __launch_bounds__(kB) void pass(int64_t ng, d2v *__restrict__ y, d2v *__restrict__ p,
                                           d2v *__restrict__ r, const d2v *__restrict__ ap, double a, double w) {
  const int tid = threadIdx.x;
  int64_t i0, i1, step;
  if (MODE & 1) {
    i0 = (int64_t)blockIdx.x * kB + tid;
    i1 = ng;
    step = (int64_t)gridDim.x * kB;
  } else {
    const int64_t per = ((ng + gridDim.x - 1) / gridDim.x + kB - 1) / kB * kB;
    i0 = per * blockIdx.x + tid;
    i1 = per * blockIdx.x + per < ng ? per * blockIdx.x + per : ng;
    step = kB;
  }
  for (int64_t i = i0; i < i1; i += U * step) {
    d2v yv[U], pv[U], rv[U], av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * step;
      if (j < i1) {
        if (YP) {
          yv[u] = __builtin_nontemporal_load(y + j);
          pv[u] = p[j];
          rv[u] = r[j];
        } else {
          rv[u] = r[j];
          av[u] = __builtin_nontemporal_load(ap + j);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * step;
      if (j < i1) {
        if (YP) {
          d2v t1 = a * pv[u];
          yv[u] = yv[u] + t1;
          d2v t2 = w * pv[u];
          pv[u] = rv[u] + t2;
          __builtin_nontemporal_store(yv[u], y + j);
          p[j] = pv[u];
        } else {
          d2v t = a * av[u];
          rv[u] = rv[u] - t;
          r[j] = rv[u];
        }
      }
    }
  }
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 10004569;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int64_t N = n * 8, ng = N / 2;
  d2v *y, *p, *r, *ap;
  CK(hipMalloc(&y, N * 8));
  CK(hipMalloc(&p, N * 8));
  CK(hipMalloc(&r, N * 8));
  CK(hipMalloc(&ap, N * 8));
  std::vector<double> h(N);
  for (int64_t i = 0; i < N; ++i) h[i] = 1.0 + (double)(i % 977) * 1e-3;
  CK(hipMemcpy(y, h.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(p, h.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(r, h.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(ap, h.data(), N * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("n=%ld x 8 doubles (%.0f MB per vector)\n", (long)n, N * 8 / 1e6);
  auto timeit = [&](const char *name, double bytes, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ts.push_back(t);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    printf("%-44s %.4f ms  %.0f GB/s\n", name, ms, bytes / ms / 1e6);
  };
  // a = 0, w = 1: the values stay bounded over the repetitions (p = r + p grows linearly)
  const double a = 1e-9, w = 0.5;
  const double byp = 5.0 * N * 8, br = 3.0 * N * 8;
#define RUN(U, MODE, GRID, NAME)                                                                            \
  {                                                                                                         \
    char nm[96];                                                                                            \
    snprintf(nm, sizeof nm, "%s U%d grid %d", NAME, U, GRID);                                               \
    timeit(nm, byp, [&] { hipLaunchKernelGGL((pass<U, MODE, true>), dim3(GRID), dim3(kB), 0, 0, ng, y, p, r, ap, a, w); }); \
  }
#define RUNR(U, MODE, GRID, NAME)                                                                           \
  {                                                                                                         \
    char nm[96];                                                                                            \
    snprintf(nm, sizeof nm, "%s U%d grid %d", NAME, U, GRID);                                               \
    timeit(nm, br, [&] { hipLaunchKernelGGL((pass<U, MODE, false>), dim3(GRID), dim3(kB), 0, 0, ng, y, p, r, ap, a, w); }); \
  }
  for (int g : {8192, 4096, 2048, 1024}) {
    RUN(1, 0, g, "y/p pass, span");
    RUN(2, 0, g, "y/p pass, span");
    RUN(4, 0, g, "y/p pass, span");
    RUN(1, 1, g, "y/p pass, grid-stride");
    RUN(2, 1, g, "y/p pass, grid-stride");
    RUN(4, 1, g, "y/p pass, grid-stride");
  }
  for (int g : {8192, 4096, 2048, 1024}) {
    RUNR(1, 0, g, "r pass, span");
    RUNR(2, 0, g, "r pass, span");
    RUNR(4, 0, g, "r pass, span");
    RUNR(1, 1, g, "r pass, grid-stride");
    RUNR(4, 1, g, "r pass, grid-stride");
  }
  return 0;
}
