// Gather ceiling of the column-blocked SpMV on a given matrix (development
// tool, not product; round 4). The library builds its column-blocked image
// (kry_csr::cb_*) for the matrix; then, on that image's arrays in storage
// order (column block after column block, so the x gathers of all CUs fall in
// one 2 MB block of x at a time, as in the SpMV), four kernels are timed:
//
//   library  the SpMV launch_spmv runs for one right-hand side (y = A x)
//   gather   a stream of the 4-B column indices and one 8-B gather of x per
//            entry, 16-B column loads, 4 gathers per thread per round,
//            grid-stride over the whole image (no row bookkeeping, no LDS,
//            no y): the access shape alone
//   image    the same plus the 8-B values (the whole image stream + gathers):
//            the ceiling the SpMV is measured against
//   window   random 8-B gathers from one L2-resident 2 MB window (no stream)
//   stream   the 12-B column + value stream alone (no gathers)
//
// The grid-stride kernels are not a ceiling for the SpMV (the library's
// blocks walk the column blocks in step and run faster); the ceiling model
// is max(nnz / window rate, stream time) if gathers and stream overlapped
// perfectly, and their sum if they share the load path serially.
// Each reports ms per launch and G gathers/s (nnz / time). Called from
// tools/gather_ceiling.py, which builds cfg3 and the permuted metric matrix
// and writes profiles/r04_gather_ceiling.json.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC \
//     tools/gather_ceiling.hip -o tools/libgather_ceiling.so -Lkrylov_amd -lkrylov_hip \
//     -Wl,-rpath,'$ORIGIN/../krylov_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../include/krylov_hip.h"
#include "../krylov_amd/csrc/device.hpp"

using namespace kry;

typedef int gi4 __attribute__((ext_vector_type(4)));
typedef double gd2 __attribute__((ext_vector_type(2)));

template <bool VAL, bool GATHER = true>
__global__ __launch_bounds__(256) void gc_stream(const gi4 *__restrict__ col, const gd2 *__restrict__ val, int64_t nnz,
                                                 const double *__restrict__ x, double *__restrict__ out) {
  const int64_t nq = (nnz + 3) / 4;
  double s = 0.0;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
    const gi4 c = __builtin_nontemporal_load(col + q);
    double a0 = 1.0, a1 = 1.0, a2 = 1.0, a3 = 1.0;
    if (VAL) {
      const gd2 v0 = __builtin_nontemporal_load(val + 2 * q), v1 = __builtin_nontemporal_load(val + 2 * q + 1);
      a0 = v0.x; a1 = v0.y; a2 = v1.x; a3 = v1.y;
    }
    const int64_t e = 4 * q;
    if (GATHER) {
      const double x0 = x[c.x];
      const double x1 = e + 1 < nnz ? x[c.y] : 0.0;
      const double x2 = e + 2 < nnz ? x[c.z] : 0.0;
      const double x3 = e + 3 < nnz ? x[c.w] : 0.0;
      s += a0 * x0 + a1 * x1 + a2 * x2 + a3 * x3;
    } else {
      s += a0 * (double)c.x + a1 * (double)c.y + a2 * (double)c.z + a3 * (double)c.w;
    }
  }
  if (s == 1234.5678) out[0] = s;  // keeps the loads; never true for these inputs
}

__global__ __launch_bounds__(256) void gc_window(const double *__restrict__ x, int64_t span, int rounds,
                                                 double *__restrict__ out) {
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
  double s = 0.0;
  for (int r = 0; r < rounds; ++r) {
    double v[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      h ^= h << 13; h ^= h >> 17; h ^= h << 5;
      v[g] = x[h % (uint32_t)span];
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) s += v[g];
  }
  if (s == 1234.5678) out[0] = s;
}

extern "C" int gc_run(int64_t n, int64_t nnz, const int *ip, const int *ix, const double *dv, int reps,
                      double *res /* [0] library ms, [1] gather ms, [2] image ms, [3] window G/s, [4] nb, [5] cols,
                                  [6] stream ms */) {
  kry_ctx *ctx;
  if (kry_ctx_create(0, &ctx) != KRY_OK) return -1;
  kry_csr *A;
  if (kry_csr_create(ctx, n, nnz, ip, ix, dv, KRY_F64, KRY_I32, &A) != KRY_OK) return -2;
  if (A->cb_nb == 0) return -3;
  std::vector<double> xh(n);
  for (int64_t i = 0; i < n; ++i) xh[i] = 1.0 + 1e-3 * (double)((i * 2654435761ull) % 1000);
  double *x, *y, *o;
  hipMalloc(&x, n * 8 + 512);
  hipMalloc(&y, n * 8 + 512);
  hipMalloc(&o, 64);
  hipMemcpy(x, xh.data(), n * 8, hipMemcpyHostToDevice);
  hipStream_t st = ctx->stream;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](auto launch) {
    launch();
    hipStreamSynchronize(st);
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      hipEventRecord(e0, st);
      launch();
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      ts.push_back(t);
    }
    std::sort(ts.begin(), ts.end());
    return (double)ts[ts.size() / 2];
  };
  res[0] = timeit([&] {
    launch_spmv<double, double, int>(A, 1, SrcPlain<double>{x, 1}, EpiStore<double>{y, 1}, nullptr, nullptr,
                                     nullptr, 0, st);
  });
  const gi4 *col = static_cast<const gi4 *>(A->cb_col);
  const gd2 *val = static_cast<const gd2 *>(A->cb_val);
  res[1] = timeit([&] { hipLaunchKernelGGL(gc_stream<false>, dim3(8192), dim3(256), 0, st, col, val, nnz, x, o); });
  res[2] = timeit([&] { hipLaunchKernelGGL(gc_stream<true>, dim3(8192), dim3(256), 0, st, col, val, nnz, x, o); });
  res[6] = timeit([&] {
    hipLaunchKernelGGL((gc_stream<true, false>), dim3(8192), dim3(256), 0, st, col, val, nnz, x, o);
  });
  const int64_t span = std::min<int64_t>(n, 262144);
  const int rounds = 64;
  const double wms = timeit([&] { hipLaunchKernelGGL(gc_window, dim3(8192), dim3(256), 0, st, x, span, rounds, o); });
  res[3] = 8192.0 * 256 * rounds * 8 / (wms * 1e-3) / 1e9;
  res[4] = (double)A->cb_nb;
  res[5] = (double)A->cb_cols;
  hipFree(x);
  hipFree(y);
  hipFree(o);
  kry_csr_destroy(A);
  kry_ctx_destroy(ctx);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
