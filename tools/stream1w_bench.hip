// Streaming rate at one or two waves per SIMD (development tool, not
// product; round 4): the premise of a streamed-MGS kernel at 256 threads per
// CU (one wave per SIMD, 512 registers per lane), which could keep w and most
// of the next basis vector on chip. Each block of T threads is alone on its
// CU (LDS_PAD bytes of static LDS) and streams its segment of a 80.6 MB
// vector with buffer loads, DEPTH chunks of U 16-B granules per lane in
// flight, accumulating a dot product with a second, register-held operand
// (W_REGS granules per lane, written back at the end so it stays live).
// Every pass reads a different vector of a 31-vector basis (no cache reuse).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream1w_bench.hip -o tools/stream1w_bench
//   ./tools/stream1w_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int T, int NV, int U, int W_REGS>
__global__ __launch_bounds__(T) void stream1w(const double *__restrict__ basis, size_t stride, int passes,
                                              double *__restrict__ wout, double *__restrict__ out) {
  __shared__ double pad[(160 * 1024 - 4096) / 8];  // one block per CU
  const int tid = threadIdx.x;
  const int64_t seg = (int64_t)NV * T * 2;  // doubles per block
  double w[W_REGS][2];
#pragma unroll
  for (int i = 0; i < W_REGS; ++i) {
    w[i][0] = 1.0 + 1e-3 * i;
    w[i][1] = 2.0 - 1e-3 * i;
  }
  double acc = 0.0;
  for (int p = 0; p < passes; ++p) {
    const double *v = basis + stride * (size_t)(p % 31) + (int64_t)blockIdx.x * seg;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(v), 0, (int)(seg * 8), 0x00020000);
    u4 buf[2][U];
#pragma unroll
    for (int u = 0; u < U; ++u) buf[0][u] = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16, u * T * 16, 2);
#pragma unroll
    for (int c = 0; c < NV / U; ++c) {
      const int b = c & 1;
      if (c + 1 < NV / U) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          buf[b ^ 1][u] = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16, ((c + 1) * U + u) * T * 16, 2);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double2 d = __builtin_bit_cast(double2, buf[b][u]);
        const int g = (c * U + u) % W_REGS;
        acc += d.x * w[g][0] + d.y * w[g][1];
        w[g][0] -= 1e-9 * d.x;
      }
    }
  }
  if (tid == 0) pad[0] = acc;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < W_REGS; ++i) wout[((int64_t)blockIdx.x * W_REGS + i) * T + tid] = w[i][0] + w[i][1];
  if (acc == 1234.5 || pad[0] == 4321.5) out[0] = acc;
}

int main() {
  const int64_t n = 10077696;
  const size_t stride = (size_t)n + 4096;
  double *basis, *wout, *out;
  CK(hipMalloc(&basis, stride * 31 * 8));
  CK(hipMemset(basis, 0, stride * 31 * 8));
  CK(hipMalloc(&wout, (size_t)256 * 80 * 512 * 8));
  CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int passes = 31;
  auto run = [&](const char *name, auto kern, int T, int NV) {
    const int G = (int)((n + (int64_t)NV * T * 2 - 1) / ((int64_t)NV * T * 2));
    hipLaunchKernelGGL(kern, dim3(G), dim3(T), 0, 0, (const double *)basis, stride, passes, wout, out);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(kern, dim3(G), dim3(T), 0, 0, (const double *)basis, stride, passes, wout, out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ts.push_back(t);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[2] * 1e3 / passes;
    printf("%-48s grid %3d: %7.2f us per 80.6 MB pass, %6.0f GB/s\n", name, G, us, n * 8.0 / (us * 1e-6) / 1e9);
  };
  run("512 thr (2 waves/SIMD), NV 40, U 2, w 40", stream1w<512, 40, 2, 40>, 512, 40);
  run("512 thr (2 waves/SIMD), NV 40, U 4, w 40", stream1w<512, 40, 4, 40>, 512, 40);
  run("256 thr (1 wave/SIMD), NV 78, U 2, w 78", stream1w<256, 78, 2, 78>, 256, 78);
  run("256 thr (1 wave/SIMD), NV 78, U 3, w 78", stream1w<256, 78, 3, 78>, 256, 78);
  run("256 thr (1 wave/SIMD), NV 78, U 6, w 78", stream1w<256, 78, 6, 78>, 256, 78);
  run("256 thr (1 wave/SIMD), NV 78, U 6, w 8", stream1w<256, 78, 6, 8>, 256, 78);
  run("256 thr (1 wave/SIMD), NV 80, U 8, w 8", stream1w<256, 80, 8, 8>, 256, 80);
  return 0;
}
