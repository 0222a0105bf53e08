// Standalone SpMV microbenchmark for gfx950 (development tool, not product).
// Builds the BASELINE metric matrix (3-D 15-point stencil, m^3) on the host,
// uploads it through the library's C-ABI (kry_csr_create -> SELL-64 image),
// and times the library's SpMV launches next to a pure streaming-read ceiling,
// checking every variant bitwise against a host csr_matvec.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     tools/spmv_bench.hip -o tools/spmv_bench -Lkrylov_amd -lkrylov_hip -Wl,-rpath,'$ORIGIN/../krylov_amd'
//   ./tools/spmv_bench [m=216] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../krylov_amd/csrc/device.hpp"

using namespace kry;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)
#define KC(x)                                                                             \
  do {                                                                                    \
    int r = (x);                                                                          \
    if (r != KRY_OK) {                                                                    \
      fprintf(stderr, "%s:%d %s: %d %s\n", __FILE__, __LINE__, #x, r, kry_last_error()); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

static void build_stencil(int m, std::vector<int> &ip, std::vector<int> &ix, std::vector<double> &dv) {
  const int64_t n = (int64_t)m * m * m;
  ip.assign(n + 1, 0);
  ix.clear();
  dv.clear();
  ix.reserve(n * 15);
  dv.reserve(n * 15);
  struct Nb { int64_t off; int di, dj, dk; };
  std::vector<Nb> nb;
  for (int dk = -1; dk <= 1; ++dk)
    for (int dj = -1; dj <= 1; ++dj)
      for (int di = -1; di <= 1; ++di) {
        int nz = (di != 0) + (dj != 0) + (dk != 0);
        if (nz == 0 || nz == 1 || nz == 3) nb.push_back({(int64_t)dk * m * m + dj * m + di, di, dj, dk});
      }
  std::sort(nb.begin(), nb.end(), [](const Nb &a, const Nb &b) { return a.off < b.off; });
  for (int64_t r = 0; r < n; ++r) {
    int i = r % m, j = (r / m) % m, k = r / ((int64_t)m * m);
    for (auto &q : nb) {
      int ii = i + q.di, jj = j + q.dj, kk = k + q.dk;
      if (ii < 0 || ii >= m || jj < 0 || jj >= m || kk < 0 || kk >= m) continue;
      ix.push_back((int)(r + q.off));
      dv.push_back(q.off == 0 ? 14.0 : -1.0);
    }
    ip[r + 1] = (int)ix.size();
  }
}

__global__ __launch_bounds__(256) void read_ceiling(const int4 *__restrict__ a, int64_t na, const double2 *__restrict__ b,
                                                    int64_t nb, double *out) {
  double s = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) {
    int4 v = a[i];
    s += v.x + v.w;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride) {
    double2 v = b[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}


// PMC calibration: the SELL matrix stream alone, with the library kernel's
// access widths (4-B index + 8-B value per lane, nontemporal, coalesced per
// wave). Algorithmic bytes = 12 * nslots; FETCH_SIZE / that = the counter's
// scale for this access pattern (MI355X_MICROARCH.md "HBM": uncalibrated
// widths must be calibrated on a known byte count).
__global__ __launch_bounds__(256) void sell_stream_calib(const int *__restrict__ idx, const double *__restrict__ val,
                                                         int64_t ns, double *out) {
  double s = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride) {
    const int c = __builtin_nontemporal_load(idx + i);
    const double v = __builtin_nontemporal_load(val + i);
    s += c >= 0 ? v : 0.0;
  }
  if (s == 12345.678) out[0] = s;
}


typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef double v2d __attribute__((ext_vector_type(2)));
// ---- prototype: SELL-64 with G consecutive columns per lane (slot-major) ----
// slot(s, j, lane) = base_s + (j / G) * 64 G + lane * G + j % G; width padded to
// a multiple of G with index -1. Index loads are G*4 B per lane, value loads
// G*8 B per lane (two 16-B loads for G = 4).
template <int G, int UNRG, bool CGP, bool NT = true, int MINW = 1>
__global__ __launch_bounds__(256, MINW) void spmv_sellg(const int64_t *__restrict__ sptr, const int *__restrict__ swid,
                                                 const int *__restrict__ sidx, const double *__restrict__ sval,
                                                 int64_t nslices, int64_t n, const double *__restrict__ x,
                                                 const double *__restrict__ pold, const double *__restrict__ omp,
                                                 double *__restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4, wg = (int64_t)g * 4 + wid;
  const int64_t s0 = nslices * wg / W, s1 = nslices * (wg + 1) / W;
  const double om = CGP ? omp[0] : 0.0;
  for (int64_t s = s0; s < s1; ++s) {
    const int ngrp = swid[s] / G;
    const int *ci = sidx + sptr[s] + lane * G;
    const double *cv = sval + sptr[s] + lane * G;
    double acc = 0.0;
    for (int q0 = 0; q0 < ngrp; q0 += UNRG) {
      int col[UNRG][G];
      double a[UNRG][G];
#pragma unroll
      for (int uq = 0; uq < UNRG; ++uq) {
        const bool in = q0 + uq < ngrp;
        const int64_t off = (int64_t)(q0 + uq) * 64 * G;
        if constexpr (G == 4) {
          v4i c4 = in ? __builtin_nontemporal_load(reinterpret_cast<const v4i *>(ci + off)) : v4i{-1, -1, -1, -1};
          col[uq][0] = c4.x; col[uq][1] = c4.y; col[uq][2] = c4.z; col[uq][3] = c4.w;
          v2d v0 = in ? __builtin_nontemporal_load(reinterpret_cast<const v2d *>(cv + off)) : v2d{0, 0};
          v2d v1 = in ? __builtin_nontemporal_load(reinterpret_cast<const v2d *>(cv + off + 2)) : v2d{0, 0};
          a[uq][0] = v0.x; a[uq][1] = v0.y; a[uq][2] = v1.x; a[uq][3] = v1.y;
        } else if constexpr (G == 2) {
          v2i c2 = in ? __builtin_nontemporal_load(reinterpret_cast<const v2i *>(ci + off)) : v2i{-1, -1};
          col[uq][0] = c2.x; col[uq][1] = c2.y;
          v2d v0 = in ? __builtin_nontemporal_load(reinterpret_cast<const v2d *>(cv + off)) : v2d{0, 0};
          a[uq][0] = v0.x; a[uq][1] = v0.y;
        } else {
          if (NT) {
            col[uq][0] = in ? __builtin_nontemporal_load(ci + off) : -1;
            a[uq][0] = in ? __builtin_nontemporal_load(cv + off) : 0.0;
          } else {
            col[uq][0] = in ? ci[off] : -1;
            a[uq][0] = in ? cv[off] : 0.0;
          }
        }
      }
      double xv[UNRG][G];
#pragma unroll
      for (int uq = 0; uq < UNRG; ++uq)
#pragma unroll
        for (int e = 0; e < G; ++e) {
          const int j = col[uq][e];
          double v = j >= 0 ? x[j] : 0.0;
          if (CGP) { const double t = om * (j >= 0 ? pold[j] : 0.0); v = v + t; }
          xv[uq][e] = v;
        }
#pragma unroll
      for (int uq = 0; uq < UNRG; ++uq)
#pragma unroll
        for (int e = 0; e < G; ++e)
          if (col[uq][e] >= 0) { const double p = a[uq][e] * xv[uq][e]; acc = acc + p; }
    }
    const int64_t row = s * 64 + lane;
    if (row < n) y[row] = acc;
  }
}

int main(int argc, char **argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 216;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<int> ip, ix;
  std::vector<double> dv;
  build_stencil(m, ip, ix, dv);
  const int64_t n = ip.size() - 1, nnz = ix.size();
  const double S = nnz * 12.0 + (n + 1) * 4.0 + 2.0 * n * 8.0;
  printf("m=%d n=%ld nnz=%ld S=%.4f GB\n", m, n, nnz, S / 1e9);

  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  kry_csr *A;
  auto t0 = std::chrono::steady_clock::now();
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
  printf("upload + SELL-64 build %.2fs: %ld slices, %ld slots (%.2f%% padding), %ld irregular\n",
         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), A->nslices, A->nslots,
         100.0 * (A->nslots - nnz) / nnz, A->nirregular);
  printf("x-window groups: %ld of %ld windowed\n", A->nwindowed, A->ngroups);

  double *d_x, *d_y, *d_p, *d_ap, *d_om, *d_out, *part;
  CK(hipMalloc(&d_x, n * 8));
  CK(hipMalloc(&d_y, n * 8));
  CK(hipMalloc(&d_p, n * 8));
  CK(hipMalloc(&d_ap, n * 8));
  CK(hipMalloc(&d_om, 64));
  CK(hipMalloc(&d_out, 64));
  CK(hipMalloc(&part, kMaxGrid * 8));
  std::vector<double> xh(n);
  for (int64_t i = 0; i < n; ++i) xh[i] = 1.0 + 1e-3 * (double)((i * 2654435761u) % 1000);
  CK(hipMemcpy(d_x, xh.data(), n * 8, hipMemcpyHostToDevice));
  const double om = 0.25;
  CK(hipMemcpy(d_om, &om, 8, hipMemcpyHostToDevice));
  // host references: y = A x, p = x + om x, Ap = A p (sequential, no FMA)
  std::vector<double> yref(n), y2ref(n), pref(n);
  for (int64_t i = 0; i < n; ++i) {
    const double t = om * xh[i];
    pref[i] = xh[i] + t;
  }
  for (int64_t i = 0; i < n; ++i) {
    double s = 0, s2 = 0;
    for (int e = ip[i]; e < ip[i + 1]; ++e) {
      const double p = dv[e] * xh[ix[e]];
      s = s + p;
      const double p2 = dv[e] * pref[ix[e]];
      s2 = s2 + p2;
    }
    yref[i] = s;
    y2ref[i] = s2;
  }

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto report = [&](const char *name, double bytes, auto &&launch) {
    launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    float tot = 0, best = 1e30;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
      best = std::min(best, ms);
    }
    printf("%-40s avg %.4f ms  best %.4f ms  %.0f GB/s  %.1f%% of 8 TB/s\n", name, tot / reps, best,
           bytes / (tot / reps) / 1e6, 100.0 * bytes / (tot / reps) / 1e6 / 8000.0);
  };
  auto check = [&](const char *name, const double *dev, const std::vector<double> &ref) {
    std::vector<double> h(n);
    CK(hipMemcpy(h.data(), dev, n * 8, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += memcmp(&h[i], &ref[i], 8) != 0;
    printf("  %-38s bitwise mismatches vs host csr_matvec: %ld\n", name, bad);
  };

  report("read ceiling (SELL idx+val, 16 B/lane)", nnz * 12.0, [&] {
    hipLaunchKernelGGL(read_ceiling, dim3(2048), dim3(256), 0, 0, (const int4 *)A->sidx, nnz / 4,
                       (const double2 *)A->sval, nnz / 2, d_out);
  });
  report("SELL stream calibration (4+8 B/lane nt)", A->nslots * 12.0, [&] {
    hipLaunchKernelGGL(sell_stream_calib, dim3(8192), dim3(256), 0, 0, (const int *)A->sidx,
                       (const double *)A->sval, A->nslots, d_out);
  });
  report("library SELL SpMV y = A x", S, [&] {
    launch_spmv<double, double, int>(A, 1, SrcPlain<double>{d_x, 1}, EpiStore<double>{d_y, 1}, nullptr, nullptr,
                                     nullptr, 0, 0);
  });
  check("y = A x", d_y, yref);
  report("library SELL SpMV + <x, y> partials", S, [&] {
    launch_spmv<double, double, int>(A, 1, SrcPlain<double>{d_x, 1}, EpiStoreDot<double>{d_y, d_x, nullptr, 1},
                                     part, nullptr, nullptr, 0, 0);
  });
  check("y = A x (dot epilogue)", d_y, yref);
  SrcCgP<double> src{d_x, d_x, d_om, 1, 0};
  report("library CG-fused p-update+SpMV+<p,Ap>", S + 16.0 * n, [&] {
    launch_spmv<double, double, int>(A, 1, src, EpiCgAp<double>{d_ap, d_p, src, nullptr, 1}, part, nullptr,
                                     nullptr, 0, 0);
  });
  check("Ap (CG-fused)", d_ap, y2ref);
  check("p  (CG-fused)", d_p, pref);

  {
    const int G = 1;
    const int64_t ns = (n + 63) / 64;
    std::vector<int64_t> sp(ns + 1, 0);
    std::vector<int> sw(ns);
    for (int64_t s2 = 0; s2 < ns; ++s2) {
      int w = 0;
      for (int64_t r = s2 * 64; r < std::min<int64_t>(n, s2 * 64 + 64); ++r) w = std::max(w, ip[r + 1] - ip[r]);
      sw[s2] = w;
      sp[s2 + 1] = sp[s2] + 64 * w;
    }
    const int64_t slots = sp[ns];
    std::vector<int> si(slots + 1024, -1);
    std::vector<double> sv(slots + 1024, 0.0);
    for (int64_t s2 = 0; s2 < ns; ++s2)
      for (int l = 0; l < 64; ++l) {
        const int64_t r = s2 * 64 + l;
        if (r >= n) continue;
        for (int e = ip[r]; e < ip[r + 1]; ++e) {
          const int j = e - ip[r];
          const int64_t slot = sp[s2] + (int64_t)(j / G) * 64 * G + l * G + j % G;
          si[slot] = ix[e];
          sv[slot] = dv[e];
        }
      }
    int64_t *d_sp;
    int *d_sw, *d_si;
    double *d_sv;
    CK(hipMalloc(&d_sp, sp.size() * 8));
    CK(hipMalloc(&d_sw, sw.size() * 4));
    CK(hipMalloc(&d_si, si.size() * 4));
    CK(hipMalloc(&d_sv, sv.size() * 8));
    CK(hipMemcpy(d_sp, sp.data(), sp.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sw, sw.data(), sw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_si, si.data(), si.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sv, sv.data(), sv.size() * 8, hipMemcpyHostToDevice));
#define PV(UNR, NTF, MINW, GRID)                                                                                 \
    {                                                                                                            \
      char nm[96];                                                                                               \
      snprintf(nm, 96, "proto U%d nt=%d minw=%d grid=%d", UNR, (int)NTF, MINW, GRID);                            \
      report(nm, S, [&] {                                                                                        \
        hipLaunchKernelGGL((spmv_sellg<1, UNR, false, NTF, MINW>), dim3(GRID), dim3(256), 0, 0, d_sp, d_sw, d_si, \
                           d_sv, ns, n, d_x, d_x, d_om, d_y);                                                    \
      });                                                                                                        \
    }
    PV(16, true, 1, 2048)
    PV(16, false, 1, 2048)
    PV(8, true, 1, 2048)
    PV(4, true, 1, 2048)
    PV(24, true, 1, 2048)
    PV(16, true, 1, 1024)
    PV(16, true, 1, 4096)
    PV(16, true, 1, 8192)
    PV(8, true, 2, 2048)
    PV(8, true, 4, 4096)
    PV(16, true, 2, 4096)
    check("last proto", d_y, yref);
  }
  KC(kry_csr_destroy(A));
  KC(kry_ctx_destroy(ctx));
  return 0;
}
