// Microbenchmark (development tool, not product) of a paired-row SELL-128
// SpMV for general CSR on gfx950, against the library's compact SELL-64
// kernel (KRY_SPMV_DIA=0) and its DIA kernel on the metric matrix (15-point
// 216^3). The image: slices of 128 rows, slot column j holds the j-th entry
// of every row, rows interleaved so that lane l owns rows 2l and 2l + 1 and
// makes ONE 16-B value load and ONE 4-B load of its two uint16 column deltas
// (over a per-slot-column int32 base, 0xFFFF = padding) per slot column.
// When the two columns are adjacent (rows 2l, 2l + 1 of a banded or stencil
// matrix), one 16-B x load serves both; otherwise the second is its own
// 8-B load behind a branch that a wave skips when all its lanes paired.
// Each row is still summed from 0 in stored order (bitwise csr_matvec,
// checked against the host).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     tools/sellp_bench.hip -o tools/sellp_bench -Lkrylov_amd -lkrylov_hip -Wl,-rpath,'$ORIGIN/../krylov_amd'
//   ./tools/sellp_bench [m=216] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/krylov_hip.h"
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
  std::vector<int64_t> offs;
  std::vector<int> ds;
  for (int dk = -1; dk <= 1; ++dk)
    for (int dj = -1; dj <= 1; ++dj)
      for (int di = -1; di <= 1; ++di) {
        const int nz = (di != 0) + (dj != 0) + (dk != 0);
        if (nz == 2) continue;  // 15-point: centre, faces, corners
        offs.push_back((int64_t)dk * m * m + dj * m + di);
        ds.push_back((di + 1) | (dj + 1) << 2 | (dk + 1) << 4);
      }
  std::vector<int> ord(offs.size());
  for (size_t q = 0; q < ord.size(); ++q) ord[q] = (int)q;
  std::sort(ord.begin(), ord.end(), [&](int a, int b) { return offs[a] < offs[b]; });
  for (int64_t r = 0; r < n; ++r) {
    const int i = r % m, j = (r / m) % m, k = (int)(r / ((int64_t)m * m));
    for (int q : ord) {
      const int di = (ds[q] & 3) - 1, dj = (ds[q] >> 2 & 3) - 1, dk = (ds[q] >> 4 & 3) - 1;
      const int ii = i + di, jj = j + dj, kk = k + dk;
      if (ii < 0 || ii >= m || jj < 0 || jj >= m || kk < 0 || kk >= m) continue;
      ix.push_back((int)(r + offs[q]));
      dv.push_back(offs[q] == 0 ? 14.0 : -1.0);
    }
    ip[r + 1] = (int)ix.size();
  }
}

constexpr int kPS = 128;  // rows per slice

struct SellP {
  int64_t nslices = 0, nslots = 0;
  int max_width = 0;
  std::vector<int64_t> sptr;    // nslices + 1, in slots (kPS per slot column)
  std::vector<int> width;       // nslices
  std::vector<int> cbase;       // nslots / kPS (+ pad)
  std::vector<uint16_t> delta;  // nslots (+ pad)
  std::vector<double> val;      // nslots (+ pad)
};

static bool build_sellp(int64_t n, const std::vector<int> &ip, const std::vector<int> &ix, const std::vector<double> &dv,
                        SellP &P) {
  P.nslices = (n + kPS - 1) / kPS;
  P.width.assign(P.nslices, 0);
  P.sptr.assign(P.nslices + 1, 0);
  for (int64_t s = 0; s < P.nslices; ++s) {
    int w = 0;
    for (int64_t r = s * kPS; r < std::min<int64_t>(n, (s + 1) * kPS); ++r) w = std::max(w, ip[r + 1] - ip[r]);
    P.width[s] = w;
    P.sptr[s + 1] = P.sptr[s] + (int64_t)w * kPS;
    P.max_width = std::max(P.max_width, w);
  }
  P.nslots = P.sptr.back();
  P.cbase.assign(P.nslots / kPS + 64, 0);
  P.delta.assign(P.nslots + 1024, 0xFFFF);
  P.val.assign(P.nslots + 1024, 0.0);
  bool ok = true;
  for (int64_t s = 0; s < P.nslices; ++s) {
    const int64_t r0 = s * kPS, r1 = std::min<int64_t>(n, r0 + kPS);
    for (int j = 0; j < P.width[s]; ++j) {
      int lo = 0x7fffffff, hi = -1;
      for (int64_t r = r0; r < r1; ++r)
        if (ip[r] + j < ip[r + 1]) {
          lo = std::min(lo, ix[ip[r] + j]);
          hi = std::max(hi, ix[ip[r] + j]);
        }
      if (hi < 0) lo = hi = 0;
      if (hi - lo > 65534) ok = false;
      const int64_t colj = P.sptr[s] / kPS + j;
      P.cbase[colj] = lo;
      for (int64_t r = r0; r < r1; ++r) {
        const int64_t slot = P.sptr[s] + (int64_t)j * kPS + (r - r0);
        if (ip[r] + j < ip[r + 1]) {
          P.delta[slot] = (uint16_t)(ix[ip[r] + j] - lo);
          P.val[slot] = dv[ip[r] + j];
        }
      }
    }
  }
  return ok;
}

typedef double d2v __attribute__((ext_vector_type(2)));

// MODE bits: 1 never pair (two 8-B gathers per lane and slot column);
// 2 nontemporal delta loads; 4 one slice per wave (grid over the slices);
// 8 the unpaired second loads of a round behind one wave-level branch
template <int UNR, int MODE, class Src, class Epi>
__global__ __launch_bounds__(256) void sellp_kernel(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                    const int *__restrict__ cbase, const uint32_t *__restrict__ dpair,
                                                    const double *__restrict__ val, int64_t nslices, int64_t n, Src src,
                                                    Epi epi, double *__restrict__ part) {
  constexpr bool NOPAIR = (MODE & 1) != 0, NTD = (MODE & 2) != 0, ONE = (MODE & 4) != 0, WB = (MODE & 8) != 0;
  __shared__ double red[256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4, m = (int64_t)g * 4 + wid;
  const int64_t s_begin = ONE ? m : nslices * m / W, s_end = ONE ? (m < nslices ? m + 1 : m) : nslices * (m + 1) / W;
  const auto bs = src.template bind<1>(0);
  double dacc = 0.0;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * kPS + 2 * lane;
    const int *cb = cbase + base / kPS;                        // wave-uniform: scalar loads
    const uint32_t *cd = dpair + base / 2 + lane;              // two uint16 deltas per lane
    const d2v *cv = reinterpret_cast<const d2v *>(val + base) + lane;
    double acc0 = 0.0, acc1 = 0.0;
    for (int j0 = 0; j0 < w; j0 += UNR) {
      int b[UNR];
      uint32_t d[UNR];
      d2v a[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        b[u] = cb[j0 + u];  // padded: read unconditionally
        if (j0 + u < w) {
          d[u] = NTD ? __builtin_nontemporal_load(cd + (int64_t)(j0 + u) * (kPS / 2)) : cd[(int64_t)(j0 + u) * (kPS / 2)];
          a[u] = __builtin_nontemporal_load(cv + (int64_t)(j0 + u) * (kPS / 2));
        } else {
          d[u] = 0xFFFFFFFFu;
          a[u] = d2v{0.0, 0.0};
        }
      }
      double x0[UNR], x1[UNR];
      bool v0[UNR], v1[UNR], need[UNR];
      int64_t c1s[UNR];
      bool anyneed = false;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t lo = d[u] & 0xFFFFu, hi = d[u] >> 16;
        v0[u] = lo != 0xFFFFu;
        v1[u] = hi != 0xFFFFu;
        const int64_t c0 = (int64_t)b[u] + lo, c1 = (int64_t)b[u] + hi;
        if (NOPAIR) {
          x0[u] = v0[u] ? bs(c0, 0) : 0.0;
          x1[u] = v1[u] ? bs(c1, 0) : 0.0;
        } else {
          const bool pr = v0[u] && v1[u] && c1 == c0 + 1;
          double xp[2];
          bs.pair(v0[u] ? c0 : (v1[u] ? c1 : 0), xp);
          x0[u] = xp[0];
          x1[u] = pr ? xp[1] : xp[0];
          need[u] = v0[u] && v1[u] && !pr;
          c1s[u] = c1;
          anyneed = anyneed || need[u];
          if (!WB && need[u]) x1[u] = bs(c1, 0);
        }
      }
      if (WB && !NOPAIR && __any(anyneed)) {
#pragma unroll
        for (int u = 0; u < UNR; ++u)
          if (need[u]) x1[u] = bs(c1s[u], 0);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const double p0 = a[u].x * x0[u];
        const double p1 = a[u].y * x1[u];
        const double t0 = acc0 + p0;
        const double t1 = acc1 + p1;
        acc0 = v0[u] ? t0 : acc0;
        acc1 = v1[u] ? t1 : acc1;
      }
    }
    if (row + 1 < n) {
      double xi[2];
      bs.pair(row, xi);
      const double pend[2] = {acc0, acc1};
      dacc += epi.rows2(row, pend, xi);
    } else if (row < n) {
      dacc += epi(row, 0, acc0, bs(row, 0));
    }
  }
  red[tid] = dacc;
  block_tree_reduce(red, 256, 1);
  if (tid == 0) part[g] = red[0];
}

int main(int argc, char **argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 216;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<int> ip, ix;
  std::vector<double> dv;
  build_stencil(m, ip, ix, dv);
  const int64_t n = (int64_t)ip.size() - 1, nnz = ix.size();
  SellP P;
  const bool ok = build_sellp(n, ip, ix, dv, P);
  printf("m=%d n=%ld nnz=%ld sellp slices=%ld slots=%ld (padding %.2f%%) max_width=%d compact=%d\n", m, (long)n,
         (long)nnz, (long)P.nslices, (long)P.nslots, 100.0 * (P.nslots - nnz) / nnz, P.max_width, (int)ok);
  if (!ok) return 1;
  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  kry_csr *Adia, *Asell;
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &Adia));
  setenv("KRY_SPMV_DIA", "0", 1);
  kry_csr *Apair;
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &Apair));
  setenv("KRY_SPMV_PAIR", "0", 1);
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &Asell));
  printf("library images: dia=%d sell compact=%d sell slots=%ld\n", (int)Adia->dia, (int)Asell->compact,
         (long)Asell->nslots);
  std::vector<double> xh(n);
  for (int64_t i = 0; i < n; ++i) xh[i] = 1.0 + (double)((i * 7919) % 1000) * 1e-3;
  kry_vec *xv, *yv;
  KC(kry_vec_create(ctx, n, 1, KRY_F64, &xv));
  KC(kry_vec_create(ctx, n, 1, KRY_F64, &yv));
  KC(kry_vec_upload(xv, xh.data()));
  double *x = (double *)xv->d, *y = (double *)yv->d, *part;
  CK(hipMalloc(&part, (size_t)65536 * 8));
  int64_t *d_sptr;
  int *d_width, *d_cbase;
  uint16_t *d_delta;
  double *d_val;
  CK(hipMalloc(&d_sptr, P.sptr.size() * 8));
  CK(hipMalloc(&d_width, P.width.size() * 4));
  CK(hipMalloc(&d_cbase, P.cbase.size() * 4));
  CK(hipMalloc(&d_delta, P.delta.size() * 2));
  CK(hipMalloc(&d_val, P.val.size() * 8));
  CK(hipMemcpy(d_sptr, P.sptr.data(), P.sptr.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_width, P.width.data(), P.width.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_cbase, P.cbase.data(), P.cbase.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_delta, P.delta.data(), P.delta.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_val, P.val.data(), P.val.size() * 8, hipMemcpyHostToDevice));
  hipStream_t st = ctx->stream;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double img_p = (double)P.nslots * 10 + (double)P.nslots / kPS * 4 + P.nslices * 12.0 + 2.0 * n * 8;
  const double img_s = (double)Asell->nslots * 10 + (double)Asell->nslots / 64 * 4 + Asell->nslices * 12.0 + 2.0 * n * 8;
  const double img_d = (double)Adia->dia_nslots * 8 + (double)Adia->dia_nslots / 128 * 20 + 2.0 * n * 8;
  auto timeit = [&](const char *name, double bytes, auto launch) {
    launch();
    CK(hipStreamSynchronize(st));
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, st));
      launch();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ts.push_back(t);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    printf("%-48s %.4f ms  %.3f GB/launch  %.0f GB/s  %.3f of 8 TB/s\n", name, ms, bytes / 1e9, bytes / ms / 1e6,
           bytes / ms / 1e6 / 8000.0);
    return ms;
  };
  // host reference y = A x (csr_matvec order)
  std::vector<double> ref(n), got(n);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&, t] {
        for (int64_t r = n * t / 8; r < n * (t + 1) / 8; ++r) {
          double acc = 0.0;
          for (int e = ip[r]; e < ip[r + 1]; ++e) {
            volatile double p = dv[e] * xh[ix[e]];
            acc = acc + p;
          }
          ref[r] = acc;
        }
      });
    for (auto &t : th) t.join();
  }
  auto check = [&](const char *name) {
    CK(hipMemcpy(got.data(), y, n * 8, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t r = 0; r < n; ++r) bad += memcmp(&got[r], &ref[r], 8) != 0;
    if (bad) printf("  !! %s: %ld rows differ from host csr_matvec\n", name, (long)bad);
  };
  for (int rep = 0; rep < 2; ++rep) {
    timeit("library DIA (spmv_dia_kernel, EpiApDot)", img_d, [&] {
      int G;
      launch_spmv<double, double, int>(Adia, 1, SrcPlain<double>{x, 1}, EpiApDot<double>{y, nullptr, 1}, part, &G,
                                       nullptr, 0, st);
    });
    check("library DIA");
    timeit("library SELL-64 compact (EpiApDot)", img_s, [&] {
      int G;
      launch_spmv<double, double, int>(Asell, 1, SrcPlain<double>{x, 1}, EpiApDot<double>{y, nullptr, 1}, part, &G,
                                       nullptr, 0, st);
    });
    check("library SELL-64");
    timeit("library pair (spmv_pair_kernel, EpiApDot)", img_p, [&] {
      int G;
      launch_spmv<double, double, int>(Apair, 1, SrcPlain<double>{x, 1}, EpiApDot<double>{y, nullptr, 1}, part, &G,
                                       nullptr, 0, st);
    });
    check("library pair");
#define PK(UNR, MODE, GRID, NAME)                                                                                     \
  {                                                                                                                   \
    char nm[96];                                                                                                      \
    snprintf(nm, sizeof nm, "%s, grid %d", NAME, (int)(GRID));                                                        \
    timeit(nm, img_p, [&] {                                                                                           \
      hipLaunchKernelGGL((sellp_kernel<UNR, MODE, SrcPlain<double>, EpiApDot<double>>), dim3(GRID), dim3(256), 0, st, \
                         (const int64_t *)d_sptr, (const int *)d_width, (const int *)d_cbase,                         \
                         (const uint32_t *)d_delta, (const double *)d_val, P.nslices, n, SrcPlain<double>{x, 1},      \
                         EpiApDot<double>{y, nullptr, 1}, part);                                                      \
    });                                                                                                               \
    check(nm);                                                                                                        \
  }
    const int64_t one = (P.nslices + 3) / 4;
    if (one <= 65536) {
      PK(8, 6, one, "sellp UNR 8 paired, nt deltas, 1 slice/wave");
      PK(8, 14, one, "sellp UNR 8 paired, nt deltas, wave branch, 1 slice/wave");
      PK(8, 7, one, "sellp UNR 8 no pairing, nt deltas, 1 slice/wave");
      PK(16, 6, one, "sellp UNR 16 paired, nt deltas, 1 slice/wave");
      PK(16, 14, one, "sellp UNR 16 paired, nt deltas, wave branch, 1 slice/wave");
      PK(16, 7, one, "sellp UNR 16 no pairing, nt deltas, 1 slice/wave");
      PK(4, 14, one, "sellp UNR 4 paired, nt deltas, wave branch, 1 slice/wave");
      PK(12, 14, one, "sellp UNR 12 paired, nt deltas, wave branch, 1 slice/wave");
    }
  }
  KC(kry_vec_destroy(xv));
  KC(kry_vec_destroy(yv));
  KC(kry_csr_destroy(Adia));
  KC(kry_csr_destroy(Asell));
  KC(kry_csr_destroy(Apair));
  KC(kry_ctx_destroy(ctx));
  return 0;
}
