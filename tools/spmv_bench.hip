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
template <typename IX>
__global__ __launch_bounds__(256) void sell_stream_calib(const IX *__restrict__ idx, const double *__restrict__ val,
                                                         int64_t ns, double *out) {
  double s = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride) {
    const IX c = __builtin_nontemporal_load(idx + i);
    const double v = __builtin_nontemporal_load(val + i);
    s += c != IX(-1) ? v : 0.0;
  }
  if (s == 12345.678) out[0] = s;
}



// ---- prototype: compact SELL with the next slice's matrix stream issued
// right after the current slice's gathers (software pipelining); w <= UNR.
template <int UNR, int MINW>
__global__ __launch_bounds__(256, MINW) void spmv_pf(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                     const uint16_t *__restrict__ sdelta,
                                                     const int *__restrict__ scbase, const double *__restrict__ sval,
                                                     int64_t nslices, int64_t n, const double *__restrict__ x,
                                                     double *__restrict__ y) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  if (s_begin >= s_end) return;
  unsigned dA[UNR], dB[UNR];
  double aA[UNR], aB[UNR];
  int bA[UNR], bB[UNR];
  auto load = [&](int64_t s, unsigned(&d)[UNR], double(&a)[UNR], int(&b)[UNR]) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const bool in = u < w;
      d[u] = in ? (unsigned)__builtin_nontemporal_load(sdelta + base + (int64_t)u * 64 + lane) : 0xFFFFu;
      a[u] = in ? __builtin_nontemporal_load(sval + base + (int64_t)u * 64 + lane) : 0.0;
      b[u] = in ? scbase[(base >> 6) + u] : 0;
    }
  };
  load(s_begin, dA, aA, bA);
  for (int64_t s = s_begin; s < s_end; ++s) {
    double xv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) xv[u] = dA[u] != 0xFFFFu ? x[bA[u] + (int)dA[u]] : 0.0;
    if (s + 1 < s_end) load(s + 1, dB, aB, bB);
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (dA[u] != 0xFFFFu) {
        const double p = aA[u] * xv[u];
        acc = acc + p;
      }
    const int64_t row = s * 64 + lane;
    if (row < n) y[row] = acc;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      dA[u] = dB[u];
      aA[u] = aB[u];
      bA[u] = bB[u];
    }
  }
}


// ---- prototype: packed compact SELL. Lane l loads 4 slots' uint16 deltas as
// one 8-B access and 2 slots' values as one 16-B access (slot pairs, odd tail
// slot alone), so a slot costs 1/4 + 1/2 + 1 (gather) vector memory
// instructions instead of 3. Same per-row order: bitwise.
template <int UNR>
__global__ __launch_bounds__(256) void spmv_packed(const int64_t *__restrict__ sptr, const int64_t *__restrict__ dptr,
                                                   const int *__restrict__ swidth, const uint16_t *__restrict__ dpk,
                                                   const int *__restrict__ scbase, const double *__restrict__ vpk,
                                                   int64_t nslices, int64_t n, const double *__restrict__ x,
                                                   double *__restrict__ y) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s], doff = dptr[s];
    unsigned d[UNR];
    double a[UNR];
    int b[UNR];
#pragma unroll
    for (int q = 0; q < UNR / 4; ++q) {
      if (4 * q < w) {
        typedef unsigned short us4 __attribute__((ext_vector_type(4)));
        const us4 v = __builtin_nontemporal_load(reinterpret_cast<const us4 *>(dpk + doff + (int64_t)q * 256 + lane * 4));
        d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
      } else {
        d[4 * q] = d[4 * q + 1] = d[4 * q + 2] = d[4 * q + 3] = 0xFFFFu;
      }
    }
#pragma unroll
    for (int p = 0; p < UNR / 2; ++p) {
      if (2 * p + 1 < w) {
        typedef double d2 __attribute__((ext_vector_type(2)));
        const d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(vpk + base + (int64_t)p * 128 + lane * 2));
        a[2 * p] = v.x;
        a[2 * p + 1] = v.y;
      } else if (2 * p < w) {
        a[2 * p] = __builtin_nontemporal_load(vpk + base + (int64_t)p * 128 + lane);
        a[2 * p + 1] = 0.0;
      } else {
        a[2 * p] = a[2 * p + 1] = 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) b[u] = u < w ? scbase[(base >> 6) + u] : 0;
    double xv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) xv[u] = (u < w && d[u] != 0xFFFFu) ? x[b[u] + (int)d[u]] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (u < w && d[u] != 0xFFFFu) {
        const double pr = a[u] * xv[u];
        acc = acc + pr;
      }
    const int64_t row = s * 64 + lane;
    if (row < n) y[row] = acc;
  }
}

// ---- probe: the d16 SpMV with the gathers replaced by x[base_j + lane]
// (contiguous, independent of the per-lane delta load). Wrong result by
// design; isolates what the data-dependent gather costs.
template <int UNR, int MODE>
__global__ __launch_bounds__(256) void spmv_probe(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                  const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase,
                                                  const double *__restrict__ sval, int64_t nslices, int64_t n,
                                                  const double *__restrict__ x, double *__restrict__ y) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  double pend = 0.0;
  int64_t prow = -1;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    unsigned d[UNR];
    double a[UNR];
    int b[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const bool in = u < w;
      d[u] = in ? (unsigned)__builtin_nontemporal_load(sdelta + base + (int64_t)u * 64 + lane) : 0xFFFFu;
      a[u] = in ? __builtin_nontemporal_load(sval + base + (int64_t)u * 64 + lane) : 0.0;
      b[u] = in ? scbase[(base >> 6) + u] : 0;
    }
    if (MODE == 6 || MODE == 7) {
      // the previous slice's y store issued behind this slice's loads: with
      // in-order vmcnt its ack no longer gates this slice's first use
      asm volatile("" ::: "memory");
      if (prow >= 0 && prow < n) y[prow] = pend;
    }
    double xv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      // 1: no gather, y stored; 3: no gather, no y store; 4: no gather,
      // nontemporal y store; 5: no gather, y stored to a small target;
      // 6: no gather, y store deferred behind the next slice's loads;
      // 7: with the x gather, y store deferred; 8: with the gather, y stored
      if (MODE >= 7)
        xv[u] = (u < w && d[u] != 0xFFFFu) ? x[b[u] + (int)d[u]] : 0.0;
      else
        xv[u] = 1.0;
    }
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (d[u] != 0xFFFFu) {
        const double pr = a[u] * xv[u];
        acc = acc + pr;
      }
    const int64_t row = s * 64 + lane;
    if (MODE == 3) {
      if (row < n && acc == 12345.678) y[row] = acc;
    } else if (MODE == 4) {
      if (row < n) __builtin_nontemporal_store(acc, y + row);
    } else if (MODE == 5) {
      // same store count into a small L2-resident target (bounded by n)
      const int64_t idx = ((int64_t)blockIdx.x * 4 + wid) * 64 + lane;
      if (row < n && idx < n) y[idx] = acc;
    } else if (MODE == 6 || MODE == 7) {
      pend = acc;
      prow = row;
    } else if (MODE == 9) {  // gather; y store with cache-policy bits
      if (row < n) asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(y + row), "v"(acc) : "memory");
    } else if (MODE == 10) {
      if (row < n) asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(y + row), "v"(acc) : "memory");
    } else if (MODE == 11) {
      if (row < n) asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1 nt" ::"v"(y + row), "v"(acc) : "memory");
    } else if (row < n) {
      y[row] = acc;
    }
  }
  if ((MODE == 6 || MODE == 7) && prow >= 0 && prow < n) y[prow] = pend;
}

// ---- prototype: the d16 SpMV with XCD-interleaved slice order. XCD x owns a
// contiguous 1/8 of the slices (x gathers stay in its L2); inside it the
// waves take slices round-robin (wave j: start + j, start + j + Wx, ...), so
// the waves resident at one time stream one compact region of the matrix
// instead of one region each.
template <int UNR>
__global__ __launch_bounds__(256) void spmv_ilv(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase,
                                                const double *__restrict__ sval, int64_t nslices, int64_t n,
                                                const double *__restrict__ x, double *__restrict__ y) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
  const int nbx = (gridDim.x - xcd + 7) / 8;  // blocks on this XCD group
  const int64_t s0 = nslices * xcd / 8, s1 = nslices * (xcd + 1) / 8;
  const int64_t Wx = (int64_t)nbx * 4;
  for (int64_t s = s0 + (int64_t)idx * 4 + wid; s < s1; s += Wx) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    unsigned d[UNR];
    double a[UNR];
    int b[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const bool in = u < w;
      d[u] = in ? (unsigned)__builtin_nontemporal_load(sdelta + base + (int64_t)u * 64 + lane) : 0xFFFFu;
      a[u] = in ? __builtin_nontemporal_load(sval + base + (int64_t)u * 64 + lane) : 0.0;
      b[u] = in ? scbase[(base >> 6) + u] : 0;
    }
    double xv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) xv[u] = (u < w && d[u] != 0xFFFFu) ? x[b[u] + (int)d[u]] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (u < w && d[u] != 0xFFFFu) {
        const double pr = a[u] * xv[u];
        acc = acc + pr;
      }
    const int64_t row = s * 64 + lane;
    if (row < n) y[row] = acc;
  }
}

// ---- probe: the d16 SpMV with every y store deferred to the end of the
// wave's slice range (staged in LDS; MODE 0 per-slice 8-B stores at the end,
// MODE 1 the whole range as 16-B vector stores).
template <int UNR, int MODE>
__global__ __launch_bounds__(256) void spmv_defer(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                  const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase,
                                                  const double *__restrict__ sval, int64_t nslices, int64_t n,
                                                  const double *__restrict__ x, double *__restrict__ y) {
  __shared__ double ys[4][8 * 64];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  int t = 0;
  for (int64_t s = s_begin; s < s_end; ++s, ++t) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    unsigned d[UNR];
    double a[UNR];
    int b[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const bool in = u < w;
      d[u] = in ? (unsigned)__builtin_nontemporal_load(sdelta + base + (int64_t)u * 64 + lane) : 0xFFFFu;
      a[u] = in ? __builtin_nontemporal_load(sval + base + (int64_t)u * 64 + lane) : 0.0;
      b[u] = in ? scbase[(base >> 6) + u] : 0;
    }
    double xv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) xv[u] = (u < w && d[u] != 0xFFFFu) ? x[b[u] + (int)d[u]] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (u < w && d[u] != 0xFFFFu) {
        const double pr = a[u] * xv[u];
        acc = acc + pr;
      }
    ys[wid][t * 64 + lane] = acc;
  }
  const int64_t r0 = s_begin * 64, r1 = s_end * 64 < n ? s_end * 64 : n;
  if (MODE == 0) {
    for (int64_t r = r0 + lane; r < r1; r += 64) y[r] = ys[wid][r - r0];
  } else {
    typedef double d2 __attribute__((ext_vector_type(2)));
    for (int64_t r = r0 + 2 * lane; r < r1; r += 128) {
      if (r + 1 < r1) *reinterpret_cast<d2 *>(y + r) = d2{ys[wid][r - r0], ys[wid][r - r0 + 1]};
      else y[r] = ys[wid][r - r0];
    }
  }
}
__global__ __launch_bounds__(256) void pupdate_kernel(const double *__restrict__ r, const double *__restrict__ pold,
                                                      const double *__restrict__ om, double *__restrict__ p,
                                                      int64_t n) {
  const double o = om[0];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; 2 * i < n; i += stride) {
    if (2 * i + 1 < n) {
      const double2 rr = reinterpret_cast<const double2 *>(r)[i];
      const double2 pp = reinterpret_cast<const double2 *>(pold)[i];
      const double t0 = o * pp.x, t1 = o * pp.y;
      reinterpret_cast<double2 *>(p)[i] = make_double2(rr.x + t0, rr.y + t1);
    } else {
      const double t0 = o * pold[2 * i];
      p[2 * i] = r[2 * i] + t0;
    }
  }
}


// Random gather study (cfg3 shape): n rows, 19 uniform random off-diagonal
// columns in [0, span) plus the diagonal, sorted per row. span = n is the
// cfg3 pattern (x = 16 MB, not L2-resident); a small span keeps x in L2.
static int random_study(int64_t n, int reps) {
  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  double *d_x, *d_y;
  CK(hipMalloc(&d_x, n * 8));
  CK(hipMalloc(&d_y, n * 8));
  std::vector<double> xh(n, 1.0);
  CK(hipMemcpy(d_x, xh.data(), n * 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int64_t span : {n, n / 2, n / 4, n / 8, n / 16, n / 64}) {
    std::vector<int> ip(n + 1, 0), ix;
    std::vector<double> dv;
    ix.reserve(n * 20);
    dv.reserve(n * 20);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    std::vector<int> row;
    for (int64_t r = 0; r < n; ++r) {
      row.clear();
      row.push_back((int)r);
      for (int j = 0; j < 19; ++j) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        row.push_back((int)(st % (uint64_t)span));
      }
      std::sort(row.begin(), row.end());
      for (int c : row) { ix.push_back(c); dv.push_back(0.5); }
      ip[r + 1] = (int)ix.size();
    }
    const int64_t nnz = ix.size();
    const double S = nnz * 12.0 + (n + 1) * 4.0 + 2.0 * n * 8.0;
    for (int cbmode : {1, 0}) {
    if (!cbmode) setenv("KRY_SPMV_CB", "0", 1);
    kry_csr *A;
    KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
    unsetenv("KRY_SPMV_CB");
    auto launch = [&] {
      launch_spmv<double, double, int>(A, 1, SrcPlain<double>{d_x, 1}, EpiStore<double>{d_y, 1}, nullptr, nullptr,
                                       nullptr, 0, 0);
    };
    launch();
    CK(hipDeviceSynchronize());
    float tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
    }
    printf("random n=%ld span=%ld (x window %.1f MB) compact=%d col_blocks=%ld: %.4f ms  %.0f GB/s (S)\n", n, span,
           span * 8 / 1e6, (int)A->compact, A->cb_nb, tot / reps, S / (tot / reps) / 1e6);
    KC(kry_csr_destroy(A));
    if (span != n) break;
    }
  }
  KC(kry_ctx_destroy(ctx));
  return 0;
}

// Variant kept for the record (measured 0.358 ms vs spmv_cbp_kernel 0.264 ms
// on cfg3, grid 1024): software-pipelined spmv_cbp_kernel (same ownership,
// same per-row order, bitwise the same result). The block's work is one sequence of
// chunks (column block b, owned group o, entry offset c0); the segment table
// of that sequence is staged in LDS once. Per chunk: gather x for the
// chunk's columns, THEN issue the column/value/row-offset loads of the next
// chunk (so a wait for the gathers never waits for the prefetch: vmcnt is in
// order), stage the products in one of two LDS buffers, one barrier, and
// every thread adds its row's products to its running sum. The HBM stream of
// chunk i+1 is in flight while chunk i is gathered, staged and summed.
constexpr int kCbMaxSteps = 512;  // nb * owned groups per block
template <typename V, typename MV, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_cbq_kernel(int nb, int64_t n, int64_t ng,
                                                          const int64_t *__restrict__ gptr,
                                                          const uint16_t *__restrict__ roff,
                                                          const int *__restrict__ col, const MV *__restrict__ val,
                                                          Src src, Epi epi, double *__restrict__ part,
                                                          const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  constexpr int U = kCbCap / kBlock;
  __shared__ V prod[2][kCbCap];
  __shared__ double red[kBlock];
  __shared__ int64_t seg_s0[kCbMaxSteps];
  __shared__ int seg_len[kCbMaxSteps];
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  const int own = (int)((ng - blockIdx.x + G - 1) / G);  // groups blk, blk + G, ... (host: own <= kCbMaxOwn)
  const int T = nb * own;                                 // steps (b, o), b major (host: T <= kCbMaxSteps)
  for (int t = tid; t < T; t += kBlock) {
    const int b = t / own, o = t - (t / own) * own;
    const int64_t q = (int64_t)b * ng + blockIdx.x + (int64_t)o * G;
    const int64_t s0 = gptr[q];
    seg_s0[t] = s0;
    seg_len[t] = (int)(gptr[q + 1] - s0);
  }
  __syncthreads();
  const auto bs = src.template bind<1>(0);
  V acc[kCbMaxOwn];
#pragma unroll
  for (int o = 0; o < kCbMaxOwn; ++o) acc[o] = V(0);

  struct Chunk {
    int j[U];
    MV a[U];
    int r0, r1;
  };
  // loads of chunk (t, c0): its entries and this thread's row range in step t
  auto load = [&](int t, int c0, Chunk &c) {
    const int64_t s0 = seg_s0[t];
    const int len = seg_len[t];
    const int c1 = len < c0 + kCbCap ? len : c0 + kCbCap;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = c0 + tid + u * kBlock;
      c.j[u] = e < c1 ? __builtin_nontemporal_load(col + s0 + e) : -1;
      c.a[u] = e < c1 ? __builtin_nontemporal_load(val + s0 + e) : MV(0);
    }
    const int b = t / own, o = t - (t / own) * own;
    const int64_t row = ((int64_t)blockIdx.x + (int64_t)o * G) * kCbRows + tid;
    c.r0 = 0;
    c.r1 = 0;
    if (row < n) {
      c.r0 = roff[(int64_t)b * n + row];
      c.r1 = (tid == kCbRows - 1 || row + 1 >= n) ? len : (int)roff[(int64_t)b * n + row + 1];
    }
  };
  int t = 0, c0 = 0, par = 0;
  // one chunk: gathers of `cur`, prefetch of the next chunk into `nxt`,
  // products to LDS, barrier, row sums. Returns false after the last chunk.
  auto body = [&](Chunk &cur, Chunk &nxt) -> bool {
    int tn = t, cn = c0 + kCbCap;
    if (cn >= seg_len[t]) {
      tn = t + 1;
      cn = 0;
    }
    V xj[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xj[u] = cur.j[u] >= 0 ? bs(cur.j[u], 0) : V(0);
    if (tn < T) load(tn, cn, nxt);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (cur.j[u] >= 0) prod[par][tid + u * kBlock] = (V)cur.a[u] * xj[u];
    __syncthreads();
    const int len = seg_len[t];
    const int c1 = len < c0 + kCbCap ? len : c0 + kCbCap;
    const int lo = cur.r0 > c0 ? cur.r0 : c0, hi = cur.r1 < c1 ? cur.r1 : c1;
    const int o = t - (t / own) * own;
    V s = acc[0];
#pragma unroll
    for (int oo = 1; oo < kCbMaxOwn; ++oo)
      if (oo == o) s = acc[oo];
    for (int e = lo; e < hi; ++e) s = s + prod[par][e - c0];
#pragma unroll
    for (int oo = 0; oo < kCbMaxOwn; ++oo)
      if (oo == o) acc[oo] = s;
    t = tn;
    c0 = cn;
    par ^= 1;
    return t < T;
  };
  Chunk A, B;
  if (T > 0) {
    load(0, 0, A);
    while (body(A, B) && body(B, A)) {
    }
  }
  double dacc = 0.0;
#pragma unroll
  for (int o = 0; o < kCbMaxOwn; ++o) {
    if (o >= own) break;
    const int64_t row = ((int64_t)blockIdx.x + (int64_t)o * G) * kCbRows + tid;
    if (row < n) dacc += epi(row, 0, acc[o], bs(row, 0));
  }
  if (part != nullptr) {
    __syncthreads();
    red[tid] = dacc;
    block_tree_reduce(red, kBlock, 1);
    if (tid == 0) part[blockIdx.x] = red[0];
  }
}


// ---- calibration: random 8-B gathers from an L2-sized window. Each lane
// performs G gathers per round at hashed indices in [0, span); returns the
// chip-wide gather rate (gathers / s) — the ceiling a random-column SpMV's x
// gathers run against.
template <int G>
__global__ __launch_bounds__(256) void gather_calib(const double *__restrict__ x, int64_t span, int rounds,
                                                    double *out) {
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
  double s = 0.0;
  for (int r = 0; r < rounds; ++r) {
    double v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      h ^= h << 13; h ^= h >> 17; h ^= h << 5;
      v[g] = x[h % (uint32_t)span];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) s += v[g];
  }
  if (s == 12345.678) out[0] = s;
}

// ---- prototype: column-blocked SpMV with owner-contiguous segments. Block b
// owns rows [b * RB, (b + 1) * RB) (RB = 256 * RPT); for column block c its
// entries are one contiguous segment, processed in chunks of 256 * GPT
// entries (GPT gathers per thread in flight), products staged in LDS; thread
// t owns rows b * RB + t + 256 i (i < RPT) and adds each row's products to
// its running sum in stored order (bitwise csr_matvec).
template <int RPT, int GPT>
__global__ __launch_bounds__(256) void spmv_cbo(int nb, int64_t n, const int64_t *__restrict__ seg,
                                                const uint16_t *__restrict__ roff, const int *__restrict__ col,
                                                const double *__restrict__ val, const double *__restrict__ x,
                                                double *__restrict__ y) {
  constexpr int RB = 256 * RPT, CH = 256 * GPT;
  __shared__ double prod[CH];
  const int tid = threadIdx.x;
  const int64_t rbase = (int64_t)blockIdx.x * RB;
  double acc[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) acc[i] = 0.0;
  for (int c = 0; c < nb; ++c) {
    const int64_t s0 = seg[(int64_t)c * gridDim.x + blockIdx.x];
    const int len = (int)(seg[(int64_t)c * gridDim.x + blockIdx.x + 1] - s0);
    int r0[RPT], r1[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int lr = tid + 256 * i;  // local row
      const int64_t row = rbase + lr;
      r0[i] = r1[i] = 0;
      if (row < n) {
        r0[i] = roff[(int64_t)c * gridDim.x * (RB + 1) + (int64_t)blockIdx.x * (RB + 1) + lr];
        r1[i] = roff[(int64_t)c * gridDim.x * (RB + 1) + (int64_t)blockIdx.x * (RB + 1) + lr + 1];
      }
    }
    for (int c0 = 0; c0 < len; c0 += CH) {
      const int c1 = len < c0 + CH ? len : c0 + CH;
      int j[GPT];
      double a[GPT];
#pragma unroll
      for (int u = 0; u < GPT; ++u) {
        const int e = c0 + tid + u * 256;
        j[u] = e < c1 ? __builtin_nontemporal_load(col + s0 + e) : -1;
        a[u] = e < c1 ? __builtin_nontemporal_load(val + s0 + e) : 0.0;
      }
      double xj[GPT];
#pragma unroll
      for (int u = 0; u < GPT; ++u) xj[u] = j[u] >= 0 ? x[j[u]] : 0.0;
      __syncthreads();  // the previous chunk's products are consumed
#pragma unroll
      for (int u = 0; u < GPT; ++u)
        if (j[u] >= 0) prod[tid + u * 256] = a[u] * xj[u];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int lo = r0[i] > c0 ? r0[i] : c0, hi = r1[i] < c1 ? r1[i] : c1;
        for (int e = lo; e < hi; ++e) acc[i] = acc[i] + prod[e - c0];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int64_t row = rbase + tid + 256 * i;
    if (row < n) y[row] = acc[i];
  }
}

template <int RPT, int GPT>
static void cbo_study(int64_t n, const std::vector<int> &ip, const std::vector<int> &ix,
                      const std::vector<double> &dv, const std::vector<double> &yref, const double *d_x, double *d_y,
                      int reps, hipEvent_t a, hipEvent_t b, int64_t cols) {
  constexpr int RB = 256 * RPT;
  const int G = (int)((n + RB - 1) / RB);
  const int nb = (int)((n + cols - 1) / cols);
  // segments: (c, block) -> contiguous entries; roff per (c, block, local row)
  std::vector<int64_t> seg((size_t)nb * G + 1, 0);
  std::vector<uint16_t> roff((size_t)nb * G * (RB + 1), 0);
  std::vector<int64_t> cnt((size_t)nb * G, 0);
  for (int64_t r = 0; r < n; ++r)
    for (int e = ip[r]; e < ip[r + 1]; ++e) cnt[(size_t)(ix[e] / cols) * G + r / RB]++;
  for (size_t i = 0; i < cnt.size(); ++i) seg[i + 1] = seg[i] + cnt[i];
  std::vector<int> col(ip[n]);
  std::vector<double> val(ip[n]);
  std::vector<int64_t> pos(seg.begin(), seg.end() - 1);
  bool fits = true;
  for (int64_t r = 0; r < n; ++r) {
    const int blk = (int)(r / RB), lr = (int)(r % RB);
    for (int c = 0; c < nb; ++c) {
      const int64_t off = pos[(size_t)c * G + blk] - seg[(size_t)c * G + blk];
      if (off > 65535) fits = false;
      roff[((size_t)c * G + blk) * (RB + 1) + lr] = (uint16_t)off;
    }
    for (int e = ip[r]; e < ip[r + 1]; ++e) {
      const int c = ix[e] / cols;
      const int64_t p = pos[(size_t)c * G + blk]++;
      col[p] = ix[e];
      val[p] = dv[e];
    }
  }
  for (int blk = 0; blk < G; ++blk)
    for (int c = 0; c < nb; ++c) {
      const int64_t rows = std::min<int64_t>(RB, n - (int64_t)blk * RB);
      for (int64_t lr = rows; lr <= RB; ++lr)
        roff[((size_t)c * G + blk) * (RB + 1) + lr] = (uint16_t)(seg[(size_t)c * G + blk + 1] - seg[(size_t)c * G + blk]);
    }
  if (!fits) { printf("cbo RPT=%d: segment too long\n", RPT); return; }
  int64_t *d_seg; uint16_t *d_roff; int *d_col; double *d_val;
  CK(hipMalloc(&d_seg, seg.size() * 8));
  CK(hipMalloc(&d_roff, roff.size() * 2));
  CK(hipMalloc(&d_col, col.size() * 4 + 4096));
  CK(hipMalloc(&d_val, val.size() * 8 + 8192));
  CK(hipMemcpy(d_seg, seg.data(), seg.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_roff, roff.data(), roff.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_col, col.data(), col.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_val, val.data(), val.size() * 8, hipMemcpyHostToDevice));
  auto launch = [&] {
    hipLaunchKernelGGL((spmv_cbo<RPT, GPT>), dim3(G), dim3(256), 0, 0, nb, n, (const int64_t *)d_seg,
                       (const uint16_t *)d_roff, (const int *)d_col, (const double *)d_val, d_x, d_y);
  };
  CK(hipMemset(d_y, 0, n * 8));
  launch();
  CK(hipDeviceSynchronize());
  float tot = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  std::vector<double> h(n);
  CK(hipMemcpy(h.data(), d_y, n * 8, hipMemcpyDeviceToHost));
  int64_t bad = 0;
  for (int64_t i = 0; i < n; ++i) bad += memcmp(&h[i], &yref[i], 8) != 0;
  printf("cbo cols=%ld RPT=%d GPT=%d grid=%d nb=%d: %.4f ms  bitwise mismatches %ld\n", cols, RPT, GPT, G, nb,
         tot / reps, bad);
  CK(hipFree(d_seg)); CK(hipFree(d_roff)); CK(hipFree(d_col)); CK(hipFree(d_val));
}
// probe epilogue: no store, the value only feeds a dot partial
struct EpiNoStore {
  __device__ __forceinline__ double operator()(int64_t i, int c, double s, double xi) const { return s * s; }
};

// Column-blocked image tuning on the cfg3 pattern: block width x launch grid.
static int cb_tune(int64_t n, int reps) {
  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  double *d_x, *d_y;
  CK(hipMalloc(&d_x, n * 8));
  CK(hipMalloc(&d_y, n * 8));
  std::vector<double> xh(n);
  for (int64_t i = 0; i < n; ++i) xh[i] = 1.0 + 1e-3 * (double)((i * 2654435761u) % 1000);
  CK(hipMemcpy(d_x, xh.data(), n * 8, hipMemcpyHostToDevice));
  std::vector<int> ip(n + 1, 0), ix;
  std::vector<double> dv;
  uint64_t st = 0x9E3779B97F4A7C15ull;
  std::vector<int> row;
  for (int64_t r = 0; r < n; ++r) {
    row.clear();
    row.push_back((int)r);
    for (int j = 0; j < 19; ++j) {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      row.push_back((int)(st % (uint64_t)n));
    }
    std::sort(row.begin(), row.end());
    for (int c : row) { ix.push_back(c); dv.push_back(0.25 + 1e-3 * (double)(c % 997)); }
    ip[r + 1] = (int)ix.size();
  }
  const int64_t nnz = ix.size();
  const double S = nnz * 12.0 + (n + 1) * 4.0 + 2.0 * n * 8.0;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<double> yref(n);
  for (int64_t r = 0; r < n; ++r) {
    double sum = 0;
    for (int e = ip[r]; e < ip[r + 1]; ++e) {
      const double pr = dv[e] * xh[ix[e]];
      sum = sum + pr;
    }
    yref[r] = sum;
  }
  auto verify = [&](const char *what) {
    std::vector<double> h(n);
    CK(hipMemcpy(h.data(), d_y, n * 8, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += memcmp(&h[i], &yref[i], 8) != 0;
    printf("  %s: bitwise mismatches %ld\n", what, bad);
  };
  {
    // epilogue cost on the single-launch kernel (default image): y store,
    // y + V store + dot (the GMRES form), and no store at all
    kry_csr *A;
    KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
    double *d_v, *d_part, *d_hs;
    CK(hipMalloc(&d_v, n * 8));
    CK(hipMalloc(&d_part, kMaxGrid * 8));
    CK(hipMalloc(&d_hs, 64));
    const double one = 1.0;
    CK(hipMemcpy(d_hs, &one, 8, hipMemcpyHostToDevice));
    const int grid = (int)std::min<int64_t>(A->cb_ng, kCbPersistGrid);
    auto timeit = [&](const char *name, auto &&launch) {
      launch();
      CK(hipDeviceSynchronize());
      float tot = 0;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        tot += ms;
      }
      printf("cb epilogue %-40s %.4f ms\n", name, tot / reps);
    };
    auto cbp = [&](auto src, auto epi, double *part) {
      hipLaunchKernelGGL((spmv_cbp_kernel<true, double, double, decltype(src), decltype(epi)>), dim3(grid), dim3(kBlock),
                         0, 0, (int)A->cb_nb, A->n, A->cb_ng, (int64_t)0, A->cb_ng, (const int64_t *)A->cb_gptr, (const uint16_t *)A->cb_roff,
                         (const int *)A->cb_col, (const double *)A->cb_val, src, epi, part, (const Ctrl *)nullptr, 0);
    };
    timeit("store y", [&] { cbp(SrcPlain<double>{d_x, 1}, EpiStore<double>{d_y, 1}, nullptr); });
    timeit("store y + V, <q, y> (GMRES)", [&] {
      cbp(SrcScaled<double>{d_x, d_hs, 1}, EpiStoreDotV<double>{d_y, d_x, d_v, nullptr, 1}, d_part);
    });
    timeit("store y, <q, y>", [&] { cbp(SrcPlain<double>{d_x, 1}, EpiStoreDot<double>{d_y, d_x, nullptr, 1}, d_part); });
    timeit("no store, <y, y>", [&] { cbp(SrcPlain<double>{d_x, 1}, EpiNoStore{}, d_part); });
    KC(kry_csr_destroy(A));
    CK(hipFree(d_v));
    CK(hipFree(d_part));
    CK(hipFree(d_hs));
  }
  cbo_study<8, 8>(n, ip, ix, dv, yref, d_x, d_y, reps, a, b, 262144);
  cbo_study<8, 4>(n, ip, ix, dv, yref, d_x, d_y, reps, a, b, 262144);
  cbo_study<4, 8>(n, ip, ix, dv, yref, d_x, d_y, reps, a, b, 262144);
  cbo_study<8, 16>(n, ip, ix, dv, yref, d_x, d_y, reps, a, b, 262144);
  cbo_study<8, 8>(n, ip, ix, dv, yref, d_x, d_y, reps, a, b, 131072);
  {
    double *d_out;
    CK(hipMalloc(&d_out, 64));
    for (int64_t span : {(int64_t)4096, (int64_t)262144, (int64_t)2000000}) {
      for (int grid : {2048, 8192}) {
        const int rounds = 64;
        hipLaunchKernelGGL((gather_calib<8>), dim3(grid), dim3(256), 0, 0, d_x, span, rounds, d_out);
        CK(hipDeviceSynchronize());
        float tot = 0;
        for (int r = 0; r < reps; ++r) {
          CK(hipEventRecord(a, 0));
          hipLaunchKernelGGL((gather_calib<8>), dim3(grid), dim3(256), 0, 0, d_x, span, rounds, d_out);
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          tot += ms;
        }
        const double ng = (double)grid * 256 * rounds * 8;
        printf("gather calib span %ld doubles (%.1f MB) grid %d: %.4f ms, %.1f G gathers/s (40M gathers -> %.1f us)\n",
               span, span * 8 / 1e6, grid, tot / reps, ng / (tot / reps) / 1e6, 40e6 / (ng / (tot / reps) / 1e3) * 1e3);
      }
    }
    CK(hipFree(d_out));
  }
  for (const char *cols : {"131072", "262144", "524288"}) {
    setenv("KRY_CB_COLS", cols, 1);
    kry_csr *A;
    KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
    for (int grid : {1024, 1536, 2048}) {
      if (A->cb_ng > (int64_t)grid * kCbMaxOwn) continue;
      auto launch = [&] {
        hipLaunchKernelGGL((spmv_cbp_kernel<true, double, double, SrcPlain<double>, EpiStore<double>>), dim3(grid),
                           dim3(kBlock), 0, 0, (int)A->cb_nb, A->n, A->cb_ng, (int64_t)0, A->cb_ng,
                           (const int64_t *)A->cb_gptr,
                           (const uint16_t *)A->cb_roff, (const int *)A->cb_col, (const double *)A->cb_val,
                           SrcPlain<double>{d_x, 1}, EpiStore<double>{d_y, 1}, (double *)nullptr, (const Ctrl *)nullptr, 0);
      };
      launch();
      CK(hipDeviceSynchronize());
      float tot = 0;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        tot += ms;
      }
      printf("cb persistent cols=%s (nb=%ld) grid=%d: %.4f ms  %.0f GB/s (S)\n", cols, A->cb_nb, grid, tot / reps,
             S / (tot / reps) / 1e6);
      verify("persistent");
    }
    for (int grid : {1024, 1536, 2048}) {
      if (A->cb_ng > (int64_t)grid * kCbMaxOwn) continue;
      if (A->cb_nb * ((A->cb_ng + grid - 1) / grid) > kCbMaxSteps) continue;
      auto launch = [&] {
        hipLaunchKernelGGL((spmv_cbq_kernel<double, double, SrcPlain<double>, EpiStore<double>>), dim3(grid),
                           dim3(kBlock), 0, 0, (int)A->cb_nb, A->n, A->cb_ng, (const int64_t *)A->cb_gptr,
                           (const uint16_t *)A->cb_roff, (const int *)A->cb_col, (const double *)A->cb_val,
                           SrcPlain<double>{d_x, 1}, EpiStore<double>{d_y, 1}, (double *)nullptr, (const Ctrl *)nullptr, 0);
      };
      CK(hipMemset(d_y, 0, n * 8));
      launch();
      CK(hipDeviceSynchronize());
      float tot = 0;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        tot += ms;
      }
      printf("cb pipelined cols=%s (nb=%ld) grid=%d: %.4f ms  %.0f GB/s (S)\n", cols, A->cb_nb, grid, tot / reps,
             S / (tot / reps) / 1e6);
      verify("pipelined");
    }
    KC(kry_csr_destroy(A));
  }
  unsetenv("KRY_CB_COLS");
  KC(kry_ctx_destroy(ctx));
  return 0;
}

// Variant kept for the record (cfg4 k = 8: 0.749 ms at UNR 4 vs the
// lane-group kernel 0.795 ms; UNR 8 and k = 16 slower): lane-group SpMV with
// broadcast matrix entries (K in {4, 8, 16}). The
// lane-group kernel above re-loads every slot's index and value once per row
// pass (K passes of 64 / K rows), so a wave issues 2K narrow matrix loads per
// slot column. Here the 64 lanes load a slot column once (lane = row, one
// coalesced access as in the k = 1 kernel) and each pass takes its row's entry
// by a cross-lane shuffle; lane (row r, column c) keeps one accumulator per
// pass. The gathers are unchanged (K contiguous values of x per row), and
// every (row, column) is still summed over the slots in stored order from 0:
// bitwise the lane-group and csr_matvecs results.
template <typename V, typename MV, typename I, int K, int UNR, bool D16, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_sell_lgb_kernel(
    const int64_t *__restrict__ sptr, const int *__restrict__ swidth, const I *__restrict__ sidx,
    const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase, const MV *__restrict__ sval,
    int64_t nslices, int64_t n, int k, const I *__restrict__ indptr, const I *__restrict__ indices,
    const MV *__restrict__ data, Src src, Epi epi, double *__restrict__ part, const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  constexpr int RPP = 64 / K;  // rows per pass
  constexpr int NP = K;        // passes per slice
  __shared__ double red[kBlock];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane / K, c = lane & (K - 1);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  const auto bs = src.template bind<1>(c);
  double dacc = 0.0;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    V acc[NP];
#pragma unroll
    for (int t = 0; t < NP; ++t) acc[t] = V(0);
    if (w >= 0) {
      const I *ci = sidx + base + lane;
      const uint16_t *cd = sdelta + base + lane;
      const int *cb = scbase + (base >> 6);
      const MV *cv = sval + base + lane;
      for (int j0 = 0; j0 < w; j0 += UNR) {
        I col[UNR];
        V a[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const bool in = j0 + u < w;
          if constexpr (D16) {
            const unsigned d = in ? (unsigned)__builtin_nontemporal_load(cd + (int64_t)(j0 + u) * 64) : 0xFFFFu;
            const int b = in ? cb[j0 + u] : 0;
            col[u] = d != 0xFFFFu ? I(b + (int)d) : I(-1);
          } else {
            col[u] = in ? __builtin_nontemporal_load(ci + (int64_t)(j0 + u) * 64) : I(-1);
          }
          a[u] = in ? (V)__builtin_nontemporal_load(cv + (int64_t)(j0 + u) * 64) : V(0);
        }
#pragma unroll
        for (int t = 0; t < NP; ++t) {
          const int src_lane = t * RPP + rl0;
          I cx[UNR];
          V ax[UNR], xv[UNR];
#pragma unroll
          for (int u = 0; u < UNR; ++u) {
            cx[u] = __shfl(col[u], src_lane);
            ax[u] = __shfl(a[u], src_lane);
          }
#pragma unroll
          for (int u = 0; u < UNR; ++u) xv[u] = cx[u] >= 0 ? bs(cx[u], 0) : V(0);
#pragma unroll
          for (int u = 0; u < UNR; ++u)
            if (cx[u] >= 0) {
              const V p = ax[u] * xv[u];
              acc[t] = acc[t] + p;
            }
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < NP; ++t) {
        const int64_t row = s * 64 + t * RPP + rl0;
        if (row < n)
          for (I e = indptr[row]; e < indptr[row + 1]; ++e) {
            const V p = (V)data[e] * bs(indices[e], 0);
            acc[t] = acc[t] + p;
          }
      }
    }
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      const int64_t row = s * 64 + t * RPP + rl0;
      if (row < n) dacc += epi(row, c, acc[t], bs(row, 0));
    }
  }
  if (part != nullptr) {
    red[tid] = dacc;  // slot tid holds column tid % k
    block_tree_reduce(red, kBlock, k);
    if (tid < k) part[(int64_t)g * k + tid] = red[tid];
  }
}


// ---- prototype: one lane per row for a k = KB row-major block, the row's KB
// x values gathered as KB/2 16-B loads, KB accumulators per lane (matrix
// entries loaded once per slot, coalesced). Same per-(row, column) order.
template <int KB, int UNR>
__global__ __launch_bounds__(256) void spmv_rowblk(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                   const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase,
                                                   const double *__restrict__ sval, int64_t nslices, int64_t n,
                                                   const double *__restrict__ x, double *__restrict__ y) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  typedef double d2 __attribute__((ext_vector_type(2)));
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    double acc[KB];
#pragma unroll
    for (int c = 0; c < KB; ++c) acc[c] = 0.0;
    for (int j0 = 0; j0 < w; j0 += UNR) {
      int col[UNR];
      double a[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const bool in = j0 + u < w;
        const unsigned d = in ? (unsigned)__builtin_nontemporal_load(sdelta + base + (int64_t)(j0 + u) * 64 + lane) : 0xFFFFu;
        const int b = in ? scbase[(base >> 6) + j0 + u] : 0;
        col[u] = d != 0xFFFFu ? b + (int)d : -1;
        a[u] = in ? __builtin_nontemporal_load(sval + base + (int64_t)(j0 + u) * 64 + lane) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (col[u] >= 0) {
          const d2 *xr = reinterpret_cast<const d2 *>(x + (int64_t)col[u] * KB);
          d2 xv[KB / 2];
#pragma unroll
          for (int q = 0; q < KB / 2; ++q) xv[q] = xr[q];
#pragma unroll
          for (int q = 0; q < KB / 2; ++q) {
            const double p0 = a[u] * xv[q].x, p1 = a[u] * xv[q].y;
            acc[2 * q] = acc[2 * q] + p0;
            acc[2 * q + 1] = acc[2 * q + 1] + p1;
          }
        }
      }
    }
    const int64_t row = s * 64 + lane;
    if (row < n) {
      d2 *yr = reinterpret_cast<d2 *>(y + row * KB);
#pragma unroll
      for (int q = 0; q < KB / 2; ++q) yr[q] = d2{acc[2 * q], acc[2 * q + 1]};
    }
  }
}

// ---- prototype: LPR = KB / CPL lanes per row, CPL columns per lane
// (CPL * 8-B vector gathers and stores), 64 / LPR rows per pass, LPR passes.
template <int KB, int CPL, int UNR, bool NTS>
__global__ __launch_bounds__(256) void spmv_lgv(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase,
                                                const double *__restrict__ sval, int64_t nslices, int64_t n,
                                                const double *__restrict__ x, double *__restrict__ y) {
  constexpr int LPR = KB / CPL, RPP = 64 / LPR;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  const int rl0 = lane / LPR, cq = lane % LPR;
  typedef double dv __attribute__((ext_vector_type(2)));
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
#pragma unroll
    for (int t = 0; t < LPR; ++t) {
      const int rl = t * RPP + rl0;
      double acc[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[c] = 0.0;
      for (int j0 = 0; j0 < w; j0 += UNR) {
        int col[UNR];
        double a[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const bool in = j0 + u < w;
          const unsigned d = in ? (unsigned)__builtin_nontemporal_load(sdelta + base + (int64_t)(j0 + u) * 64 + rl) : 0xFFFFu;
          const int b = in ? scbase[(base >> 6) + j0 + u] : 0;
          col[u] = d != 0xFFFFu ? b + (int)d : -1;
          a[u] = in ? __builtin_nontemporal_load(sval + base + (int64_t)(j0 + u) * 64 + rl) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (col[u] >= 0) {
            const dv *xr = reinterpret_cast<const dv *>(x + (int64_t)col[u] * KB + cq * CPL);
            dv xv[CPL / 2];
#pragma unroll
            for (int q = 0; q < CPL / 2; ++q) xv[q] = xr[q];
#pragma unroll
            for (int q = 0; q < CPL / 2; ++q) {
              const double p0 = a[u] * xv[q].x, p1 = a[u] * xv[q].y;
              acc[2 * q] = acc[2 * q] + p0;
              acc[2 * q + 1] = acc[2 * q + 1] + p1;
            }
          }
        }
      }
      const int64_t row = s * 64 + rl;
      if (row < n) {
        dv *yr = reinterpret_cast<dv *>(y + row * KB + cq * CPL);
#pragma unroll
        for (int q = 0; q < CPL / 2; ++q) {
          if (NTS) __builtin_nontemporal_store(dv{acc[2 * q], acc[2 * q + 1]}, yr + q);
          else yr[q] = dv{acc[2 * q], acc[2 * q + 1]};
        }
      }
    }
  }
}
// cfg4 block SpMV (5-pt Poisson m^2, k = 8 row-major RHS): lane-group kernel
// vs the broadcast lane-group kernel, both checked bitwise against csr_matvecs.
static int block_study(int m, int k, int reps) {
  const int64_t n = (int64_t)m * m;
  std::vector<int> ip(n + 1, 0), ix;
  std::vector<double> dv;
  ix.reserve(n * 5);
  dv.reserve(n * 5);
  for (int64_t r = 0; r < n; ++r) {
    const int64_t i = r % m, j = r / m;
    if (j > 0) { ix.push_back((int)(r - m)); dv.push_back(-1.0); }
    if (i > 0) { ix.push_back((int)(r - 1)); dv.push_back(-1.0); }
    ix.push_back((int)r); dv.push_back(4.0);
    if (i + 1 < m) { ix.push_back((int)(r + 1)); dv.push_back(-1.0); }
    if (j + 1 < m) { ix.push_back((int)(r + m)); dv.push_back(-1.0); }
    ip[r + 1] = (int)ix.size();
  }
  const int64_t nnz = ix.size();
  const double S = nnz * 12.0 + (n + 1) * 4.0 + 2.0 * n * k * 8.0;
  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  kry_csr *A;
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
  printf("block study: poisson %d^2 n=%ld nnz=%ld k=%d compact=%d S=%.3f GB\n", m, n, nnz, k, (int)A->compact, S / 1e9);
  double *d_x, *d_y;
  CK(hipMalloc(&d_x, n * k * 8));
  CK(hipMalloc(&d_y, n * k * 8));
  std::vector<double> xh(n * k);
  for (int64_t i = 0; i < n * k; ++i) xh[i] = 1.0 + 1e-3 * (double)((i * 2654435761u) % 1000);
  CK(hipMemcpy(d_x, xh.data(), n * k * 8, hipMemcpyHostToDevice));
  std::vector<double> yref(n * k);
  for (int64_t r = 0; r < n; ++r)
    for (int c = 0; c < k; ++c) {
      double sum = 0;
      for (int e = ip[r]; e < ip[r + 1]; ++e) {
        const double p = dv[e] * xh[(int64_t)ix[e] * k + c];
        sum = sum + p;
      }
      yref[r * k + c] = sum;
    }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxGrid, (A->nslices + 3) / 4));
  auto run = [&](const char *name, auto kern) {
    CK(hipMemset(d_y, 0, n * k * 8));
    auto launch = [&] {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, 0, (const int64_t *)A->sptr, (const int *)A->swidth,
                         (const int *)A->sidx, (const uint16_t *)A->sdelta, (const int *)A->scbase,
                         (const double *)A->sval, A->nslices, A->n, k, (const int *)A->indptr,
                         (const int *)A->indices, (const double *)A->data, SrcPlain<double>{d_x, k},
                         EpiStore<double>{d_y, k}, (double *)nullptr, (const Ctrl *)nullptr, 0);
    };
    launch();
    CK(hipDeviceSynchronize());
    float tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
    }
    std::vector<double> h(n * k);
    CK(hipMemcpy(h.data(), d_y, n * k * 8, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < n * k; ++i) bad += memcmp(&h[i], &yref[i], 8) != 0;
    printf("  %s: %.4f ms  %.0f GB/s (S)  bitwise mismatches %ld\n", name, tot / reps, S / (tot / reps) / 1e6, bad);
  };
  if (k == 8) {
    run("lane-group", spmv_sell_lg_kernel<double, double, int, 4, 8, true, SrcPlain<double>, EpiStore<double>>);
    run("broadcast lane-group UNR8", spmv_sell_lgb_kernel<double, double, int, 8, 8, true, SrcPlain<double>, EpiStore<double>>);
    run("broadcast lane-group UNR4", spmv_sell_lgb_kernel<double, double, int, 8, 4, true, SrcPlain<double>, EpiStore<double>>);
    auto rowblk = [&](const char *name, auto kern, int gsz) {
      CK(hipMemset(d_y, 0, n * k * 8));
      auto launch = [&] {
        hipLaunchKernelGGL(kern, dim3(gsz), dim3(kBlock), 0, 0, (const int64_t *)A->sptr, (const int *)A->swidth,
                           (const uint16_t *)A->sdelta, (const int *)A->scbase, (const double *)A->sval, A->nslices,
                           A->n, (const double *)d_x, d_y);
      };
      launch();
      CK(hipDeviceSynchronize());
      float tot = 0;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        tot += ms;
      }
      std::vector<double> h(n * k);
      CK(hipMemcpy(h.data(), d_y, n * k * 8, hipMemcpyDeviceToHost));
      int64_t bad = 0;
      for (int64_t i = 0; i < n * k; ++i) bad += memcmp(&h[i], &yref[i], 8) != 0;
      printf("  %s grid %d: %.4f ms  %.0f GB/s (S)  bitwise mismatches %ld\n", name, gsz, tot / reps,
             S / (tot / reps) / 1e6, bad);
    };
    for (int gsz : {8192}) {
      rowblk("row-per-lane k=8 UNR4", spmv_rowblk<8, 4>, gsz);
      rowblk("lgv CPL2 UNR4", spmv_lgv<8, 2, 4, false>, gsz);
      rowblk("lgv CPL2 UNR8", spmv_lgv<8, 2, 8, false>, gsz);
      rowblk("lgv CPL4 UNR4", spmv_lgv<8, 4, 4, false>, gsz);
      rowblk("lgv CPL4 UNR8", spmv_lgv<8, 4, 8, false>, gsz);
      rowblk("lgv CPL8 UNR4", spmv_lgv<8, 8, 4, false>, gsz);
      rowblk("lgv CPL2 UNR4 nt-store", spmv_lgv<8, 2, 4, true>, gsz);
      rowblk("lgv CPL4 UNR4 nt-store", spmv_lgv<8, 4, 4, true>, gsz);
      rowblk("lgv CPL8 UNR4 nt-store", spmv_lgv<8, 8, 4, true>, gsz);
    }
  } else if (k == 4) {
    run("lane-group", spmv_sell_lg_kernel<double, double, int, 4, 8, true, SrcPlain<double>, EpiStore<double>>);
    run("broadcast lane-group UNR8", spmv_sell_lgb_kernel<double, double, int, 4, 8, true, SrcPlain<double>, EpiStore<double>>);
  } else if (k == 16) {
    run("lane-group", spmv_sell_lg_kernel<double, double, int, 4, 8, true, SrcPlain<double>, EpiStore<double>>);
    run("broadcast lane-group UNR8", spmv_sell_lgb_kernel<double, double, int, 16, 8, true, SrcPlain<double>, EpiStore<double>>);
  }
  KC(kry_csr_destroy(A));
  KC(kry_ctx_destroy(ctx));
  return 0;
}

// The library's CG SpMV (compact image, Ap stored + <p, Ap> partials) alone on
// the m^3 15-point stencil: `spmv_bench cgonly m reps`.
static int cg_only(int m, int reps) {
  std::vector<int> ip, ix;
  std::vector<double> dv;
  build_stencil(m, ip, ix, dv);
  const int64_t n = ip.size() - 1, nnz = ix.size();
  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  kry_csr *A;
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
  double *d_p, *d_ap, *part;
  CK(hipMalloc(&d_p, n * 8));
  CK(hipMalloc(&d_ap, n * 8));
  CK(hipMalloc(&part, kMaxGrid * 8));
  CK(hipMemset(d_p, 0, n * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto launch = [&] {
    launch_spmv<double, double, int>(A, 1, SrcPlain<double>{d_p, 1}, EpiApDot<double>{d_ap, nullptr, 1}, part, nullptr,
                                     nullptr, 0, 0);
  };
  launch();
  CK(hipDeviceSynchronize());
  float tot = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  printf("cgonly m=%d n=%ld nnz=%ld: CG SpMV %.4f ms\n", m, n, nnz, tot / reps);
  KC(kry_csr_destroy(A));
  KC(kry_ctx_destroy(ctx));
  return 0;
}


// Persistent-CG premise probe (`spmv_bench pstudy m reps`): the CG SpMV run
// as ONE resident block of 1024 threads per CU (the shape a persistent
// large-n CG would have), each wave over a contiguous slice range, with the
// result kept on chip (LDS) for the first LSL slices of each wave and
// stored to y for the rest. LSL = 0: all stored; LSL = 1 << 30: none stored
// (LDS slots reused round-robin).
template <int UNR, int LSL>
__global__ __launch_bounds__(1024) void spmv_1pc(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                 const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase,
                                                 const double *__restrict__ sval, int64_t nslices, int64_t n,
                                                 const double *__restrict__ x, double *__restrict__ y,
                                                 double *__restrict__ part) {
  __shared__ double keep[16 * 1024];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t W = (int64_t)gridDim.x * 16, wg = (int64_t)blockIdx.x * 16 + wid;
  const int64_t sb = nslices * wg / W, se = nslices * (wg + 1) / W;
  double dacc = 0.0;
  for (int64_t s = sb; s < se; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const uint16_t *cd = sdelta + base + lane;
    const int *cb = scbase + (base >> 6);
    const double *cv = sval + base + lane;
    double acc = 0.0;
    for (int j0 = 0; j0 < w; j0 += UNR) {
      int col[UNR];
      double a[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const bool in = j0 + u < w;
        const unsigned d = in ? (unsigned)__builtin_nontemporal_load(cd + (int64_t)(j0 + u) * 64) : 0xFFFFu;
        const int b = in ? cb[j0 + u] : 0;
        col[u] = d != 0xFFFFu ? b + (int)d : -1;
        a[u] = in ? __builtin_nontemporal_load(cv + (int64_t)(j0 + u) * 64) : 0.0;
      }
      double xv[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) xv[u] = col[u] >= 0 ? x[col[u]] : 0.0;
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (col[u] >= 0) acc = acc + a[u] * xv[u];
    }
    const int64_t row = s * 64 + lane;
    if (row < n) {
      dacc += acc * x[row];
      const int64_t j = s - sb;
      if (j < LSL)
        keep[wid * 1024 + (int)(j & 15) * 64 + lane] = acc;
      else
        __builtin_nontemporal_store(acc, y + row);
    }
  }
  for (int off = 32; off >= 1; off >>= 1) dacc += __shfl_xor(dacc, off);
  if (lane == 0) keep[wid] += dacc;  // keep the LDS writes live
  __syncthreads();
  if (tid == 0) {
    double t = 0;
    for (int i = 0; i < 16; ++i) t += keep[i];
    part[blockIdx.x] = t;
  }
}

static int persist_study(int m, int reps) {
  std::vector<int> ip, ix;
  std::vector<double> dv;
  build_stencil(m, ip, ix, dv);
  const int64_t n = ip.size() - 1, nnz = ix.size();
  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  kry_csr *A;
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
  if (!A->compact) {
    printf("not compact\n");
    return 1;
  }
  double *d_p, *d_ap, *part;
  CK(hipMalloc(&d_p, n * 8));
  CK(hipMalloc(&d_ap, n * 8));
  CK(hipMalloc(&part, kMaxGrid * 8));
  CK(hipMemset(d_p, 0, n * 8));
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time = [&](const char *name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
    }
    printf("%-44s %.4f ms\n", name, tot / reps);
  };
  time("library CG SpMV (EpiApDot)", [&] {
    launch_spmv<double, double, int>(A, 1, SrcPlain<double>{d_p, 1}, EpiApDot<double>{d_ap, nullptr, 1}, part,
                                     nullptr, nullptr, 0, 0);
  });
  auto one = [&](const char *name, auto kern) {
    time(name, [&] {
      hipLaunchKernelGGL(kern, dim3(ncu), dim3(1024), 0, 0, (const int64_t *)A->sptr, (const int *)A->swidth,
                         (const uint16_t *)A->sdelta, (const int *)A->scbase, (const double *)A->sval, A->nslices, n,
                         d_p, d_ap, part);
    });
  };
  one("1 block/CU, UNR8, all stored", spmv_1pc<8, 0>);
  one("1 block/CU, UNR8, first 16 slices/wave kept", spmv_1pc<8, 16>);
  one("1 block/CU, UNR8, first 32 slices/wave kept", spmv_1pc<8, 32>);
  one("1 block/CU, UNR8, none stored", spmv_1pc<8, (1 << 30)>);
  one("1 block/CU, UNR16, all stored", spmv_1pc<16, 0>);
  one("1 block/CU, UNR16, none stored", spmv_1pc<16, (1 << 30)>);
  KC(kry_csr_destroy(A));
  KC(kry_ctx_destroy(ctx));
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && strcmp(argv[1], "pstudy") == 0)
    return persist_study(argc > 2 ? atoi(argv[2]) : 216, argc > 3 ? atoi(argv[3]) : 20);
  if (argc > 1 && strcmp(argv[1], "cgonly") == 0)
    return cg_only(argc > 2 ? atoi(argv[2]) : 216, argc > 3 ? atoi(argv[3]) : 20);
  if (argc > 1 && strcmp(argv[1], "block") == 0)
    return block_study(argc > 2 ? atoi(argv[2]) : 3163, argc > 3 ? atoi(argv[3]) : 8, 10);
  if (argc > 1 && strcmp(argv[1], "random") == 0) return random_study(argc > 2 ? atol(argv[2]) : 2000000, 10);
  if (argc > 1 && strcmp(argv[1], "cbtune") == 0) return cb_tune(argc > 2 ? atol(argv[2]) : 2000000, 10);
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
  // A: the library's default image (compact uint16 deltas for this stencil);
  // A32: the same matrix with int32 indices (KRY_SELL_COMPACT=0)
  kry_csr *A, *A32;
  auto t0 = std::chrono::steady_clock::now();
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
  printf("upload + SELL-64 build %.2fs: %ld slices, %ld slots (%.2f%% padding), %ld irregular, compact %d\n",
         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), A->nslices, A->nslots,
         100.0 * (A->nslots - nnz) / nnz, A->nirregular, (int)A->compact);
  setenv("KRY_SELL_COMPACT", "0", 1);
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A32));
  unsetenv("KRY_SELL_COMPACT");
  if (!A->compact || A32->compact || !A32->sidx) {
    fprintf(stderr, "unexpected images (compact %d / %d)\n", (int)A->compact, (int)A32->compact);
    return 1;
  }

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

  CK(hipMemcpy(d_p, pref.data(), n * 8, hipMemcpyHostToDevice));
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

  if (getenv("SPMV_STORE_PROBE")) {  // the y-store cost only: library kernel vs probe modes
    report("SELL d16 y = A x (library)", S, [&] {
      launch_spmv<double, double, int>(A, 1, SrcPlain<double>{d_x, 1}, EpiStore<double>{d_y, 1}, nullptr, nullptr,
                                       nullptr, 0, 0);
    });
    check("SELL d16 y = A x (library)", d_y, yref);
    for (int mode : {8, 9, 10, 11, 7, 1, 6, 3}) {
      char nm[96];
      snprintf(nm, 96, "probe mode %d (%s)", mode, mode == 1 ? "no gather, store" : mode == 3 ? "no gather, no store" : mode == 6 ? "no gather, deferred store" : mode == 7 ? "gather, deferred store" : mode == 9 ? "gather, store sc0 sc1" : mode == 10 ? "gather, store sc1" : mode == 11 ? "gather, store sc0 sc1 nt" : "gather, store");
      CK(hipMemset(d_y, 0, n * 8));
      report(nm, S, [&] {
        auto go = [&](auto kern) {
          hipLaunchKernelGGL(kern, dim3(8192), dim3(256), 0, 0, (const int64_t *)A->sptr, (const int *)A->swidth,
                             (const uint16_t *)A->sdelta, (const int *)A->scbase, (const double *)A->sval, A->nslices,
                             n, d_x, d_y);
        };
        if (mode == 1) go(spmv_probe<16, 1>);
        else if (mode == 3) go(spmv_probe<16, 3>);
        else if (mode == 6) go(spmv_probe<16, 6>);
        else if (mode == 7) go(spmv_probe<16, 7>);
        else if (mode == 9) go(spmv_probe<16, 9>);
        else if (mode == 10) go(spmv_probe<16, 10>);
        else if (mode == 11) go(spmv_probe<16, 11>);
        else go(spmv_probe<16, 8>);
      });
      if (mode >= 7) check(nm, d_y, yref);
    }
    return 0;
  }
  report("read ceiling (SELL idx+val, 16 B/lane)", nnz * 12.0, [&] {
    hipLaunchKernelGGL(read_ceiling, dim3(2048), dim3(256), 0, 0, (const int4 *)A32->sidx, nnz / 4,
                       (const double2 *)A32->sval, nnz / 2, d_out);
  });
  report("SELL stream calibration (4+8 B/lane nt)", A32->nslots * 12.0, [&] {
    hipLaunchKernelGGL(sell_stream_calib<int>, dim3(8192), dim3(256), 0, 0, (const int *)A32->sidx,
                       (const double *)A32->sval, A32->nslots, d_out);
  });
  report("d16 stream calibration (2+8 B/lane nt)", A->nslots * 10.0, [&] {
    hipLaunchKernelGGL(sell_stream_calib<uint16_t>, dim3(8192), dim3(256), 0, 0, (const uint16_t *)A->sdelta,
                       (const double *)A->sval, A->nslots, d_out);
  });
  for (kry_csr *M : {A32, A}) {
    const char *tag = M->compact ? "d16" : "i32";
    char nm[96];
    snprintf(nm, 96, "SELL %s y = A x", tag);
    report(nm, S, [&] {
      launch_spmv<double, double, int>(M, 1, SrcPlain<double>{d_x, 1}, EpiStore<double>{d_y, 1}, nullptr, nullptr,
                                       nullptr, 0, 0);
    });
    check(nm, d_y, yref);
    snprintf(nm, 96, "SELL %s CG: Ap = A p, <p, Ap>", tag);
    report(nm, S, [&] {
      launch_spmv<double, double, int>(M, 1, SrcPlain<double>{d_p, 1}, EpiApDot<double>{d_ap, nullptr, 1}, part,
                                       nullptr, nullptr, 0, 0);
    });
    check(nm, d_ap, y2ref);
  }
#define PF(UNR, MINW, GRID)                                                                                  \
  {                                                                                                          \
    char nm[96];                                                                                             \
    snprintf(nm, 96, "proto pipelined d16 U%d minw=%d grid=%d", UNR, MINW, GRID);                            \
    report(nm, S, [&] {                                                                                      \
      hipLaunchKernelGGL((spmv_pf<UNR, MINW>), dim3(GRID), dim3(256), 0, 0, (const int64_t *)A->sptr,          \
                         (const int *)A->swidth, (const uint16_t *)A->sdelta, (const int *)A->scbase,           \
                         (const double *)A->sval, A->nslices, n, d_x, d_y);                                    \
    });                                                                                                      \
    check(nm, d_y, yref);                                                                                    \
  }
  PF(16, 1, 8192)
  PF(16, 1, 2048)
  PF(16, 1, 1024)
  PF(16, 2, 2048)
  {
    // the library kernel at other grid sizes (KRY_SPMV_GRID)
    for (int gsz : {1024, 2048, 4096}) {
      char nm[96];
      snprintf(nm, 96, "SELL d16 y = A x grid=%d", gsz);
      report(nm, S, [&] {
        hipLaunchKernelGGL((spmv_sell_kernel<double, double, int, 1, 16, true, SrcPlain<double>, EpiStore<double>>),
                           dim3(gsz), dim3(256), 0, 0, (const int64_t *)A->sptr, (const int *)A->swidth,
                           (const int *)nullptr, (const uint16_t *)A->sdelta, (const int *)A->scbase,
                           (const double *)A->sval, A->nslices, n, 1, (const int *)nullptr, (const int *)nullptr,
                           (const double *)nullptr, SrcPlain<double>{d_x, 1}, EpiStore<double>{d_y, 1},
                           (double *)nullptr, (const Ctrl *)nullptr, 0);
      });
      check(nm, d_y, yref);
    }
  }
  {
    // packed image from the library's compact image (host repack)
    const int64_t ns = A->nslices;
    std::vector<int64_t> sp(ns + 1);
    std::vector<int> sw(ns);
    CK(hipMemcpy(sp.data(), A->sptr, (ns + 1) * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sw.data(), A->swidth, ns * 4, hipMemcpyDeviceToHost));
    std::vector<uint16_t> dl(A->nslots);
    std::vector<double> vl(A->nslots);
    CK(hipMemcpy(dl.data(), A->sdelta, A->nslots * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(vl.data(), A->sval, A->nslots * 8, hipMemcpyDeviceToHost));
    std::vector<int64_t> dp(ns + 1, 0);
    int maxw = 0;
    for (int64_t s = 0; s < ns; ++s) {
      maxw = std::max(maxw, sw[s]);
      dp[s + 1] = dp[s] + 256 * ((std::max(sw[s], 0) + 3) / 4);
    }
    if (maxw <= 16) {
      std::vector<uint16_t> dpk(dp[ns] + 256, 0xFFFF);
      std::vector<double> vpk(A->nslots + 128, 0.0);
      for (int64_t s = 0; s < ns; ++s) {
        const int w = sw[s];
        const int64_t base = sp[s];
        for (int j = 0; j < w; ++j)
          for (int l = 0; l < 64; ++l) {
            dpk[dp[s] + (j / 4) * 256 + l * 4 + (j & 3)] = dl[base + 64 * j + l];
            const double v = vl[base + 64 * j + l];
            if (j < 2 * (w / 2)) vpk[base + (j / 2) * 128 + l * 2 + (j & 1)] = v;
            else vpk[base + (w / 2) * 128 + l] = v;
          }
      }
      int64_t *d_dp;
      uint16_t *d_dpk;
      double *d_vpk;
      CK(hipMalloc(&d_dp, (ns + 1) * 8));
      CK(hipMalloc(&d_dpk, dpk.size() * 2));
      CK(hipMalloc(&d_vpk, vpk.size() * 8));
      CK(hipMemcpy(d_dp, dp.data(), (ns + 1) * 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(d_dpk, dpk.data(), dpk.size() * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(d_vpk, vpk.data(), vpk.size() * 8, hipMemcpyHostToDevice));
      for (int gsz : {2048, 4096, 8192}) {
        char nm[96];
        snprintf(nm, 96, "proto packed d16 (8B deltas, 16B vals) grid=%d", gsz);
        report(nm, S, [&] {
          hipLaunchKernelGGL((spmv_packed<16>), dim3(gsz), dim3(256), 0, 0, (const int64_t *)A->sptr,
                             (const int64_t *)d_dp, (const int *)A->swidth, (const uint16_t *)d_dpk,
                             (const int *)A->scbase, (const double *)d_vpk, ns, n, d_x, d_y);
        });
        check(nm, d_y, yref);
      }
      CK(hipFree(d_dp));
      CK(hipFree(d_dpk));
      CK(hipFree(d_vpk));
    }
  }
  for (int gsz : {1024, 1280, 2048, 4096, 8192}) {
    char nm[96];
    snprintf(nm, 96, "proto XCD-interleaved d16 grid=%d", gsz);
    report(nm, S, [&] {
      hipLaunchKernelGGL((spmv_ilv<16>), dim3(gsz), dim3(256), 0, 0, (const int64_t *)A->sptr, (const int *)A->swidth,
                         (const uint16_t *)A->sdelta, (const int *)A->scbase, (const double *)A->sval, A->nslices, n,
                         d_x, d_y);
    });
    check(nm, d_y, yref);
  }
  for (int mode = 0; mode < 2; ++mode) {
    char nm[96];
    snprintf(nm, 96, "proto deferred y stores mode %d", mode);
    if ((A->nslices + 32767) / 32768 > 8) break;
    report(nm, S, [&] {
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(8192), dim3(256), 0, 0, (const int64_t *)A->sptr, (const int *)A->swidth,
                           (const uint16_t *)A->sdelta, (const int *)A->scbase, (const double *)A->sval, A->nslices, n,
                           d_x, d_y);
      };
      if (mode == 0) go(spmv_defer<16, 0>);
      else go(spmv_defer<16, 1>);
    });
    check(nm, d_y, yref);
  }
  for (int mode = 1; mode < 8; mode += (mode == 1 ? 2 : 1)) {
    char nm[96];
    snprintf(nm, 96, "probe mode %d (%s)", mode, mode == 1 ? "no gather" : mode == 3 ? "no gather, no store" : mode == 4 ? "no gather, nt store" : mode == 5 ? "no gather, store to 8 MB" : mode == 6 ? "no gather, deferred store" : "gather, deferred store");
    report(nm, S, [&] {
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(8192), dim3(256), 0, 0, (const int64_t *)A->sptr, (const int *)A->swidth,
                           (const uint16_t *)A->sdelta, (const int *)A->scbase, (const double *)A->sval, A->nslices, n,
                           d_x, d_y);
      };
      if (mode == 1) go(spmv_probe<16, 1>);
      else if (mode == 3) go(spmv_probe<16, 3>);
      else if (mode == 4) go(spmv_probe<16, 4>);
      else if (mode == 5) go(spmv_probe<16, 5>);
      else if (mode == 6) go(spmv_probe<16, 6>);
      else go(spmv_probe<16, 7>);
    });
  }
  report("CG p pass p = r + om p_old (3 vectors)", 24.0 * n, [&] {
    hipLaunchKernelGGL(pupdate_kernel, dim3(4096), dim3(256), 0, 0, d_x, d_x, d_om, d_y, n);
  });
  check("p pass", d_y, pref);
  KC(kry_csr_destroy(A32));
  KC(kry_csr_destroy(A));
  KC(kry_ctx_destroy(ctx));
  return 0;
}
