// Microbenchmark of the diagonal-offset (SELL-128/DIA, two rows per lane)
// SpMV on gfx950 (development tool, not product). Uploads the BASELINE metric
// matrix (3-D 15-point stencil m^3) through the library's C-ABI, then times
// the library's CG SpMV (Ap stored + <p, Ap> partials) next to probe
// variants on the same image: no store, no gathers, the value stream alone
// (also the read-side calibration of tools/pmc_traffic.sh: 8 B x dia_slots
// known bytes, 16 B per lane), other unrolls, interleaved slice order.
// Every full variant is checked bitwise against the library kernel.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     tools/dia_bench.hip -o tools/dia_bench -Lkrylov_amd -lkrylov_hip -Wl,-rpath,'$ORIGIN/../krylov_amd'
//   ./tools/dia_bench [m=216] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
  struct Nb {
    int64_t off;
    int di, dj, dk;
  };
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

typedef double d2v __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void read_ceiling(const d2v *__restrict__ b, int64_t nb, double *out) {
  double s = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride) {
    d2v v = __builtin_nontemporal_load(b + i);
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}

// MODE bits: 1 no store, 2 no gathers, 4 values only (no descriptors, no
// gathers, no store), 16 interleaved slice order, 32 plain (not nt) store
template <int UNR, int MODE>
__global__ __launch_bounds__(256) void dia_probe(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                 const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                 const double *__restrict__ val, int64_t nslices, int64_t n,
                                                 const double *__restrict__ x, double *__restrict__ y,
                                                 double *__restrict__ part) {
  __shared__ double red[256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  int64_t s_begin, s_end, s_step;
  if (MODE & 16) {
    s_begin = m;
    s_end = nslices;
    s_step = W;
  } else {
    s_begin = nslices * m / W;
    s_end = nslices * (m + 1) / W;
    s_step = 1;
  }
  double dacc = 0.0;
  for (int64_t s = s_begin; s < s_end; s += s_step) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * 128 + 2 * lane;
    const int64_t c0 = base / 128;
    const double *cv = val + base + 2 * lane;
    double acc0 = 0.0, acc1 = 0.0;
    if (MODE & 4) {
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (u < w) {
          double a[2];
          pload_nt<double>(cv + u * 128, a);
          acc0 += a[0];
          acc1 += a[1];
        }
    } else {
      for (int j0 = 0; j0 < w; j0 += UNR) {
        int off[UNR];
        uint64_t me[UNR], md[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          off[u] = doff[c0 + j0 + u];
          me[u] = dmask[2 * (c0 + j0 + u)];
          md[u] = dmask[2 * (c0 + j0 + u) + 1];
        }
        double a[UNR][2];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (j0 + u < w) pload_nt<double>(cv + (int64_t)(j0 + u) * 128, a[u]);
          else a[u][0] = a[u][1] = 0.0;
        }
        bool on0[UNR], on1[UNR];
        double xv[UNR][2];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          on0[u] = j0 + u < w && ((me[u] >> lane) & 1u) != 0;
          on1[u] = j0 + u < w && ((md[u] >> lane) & 1u) != 0;
          if (MODE & 2) xv[u][0] = xv[u][1] = 1.0;
          else pload<double>(x + ((on0[u] || on1[u]) ? row + off[u] : 0), xv[u]);
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const double p0 = a[u][0] * xv[u][0], p1 = a[u][1] * xv[u][1];
          const double t0 = acc0 + p0, t1 = acc1 + p1;
          acc0 = on0[u] ? t0 : acc0;
          acc1 = on1[u] ? t1 : acc1;
        }
      }
    }
    if (row + 1 < n) {
      const double sv[2] = {acc0, acc1};
      if (!(MODE & 1) && !(MODE & 4)) {
        if (MODE & 32) pstore<double>(y + row, sv);
        else pstore<double, true>(y + row, sv);
      }
      double xr[2];
      pload<double>(x + row, xr);
      dacc += (MODE & 4) ? acc0 + acc1 : xr[0] * acc0 + xr[1] * acc1;
    } else if (row < n) {
      if (!(MODE & 1) && !(MODE & 4)) y[row] = acc0;
      dacc += x[row] * acc0;
    }
  }
  red[tid] = dacc;
  block_tree_reduce(red, 256, 1);
  if (tid == 0) part[g] = red[0];
}

// Deferred store: slice s's result is stored after slice s + 1's loads have
// been issued (sched_barrier keeps the order), so a wait on those loads never
// waits for the store's acknowledgement. One round of UNR >= width.
template <int UNR>
__global__ __launch_bounds__(256) void dia_defer(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                 const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                 const double *__restrict__ val, int64_t nslices, int64_t n,
                                                 const double *__restrict__ x, double *__restrict__ y,
                                                 double *__restrict__ part) {
  __shared__ double red[256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  double dacc = 0.0;
  double pend[2] = {0.0, 0.0};
  int64_t prow = -1;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * 128 + 2 * lane;
    const int64_t c0 = base / 128;
    const double *cv = val + base + 2 * lane;
    int off[UNR];
    uint64_t me[UNR], md[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      off[u] = doff[c0 + u];
      me[u] = dmask[2 * (c0 + u)];
      md[u] = dmask[2 * (c0 + u) + 1];
    }
    double a[UNR][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (u < w) pload_nt<double>(cv + (int64_t)u * 128, a[u]);
      else a[u][0] = a[u][1] = 0.0;
    }
    bool on0[UNR], on1[UNR];
    double xv[UNR][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      on0[u] = u < w && ((me[u] >> lane) & 1u) != 0;
      on1[u] = u < w && ((md[u] >> lane) & 1u) != 0;
      pload<double>(x + ((on0[u] || on1[u]) ? row + off[u] : 0), xv[u]);
    }
    double xr[2];
    pload<double>(x + (row < n ? row : 0), xr);
    __builtin_amdgcn_sched_barrier(0);
    if (prow >= 0) {
      if (prow + 1 < n) pstore<double, true>(y + prow, pend);
      else if (prow < n) y[prow] = pend[0];
    }
    __builtin_amdgcn_sched_barrier(0);
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const double p0 = a[u][0] * xv[u][0], p1 = a[u][1] * xv[u][1];
      const double t0 = acc0 + p0, t1 = acc1 + p1;
      acc0 = on0[u] ? t0 : acc0;
      acc1 = on1[u] ? t1 : acc1;
    }
    if (row + 1 < n) dacc += xr[0] * acc0 + xr[1] * acc1;
    else if (row < n) dacc += xr[0] * acc0;
    pend[0] = acc0;
    pend[1] = acc1;
    prow = row;
  }
  if (prow >= 0) {
    if (prow + 1 < n) pstore<double, true>(y + prow, pend);
    else if (prow < n) y[prow] = pend[0];
  }
  red[tid] = dacc;
  block_tree_reduce(red, 256, 1);
  if (tid == 0) part[g] = red[0];
}

// x-run reuse: a slot column whose offset is 1 or 2 above an earlier loaded
// column's (the base) takes its x pair from the neighbouring lane's base pair
// (DPP wave_shl:1) instead of a load; lane 63 takes the element(s) past the
// base run from one extra 16-byte load. src[j] = 0: load; else (j - b) << 2 | d.
// Base runs are loaded for every lane (address clamped to [-1, n - 1]: a lane
// that consumes a shifted value has its source in range).
__device__ __forceinline__ double shl1(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int UNR>
__global__ __launch_bounds__(256) void dia_reuse(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                 const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                 const signed char *__restrict__ dsrc,
                                                 const double *__restrict__ val, int64_t nslices, int64_t n,
                                                 const double *__restrict__ x, double *__restrict__ y,
                                                 double *__restrict__ part) {
  __shared__ double red[256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  double dacc = 0.0;
  double pend[2] = {0.0, 0.0};
  int64_t prow = -1;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * 128 + 2 * lane;
    const int64_t c0 = base / 128;
    const double *cv = val + base + 2 * lane;
    int off[UNR], src[UNR];
    uint64_t me[UNR], md[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      off[u] = doff[c0 + u];
      me[u] = dmask[2 * (c0 + u)];
      md[u] = dmask[2 * (c0 + u) + 1];
      src[u] = dsrc[c0 + u];
    }
    double a[UNR][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (u < w) pload_nt<double>(cv + (int64_t)u * 128, a[u]);
      else a[u][0] = a[u][1] = 0.0;
    }
    bool on0[UNR], on1[UNR];
    double xv[UNR][2];
    double ex[UNR][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      on0[u] = u < w && ((me[u] >> lane) & 1u) != 0;
      on1[u] = u < w && ((md[u] >> lane) & 1u) != 0;
      if (u < w && src[u] == 0) {
        int64_t ix = row + off[u];
        ix = ix < -1 ? -1 : (ix > n - 1 ? n - 1 : ix);
        pload<double>(x + ix, xv[u]);
        int64_t ie = s * 128 + 128 + off[u];  // the pair past the run (lane 63's shifted source)
        ie = ie < -1 ? -1 : (ie > n - 1 ? n - 1 : ie);
        pload<double>(x + ie, ex[u]);
      } else {
        xv[u][0] = xv[u][1] = 0.0;
        ex[u][0] = ex[u][1] = 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (u < w && src[u] != 0) {
        const int b = u - (src[u] >> 2), d = src[u] & 3;
#pragma unroll
        for (int bb = 0; bb < UNR; ++bb)
          if (bb == b) {
            const double s0 = shl1(xv[bb][0]);
            if (d == 2) {
              const double s1 = shl1(xv[bb][1]);
              xv[u][0] = lane < 63 ? s0 : ex[bb][0];
              xv[u][1] = lane < 63 ? s1 : ex[bb][1];
            } else {
              xv[u][0] = xv[bb][1];
              xv[u][1] = lane < 63 ? s0 : ex[bb][0];
            }
          }
      }
    }
    double xr[2];
    pload<double>(x + (row < n ? row : 0), xr);
    __builtin_amdgcn_sched_barrier(0);
    if (prow >= 0) {
      if (prow + 1 < n) pstore<double, true>(y + prow, pend);
      else if (prow < n) y[prow] = pend[0];
    }
    __builtin_amdgcn_sched_barrier(0);
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const double p0 = a[u][0] * xv[u][0], p1 = a[u][1] * xv[u][1];
      const double t0 = acc0 + p0, t1 = acc1 + p1;
      acc0 = on0[u] ? t0 : acc0;
      acc1 = on1[u] ? t1 : acc1;
    }
    if (row + 1 < n) dacc += xr[0] * acc0 + xr[1] * acc1;
    else if (row < n) dacc += xr[0] * acc0;
    pend[0] = acc0;
    pend[1] = acc1;
    prow = row;
  }
  if (prow >= 0) {
    if (prow + 1 < n) pstore<double, true>(y + prow, pend);
    else if (prow < n) y[prow] = pend[0];
  }
  red[tid] = dacc;
  block_tree_reduce(red, 256, 1);
  if (tid == 0) part[g] = red[0];
}

// Persistent DIA SpMV (round 4 probe for a fused CG iteration at n = 10 M):
// one block of 512 threads per CU, laid out as cg_upd_kernel's granules, so
// granule u of wave wv of block b is slice b * 8 NV + 8 u + wv and the lane's
// two rows are its 16-B granule. Every slice's two row sums stay in
// registers (acc[NV][2], 160 VGPRs at NV = 40) until the end of the launch,
// where the fused kernel would exchange <p, Ap> and update r in place. MODE
// bits: 1 Ap not stored (what the fused kernel's SpMV phase would cost);
// otherwise stored at the end (bitwise check against the library kernel).
template <int NV, int UNR, int MODE>
__global__ __launch_bounds__(512) void dia_persist(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                   const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                   const double *__restrict__ val, int64_t nslices, int64_t n,
                                                   const double *__restrict__ x, double *__restrict__ y,
                                                   double *__restrict__ part) {
  __shared__ double red[512];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t sb = (int64_t)blockIdx.x * NV * 8;
  double acc[NV][2];
  double dacc = 0.0;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    acc[u][0] = acc[u][1] = 0.0;
    const int64_t s = sb + 8 * u + wv;
    if (s >= nslices) continue;
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * kDiaSlice + 2 * lane;
    const int64_t c0 = base / kDiaSlice;
    const int *mo = doff + c0;
    const uint64_t *mk = dmask + 2 * c0;
    const double *cv = val + base + 2 * lane;
    double a0 = 0.0, a1 = 0.0;
    for (int j0 = 0; j0 < w; j0 += UNR) {
      int off[UNR];
      uint64_t me[UNR], md[UNR];
#pragma unroll
      for (int q = 0; q < UNR; ++q) {
        off[q] = mo[j0 + q];
        me[q] = mk[2 * (j0 + q)];
        md[q] = mk[2 * (j0 + q) + 1];
      }
      d2v a[UNR], xv[UNR];
#pragma unroll
      for (int q = 0; q < UNR; ++q)
        a[q] = j0 + q < w ? __builtin_nontemporal_load(reinterpret_cast<const d2v *>(cv + (int64_t)(j0 + q) * kDiaSlice))
                          : d2v{0.0, 0.0};
      bool on0[UNR], on1[UNR];
#pragma unroll
      for (int q = 0; q < UNR; ++q) {
        on0[q] = j0 + q < w && ((me[q] >> lane) & 1u) != 0;
        on1[q] = j0 + q < w && ((md[q] >> lane) & 1u) != 0;
        xv[q] = *reinterpret_cast<const d2v *>(x + ((on0[q] || on1[q]) ? row + off[q] : 0));
      }
#pragma unroll
      for (int q = 0; q < UNR; ++q) {
        const double p0 = a[q].x * xv[q].x, p1 = a[q].y * xv[q].y;
        const double t0 = a0 + p0, t1 = a1 + p1;
        a0 = on0[q] ? t0 : a0;
        a1 = on1[q] ? t1 : a1;
      }
    }
    acc[u][0] = a0;
    acc[u][1] = a1;
  }
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int64_t s = sb + 8 * u + wv;
    if (s >= nslices) continue;
    const int64_t row = s * kDiaSlice + 2 * lane;
    const d2v p = *reinterpret_cast<const d2v *>(x + row);
    dacc += p.x * acc[u][0];
    if (row + 1 < n) dacc += p.y * acc[u][1];
    if (!(MODE & 1)) {
      if (row + 1 < n) __builtin_nontemporal_store(d2v{acc[u][0], acc[u][1]}, reinterpret_cast<d2v *>(y + row));
      else if (row < n) y[row] = acc[u][0];
    }
  }
  red[tid] = dacc;
  __syncthreads();
  for (int h = 256; h > 0; h >>= 1) {
    if (tid < h) red[tid] += red[tid + h];
    __syncthreads();
  }
  if (tid == 0) part[blockIdx.x] = red[0];
}

__global__ void dpp_direction(int *o) { o[threadIdx.x] = __builtin_amdgcn_update_dpp(-7, (int)threadIdx.x, 0x130, 0xf, 0xf, false); }

int main(int argc, char **argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 216;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<int> ip, ix;
  std::vector<double> dv;
  build_stencil(m, ip, ix, dv);
  const int64_t n = (int64_t)ip.size() - 1, nnz = ix.size();
  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  kry_csr *A;
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
  if (!A->dia) {
    fprintf(stderr, "no DIA image\n");
    return 1;
  }
  printf("m=%d n=%ld nnz=%ld dia_slices=%ld dia_slots=%ld max_width=%d\n", m, (long)n, (long)nnz,
         (long)A->dia_nslices, (long)A->dia_nslots, A->dia_max_width);
  std::vector<double> xh(n);
  for (int64_t i = 0; i < n; ++i) xh[i] = 1.0 + (double)((i * 7919) % 1000) * 1e-3;
  kry_vec *xv, *yv, *yrefv;  // library vectors: the allocation slack the kernel relies on
  KC(kry_vec_create(ctx, n, 1, KRY_F64, &xv));
  KC(kry_vec_create(ctx, n, 1, KRY_F64, &yv));
  KC(kry_vec_create(ctx, n, 1, KRY_F64, &yrefv));
  KC(kry_vec_upload(xv, xh.data()));
  double *x = (double *)xv->d, *y = (double *)yv->d, *yref = (double *)yrefv->d, *part, *dummy;
  CK(hipMalloc(&part, (size_t)65536 * 8));  // grids up to 65536 blocks (the sweep goes past kMaxGrid)
  CK(hipMalloc(&dummy, 64));
  hipStream_t st = ctx->stream;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double S = (double)nnz * 12 + (double)(n + 1) * 4 + 2.0 * n * 8;
  const double phys = (double)A->dia_nslots * 8 + (double)A->dia_nslots / 128 * 20 + 2.0 * n * 8;
  auto timeit = [&](const char *name, auto launch) {
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
    printf("%-44s %.4f ms  S-rate %.0f GB/s  image-rate %.0f GB/s\n", name, ms, S / ms / 1e6, phys / ms / 1e6);
    return ms;
  };
  // the library kernel (CG SpMV epilogue)
  timeit("library spmv_dia (EpiApDot)", [&] {
    int P;
    launch_spmv<double, double, int>(A, 1, SrcPlain<double>{x, 1}, EpiApDot<double>{yref, nullptr, 1}, part, &P,
                                     nullptr, 0, st);
  });
  std::vector<double> ref(n), got(n);
  CK(hipMemcpy(ref.data(), yref, n * 8, hipMemcpyDeviceToHost));
  // the library result against a host csr_matvec (sequential, no FMA)
  {
    int64_t bad = 0;
    for (int64_t r = 0; r < n; ++r) {
      double acc = 0.0;
      for (int e = ip[r]; e < ip[r + 1]; ++e) {
        volatile double p = dv[e] * xh[ix[e]];
        acc = acc + p;
      }
      bad += memcmp(&acc, &ref[r], 8) != 0;
    }
    printf("library vs host csr_matvec: %ld rows differ\n", (long)bad);
  }
  const int grid = (int)std::min<int64_t>(kMaxGrid, (A->dia_nslices + 3) / 4);
  auto check = [&](const char *name) {
    CK(hipMemcpy(got.data(), y, n * 8, hipMemcpyDeviceToHost));
    if (memcmp(got.data(), ref.data(), n * 8) != 0) printf("  !! %s differs from the library kernel\n", name);
  };
  const double vals_bytes = (double)A->dia_nslots * 8;
  {
    const int64_t nb = A->dia_nslots / 2;
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, st));
      hipLaunchKernelGGL(read_ceiling, dim3(4096), dim3(256), 0, st, (const d2v *)A->dia_val, nb, dummy);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ts.push_back(t);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-44s %.4f ms  %.0f GB/s\n", "read ceiling (value array, 16 B/lane)", ts[reps / 2],
           vals_bytes / ts[reps / 2] / 1e6);
  }
#define PROBE(U, MODE, NAME, CHECK)                                                                              \
  timeit(NAME, [&] {                                                                                            \
    hipLaunchKernelGGL((dia_probe<U, MODE>), dim3(grid), dim3(256), 0, st, (const int64_t *)A->dia_sptr,        \
                       (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,       \
                       (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);              \
  });                                                                                                           \
  if (CHECK) check(NAME);
  PROBE(16, 0, "probe: full (same as library)", true);
  PROBE(16, 1, "probe: no store", false);
  PROBE(16, 2, "probe: no gathers", false);
  PROBE(16, 3, "probe: no gathers, no store", false);
  PROBE(16, 4, "probe: values only", false);
  PROBE(8, 0, "probe: UNR 8", true);
  PROBE(16, 16, "probe: interleaved slices", true);
  PROBE(16, 32, "probe: plain (not nt) store", true);
  if (getenv("DIA_PERSIST")) {
    const int pg = (int)((A->dia_nslices + 319) / 320);
#define PERSIST(U, MODE, NAME, CHECK)                                                                            \
  timeit(NAME, [&] {                                                                                            \
    hipLaunchKernelGGL((dia_persist<40, U, MODE>), dim3(pg), dim3(512), 0, st, (const int64_t *)A->dia_sptr,    \
                       (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,       \
                       (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);              \
  });                                                                                                           \
  if (CHECK) check(NAME);
    PERSIST(4, 0, "persist NV40 UNR4: Ap stored", true);
    PERSIST(4, 1, "persist NV40 UNR4: Ap kept", false);
    PERSIST(8, 0, "persist NV40 UNR8: Ap stored", true);
    PERSIST(8, 1, "persist NV40 UNR8: Ap kept", false);
    PERSIST(5, 1, "persist NV40 UNR5: Ap kept", false);
    PERSIST(16, 1, "persist NV40 UNR16: Ap kept", false);
    timeit("library spmv_dia (EpiApDot), again", [&] {
      int P;
      launch_spmv<double, double, int>(A, 1, SrcPlain<double>{x, 1}, EpiApDot<double>{yref, nullptr, 1}, part, &P,
                                       nullptr, 0, st);
    });
    return 0;
  }
  const int full = (int)std::min<int64_t>(65536, (A->dia_nslices + 3) / 4);  // one slice per wave
  for (int gr : {grid, 4096, full}) {
    char nm[80];
    snprintf(nm, sizeof nm, "probe: deferred store, grid %d", gr);
    timeit(nm, [&] {
      hipLaunchKernelGGL(dia_defer<16>, dim3(gr), dim3(256), 0, st, (const int64_t *)A->dia_sptr,
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);
    });
    check(nm);
  }
  {
    int *od;
    CK(hipMalloc(&od, 64 * 4));
    hipLaunchKernelGGL(dpp_direction, dim3(1), dim3(64), 0, st, od);
    int oh[64];
    CK(hipMemcpy(oh, od, 256, hipMemcpyDeviceToHost));
    printf("dpp wave_shl:1 -> lane 0 gets %d, lane 62 gets %d, lane 63 gets %d\n", oh[0], oh[62], oh[63]);
    CK(hipFree(od));
    // x-run reuse codes from the image's offsets
    const int64_t cols = A->dia_nslots / 128;
    std::vector<int> offh(cols), wh(A->dia_nslices);
    std::vector<int64_t> sp(A->dia_nslices + 1);
    CK(hipMemcpy(offh.data(), A->dia_off, cols * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(wh.data(), A->dia_width, wh.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sp.data(), A->dia_sptr, sp.size() * 8, hipMemcpyDeviceToHost));
    std::vector<signed char> srch(cols + 64, 0);
    int64_t derived = 0;
    for (int64_t s = 0; s < A->dia_nslices; ++s) {
      const int64_t c0 = sp[s] / 128;
      int lastb = -1;
      for (int j = 0; j < wh[s]; ++j) {
        const int o = offh[c0 + j];
        if (lastb >= 0 && o - offh[c0 + lastb] >= 1 && o - offh[c0 + lastb] <= 2 && j - lastb < 32) {
          srch[c0 + j] = (signed char)(((j - lastb) << 2) | (o - offh[c0 + lastb]));
          ++derived;
        } else {
          lastb = j;
        }
      }
    }
    printf("x-run reuse: %ld of %ld slot columns derived\n", (long)derived, (long)cols);
    signed char *srcd;
    CK(hipMalloc(&srcd, srch.size()));
    CK(hipMemcpy(srcd, srch.data(), srch.size(), hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep) {
      timeit("probe: deferred store + x-run reuse", [&] {
        hipLaunchKernelGGL(dia_reuse<16>, dim3(grid), dim3(256), 0, st, (const int64_t *)A->dia_sptr,
                           (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,
                           (const signed char *)srcd, (const double *)A->dia_val, A->dia_nslices, n,
                           (const double *)x, y, part);
      });
      check("probe: deferred store + x-run reuse");
      timeit("probe: deferred store", [&] {
        hipLaunchKernelGGL(dia_defer<16>, dim3(grid), dim3(256), 0, st, (const int64_t *)A->dia_sptr,
                           (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,
                           (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);
      });
    }
    CK(hipFree(srcd));
  }
  KC(kry_vec_destroy(xv));
  KC(kry_vec_destroy(yv));
  KC(kry_vec_destroy(yrefv));
  KC(kry_csr_destroy(A));
  KC(kry_ctx_destroy(ctx));
  return 0;
}
