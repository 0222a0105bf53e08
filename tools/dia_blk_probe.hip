// The block right-hand-side DIA SpMV (k = 8, cfg4's 5-point Poisson N^2) on
// gfx950: development probe, not product. Round 5 folds the round 2-4
// variant benches (split slices, shifted windows, LDS windows, column-major
// vectors, grid sweeps: source in git history before round 5, numbers in
// profiles/r02_dia_blk_*, r03_dia_blk_*, r04_dia_blk_*, r04_pmc_dia_blk.json)
// into the variants DESIGN (f) still argues from:
//
//   library     launch_spmv's spmv_dia_blk_kernel (EpiApDot: Ap stored + <p, Ap>)
//   floor       p read + Ap write, 16 B per lane (the vector traffic alone)
//   slot-major  one slice per wave, every row group's value and x run of a slot
//               column loaded together (the library kernel's structure)
//   shuffled    the slot column's 128 values loaded once (16 B per lane,
//               nontemporal) and handed to the row groups by lane shuffles:
//               8 fewer vector memory instructions per slot column
//   no x        the x runs not loaded (values + p + Ap only; wrong results)
//
// Full variants are checked bitwise against the library kernel.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     tools/dia_blk_probe.hip -o tools/dia_blk_probe -Lkrylov_amd -lkrylov_hip -Wl,-rpath,'$ORIGIN/../krylov_amd'
//   ./tools/dia_blk_probe [N=3163] [reps=20]
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

constexpr int K = 8, CPL = 2, LPR = K / CPL, RPG = 64 / LPR, NG = kDiaSlice / RPG;

static void build_poisson(int N, std::vector<int> &ip, std::vector<int> &ix, std::vector<double> &dv) {
  const int64_t n = (int64_t)N * N;
  ip.assign(n + 1, 0);
  for (int64_t r = 0; r < n; ++r) {
    const int i = r % N, j = r / N;
    if (j > 0) ix.push_back((int)(r - N)), dv.push_back(-1.0);
    if (i > 0) ix.push_back((int)(r - 1)), dv.push_back(-1.0);
    ix.push_back((int)r), dv.push_back(4.0);
    if (i < N - 1) ix.push_back((int)(r + 1)), dv.push_back(-1.0);
    if (j < N - 1) ix.push_back((int)(r + N)), dv.push_back(-1.0);
    ip[r + 1] = (int)ix.size();
  }
}

typedef double d2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void copy_floor(const d2v *__restrict__ a, d2v *__restrict__ b, int64_t nb) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride)
    __builtin_nontemporal_store(a[i], b + i);
}

// MODE bits: 1 shuffled nontemporal values; 2 no x loads
template <int MODE>
__global__ __launch_bounds__(256) void slot_major(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                  const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                  const double *__restrict__ val, int64_t nslices, int64_t n,
                                                  const double *__restrict__ x, double *__restrict__ y,
                                                  double *__restrict__ part) {
  constexpr bool SHUF = (MODE & 1) != 0, NOX = (MODE & 2) != 0;
  __shared__ double red[256 * CPL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane / LPR, c0 = (lane % LPR) * CPL;
  double dacc[CPL] = {0.0, 0.0};
  for (int64_t s = (int64_t)g * 4 + wid; s < nslices; s += (int64_t)gridDim.x * 4) {
    const int w = swidth[s];
    const int64_t base = sptr[s], cb = base / kDiaSlice;
    double acc[NG][CPL];
#pragma unroll
    for (int r = 0; r < NG; ++r) acc[r][0] = acc[r][1] = 0.0;
    for (int j = 0; j < w; ++j) {
      const int off = doff[cb + j];
      const uint64_t m0 = dmask[2 * (cb + j)], m1 = dmask[2 * (cb + j) + 1];
      double a[NG], xv[NG][CPL];
      bool on[NG];
      d2v vv;
      if (SHUF) vv = __builtin_nontemporal_load(reinterpret_cast<const d2v *>(val + base + (int64_t)j * kDiaSlice) + lane);
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int rl = r * RPG + rl0;
        if (!SHUF) a[r] = val[base + (int64_t)j * kDiaSlice + rl];
        on[r] = (((rl & 1) ? m1 : m0) >> (rl >> 1) & 1u) != 0;
        if (NOX) {
          xv[r][0] = xv[r][1] = 1.0;
        } else {
          const d2v t = *reinterpret_cast<const d2v *>(x + (on[r] ? s * kDiaSlice + rl + off : 0) * K + c0);
          xv[r][0] = t.x;
          xv[r][1] = t.y;
        }
      }
      if (SHUF) {
#pragma unroll
        for (int r = 0; r < NG; ++r) {
          const int rl = r * RPG + rl0;
          const double lo = __shfl(vv.x, rl >> 1), hi = __shfl(vv.y, rl >> 1);
          a[r] = (rl & 1) ? hi : lo;
        }
      }
#pragma unroll
      for (int r = 0; r < NG; ++r)
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const double t = acc[r][c] + a[r] * xv[r][c];
          acc[r][c] = on[r] ? t : acc[r][c];
        }
    }
#pragma unroll
    for (int r = 0; r < NG; ++r) {
      const int64_t row = s * kDiaSlice + r * RPG + rl0;
      if (row < n) {
        const d2v q = *reinterpret_cast<const d2v *>(x + row * K + c0);
        d2v v;
        v.x = acc[r][0];
        v.y = acc[r][1];
        __builtin_nontemporal_store(v, reinterpret_cast<d2v *>(y + row * K + c0));
        dacc[0] += q.x * acc[r][0];
        dacc[1] += q.y * acc[r][1];
      }
    }
  }
  red[tid * CPL] = dacc[0];
  red[tid * CPL + 1] = dacc[1];
  block_tree_reduce(red, 256 * CPL, K);
  if (tid < K) part[(int64_t)g * K + tid] = red[tid];
}

// Row-per-lane-in-DPP-row layout (round 5): lane l owns row (l & 15) of each
// 16-row group and column pair l >> 4, so the rows r +- 1 of a lane are its
// neighbours inside its 16-lane DPP row. MODE bit 4: the slice's offset-0 x
// window is loaded once (every row < n, mask or not) and the -1 / +1 slot
// columns take their x from it by DPP row rotations (v_mov_dpp row_ror:1 /
// row_ror:15, the group's edge lane from the neighbouring group's register,
// the slice's edge rows from two halo loads); the epilogue's p is the same
// window. Products and their order are the library's: bitwise.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

template <int MODE>
__global__ __launch_bounds__(256) void slot_rowdpp(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                   const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                   const double *__restrict__ val, int64_t nslices, int64_t n,
                                                   const double *__restrict__ x, double *__restrict__ y,
                                                   double *__restrict__ part) {
  constexpr bool DERIVE = (MODE & 4) != 0;
  __shared__ double red[256 * CPL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane & 15, c0 = (lane >> 4) * CPL;
  const bool first = rl0 == 0, last = rl0 == 15;
  double dacc[CPL] = {0.0, 0.0};
  for (int64_t s = (int64_t)g * 4 + wid; s < nslices; s += (int64_t)gridDim.x * 4) {
    const int w = swidth[s];
    const int64_t base = sptr[s], cb = base / kDiaSlice, r0 = s * kDiaSlice;
    double acc[NG][CPL], xc[NG][CPL], hp[CPL], hm[CPL];
#pragma unroll
    for (int r = 0; r < NG; ++r) acc[r][0] = acc[r][1] = 0.0;
    if (DERIVE) {
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int64_t row = r0 + r * 16 + rl0;
        const d2v t = *reinterpret_cast<const d2v *>(x + (row < n ? row : n - 1) * K + c0);
        xc[r][0] = t.x;
        xc[r][1] = t.y;
      }
      const int64_t rp = r0 + kDiaSlice < n ? r0 + kDiaSlice : n - 1, rm = r0 > 0 ? r0 - 1 : 0;
      const d2v tp = *reinterpret_cast<const d2v *>(x + rp * K + c0);
      const d2v tm = *reinterpret_cast<const d2v *>(x + rm * K + c0);
      hp[0] = tp.x, hp[1] = tp.y, hm[0] = tm.x, hm[1] = tm.y;
    }
    for (int j = 0; j < w; ++j) {
      const int off = doff[cb + j];
      const uint64_t m0 = dmask[2 * (cb + j)], m1 = dmask[2 * (cb + j) + 1];
      double a[NG], xv[NG][CPL];
      bool on[NG];
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int rl = r * 16 + rl0;
        a[r] = val[base + (int64_t)j * kDiaSlice + rl];
        on[r] = (((rl & 1) ? m1 : m0) >> (rl >> 1) & 1u) != 0;
      }
      if (DERIVE && off == 0) {
#pragma unroll
        for (int r = 0; r < NG; ++r) xv[r][0] = xc[r][0], xv[r][1] = xc[r][1];
      } else if (DERIVE && off == 1) {
#pragma unroll
        for (int r = 0; r < NG; ++r)
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const double own = dpp_d<0x12F>(xc[r][c]);  // row_ror:15: lane i <- lane i + 1
            const double nxt = r + 1 < NG ? dpp_d<0x12F>(xc[r + 1 < NG ? r + 1 : r][c]) : hp[c];
            xv[r][c] = last ? nxt : own;
          }
      } else if (DERIVE && off == -1) {
#pragma unroll
        for (int r = 0; r < NG; ++r)
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const double own = dpp_d<0x121>(xc[r][c]);  // row_ror:1: lane i <- lane i - 1
            const double prv = r > 0 ? dpp_d<0x121>(xc[r > 0 ? r - 1 : 0][c]) : hm[c];
            xv[r][c] = first ? prv : own;
          }
      } else {
#pragma unroll
        for (int r = 0; r < NG; ++r) {
          const int64_t row = r0 + r * 16 + rl0;
          const d2v t = *reinterpret_cast<const d2v *>(x + (on[r] ? row + off : 0) * K + c0);
          xv[r][0] = t.x;
          xv[r][1] = t.y;
        }
      }
#pragma unroll
      for (int r = 0; r < NG; ++r)
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const double t = acc[r][c] + a[r] * xv[r][c];
          acc[r][c] = on[r] ? t : acc[r][c];
        }
    }
#pragma unroll
    for (int r = 0; r < NG; ++r) {
      const int64_t row = r0 + r * 16 + rl0;
      if (row < n) {
        double q[CPL];
        if (DERIVE) {
          q[0] = xc[r][0], q[1] = xc[r][1];
        } else {
          const d2v t = *reinterpret_cast<const d2v *>(x + row * K + c0);
          q[0] = t.x, q[1] = t.y;
        }
        d2v v;
        v.x = acc[r][0];
        v.y = acc[r][1];
        __builtin_nontemporal_store(v, reinterpret_cast<d2v *>(y + row * K + c0));
        dacc[0] += q[0] * acc[r][0];
        dacc[1] += q[1] * acc[r][1];
      }
    }
  }
  red[tid * CPL] = dacc[0];
  red[tid * CPL + 1] = dacc[1];
  block_tree_reduce(red, 256 * CPL, K);
  if (tid < K) part[(int64_t)g * K + tid] = red[tid];
}

// LDS window (round 5), the library's coalesced layout (lane l: row l >> 2 of
// each 16-row group, column pair l & 3). The slice's offset-0 x window is
// loaded once into registers (every row < n, mask or not) and written to the
// wave's own LDS window together with the rows just outside the slice; the
// -1 / +1 slot columns read their x runs from it (ds_read_b128 at +-64 B),
// and the epilogue's p is the register window. No barrier: each wave reads
// only its own window (s_waitcnt on LDS). MODE bit 1: shuffled nt values.
template <int MODE>
__global__ __launch_bounds__(256) void slot_ldswin(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                   const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                   const double *__restrict__ val, int64_t nslices, int64_t n,
                                                   const double *__restrict__ x, double *__restrict__ y,
                                                   double *__restrict__ part) {
  constexpr bool SHUF = (MODE & 1) != 0;
  constexpr int WROWS = kDiaSlice + 2;  // rows r0 - 1 .. r0 + 128
  __shared__ d2v win[4][WROWS * 4];
  __shared__ double red[256 * CPL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane / LPR, cp = lane % LPR, c0 = cp * CPL;
  d2v *W = win[wid];
  double dacc[CPL] = {0.0, 0.0};
  for (int64_t s = (int64_t)g * 4 + wid; s < nslices; s += (int64_t)gridDim.x * 4) {
    const int w = swidth[s];
    const int64_t base = sptr[s], cb = base / kDiaSlice, r0 = s * kDiaSlice;
    double acc[NG][CPL];
#pragma unroll
    for (int r = 0; r < NG; ++r) acc[r][0] = acc[r][1] = 0.0;
    {
      // the window: rows r0 .. r0 + 127 (clamped below n) and the halo rows
      // r0 - 1 (lanes 0..3) and r0 + 128 (lanes 4..7), clamped
      d2v xc[NG];
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int64_t row = r0 + r * RPG + rl0;
        xc[r] = *reinterpret_cast<const d2v *>(x + (row < n ? row : n - 1) * K + c0);
      }
      const int64_t hr = lane < 4 ? (r0 > 0 ? r0 - 1 : 0) : (r0 + kDiaSlice < n ? r0 + kDiaSlice : n - 1);
      const d2v h = *reinterpret_cast<const d2v *>(x + hr * K + c0);
      if (lane < 8) W[(lane < 4 ? 0 : WROWS - 1) * 4 + cp] = h;
#pragma unroll
      for (int r = 0; r < NG; ++r) W[(r * RPG + rl0 + 1) * 4 + cp] = xc[r];
    }
    for (int j = 0; j < w; ++j) {
      const int off = doff[cb + j];
      const uint64_t m0 = dmask[2 * (cb + j)], m1 = dmask[2 * (cb + j) + 1];
      double a[NG];
      d2v xv[NG];
      bool on[NG];
      d2v vv;
      if (SHUF) vv = __builtin_nontemporal_load(reinterpret_cast<const d2v *>(val + base + (int64_t)j * kDiaSlice) + lane);
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int rl = r * RPG + rl0;
        if (!SHUF) a[r] = val[base + (int64_t)j * kDiaSlice + rl];
        on[r] = (((rl & 1) ? m1 : m0) >> (rl >> 1) & 1u) != 0;
      }
      if (off >= -1 && off <= 1) {
#pragma unroll
        for (int r = 0; r < NG; ++r) xv[r] = W[(r * RPG + rl0 + 1 + off) * 4 + cp];
      } else {
#pragma unroll
        for (int r = 0; r < NG; ++r)
          xv[r] = *reinterpret_cast<const d2v *>(x + (on[r] ? r0 + r * RPG + rl0 + off : 0) * K + c0);
      }
      if (SHUF) {
#pragma unroll
        for (int r = 0; r < NG; ++r) {
          const int rl = r * RPG + rl0;
          const double lo = __shfl(vv.x, rl >> 1), hi = __shfl(vv.y, rl >> 1);
          a[r] = (rl & 1) ? hi : lo;
        }
      }
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const double t0 = acc[r][0] + a[r] * xv[r].x, t1 = acc[r][1] + a[r] * xv[r].y;
        acc[r][0] = on[r] ? t0 : acc[r][0];
        acc[r][1] = on[r] ? t1 : acc[r][1];
      }
    }
#pragma unroll
    for (int r = 0; r < NG; ++r) {
      const int64_t row = r0 + r * RPG + rl0;
      if (row < n) {
        d2v v;
        v.x = acc[r][0];
        v.y = acc[r][1];
        __builtin_nontemporal_store(v, reinterpret_cast<d2v *>(y + row * K + c0));
        const d2v q = W[(r * RPG + rl0 + 1) * 4 + cp];
        dacc[0] += q.x * acc[r][0];
        dacc[1] += q.y * acc[r][1];
      }
    }
  }
  red[tid * CPL] = dacc[0];
  red[tid * CPL + 1] = dacc[1];
  block_tree_reduce(red, 256 * CPL, K);
  if (tid < K) part[(int64_t)g * K + tid] = red[tid];
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 3163;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<int> ip, ix;
  std::vector<double> dv;
  build_poisson(N, ip, ix, dv);
  const int64_t n = (int64_t)ip.size() - 1, nnz = ix.size();
  kry_ctx *ctx;
  KC(kry_ctx_create(0, &ctx));
  kry_csr *A;
  KC(kry_csr_create(ctx, n, nnz, ip.data(), ix.data(), dv.data(), KRY_F64, KRY_I32, &A));
  if (!A->dia) {
    fprintf(stderr, "no DIA image\n");
    return 1;
  }
  printf("N=%d n=%ld nnz=%ld k=%d dia_slices=%ld dia_slots=%ld\n", N, (long)n, (long)nnz, K, (long)A->dia_nslices,
         (long)A->dia_nslots);
  std::vector<double> xh(n * K);
  for (int64_t i = 0; i < n * K; ++i) xh[i] = 1.0 + (double)((i * 7919) % 1000) * 1e-3;
  kry_vec *xv, *yv, *yrefv;
  KC(kry_vec_create(ctx, n, K, KRY_F64, &xv));
  KC(kry_vec_create(ctx, n, K, KRY_F64, &yv));
  KC(kry_vec_create(ctx, n, K, KRY_F64, &yrefv));
  KC(kry_vec_upload(xv, xh.data()));
  double *x = (double *)xv->d, *y = (double *)yv->d, *yref = (double *)yrefv->d, *part;
  const int full = (int)((A->dia_nslices + 3) / 4);  // one slice per wave
  CK(hipMalloc(&part, (size_t)std::max(full, kMaxGridBlk) * K * 8));
  hipStream_t st = ctx->stream;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double S = (double)nnz * 12 + (double)(n + 1) * 4 + 2.0 * n * K * 8;
  const double img = (double)A->dia_nslots * 8 + (double)A->dia_nslices * 20 + 2.0 * n * K * 8;
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
    printf("%-44s %.4f ms  S-rate %.0f GB/s  image-rate %.0f GB/s\n", name, ms, S / ms / 1e6, img / ms / 1e6);
  };
  auto library = [&] {
    int P;
    launch_spmv<double, double, int>(A, K, SrcPlain<double>{x, K}, EpiApDot<double>{yref, nullptr, K}, part, &P,
                                     nullptr, 0, st);
  };
  library();
  CK(hipStreamSynchronize(st));
  std::vector<double> ref(n * K), got(n * K);
  CK(hipMemcpy(ref.data(), yref, n * K * 8, hipMemcpyDeviceToHost));
  int64_t bad = 0;
  for (int64_t r = 0; r < n; ++r)
    for (int c = 0; c < K; ++c) {
      double acc = 0.0;
      for (int e = ip[r]; e < ip[r + 1]; ++e) {
        volatile double p = dv[e] * xh[(int64_t)ix[e] * K + c];
        acc = acc + p;
      }
      bad += memcmp(&acc, &ref[r * K + c], 8) != 0;
    }
  printf("library vs host csr_matvecs: %ld entries differ\n", (long)bad);
#define SM(MODE, NAME, CHECK)                                                                                  \
  {                                                                                                            \
    timeit(NAME, [&] {                                                                                         \
      hipLaunchKernelGGL((slot_major<MODE>), dim3(full), dim3(256), 0, st, (const int64_t *)A->dia_sptr,       \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,   \
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);          \
    });                                                                                                        \
    if (CHECK) {                                                                                               \
      CK(hipMemcpy(got.data(), y, n * K * 8, hipMemcpyDeviceToHost));                                          \
      if (memcmp(got.data(), ref.data(), n * K * 8) != 0) printf("  !! %s differs from the library\n", NAME); \
    }                                                                                                          \
  }
#define RD(MODE, NAME)                                                                                         \
  {                                                                                                            \
    timeit(NAME, [&] {                                                                                         \
      hipLaunchKernelGGL((slot_rowdpp<MODE>), dim3(full), dim3(256), 0, st, (const int64_t *)A->dia_sptr,      \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,   \
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);          \
    });                                                                                                        \
    CK(hipMemcpy(got.data(), y, n * K * 8, hipMemcpyDeviceToHost));                                            \
    if (memcmp(got.data(), ref.data(), n * K * 8) != 0) printf("  !! %s differs from the library\n", NAME);   \
  }
#define LW(MODE, NAME)                                                                                         \
  {                                                                                                            \
    timeit(NAME, [&] {                                                                                         \
      hipLaunchKernelGGL((slot_ldswin<MODE>), dim3(full), dim3(256), 0, st, (const int64_t *)A->dia_sptr,      \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,   \
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);          \
    });                                                                                                        \
    CK(hipMemcpy(got.data(), y, n * K * 8, hipMemcpyDeviceToHost));                                            \
    if (memcmp(got.data(), ref.data(), n * K * 8) != 0) printf("  !! %s differs from the library\n", NAME);   \
  }
  for (int rep = 0; rep < 2; ++rep) {
    timeit("library spmv_dia_blk (EpiApDot)", library);
    timeit("floor: p read + Ap write", [&] {
      hipLaunchKernelGGL(copy_floor, dim3(8192), dim3(256), 0, st, (const d2v *)x, (d2v *)y, n * K / 2);
    });
    SM(0, "slot-major", true);
    SM(1, "slot-major, shuffled nt values", true);
    SM(2, "slot-major, no x", false);
    SM(3, "slot-major, shuffled nt values, no x", false);
    RD(0, "row-per-lane layout");
    RD(4, "row-per-lane layout, -1/0/+1 x by DPP");
    LW(0, "LDS window, -1/0/+1 x from registers");
    LW(1, "LDS window + shuffled nt values");
  }
  CK(hipFree(part));
  KC(kry_vec_destroy(xv));
  KC(kry_vec_destroy(yv));
  KC(kry_vec_destroy(yrefv));
  KC(kry_csr_destroy(A));
  KC(kry_ctx_destroy(ctx));
  return 0;
}
