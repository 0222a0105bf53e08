// Microbenchmark of the block right-hand-side DIA SpMV (k = 8, cfg4's 5-point
// Poisson N^2) on gfx950 (development tool, not product). Uploads the matrix
// through the library's C-ABI, times the library's block CG SpMV (Ap stored +
// <p, Ap> partials) and probe variants on the same image: no store, a pure
// p-read + Ap-write stream (the traffic floor), and slot-major kernels in
// which a wave loads one slot column for ALL row groups of its slice at once
// (CPL = 2, 4 or 8 columns per lane). Every full variant is checked bitwise
// against the library kernel.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     tools/dia_blk_bench.hip -o tools/dia_blk_bench -Lkrylov_amd -lkrylov_hip -Wl,-rpath,'$ORIGIN/../krylov_amd'
//   ./tools/dia_blk_bench [N=3163] [reps=20]
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

constexpr int K = 8;

static void build_poisson(int N, std::vector<int> &ip, std::vector<int> &ix, std::vector<double> &dv) {
  const int64_t n = (int64_t)N * N;
  ip.assign(n + 1, 0);
  ix.clear();
  dv.clear();
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

// p read + Ap write, 16 B per lane: the SpMV's vector traffic alone
__global__ __launch_bounds__(256) void copy_floor(const d2v *__restrict__ a, d2v *__restrict__ b, int64_t nb) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride)
    __builtin_nontemporal_store(a[i], b + i);
}

template <int C>
__device__ __forceinline__ void ldx(const double *p, double (&o)[C]) {
#pragma unroll
  for (int c = 0; c < C; c += 2) {
    const d2v v = *reinterpret_cast<const d2v *>(p + c);
    o[c] = v.x;
    o[c + 1] = v.y;
  }
}

// Slot-major: per slot column j of the slice, every row group's value and x
// run are loaded together (NG = 128 / rows-per-group loads of each), then
// accumulated; each (row, column) still sums its slot columns in ascending
// order from 0. MODE bits: 1 no store (dot terms only); 2 nontemporal value
// loads; 4 the slice's epilogue deferred behind the next slice's first slot
// column loads; 8 the epilogue's p values taken from the offset-0 slot
// column's x run (reloaded only where that slot is a hole); 16 the slot
// column's 128 values loaded once (16 B per lane) and handed to the row
// groups by lane shuffles; 32 every x run read at offset 0 (locality probe,
// wrong results); 64 no x loads; 256 no XCD remap of the block index; 512
// wave m takes slices m, m + W, m + 2W, ... (W waves) instead of a contiguous run.
template <int CPL, int MODE, int BS = 256>
__global__ __launch_bounds__(BS) void dia_slot_major(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                      const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                      const double *__restrict__ val, int64_t nslices, int64_t n,
                                                      const double *__restrict__ x, double *__restrict__ y,
                                                      double *__restrict__ part) {
  constexpr int LPR = K / CPL, RPG = 64 / LPR, NG = kDiaSlice / RPG;
  constexpr bool DEFER = (MODE & 4) != 0, CAPT = (MODE & 8) != 0, SHUF = (MODE & 16) != 0;
  __shared__ double red[BS * CPL];
  constexpr int WPB = BS / 64;  // waves per block
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = (MODE & 256) ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane / LPR, c0 = (lane % LPR) * CPL;
  const int64_t W = (int64_t)gridDim.x * WPB, m = (int64_t)g * WPB + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  double dacc[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) dacc[c] = 0.0;
  double pend[DEFER ? NG : 1][CPL];
  double xi[CAPT ? NG : 1][CPL];
  bool have[CAPT ? NG : 1];
  int64_t prow0 = -1;  // first row (group 0, lane's rl0) of the pending slice
  auto finish = [&](int64_t row0, auto &&accs) {
#pragma unroll
    for (int r = 0; r < NG; ++r) {
      const int64_t row = row0 + r * RPG;
      if (row < n) {
        double q[CPL];
        if (CAPT) {
          if (have[r]) {
#pragma unroll
            for (int c = 0; c < CPL; ++c) q[c] = xi[CAPT ? r : 0][c];
          } else {
            ldx<CPL>(x + row * K + c0, q);
          }
        } else {
          ldx<CPL>(x + row * K + c0, q);
        }
        if (!(MODE & 1)) {
#pragma unroll
          for (int c = 0; c < CPL; c += 2) {
            d2v v;
            v.x = accs(r, c);
            v.y = accs(r, c + 1);
            __builtin_nontemporal_store(v, reinterpret_cast<d2v *>(y + row * K + c0 + c));
          }
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) dacc[c] += dterm(q[c], accs(r, c));
      }
    }
  };
  const bool strided = (MODE & 512) != 0;
  for (int64_t s = strided ? m : s_begin; s < (strided ? nslices : s_end); s += strided ? W : 1) {
    const int w = swidth[s];
    const int64_t base = sptr[s], cb = base / kDiaSlice;
    double acc[NG][CPL];
#pragma unroll
    for (int r = 0; r < NG; ++r)
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[r][c] = 0.0;
    for (int j = 0; j < w; ++j) {
      const int off = doff[cb + j];
      const uint64_t m0 = dmask[2 * (cb + j)], m1 = dmask[2 * (cb + j) + 1];
      double a[NG], xv[NG][CPL];
      bool on[NG];
      d2v vv;
      if (SHUF) {
        const d2v *vp = reinterpret_cast<const d2v *>(val + base + (int64_t)j * kDiaSlice) + lane;
        vv = (MODE & 2) ? __builtin_nontemporal_load(vp) : *vp;
      }
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int rl = r * RPG + rl0;
        if (!SHUF) {
          const double *vp = val + base + (int64_t)j * kDiaSlice + rl;
          a[r] = (MODE & 2) ? __builtin_nontemporal_load(vp) : *vp;
        }
        on[r] = (((rl & 1) ? m1 : m0) >> (rl >> 1) & 1u) != 0;
        const int64_t row = s * kDiaSlice + rl;
        if (MODE & 64) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) xv[r][c] = 1.0;
        } else {
          ldx<CPL>(x + (on[r] ? row + ((MODE & 32) ? 0 : off) : 0) * K + c0, xv[r]);
        }
      }
      if (DEFER && j == 0 && prow0 >= 0) {
        __builtin_amdgcn_sched_barrier(0);
        finish(prow0, [&](int r, int c) { return pend[DEFER ? r : 0][c]; });
        __builtin_amdgcn_sched_barrier(0);
        prow0 = -1;
      }
      if (SHUF) {
#pragma unroll
        for (int r = 0; r < NG; ++r) {
          const int rl = r * RPG + rl0;
          const double lo = __shfl(vv.x, rl >> 1), hi = __shfl(vv.y, rl >> 1);
          a[r] = (rl & 1) ? hi : lo;
        }
      }
      if (CAPT && off == 0) {
#pragma unroll
        for (int r = 0; r < NG; ++r) {
          have[CAPT ? r : 0] = on[r];
#pragma unroll
          for (int c = 0; c < CPL; ++c) xi[CAPT ? r : 0][c] = xv[r][c];
        }
      }
#pragma unroll
      for (int r = 0; r < NG; ++r)
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const double p = a[r] * xv[r][c];
          const double t = acc[r][c] + p;
          acc[r][c] = on[r] ? t : acc[r][c];
        }
    }
    if (CAPT) {
      bool any0 = false;
      for (int j = 0; j < w; ++j) any0 = any0 || doff[cb + j] == 0;
      if (!any0)
#pragma unroll
        for (int r = 0; r < NG; ++r) have[CAPT ? r : 0] = false;
    }
    if (DEFER) {
      if (w == 0 && prow0 >= 0) finish(prow0, [&](int r, int c) { return pend[DEFER ? r : 0][c]; });
#pragma unroll
      for (int r = 0; r < NG; ++r)
#pragma unroll
        for (int c = 0; c < CPL; ++c) pend[DEFER ? r : 0][c] = acc[r][c];
      prow0 = s * kDiaSlice + rl0;
    } else {
      finish(s * kDiaSlice + rl0, [&](int r, int c) { return acc[r][c]; });
    }
  }
  if (DEFER && prow0 >= 0) finish(prow0, [&](int r, int c) { return pend[DEFER ? r : 0][c]; });
#pragma unroll
  for (int c = 0; c < CPL; ++c) red[tid * CPL + c] = dacc[c];
  block_tree_reduce(red, BS * CPL, K);
  if (tid < K) part[(int64_t)g * K + tid] = red[tid];
}

// Split slices: wave (s, part) handles GPW of the slice's 8 row groups (CPL 2,
// k = 8), one (slice, part) per wave; SPR slot columns per round (all their
// loads issued together). Fewer registers per wave (more resident waves) or
// more loads in flight per wave than the whole-slice kernel.
template <int GPW, int SPR>
__global__ __launch_bounds__(256) void dia_split(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                 const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                 const double *__restrict__ val, int64_t nslices, int64_t n,
                                                 const double *__restrict__ x, double *__restrict__ y,
                                                 double *__restrict__ part) {
  constexpr int CPL = 2, LPR = K / CPL, RPG = 64 / LPR, NG = kDiaSlice / RPG, PARTS = NG / GPW;
  __shared__ double red[256 * CPL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane / LPR, c0 = (lane % LPR) * CPL;
  const int64_t W = (int64_t)gridDim.x * 4;
  double dacc[CPL] = {0.0, 0.0};
  for (int64_t t = (int64_t)g * 4 + wid; t < nslices * PARTS; t += W) {
    const int64_t s = t / PARTS;
    const int pt = (int)(t % PARTS);
    const int w = swidth[s];
    const int64_t base = sptr[s], cb = base / kDiaSlice;
    double acc[GPW][CPL];
#pragma unroll
    for (int r = 0; r < GPW; ++r) acc[r][0] = acc[r][1] = 0.0;
    for (int j0 = 0; j0 < w; j0 += SPR) {
      double a[SPR][GPW], xv[SPR][GPW][CPL];
      bool on[SPR][GPW];
#pragma unroll
      for (int q = 0; q < SPR; ++q) {
        const int j = j0 + q < w ? j0 + q : w - 1;  // a slot past the width repeats the last (dropped below)
        const int off = doff[cb + j];
        const uint64_t m0 = dmask[2 * (cb + j)], m1 = dmask[2 * (cb + j) + 1];
#pragma unroll
        for (int r = 0; r < GPW; ++r) {
          const int rl = (pt * GPW + r) * RPG + rl0;
          a[q][r] = val[base + (int64_t)j * kDiaSlice + rl];
          on[q][r] = j0 + q < w && ((((rl & 1) ? m1 : m0) >> (rl >> 1)) & 1u) != 0;
          ldx<CPL>(x + (on[q][r] ? s * kDiaSlice + rl + off : 0) * K + c0, xv[q][r]);
        }
      }
#pragma unroll
      for (int q = 0; q < SPR; ++q)
#pragma unroll
        for (int r = 0; r < GPW; ++r)
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const double p = a[q][r] * xv[q][r][c];
            const double tt = acc[r][c] + p;
            acc[r][c] = on[q][r] ? tt : acc[r][c];
          }
    }
#pragma unroll
    for (int r = 0; r < GPW; ++r) {
      const int64_t row = s * kDiaSlice + (pt * GPW + r) * RPG + rl0;
      if (row < n) {
        double q[CPL];
        ldx<CPL>(x + row * K + c0, q);
        d2v v;
        v.x = acc[r][0];
        v.y = acc[r][1];
        __builtin_nontemporal_store(v, reinterpret_cast<d2v *>(y + row * K + c0));
        for (int c = 0; c < CPL; ++c) dacc[c] += dterm(q[c], acc[r][c]);
      }
    }
  }
  for (int c = 0; c < CPL; ++c) red[tid * CPL + c] = dacc[c];
  block_tree_reduce(red, 256 * CPL, K);
  if (tid < K) part[(int64_t)g * K + tid] = red[tid];
}

// Shifted windows (round 3): one slice per wave, CPL 2 (lane = row rl0 of
// each 16-row group, columns c0, c0 + 1). A slot column whose offset is the
// previous one's + 1 reads the previous window one row further on: lane l
// takes lane l + 4's value of the same group register, lanes 60..63 take
// lanes 0..3 of the next group (the same rotation of register r + 1), and
// the last group's last row is one extra 16-B load. The 5-point stencil's
// -1 / 0 / +1 slots then cost one window of loads instead of three, and the
// offset-0 window is kept for the epilogue's p (no reload). Every window
// position is loaded at its clamped row whether or not its mask bit is set,
// so a derived position is always the true x row (a row out of range is a
// hole in every slot). MODE bits: 1 values loaded once per slot (16 B per
// lane) and handed to the row groups by lane shuffles; 2 nontemporal value
// loads; 4 never derive (full window loads, clamped; epilogue p captured).
template <int MODE>
__global__ __launch_bounds__(256) void dia_shift(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                                 const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                                 const double *__restrict__ val, int64_t nslices, int64_t n,
                                                 const double *__restrict__ x, double *__restrict__ y,
                                                 double *__restrict__ part) {
  constexpr int CPL = 2, LPR = K / CPL, RPG = 64 / LPR, NG = kDiaSlice / RPG;
  constexpr bool SHUF = (MODE & 1) != 0, NTV = (MODE & 2) != 0, NODER = (MODE & 4) != 0;
  __shared__ double red[256 * CPL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane / LPR, c0 = (lane % LPR) * CPL;
  const int src4 = (lane + 4) & 63;
  const bool tail = lane >= 64 - LPR;  // row rl0 = RPG - 1: its +1 neighbour is the next group's row 0
  const int64_t W = (int64_t)gridDim.x * 4;
  double dacc[CPL] = {0.0, 0.0};
  auto ldrow = [&](int64_t row, double (&o)[CPL]) {
    row = row < 0 ? 0 : (row >= n ? n - 1 : row);
    ldx<CPL>(x + row * K + c0, o);
  };
  for (int64_t s = (int64_t)g * 4 + wid; s < nslices; s += W) {
    const int w = swidth[s];
    const int64_t base = sptr[s], cb = base / kDiaSlice;
    const int64_t row0 = s * kDiaSlice + rl0;
    double acc[NG][CPL], xw[NG][CPL], xi[NG][CPL];
#pragma unroll
    for (int r = 0; r < NG; ++r)
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[r][c] = 0.0;
    bool have_i = false;
    int prev = 0;
    for (int j = 0; j < w; ++j) {
      const int off = doff[cb + j];
      const uint64_t m0 = dmask[2 * (cb + j)], m1 = dmask[2 * (cb + j) + 1];
      double a[NG];
      d2v vv;
      if (SHUF) {
        const d2v *vp = reinterpret_cast<const d2v *>(val + base + (int64_t)j * kDiaSlice) + lane;
        vv = NTV ? __builtin_nontemporal_load(vp) : *vp;
      } else {
#pragma unroll
        for (int r = 0; r < NG; ++r) {
          const double *vp = val + base + (int64_t)j * kDiaSlice + r * RPG + rl0;
          a[r] = NTV ? __builtin_nontemporal_load(vp) : *vp;
        }
      }
      if (!NODER && j > 0 && off == prev + 1) {
        double e[CPL];
        ldrow(s * kDiaSlice + kDiaSlice + prev, e);  // row 128 of the previous window
        double R[NG][CPL];
#pragma unroll
        for (int r = 0; r < NG; ++r)
#pragma unroll
          for (int c = 0; c < CPL; ++c) R[r][c] = __shfl(xw[r][c], src4);
#pragma unroll
        for (int r = 0; r < NG; ++r)
#pragma unroll
          for (int c = 0; c < CPL; ++c) xw[r][c] = tail ? (r + 1 < NG ? R[r + 1 < NG ? r + 1 : r][c] : e[c]) : R[r][c];
      } else {
#pragma unroll
        for (int r = 0; r < NG; ++r) ldrow(row0 + r * RPG + off, xw[r]);
      }
      prev = off;
      if (SHUF) {
#pragma unroll
        for (int r = 0; r < NG; ++r) {
          const int rl = r * RPG + rl0;
          const double lo = __shfl(vv.x, rl >> 1), hi = __shfl(vv.y, rl >> 1);
          a[r] = (rl & 1) ? hi : lo;
        }
      }
      if (off == 0) {
        have_i = true;
#pragma unroll
        for (int r = 0; r < NG; ++r)
#pragma unroll
          for (int c = 0; c < CPL; ++c) xi[r][c] = xw[r][c];
      }
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int rl = r * RPG + rl0;
        const bool on = ((((rl & 1) ? m1 : m0) >> (rl >> 1)) & 1u) != 0;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const double p = a[r] * xw[r][c];
          const double t = acc[r][c] + p;
          acc[r][c] = on ? t : acc[r][c];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < NG; ++r) {
      const int64_t row = row0 + r * RPG;
      if (row < n) {
        double q[CPL];
        if (have_i) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) q[c] = xi[r][c];
        } else {
          ldx<CPL>(x + row * K + c0, q);
        }
        d2v v;
        v.x = acc[r][0];
        v.y = acc[r][1];
        __builtin_nontemporal_store(v, reinterpret_cast<d2v *>(y + row * K + c0));
#pragma unroll
        for (int c = 0; c < CPL; ++c) dacc[c] += dterm(q[c], acc[r][c]);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CPL; ++c) red[tid * CPL + c] = dacc[c];
  block_tree_reduce(red, 256 * CPL, K);
  if (tid < K) part[(int64_t)g * K + tid] = red[tid];
}

// LDS window (round 4): the slot columns whose offsets lie within +-kNear of
// the diagonal (Poisson: -1, 0, +1) read x from ONE window of the slice's x
// rows [128 s + lo, 128 s + hi + 128), staged in LDS by global_load_lds (16 B
// per lane, 1 KB per instruction) instead of three overlapping 1 KB runs per
// row group through L1; the epilogue's p comes from the same window. MODE bit
// 1: the slice's values staged in LDS too (one 1 KB DMA per slot column, then
// ds_read_b64 per row group) instead of 8-B loads replicated over a row's
// lanes. Far columns (+-m) load straight to registers as before. One slice per
// wave. Bitwise the library kernel (same products, same order).
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;
constexpr int kNear = 4;
constexpr int kWinB = ((128 + 2 * kNear) * 64 + 1023) / 1024 * 1024;  // whole 1 KB DMA pieces
constexpr int kValMax = 8;
template <int MODE>
__global__ __launch_bounds__(256) void dia_lds(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                               const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                               const double *__restrict__ val, int64_t nslices, int64_t n,
                                               const double *__restrict__ x, double *__restrict__ y,
                                               double *__restrict__ part) {
  constexpr int CPL = 2, LPR = K / CPL, RPG = 64 / LPR, NG = kDiaSlice / RPG;
  constexpr bool VL = (MODE & 1) != 0;
  constexpr bool HOIST = (MODE & 4) != 0;  // the first / last slot column, when far, loaded before the wait
  constexpr int PERW = kWinB + (VL ? kValMax * 1024 : 0);
  __shared__ __attribute__((aligned(16))) char lds[4 * PERW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane / LPR, c0 = (lane % LPR) * CPL;
  char *my = lds + wid * PERW;
  const int64_t s = (int64_t)g * 4 + wid;
  double dacc[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) dacc[c] = 0.0;
  if (s < nslices) {
    const int w = swidth[s];
    const int64_t base = sptr[s], cb = base / kDiaSlice;
    int lo = 1 << 30, hi = -(1 << 30);
    for (int j = 0; j < w; ++j) {
      const int o = doff[cb + j];
      if (o >= -kNear && o <= kNear) {
        lo = o < lo ? o : lo;
        hi = o > hi ? o : hi;
      }
    }
    const bool win = lo <= hi;
    const int64_t r0 = s * kDiaSlice;
    const int64_t nx = n * K;
    if (win) {
      const int nb = (hi - lo + kDiaSlice) * K * 8;
      const int64_t e0 = (r0 + lo) * K;
      for (int i = 0; i * 1024 < nb; ++i) {
        int64_t e = e0 + (i * 1024 + lane * 16) / 8;
        e = e < 0 ? 0 : (e > nx - 2 ? nx - 2 : e);  // rows outside x: holes, never added
        __builtin_amdgcn_global_load_lds((glb_void *)(x + e), (lds_void *)(my + i * 1024), 16, 0, 0);
      }
    }
    const bool vl = VL && w <= kValMax;
    if (vl)
      for (int j = 0; j < w; ++j)
        __builtin_amdgcn_global_load_lds((glb_void *)(val + base + (int64_t)j * kDiaSlice + 2 * lane),
                                         (lds_void *)(my + kWinB + j * 1024), 16, 0, 0);
    // far edge columns (Poisson: offsets -m and +m) into registers now, so
    // their loads travel with the DMAs (one round trip per slice)
    double xl[HOIST ? NG : 1][CPL], xr[HOIST ? NG : 1][CPL];
    bool hl = false, hr = false;
    if (HOIST && w > 0) {
      const int o0 = doff[cb], o1 = doff[cb + w - 1];
      hl = !(win && o0 >= lo && o0 <= hi);
      hr = w > 1 && !(win && o1 >= lo && o1 <= hi);
      const uint64_t l0 = dmask[2 * cb], l1 = dmask[2 * cb + 1];
      const uint64_t h0 = dmask[2 * (cb + w - 1)], h1 = dmask[2 * (cb + w - 1) + 1];
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int rl = r * RPG + rl0;
        const bool onl = hl && (((rl & 1) ? l1 : l0) >> (rl >> 1) & 1u) != 0;
        const bool onr = hr && (((rl & 1) ? h1 : h0) >> (rl >> 1) & 1u) != 0;
        ldx<CPL>(x + (onl ? r0 + rl + o0 : 0) * K + c0, xl[HOIST ? r : 0]);
        ldx<CPL>(x + (onr ? r0 + rl + o1 : 0) * K + c0, xr[HOIST ? r : 0]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    double acc[NG][CPL];
#pragma unroll
    for (int r = 0; r < NG; ++r)
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[r][c] = 0.0;
    for (int j = 0; j < w; ++j) {
      const int off = doff[cb + j];
      const uint64_t m0 = dmask[2 * (cb + j)], m1 = dmask[2 * (cb + j) + 1];
      const bool near = win && off >= lo && off <= hi;
      double a[NG], xv[NG][CPL];
      bool on[NG];
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int rl = r * RPG + rl0;
        on[r] = (((rl & 1) ? m1 : m0) >> (rl >> 1) & 1u) != 0;
        a[r] = vl ? *reinterpret_cast<const double *>(my + kWinB + j * 1024 + rl * 8)
                  : val[base + (int64_t)j * kDiaSlice + rl];
        if (near) {
          const d2v v = *reinterpret_cast<const d2v *>(my + (rl + off - lo) * K * 8 + c0 * 8);
          xv[r][0] = v.x;
          xv[r][1] = v.y;
        } else if (HOIST && j == 0 && hl) {
          xv[r][0] = xl[HOIST ? r : 0][0];
          xv[r][1] = xl[HOIST ? r : 0][1];
        } else if (HOIST && j == w - 1 && hr) {
          xv[r][0] = xr[HOIST ? r : 0][0];
          xv[r][1] = xr[HOIST ? r : 0][1];
        } else {
          ldx<CPL>(x + (on[r] ? r0 + rl + off : 0) * K + c0, xv[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < NG; ++r)
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const double p = a[r] * xv[r][c];
          const double t = acc[r][c] + p;
          acc[r][c] = on[r] ? t : acc[r][c];
        }
    }
    const bool pin = win && lo <= 0 && hi >= 0;
#pragma unroll
    for (int r = 0; r < NG; ++r) {
      const int rl = r * RPG + rl0;
      const int64_t row = r0 + rl;
      if (row < n) {
        double q[CPL];
        if (pin) {
          const d2v v = *reinterpret_cast<const d2v *>(my + (rl - lo) * K * 8 + c0 * 8);
          q[0] = v.x;
          q[1] = v.y;
        } else {
          ldx<CPL>(x + row * K + c0, q);
        }
        d2v o;
        o.x = acc[r][0];
        o.y = acc[r][1];
        __builtin_nontemporal_store(o, reinterpret_cast<d2v *>(y + row * K + c0));
#pragma unroll
        for (int c = 0; c < CPL; ++c) dacc[c] += dterm(q[c], acc[r][c]);
      }
    }
  }
  __syncthreads();  // every wave is done with its window: the LDS serves the reduction
  double *red = reinterpret_cast<double *>(lds);
#pragma unroll
  for (int c = 0; c < CPL; ++c) red[tid * CPL + c] = dacc[c];
  block_tree_reduce(red, 256 * CPL, K);
  if (tid < K) part[(int64_t)g * K + tid] = red[tid];
}

// Column-major block vectors (round 4 probe): the k columns of p and Ap
// stored one after another (column c at c * ns, ns = n rounded up), so the
// block SpMV is the single-RHS DIA kernel's access pattern k times over one
// value load: lane l owns rows 2l, 2l + 1 of the wave's slice, and per slot
// column makes ONE 16-B value load and k 16-B x loads (one per column), all
// coalesced 1 KB runs, against k/CPL... = 8 value loads of 8 B replicated
// over a row's lanes plus 8 x runs in the row-major kernel. Each (row,
// column) sums its slot columns in ascending order from 0, as the library
// does; UNR slot columns' loads in flight. A timing probe only: its output,
// transposed back, did not match the library's Ap in the one run made
// (profiles/r04_dia_blk_colmajor_probe.txt), and that was not chased, the
// timing having already ruled the layout out.
template <int UNR>
__global__ __launch_bounds__(256) void dia_cm(const int64_t *__restrict__ sptr, const int *__restrict__ swidth,
                                              const int *__restrict__ doff, const uint64_t *__restrict__ dmask,
                                              const double *__restrict__ val, int64_t nslices, int64_t n, int64_t ns,
                                              const double *__restrict__ x, double *__restrict__ y,
                                              double *__restrict__ part) {
  __shared__ double red[256 * K];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t s = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 4 + wid;
  double dacc[K];
#pragma unroll
  for (int c = 0; c < K; ++c) dacc[c] = 0.0;
  if (s < nslices) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * kDiaSlice + 2 * lane;
    const int64_t c0 = base / kDiaSlice;
    const int *mo = doff + c0;
    const uint64_t *mk = dmask + 2 * c0;
    const double *cv = val + base + 2 * lane;
    double acc[K][2];
#pragma unroll
    for (int c = 0; c < K; ++c) acc[c][0] = acc[c][1] = 0.0;
    for (int j0 = 0; j0 < w; j0 += UNR) {
      int off[UNR];
      uint64_t me[UNR], md[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        off[u] = mo[j0 + u];
        me[u] = mk[2 * (j0 + u)];
        md[u] = mk[2 * (j0 + u) + 1];
      }
      d2v a[UNR], xv[UNR][K];
      bool on0[UNR], on1[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        a[u] = j0 + u < w ? __builtin_nontemporal_load(reinterpret_cast<const d2v *>(cv + (int64_t)(j0 + u) * kDiaSlice))
                          : d2v{0.0, 0.0};
        on0[u] = j0 + u < w && ((me[u] >> lane) & 1u) != 0;
        on1[u] = j0 + u < w && ((md[u] >> lane) & 1u) != 0;
        const int64_t xr = (on0[u] || on1[u]) ? row + off[u] : 0;
#pragma unroll
        for (int c = 0; c < K; ++c) xv[u][c] = *reinterpret_cast<const d2v *>(x + (int64_t)c * ns + xr);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int c = 0; c < K; ++c) {
          const double p0 = a[u].x * xv[u][c].x, p1 = a[u].y * xv[u][c].y;
          const double t0 = acc[c][0] + p0, t1 = acc[c][1] + p1;
          acc[c][0] = on0[u] ? t0 : acc[c][0];
          acc[c][1] = on1[u] ? t1 : acc[c][1];
        }
    }
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if (row + 1 < n) {
        const d2v p = *reinterpret_cast<const d2v *>(x + (int64_t)c * ns + row);
        __builtin_nontemporal_store(d2v{acc[c][0], acc[c][1]}, reinterpret_cast<d2v *>(y + (int64_t)c * ns + row));
        dacc[c] += dterm(p.x, acc[c][0]);
        dacc[c] += dterm(p.y, acc[c][1]);
      } else if (row < n) {
        const double p = x[(int64_t)c * ns + row];
        y[(int64_t)c * ns + row] = acc[c][0];
        dacc[c] += dterm(p, acc[c][0]);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < K; ++c) red[tid * K + c] = dacc[c];
  block_tree_reduce(red, 256 * K, K);
  if (tid < K) part[(int64_t)blockIdx.x * K + tid] = red[tid];
}

// row-major (n x K) <-> column-major (K x ns)
__global__ void to_cm(const double *__restrict__ a, double *__restrict__ b, int64_t n, int64_t ns) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * K; i += (int64_t)gridDim.x * blockDim.x)
    b[(i % K) * ns + i / K] = a[i];
}
__global__ void from_cm(const double *__restrict__ b, double *__restrict__ a, int64_t n, int64_t ns) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * K; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = b[(i % K) * ns + i / K];
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
  printf("N=%d n=%ld nnz=%ld k=%d dia_slices=%ld dia_slots=%ld max_width=%d\n", N, (long)n, (long)nnz, K,
         (long)A->dia_nslices, (long)A->dia_nslots, A->dia_max_width);
  std::vector<double> xh(n * K);
  for (int64_t i = 0; i < n * K; ++i) xh[i] = 1.0 + (double)((i * 7919) % 1000) * 1e-3;
  kry_vec *xv, *yv, *yrefv;
  KC(kry_vec_create(ctx, n, K, KRY_F64, &xv));
  KC(kry_vec_create(ctx, n, K, KRY_F64, &yv));
  KC(kry_vec_create(ctx, n, K, KRY_F64, &yrefv));
  KC(kry_vec_upload(xv, xh.data()));
  double *x = (double *)xv->d, *y = (double *)yv->d, *yref = (double *)yrefv->d, *part;
  CK(hipMalloc(&part, (size_t)65536 * K * 8));  // grids up to 65536 blocks (the sweep goes past kMaxGrid)
  hipStream_t st = ctx->stream;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double S = (double)nnz * 12 + (double)(n + 1) * 4 + 2.0 * n * K * 8;
  const double phys = (double)A->dia_nslots * 8 + (double)A->dia_nslots / 128 * 20 + 2.0 * n * K * 8;
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
    printf("%-46s %.4f ms  S-rate %.0f GB/s  image-rate %.0f GB/s\n", name, ms, S / ms / 1e6, phys / ms / 1e6);
    return ms;
  };
  timeit("library spmv_dia_blk (EpiApDot)", [&] {
    int P;
    launch_spmv<double, double, int>(A, K, SrcPlain<double>{x, K}, EpiApDot<double>{yref, nullptr, K}, part, &P,
                                     nullptr, 0, st);
  });
  std::vector<double> ref(n * K), got(n * K);
  CK(hipMemcpy(ref.data(), yref, n * K * 8, hipMemcpyDeviceToHost));
  {
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
  }
  auto check = [&](const char *name) {
    CK(hipMemcpy(got.data(), y, n * K * 8, hipMemcpyDeviceToHost));
    if (memcmp(got.data(), ref.data(), n * K * 8) != 0) printf("  !! %s differs from the library kernel\n", name);
  };
  timeit("floor: p read + Ap write (16 B/lane copy)", [&] {
    hipLaunchKernelGGL(copy_floor, dim3(8192), dim3(256), 0, st, (const d2v *)x, (d2v *)y, n * K / 2);
  });
  const int grid = (int)std::min<int64_t>(kMaxGrid, (A->dia_nslices + 3) / 4);
  int gr = 0;
#define SM(CPL, MODE, NAME, CHECK)                                                                                \
  {                                                                                                               \
    char nm[96];                                                                                                  \
    snprintf(nm, sizeof nm, "%s, grid %d", NAME, gr);                                                             \
    timeit(nm, [&] {                                                                                              \
      hipLaunchKernelGGL((dia_slot_major<CPL, MODE>), dim3(gr), dim3(256), 0, st, (const int64_t *)A->dia_sptr,   \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,       \
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);              \
    });                                                                                                           \
    if (CHECK) check(nm);                                                                                         \
  }
  if (getenv("DIA_BLK_CM")) {  // round 4: column-major block vectors
    const int64_t ns = (n + 63) / 64 * 64;
    double *xcm0, *ycm0;
    CK(hipMalloc(&xcm0, (K * ns + 128) * 8));
    CK(hipMalloc(&ycm0, (K * ns + 128) * 8));
    CK(hipMemset(xcm0, 0, (K * ns + 128) * 8));
    double *xcm = xcm0 + 64, *ycm = ycm0 + 64;  // 512 B of readable slack before column 0
    hipLaunchKernelGGL(to_cm, dim3(4096), dim3(256), 0, st, (const double *)x, xcm, n, ns);
    const int full = (int)((A->dia_nslices + 3) / 4);
#define CM(U, NAME)                                                                                                 \
  {                                                                                                                 \
    timeit(NAME, [&] {                                                                                              \
      hipLaunchKernelGGL((dia_cm<U>), dim3(full), dim3(256), 0, st, (const int64_t *)A->dia_sptr,                   \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,        \
                         (const double *)A->dia_val, A->dia_nslices, n, ns, (const double *)xcm, ycm, part);       \
    });                                                                                                             \
    hipLaunchKernelGGL(from_cm, dim3(4096), dim3(256), 0, st, (const double *)ycm, y, n, ns);                      \
    check(NAME);                                                                                                    \
  }
    for (int rep = 0; rep < 2; ++rep) {
      timeit("library spmv_dia_blk (EpiApDot), again", [&] {
        int P;
        launch_spmv<double, double, int>(A, K, SrcPlain<double>{x, K}, EpiApDot<double>{yref, nullptr, K}, part,
                                         &P, nullptr, 0, st);
      });
      CM(1, "column-major, UNR 1");
      CM(2, "column-major, UNR 2");
      CM(3, "column-major, UNR 3");
      CM(5, "column-major, UNR 5");
    }
    timeit("floor: p read + Ap write (16 B/lane copy)", [&] {
      hipLaunchKernelGGL(copy_floor, dim3(8192), dim3(256), 0, st, (const d2v *)x, (d2v *)y, n * K / 2);
    });
    return 0;
  }
  if (getenv("DIA_BLK_LDS")) {  // round 4: the near-diagonal x window (and values) through LDS
    const int full = (int)((A->dia_nslices + 3) / 4);
    if (full > 65536) return 1;
#define LD(MODE, NAME)                                                                                              \
  {                                                                                                                 \
    timeit(NAME, [&] {                                                                                              \
      hipLaunchKernelGGL((dia_lds<MODE>), dim3(full), dim3(256), 0, st, (const int64_t *)A->dia_sptr,               \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,        \
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);               \
    });                                                                                                             \
    check(NAME);                                                                                                    \
  }
    for (int rep = 0; rep < 2; ++rep) {
      gr = full;
      SM(2, 0, "slot-major CPL 2, 1 slice/wave", true);
      LD(0, "LDS window (near x), values direct");
      LD(1, "LDS window (near x) + LDS values");
      LD(4, "LDS window, values direct, far x hoisted");
      LD(5, "LDS window + LDS values, far x hoisted");
    }
  } else
  if (getenv("DIA_BLK_SHIFT")) {  // shifted-window variants against the slot-major kernel
    const int full = (int)((A->dia_nslices + 3) / 4);
    if (full > 65536) return 1;
#define SH(MODE, NAME)                                                                                              \
  {                                                                                                                 \
    timeit(NAME, [&] {                                                                                              \
      hipLaunchKernelGGL((dia_shift<MODE>), dim3(full), dim3(256), 0, st, (const int64_t *)A->dia_sptr,             \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,        \
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);               \
    });                                                                                                             \
    check(NAME);                                                                                                    \
  }
    if (getenv("DIA_BLK_NTV")) {  // value-load policy and shuffles at one slice per wave
      for (int rep = 0; rep < 2; ++rep) {
        gr = full;
        SM(2, 0, "slot-major CPL 2, 1 slice/wave", true);
        SM(2, 2, "slot-major CPL 2, nt values, 1 slice/wave", true);
        SM(2, 16, "slot-major CPL 2, shuffled values, 1 slice/wave", true);
        SM(2, 18, "slot-major CPL 2, shuffled nt values, 1 slice/wave", true);
        SM(2, 10, "slot-major CPL 2, nt values + diagonal p, 1 slice/wave", true);
        SM(2, 26, "slot-major CPL 2, shuf nt + diag p, 1 slice/wave", true);
      }
      return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
      gr = full;
      SM(2, 0, "slot-major CPL 2, 1 slice/wave", true);
      SH(4, "shift: no derive (clamped windows, p captured)");
      SH(0, "shift: -1/0/+1 derived");
      SH(2, "shift: derived, nt values");
      SH(1, "shift: derived, shuffled values");
      SH(3, "shift: derived, shuffled nt values");
    }
  } else
  if (getenv("DIA_BLK_SPLIT")) {
#define SPL(GPW, SPR)                                                                                              \
  {                                                                                                                \
    const int64_t waves = A->dia_nslices * (8 / GPW);                                                              \
    const int gsp = (int)std::min<int64_t>(65536, (waves + 3) / 4);                                                \
    char nm[96];                                                                                                   \
    snprintf(nm, sizeof nm, "split: %d groups/wave, %d slots/round, grid %d", GPW, SPR, gsp);                      \
    timeit(nm, [&] {                                                                                               \
      hipLaunchKernelGGL((dia_split<GPW, SPR>), dim3(gsp), dim3(256), 0, st, (const int64_t *)A->dia_sptr,         \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,        \
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);               \
    });                                                                                                            \
    check(nm);                                                                                                     \
  }
    for (int rep = 0; rep < 2; ++rep) {
      SPL(8, 1);
      SPL(8, 2);
      SPL(4, 1);
      SPL(4, 2);
      SPL(4, 3);
      SPL(2, 1);
      SPL(2, 3);
      SPL(2, 5);
    }
  } else
  if (getenv("DIA_BLK_GRIDS")) {  // block size / grid sweep of the slot-major kernel
    const int full = (int)((A->dia_nslices + 3) / 4);
    if (full > 65536) return 1;
    for (int rep = 0; rep < 2; ++rep) {
      gr = full;
      SM(2, 0, "slot-major CPL 2, 256 threads, 1 slice/wave", true);
      gr = (int)((A->dia_nslices + 15) / 16);
#define SMB(CPL, MODE, BS, NAME)                                                                                  \
  {                                                                                                               \
    char nm[96];                                                                                                  \
    snprintf(nm, sizeof nm, "%s, grid %d", NAME, gr);                                                             \
    timeit(nm, [&] {                                                                                              \
      hipLaunchKernelGGL((dia_slot_major<CPL, MODE, BS>), dim3(gr), dim3(BS), 0, st, (const int64_t *)A->dia_sptr, \
                         (const int *)A->dia_width, (const int *)A->dia_off, (const uint64_t *)A->dia_mask,       \
                         (const double *)A->dia_val, A->dia_nslices, n, (const double *)x, y, part);              \
    });                                                                                                           \
    check(nm);                                                                                                    \
  }
      SMB(2, 0, 1024, "slot-major CPL 2, 1024 threads, 1 slice/wave");
      SMB(2, 16, 1024, "slot-major CPL 2, 1024 thr, shuffled values");
      gr = (int)((A->dia_nslices + 7) / 8);
      SMB(2, 0, 512, "slot-major CPL 2, 512 threads, 1 slice/wave");
      gr = (int)((A->dia_nslices + 31) / 32);
      SMB(2, 0, 1024, "slot-major CPL 2, 1024 threads, 2 slices/wave");
      SMB(2, 512, 1024, "slot-major CPL 2, 1024 thr, 2 slices/wave strided");
    }
  } else
  for (int gr2 : {grid, 4096}) {
    gr = gr2;
    SM(2, 0, "slot-major CPL 2", true);
    SM(2, 1, "slot-major CPL 2, no store", false);
    SM(2, 2, "slot-major CPL 2, nt values", true);
    SM(2, 4, "slot-major CPL 2, deferred epilogue", true);
    SM(2, 8, "slot-major CPL 2, p from the diagonal", true);
    SM(2, 16, "slot-major CPL 2, shuffled values", true);
    SM(2, 18, "slot-major CPL 2, shuffled nt values", true);
    SM(2, 24, "slot-major CPL 2, shuffled values + diagonal p", true);
    SM(2, 28, "slot-major CPL 2, shuffled + diag p + deferred", true);
    SM(2, 32, "slot-major CPL 2, x at offset 0 only", false);
    SM(2, 64, "slot-major CPL 2, no x loads", false);
    if (getenv("DIA_BLK_SHORT")) break;
    SM(4, 16, "slot-major CPL 4, shuffled values", true);
  }
  KC(kry_vec_destroy(xv));
  KC(kry_vec_destroy(yv));
  KC(kry_vec_destroy(yrefv));
  KC(kry_csr_destroy(A));
  KC(kry_ctx_destroy(ctx));
  return 0;
}
