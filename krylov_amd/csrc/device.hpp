// gfx950 kernel templates: CSR SpMV (LDS-staged streaming form for one RHS,
// register form for row-major RHS blocks), fused elementwise passes with
// deterministic per-column dot partials, partial reducers, LAPACK lartg.
//
// Numerics contract (compiled with -ffp-contract=off):
//  * SpMV sums every row sequentially in stored nonzero order starting from 0,
//    one rounding per product and per add: bitwise SciPy csr_matvec(s).
//  * Elementwise updates evaluate exactly the NumPy expression tree of the
//    reference line they replace (e.g. `y + (alpha * p)`), no contraction.
//  * Inner products accumulate per-product doubles in a fixed order (per thread,
//    then a fixed LDS tree per block, then a fixed tree over block partials):
//    reproducible run to run, though not in OpenBLAS's summation order.
#pragma once

#include "common.hpp"
#include "objects.hpp"

namespace kry {

// ------------------------------------------------------------------ dot terms
__device__ __forceinline__ double dterm(double x, double y) { return x * y; }
__device__ __forceinline__ double dterm_w(double x, double w, double y) { return x * (w * y); }

// ------------------------------------------------------------- x sources
// The SpMV input x[j, c] may be materialised on the fly from other vectors
// (the p-update of CG, the normalisation of GMRES), so the gather never
// needs a separate pass over HBM. The owner row writes the same value out.
template <typename V>
struct SrcPlain {
  const V *x;
  int k;
  __device__ __forceinline__ V operator()(int64_t j, int c) const { return x[j * k + c]; }
};

// p = r + omega * p_old (cg.py:178); first iteration p = r (cg.py:138).
template <typename V>
struct SrcCgP {
  const V *r;
  const V *pold;
  const double *omega;
  int k;
  int first;
  __device__ __forceinline__ V operator()(int64_t j, int c) const {
    const V rj = r[j * k + c];
    if (first) return rj;
    const V om = (V)omega[c];
    const V t = om * pold[j * k + c];
    return rj + t;
  }
};

// -------------------------------------------------------------- epilogues
// store(row, c, sum) writes the SpMV result and returns this row/column's
// contribution to the fused inner product (0 if the epilogue has none).
template <typename V>
struct EpiStore {
  V *y;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s) const {
    y[i * k + c] = s;
    return 0.0;
  }
};

// y = A v and the first MGS inner product <q, y> (arnoldi.py:176,159).
template <typename V>
struct EpiStoreDot {
  V *y;
  const V *q;
  const double *w;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s) const {
    y[i * k + c] = s;
    const double qv = (double)q[i * k + c];
    return w ? dterm_w(qv, w[i], (double)s) : dterm(qv, (double)s);
  }
};

// r = b - A z and <r, r> (cg.py:86-90, gmres.py:106-108).
template <typename V>
struct EpiResidual {
  const V *b;
  V *r;
  const double *w;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s) const {
    const V ri = b[i * k + c] - s;
    r[i * k + c] = ri;
    const double rv = (double)ri;
    return w ? dterm_w(rv, w[i], rv) : dterm(rv, rv);
  }
};

// CG: Ap = A p, write p (materialised by SrcCgP), <p, Ap> (cg.py:178-183).
template <typename V>
struct EpiCgAp {
  V *Ap;
  V *pnew;
  SrcCgP<V> src;
  const double *w;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s) const {
    const V pi = src(i, c);
    pnew[i * k + c] = pi;
    Ap[i * k + c] = s;
    const double pv = (double)pi;
    return w ? dterm_w(pv, w[i], (double)s) : dterm(pv, (double)s);
  }
};

// MINRES Lanczos: w = A v - h0 * p_old (arnoldi.py:244-249) and <v, w>.
template <typename V>
struct EpiLanczos {
  V *out;
  const V *v;
  const V *pold;      // null on the first step
  const double *h0;   // stored in the Lanczos dtype
  const double *w;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s) const {
    V o = s;
    if (pold) {
      const V t = (V)h0[c] * pold[i * k + c];
      o = o - t;
    }
    out[i * k + c] = o;
    const double vv = (double)v[i * k + c];
    return w ? dterm_w(vv, w[i], (double)o) : dterm(vv, (double)o);
  }
};

// ---------------------------------------------------------- control word
__device__ __forceinline__ bool halted(const Ctrl *ctrl, int step) {
  return ctrl != nullptr && step >= ctrl->stop_at;
}

// ------------------------------------------------- streaming SpMV (k = 1)
// One persistent workgroup walks a contiguous run of row tiles (<= kTileNnz
// nonzeros, <= 256 rows). Phase 1: all 256 lanes stream the tile's
// (indices, data) with 16-byte loads and store data[e] * x[indices[e]] into
// LDS. Phase 2: lane r sums row r's products sequentially from LDS. HBM sees
// every matrix byte exactly once, coalesced; x gathers hit L2 (XCD-contiguous
// tiles). A row longer than a tile is streamed through LDS in chunks and
// summed by lane 0 (exact order kept).
template <typename V, typename MV, typename I, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_stream_kernel(
    const I *__restrict__ indptr, const I *__restrict__ indices, const MV *__restrict__ data,
    const I *__restrict__ tiles, int64_t ntiles, Src src, Epi epi, double *__restrict__ part,
    const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ V prod[kTileNnz];
  __shared__ double red[kBlock];
  const int tid = threadIdx.x;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t t_begin = ntiles * g / gridDim.x;
  const int64_t t_end = ntiles * (g + 1) / gridDim.x;
  double acc = 0.0;
  for (int64_t t = t_begin; t < t_end; ++t) {
    const int64_t r0 = tiles[t], r1 = tiles[t + 1];
    const int64_t e0 = indptr[r0], e1 = indptr[r1];
    if (e1 - e0 <= kTileNnz) {
      const int64_t eb = e0 & ~int64_t(3);
      for (int64_t e = eb + 4 * tid; e < e1; e += 4 * kBlock) {
        I col[4];
        V val[4];
        if constexpr (sizeof(I) == 4) {
          const int4 c4 = *reinterpret_cast<const int4 *>(indices + e);
          col[0] = c4.x; col[1] = c4.y; col[2] = c4.z; col[3] = c4.w;
        } else {
          const longlong2 a = *reinterpret_cast<const longlong2 *>(indices + e);
          const longlong2 b = *reinterpret_cast<const longlong2 *>(indices + e + 2);
          col[0] = a.x; col[1] = a.y; col[2] = b.x; col[3] = b.y;
        }
        if constexpr (sizeof(MV) == 8) {
          const double2 a = *reinterpret_cast<const double2 *>(data + e);
          const double2 b = *reinterpret_cast<const double2 *>(data + e + 2);
          val[0] = a.x; val[1] = a.y; val[2] = b.x; val[3] = b.y;
        } else {
          const float4 a = *reinterpret_cast<const float4 *>(data + e);
          val[0] = (V)a.x; val[1] = (V)a.y; val[2] = (V)a.z; val[3] = (V)a.w;
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int64_t ee = e + v;
          if (ee >= e0 && ee < e1) prod[ee - e0] = val[v] * src(col[v], 0);
        }
      }
      __syncthreads();
      const int nr = (int)(r1 - r0);
      if (tid < nr) {
        const int64_t row = r0 + tid;
        const int a = (int)(indptr[row] - e0), b = (int)(indptr[row + 1] - e0);
        V s = 0;
        for (int e = a; e < b; ++e) s = s + prod[e];
        acc += epi(row, 0, s);
      }
      __syncthreads();
    } else {
      // a single long row: chunked through LDS, sequential sum by lane 0
      V s = 0;
      for (int64_t cb = e0; cb < e1; cb += kTileNnz) {
        const int64_t ce = cb + kTileNnz < e1 ? cb + kTileNnz : e1;
        for (int64_t e = cb + tid; e < ce; e += kBlock) prod[e - cb] = (V)data[e] * src(indices[e], 0);
        __syncthreads();
        if (tid == 0)
          for (int e = 0; e < (int)(ce - cb); ++e) s = s + prod[e];
        __syncthreads();
      }
      if (tid == 0) acc += epi(r0, 0, s);
    }
  }
  if (part != nullptr) {
    red[tid] = acc;
    block_tree_reduce(red, kBlock, 1);
    if (tid == 0) part[g] = red[0];
  }
}

// ------------------------------------------- row-major block SpMV (k >= 2)
// Thread per (row, chunk of KT columns): y[i, c0:c0+KT] accumulated in
// registers in stored nonzero order (csr_matvecs semantics), the row's
// nonzeros loaded once per chunk, x rows (k contiguous values) gathered.
template <typename V, typename MV, typename I, int KT, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_rows_kernel(
    const I *__restrict__ indptr, const I *__restrict__ indices, const MV *__restrict__ data,
    int64_t n, int k, Src src, Epi epi, double *__restrict__ part, const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock * KT];
  const int tid = threadIdx.x;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int nch = k / KT;
  const int64_t total = n * nch;
  const int64_t per = ((total + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
  const int64_t q0 = per * g;
  const int64_t q1 = q0 + per < total ? q0 + per : total;
  double acc[KT];
#pragma unroll
  for (int c = 0; c < KT; ++c) acc[c] = 0.0;
  for (int64_t q = q0 + tid; q < q1; q += kBlock) {
    const int64_t row = q / nch;
    const int c0 = (int)(q % nch) * KT;
    V s[KT];
#pragma unroll
    for (int c = 0; c < KT; ++c) s[c] = 0;
    const int64_t eb = indptr[row], ee = indptr[row + 1];
    for (int64_t e = eb; e < ee; ++e) {
      const int64_t j = indices[e];
      const V a = (V)data[e];
#pragma unroll
      for (int c = 0; c < KT; ++c) {
        const V t = a * src(j, c0 + c);
        s[c] = s[c] + t;
      }
    }
#pragma unroll
    for (int c = 0; c < KT; ++c) acc[c] += epi(row, c0 + c, s[c]);
  }
  if (part != nullptr) {
#pragma unroll
    for (int c = 0; c < KT; ++c) red[tid * KT + c] = acc[c];
    block_tree_reduce(red, kBlock * KT, k);
    if (tid < k) part[(int64_t)g * k + tid] = red[tid];
  }
}

// ---------------------------------------------------- elementwise passes
// Op(e, N, acc) handles the W = 16/sizeof(V) consecutive elements at flat
// index e (a multiple of W) and adds its dot terms to acc[0..W). Each block
// owns a contiguous span of W*256-element groups, so slot p = tid*W + v maps
// to column p % k (k a power of two <= 256).
template <typename V, class Op>
__global__ __launch_bounds__(kBlock) void elementwise_kernel(int64_t N, int k, Op op,
                                                             double *__restrict__ part,
                                                             const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  __shared__ double red[kBlock * W];
  const int tid = threadIdx.x;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t ngrp = (N + W - 1) / W;
  const int64_t per = ((ngrp + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
  const int64_t v0 = per * g;
  const int64_t v1 = v0 + per < ngrp ? v0 + per : ngrp;
  double acc[W];
#pragma unroll
  for (int v = 0; v < W; ++v) acc[v] = 0.0;
  for (int64_t v = v0 + tid; v < v1; v += kBlock) op(v * W, N, acc);
  if (part != nullptr) {
#pragma unroll
    for (int v = 0; v < W; ++v) red[tid * W + v] = acc[v];
    block_tree_reduce(red, kBlock * W, k);
    if (tid < k) part[(int64_t)g * k + tid] = red[tid];
  }
}

// W-wide load/store of V with a scalar tail.
template <typename V>
struct VIO {
  static constexpr int W = Vec16<V>::W;
  __device__ __forceinline__ static void load(const V *p, int64_t e, int64_t N, V (&o)[W]) {
    if (e + W <= N) {
      if constexpr (W == 2) {
        const double2 t = *reinterpret_cast<const double2 *>(p + e);
        o[0] = t.x; o[1] = t.y;
      } else {
        const float4 t = *reinterpret_cast<const float4 *>(p + e);
        o[0] = t.x; o[1] = t.y; o[2] = t.z; o[3] = t.w;
      }
    } else {
#pragma unroll
      for (int v = 0; v < W; ++v) o[v] = e + v < N ? p[e + v] : V(0);
    }
  }
  __device__ __forceinline__ static void store(V *p, int64_t e, int64_t N, const V (&o)[W]) {
    if (e + W <= N) {
      if constexpr (W == 2) {
        *reinterpret_cast<double2 *>(p + e) = make_double2(o[0], o[1]);
      } else {
        *reinterpret_cast<float4 *>(p + e) = make_float4(o[0], o[1], o[2], o[3]);
      }
    } else {
#pragma unroll
      for (int v = 0; v < W; ++v)
        if (e + v < N) p[e + v] = o[v];
    }
  }
};

// ------------------------------------------------------- partial reducers
// Sum part[p * k + c] over p < P for every column c < k into red[c]
// (fixed order; all of one block). Must be called by every thread.
__device__ __forceinline__ void reduce_partials(const double *part, int P, int k, double *red) {
  const int tid = threadIdx.x;
  const int c = tid & (k - 1);
  const int step = kBlock / k;
  double s = 0.0;
  for (int p = tid / k; p < P; p += step) s += part[(int64_t)p * k + c];
  red[tid] = s;
  block_tree_reduce(red, kBlock, k);
}

// one-block finalize: out[c] = sum over the partials of column c
template <int D = 0>
__global__ void reduce_to_kernel(const double *part, int P, int k, double *out) {
  __shared__ double red[kBlock];
  reduce_partials(part, P, k, red);
  if (threadIdx.x < k) out[threadIdx.x] = red[threadIdx.x];
}

// ------------------------------------------------------------ lartg
// LAPACK >= 3.10 xLARTG (la_xlartg.f90) restated; bitwise scipy ?lartg.
template <typename T>
struct LartgConst;
template <>
struct LartgConst<double> {
  static constexpr double safmin = 2.2250738585072014e-308;
};
template <>
struct LartgConst<float> {
  static constexpr float safmin = 1.17549435e-38f;
};

template <typename T>
__device__ __forceinline__ void lartg(T f, T g, T &c, T &s, T &r) {
  const T safmin = LartgConst<T>::safmin;
  const T safmax = T(1) / safmin;
  const T rtmin = sqrt(safmin);
  const T rtmax = sqrt(safmax / T(2));
  const T f1 = fabs(f), g1 = fabs(g);
  if (g == T(0)) {
    c = T(1); s = T(0); r = f;
  } else if (f == T(0)) {
    c = T(0); s = g > T(0) ? T(1) : T(-1); r = g1;
  } else if (f1 > rtmin && f1 < rtmax && g1 > rtmin && g1 < rtmax) {
    const T ff = f * f, gg = g * g;
    const T d = sqrt(ff + gg);
    c = f1 / d;
    r = f >= T(0) ? d : -d;
    s = g / r;
  } else {
    T m = f1 > g1 ? f1 : g1;
    if (m < safmin) m = safmin;
    const T u = m < safmax ? m : safmax;
    const T fs = f / u, gs = g / u;
    const T ff = fs * fs, gg = gs * gs;
    const T d = sqrt(ff + gg);
    c = fabs(fs) / d;
    const T rr = f >= T(0) ? d : -d;
    s = gs / rr;
    r = rr * u;
  }
}

// -------------------------------------------------------- host launchers
template <typename V, typename MV, typename I, class Src, class Epi>
void launch_spmv(const kry_csr *A, int k, Src src, Epi epi, double *part, int *grid_out,
                 const Ctrl *ctrl, int step, hipStream_t st) {
  const I *ip = static_cast<const I *>(A->indptr);
  const I *ix = static_cast<const I *>(A->indices);
  const MV *dv = static_cast<const MV *>(A->data);
  int grid;
  if (k == 1) {
    grid = (int)(A->ntiles < kMaxGrid ? A->ntiles : kMaxGrid);
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((spmv_stream_kernel<V, MV, I, Src, Epi>), dim3(grid), dim3(kBlock), 0, st, ip, ix,
                       dv, static_cast<const I *>(A->tiles), A->ntiles, src, epi, part, ctrl, step);
  } else {
    const int KT = k >= 8 ? 8 : k;
    const int64_t total = A->n * (k / KT);
    grid = grid_for(total, kBlock * 2);
    switch (KT) {
      case 2:
        hipLaunchKernelGGL((spmv_rows_kernel<V, MV, I, 2, Src, Epi>), dim3(grid), dim3(kBlock), 0, st, ip,
                           ix, dv, A->n, k, src, epi, part, ctrl, step);
        break;
      case 4:
        hipLaunchKernelGGL((spmv_rows_kernel<V, MV, I, 4, Src, Epi>), dim3(grid), dim3(kBlock), 0, st, ip,
                           ix, dv, A->n, k, src, epi, part, ctrl, step);
        break;
      default:
        hipLaunchKernelGGL((spmv_rows_kernel<V, MV, I, 8, Src, Epi>), dim3(grid), dim3(kBlock), 0, st, ip,
                           ix, dv, A->n, k, src, epi, part, ctrl, step);
        break;
    }
  }
  KRY_HIP(hipGetLastError());
  if (grid_out) *grid_out = grid;
}

template <typename V, class Op>
int launch_elementwise(int64_t N, int k, Op op, double *part, const Ctrl *ctrl, int step,
                       hipStream_t st) {
  constexpr int W = Vec16<V>::W;
  const int grid = grid_for((N + W - 1) / W, kBlock * 2);
  hipLaunchKernelGGL((elementwise_kernel<V, Op>), dim3(grid), dim3(kBlock), 0, st, N, k, op, part,
                     ctrl, step);
  KRY_HIP(hipGetLastError());
  return grid;
}

// Dispatch on (vector value, matrix value, index) type. A float32 matrix may
// drive float64 vectors (SciPy upcasts the data: (double)a * x is exact).
template <class F>
void dispatch_vmi(int vtype, int mtype, int itype, F &&f) {
  auto with_i = [&](auto v0, auto m0) {
    if (itype == KRY_I32) f(v0, m0, (int32_t)0);
    else if (itype == KRY_I64) f(v0, m0, (int64_t)0);
    else throw Error{KRY_EINVAL, "unsupported index type"};
  };
  if (vtype == KRY_F64 && mtype == KRY_F64) with_i((double)0, (double)0);
  else if (vtype == KRY_F64 && mtype == KRY_F32) with_i((double)0, (float)0);
  else if (vtype == KRY_F32 && mtype == KRY_F32) with_i((float)0, (float)0);
  else throw Error{KRY_EINVAL, "unsupported vector/matrix dtype combination"};
}

}  // namespace kry
