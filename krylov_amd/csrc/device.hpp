// gfx950 kernel templates: SpMV over the SELL-64 image (lane per row for one
// or two RHS, lane groups for 4..64 row-major RHS, int32 or compact uint16
// column deltas) and over the column-blocked image (scattered sparsity, one
// RHS), fused elementwise passes with deterministic per-column dot partials,
// partial reducers, LAPACK lartg.
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

#include <type_traits>

#include "common.hpp"
#include "objects.hpp"

namespace kry {

// ------------------------------------------------------------------ dot terms
__device__ __forceinline__ double dterm(double x, double y) { return x * y; }
__device__ __forceinline__ double dterm_w(double x, double w, double y) { return x * (w * y); }

// ------------------------------------------------------------- x sources
// C consecutive values starting at p (16-B aligned: p's element offset is a
// multiple of C, C in {2, 4}, and allocations are 256-B aligned) as 16-B
// vector loads.
template <typename V, int C>
__device__ __forceinline__ void vload_row(const V *p, V (&o)[C]) {
  if constexpr (sizeof(V) == 8) {
    typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int q = 0; q < C / 2; ++q) {
      const d2 t = reinterpret_cast<const d2 *>(p)[q];
      o[2 * q] = t.x;
      o[2 * q + 1] = t.y;
    }
  } else {
    typedef float fC __attribute__((ext_vector_type(C)));
    const fC t = *reinterpret_cast<const fC *>(p);
#pragma unroll
    for (int q = 0; q < C; ++q) o[q] = t[q];
  }
}
template <typename V, int C, bool NT = false>
__device__ __forceinline__ void vstore_row(V *p, const V (&o)[C]) {
  if constexpr (sizeof(V) == 8) {
    typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int q = 0; q < C / 2; ++q) {
      const d2 t = d2{o[2 * q], o[2 * q + 1]};
      if (NT) __builtin_nontemporal_store(t, reinterpret_cast<d2 *>(p) + q);
      else reinterpret_cast<d2 *>(p)[q] = t;
    }
  } else {
    typedef float fC __attribute__((ext_vector_type(C)));
    fC t;
#pragma unroll
    for (int q = 0; q < C; ++q) t[q] = o[q];
    if (NT) __builtin_nontemporal_store(t, reinterpret_cast<fC *>(p));
    else *reinterpret_cast<fC *>(p) = t;
  }
}

// Two consecutive values at p, aligned to the element only (the
// diagonal-offset SpMV's x pairs start at row + offset): one 16-byte access
// for double, 8-byte for float.
template <typename V>
struct PairT;
template <>
struct PairT<double> {
  typedef double T __attribute__((ext_vector_type(2), aligned(8)));
};
template <>
struct PairT<float> {
  typedef float T __attribute__((ext_vector_type(2), aligned(4)));
};
template <typename V>
__device__ __forceinline__ void pload(const V *p, V (&o)[2]) {
  const typename PairT<V>::T t = *reinterpret_cast<const typename PairT<V>::T *>(p);
  o[0] = t.x;
  o[1] = t.y;
}
template <typename V>
__device__ __forceinline__ void pload_nt(const V *p, V (&o)[2]) {
  const typename PairT<V>::T t = __builtin_nontemporal_load(reinterpret_cast<const typename PairT<V>::T *>(p));
  o[0] = t.x;
  o[1] = t.y;
}
template <typename V, bool NT = false>
__device__ __forceinline__ void pstore(V *p, const V (&o)[2]) {
  const typename PairT<V>::T t = {o[0], o[1]};
  if (NT) __builtin_nontemporal_store(t, reinterpret_cast<typename PairT<V>::T *>(p));
  else *reinterpret_cast<typename PairT<V>::T *>(p) = t;
}
// dot terms of two consecutive rows i, i + 1 (one column), summed in order
__device__ __forceinline__ double dterm2(const double *w, int64_t i, double x0, double y0, double x1, double y1) {
  if (w) return dterm_w(x0, w[i], y0) + dterm_w(x1, w[i + 1], y1);
  return dterm(x0, y0) + dterm(x1, y1);
}

// The SpMV input x[j, c] may be materialised on the fly from other vectors
// (the p-update of CG, the normalisation of GMRES), so the gather never
// needs a separate pass over HBM. The owner row writes the same value out.
// operator()(j, c) reads global column c; bind<KT>(c0) returns a copy for the
// SpMV inner loop that serves local columns c0 + [0, KT) with any per-column
// scalars held in registers.
template <typename V>
struct SrcPlain {
  const V *x;
  int k;
  __device__ __forceinline__ V operator()(int64_t j, int c) const { return x[j * k + c]; }
  template <int KT>
  struct Bound {
    const V *x;
    int k, c0;
    __device__ __forceinline__ V operator()(int64_t j, int c) const { return x[j * k + c0 + c]; }
    // the KT values of row j (lane-group kernel, KT in {2, 4})
    __device__ __forceinline__ void row(int64_t j, V (&o)[KT]) const { vload_row<V, KT>(x + j * k + c0, o); }
    // rows j and j + 1 of a single column (k = 1, diagonal-offset kernel)
    __device__ __forceinline__ void pair(int64_t j, V (&o)[2]) const { pload<V>(x + j, o); }
  };
  template <int KT>
  __device__ __forceinline__ Bound<KT> bind(int c0) const {
    return Bound<KT>{x, k, c0};
  }
};

// x = w / hsafe (GMRES: the next basis vector V_{k+1} = w / guard(h[k+1]),
// arnoldi.py:191-196, formed on the fly at every gather of the next SpMV).
template <typename V>
struct SrcScaled {
  const V *w;
  const double *hs;
  int k;
  __device__ __forceinline__ V operator()(int64_t j, int c) const { return w[j * k + c] / (V)hs[c]; }
  template <int KT>
  struct Bound {
    const V *w;
    V h[KT];
    int k, c0;
    __device__ __forceinline__ V operator()(int64_t j, int c) const { return w[j * k + c0 + c] / h[c]; }
    __device__ __forceinline__ void pair(int64_t j, V (&o)[2]) const {
      pload<V>(w + j, o);
      o[0] = o[0] / h[0];
      o[1] = o[1] / h[0];
    }
    __device__ __forceinline__ void row(int64_t j, V (&o)[KT]) const {
      vload_row<V, KT>(w + j * k + c0, o);
#pragma unroll
      for (int c = 0; c < KT; ++c) o[c] = o[c] / h[c];
    }
  };
  template <int KT>
  __device__ __forceinline__ Bound<KT> bind(int c0) const {
    Bound<KT> b;
    b.w = w;
    b.k = k;
    b.c0 = c0;
#pragma unroll
    for (int c = 0; c < KT; ++c) b.h[c] = (V)hs[c0 + c];
    return b;
  }
};

// -------------------------------------------------------------- epilogues
// store(row, c, sum) writes the SpMV result and returns this row/column's
// contribution to the fused inner product (0 if the epilogue has none).
template <typename V>
struct EpiStore {
  V *y;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s, V xi) const {
    y[i * k + c] = s;
    return 0.0;
  }
  // C consecutive columns c0.. of row i at once (lane-group kernel): 16-B
  // stores, dot contributions added to d[]
  template <int C>
  __device__ __forceinline__ void row(int64_t i, int c0, const V (&s)[C], const V (&xi)[C], double (&d)[C]) const {
    vstore_row<V, C>(y + i * k + c0, s);
  }
  // rows i and i + 1 of a single column (k = 1, diagonal-offset kernel)
  __device__ __forceinline__ double rows2(int64_t i, const V (&s)[2], const V (&xi)[2]) const {
    pstore<V>(y + i, s);
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
  __device__ __forceinline__ double operator()(int64_t i, int c, V s, V xi) const {
    y[i * k + c] = s;
    const double qv = (double)q[i * k + c];
    return w ? dterm_w(qv, w[i], (double)s) : dterm(qv, (double)s);
  }
  template <int C>
  __device__ __forceinline__ void row(int64_t i, int c0, const V (&s)[C], const V (&xi)[C], double (&d)[C]) const {
    vstore_row<V, C>(y + i * k + c0, s);
    V qv[C];
    vload_row<V, C>(q + i * k + c0, qv);
#pragma unroll
    for (int c = 0; c < C; ++c) d[c] += w ? dterm_w((double)qv[c], w[i], (double)s[c]) : dterm((double)qv[c], (double)s[c]);
  }
  __device__ __forceinline__ double rows2(int64_t i, const V (&s)[2], const V (&xi)[2]) const {
    pstore<V>(y + i, s);
    V qv[2];
    pload<V>(q + i, qv);
    return dterm2(w, i, (double)qv[0], (double)s[0], (double)qv[1], (double)s[1]);
  }
};

// y = A x and <y, y> (weighted): a preconditioned residual M_l r and its norm.
template <typename V>
struct EpiStoreNorm {
  V *y;
  const double *w;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s, V xi) const {
    y[i * k + c] = s;
    const double sv = (double)s;
    return w ? dterm_w(sv, w[i], sv) : dterm(sv, sv);
  }
  template <int C>
  __device__ __forceinline__ void row(int64_t i, int c0, const V (&s)[C], const V (&xi)[C], double (&d)[C]) const {
    vstore_row<V, C>(y + i * k + c0, s);
#pragma unroll
    for (int c = 0; c < C; ++c) d[c] += w ? dterm_w((double)s[c], w[i], (double)s[c]) : dterm((double)s[c], (double)s[c]);
  }
  __device__ __forceinline__ double rows2(int64_t i, const V (&s)[2], const V (&xi)[2]) const {
    pstore<V>(y + i, s);
    return dterm2(w, i, (double)s[0], (double)s[0], (double)s[1], (double)s[1]);
  }
};

// out = x0 + A y (gmres.py:97-99 / minres.py: x0 + Mr @ yk).
template <typename V>
struct EpiAddStore {
  V *out;
  const V *x0;  // may be null (x0 = 0)
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s, V xi) const {
    out[i * k + c] = x0 ? x0[i * k + c] + s : s;
    return 0.0;
  }
  template <int C>
  __device__ __forceinline__ void row(int64_t i, int c0, const V (&s)[C], const V (&xi)[C], double (&d)[C]) const {
    V o[C];
    if (x0) {
      vload_row<V, C>(x0 + i * k + c0, o);
#pragma unroll
      for (int c = 0; c < C; ++c) o[c] = o[c] + s[c];
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) o[c] = s[c];
    }
    vstore_row<V, C>(out + i * k + c0, o);
  }
  __device__ __forceinline__ double rows2(int64_t i, const V (&s)[2], const V (&xi)[2]) const {
    V o[2] = {s[0], s[1]};
    if (x0) {
      pload<V>(x0 + i, o);
      o[0] = o[0] + s[0];
      o[1] = o[1] + s[1];
    }
    pstore<V>(out + i, o);
    return 0.0;
  }
};

// EpiStoreDot that also stores the row's source value: with SrcScaled the
// SpMV materialises V_{k+1} = w / guard(h[k+1]) while it multiplies by it.
template <typename V>
struct EpiStoreDotV {
  V *y;
  const V *q;
  V *vout;
  const double *w;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s, V xi) const {
    vout[i * k + c] = xi;
    y[i * k + c] = s;
    const double qv = (double)q[i * k + c];
    return w ? dterm_w(qv, w[i], (double)s) : dterm(qv, (double)s);
  }
  template <int C>
  __device__ __forceinline__ void row(int64_t i, int c0, const V (&s)[C], const V (&xi)[C], double (&d)[C]) const {
    vstore_row<V, C>(vout + i * k + c0, xi);
    vstore_row<V, C>(y + i * k + c0, s);
    V qv[C];
    vload_row<V, C>(q + i * k + c0, qv);
#pragma unroll
    for (int c = 0; c < C; ++c) d[c] += w ? dterm_w((double)qv[c], w[i], (double)s[c]) : dterm((double)qv[c], (double)s[c]);
  }
  __device__ __forceinline__ double rows2(int64_t i, const V (&s)[2], const V (&xi)[2]) const {
    pstore<V>(vout + i, xi);
    pstore<V>(y + i, s);
    V qv[2];
    pload<V>(q + i, qv);
    return dterm2(w, i, (double)qv[0], (double)s[0], (double)qv[1], (double)s[1]);
  }
};

// r = b - A z and <r, r> (cg.py:86-90, gmres.py:106-108).
template <typename V>
struct EpiResidual {
  const V *b;
  V *r;
  const double *w;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s, V xi) const {
    const V ri = b[i * k + c] - s;
    r[i * k + c] = ri;
    const double rv = (double)ri;
    return w ? dterm_w(rv, w[i], rv) : dterm(rv, rv);
  }
  template <int C>
  __device__ __forceinline__ void row(int64_t i, int c0, const V (&s)[C], const V (&xi)[C], double (&d)[C]) const {
    V ri[C];
    vload_row<V, C>(b + i * k + c0, ri);
#pragma unroll
    for (int c = 0; c < C; ++c) ri[c] = ri[c] - s[c];
    vstore_row<V, C>(r + i * k + c0, ri);
#pragma unroll
    for (int c = 0; c < C; ++c) d[c] += w ? dterm_w((double)ri[c], w[i], (double)ri[c]) : dterm((double)ri[c], (double)ri[c]);
  }
  __device__ __forceinline__ double rows2(int64_t i, const V (&s)[2], const V (&xi)[2]) const {
    V ri[2];
    pload<V>(b + i, ri);
    ri[0] = ri[0] - s[0];
    ri[1] = ri[1] - s[1];
    pstore<V>(r + i, ri);
    return dterm2(w, i, (double)ri[0], (double)ri[0], (double)ri[1], (double)ri[1]);
  }
};

// CG: Ap = A p (nontemporal: read once, by the update pass) and <p, Ap>
// (cg.py:178-183); xi is p_i, read by the bound source at row i.
template <typename V>
struct EpiApDot {
  V *Ap;
  const double *w;
  int k;
  __device__ __forceinline__ double operator()(int64_t i, int c, V s, V xi) const {
    __builtin_nontemporal_store(s, Ap + i * k + c);
    const double pv = (double)xi;
    return w ? dterm_w(pv, w[i], (double)s) : dterm(pv, (double)s);
  }
  template <int C>
  __device__ __forceinline__ void row(int64_t i, int c0, const V (&s)[C], const V (&xi)[C], double (&d)[C]) const {
    vstore_row<V, C, true>(Ap + i * k + c0, s);
#pragma unroll
    for (int c = 0; c < C; ++c) d[c] += w ? dterm_w((double)xi[c], w[i], (double)s[c]) : dterm((double)xi[c], (double)s[c]);
  }
  __device__ __forceinline__ double rows2(int64_t i, const V (&s)[2], const V (&xi)[2]) const {
    pstore<V, true>(Ap + i, s);
    return dterm2(w, i, (double)xi[0], (double)s[0], (double)xi[1], (double)s[1]);
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
  __device__ __forceinline__ double operator()(int64_t i, int c, V s, V xi) const {
    V o = s;
    if (pold) {
      const V t = (V)h0[c] * pold[i * k + c];
      o = o - t;
    }
    out[i * k + c] = o;
    const double vv = (double)v[i * k + c];
    return w ? dterm_w(vv, w[i], (double)o) : dterm(vv, (double)o);
  }
  template <int C>
  __device__ __forceinline__ void row(int64_t i, int c0, const V (&s)[C], const V (&xi)[C], double (&d)[C]) const {
    V o[C];
#pragma unroll
    for (int c = 0; c < C; ++c) o[c] = s[c];
    if (pold) {
      V po[C];
      vload_row<V, C>(pold + i * k + c0, po);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const V t = (V)h0[c0 + c] * po[c];
        o[c] = o[c] - t;
      }
    }
    vstore_row<V, C>(out + i * k + c0, o);
    V vv[C];
    vload_row<V, C>(v + i * k + c0, vv);
#pragma unroll
    for (int c = 0; c < C; ++c) d[c] += w ? dterm_w((double)vv[c], w[i], (double)o[c]) : dterm((double)vv[c], (double)o[c]);
  }
  __device__ __forceinline__ double rows2(int64_t i, const V (&s)[2], const V (&xi)[2]) const {
    V o[2] = {s[0], s[1]};
    if (pold) {
      V po[2];
      pload<V>(pold + i, po);
      const V h = (V)h0[0];
      const V t0 = h * po[0];
      const V t1 = h * po[1];
      o[0] = o[0] - t0;
      o[1] = o[1] - t1;
    }
    pstore<V>(out + i, o);
    V vv[2];
    pload<V>(v + i, vv);
    return dterm2(w, i, (double)vv[0], (double)o[0], (double)vv[1], (double)o[1]);
  }
};

// ---------------------------------------------------------- control word
__device__ __forceinline__ bool halted(const Ctrl *ctrl, int step) {
  return ctrl != nullptr && step >= ctrl->stop_at;
}

// ------------------------------------------------------ SELL-64 SpMV
// The operator is stored once, at upload, as SELL-64: rows in slices of 64
// (one wavefront), each slice column-major with width = its longest row and
// padding marked by column index -1. Lane r of a wave owns row r of the slice
// and sums it sequentially over the slice columns, so:
//  * every value / index load is one contiguous 64-lane access (HBM streamed
//    once, no LDS staging, no barriers);
//  * for stencil-like matrices lane r's gather x[col] sits next to lane r+1's
//    (a few cache lines per wave-instruction, served from the XCD's L2);
//  * the per-row summation order is the stored CSR order: bitwise
//    csr_matvec / csr_matvecs.
// Slices whose padding would exceed ~2x their nonzeros (very uneven rows) are
// flagged irregular (width -1) and walked in CSR form by the same lanes.
// k > 1 right-hand sides: each lane keeps KT column accumulators; for k > 8
// the waves split into k/8 column groups.
template <typename V, typename MV, typename I, int KT, int UNR, bool D16, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_sell_kernel(
    const int64_t *__restrict__ sptr, const int *__restrict__ swidth, const I *__restrict__ sidx,
    const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase,
    const MV *__restrict__ sval, int64_t nslices, int64_t n, int k, const I *__restrict__ indptr,
    const I *__restrict__ indices, const MV *__restrict__ data, Src src, Epi epi, double *__restrict__ part,
    const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock * KT];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int nch = k / KT;                        // column groups (1 unless k > 8)
  const int64_t W = (int64_t)gridDim.x * 4 / nch;  // waves per column group
  const int64_t wg = (int64_t)g * 4 + wid;
  const int ch = (int)(wg % nch);
  const int64_t m = wg / nch;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  const int c0 = ch * KT;
  const auto bs = src.template bind<KT>(c0);
  double dacc[KT];
#pragma unroll
  for (int c = 0; c < KT; ++c) dacc[c] = 0.0;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t row = s * 64 + lane;
    V acc[KT];
#pragma unroll
    for (int c = 0; c < KT; ++c) acc[c] = V(0);
    if (w >= 0) {
      const int64_t base = sptr[s];
      const I *ci = sidx + base + lane;
      const uint16_t *cd = sdelta + base + lane;
      const int *cb = scbase + (base >> 6);  // slot-column bases: wave-uniform (scalar loads)
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
        V xv[UNR][KT];
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
          for (int c = 0; c < KT; ++c) xv[u][c] = col[u] >= 0 ? bs(col[u], c) : V(0);
#pragma unroll
        for (int u = 0; u < UNR; ++u)
          if (col[u] >= 0) {
#pragma unroll
            for (int c = 0; c < KT; ++c) {
              const V p = a[u] * xv[u][c];
              acc[c] = acc[c] + p;
            }
          }
      }
    } else if (row < n) {
      for (I e = indptr[row]; e < indptr[row + 1]; ++e) {
        const I j = indices[e];
        const V a = (V)data[e];
#pragma unroll
        for (int c = 0; c < KT; ++c) {
          const V p = a * bs(j, c);
          acc[c] = acc[c] + p;
        }
      }
    }
    if (row < n) {
#pragma unroll
      for (int c = 0; c < KT; ++c) dacc[c] += epi(row, c0 + c, acc[c], bs(row, c));
    }
  }
  if (part != nullptr) {
#pragma unroll
    for (int c = 0; c < KT; ++c) red[tid * KT + c] = dacc[c];
    if (nch == 1) {
      block_tree_reduce(red, kBlock * KT, k);
      if (tid < k) part[(int64_t)g * k + tid] = red[tid];
    } else {
      // column group of wave w in this block: (g*4 + w) % nch; fixed order
      __syncthreads();
      double sum = 0.0;
      if (tid < k) {
        const int cg = tid / KT, cc = tid % KT;
        for (int t = 0; t < kBlock; ++t)
          if ((int)(((int64_t)g * 4 + (t >> 6)) % nch) == cg) sum += red[t * KT + cc];
      }
      __syncthreads();
      if (tid < k) part[(int64_t)g * k + tid] = sum;
    }
  }
}


// -------------------------------------------- diagonal-offset SpMV (k = 1)
// The SELL-128/DIA image (kry_csr::dia_*): lane l of the wave owns rows
// 128 s + 2l and 128 s + 2l + 1 of slice s; slot column j of the slice holds,
// for every row whose mask bit is set, the entry at column row + off_j. The
// slot column's offset and its two lane masks are wave-uniform (scalar
// loads); per slot column a lane makes one 16-byte value load, one 16-byte x
// load (x[row + off_j], x[row + 1 + off_j]: the wave reads the contiguous run
// x[128 s + off_j, 128 s + off_j + 128)) and, at the end of the slice, one
// 16-byte store: no index stream, and half the memory instructions of one
// row per lane. A hole's x entry is loaded with its partner (at worst one
// element past either end of x, inside the allocation slack) and its product
// is dropped by a select, never added: an inf or NaN there cannot leak in.
// The offsets of a slice ascend and every row is sorted, so each row is still
// summed from 0 in stored order, one rounding per product and per add:
// bitwise csr_matvec.
template <typename V, typename MV, int UNR, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_dia_kernel(const int64_t *__restrict__ sptr,
                                                          const int *__restrict__ swidth,
                                                          const int *__restrict__ doff,
                                                          const uint64_t *__restrict__ dmask,
                                                          const MV *__restrict__ val, int64_t nslices, int64_t n,
                                                          Src src, Epi epi, double *__restrict__ part,
                                                          const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  const auto bs = src.template bind<1>(0);
  double dacc = 0.0;
  // The epilogue (result store, dot term) of slice s - 1 runs after slice s's
  // first round of loads is issued: on gfx9's in-order vmcnt a wait on those
  // loads then never waits for the store's acknowledgement
  // (tools/dia_bench "deferred store": -3.5 % on the metric SpMV).
  V pend[2] = {V(0), V(0)};
  int64_t prow = -1;
  auto flush = [&]() {
    if (prow + 1 < n) {
      V xi[2];
      bs.pair(prow, xi);
      dacc += epi.rows2(prow, pend, xi);
    } else if (prow < n) {
      dacc += epi(prow, 0, pend[0], bs(prow, 0));
    }
  };
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * kDiaSlice + 2 * lane;
    const int64_t c0 = base / kDiaSlice;
    const int *mo = doff + c0;  // wave-uniform: scalar loads
    const uint64_t *mk = dmask + 2 * c0;
    const MV *cv = val + base + 2 * lane;
    V acc0 = V(0), acc1 = V(0);
    for (int j0 = 0; j0 < w; j0 += UNR) {
      // descriptors: read unconditionally (the arrays are padded by kDiaPad
      // columns), all scalar loads in flight before the first use; values:
      // behind the wave-uniform `j0 + u < w` (a scalar branch, no wait)
      int off[UNR];
      uint64_t me[UNR], md[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        off[u] = mo[j0 + u];
        me[u] = mk[2 * (j0 + u)];
        md[u] = mk[2 * (j0 + u) + 1];
      }
      MV a[UNR][2];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (j0 + u < w) {
          pload_nt<MV>(cv + (int64_t)(j0 + u) * kDiaSlice, a[u]);
        } else {
          a[u][0] = MV(0);
          a[u][1] = MV(0);
        }
      }
      bool on0[UNR], on1[UNR];
      V xv[UNR][2];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        on0[u] = j0 + u < w && ((me[u] >> lane) & 1u) != 0;
        on1[u] = j0 + u < w && ((md[u] >> lane) & 1u) != 0;
        bs.pair((on0[u] || on1[u]) ? row + off[u] : 0, xv[u]);
      }
      if (j0 == 0 && prow >= 0) {  // the previous slice's epilogue, behind this round's loads
        __builtin_amdgcn_sched_barrier(0);
        flush();
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const V p0 = (V)a[u][0] * xv[u][0];
        const V p1 = (V)a[u][1] * xv[u][1];
        const V t0 = acc0 + p0;
        const V t1 = acc1 + p1;
        acc0 = on0[u] ? t0 : acc0;
        acc1 = on1[u] ? t1 : acc1;
      }
    }
    if (w == 0 && prow >= 0) flush();
    pend[0] = acc0;
    pend[1] = acc1;
    prow = row;
  }
  if (prow >= 0) flush();
  if (part != nullptr) {
    red[tid] = dacc;
    block_tree_reduce(red, kBlock, 1);
    if (tid == 0) part[g] = red[0];
  }
}

// ------------------------------------ paired-row SELL-128 SpMV (k = 1)
// The general-CSR image for one right-hand side (kry_csr::sp_*): slices of
// 128 rows, slot column j of a slice holds the j-th stored entry of every row
// (padding: delta 0xFFFF, value 0), rows interleaved so that lane l of the
// wave owns rows 2l and 2l + 1. Per slot column a lane makes one 16-B value
// load, one 4-B load of its two uint16 column deltas over the slot column's
// int32 base (wave-uniform: scalar load) and one 16-B x load at its first
// column: when the second row's column is the next one (banded and stencil
// rows, where the slice's rows share their offsets) that load serves both;
// otherwise the second value is an 8-B load behind one wave-level branch per
// round, skipped by waves whose lanes all paired. Against SELL-64 that is
// half the memory instructions per nonzero with the same 10 bytes
// (archive:sellp_bench: 0.297 against 0.352 ms on the metric matrix). Each row
// is summed from 0 in stored order, a hole or padding slot dropped by a
// select, never added: bitwise csr_matvec, for unsorted rows, duplicates
// and explicit zeros too. One slice per wave (grid over the slices).
template <typename V, typename MV, int UNR, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_pair_kernel(const int64_t *__restrict__ sptr,
                                                           const int *__restrict__ swidth,
                                                           const int *__restrict__ cbase,
                                                           const uint32_t *__restrict__ dpair,
                                                           const MV *__restrict__ val, int64_t nslices, int64_t n,
                                                           Src src, Epi epi, double *__restrict__ part,
                                                           const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const auto bs = src.template bind<1>(0);
  double dacc = 0.0;
  for (int64_t s = (int64_t)g * 4 + wid; s < nslices; s += W) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * kPairSlice + 2 * lane;
    const int *cb = cbase + base / kPairSlice;  // wave-uniform: scalar loads (padded by kDiaPad)
    const uint32_t *cd = dpair + base / 2 + lane;
    const MV *cv = val + base + 2 * lane;
    V acc0 = V(0), acc1 = V(0);
    for (int j0 = 0; j0 < w; j0 += UNR) {
      int b[UNR];
      uint32_t d[UNR];
      MV a[UNR][2];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        b[u] = cb[j0 + u];
        if (j0 + u < w) {
          d[u] = __builtin_nontemporal_load(cd + (int64_t)(j0 + u) * (kPairSlice / 2));
          pload_nt<MV>(cv + (int64_t)(j0 + u) * kPairSlice, a[u]);
        } else {
          d[u] = 0xFFFFFFFFu;
          a[u][0] = MV(0);
          a[u][1] = MV(0);
        }
      }
      V x0[UNR], x1[UNR];
      bool v0[UNR], v1[UNR], need[UNR];
      int64_t c1[UNR];
      bool any = false;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t lo = d[u] & 0xFFFFu, hi = d[u] >> 16;
        v0[u] = lo != 0xFFFFu;
        v1[u] = hi != 0xFFFFu;
        const int64_t c0 = (int64_t)b[u] + lo;
        c1[u] = (int64_t)b[u] + hi;
        const bool pr = v0[u] && v1[u] && c1[u] == c0 + 1;
        V xp[2];
        bs.pair(v0[u] ? c0 : (v1[u] ? c1[u] : 0), xp);  // at worst x[n]: inside the allocation slack
        x0[u] = xp[0];
        x1[u] = pr ? xp[1] : xp[0];
        need[u] = v0[u] && v1[u] && !pr;
        any = any || need[u];
      }
      if (__any(any)) {
#pragma unroll
        for (int u = 0; u < UNR; ++u)
          if (need[u]) x1[u] = bs(c1[u], 0);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const V p0 = (V)a[u][0] * x0[u];
        const V p1 = (V)a[u][1] * x1[u];
        const V t0 = acc0 + p0;
        const V t1 = acc1 + p1;
        acc0 = v0[u] ? t0 : acc0;
        acc1 = v1[u] ? t1 : acc1;
      }
    }
    if (row + 1 < n) {
      V xi[2];
      bs.pair(row, xi);
      const V o[2] = {acc0, acc1};
      dacc += epi.rows2(row, o, xi);
    } else if (row < n) {
      dacc += epi(row, 0, acc0, bs(row, 0));
    }
  }
  if (part != nullptr) {
    red[tid] = dacc;
    block_tree_reduce(red, kBlock, 1);
    if (tid == 0) part[g] = red[0];
  }
}


// ---------------------------------- rank-sorted SELL-128 SpMV (k = 1)
// Round 5, kry_csr::rs_* (host_image.hpp rs_build): the paired-row slice
// geometry (lane l owns rows 2l, 2l + 1; one 16-B value load and one 8-B
// load of the two rows' column words per slot column) with int32 columns, for
// matrices the DIA, column-blocked and paired images do not take: unsorted
// rows, or slot columns wider than a uint16 delta (a renumbered matrix). In
// every run of kRsChunk stored entries of a row the entries sit in column
// order, so slot column j of neighbouring rows gathers neighbouring x entries
// (the renumbered permuted metric: 0.155 cache lines per gather against 0.65
// in stored order). The run's products are written to LDS at their stored
// position (the word's top 4 bits) and summed back in that order, from 0,
// one rounding per product and per add: bitwise csr_matvec. LDS: 2 x 16 x 64
// products per wave, each lane reading back only what it wrote (no barrier).
// The second row's x is the first row's 16-B pair load when its column is
// the next one (neighbouring rows of a banded numbering), else an 8-B load
// behind one wave-level branch, as in the paired kernel.
constexpr int kRsRun = kRsChunk;
template <typename V, typename MV, int UNR, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_rs_kernel(const int64_t *__restrict__ sptr,
                                                         const int *__restrict__ swidth,
                                                         const uint32_t *__restrict__ colrank,
                                                         const MV *__restrict__ val, int64_t nslices, int64_t n,
                                                         Src src, Epi epi, double *__restrict__ part,
                                                         const Ctrl *ctrl, int step) {
  static_assert(kRsRun % UNR == 0, "a run is a whole number of unrolled rounds");
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  __shared__ V prod[kBlock / 64][2][kRsRun][64];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const auto bs = src.template bind<1>(0);
  V(*pw)[kRsRun][64] = prod[wid];
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  double dacc = 0.0;
  for (int64_t s = (int64_t)g * 4 + wid; s < nslices; s += W) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * kPairSlice + 2 * lane;
    const u2 *cr = reinterpret_cast<const u2 *>(colrank + base) + lane;
    const MV *cv = val + base + 2 * lane;
    V acc0 = V(0), acc1 = V(0);
    for (int r0 = 0; r0 < w; r0 += kRsRun) {
      const int re = w < r0 + kRsRun ? w : r0 + kRsRun;
      int n0 = 0, n1 = 0;
      for (int j0 = r0; j0 < re; j0 += UNR) {
        uint32_t d0[UNR], d1[UNR];
        MV a[UNR][2];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (j0 + u < re) {
            const u2 t = __builtin_nontemporal_load(cr + (int64_t)(j0 + u) * (kPairSlice / 2));
            d0[u] = t.x;
            d1[u] = t.y;
            pload_nt<MV>(cv + (int64_t)(j0 + u) * kPairSlice, a[u]);
          } else {
            d0[u] = 0xFFFFFFFFu;
            d1[u] = 0xFFFFFFFFu;
            a[u][0] = MV(0);
            a[u][1] = MV(0);
          }
        }
        V x0[UNR], x1[UNR];
        bool v0[UNR], v1[UNR], need[UNR];
        int64_t c1[UNR];
        bool any = false;
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          v0[u] = d0[u] != 0xFFFFFFFFu;
          v1[u] = d1[u] != 0xFFFFFFFFu;
          const int64_t c0 = (int64_t)(d0[u] & 0x0FFFFFFFu);
          c1[u] = (int64_t)(d1[u] & 0x0FFFFFFFu);
          const bool pr = v0[u] && v1[u] && c1[u] == c0 + 1;
          V xp[2];
          bs.pair(v0[u] ? c0 : (v1[u] ? c1[u] : 0), xp);  // at worst x[n]: inside the allocation slack
          x0[u] = xp[0];
          x1[u] = pr ? xp[1] : xp[0];
          need[u] = v0[u] && v1[u] && !pr;
          any = any || need[u];
        }
        if (__any(any)) {
#pragma unroll
          for (int u = 0; u < UNR; ++u)
            if (need[u]) x1[u] = bs(c1[u], 0);
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const V p0 = (V)a[u][0] * x0[u];
          const V p1 = (V)a[u][1] * x1[u];
          if (v0[u]) pw[0][d0[u] >> 28][lane] = p0;
          if (v1[u]) pw[1][d1[u] >> 28][lane] = p1;
          n0 += v0[u] ? 1 : 0;
          n1 += v1[u] ? 1 : 0;
        }
      }
      // the run in stored order (entries of a row fill its first slots: the
      // run's positions are 0 .. n - 1)
      const int nm = n0 > n1 ? n0 : n1;
      for (int k = 0; k < nm; ++k) {
        if (k < n0) acc0 = acc0 + pw[0][k][lane];
        if (k < n1) acc1 = acc1 + pw[1][k][lane];
      }
    }
    if (row + 1 < n) {
      V xi[2];
      bs.pair(row, xi);
      const V o[2] = {acc0, acc1};
      dacc += epi.rows2(row, o, xi);
    } else if (row < n) {
      dacc += epi(row, 0, acc0, bs(row, 0));
    }
  }
  if (part != nullptr) {
    red[tid] = dacc;
    block_tree_reduce(red, kBlock, 1);
    if (tid == 0) part[g] = red[0];
  }
}

// The same rank-sorted image, one row per lane (the default since round 5;
// KRY_SPMV_RS1=0 selects the paired kernel above): a wave takes half a slice
// (64 rows: row r of the half is image slot r, so the column-word, value and
// x loads of a slot column stay contiguous 4-, 8- and 8-byte runs), and the
// run's products need 16 x 64 doubles of LDS per wave instead of 2 x 16 x 64:
// five blocks of four waves per CU instead of two (the paired kernel's
// occupancy is set by its 66 KB of LDS per block). UNR = 16 puts a whole
// run's loads in flight. Same products, same stored-order sums: bitwise the
// paired kernel and csr_matvec. Renumbered permuted metric: 0.561 -> 0.499
// ms per SpMV at four blocks per CU (tools/rs_ab.py,
// profiles/r05_rs_ab.txt).
template <typename V, typename MV, int UNR, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_rs1_kernel(const int64_t *__restrict__ sptr,
                                                          const int *__restrict__ swidth,
                                                          const uint32_t *__restrict__ colrank,
                                                          const MV *__restrict__ val, int64_t nslices, int64_t n,
                                                          Src src, Epi epi, double *__restrict__ part,
                                                          const Ctrl *ctrl, int step) {
  static_assert(kRsRun % UNR == 0, "a run is a whole number of unrolled rounds");
  if (halted(ctrl, step)) return;
  // 32 KB (fp64): five blocks per CU; the block reduction reuses it
  __shared__ __attribute__((aligned(16))) V prod[kBlock / 64][kRsRun][64];
  static_assert(sizeof(prod) >= kBlock * sizeof(double), "the reduction fits the product buffer");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t W = (int64_t)gridDim.x * 4;
  const auto bs = src.template bind<1>(0);
  V(*pw)[64] = prod[wid];
  double dacc = 0.0;
  for (int64_t hs = (int64_t)g * 4 + wid; hs < 2 * nslices; hs += W) {
    const int64_t s = hs >> 1;
    const int q = (int)(hs & 1) * 64 + lane;  // the row's slot within the slice
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t row = s * kPairSlice + q;
    const uint32_t *cr = colrank + base + q;
    const MV *cv = val + base + q;
    const V xi = bs(row < n ? row : 0, 0);  // the epilogue's x, in flight with the run's loads
    V acc = V(0);
    for (int r0 = 0; r0 < w; r0 += kRsRun) {
      const int re = w < r0 + kRsRun ? w : r0 + kRsRun;
      int nv = 0;
      for (int j0 = r0; j0 < re; j0 += UNR) {
        uint32_t d[UNR];
        MV a[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (j0 + u < re) {
            d[u] = __builtin_nontemporal_load(cr + (int64_t)(j0 + u) * kPairSlice);
            a[u] = __builtin_nontemporal_load(cv + (int64_t)(j0 + u) * kPairSlice);
          } else {
            d[u] = 0xFFFFFFFFu;
            a[u] = MV(0);
          }
        }
        V xv[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const bool v = d[u] != 0xFFFFFFFFu;
          xv[u] = bs(v ? (int64_t)(d[u] & 0x0FFFFFFFu) : 0, 0);
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if (d[u] != 0xFFFFFFFFu) pw[d[u] >> 28][lane] = (V)a[u] * xv[u];
          nv += d[u] != 0xFFFFFFFFu ? 1 : 0;
        }
      }
      // the run in stored order: all sixteen LDS reads issued together (the
      // slots past the run's nv entries are read and dropped), then the adds
      V t[kRsRun];
#pragma unroll
      for (int k = 0; k < kRsRun; ++k) t[k] = pw[k][lane];
#pragma unroll
      for (int k = 0; k < kRsRun; ++k) acc = k < nv ? acc + t[k] : acc;
    }
    if (row < n) dacc += epi(row, 0, acc, xi);
  }
  if (part != nullptr) {
    double *red = reinterpret_cast<double *>(&prod[0][0][0]);
    __syncthreads();  // every wave is done with its products
    red[tid] = dacc;
    block_tree_reduce(red, kBlock, 1);
    if (tid == 0) part[g] = red[0];
  }
}

// ------------------------------ diagonal-offset SpMV, block RHS (k = 2..8)
// The same SELL-128/DIA image for k right-hand sides stored row-major
// (n x k): for a slot column of offset o the x rows of the slice's rows are
// the contiguous block x[128 s + o, +128) x k. A lane owns CPL consecutive
// columns (16 bytes) of one row per row group; a wave covers RPG = 64 / (k /
// CPL) rows per group and NG = 128 / RPG groups per slice. Slot-major: for
// each slot column the wave loads every group's value and x run at once (NG
// contiguous runs of RPG x k elements, 1 KB each for k = 8) and accumulates;
// each (row, column) is summed from 0 over the slot columns in ascending
// offset order, holes skipped: bitwise csr_matvecs. One slice per wave (the
// grid covers the slices, kMaxGridBlk blocks at most): the waves resident on
// an XCD then work on neighbouring slices together, so the x rows a slot
// column at offset +-o reads again were fetched by a neighbouring wave
// moments before and are L2 hits (archive:dia_blk_bench: x fetched ~1x from
// HBM, against ~3x with 2.4 contiguous slices per wave at 8192 blocks).
// Round 5, the x window: the slice's own x rows (every row < n, mask or
// not) and the two rows just outside it are loaded once per slice into the
// wave's LDS window; the slot columns of offset -1, 0 and +1 (the
// near-diagonal runs of a 2-D / 3-D stencil) and the epilogue's p read their
// runs from it (ds_read_b128) instead of three more 1 KB runs per group
// through L1 / L2. cfg4 (5-point Poisson 3163^2, k = 8): 0.458 -> 0.372 ms
// per launch (tools/dia_blk_probe.hip, profiles/r05_dia_blk_probe.txt). The
// values and their order are unchanged: a window row holds the same x the
// direct load would return. Each wave reads only its own window (no
// barrier: a wave's LDS accesses execute in order; compiler-only barriers
// keep a read of a neighbour lane's row below the write of it).
// The epilogue is the lane-group kernel's row<CPL>.
template <typename V, typename MV, int CPL, int NG, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_dia_blk_kernel(const int64_t *__restrict__ sptr,
                                                              const int *__restrict__ swidth,
                                                              const int *__restrict__ doff,
                                                              const uint64_t *__restrict__ dmask,
                                                              const MV *__restrict__ val, int64_t nslices, int64_t n,
                                                              int k, Src src, Epi epi, double *__restrict__ part,
                                                              const Ctrl *ctrl, int step) {
  constexpr int RPG = kDiaSlice / NG;  // rows per group
  constexpr int LPR = 64 / RPG;        // lanes per row (k / CPL)
  constexpr int WROWS = kDiaSlice + 2;  // window rows 128 s - 1 .. 128 s + 128
  typedef V vec_t __attribute__((ext_vector_type(CPL)));
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock * CPL];
  __shared__ vec_t win[kBlock / 64][WROWS * LPR];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int rl0 = lane / LPR, cl = lane % LPR, c0 = cl * CPL;
  const int64_t W = (int64_t)gridDim.x * 4;
  const auto bs = src.template bind<CPL>(c0);
  vec_t *wn = win[wid];
  auto wput = [&](int wr, const V(&t)[CPL]) {
    vec_t v;
#pragma unroll
    for (int c = 0; c < CPL; ++c) v[c] = t[c];
    wn[wr * LPR + cl] = v;
  };
  auto wget = [&](int wr, V(&t)[CPL]) {
    const vec_t v = wn[wr * LPR + cl];
#pragma unroll
    for (int c = 0; c < CPL; ++c) t[c] = v[c];
  };
  double dacc[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) dacc[c] = 0.0;
  for (int64_t s = (int64_t)g * 4 + wid; s < nslices; s += W) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    const int64_t cb = base / kDiaSlice;
    const int64_t r0 = s * kDiaSlice;
    V acc[NG][CPL];
#pragma unroll
    for (int r = 0; r < NG; ++r)
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[r][c] = V(0);
    {
      // the window (rows clamped below n: a row >= n is never read through
      // a set mask bit, nor stored); lanes < LPR add row r0 - 1, the next
      // LPR lanes row r0 + 128 (clamped to [0, n))
      V t[NG][CPL], h[CPL];
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int64_t row = r0 + r * RPG + rl0;
        bs.row(row < n ? row : n - 1, t[r]);
      }
      const int64_t hr = lane < LPR ? (r0 > 0 ? r0 - 1 : 0) : (r0 + kDiaSlice < n ? r0 + kDiaSlice : n - 1);
      bs.row(hr, h);
      // LDS accesses of one wave execute in order, so a lane's read of a
      // neighbour's row sees its write; only the compiler must not move one
      // across the other (the previous slice's reads stay above the writes)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int r = 0; r < NG; ++r) wput(r * RPG + rl0 + 1, t[r]);
      if (lane < 2 * LPR) wput(lane < LPR ? 0 : WROWS - 1, h);
      asm volatile("" ::: "memory");
    }
    for (int j = 0; j < w; ++j) {
      const int off = doff[cb + j];  // wave-uniform: scalar loads
      const uint64_t m0 = dmask[2 * (cb + j)], m1 = dmask[2 * (cb + j) + 1];
      const MV *cv = val + base + (int64_t)j * kDiaSlice;
      V a[NG];
      bool on[NG];
      V xv[NG][CPL];
#pragma unroll
      for (int r = 0; r < NG; ++r) {
        const int rl = r * RPG + rl0;
        a[r] = (V)cv[rl];
        on[r] = ((((rl & 1) ? m1 : m0) >> (rl >> 1)) & 1u) != 0;  // mask word (rl & 1), bit (rl >> 1)
      }
      if (off >= -1 && off <= 1) {  // wave-uniform branch around all the groups' runs
#pragma unroll
        for (int r = 0; r < NG; ++r) wget(r * RPG + rl0 + 1 + off, xv[r]);
      } else {
#pragma unroll
        for (int r = 0; r < NG; ++r) bs.row(on[r] ? r0 + r * RPG + rl0 + off : 0, xv[r]);
      }
#pragma unroll
      for (int r = 0; r < NG; ++r)
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const V p = a[r] * xv[r][c];
          const V t = acc[r][c] + p;
          acc[r][c] = on[r] ? t : acc[r][c];
        }
    }
#pragma unroll
    for (int r = 0; r < NG; ++r) {
      const int64_t row = r0 + r * RPG + rl0;
      if (row < n) {
        V xi[CPL];
        wget(r * RPG + rl0 + 1, xi);
        epi.template row<CPL>(row, c0, acc[r], xi, dacc);
      }
    }
  }
  if (part != nullptr) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) red[tid * CPL + c] = dacc[c];  // slot tid * CPL + c holds column (c0 + c)
    block_tree_reduce(red, kBlock * CPL, k);
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
  // non-temporal forms for streams nobody re-reads soon (keeps the vectors the
  // next SpMV gathers resident in L2 / MALL)
  __device__ __forceinline__ static void load_nt(const V *p, int64_t e, int64_t N, V (&o)[W]) {
    if (e + W <= N) {
      typedef V vec_t __attribute__((ext_vector_type(W)));
      const vec_t t = __builtin_nontemporal_load(reinterpret_cast<const vec_t *>(p + e));
#pragma unroll
      for (int v = 0; v < W; ++v) o[v] = t[v];
    } else {
#pragma unroll
      for (int v = 0; v < W; ++v) o[v] = e + v < N ? p[e + v] : V(0);
    }
  }
  __device__ __forceinline__ static void store_nt(V *p, int64_t e, int64_t N, const V (&o)[W]) {
    if (e + W <= N) {
      typedef V vec_t __attribute__((ext_vector_type(W)));
      vec_t t;
#pragma unroll
      for (int v = 0; v < W; ++v) t[v] = o[v];
      __builtin_nontemporal_store(t, reinterpret_cast<vec_t *>(p + e));
    } else {
#pragma unroll
      for (int v = 0; v < W; ++v)
        if (e + v < N) p[e + v] = o[v];
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
// NT threads (the block size), red[NT]
template <int NT = kBlock>
__device__ __forceinline__ void reduce_partials(const double *part, int P, int k, double *red) {
  const int tid = threadIdx.x;
  const int c = tid & (k - 1);
  const int step = NT / k;
  double s = 0.0;
  // loads issued 32 (then 8) at a time (independent), added in the fixed
  // sequential order: one L2 round trip per 32 partials (k = 8 over 8192
  // blocks: 256 partials per thread), same bits as a plain loop
  int p = tid / k;
  for (; p + 31 * step < P; p += 32 * step) {
    double v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) v[u] = part[(int64_t)(p + u * step) * k + c];
#pragma unroll
    for (int u = 0; u < 32; ++u) s += v[u];
  }
  for (; p + 7 * step < P; p += 8 * step) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(p + u * step) * k + c];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; p < P; p += step) s += part[(int64_t)p * k + c];
  red[tid] = s;
  block_tree_reduce(red, NT, k);
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

// ---------------------------------------------- lane-group SELL SpMV (4 <= k <= 64)
// For a block of k right-hand sides stored row-major (row i's k values are
// contiguous), LPR = k / CPL lanes share a row and each owns CPL consecutive
// columns: a wave covers 64 / LPR rows of a slice per pass (LPR passes), and
// each lane gathers its CPL values of an x row with 16-B vector loads, so one
// pass's gathers read whole contiguous rows (k * 8 bytes each). Same slot
// order, same per-(row, column) sequential sum, so the result is bitwise the
// lane-per-row kernel's (and csr_matvecs'). CPL = 4 measured 0.53 ms against
// 0.80 ms for one column per lane on cfg4 (k = 8, archive:spmv_bench block).
template <typename V, typename MV, typename I, int CPL, int UNR, bool D16, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_sell_lg_kernel(
    const int64_t *__restrict__ sptr, const int *__restrict__ swidth, const I *__restrict__ sidx,
    const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase, const MV *__restrict__ sval,
    int64_t nslices, int64_t n, int k, const I *__restrict__ indptr, const I *__restrict__ indices,
    const MV *__restrict__ data, Src src, Epi epi, double *__restrict__ part, const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock * CPL];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int lpr = k / CPL;          // lanes per row
  const int rows_per_pass = 64 / lpr;
  const int rl0 = lane / lpr, c0 = (lane % lpr) * CPL;
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t m = (int64_t)g * 4 + wid;
  const int64_t s_begin = nslices * m / W, s_end = nslices * (m + 1) / W;
  const auto bs = src.template bind<CPL>(c0);
  double dacc[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) dacc[c] = 0.0;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const int w = swidth[s];
    const int64_t base = sptr[s];
    for (int rl = rl0; rl < 64; rl += rows_per_pass) {
      const int64_t row = s * 64 + rl;
      V acc[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[c] = V(0);
      if (w >= 0) {
        const I *ci = sidx + base + rl;
        const uint16_t *cd = sdelta + base + rl;
        const int *cb = scbase + (base >> 6);
        const MV *cv = sval + base + rl;
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
          for (int u = 0; u < UNR; ++u)
            if (col[u] >= 0) {
              V xv[CPL];
              bs.row(col[u], xv);
#pragma unroll
              for (int c = 0; c < CPL; ++c) {
                const V p = a[u] * xv[c];
                acc[c] = acc[c] + p;
              }
            }
        }
      } else if (row < n) {
        for (I e = indptr[row]; e < indptr[row + 1]; ++e) {
          const V a = (V)data[e];
          V xv[CPL];
          bs.row(indices[e], xv);
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const V p = a * xv[c];
            acc[c] = acc[c] + p;
          }
        }
      }
      if (row < n) {
        V xi[CPL];
        bs.row(row, xi);
        epi.template row<CPL>(row, c0, acc, xi, dacc);
      }
    }
  }
  if (part != nullptr) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) red[tid * CPL + c] = dacc[c];  // slot tid * CPL + c holds column (c0 + c)
    block_tree_reduce(red, kBlock * CPL, k);
    if (tid < k) part[(int64_t)g * k + tid] = red[tid];
  }
}

// One (column block, row group) segment of the column-blocked image: its
// entries [s0, s0 + len) are multiplied against the x block in chunks of
// kCbCap products staged in LDS, then thread r adds its row's products
// [r0, r1) to acc in stored order. VEC: each thread loads 4 consecutive
// entries (one 16-B column load, 16-B value loads) from the 4-entry-aligned
// quads covering the segment (entries outside it are masked), against one
// 4- or 8-B load per entry and array.
template <bool VEC, typename V, typename MV, class BS>
__device__ __forceinline__ void cb_segment(int64_t s0, int len, int r0, int r1, const int *__restrict__ col,
                                           const MV *__restrict__ val, const BS &bs, V *prod, V &acc, int tid) {
  constexpr int U = kCbCap / kBlock;
  if constexpr (VEC) {
    static_assert(U == 4, "one quad of entries per thread and chunk");
    typedef int i4 __attribute__((ext_vector_type(4)));
    const int64_t q0 = s0 >> 2, qend = (s0 + len + 3) >> 2;
    for (int64_t qc = q0; qc < qend; qc += kBlock) {
      const int64_t base = qc * 4 - s0;  // segment-relative entry held by prod[0]
      __syncthreads();                   // the previous chunk has been consumed
      const int64_t q = qc + tid;
      int j[4];
      V a[4];
      if (q < qend) {
        const i4 c = __builtin_nontemporal_load(reinterpret_cast<const i4 *>(col) + q);
        MV m[4];
        if constexpr (sizeof(MV) == 8) {
          typedef double d2 __attribute__((ext_vector_type(2)));
          const d2 v0 = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(val) + 2 * q);
          const d2 v1 = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(val) + 2 * q + 1);
          m[0] = v0.x; m[1] = v0.y; m[2] = v1.x; m[3] = v1.y;
        } else {
          typedef float f4 __attribute__((ext_vector_type(4)));
          const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(val) + q);
          m[0] = v.x; m[1] = v.y; m[2] = v.z; m[3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t e = base + 4 * (int64_t)tid + i;
          const bool in = e >= 0 && e < len;
          j[i] = in ? c[i] : -1;
          a[i] = (V)m[i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) { j[i] = -1; a[i] = V(0); }
      }
      V xj[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) xj[i] = j[i] >= 0 ? bs(j[i], 0) : V(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (j[i] >= 0) prod[4 * tid + i] = a[i] * xj[i];
      __syncthreads();
      const int64_t lo = r0 > base ? r0 : base, hi = r1 < base + kCbCap ? r1 : base + kCbCap;
      for (int64_t e = lo; e < hi; ++e) acc = acc + prod[e - base];
    }
  } else {
    for (int c0 = 0; c0 < len; c0 += kCbCap) {
      const int c1 = len < c0 + kCbCap ? len : c0 + kCbCap;
      __syncthreads();  // the previous chunk has been consumed
      // U entries per thread, all loads issued before the gathers
      int j[U];
      V a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = c0 + tid + u * kBlock;
        j[u] = e < c1 ? __builtin_nontemporal_load(col + s0 + e) : -1;
        a[u] = e < c1 ? (V)__builtin_nontemporal_load(val + s0 + e) : V(0);
      }
      V xj[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xj[u] = j[u] >= 0 ? bs(j[u], 0) : V(0);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j[u] >= 0) prod[tid + u * kBlock] = a[u] * xj[u];
      __syncthreads();
      const int lo = r0 > c0 ? r0 : c0, hi = r1 < c1 ? r1 : c1;
      for (int e = lo; e < hi; ++e) acc = acc + prod[e - c0];
    }
  }
}

// ------------------------------------------- column-blocked SpMV (k = 1)
// Block `blk` owns the 256-row groups g0 + blk, g0 + blk + G, ... below g1
// (at most kCbMaxOwn of them) and walks the column blocks in order for all of
// them: per (column block, group) segment the entries are multiplied against
// the L2-resident x block with coalesced loads and staged in LDS, then thread
// r adds its row's products to the row's running sum (a register), in stored
// order (the same sequence of roundings as csr_matvec: sum from 0, product
// rounded, then added; rows are sorted, so block order is stored order). The
// last column block applies the epilogue. Blocks never wait for each other
// (no residency assumption); they stay roughly in step on the column blocks
// because their work per block is similar, which is what keeps the current x
// block L2-resident. A matrix with more than kCbPersistGrid * kCbMaxOwn groups
// takes one launch per range of that many groups (round 4; before, one launch
// per column block with the running sums carried through HBM: 2.4 GB per
// SpMV at n = 10 M).
constexpr int kCbMaxOwn = 16;
constexpr int kCbPersistGrid = 1024;  // 4 blocks per CU: all resident, so they start together
template <bool VEC, typename V, typename MV, class Src, class Epi>
__global__ __launch_bounds__(kBlock) void spmv_cbp_kernel(int nb, int64_t n, int64_t ng, int64_t g0, int64_t g1,
                                                          const int64_t *__restrict__ gptr,
                                                          const uint16_t *__restrict__ roff,
                                                          const int *__restrict__ col, const MV *__restrict__ val,
                                                          Src src, Epi epi, double *__restrict__ part,
                                                          const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ V prod[kCbCap];
  __shared__ double red[kBlock];
  const int tid = threadIdx.x;
  const auto bs = src.template bind<1>(0);
  V acc[kCbMaxOwn];
#pragma unroll
  for (int o = 0; o < kCbMaxOwn; ++o) acc[o] = V(0);
  for (int b = 0; b < nb; ++b) {
#pragma unroll
    for (int o = 0; o < kCbMaxOwn; ++o) {
      const int64_t g = g0 + (int64_t)blockIdx.x + (int64_t)o * gridDim.x;
      if (g >= g1) break;
      const int64_t s0 = gptr[(int64_t)b * ng + g];
      const int len = (int)(gptr[(int64_t)b * ng + g + 1] - s0);
      const int64_t row = g * kCbRows + tid;
      const bool has = row < n;
      int r0 = 0, r1 = 0;
      if (has) {
        r0 = roff[(int64_t)b * n + row];
        r1 = (tid == kCbRows - 1 || row + 1 >= n) ? len : (int)roff[(int64_t)b * n + row + 1];
      }
      cb_segment<VEC, V, MV>(s0, len, r0, r1, col, val, bs, prod, acc[o], tid);
    }
  }
  double dacc = 0.0;
#pragma unroll
  for (int o = 0; o < kCbMaxOwn; ++o) {
    const int64_t g = g0 + (int64_t)blockIdx.x + (int64_t)o * gridDim.x;
    if (g >= g1) break;
    const int64_t row = g * kCbRows + tid;
    if (row < n) dacc += epi(row, 0, acc[o], bs(row, 0));
  }
  if (part != nullptr) {
    __syncthreads();
    red[tid] = dacc;
    block_tree_reduce(red, kBlock, 1);
    if (tid == 0) part[blockIdx.x] = red[0];
  }
}

// -------------------------------------------------------- host launchers
template <typename V, typename MV, typename I, int KT, int UNR, bool D16, class Src, class Epi>
int launch_sell_img(const kry_csr *A, int k, Src src, Epi epi, double *part, const Ctrl *ctrl, int step,
                    hipStream_t st) {
  const int nch = k / KT;
  int64_t waves = A->nslices * nch;
  int grid = (int)((waves + 3) / 4);
  if (grid > kMaxGrid) grid = kMaxGrid;
  if (grid < 1) grid = 1;
  if (nch > 1) grid = (grid + 7) / 8 * 8;  // 4 * grid must be a multiple of nch (<= 32)
  if (grid > kMaxGrid) grid = kMaxGrid;
  hipLaunchKernelGGL((spmv_sell_kernel<V, MV, I, KT, UNR, D16, Src, Epi>), dim3(grid), dim3(kBlock), 0, st,
                     static_cast<const int64_t *>(A->sptr), static_cast<const int *>(A->swidth),
                     static_cast<const I *>(A->sidx), static_cast<const uint16_t *>(A->sdelta),
                     static_cast<const int *>(A->scbase), static_cast<const MV *>(A->sval), A->nslices, A->n, k,
                     static_cast<const I *>(A->indptr), static_cast<const I *>(A->indices),
                     static_cast<const MV *>(A->data), src, epi, part, ctrl, step);
  return grid;
}

template <typename V, typename MV, typename I, int KT, int UNR, class Src, class Epi>
int launch_sell(const kry_csr *A, int k, Src src, Epi epi, double *part, const Ctrl *ctrl, int step,
                hipStream_t st) {
  if constexpr (sizeof(I) == 4) {
    if (A->compact) return launch_sell_img<V, MV, I, KT, UNR, true>(A, k, src, epi, part, ctrl, step, st);
  }
  return launch_sell_img<V, MV, I, KT, UNR, false>(A, k, src, epi, part, ctrl, step, st);
}

// 16-B quad loads in the column-blocked kernels (KRY_CB_VEC=0: one load per
// entry and array, the round-2 form; A/B switch)
inline bool cb_vec() {
  static const bool on = [] {
    const char *e = getenv("KRY_CB_VEC");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// KRY_SPMV_DIA_BLK=0: block right-hand sides on the lane-group SELL kernel
// instead of the diagonal-offset image (A/B and tests)
inline bool dia_blk_off() {
  static const bool off = [] {
    const char *e = getenv("KRY_SPMV_DIA_BLK");
    return e && atoi(e) == 0;
  }();
  return off;
}

// launch_spmv takes the column-blocked kernels for this operator and k: its
// SpMV is bound by the random x gathers, so a source that computes on every
// gathered value (SrcScaled's division) costs more than a pass forming the
// vector first.
// The rank-sorted image's kernel: one row per lane with sixteen slot
// columns' loads in flight (default, KRY_SPMV_RS1=2), eight (1), or the
// paired two-rows-per-lane kernel (0); tools/rs_ab.py.
inline int rs1_on() {
  const char *e = getenv("KRY_SPMV_RS1");  // read per launch: the tests switch it within one process
  return e ? atoi(e) : 2;
}

template <typename I>
inline bool spmv_column_blocked(const kry_csr *A, int k) {
  return sizeof(I) == 4 && k == 1 && !A->dia && A->cb_nb > 0;
}

// y-side epilogue Epi / x-side source Src composition of one SpMV launch;
// returns the number of block partials written to `part` (if non-null).
template <typename V, typename MV, typename I, class Src, class Epi>
void launch_spmv(const kry_csr *A, int k, Src src, Epi epi, double *part, int *grid_out, const Ctrl *ctrl,
                 int step, hipStream_t st) {
  KRY_REQUIRE(k >= 1 && k <= kMaxCols && is_pow2(k), KRY_EUNSUPPORTED, "k must be a power of two <= 256");
  int grid;
  if (k == 1 && A->sp) {
    // one slice per wave (archive:sellp_bench: 0.32 ms against 0.36 ms at 8192
    // blocks of 2.4 slices per wave on the metric matrix); partial buffers
    // hold kMaxGridBlk rows for k = 1
    grid = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxGridBlk, (A->sp_nslices + 3) / 4));
    hipLaunchKernelGGL((spmv_pair_kernel<V, MV, 8, Src, Epi>), dim3(grid), dim3(kBlock), 0, st,
                       static_cast<const int64_t *>(A->sp_sptr), static_cast<const int *>(A->sp_width),
                       static_cast<const int *>(A->sp_cbase), static_cast<const uint32_t *>(A->sp_delta),
                       static_cast<const MV *>(A->sp_val), A->sp_nslices, A->n, src, epi, part, ctrl, step);
    KRY_HIP(hipGetLastError());
    if (grid_out) *grid_out = grid;
    return;
  }
  if (k == 1 && A->rs && rs1_on()) {
    grid = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxGridBlk, (2 * A->rs_nslices + 3) / 4));
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, st, static_cast<const int64_t *>(A->rs_sptr),
                         static_cast<const int *>(A->rs_width), static_cast<const uint32_t *>(A->rs_colrank),
                         static_cast<const MV *>(A->rs_val), A->rs_nslices, A->n, src, epi, part, ctrl, step);
    };
    if (rs1_on() == 2)
      go(spmv_rs1_kernel<V, MV, 16, Src, Epi>);
    else
      go(spmv_rs1_kernel<V, MV, 8, Src, Epi>);
    KRY_HIP(hipGetLastError());
    if (grid_out) *grid_out = grid;
    return;
  }
  if (k == 1 && A->rs) {
    grid = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxGridBlk, (A->rs_nslices + 3) / 4));
    hipLaunchKernelGGL((spmv_rs_kernel<V, MV, 8, Src, Epi>), dim3(grid), dim3(kBlock), 0, st,
                       static_cast<const int64_t *>(A->rs_sptr), static_cast<const int *>(A->rs_width),
                       static_cast<const uint32_t *>(A->rs_colrank), static_cast<const MV *>(A->rs_val),
                       A->rs_nslices, A->n, src, epi, part, ctrl, step);
    KRY_HIP(hipGetLastError());
    if (grid_out) *grid_out = grid;
    return;
  }
  if constexpr (sizeof(I) == 4) {
    if (k == 1 && A->dia) {
      // Wide images (more than 8 slot columns, the metric's 15): one slice
      // per wave (tools/dia_bench "deferred store, grid": 0.227 ms on the
      // metric against 0.252 ms at 8192 blocks of 2.4 slices per wave; CG
      // 2896 -> 3040 it/s). Narrow ones keep 8192 blocks: on cfg5 (7 slot
      // columns, fp32 values) the larger grid measured 1.8 % slower per
      // MINRES iteration, its consumers summing twice the partials.
      static const int dia_cap_env = [] {
        const char *e = getenv("KRY_DIA_GRID");  // tuning override: grid cap
        return e ? std::max(1, std::min(atoi(e), kMaxGridBlk)) : 0;
      }();
      const int dia_cap = dia_cap_env ? dia_cap_env : (A->dia_max_width > 8 ? kMaxGridBlk : kMaxGrid);
      grid = (int)std::max<int64_t>(1, std::min<int64_t>(dia_cap, (A->dia_nslices + 3) / 4));
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, st, static_cast<const int64_t *>(A->dia_sptr),
                           static_cast<const int *>(A->dia_width), static_cast<const int *>(A->dia_off),
                           static_cast<const uint64_t *>(A->dia_mask), static_cast<const MV *>(A->dia_val),
                           A->dia_nslices, A->n, src, epi, part, ctrl, step);
      };
      if (A->dia_max_width <= 8) go(spmv_dia_kernel<V, MV, 8, Src, Epi>);
      else go(spmv_dia_kernel<V, MV, 16, Src, Epi>);
      KRY_HIP(hipGetLastError());
      if (grid_out) *grid_out = grid;
      return;
    }
    constexpr int CPLB = 16 / (int)sizeof(V);  // columns per lane of the block DIA kernel
    if (k >= CPLB && k <= 8 && A->dia && !dia_blk_off()) {
      // one slice per wave (partial buffers hold part_rows(k) = kMaxGridBlk rows for k <= 8)
      grid = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxGridBlk, (A->dia_nslices + 3) / 4));
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, st, static_cast<const int64_t *>(A->dia_sptr),
                           static_cast<const int *>(A->dia_width), static_cast<const int *>(A->dia_off),
                           static_cast<const uint64_t *>(A->dia_mask), static_cast<const MV *>(A->dia_val),
                           A->dia_nslices, A->n, k, src, epi, part, ctrl, step);
      };
      // NG = 128 / (64 / (k / CPLB)) = 2 k / CPLB row groups per slice
      switch (k / CPLB) {
        case 1: go(spmv_dia_blk_kernel<V, MV, CPLB, 2, Src, Epi>); break;
        case 2: go(spmv_dia_blk_kernel<V, MV, CPLB, 4, Src, Epi>); break;
        default: go(spmv_dia_blk_kernel<V, MV, CPLB, 8, Src, Epi>); break;
      }
      KRY_HIP(hipGetLastError());
      if (grid_out) *grid_out = grid;
      return;
    }
    if (k == 1 && A->cb_nb > 0) {
      // one launch per range of kCbPersistGrid * kCbMaxOwn groups (one for n
      // up to 4.2 M); launch l writes its block partials (every block writes
      // one, 0 without groups) at part + l * grid: at most 32 launches
      // (cb_build refuses more), so they fit the kMaxGridBlk partial rows
      const int64_t per = (int64_t)kCbPersistGrid * kCbMaxOwn;
      grid = (int)std::min<int64_t>(A->cb_ng, kCbPersistGrid);
      int nl = 0;
      for (int64_t g0 = 0; g0 < A->cb_ng; g0 += per, ++nl) {
        const int64_t g1 = std::min<int64_t>(A->cb_ng, g0 + per);
        double *pl = part ? part + (int64_t)nl * grid : nullptr;
        auto go = [&](auto kern) {
          hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, st, (int)A->cb_nb, A->n, A->cb_ng, g0, g1,
                             static_cast<const int64_t *>(A->cb_gptr), static_cast<const uint16_t *>(A->cb_roff),
                             static_cast<const int *>(A->cb_col), static_cast<const MV *>(A->cb_val), src, epi, pl,
                             ctrl, step);
        };
        if (cb_vec()) go(spmv_cbp_kernel<true, V, MV, Src, Epi>);
        else go(spmv_cbp_kernel<false, V, MV, Src, Epi>);
      }
      KRY_HIP(hipGetLastError());
      if (grid_out) *grid_out = grid * nl;
      return;
    }
  }
  if (k >= 4 && k <= 64) {
    grid = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxGrid, (A->nslices + 3) / 4));
    const bool d16 = sizeof(I) == 4 && A->compact;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, st, static_cast<const int64_t *>(A->sptr),
                         static_cast<const int *>(A->swidth), static_cast<const I *>(A->sidx),
                         static_cast<const uint16_t *>(A->sdelta), static_cast<const int *>(A->scbase),
                         static_cast<const MV *>(A->sval), A->nslices, A->n, k, static_cast<const I *>(A->indptr),
                         static_cast<const I *>(A->indices), static_cast<const MV *>(A->data), src, epi, part, ctrl,
                         step);
    };
    if (d16) go(spmv_sell_lg_kernel<V, MV, I, 4, 8, true, Src, Epi>);
    else go(spmv_sell_lg_kernel<V, MV, I, 4, 8, false, Src, Epi>);
    KRY_HIP(hipGetLastError());
    if (grid_out) *grid_out = grid;
    return;
  }
  switch (k) {
    case 1:  // one pass over a slice's slot columns when they all fit the unroll
      grid = A->max_width <= 8 ? launch_sell<V, MV, I, 1, 8>(A, k, src, epi, part, ctrl, step, st)
                               : launch_sell<V, MV, I, 1, 16>(A, k, src, epi, part, ctrl, step, st);
      break;
    case 2: grid = launch_sell<V, MV, I, 2, 8>(A, k, src, epi, part, ctrl, step, st); break;
    case 4: grid = launch_sell<V, MV, I, 4, 4>(A, k, src, epi, part, ctrl, step, st); break;
    default: grid = launch_sell<V, MV, I, 8, 4>(A, k, src, epi, part, ctrl, step, st); break;
  }
  KRY_HIP(hipGetLastError());
  if (grid_out) *grid_out = grid;
}

// SpMV with an operator of any stored type (preconditioners M, Ml, Mr): the
// matrix value type may be float under double vectors (exact upcast).
template <typename V, class Src, class Epi>
void launch_spmv_any(const kry_csr *Op, int k, Src src, Epi epi, double *part, int *grid_out, const Ctrl *ctrl,
                     int step, hipStream_t st) {
  const bool f64 = Op->dtype == KRY_F64, i32 = Op->itype == KRY_I32;
  if constexpr (std::is_same<V, double>::value) {
    if (f64 && i32) return launch_spmv<V, double, int32_t>(Op, k, src, epi, part, grid_out, ctrl, step, st);
    if (f64) return launch_spmv<V, double, int64_t>(Op, k, src, epi, part, grid_out, ctrl, step, st);
  } else {
    KRY_REQUIRE(!f64, KRY_EINVAL, "a float64 operator cannot act on float32 vectors");
  }
  if (i32) return launch_spmv<V, float, int32_t>(Op, k, src, epi, part, grid_out, ctrl, step, st);
  return launch_spmv<V, float, int64_t>(Op, k, src, epi, part, grid_out, ctrl, step, st);
}

template <typename V, class Op>
int launch_elementwise(int64_t N, int k, Op op, double *part, const Ctrl *ctrl, int step,
                       hipStream_t st, int max_grid = kMaxGrid) {
  constexpr int W = Vec16<V>::W;
  int grid = grid_for((N + W - 1) / W, kBlock * 2);
  if (grid > max_grid) grid = max_grid;
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
