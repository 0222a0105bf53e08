// Pieces shared by the CG / GMRES / MINRES device loops.
#pragma once

#include <climits>

#include <rccl/rccl.h>

#include "device.hpp"

struct kry_comm {
  kry_ctx *ctx = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  double *dbuf = nullptr;  // scratch for host allreduces
  int dbuf_len = 0;
};

namespace kry {

// guarded divisor, np.where(d != 0, d, 1.0)
template <typename S>
__device__ __forceinline__ S safe(S d) {
  return d != S(0) ? d : S(1);
}

// Column-wise convergence test np.all(resnorm <= criterion) over `count`
// columns held in slots[0..count) by the first `count` threads. All threads
// of the block must call it; returns the same answer in every thread.
__device__ __forceinline__ bool all_le(const double *vals, const double *crit, int count, int *flag) {
  if (threadIdx.x == 0) *flag = 1;
  __syncthreads();
  for (int c = threadIdx.x; c < count; c += blockDim.x)
    if (!(vals[c] <= crit[c])) *flag = 0;
  __syncthreads();
  const bool r = *flag != 0;
  __syncthreads();
  return r;
}

// Host helper: reset the control word to "run everything".
inline void reset_ctrl(Ctrl *d_ctrl, hipStream_t st) {
  static const Ctrl fresh = {INT_MAX, 0, 0, 0};
  KRY_HIP(hipMemcpyAsync(d_ctrl, &fresh, sizeof(Ctrl), hipMemcpyHostToDevice, st));
}

inline void check_vec(const kry_vec *v, int64_t n, int k, int dtype, const char *what) {
  KRY_REQUIRE(v != nullptr, KRY_EINVAL, std::string("null ") + what);
  KRY_REQUIRE(v->n == n && v->k == k && v->dtype == dtype, KRY_EINVAL,
              std::string(what) + ": shape/dtype mismatch with the solver");
}

inline void check_weights(const kry_vec *w, int64_t n) {
  KRY_REQUIRE(!w || (w->n == n && w->k == 1 && w->dtype == KRY_F64), KRY_EINVAL,
              "inner-product weights must be an (n,) float64 vector");
}

// xk = x0 + y (cg.py:59-66 _get_xk / minres.py:95-98); x0 == null means the
// reference's zeros_like(b), i.e. 0.0 + y (which maps -0.0 to +0.0).
template <typename V>
struct OpXk {
  const V *x0;
  const V *y;
  V *xk;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V a[W], b[W];
    VIO<V>::load(y, e, N, b);
    if (x0) {
      VIO<V>::load(x0, e, N, a);
    } else {
#pragma unroll
      for (int v = 0; v < W; ++v) a[v] = V(0);
    }
#pragma unroll
    for (int v = 0; v < W; ++v) a[v] = a[v] + b[v];
    VIO<V>::store(xk, e, N, a);
  }
};

template <typename V>
struct OpCopy {
  const V *src;
  V *dst;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V a[W];
    VIO<V>::load(src, e, N, a);
    VIO<V>::store(dst, e, N, a);
  }
};

}  // namespace kry
