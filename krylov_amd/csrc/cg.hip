// CG device loop (reference cg.py:16-259). Preconditioners M and Ml are
// device CSR operators (kry_cg_set_preconditioners); without them the loop is
// the five launches below. With Ml, step 1 is A p then Ml (A p); with M, the
// update's <r, r> partials are replaced by z = M r with <r, z> (cg.py:207-209)
// and the p pass reads z.
//
// One iteration (no M, k <= 8) = four launches on the context stream, no
// host sync:
//   1. SpMV   Ap = A p, partial <p, Ap>                 cg.py:180-183
//   2. tiny   alpha = rho / guard(<p, Ap>)              cg.py:185
//   3. r pass r -= alpha Ap, partial <r, r>             cg.py:200-209
//   4. yp     every block finishes <r, r> itself: omega; y += alpha p and
//             p = r + omega p for the next iteration; block 0 shifts rho,
//             writes resnorm = sqrt(rho) to the history and the stop test
//             np.all(resnorm <= criterion) -> ctrl.stop_at
//                                                       cg.py:156,175-178,196,214-217
// With M (or k > 8) steps 3-4 are the update pass (y and r), z = M r, a
// one-block rho kernel and a p pass.
// (+ with an attached communicator: one ncclAllReduce of the zero-padded
//  residual-norm vector and a tiny global stop test.)
// The p update is its own streaming pass (not folded into the SpMV's gather):
// the SpMV then gathers one vector instead of two, which is what bounds it.
#include <string>
#include <tuple>
#include <utility>

#include "solver_common.hpp"

using namespace kry;

struct kry_cg {
  kry_ctx *ctx = nullptr;
  kry_csr *A = nullptr;
  int64_t n = 0;
  int k = 1;
  int dtype = 0;
  bool scalar_f32 = false;
  void *b = nullptr, *x0 = nullptr, *y = nullptr, *r = nullptr, *p = nullptr;
  void *Ap = nullptr, *xk = nullptr, *rt = nullptr;
  kry_csr *M = nullptr, *Ml = nullptr;  // preconditioners (null = identity)
  void *z = nullptr;                    // M Ml_r (with M)
  void *t = nullptr;                    // A p / scratch (with Ml)
  double *w = nullptr;
  double *part = nullptr;  // 2 * part_rows(k) * k
  double *scal = nullptr;  // scalar slots, see S_* below
  double *hist = nullptr;  // chunk_cap * hist_k
  Ctrl *ctrl = nullptr;
  int chunk_cap = 0;
  int64_t it = 0;
  // deferred yk (ydefer = D > 0): the ring is indexed by the GLOBAL step
  // (p_g in pring[g % (D + 1)], alpha_g in alpha_ring[g % D]) across run
  // calls, so a chunk's end costs nothing: y holds every update below yfb,
  // the in-kernel flushes fall every D steps from yfb, and the ones pending
  // at a chunk's end are applied only when the host needs y (cg_ydefer_flush:
  // kry_cg_get x, kry_cg_residual). it_base: the global step of a run's step 0
  int64_t yfb = 0;
  int64_t it_base = 0;
  bool started = false;
  // multi-GPU
  kry_comm *comm = nullptr;
  int col_offset = 0, total_k = 0;
  double *gbuf = nullptr;  // total_k + 1 (allreduced residual norms, fault count)
  double *gcrit = nullptr; // total_k
  // persistent small-n loop (cg_persist_kernel): its scratch r, two p
  // buffers, the y output, the scalar staging slots, barrier and granule
  // words; cgp_spw = -1 undecided, 0 not used, else slices/wave. The kernel
  // never writes the solver's own y, r, p or scalar slots: after a clean
  // chunk the host swaps the buffers in, after a timed-out one it keeps the
  // chunk-start state and reruns the chunk on the launch-per-pass path.
  void *rs = nullptr, *pb = nullptr, *pb2 = nullptr, *yb = nullptr;
  double *cgp_scal = nullptr;  // S_COUNT slots
  unsigned *cgp_words = nullptr;
  int cgp_spw = -1;
  int cgp_fallbacks = 0;  // chunks rerun on the launch-per-pass path after a timeout
  bool cgp_last = false;  // the last kry_cg_run chunk ran the persistent loop
  // one-launch update (cg_upd_kernel): upd_nv = -1 undecided, 0 not used,
  // else granules per thread; its abort word and granule region
  int upd_nv = -1;
  unsigned *upd_words = nullptr;
  int upd_fallbacks = 0;
  bool upd_used = false;  // an update kernel was launched in the current chunk
  bool upd_last = false;  // ... in the last kry_cg_run chunk
  // block right-hand sides on the separate passes: yk += alpha p (cg.py:196)
  // deferred and applied ydefer steps at a time (cg_pdefer_kernel, then
  // cg_yflush at the chunk's end), p_i in pring[i % (ydefer + 1)] within a
  // chunk (pring[0] is p). ydefer = -1 undecided, 0 not used.
  int ydefer = -1;
  void *pring[33] = {};  // [1 .. ydefer] allocated (kCgYDeferMax = 31 at most)
  double *alpha_ring = nullptr;  // ydefer x k: alpha of step j at row j % ydefer
  int64_t ydefer_bytes = 0;      // what the rings hold (kry_cg_defer_info)
};

namespace {

enum { S_RHO = 0, S_RHO_PREV = 1, S_ALPHA = 2, S_OMEGA = 3, S_CRIT = 4, S_TMP = 5, S_RHO_OLD = 6, S_COUNT = 7 };

constexpr int kCgUpdateGrid = 1024;  // update-pass blocks: the <r, r> partials every yp block re-reduces
constexpr size_t kCgYDeferBudget = size_t(10) << 30;  // default ring budget (bytes)
constexpr int kCgYDefer = 7;         // deferred yk updates per flush: the policy tries 31, 15, 7, 3 (KRY_CG_YDEFER)
constexpr int kCgYDeferMax = 31;     // the ring holds at most 32 p buffers

template <typename V>
struct OpCgUpdate {
  V *y, *r;
  const V *p, *Ap;
  const double *alpha;
  const double *w;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&acc)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V yv[W], rv[W], pv[W], av[W];
    VIO<V>::load_nt(y, e, N, yv);   // y and Ap: streamed once per iteration
    VIO<V>::load(r, e, N, rv);
    VIO<V>::load(p, e, N, pv);
    VIO<V>::load_nt(Ap, e, N, av);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const V a = (V)alpha[(e + v) & (k - 1)];
      const V t1 = a * pv[v];
      yv[v] = yv[v] + t1;        // yk += alpha * p        (cg.py:196)
      const V t2 = a * av[v];
      rv[v] = rv[v] - t2;        // Ml_rk -= alpha * Ap    (cg.py:200)
      if (e + v < N) {
        const double rd = (double)rv[v];
        acc[v] += w ? dterm_w(rd, w[(e + v) / k], rd) : dterm(rd, rd);
      }
    }
    VIO<V>::store_nt(y, e, N, yv);
    VIO<V>::store(r, e, N, rv);  // r and p are the next SpMV's gather sources
  }
};

// Ml_rk -= alpha * Ap (cg.py:200) with <r, r> partials (cg.py:209); the y
// update moves to the yp pass, which reads p anyway.
template <typename V>
struct OpCgR {
  V *r;
  const V *Ap;
  const double *alpha;
  const double *w;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&acc)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V rv[W], av[W];
    VIO<V>::load(r, e, N, rv);
    VIO<V>::load_nt(Ap, e, N, av);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const V a = (V)alpha[(e + v) & (k - 1)];
      const V t2 = a * av[v];
      rv[v] = rv[v] - t2;
      if (e + v < N) {
        const double rd = (double)rv[v];
        acc[v] += w ? dterm_w(rd, w[(e + v) / k], rd) : dterm(rd, rd);
      }
    }
    VIO<V>::store(r, e, N, rv);
  }
};

// p = r + omega * p, in place (cg.py:178 with M = I: p = MPr + omega p).
template <typename V>
struct OpCgP {
  V *p;
  const V *r;
  const double *omega;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&acc)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V pv[W], rv[W];
    VIO<V>::load(p, e, N, pv);
    VIO<V>::load(r, e, N, rv);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const V om = (V)omega[(e + v) & (k - 1)];
      const V t = om * pv[v];
      pv[v] = rv[v] + t;
    }
    VIO<V>::store(p, e, N, pv);
  }
};

// rho0 = <r0, r0> -> rho slot (cg.py:116, 131).
template <typename S>
__global__ void cg_start_finalize(const double *part, int P, int k, double *scal) {
  __shared__ double red[kBlock];
  reduce_partials(part, P, k, red);
  const int c = threadIdx.x;
  if (c < k) {
    const S rho = (S)red[c];
    scal[S_RHO * k + c] = (double)rho;
    scal[S_RHO_PREV * k + c] = 0.0;
    scal[S_OMEGA * k + c] = 0.0;
    scal[S_TMP * k + c] = (double)rho;
  }
}

// alpha = rhos[-1] / np.where(pAp != 0, pAp, 1.0)  (cg.py:183-185)
// 1024 threads: the SpMV's partials (up to part_rows(k) blocks x k) in 32-load rounds
constexpr int kAlphaBlock = 1024;
template <typename S>
__global__ __launch_bounds__(kAlphaBlock) void cg_alpha_kernel(const double *part, int P, int k, double *scal,
                                                               const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kAlphaBlock];
  reduce_partials<kAlphaBlock>(part, P, k, red);
  const int c = threadIdx.x;
  if (c < k) {
    const S pAp = (S)red[c];
    const S rho = (S)scal[S_RHO * k + c];
    scal[S_ALPHA * k + c] = (double)(rho / safe<S>(pAp));
    scal[S_RHO_OLD * k + c] = (double)rho;  // stable copy for the yp pass (S_RHO is rewritten there)
  }
}

// First stage of the alpha reduction when the SpMV left many block partials
// (the block DIA kernel at cfg4: 19,541 rows of k): block b sums rows
// [b P / G, (b + 1) P / G) in reduce_partials' fixed order into row b of
// `out`, so the one-block alpha kernel sums G rows instead of P (one block
// reading 1.25 MB took 29 us per iteration, profiles/r03_bench_kernel_stats.csv).
constexpr int kAlphaStage = 128;
__global__ __launch_bounds__(kBlock) void partial_stage_kernel(const double *part, int P, int k, double *out,
                                                               const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  const int r0 = (int)((int64_t)blockIdx.x * P / gridDim.x), r1 = (int)((int64_t)(blockIdx.x + 1) * P / gridDim.x);
  reduce_partials(part + (int64_t)r0 * k, r1 - r0, k, red);
  if ((int)threadIdx.x < k) out[(int64_t)blockIdx.x * k + threadIdx.x] = red[threadIdx.x];
}

// rhos = [rhos[-1], <r, r>]; omega for the next p-update; resnorm =
// sqrt(<r, r>); global stop test (cg.py:209-217, 156, 177).
template <typename S>
__global__ void cg_rho_kernel(const double *part, int P, int k, double *scal, double *hist, Ctrl *ctrl,
                              int step, double *gbuf, int col_offset, int total_k) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  __shared__ double rn[kMaxCols];
  __shared__ int flag;
  reduce_partials(part, P, k, red);
  const int c = threadIdx.x;
  if (c < k) {
    const S rr = (S)red[c];
    const S old = (S)scal[S_RHO * k + c];
    scal[S_RHO_PREV * k + c] = (double)old;
    scal[S_RHO * k + c] = (double)rr;
    scal[S_OMEGA * k + c] = (double)(rr / safe<S>(old));
    const S nrm = sqrt(rr);
    rn[c] = (double)nrm;
    if (!gbuf) hist[(int64_t)step * k + c] = (double)nrm;
  }
  __syncthreads();
  if (gbuf) {
    // zero-padded residual-norm vector for the RCCL allreduce
    for (int t = threadIdx.x; t <= total_k; t += blockDim.x) {  // + the fault slot (0)
      const int lc = t - col_offset;
      gbuf[t] = (lc >= 0 && lc < k) ? rn[lc] : 0.0;
    }
    return;
  }
  if (all_le(rn, scal + S_CRIT * k, k, &flag) && threadIdx.x == 0) ctrl->stop_at = step + 1;
}

// global stop test on the allreduced residual norms (slot total_k: the fault
// count, post_fault)
__global__ void cg_global_check(const double *gbuf, const double *gcrit, int total_k, double *hist, Ctrl *ctrl,
                                int step) {
  if (halted(ctrl, step)) return;
  if (peer_fault(gbuf, total_k + 1, ctrl, step)) return;
  __shared__ int flag;
  for (int t = threadIdx.x; t < total_k; t += blockDim.x) hist[(int64_t)step * total_k + t] = gbuf[t];
  if (all_le(gbuf, gcrit, total_k, &flag) && threadIdx.x == 0) ctrl->stop_at = step + 1;
}

// Ml r and M Ml r with <Ml r, M Ml r> partials for r = b - A src
// (cg.py:70-90); returns the partial count. Leaves Ml r in `mlr` and M Ml r in
// `z` (when M is set).
// Steps 4-5 fused (no preconditioner): every block finishes <r, r> from the
// update pass's partials in the same fixed order, derives omega, and applies
// yk += alpha p (cg.py:196) and p = r + omega p (cg.py:178) to its span; block
// 0 also shifts rho, writes the history and the stop word (cg.py:156,
// 209-217). Saves the one-block rho launch and one pass over p.
template <typename V, typename S>
__global__ __launch_bounds__(kBlock) void cg_yp_kernel(int64_t N, int k, V *__restrict__ y, V *__restrict__ p,
                                                       const V *__restrict__ r, const double *__restrict__ part,
                                                       int P, double *scal, double *hist, Ctrl *ctrl, int step,
                                                       double *gbuf, int col_offset, int total_k) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  __shared__ double red[kBlock];
  __shared__ double sh_a[kMaxCols], sh_om[kMaxCols], rn[kMaxCols];
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  reduce_partials(part, P, k, red);
  if (tid < k) {
    const S rr = (S)red[tid];
    const S old = (S)scal[S_RHO_OLD * k + tid];
    const S om = rr / safe<S>(old);
    sh_om[tid] = (double)om;
    sh_a[tid] = scal[S_ALPHA * k + tid];
    const S nrm = sqrt(rr);
    rn[tid] = (double)nrm;
    if (g == 0) {
      scal[S_RHO_PREV * k + tid] = (double)old;
      scal[S_RHO * k + tid] = (double)rr;
      scal[S_OMEGA * k + tid] = (double)om;
      if (!gbuf) hist[(int64_t)step * k + tid] = (double)nrm;
    }
  }
  __syncthreads();
  const int64_t ngrp = (N + W - 1) / W;
  const int64_t per = ((ngrp + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
  const int64_t v0 = per * g;
  const int64_t v1 = v0 + per < ngrp ? v0 + per : ngrp;
  for (int64_t gi = v0 + tid; gi < v1; gi += kBlock) {
    const int64_t e = gi * W;
    V yv[W], pv[W], rv[W];
    VIO<V>::load_nt(y, e, N, yv);
    VIO<V>::load(p, e, N, pv);
    VIO<V>::load(r, e, N, rv);
#pragma unroll
    for (int u = 0; u < W; ++u) {
      const int c = (int)((e + u) & (k - 1));
      const V a = (V)sh_a[c];
      const V t1 = a * pv[u];
      yv[u] = yv[u] + t1;
      const V om = (V)sh_om[c];
      const V t = om * pv[u];
      pv[u] = rv[u] + t;
    }
    VIO<V>::store_nt(y, e, N, yv);
    VIO<V>::store(p, e, N, pv);
  }
  if (g == 0) {
    if (gbuf) {
      for (int t = tid; t <= total_k; t += kBlock) {  // + the fault slot (0)
        const int lc = t - col_offset;
        gbuf[t] = (lc >= 0 && lc < k) ? rn[lc] : 0.0;
      }
    } else if (all_le(rn, scal + S_CRIT * k, k, &flag) && tid == 0) {
      ctrl->stop_at = step + 1;
    }
  }
}

// The yp pass with yk += alpha p deferred (block right-hand sides, separate
// passes): step i computes omega from the <r, r> partials exactly as
// cg_yp_kernel does, records alpha_i in alpha_ring, and writes p_{i+1} = r +
// omega p_i (cg.py:178) into the next ring buffer; every D-th step it also
// applies the D deferred updates yk += alpha_j p_j (cg.py:196), j = i - D + 1
// .. i, in that order (the same sequence of roundings as one update per
// step: bitwise the same yk). Per D steps the passes read and write yk once
// instead of D times: 3 vectors per step and D + 4 on the flushing one,
// against 5 per step.
template <typename V>
struct PRing {
  V *s[kCgYDeferMax + 1];
};

template <typename V, typename S, bool FLUSH>
__global__ __launch_bounds__(kBlock) void cg_pdefer_kernel(int64_t N, int k, V *__restrict__ y, PRing<V> ring, int D,
                                                           const V *__restrict__ r, const double *__restrict__ part,
                                                           int P, double *scal, double *alpha_ring, double *hist,
                                                           Ctrl *ctrl, int step, double *gbuf, int col_offset,
                                                           int total_k, int64_t gstep, int64_t fb) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  __shared__ double red[kBlock];
  __shared__ double sh_a[kCgYDeferMax][8];  // alpha of the flushed steps, oldest first (k <= 8 on this path)
  __shared__ double sh_om[kMaxCols], rn[kMaxCols];
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  // gstep: this step's global index; flushes fall every D steps from fb (the
  // host picks FLUSH by the same rule, so the common step carries no flush code)
  const int nf = FLUSH ? D : 0;
  reduce_partials(part, P, k, red);
  if (tid < k) {
    const S rr = (S)red[tid];
    const S old = (S)scal[S_RHO_OLD * k + tid];
    const S om = rr / safe<S>(old);
    sh_om[tid] = (double)om;
    const double a = scal[S_ALPHA * k + tid];
    for (int q = 0; q + 1 < nf; ++q) sh_a[q][tid] = alpha_ring[((gstep - nf + 1 + q) % D) * k + tid];
    if (nf) sh_a[nf - 1][tid] = a;
    const S nrm = sqrt(rr);
    rn[tid] = (double)nrm;
    if (g == 0) {
      alpha_ring[(gstep % D) * k + tid] = a;
      scal[S_RHO_PREV * k + tid] = (double)old;
      scal[S_RHO * k + tid] = (double)rr;
      scal[S_OMEGA * k + tid] = (double)om;
      if (!gbuf) hist[(int64_t)step * k + tid] = (double)nrm;
    }
  }
  __syncthreads();
  const V *pi = ring.s[gstep % (D + 1)];
  V *pn = ring.s[(gstep + 1) % (D + 1)];
  const int64_t ngrp = (N + W - 1) / W;
  const int64_t per = ((ngrp + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
  const int64_t v0 = per * g;
  const int64_t v1 = v0 + per < ngrp ? v0 + per : ngrp;
  for (int64_t gi = v0 + tid; gi < v1; gi += kBlock) {
    const int64_t e = gi * W;
    V pv[W], rv[W];
    VIO<V>::load(pi, e, N, pv);
    VIO<V>::load(r, e, N, rv);
    if constexpr (FLUSH) {
      V yv[W];
      VIO<V>::load_nt(y, e, N, yv);
      for (int q = 0; q < nf; ++q) {
        V pj[W];
        if (q + 1 < nf) VIO<V>::load_nt(ring.s[(gstep - nf + 1 + q) % (D + 1)], e, N, pj);
#pragma unroll
        for (int u = 0; u < W; ++u) {
          const V a = (V)sh_a[q][(int)((e + u) & (k - 1))];
          const V t1 = a * (q + 1 < nf ? pj[u] : pv[u]);
          yv[u] = yv[u] + t1;  // yk += alpha_j p_j (cg.py:196), j ascending
        }
      }
      VIO<V>::store_nt(y, e, N, yv);
    }
#pragma unroll
    for (int u = 0; u < W; ++u) {
      const V om = (V)sh_om[(int)((e + u) & (k - 1))];
      const V t = om * pv[u];
      pv[u] = rv[u] + t;  // p = r + omega p (cg.py:178)
    }
    VIO<V>::store(pn, e, N, pv);
  }
  if (g == 0) {
    if (gbuf) {
      for (int t = tid; t <= total_k; t += kBlock) {  // + the fault slot (0)
        const int lc = t - col_offset;
        gbuf[t] = (lc >= 0 && lc < k) ? rn[lc] : 0.0;
      }
    } else if (all_le(rn, scal + S_CRIT * k, k, &flag) && tid == 0) {
      ctrl->stop_at = step + 1;
    }
  }
}

// yk += alpha_j p_j for global steps j = j0 .. j1 - 1 in order (cg.py:196):
// the deferred updates of a flushing step of the one-launch update path, and
// those pending when the host needs y (cg_ydefer_flush).
template <typename V>
struct OpCgYSteps {
  V *y;
  PRing<V> ring;
  int D;
  const double *alpha_ring;
  int64_t j0, j1;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V yv[W];
    VIO<V>::load_nt(y, e, N, yv);
    for (int64_t j = j0; j < j1; ++j) {
      V pj[W];
      VIO<V>::load_nt(ring.s[j % (D + 1)], e, N, pj);
#pragma unroll
      for (int u = 0; u < W; ++u) {
        const V a = (V)alpha_ring[(int64_t)(j % D) * k + (int)((e + u) & (k - 1))];
        const V t1 = a * pj[u];
        yv[u] = yv[u] + t1;
      }
    }
    VIO<V>::store_nt(y, e, N, yv);
  }
};

// ------------------------------------- one-launch CG update (large n, k = 1)
// Replaces the alpha kernel, the r pass and the fused rho / y / p pass of an
// iteration for one right-hand side, no M / Ml, Euclidean inner and n up to
// 512 * 40 * 2 per block at one 512-thread block per CU (n = 10.5 M doubles),
// with the same scalar arithmetic (one launch of at most one block per CU,
// all resident):
//   alpha = rho / guard(<p, Ap>)  (every block sums the SpMV's partials in
//                                  the alpha kernel's fixed order)
//   r' = r - alpha Ap, <r', r'>   (r' kept in registers; block partial)
//   all-gather of the block partials -> rho' = <r', r'>, omega = rho' / guard(rho)
//   y += alpha p, p = r' + omega p; y, p and r' stored
// so an iteration streams Ap, r, y, p in and r, y, p out (7 vectors, the
// launch-per-pass form moves 8: r twice) with one kernel boundary instead of
// three. Nothing is stored before the exchange has completed: a timed-out
// exchange (a block not resident) leaves the iteration's state untouched, the
// kernel halts the chunk at this step and kry_cg_run reruns it launch per
// pass. A block that comes late to a finished exchange re-checks the abort
// word before it writes anything.
constexpr int kUpdBlock = 512;
constexpr int kUpdU = 2;  // granules per streamed chunk
constexpr size_t kUpdWords = 16 + 2 * 2 * 256 * 2;  // abort word area + two parity regions of G <= 256 granule pairs
// DEF (deferred yk, see cg_pdefer_kernel): y is neither read nor written,
// p_{i+1} goes to pout (the next ring buffer) and alpha to alpha_ring[step %
// D]; 5 vectors per iteration, the yk updates applied D steps at a time by
// OpCgYSteps.
template <typename V, typename S, int NV, bool DEF>
__global__ __launch_bounds__(kUpdBlock) void cg_upd_kernel(int64_t N, V *__restrict__ y, V *__restrict__ r,
                                                           V *__restrict__ p, const V *__restrict__ Ap,
                                                           const double *__restrict__ partA, int PA, double *scal,
                                                           double *hist, Ctrl *ctrl, int step, double *gbuf,
                                                           int col_offset, int total_k, unsigned *words,
                                                           int fault_step, V *__restrict__ pout,
                                                           double *__restrict__ alpha_ring, int D) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  constexpr int U = kUpdU;
  constexpr int NC = NV / U;
  static_assert(NV % U == 0, "chunks must tile the thread's granules");
  __shared__ double red[kUpdBlock];
  __shared__ double shv[2];
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  if (fault_step >= 0 && (fault_step & 0xffff) == step && (int)blockIdx.x == G - 1) {
    // fault injection (tests, KRY_CGU_FAULT): the last block drops out, or, with
    // KRY_CGU_FAULT_LATE = L, joins the exchange L x 0.25 ms late (the others' spin
    // gives up after kSpinLimitFault = 1 ms: either outcome must be consistent)
    const unsigned late = (unsigned)fault_step >> 16;
    if (late == 0) return;
    const unsigned long long t0 = wall_clock64();
    while (!spin_expired(t0, late * (kSpinLimitFault / 4))) __builtin_amdgcn_s_sleep(8);
  }
  const unsigned spin_limit = fault_step >= 0 ? kSpinLimitFault : kSpinLimit;
  const int64_t seg = (int64_t)NV * kUpdBlock * W;
  const int64_t e0 = (int64_t)blockIdx.x * seg;
  const BufSeg<V, kUpdBlock> sr(r, e0, N, seg), sa(Ap, e0, N, seg), sy(y, e0, N, seg), sp(p, e0, N, seg),
      spo(pout, e0, N, seg);
  V ca[2][U][W], cb[2][U][W];
  auto ld2 = [&](const BufSeg<V, kUpdBlock> &s1, const BufSeg<V, kUpdBlock> &s2, int c, V(&d1)[U][W],
                 V(&d2)[U][W]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s1.template load<W>(c * U + u, d1[u]);
      s2.template load<W, 2>(c * U + u, d2[u]);  // second stream (Ap / p... see callers) nontemporal
    }
  };
  ld2(sr, sa, 0, ca[0], cb[0]);  // chunk 0 of r and Ap travels during the alpha reduction
  // alpha = rho / guard(<p, Ap>)  (cg.py:183-185), same order as cg_alpha_kernel
  reduce_partials<kUpdBlock>(partA, PA, 1, red);
  const S rho = (S)scal[S_RHO];
  const S alpha = rho / safe<S>((S)red[0]);
  const V a = (V)alpha;
  // r' = r - alpha Ap (cg.py:200) and <r', r'>
  V rr[NV][W];
  double acc = 0.0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int b = c & 1;
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 < NC) ld2(sr, sa, c + 1, ca[b ^ 1], cb[b ^ 1]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int g = c * U + u;
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const V t2 = a * cb[b][u][v];
        rr[g][v] = ca[b][u][v] - t2;
        const double rd = (double)rr[g][v];
        acc += dterm(rd, rd);  // out-of-range elements are 0: they add 0
      }
    }
  }
  const double bp = block_sum1_t0(acc, red);
  unsigned long long *gran = reinterpret_cast<unsigned long long *>(words + 16) + (size_t)(step & 1) * 2 * 256;
  const unsigned tag = (unsigned)step + 1u;
  if (tid == 0) publish_partial(gran + 2 * blockIdx.x, tag, bp);
  auto ld1 = [&](int c, V(&d1)[U][W]) {
#pragma unroll
    for (int u = 0; u < U; ++u) sp.template load<W>(c * U + u, d1[u]);
  };
  if constexpr (DEF) ld1(0, ca[0]);
  else ld2(sp, sy, 0, ca[0], cb[0]);  // chunk 0 of p and y travels during the exchange
  if (tid < 64) {
    // every block commits or every block aborts (decide_exchange): no block
    // stores its segment after another gave up
    const bool ok = sweep_partials<true>(gran, G, tag, words, ctrl, &shv[0], spin_limit);
    if (tid == 0) flag = ok ? 1 : 0;
  }
  __syncthreads();
  if (!__builtin_amdgcn_readfirstlane(flag)) {
    if (tid == 0) atomicMin(&ctrl->stop_at, step);
    if (gbuf && blockIdx.x == 0) post_fault(gbuf, total_k + 1);  // sharded: tell the other ranks
    return;
  }
  const S rrs = (S)shv[0];
  const S om = rrs / safe<S>(rho);  // omega = rhos[-1] / rhos[-2] (cg.py:177)
  const V o = (V)om;
  // y += alpha p (cg.py:196), p = r' + omega p (cg.py:178); y, p, r' stored
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int b = c & 1;
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 < NC) {
      if constexpr (DEF) ld1(c + 1, ca[b ^ 1]);
      else ld2(sp, sy, c + 1, ca[b ^ 1], cb[b ^ 1]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int g = c * U + u;
      V yv[W], pv[W];
#pragma unroll
      for (int v = 0; v < W; ++v) {
        if constexpr (!DEF) {
          const V t1 = a * ca[b][u][v];
          yv[v] = cb[b][u][v] + t1;
        }
        const V t = o * ca[b][u][v];
        pv[v] = rr[g][v] + t;
      }
      if constexpr (DEF) {
        spo.template store<W>(g, pv);
      } else {
        sy.template store<W, 2>(g, yv);
        sp.template store<W>(g, pv);
      }
      sr.template store<W>(g, rr[g]);
    }
  }
  if (blockIdx.x == 0) {
    if (tid == 0) {
      if (DEF) alpha_ring[0] = (double)alpha;  // the host passes this step's slot
      scal[S_ALPHA] = (double)alpha;
      scal[S_RHO_OLD] = (double)rho;
      scal[S_RHO_PREV] = (double)rho;
      scal[S_RHO] = (double)rrs;
      scal[S_OMEGA] = (double)om;
      const double nrm = (double)sqrt(rrs);
      red[0] = nrm;
      if (!gbuf) hist[step] = nrm;
    }
    __syncthreads();
    if (gbuf) {
      for (int t = tid; t <= total_k; t += kUpdBlock) gbuf[t] = t == col_offset ? red[0] : 0.0;  // + fault slot
    } else if (all_le(red, scal + S_CRIT, 1, &flag) && tid == 0) {
      ctrl->stop_at = step + 1;
    }
  }
}

// ------------------------------------- persistent CG for launch-bound sizes
// One launch runs a whole chunk of iterations of the fused path (no M / Ml,
// one RHS, default inner) on at most one 1024-thread block per CU, all
// resident. Wave gw owns SPW consecutive SELL slices; each lane keeps r of its
// rows in registers across iterations, y, Ap and p_t in LDS. Per iteration:
//   SpMV of the own rows, <p, Ap> block partial   -> all-gather #1 -> alpha
//   r -= alpha Ap (stored write-through), <r, r>  -> drain, all-gather #2
//                                                    -> rho, omega
//   y += alpha p, p = r + omega p (p stored write-through, ping-pong buffer)
// The SpMV gathers p_t(j) of the block's own rows from LDS and of other
// blocks' rows as r_t(j) + omega_{t-1} p_{t-1}(j) (the owner's exact
// operations) with agent-scope loads: r_t was stored before all-gather #2 of
// the previous iteration and p_{t-1} one iteration earlier, so both are
// visible once it has been observed, and the loop needs two grid-wide
// exchanges, not three.
// Scalar arithmetic is that of cg_alpha_kernel / cg_yp_kernel and every
// block derives the same bits (fixed-order sums); the dot products are summed
// in another order than the launch-per-pass path's, so the two agree to
// rounding, not bitwise.
// Inputs are read-only: r_t lives in Rs, p_{t+1} in Pb[t & 1], y in LDS and,
// after a clean chunk, in Yout; the scalar slots go to Sout. A timed-out
// exchange (a block that is not resident, kSpinLimit) therefore leaves the
// chunk-start state intact, whichever blocks got how far.
constexpr int kCgpBlock = 1024;
constexpr int kCgpWaves = kCgpBlock / 64;
constexpr int kCgpGran = 4 * 2 * 256;                 // (exchange, parity) regions x 2 words x G <= 256
constexpr size_t kCgpBytes = 64 + (size_t)kCgpGran * 8;  // 16 barrier words, then the granules

// write-through store (sc1): visible at agent scope once the wave's vmcnt
// drains, so the exchange needs no L2 writeback (buffer_wbl2) on its release
// side
template <typename V>
__device__ __forceinline__ void st_wt(V *p, V v) {
  if constexpr (sizeof(V) == 8)
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), (unsigned long long)__double_as_longlong((double)v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    __hip_atomic_store(reinterpret_cast<unsigned *>(p), __float_as_uint((float)v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// its reader: an agent-scope (sc1) load sees the write-through stores once the
// writer's all-gather has been observed, with no L2 invalidate (buffer_inv)
template <typename V>
__device__ __forceinline__ V ld_wt(const V *p) {
  if constexpr (sizeof(V) == 8)
    return (V)__longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p),
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  else
    return (V)__uint_as_float(
        __hip_atomic_load(reinterpret_cast<const unsigned *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// &base[idx] as a uniform 64-bit base plus a 32-bit byte offset (the
// persistent loop's n <= 1 M rows): the store/load then takes the base in
// SGPRs and one VGPR of offset, where a 64-bit per-lane address costs two
// VGPRs per row and was spilled and reloaded (a reload's vmcnt wait then
// serialised the write-through stores behind it)
template <typename T>
__device__ __forceinline__ T *at32(T *base, int64_t idx) {
  return reinterpret_cast<T *>(reinterpret_cast<char *>(base) + (size_t)((unsigned)idx * (unsigned)sizeof(T)));
}
template <typename T>
__device__ __forceinline__ const T *at32(const T *base, int64_t idx) {
  return reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) +
                                     (size_t)((unsigned)idx * (unsigned)sizeof(T)));
}

template <typename V>
struct CgpBufs {
  const V *Yin, *Rin, *Pin;  // chunk-start state (never written)
  V *Yout, *Rs, *Pa, *Pb;    // y after a clean chunk; scratch r; p_{t+1} in (t & 1 ? Pb : Pa)
  const double *Sin;         // scalar slots (read)
  double *Sout;              // scalar slots after a clean chunk
};

// The SELL-128/DIA image for the persistent loop's SpMV (round 5; DIA = true):
// a wave's SPW SELL-64 slices are SPW / 2 DIA slices of the same rows, lane l
// owning rows 2l, 2l + 1 of each; one 16-B value load per slot column and no
// index stream, against a 2-B delta and an 8-B value load per row.
template <typename MV>
struct CgpDia {
  const int64_t *sptr;
  const int *width;
  const int *off;
  const uint64_t *mask;
  const MV *val;
  int64_t nslices;
  int span;  // max |offset| over the image (WR > 0: the LDS halo's rows per side)
};

// The register-resident DIA form (WR > 0): the wave's values stay in
// registers for the whole chunk (a 5-point stencil: 2 x 5 x 2 values per lane
// at SPW = 4, 40 VGPRs for fp64) instead of being re-read every iteration,
// and the SpMV's x comes from LDS alone: the block's own p_t rows and, formed
// at the top of every iteration by one coalesced pass of the whole block, the
// span rows on either side (a halo of at most kCgpHalo rows per side). A
// matrix with wider slices or a larger span takes the streamed form (WR = 0).
constexpr int kCgpWr = 5;
constexpr int kCgpHalo = 3072;

template <typename V, typename S, typename MV, typename I, bool D16, int SPW, bool DIA = false, int WR = 0>
__global__ __launch_bounds__(kCgpBlock) void cg_persist_kernel(
    const int64_t *__restrict__ sptr, const int *__restrict__ swidth, const I *__restrict__ sidx,
    const uint16_t *__restrict__ sdelta, const int *__restrict__ scbase, const MV *__restrict__ sval,
    int64_t nslices, int64_t n, CgpBufs<V> B, double *hist, unsigned *words, Ctrl *ctrl, int max_steps,
    unsigned long long *tbuf, int fault_step, CgpDia<MV> Dg) {
  static_assert(!DIA || SPW % 2 == 0, "a DIA slice is two SELL-64 slices");
  static_assert(WR == 0 || DIA, "register-resident values are the DIA form's");
  if (halted(ctrl, 0)) return;
  // optional phase trace (tbuf != null, KRY_CGP_TRACE): thread 0's wall-clock
  // split of an iteration into SpMV / all-gather #1 wait / r update / store
  // drain / all-gather #2 wait / y and p update
  // (in LDS: per-lane registers for one thread's counters cost 14 VGPRs
  // across the whole loop)
  __shared__ unsigned long long tacc[7];  // 6 phases, then the last mark
  auto tmark = [&](int k) {
    if (tbuf && threadIdx.x == 0) {
      const unsigned long long now = wall_clock64();
      if (k >= 0) tacc[k] += now - tacc[6];
      tacc[6] = now;
    }
  };
  if (tbuf && threadIdx.x == 0)
    for (int k = 0; k < 7; ++k) tacc[k] = 0;
  constexpr int UNR = 5;  // a 5-point row in one round of loads; 8 spills at 128 VGPRs
  constexpr int ROWS = SPW * kCgpBlock;  // rows of this block: [row0, row0 + ROWS)
  __shared__ double wsum[kCgpWaves];
  __shared__ double shv[2];
  __shared__ int flag;
  // LDS: y and Ap of the block's rows (r stays in registers) and p_t of the
  // block's rows by local row, so that in-block columns (most of a banded
  // matrix's) are gathered from LDS; SPW = 4 doubles is 96 KB of 160
  // WR > 0: ps holds the halo too, own row lr at ps[po + lr] (po = span)
  __shared__ V ys[ROWS], aps[ROWS], ps[ROWS + (WR > 0 ? 2 * kCgpHalo : 0)];
  const int po = WR > 0 ? Dg.span : 0;
  unsigned long long *gran = reinterpret_cast<unsigned long long *>(words + 16);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  // fault injection (tests): the last block stops publishing at iteration
  // fault_step, as a block that never became resident would
  const bool faulty = fault_step >= 0 && (int)blockIdx.x == G - 1;
  const unsigned spin_limit = fault_step >= 0 ? kSpinLimitFault : kSpinLimit;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;
  const int64_t s0 = ((int64_t)blockIdx.x * kCgpWaves + wid) * SPW;
  const int lr0 = wid * SPW * 64 + lane;  // local row of slice i: lr0 + 64 i
  V r[SPW];
#pragma unroll
  for (int i = 0; i < SPW; ++i) {
    const int64_t row = (s0 + i) * 64 + lane;
    const bool own = s0 + i < nslices && row < n;
    ys[i * kCgpBlock + tid] = own ? *at32(B.Yin, row) : V(0);
    r[i] = own ? *at32(B.Rin, row) : V(0);
    ps[po + lr0 + 64 * i] = own ? *at32(B.Pin, row) : V(0);
  }
  // WR > 0: the wave's DIA values, slot offsets and lane masks, loaded once
  // per chunk: pair q's slot column u in ar[q][u] (holes and columns past the
  // slice's width are 0), its offset in aoff[q][u] (wave-uniform), row 2l + h
  // present in bit 2 (q WR + u) + h of abits
  constexpr int NQ = WR > 0 ? SPW / 2 : 1, NU = WR > 0 ? WR : 1;
  MV ar[NQ][NU][2];
  int aoff[NQ][NU];
  unsigned abits = 0;
  if constexpr (WR > 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int64_t sd = s0 / 2 + q;
      const int w = sd < Dg.nslices ? Dg.width[sd] : 0;
      const int64_t base = w > 0 ? Dg.sptr[sd] : 0, cb = base / kDiaSlice;
      const MV *cv = Dg.val + base + 2 * lane;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const bool in = u < w;
        aoff[q][u] = in ? Dg.off[cb + u] : 0;
        const uint64_t m0 = in ? Dg.mask[2 * (cb + u)] : 0, m1 = in ? Dg.mask[2 * (cb + u) + 1] : 0;
        abits |= (unsigned)((m0 >> lane) & 1u) << (2 * (q * NU + u));
        abits |= (unsigned)((m1 >> lane) & 1u) << (2 * (q * NU + u) + 1);
        if (in) {
          pload<MV>(cv + (int64_t)u * kDiaSlice, ar[q][u]);
        } else {
          ar[q][u][0] = MV(0);
          ar[q][u][1] = MV(0);
        }
      }
    }
  }
  S rho = (S)B.Sin[S_RHO];
  const double crit = B.Sin[S_CRIT];
  S alpha = (S)B.Sin[S_ALPHA], rho_prev = (S)B.Sin[S_RHO_PREV], omega = (S)B.Sin[S_OMEGA];
  V om_prev = V(0);
  // all-gather of one double per block (fixed-order sum, same in every block);
  // `data`: R / P stores precede it (write-through: drained before the publish)
  auto exchange = [&](double part, int t, int xid, bool data) -> bool {
    const double bp = block_sum1_t0_dpp(part, wsum);
    tmark(xid == 0 ? 0 : 2);
    unsigned long long *gr = gran + (size_t)(xid * 2 + (t & 1)) * 2 * 256;
    const unsigned tag = ((unsigned)(t + 1) << 2) | (unsigned)(xid + 1);
    if (data) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      tmark(3);
    }
    if (tid == 0) publish_partial(gr + 2 * blockIdx.x, tag, bp);
    if (tid < 64) {
      const bool ok = sweep_partials<false, true>(gr, G, tag, words, ctrl, &shv[0], spin_limit);
      if (tid == 0) {
        flag = ok ? 1 : 0;
      }
    }
    __syncthreads();
    tmark(xid == 0 ? 1 : 4);
    return flag != 0;
  };
  int t = 0;
  tmark(-1);
  for (; t < max_steps; ++t) {
    __syncthreads();  // p_t of the block's rows complete in LDS
    // p_t(j) of other blocks' rows: at t = 0 from Pin (kernel boundary); after
    // that r_t(j) + omega p_{t-1}(j), the owner's operations
    const V *Pprev = t == 1 ? B.Pin : ((t & 1) ? B.Pb : B.Pa);  // holds p_{t-1} (t >= 1)
    double pap = 0.0;
    // x of global row c for the SpMV: this block's p_t from LDS, another
    // block's formed as the owner does (r_t(c) + omega p_{t-1}(c))
    auto xval = [&](int64_t c) -> V {
      const int64_t lc = c - row0;
      if ((uint64_t)lc < (uint64_t)ROWS) return ps[po + lc];
      if (t == 0) return *at32(B.Pin, c);
      const V rj = ld_wt(at32(B.Rs, c)), pj = ld_wt(at32(Pprev, c));
      const V tt = om_prev * pj;  // p = r + omega p (cg.py:178)
      return rj + tt;
    };
    if constexpr (WR > 0) {
      // the halo: rows [row0 - span, row0) and [row0 + ROWS, row0 + ROWS +
      // span) of p_t, formed as xval forms them, from the owners' r_t and
      // the halo's own p_{t-1} (kept in LDS from the previous iteration: the
      // same bits the owner holds), so p never crosses blocks in the loop
      for (int h = tid; h < 2 * po; h += kCgpBlock) {
        const int64_t c = h < po ? row0 - po + h : row0 + ROWS + (h - po);
        if (c < 0 || c >= n) continue;
        const int hs = h < po ? h : po + ROWS + (h - po);
        V v;
        if (t == 0) {
          v = *at32(B.Pin, c);
        } else {
          const V rj = ld_wt(at32(B.Rs, c));
          const V tt = om_prev * ps[hs];  // p = r + omega p (cg.py:178)
          v = rj + tt;
        }
        ps[hs] = v;
      }
      __syncthreads();
      // opaque per iteration, so that the 2 NQ NU LDS addresses and lane
      // masks are formed here and not held in registers across the loop
      int lb = po + wid * SPW * 64 + 2 * lane;
      unsigned ab = abits;
      asm volatile("" : "+v"(lb), "+v"(ab));
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int la = wid * SPW * 64 + q * 128 + 2 * lane;  // local row of the lane's first row
        const int64_t ra = row0 + la;
        V acc0 = V(0), acc1 = V(0);
#pragma unroll
        for (int u = 0; u < NU; ++u) {  // ascending offsets, as the streamed form below
          if ((ab >> (2 * (q * NU + u))) & 1u) {
            const V pr = (V)ar[q][u][0] * ps[lb + q * 128 + aoff[q][u]];
            acc0 = acc0 + pr;
          }
          if ((ab >> (2 * (q * NU + u) + 1)) & 1u) {
            const V pr = (V)ar[q][u][1] * ps[lb + q * 128 + 1 + aoff[q][u]];
            acc1 = acc1 + pr;
          }
        }
        aps[la] = acc0;
        aps[la + 1] = acc1;
        if (ra < n) pap += dterm((double)ps[po + la], (double)acc0);
        if (ra + 1 < n) pap += dterm((double)ps[po + la + 1], (double)acc1);
      }
    } else if constexpr (DIA) {
      constexpr int UNRD = SPW == 4 ? 2 : 3;  // slot columns per round (more spill at 128 VGPRs)
#pragma unroll 1
      for (int q = 0; q < SPW / 2; ++q) {
        const int64_t sd = s0 / 2 + q;
        const int la = wid * SPW * 64 + q * 128 + 2 * lane;  // local row of the lane's first row
        const int64_t ra = row0 + la;
        V acc0 = V(0), acc1 = V(0);
        if (sd < Dg.nslices) {
          const int w = Dg.width[sd];
          const int64_t base = Dg.sptr[sd], cb = base / kDiaSlice;
          const MV *cv = Dg.val + base + 2 * lane;
          for (int j0 = 0; j0 < w; j0 += UNRD) {
            int off[UNRD];
            bool on0[UNRD], on1[UNRD];
            MV a[UNRD][2];
#pragma unroll
            for (int u = 0; u < UNRD; ++u) {
              const bool in = j0 + u < w;
              off[u] = in ? Dg.off[cb + j0 + u] : 0;
              const uint64_t m0 = in ? Dg.mask[2 * (cb + j0 + u)] : 0, m1 = in ? Dg.mask[2 * (cb + j0 + u) + 1] : 0;
              on0[u] = ((m0 >> lane) & 1u) != 0;
              on1[u] = ((m1 >> lane) & 1u) != 0;
              if (in) {
                pload<MV>(cv + (int64_t)(j0 + u) * kDiaSlice, a[u]);
              } else {
                a[u][0] = MV(0);
                a[u][1] = MV(0);
              }
            }
#pragma unroll
            for (int u = 0; u < UNRD; ++u) {  // ascending offsets: csr_matvec's order for sorted rows
              if (on0[u]) {
                const V pr = (V)a[u][0] * xval(ra + off[u]);
                acc0 = acc0 + pr;
              }
              if (on1[u]) {
                const V pr = (V)a[u][1] * xval(ra + 1 + off[u]);
                acc1 = acc1 + pr;
              }
            }
          }
        }
        aps[la] = acc0;
        aps[la + 1] = acc1;
        if (ra < n) pap += dterm((double)ps[po + la], (double)acc0);
        if (ra + 1 < n) pap += dterm((double)ps[po + la + 1], (double)acc1);
      }
    } else {
#pragma unroll
      for (int i = 0; i < SPW; ++i) {
        const int64_t sl = s0 + i;
        V acc = V(0);
        if (sl < nslices) {
          const int w = swidth[sl];
          const int64_t base = sptr[sl];
          for (int j0 = 0; j0 < w; j0 += UNR) {
            I col[UNR];
            V a[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
              const bool in = j0 + u < w;
              if constexpr (D16) {
                const unsigned d = in ? (unsigned)sdelta[base + (int64_t)(j0 + u) * 64 + lane] : 0xFFFFu;
                const int b = in ? scbase[(base >> 6) + j0 + u] : 0;
                col[u] = d != 0xFFFFu ? I(b + (int)d) : I(-1);
              } else {
                col[u] = in ? sidx[base + (int64_t)(j0 + u) * 64 + lane] : I(-1);
              }
              a[u] = in ? (V)sval[base + (int64_t)(j0 + u) * 64 + lane] : V(0);
            }
            V xv[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) xv[u] = col[u] < 0 ? V(0) : xval(col[u]);
#pragma unroll
            for (int u = 0; u < UNR; ++u)
              if (col[u] >= 0) {
                const V pr = a[u] * xv[u];
                acc = acc + pr;
              }
          }
          if (sl * 64 + lane < n) pap += dterm((double)ps[po + lr0 + 64 * i], (double)acc);
        }
        aps[lr0 + 64 * i] = acc;  // by local row (the DIA form's layout)
      }
    }
    if (faulty && t == fault_step) return;
    if (!exchange(pap, t, 0, false)) return;
    const S pAp = (S)shv[0];
    alpha = rho / safe<S>(pAp);  // cg.py:183-185
    const V a = (V)(double)alpha;
    double rr = 0.0;
    // the rows' store offsets are formed here each iteration from an opaque
    // lane index: hoisted out of the loop they were spilled (see at32)
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < SPW; ++i) {
      const int64_t row = (s0 + i) * 64 + ln;
      const V t2 = a * aps[lr0 + 64 * i];
      r[i] = r[i] - t2;  // cg.py:200
      if (s0 + i < nslices && row < n) {
        // WR: only the rows within span of the block's edges are another
        // block's halo; the rest go out once, after the loop
        const int lr = lr0 + 64 * i;
        if (WR == 0 || lr < po || lr >= ROWS - po) st_wt(at32(B.Rs, row), r[i]);
        rr += dterm((double)r[i], (double)r[i]);
      }
    }
    if (!exchange(rr, t, 1, true)) return;
    const S rrS = (S)shv[0];
    const S om = rrS / safe<S>(rho);
    const V omV = (V)(double)om;
    V *Pnext = (t & 1) ? B.Pb : B.Pa;  // p_{t+1}
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < SPW; ++i) {
      const int64_t row = (s0 + i) * 64 + ln;
      const V pv = ps[po + lr0 + 64 * i];
      const V t1 = a * pv;
      ys[i * kCgpBlock + tid] = ys[i * kCgpBlock + tid] + t1;  // cg.py:196
      const V tt = omV * pv;
      const V pn = r[i] + tt;  // cg.py:178
      ps[po + lr0 + 64 * i] = pn;  // every wave is past this iteration's SpMV (exchange barriers)
      // (WR: no peer reads p; the last p goes out once, after the loop)
      if (WR == 0 && s0 + i < nslices && row < n) st_wt(at32(Pnext, row), pn);
    }
    tmark(5);
    const S nrm = sqrt(rrS);
    if (blockIdx.x == 0 && tid == 0) hist[t] = (double)nrm;
    rho_prev = rho;
    rho = rrS;
    omega = om;
    om_prev = omV;
    if ((double)nrm <= crit) {  // cg.py:156 (uniform: every block has the same bits)
      if (blockIdx.x == 0 && tid == 0) ctrl->stop_at = t + 1;
      ++t;
      break;
    }
  }
  if (tbuf && tid == 0)
    for (int k = 0; k < 6; ++k) tbuf[blockIdx.x * 8 + k] = tacc[k];
  // a clean chunk: y to Yout (r, and p but in the WR form, are already in
  // Rs and Pa / Pb), the scalar
  // slots to Sout (the fused path's layout; S_RHO_OLD = the rho alpha used)
  if (blockIdx.x == 0 && tid == 0 && t > 0) {
    B.Sout[S_ALPHA] = (double)alpha;
    B.Sout[S_RHO_OLD] = (double)rho_prev;
    B.Sout[S_RHO_PREV] = (double)rho_prev;
    B.Sout[S_RHO] = (double)rho;
    B.Sout[S_OMEGA] = (double)omega;
    B.Sout[S_CRIT] = crit;
    B.Sout[S_TMP] = B.Sin[S_TMP];
  }
  V *Plast = ((t - 1) & 1) ? B.Pb : B.Pa;  // p_t, where the iteration that formed it would have stored it
#pragma unroll
  for (int i = 0; i < SPW; ++i) {
    const int64_t row = (s0 + i) * 64 + lane;
    if (s0 + i < nslices && row < n) {
      *at32(B.Yout, row) = ys[i * kCgpBlock + tid];
      if (WR > 0 && t > 0) {
        *at32(Plast, row) = ps[po + lr0 + 64 * i];
        *at32(B.Rs, row) = r[i];
      }
    }
  }
}

template <typename V, typename MV, typename I>
int cg_residual_chain(kry_cg *s, const V *src, V *raw, V *mlr) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  int P = 0;
  const V *bb = static_cast<const V *>(s->b);
  if (!s->Ml && !s->M) {
    launch_spmv<V, MV, I>(s->A, k, SrcPlain<V>{src, k}, EpiResidual<V>{bb, mlr, s->w, k}, s->part, &P, nullptr, 0,
                          st);
    return P;
  }
  if (s->Ml) {
    launch_spmv<V, MV, I>(s->A, k, SrcPlain<V>{src, k}, EpiResidual<V>{bb, raw, s->w, k}, s->part, &P, nullptr, 0,
                          st);
    launch_spmv_any<V>(s->Ml, k, SrcPlain<V>{raw, k}, EpiStoreNorm<V>{mlr, s->w, k}, s->part, &P, nullptr, 0, st);
  } else {
    launch_spmv<V, MV, I>(s->A, k, SrcPlain<V>{src, k}, EpiResidual<V>{bb, mlr, s->w, k}, s->part, &P, nullptr, 0,
                          st);
  }
  if (s->M)
    launch_spmv_any<V>(s->M, k, SrcPlain<V>{mlr, k}, EpiStoreDot<V>{static_cast<V *>(s->z), mlr, s->w, k}, s->part,
                       &P, nullptr, 0, st);
  return P;
}

template <typename V, typename MV, typename I>
void cg_start_impl(kry_cg *s) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  // r0 = b - A x0 (x0 = 0: r0 = b - A 0 evaluated the same way)
  const V *src = static_cast<const V *>(s->x0);
  if (!src) src = static_cast<const V *>(s->xk);  // zero-filled scratch
  const int P = cg_residual_chain<V, MV, I>(s, src, static_cast<V *>(s->t), static_cast<V *>(s->r));
  if (s->scalar_f32)
    hipLaunchKernelGGL(cg_start_finalize<float>, dim3(1), dim3(kBlock), 0, st, s->part, P, k, s->scal);
  else
    hipLaunchKernelGGL(cg_start_finalize<double>, dim3(1), dim3(kBlock), 0, st, s->part, P, k, s->scal);
  KRY_HIP(hipGetLastError());
}

// The persistent loop when the whole problem fits one resident block per CU
// (SPW slices per wave, SPW in 1..4: n <= 1 M at 256 CUs; 8 spills); false = use the
// launch-per-pass path. Decided once per solver (s->cgp_spw); the words are
// zeroed per launch so the granule tags restart at step 0.
// The launch is cooperative: the runtime refuses a grid larger than the
// occupancy query admits (hipErrorCooperativeLaunchTooLarge), and the solve
// then stays on the launch-per-pass path. That check is all a cooperative
// launch adds on this chip (MI355X_MICROARCH.md "coop-launch": same residency
// as a plain launch, +15-19 us per launch = < 0.1 us per iteration at 256
// iterations per chunk); CUs held by another stream or process can still keep
// a block from becoming resident, which the bounded exchanges and the host's
// rerun (kry_cg_run) cover.
// The DIA image's largest |offset| (the register-resident form's halo),
// read back once per operator; concurrent first callers compute the same value.
static int dia_span_of(const kry_csr *A, hipStream_t st) {
  int sp = __atomic_load_n(&A->dia_span, __ATOMIC_ACQUIRE);
  if (sp >= 0) return sp;
  const int64_t ncol = A->dia_nslots / kDiaSlice;
  std::vector<int> off((size_t)ncol);
  if (ncol > 0) {
    KRY_HIP(hipMemcpyAsync(off.data(), A->dia_off, (size_t)ncol * 4, hipMemcpyDeviceToHost, st));
    KRY_HIP(hipStreamSynchronize(st));
  }
  sp = 0;
  for (int o : off) sp = std::max(sp, o < 0 ? -o : o);
  __atomic_store_n(const_cast<int *>(&A->dia_span), sp, __ATOMIC_RELEASE);
  return sp;
}

template <typename V, typename S, typename MV, typename I, bool D16>
bool cgp_launch_t(kry_cg *s, int max_steps, bool decide_only) {
  const kry_csr *A = s->A;
  // the SpMV over the DIA image when there is one and a wave's slices pair
  // up (SPW even); KRY_CGP_DIA=0: the SELL image as before round 5
  const bool dia_ok = A->dia && !env_off("KRY_CGP_DIA");
  // its values held in registers for the chunk and x from LDS when every
  // slice is at most kCgpWr slot columns wide and the offsets span at most
  // kCgpHalo rows; KRY_CGP_WR=0: the streamed form
  const bool wr_ok = dia_ok && A->dia_max_width <= kCgpWr && !env_off("KRY_CGP_WR") &&
                     dia_span_of(A, s->ctx->stream) <= kCgpHalo;
  auto kern_for = [&](int spw) {
    if (wr_ok && spw == 2) return cg_persist_kernel<V, S, MV, I, D16, 2, true, kCgpWr>;
    if (wr_ok && spw == 4) return cg_persist_kernel<V, S, MV, I, D16, 4, true, kCgpWr>;
    if (dia_ok && spw == 2) return cg_persist_kernel<V, S, MV, I, D16, 2, true>;
    if (dia_ok && spw == 4) return cg_persist_kernel<V, S, MV, I, D16, 4, true>;
    switch (spw) {
      case 1: return cg_persist_kernel<V, S, MV, I, D16, 1>;
      case 2: return cg_persist_kernel<V, S, MV, I, D16, 2>;
      default: return cg_persist_kernel<V, S, MV, I, D16, 4>;
    }
  };
  if (s->cgp_spw < 0) {
    s->cgp_spw = 0;
    const char *e = getenv("KRY_CG_PERSIST");
    if (!(e && atoi(e) == 0)) {
      int dev = 0, ncu = 0;
      KRY_HIP(hipGetDevice(&dev));
      KRY_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      const int gmax = ncu < 256 ? ncu : 256;
      for (int spw = 1; spw <= 4; spw *= 2) {
        const int64_t G = (A->nslices + (int64_t)kCgpWaves * spw - 1) / ((int64_t)kCgpWaves * spw);
        if (G > gmax) continue;
        int per_cu = 0;
        KRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern_for(spw), kCgpBlock, 0));
        if (per_cu >= 1) s->cgp_spw = spw;
        break;
      }
      if (s->cgp_spw > 0) {
        const size_t vb = ((size_t)s->n + 15) / 16 * 16 * sizeof(V);
        s->rs = dev_alloc(vb);
        s->pb = dev_alloc(vb);
        s->pb2 = dev_alloc(vb);
        s->yb = dev_alloc(vb);
        s->cgp_scal = static_cast<double *>(dev_alloc(S_COUNT * 8));
        s->cgp_words = static_cast<unsigned *>(dev_alloc(kCgpBytes));
      }
    }
  }
  if (s->cgp_spw == 0) return false;
  if (decide_only) return true;
  const int spw = s->cgp_spw;
  const int G = (int)((A->nslices + (int64_t)kCgpWaves * spw - 1) / ((int64_t)kCgpWaves * spw));
  hipStream_t st = s->ctx->stream;
  KRY_HIP(hipMemsetAsync(s->cgp_words, 0, kCgpBytes, st));
  KRY_HIP(hipMemcpyAsync(s->cgp_scal, s->scal, S_COUNT * 8, hipMemcpyDeviceToDevice, st));
  unsigned long long *tb = nullptr;
  if (getenv("KRY_CGP_TRACE")) {
    KRY_HIP(hipMalloc(&tb, (size_t)G * 64));
    KRY_HIP(hipMemsetAsync(tb, 0, (size_t)G * 64, st));
  }
  const char *fe = getenv("KRY_CGP_FAULT");  // fault injection (tests): iteration at which a block drops out
  int fault_step = fe ? atoi(fe) : -1;
  CgpBufs<V> bufs{static_cast<const V *>(s->y), static_cast<const V *>(s->r), static_cast<const V *>(s->p),
                  static_cast<V *>(s->yb),      static_cast<V *>(s->rs),      static_cast<V *>(s->pb),
                  static_cast<V *>(s->pb2),     s->scal,                      s->cgp_scal};
  const int64_t *a_sptr = static_cast<const int64_t *>(A->sptr);
  const int *a_swidth = static_cast<const int *>(A->swidth);
  const I *a_sidx = static_cast<const I *>(A->sidx);
  const uint16_t *a_sdelta = static_cast<const uint16_t *>(A->sdelta);
  const int *a_scbase = static_cast<const int *>(A->scbase);
  const MV *a_sval = static_cast<const MV *>(A->sval);
  int64_t nsl = A->nslices, n = A->n;
  double *hist = s->hist;
  unsigned *words = s->cgp_words;
  Ctrl *ctrl = s->ctrl;
  CgpDia<MV> dg{static_cast<const int64_t *>(A->dia_sptr), static_cast<const int *>(A->dia_width),
                static_cast<const int *>(A->dia_off), static_cast<const uint64_t *>(A->dia_mask),
                static_cast<const MV *>(A->dia_val), A->dia ? A->dia_nslices : 0, wr_ok ? A->dia_span : 0};
  void *args[] = {&a_sptr, &a_swidth, &a_sidx, &a_sdelta, &a_scbase, &a_sval, &nsl,        &n,
                  &bufs,   &hist,     &words,  &ctrl,     &max_steps, &tb,    &fault_step, &dg};
  hipError_t le;
  {
    // A plain launch, as for cg_upd_kernel: residency is the occupancy check
    // above (at most one block per CU) and a block that still does not become
    // resident makes the exchange time out, the chunk then reruns launch per
    // pass from its untouched start state. A cooperative launch guaranteed
    // residency but left HIP runtime state behind that crashed the process at
    // exit under rocprofv3 (libamdhip64's exit handler into
    // libhsa-runtime64, profiles/r03_exit_crash.txt); KRY_CGP_COOP=1 keeps
    // it for comparison.
    ProfScope ps(s->ctx, PROF_OTHER);
    const char *ce = getenv("KRY_CGP_COOP");
    const void *kf = reinterpret_cast<const void *>(kern_for(spw));
    le = (ce && atoi(ce) == 1) ? hipLaunchCooperativeKernel(kf, dim3(G), dim3(kCgpBlock), args, 0, st)
                               : hipLaunchKernel(kf, dim3(G), dim3(kCgpBlock), args, 0, st);
  }
  if (le != hipSuccess) {
    (void)hipGetLastError();  // clear the refusal; the solve continues on the launch-per-pass path
    s->cgp_spw = 0;
    if (tb) KRY_HIP(hipFree(tb));
    return false;
  }
  if (tb) {  // KRY_CGP_TRACE: per-phase split, per-block sums of wall_clock64 ticks (100 MHz), to stderr
    std::vector<unsigned long long> h((size_t)G * 8);
    KRY_HIP(hipMemcpyAsync(h.data(), tb, h.size() * 8, hipMemcpyDeviceToHost, st));
    KRY_HIP(hipStreamSynchronize(st));
    Ctrl c;
    KRY_HIP(hipMemcpy(&c, s->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost));
    const int its = c.stop_at < max_steps ? c.stop_at : max_steps;
    const char *names[6] = {"spmv", "x1wait", "rupd", "drain", "x2wait", "pupd"};
    fprintf(stderr, "cgp trace G=%d its=%d (us/it: mean / min / max over blocks):", G, its);
    for (int k = 0; k < 6; ++k) {
      double mn = 1e30, mx = 0, sm = 0;
      for (int b = 0; b < G; ++b) {
        const double v = h[(size_t)b * 8 + k] * 0.01 / (its > 0 ? its : 1);
        mn = v < mn ? v : mn;
        mx = v > mx ? v : mx;
        sm += v;
      }
      fprintf(stderr, " %s %.2f/%.2f/%.2f", names[k], sm / G, mn, mx);
    }
    fprintf(stderr, "\n");
    KRY_HIP(hipFree(tb));
  }
  return true;
}

// After a persistent chunk of `done` clean iterations: the state it left in
// its own buffers becomes the solver's (r_T in rs, p_T in pb / pb2 by the
// parity of T, y_T in yb, the scalar slots in cgp_scal).
static void cgp_commit(kry_cg *s, int done) {
  if (done <= 0) return;
  std::swap(s->r, s->rs);
  std::swap(s->y, s->yb);
  if ((done - 1) & 1)
    std::swap(s->p, s->pb2);
  else
    std::swap(s->p, s->pb);
  KRY_HIP(hipMemcpyAsync(s->scal, s->cgp_scal, S_COUNT * 8, hipMemcpyDeviceToDevice, s->ctx->stream));
}

// KRY_CG_PERSIST=0 disables the persistent loop; =2 requires it (tests).
// decide_only: report eligibility (deciding it once) without launching.
template <typename V, typename MV, typename I>
bool cgp_launch(kry_cg *s, int max_steps, bool decide_only = false) {
  const kry_csr *A = s->A;
  bool taken = false;
  if (s->cgp_spw != 0 && s->k == 1 && !s->M && !s->Ml && !s->w && !s->comm && A->nirregular == 0 && A->cb_nb == 0 &&
      A->sptr && A->nslices > 0 && max_steps > 0) {
    const bool f32 = s->scalar_f32;
    if (A->compact)
      taken = f32 ? cgp_launch_t<V, float, MV, I, true>(s, max_steps, decide_only)
                  : cgp_launch_t<V, double, MV, I, true>(s, max_steps, decide_only);
    else
      taken = f32 ? cgp_launch_t<V, float, MV, I, false>(s, max_steps, decide_only)
                  : cgp_launch_t<V, double, MV, I, false>(s, max_steps, decide_only);
  }
  if (decide_only) return taken;
  const char *e = getenv("KRY_CG_PERSIST");
  KRY_REQUIRE(taken || max_steps <= 0 || !(e && atoi(e) == 2), KRY_EUNSUPPORTED,
              "KRY_CG_PERSIST=2: this solve is not eligible for the persistent CG loop");
  return taken;
}

// One-launch update of step `step` (cg_upd_kernel) if eligible: one RHS, no
// M / Ml, Euclidean inner, n larger than the persistent loop serves and at
// most 512 * 40 granules per block at one block per CU (decided once per
// solver; KRY_CG_UPD=0 disables). Returns false when not launched.
template <typename V, typename S, int NV>
void *cgu_kern(bool def) {
  return def ? reinterpret_cast<void *>(cg_upd_kernel<V, S, NV, true>)
             : reinterpret_cast<void *>(cg_upd_kernel<V, S, NV, false>);
}
template <typename V>
bool cgu_launch(kry_cg *s, const double *partA, int PA, int step, double *gbuf, const PRing<V> &ring, int D) {
  constexpr int W = Vec16<V>::W;
  using S = V;
  const int64_t N = s->n;
  auto kern = [&](int nv, bool def = false) -> void * {
    switch (nv) {
      case 8: return cgu_kern<V, S, 8>(def);
      case 16: return cgu_kern<V, S, 16>(def);
      case 24: return cgu_kern<V, S, 24>(def);
      case 32: return cgu_kern<V, S, 32>(def);
      default: return cgu_kern<V, S, 40>(def);
    }
  };
  if (s->upd_nv < 0) {
    s->upd_nv = 0;
    const char *e = getenv("KRY_CG_UPD");
    const bool scalars_match = (sizeof(V) == 8) != s->scalar_f32;
    if (!(e && atoi(e) == 0) && s->k == 1 && !s->M && !s->Ml && !s->w && scalars_match) {
      int dev = 0, ncu = 0;
      KRY_HIP(hipGetDevice(&dev));
      KRY_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      const int gmax = ncu < 256 ? ncu : 256;
      for (int nv : {8, 16, 24, 32, 40}) {
        const int64_t G = (N + (int64_t)kUpdBlock * nv * W - 1) / ((int64_t)kUpdBlock * nv * W);
        if (G > gmax) continue;
        int per_cu = 0;
        KRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(kern(nv)),
                                                             kUpdBlock, 0));
        if (per_cu >= 1) s->upd_nv = nv;
        break;
      }
      if (s->upd_nv > 0) s->upd_words = static_cast<unsigned *>(dev_alloc(kUpdWords * 4));
    }
  }
  if (s->upd_nv == 0) return false;
  const int nv = s->upd_nv;
  const int G = (int)((N + (int64_t)kUpdBlock * nv * W - 1) / ((int64_t)kUpdBlock * nv * W));
  hipStream_t st = s->ctx->stream;
  if (step == 0) KRY_HIP(hipMemsetAsync(s->upd_words, 0, kUpdWords * 4, st));
  const char *fe = getenv("KRY_CGU_FAULT");  // fault injection (tests): step at which a block drops out
  int fault_step = fe ? atoi(fe) : -1;
  const char *fl = getenv("KRY_CGU_FAULT_LATE");  // ... or joins late (decide_exchange tests)
  if (fault_step >= 0 && fl) fault_step |= (atoi(fl) & 0x7fff) << 16;
  V *y = static_cast<V *>(s->y), *r = static_cast<V *>(s->r);
  const int64_t gstep = s->it_base + step;
  V *p = D ? ring.s[gstep % (D + 1)] : static_cast<V *>(s->p);
  V *pout = D ? ring.s[(gstep + 1) % (D + 1)] : p;
  double *alpha_ring = D ? s->alpha_ring + gstep % D : s->alpha_ring;  // this step's slot
  int Dv = D ? D : 1;
  const V *Ap = static_cast<const V *>(s->Ap);
  double *scal = s->scal, *hist = s->hist;
  Ctrl *ctrl = s->ctrl;
  int col_offset = s->col_offset, total_k = s->total_k;
  unsigned *words = s->upd_words;
  int64_t n = N;
  void *args[] = {&n,    &y,        &r,          &p,       &Ap,    &partA,       &PA,        &scal,
                  &hist, &ctrl,     &step,       &gbuf,    &col_offset, &total_k, &words,  &fault_step,
                  &pout, &alpha_ring, &Dv};
  hipError_t le;
  {
    // A plain launch: a cooperative one costs ~8 us more stream time on each
    // side of the kernel, which is most of what the fusion saves. Residency
    // is the occupancy check above (one block per CU, G <= CUs) and the
    // exchange's bounded spin with rollback covers a block that still does
    // not become resident.
    ProfScope ps(s->ctx, PROF_UPDATE);
    le = hipLaunchKernel(kern(nv, D != 0), dim3(G), dim3(kUpdBlock), args, 0, st);
  }
  if (le == hipSuccess && D && (gstep + 1 - s->yfb) % D == 0) {  // the D deferred updates of steps gstep - D + 1 .. gstep
    ProfScope ps(s->ctx, PROF_OTHER);
    launch_elementwise<V>(N, 1, OpCgYSteps<V>{y, ring, D, s->alpha_ring, gstep - D + 1, gstep + 1, 1}, nullptr, ctrl,
                          step, st);
  }
  if (le != hipSuccess) {
    (void)hipGetLastError();
    s->upd_nv = 0;
    return false;
  }
  s->upd_used = true;
  return true;
}

// alpha = rho / <p, Ap> from the SpMV's PA partial rows (cg_alpha_kernel),
// through partial_stage_kernel first when there are many; `scratch` (k x
// kAlphaStage doubles) is free until the r pass writes its partials there.
static void launch_alpha(kry_cg *s, const double *partA, int PA, double *scratch, int step) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  static const bool stage = [] {
    const char *e = getenv("KRY_ALPHA_STAGE");  // A/B switch: 0 = one-block alpha only
    return !(e && atoi(e) == 0);
  }();
  if (stage && PA > 4 * kAlphaStage) {
    hipLaunchKernelGGL(partial_stage_kernel, dim3(kAlphaStage), dim3(kBlock), 0, st, partA, PA, k, scratch, s->ctrl,
                       step);
    partA = scratch;
    PA = kAlphaStage;
  }
  if (s->scalar_f32)
    hipLaunchKernelGGL(cg_alpha_kernel<float>, dim3(1), dim3(kAlphaBlock), 0, st, partA, PA, k, s->scal, s->ctrl, step);
  else
    hipLaunchKernelGGL(cg_alpha_kernel<double>, dim3(1), dim3(kAlphaBlock), 0, st, partA, PA, k, s->scal, s->ctrl,
                       step);
  KRY_HIP(hipGetLastError());
}

// Deferred yk updates on the block path (KRY_CG_YDEFER = D, 0 = off): the
// ring of D p buffers is chosen and allocated once per solver, by
// kry_cg_start (setup, not the iteration loop), and every buffer is written
// once there (hipMemsetAsync): the first kernel to write a fresh multi-GB
// allocation pays for mapping its pages (cfg4: a 2.2 ms first p pass against
// ~0.39 ms, profiles/r05_cfg4_kernel_stats.csv), which then happens before
// the solve's first iteration.
static void cg_ydefer_setup(kry_cg *s) {
  const int k = s->k;
  if (s->ydefer < 0) {
    s->ydefer = 0;
    const char *e = getenv("KRY_CG_YDEFER");
    const size_t vb = ((size_t)s->n * k + 15) / 16 * 16 * dsize(s->dtype);
    size_t fr = 0, tot = 0;
    KRY_HIP(hipMemGetInfo(&fr, &tot));
    // the default: only for vectors larger than half the 256 MB MALL (a
    // smaller y / p stay cache-resident between the passes, and reading the
    // ring's older p vectors back costs more than the y pass it saves: metric
    // CG, 80 MB vectors, 3,016 -> 2,874 it/s with D = 7; cfg4, 640 MB, 690 ->
    // 748 it/s at D = 7: the flush reads D + 2 vectors every D steps), the
    // deepest ring of 15, 7 or 3 whose D buffers fit kCgYDeferBudget (10 GB)
    // and a quarter of the memory free right now. Round 4 defaulted to 31
    // steps within an eighth of the device (19.8 GB at cfg4) for +1.2 % over
    // D = 15 (748 -> 757 it/s, profiles/r04_ydefer_depth.json): not worth 7 %
    // of the device held per solver. cfg4 at D = 15: 9.6 GB. KRY_CG_YDEFER
    // still selects any depth up to 31; an allocation failure falls back to
    // one update per step
    const bool big = vb > (size_t(128) << 20);
    const size_t budget = std::min(kCgYDeferBudget, fr / 4);
    int D = 0;
    if (e) {
      D = atoi(e);
    } else if (big) {
      for (int d : {15, kCgYDefer, 3})
        if ((size_t)d * vb <= budget) {
          D = d;
          break;
        }
    }
    if (D >= 1 && D <= kCgYDeferMax && k <= 8 && !s->M) {
      try {
        for (int q = 1; q <= D; ++q) s->pring[q] = dev_alloc(vb);
        s->alpha_ring = static_cast<double *>(dev_alloc((size_t)D * k * 8));
        for (int q = 1; q <= D; ++q) KRY_HIP(hipMemsetAsync(s->pring[q], 0, vb, s->ctx->stream));
        s->ydefer = D;
        s->ydefer_bytes = (int64_t)D * (int64_t)vb + (int64_t)D * k * 8;
      } catch (const Error &err) {
        if (err.code != KRY_ENOMEM) throw;
        for (int q = 1; q <= D; ++q) {
          dev_free(s->pring[q]);
          s->pring[q] = nullptr;
        }
      }
    }
  }
}

// Returns true when the chunk ran as one persistent launch.
template <typename V, typename MV, typename I>
bool cg_run_impl(kry_cg *s, int max_steps) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const int64_t N = s->n * (int64_t)k;
  if (cgp_launch<V, MV, I>(s, max_steps)) return true;
  double *partA = s->part, *partB = s->part + part_rows(k) * k;
  cg_ydefer_setup(s);  // normally done by kry_cg_start already
  const int D = (!s->M && k <= 8) ? s->ydefer : 0;
  PRing<V> ring{};
  if (D) {
    ring.s[0] = static_cast<V *>(s->p);
    for (int q = 1; q <= D; ++q) ring.s[q] = static_cast<V *>(s->pring[q]);
  }
  for (int step = 0; step < max_steps; ++step) {
    const int64_t gstep = s->it_base + step;
    V *p = D ? ring.s[gstep % (D + 1)] : static_cast<V *>(s->p);
    int PA, PB;
    {
      ProfScope ps(s->ctx, PROF_SPMV);
      if (s->Ml) {  // Ap = Ml (A p) (Product(Ml, A), cg.py:110,180)
        V *t = static_cast<V *>(s->t);
        launch_spmv<V, MV, I>(s->A, k, SrcPlain<V>{p, k}, EpiStore<V>{t, k}, nullptr, nullptr, s->ctrl, step, st);
        launch_spmv_any<V>(s->Ml, k, SrcPlain<V>{t, k}, EpiStoreDot<V>{static_cast<V *>(s->Ap), p, s->w, k}, partA,
                           &PA, s->ctrl, step, st);
      } else {
        launch_spmv<V, MV, I>(s->A, k, SrcPlain<V>{p, k}, EpiApDot<V>{static_cast<V *>(s->Ap), s->w, k}, partA, &PA,
                              s->ctrl, step, st);
      }
    }
    double *gb = s->comm ? s->gbuf : nullptr;
    if (!s->M && !s->Ml && k == 1 && cgu_launch<V>(s, partA, PA, step, gb, ring, D)) {
      // alpha, r, rho, omega, y and p in one launch (cg_upd_kernel)
    } else if (!s->M && k <= 8) {  // alpha kernel, r pass, then the fused rho / y / p pass
      launch_alpha(s, partA, PA, partB, step);
      {
        ProfScope ps(s->ctx, PROF_UPDATE);
        PB = launch_elementwise<V>(N, k,
                                   OpCgR<V>{static_cast<V *>(s->r), static_cast<const V *>(s->Ap),
                                            s->scal + S_ALPHA * k, s->w, k},
                                   partB, s->ctrl, step, st, kCgUpdateGrid);
      }
      ProfScope ps(s->ctx, PROF_OTHER);
      constexpr int W = Vec16<V>::W;
      const int G = grid_for((N + W - 1) / W, kBlock * 2);
      if (D) {
        const bool flush = (gstep + 1 - s->yfb) % D == 0;  // the kernel's rule (cg_pdefer_kernel)
        auto go = [&](auto kern) {
          hipLaunchKernelGGL(kern, dim3(G), dim3(kBlock), 0, st, N, k, static_cast<V *>(s->y), ring, D,
                             static_cast<const V *>(s->r), partB, PB, s->scal, s->alpha_ring, s->hist, s->ctrl, step,
                             gb, s->col_offset, s->total_k, gstep, s->yfb);
        };
        if (s->scalar_f32) {
          if (flush) go(cg_pdefer_kernel<V, float, true>);
          else go(cg_pdefer_kernel<V, float, false>);
        } else {
          if (flush) go(cg_pdefer_kernel<V, double, true>);
          else go(cg_pdefer_kernel<V, double, false>);
        }
      } else if (s->scalar_f32)
        hipLaunchKernelGGL((cg_yp_kernel<V, float>), dim3(G), dim3(kBlock), 0, st, N, k, static_cast<V *>(s->y), p,
                           static_cast<const V *>(s->r), partB, PB, s->scal, s->hist, s->ctrl, step, gb,
                           s->col_offset, s->total_k);
      else
        hipLaunchKernelGGL((cg_yp_kernel<V, double>), dim3(G), dim3(kBlock), 0, st, N, k, static_cast<V *>(s->y), p,
                           static_cast<const V *>(s->r), partB, PB, s->scal, s->hist, s->ctrl, step, gb,
                           s->col_offset, s->total_k);
      KRY_HIP(hipGetLastError());
    } else {  // alpha kernel, update pass, [z = M r], one-block rho kernel, p pass
      if (s->scalar_f32)
        hipLaunchKernelGGL(cg_alpha_kernel<float>, dim3(1), dim3(kAlphaBlock), 0, st, partA, PA, k, s->scal, s->ctrl,
                           step);
      else
        hipLaunchKernelGGL(cg_alpha_kernel<double>, dim3(1), dim3(kAlphaBlock), 0, st, partA, PA, k, s->scal, s->ctrl,
                           step);
      {
        ProfScope ps(s->ctx, PROF_UPDATE);
        PB = launch_elementwise<V>(N, k,
                                   OpCgUpdate<V>{static_cast<V *>(s->y), static_cast<V *>(s->r), p,
                                                 static_cast<const V *>(s->Ap), s->scal + S_ALPHA * k, s->w, k},
                                   s->M ? nullptr : partB, s->ctrl, step, st);
      }
      if (s->M) {  // M_Ml_rk = M Ml_rk and <Ml_rk, M_Ml_rk> (cg.py:207-209)
        V *r = static_cast<V *>(s->r);
        launch_spmv_any<V>(s->M, k, SrcPlain<V>{r, k}, EpiStoreDot<V>{static_cast<V *>(s->z), r, s->w, k}, partB,
                           &PB, s->ctrl, step, st);
      }
      if (s->scalar_f32)
        hipLaunchKernelGGL(cg_rho_kernel<float>, dim3(1), dim3(kBlock), 0, st, partB, PB, k, s->scal, s->hist,
                           s->ctrl, step, gb, s->col_offset, s->total_k);
      else
        hipLaunchKernelGGL(cg_rho_kernel<double>, dim3(1), dim3(kBlock), 0, st, partB, PB, k, s->scal, s->hist,
                           s->ctrl, step, gb, s->col_offset, s->total_k);
      KRY_HIP(hipGetLastError());
      {
        ProfScope ps(s->ctx, PROF_OTHER);
        const V *zv = static_cast<const V *>(s->M ? s->z : s->r);
        launch_elementwise<V>(N, k, OpCgP<V>{p, zv, s->scal + S_OMEGA * k, k}, nullptr, s->ctrl, step, st);
      }
    }
    if (s->comm) {
      // exactly one collective per iteration: the residual-norm vector and the
      // fault count (post_fault)
      inject_peer_fault(s->gbuf, s->total_k + 1, step, st);
      comm_allreduce(s->comm, s->gbuf, s->total_k + 1, st);
      hipLaunchKernelGGL(cg_global_check, dim3(1), dim3(kBlock), 0, st, s->gbuf, s->gcrit, s->total_k, s->hist,
                         s->ctrl, step);
      KRY_HIP(hipGetLastError());
    }
  }
  return false;  // (deferred yk: the updates pending now wait for cg_ydefer_flush)
}

// The deferred yk updates still pending (global steps yfb .. it - 1), applied
// in step order when the host needs y: then y is bitwise what one update per
// step gives. Nothing to do off the deferred path.
template <typename V>
void cg_ydefer_flush(kry_cg *s) {
  const int D = (!s->M && s->k <= 8) ? s->ydefer : 0;
  if (D <= 0 || s->yfb >= s->it) return;
  PRing<V> ring{};
  ring.s[0] = static_cast<V *>(s->p);
  for (int q = 1; q <= D; ++q) ring.s[q] = static_cast<V *>(s->pring[q]);
  ProfScope ps(s->ctx, PROF_OTHER);
  launch_elementwise<V>(s->n * (int64_t)s->k, s->k, OpCgYSteps<V>{static_cast<V *>(s->y), ring, D, s->alpha_ring, s->yfb,
                                                                s->it, s->k},
                        nullptr, nullptr, 0, s->ctx->stream);
  s->yfb = s->it;
}

template <typename V, typename MV, typename I>
void cg_residual_impl(kry_cg *s, double *norm2) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const int64_t N = s->n * (int64_t)k;
  cg_ydefer_flush<V>(s);
  launch_elementwise<V>(N, k, OpXk<V>{static_cast<const V *>(s->x0), static_cast<const V *>(s->y), static_cast<V *>(s->xk)},
                        nullptr, nullptr, 0, st);
  // explicit ||M Ml (b - A xk)||: t and z are free between iterations
  V *mlr = static_cast<V *>(s->Ml ? s->t : s->rt);
  const int P = cg_residual_chain<V, MV, I>(s, static_cast<const V *>(s->xk), static_cast<V *>(s->rt), mlr);
  double *out = s->scal + S_TMP * k;
  hipLaunchKernelGGL(reduce_to_kernel<0>, dim3(1), dim3(kBlock), 0, st, s->part, P, k, out);
  KRY_HIP(hipGetLastError());
  KRY_HIP(hipMemcpyAsync(norm2, out, k * 8, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
}

}  // namespace

#define KRY_API_BEGIN try {
#define KRY_API_END                  \
  return KRY_OK;                     \
  }                                  \
  catch (const kry::Error &e) {      \
    kry::set_error(e.msg);           \
    return e.code;                   \
  }                                  \
  catch (const std::exception &e) {  \
    kry::set_error(e.what());        \
    return KRY_EDEVICE;              \
  }

static void cg_free(kry_cg *s) {
  void *bufs[] = {s->b,    s->x0,   s->y,     s->r,    s->p,    s->Ap,       s->z,
                  s->t,    s->xk,   s->rt,    s->w,    s->part, s->scal,     s->hist,
                  s->ctrl, s->gbuf, s->gcrit, s->rs,   s->pb,   s->pb2,      s->yb,
                  s->cgp_scal, s->cgp_words, s->upd_words, s->alpha_ring};
  for (void *b : bufs) dev_free(b);
  for (int q = 1; q <= kCgYDeferMax; ++q) dev_free(s->pring[q]);
}

extern "C" {

int kry_cg_create(kry_ctx *ctx, kry_csr *A, int32_t k, int dtype, kry_cg **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && A && out, KRY_EINVAL, "null argument");
  KRY_REQUIRE(is_pow2(k) && k <= kMaxCols, KRY_EUNSUPPORTED, "k must be a power of two <= 256");
  KRY_REQUIRE(dtype == A->dtype || (dtype == KRY_F64 && A->dtype == KRY_F32), KRY_EINVAL,
              "vectors must have the operator dtype (or float64 over a float32 operator)");
  KRY_HIP(hipSetDevice(ctx->device));
  auto *s = new kry_cg();
  try {
    s->ctx = ctx;
    s->A = A;
    s->n = A->n;
    s->k = k;
    s->dtype = dtype;
    const size_t vb = ((size_t)A->n * k + 15) / 16 * 16 * dsize(dtype);
    void **vecs[] = {&s->b, &s->y, &s->r, &s->p, &s->Ap, &s->xk, &s->rt};
    for (void **v : vecs) {
      *v = dev_alloc(vb);
      KRY_HIP(hipMemsetAsync(*v, 0, vb, ctx->stream));
    }
    s->part = static_cast<double *>(dev_alloc(2 * part_rows(k) * k * 8));
    s->scal = static_cast<double *>(dev_alloc(S_COUNT * (size_t)k * 8));
    KRY_HIP(hipMemsetAsync(s->scal, 0, S_COUNT * (size_t)k * 8, ctx->stream));
    s->chunk_cap = 64;
    s->hist = static_cast<double *>(dev_alloc((size_t)s->chunk_cap * k * 8));
    s->ctrl = static_cast<Ctrl *>(dev_alloc(sizeof(Ctrl)));
    reset_ctrl(s->ctrl, ctx->stream);
    KRY_HIP(hipStreamSynchronize(ctx->stream));
  } catch (...) {
    cg_free(s);
    delete s;
    throw;
  }
  *out = s;
  KRY_API_END
}

int kry_cg_destroy(kry_cg *s) {
  KRY_API_BEGIN
  if (!s) return KRY_OK;
  (void)hipSetDevice(s->ctx->device);
  (void)hipStreamSynchronize(s->ctx->stream);
  cg_free(s);
  delete s;
  KRY_API_END
}

int kry_cg_start(kry_cg *s, kry_vec *b, kry_vec *x0, kry_vec *w, double *rho0) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && rho0, KRY_EINVAL, "null argument");
  check_vec(b, s->n, s->k, s->dtype, "b");
  if (x0) check_vec(x0, s->n, s->k, s->dtype, "x0");
  check_weights(w, s->n);
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  const size_t vb = b->bytes();
  // b, x0 and the weights arrive in the caller's numbering (load_in: into a
  // renumbered operator's, a plain copy otherwise)
  load_in(s->A, b->d, s->b, s->k, dsize(s->dtype), st);
  dev_free(s->x0);
  s->x0 = nullptr;
  if (x0) {
    s->x0 = dev_alloc(((size_t)s->n * s->k + 15) / 16 * 16 * dsize(s->dtype));
    load_in(s->A, x0->d, s->x0, s->k, dsize(s->dtype), st);
  }
  dev_free(s->w);
  s->w = nullptr;
  if (w) {
    s->w = static_cast<double *>(dev_alloc(((size_t)s->n + 1) * 8));
    load_in(s->A, w->d, s->w, 1, 8, st);
  }
  // the inner product's dtype: float32 for an unweighted fp32 solve (np.dot of
  // float32), float64 otherwise (weights are float64)
  s->scalar_f32 = (s->dtype == KRY_F32 && !w);
  KRY_HIP(hipMemsetAsync(s->y, 0, vb, st));
  KRY_HIP(hipMemsetAsync(s->xk, 0, vb, st));
  s->it = 0;
  s->yfb = 0;
  s->it_base = 0;
  cg_ydefer_setup(s);
  dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { cg_start_impl<decltype(v0), decltype(m0), decltype(i0)>(s); });
  // p0 = M_Ml_r0 (cg.py:138)
  KRY_HIP(hipMemcpyAsync(s->p, s->M ? s->z : s->r, vb, hipMemcpyDeviceToDevice, st));
  KRY_HIP(hipMemcpyAsync(rho0, s->scal + S_TMP * s->k, s->k * 8, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  s->started = true;
  KRY_API_END
}

int kry_cg_set_criterion(kry_cg *s, const double *criterion) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && criterion, KRY_EINVAL, "null argument");
  hipStream_t st = s->ctx->stream;
  if (s->comm) {
    KRY_HIP(hipMemcpyAsync(s->gcrit, criterion, s->total_k * 8, hipMemcpyHostToDevice, st));
  } else {
    KRY_HIP(hipMemcpyAsync(s->scal + S_CRIT * s->k, criterion, s->k * 8, hipMemcpyHostToDevice, st));
  }
  KRY_HIP(hipStreamSynchronize(st));
  KRY_API_END
}

int kry_cg_run(kry_cg *s, int32_t max_steps, int32_t *steps_done, double *resnorms) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && steps_done && resnorms && max_steps >= 0, KRY_EINVAL, "bad argument");
  KRY_REQUIRE(s->started, KRY_EINVAL, "kry_cg_start has not been called");
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  const int hk = s->comm ? s->total_k : s->k;
  if (max_steps > s->chunk_cap) {
    dev_free(s->hist);
    s->hist = nullptr;
    s->hist = static_cast<double *>(dev_alloc((size_t)max_steps * hk * 8));
    s->chunk_cap = max_steps;
  }
  auto run_steps = [&](int steps, double *rows, Ctrl *c) -> std::pair<int, bool> {
    reset_ctrl(s->ctrl, st);
    bool persistent = false;
    s->upd_used = false;
    dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) {
      persistent = cg_run_impl<decltype(v0), decltype(m0), decltype(i0)>(s, steps);
    });
    return {read_chunk(s->ctx, st, s->ctrl, s->hist, steps, hk, rows, c), persistent};
  };
  auto run_chunk = [&](Ctrl *c) { return run_steps(max_steps, resnorms, c); };
  s->it_base = s->it;
  Ctrl c;
  auto [done, persistent] = run_chunk(&c);
  bool upd = s->upd_used;
  if (persistent && c.status == KRY_EDEVICE) {
    // an in-launch exchange timed out (a block was not resident): the kernel
    // left the chunk-start state untouched; rerun the chunk launch per pass
    s->cgp_spw = 0;
    ++s->cgp_fallbacks;
    std::tie(done, persistent) = run_chunk(&c);
    upd = s->upd_used;
  } else if (persistent) {
    cgp_commit(s, done);
  } else if (s->comm && c.status == KRY_ECOMM) {
    // the healthy rank's state has moved past the recorded history (the
    // step's update kernels ran before the global check stopped it): the
    // solver refuses further runs until kry_*_start
    s->started = false;
    throw Error{KRY_ECOMM, "CG: another rank's in-launch exchange failed at step " + std::to_string(done) +
                               " of this run call; every rank stopped before it"};
  } else if (upd && c.status == KRY_EDEVICE && s->comm) {
    // under a communicator every step posts one allreduce on every rank: a
    // rank that reran part of its chunk alone would pair its collectives with
    // other iterations of the other ranks, so a timed-out exchange is a hard
    // error here; the step's allreduce carried the fault to every rank
    // (post_fault), which all stopped before it
    s->upd_nv = 0;
    ++s->upd_fallbacks;
    s->started = false;  // refuse further runs until kry_*_start (the state is past the history)
    throw Error{KRY_EDEVICE, "CG: the one-launch update's exchange timed out at step " + std::to_string(done) +
                                 " (a block was not resident); every rank of the communicator stopped before it"};
  } else if (upd && c.status == KRY_EDEVICE) {
    // a one-launch update timed out at step `done` and wrote nothing: the
    // steps before it stand; rerun the rest of the chunk launch per pass,
    // from that step's SpMV (p is unchanged, so it recomputes the same Ap)
    s->upd_nv = 0;
    ++s->upd_fallbacks;
    const int first = done;
    s->it_base = s->it + first;
    auto [more, pers2] = run_steps(max_steps - first, resnorms + (size_t)first * hk, &c);
    (void)pers2;
    done = first + more;
  }
  KRY_REQUIRE(c.status == 0, KRY_EDEVICE, "CG: device error status " + std::to_string(c.status));
  s->cgp_last = persistent;
  s->upd_last = upd;
  s->it += done;
  if (s->ydefer > 0 && !s->M && s->k <= 8 && !persistent)  // the in-kernel flushes of this run
    s->yfb += (s->it - s->yfb) / s->ydefer * s->ydefer;
  *steps_done = done;
  KRY_API_END
}

int kry_cg_preferred_chunk(kry_cg *s, int32_t *steps) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && steps, KRY_EINVAL, "null argument");
  KRY_REQUIRE(s->started, KRY_EINVAL, "kry_cg_start has not been called");
  KRY_HIP(hipSetDevice(s->ctx->device));
  bool persist = false;
  dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) {
    persist = cgp_launch<decltype(v0), decltype(m0), decltype(i0)>(s, 1, true);
  });
  // one launch per chunk and no halted launches after convergence: long
  // chunks cost nothing; the launch-per-pass path keeps 32
  *steps = persist ? 256 : 32;
  KRY_API_END
}

int kry_cg_path(kry_cg *s, int32_t *info) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && info, KRY_EINVAL, "null argument");
  info[0] = s->cgp_last ? 1 : 0;
  info[1] = s->cgp_fallbacks;
  KRY_API_END
}

int kry_cg_update_path(kry_cg *s, int32_t *info) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && info, KRY_EINVAL, "null argument");
  info[0] = s->upd_last ? 1 : 0;
  info[1] = s->upd_fallbacks;
  KRY_API_END
}

int kry_cg_defer_info(kry_cg *s, int32_t *D, int64_t *bytes) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && D && bytes, KRY_EINVAL, "null argument");
  *D = s->ydefer > 0 ? s->ydefer : 0;
  *bytes = s->ydefer > 0 ? s->ydefer_bytes : 0;
  KRY_API_END
}

int kry_cg_residual(kry_cg *s, double *norm2) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && norm2, KRY_EINVAL, "null argument");
  KRY_REQUIRE(s->started, KRY_EINVAL, "kry_cg_start has not been called");
  KRY_HIP(hipSetDevice(s->ctx->device));
  dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { cg_residual_impl<decltype(v0), decltype(m0), decltype(i0)>(s, norm2); });
  KRY_API_END
}

int kry_cg_get(kry_cg *s, int which, void *host) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && host && which >= 0 && which <= 2, KRY_EINVAL, "bad argument");
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  const int64_t N = s->n * (int64_t)s->k;
  if (which == 0) {
    if (s->dtype == KRY_F64) cg_ydefer_flush<double>(s);
    else cg_ydefer_flush<float>(s);
    if (s->dtype == KRY_F64)
      launch_elementwise<double>(N, s->k, OpXk<double>{static_cast<const double *>(s->x0), static_cast<const double *>(s->y), static_cast<double *>(s->xk)},
                                 nullptr, nullptr, 0, st);
    else
      launch_elementwise<float>(N, s->k, OpXk<float>{static_cast<const float *>(s->x0), static_cast<const float *>(s->y), static_cast<float *>(s->xk)},
                                nullptr, nullptr, 0, st);
    store_out(s->A, s->xk, host, s->k, dsize(s->dtype), st);
  } else {
    // 1: Ml_rk; 2: M_Ml_rk (= Ml_rk without M)
    store_out(s->A, which == 2 && s->M ? s->z : s->r, host, s->k, dsize(s->dtype), st);
  }
  KRY_HIP(hipStreamSynchronize(st));
  KRY_API_END
}

int kry_cg_scalars(kry_cg *s, double *out) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && out, KRY_EINVAL, "null argument");
  const int k = s->k;
  const int slots[4] = {S_RHO, S_RHO_PREV, S_ALPHA, S_OMEGA};
  for (int i = 0; i < 4; ++i)
    KRY_HIP(hipMemcpyAsync(out + (size_t)i * k, s->scal + (size_t)slots[i] * k, k * 8, hipMemcpyDeviceToHost,
                           s->ctx->stream));
  KRY_HIP(hipStreamSynchronize(s->ctx->stream));
  KRY_API_END
}

int kry_cg_set_preconditioners(kry_cg *s, kry_csr *M, kry_csr *Ml) {
  KRY_API_BEGIN
  KRY_REQUIRE(s, KRY_EINVAL, "null solver");
  for (kry_csr *op : {M, Ml}) {
    if (!op) continue;
    KRY_REQUIRE(op->n == s->n, KRY_EINVAL, "preconditioner shape does not match the operator");
    KRY_REQUIRE(op->dtype == s->dtype || (s->dtype == KRY_F64 && op->dtype == KRY_F32), KRY_EINVAL,
                "preconditioner dtype must match the vectors (or be float32 under float64 vectors)");
    KRY_REQUIRE(op->renumbered == s->A->renumbered && op->perm_hash == s->A->perm_hash, KRY_EINVAL,
                "preconditioner renumbered differently from the operator (build it with kry_csr_create_like)");
  }
  KRY_HIP(hipSetDevice(s->ctx->device));
  const size_t vb = ((size_t)s->n * s->k + 15) / 16 * 16 * dsize(s->dtype);
  s->M = M;
  s->Ml = Ml;
  if (M && !s->z) {
    s->z = dev_alloc(vb);
    KRY_HIP(hipMemsetAsync(s->z, 0, vb, s->ctx->stream));
  }
  if (Ml && !s->t) {
    s->t = dev_alloc(vb);
    KRY_HIP(hipMemsetAsync(s->t, 0, vb, s->ctx->stream));
  }
  KRY_HIP(hipStreamSynchronize(s->ctx->stream));
  s->started = false;
  KRY_API_END
}

int kry_cg_attach_comm(kry_cg *s, kry_comm *c, int32_t col_offset, int32_t total_k) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && c, KRY_EINVAL, "null argument");
  KRY_REQUIRE(col_offset >= 0 && total_k >= col_offset + s->k && total_k <= 4096, KRY_EINVAL,
              "bad column range");
  KRY_HIP(hipSetDevice(s->ctx->device));
  dev_free(s->gbuf);
  dev_free(s->gcrit);
  s->gbuf = nullptr;
  s->gcrit = nullptr;
  s->gbuf = static_cast<double *>(dev_alloc(((size_t)total_k + 1) * 8));  // + the fault count
  s->gcrit = static_cast<double *>(dev_alloc((size_t)total_k * 8));
  dev_free(s->hist);
  s->hist = nullptr;
  s->hist = static_cast<double *>(dev_alloc((size_t)s->chunk_cap * total_k * 8));
  s->comm = c;
  s->col_offset = col_offset;
  s->total_k = total_k;
  KRY_API_END
}

}  // extern "C"
