// MINRES device loop (reference minres.py:28-253 with the Lanczos process of
// arnoldi.py:203-281). Preconditioners are device CSR operators
// (kry_minres_set_preconditioners): the Lanczos operator is Ml A Mr, M splits
// the Lanczos vectors into p and v = M p with h[2] = sqrt(<w, M w>)
// (arnoldi.py:268-277), and x = x0 + Mr yk (minres.py:95-98).
//
// One iteration = five launches, no host sync:
//   SpMV   w = A v - h0 p_old, partial <v, w>             arnoldi.py:244-252
//   tiny   alpha = <v, w>, h[1] = alpha                   arnoldi.py:252-264
//   ortho  w -= alpha p, partial <w, w>                   arnoldi.py:264-267
//   tiny   h[2] = sqrt(<w, w>), invariance, the two old rotations and the new
//          one on R (float64), y update, resnorm = |y1|, stop test
//                                                        minres.py:193-228
//   update z = (v - R0 W0 - R1 W1) / guard(R2), W shift, yk += y0 z,
//          p_old <- p, p = v = w / guard(h[2])           minres.py:219-221,
//                                                        arnoldi.py:274-277
// Precision follows the reference under NumPy-2 promotion: Lanczos scalars
// in the vector dtype, the inner products in the inner's dtype, R / rotations
// / y / z / W in float64 (minres.py:195, 219).
#include "solver_common.hpp"

using namespace kry;

struct kry_minres {
  kry_ctx *ctx = nullptr;
  kry_csr *A = nullptr;
  int64_t n = 0;
  int k = 1;
  int dtype = 0;
  bool inner_f32 = false;  // inner products in float32 (unweighted fp32)
  void *b = nullptr, *x0 = nullptr, *yk = nullptr, *wv = nullptr, *xk = nullptr, *rt = nullptr;
  void *P[3] = {nullptr, nullptr, nullptr};  // ring: p_old, p (= v), p_new
  double *W[2] = {nullptr, nullptr};         // float64 W ring
  kry_csr *M = nullptr, *Ml = nullptr, *Mr = nullptr;  // preconditioners (null = identity)
  void *Vr[2] = {nullptr, nullptr};  // v = M p ring (with M; else v = p)
  void *mw = nullptr;                // M w (with M)
  void *t1 = nullptr, *t2 = nullptr; // Mr v (with Mr), A Mr v / raw residual (with Ml)
  double *w = nullptr;
  double *part = nullptr;
  double *scal = nullptr;
  double *hist = nullptr;
  Ctrl *ctrl = nullptr;
  // RHS sharding (kry_minres_attach_comm), as in GMRES
  kry_comm *comm = nullptr;
  double *gbuf = nullptr;   // total_k + 2 (norms, non-invariant count, fault count)
  double *gcrit = nullptr;  // total_k
  int col_offset = 0, total_k = 0;
  int chunk_cap = 0;
  int64_t it = 0;
  int wflip = 0;
  bool invariant = false;
  bool started = false;
  // one-launch update (mr_upd_kernel): upd_nv = -1 undecided, 0 not used,
  // else granules per thread; its abort word and granule region
  int upd_nv = -1;
  unsigned *upd_words = nullptr;
  int upd_fallbacks = 0;
  bool upd_used = false;
  bool upd_last = false;
};

namespace {

// scalar slots (x k each)
enum {
  M_H0 = 0, M_H1, M_H2, M_HSAFE, M_ALPHA, M_Y0, M_Y1, M_G0C, M_G0S, M_G1C, M_G1S,
  M_Z0, M_Z1, M_Z2, M_ZY, M_CRIT, M_TMP, M_COUNT
};

// store = 0 (no preconditioner M, so p is the v the update pass reads
// anyway): only the <Av, Av> partials; the update pass recomputes
// Av - alpha p with the same operations instead of re-reading a stored copy.
template <typename V, typename S>
struct OpLanczosOrtho {
  V *w;
  const V *p;
  const double *alpha;
  const double *wt;
  int k;
  int store;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&acc)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V wv[W], pv[W];
    VIO<V>::load(w, e, N, wv);
    VIO<V>::load(p, e, N, pv);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const S a = (S)alpha[(e + v) & (k - 1)];
      const S t = a * (S)pv[v];
      wv[v] = (V)((S)wv[v] - t);  // Av -= alpha * p   (arnoldi.py:264)
      if (e + v < N) {
        const double d = (double)wv[v];
        acc[v] += wt ? dterm_w(d, wt[(e + v) / k], d) : dterm(d, d);
      }
    }
    if (store) VIO<V>::store(w, e, N, wv);
  }
};

template <typename V, typename S>
struct OpMinresUpdate {
  const V *vold;   // the v this step multiplied (minres.py:187)
  const double *W0;
  double *W1z;     // holds W[0] on entry; receives z (becomes the new W[1])
  const double *W1;
  V *yk;
  const V *wv;     // Av, or Av - alpha p when ortho_here == 0
  V *pnew;         // null when the space is invariant
  const double *scal;
  int k;
  int ortho_here;  // apply Av -= alpha p here (p = vold; arnoldi.py:264)
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V va[W], ya[W], wa[W];
    VIO<V>::load(vold, e, N, va);
    VIO<V>::load(yk, e, N, ya);
    if (pnew) VIO<V>::load(wv, e, N, wa);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      if (e + v >= N) continue;
      const int c = (int)((e + v) & (k - 1));
      const double r0 = scal[M_Z0 * k + c], r1 = scal[M_Z1 * k + c], r2 = scal[M_Z2 * k + c];
      const double y0 = scal[M_ZY * k + c];
      const double t0 = r0 * W0[e + v];
      const double t1 = r1 * W1[e + v];
      const double z = (((double)va[v] - t0) - t1) / r2;  // minres.py:219
      W1z[e + v] = z;
      const double dy = y0 * z;
      ya[v] = (V)((double)ya[v] + dy);                     // minres.py:221
      if (pnew) {
        if (ortho_here) {  // the same operations as OpLanczosOrtho
          const S a = (S)scal[M_ALPHA * k + c];
          const S t = a * (S)va[v];
          wa[v] = (V)((S)wa[v] - t);
        }
        wa[v] = wa[v] / (V)scal[M_HSAFE * k + c];  // arnoldi.py:276-277
      }
    }
    VIO<V>::store(yk, e, N, ya);
    if (pnew) VIO<V>::store(pnew, e, N, wa);
  }
};

template <typename V>
struct OpDivInto {
  const V *src;
  V *dst;
  const double *den;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V a[W];
    VIO<V>::load(src, e, N, a);
#pragma unroll
    for (int v = 0; v < W; ++v) a[v] = a[v] / (V)den[(e + v) & (k - 1)];
    VIO<V>::store(dst, e, N, a);
  }
};

// ||r0|| (inner dtype S), y = [||r0||, 0], Lanczos scale guard.
template <typename V, typename S>
__global__ void mr_start_finalize(const double *part, int P, int k, double *scal) {
  __shared__ double red[kBlock];
  reduce_partials(part, P, k, red);
  const int c = threadIdx.x;
  if (c < k) {
    const S nrm = sqrt((S)red[c]);
    scal[M_TMP * k + c] = (double)nrm;
    scal[M_Y0 * k + c] = (double)nrm;
    scal[M_Y1 * k + c] = 0.0;
    scal[M_HSAFE * k + c] = (double)(nrm != S(0) ? nrm : S(1));
    for (int s = M_H0; s <= M_H2; ++s) scal[s * k + c] = 0.0;
  }
}

template <typename V, typename S>
__global__ void mr_alpha_kernel(const double *part, int P, int k, double *scal, const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  reduce_partials(part, P, k, red);
  const int c = threadIdx.x;
  if (c < k) {
    const S a = (S)red[c];
    scal[M_ALPHA * k + c] = (double)a;
    scal[M_H1 * k + c] = (double)(V)a;  // h stored in the Lanczos dtype
  }
}

template <typename V, typename S>
__global__ void mr_qr_kernel(const double *part, int P, int k, double *scal, int have_g0, int have_g1, double *hist,
                             Ctrl *ctrl, int step, double *gbuf = nullptr, int col_offset = 0, int total_k = 0) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  __shared__ double rn[kMaxCols];
  __shared__ int flag;
  reduce_partials(part, P, k, red);
  const int c = threadIdx.x;
  if (c < k) {
    const V h2 = (V)sqrt((S)red[c]);
    scal[M_H2 * k + c] = (double)h2;
    red[c] = (double)h2;
  }
  __syncthreads();
  if (threadIdx.x == 0) flag = 1;
  __syncthreads();
  if (c < k && !(red[c] <= 1.0e-14)) flag = 0;  // np.all(h[2] <= 1e-14)
  __syncthreads();
  const bool inv = flag != 0;
  __syncthreads();
  if (c < k) {
    const V h2 = (V)scal[M_H2 * k + c];
    scal[M_HSAFE * k + c] = (double)(h2 != V(0) ? h2 : V(1));
    double R0 = 0.0, R1 = scal[M_H0 * k + c], R2, R3;
    if (have_g1) {
      const double cc = scal[M_G1C * k + c], ss = scal[M_G1S * k + c];
      const double a0 = cc * R0, a1 = ss * R1, b0 = -ss * R0, b1 = cc * R1;
      R0 = a0 + a1;
      R1 = b0 + b1;
    }
    R2 = scal[M_H1 * k + c];
    R3 = (double)h2;
    if (have_g0) {
      const double cc = scal[M_G0C * k + c], ss = scal[M_G0S * k + c];
      const double a0 = cc * R1, a1 = ss * R2, b0 = -ss * R1, b1 = cc * R2;
      R1 = a0 + a1;
      R2 = b0 + b1;
      scal[M_G1C * k + c] = cc;
      scal[M_G1S * k + c] = ss;
    }
    double cs, sn, rr;
    lartg<double>(R2, R3, cs, sn, rr);
    scal[M_G0C * k + c] = cs;
    scal[M_G0S * k + c] = sn;
    R2 = rr;
    const double y0 = scal[M_Y0 * k + c], y1 = scal[M_Y1 * k + c];
    const double a0 = cs * y0, a1 = sn * y1, b0 = -sn * y0, b1 = cs * y1;
    const double ny0 = a0 + a1, ny1 = b0 + b1;
    scal[M_Z0 * k + c] = R0;
    scal[M_Z1 * k + c] = R1;
    scal[M_Z2 * k + c] = R2 != 0.0 ? R2 : 1.0;
    scal[M_ZY * k + c] = ny0;
    scal[M_Y0 * k + c] = ny1;  // y = [y[1], 0]
    scal[M_Y1 * k + c] = 0.0;
    // next step's h[0] = this step's h[2] (arnoldi.py:246-247)
    scal[M_H0 * k + c] = (double)h2;
    rn[c] = fabs(ny1);
    if (!gbuf) hist[(int64_t)step * k + c] = rn[c];
  }
  __syncthreads();
  if (gbuf) {  // sharded: this rank's share of the global vector; mr_global_check decides
    for (int t = threadIdx.x; t < total_k; t += blockDim.x) {
      const int lc = t - col_offset;
      gbuf[t] = (lc >= 0 && lc < k) ? rn[lc] : 0.0;
    }
    if (threadIdx.x == 0) {
      gbuf[total_k] = inv ? 0.0 : 1.0;  // ranks with a non-invariant column
      gbuf[total_k + 1] = 0.0;          // the fault count (post_fault)
    }
    return;
  }
  const bool conv = all_le(rn, scal + M_CRIT * k, k, &flag);
  if (threadIdx.x == 0) {
    if (inv) ctrl->invariant = 1;
    if (inv || conv) ctrl->stop_at = step + 1;
  }
}

// ------------------------------ one-launch MINRES step tail (large n, k = 1)
// Replaces mr_alpha_kernel, the Lanczos ortho pass, mr_qr_kernel and the
// update pass of a step for one right-hand side without preconditioners
// (float64 vectors, Euclidean or weighted inner), at one 512-thread block per
// CU, all resident, with the same arithmetic:
//   alpha = <v, w> (every block sums the SpMV's partials in one fixed order)
//   w' = w - alpha p kept in registers, <w', w'>_W block partial
//   all-gather -> h2 = sqrt(<w', w'>); every block then runs the scalar
//   recurrence of mr_qr_kernel (old rotations, lartg, y) from the same
//   values, so the update needs no second exchange
//   z = (v - R0 W0 - R1 W1) / guard(R2) into W0's buffer, yk += y0 z,
//   p_new = w' / guard(h2)
// so a step streams w, p, [weights,] v (= p), W0, W1, yk in and z, yk, p_new
// out in one launch instead of four. Nothing is stored before the exchange has
// completed: a timed-out exchange leaves the step's state untouched, halts
// the chunk at this step, and kry_minres_run reruns the rest with the
// separate kernels. Block 0 writes the scalar slots and the history.
constexpr int kMrBlock = 512;
constexpr int kMrU = 2;
constexpr size_t kMrWords = 16 + 2 * 2 * 256 * 2;
template <bool WT, int NV>
__global__ __launch_bounds__(kMrBlock) void mr_upd_kernel(int64_t N, const double *__restrict__ w,
                                                          const double *__restrict__ p, const double *__restrict__ wt,
                                                          double *__restrict__ W0z, const double *__restrict__ W1,
                                                          double *__restrict__ yk, double *__restrict__ pnew,
                                                          const double *__restrict__ partA, int PA, double *scal,
                                                          int have_g0, int have_g1, double *hist, Ctrl *ctrl, int step,
                                                          double *gbuf, int col_offset, int total_k, unsigned *words,
                                                          int fault_step) {
  using V = double;
  if (halted(ctrl, step)) return;
  constexpr int W = 2;
  constexpr int U = kMrU;
  constexpr int NC = NV / U;
  static_assert(NV % U == 0, "chunks must tile the thread's granules");
  __shared__ double red[kMrBlock];
  __shared__ double shv[2];
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  if (fault_step >= 0 && (fault_step & 0xffff) == step && (int)blockIdx.x == G - 1) {
    // fault injection (tests, KRY_MRU_FAULT): the last block drops out, or, with
    // KRY_MRU_FAULT_LATE = L, joins the exchange L x 0.25 ms late (the others' spin
    // gives up after kSpinLimitFault = 1 ms: either outcome must be consistent)
    const unsigned late = (unsigned)fault_step >> 16;
    if (late == 0) return;
    const unsigned long long t0 = wall_clock64();
    while (!spin_expired(t0, late * (kSpinLimitFault / 4))) __builtin_amdgcn_s_sleep(8);
  }
  const unsigned spin_limit = fault_step >= 0 ? kSpinLimitFault : kSpinLimit;
  const int64_t seg = (int64_t)NV * kMrBlock * W;
  const int64_t e0 = (int64_t)blockIdx.x * seg;
  using Seg = BufSeg<V, kMrBlock>;
  const Seg sw(w, e0, N, seg), sp(p, e0, N, seg), swt(WT ? wt : p, e0, N, seg), sW0(W0z, e0, N, seg),
      sW1(W1, e0, N, seg), sy(yk, e0, N, seg), spn(pnew, e0, N, seg);
  // phase A buffers: w, p, weights; phase B: v (= p), W0, W1, yk
  V c1[2][U][W], c2[2][U][W], c3[2][U][W], c4[2][U][W];
  auto ldA = [&](int c, int b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      sw.template load<W, 2>(c * U + u, c1[b][u]);
      sp.template load<W>(c * U + u, c2[b][u]);
      if (WT) swt.template load<W>(c * U + u, c3[b][u]);
    }
  };
  auto ldB = [&](int c, int b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      sp.template load<W>(c * U + u, c1[b][u]);
      sW0.template load<W, 2>(c * U + u, c2[b][u]);
      sW1.template load<W, 2>(c * U + u, c3[b][u]);
      sy.template load<W, 2>(c * U + u, c4[b][u]);
    }
  };
  ldA(0, 0);
  // alpha = <v, w> (arnoldi.py:252), h[1] = alpha in the Lanczos dtype
  reduce_partials<kMrBlock>(partA, PA, 1, red);
  const double alpha = red[0];
  // the old scalars, read before this block publishes (block 0 rewrites them
  // only after every block has published)
  const double h0 = scal[M_H0], g0c = scal[M_G0C], g0s = scal[M_G0S], g1c = scal[M_G1C], g1s = scal[M_G1S];
  const double y0o = scal[M_Y0], y1o = scal[M_Y1];
  // w' = w - alpha p (arnoldi.py:264) and <w', w'>_W
  V wr[NV][W];
  double acc = 0.0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int b = c & 1;
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 < NC) ldA(c + 1, b ^ 1);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int g = c * U + u;
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const V t = alpha * c2[b][u][v];
        wr[g][v] = c1[b][u][v] - t;
        const double d = wr[g][v];
        acc += WT ? dterm_w(d, c3[b][u][v], d) : dterm(d, d);  // out-of-range elements are 0
      }
    }
  }
  const double bp = block_sum1_t0(acc, red);
  unsigned long long *gran = reinterpret_cast<unsigned long long *>(words + 16) + (size_t)(step & 1) * 2 * 256;
  const unsigned tag = (unsigned)step + 1u;
  if (tid == 0) publish_partial(gran + 2 * blockIdx.x, tag, bp);
  ldB(0, 0);  // phase B's first chunk travels during the exchange
  if (tid < 64) {
    // every block commits or every block aborts (decide_exchange): no block
    // stores its segment after another gave up
    const bool ok = sweep_partials<true>(gran, G, tag, words, ctrl, &shv[0], spin_limit);
    if (tid == 0) flag = ok ? 1 : 0;
  }
  __syncthreads();
  if (!__builtin_amdgcn_readfirstlane(flag)) {
    if (tid == 0) atomicMin(&ctrl->stop_at, step);
    if (gbuf && blockIdx.x == 0) post_fault(gbuf, total_k + 2);  // sharded: tell the other ranks
    return;
  }
  // mr_qr_kernel's scalar recurrence (minres.py:193-228), same in every block
  const V h2 = (V)sqrt(shv[0]);
  const bool inv = h2 <= 1.0e-14;  // np.all(h[2] <= 1e-14)
  const V hsafe = h2 != V(0) ? h2 : V(1);
  double R0 = 0.0, R1 = h0, R2, R3;
  if (have_g1) {
    const double a0 = g1c * R0, a1 = g1s * R1, b0 = -g1s * R0, b1 = g1c * R1;
    R0 = a0 + a1;
    R1 = b0 + b1;
  }
  R2 = (double)(V)alpha;
  R3 = (double)h2;
  if (have_g0) {
    const double a0 = g0c * R1, a1 = g0s * R2, b0 = -g0s * R1, b1 = g0c * R2;
    R1 = a0 + a1;
    R2 = b0 + b1;
  }
  double cs, sn, rr;
  lartg<double>(R2, R3, cs, sn, rr);
  R2 = rr;
  const double a0 = cs * y0o, a1 = sn * y1o, b0 = -sn * y0o, b1 = cs * y1o;
  const double ny0 = a0 + a1, ny1 = b0 + b1;
  const double z2 = R2 != 0.0 ? R2 : 1.0;
  // z = (v - R0 W0 - R1 W1) / R2 (minres.py:219), yk += y0 z (221), p_new = w' / guard(h2) (arnoldi.py:274-277)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int b = c & 1;
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 < NC) ldB(c + 1, b ^ 1);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int g = c * U + u;
      V zv[W], yv[W], pv[W];
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const double t0 = R0 * c2[b][u][v];
        const double t1 = R1 * c3[b][u][v];
        const double z = ((c1[b][u][v] - t0) - t1) / z2;
        zv[v] = z;
        const double dy = ny0 * z;
        yv[v] = c4[b][u][v] + dy;
        pv[v] = wr[g][v] / hsafe;
      }
      sW0.template store<W, 2>(g, zv);
      sy.template store<W, 2>(g, yv);
      spn.template store<W>(g, pv);
    }
  }
  if (blockIdx.x == 0) {
    if (tid == 0) {
      scal[M_ALPHA] = alpha;
      scal[M_H1] = (double)(V)alpha;
      scal[M_H2] = (double)h2;
      scal[M_HSAFE] = (double)hsafe;
      if (have_g0) {
        scal[M_G1C] = g0c;
        scal[M_G1S] = g0s;
      }
      scal[M_G0C] = cs;
      scal[M_G0S] = sn;
      scal[M_Z0] = R0;
      scal[M_Z1] = R1;
      scal[M_Z2] = z2;
      scal[M_ZY] = ny0;
      scal[M_Y0] = ny1;
      scal[M_Y1] = 0.0;
      scal[M_H0] = (double)h2;
      red[0] = fabs(ny1);
      if (!gbuf) hist[step] = red[0];
    }
    __syncthreads();
    if (gbuf) {
      for (int t = tid; t < total_k; t += kMrBlock) gbuf[t] = t == col_offset ? red[0] : 0.0;
      if (tid == 0) {
        gbuf[total_k] = inv ? 0.0 : 1.0;
        gbuf[total_k + 1] = 0.0;  // the fault count (post_fault)
      }
    } else {
      const bool conv = all_le(red, scal + M_CRIT, 1, &flag);
      if (tid == 0) {
        if (inv) ctrl->invariant = 1;
        if (inv || conv) ctrl->stop_at = step + 1;
      }
    }
  }
}

template <bool WT, int NV>
void *mru_kern() {
  return reinterpret_cast<void *>(mr_upd_kernel<WT, NV>);
}

// Sharded global step decision (Lanczos invariance over all columns,
// arnoldi.py:270-272; stop rule over all columns, minres.py:162).
__global__ void mr_global_check(const double *gbuf, const double *gcrit, int total_k, double *hist, Ctrl *ctrl,
                                int step) {
  if (halted(ctrl, step)) return;
  if (peer_fault(gbuf, total_k + 2, ctrl, step)) return;
  __shared__ int flag;
  for (int t = threadIdx.x; t < total_k; t += blockDim.x) hist[(int64_t)step * total_k + t] = gbuf[t];
  const bool inv = gbuf[total_k] == 0.0;
  const bool conv = all_le(gbuf, gcrit, total_k, &flag);
  if (threadIdx.x == 0) {
    if (inv) ctrl->invariant = 1;
    if (inv || conv) ctrl->stop_at = step + 1;
  }
}

// w = Ml (A (Mr v)) (Product(Ml, A, Mr), minres.py:151), `epi` on the last product.
template <typename V, typename MV, typename I, class Epi>
void mr_apply_op(kry_minres *s, const V *v, Epi epi, double *part, int *P, const Ctrl *ctrl, int step) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const V *src = v;
  if (s->Mr) {
    V *t1 = static_cast<V *>(s->t1);
    launch_spmv_any<V>(s->Mr, k, SrcPlain<V>{v, k}, EpiStore<V>{t1, k}, nullptr, nullptr, ctrl, step, st);
    src = t1;
  }
  if (s->Ml) {
    V *t2 = static_cast<V *>(s->t2);
    launch_spmv<V, MV, I>(s->A, k, SrcPlain<V>{src, k}, EpiStore<V>{t2, k}, nullptr, nullptr, ctrl, step, st);
    launch_spmv_any<V>(s->Ml, k, SrcPlain<V>{t2, k}, epi, part, P, ctrl, step, st);
  } else {
    launch_spmv<V, MV, I>(s->A, k, SrcPlain<V>{src, k}, epi, part, P, ctrl, step, st);
  }
}

// Ml (b - A z) -> mlr, M Ml (b - A z) -> mw (with M), partials of
// <Ml r, M Ml r> (minres.py:105-118, 131-136); returns the partial count.
template <typename V, typename MV, typename I>
int mr_residual_chain(kry_minres *s, const V *z, V *mlr) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  int P = 0;
  V *raw = s->Ml ? static_cast<V *>(s->t2) : mlr;
  launch_spmv<V, MV, I>(s->A, k, SrcPlain<V>{z, k}, EpiResidual<V>{static_cast<const V *>(s->b), raw, s->w, k},
                        s->part, &P, nullptr, 0, st);
  if (s->Ml)
    launch_spmv_any<V>(s->Ml, k, SrcPlain<V>{raw, k}, EpiStoreNorm<V>{mlr, s->w, k}, s->part, &P, nullptr, 0, st);
  if (s->M)
    launch_spmv_any<V>(s->M, k, SrcPlain<V>{mlr, k}, EpiStoreDot<V>{static_cast<V *>(s->mw), mlr, s->w, k},
                       s->part, &P, nullptr, 0, st);
  return P;
}

// xk = x0 + Mr yk (minres.py:95-98)
template <typename V>
void mr_compute_xk(kry_minres *s) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const int64_t N = s->n * (int64_t)k;
  if (s->Mr)
    launch_spmv_any<V>(s->Mr, k, SrcPlain<V>{static_cast<const V *>(s->yk), k},
                       EpiAddStore<V>{static_cast<V *>(s->xk), static_cast<const V *>(s->x0), k}, nullptr, nullptr,
                       nullptr, 0, st);
  else
    launch_elementwise<V>(N, k,
                          OpXk<V>{static_cast<const V *>(s->x0), static_cast<const V *>(s->yk),
                                  static_cast<V *>(s->xk)},
                          nullptr, nullptr, 0, st);
}

template <typename V, typename MV, typename I>
void mr_start_impl(kry_minres *s) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const int64_t N = s->n * (int64_t)k;
  const V *src = s->x0 ? static_cast<const V *>(s->x0) : static_cast<const V *>(s->xk);
  V *wv = static_cast<V *>(s->wv);
  const int P = mr_residual_chain<V, MV, I>(s, src, wv);
  if (s->inner_f32)
    hipLaunchKernelGGL((mr_start_finalize<V, float>), dim3(1), dim3(kBlock), 0, st, s->part, P, k, s->scal);
  else
    hipLaunchKernelGGL((mr_start_finalize<V, double>), dim3(1), dim3(kBlock), 0, st, s->part, P, k, s->scal);
  KRY_HIP(hipGetLastError());
  // p = Ml r0 / guard(norm), v = M Ml r0 / guard(norm) (ArnoldiLanczos.__init__,
  // arnoldi.py:220-230)
  launch_elementwise<V>(N, k, OpDivInto<V>{wv, static_cast<V *>(s->P[0]), s->scal + M_HSAFE * k, k}, nullptr, nullptr,
                        0, st);
  if (s->M)
    launch_elementwise<V>(N, k,
                          OpDivInto<V>{static_cast<const V *>(s->mw), static_cast<V *>(s->Vr[0]),
                                       s->scal + M_HSAFE * k, k},
                          nullptr, nullptr, 0, st);
}

// One launch for the step tail (mr_upd_kernel) if eligible: one RHS, no
// preconditioners, float64 vectors, at most 512 * 40 granules per block at
// one block per CU (decided once per solver; KRY_MR_UPD=0 disables).
inline bool mru_launch(kry_minres *s, const double *w, const double *p, double *W0z, const double *W1, double *pnew,
                       const double *partA, int PA, int step, int64_t i) {
  const int64_t N = s->n;
  auto kern = [&](bool wt, int nv) -> void * {
    switch (nv) {
      case 8: return wt ? mru_kern<true, 8>() : mru_kern<false, 8>();
      case 16: return wt ? mru_kern<true, 16>() : mru_kern<false, 16>();
      case 24: return wt ? mru_kern<true, 24>() : mru_kern<false, 24>();
      case 32: return wt ? mru_kern<true, 32>() : mru_kern<false, 32>();
      default: return wt ? mru_kern<true, 40>() : mru_kern<false, 40>();
    }
  };
  const bool wt = s->w != nullptr;
  if (s->upd_nv < 0) {
    s->upd_nv = 0;
    const char *e = getenv("KRY_MR_UPD");
    if (!(e && atoi(e) == 0) && s->k == 1 && !s->M && !s->Ml && !s->Mr && s->dtype == KRY_F64) {
      int dev = 0, ncu = 0;
      KRY_HIP(hipGetDevice(&dev));
      KRY_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      const int gmax = ncu < 256 ? ncu : 256;
      for (int nv : {8, 16, 24, 32, 40}) {
        const int64_t G = (N + (int64_t)kMrBlock * nv * 2 - 1) / ((int64_t)kMrBlock * nv * 2);
        if (G > gmax) continue;
        int per_cu = 0;
        KRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(kern(wt, nv)),
                                                             kMrBlock, 0));
        if (per_cu >= 1) s->upd_nv = nv;
        break;
      }
      if (s->upd_nv > 0) s->upd_words = static_cast<unsigned *>(dev_alloc(kMrWords * 4));
    }
  }
  if (s->upd_nv == 0) return false;
  const int nv = s->upd_nv;
  const int G = (int)((N + (int64_t)kMrBlock * nv * 2 - 1) / ((int64_t)kMrBlock * nv * 2));
  hipStream_t st = s->ctx->stream;
  if (step == 0) KRY_HIP(hipMemsetAsync(s->upd_words, 0, kMrWords * 4, st));
  const char *fe = getenv("KRY_MRU_FAULT");  // fault injection (tests): step at which a block drops out
  int fault_step = fe ? atoi(fe) : -1;
  const char *fl = getenv("KRY_MRU_FAULT_LATE");  // ... or joins late (decide_exchange tests)
  if (fault_step >= 0 && fl) fault_step |= (atoi(fl) & 0x7fff) << 16;
  int64_t n = N;
  const double *wtp = s->w;
  double *yk = static_cast<double *>(s->yk), *scal = s->scal, *hist = s->hist;
  int have_g0 = i >= 1 ? 1 : 0, have_g1 = i >= 2 ? 1 : 0;
  Ctrl *ctrl = s->ctrl;
  double *gbuf = s->comm ? s->gbuf : nullptr;
  int col_offset = s->col_offset, total_k = s->total_k;
  unsigned *words = s->upd_words;
  void *args[] = {&n,       &w,   &p,       &wtp,        &W0z,     &W1,    &yk,    &pnew,  &partA, &PA,
                  &scal,    &have_g0, &have_g1, &hist,  &ctrl,   &step,   &gbuf, &col_offset, &total_k,
                  &words,   &fault_step};
  hipError_t le;
  {
    ProfScope ps(s->ctx, PROF_UPDATE);
    le = hipLaunchKernel(kern(wt, nv), dim3(G), dim3(kMrBlock), args, 0, st);
  }
  if (le != hipSuccess) {
    (void)hipGetLastError();
    s->upd_nv = 0;
    return false;
  }
  s->upd_used = true;
  return true;
}

template <typename V, typename S, typename MV, typename I>
void mr_run_typed(kry_minres *s, int max_steps) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const int64_t N = s->n * (int64_t)k;
  V *w = static_cast<V *>(s->wv);
  double *partA = s->part, *partB = s->part + part_rows(k) * k;
  for (int step = 0; step < max_steps; ++step) {
    const int64_t i = s->it + step;
    const V *p = static_cast<const V *>(s->P[i % 3]);
    const V *v = s->M ? static_cast<const V *>(s->Vr[i % 2]) : p;
    const V *pold = i > 0 ? static_cast<const V *>(s->P[(i + 2) % 3]) : nullptr;
    V *pnew = static_cast<V *>(s->P[(i + 1) % 3]);
    int PA, PB;
    {
      ProfScope ps(s->ctx, PROF_SPMV);
      mr_apply_op<V, MV, I>(s, v, EpiLanczos<V>{w, v, pold, s->scal + M_H0 * k, s->w, k}, partA, &PA, s->ctrl, step);
    }
    const int f = (s->wflip + step) & 1;
    if constexpr (std::is_same<V, double>::value) {
      if (mru_launch(s, w, p, s->W[f], s->W[f ^ 1], pnew, partA, PA, step, i)) {
        if (s->comm) {  // one collective per iteration: residual norms + non-invariant count
          inject_peer_fault(s->gbuf, s->total_k + 2, step, st);
          comm_allreduce(s->comm, s->gbuf, s->total_k + 2, st);
          hipLaunchKernelGGL(mr_global_check, dim3(1), dim3(kBlock), 0, st, (const double *)s->gbuf,
                             (const double *)s->gcrit, s->total_k, s->hist, s->ctrl, step);
          KRY_HIP(hipGetLastError());
        }
        continue;
      }
    }
    hipLaunchKernelGGL((mr_alpha_kernel<V, S>), dim3(1), dim3(kBlock), 0, st, partA, PA, k, s->scal, s->ctrl, step);
    PB = launch_elementwise<V>(N, k, OpLanczosOrtho<V, S>{w, p, s->scal + M_ALPHA * k, s->w, k, s->M ? 1 : 0},
                               s->M ? nullptr : partB, s->ctrl, step, st);
    if (s->M)  // MAv = M Av, h[2] = sqrt(<Av, MAv>) (arnoldi.py:268-269)
      launch_spmv_any<V>(s->M, k, SrcPlain<V>{w, k}, EpiStoreDot<V>{static_cast<V *>(s->mw), w, s->w, k}, partB, &PB,
                         s->ctrl, step, st);
    hipLaunchKernelGGL((mr_qr_kernel<V, S>), dim3(1), dim3(kBlock), 0, st, partB, PB, k, s->scal, i >= 1 ? 1 : 0,
                       i >= 2 ? 1 : 0, s->hist, s->ctrl, step, s->comm ? s->gbuf : nullptr, s->col_offset,
                       s->total_k);
    KRY_HIP(hipGetLastError());
    if (s->comm) {  // one collective per iteration: residual norms + non-invariant count
      inject_peer_fault(s->gbuf, s->total_k + 2, step, st);
      comm_allreduce(s->comm, s->gbuf, s->total_k + 2, st);
      hipLaunchKernelGGL(mr_global_check, dim3(1), dim3(kBlock), 0, st, (const double *)s->gbuf,
                         (const double *)s->gcrit, s->total_k, s->hist, s->ctrl, step);
      KRY_HIP(hipGetLastError());
    }
    {
      ProfScope ps(s->ctx, PROF_UPDATE);
      launch_elementwise<V>(N, k,
                            OpMinresUpdate<V, S>{v, s->W[f], s->W[f], s->W[f ^ 1], static_cast<V *>(s->yk), w,
                                                 pnew, s->scal, k, s->M ? 0 : 1},
                            nullptr, s->ctrl, step, st);
    }
    if (s->M)  // v = MAv / guard(h[2]) (arnoldi.py:277)
      launch_elementwise<V>(N, k,
                            OpDivInto<V>{static_cast<const V *>(s->mw), static_cast<V *>(s->Vr[(i + 1) % 2]),
                                         s->scal + M_HSAFE * k, k},
                            nullptr, s->ctrl, step, st);
  }
}

template <typename V, typename MV, typename I>
void mr_run_impl(kry_minres *s, int max_steps) {
  if (s->inner_f32)
    mr_run_typed<V, float, MV, I>(s, max_steps);
  else
    mr_run_typed<V, double, MV, I>(s, max_steps);
}

template <typename V, typename MV, typename I>
void mr_residual_impl(kry_minres *s, double *norm2) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  mr_compute_xk<V>(s);
  const int P = mr_residual_chain<V, MV, I>(s, static_cast<const V *>(s->xk), static_cast<V *>(s->rt));
  double *out = s->scal + M_TMP * k;
  hipLaunchKernelGGL(reduce_to_kernel<0>, dim3(1), dim3(kBlock), 0, st, s->part, P, k, out);
  KRY_HIP(hipGetLastError());
  KRY_HIP(hipMemcpyAsync(norm2, out, k * 8, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
}

void mr_free(kry_minres *s) {
  void *bufs[] = {s->b,  s->x0,   s->yk,   s->wv,   s->xk,    s->rt,  s->P[0], s->P[1], s->P[2], s->W[0],
                  s->W[1], s->w, s->part, s->scal, s->hist, s->ctrl, s->Vr[0], s->Vr[1], s->mw, s->t1, s->t2,
                  s->gbuf, s->gcrit, s->upd_words};
  for (void *b : bufs) dev_free(b);
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

extern "C" {

int kry_minres_create(kry_ctx *ctx, kry_csr *A, int32_t k, int dtype, kry_minres **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && A && out, KRY_EINVAL, "null argument");
  KRY_REQUIRE(is_pow2(k) && k <= kMaxCols, KRY_EUNSUPPORTED, "k must be a power of two <= 256");
  KRY_REQUIRE(dtype == A->dtype || (dtype == KRY_F64 && A->dtype == KRY_F32), KRY_EINVAL,
              "vectors must have the operator dtype (or float64 over a float32 operator)");
  KRY_HIP(hipSetDevice(ctx->device));
  auto *s = new kry_minres();
  try {
    s->ctx = ctx;
    s->A = A;
    s->n = A->n;
    s->k = k;
    s->dtype = dtype;
    const size_t elems = ((size_t)A->n * k + 15) / 16 * 16;
    const size_t vb = elems * dsize(dtype);
    void **vecs[] = {&s->b, &s->yk, &s->wv, &s->xk, &s->rt, &s->P[0], &s->P[1], &s->P[2]};
    for (void **v : vecs) {
      *v = dev_alloc(vb);
      KRY_HIP(hipMemsetAsync(*v, 0, vb, ctx->stream));
    }
    for (int i = 0; i < 2; ++i) {
      s->W[i] = static_cast<double *>(dev_alloc(elems * 8));
      KRY_HIP(hipMemsetAsync(s->W[i], 0, elems * 8, ctx->stream));
    }
    s->part = static_cast<double *>(dev_alloc(2 * part_rows(k) * k * 8));
    s->scal = static_cast<double *>(dev_alloc(M_COUNT * (size_t)k * 8));
    KRY_HIP(hipMemsetAsync(s->scal, 0, M_COUNT * (size_t)k * 8, ctx->stream));
    s->chunk_cap = 64;
    s->hist = static_cast<double *>(dev_alloc((size_t)s->chunk_cap * k * 8));
    s->ctrl = static_cast<Ctrl *>(dev_alloc(sizeof(Ctrl)));
    KRY_HIP(hipStreamSynchronize(ctx->stream));
  } catch (...) {
    mr_free(s);
    delete s;
    throw;
  }
  *out = s;
  KRY_API_END
}

int kry_minres_set_preconditioners(kry_minres *s, kry_csr *M, kry_csr *Ml, kry_csr *Mr) {
  KRY_API_BEGIN
  KRY_REQUIRE(s, KRY_EINVAL, "null solver");
  for (kry_csr *op : {M, Ml, Mr}) {
    if (!op) continue;
    KRY_REQUIRE(op->n == s->n, KRY_EINVAL, "preconditioner shape does not match the operator");
    KRY_REQUIRE(op->dtype == s->dtype || (s->dtype == KRY_F64 && op->dtype == KRY_F32), KRY_EINVAL,
                "preconditioner dtype must match the vectors (or be float32 under float64 vectors)");
    KRY_REQUIRE(op->renumbered == s->A->renumbered && op->perm_hash == s->A->perm_hash, KRY_EINVAL,
                "preconditioner renumbered differently from the operator (build it with kry_csr_create_like)");
  }
  KRY_HIP(hipSetDevice(s->ctx->device));
  const size_t vb = ((size_t)s->n * s->k + 15) / 16 * 16 * dsize(s->dtype);
  auto need = [&](void *&buf) {
    if (!buf) {
      buf = dev_alloc(vb);
      KRY_HIP(hipMemsetAsync(buf, 0, vb, s->ctx->stream));
    }
  };
  s->M = M;
  s->Ml = Ml;
  s->Mr = Mr;
  if (M) {
    need(s->Vr[0]);
    need(s->Vr[1]);
    need(s->mw);
  }
  if (Mr) need(s->t1);
  if (Ml) need(s->t2);
  KRY_HIP(hipStreamSynchronize(s->ctx->stream));
  s->started = false;
  KRY_API_END
}

int kry_minres_destroy(kry_minres *s) {
  KRY_API_BEGIN
  if (!s) return KRY_OK;
  (void)hipSetDevice(s->ctx->device);
  (void)hipStreamSynchronize(s->ctx->stream);
  mr_free(s);
  delete s;
  KRY_API_END
}

int kry_minres_start(kry_minres *s, kry_vec *b, kry_vec *x0, kry_vec *w, double *r0norm) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && r0norm, KRY_EINVAL, "null argument");
  check_vec(b, s->n, s->k, s->dtype, "b");
  if (x0) check_vec(x0, s->n, s->k, s->dtype, "x0");
  check_weights(w, s->n);
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  const size_t elems = ((size_t)s->n * s->k + 15) / 16 * 16;
  const size_t vb = b->bytes();
  load_in(s->A, b->d, s->b, s->k, dsize(s->dtype), st);  // the caller's numbering in
  dev_free(s->x0);
  s->x0 = nullptr;
  if (x0) {
    s->x0 = dev_alloc(elems * dsize(s->dtype));
    load_in(s->A, x0->d, s->x0, s->k, dsize(s->dtype), st);
  }
  dev_free(s->w);
  s->w = nullptr;
  if (w) {
    s->w = static_cast<double *>(dev_alloc(((size_t)s->n + 1) * 8));
    load_in(s->A, w->d, s->w, 1, 8, st);
  }
  s->inner_f32 = (s->dtype == KRY_F32 && !w);
  KRY_HIP(hipMemsetAsync(s->yk, 0, vb, st));
  KRY_HIP(hipMemsetAsync(s->xk, 0, vb, st));
  for (int i = 0; i < 2; ++i) KRY_HIP(hipMemsetAsync(s->W[i], 0, elems * 8, st));
  KRY_HIP(hipMemsetAsync(s->scal, 0, M_COUNT * (size_t)s->k * 8, st));
  s->it = 0;
  s->wflip = 0;
  s->invariant = false;
  dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { mr_start_impl<decltype(v0), decltype(m0), decltype(i0)>(s); });
  KRY_HIP(hipMemcpyAsync(r0norm, s->scal + M_TMP * s->k, s->k * 8, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  s->started = true;
  KRY_API_END
}

int kry_minres_set_criterion(kry_minres *s, const double *criterion) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && criterion, KRY_EINVAL, "null argument");
  if (s->comm)  // all total_k columns, in rank order
    KRY_HIP(hipMemcpyAsync(s->gcrit, criterion, s->total_k * 8, hipMemcpyHostToDevice, s->ctx->stream));
  else
    KRY_HIP(hipMemcpyAsync(s->scal + M_CRIT * s->k, criterion, s->k * 8, hipMemcpyHostToDevice, s->ctx->stream));
  KRY_HIP(hipStreamSynchronize(s->ctx->stream));
  KRY_API_END
}

int kry_minres_run(kry_minres *s, int32_t max_steps, int32_t *steps_done, double *resnorms, int32_t *invariant) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && steps_done && resnorms && invariant && max_steps >= 0, KRY_EINVAL, "bad argument");
  KRY_REQUIRE(s->started, KRY_EINVAL, "kry_minres_start has not been called");
  if (s->invariant)
    throw Error{KRY_EINVARIANT, "Krylov subspace was found to be invariant in the previous iteration."};
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  if (max_steps > s->chunk_cap) {
    dev_free(s->hist);
    s->hist = nullptr;
    s->hist = static_cast<double *>(dev_alloc((size_t)max_steps * (s->comm ? s->total_k : s->k) * 8));
    s->chunk_cap = max_steps;
  }
  const int hk = s->comm ? s->total_k : s->k;
  auto run_steps = [&](int steps, double *rows, Ctrl *c) {
    reset_ctrl(s->ctrl, st);
    s->upd_used = false;
    dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { mr_run_impl<decltype(v0), decltype(m0), decltype(i0)>(s, steps); });
    return read_chunk(s->ctx, st, s->ctrl, s->hist, steps, hk, rows, c);
  };
  Ctrl c;
  int done = run_steps(max_steps, resnorms, &c);
  const bool upd = s->upd_used;
  if (s->comm && c.status == KRY_ECOMM) {
    // the healthy rank's state has moved past the recorded history (the
    // step's update kernels ran before the global check stopped it): the
    // solver refuses further runs until kry_*_start
    s->started = false;
    throw Error{KRY_ECOMM, "MINRES: another rank's in-launch exchange failed at step " + std::to_string(done) +
                               " of this run call; every rank stopped before it"};
  }
  if (upd && c.status == KRY_EDEVICE && s->comm) {
    // one allreduce per step on every rank: no rank may rerun part of a chunk
    // alone (see kry_cg_run); the step's allreduce carried the fault to every
    // rank (post_fault), which all stopped before it
    s->upd_nv = 0;
    ++s->upd_fallbacks;
    s->started = false;  // refuse further runs until kry_*_start (the state is past the history)
    throw Error{KRY_EDEVICE, "MINRES: the one-launch step tail's exchange timed out at step " + std::to_string(done) +
                                 " (a block was not resident); every rank of the communicator stopped before it"};
  }
  if (upd && c.status == KRY_EDEVICE) {
    // the one-launch step tail timed out at step `done` and wrote nothing:
    // keep the steps before it and rerun the rest with the separate kernels,
    // from that step's SpMV (its inputs are unchanged)
    s->it += done;
    s->wflip = (s->wflip + done) & 1;
    s->upd_nv = 0;
    ++s->upd_fallbacks;
    const int more = run_steps(max_steps - done, resnorms + (size_t)done * hk, &c);
    s->it -= done;
    s->wflip = (s->wflip + 2 - (done & 1)) & 1;
    done += more;
  }
  KRY_REQUIRE(c.status == 0, KRY_EDEVICE, "MINRES: device error status " + std::to_string(c.status));
  s->upd_last = upd;
  s->it += done;
  s->wflip = (s->wflip + done) & 1;
  s->invariant = c.invariant != 0;
  *steps_done = done;
  *invariant = s->invariant ? 1 : 0;
  KRY_API_END
}

int kry_minres_update_path(kry_minres *s, int32_t *info) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && info, KRY_EINVAL, "null argument");
  info[0] = s->upd_last ? 1 : 0;
  info[1] = s->upd_fallbacks;
  KRY_API_END
}

int kry_minres_residual(kry_minres *s, double *norm2) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && norm2, KRY_EINVAL, "null argument");
  KRY_REQUIRE(s->started, KRY_EINVAL, "kry_minres_start has not been called");
  KRY_HIP(hipSetDevice(s->ctx->device));
  dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { mr_residual_impl<decltype(v0), decltype(m0), decltype(i0)>(s, norm2); });
  KRY_API_END
}

// which = 0: xk = x0 + Mr yk; 1: the current Lanczos vector p (the next step
// multiplies it); 2: v = M p; 3: the scalars [h0, h1, h2] of the last step
// (3 x k; h0 already holds the next step's h[0] = this step's h[2]).
int kry_minres_get(kry_minres *s, int which, void *host) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && host && which >= 0 && which <= 3, KRY_EINVAL, "bad argument");
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  if (which != 0) {
    KRY_REQUIRE(s->started, KRY_EINVAL, "kry_minres_start has not been called");
    if (which == 3) {
      KRY_HIP(hipMemcpyAsync(host, s->scal + M_H0 * s->k, 3 * (size_t)s->k * 8, hipMemcpyDeviceToHost, st));
    } else {
      const void *src = s->P[s->it % 3];
      if (which == 2 && s->M) src = s->Vr[s->it % 2];
      store_out(s->A, src, host, s->k, dsize(s->dtype), st);
    }
    KRY_HIP(hipStreamSynchronize(st));
    return KRY_OK;
  }
  if (s->dtype == KRY_F64)
    mr_compute_xk<double>(s);
  else
    mr_compute_xk<float>(s);
  store_out(s->A, s->xk, host, s->k, dsize(s->dtype), st);
  KRY_HIP(hipStreamSynchronize(st));
  KRY_API_END
}

// RHS sharding: see kry_gmres_attach_comm.
int kry_minres_attach_comm(kry_minres *s, kry_comm *c, int32_t col_offset, int32_t total_k) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && c, KRY_EINVAL, "null argument");
  KRY_REQUIRE(col_offset >= 0 && total_k >= col_offset + s->k && total_k <= 4096, KRY_EINVAL,
              "bad column range");
  KRY_HIP(hipSetDevice(s->ctx->device));
  dev_free(s->gbuf);
  dev_free(s->gcrit);
  s->gbuf = nullptr;
  s->gcrit = nullptr;
  s->gbuf = static_cast<double *>(dev_alloc(((size_t)total_k + 2) * 8));  // + non-invariant and fault counts
  s->gcrit = static_cast<double *>(dev_alloc((size_t)total_k * 8));
  dev_free(s->hist);
  s->hist = nullptr;
  s->hist = static_cast<double *>(dev_alloc((size_t)(s->chunk_cap > 0 ? s->chunk_cap : 1) * total_k * 8));
  s->comm = c;
  s->col_offset = col_offset;
  s->total_k = total_k;
  KRY_API_END
}

}  // extern "C"
