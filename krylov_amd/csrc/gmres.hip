// GMRES device loop (reference gmres.py:41-251, ArnoldiMGS arnoldi.py:107-200).
// Preconditioners are device CSR operators (kry_gmres_set_preconditioners):
// the Arnoldi operator is Ml A Mr (Product, gmres.py:139), M splits the basis
// into P (MGS subtraction) and V = M P (MGS inner products, solution), and
// h[k+1] = sqrt(<w, M w>) (arnoldi.py:185); without M the bases coincide.
//
// One Arnoldi step k (sweeps = 1 for "mgs", K for "mgsK"):
//   SpMV      w = A V_k, partial <V_0, w>                      arnoldi.py:176
//   per sweep, per j = 0..k:
//     tiny    alpha_j = reduce, h[j] += alpha_j                 arnoldi.py:160-161
//     MGS     w -= alpha_j V_j, partial of the next inner product
//             (<V_{j+1}, w>, or <V_0, w> for the next sweep, or <w, w>)
//   tiny      h[k+1] = sqrt(<w, w>), invariant test, Givens QR update of the
//             Hessenberg column, y update, resnorm = |y[k+1]|, stop test
//             (arnoldi.py:185-189, gmres.py:206-221)
//   normalise V_{k+1} = w / guard(h[k+1])                       arnoldi.py:191-196
// All scalars stay on the device; the host sees the residual-norm history.
#include "solver_common.hpp"

using namespace kry;

struct kry_gmres {
  kry_ctx *ctx = nullptr;
  kry_csr *A = nullptr;
  int64_t n = 0;
  int k = 1;
  int dtype = 0;
  int maxiter = 0;
  int sweeps = 1;
  size_t vstride = 0;  // elements per basis vector (padded)
  void *b = nullptr, *x0 = nullptr, *V = nullptr, *wv = nullptr, *xk = nullptr, *rt = nullptr;
  kry_csr *M = nullptr, *Ml = nullptr, *Mr = nullptr;  // preconditioners (null = identity)
  void *P = nullptr;    // (maxiter + 1) basis vectors P_j (with M; else P = V)
  void *mw = nullptr;   // M w (with M)
  void *t1 = nullptr;   // Mr v / solution scratch (with Mr)
  void *t2 = nullptr;   // A Mr v / raw residual (with Ml)
  // normalisation fused into the next SpMV (no preconditioners, MGS): w is
  // double-buffered; vpending = V_steps is still w[wcur] / hsafe
  void *wv2 = nullptr;
  int wcur = 0;
  bool vpending = false;
  // Householder Arnoldi (sweeps == 0, one right-hand side): reflector vectors
  // U_j (zero below j) and their scalars (householder.py:8-53)
  bool householder = false;
  void *U = nullptr;      // (maxiter + 2) vectors
  void *vnew = nullptr;   // the next basis vector under construction
  double *hh = nullptr;   // (maxiter + 2) x HH_COUNT
  double *w = nullptr;
  double *part = nullptr, *part1 = nullptr, *part2 = nullptr;  // partial rows (MGS ping-pong)
  double *scal = nullptr;  // alpha[k], hsafe[k], crit[k], tmp[k]
  double *h = nullptr;     // (maxiter + 2) x k, current Arnoldi column
  double *R = nullptr;     // (maxiter + 1) x maxiter x k
  double *Hs = nullptr;    // (maxiter + 1) x maxiter x k: the Hessenberg columns before rotation
  double *y = nullptr;     // (maxiter + 1) x k
  double *Gc = nullptr, *Gs = nullptr;  // maxiter x k rotations
  double *yy = nullptr;    // maxiter x k triangular-solve result
  double *hist = nullptr;
  Ctrl *ctrl = nullptr;
  // grid-barrier words of the persistent MGS kernel: 16 per chunk step,
  // zeroed once per chunk (kry_gmres_run)
  unsigned *bar = nullptr;
  // RHS sharding (kry_gmres_attach_comm): one allreduce per step of the
  // zero-padded residual-norm vector + a non-invariant count, global stop
  kry_comm *comm = nullptr;
  double *gbuf = nullptr;   // total_k + 2 (norms, non-invariant count, fault count)
  double *gcrit = nullptr;  // total_k
  int col_offset = 0, total_k = 0;
  int mgsp_E = -1;  // persistent MGS: -1 undecided, 0 not used, else elements per thread
  bool mgsp_large = false;  // gm_mgsl_kernel (basis streamed) rather than gm_mgsp_kernel
  bool mgsp_norm = false;   // the last launch also wrote V_{k+1} (no w / hsafe pending)
  int mgsp_grid = 0;
  int mgsp_fallbacks = 0;  // chunks finished launch per pass after a persistent MGS timeout
  double *mgsp_out = nullptr;  // <w, w> partials of the last persistent pass
  unsigned long long *mgs_tbuf = nullptr;  // KRY_MGS_TRACE phase sums (256 blocks x 4)
  int64_t mgs_tpasses = 0;
  int mgs_tgrid = 0;
  int chunk_cap = 0;
  int steps = 0;           // Arnoldi iterations done (arnoldi.iter)
  bool invariant = false;
  bool started = false;
  bool have_solution = false;
};

namespace {

enum { G_ALPHA = 0, G_HSAFE = 1, G_CRIT = 2, G_TMP = 3, G_COUNT = 4 };

template <typename V>
__host__ __device__ __forceinline__ V *basis(void *Vb, size_t stride, int i) {
  return static_cast<V *>(Vb) + stride * (size_t)i;
}

// One MGS pass j (arnoldi.py:159-162) in a single launch: every block first
// reduces the previous pass's partials into alpha_j = <V_j, w> (fixed order,
// identical in every block), block 0 records h[j] += alpha_j, then the block
// applies w -= alpha_j V_j to its span and emits partials of the next inner
// product (<V_{j+1}, w>, <V_0, w> for the next sweep, or <w, w>).
template <typename V>
__global__ __launch_bounds__(kBlock) void gm_mgs_kernel(int64_t N, int k, V *__restrict__ w,
                                                        const V *__restrict__ Vj, const V *__restrict__ q,
                                                        const double *__restrict__ part_in, int P_in,
                                                        double *__restrict__ part_out, double *__restrict__ h, int j,
                                                        int first_sweep, const double *__restrict__ wt,
                                                        const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  __shared__ double red[kBlock * W];
  __shared__ double alpha[kMaxCols];
  const int tid = threadIdx.x;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t ngrp = (N + W - 1) / W;
  const int64_t per = ((ngrp + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
  const int64_t v0 = per * g;
  const int64_t v1 = v0 + per < ngrp ? v0 + per : ngrp;
  // U chunks per thread per round, every load issued before any store
  constexpr int U = 4;
  V wv[U][W], vj[U][W], qv[U][W];
  auto load_round = [&](int64_t gb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t gi = gb + (int64_t)u * kBlock;
      if (gi < v1) {
        const int64_t e = gi * W;
        VIO<V>::load(w, e, N, wv[u]);
        VIO<V>::load(Vj, e, N, vj[u]);
        if (q) VIO<V>::load(q, e, N, qv[u]);
      }
    }
  };
  // the first round's vector loads do not depend on alpha_j: they are in
  // flight while the previous pass's partials are read and reduced
  int64_t gb = v0 + tid;
  if (gb < v1) load_round(gb);
  reduce_partials(part_in, P_in, k, red);
  if (tid < k) {
    const V a = (V)red[tid];
    alpha[tid] = (double)a;
    if (blockIdx.x == 0) {
      const V prev = first_sweep ? V(0) : (V)h[(int64_t)j * k + tid];
      h[(int64_t)j * k + tid] = (double)(prev + a);
    }
  }
  __syncthreads();
  double acc[W];
#pragma unroll
  for (int v = 0; v < W; ++v) acc[v] = 0.0;
  for (; gb < v1; gb += U * kBlock) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t gi = gb + (int64_t)u * kBlock;
      if (gi < v1) {
        const int64_t e = gi * W;
#pragma unroll
        for (int v = 0; v < W; ++v) {
          const V t = (V)alpha[(e + v) & (k - 1)] * vj[u][v];
          wv[u][v] = wv[u][v] - t;  // Av -= alpha * P[j]
          if (e + v < N) {
            const double a = q ? (double)qv[u][v] : (double)wv[u][v];
            const double b = (double)wv[u][v];
            acc[v] += wt ? dterm_w(a, wt[(e + v) / k], b) : dterm(a, b);
          }
        }
        VIO<V>::store(w, e, N, wv[u]);
      }
    }
    if (gb + U * kBlock < v1) load_round(gb + U * kBlock);
  }
  __syncthreads();
#pragma unroll
  for (int v = 0; v < W; ++v) red[tid * W + v] = acc[v];
  block_tree_reduce(red, kBlock * W, k);
  if (tid < k) part_out[(int64_t)g * k + tid] = red[tid];
}

// ---------------------------------------------- persistent MGS (one launch)
// All k + 1 MGS passes of Arnoldi step k (times the sweeps) in ONE launch of
// at most one 512-thread block per CU, so every block is resident and a
// grid-wide barrier is safe. Each thread keeps its E elements of w in
// registers for the whole step, so a pass moves only V_{j+1} from HBM (read
// once, prefetched while the block waits at the previous barrier) instead of
// w, V_j and V_{j+1} in and w out.
//   pass p (sweep sw, index j):  w -= alpha_j V_j  (V_j in registers)
//                                partial of <next, w>, next = V_{j+1}, V_0 of
//                                the next sweep, or w itself after the last
//   grid barrier; every block sums the G partials in the same fixed order
//   -> alpha_{j+1}, identical bits in every block (no atomics on data).
// Barrier: per-group arrival counters (group = blockIdx % 8, the XCD under
// round-robin dispatch: speed only, the counts are exact for any placement),
// the last arriver of a group bumps the top counter, one lane per block polls
// it. Partials are stored write-through (agent-scope atomic stores) and read
// back after an agent-scope acquire. Every spin is bounded: on timeout the
// kernel raises ctrl->status = KRY_EDEVICE and every block leaves.
constexpr int kMgsBlock = 512;
constexpr int kBarWords = 16;  // [0, 8) group counters, 8 top counter, 9 abort

__device__ __forceinline__ void st_agent(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double *p) {
  return __longlong_as_double(__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT));
}

// Grid barrier, split so the block can issue its next prefetch between
// arriving and waiting. Arrive after this block's partials are stored
// write-through and drained by every storing wave; the partials are read back
// with write-through-coherent loads only (ld_agent), so no L1 invalidate is
// needed. Counters: per-group arrivals (group = blockIdx % 8, the XCD under
// round-robin dispatch: speed only, the counts are exact for any placement);
// the last arriver of a group bumps the top counter.
__device__ __forceinline__ void mgs_arrive(unsigned *bar, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const int G = gridDim.x;
    const int grp = blockIdx.x & 7;
    const unsigned gsize = (unsigned)((G - grp + 7) / 8);
    const unsigned old = __hip_atomic_fetch_add(bar + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == gsize * epoch) __hip_atomic_fetch_add(bar + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Wait for every block's arrival. Every spin is bounded: on timeout the block
// raises ctrl->status = KRY_EDEVICE and the abort word, and every block
// leaves. Returns false (in every thread) in that case.
__device__ bool mgs_wait(unsigned *bar, unsigned epoch, Ctrl *ctrl, int *flag, unsigned spin_limit = kSpinLimit) {
  if (threadIdx.x == 0) {
    const int G = gridDim.x;
    const unsigned ngroups = G < 8 ? (unsigned)G : 8u;
    int ok = 1;
    unsigned spins = 0;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(bar + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ngroups * epoch) {
      __builtin_amdgcn_s_sleep(1);
      ++spins;
      if ((spins & 255u) != 0) continue;
      if (__hip_atomic_load(bar + 9, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        ok = 0;
        break;
      }
      if (spin_expired(t0, spin_limit)) {
        __hip_atomic_store(bar + 9, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&ctrl->status, (int32_t)KRY_EDEVICE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the partial loads below the poll
    *flag = ok;
  }
  __syncthreads();
  return *flag != 0;
}

// Fixed-order sum of P partial rows (same order in every block of size B).
template <int B, bool AGENT>
__device__ __forceinline__ void reduce_rows(const double *part, int P, int k, double *red) {
  const int tid = threadIdx.x;
  if (k == 1) {
    double s = 0.0;
    for (int p = tid; p < P; p += B) s += AGENT ? ld_agent(part + p) : part[p];
    block_sum1(s, red + B, red);
    return;
  }
  const int c = tid & (k - 1);
  const int step = B / k;
  double s = 0.0;
  int p = tid / k;
  for (; p + 3 * step < P; p += 4 * step) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double *a = part + (int64_t)(p + u * step) * k + c;
      v[u] = AGENT ? ld_agent(a) : *a;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s += v[u];
  }
  for (; p < P; p += step) {
    const double *a = part + (int64_t)p * k + c;
    s += AGENT ? ld_agent(a) : *a;
  }
  red[tid] = s;
  block_tree_reduce(red, B, k);
}

// One column (k = 1): the partials travel as self-validating granules
// {tag, 32 data bits} (two per block: the double's low and high words), stored
// write-through; no counters, no flag. Wave 0 of every block sweeps all G
// blocks' granules until every tag matches, then sums the values in a fixed
// order (lane l: blocks l, l + 64, ..., then a fixed xor butterfly; lane 0's
// value). tag = (step + 1) << 12 | (pass + 1) is unique within a chunk, and
// the granule words are zeroed once per chunk.
constexpr int kGranWords = 2 * 2 * 256;  // two pass parities x two words x G <= 256 blocks
// barrier words for `steps` chunk steps, then the (shared) granule words
inline size_t bar_bytes(int steps);
template <typename V, int E>
__global__ __launch_bounds__(kMgsBlock) void gm_mgsp_kernel(int64_t N, int k, V *__restrict__ w,
                                                            const V *__restrict__ Vb, size_t stride, int col,
                                                            int sweeps, const double *__restrict__ part0, int P0,
                                                            double *__restrict__ pbuf, double *__restrict__ h,
                                                            unsigned *bar, unsigned long long *gran, Ctrl *ctrl,
                                                            int step, int fault_step,
                                                            unsigned long long *tbuf = nullptr) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  constexpr int NV = E / W;
  __shared__ double red[kMgsBlock * W];
  __shared__ double alpha[kMaxCols];
  // optional phase trace (KRY_MGS_TRACE): thread 0's wall-clock split of the
  // passes into compute (incl. the wait for the prefetched vectors), block
  // reduction + publish, exchange wait
  __shared__ unsigned long long tacc[4];
  auto tmark = [&](int ph) {
    if (tbuf && threadIdx.x == 0) {
      const unsigned long long now = wall_clock64();
      if (ph >= 0) tacc[ph] += now - tacc[3];
      tacc[3] = now;
    }
  };
  if (tbuf && threadIdx.x == 0) tacc[0] = tacc[1] = tacc[2] = 0;
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  // fault injection (tests, KRY_MGS_FAULT): the last block never takes part
  // in chunk step fault_step, as a block that never became resident
  if (fault_step == step && (int)blockIdx.x == G - 1) return;
  const unsigned spin_limit = fault_step >= 0 ? kSpinLimitFault : kSpinLimit;
  // A timed-out exchange ends the launch with w (this step's A V_k) and the
  // partial buffers as they were, and halts the rest of the chunk from this
  // step on (stop_at); kry_gmres_run reruns the step on the launch-per-pass
  // path, whose first sweep rewrites every h[j] this launch may have touched.
  auto abort_step = [&]() {
    if (tid == 0) atomicMin(&ctrl->stop_at, step);
  };
  const int64_t base = (int64_t)blockIdx.x * NV * kMgsBlock;
  V wr[NV][W], vc[NV][W], vn[NV][W];
  auto ld = [&](const V *src, V(&dst)[NV][W]) {
#pragma unroll
    for (int u = 0; u < NV; ++u) VIO<V>::load(src, (base + (int64_t)u * kMgsBlock + tid) * W, N, dst[u]);
  };
  const int np = sweeps * (col + 1);
  auto next_of = [&](int p) -> const V * {  // the vector of pass p's inner product (null = w)
    const int j = p % (col + 1), sw = p / (col + 1);
    if (j < col) return Vb + stride * (size_t)(j + 1);
    if (sw + 1 < sweeps) return Vb;
    return nullptr;
  };
  ld(w, wr);
  ld(Vb, vc);
  if (const V *q = next_of(0)) ld(q, vn);
  // alpha_0 = <V_0, w> from the SpMV's partials
  reduce_rows<kMgsBlock, false>(part0, P0, k, red);
  if (tid < k) alpha[tid] = red[tid];
  __syncthreads();
  tmark(-1);
  for (int p = 0; p < np; ++p) {
    const int j = p % (col + 1);
    const bool first_sweep = p <= col;
    if (blockIdx.x == 0 && tid < k) {  // h[j] += alpha_j (arnoldi.py:160-161)
      const V a = (V)alpha[tid];
      const V prev = first_sweep ? V(0) : (V)h[(int64_t)j * k + tid];
      h[(int64_t)j * k + tid] = (double)(prev + a);
    }
    const V *q = next_of(p);
    double acc[W];
#pragma unroll
    for (int v = 0; v < W; ++v) acc[v] = 0.0;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int64_t e = (base + (int64_t)u * kMgsBlock + tid) * W;
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const V t = (V)alpha[(e + v) & (k - 1)] * vc[u][v];
        wr[u][v] = wr[u][v] - t;  // Av -= alpha * V[j] (arnoldi.py:162)
        if (e + v < N) {
          const double a = q ? (double)vn[u][v] : (double)wr[u][v];
          const double b = (double)wr[u][v];
          acc[v] += dterm(a, b);
        }
      }
    }
    tmark(0);
    if (q) {  // V_{j+1} becomes the next pass's subtrahend
#pragma unroll
      for (int u = 0; u < NV; ++u)
#pragma unroll
        for (int v = 0; v < W; ++v) vc[u][v] = vn[u][v];
    }
    double part1 = 0.0;  // k == 1: the block partial, in thread 0
    if (k == 1) {
      double t = acc[0];
#pragma unroll
      for (int v = 1; v < W; ++v) t += acc[v];
      part1 = block_sum1_t0_dpp(t, red + kMgsBlock);
    } else {
      __syncthreads();
#pragma unroll
      for (int v = 0; v < W; ++v) red[tid * W + v] = acc[v];
      block_tree_reduce(red, kMgsBlock * W, k);
    }
    double *slot = pbuf + (size_t)(p < np - 1 ? (p & 1) : 2) * G * k;
    if (p == np - 1) {  // <w, w> partials for the QR kernel; w back to HBM
      if (k == 1) {
        if (tid == 0) slot[blockIdx.x] = part1;
      } else if (tid < k) {
        slot[(int64_t)blockIdx.x * k + tid] = red[tid];
      }
#pragma unroll
      for (int u = 0; u < NV; ++u) VIO<V>::store(w, (base + (int64_t)u * kMgsBlock + tid) * W, N, wr[u]);
      tmark(1);
      if (tbuf && tid == 0)
        for (int q3 = 0; q3 < 3; ++q3) tbuf[blockIdx.x * 4 + q3] += tacc[q3];
      return;
    }
    if (k == 1) {  // granule all-gather of the block partials
      unsigned long long *gr = gran + (size_t)(p & 1) * 2 * G;
      const unsigned tag = ((unsigned)(step + 1) << 12) | (unsigned)(p + 1);
      if (tid == 0) publish_partial(gr + 2 * blockIdx.x, tag, part1);
      tmark(1);
      if (const V *q2 = next_of(p + 1)) ld(q2, vn);
      if (tid < 64) {
        const bool ok = sweep_partials<false, true>(gr, G, tag, bar, ctrl, alpha, spin_limit);
        if (tid == 0) flag = ok ? 1 : 0;
      }
      __syncthreads();
      if (!flag) return abort_step();
      tmark(2);
      continue;
    }
    if (tid < k) st_agent(slot + (int64_t)blockIdx.x * k + tid, red[tid]);
    mgs_arrive(bar, (unsigned)(p + 1));
    // prefetch the vector after next only now: the drain in mgs_arrive must
    // not wait for it (vmcnt is in order); it travels during the wait
    if (const V *q2 = next_of(p + 1)) ld(q2, vn);
    if (!mgs_wait(bar, (unsigned)(p + 1), ctrl, &flag, spin_limit)) return abort_step();
    reduce_rows<kMgsBlock, true>(slot, G, k, red);
    if (tid < k) alpha[tid] = red[tid];
    __syncthreads();
  }
}

// ------------------------ persistent MGS, next vector two passes ahead (k = 1)
// gm_mgsp_kernel's passes, exchanges and sums (bitwise the same results), with
// the partner of pass p + 1 already on chip when pass p's exchange ends: each
// wave copies its rows of the partner of pass p + 2 into LDS with
// buffer_load ... lds (no VGPRs) during pass p's exchange, so the copy has a
// whole pass to land instead of the exchange's few microseconds, and reads
// them into registers at the start of pass p + 1 after a counted vmcnt wait
// for the older copy only. Wave 0, which polls the exchange, issues its copy
// after the exchange (its polls would otherwise wait behind it: vmcnt counts
// in order). The barriers that may have a copy in flight are raw s_barriers
// with lgkmcnt waits only: __syncthreads would drain every copy.
// a workgroup barrier that leaves vector-memory copies in flight
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// The same copy issued from inline asm: the compiler then does not know the
// LDS is written by a pending vector-memory op, and does not put vmcnt(0)
// before the kernel's LDS reads (its tracking cannot tell the copy's rows
// from alpha / red); the kernel waits for the copies itself, with counted
// vmcnt. desc: {base lo, base hi, bytes, 0x00020000} (no stride), lds: the
// wave's LDS byte address (m0), voff: the lane's byte offset, soff: the
// granule's.
typedef int sdesc4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_dma16_asm(sdesc4 desc, unsigned lds, int voff, int soff) {
  int keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(desc), "s"(lds), "s"(soff)
      : "memory");
}
template <typename V, int E>
__global__ __launch_bounds__(kMgsBlock) void gm_mgsp3_kernel(int64_t N, int k, V *__restrict__ w,
                                                             const V *__restrict__ Vb, size_t stride, int col,
                                                             int sweeps, const double *__restrict__ part0, int P0,
                                                             double *__restrict__ pbuf, double *__restrict__ h,
                                                             unsigned *bar, unsigned long long *gran, Ctrl *ctrl,
                                                             int step, int fault_step,
                                                             unsigned long long *tbuf = nullptr) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  constexpr int NV = E / W;
  __shared__ __attribute__((aligned(16))) V nb[2][NV][kMgsBlock * W];  // partners two passes ahead
  __shared__ double red[kMgsBlock * W];
  __shared__ double alpha[kMaxCols];
  __shared__ unsigned long long tacc[4];  // phase trace (KRY_MGS_TRACE), as gm_mgsp_kernel's
  auto tmark = [&](int ph) {
    if (tbuf && threadIdx.x == 0) {
      const unsigned long long now = wall_clock64();
      if (ph >= 0) tacc[ph] += now - tacc[3];
      tacc[3] = now;
    }
  };
  if (tbuf && threadIdx.x == 0) tacc[0] = tacc[1] = tacc[2] = 0;
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  if (fault_step == step && (int)blockIdx.x == G - 1) return;  // KRY_MGS_FAULT (tests)
  const unsigned spin_limit = fault_step >= 0 ? kSpinLimitFault : kSpinLimit;
  auto abort_step = [&]() {
    if (tid == 0) atomicMin(&ctrl->stop_at, step);
  };
  const int64_t base = (int64_t)blockIdx.x * NV * kMgsBlock;
  V wr[NV][W], vc[NV][W], vn[NV][W];
  auto ld = [&](const V *src, V(&dst)[NV][W]) {
#pragma unroll
    for (int u = 0; u < NV; ++u) VIO<V>::load(src, (base + (int64_t)u * kMgsBlock + tid) * W, N, dst[u]);
  };
  const int wave0 = tid & ~63;
  // LDS byte addresses (the low 32 bits of a generic LDS address are the offset)
  const unsigned nb0 = (unsigned)(uintptr_t)&nb[0][0][0];
  constexpr unsigned kRow = kMgsBlock * W * sizeof(V), kBuf = NV * kRow;
  auto dma = [&](const V *src, int buf) {  // this wave's rows of src into nb[buf] (out of range: 0)
    const int64_t e0 = base * W;
    const int64_t rem = N - e0, seg = (int64_t)NV * kMgsBlock * W;
    const int64_t cnt = rem < seg ? (rem > 0 ? rem : 0) : seg;
    const uint64_t a = reinterpret_cast<uint64_t>(src + e0);
    sdesc4 d;
    d.x = (int)__builtin_amdgcn_readfirstlane((uint32_t)a);
    d.y = (int)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    d.z = __builtin_amdgcn_readfirstlane((int)(cnt * (int64_t)sizeof(V)));
    d.w = 0x00020000;
    const unsigned l0 = (unsigned)__builtin_amdgcn_readfirstlane(nb0 + buf * kBuf + wave0 * W * sizeof(V));
#pragma unroll
    for (int u = 0; u < NV; ++u)
      lds_dma16_asm(d, __builtin_amdgcn_readfirstlane(l0 + u * kRow), tid * 16,
                    __builtin_amdgcn_readfirstlane(u * kMgsBlock * 16));
  };
  auto nb_ld = [&](int buf) {  // this thread's rows of nb[buf] into vn (after the counted wait below)
    asm volatile("" ::: "memory");  // the reads stay below the wait
    typedef V vec_t __attribute__((ext_vector_type(W)));
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const vec_t t = *reinterpret_cast<const vec_t *>(&nb[buf][u][tid * W]);
#pragma unroll
      for (int v = 0; v < W; ++v) vn[u][v] = t[v];
    }
  };
  const int np = sweeps * (col + 1);
  auto next_of = [&](int p) -> const V * {  // the vector of pass p's inner product (null = w)
    if (p >= np) return nullptr;
    const int j = p % (col + 1), sw = p / (col + 1);
    if (j < col) return Vb + stride * (size_t)(j + 1);
    if (sw + 1 < sweeps) return Vb;
    return nullptr;
  };
  // h[j] += alpha_j of pass p (arnoldi.py:160-161), block 0; issued where
  // no copy of this wave is in flight (its load would wait behind them)
  auto h_update = [&](int p) {
    if (blockIdx.x == 0 && tid < k) {
      const int j = p % (col + 1);
      const V a = (V)alpha[tid];
      const V prev = p <= col ? V(0) : (V)h[(int64_t)j * k + tid];
      h[(int64_t)j * k + tid] = (double)(prev + a);
    }
  };
  ld(w, wr);
  ld(Vb, vc);
  reduce_rows<kMgsBlock, false>(part0, P0, k, red);  // alpha_0 = <V_0, w> from the SpMV's partials
  if (tid < k) alpha[tid] = red[tid];
  __syncthreads();
  h_update(0);
  // w, V_0 and h in: only copies from here on. (s_waitcnt encodings on gfx9:
  // vmcnt in bits 3:0 and 15:14, expcnt 6:4, lgkmcnt 11:8; the builtin, not
  // inline asm, so the compiler's own wait tracking sees it)
  __builtin_amdgcn_s_waitcnt(0x0F70);
  if (const V *q0 = next_of(0)) dma(q0, 0);  // the partners of passes 0 and 1
  if (const V *q1 = next_of(1)) dma(q1, 1);
  tmark(-1);
  for (int p = 0; p < np; ++p) {
    const V *q = next_of(p);
    if (q) {
      // this pass's partner was copied during an earlier exchange; the copy
      // of the next pass's (NV instructions, issued since, if any) may stay
      // in flight
      static_assert(NV < 16, "vmcnt(NV) in the low field");
      if (next_of(p + 1)) __builtin_amdgcn_s_waitcnt(0x0F70 | NV);
      else __builtin_amdgcn_s_waitcnt(0x0F70);
      nb_ld(p & 1);
    }
    double acc[W];
#pragma unroll
    for (int v = 0; v < W; ++v) acc[v] = 0.0;
    const V al = (V)alpha[0];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int64_t e = (base + (int64_t)u * kMgsBlock + tid) * W;
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const V t = al * vc[u][v];
        wr[u][v] = wr[u][v] - t;  // Av -= alpha * V[j] (arnoldi.py:162)
        if (e + v < N) {
          const double a = q ? (double)vn[u][v] : (double)wr[u][v];
          const double b = (double)wr[u][v];
          acc[v] += dterm(a, b);
        }
      }
    }
    tmark(0);
    if (q) {  // V_{j+1} becomes the next pass's subtrahend
#pragma unroll
      for (int u = 0; u < NV; ++u)
#pragma unroll
        for (int v = 0; v < W; ++v) vc[u][v] = vn[u][v];
    }
    // block sum as block_sum1_t0_dpp (same tree, same bits) over a raw barrier
    double part1 = 0.0;
    {
      double t = acc[0];
#pragma unroll
      for (int v = 1; v < W; ++v) t += acc[v];
      t = wave_sum_dpp(t);
      const int lane = tid & 63, wv = tid >> 6;
      if (lane == 0) red[kMgsBlock + wv] = t;
      raw_barrier();
      if (wv == 0) part1 = wave_sum_dpp(lane < kMgsBlock / 64 ? red[kMgsBlock + lane] : 0.0);
    }
    if (p == np - 1) {  // <w, w> partials for the QR kernel; w back to HBM
      double *slot = pbuf + (size_t)2 * G;
      if (tid == 0) slot[blockIdx.x] = part1;
#pragma unroll
      for (int u = 0; u < NV; ++u) VIO<V>::store(w, (base + (int64_t)u * kMgsBlock + tid) * W, N, wr[u]);
      tmark(1);
      if (tbuf && tid == 0)
        for (int q3 = 0; q3 < 3; ++q3) tbuf[blockIdx.x * 4 + q3] += tacc[q3];
      __builtin_amdgcn_s_waitcnt(0x0F70);
      return;
    }
    unsigned long long *gr = gran + (size_t)(p & 1) * 2 * G;
    const unsigned tag = ((unsigned)(step + 1) << 12) | (unsigned)(p + 1);
    if (tid == 0) publish_partial(gr + 2 * blockIdx.x, tag, part1);
    tmark(1);
    const V *q2 = next_of(p + 2);
    if (q2 && tid >= 64) dma(q2, p & 1);  // the partner of pass p + 2 (nb[p & 1] held pass p's, now in vn / vc)
    if (tid < 64) {
      const bool ok = sweep_partials<false, true>(gr, G, tag, bar, ctrl, alpha, spin_limit);
      if (tid == 0) flag = ok ? 1 : 0;
    }
    raw_barrier();
    if (!flag) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // no copy left in flight when the block leaves
      return abort_step();
    }
    if (tid < 64) {
      h_update(p + 1);  // (wave 0 has no copy in flight here)
      if (q2) dma(q2, p & 1);  // wave 0's rows, after its polls
    }
    tmark(2);
  }
}

// ------------------------------ persistent MGS with a two-vector lookahead
// The same Arnoldi step as gm_mgsp_kernel with half the dependent grid
// exchanges. The flattened MGS index list m = 0 .. np - 1 (vector
// V_{m mod (col + 1)}, sweep m / (col + 1)) is split into groups {0} (alpha_0
// from the SpMV's partials), {1, 2}, {3, 4}, ... (the last one single when
// np - 1 is odd). Pass t subtracts group t, whose alphas are known,
//   w -= alpha_a V_a;  w -= alpha_b V_b            (arnoldi.py:162, in order)
// and forms the partials of group t + 1 = {a', b'} in the same sweep over w:
//   c_a = <V_a', w>,  c_b = <V_b', w>,  g = <V_b', V_a'>
// so ONE exchange gives alpha_a' = c_a and
//   alpha_b' = <V_b', w - alpha_a' V_a'> = c_b - alpha_a' g
// which is MGS in exact arithmetic (arnoldi.py:159-162); in floating point
// alpha_b' moves by ~eps |alpha_a' g|, with g ~ eps for an orthonormal basis.
// After the last group, <w, w> as before. Group t + 1's vectors are
// prefetched into registers during pass t's predecessor's exchange and are
// the subtrahends of pass t + 1 (read from HBM once per step, as in
// gm_mgsp_kernel). KRY_MGS_LOOKAHEAD=0 restores gm_mgsp_kernel.
__device__ __forceinline__ int la_groups(int np) { return 1 + np / 2; }
__device__ __forceinline__ int la_first(int t) { return t == 0 ? 0 : 2 * t - 1; }
__device__ __forceinline__ int la_size(int t, int np) {
  return t >= la_groups(np) ? 0 : (t == 0 ? 1 : (np - (2 * t - 1) >= 2 ? 2 : 1));
}
// granule words: two pass parities x three values x two words x G <= 256 blocks
constexpr int kGranWordsLa = 2 * 3 * 2 * 256;
inline size_t bar_bytes(int steps) {
  return (size_t)steps * kBarWords * 4 + (size_t)(kGranWords > kGranWordsLa ? kGranWords : kGranWordsLa) * 8;
}

template <typename V, int E>
__global__ __launch_bounds__(kMgsBlock) void gm_mgsp2_kernel(int64_t N, int k, V *__restrict__ w,
                                                             const V *__restrict__ Vb, size_t stride, int col,
                                                             int sweeps, const double *__restrict__ part0, int P0,
                                                             double *__restrict__ pbuf, double *__restrict__ h,
                                                             unsigned *bar, unsigned long long *gran, Ctrl *ctrl,
                                                             int step, int fault_step,
                                                             unsigned long long *tbuf = nullptr) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  constexpr int NV = E / W;
  __shared__ unsigned long long tacc[4];  // phase trace (KRY_MGS_TRACE), as gm_mgsp_kernel's
  auto tmark = [&](int ph) {
    if (tbuf && threadIdx.x == 0) {
      const unsigned long long now = wall_clock64();
      if (ph >= 0) tacc[ph] += now - tacc[3];
      tacc[3] = now;
    }
  };
  if (tbuf && threadIdx.x == 0) tacc[0] = tacc[1] = tacc[2] = 0;
  // the current pass's subtrahends, per-thread storage (each thread reads back
  // only what it wrote: no barrier): registers hold w and the partners only
  __shared__ __attribute__((aligned(16))) V sub[2][NV][kMgsBlock * W];
  __shared__ double red[kMgsBlock * W];
  __shared__ double alpha[2 * kMaxCols];  // the current group's alphas: [i * k + column]
  __shared__ double xs[3];                // k == 1: the exchanged sums
  __shared__ int flags[3];
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  if (fault_step == step && (int)blockIdx.x == G - 1) return;  // KRY_MGS_FAULT (tests)
  const unsigned spin_limit = fault_step >= 0 ? kSpinLimitFault : kSpinLimit;
  auto abort_step = [&]() {
    if (tid == 0) atomicMin(&ctrl->stop_at, step);
  };
  // the block's segment of every vector through a buffer descriptor (no
  // per-granule address registers; out-of-range elements read as 0, so they
  // add 0 to every partial, and their stores are dropped), laid out as in
  // gm_mgsp_kernel: granule u of thread tid = elements (u B + tid) W ...
  const int64_t seg = (int64_t)NV * kMgsBlock * W;
  const int64_t e0 = (int64_t)blockIdx.x * seg;
  int colv[W];  // the column of element v of every granule (strides are multiples of 1024 >= k)
#pragma unroll
  for (int v = 0; v < W; ++v) colv[v] = (tid * W + v) & (k - 1);
  V wr[NV][W], ta[NV][W], tb[NV][W];
  typedef V vec_t __attribute__((ext_vector_type(W)));
  auto sub_ld = [&](int i, int u, V(&o)[W]) {
    const vec_t t = *reinterpret_cast<const vec_t *>(&sub[i][u][tid * W]);
#pragma unroll
    for (int v = 0; v < W; ++v) o[v] = t[v];
  };
  auto sub_st = [&](int i, int u, const V(&o)[W]) {
    vec_t t;
#pragma unroll
    for (int v = 0; v < W; ++v) t[v] = o[v];
    *reinterpret_cast<vec_t *>(&sub[i][u][tid * W]) = t;
  };
  auto ld = [&](const V *src, V(&dst)[NV][W]) {
    const BufSeg<V, kMgsBlock> sg(src, e0, N, seg);
#pragma unroll
    for (int u = 0; u < NV; ++u) sg.template load<W>(u, dst[u]);
  };
  const int np = sweeps * (col + 1);
  const int ng = la_groups(np);
  auto vec_of = [&](int m) -> const V * { return Vb + stride * (size_t)(m % (col + 1)); };
  auto ld_group = [&](int t) {  // group t's vectors into ta, tb
    const int sz = la_size(t, np);
    if (sz >= 1) ld(vec_of(la_first(t)), ta);
    if (sz == 2) ld(vec_of(la_first(t) + 1), tb);
  };
  ld(w, wr);
  ld(Vb, ta);  // V_0, the first pass's subtrahend
#pragma unroll
  for (int u = 0; u < NV; ++u) sub_st(0, u, ta[u]);
  ld_group(1);
  reduce_rows<kMgsBlock, false>(part0, P0, k, red);  // alpha_0 = <V_0, w> from the SpMV's partials
  if (tid < k) alpha[tid] = red[tid];
  __syncthreads();
  tmark(-1);
  for (int t = 0; t < ng; ++t) {
    const int sS = la_size(t, np), sT = la_size(t + 1, np);
    const int m0 = la_first(t);
    if (blockIdx.x == 0 && tid < k) {  // h[j] += alpha_j (arnoldi.py:160-161)
      for (int i = 0; i < sS; ++i) {
        const int m = m0 + i, j = m % (col + 1);
        const V a = (V)alpha[i * k + tid];
        const V prev = m <= col ? V(0) : (V)h[(int64_t)j * k + tid];
        h[(int64_t)j * k + tid] = (double)(prev + a);
      }
    }
    double acc[3][W];
#pragma unroll
    for (int n = 0; n < 3; ++n)
#pragma unroll
      for (int v = 0; v < W; ++v) acc[n][v] = 0.0;
    V a1[W], a2[W];
#pragma unroll
    for (int v = 0; v < W; ++v) {
      a1[v] = (V)alpha[colv[v]];
      a2[v] = (V)alpha[k + colv[v]];
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      V sa[W], sb[W];
      sub_ld(0, u, sa);
      if (sS == 2) sub_ld(1, u, sb);
#pragma unroll
      for (int v = 0; v < W; ++v) {
        wr[u][v] = wr[u][v] - a1[v] * sa[v];
        if (sS == 2) wr[u][v] = wr[u][v] - a2[v] * sb[v];
        const double b = (double)wr[u][v];
        if (sT == 0) {
          acc[0][v] += dterm(b, b);
        } else {
          acc[0][v] += dterm((double)ta[u][v], b);
          if (sT == 2) {
            acc[1][v] += dterm((double)tb[u][v], b);
            acc[2][v] += dterm((double)tb[u][v], (double)ta[u][v]);
          }
        }
      }
    }
    tmark(0);
    if (sT) {  // group t + 1 becomes the next pass's subtrahends
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        sub_st(0, u, ta[u]);
        if (sT == 2) sub_st(1, u, tb[u]);
      }
    }
    const int nval = sT == 2 ? 3 : 1;
    double pv[3] = {0.0, 0.0, 0.0};  // k == 1: the block partials, in wave 0
    if (k == 1) {
      double t3[3];
#pragma unroll
      for (int n = 0; n < 3; ++n) {
        t3[n] = acc[n][0];
#pragma unroll
        for (int v = 1; v < W; ++v) t3[n] += acc[n][v];
      }
      if (nval == 3) {
        block_sumn_t0_dpp<3>(t3, red + kMgsBlock);
      } else {
        double t1[1] = {t3[0]};
        block_sumn_t0_dpp<1>(t1, red + kMgsBlock);
        t3[0] = t1[0];
      }
#pragma unroll
      for (int n = 0; n < 3; ++n) pv[n] = t3[n];
    }
    if (t == ng - 1) {  // <w, w> partials for the QR kernel; w back to HBM
      double *slot = pbuf + (size_t)6 * G * k;
      if (k == 1) {
        if (tid == 0) slot[blockIdx.x] = pv[0];
      } else {
        __syncthreads();
#pragma unroll
        for (int v = 0; v < W; ++v) red[tid * W + v] = acc[0][v];
        block_tree_reduce(red, kMgsBlock * W, k);
        if (tid < k) slot[(int64_t)blockIdx.x * k + tid] = red[tid];
      }
      const BufSeg<V, kMgsBlock> ws(w, e0, N, seg);
#pragma unroll
      for (int u = 0; u < NV; ++u) ws.template store<W>(u, wr[u]);
      tmark(1);
      if (tbuf && tid == 0)
        for (int q3 = 0; q3 < 3; ++q3) tbuf[blockIdx.x * 4 + q3] += tacc[q3];
      return;
    }
    if (k == 1) {  // granule all-gather of the block partials
      unsigned long long *gr = gran + (size_t)(t & 1) * 3 * 2 * G;
      const unsigned tag = ((unsigned)(step + 1) << 12) | (unsigned)(t + 1);
      if (tid == 0) {
        if (nval == 3) publish_partials_n<3>(gr, G, tag, pv);
        else publish_partials_n<1>(gr, G, tag, pv);
      }
      tmark(1);
      ld_group(t + 2);  // travels during the wait
      // wave v sweeps value v's granules (one wave's poll state each, as in
      // the one-value kernels)
      if (tid < 64 * nval) {
        const int v = tid >> 6;
        const bool ok = sweep_partials_n<1>(gr + (size_t)2 * v * G, G, tag, bar, ctrl, xs + v, spin_limit);
        if ((tid & 63) == 0) flags[v] = ok ? 1 : 0;
      }
      __syncthreads();
      if (!(flags[0] && (nval == 1 || (flags[1] && flags[2])))) return abort_step();
      if (tid == 0) {
        const V aa = (V)xs[0];
        alpha[0] = xs[0];
        if (nval == 3) alpha[1] = xs[1] - (double)aa * xs[2];
      }
      __syncthreads();
      tmark(2);
      continue;
    }
    double *slot = pbuf + (size_t)(t & 1) * 3 * G * k;
    for (int n = 0; n < nval; ++n) {
      __syncthreads();
#pragma unroll
      for (int v = 0; v < W; ++v) red[tid * W + v] = acc[n][v];
      block_tree_reduce(red, kMgsBlock * W, k);
      if (tid < k) st_agent(slot + ((int64_t)n * G + blockIdx.x) * k + tid, red[tid]);
    }
    mgs_arrive(bar, (unsigned)(t + 1));
    ld_group(t + 2);
    if (!mgs_wait(bar, (unsigned)(t + 1), ctrl, &flag, spin_limit)) return abort_step();
    double xv[3] = {0.0, 0.0, 0.0};
    for (int n = 0; n < nval; ++n) {
      reduce_rows<kMgsBlock, true>(slot + (int64_t)n * G * k, G, k, red);
      if (tid < k) xv[n] = red[tid];
      __syncthreads();
    }
    if (tid < k) {
      const V aa = (V)xv[0];
      alpha[tid] = xv[0];
      if (nval == 3) alpha[k + tid] = xv[1] - (double)aa * xv[2];
    }
    __syncthreads();
  }
}

// ------------------------------- persistent MGS for large n (one launch)
// As gm_mgsp_kernel (same passes, exchange, abort and partial buffers), for
// n·k up to 512 · NV · W per block and one block per CU (n = 10 M doubles at
// NV = 40): only w stays in registers (NV granules of W elements per thread,
// 160 VGPRs at NV = 40); the pass's two basis vectors are streamed in chunks
// of U granules, chunk c + 1 loaded while chunk c is used, and chunk 0 of the
// next pass loaded before the exchange so it travels during the wait. A pass
// therefore reads V_j (the subtrahend) and V_{j+1} (the next inner product's
// partner) once each; V_{j+1} is read again as the next pass's subtrahend,
// with default-policy loads that leave it in the 256 MB MALL between the two
// uses. The launch-per-pass kernel moves w in and out as well: 4 vectors per
// pass against 2.
// Memory access: buffer loads/stores over the block's segment of each vector
// (descriptor from wave-uniform values; per-lane byte offset tid * 16, the
// granule's offset u * 8192 as a scalar), so no per-granule address
// registers; the descriptor's record count ends at N, so the tail's
// out-of-range granules read as 0 (they add 0 to the partials and stay 0 in
// w) and their stores are dropped.
template <typename V>
using MgslSeg = BufSeg<V, kMgsBlock>;

template <typename V, int NV, int U, bool NT>
__global__ __launch_bounds__(kMgsBlock) void gm_mgsl_kernel(int64_t N, int k, V *__restrict__ w,
                                                            const V *__restrict__ Vb, size_t stride, int col,
                                                            int sweeps, const double *__restrict__ part0, int P0,
                                                            double *__restrict__ pbuf, double *__restrict__ h,
                                                            unsigned *bar, unsigned long long *gran, Ctrl *ctrl,
                                                            int step, int fault_step, V *__restrict__ vnext) {
  static_assert(NV % U == 0, "chunks must tile the thread's granules");
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  constexpr int NC = NV / U;
  // The partner V_{j+1} of pass j is the subtrahend of pass j + 1. Its first
  // KU granule rows (KC chunks) are kept in LDS from one pass to the next, as
  // per-thread storage (each thread reads back only what it wrote: no
  // barrier), so a pass reads them from HBM once, not twice. The rest of the
  // 160 KiB holds the reduction scratch.
  constexpr int KEEP = W == 2 ? 18 : 16;
  constexpr int KU = (NV < KEEP ? NV : KEEP) / U * U;
  constexpr int KC = KU / U;
  __shared__ __attribute__((aligned(16))) V keep[KU > 0 ? KU : 1][kMgsBlock * W];
  __shared__ double red[kMgsBlock * W];
  __shared__ double alpha[kMaxCols];
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  // fault injection (tests, KRY_MGS_FAULT): the last block drops out at chunk
  // step fault_step, at its start, or (KRY_MGS_FAULT_FINAL=1, bit 16) at the
  // final normalising exchange, after the other blocks' passes are done
  const bool fault_here = fault_step >= 0 && (fault_step & 0xffff) == step && (int)blockIdx.x == G - 1;
  const bool fault_final = (fault_step >> 16) == 1;
  if (fault_here && !fault_final) return;
  const unsigned spin_limit = fault_step >= 0 ? kSpinLimitFault : kSpinLimit;
  auto abort_step = [&]() {
    if (tid == 0) atomicMin(&ctrl->stop_at, step);
  };
  const int64_t seg = (int64_t)NV * kMgsBlock * W;  // elements of the block's segment
  const int64_t e0 = (int64_t)blockIdx.x * seg;
  // element v of every granule of this thread belongs to column (tid W + v) & (k - 1)
  // (the segment and granule strides are multiples of 1024 >= k)
  int colv[W];
#pragma unroll
  for (int v = 0; v < W; ++v) colv[v] = (tid * W + v) & (k - 1);
  const MgslSeg<V> ws(w, e0, N, seg);
  V wr[NV][W];
#pragma unroll
  for (int u = 0; u < NV; ++u) ws.template load<W>(u, wr[u]);
  const int np = sweeps * (col + 1);
  auto sub_of = [&](int p) -> const V * { return Vb + stride * (size_t)(p % (col + 1)); };  // V_j of pass p
  auto next_of = [&](int p) -> const V * {  // the vector of pass p's inner product (null = w)
    const int j = p % (col + 1), sw = p / (col + 1);
    if (j < col) return Vb + stride * (size_t)(j + 1);
    if (sw + 1 < sweeps) return Vb;
    return nullptr;
  };
  // chunk buffers: [parity][granule of the chunk][element]
  V cs[2][U][W], cn[2][U][W];
  auto ld_chunk = [&](const MgslSeg<V> &sg, int c, V(&dst)[U][W]) {
#pragma unroll
    for (int u = 0; u < U; ++u) sg.template load<W>(c * U + u, dst[u]);
  };
  // the subtrahend V_j is read for the last time in this step: nontemporal
  // (NT), so the MALL keeps V_{j+1} for its second read in the next pass
  auto ld_chunk_sub = [&](const MgslSeg<V> &sg, int c, V(&dst)[U][W]) {
#pragma unroll
    for (int u = 0; u < U; ++u) sg.template load<W, NT ? 2 : 0>(c * U + u, dst[u]);
  };
  auto keep_ld = [&](int g, V(&o)[W]) {
    typedef V vec_t __attribute__((ext_vector_type(W)));
    const vec_t t = *reinterpret_cast<const vec_t *>(&keep[g][tid * W]);
#pragma unroll
    for (int v = 0; v < W; ++v) o[v] = t[v];
  };
  auto keep_st = [&](int g, const V(&o)[W]) {
    typedef V vec_t __attribute__((ext_vector_type(W)));
    vec_t t;
#pragma unroll
    for (int v = 0; v < W; ++v) t[v] = o[v];
    *reinterpret_cast<vec_t *>(&keep[g][tid * W]) = t;
  };
  {
    const MgslSeg<V> s0(sub_of(0), e0, N, seg);
#pragma unroll
    for (int g = 0; g < KU; ++g) {  // V_0's kept rows
      V t[W];
      s0.template load<W>(g, t);
      keep_st(g, t);
    }
    if (KC == 0) ld_chunk_sub(s0, 0, cs[0]);
    const V *q = next_of(0);
    ld_chunk(MgslSeg<V>(q ? q : Vb, e0, N, seg), 0, cn[0]);
  }
  reduce_rows<kMgsBlock, false>(part0, P0, k, red);  // alpha_0 = <V_0, w> from the SpMV's partials
  if (tid < k) alpha[tid] = red[tid];
  __syncthreads();
  for (int p = 0; p < np; ++p) {
    const int j = p % (col + 1);
    const bool first_sweep = p <= col;
    if (blockIdx.x == 0 && tid < k) {  // h[j] += alpha_j (arnoldi.py:160-161)
      const V a = (V)alpha[tid];
      const V prev = first_sweep ? V(0) : (V)h[(int64_t)j * k + tid];
      h[(int64_t)j * k + tid] = (double)(prev + a);
    }
    const MgslSeg<V> sv(sub_of(p), e0, N, seg);
    const V *qp = next_of(p);
    const MgslSeg<V> sq(qp ? qp : Vb, e0, N, seg);
    V al[W];
#pragma unroll
    for (int v = 0; v < W; ++v) al[v] = (V)alpha[colv[v]];
    double acc[W];
#pragma unroll
    for (int v = 0; v < W; ++v) acc[v] = 0.0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int b = c & 1;
      // keeps the scheduler from hoisting later chunks' loads (their buffers
      // would be live all at once: spills)
      __builtin_amdgcn_sched_barrier(0);
      if (c + 1 < NC) {  // the next chunk travels while this one is used
        // (the partner is loaded even when the pass pairs w with itself: no
        // branch, so the chunks stay in one block for the scheduler)
        if (c + 1 >= KC) ld_chunk_sub(sv, c + 1, cs[b ^ 1]);
        ld_chunk(sq, c + 1, cn[b ^ 1]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int g = c * U + u;
        V sub[W];
        if (c < KC) {
          keep_ld(g, sub);
          keep_st(g, cn[b][u]);  // the next pass's subtrahend
        } else {
#pragma unroll
          for (int v = 0; v < W; ++v) sub[v] = cs[b][u][v];
        }
#pragma unroll
        for (int v = 0; v < W; ++v) {
          const V t = al[v] * sub[v];
          wr[g][v] = wr[g][v] - t;  // Av -= alpha * V[j] (arnoldi.py:162)
          const double a = qp ? (double)cn[b][u][v] : (double)wr[g][v];
          acc[v] += dterm(a, (double)wr[g][v]);  // out-of-range elements are 0: they add 0
          // keeps the accumulation in program order: otherwise, for float
          // vectors, LLVM schedules the products of a whole chunk ahead of
          // the float64 adds and holds them in registers (218-578 VGPRs
          // spilled at NV = 24-40; 4-15 with this)
          asm volatile("" : "+v"(acc[v]));
        }
      }
    }
    double part1 = 0.0;  // k == 1: the block partial, in thread 0
    if (k == 1) {
      double t = acc[0];
#pragma unroll
      for (int v = 1; v < W; ++v) t += acc[v];
      part1 = block_sum1_t0_dpp(t, red + kMgsBlock);
    } else {
      __syncthreads();
#pragma unroll
      for (int v = 0; v < W; ++v) red[tid * W + v] = acc[v];
      block_tree_reduce(red, kMgsBlock * W, k);
    }
    double *slot = pbuf + (size_t)(p < np - 1 ? (p & 1) : 2) * G * k;
    if (p == np - 1 && vnext == nullptr) {  // <w, w> partials for the QR kernel; w back to HBM
      if (k == 1) {
        if (tid == 0) slot[blockIdx.x] = part1;
      } else if (tid < k) {
        slot[(int64_t)blockIdx.x * k + tid] = red[tid];
      }
#pragma unroll
      for (int u = 0; u < NV; ++u) ws.template store<W>(u, wr[u]);
      return;
    }
    if (p == np - 1) {
      // one more exchange: every block gets <w, w>, forms h[k+1] =
      // sqrt(<w, w>) and its guard exactly as the QR kernel does (same
      // value, same operations) and writes the next basis vector
      // V_{k+1} = w / guard(h[k+1]) (arnoldi.py:185,191-196) straight from
      // its registers; w itself is not written back. The QR kernel reads
      // the exchanged sum as a single partial row (slot 2, row 0).
      double *tot = pbuf + (size_t)2 * G * k;
      if (fault_here) return;  // KRY_MGS_FAULT_FINAL: never joins the normalising exchange
      if (k == 1) {
        unsigned long long *gr = gran + (size_t)(p & 1) * 2 * G;
        const unsigned tag = ((unsigned)(step + 1) << 12) | (unsigned)(p + 1);
        if (tid == 0) publish_partial(gr + 2 * blockIdx.x, tag, part1);
        if (tid < 64) {
          const bool ok = sweep_partials<false, true>(gr, G, tag, bar, ctrl, alpha, spin_limit);
          if (tid == 0) flag = ok ? 1 : 0;
        }
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(flag)) return abort_step();
      } else {
        double *xs = pbuf + (size_t)(p & 1) * G * k;
        if (tid < k) st_agent(xs + (int64_t)blockIdx.x * k + tid, red[tid]);
        mgs_arrive(bar, (unsigned)(p + 1));
        if (!mgs_wait(bar, (unsigned)(p + 1), ctrl, &flag, spin_limit)) return abort_step();
        reduce_rows<kMgsBlock, true>(xs, G, k, red);
        if (tid < k) alpha[tid] = red[tid];
        __syncthreads();
      }
      if (blockIdx.x == 0 && tid < k) tot[tid] = alpha[tid];
      V hs[W];
#pragma unroll
      for (int v = 0; v < W; ++v) hs[v] = safe<V>(sqrt((V)alpha[colv[v]]));
      const MgslSeg<V> vs(vnext, e0, N, seg);
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        V o[W];
#pragma unroll
        for (int v = 0; v < W; ++v) o[v] = wr[u][v] / hs[v];
        vs.template store<W>(u, o);
      }
      return;
    }
    // chunk 0 of the next pass: its loads must not be waited on by the
    // exchange's drains (vmcnt is in order), so they are issued after the
    // publish / arrive and travel during the wait
    const MgslSeg<V> sv2(sub_of(p + 1), e0, N, seg);
    const V *q2 = next_of(p + 1);
    if (k == 1) {  // granule all-gather of the block partials
      unsigned long long *gr = gran + (size_t)(p & 1) * 2 * G;
      const unsigned tag = ((unsigned)(step + 1) << 12) | (unsigned)(p + 1);
      if (tid == 0) publish_partial(gr + 2 * blockIdx.x, tag, part1);
      if (KC == 0) ld_chunk_sub(sv2, 0, cs[0]);
      ld_chunk(MgslSeg<V>(q2 ? q2 : Vb, e0, N, seg), 0, cn[0]);
      if (tid < 64) {
        const bool ok = sweep_partials<false, true>(gr, G, tag, bar, ctrl, alpha, spin_limit);
        if (tid == 0) flag = ok ? 1 : 0;
      }
      __syncthreads();
      if (!__builtin_amdgcn_readfirstlane(flag)) return abort_step();
      continue;
    }
    if (tid < k) st_agent(slot + (int64_t)blockIdx.x * k + tid, red[tid]);
    mgs_arrive(bar, (unsigned)(p + 1));
    if (KC == 0) ld_chunk_sub(sv2, 0, cs[0]);
    ld_chunk(MgslSeg<V>(q2 ? q2 : Vb, e0, N, seg), 0, cn[0]);
    if (!mgs_wait(bar, (unsigned)(p + 1), ctrl, &flag, spin_limit)) return abort_step();
    reduce_rows<kMgsBlock, true>(slot, G, k, red);
    if (tid < k) alpha[tid] = red[tid];
    __syncthreads();
  }
}

// ----------------------- streamed persistent MGS with the two-vector lookahead
// gm_mgsl_kernel's streaming (w in registers, the basis streamed in chunks of
// one granule per vector, chunk c + 1 loaded while chunk c is used, chunk 0
// of the next pass loaded before the exchange) with gm_mgsp2_kernel's groups:
// pass t streams its two subtrahends (group t) and its two partners (group
// t + 1) and performs ONE exchange of <V_a', w>, <V_b', w>, <V_b', V_a'>. The
// first KU granule rows of each partner are kept in LDS for its second read
// as a subtrahend in the next pass (per-thread storage, no barrier), as the
// one-vector kernel keeps its partner's. After the last group: the <w, w>
// exchange and V_{k+1} = w / guard(h[k+1]) from the registers, as there.
template <typename V, int NV, bool NT>
__global__ __launch_bounds__(kMgsBlock) void gm_mgsl2_kernel(int64_t N, int k, V *__restrict__ w,
                                                             const V *__restrict__ Vb, size_t stride, int col,
                                                             int sweeps, const double *__restrict__ part0, int P0,
                                                             double *__restrict__ pbuf, double *__restrict__ h,
                                                             unsigned *bar, unsigned long long *gran, Ctrl *ctrl,
                                                             int step, int fault_step, V *__restrict__ vnext) {
  if (halted(ctrl, step)) return;
  constexpr int W = Vec16<V>::W;
  constexpr int KEEP = W == 2 ? 9 : 8;  // granule rows kept per partner (two partners: ~147 KiB)
  constexpr int KU = NV < KEEP ? NV : KEEP;
  __shared__ __attribute__((aligned(16))) V keep[2][KU][kMgsBlock * W];
  __shared__ double red[kMgsBlock * W];
  __shared__ double alpha[2 * kMaxCols];
  __shared__ double xs[3];
  __shared__ int flags[3];
  __shared__ int flag;
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  const bool fault_here = fault_step >= 0 && (fault_step & 0xffff) == step && (int)blockIdx.x == G - 1;
  const bool fault_final = (fault_step >> 16) == 1;
  if (fault_here && !fault_final) return;
  const unsigned spin_limit = fault_step >= 0 ? kSpinLimitFault : kSpinLimit;
  auto abort_step = [&]() {
    if (tid == 0) atomicMin(&ctrl->stop_at, step);
  };
  const int64_t seg = (int64_t)NV * kMgsBlock * W;
  const int64_t e0 = (int64_t)blockIdx.x * seg;
  int colv[W];
#pragma unroll
  for (int v = 0; v < W; ++v) colv[v] = (tid * W + v) & (k - 1);
  typedef BufSeg<V, kMgsBlock> Seg;
  const Seg ws(w, e0, N, seg);
  V wr[NV][W];
#pragma unroll
  for (int u = 0; u < NV; ++u) ws.template load<W>(u, wr[u]);
  const int np = sweeps * (col + 1);
  const int ng = la_groups(np);
  auto vec_of = [&](int m) -> const V * { return Vb + stride * (size_t)(m % (col + 1)); };
  typedef V vec_t __attribute__((ext_vector_type(W)));
  auto keep_ld = [&](int s, int g, V(&o)[W]) {
    const vec_t t = *reinterpret_cast<const vec_t *>(&keep[s][g][tid * W]);
#pragma unroll
    for (int v = 0; v < W; ++v) o[v] = t[v];
  };
  auto keep_st = [&](int s, int g, const V(&o)[W]) {
    vec_t t;
#pragma unroll
    for (int v = 0; v < W; ++v) t[v] = o[v];
    *reinterpret_cast<vec_t *>(&keep[s][g][tid * W]) = t;
  };
  // chunk buffers [parity][stream][element]: streams S_a, S_b, T_a, T_b
  V cb[2][4][W];
  // chunk c of pass t's streams into cb[par] (the subtrahends only beyond the kept rows)
  auto ld_chunk = [&](int t, int c, int par) {
    const int sS = la_size(t, np), sT = la_size(t + 1, np);
    const int m0 = la_first(t), m1 = la_first(t + 1);
    if (c >= KU) {
      Seg(vec_of(m0), e0, N, seg).template load<W, NT ? 2 : 0>(c, cb[par][0]);
      if (sS == 2) Seg(vec_of(m0 + 1), e0, N, seg).template load<W, NT ? 2 : 0>(c, cb[par][1]);
    }
    if (sT >= 1) Seg(vec_of(m1), e0, N, seg).template load<W>(c, cb[par][2]);
    if (sT == 2) Seg(vec_of(m1 + 1), e0, N, seg).template load<W>(c, cb[par][3]);
  };
  {
    const Seg s0(Vb, e0, N, seg);
#pragma unroll
    for (int g = 0; g < KU; ++g) {  // V_0's kept rows
      V t[W];
      s0.template load<W>(g, t);
      keep_st(0, g, t);
    }
    ld_chunk(0, 0, 0);
  }
  reduce_rows<kMgsBlock, false>(part0, P0, k, red);  // alpha_0 = <V_0, w> from the SpMV's partials
  if (tid < k) alpha[tid] = red[tid];
  __syncthreads();
  for (int t = 0; t < ng; ++t) {
    const int sS = la_size(t, np), sT = la_size(t + 1, np);
    const int m0 = la_first(t);
    if (blockIdx.x == 0 && tid < k) {  // h[j] += alpha_j (arnoldi.py:160-161)
      for (int i = 0; i < sS; ++i) {
        const int m = m0 + i, j = m % (col + 1);
        const V a = (V)alpha[i * k + tid];
        const V prev = m <= col ? V(0) : (V)h[(int64_t)j * k + tid];
        h[(int64_t)j * k + tid] = (double)(prev + a);
      }
    }
    V a1[W], a2[W];
#pragma unroll
    for (int v = 0; v < W; ++v) {
      a1[v] = (V)alpha[colv[v]];
      a2[v] = (V)alpha[k + colv[v]];
    }
    double acc[3][W];
#pragma unroll
    for (int n = 0; n < 3; ++n)
#pragma unroll
      for (int v = 0; v < W; ++v) acc[n][v] = 0.0;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int b = c & 1;
      __builtin_amdgcn_sched_barrier(0);
      if (c + 1 < NV) ld_chunk(t, c + 1, b ^ 1);
      V sa[W], sb[W];
      if (c < KU) {
        keep_ld(0, c, sa);
        if (sS == 2) keep_ld(1, c, sb);
        if (sT >= 1) keep_st(0, c, cb[b][2]);  // the next pass's subtrahends
        if (sT == 2) keep_st(1, c, cb[b][3]);
      } else {
#pragma unroll
        for (int v = 0; v < W; ++v) {
          sa[v] = cb[b][0][v];
          sb[v] = cb[b][1][v];
        }
      }
#pragma unroll
      for (int v = 0; v < W; ++v) {
        wr[c][v] = wr[c][v] - a1[v] * sa[v];
        if (sS == 2) wr[c][v] = wr[c][v] - a2[v] * sb[v];
        const double x = (double)wr[c][v];
        if (sT == 0) {
          acc[0][v] += dterm(x, x);
        } else {
          acc[0][v] += dterm((double)cb[b][2][v], x);
          if (sT == 2) {
            acc[1][v] += dterm((double)cb[b][3][v], x);
            acc[2][v] += dterm((double)cb[b][3][v], (double)cb[b][2][v]);
          }
        }
        asm volatile("" : "+v"(acc[0][v]));  // the accumulation in program order (see gm_mgsl_kernel)
      }
    }
    const int nval = sT == 2 ? 3 : 1;
    double pv[3] = {0.0, 0.0, 0.0};
    if (k == 1) {
      double t3[3];
#pragma unroll
      for (int n = 0; n < 3; ++n) {
        t3[n] = acc[n][0];
#pragma unroll
        for (int v = 1; v < W; ++v) t3[n] += acc[n][v];
      }
      if (nval == 3) {
        block_sumn_t0_dpp<3>(t3, red + kMgsBlock);
      } else {
        double t1[1] = {t3[0]};
        block_sumn_t0_dpp<1>(t1, red + kMgsBlock);
        t3[0] = t1[0];
      }
#pragma unroll
      for (int n = 0; n < 3; ++n) pv[n] = t3[n];
    }
    if (t == ng - 1) {
      double *tot = pbuf + (size_t)6 * G * k;
      if (vnext == nullptr) {  // <w, w> partials for the QR kernel; w back to HBM
        if (k == 1) {
          if (tid == 0) tot[blockIdx.x] = pv[0];
        } else {
          __syncthreads();
#pragma unroll
          for (int v = 0; v < W; ++v) red[tid * W + v] = acc[0][v];
          block_tree_reduce(red, kMgsBlock * W, k);
          if (tid < k) tot[(int64_t)blockIdx.x * k + tid] = red[tid];
        }
#pragma unroll
        for (int u = 0; u < NV; ++u) ws.template store<W>(u, wr[u]);
        return;
      }
      // the <w, w> exchange, h[k+1] and its guard as the QR kernel forms
      // them, and V_{k+1} = w / guard(h[k+1]) from the registers
      // (arnoldi.py:185,191-196); the QR kernel reads the sum as one row
      if (fault_here) return;  // KRY_MGS_FAULT_FINAL: never joins the normalising exchange
      if (k == 1) {
        unsigned long long *gr = gran + (size_t)(t & 1) * 3 * 2 * G;
        const unsigned tag = ((unsigned)(step + 1) << 12) | (unsigned)(t + 1);
        if (tid == 0) publish_partials_n<1>(gr, G, tag, pv);
        if (tid < 64) {
          const bool ok = sweep_partials_n<1>(gr, G, tag, bar, ctrl, xs, spin_limit);
          if (tid == 0) {
            flag = ok ? 1 : 0;
            alpha[0] = xs[0];
          }
        }
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(flag)) return abort_step();
      } else {
        double *xsl = pbuf + (size_t)(t & 1) * 3 * G * k;
        __syncthreads();
#pragma unroll
        for (int v = 0; v < W; ++v) red[tid * W + v] = acc[0][v];
        block_tree_reduce(red, kMgsBlock * W, k);
        if (tid < k) st_agent(xsl + (int64_t)blockIdx.x * k + tid, red[tid]);
        mgs_arrive(bar, (unsigned)(t + 1));
        if (!mgs_wait(bar, (unsigned)(t + 1), ctrl, &flag, spin_limit)) return abort_step();
        reduce_rows<kMgsBlock, true>(xsl, G, k, red);
        if (tid < k) alpha[tid] = red[tid];
        __syncthreads();
      }
      if (blockIdx.x == 0 && tid < k) tot[tid] = alpha[tid];
      V hs[W];
#pragma unroll
      for (int v = 0; v < W; ++v) hs[v] = safe<V>(sqrt((V)alpha[colv[v]]));
      const Seg vs(vnext, e0, N, seg);
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        V o[W];
#pragma unroll
        for (int v = 0; v < W; ++v) o[v] = wr[u][v] / hs[v];
        vs.template store<W>(u, o);
      }
      return;
    }
    if (k == 1) {  // granule all-gather of the block partials, one wave per value
      unsigned long long *gr = gran + (size_t)(t & 1) * 3 * 2 * G;
      const unsigned tag = ((unsigned)(step + 1) << 12) | (unsigned)(t + 1);
      if (tid == 0) {
        if (nval == 3) publish_partials_n<3>(gr, G, tag, pv);
        else publish_partials_n<1>(gr, G, tag, pv);
      }
      ld_chunk(t + 1, 0, 0);  // chunk 0 of the next pass travels during the wait
      if (tid < 64 * nval) {
        const int v = tid >> 6;
        const bool ok = sweep_partials_n<1>(gr + (size_t)2 * v * G, G, tag, bar, ctrl, xs + v, spin_limit);
        if ((tid & 63) == 0) flags[v] = ok ? 1 : 0;
      }
      __syncthreads();
      if (!(flags[0] && (nval == 1 || (flags[1] && flags[2])))) return abort_step();
      if (tid == 0) {
        const V aa = (V)xs[0];
        alpha[0] = xs[0];
        if (nval == 3) alpha[1] = xs[1] - (double)aa * xs[2];
      }
      __syncthreads();
      continue;
    }
    double *slot = pbuf + (size_t)(t & 1) * 3 * G * k;
    for (int n = 0; n < nval; ++n) {
      __syncthreads();
#pragma unroll
      for (int v = 0; v < W; ++v) red[tid * W + v] = acc[n][v];
      block_tree_reduce(red, kMgsBlock * W, k);
      if (tid < k) st_agent(slot + ((int64_t)n * G + blockIdx.x) * k + tid, red[tid]);
    }
    mgs_arrive(bar, (unsigned)(t + 1));
    ld_chunk(t + 1, 0, 0);
    if (!mgs_wait(bar, (unsigned)(t + 1), ctrl, &flag, spin_limit)) return abort_step();
    double xv[3] = {0.0, 0.0, 0.0};
    for (int n = 0; n < nval; ++n) {
      reduce_rows<kMgsBlock, true>(slot + (int64_t)n * G * k, G, k, red);
      if (tid < k) xv[n] = red[tid];
      __syncthreads();
    }
    if (tid < k) {
      const V aa = (V)xv[0];
      alpha[tid] = xv[0];
      if (nval == 3) alpha[k + tid] = xv[1] - (double)aa * xv[2];
    }
    __syncthreads();
  }
}

// out = src / hsafe  (arnoldi.py:193-195, the guarded normalisation)
template <typename V>
struct OpScaleDiv {
  const V *src;
  V *dst;
  const double *hsafe;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V a[W];
    VIO<V>::load(src, e, N, a);
#pragma unroll
    for (int v = 0; v < W; ++v) a[v] = a[v] / (V)hsafe[(e + v) & (k - 1)];
    VIO<V>::store(dst, e, N, a);
  }
};

// xk = x0 + sum_i yy_i V_i, summed left to right from 0 (gmres.py:97-98)
template <typename V>
struct OpBasisCombo {
  const V *Vb;
  size_t stride;
  int m;
  const double *yy;
  const V *x0;
  V *xk;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V acc[W], t[W];
#pragma unroll
    for (int v = 0; v < W; ++v) acc[v] = V(0);
    for (int i = 0; i < m; ++i) {
      VIO<V>::load(Vb + stride * (size_t)i, e, N, t);
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const V p = (V)yy[(int64_t)i * k + ((e + v) & (k - 1))] * t[v];
        acc[v] = acc[v] + p;
      }
    }
    if (x0) {
      VIO<V>::load(x0, e, N, t);
    } else {
#pragma unroll
      for (int v = 0; v < W; ++v) t[v] = V(0);
    }
#pragma unroll
    for (int v = 0; v < W; ++v) t[v] = t[v] + acc[v];
    VIO<V>::store(xk, e, N, t);
  }
};

// ||r0|| -> y[0], hsafe (for V_0 = r0 / guard(||r0||)), tmp (host copy)
template <typename S>
__global__ void gm_start_finalize(const double *part, int P, int k, double *scal, double *y) {
  __shared__ double red[kBlock];
  reduce_partials(part, P, k, red);
  const int c = threadIdx.x;
  if (c < k) {
    const S nrm = sqrt((S)red[c]);
    y[c] = (double)nrm;
    scal[G_HSAFE * k + c] = (double)safe<S>(nrm);
    scal[G_TMP * k + c] = (double)nrm;
  }
}

// alpha_j = <V_j, w>; h[j] += alpha_j   (h[j] starts at 0.0 each step)
template <typename S>
__global__ void gm_coef_kernel(const double *part, int P, int k, double *scal, double *h, int j, int first_sweep,
                               const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  reduce_partials(part, P, k, red);
  const int c = threadIdx.x;
  if (c < k) {
    const S a = (S)red[c];
    scal[G_ALPHA * k + c] = (double)a;
    const S prev = first_sweep ? S(0) : (S)h[(int64_t)j * k + c];
    h[(int64_t)j * k + c] = (double)(prev + a);
  }
}

constexpr int kQrTile = 2048;  // doubles per LDS-staged array of gm_qr_kernel (3 x 16 KB)

// h[k+1] = sqrt(<w, w>); invariance; Givens update of column `col`
// (gmres.py:206-221); resnorm |y[col+1]|; stop test.
template <typename S>
__global__ void gm_qr_kernel(const double *part, int P, int k, double *scal, double *h, double *R, double *y,
                             double *Gc, double *Gs, int col, int maxiter, double *hist, Ctrl *ctrl, int step,
                             int hgiven = 0, double *gbuf = nullptr, int col_offset = 0, int total_k = 0,
                             double *Hs = nullptr) {
  __shared__ double red[kBlock];
  __shared__ double rn[kMaxCols];
  __shared__ double qGc[kQrTile], qGs[kQrTile], qH[kQrTile];
  __shared__ int flag;
  const int c = threadIdx.x;
  const int64_t ld = (int64_t)maxiter * k;  // R row stride
  const int T = kQrTile / k > 0 ? kQrTile / k : 1;  // rotations per LDS tile (below)
  const int nt0 = col < T ? col : T;
  // The step's independent loads go out together, before the first wait
  // (each is a miss to data an earlier kernel wrote, ~1 us when chained):
  // this thread's item of rotation tile 0, y[col], y[col + 1] and h[0].
  const bool own0 = c < nt0 * k;
  double pg0 = 0.0, ps0 = 0.0, ph0 = 0.0, py0 = 0.0, py1 = 0.0, pc0 = 0.0;
  if (own0) {
    pg0 = Gc[c];
    ps0 = Gs[c];
    ph0 = h[c + k];
  }
  if (c < k) {
    py0 = y[(int64_t)col * k + c];
    py1 = y[(int64_t)(col + 1) * k + c];
    pc0 = h[c];
  }
  if (halted(ctrl, step)) {
    // sharded: this step's MGS exchange timed out here, tell the other ranks
    if (gbuf && local_fault_at(ctrl, step)) post_fault(gbuf, total_k + 2);
    return;
  }
  if (!hgiven) reduce_partials(part, P, k, red);  // else h[k+1] is already in h (Householder)
  if (c < k) {
    const S hk1 = hgiven ? (S)h[(int64_t)(col + 1) * k + c] : sqrt((S)red[c]);
    h[(int64_t)(col + 1) * k + c] = (double)hk1;
    red[c] = (double)hk1;
  }
  __syncthreads();
  if (Hs)  // the Arnoldi relation's H[:col+2, col] (the reference's h column)
    for (int t = threadIdx.x; t < (col + 2) * k; t += blockDim.x)
      Hs[(t / k) * ld + (int64_t)col * k + t % k] = h[t];
  // np.all(h[k+1] <= 1e-14) over the columns (arnoldi.py:187)
  if (threadIdx.x == 0) flag = 1;
  __syncthreads();
  if (c < k && !(red[c] <= 1.0e-14)) flag = 0;
  __syncthreads();
  const bool inv = flag != 0;
  __syncthreads();
  // R[:col+2, col] = h[:col+2], then the previous rotations (gmres.py:208-210).
  // Rotation i finalises R[i] and hands R[i+1] on: carry it in a register
  // so the chain is arithmetic only (same operations, same bits). The
  // rotations and the h column are first staged through LDS by the whole
  // block, a tile at a time: the chain then waits on LDS, not on one global
  // round trip per rotation (the R store of rotation i kept the loads of
  // rotation i + 1 behind it: ~0.35 us per rotation, 10 us per step at j = 30).
  S carry = c < k ? (S)pc0 : S(0);
  {
    for (int i0 = 0; i0 < col; i0 += T) {
      const int nt = col - i0 < T ? col - i0 : T;
      __syncthreads();
      int t0 = threadIdx.x;
      if (i0 == 0) {  // the prefetched item
        if (own0) {
          qGc[c] = pg0;
          qGs[c] = ps0;
          qH[c] = ph0;
        }
        t0 += blockDim.x;
      }
      for (int t = t0; t < nt * k; t += blockDim.x) {
        const int64_t g = (int64_t)i0 * k + t;  // rotation i0 + t / k, column t % k
        qGc[t] = Gc[g];
        qGs[t] = Gs[g];
        qH[t] = h[g + k];
      }
      __syncthreads();
      if (c < k) {
        for (int i = 0; i < nt; ++i) {
          const S cc = (S)qGc[i * k + c], ss = (S)qGs[i * k + c];
          const S r0 = carry, r1 = (S)qH[i * k + c];
          const S a0 = cc * r0, a1 = ss * r1;
          const S b0 = -ss * r0, b1 = cc * r1;
          R[(int64_t)(i0 + i) * ld + (int64_t)col * k + c] = (double)(a0 + a1);
          carry = b0 + b1;
        }
      }
    }
  }
  if (c < k) {
    const S hk1 = (S)red[c];
    scal[G_HSAFE * k + c] = (double)safe<S>(hk1);
    S cs, sn, rr;
    lartg<S>(carry, (S)h[(int64_t)(col + 1) * k + c], cs, sn, rr);
    Gc[(int64_t)col * k + c] = (double)cs;
    Gs[(int64_t)col * k + c] = (double)sn;
    R[col * ld + (int64_t)col * k + c] = (double)rr;
    R[(col + 1) * ld + (int64_t)col * k + c] = 0.0;
    const S y0 = (S)py0, y1 = (S)py1;
    const S a0 = cs * y0, a1 = sn * y1;
    const S b0 = -sn * y0, b1 = cs * y1;
    const S ny1 = b0 + b1;
    y[(int64_t)col * k + c] = (double)(a0 + a1);
    y[(int64_t)(col + 1) * k + c] = (double)ny1;
    rn[c] = (double)fabs(ny1);
    if (!gbuf) hist[(int64_t)step * k + c] = rn[c];
  }
  __syncthreads();
  if (gbuf) {  // sharded: this rank's share of the global vector; gm_global_check decides
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
  const bool conv = all_le(rn, scal + G_CRIT * k, k, &flag);
  if (threadIdx.x == 0) {
    if (inv) ctrl->invariant = 1;
    if (inv || conv) ctrl->stop_at = step + 1;
  }
}

// Sharded global step decision on the allreduced vector: the history row,
// np.all(h[k+1] <= 1e-14) over ALL columns of all ranks (arnoldi.py:187) and
// the stop rule over all columns (gmres.py:193).
__global__ void gm_global_check(const double *gbuf, const double *gcrit, int total_k, double *hist, Ctrl *ctrl,
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

// yy = R[:m,:m]^-1 y[:m] per column (gmres.py:24-38; LAPACK ?trtrs semantics:
// zero rhs -> 0, non-finite input -> error, zero diagonal -> singular).
// One 64-lane block per column c (m <= 64): the column's R and y are read in
// parallel, lane i owns x[i], and the back substitution walks j = m-1..0 with
// x[j] broadcast through LDS, so every x[i] sees the same operations in the
// same order as the serial column-oriented loop (reference BLAS xTRSV 'U','N',
// 'N'): bitwise the same solution without m^2 dependent global loads.
template <typename S>
__global__ __launch_bounds__(64) void gm_trsv_kernel(const double *R, const double *y, double *yy, int m, int k,
                                                     int maxiter, Ctrl *ctrl) {
  __shared__ S Rs[64 * 64];
  __shared__ S fin[64];
  __shared__ int did[64];
  const int c = blockIdx.x, i = threadIdx.x;
  const int64_t ld = (int64_t)maxiter * k;
  bool nz = false, bad = false, sing = false;
  S xi = S(0);
  if (i < m) {
    const double yv = y[(int64_t)i * k + c];
    nz = yv != 0.0;
    bad = !isfinite(yv);
    xi = (S)yv;
  }
  for (int idx = i; idx < m * m; idx += 64) {
    const int r = idx / m, q = idx - (idx / m) * m;
    const double v = R[r * ld + (int64_t)q * k + c];
    bad = bad || !isfinite(v);
    sing = sing || (r == q && v == 0.0);
    Rs[r * 64 + q] = (S)v;
  }
  // precedence of the reference: zero rhs -> 0, then non-finite, then singular
  if (!__any(nz)) {
    if (i < m) yy[(int64_t)i * k + c] = 0.0;
    return;
  }
  if (__any(bad)) {
    if (i == 0) ctrl->status = KRY_ENONFINITE;
    return;
  }
  if (__any(sing)) {
    if (i == 0) ctrl->status = KRY_ESINGULAR;
    return;
  }
  __syncthreads();
  for (int j = m - 1; j >= 0; --j) {
    if (i == j) {
      did[j] = xi != S(0);
      if (xi != S(0)) xi = xi / Rs[j * 64 + j];
      fin[j] = xi;
    }
    __syncthreads();
    if (did[j] && i < j) {
      const S p = fin[j] * Rs[i * 64 + j];
      xi = xi - p;
    }
  }
  if (i < m) yy[(int64_t)i * k + c] = (double)xi;
}

// Larger triangular systems: same algorithm, solution kept in global memory.
template <typename S>
__global__ void gm_trsv_big_kernel(const double *R, const double *y, double *yy, int m, int k, int maxiter,
                                   Ctrl *ctrl) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= k) return;
  const int64_t ld = (int64_t)maxiter * k;
  bool allzero = true;
  for (int i = 0; i < m; ++i) allzero = allzero && (y[(int64_t)i * k + c] == 0.0);
  if (allzero) {
    for (int i = 0; i < m; ++i) yy[(int64_t)i * k + c] = 0.0;
    return;
  }
  bool finite = true;
  for (int i = 0; i < m; ++i) {
    finite = finite && isfinite(y[(int64_t)i * k + c]);
    for (int j = 0; j < m; ++j) finite = finite && isfinite(R[i * ld + (int64_t)j * k + c]);
  }
  if (!finite) {
    ctrl->status = KRY_ENONFINITE;
    return;
  }
  for (int i = 0; i < m; ++i)
    if (R[i * ld + (int64_t)i * k + c] == 0.0) {
      ctrl->status = KRY_ESINGULAR;
      return;
    }
  for (int i = 0; i < m; ++i) yy[(int64_t)i * k + c] = (double)(S)y[(int64_t)i * k + c];
  for (int j = m - 1; j >= 0; --j) {
    S xj = (S)yy[(int64_t)j * k + c];
    if (xj != S(0)) {
      xj = xj / (S)R[j * ld + (int64_t)j * k + c];
      yy[(int64_t)j * k + c] = (double)xj;
      for (int i = j - 1; i >= 0; --i) {
        const S p = xj * (S)R[i * ld + (int64_t)j * k + c];
        yy[(int64_t)i * k + c] = (double)((S)yy[(int64_t)i * k + c] - p);
      }
    }
  }
}

// ------------------------------------------------ Householder Arnoldi
// ArnoldiHouseholder (arnoldi.py:33-104) with Householder(x) of
// householder.py:8-53, one right-hand side. Reflector j is stored as a full
// vector U_j (zeros below index j) with scalars beta (0 or 2), alpha, and the
// values it was built from. Applying it to x[j:] is x - (beta * u) * <u, x>,
// each a streaming pass whose <u, x> arrives as block partials from the pass
// before (fixed-order reduction in every block, as in the MGS passes).
enum { HH_BETA = 0, HH_ALPHA = 1, HH_V0 = 2, HH_NRM = 3, HH_XNORM = 4, HH_COUNT = 5 };

// Householder(x[j:]): gamma = x[j], sigma2 = <x[j+1:], x[j+1:]> from the partials
// (arithmetic in the vector dtype, as the reference's arrays)
template <typename S>
__global__ void hh_make_kernel(const S *x, int64_t j, const double *part, int P, double *hh, const Ctrl *ctrl,
                               int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  reduce_partials(part, P, 1, red);
  if (threadIdx.x != 0) return;
  const S g = x[j];
  const S sig2 = (S)red[0];
  const S ag = fabs(g);
  S xnorm = sqrt(ag * ag + sig2);
  S beta, alpha, v0 = S(1);
  if (sig2 == S(0)) {
    beta = S(0);
    xnorm = ag;
    alpha = g == S(0) ? S(1) : g / xnorm;
  } else {
    beta = S(2);
    if (g == S(0)) {
      v0 = -sqrt(sig2);
      alpha = S(1);
    } else {
      const S t = g / ag * xnorm;
      v0 = g + t;
      alpha = -g / ag;
    }
  }
  const S av0 = fabs(v0);
  const S nrm = sqrt(av0 * av0 + sig2);
  hh[HH_BETA] = (double)beta;
  hh[HH_ALPHA] = (double)alpha;
  hh[HH_V0] = (double)v0;
  hh[HH_NRM] = (double)nrm;
  hh[HH_XNORM] = (double)xnorm;
}

// U_j = (v0 at j, x[i] beyond) / nrm, zero below j; partials of <U_j, x>.
template <typename V>
__global__ __launch_bounds__(kBlock) void hh_vec_kernel(int64_t N, const V *__restrict__ x, V *__restrict__ u,
                                                        int64_t j, const double *hh, double *__restrict__ part,
                                                        const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  const V v0 = (V)hh[HH_V0], nrm = (V)hh[HH_NRM];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) {
    V ui = V(0);
    const V xi = x[i];
    if (i >= j) {
      ui = (i == j ? v0 : xi) / nrm;
      acc += (double)ui * (double)xi;
    }
    u[i] = ui;
  }
  red[threadIdx.x] = acc;
  block_tree_reduce(red, kBlock, 1);
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// x[j:] = x[j:] - (beta U_j) s, s = <U_j, x> (from part_in, or *s_direct
// when P_in == 0); optionally x[j] *= alpha_j (arnoldi.py:75-77). Emits the
// partials of the next inner product: <q, x_new> over i >= qoff (q = x_new
// itself when q_is_x), if qoff >= 0. With `out`, writes x_new * (*scale) to out.
template <typename V>
__global__ __launch_bounds__(kBlock) void hh_apply_kernel(int64_t N, V *__restrict__ x, const V *__restrict__ u,
                                                          int64_t j, const double *hh, const double *part_in,
                                                          int P_in, const V *s_direct, int apply_alpha,
                                                          const V *__restrict__ q, int q_is_x, int64_t qoff,
                                                          double *__restrict__ part_out, V *__restrict__ out,
                                                          const double *scale, const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  V sv;
  if (P_in > 0) {
    reduce_partials(part_in, P_in, 1, red);
    sv = (V)red[0];
    __syncthreads();
  } else {
    sv = *s_direct;
  }
  const V beta = (V)hh[HH_BETA], alpha = (V)hh[HH_ALPHA];
  const V sc = out ? (V)*scale : V(1);
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) {
    V xi = x[i];
    if (i >= j && beta != V(0)) {
      const V bu = beta * u[i];
      const V t = bu * sv;
      xi = xi - t;
    }
    if (apply_alpha && i == j) xi = xi * alpha;
    if (out) out[i] = xi * sc;
    else x[i] = xi;
    if (qoff >= 0 && i >= qoff) acc += (double)(q_is_x ? xi : q[i]) * (double)xi;
  }
  if (qoff >= 0) {
    red[threadIdx.x] = acc;
    block_tree_reduce(red, kBlock, 1);
    if (threadIdx.x == 0) part_out[blockIdx.x] = red[0];
  }
}

// The Hessenberg column of step k: h[:k+1] = w[:k+1] after the forward
// reflections; h[k+1] = |(w[k+1] - (beta u) s) alpha| for the new reflector
// (arnoldi.py:79-86), or 0 when k + 1 == N (the space is exhausted).
template <typename V>
__global__ void hh_col_kernel(const V *w, const V *u, int64_t k, int64_t N, const double *hh, const double *part,
                              int P, double *h, const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  if (k + 1 < N) reduce_partials(part, P, 1, red);
  for (int64_t i = threadIdx.x; i <= k; i += kBlock) h[i] = (double)w[i];
  if (threadIdx.x == 0) {
    V hk1 = V(0);
    if (k + 1 < N) {
      const V beta = (V)hh[HH_BETA], alpha = (V)hh[HH_ALPHA];
      V xi = w[k + 1];
      if (beta != V(0)) {
        const V bu = beta * u[k + 1];
        const V t = bu * (V)red[0];
        xi = xi - t;
      }
      hk1 = fabs(xi * alpha);
    }
    h[k + 1] = (double)hk1;
  }
}

template <typename V>
__global__ void hh_unit_kernel(V *x, int64_t i, const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  if (threadIdx.x == 0 && blockIdx.x == 0) x[i] = V(1);
}

template <typename V>
struct OpSuffixSq {  // partials of <x[off:], x[off:]> (householder.py:32)
  const V *x;
  int64_t off;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&acc)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V a[W];
    VIO<V>::load(x, e, N, a);
#pragma unroll
    for (int v = 0; v < W; ++v)
      if (e + v < N && e + v >= off) acc[v] += (double)a[v] * (double)a[v];
  }
};

// w = Ml (A (Mr v)) (Product(Ml, A, Mr), gmres.py:139), `epi` on the last product.
template <typename V, typename MV, typename I, class Epi>
void gm_apply_op(kry_gmres *s, const V *v, Epi epi, double *part, int *P, const Ctrl *ctrl, int step) {
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

// Ml (b - A z) -> mlr, M Ml (b - A z) -> mw (with M), and the partials of
// <Ml r, M Ml r> (gmres.py:111-118); returns the partial count.
template <typename V, typename MV, typename I>
int gm_residual_chain(kry_gmres *s, const V *z, V *mlr) {
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

template <typename V, typename MV, typename I>
void gm_start_impl(kry_gmres *s) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const int64_t N = s->n * (int64_t)k;
  const V *src = s->x0 ? static_cast<const V *>(s->x0) : static_cast<const V *>(s->xk);  // xk zero-filled
  V *wv = static_cast<V *>(s->wv);
  const int P = gm_residual_chain<V, MV, I>(s, src, wv);
  hipLaunchKernelGGL(gm_start_finalize<V>, dim3(1), dim3(kBlock), 0, st, s->part, P, k, s->scal, s->y);
  KRY_HIP(hipGetLastError());
  // P_0 = Ml r0 / norm, V_0 = M Ml r0 / norm (arnoldi.py:147-150)
  if (s->M)
    launch_elementwise<V>(N, k, OpScaleDiv<V>{wv, static_cast<V *>(s->P), s->scal + G_HSAFE * k, k}, nullptr, nullptr,
                          0, st);
  const V *v0src = s->M ? static_cast<const V *>(s->mw) : wv;
  launch_elementwise<V>(N, k, OpScaleDiv<V>{v0src, static_cast<V *>(s->V), s->scal + G_HSAFE * k, k}, nullptr,
                        nullptr, 0, st);
  if (s->householder) {  // houses = [Householder(Ml r0)] (arnoldi.py:51)
    const int Ps = launch_elementwise<V>(N, 1, OpSuffixSq<V>{wv, 1}, s->part, nullptr, 0, st);
    hipLaunchKernelGGL(hh_make_kernel<V>, dim3(1), dim3(kBlock), 0, st, (const V *)wv, (int64_t)0,
                       (const double *)s->part, Ps, s->hh, (const Ctrl *)nullptr, 0);
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (N + 4 * kBlock - 1) / (4 * kBlock)));
    hipLaunchKernelGGL(hh_vec_kernel<V>, dim3(G), dim3(kBlock), 0, st, N, (const V *)wv, static_cast<V *>(s->U),
                       (int64_t)0, (const double *)s->hh, s->part2, (const Ctrl *)nullptr, 0);
    KRY_HIP(hipGetLastError());
  }
}

// One Householder Arnoldi step per iteration (arnoldi.py:65-104).
template <typename V, typename MV, typename I>
void hh_run_impl(kry_gmres *s, int max_steps) {
  hipStream_t st = s->ctx->stream;
  const int64_t N = s->n;
  V *w = static_cast<V *>(s->wv);
  V *vnew = static_cast<V *>(s->vnew);
  auto U = [&](int64_t j) { return basis<V>(s->U, s->vstride, (int)j); };
  auto hh = [&](int64_t j) { return s->hh + j * HH_COUNT; };
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (N + 4 * kBlock - 1) / (4 * kBlock)));
  for (int step = 0; step < max_steps; ++step) {
    const int64_t k = s->steps + step;
    if (k >= s->maxiter) break;
    int P;
    {
      ProfScope ps(s->ctx, PROF_SPMV);  // Av = A V_k with <U_0, Av> partials
      gm_apply_op<V, MV, I>(s, basis<V>(s->V, s->vstride, (int)k), EpiStoreDot<V>{w, U(0), nullptr, 1}, s->part, &P,
                            s->ctrl, step);
    }
    hipLaunchKernelGGL(reduce_to_kernel<0>, dim3(1), dim3(kBlock), 0, st, s->part, P, 1, s->part1);
    const double *pin = s->part1;
    int Pin = 1;
    double *pbuf[2] = {s->part, s->part2};
    int flip = 0;
    // Av[j:] = H_j Av[j:]; Av[j] *= alpha_j for j = 0..k (arnoldi.py:74-77)
    for (int64_t j = 0; j <= k; ++j) {
      const bool last = j == k;
      double *pout = pbuf[flip];
      ProfScope ps(s->ctx, PROF_MGS);
      hipLaunchKernelGGL(hh_apply_kernel<V>, dim3(G), dim3(kBlock), 0, st, N, w, (const V *)U(j), j,
                         (const double *)hh(j), pin, Pin, (const V *)nullptr, 1, last ? (const V *)nullptr : (const V *)U(j + 1),
                         last ? 1 : 0, last ? k + 2 : j + 1, pout, (V *)nullptr, (const double *)nullptr, s->ctrl, step);
      pin = pout;
      Pin = G;
      flip ^= 1;
    }
    const bool more = k + 1 < N;
    double *pout = pbuf[flip];
    if (more) {  // the new reflector from Av[k+1:] (arnoldi.py:79-81)
      hipLaunchKernelGGL(hh_make_kernel<V>, dim3(1), dim3(kBlock), 0, st, (const V *)w, k + 1, pin, Pin, hh(k + 1),
                         s->ctrl, step);
      hipLaunchKernelGGL(hh_vec_kernel<V>, dim3(G), dim3(kBlock), 0, st, N, (const V *)w, U(k + 1), k + 1,
                         (const double *)hh(k + 1), pout, s->ctrl, step);
    }
    hipLaunchKernelGGL(hh_col_kernel<V>, dim3(1), dim3(kBlock), 0, st, (const V *)w,
                       more ? (const V *)U(k + 1) : (const V *)nullptr, k, N, (const double *)hh(more ? k + 1 : 0),
                       (const double *)pout, G, s->h, s->ctrl, step);
    hipLaunchKernelGGL(gm_qr_kernel<V>, dim3(1), dim3(kBlock), 0, st, (const double *)nullptr, 0, 1, s->scal, s->h,
                       s->R, s->y, s->Gc, s->Gs, (int)k, s->maxiter, s->hist, s->ctrl, step, 1, (double *)nullptr, 0,
                       0, s->Hs);
    KRY_HIP(hipGetLastError());
    if (!more) continue;  // invariant: no new basis vector
    // vnew = e_{k+1}; vnew[j:] = H_j vnew[j:] for j = k+1..0; V_{k+1} = vnew alpha_{k+1}
    // (arnoldi.py:91-95)
    KRY_HIP(hipMemsetAsync(vnew, 0, (size_t)N * sizeof(V), st));
    hipLaunchKernelGGL(hh_unit_kernel<V>, dim3(1), dim3(64), 0, st, vnew, k + 1, s->ctrl, step);
    double *po = pbuf[flip ^ 1];
    hipLaunchKernelGGL(hh_apply_kernel<V>, dim3(G), dim3(kBlock), 0, st, N, vnew, (const V *)U(k + 1), k + 1,
                       (const double *)hh(k + 1), (const double *)nullptr, 0, (const V *)(U(k + 1) + (k + 1)), 0,
                       (const V *)U(k), 0, k, po, (V *)nullptr, (const double *)nullptr, s->ctrl, step);
    pin = po;
    for (int64_t j = k; j >= 0; --j) {
      const bool last = j == 0;
      double *pn = (pin == pbuf[0]) ? pbuf[1] : pbuf[0];
      hipLaunchKernelGGL(hh_apply_kernel<V>, dim3(G), dim3(kBlock), 0, st, N, vnew, (const V *)U(j), j,
                         (const double *)hh(j), pin, G, (const V *)nullptr, 0, last ? (const V *)nullptr : (const V *)U(j - 1),
                         0, last ? (int64_t)-1 : j - 1, pn, last ? basis<V>(s->V, s->vstride, (int)k + 1) : (V *)nullptr,
                         last ? (const double *)(hh(k + 1) + HH_ALPHA) : (const double *)nullptr, s->ctrl, step);
      pin = pn;
    }
    KRY_HIP(hipGetLastError());
  }
}

// Launch the persistent MGS kernel for this Arnoldi step if w fits the
// registers of one resident 512-thread block per CU; false = not eligible
// (decided once per solver: s->mgsp_E = 0 no, else elements per thread).
// Up to 16 doubles per thread w and the two basis vectors stay in registers
// (gm_mgsp_kernel); up to 80 only w does and the basis is streamed
// (gm_mgsl_kernel, n = 10 M at one column).
// granules per streamed chunk: 4 (2 from NV = 32 on, where 4 would spill)
template <int NV>
constexpr int mgsl_u() {
  return NV >= 32 ? 2 : 4;
}
// The two-vector lookahead MGS (gm_mgsp2_kernel / gm_mgsl2_kernel) is
// opt-in: KRY_MGS_LOOKAHEAD=1 (register-resident kernel), KRY_MGSL_LOOKAHEAD=1
// (streamed kernel). Both measured slower than the one-exchange-per-pass
// forms on one box, alternating processes (profiles/r06_mgs_lookahead_ab.txt):
// cfg3 0.100 against 0.082 ms per step, the metric 0.405 against 0.356 ms
// (its two partners share the LDS room one partner had, so it re-reads more
// of the basis).
inline bool mgs_lookahead() {
  static const bool on = [] {
    const char *e = getenv("KRY_MGS_LOOKAHEAD");
    return e && atoi(e) == 1;
  }();
  return on;
}
// the register-resident MGS at k = 1 with the partner copied two passes
// ahead into LDS (gm_mgsp3_kernel): default; KRY_MGS_PF2=0 restores
// gm_mgsp_kernel (bitwise the same results). cfg3 GMRES(30): MGS 0.084 ->
// 0.079 ms per step, 2,867 -> 2,920 it/s, same box, alternating processes
// (profiles/r06_mgs_pf2_ab.txt)
inline bool mgs_pf2() {
  const char *e = getenv("KRY_MGS_PF2");  // read per launch: the tests switch it within one process
  return !(e && atoi(e) == 0);
}
inline bool mgsl_lookahead() {
  static const bool on = [] {
    const char *e = getenv("KRY_MGSL_LOOKAHEAD");
    return e && atoi(e) == 1;
  }();
  return on;
}
template <typename V>
bool mgsp_launch(kry_gmres *s, V *w, const double *pin, int Pin, int col, int step) {
  const int64_t N = s->n * (int64_t)s->k;
  constexpr int W = Vec16<V>::W;
  if (s->mgsp_E < 0) {
    s->mgsp_E = 0;
    s->mgsp_large = false;
    const char *e = getenv("KRY_MGS_PERSIST");
    if (!(e && atoi(e) == 0)) {
      int dev = 0, ncu = 0;
      KRY_HIP(hipGetDevice(&dev));
      KRY_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      auto fits = [&](auto kern, int E) {
        const int64_t G = (N + (int64_t)kMgsBlock * E - 1) / ((int64_t)kMgsBlock * E);
        int per_cu = 0;
        KRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kMgsBlock, 0));
        // one block per CU: VGPR-bound residency (<= 256 VGPRs at 2 waves
        // per SIMD), far from the SGPR band where the answer runs high
        return G <= ncu && G <= 256 && per_cu >= 1 && (int64_t)s->sweeps * (s->maxiter + 1) < 4095;
      };
      // (E = 32 doubles per thread would spill: float only)
      const bool pf2 = !mgs_lookahead() && s->k == 1 && mgs_pf2();
      if (pf2 ? fits(gm_mgsp3_kernel<V, 8>, 8)
              : (mgs_lookahead() ? fits(gm_mgsp2_kernel<V, 8>, 8) : fits(gm_mgsp_kernel<V, 8>, 8)))
        s->mgsp_E = 8;
      else if (pf2 ? fits(gm_mgsp3_kernel<V, 16>, 16)
                   : (mgs_lookahead() ? fits(gm_mgsp2_kernel<V, 16>, 16) : fits(gm_mgsp_kernel<V, 16>, 16)))
        s->mgsp_E = 16;
      else if constexpr (sizeof(V) == 4) {
        if (mgs_lookahead() ? fits(gm_mgsp2_kernel<V, 32>, 32) : fits(gm_mgsp_kernel<V, 32>, 32)) s->mgsp_E = 32;
      }
      if (s->mgsp_E == 0 && !(e && atoi(e) == 1)) {  // KRY_MGS_PERSIST=1: the register-resident kernel only
        s->mgsp_large = true;
        const bool la = mgsl_lookahead();
        if (la ? fits(gm_mgsl2_kernel<V, 12, true>, 12 * W) : fits(gm_mgsl_kernel<V, 12, mgsl_u<12>(), true>, 12 * W))
          s->mgsp_E = 12 * W;
        else if (la ? fits(gm_mgsl2_kernel<V, 16, true>, 16 * W)
                    : fits(gm_mgsl_kernel<V, 16, mgsl_u<16>(), true>, 16 * W))
          s->mgsp_E = 16 * W;
        else if (la ? fits(gm_mgsl2_kernel<V, 24, true>, 24 * W)
                    : fits(gm_mgsl_kernel<V, 24, mgsl_u<24>(), true>, 24 * W))
          s->mgsp_E = 24 * W;
        else if (la ? fits(gm_mgsl2_kernel<V, 32, true>, 32 * W)
                    : fits(gm_mgsl_kernel<V, 32, mgsl_u<32>(), true>, 32 * W))
          s->mgsp_E = 32 * W;
        else if (la ? fits(gm_mgsl2_kernel<V, 40, true>, 40 * W)
                    : fits(gm_mgsl_kernel<V, 40, mgsl_u<40>(), true>, 40 * W))
          s->mgsp_E = 40 * W;
        else s->mgsp_large = false;
      }
    }
  }
  if (s->mgsp_E == 0) return false;
  hipStream_t st = s->ctx->stream;
  const int E = s->mgsp_E;
  const int G = (int)((N + (int64_t)kMgsBlock * E - 1) / ((int64_t)kMgsBlock * E));
  if (step == 0) KRY_HIP(hipMemsetAsync(s->bar, 0, bar_bytes(s->chunk_cap), st));
  unsigned *bar = s->bar + (size_t)step * kBarWords;
  unsigned long long *gran = reinterpret_cast<unsigned long long *>(s->bar + (size_t)s->chunk_cap * kBarWords);
  double *pbuf = s->part2;  // [pass parity 0 | parity 1 | last pass], G * k each
  ProfScope ps(s->ctx, PROF_MGS);
  const char *fe = getenv("KRY_MGS_FAULT");  // fault injection (tests): chunk step at which a block drops out
  const char *ff = getenv("KRY_MGS_FAULT_FINAL");  // ... at the streamed kernel's final exchange instead
  const int fault_step = fe ? (atoi(fe) | ((ff && atoi(ff) == 1) ? (1 << 16) : 0)) : -1;
  // KRY_MGS_TRACE: per-block phase sums of the register-resident kernels,
  // accumulated over the solver's launches and printed at its destroy
  static const bool trace = getenv("KRY_MGS_TRACE") != nullptr;
  if (trace && !s->mgs_tbuf) {
    KRY_HIP(hipMalloc(&s->mgs_tbuf, 256 * 4 * 8));
    KRY_HIP(hipMemsetAsync(s->mgs_tbuf, 0, 256 * 4 * 8, st));
  }
  if (trace) {
    s->mgs_tpasses += (int64_t)(mgs_lookahead() ? (1 + s->sweeps * (col + 1) / 2) : s->sweeps * (col + 1));
    s->mgs_tgrid = G;
  }
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(kMgsBlock), 0, st, N, s->k, w, (const V *)s->V, s->vstride, col, s->sweeps,
                       pin, Pin, pbuf, s->h, bar, gran, s->ctrl, step, fault_step, s->mgs_tbuf);
  };
  // the streamed kernel also normalises: V_{col+1} = w / guard(h[col+1])
  V *vnext = basis<V>(s->V, s->vstride, col + 1);
  auto gol = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(kMgsBlock), 0, st, N, s->k, w, (const V *)s->V, s->vstride, col, s->sweeps,
                       pin, Pin, pbuf, s->h, bar, gran, s->ctrl, step, fault_step, vnext);
  };
  s->mgsp_norm = s->mgsp_large;
  static const bool mgsl_nt = [] {
    const char *e = getenv("KRY_MGSL_NT");  // tuning override: subtrahend loads nontemporal (1) or not (0)
    return e ? atoi(e) != 0 : true;
  }();
  static const int mgsl_u_env = [] {
    const char *e = getenv("KRY_MGSL_U");  // tuning override: granules per streamed chunk at NV >= 32 (2 or 4)
    return e ? atoi(e) : 0;
  }();
  bool u4 = false;
  if constexpr (sizeof(V) == 8) u4 = s->mgsp_large && mgsl_nt && mgsl_u_env == 4 && E / W >= 32;
  const bool la = s->mgsp_large ? mgsl_lookahead() : mgs_lookahead();
  if (s->mgsp_large && la) {
    switch (E / W) {
      case 12: gol(gm_mgsl2_kernel<V, 12, true>); break;
      case 16: gol(gm_mgsl2_kernel<V, 16, true>); break;
      case 24: gol(gm_mgsl2_kernel<V, 24, true>); break;
      case 32: gol(gm_mgsl2_kernel<V, 32, true>); break;
      default: gol(gm_mgsl2_kernel<V, 40, true>); break;
    }
  } else if (u4) {
    if constexpr (sizeof(V) == 8) {
      if (E / W == 32) gol(gm_mgsl_kernel<V, 32, 4, true>);
      else gol(gm_mgsl_kernel<V, 40, 4, true>);
    }
  } else if (s->mgsp_large && mgsl_nt) {
    switch (E / W) {
      case 12: gol(gm_mgsl_kernel<V, 12, mgsl_u<12>(), true>); break;
      case 16: gol(gm_mgsl_kernel<V, 16, mgsl_u<16>(), true>); break;
      case 24: gol(gm_mgsl_kernel<V, 24, mgsl_u<24>(), true>); break;
      case 32: gol(gm_mgsl_kernel<V, 32, mgsl_u<32>(), true>); break;
      default: gol(gm_mgsl_kernel<V, 40, mgsl_u<40>(), true>); break;
    }
  } else if (s->mgsp_large) {
    switch (E / W) {
      case 12: gol(gm_mgsl_kernel<V, 12, mgsl_u<12>(), false>); break;
      case 16: gol(gm_mgsl_kernel<V, 16, mgsl_u<16>(), false>); break;
      case 24: gol(gm_mgsl_kernel<V, 24, mgsl_u<24>(), false>); break;
      case 32: gol(gm_mgsl_kernel<V, 32, mgsl_u<32>(), false>); break;
      default: gol(gm_mgsl_kernel<V, 40, mgsl_u<40>(), false>); break;
    }
  } else if (!la && s->k == 1 && mgs_pf2()) {
    if (E == 8) go(gm_mgsp3_kernel<V, 8>);
    else if (E == 16) go(gm_mgsp3_kernel<V, 16>);
    else if constexpr (sizeof(V) == 4) go(gm_mgsp3_kernel<V, 32>);
  } else if (la) {
    if (E == 8) go(gm_mgsp2_kernel<V, 8>);
    else if (E == 16) go(gm_mgsp2_kernel<V, 16>);
    else if constexpr (sizeof(V) == 4) go(gm_mgsp2_kernel<V, 32>);
  } else if (E == 8) {
    go(gm_mgsp_kernel<V, 8>);
  } else if (E == 16) {
    go(gm_mgsp_kernel<V, 16>);
  } else if constexpr (sizeof(V) == 4) {
    go(gm_mgsp_kernel<V, 32>);
  }
  KRY_HIP(hipGetLastError());
  s->mgsp_grid = s->mgsp_norm ? 1 : G;  // normalising: the exchanged sum, one row
  // the <w, w> partials: slot 2 of the one-value kernels, slot 6 of the lookahead's three-value parities
  s->mgsp_out = pbuf + (size_t)(la ? 6 : 2) * G * s->k;
  return true;
}

// h[k+1], Givens QR, resnorm and the step decision; sharded: one RCCL
// allreduce of the residual-norm vector (+ non-invariant count) per step and
// the global decision.
template <typename V>
void gm_qr_step(kry_gmres *s, const double *pin, int P, int col, int step) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  hipLaunchKernelGGL(gm_qr_kernel<V>, dim3(1), dim3(kBlock), 0, st, pin, P, k, s->scal, s->h, s->R, s->y, s->Gc,
                     s->Gs, col, s->maxiter, s->hist, s->ctrl, step, 0, s->comm ? s->gbuf : nullptr, s->col_offset,
                     s->total_k, s->Hs);
  KRY_HIP(hipGetLastError());
  if (!s->comm) return;
  inject_peer_fault(s->gbuf, s->total_k + 2, step, st);
  comm_allreduce(s->comm, s->gbuf, s->total_k + 2, st);
  hipLaunchKernelGGL(gm_global_check, dim3(1), dim3(kBlock), 0, st, (const double *)s->gbuf,
                     (const double *)s->gcrit, s->total_k, s->hist, s->ctrl, step);
  KRY_HIP(hipGetLastError());
}

template <typename V, typename MV, typename I>
void gm_run_impl(kry_gmres *s, int max_steps) {
  if (s->householder) return hh_run_impl<V, MV, I>(s, max_steps);
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const int64_t N = s->n * (int64_t)k;
  V *wb[2] = {static_cast<V *>(s->wv), static_cast<V *>(s->wv2)};
  const bool fuse_norm = !s->M && !s->Ml && !s->Mr;
  for (int step = 0; step < max_steps; ++step) {
    const int col = s->steps + step;
    if (col >= s->maxiter) break;
    V *Vk = basis<V>(s->V, s->vstride, col);
    const V *V0 = basis<V>(s->V, s->vstride, 0);
    int P;
    V *w;
    {
      ProfScope ps(s->ctx, PROF_SPMV);
      if (s->vpending) {  // V_k = w_prev / hsafe, formed in the gather and stored by the epilogue
        const V *wprev = wb[s->wcur];
        w = wb[s->wcur ^ 1];
        launch_spmv<V, MV, I>(s->A, k, SrcScaled<V>{wprev, s->scal + G_HSAFE * k, k},
                              EpiStoreDotV<V>{w, V0, Vk, s->w, k}, s->part, &P, s->ctrl, step, st);
        s->wcur ^= 1;
        s->vpending = false;
      } else {
        w = wb[s->wcur];
        gm_apply_op<V, MV, I>(s, Vk, EpiStoreDot<V>{w, V0, s->w, k}, s->part, &P, s->ctrl, step);
      }
    }
    if (fuse_norm && !s->w && mgsp_launch<V>(s, w, s->part, P, col, step)) {
      // the QR kernel reads the persistent kernel's <w, w> partials
      gm_qr_step<V>(s, s->mgsp_out, s->mgsp_grid, col, step);
      if (s->mgsp_norm) continue;  // V_{col+1} is in the basis already
      if (col + 1 < s->maxiter && !spmv_column_blocked<I>(s->A, k)) {
        s->vpending = true;  // V_{col+1} is formed by the next step's SpMV
        continue;
      }
      // last column, or a gather-bound SpMV (cfg3: the division on every
      // gathered value cost 269 -> 285 us with the quad-loading kernel, the
      // separate pass ~6 us): V_{col+1} = w / hsafe as its own pass
      launch_elementwise<V>(N, k, OpScaleDiv<V>{w, basis<V>(s->V, s->vstride, col + 1), s->scal + G_HSAFE * k, k},
                            nullptr, s->ctrl, step, st);
      continue;
    }
    // the SpMV's partials of <V_0, w> -> one value per column, so every MGS
    // block reduces a single partial row for its first coefficient
    hipLaunchKernelGGL(reduce_to_kernel<0>, dim3(1), dim3(kBlock), 0, st, s->part, P, k, s->part1);
    const double *pin = s->part1;
    int Pin = 1;
    double *pbuf[2] = {s->part, s->part2};
    int flip = 0;
    const int64_t ngrp = (N + Vec16<V>::W - 1) / Vec16<V>::W;
    static const int mgs_cap = [] {
      const char *e = getenv("KRY_MGS_GRID");  // tuning override
      return e ? std::max(1, std::min(atoi(e), kMaxGrid)) : 1024;
    }();
    static const int mgs_per = [] {
      const char *e = getenv("KRY_MGS_PER");  // tuning override: chunks per block
      return e ? std::max(64, atoi(e)) : 1024;
    }();
    const int Gm = (int)std::max<int64_t>(1, std::min<int64_t>(mgs_cap, (ngrp + mgs_per - 1) / mgs_per));
    for (int sw = 0; sw < s->sweeps; ++sw) {
      for (int j = 0; j <= col; ++j) {
        const V *Pj = basis<V>(s->M ? s->P : s->V, s->vstride, j);  // Av -= alpha P_j (arnoldi.py:162)
        const V *q = j < col ? basis<V>(s->V, s->vstride, j + 1) : (sw + 1 < s->sweeps ? V0 : nullptr);
        double *pout = pbuf[flip];
        ProfScope ps(s->ctx, PROF_MGS);
        hipLaunchKernelGGL(gm_mgs_kernel<V>, dim3(Gm), dim3(kBlock), 0, st, N, k, w, Pj, q, pin, Pin, pout, s->h, j,
                           sw == 0 ? 1 : 0, s->w, s->ctrl, step);
        pin = pout;
        Pin = Gm;
        flip ^= 1;
      }
    }
    P = Pin;
    if (s->M) {  // MAv = M Av, h[k+1] = sqrt(<Av, MAv>) (arnoldi.py:184-185)
      launch_spmv_any<V>(s->M, k, SrcPlain<V>{w, k}, EpiStoreDot<V>{static_cast<V *>(s->mw), w, s->w, k}, s->part,
                         &P, s->ctrl, step, st);
      pin = s->part;
    }
    gm_qr_step<V>(s, pin, P, col, step);
    // P_{col+1} = w / guard(h[col+1]), V_{col+1} = M w / guard(h[col+1]) unless
    // invariant; these run for this step even when the QR kernel just raised
    // stop_at to step + 1 (arnoldi.py:191-196).
    if (fuse_norm && col + 1 < s->maxiter) {
      s->vpending = true;  // V_{col+1} is formed by the next step's SpMV
      continue;
    }
    if (s->M)
      launch_elementwise<V>(N, k, OpScaleDiv<V>{w, basis<V>(s->P, s->vstride, col + 1), s->scal + G_HSAFE * k, k},
                            nullptr, s->ctrl, step, st);
    const V *vsrc = s->M ? static_cast<const V *>(s->mw) : w;
    launch_elementwise<V>(N, k,
                          OpScaleDiv<V>{vsrc, basis<V>(s->V, s->vstride, col + 1), s->scal + G_HSAFE * k, k},
                          nullptr, s->ctrl, step, st);
  }
}

template <typename V, typename MV, typename I>
void gm_solution_impl(kry_gmres *s) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k, m = s->steps;
  const int64_t N = s->n * (int64_t)k;
  if (m > 0) {
    const int g = (k + kBlock - 1) / kBlock;
    if (m <= 64)
      hipLaunchKernelGGL(gm_trsv_kernel<V>, dim3(k), dim3(64), 0, st, s->R, s->y, s->yy, m, k, s->maxiter, s->ctrl);
    else
      hipLaunchKernelGGL(gm_trsv_big_kernel<V>, dim3(g), dim3(kBlock), 0, st, s->R, s->y, s->yy, m, k, s->maxiter,
                         s->ctrl);
    KRY_HIP(hipGetLastError());
  }
  if (!s->Mr) {
    launch_elementwise<V>(N, k,
                          OpBasisCombo<V>{static_cast<const V *>(s->V), s->vstride, m, s->yy,
                                          static_cast<const V *>(s->x0), static_cast<V *>(s->xk), k},
                          nullptr, nullptr, 0, st);
    return;
  }
  // xk = x0 + Mr (sum_i yy_i V_i) (gmres.py:97-99)
  V *t1 = static_cast<V *>(s->t1);
  launch_elementwise<V>(N, k, OpBasisCombo<V>{static_cast<const V *>(s->V), s->vstride, m, s->yy, nullptr, t1, k},
                        nullptr, nullptr, 0, st);
  launch_spmv_any<V>(s->Mr, k, SrcPlain<V>{t1, k},
                     EpiAddStore<V>{static_cast<V *>(s->xk), static_cast<const V *>(s->x0), k}, nullptr, nullptr,
                     nullptr, 0, st);
}

template <typename V, typename MV, typename I>
void gm_residual_impl(kry_gmres *s, double *norm2) {
  hipStream_t st = s->ctx->stream;
  const int k = s->k;
  const int P = gm_residual_chain<V, MV, I>(s, static_cast<const V *>(s->xk), static_cast<V *>(s->rt));
  double *out = s->scal + G_TMP * k;
  hipLaunchKernelGGL(reduce_to_kernel<0>, dim3(1), dim3(kBlock), 0, st, s->part, P, k, out);
  KRY_HIP(hipGetLastError());
  KRY_HIP(hipMemcpyAsync(norm2, out, k * 8, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
}

void gm_free(kry_gmres *s) {
  void *bufs[] = {s->b,  s->x0,   s->V,     s->wv,   s->xk,   s->rt, s->w,  s->part, s->part1, s->part2,
                  s->scal, s->h, s->R, s->y, s->Gc, s->Gs, s->yy, s->hist, s->ctrl, s->P, s->mw, s->t1, s->t2,
                  s->U, s->vnew, s->hh, s->wv2, s->bar, s->gbuf, s->gcrit, s->Hs};
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

int kry_gmres_create(kry_ctx *ctx, kry_csr *A, int32_t k, int dtype, int32_t maxiter, int32_t sweeps,
                     kry_gmres **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && A && out, KRY_EINVAL, "null argument");
  KRY_REQUIRE(is_pow2(k) && k <= kMaxCols, KRY_EUNSUPPORTED, "k must be a power of two <= 256");
  KRY_REQUIRE(dtype == A->dtype || (dtype == KRY_F64 && A->dtype == KRY_F32), KRY_EINVAL,
              "vectors must have the operator dtype (or float64 over a float32 operator)");
  KRY_REQUIRE(maxiter >= 0 && sweeps >= 0, KRY_EINVAL, "bad maxiter / sweeps");
  KRY_REQUIRE(sweeps >= 1 || k == 1, KRY_EUNSUPPORTED, "Householder Arnoldi works on one right-hand side");
  KRY_HIP(hipSetDevice(ctx->device));
  auto *s = new kry_gmres();
  try {
    s->ctx = ctx;
    s->A = A;
    s->n = A->n;
    s->k = k;
    s->dtype = dtype;
    s->maxiter = maxiter;
    s->sweeps = sweeps;
    s->vstride = ((size_t)A->n * k + 15) / 16 * 16;
    const size_t vb = s->vstride * dsize(dtype);
    s->b = dev_alloc(vb);
    s->wv = dev_alloc(vb);
    s->wv2 = dev_alloc(vb);
    s->xk = dev_alloc(vb);
    s->rt = dev_alloc(vb);
    s->V = dev_alloc(vb * ((size_t)maxiter + 1));
    if (sweeps == 0) {
      s->householder = true;
      s->U = dev_alloc(vb * ((size_t)maxiter + 2));
      s->vnew = dev_alloc(vb);
      s->hh = static_cast<double *>(dev_alloc(((size_t)maxiter + 2) * HH_COUNT * 8));
    }
    KRY_HIP(hipMemsetAsync(s->xk, 0, vb, ctx->stream));
    KRY_HIP(hipMemsetAsync(s->wv, 0, vb, ctx->stream));
    KRY_HIP(hipMemsetAsync(s->wv2, 0, vb, ctx->stream));
    s->part = static_cast<double *>(dev_alloc(part_rows(k) * k * 8));
    s->part1 = static_cast<double *>(dev_alloc((size_t)k * 8));
    s->part2 = static_cast<double *>(dev_alloc(part_rows(k) * k * 8));
    s->scal = static_cast<double *>(dev_alloc(G_COUNT * (size_t)k * 8));
    s->h = static_cast<double *>(dev_alloc(((size_t)maxiter + 2) * k * 8));
    s->R = static_cast<double *>(dev_alloc(((size_t)maxiter + 1) * (maxiter > 0 ? maxiter : 1) * k * 8));
    s->Hs = static_cast<double *>(dev_alloc(((size_t)maxiter + 1) * (maxiter > 0 ? maxiter : 1) * k * 8));
    KRY_HIP(hipMemsetAsync(s->Hs, 0, ((size_t)maxiter + 1) * (maxiter > 0 ? maxiter : 1) * k * 8, ctx->stream));
    s->y = static_cast<double *>(dev_alloc(((size_t)maxiter + 1) * k * 8));
    s->Gc = static_cast<double *>(dev_alloc(((size_t)maxiter + 1) * k * 8));
    s->Gs = static_cast<double *>(dev_alloc(((size_t)maxiter + 1) * k * 8));
    s->yy = static_cast<double *>(dev_alloc(((size_t)maxiter + 1) * k * 8));
    s->chunk_cap = 64;
    s->hist = static_cast<double *>(dev_alloc((size_t)s->chunk_cap * k * 8));
    s->bar = static_cast<unsigned *>(dev_alloc(bar_bytes(s->chunk_cap)));
    s->ctrl = static_cast<Ctrl *>(dev_alloc(sizeof(Ctrl)));
    KRY_HIP(hipStreamSynchronize(ctx->stream));
  } catch (...) {
    gm_free(s);
    delete s;
    throw;
  }
  *out = s;
  KRY_API_END
}

int kry_gmres_set_preconditioners(kry_gmres *s, kry_csr *M, kry_csr *Ml, kry_csr *Mr) {
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
  KRY_REQUIRE(!(M && s->householder), KRY_EINVAL, "Householder Arnoldi does not take M (gmres.py:160)");
  KRY_HIP(hipSetDevice(s->ctx->device));
  const size_t vb = s->vstride * dsize(s->dtype);
  auto need = [&](void *&buf, size_t bytes) {
    if (!buf) {
      buf = dev_alloc(bytes);
      KRY_HIP(hipMemsetAsync(buf, 0, bytes, s->ctx->stream));
    }
  };
  s->M = M;
  s->Ml = Ml;
  s->Mr = Mr;
  if (M) {
    need(s->P, vb * ((size_t)s->maxiter + 1));
    need(s->mw, vb);
  }
  if (Mr) need(s->t1, vb);
  if (Ml) need(s->t2, vb);
  KRY_HIP(hipStreamSynchronize(s->ctx->stream));
  s->started = false;
  KRY_API_END
}

int kry_gmres_destroy(kry_gmres *s) {
  KRY_API_BEGIN
  if (!s) return KRY_OK;
  (void)hipSetDevice(s->ctx->device);
  (void)hipStreamSynchronize(s->ctx->stream);
  if (s->mgs_tbuf) {  // KRY_MGS_TRACE: mean over blocks of the per-pass phase times
    unsigned long long h[256 * 4];
    if (hipMemcpy(h, s->mgs_tbuf, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess && s->mgs_tgrid > 0) {
      double sum[3] = {0, 0, 0};
      for (int b = 0; b < s->mgs_tgrid; ++b)
        for (int q = 0; q < 3; ++q) sum[q] += (double)h[b * 4 + q];
      const double np = (double)(s->mgs_tpasses > 0 ? s->mgs_tpasses : 1);
      fprintf(stderr, "mgs trace G=%d passes=%lld (us/pass, mean over blocks): compute %.2f reduce+publish %.2f xwait %.2f\n",
              s->mgs_tgrid, (long long)s->mgs_tpasses, sum[0] * 0.01 / s->mgs_tgrid / np,
              sum[1] * 0.01 / s->mgs_tgrid / np, sum[2] * 0.01 / s->mgs_tgrid / np);
    }
    (void)hipFree(s->mgs_tbuf);
    s->mgs_tbuf = nullptr;
  }
  gm_free(s);
  delete s;
  KRY_API_END
}

int kry_gmres_start(kry_gmres *s, kry_vec *b, kry_vec *x0, kry_vec *w, double *r0norm) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && r0norm, KRY_EINVAL, "null argument");
  check_vec(b, s->n, s->k, s->dtype, "b");
  if (x0) check_vec(x0, s->n, s->k, s->dtype, "x0");
  check_weights(w, s->n);
  KRY_REQUIRE(!(w && s->householder), KRY_EINVAL, "Householder Arnoldi needs the Euclidean inner product");
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  const size_t vb = b->bytes();
  const int k = s->k;
  // b, x0 and the weights arrive in the caller's numbering (load_in: into a
  // renumbered operator's, a plain copy otherwise)
  load_in(s->A, b->d, s->b, k, dsize(s->dtype), st);
  dev_free(s->x0);
  s->x0 = nullptr;
  if (x0) {
    s->x0 = dev_alloc(s->vstride * dsize(s->dtype));
    load_in(s->A, x0->d, s->x0, k, dsize(s->dtype), st);
  }
  dev_free(s->w);
  s->w = nullptr;
  if (w) {
    s->w = static_cast<double *>(dev_alloc(((size_t)s->n + 1) * 8));
    load_in(s->A, w->d, s->w, 1, 8, st);
  }
  const size_t m1 = (size_t)s->maxiter + 1;
  KRY_HIP(hipMemsetAsync(s->xk, 0, vb, st));
  KRY_HIP(hipMemsetAsync(s->R, 0, m1 * (s->maxiter > 0 ? s->maxiter : 1) * k * 8, st));
  KRY_HIP(hipMemsetAsync(s->y, 0, m1 * k * 8, st));
  KRY_HIP(hipMemsetAsync(s->h, 0, (m1 + 1) * k * 8, st));
  KRY_HIP(hipMemsetAsync(s->yy, 0, m1 * k * 8, st));
  reset_ctrl(s->ctrl, st);
  s->steps = 0;
  s->invariant = false;
  s->have_solution = false;
  s->wcur = 0;
  s->vpending = false;
  dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { gm_start_impl<decltype(v0), decltype(m0), decltype(i0)>(s); });
  KRY_HIP(hipMemcpyAsync(r0norm, s->scal + G_TMP * k, k * 8, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  s->started = true;
  KRY_API_END
}

int kry_gmres_set_criterion(kry_gmres *s, const double *criterion) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && criterion, KRY_EINVAL, "null argument");
  if (s->comm)  // all total_k columns, in rank order
    KRY_HIP(hipMemcpyAsync(s->gcrit, criterion, s->total_k * 8, hipMemcpyHostToDevice, s->ctx->stream));
  else
    KRY_HIP(hipMemcpyAsync(s->scal + G_CRIT * s->k, criterion, s->k * 8, hipMemcpyHostToDevice, s->ctx->stream));
  KRY_HIP(hipStreamSynchronize(s->ctx->stream));
  KRY_API_END
}

int kry_gmres_run(kry_gmres *s, int32_t max_steps, int32_t *steps_done, double *resnorms, int32_t *invariant) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && steps_done && resnorms && invariant && max_steps >= 0, KRY_EINVAL, "bad argument");
  KRY_REQUIRE(s->started, KRY_EINVAL, "kry_gmres_start has not been called");
  if (s->invariant)
    throw Error{KRY_EINVARIANT, "Krylov subspace was found to be invariant in the previous iteration."};
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  if (max_steps > s->maxiter - s->steps) max_steps = s->maxiter - s->steps;
  if (max_steps > s->chunk_cap) {
    dev_free(s->hist);
    s->hist = nullptr;
    s->hist = static_cast<double *>(dev_alloc((size_t)max_steps * (s->comm ? s->total_k : s->k) * 8));
    dev_free(s->bar);
    s->bar = nullptr;
    s->bar = static_cast<unsigned *>(dev_alloc(bar_bytes(max_steps)));
    s->chunk_cap = max_steps;
  }
  const int hk = s->comm ? s->total_k : s->k;
  auto run_chunk = [&](int steps, double *rows, Ctrl *c) {
    reset_ctrl(s->ctrl, st);
    dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { gm_run_impl<decltype(v0), decltype(m0), decltype(i0)>(s, steps); });
    return read_chunk(s->ctx, st, s->ctrl, s->hist, steps, hk, rows, c);
  };
  Ctrl c;
  int done = run_chunk(max_steps, resnorms, &c);
  if (s->comm && c.status == KRY_ECOMM) {
    // the healthy rank's state has moved past the recorded history (the
    // step's update kernels ran before the global check stopped it): the
    // solver refuses further runs until kry_*_start
    s->started = false;
    throw Error{KRY_ECOMM, "GMRES: another rank's in-launch exchange failed at step " + std::to_string(done) +
                               " of this run call; every rank stopped before it"};
  }
  if (c.status == KRY_EDEVICE && s->mgsp_E > 0 && s->comm) {
    // one allreduce per step on every rank: no rank may rerun part of a chunk
    // alone (see kry_cg_run); the step's allreduce carried the fault to every
    // rank (post_fault), which all stopped before it
    s->mgsp_E = 0;
    ++s->mgsp_fallbacks;
    s->started = false;  // refuse further runs until kry_*_start (the state is past the history)
    throw Error{KRY_EDEVICE, "GMRES: the persistent MGS exchange timed out at step " + std::to_string(done) +
                                 " (a block was not resident); every rank of the communicator stopped before it"};
  }
  if (c.status == KRY_EDEVICE && s->mgsp_E > 0) {
    // the persistent MGS kernel timed out at step `done` (a block was not
    // resident) and halted the chunk there: keep the steps before it and run
    // the rest of the chunk launch per pass, from that step's SpMV (V_k is in
    // the basis; the step's h entries are rewritten by its first sweep)
    s->steps += done;
    s->mgsp_E = 0;
    s->vpending = false;
    ++s->mgsp_fallbacks;
    const int more = run_chunk(max_steps - done, resnorms + (size_t)done * hk, &c);
    s->steps -= done;
    done += more;
  }
  if (c.status == KRY_EDEVICE) throw Error{KRY_EDEVICE, "GMRES: device error during the chunk"};
  s->steps += done;
  s->invariant = c.invariant != 0;
  s->have_solution = false;
  *steps_done = done;
  *invariant = s->invariant ? 1 : 0;
  KRY_API_END
}

int kry_gmres_solution(kry_gmres *s) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && s->started, KRY_EINVAL, "solver not started");
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  reset_ctrl(s->ctrl, st);
  dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { gm_solution_impl<decltype(v0), decltype(m0), decltype(i0)>(s); });
  Ctrl c;
  KRY_HIP(hipMemcpyAsync(&c, s->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  if (c.status == KRY_ESINGULAR) throw Error{KRY_ESINGULAR, "singular matrix: resolution failed at a zero diagonal"};
  if (c.status == KRY_ENONFINITE) throw Error{KRY_ENONFINITE, "array must not contain infs or NaNs"};
  s->have_solution = true;
  KRY_API_END
}

// xk (after kry_gmres_solution) into a device vector: the restart chain's
// next x0 without a round trip through the host (gmres_restarted).
int kry_gmres_xk_device(kry_gmres *s, kry_vec *out) {
  KRY_API_BEGIN
  KRY_REQUIRE(s, KRY_EINVAL, "null solver");
  KRY_REQUIRE(s->have_solution, KRY_EINVAL, "call kry_gmres_solution first");
  check_vec(out, s->n, s->k, s->dtype, "out");
  KRY_REQUIRE(out->ctx && out->ctx->device == s->ctx->device, KRY_EINVAL, "out: a vector on another device");
  KRY_HIP(hipSetDevice(s->ctx->device));
  permute_rows(s->A, s->xk, out->d, s->k, dsize(s->dtype), false, s->ctx->stream);  // the caller's numbering
  KRY_API_END
}

int kry_gmres_residual(kry_gmres *s, double *norm2) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && norm2, KRY_EINVAL, "null argument");
  KRY_REQUIRE(s->have_solution, KRY_EINVAL, "call kry_gmres_solution first");
  KRY_HIP(hipSetDevice(s->ctx->device));
  dispatch_vmi(s->dtype, s->A->dtype, s->A->itype, [&](auto v0, auto m0, auto i0) { gm_residual_impl<decltype(v0), decltype(m0), decltype(i0)>(s, norm2); });
  KRY_API_END
}

// which = 0: xk (after kry_gmres_solution); 1: the basis V_0..V_m, 2: P_0..P_m
// (= V without M), m = steps (steps - 1 after an invariant step), each n x k;
// 3: the Hessenberg matrix H, (maxiter + 1) x maxiter x k, column j filled
// for j < steps (arnoldi.py:158-196, the relation A V_m = V_{m+1} H).
int kry_gmres_path(kry_gmres *s, int32_t *info) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && info, KRY_EINVAL, "null argument");
  info[0] = s->mgsp_E > 0 ? 1 : 0;
  info[1] = s->mgsp_fallbacks;
  KRY_API_END
}

int kry_gmres_get(kry_gmres *s, int which, void *host) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && host && which >= 0 && which <= 3, KRY_EINVAL, "bad argument");
  KRY_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  const size_t vb = (size_t)s->n * s->k * dsize(s->dtype);
  if (which == 0) {
    KRY_REQUIRE(s->have_solution, KRY_EINVAL, "call kry_gmres_solution first");
    store_out(s->A, s->xk, host, s->k, dsize(s->dtype), st);
  } else if (which == 3) {
    const int mi = s->maxiter > 0 ? s->maxiter : 1;
    KRY_HIP(hipMemcpyAsync(host, s->Hs, ((size_t)s->maxiter + 1) * mi * s->k * 8, hipMemcpyDeviceToHost, st));
  } else {
    KRY_REQUIRE(s->started, KRY_EINVAL, "solver not started");
    KRY_REQUIRE(!s->householder || which == 1, KRY_EINVAL, "Householder Arnoldi has no P basis");
    const int nv = s->steps + (s->invariant ? 0 : 1);
    if (s->vpending && !s->invariant) {  // V_steps is still w / guard(h[steps]): form it now
      const int64_t N = s->n * (int64_t)s->k;
      const int k = s->k;
      auto go = [&](auto v0) {
        using V = decltype(v0);
        V *wb[2] = {static_cast<V *>(s->wv), static_cast<V *>(s->wv2)};
        launch_elementwise<V>(N, k,
                              OpScaleDiv<V>{wb[s->wcur], basis<V>(s->V, s->vstride, s->steps), s->scal + G_HSAFE * k, k},
                              nullptr, nullptr, 0, st);
      };
      if (s->dtype == KRY_F64) go(0.0);
      else go(0.0f);
    }
    const void *base = (which == 2 && s->M) ? s->P : s->V;
    const size_t stride = s->vstride * dsize(s->dtype);
    for (int i = 0; i < nv; ++i)
      store_out(s->A, static_cast<const char *>(base) + i * stride, static_cast<char *>(host) + (size_t)i * vb, s->k,
                dsize(s->dtype), st);
  }
  KRY_HIP(hipStreamSynchronize(st));
  KRY_API_END
}

// RHS sharding: this solver's k columns are global columns
// [col_offset, col_offset + k) of total_k; every step allreduces the residual
// norms (and a non-invariant count) over the communicator and applies the
// reference's stop and invariance rules to all columns. The history rows
// returned by kry_gmres_run then hold total_k values.
int kry_gmres_attach_comm(kry_gmres *s, kry_comm *c, int32_t col_offset, int32_t total_k) {
  KRY_API_BEGIN
  KRY_REQUIRE(s && c, KRY_EINVAL, "null argument");
  KRY_REQUIRE(col_offset >= 0 && total_k >= col_offset + s->k && total_k <= 4096, KRY_EINVAL,
              "bad column range");
  KRY_REQUIRE(!s->householder, KRY_EUNSUPPORTED, "Householder Arnoldi is single right-hand side");
  KRY_HIP(hipSetDevice(s->ctx->device));
  dev_free(s->gbuf);
  dev_free(s->gcrit);
  s->gbuf = nullptr;
  s->gcrit = nullptr;
  s->gbuf = static_cast<double *>(dev_alloc(((size_t)total_k + 2) * 8));  // + non-invariant and fault counts
  s->gcrit = static_cast<double *>(dev_alloc((size_t)total_k * 8));
  dev_free(s->hist);
  s->hist = nullptr;
  s->hist = static_cast<double *>(dev_alloc((size_t)s->chunk_cap * total_k * 8));
  s->comm = c;
  s->col_offset = col_offset;
  s->total_k = total_k;
  KRY_API_END
}

// multi_solve_triangular (gmres.py:24-38) as a standalone device call: per
// column c of k, yy = R[:, :, c]^-1 y[:, c] for upper-triangular R (m x m x k,
// C order) and y (m x k), with the reference's semantics (zero rhs -> 0,
// non-finite input -> KRY_ENONFINITE, zero diagonal -> KRY_ESINGULAR). The
// arithmetic runs in `dtype` (float64 / float32, as scipy's dtrtrs / strtrs);
// host arrays are float64.
int kry_trsv_upper(kry_ctx *ctx, int32_t m, int32_t k, int dtype, const double *R, const double *y, double *out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && R && y && out && m >= 1 && k >= 1, KRY_EINVAL, "bad argument");
  KRY_REQUIRE(dtype == KRY_F64 || dtype == KRY_F32, KRY_EINVAL, "dtype must be float64 or float32");
  KRY_HIP(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const size_t rb = (size_t)m * m * k * 8, yb = (size_t)m * k * 8;
  double *dR = static_cast<double *>(dev_alloc(rb));
  double *dy = nullptr, *dout = nullptr;
  Ctrl *c = nullptr;
  try {
    dy = static_cast<double *>(dev_alloc(yb));
    dout = static_cast<double *>(dev_alloc(yb));
    c = static_cast<Ctrl *>(dev_alloc(sizeof(Ctrl)));
    reset_ctrl(c, st);
    KRY_HIP(hipMemcpyAsync(dR, R, rb, hipMemcpyHostToDevice, st));
    KRY_HIP(hipMemcpyAsync(dy, y, yb, hipMemcpyHostToDevice, st));
    auto go = [&](auto s0) {
      using S = decltype(s0);
      if (m <= 64)
        hipLaunchKernelGGL(gm_trsv_kernel<S>, dim3(k), dim3(64), 0, st, (const double *)dR, (const double *)dy, dout,
                           m, k, m, c);
      else
        hipLaunchKernelGGL(gm_trsv_big_kernel<S>, dim3((k + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                           (const double *)dR, (const double *)dy, dout, m, k, m, c);
    };
    if (dtype == KRY_F64) go(0.0);
    else go(0.0f);
    KRY_HIP(hipGetLastError());
    Ctrl hc;
    KRY_HIP(hipMemcpyAsync(&hc, c, sizeof(Ctrl), hipMemcpyDeviceToHost, st));
    KRY_HIP(hipMemcpyAsync(out, dout, yb, hipMemcpyDeviceToHost, st));
    KRY_HIP(hipStreamSynchronize(st));
    if (hc.status == KRY_ESINGULAR) throw Error{KRY_ESINGULAR, "singular matrix: resolution failed at a zero diagonal"};
    if (hc.status == KRY_ENONFINITE) throw Error{KRY_ENONFINITE, "array must not contain infs or NaNs"};
  } catch (...) {
    dev_free(dR);
    dev_free(dy);
    dev_free(dout);
    dev_free(c);
    throw;
  }
  dev_free(dR);
  dev_free(dy);
  dev_free(dout);
  dev_free(c);
  KRY_API_END
}

// Householder(x) (householder.py:6-53) on its own, for a single vector x
// (n x 1): v_out = v / sqrt(|v0|^2 + sigma2), out3 = [beta, alpha, xnorm],
// with the same kernels (and arithmetic in x's dtype) as Householder Arnoldi.
int kry_householder(kry_ctx *ctx, kry_vec *x, kry_vec *v_out, double *out3) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && x && v_out && out3, KRY_EINVAL, "null argument");
  KRY_REQUIRE(x->k == 1 && v_out->k == 1 && x->n == v_out->n && x->dtype == v_out->dtype && x->n >= 1, KRY_EINVAL,
              "x and v_out must be matching single vectors");
  KRY_HIP(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const int64_t N = x->n;
  double *part = ctx_scratch(ctx, ((size_t)kMaxGrid + HH_COUNT) * 8);
  double *hh = part + kMaxGrid;
  auto go = [&](auto v0) {
    using V = decltype(v0);
    const int P = launch_elementwise<V>(N, 1, OpSuffixSq<V>{static_cast<const V *>(x->d), 1}, part, nullptr, 0, st);
    hipLaunchKernelGGL(hh_make_kernel<V>, dim3(1), dim3(kBlock), 0, st, static_cast<const V *>(x->d), (int64_t)0,
                       (const double *)part, P, hh, (const Ctrl *)nullptr, 0);
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (N + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(hh_vec_kernel<V>, dim3(G), dim3(kBlock), 0, st, N, static_cast<const V *>(x->d),
                       static_cast<V *>(v_out->d), (int64_t)0, (const double *)hh, part, (const Ctrl *)nullptr, 0);
  };
  if (x->dtype == KRY_F64) go(0.0);
  else go(0.0f);
  KRY_HIP(hipGetLastError());
  double h[HH_COUNT];
  KRY_HIP(hipMemcpyAsync(h, hh, sizeof(h), hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  out3[0] = h[HH_BETA];
  out3[1] = h[HH_ALPHA];
  out3[2] = h[HH_XNORM];
  KRY_API_END
}

}  // extern "C"
