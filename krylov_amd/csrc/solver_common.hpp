// Pieces shared by the CG / GMRES / MINRES device loops.
#pragma once

#include <atomic>
#include <chrono>
#include <climits>
#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "device.hpp"

// One rank's RCCL communicator. Several host threads may hold one (the
// devices=[...] driver aborts every device's communicator from the thread
// that failed while the others are inside their solver loops), so: `aborted`
// is atomic, and every collective ENQUEUE and the abort itself run under
// `mu` (not the stream syncs that follow an enqueue: an abort must be able to
// release a rank blocked in one). After an abort `comm` is null.
struct kry_comm {
  kry_ctx *ctx = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  double *dbuf = nullptr;  // scratch for host allreduces
  int dbuf_len = 0;
  std::atomic<bool> aborted{false};  // kry_comm_abort ran: destroy skips ncclCommDestroy
  std::timed_mutex mu;
};

namespace kry {

// In-place float64 sum over the communicator's ranks of `count` device
// doubles, enqueued on `st` under the communicator's lock; KRY_ECOMM once the
// communicator was aborted (by any thread).
inline void comm_allreduce(kry_comm *c, double *buf, size_t count, hipStream_t st) {
  std::lock_guard<std::timed_mutex> g(c->mu);
  if (c->aborted.load(std::memory_order_acquire) || !c->comm)
    throw Error{KRY_ECOMM, "the communicator was aborted"};
  ncclResult_t nr = ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, c->comm, st);
  if (nr != ncclSuccess) throw Error{KRY_ECOMM, std::string("ncclAllReduce: ") + ncclGetErrorString(nr)};
}

// ------------------------------------------------ in-launch all-gathers
// Persistent kernels (GMRES MGS, small-n CG) exchange one double per block
// per phase as self-validating granules {tag, 32 data bits} (two per block:
// the low and high words), stored write-through with agent-scope atomics; no
// counters, no flag. Wave 0 of every block sweeps all G <= 256 blocks'
// granules until every tag matches, then sums the values in a fixed order
// (lane l: blocks l, l + 64, ..., then a fixed xor butterfly; lane 0's value),
// so every block derives the same bits. Tags must be unique among the words
// a region holds between zeroings. Every spin is bounded: on timeout the
// kernel raises ctrl->status = KRY_EDEVICE and the abort word, and every
// block leaves; the host then reruns the work on the launch-per-pass path
// (kry_cg_run / kry_gmres_run), which needs no co-residency.
//
// Memory-ordering argument (gfx950 only, see the guard below). The protocol
// uses relaxed operations only, and rests on how gfx950 lowers them
// (MI355X_MICROARCH.md, "Valid forms" and its hand-off table, row 1):
//  - data handed to other blocks (CG's r and p, the MGS partials) is stored
//    with agent-scope relaxed atomic stores = `global_store ... sc1`, which
//    write through the XCD's L2 to the fabric;
//  - every storing wave runs `s_waitcnt vmcnt(0)` and then the workgroup
//    barrier before ONE lane publishes the block's granule (also `sc1`), so
//    every data store has been acknowledged before the tag can be seen;
//  - the reader polls the granules with agent-scope relaxed loads
//    (`global_load ... sc1`, which bypass the CU's L1), then a workgroup
//    barrier, and reads the data only with `sc1` loads (ld_wt / ld_agent):
//    never from L1, so no `buffer_inv` is needed.
// The granule itself is a single naturally aligned 8-byte store, observed
// untorn. None of this is promised by the HIP memory model: a different
// target (gfx942's non-coherent per-XCD L2 with other cache policies) or a
// compiler that reorders relaxed atomics across the inline-asm wait could
// read stale data. Hence the compile-time guard, and the cross-XCD parity
// tests (CG at G = 245 blocks, tests/test_gpu_solvers.py) as the guard for
// compiler upgrades.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "the in-launch exchanges of the persistent kernels are validated for gfx950 (MI355X) only"
#endif
// Bounds on the exchanges' spins, in ticks of the 100 MHz constant clock
// (wall_clock64): a block that has not seen every partial after 20 ms gives
// up (the callers then fall back to kernels that need no co-residency), so a
// non-resident block costs at most ~20 ms once per solver, not an unbounded
// or poll-count-dependent stall (round 2 counted 2^20 polls: about a second).
constexpr unsigned kSpinLimit = 2000000u;
// Shorter bound for the fault-injection runs (KRY_CGP_FAULT / KRY_MGS_FAULT /
// KRY_CGU_FAULT / KRY_MRU_FAULT), so that a test of the timeout path
// finishes in milliseconds: 1 ms.
constexpr unsigned kSpinLimitFault = 100000u;
// Time since `t0` has exceeded `limit` ticks (checked every 256 polls).
__device__ __forceinline__ bool spin_expired(unsigned long long t0, unsigned limit) {
  return wall_clock64() - t0 > (unsigned long long)limit;
}

__device__ __forceinline__ void publish_partial(unsigned long long *g, unsigned tag, double v) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
  const unsigned long long t = (unsigned long long)tag << 32;
  __hip_atomic_store(g, t | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, t | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Commit / abort agreement of one exchange (kernels that update their inputs
// in place after it: cg_upd_kernel, mr_upd_kernel). Word bar[10] records the
// decision for the exchange tagged `tag` as tag * 4 + {1 abort, 2 commit}; the
// first block to decide (a block that saw every partial: commit; a block
// whose spin ran out: abort) wins by compare-and-swap, and every other block
// follows it. So no block stores after another gave up, and a block whose
// spin runs out after some block committed keeps waiting: every partial has
// been published by then, so its sweep completes. bar[10] starts at 0 (the
// host clears the words at the start of a chunk) and tags grow within it.
constexpr unsigned kDecAbort = 1u, kDecCommit = 2u;
__device__ inline unsigned decide_exchange(unsigned *bar, unsigned tag, unsigned want) {
  unsigned old = __hip_atomic_load(bar + 10, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while ((old >> 2) != tag) {
    if (__hip_atomic_compare_exchange_strong(bar + 10, &old, tag * 4u + want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return want;
  }
  return old & 3u;
}

// One poll of a granule pair {lo, hi} = 16 B at agent scope (sc1: past the
// CU's L1), through a wave-uniform buffer descriptor over the whole region
// and a per-lane byte offset (no per-lane descriptors, no waterfall loop).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t granule_rsrc(const unsigned long long *gr, int G) {
  const uint64_t a = reinterpret_cast<uint64_t>(gr);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(G * 16), 0x00020000);
}
typedef unsigned int granule_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ granule_u4 poll_granule(__amdgpu_buffer_rsrc_t r, int b) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, b * 16, 0, 16 /* sc1 */);
}

// Wave 0 only; returns the same value in every lane (false = timed out /
// aborted). spin_limit: ticks of wall_clock64 (kSpinLimit). AGREE: the commit / abort decision is shared by all blocks
// (decide_exchange); otherwise a timed-out block only raises bar[9] and a
// caller that has stored nothing yet re-checks it.
// Round 5: each block's granule pair is read with ONE 16-B load, and a lane
// re-polls only the pairs whose tags have not matched yet (the round-4 form
// re-read every pair with two 8-B loads per poll). tools/xchg_probe.hip at
// 256 blocks: 3.74 -> 3.21 us per exchange round with nothing in flight,
// 3.4-4.6 -> 2.7-2.8 us with the MGS kernel's prefetch loads in flight
// (profiles/r05_xchg_probe.jsonl); two-level (per-XCD) trees and 8 or 32
// reader blocks were slower (a second hop). The values and their summation
// order are unchanged (lane l: blocks l, l + 64, ..., then the butterfly).
// Wave sum of a double by DPP moves (VALU lane exchanges, no LDS round
// trip): xor 1 and 2 within quads, the half-row and row mirrors, then the
// row broadcasts 15 and 31; a fixed tree whose total lands in lane 63 and is
// returned, read back as a wave-uniform value, in every lane. Masked rows
// add 0 (the update keeps `old` = 0 there).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ double dpp_mov_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v = v + dpp_mov_f64<0xB1>(v);        // quad_perm [1, 0, 3, 2]
  v = v + dpp_mov_f64<0x4E>(v);        // quad_perm [2, 3, 0, 1]
  v = v + dpp_mov_f64<0x141>(v);       // row_half_mirror
  v = v + dpp_mov_f64<0x140>(v);       // row_mirror
  v = v + dpp_mov_f64<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
  v = v + dpp_mov_f64<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// DPP: the final wave sum by wave_sum_dpp (the persistent CG loop; its sums
// have their own fixed order) instead of the xor butterfly of shuffles.
template <bool AGREE = false, bool DPP = false>
__device__ inline bool sweep_partials(unsigned long long *gr, int G, unsigned tag, unsigned *bar, Ctrl *ctrl, double *out,
                                      unsigned spin_limit = kSpinLimit) {
  const int lane = threadIdx.x;
  const __amdgpu_buffer_rsrc_t rs = granule_rsrc(gr, G);
  granule_u4 g[4];
  bool got[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    got[i] = lane + 64 * i >= G;
    g[i] = granule_u4{0u, 0u, 0u, 0u};
  }
  unsigned spins = 0;
  bool expired = false;
  const unsigned long long t0 = wall_clock64();
  bool committed = false;  // AGREE: another block has committed this exchange
  const bool legacy = __builtin_amdgcn_readfirstlane(ctrl->xchg) != 0;
  for (;;) {
    asm volatile("" ::: "memory");  // a fresh poll every round: the loads are not hoisted
    if (legacy) {  // the round-4 poll, for A/B runs: every pair, two 8-B loads
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = lane + 64 * i;
        got[i] = b >= G;
        if (b < G) {
          const unsigned long long lo = __hip_atomic_load(gr + 2 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const unsigned long long hi = __hip_atomic_load(gr + 2 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          g[i] = granule_u4{(unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32)};
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (!got[i]) g[i] = poll_granule(rs, lane + 64 * i);
    }
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!got[i]) got[i] = g[i].y == tag && g[i].w == tag;
      ok = ok && got[i];
    }
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(1);
    ++spins;
    if (committed) continue;
    if ((spins & 255u) == 0) {
      expired = spin_expired(t0, spin_limit);
      if (AGREE) {
        const unsigned d = __hip_atomic_load(bar + 10, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == tag * 4u + kDecAbort) return false;
        if (d == tag * 4u + kDecCommit) committed = true;
      } else if (__hip_atomic_load(bar + 9, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        return false;
      }
    }
    if (expired && !committed) {
      unsigned d = kDecAbort;
      if (AGREE) {
        if (lane == 0) d = decide_exchange(bar, tag, kDecAbort);
        d = __shfl(d, 0);
        if (d == kDecCommit) {
          committed = true;
          continue;
        }
      }
      if (lane == 0) {
        __hip_atomic_store(bar + 9, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&ctrl->status, (int32_t)KRY_EDEVICE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return false;
    }
  }
  if (AGREE) {
    unsigned d = 0;
    if (lane == 0) d = decide_exchange(bar, tag, kDecCommit);
    if (__shfl(d, 0) != kDecCommit) return false;
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = lane + 64 * i;
    if (b < G) s += __longlong_as_double((long long)(((unsigned long long)g[i].z << 32) | (unsigned long long)g[i].x));
  }
  if constexpr (DPP) {
    s = wave_sum_dpp(s);
  } else {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  }
  if (lane == 0) *out = s;
  return true;
}

// sweep_partials<false, true> for NVAL doubles per block (the lookahead MGS
// kernels exchange <V_a, w>, <V_b, w> and <V_b, V_a> at once): value v of
// block b is the granule pair gr[2 (v G + b)], gr[2 (v G + b) + 1], read with
// one 16-B load; the exchange completes when every value's tags match. Each
// value is summed in sweep_partials' order (lane l: blocks l, l + 64, ...,
// then wave_sum_dpp), so NVAL = 1 gives its bits; out[v] in lane 0.
template <int NVAL>
__device__ inline bool sweep_partials_n(unsigned long long *gr, int G, unsigned tag, unsigned *bar, Ctrl *ctrl,
                                        double *out, unsigned spin_limit = kSpinLimit) {
  const int lane = threadIdx.x & 63;  // any one wave
  const __amdgpu_buffer_rsrc_t rs = granule_rsrc(gr, NVAL * G);
  granule_u4 g[NVAL][4];
  bool got[NVAL][4];
#pragma unroll
  for (int v = 0; v < NVAL; ++v)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      got[v][i] = lane + 64 * i >= G;
      g[v][i] = granule_u4{0u, 0u, 0u, 0u};
    }
  unsigned spins = 0;
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    asm volatile("" ::: "memory");  // a fresh poll every round: the loads are not hoisted
#pragma unroll
    for (int v = 0; v < NVAL; ++v)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (!got[v][i]) g[v][i] = poll_granule(rs, v * G + lane + 64 * i);
    bool ok = true;
#pragma unroll
    for (int v = 0; v < NVAL; ++v)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!got[v][i]) got[v][i] = g[v][i].y == tag && g[v][i].w == tag;
        ok = ok && got[v][i];
      }
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(1);
    ++spins;
    if ((spins & 255u) == 0) {
      if (__hip_atomic_load(bar + 9, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
      if (spin_expired(t0, spin_limit)) {
        if (lane == 0) {
          __hip_atomic_store(bar + 9, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ctrl->status, (int32_t)KRY_EDEVICE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return false;
      }
    }
  }
#pragma unroll
  for (int v = 0; v < NVAL; ++v) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = lane + 64 * i;
      if (b < G)
        s += __longlong_as_double((long long)(((unsigned long long)g[v][i].z << 32) | (unsigned long long)g[v][i].x));
    }
    s = wave_sum_dpp(s);
    if (lane == 0) out[v] = s;
  }
  return true;
}

// Publish NVAL doubles of this block (sweep_partials_n's layout); one lane.
template <int NVAL>
__device__ __forceinline__ void publish_partials_n(unsigned long long *gr, int G, unsigned tag, const double *v) {
#pragma unroll
  for (int n = 0; n < NVAL; ++n) publish_partial(gr + 2 * ((size_t)n * G + blockIdx.x), tag, v[n]);
}

// Deterministic block sum for one column: each wave sums by a fixed xor
// butterfly (lane 0's value is used), one barrier, then wave 0 adds the wave
// sums by a fixed butterfly over lanes 0..nwaves-1 (blockDim <= 1024). The result is
// returned in thread 0 (no trailing barrier); block_sum1 also stores it to
// *out and makes it visible to the block.
__device__ __forceinline__ double block_sum1_t0(double v, double *wsum) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) wsum[wv] = v;
  __syncthreads();
  double s = 0.0;
  if (wv == 0) {
    s = lane < (int)(blockDim.x >> 6) ? wsum[lane] : 0.0;
    for (int off = 1; off < (int)(blockDim.x >> 6); off <<= 1) s += __shfl_xor(s, off);
  }
  return s;
}
// block_sum1_t0 with DPP wave sums (the persistent CG loop): every wave's
// sum by wave_sum_dpp, then wave 0 sums the wave sums the same way; the
// result is valid in every lane of wave 0
__device__ __forceinline__ double block_sum1_t0_dpp(double v, double *wsum) {
  v = wave_sum_dpp(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) wsum[wv] = v;
  __syncthreads();
  double s = 0.0;
  if (wv == 0) s = wave_sum_dpp(lane < (int)(blockDim.x >> 6) ? wsum[lane] : 0.0);
  return s;
}
// block_sum1_t0_dpp for NVAL values at once (one barrier); wsum holds
// NVAL * 16 doubles. Each value's bits are block_sum1_t0_dpp's; valid in
// every lane of wave 0.
template <int NVAL>
__device__ __forceinline__ void block_sumn_t0_dpp(double (&v)[NVAL], double *wsum) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int n = 0; n < NVAL; ++n) {
    v[n] = wave_sum_dpp(v[n]);
    if (lane == 0) wsum[n * 16 + wv] = v[n];
  }
  __syncthreads();
  if (wv == 0) {
#pragma unroll
    for (int n = 0; n < NVAL; ++n) v[n] = wave_sum_dpp(lane < (int)(blockDim.x >> 6) ? wsum[n * 16 + lane] : 0.0);
  }
}
__device__ __forceinline__ void block_sum1(double v, double *wsum, double *out) {
  const double s = block_sum1_t0(v, wsum);
  if (threadIdx.x == 0) *out = s;
  __syncthreads();
}

// ------------------------------------------ block-segment buffer access
// The persistent kernels that hold a vector segment per thread in registers
// (streamed MGS, one-launch CG update) address it with buffer loads/stores
// over the block's segment of each vector: a descriptor from wave-uniform
// values, the per-lane byte offset tid * 16 and the granule's offset
// u * BLOCK * 16 as a scalar, so no per-granule address registers; the
// descriptor's record count ends at N, so out-of-range granules read as 0
// and their stores are dropped.
typedef unsigned int bufseg_u4 __attribute__((ext_vector_type(4)));
template <typename V, int BLOCK>
struct BufSeg {
  __amdgpu_buffer_rsrc_t r;
  V *base;      // the segment's first element (wave-uniform)
  int64_t cnt;  // its elements inside [0, N)
  __device__ __forceinline__ BufSeg(const V *vec, int64_t e0, int64_t N, int64_t seg) {
    const int64_t rem = N - e0;
    cnt = rem < seg ? (rem > 0 ? rem : 0) : seg;
    // wave-uniform by construction; readfirstlane makes it provable, so the
    // buffer ops take the descriptor from SGPRs without a waterfall loop
    const uint64_t a = reinterpret_cast<uint64_t>(vec + e0);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane((int)(cnt * (int64_t)sizeof(V)));
    base = reinterpret_cast<V *>(((uint64_t)hi << 32) | lo);
    r = __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
  }
  template <int W, int AUX = 0>
  __device__ __forceinline__ void load(int u, V (&o)[W]) const {
    const bufseg_u4 t = __builtin_amdgcn_raw_buffer_load_b128(r, (int)threadIdx.x * 16, u * BLOCK * 16, AUX);
    if constexpr (W == 2) {
      const double2 d = __builtin_bit_cast(double2, t);
      o[0] = d.x;
      o[1] = d.y;
    } else {
      const float4 f = __builtin_bit_cast(float4, t);
      o[0] = f.x;
      o[1] = f.y;
      o[2] = f.z;
      o[3] = f.w;
    }
  }
  // Stores are plain global stores, guarded at the segment's end: with
  // __builtin_amdgcn_raw_buffer_store_b128 hipcc (ROCm 7.2, gfx950) may let a
  // VALU overwrite the store's data VGPRs in the very next instruction, before
  // the 16-byte store has read them (seen as corrupted lanes 12-15 of every 16
  // in one element: archive:cgu_debug.py); for global stores it keeps the wait
  // states.
  // The element offset is built from an opaque zero (a volatile s_mov):
  // otherwise LLVM hoists the NV per-granule offsets of an epilogue that
  // sits inside the pass loop out of it and spills them (the streamed MGS
  // kernel at NV = 40 spilled 148 VGPRs: ~150 MB of scratch traffic per
  // launch); recomputed here they cost two VALU ops per store.
  template <int W, int AUX = 0>
  __device__ __forceinline__ void store(int u, const V (&o)[W]) const {
    typedef V vec_t __attribute__((ext_vector_type(W)));
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    const int tz = (int)threadIdx.x ^ z;  // everything per-thread below depends on z
    const int64_t e = ((int64_t)u * BLOCK + tz) * W;
    if (e + W <= cnt) {
      vec_t t;
#pragma unroll
      for (int v = 0; v < W; ++v) t[v] = o[v];
      if (AUX & 2) __builtin_nontemporal_store(t, reinterpret_cast<vec_t *>(base + e));
      else *reinterpret_cast<vec_t *>(base + e) = t;
    } else {
#pragma unroll
      for (int v = 0; v < W; ++v)
        if (e + v < cnt) base[e + v] = o[v];
    }
  }
};

// guarded divisor, np.where(d != 0, d, 1.0)
template <typename S>
__device__ __forceinline__ S safe(S d) {
  return d != S(0) ? d : S(1);
}

// ------------------------------------------ sharded runs: fault agreement
// Under a communicator every step posts one allreduce of the global vector on
// every rank, and its LAST slot is a fault count. A rank whose in-launch
// exchange timed out at `step` (that kernel left ctrl->stop_at = step and
// ctrl->status = KRY_EDEVICE, and stored nothing) posts zeros and a fault in
// place of its norms; every rank's global check of that step sees the count,
// stops the chunk at `step` (the step does not count) and raises KRY_ECOMM.
// So every rank leaves the chunk after the same collectives and reports the
// failure: the healthy ranks never block in the next chunk's allreduce, and
// none of them reads the faulting rank's stale slots as a step's norms.
// nslots = the allreduced length (fault slot = nslots - 1). One block.
__device__ inline void post_fault(double *gbuf, int nslots) {
  for (int t = threadIdx.x; t < nslots; t += blockDim.x) gbuf[t] = t == nslots - 1 ? 1.0 : 0.0;
}
// This rank's step `step` was abandoned by a timed-out exchange (read by the
// kernel that would have posted the step's norms).
__device__ inline bool local_fault_at(const Ctrl *ctrl, int step) {
  return ctrl->stop_at == step && ctrl->status == (int32_t)KRY_EDEVICE;
}
// In a global check: a rank posted a fault for this step. Stops the chunk
// before the step and records KRY_ECOMM (block-uniform answer).
__device__ inline bool peer_fault(const double *gbuf, int nslots, Ctrl *ctrl, int step) {
  if (gbuf[nslots - 1] == 0.0) return false;
  if (threadIdx.x == 0) {
    ctrl->stop_at = step;
    if (ctrl->status == 0) ctrl->status = (int32_t)KRY_ECOMM;
  }
  return true;
}

// Test hook for the receiving side on one GPU (a 1-rank communicator has no
// peer that could fail): KRY_COMM_PEER_FAULT = s makes step s's allreduce
// carry a fault count, as if another rank had posted one (s counts the steps
// of a run call, like the other fault switches).
inline void inject_peer_fault(double *gbuf, int nslots, int step, hipStream_t st) {
  const char *e = getenv("KRY_COMM_PEER_FAULT");
  if (e && atoi(e) == step) KRY_HIP(hipMemsetAsync(gbuf + nslots - 1, 0x3f, 8, st));
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

template <int D = 0>
__global__ void ctrl_reset_kernel(Ctrl *c, int xchg) {
  c->stop_at = INT_MAX;
  c->invariant = 0;
  c->status = 0;
  c->xchg = xchg;
}

inline int xchg_mode() {
  static const int m = [] {
    const char *e = getenv("KRY_XCHG_LEGACY");
    return e && atoi(e) != 0 ? 1 : 0;
  }();
  return m;
}

// Host helper: reset the control word to "run everything" (a one-thread
// kernel on the stream: no pageable host copy in the chunk's critical path).
inline void reset_ctrl(Ctrl *d_ctrl, hipStream_t st) {
  hipLaunchKernelGGL(ctrl_reset_kernel<0>, dim3(1), dim3(1), 0, st, d_ctrl, xchg_mode());
  KRY_HIP(hipGetLastError());
}

// End of a chunk: the control word and the chunk's history rows (all
// max_steps of them, a few KB) through pinned staging with ONE host sync;
// returns the steps done (min(stop_at, max_steps)) and copies their rows.
inline int read_chunk(kry_ctx *ctx, hipStream_t st, const Ctrl *d_ctrl, const double *d_hist, int max_steps, int hk,
                      double *resnorms, Ctrl *c) {
  const size_t hb = (size_t)(max_steps > 0 ? max_steps : 0) * hk * 8;
  const size_t need = 64 + hb;
  if (ctx->pinned_bytes < need) {
    if (ctx->pinned) KRY_HIP(hipHostFree(ctx->pinned));
    ctx->pinned = nullptr;
    ctx->pinned_bytes = 0;
    const size_t sz = need < 65536 ? 65536 : need;
    KRY_HIP(hipHostMalloc(&ctx->pinned, sz, hipHostMallocDefault));
    ctx->pinned_bytes = sz;
  }
  char *h = static_cast<char *>(ctx->pinned);
  KRY_HIP(hipMemcpyAsync(h, d_ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, st));
  if (hb) KRY_HIP(hipMemcpyAsync(h + 64, d_hist, hb, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  memcpy(c, h, sizeof(Ctrl));
  const int done = c->stop_at < max_steps ? c->stop_at : max_steps;
  if (done > 0) memcpy(resnorms, h + 64, (size_t)done * hk * 8);
  return done;
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
