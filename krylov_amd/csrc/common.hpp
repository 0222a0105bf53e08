// Shared device/host plumbing for libkrylov_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/krylov_hip.h"
#include "host_common.hpp"

namespace kry {

constexpr int kBlock = 256;          // threads per workgroup (4 waves of 64)
constexpr int kWave = 64;            // CDNA wavefront
constexpr int kMaxGrid = 8192;       // grid cap (and partial-buffer rows)
// The block right-hand-side SpMV (k <= 8) runs one slice per wave, up to
// kMaxGridBlk blocks, so partial buffers for k <= 8 hold that many rows.
constexpr int kMaxGridBlk = 32768;
inline size_t part_rows(int k) { return k <= 8 ? (size_t)kMaxGridBlk : (size_t)kMaxGrid; }
constexpr int kMaxCols = 256;        // RHS columns per device (power of two)
constexpr int kCbCap = 1024;         // products staged in LDS per chunk
constexpr int kNumXcd = 8;

#define KRY_HIP(call)                                                          \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess)                                                      \
      throw ::kry::Error{e_ == hipErrorOutOfMemory ? KRY_ENOMEM : KRY_EDEVICE, \
                         std::string(#call) + ": " + hipGetErrorString(e_)};   \
  } while (0)

// ------------------------------------------------------------- scalars
// Per-solve control word shared by every kernel of a chunk. Kernels of chunk
// step s run only while s < stop_at; the finalize kernel that detects
// convergence (or an invariant Krylov space) at step s sets stop_at = s + 1,
// so the rest of step s completes and every later launch returns at its first
// instruction (same stream => kernel boundaries order the stores).
struct Ctrl {
  int32_t stop_at;     // first chunk step that must not run (INT32_MAX = none)
  int32_t invariant;   // Arnoldi / Lanczos invariant flag
  int32_t status;      // device-detected error (KRY_ESINGULAR, ...)
  int32_t xchg;        // in-launch exchange poll form: 0 one 16-B load per block pair; 1 the round-4
                       // form (two 8-B loads, every pair re-read per poll; KRY_XCHG_LEGACY=1, A/B runs only)
};

// ---------------------------------------------------------- device utils
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  // Blocks are dealt round-robin over the 8 XCDs: give each XCD a contiguous
  // range of logical blocks so neighbouring tiles share one L2 (speed only).
  const int q = nb / kNumXcd, r = nb % kNumXcd;
  const int xcd = b % kNumXcd, idx = b / kNumXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Deterministic in-block reduction of `vals` laid out as slots[p], p < nslot,
// where slot p belongs to column (p % k) (k a power of two <= nslot). Leaves
// column sums in slots[0..k). Fixed tree => bitwise reproducible.
__device__ __forceinline__ void block_tree_reduce(double *slots, int nslot, int k) {
  for (int s = nslot >> 1; s >= k; s >>= 1) {
    __syncthreads();
    for (int p = threadIdx.x; p < s; p += blockDim.x) slots[p] = slots[p] + slots[p + s];
  }
  __syncthreads();
}

template <typename V>
struct Vec16;
template <>
struct Vec16<double> {
  using T = double2;
  static constexpr int W = 2;
};
template <>
struct Vec16<float> {
  using T = float4;
  static constexpr int W = 4;
};

inline int grid_for(int64_t work_items, int per_block) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (int)g;
}

inline bool is_pow2(int64_t x) { return x > 0 && (x & (x - 1)) == 0; }

}  // namespace kry
