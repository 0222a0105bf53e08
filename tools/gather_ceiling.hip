// Gather ceiling of the column-blocked SpMV on a given matrix (development
// tool, not product; round 4). The library builds its column-blocked image
// (kry_csr::cb_*) for the matrix; then, on that image's arrays in storage
// order (column block after column block, so the x gathers of all CUs fall in
// one 2 MB block of x at a time, as in the SpMV), four kernels are timed:
//
//   library  the SpMV launch_spmv runs for one right-hand side (y = A x)
//   gather   a stream of the 4-B column indices and one 8-B gather of x per
//            entry, 16-B column loads, 4 gathers per thread per round,
//            grid-stride over the whole image (no row bookkeeping, no LDS,
//            no y): the access shape alone
//   image    the same plus the 8-B values (the whole image stream + gathers):
//            the ceiling the SpMV is measured against
//   window   random 8-B gathers from one L2-resident 2 MB window (no stream)
//   stream   the 12-B column + value stream alone (no gathers)
//
// The grid-stride kernels are not a ceiling for the SpMV (the library's
// blocks walk the column blocks in step and run faster); the ceiling model
// is max(nnz / window rate, stream time) if gathers and stream overlapped
// perfectly, and their sum if they share the load path serially.
// Each reports ms per launch and G gathers/s (nnz / time). Called from
// tools/gather_ceiling.py, which builds cfg3 and the permuted metric matrix
// and writes profiles/r04_gather_ceiling.json.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC \
//     tools/gather_ceiling.hip -o tools/libgather_ceiling.so -Lkrylov_amd -lkrylov_hip \
//     -Wl,-rpath,'$ORIGIN/../krylov_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/krylov_hip.h"
#include "../krylov_amd/csrc/device.hpp"

using namespace kry;

typedef int gi4 __attribute__((ext_vector_type(4)));
typedef double gd2 __attribute__((ext_vector_type(2)));

template <bool VAL, bool GATHER = true>
__global__ __launch_bounds__(256) void gc_stream(const gi4 *__restrict__ col, const gd2 *__restrict__ val, int64_t nnz,
                                                 const double *__restrict__ x, double *__restrict__ out) {
  const int64_t nq = (nnz + 3) / 4;
  double s = 0.0;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
    const gi4 c = __builtin_nontemporal_load(col + q);
    double a0 = 1.0, a1 = 1.0, a2 = 1.0, a3 = 1.0;
    if (VAL) {
      const gd2 v0 = __builtin_nontemporal_load(val + 2 * q), v1 = __builtin_nontemporal_load(val + 2 * q + 1);
      a0 = v0.x; a1 = v0.y; a2 = v1.x; a3 = v1.y;
    }
    const int64_t e = 4 * q;
    if (GATHER) {
      const double x0 = x[c.x];
      const double x1 = e + 1 < nnz ? x[c.y] : 0.0;
      const double x2 = e + 2 < nnz ? x[c.z] : 0.0;
      const double x3 = e + 3 < nnz ? x[c.w] : 0.0;
      s += a0 * x0 + a1 * x1 + a2 * x2 + a3 * x3;
    } else {
      s += a0 * (double)c.x + a1 * (double)c.y + a2 * (double)c.z + a3 * (double)c.w;
    }
  }
  if (s == 1234.5678) out[0] = s;  // keeps the loads; never true for these inputs
}

__global__ __launch_bounds__(256) void gc_window(const double *__restrict__ x, int64_t span, int rounds,
                                                 double *__restrict__ out) {
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
  double s = 0.0;
  for (int r = 0; r < rounds; ++r) {
    double v[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      h ^= h << 13; h ^= h >> 17; h ^= h << 5;
      v[g] = x[h % (uint32_t)span];
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) s += v[g];
  }
  if (s == 1234.5678) out[0] = s;
}

// Candidate (round 4): contiguous ownership. Block blk owns the row groups
// [gb, gb + own) (own <= OWN), so for column block b their segments are ONE
// contiguous entry range: it is walked in full 1024-entry chunks (quads of
// entries, as the library kernel), the products staged in LDS, and every
// thread adds to each of its OWN rows' running sums the chunk's entries of
// that row (its range from the row offsets), in stored order: bitwise the
// library kernel. The library walks every (column block, group) segment as
// its own chunk, and a segment of 256 rows holds ~240 (permuted metric) to
// ~640 (cfg3) entries: most of each 1024-entry chunk idles.
template <int OWN, class Epi>
__global__ __launch_bounds__(256) void spmv_cbc(int nb, int64_t n, int64_t ng, int64_t g0, int64_t g1, int own,
                                                const int64_t *__restrict__ gptr, const uint16_t *__restrict__ roff,
                                                const int *__restrict__ col, const double *__restrict__ val,
                                                const double *__restrict__ x, Epi epi) {
  __shared__ double prod[kCbCap];
  const int tid = threadIdx.x;
  const int64_t gb = g0 + (int64_t)blockIdx.x * own;
  const int no = (int)std::min<int64_t>(own, g1 - gb);
  if (no <= 0) return;
  double acc[OWN];
#pragma unroll
  for (int o = 0; o < OWN; ++o) acc[o] = 0.0;
  for (int b = 0; b < nb; ++b) {
    const int64_t eb = gptr[(int64_t)b * ng + gb], ee = gptr[(int64_t)b * ng + gb + no];
    int r0[OWN], r1[OWN];  // this thread's row of each owned group: entries [r0, r1) of the block's range
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      r0[o] = r1[o] = 0;
      if (o < no) {
        const int64_t s0 = gptr[(int64_t)b * ng + gb + o];
        const int len = (int)(gptr[(int64_t)b * ng + gb + o + 1] - s0);
        const int64_t row = (gb + o) * kCbRows + tid;
        if (row < n) {
          const int a = roff[(int64_t)b * n + row];
          const int z = (tid == kCbRows - 1 || row + 1 >= n) ? len : (int)roff[(int64_t)b * n + row + 1];
          r0[o] = (int)(s0 - eb) + a;
          r1[o] = (int)(s0 - eb) + z;
        }
      }
    }
    typedef int i4 __attribute__((ext_vector_type(4)));
    typedef double d2 __attribute__((ext_vector_type(2)));
    const int64_t q0 = eb >> 2, qend = (ee + 3) >> 2;
    for (int64_t qc = q0; qc < qend; qc += 256) {
      const int64_t base = qc * 4 - eb;  // block-range-relative entry held by prod[0]
      __syncthreads();                   // the previous chunk has been consumed
      const int64_t q = qc + tid;
      if (q < qend) {
        const i4 c = __builtin_nontemporal_load(reinterpret_cast<const i4 *>(col) + q);
        const d2 v0 = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(val) + 2 * q);
        const d2 v1 = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(val) + 2 * q + 1);
        const int jj[4] = {c.x, c.y, c.z, c.w};
        const double aa[4] = {v0.x, v0.y, v1.x, v1.y};
        double xj[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t e = base + 4 * (int64_t)tid + i;
          xj[i] = (e >= 0 && e < ee - eb) ? x[jj[i]] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t e = base + 4 * (int64_t)tid + i;
          if (e >= 0 && e < ee - eb) prod[4 * tid + i] = aa[i] * xj[i];
        }
      }
      __syncthreads();
#pragma unroll
      for (int o = 0; o < OWN; ++o) {
        if (o >= no) break;
        const int64_t lo = r0[o] > base ? r0[o] : base, hi = r1[o] < base + kCbCap ? r1[o] : base + kCbCap;
        for (int64_t e = lo; e < hi; ++e) acc[o] = acc[o] + prod[e - base];
      }
    }
  }
#pragma unroll
  for (int o = 0; o < OWN; ++o) {
    if (o >= no) break;
    const int64_t row = (gb + o) * kCbRows + tid;
    if (row < n) epi(row, 0, acc[o], 0.0);
  }
}

// Candidates (round 4, second set): contiguous ownership as spmv_cbc, plus
//   QPT  quads per thread and chunk (chunk = 1024 * QPT entries): more
//        loads and gathers in flight per wave;
//   PF   the next chunk's column / value quads are loaded into registers
//        before this chunk's gathers, across column blocks too (the chunk
//        after a block's last one is the next block's first), so the stream
//        latency hides behind the gathers;
//   the products are double-buffered in LDS: one barrier per chunk.
// The grid and the groups a block owns are the launcher's (OWN at most).
template <int OWN, int QPT, bool PF, class Epi, bool NOROFF = false>
__global__ __launch_bounds__(256) void spmv_cbx(int nb, int64_t n, int64_t ng, int64_t g0, int64_t g1, int own,
                                                const int64_t *__restrict__ gptr, const uint16_t *__restrict__ roff,
                                                const int *__restrict__ col, const double *__restrict__ val,
                                                const double *__restrict__ x, Epi epi) {
  constexpr int CAP = 1024 * QPT;
  typedef int i4 __attribute__((ext_vector_type(4)));
  typedef double d2 __attribute__((ext_vector_type(2)));
  __shared__ double prod[2][CAP];
  const int tid = threadIdx.x;
  const int64_t gb = g0 + (int64_t)blockIdx.x * own;
  const int no = (int)std::min<int64_t>(own, g1 - gb);
  if (no <= 0) return;
  double acc[OWN];
#pragma unroll
  for (int o = 0; o < OWN; ++o) acc[o] = 0.0;
  int r0[OWN], r1[OWN];
  auto setup = [&](int b, int64_t eb) {
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      r0[o] = r1[o] = 0;
      if (!NOROFF && o < no) {
        const int64_t s0 = gptr[(int64_t)b * ng + gb + o];
        const int len = (int)(gptr[(int64_t)b * ng + gb + o + 1] - s0);
        const int64_t row = (gb + o) * kCbRows + tid;
        if (row < n) {
          const int a = roff[(int64_t)b * n + row];
          const int z = (tid == kCbRows - 1 || row + 1 >= n) ? len : (int)roff[(int64_t)b * n + row + 1];
          r0[o] = (int)(s0 - eb) + a;
          r1[o] = (int)(s0 - eb) + z;
        }
      }
    }
  };
  // chunk cursor: column block b, entries [eb, ee), quad qc
  int b = 0;
  int64_t eb = gptr[gb], ee = gptr[gb + no];
  int64_t qc = eb >> 2;
  auto advance = [&](int &bb, int64_t &ebb, int64_t &eee, int64_t &q) {  // to the next chunk; false at the end
    q += 256 * QPT;
    while (q >= ((eee + 3) >> 2)) {
      if (++bb >= nb) return false;
      ebb = gptr[(int64_t)bb * ng + gb];
      eee = gptr[(int64_t)bb * ng + gb + no];
      q = ebb >> 2;
    }
    return true;
  };
  // the first chunk may be empty too
  {
    int64_t q = qc - 256 * QPT;
    if (!advance(b, eb, ee, q)) b = nb;
    qc = q;
  }
  if (b < nb) setup(b, eb);
  i4 c[QPT];
  d2 v[2 * QPT];
  auto load = [&](int64_t q0, int64_t qe, i4 *cc, d2 *vv) {
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
      const int64_t q = q0 + u * 256 + tid;
      if (q < qe) {
        cc[u] = __builtin_nontemporal_load(reinterpret_cast<const i4 *>(col) + q);
        vv[2 * u] = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(val) + 2 * q);
        vv[2 * u + 1] = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(val) + 2 * q + 1);
      }
    }
  };
  if (b < nb) load(qc, (ee + 3) >> 2, c, v);
  int buf = 0;
  while (b < nb) {
    int nbk = b;
    int64_t neb = eb, nee = ee, nq = qc;
    const bool more = advance(nbk, neb, nee, nq);
    i4 cn[QPT];
    d2 vn[2 * QPT];
    if (PF && more) load(nq, (nee + 3) >> 2, cn, vn);
    const int64_t base = qc * 4 - eb;
    const int64_t len = ee - eb;
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
      const int jj[4] = {c[u].x, c[u].y, c[u].z, c[u].w};
      const double aa[4] = {v[2 * u].x, v[2 * u].y, v[2 * u + 1].x, v[2 * u + 1].y};
      double xj[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t e = base + 4 * (int64_t)(u * 256 + tid) + i;
        xj[i] = (e >= 0 && e < len) ? x[jj[i]] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t e = base + 4 * (int64_t)(u * 256 + tid) + i;
        if (e >= 0 && e < len) prod[buf][4 * (u * 256 + tid) + i] = aa[i] * xj[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int o = 0; o < OWN; ++o) {
      if (o >= no) break;
      const int64_t lo = r0[o] > base ? r0[o] : base, hi = r1[o] < base + CAP ? r1[o] : base + CAP;
      for (int64_t e = lo; e < hi; ++e) acc[o] = acc[o] + prod[buf][e - base];
    }
    buf ^= 1;
    if (!more) break;
    if (nbk != b) setup(nbk, neb);
    b = nbk; eb = neb; ee = nee; qc = nq;
    if (PF) {
#pragma unroll
      for (int u = 0; u < QPT; ++u) { c[u] = cn[u]; v[2 * u] = vn[2 * u]; v[2 * u + 1] = vn[2 * u + 1]; }
    } else {
      load(qc, (ee + 3) >> 2, c, v);
    }
  }
#pragma unroll
  for (int o = 0; o < OWN; ++o) {
    if (o >= no) break;
    const int64_t row = (gb + o) * kCbRows + tid;
    if (row < n) epi(row, 0, acc[o], 0.0);
  }
}

extern "C" int gc_run(int64_t n, int64_t nnz, const int *ip, const int *ix, const double *dv, int reps,
                      double *res /* [0] library ms, [1] gather ms, [2] image ms, [3] window G/s, [4] nb, [5] cols,
                                  [6] stream ms, [7] contiguous-ownership candidate ms, [8] its
                                  entries differing from the library's y, [9 + 2 i], [10 + 2 i]: the same for
                                  spmv_cbx variant i (i < 8) */) {
  kry_ctx *ctx;
  if (kry_ctx_create(0, &ctx) != KRY_OK) return -1;
  kry_csr *A;
  if (kry_csr_create(ctx, n, nnz, ip, ix, dv, KRY_F64, KRY_I32, &A) != KRY_OK) return -2;
  if (A->cb_nb == 0) return -3;
  std::vector<double> xh(n);
  for (int64_t i = 0; i < n; ++i) xh[i] = 1.0 + 1e-3 * (double)((i * 2654435761ull) % 1000);
  double *x, *y, *o;
  hipMalloc(&x, n * 8 + 512);
  hipMalloc(&y, n * 8 + 512);
  hipMalloc(&o, 64);
  hipMemcpy(x, xh.data(), n * 8, hipMemcpyHostToDevice);
  hipStream_t st = ctx->stream;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](auto launch) {
    launch();
    hipStreamSynchronize(st);
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      hipEventRecord(e0, st);
      launch();
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      ts.push_back(t);
    }
    std::sort(ts.begin(), ts.end());
    return (double)ts[ts.size() / 2];
  };
  res[0] = timeit([&] {
    launch_spmv<double, double, int>(A, 1, SrcPlain<double>{x, 1}, EpiStore<double>{y, 1}, nullptr, nullptr,
                                     nullptr, 0, st);
  });
  const gi4 *col = static_cast<const gi4 *>(A->cb_col);
  const gd2 *val = static_cast<const gd2 *>(A->cb_val);
  res[1] = timeit([&] { hipLaunchKernelGGL(gc_stream<false>, dim3(8192), dim3(256), 0, st, col, val, nnz, x, o); });
  res[2] = timeit([&] { hipLaunchKernelGGL(gc_stream<true>, dim3(8192), dim3(256), 0, st, col, val, nnz, x, o); });
  {
    // the contiguous-ownership candidate: bitwise against the library's y
    std::vector<double> yl(n), yc(n);
    hipMemcpy(yl.data(), y, n * 8, hipMemcpyDeviceToHost);
    double *yc_d;
    hipMalloc(&yc_d, n * 8 + 512);
    const int grid = 1024;
    const int64_t per = (int64_t)grid * 16;
    res[7] = timeit([&] {
      for (int64_t g0 = 0; g0 < A->cb_ng; g0 += per) {
        const int64_t g1 = std::min<int64_t>(A->cb_ng, g0 + per);
        const int own = (int)((g1 - g0 + grid - 1) / grid);
        hipLaunchKernelGGL((spmv_cbc<16, EpiStore<double>>), dim3(grid), dim3(256), 0, st, (int)A->cb_nb, n, A->cb_ng,
                           g0, g1, own, (const int64_t *)A->cb_gptr, (const uint16_t *)A->cb_roff,
                           (const int *)A->cb_col, (const double *)A->cb_val, (const double *)x,
                           EpiStore<double>{yc_d, 1});
      }
    });
    hipMemcpy(yc.data(), yc_d, n * 8, hipMemcpyDeviceToHost);
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += memcmp(&yl[i], &yc[i], 8) != 0;
    res[8] = (double)bad;
    auto variant = [&](int i, auto kern, int grid, int ownmax) {
      hipMemset(yc_d, 0, n * 8);
      const int64_t per = (int64_t)grid * ownmax;
      res[9 + 2 * i] = timeit([&] {
        for (int64_t g0 = 0; g0 < A->cb_ng; g0 += per) {
          const int64_t g1 = std::min<int64_t>(A->cb_ng, g0 + per);
          const int own = (int)((g1 - g0 + grid - 1) / grid);
          hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, (int)A->cb_nb, n, A->cb_ng, g0, g1, own,
                             (const int64_t *)A->cb_gptr, (const uint16_t *)A->cb_roff, (const int *)A->cb_col,
                             (const double *)A->cb_val, (const double *)x, EpiStore<double>{yc_d, 1});
        }
      });
      hipMemcpy(yc.data(), yc_d, n * 8, hipMemcpyDeviceToHost);
      int64_t bd = 0;
      for (int64_t r = 0; r < n; ++r) bd += memcmp(&yl[r], &yc[r], 8) != 0;
      res[10 + 2 * i] = (double)bd;
    };
    using E = EpiStore<double>;
    variant(0, spmv_cbx<16, 1, false, E>, 1024, 16);
    variant(1, spmv_cbx<16, 1, true, E>, 1024, 16);
    variant(2, spmv_cbx<16, 2, false, E>, 768, 16);
    variant(3, spmv_cbx<16, 1, false, E, true>, 1024, 16);  // no row offsets (wrong y): their cost
    variant(4, spmv_cbx<8, 1, true, E>, 1280, 8);
    variant(5, spmv_cbx<8, 2, true, E>, 768, 8);
    variant(6, spmv_cbx<16, 1, true, E, true>, 1024, 16);  // no row offsets, prefetch
    variant(7, spmv_cbx<16, 1, true, E>, 768, 16);
    hipFree(yc_d);
  }
  res[6] = timeit([&] {
    hipLaunchKernelGGL((gc_stream<true, false>), dim3(8192), dim3(256), 0, st, col, val, nnz, x, o);
  });
  const int64_t span = std::min<int64_t>(n, 262144);
  const int rounds = 64;
  const double wms = timeit([&] { hipLaunchKernelGGL(gc_window, dim3(8192), dim3(256), 0, st, x, span, rounds, o); });
  res[3] = 8192.0 * 256 * rounds * 8 / (wms * 1e-3) / 1e9;
  // random-gather rate against the window size: 2, 3, 4, 5, 8 MB and the whole x
  const int64_t spans[6] = {262144, 393216, 524288, 655360, 1048576, n};
  for (int i = 0; i < 6; ++i) {
    const int64_t sp = std::min<int64_t>(n, spans[i]);
    const double t = timeit([&] { hipLaunchKernelGGL(gc_window, dim3(8192), dim3(256), 0, st, x, sp, rounds, o); });
    res[25 + i] = 8192.0 * 256 * rounds * 8 / (t * 1e-3) / 1e9;
  }
  res[4] = (double)A->cb_nb;
  res[5] = (double)A->cb_cols;
  hipFree(x);
  hipFree(y);
  hipFree(o);
  kry_csr_destroy(A);
  kry_ctx_destroy(ctx);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
