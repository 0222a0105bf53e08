/*
 * ORACLE — plain-C restatement of the third-party arithmetic under the
 * reference hot path (TEST INFRASTRUCTURE ONLY; never linked into the product).
 *
 * The reference (ju-liu/krylov 0.0.3) has no native code; its SpMV and plane
 * rotations live in dependencies that are present in this image but not in
 * /root/reference:
 *
 *  - SciPy 1.15.3 sparsetools ``csr_matvec`` / ``csr_matvecs`` (sparsetools/csr.h),
 *    reached from ``A @ x`` at _helpers.py:47, cg.py:86, gmres.py:106,
 *    minres.py:111,121. Algorithm: for each row, ``sum = 0; for jj in
 *    [indptr[i], indptr[i+1]): sum += data[jj] * x[indices[jj]]`` in stored
 *    order (unsorted indices, duplicates and explicit zeros are honoured), in
 *    the value type, with no fused multiply-add (x86-64 baseline build).
 *    The multivector form applies the same recurrence to every column.
 *  - LAPACK >= 3.10 ``?lartg`` (la_xlartg.f90, Anderson's safe-scaling
 *    version) via scipy.linalg.lapack, called at givens.py:35-40.
 *
 * Pinned against SciPy itself in tests/test_oracle.py (tests/golden/spmv.npz,
 * tests/golden/lartg.npz). Build: ``make -C oracle`` (gcc, -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>

#define DEF_MATVEC(NAME, V, I)                                                  \
  void NAME(int64_t n, const I *indptr, const I *indices, const V *data,       \
            const V *x, V *y) {                                                 \
    for (int64_t i = 0; i < n; ++i) {                                           \
      V sum = 0;                                                                \
      for (I jj = indptr[i]; jj < indptr[i + 1]; ++jj) {                        \
        V prod = data[jj] * x[indices[jj]];                                     \
        sum = sum + prod;                                                       \
      }                                                                         \
      y[i] = sum;                                                               \
    }                                                                           \
  }                                                                             \
  void NAME##s(int64_t n, int64_t k, const I *indptr, const I *indices,         \
               const V *data, const V *x, V *y) {                               \
    for (int64_t i = 0; i < n; ++i) {                                           \
      V *yi = y + i * k;                                                        \
      for (int64_t c = 0; c < k; ++c) yi[c] = 0;                                \
      for (I jj = indptr[i]; jj < indptr[i + 1]; ++jj) {                        \
        const V a = data[jj];                                                   \
        const V *xj = x + (int64_t)indices[jj] * k;                             \
        for (int64_t c = 0; c < k; ++c) {                                       \
          V prod = a * xj[c];                                                   \
          yi[c] = yi[c] + prod;                                                 \
        }                                                                       \
      }                                                                         \
    }                                                                           \
  }

DEF_MATVEC(oracle_csr_matvec_f64_i32, double, int32_t)
DEF_MATVEC(oracle_csr_matvec_f64_i64, double, int64_t)
DEF_MATVEC(oracle_csr_matvec_f32_i32, float, int32_t)
DEF_MATVEC(oracle_csr_matvec_f32_i64, float, int64_t)

/* LAPACK 3.10+ xLARTG: safmin = radix^max(minexp-1, 1-maxexp), safmax = 1/safmin,
 * rtmin = sqrt(safmin), rtmax = sqrt(safmax/2). */
#define DEF_LARTG(NAME, T, SQRT, FABS, SAFMIN)                                  \
  void NAME(T f, T g, T *c, T *s, T *r) {                                       \
    const T safmin = SAFMIN, safmax = (T)1 / SAFMIN;                            \
    const T rtmin = SQRT(safmin), rtmax = SQRT(safmax / 2);                     \
    const T f1 = FABS(f), g1 = FABS(g);                                         \
    if (g == 0) {                                                               \
      *c = 1; *s = 0; *r = f;                                                   \
    } else if (f == 0) {                                                        \
      *c = 0; *s = g > 0 ? (T)1 : (T)-1; *r = g1;                               \
    } else if (f1 > rtmin && f1 < rtmax && g1 > rtmin && g1 < rtmax) {          \
      T ff = f * f, gg = g * g;                                                 \
      T d = SQRT(ff + gg);                                                      \
      *c = f1 / d;                                                              \
      T rr = f >= 0 ? d : -d;                                                   \
      *r = rr;                                                                  \
      *s = g / rr;                                                              \
    } else {                                                                    \
      T m = f1 > g1 ? f1 : g1;                                                  \
      if (m < safmin) m = safmin;                                               \
      T u = m < safmax ? m : safmax;                                            \
      T fs = f / u, gs = g / u;                                                 \
      T ff = fs * fs, gg = gs * gs;                                             \
      T d = SQRT(ff + gg);                                                      \
      *c = FABS(fs) / d;                                                        \
      T rr = f >= 0 ? d : -d;                                                   \
      *s = gs / rr;                                                             \
      *r = rr * u;                                                              \
    }                                                                           \
  }

DEF_LARTG(oracle_dlartg, double, sqrt, fabs, 2.2250738585072014e-308)
DEF_LARTG(oracle_slartg, float, sqrtf, fabsf, 1.17549435e-38f)
