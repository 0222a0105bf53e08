// Device vector operations for the host-driven solver loops (bicgstab, cgs,
// cgr, gcr, ... of the reference; krylov_amd/extra.py). Each call is one
// stream-ordered launch evaluating exactly the NumPy expression tree of the
// reference line it replaces, with per-column scalars handed over by value.
#include "solver_common.hpp"

using namespace kry;

namespace {

constexpr int kLincombCols = 64;  // by-value scalars: 2 x 64 doubles of kernel arguments

struct Scal2 {
  double a[kLincombCols];
  double b[kLincombCols];
};

enum {
  LC_AXPY = 0,      // z = x + a y
  LC_NEST_ADD = 1,  // z = x + a (y + b w)
  LC_NEST_SUB = 2,  // z = x + a (y - b w)
  LC_DIV = 3,       // z = x / a
  LC_SUB = 4,       // z = x - y
  LC_ADD = 5,       // z = x + y
  LC_COPY = 6,      // z = x
  LC_SCALE = 7,     // z = a x
  LC_COUNT = 8
};

template <typename V>
struct OpLincomb {
  V *z;
  const V *x, *y, *w;
  Scal2 s;
  int form, k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V xv[W], yv[W], wv[W];
    VIO<V>::load(x, e, N, xv);
    if (y) VIO<V>::load(y, e, N, yv);
    if (w) VIO<V>::load(w, e, N, wv);
#pragma unroll
    for (int v = 0; v < W; ++v) {
      const int c = (int)((e + v) & (k - 1));
      const V a = (V)s.a[c], b = (V)s.b[c];
      V r;
      switch (form) {
        case LC_AXPY: { const V t = a * yv[v]; r = xv[v] + t; break; }
        case LC_NEST_ADD: { const V t1 = b * wv[v]; const V t2 = yv[v] + t1; const V t3 = a * t2; r = xv[v] + t3; break; }
        case LC_NEST_SUB: { const V t1 = b * wv[v]; const V t2 = yv[v] - t1; const V t3 = a * t2; r = xv[v] + t3; break; }
        case LC_DIV: r = xv[v] / a; break;
        case LC_SUB: r = xv[v] - yv[v]; break;
        case LC_ADD: r = xv[v] + yv[v]; break;
        case LC_SCALE: r = a * xv[v]; break;
        default: r = xv[v]; break;
      }
      xv[v] = r;
    }
    VIO<V>::store(z, e, N, xv);
  }
};

void check_same(const kry_vec *a, const kry_vec *b, const char *what) {
  KRY_REQUIRE(a->n == b->n && a->k == b->k && a->dtype == b->dtype, KRY_EINVAL,
              std::string("shape/dtype mismatch: ") + what);
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

int kry_vec_lincomb(kry_ctx *ctx, int form, kry_vec *z, kry_vec *x, kry_vec *y, kry_vec *w, const double *a,
                    const double *b) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && z && x, KRY_EINVAL, "null argument");
  KRY_REQUIRE(form >= 0 && form < LC_COUNT, KRY_EINVAL, "unknown lincomb form");
  const bool needs_y = form == LC_AXPY || form == LC_NEST_ADD || form == LC_NEST_SUB || form == LC_SUB || form == LC_ADD;
  const bool needs_w = form == LC_NEST_ADD || form == LC_NEST_SUB;
  const bool needs_a = form == LC_AXPY || form == LC_NEST_ADD || form == LC_NEST_SUB || form == LC_DIV || form == LC_SCALE;
  KRY_REQUIRE(!needs_y || y, KRY_EINVAL, "this form needs y");
  KRY_REQUIRE(!needs_w || w, KRY_EINVAL, "this form needs w");
  KRY_REQUIRE(!needs_a || a, KRY_EINVAL, "this form needs a");
  KRY_REQUIRE(!needs_w || b, KRY_EINVAL, "this form needs b");
  check_same(z, x, "z / x");
  if (needs_y) check_same(y, x, "y / x");
  if (needs_w) check_same(w, x, "w / x");
  const int k = x->k;
  KRY_REQUIRE(is_pow2(k) && k <= kLincombCols, KRY_EUNSUPPORTED, "lincomb handles up to 64 columns");
  KRY_HIP(hipSetDevice(ctx->device));
  Scal2 sc{};
  for (int c = 0; c < k; ++c) {
    sc.a[c] = needs_a ? a[c] : 0.0;
    sc.b[c] = needs_w ? b[c] : 0.0;
  }
  const int64_t N = x->n * (int64_t)k;
  if (x->dtype == KRY_F64)
    launch_elementwise<double>(N, k,
                               OpLincomb<double>{static_cast<double *>(z->d), static_cast<const double *>(x->d),
                                                 needs_y ? static_cast<const double *>(y->d) : nullptr,
                                                 needs_w ? static_cast<const double *>(w->d) : nullptr, sc, form, k},
                               nullptr, nullptr, 0, ctx->stream);
  else
    launch_elementwise<float>(N, k,
                              OpLincomb<float>{static_cast<float *>(z->d), static_cast<const float *>(x->d),
                                               needs_y ? static_cast<const float *>(y->d) : nullptr,
                                               needs_w ? static_cast<const float *>(w->d) : nullptr, sc, form, k},
                              nullptr, nullptr, 0, ctx->stream);
  KRY_API_END
}

}  // extern "C"
