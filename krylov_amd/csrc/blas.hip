// Device vector operations for the other solver loops (bicgstab, cgs,
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

// ---------------------------------------------- device-resident scalar chain
// These solvers (bicgstab, cgs, cgr, gcr) keep their per-iteration
// scalars in a device register file (kry_prog: nregs rows of k doubles), so
// a whole chunk of iterations is enqueued without a host round trip: inner
// products reduce into registers, scalar lines of the reference evaluate on
// registers, lincombs read their coefficients from registers, and every
// launch of chunk step s runs iff s < ctrl.stop_at (the convergence checks
// set it). Scalars are float64, as the host loop evaluated them.
enum {
  SOP_COPY = 0,     // d = a
  SOP_DIVG = 1,     // d = a / guard(b)              guard(x) = x != 0 ? x : 1
  SOP_MULDIVG = 2,  // d = (a * b) / guard(c * e)
  SOP_SQRT = 3,     // d = sqrt(a)
  SOP_GUARD = 4,    // d = guard(a)
  SOP_SET = 5,      // d = value
  SOP_COUNT = 6
};

__device__ __forceinline__ double guard1(double x) { return x != 0.0 ? x : 1.0; }

__global__ void prog_scalar_kernel(double *regs, int k, int op, int d, int a, int b, int c, int e, double value,
                                   const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  const int i = threadIdx.x;
  if (i >= k) return;
  const double *ra = regs + (int64_t)a * k, *rb = regs + (int64_t)b * k;
  double r;
  switch (op) {
    case SOP_COPY: r = ra[i]; break;
    case SOP_DIVG: r = ra[i] / guard1(rb[i]); break;
    case SOP_MULDIVG: {
      const double num = ra[i] * rb[i];
      const double den = regs[(int64_t)c * k + i] * regs[(int64_t)e * k + i];
      r = num / guard1(den);
      break;
    }
    case SOP_SQRT: r = sqrt(ra[i]); break;
    case SOP_GUARD: r = guard1(ra[i]); break;
    default: r = value; break;
  }
  regs[(int64_t)d * k + i] = r;
}

// d = fixed-order sum of the partials (the dot's second stage), halted-aware
__global__ void prog_reduce_kernel(const double *part, int P, int k, double *out, const Ctrl *ctrl, int step) {
  if (halted(ctrl, step)) return;
  __shared__ double red[kBlock];
  reduce_partials(part, P, k, red);
  if ((int)threadIdx.x < k) out[threadIdx.x] = red[threadIdx.x];
}

// convergence checks on a register of norms against the criterion (padded
// columns +inf): mode 0 appends the row to the chunk history and stops the
// chunk after this step when every column meets it (the top-of-loop test of
// the reference's next iteration); mode 1 (bicgstab's mid-step test,
// bicgstab.py:123-127) on success writes the row at this step, sets
// ctrl.invariant = 2 and stops the chunk at this step.
// Bit 2 of mode: compare the norm rounded to float32 (the reference's
// history entries of a float32 solve are float32; the top-of-loop test
// compares those).
__global__ void prog_check_kernel(const double *nrm, const double *crit, int k, double *hist, Ctrl *ctrl, int step,
                                  int mode) {
  if (halted(ctrl, step)) return;
  __shared__ int flag;
  if (threadIdx.x == 0) flag = 1;
  __syncthreads();
  const int i = threadIdx.x;
  const bool r32 = (mode & 4) != 0;
  mode &= 3;
  if (i < k) {
    const double v = r32 ? (double)(float)nrm[i] : nrm[i];
    if (!(v <= crit[i])) flag = 0;
  }
  __syncthreads();
  const bool all = flag != 0;
  if (mode == 0) {
    if (i < k) hist[(int64_t)step * k + i] = nrm[i];
    if (all && i == 0) ctrl->stop_at = step + 1;
  } else if (all) {
    if (i < k) hist[(int64_t)step * k + i] = nrm[i];
    if (i == 0) {
      ctrl->invariant = 2;
      ctrl->stop_at = step;
    }
  }
}

template <typename V>
struct OpDotP {
  const V *x, *y;
  const double *w;
  int k;
  __device__ __forceinline__ void operator()(int64_t e, int64_t N, double (&acc)[Vec16<V>::W]) const {
    constexpr int W = Vec16<V>::W;
    V a[W], b[W];
    VIO<V>::load(x, e, N, a);
    VIO<V>::load(y, e, N, b);
#pragma unroll
    for (int v = 0; v < W; ++v)
      if (e + v < N)
        acc[v] += w ? dterm_w((double)a[v], w[(e + v) / k], (double)b[v]) : dterm((double)a[v], (double)b[v]);
  }
};

// lincomb with its coefficients in device registers (sa, sb: +1 / -1, the
// reference's `- alpha * v` as `+ (-alpha) * v`, an exact negation)
template <typename V>
struct OpLincombD {
  V *z;
  const V *x, *y, *w;
  const double *a, *b;
  double sa, sb;
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
      const V av = a ? (V)(sa * a[c]) : V(0), bv = b ? (V)(sb * b[c]) : V(0);
      V r;
      switch (form) {
        case LC_AXPY: { const V t = av * yv[v]; r = xv[v] + t; break; }
        case LC_NEST_ADD: { const V t1 = bv * wv[v]; const V t2 = yv[v] + t1; const V t3 = av * t2; r = xv[v] + t3; break; }
        case LC_NEST_SUB: { const V t1 = bv * wv[v]; const V t2 = yv[v] - t1; const V t3 = av * t2; r = xv[v] + t3; break; }
        case LC_DIV: r = xv[v] / av; break;
        case LC_SUB: r = xv[v] - yv[v]; break;
        case LC_ADD: r = xv[v] + yv[v]; break;
        case LC_SCALE: r = av * xv[v]; break;
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

struct kry_prog {
  kry_ctx *ctx = nullptr;
  int nregs = 0, k = 1, cap = 0;
  double *regs = nullptr;  // nregs x k
  double *crit = nullptr;  // k
  double *hist = nullptr;  // cap x k
  double *part = nullptr;  // part_rows(k) x k (the dots' first stage)
  Ctrl *ctrl = nullptr;
};

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

// ---- device-resident scalar chain (kry_prog) ----------------------------

int kry_prog_create(kry_ctx *ctx, int32_t nregs, int32_t k, int32_t cap, kry_prog **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && out && nregs > 0 && cap > 0, KRY_EINVAL, "bad argument");
  KRY_REQUIRE(is_pow2(k) && k <= kLincombCols, KRY_EUNSUPPORTED, "the scalar chain handles up to 64 columns");
  KRY_HIP(hipSetDevice(ctx->device));
  auto *p = new kry_prog();
  try {
    p->ctx = ctx;
    p->nregs = nregs;
    p->k = k;
    p->cap = cap;
    p->regs = static_cast<double *>(dev_alloc((size_t)nregs * k * 8));
    p->crit = static_cast<double *>(dev_alloc((size_t)k * 8));
    p->hist = static_cast<double *>(dev_alloc((size_t)cap * k * 8));
    p->part = static_cast<double *>(dev_alloc((size_t)part_rows(k) * k * 8));
    p->ctrl = static_cast<Ctrl *>(dev_alloc(sizeof(Ctrl)));
    KRY_HIP(hipMemsetAsync(p->regs, 0, (size_t)nregs * k * 8, ctx->stream));
    reset_ctrl(p->ctrl, ctx->stream);
    KRY_HIP(hipStreamSynchronize(ctx->stream));
  } catch (...) {
    for (void *b : {(void *)p->regs, (void *)p->crit, (void *)p->hist, (void *)p->part, (void *)p->ctrl}) dev_free(b);
    delete p;
    throw;
  }
  *out = p;
  KRY_API_END
}

int kry_prog_destroy(kry_prog *p) {
  KRY_API_BEGIN
  if (!p) return KRY_OK;
  (void)hipSetDevice(p->ctx->device);
  for (void *b : {(void *)p->regs, (void *)p->crit, (void *)p->hist, (void *)p->part, (void *)p->ctrl}) dev_free(b);
  delete p;
  KRY_API_END
}

// register r <- host values (k doubles); crit (r = -1) <- host values
int kry_prog_set(kry_prog *p, int32_t r, const double *vals) {
  KRY_API_BEGIN
  KRY_REQUIRE(p && vals && r >= -1 && r < p->nregs, KRY_EINVAL, "bad register");
  double *dst = r < 0 ? p->crit : p->regs + (int64_t)r * p->k;
  KRY_HIP(hipMemcpyAsync(dst, vals, (size_t)p->k * 8, hipMemcpyHostToDevice, p->ctx->stream));
  KRY_HIP(hipStreamSynchronize(p->ctx->stream));
  KRY_API_END
}

int kry_prog_get(kry_prog *p, int32_t r, double *vals) {
  KRY_API_BEGIN
  KRY_REQUIRE(p && vals && r >= 0 && r < p->nregs, KRY_EINVAL, "bad register");
  KRY_HIP(hipMemcpyAsync(vals, p->regs + (int64_t)r * p->k, (size_t)p->k * 8, hipMemcpyDeviceToHost, p->ctx->stream));
  KRY_HIP(hipStreamSynchronize(p->ctx->stream));
  KRY_API_END
}

// start of a chunk: every step runs until a check stops it
int kry_prog_begin(kry_prog *p) {
  KRY_API_BEGIN
  KRY_REQUIRE(p, KRY_EINVAL, "null argument");
  reset_ctrl(p->ctrl, p->ctx->stream);
  KRY_API_END
}

// end of a chunk of `steps`: one host sync; *done = steps that ran in full,
// *midstep = 1 if a mode-1 check stopped step *done (its row is rows[*done]);
// rows gets done (+ midstep) rows of k
int kry_prog_end(kry_prog *p, int32_t steps, int32_t *done, int32_t *midstep, double *rows) {
  KRY_API_BEGIN
  KRY_REQUIRE(p && done && midstep && rows && steps >= 0 && steps <= p->cap, KRY_EINVAL, "bad argument");
  Ctrl c;
  const int d = read_chunk(p->ctx, p->ctx->stream, p->ctrl, p->hist, steps, p->k, rows, &c);
  *done = d;
  *midstep = (c.invariant == 2 && d < steps) ? 1 : 0;
  if (*midstep) KRY_HIP(hipMemcpy(rows + (size_t)d * p->k, p->hist + (size_t)d * p->k, p->k * 8, hipMemcpyDeviceToHost));
  KRY_API_END
}

int kry_prog_scalar(kry_prog *p, int32_t op, int32_t d, int32_t a, int32_t b, int32_t c, int32_t e, double value,
                    int32_t step) {
  KRY_API_BEGIN
  KRY_REQUIRE(p && op >= 0 && op < SOP_COUNT, KRY_EINVAL, "bad scalar op");
  for (int r : {d, a, b, c, e}) KRY_REQUIRE(r >= 0 && r < p->nregs, KRY_EINVAL, "bad register");
  hipLaunchKernelGGL(prog_scalar_kernel, dim3(1), dim3(64), 0, p->ctx->stream, p->regs, p->k, op, d, a, b, c, e, value,
                     p->ctrl, step);
  KRY_HIP(hipGetLastError());
  KRY_API_END
}

// register d <- inner(x, y) per column (weights w or null)
int kry_prog_dot(kry_prog *p, kry_vec *x, kry_vec *y, kry_vec *w, int32_t d, int32_t step) {
  KRY_API_BEGIN
  KRY_REQUIRE(p && x && y && d >= 0 && d < p->nregs, KRY_EINVAL, "bad argument");
  check_same(x, y, "dot x / y");
  KRY_REQUIRE(x->k == p->k, KRY_EINVAL, "column count differs from the chain's");
  KRY_REQUIRE(!w || (w->n == x->n && w->k == 1 && w->dtype == KRY_F64), KRY_EINVAL, "weights must be (n,) float64");
  const int k = p->k;
  const int64_t N = x->n * (int64_t)k;
  const double *wd = w ? static_cast<const double *>(w->d) : nullptr;
  hipStream_t st = p->ctx->stream;
  int P;
  if (x->dtype == KRY_F64)
    P = launch_elementwise<double>(N, k, OpDotP<double>{static_cast<const double *>(x->d), static_cast<const double *>(y->d), wd, k},
                                   p->part, p->ctrl, step, st);
  else
    P = launch_elementwise<float>(N, k, OpDotP<float>{static_cast<const float *>(x->d), static_cast<const float *>(y->d), wd, k},
                                  p->part, p->ctrl, step, st);
  hipLaunchKernelGGL(prog_reduce_kernel, dim3(1), dim3(kBlock), 0, st, p->part, P, k, p->regs + (int64_t)d * k, p->ctrl,
                     step);
  KRY_HIP(hipGetLastError());
  KRY_API_END
}

// z = form(x, y, w; sa * reg_a, sb * reg_b) (register -1: unused)
int kry_prog_lincomb(kry_prog *p, int32_t form, kry_vec *z, kry_vec *x, kry_vec *y, kry_vec *w, int32_t ra, double sa,
                     int32_t rb, double sb, int32_t step) {
  KRY_API_BEGIN
  KRY_REQUIRE(p && z && x && form >= 0 && form < LC_COUNT, KRY_EINVAL, "bad argument");
  KRY_REQUIRE(ra >= -1 && ra < p->nregs && rb >= -1 && rb < p->nregs, KRY_EINVAL, "bad register");
  check_same(z, x, "z / x");
  if (y) check_same(y, x, "y / x");
  if (w) check_same(w, x, "w / x");
  KRY_REQUIRE(x->k == p->k, KRY_EINVAL, "column count differs from the chain's");
  const int k = p->k;
  const int64_t N = x->n * (int64_t)k;
  const double *a = ra >= 0 ? p->regs + (int64_t)ra * k : nullptr;
  const double *b = rb >= 0 ? p->regs + (int64_t)rb * k : nullptr;
  if (x->dtype == KRY_F64)
    launch_elementwise<double>(N, k,
                               OpLincombD<double>{static_cast<double *>(z->d), static_cast<const double *>(x->d),
                                                  y ? static_cast<const double *>(y->d) : nullptr,
                                                  w ? static_cast<const double *>(w->d) : nullptr, a, b, sa, sb, form, k},
                               nullptr, p->ctrl, step, p->ctx->stream);
  else
    launch_elementwise<float>(N, k,
                              OpLincombD<float>{static_cast<float *>(z->d), static_cast<const float *>(x->d),
                                                y ? static_cast<const float *>(y->d) : nullptr,
                                                w ? static_cast<const float *>(w->d) : nullptr, a, b, sa, sb, form, k},
                              nullptr, p->ctrl, step, p->ctx->stream);
  KRY_API_END
}

// y = A x, halted-aware (the chain's SpMV)
int kry_prog_spmv(kry_prog *p, kry_csr *A, kry_vec *x, kry_vec *y, int32_t step) {
  KRY_API_BEGIN
  KRY_REQUIRE(p && A && x && y, KRY_EINVAL, "null argument");
  KRY_REQUIRE(x->n == A->n && y->n == A->n && x->k == y->k && x->dtype == y->dtype, KRY_EINVAL, "shape mismatch");
  const int k = x->k;
  dispatch_vmi(x->dtype, A->dtype, A->itype, [&](auto v0, auto m0, auto i0) {
    using V = decltype(v0);
    using MV = decltype(m0);
    using I = decltype(i0);
    ProfScope ps(p->ctx, PROF_SPMV);
    launch_spmv<V, MV, I>(A, k, SrcPlain<V>{static_cast<const V *>(x->d), k}, EpiStore<V>{static_cast<V *>(y->d), k},
                          nullptr, nullptr, p->ctrl, step, p->ctx->stream);
  });
  KRY_API_END
}

// convergence check on register r (see prog_check_kernel)
int kry_prog_check(kry_prog *p, int32_t r, int32_t mode, int32_t step) {
  KRY_API_BEGIN
  KRY_REQUIRE(p && r >= 0 && r < p->nregs && ((mode & 3) == 0 || (mode & 3) == 1) && mode < 8, KRY_EINVAL,
              "bad argument");
  KRY_REQUIRE(step >= 0 && step < p->cap, KRY_EINVAL, "step beyond the chain's history capacity");
  hipLaunchKernelGGL(prog_check_kernel, dim3(1), dim3(64), 0, p->ctx->stream, p->regs + (int64_t)r * p->k, p->crit,
                     p->k, p->hist, p->ctrl, step, mode);
  KRY_HIP(hipGetLastError());
  KRY_API_END
}

}  // extern "C"
