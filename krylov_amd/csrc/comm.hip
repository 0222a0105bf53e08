// RCCL communicator for RHS-column sharding (one process per GPU over xGMI).
#include <cstring>

#include <vector>

#include "solver_common.hpp"

using namespace kry;

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

#define KRY_NCCL(call)                                                                         \
  do {                                                                                         \
    ncclResult_t r_ = (call);                                                                  \
    if (r_ != ncclSuccess) throw Error{KRY_ECOMM, std::string(#call) + ": " + ncclGetErrorString(r_)}; \
  } while (0)

static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");

extern "C" {

int kry_comm_unique_id(void *id128) {
  KRY_API_BEGIN
  KRY_REQUIRE(id128, KRY_EINVAL, "null id");
  ncclUniqueId id;
  KRY_NCCL(ncclGetUniqueId(&id));
  std::memcpy(id128, &id, sizeof(id));
  KRY_API_END
}

int kry_comm_create(kry_ctx *ctx, int32_t nranks, int32_t rank, const void *id128, kry_comm **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctx && id128 && out, KRY_EINVAL, "null argument");
  KRY_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, KRY_EINVAL, "bad rank / nranks");
  KRY_HIP(hipSetDevice(ctx->device));
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  auto *c = new kry_comm();
  c->ctx = ctx;
  c->nranks = nranks;
  c->rank = rank;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    throw Error{KRY_ECOMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)};
  }
  *out = c;
  KRY_API_END
}

// One communicator per context of ONE process (ncclCommInitAll over the
// contexts' devices, rank i = ctxs[i]): the single-process multi-GPU path
// (krylov_amd.cg(..., devices=[...])), one host thread per device.
int kry_comm_create_all(kry_ctx **ctxs, int32_t n, kry_comm **out) {
  KRY_API_BEGIN
  KRY_REQUIRE(ctxs && out && n >= 1, KRY_EINVAL, "bad argument");
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) {
    KRY_REQUIRE(ctxs[i], KRY_EINVAL, "null context");
    devs[i] = ctxs[i]->device;
    for (int j = 0; j < i; ++j) KRY_REQUIRE(devs[j] != devs[i], KRY_EINVAL, "a device listed twice");
  }
  std::vector<ncclComm_t> comms(n, nullptr);
  ncclResult_t r = ncclCommInitAll(comms.data(), n, devs.data());
  if (r != ncclSuccess) throw Error{KRY_ECOMM, std::string("ncclCommInitAll: ") + ncclGetErrorString(r)};
  for (int i = 0; i < n; ++i) {
    auto *c = new kry_comm();
    c->ctx = ctxs[i];
    c->comm = comms[i];
    c->nranks = n;
    c->rank = i;
    out[i] = c;
  }
  KRY_API_END
}

int kry_comm_destroy(kry_comm *c) {
  KRY_API_BEGIN
  if (!c) return KRY_OK;
  (void)hipSetDevice(c->ctx->device);
  (void)hipStreamSynchronize(c->ctx->stream);
  if (c->comm && !c->aborted.load()) (void)ncclCommDestroy(c->comm);
  dev_free(c->dbuf);
  delete c;
  KRY_API_END
}

// Abort the communicator (ncclCommAbort), callable from another thread while
// a collective on it is pending: the pending and every later collective
// fails (the solvers then stop with KRY_ECOMM) instead of waiting for a rank
// that will not come. The single-process multi-GPU driver calls it on every
// device's communicator when one device's thread fails.
int kry_comm_abort(kry_comm *c) {
  KRY_API_BEGIN
  KRY_REQUIRE(c, KRY_EINVAL, "null communicator");
  // the flag first: a peer thread's next enqueue fails without touching the
  // handle; then the lock, so no enqueue is in flight on the handle the abort
  // frees. A lock not obtained within 10 s means an enqueue is itself blocked
  // inside RCCL (a connection waiting for a peer): abort anyway, which is
  // what releases it.
  if (c->aborted.exchange(true, std::memory_order_acq_rel)) return KRY_OK;
  bool locked = c->mu.try_lock_for(std::chrono::seconds(10));
  ncclComm_t h = c->comm;
  c->comm = nullptr;
  ncclResult_t r = ncclSuccess;
  if (h) {
    (void)hipSetDevice(c->ctx->device);
    r = ncclCommAbort(h);
  }
  if (locked) c->mu.unlock();
  if (r != ncclSuccess) throw Error{KRY_ECOMM, std::string("ncclCommAbort: ") + ncclGetErrorString(r)};
  KRY_API_END
}

int kry_comm_info(kry_comm *c, int32_t *nranks, int32_t *rank) {
  KRY_API_BEGIN
  KRY_REQUIRE(c && nranks && rank, KRY_EINVAL, "null argument");
  std::lock_guard<std::timed_mutex> g(c->mu);
  KRY_REQUIRE(!c->aborted.load() && c->comm, KRY_ECOMM, "the communicator was aborted");
  int n = 0, r = 0;
  KRY_NCCL(ncclCommCount(c->comm, &n));
  KRY_NCCL(ncclCommUserRank(c->comm, &r));
  *nranks = n;
  *rank = r;
  KRY_API_END
}

// Host-side convenience: in-place sum over ranks of `count` doubles (setup-time
// exchanges such as the initial residual norms; not used inside iterations).
int kry_comm_allreduce(kry_comm *c, double *host, int32_t count) {
  KRY_API_BEGIN
  KRY_REQUIRE(c && host && count >= 0, KRY_EINVAL, "bad argument");
  KRY_REQUIRE(!c->aborted.load(), KRY_ECOMM, "the communicator was aborted");
  if (count == 0) return KRY_OK;
  KRY_HIP(hipSetDevice(c->ctx->device));
  hipStream_t st = c->ctx->stream;
  if (c->dbuf_len < count) {
    dev_free(c->dbuf);
    c->dbuf = nullptr;
    c->dbuf = static_cast<double *>(dev_alloc((size_t)count * 8));
    c->dbuf_len = count;
  }
  KRY_HIP(hipMemcpyAsync(c->dbuf, host, (size_t)count * 8, hipMemcpyHostToDevice, st));
  comm_allreduce(c, c->dbuf, (size_t)count, st);
  KRY_HIP(hipMemcpyAsync(host, c->dbuf, (size_t)count * 8, hipMemcpyDeviceToHost, st));
  KRY_HIP(hipStreamSynchronize(st));
  KRY_API_END
}

}  // extern "C"
