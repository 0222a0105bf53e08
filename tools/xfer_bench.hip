// Host <-> device vector transfer rates on the GPU box (development tool,
// not product; round 4): what a solve's b upload and x download cost at the
// metric size (80.6 MB) by the runtime's pageable path, against a pinned
// staging buffer (DMA only, and DMA + a multithreaded copy between the
// pinned buffer and ordinary memory), and a chunked pipeline of the two.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xfer_bench.hip -o tools/xfer_bench -lpthread
//   ./tools/xfer_bench [MB=80.6] [threads=8] [chunk_MB=8]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include <sys/mman.h>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(char *dst, const char *src, size_t bytes, int nt) {
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([=] {
      const size_t a = bytes * t / nt / 64 * 64, b = t == nt - 1 ? bytes : bytes * (t + 1) / nt / 64 * 64;
      memcpy(dst + a, src + a, b - a);
    });
  for (auto &x : th) x.join();
}

int main(int argc, char **argv) {
  const double mb = argc > 1 ? atof(argv[1]) : 80.6;
  const int nt = argc > 2 ? atoi(argv[2]) : 8;
  const double cmb = argc > 3 ? atof(argv[3]) : 8.0;
  const size_t bytes = (size_t)(mb * 1e6) / 64 * 64;
  const size_t chunk = (size_t)(cmb * 1e6) / 64 * 64;
  char *host = (char *)aligned_alloc(4096, bytes), *dev, *pin;
  memset(host, 1, bytes);
  CK(hipMalloc(&dev, bytes));
  CK(hipHostMalloc(&pin, bytes, hipHostMallocDefault));
  memset(pin, 2, bytes);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto med = [&](auto f) {
    f();
    std::vector<double> ts;
    for (int r = 0; r < 7; ++r) {
      const double t0 = now();
      f();
      ts.push_back(now() - t0);
    }
    std::sort(ts.begin(), ts.end());
    return ts[3] * 1e3;
  };
  auto rep = [&](const char *name, double ms) {
    printf("%-52s %8.3f ms  %6.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  rep("D2H pageable hipMemcpy", med([&] { CK(hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost)); }));
  rep("H2D pageable hipMemcpy", med([&] { CK(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice)); }));
  rep("D2H pinned hipMemcpy (DMA only)", med([&] { CK(hipMemcpy(pin, dev, bytes, hipMemcpyDeviceToHost)); }));
  rep("H2D pinned hipMemcpy (DMA only)", med([&] { CK(hipMemcpy(dev, pin, bytes, hipMemcpyHostToDevice)); }));
  rep("host copy pinned -> pageable, threads", med([&] { par_copy(host, pin, bytes, nt); }));
  rep("host copy pageable -> pinned, threads", med([&] { par_copy(pin, host, bytes, nt); }));
  rep("host copy 1 thread", med([&] { memcpy(host, pin, bytes); }));
  // chunked pipeline, download: DMA chunk i into the pinned buffer while the
  // host threads copy chunk i - 1 out
  rep("D2H chunked: pinned DMA || threaded copy out", med([&] {
        const size_t nc = (bytes + chunk - 1) / chunk;
        std::vector<hipEvent_t> ev(nc);
        for (size_t c = 0; c < nc; ++c) {
          CK(hipEventCreateWithFlags(&ev[c], hipEventDisableTiming));
          const size_t a = c * chunk, l = std::min(chunk, bytes - a);
          CK(hipMemcpyAsync(pin + a, dev + a, l, hipMemcpyDeviceToHost, st));
          CK(hipEventRecord(ev[c], st));
        }
        for (size_t c = 0; c < nc; ++c) {
          CK(hipEventSynchronize(ev[c]));
          const size_t a = c * chunk, l = std::min(chunk, bytes - a);
          par_copy(host + a, pin + a, l, nt);
          CK(hipEventDestroy(ev[c]));
        }
      }));
  rep("H2D chunked: threaded copy in || pinned DMA", med([&] {
        const size_t nc = (bytes + chunk - 1) / chunk;
        for (size_t c = 0; c < nc; ++c) {
          const size_t a = c * chunk, l = std::min(chunk, bytes - a);
          par_copy(pin + a, host + a, l, nt);
          CK(hipMemcpyAsync(dev + a, pin + a, l, hipMemcpyHostToDevice, st));
        }
        CK(hipStreamSynchronize(st));
      }));
  rep("hipHostRegister + D2H + unregister", med([&] {
        CK(hipHostRegister(host, bytes, hipHostRegisterDefault));
        CK(hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost));
        CK(hipHostUnregister(host));
      }));
  // a fresh destination (numpy's np.empty for a downloaded x): its pages are
  // faulted in, and zeroed by the kernel, during the copy. HUGE: madvised for
  // transparent huge pages, as numpy does for large arrays
  auto fresh = [&](bool huge, int touch, bool copy) {
    char *f = (char *)aligned_alloc(2 << 20, (bytes + (2 << 20) - 1) / (2 << 20) * (2 << 20));
    if (huge) madvise(f, bytes, MADV_HUGEPAGE);
    if (touch > 0) {
      std::vector<std::thread> th;
      const size_t pg = huge ? (2 << 20) : 4096;
      for (int t = 0; t < touch; ++t)
        th.emplace_back([=] {
          for (size_t o = (size_t)t * pg; o < bytes; o += (size_t)touch * pg) reinterpret_cast<volatile char *>(f)[o] = 0;
        });
      for (auto &x : th) x.join();
    }
    if (copy) CK(hipMemcpy(f, dev, bytes, hipMemcpyDeviceToHost));
    free(f);
  };
  rep("fresh 4K pages: alloc + free only", med([&] { fresh(false, 0, false); }));
  rep("fresh 4K pages: D2H", med([&] { fresh(false, 0, true); }));
  rep("fresh huge pages: alloc + free only", med([&] { fresh(true, 0, false); }));
  rep("fresh huge pages: D2H", med([&] { fresh(true, 0, true); }));
  rep("fresh huge pages: threads touch, no D2H", med([&] { fresh(true, nt, false); }));
  rep("fresh huge pages: threads touch + D2H", med([&] { fresh(true, nt, true); }));
  CK(hipHostFree(pin));
  CK(hipFree(dev));
  free(host);
  return 0;
}
