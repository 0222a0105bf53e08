// Host-side image builders and host-only plans (see host_image.hpp). Plain
// C++: the library links this translation unit, and `make sanitize` builds it
// alone with ASan + UBSan and with TSan (the builders run multi-threaded, and
// release_later frees staging memory on a detached thread).
#include "host_image.hpp"

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>

namespace kry {

static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }

// A staging vector's pages are returned on a detached thread once its H2D
// copies have completed (the caller has synchronised the stream): unmapping
// ~1 GB takes ~0.1 s that kry_csr_create then does not wait for.
template <class T>
void release_later(hvec<T> &v) {
  if (v.capacity() < (size_t(64) << 20) / sizeof(T)) {
    hvec<T>().swap(v);
    return;
  }
  auto *h = new hvec<T>();
  h->swap(v);
  std::thread([h] { delete h; }).detach();
}

template <class T>
static void par_fill(hvec<T> &v, size_t n, T val) {
  v.resize(n);
  const unsigned nt = n < (size_t(1) << 20) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (nt == 1) {
    std::fill(v.begin(), v.end(), val);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] { std::fill(v.data() + n * t / nt, v.data() + n * (t + 1) / nt, val); });
  for (auto &x : th) x.join();
}

template <typename I>
void check_csr(int64_t n, int64_t nnz, const I *ip, const I *ix) {
  KRY_REQUIRE(n >= 0 && nnz >= 0 && ip, KRY_EINVAL, "bad CSR arguments");
  KRY_REQUIRE(ip[0] == 0 && (int64_t)ip[n] == nnz, KRY_EINVAL, "indptr must start at 0 and end at nnz");
  KRY_REQUIRE(nnz == 0 || ix, KRY_EINVAL, "null indices");
  const unsigned nt = n + nnz < (int64_t(1) << 20) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::atomic<int> bad{0};  // 1: indptr decreases, 2: a column out of range
  auto work = [&](unsigned t) {
    const int64_t r0 = n * t / nt, r1 = n * (t + 1) / nt;
    for (int64_t r = r0; r < r1; ++r)
      if (ip[r + 1] < ip[r]) {
        bad = 1;
        return;
      }
    // the rows are monotone here; the entries of [r0, r1) are [ip[r0], ip[r1])
    const int64_t e0 = (int64_t)ip[r0], e1 = (int64_t)ip[r1];
    for (int64_t e = e0; e < e1; ++e)
      if (ix[e] < 0 || (int64_t)ix[e] >= n) {
        bad = 2;
        return;
      }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto &x : th) x.join();
  }
  KRY_REQUIRE(bad != 1, KRY_EINVAL, "indptr must be non-decreasing");
  KRY_REQUIRE(bad != 2, KRY_EINVAL, "column index out of range [0, n)");
}

// ---------------------------------------------------------- SELL-64 layout
// Host-side plan: slice s = rows [64 s, 64 s + 64); width = longest row;
// a slice is irregular (CSR walk) when 64 * width > 2 * nnz_slice + 1024.
template <typename I>
void sell_plan(int64_t n, const I *ip, std::vector<int64_t> *sptr, std::vector<int32_t> *width,
                      int64_t *nslices, int64_t *nslots, int64_t *nirr) {
  const int64_t ns = (n + kSlice - 1) / kSlice;
  if (sptr) sptr->assign(ns + 1, 0);
  if (width) width->assign(ns, 0);
  int64_t slots = 0, irr = 0;
  for (int64_t s = 0; s < ns; ++s) {
    const int64_t r0 = s * kSlice, r1 = std::min<int64_t>(n, r0 + kSlice);
    int64_t w = 0;
    for (int64_t r = r0; r < r1; ++r) w = std::max<int64_t>(w, (int64_t)ip[r + 1] - (int64_t)ip[r]);
    const int64_t snnz = (int64_t)ip[r1] - (int64_t)ip[r0];
    const bool irregular = kSlice * w > 2 * snnz + 1024 || w > (int64_t(1) << 30);
    if (irregular) ++irr;
    if (width) (*width)[s] = irregular ? -1 : (int32_t)w;
    if (!irregular) slots += kSlice * w;
    if (sptr) (*sptr)[s + 1] = slots;
  }
  *nslices = ns;
  *nslots = slots;
  *nirr = irr;
}

template <typename I, typename MV>
void sell_fill(int64_t n, const I *ip, const I *ix, const MV *dv, const std::vector<int64_t> &sptr,
                      const std::vector<int32_t> &width, hvec<I> &sidx, hvec<MV> &sval) {
  const int64_t ns = (int64_t)width.size();
  const int64_t slots = sptr[ns];
  par_fill(sidx, slots + 256, I(-1));
  par_fill(sval, slots + 256, MV(0));
  auto work = [&](int64_t sa, int64_t sb) {
    for (int64_t s = sa; s < sb; ++s) {
      if (width[s] < 0) continue;
      const int64_t base = sptr[s];
      const int64_t r0 = s * kSlice, r1 = std::min<int64_t>(n, r0 + kSlice);
      for (int64_t r = r0; r < r1; ++r) {
        const int64_t lane = r - r0;
        int64_t j = 0;
        for (int64_t e = ip[r]; e < ip[r + 1]; ++e, ++j) {
          sidx[base + j * kSlice + lane] = ix[e];
          sval[base + j * kSlice + lane] = dv[e];
        }
      }
    }
  };
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (ns < 4096) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(work, ns * t / nt, ns * (t + 1) / nt);
  for (auto &x : th) x.join();
}
// Compact column image: for every slot column (slice s, column j) the base is
// the smallest column index among its lanes and every lane stores col - base
// as uint16 (0xFFFF = padding). Possible when each slot column spans at most
// 65534 columns (banded and stencil matrices); the gathers then read 2 B of
// index per nonzero instead of 4. Returns false (nothing built) otherwise.
template <typename I>
bool compact_fill(const std::vector<int64_t> &sptr, const std::vector<int32_t> &width,
                         const hvec<I> &sidx, hvec<uint16_t> &sdelta, std::vector<int32_t> &scbase) {
  const int64_t ns = (int64_t)width.size();
  const int64_t slots = sptr[ns];
  par_fill(sdelta, slots + 256, (uint16_t)0xFFFF);
  scbase.assign(slots / kSlice + 16, 0);
  std::atomic<bool> ok{true};
  auto work = [&](int64_t sa, int64_t sb) {
    for (int64_t s = sa; s < sb && ok.load(std::memory_order_relaxed); ++s) {
      const int64_t base = sptr[s];
      for (int64_t j = 0; j < width[s]; ++j) {
        const I *c = sidx.data() + base + j * kSlice;
        int64_t mn = INT64_MAX, mx = -1;
        for (int l = 0; l < kSlice; ++l)
          if (c[l] >= 0) {
            mn = std::min<int64_t>(mn, c[l]);
            mx = std::max<int64_t>(mx, c[l]);
          }
        if (mx < 0) mn = 0;
        if (mx - mn > 65534 || mn > INT32_MAX) {
          ok = false;
          return;
        }
        scbase[base / kSlice + j] = (int32_t)mn;
        uint16_t *d = sdelta.data() + base + j * kSlice;
        for (int l = 0; l < kSlice; ++l)
          if (c[l] >= 0) d[l] = (uint16_t)(c[l] - mn);
      }
    }
  };
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (ns < 4096) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(work, ns * t / nt, ns * (t + 1) / nt);
  for (auto &x : th) x.join();
  return ok.load();
}

// Diagonal-offset image (see kry_csr::dia_*). Pass 1 collects every slice's
// sorted offset list (col - row over its entries) and checks that each row is
// strictly sorted, so a row's entries occur in the slot order of their
// offsets: the per-row summation order stays the stored order (bitwise
// csr_matvec). Pass 2 places entry (row, col) in the slot column of offset
// col - row and sets the row's mask bit. Returns false (nothing built) for
// unsorted or duplicate entries, or when the image would hold more than
// 1.25x the SELL image's slots (offsets not shared across the slice's rows).

template <typename I, typename MV>
bool dia_build(int64_t n, const I *ip, const I *ix, const MV *dv, int64_t sell_slots, DiaHost<MV> &d) {
  if (sizeof(I) != 4 || n == 0) return false;
  constexpr int H = kDiaSlice;
  const int64_t ns = (n + H - 1) / H;
  std::vector<std::vector<int32_t>> offs(ns);
  std::atomic<bool> ok{true};
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (ns < 2048) nt = 1;
  auto pass1 = [&](int64_t sa, int64_t sb) {
    std::vector<int32_t> o;
    for (int64_t s = sa; s < sb && ok.load(std::memory_order_relaxed); ++s) {
      const int64_t r0 = s * H, r1 = std::min<int64_t>(n, r0 + H);
      o.clear();
      for (int64_t r = r0; r < r1; ++r) {
        // a row whose offsets repeat the previous row's adds nothing new to
        // the list (stencil rows, away from the grid's faces): checked
        // against it entry by entry, not pushed
        const int64_t len = (int64_t)ip[r + 1] - (int64_t)ip[r];
        bool same = r > r0 && len == (int64_t)ip[r] - (int64_t)ip[r - 1];
        for (int64_t e = ip[r]; e < ip[r + 1]; ++e) {
          if (e > ip[r] && ix[e] <= ix[e - 1]) {  // unsorted or duplicate: stored order is not offset order
            ok = false;
            return;
          }
          same = same && (int64_t)ix[e] - r == (int64_t)ix[e - len] - (r - 1);
        }
        if (!same)
          for (int64_t e = ip[r]; e < ip[r + 1]; ++e) o.push_back((int32_t)((int64_t)ix[e] - r));
      }
      std::sort(o.begin(), o.end());
      o.erase(std::unique(o.begin(), o.end()), o.end());
      if ((int64_t)o.size() * H > 2 * ((int64_t)ip[r1] - (int64_t)ip[r0]) + 2048) {
        ok = false;  // offsets not shared across the slice's rows
        return;
      }
      offs[s] = o;
    }
  };
  {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back(pass1, ns * t / nt, ns * (t + 1) / nt);
    for (auto &x : th) x.join();
  }
  if (!ok) return false;
  d.sptr.assign(ns + 1, 0);
  d.width.assign(ns, 0);
  for (int64_t s = 0; s < ns; ++s) {
    d.width[s] = (int32_t)offs[s].size();
    d.max_width = std::max(d.max_width, d.width[s]);
    d.sptr[s + 1] = d.sptr[s] + (int64_t)H * d.width[s];
  }
  const int64_t slots = d.sptr[ns];
  // the 128-row slices may hold up to one slice more padding than SELL-64's
  if (slots * 4 > sell_slots * 5 + (int64_t)4 * H * d.max_width) return false;
  const int64_t cols = slots / H;
  d.off.assign(cols + kDiaPad, 0);
  par_fill(d.mask, 2 * (cols + kDiaPad), (uint64_t)0);
  par_fill(d.val, slots + 2 * H, MV(0));
  auto pass2 = [&](int64_t sa, int64_t sb) {
    for (int64_t s = sa; s < sb; ++s) {
      const std::vector<int32_t> &o = offs[s];
      const int64_t base = d.sptr[s], c0 = base / H;
      for (size_t j = 0; j < o.size(); ++j) d.off[c0 + j] = o[j];
      const int64_t r0 = s * H, r1 = std::min<int64_t>(n, r0 + H);
      for (int64_t r = r0; r < r1; ++r) {
        const int rl = (int)(r - r0);
        size_t j = 0;
        for (int64_t e = ip[r]; e < ip[r + 1]; ++e) {
          const int32_t off = (int32_t)((int64_t)ix[e] - r);
          while (o[j] != off) ++j;  // the row's offsets ascend, as the list's do
          d.mask[2 * (c0 + j) + (rl & 1)] |= uint64_t(1) << (rl >> 1);
          d.val[base + (int64_t)j * H + rl] = dv[e];
          ++j;
        }
      }
    }
  };
  {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back(pass2, ns * t / nt, ns * (t + 1) / nt);
    for (auto &x : th) x.join();
  }
  return true;
}


// ------------------------------------------- bandwidth-reducing renumbering
// A fork-join team for the level-synchronous passes: up to 16 threads that
// live for one rcm_order call and meet at a spin barrier per level (a few
// microseconds; a thread start per level would cost ~50 us each).
namespace {
struct Team {
  unsigned nt;
  std::vector<std::thread> th;
  std::atomic<unsigned> gen{0}, left{0};
  std::atomic<bool> quit{false};
  std::function<void(unsigned)> job;
  explicit Team(unsigned want) : nt(std::max(1u, want)) {
    for (unsigned t = 1; t < nt; ++t)
      th.emplace_back([this, t] {
        unsigned seen = 0;
        for (;;) {
          unsigned g;
          while ((g = gen.load(std::memory_order_acquire)) == seen) {
            if (quit.load(std::memory_order_acquire)) return;
            std::this_thread::yield();
          }
          seen = g;
          job(t);
          left.fetch_sub(1, std::memory_order_acq_rel);
        }
      });
  }
  void run(const std::function<void(unsigned)> &f) {
    if (nt == 1) {
      f(0);
      return;
    }
    job = f;
    left.store(nt - 1, std::memory_order_release);
    gen.fetch_add(1, std::memory_order_acq_rel);
    f(0);
    while (left.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }
  ~Team() {
    quit.store(true, std::memory_order_release);
    for (auto &x : th) x.join();
  }
};

// One BFS level step: level[] of the frontier's unvisited neighbours set to
// `next` (compare-and-swap: one owner each); returns them, in thread order.
template <typename I>
void bfs_expand(Team &tm, const I *ip, const I *ix, const int32_t *front, int64_t nf, int32_t next,
                std::atomic<int32_t> *level, std::vector<std::vector<int32_t>> &loc, std::vector<int32_t> &out) {
  tm.run([&](unsigned t) {
    auto &v = loc[t];
    v.clear();
    const int64_t a = nf * t / tm.nt, b = nf * (t + 1) / tm.nt;
    for (int64_t q = a; q < b; ++q) {
      const int32_t u = front[q];
      for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
        const int32_t w = (int32_t)ix[e];
        int32_t expect = -1;
        if (level[w].load(std::memory_order_relaxed) == -1 &&
            level[w].compare_exchange_strong(expect, next, std::memory_order_relaxed))
          v.push_back(w);
      }
    }
  });
  out.clear();
  for (auto &v : loc) out.insert(out.end(), v.begin(), v.end());
}
}  // namespace

template <typename I>
bool scattered(int64_t n, const I *ip, const I *ix) {
  if (n * 8 < (int64_t(8) << 20)) return false;
  const int64_t nnz = (int64_t)ip[n];
  if (nnz == 0) return false;
  const int64_t cols = std::max<int64_t>(int64_t(1) << 18, (n + 15) / 16);
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<int64_t> far(nt, 0);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      const int64_t r0 = n * t / nt, r1 = n * (t + 1) / nt;
      int64_t f = 0;
      for (int64_t r = r0; r < r1; ++r)
        for (int64_t e = ip[r]; e < ip[r + 1]; ++e) {
          const int64_t d = (int64_t)ix[e] - r;
          f += (d > cols / 2 || d < -cols / 2);
        }
      far[t] = f;
    });
  for (auto &x : th) x.join();
  int64_t nfar = 0;
  for (int64_t f : far) nfar += f;
  return nfar * 4 >= nnz;
}

template <typename I>
bool rcm_order(int64_t n, const I *ip, const I *ix, int64_t wlimit, std::vector<int32_t> &perm, int64_t *levels) {
  if (n <= 0 || n >= (int64_t(1) << 31) - 1) return false;
  const unsigned nt = n < (int64_t(1) << 16) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  Team tm(nt);
  std::vector<std::vector<int32_t>> loc(nt);
  std::unique_ptr<std::atomic<int32_t>[]> level(new std::atomic<int32_t>[n]);
  auto deg = [&](int64_t v) { return (int64_t)ip[v + 1] - (int64_t)ip[v]; };
  auto clear_levels = [&] {
    tm.run([&](unsigned t) {
      for (int64_t v = n * t / tm.nt; v < n * (t + 1) / tm.nt; ++v) level[v].store(-1, std::memory_order_relaxed);
    });
  };
  // levels-only BFS from `root`: the level count, and the last level's
  // smallest-degree (lowest-index) node; -1 if a level exceeds wlimit
  std::vector<int32_t> front, next;
  auto sweep = [&](int32_t root, int32_t *far_node) -> int64_t {
    clear_levels();
    level[root].store(0, std::memory_order_relaxed);
    front.assign(1, root);
    int64_t nl = 1;
    for (;;) {
      bfs_expand(tm, ip, ix, front.data(), (int64_t)front.size(), (int32_t)nl, level.get(), loc, next);
      if (next.empty()) break;
      if ((int64_t)next.size() > wlimit) return -1;
      front.swap(next);
      ++nl;
    }
    int32_t best = front[0];
    for (int32_t v : front)
      if (deg(v) < deg(best) || (deg(v) == deg(best) && v < best)) best = v;
    *far_node = best;
    return nl;
  };
  int32_t root = 0;
  for (int64_t v = 1; v < n; ++v)
    if (deg(v) < deg(root)) root = (int32_t)v;
  int32_t cand = root;
  int64_t ecc = sweep(root, &cand);
  if (ecc < 0) return false;
  static const int max_sweeps = [] {  // tuning override: George-Liu sweeps after the first BFS
    const char *e = getenv("KRY_RCM_SWEEPS");
    return e ? std::max(0, atoi(e)) : 3;
  }();
  for (int it = 0; it < max_sweeps && cand != root; ++it) {
    int32_t c2 = cand;
    const int64_t e2 = sweep(cand, &c2);
    if (e2 < 0) return false;
    if (e2 <= ecc) break;
    root = cand;
    ecc = e2;
    cand = c2;
  }
  // Cuthill-McKee numbering, level by level
  clear_levels();
  std::vector<int32_t> cm;
  cm.reserve(n);
  std::vector<int32_t> key(n, INT32_MAX);  // smallest parent number, written under the per-level owner rule below
  std::unique_ptr<std::atomic<int32_t>[]> akey(new std::atomic<int32_t>[n]);
  tm.run([&](unsigned t) {
    for (int64_t v = n * t / tm.nt; v < n * (t + 1) / tm.nt; ++v) akey[v].store(INT32_MAX, std::memory_order_relaxed);
  });
  int64_t scan = 0;  // lowest index that may still be unnumbered (new components)
  int64_t nlev = 0;
  std::vector<int64_t> cnt;
  while ((int64_t)cm.size() < n) {
    if (cm.empty()) {
      level[root].store(0, std::memory_order_relaxed);
      cm.push_back(root);
    } else {
      while (level[scan].load(std::memory_order_relaxed) != -1) ++scan;
      level[scan].store(0, std::memory_order_relaxed);
      cm.push_back((int32_t)scan);
    }
    int64_t a = (int64_t)cm.size() - 1, b = (int64_t)cm.size();  // the current level: numbers [a, b)
    ++nlev;
    for (;;) {
      // children of the level: claim (level = 1) and the smallest parent number
      tm.run([&](unsigned t) {
        auto &v = loc[t];
        v.clear();
        const int64_t qa = a + (b - a) * t / tm.nt, qb = a + (b - a) * (t + 1) / tm.nt;
        for (int64_t q = qa; q < qb; ++q) {
          const int32_t u = cm[q];
          for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
            const int32_t w = (int32_t)ix[e];
            int32_t expect = -1;
            if (level[w].load(std::memory_order_relaxed) == -1 &&
                level[w].compare_exchange_strong(expect, 1, std::memory_order_relaxed))
              v.push_back(w);
            if (level[w].load(std::memory_order_relaxed) == 1) {
              int32_t k = akey[w].load(std::memory_order_relaxed);
              while ((int32_t)q < k && !akey[w].compare_exchange_weak(k, (int32_t)q, std::memory_order_relaxed)) {
              }
            }
          }
        }
      });
      next.clear();
      for (auto &v : loc) next.insert(next.end(), v.begin(), v.end());
      if (next.empty()) break;
      if ((int64_t)next.size() > wlimit) return false;
      // counting sort by parent number, then (degree, index) within a parent
      const int64_t span = b - a;
      cnt.assign(span + 1, 0);
      for (int32_t w : next) cnt[akey[w].load(std::memory_order_relaxed) - a + 1]++;
      for (int64_t i = 0; i < span; ++i) cnt[i + 1] += cnt[i];
      front.resize(next.size());
      for (int32_t w : next) front[cnt[akey[w].load(std::memory_order_relaxed) - a]++] = w;
      int64_t i0 = 0;
      while (i0 < (int64_t)front.size()) {
        const int32_t k0 = akey[front[i0]].load(std::memory_order_relaxed);
        int64_t i1 = i0 + 1;
        while (i1 < (int64_t)front.size() && akey[front[i1]].load(std::memory_order_relaxed) == k0) ++i1;
        std::sort(front.begin() + i0, front.begin() + i1, [&](int32_t x, int32_t y) {
          return deg(x) != deg(y) ? deg(x) < deg(y) : x < y;
        });
        i0 = i1;
      }
      for (int32_t w : front) level[w].store(2, std::memory_order_relaxed);  // numbered
      a = (int64_t)cm.size();
      cm.insert(cm.end(), front.begin(), front.end());
      b = (int64_t)cm.size();
      ++nlev;
    }
  }
  (void)key;
  perm.resize(n);
  for (int64_t r = 0; r < n; ++r) perm[r] = cm[n - 1 - r];
  if (levels) *levels = nlev;
  return true;
}

template <typename I, typename MV>
void renumber_csr(int64_t n, const I *ip, const I *ix, const MV *dv, const std::vector<int32_t> &perm,
                  hvec<I> &ip2, hvec<I> &ix2, hvec<MV> &dv2) {
  std::vector<int32_t> iperm(n);
  for (int64_t r = 0; r < n; ++r) iperm[perm[r]] = (int32_t)r;
  ip2.resize(n + 1);
  ip2[0] = 0;
  for (int64_t r = 0; r < n; ++r) ip2[r + 1] = ip2[r] + (ip[perm[r] + 1] - ip[perm[r]]);
  const int64_t nnz = (int64_t)ip[n];
  ix2.resize(nnz + 1);
  dv2.resize(nnz + 1);
  const unsigned nt = n < (int64_t(1) << 16) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int64_t r = n * t / nt; r < n * (t + 1) / nt; ++r) {
        const int64_t o = perm[r];
        int64_t q = (int64_t)ip2[r];
        for (int64_t e = ip[o]; e < ip[o + 1]; ++e, ++q) {
          ix2[q] = (I)iperm[ix[e]];
          dv2[q] = dv[e];
        }
      }
    });
  for (auto &x : th) x.join();
}

template <typename I, typename MV>
bool rs_build(int64_t n, const I *ip, const I *ix, const MV *dv, int64_t sell_slots, RsHost<MV> &p) {
  constexpr int H = kPairSlice;
  if (n == 0 || n >= (int64_t(1) << 28) - 1) return false;
  const int64_t ns = (n + H - 1) / H;
  p.width.assign(ns, 0);
  p.sptr.assign(ns + 1, 0);
  for (int64_t s = 0; s < ns; ++s) {
    int64_t w = 0;
    for (int64_t r = s * H; r < std::min<int64_t>(n, (s + 1) * H); ++r) w = std::max<int64_t>(w, ip[r + 1] - ip[r]);
    if (w > INT32_MAX / H) return false;
    p.width[s] = (int32_t)w;
    p.max_width = std::max(p.max_width, (int)w);
    p.sptr[s + 1] = p.sptr[s] + H * w;
  }
  const int64_t slots = p.sptr[ns];
  if (slots == 0 || slots * 4 > sell_slots * 5 + (int64_t)4 * H * p.max_width) return false;
  par_fill(p.colrank, slots + 2 * H, 0xFFFFFFFFu);
  par_fill(p.val, slots + 2 * H, MV(0));
  auto fill = [&](int64_t sa, int64_t sb) {
    std::vector<std::pair<int64_t, int>> run;  // (column, position in run)
    for (int64_t s = sa; s < sb; ++s) {
      const int64_t r0 = s * H, r1 = std::min<int64_t>(n, r0 + H), base = p.sptr[s];
      for (int64_t r = r0; r < r1; ++r) {
        const int64_t e0 = (int64_t)ip[r], len = (int64_t)ip[r + 1] - e0;
        for (int64_t c0 = 0; c0 < len; c0 += kRsChunk) {
          const int m = (int)std::min<int64_t>(kRsChunk, len - c0);
          run.clear();
          for (int k = 0; k < m; ++k) run.emplace_back((int64_t)ix[e0 + c0 + k], k);
          std::stable_sort(run.begin(), run.end(),
                           [](const std::pair<int64_t, int> &x, const std::pair<int64_t, int> &y) { return x.first < y.first; });
          for (int j = 0; j < m; ++j) {
            const int64_t q = base + (c0 + j) * H + (r - r0);
            p.colrank[q] = (uint32_t)run[j].first | ((uint32_t)run[j].second << 28);
            p.val[q] = dv[e0 + c0 + run[j].second];
          }
        }
      }
    }
  };
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (ns < 2048) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(fill, ns * t / nt, ns * (t + 1) / nt);
  for (auto &x : th) x.join();
  return true;
}

// Host-only view of the diagonal-offset plan (kry_dia_plan): the image
// kry_csr_create would build for these CSR arrays, without a device.
template <typename I>
static void dia_plan_host(int64_t n, int64_t nnz, const I *ip, const I *ix, int64_t *info, int32_t *widths,
                          int32_t *offsets, uint64_t *masks) {
  check_csr(n, nnz, ip, ix);
  int64_t ns = 0, sell_slots = 0, irr = 0;
  sell_plan(n, ip, nullptr, nullptr, &ns, &sell_slots, &irr);
  hvec<double> zeros;
  par_fill(zeros, (size_t)std::max<int64_t>(nnz, 1), 0.0);
  DiaHost<double> d;
  const bool built = dia_build(n, ip, ix, zeros.data(), sell_slots, d);
  info[0] = built ? 1 : 0;
  info[1] = built ? (int64_t)d.width.size() : 0;
  info[2] = built ? d.sptr.back() : 0;
  info[3] = built ? d.max_width : 0;
  if (!built) return;
  if (widths) std::copy(d.width.begin(), d.width.end(), widths);
  const int64_t cols = d.sptr.back() / kDiaSlice;
  if (offsets) std::copy(d.off.begin(), d.off.begin() + cols, offsets);
  if (masks) std::copy(d.mask.begin(), d.mask.begin() + 2 * cols, masks);
}

// Column-blocked image (see kry_csr::cb_*). Returns false when not useful or
// not possible: rows not sorted, x small enough to stay cache-resident, the
// columns not scattered (most entries within half a block of the diagonal),
// or a segment too long for uint16 offsets.

template <typename I, typename MV>
bool cb_build(int64_t n, const I *ip, const I *ix, const MV *dv, CbHost<MV> &cb) {
  if (sizeof(I) != 4 || n * 8 < (int64_t(8) << 20)) return false;
  const int64_t nnz = (int64_t)ip[n];
  const char *cenv = getenv("KRY_CB_COLS");  // tuning override: columns per block
  int64_t cols = cenv ? std::max<int64_t>(1024, atoll(cenv)) : std::max<int64_t>(int64_t(1) << 18, (n + 15) / 16);
  const int64_t nb = (n + cols - 1) / cols;
  if (nb < 2) return false;
  // sorted rows and scattered columns
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<int64_t> far(nt, 0);
  std::atomic<bool> sorted{true};
  {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        const int64_t r0 = n * t / nt, r1 = n * (t + 1) / nt;
        int64_t f = 0;
        for (int64_t r = r0; r < r1; ++r)
          for (int64_t e = ip[r]; e < ip[r + 1]; ++e) {
            if (e > ip[r] && ix[e] < ix[e - 1]) sorted = false;
            const int64_t d = (int64_t)ix[e] - r;
            f += (d > cols / 2 || d < -cols / 2);
          }
        far[t] = f;
      });
    for (auto &x : th) x.join();
  }
  int64_t nfar = 0;
  for (int64_t f : far) nfar += f;
  if (!sorted || nnz == 0 || nfar * 4 < nnz) return false;
  const int64_t ng = (n + kCbRows - 1) / kCbRows;
  // the SpMV takes one launch per 16,384 groups (1024 blocks x 16 owned
  // groups) with 1024 block partials each, at most kMaxGridBlk = 32768 rows
  if (ng > 32 * 16384) return false;
  // per (block, row) counts -> per (block, group) segment lengths
  hvec<uint16_t> roff;
  par_fill(roff, nb * n + 256, (uint16_t)0);
  std::vector<int64_t> seg(nb * ng, 0);
  std::atomic<bool> fits{true};
  auto pass1 = [&](int64_t g0, int64_t g1) {
    std::vector<int64_t> cnt(nb);
    for (int64_t g = g0; g < g1; ++g) {
      std::fill(cnt.begin(), cnt.end(), 0);
      const int64_t r0 = g * kCbRows, r1 = std::min<int64_t>(n, r0 + kCbRows);
      for (int64_t r = r0; r < r1; ++r) {
        for (int64_t b = 0; b < nb; ++b) {
          if (cnt[b] > 65535) fits = false;
          roff[b * n + r] = (uint16_t)cnt[b];
        }
        for (int64_t e = ip[r]; e < ip[r + 1]; ++e) cnt[ix[e] / cols]++;
      }
      for (int64_t b = 0; b < nb; ++b) {
        if (cnt[b] > 65535) fits = false;
        seg[b * ng + g] = cnt[b];
      }
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(pass1, ng * t / nt, ng * (t + 1) / nt);
  for (auto &x : th) x.join();
  th.clear();
  if (!fits) return false;
  cb.gptr.assign(nb * ng + 1, 0);
  for (int64_t i = 0; i < nb * ng; ++i) cb.gptr[i + 1] = cb.gptr[i] + seg[i];
  par_fill(cb.col, nnz + 256, (int32_t)0);
  par_fill(cb.val, nnz + 256, MV(0));
  auto pass2 = [&](int64_t g0, int64_t g1) {
    std::vector<int64_t> pos(nb);
    for (int64_t g = g0; g < g1; ++g) {
      for (int64_t b = 0; b < nb; ++b) pos[b] = cb.gptr[b * ng + g];
      const int64_t r0 = g * kCbRows, r1 = std::min<int64_t>(n, r0 + kCbRows);
      for (int64_t r = r0; r < r1; ++r)
        for (int64_t e = ip[r]; e < ip[r + 1]; ++e) {
          const int64_t p = pos[ix[e] / cols]++;
          cb.col[p] = (int32_t)ix[e];
          cb.val[p] = dv[e];
        }
    }
  };
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(pass2, ng * t / nt, ng * (t + 1) / nt);
  for (auto &x : th) x.join();
  cb.nb = nb;
  cb.cols = cols;
  cb.ng = ng;
  cb.roff = std::move(roff);
  return true;
}

// Paired-row SELL-128 image (see kry_csr::sp_*). Pass 1: slice widths (the
// longest row of each 128 rows); pass 2: per slot column the smallest column
// as base and every entry's delta and value at row position r - 128 s.
// Returns false (nothing built) when a slot column spans more than 65534
// columns, a column does not fit int32, or the image would hold more than
// 1.25x the SELL-64 image's slots (very uneven rows).

template <typename I, typename MV>
bool pair_build(int64_t n, const I *ip, const I *ix, const MV *dv, int64_t sell_slots, PairHost<MV> &p) {
  constexpr int H = kPairSlice;
  if (n == 0 || n >= (int64_t(1) << 31)) return false;
  const int64_t ns = (n + H - 1) / H;
  p.width.assign(ns, 0);
  p.sptr.assign(ns + 1, 0);
  for (int64_t s = 0; s < ns; ++s) {
    int64_t w = 0;
    for (int64_t r = s * H; r < std::min<int64_t>(n, (s + 1) * H); ++r) w = std::max<int64_t>(w, ip[r + 1] - ip[r]);
    if (w > INT32_MAX / H) return false;
    p.width[s] = (int32_t)w;
    p.max_width = std::max(p.max_width, (int)w);
    p.sptr[s + 1] = p.sptr[s] + H * w;
  }
  const int64_t slots = p.sptr[ns];
  if (slots == 0 || slots * 4 > sell_slots * 5 + (int64_t)4 * H * p.max_width) return false;
  p.cbase.assign(slots / H + kDiaPad, 0);
  par_fill(p.delta, slots + 2 * H, (uint16_t)0xFFFF);
  par_fill(p.val, slots + 2 * H, MV(0));
  std::atomic<bool> ok{true};
  auto fill = [&](int64_t sa, int64_t sb) {
    for (int64_t s = sa; s < sb && ok.load(std::memory_order_relaxed); ++s) {
      const int64_t r0 = s * H, r1 = std::min<int64_t>(n, r0 + H), base = p.sptr[s];
      for (int64_t j = 0; j < p.width[s]; ++j) {
        int64_t mn = INT64_MAX, mx = -1;
        for (int64_t r = r0; r < r1; ++r)
          if ((int64_t)ip[r] + j < (int64_t)ip[r + 1]) {
            const int64_t c = (int64_t)ix[ip[r] + j];
            mn = std::min(mn, c);
            mx = std::max(mx, c);
          }
        if (mx < 0) mn = 0;
        if (mx - mn > 65534 || mn > INT32_MAX) {
          ok = false;
          return;
        }
        p.cbase[base / H + j] = (int32_t)mn;
        for (int64_t r = r0; r < r1; ++r)
          if ((int64_t)ip[r] + j < (int64_t)ip[r + 1]) {
            const int64_t q = base + j * H + (r - r0);
            p.delta[q] = (uint16_t)((int64_t)ix[ip[r] + j] - mn);
            p.val[q] = dv[ip[r] + j];
          }
      }
    }
  };
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (ns < 2048) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(fill, ns * t / nt, ns * (t + 1) / nt);
  for (auto &x : th) x.join();
  return ok.load();
}

// Host-only view of the paired-row plan (kry_pair_plan): the image
// kry_csr_create would build for these CSR arrays when neither the DIA nor the
// column-blocked image is built, without a device.
template <typename I>
static void pair_plan_host(int64_t n, int64_t nnz, const I *ip, const I *ix, int64_t *info, int32_t *widths,
                           int32_t *cbase, uint16_t *deltas) {
  check_csr(n, nnz, ip, ix);
  int64_t ns = 0, sell_slots = 0, irr = 0;
  sell_plan(n, ip, nullptr, nullptr, &ns, &sell_slots, &irr);
  hvec<double> zeros;
  par_fill(zeros, (size_t)std::max<int64_t>(nnz, 1), 0.0);
  PairHost<double> p;
  const bool built = pair_build(n, ip, ix, zeros.data(), sell_slots, p);
  info[0] = built ? 1 : 0;
  info[1] = built ? (int64_t)p.width.size() : 0;
  info[2] = built ? p.sptr.back() : 0;
  info[3] = built ? p.max_width : 0;
  if (!built) return;
  if (widths) std::copy(p.width.begin(), p.width.end(), widths);
  const int64_t slots = p.sptr.back();
  if (cbase) std::copy(p.cbase.begin(), p.cbase.begin() + slots / kPairSlice, cbase);
  if (deltas) std::copy(p.delta.begin(), p.delta.begin() + slots, deltas);
}


// Host-only view of the column-blocked plan (kry_cb_plan): the image
// kry_csr_create would build for these CSR arrays when the diagonal-offset
// image is not, without a device.
template <typename I>
static void cb_plan_host(int64_t n, int64_t nnz, const I *ip, const I *ix, int64_t *info, int64_t *gptr) {
  check_csr(n, nnz, ip, ix);
  hvec<double> vals;
  par_fill(vals, (size_t)std::max<int64_t>(nnz, 1), 1.0);
  CbHost<double> cb;
  const bool built = cb_build(n, ip, ix, vals.data(), cb);
  info[0] = built ? 1 : 0;
  info[1] = built ? cb.nb : 0;
  info[2] = built ? cb.cols : 0;
  info[3] = built ? cb.ng : 0;
  if (built && gptr) std::copy(cb.gptr.begin(), cb.gptr.end(), gptr);
  release_later(cb.val);
  release_later(cb.col);
  release_later(cb.roff);
  release_later(vals);
}

// explicit instantiations: the combinations kry_csr_create dispatches
#define KRY_HOST_I(I)                                                                                              \
  template void check_csr<I>(int64_t, int64_t, const I *, const I *);                                            \
  template bool scattered<I>(int64_t, const I *, const I *);                                                     \
  template bool rcm_order<I>(int64_t, const I *, const I *, int64_t, std::vector<int32_t> &, int64_t *);          \
  template void sell_plan<I>(int64_t, const I *, std::vector<int64_t> *, std::vector<int32_t> *, int64_t *,     \
                             int64_t *, int64_t *);                                                              \
  template bool compact_fill<I>(const std::vector<int64_t> &, const std::vector<int32_t> &, const hvec<I> &,     \
                                hvec<uint16_t> &, std::vector<int32_t> &);
#define KRY_HOST_IM(I, MV)                                                                                         \
  template void sell_fill<I, MV>(int64_t, const I *, const I *, const MV *, const std::vector<int64_t> &,       \
                                 const std::vector<int32_t> &, hvec<I> &, hvec<MV> &);                          \
  template bool dia_build<I, MV>(int64_t, const I *, const I *, const MV *, int64_t, DiaHost<MV> &);            \
  template bool cb_build<I, MV>(int64_t, const I *, const I *, const MV *, CbHost<MV> &);                       \
  template bool pair_build<I, MV>(int64_t, const I *, const I *, const MV *, int64_t, PairHost<MV> &);          \
  template void renumber_csr<I, MV>(int64_t, const I *, const I *, const MV *, const std::vector<int32_t> &,    \
                                    hvec<I> &, hvec<I> &, hvec<MV> &);                                          \
  template bool rs_build<I, MV>(int64_t, const I *, const I *, const MV *, int64_t, RsHost<MV> &);
KRY_HOST_I(int32_t)
KRY_HOST_I(int64_t)
KRY_HOST_IM(int32_t, float)
KRY_HOST_IM(int32_t, double)
KRY_HOST_IM(int64_t, float)
KRY_HOST_IM(int64_t, double)
template void release_later<int32_t>(hvec<int32_t> &);
template void release_later<int64_t>(hvec<int64_t> &);
template void release_later<float>(hvec<float> &);
template void release_later<double>(hvec<double> &);
template void release_later<uint16_t>(hvec<uint16_t> &);
template void release_later<uint64_t>(hvec<uint64_t> &);
template void release_later<uint32_t>(hvec<uint32_t> &);

}  // namespace kry

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

template <typename I>
static void rs_plan_host(int64_t n, int64_t nnz, const I *ip, const I *ix, int64_t *info, int32_t *widths,
                         uint32_t *colrank) {
  check_csr(n, nnz, ip, ix);
  int64_t ns = 0, sell_slots = 0, irr = 0;
  sell_plan(n, ip, nullptr, nullptr, &ns, &sell_slots, &irr);
  hvec<double> zeros;
  par_fill(zeros, (size_t)std::max<int64_t>(nnz, 1), 0.0);
  RsHost<double> r;
  const bool built = rs_build(n, ip, ix, zeros.data(), sell_slots, r);
  info[0] = built ? 1 : 0;
  info[1] = built ? (int64_t)r.width.size() : 0;
  info[2] = built ? r.sptr.back() : 0;
  info[3] = built ? r.max_width : 0;
  if (!built) return;
  if (widths) std::copy(r.width.begin(), r.width.end(), widths);
  if (colrank) std::copy(r.colrank.begin(), r.colrank.begin() + r.sptr.back(), colrank);
}

extern "C" {

const char *kry_last_error(void) { return kry::g_last_error.c_str(); }

int kry_csr_layout(int64_t n, const void *indptr, int itype, int64_t *nslices, int64_t *nslots,
                   int64_t *nirregular) {
  KRY_API_BEGIN
  KRY_REQUIRE(indptr && nslices && nslots && nirregular && n >= 0, KRY_EINVAL, "bad layout arguments");
  if (itype == KRY_I32)
    sell_plan(n, static_cast<const int32_t *>(indptr), nullptr, nullptr, nslices, nslots, nirregular);
  else if (itype == KRY_I64)
    sell_plan(n, static_cast<const int64_t *>(indptr), nullptr, nullptr, nslices, nslots, nirregular);
  else
    throw Error{KRY_EINVAL, "bad itype"};
  KRY_API_END
}

int kry_dia_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t *info,
                 int32_t *widths, int32_t *offsets, uint64_t *masks) {
  KRY_API_BEGIN
  KRY_REQUIRE(indptr && info && n >= 0 && nnz >= 0 && (nnz == 0 || indices), KRY_EINVAL, "bad plan arguments");
  if (itype == KRY_I32)
    dia_plan_host(n, nnz, static_cast<const int32_t *>(indptr), static_cast<const int32_t *>(indices), info, widths,
                  offsets, masks);
  else if (itype == KRY_I64)
    dia_plan_host(n, nnz, static_cast<const int64_t *>(indptr), static_cast<const int64_t *>(indices), info, widths,
                  offsets, masks);
  else
    throw Error{KRY_EINVAL, "bad itype"};
  KRY_API_END
}

int kry_pair_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t *info,
                  int32_t *widths, int32_t *cbase, uint16_t *deltas) {
  KRY_API_BEGIN
  KRY_REQUIRE(indptr && info && n >= 0 && nnz >= 0 && (nnz == 0 || indices), KRY_EINVAL, "bad plan arguments");
  if (itype == KRY_I32)
    pair_plan_host(n, nnz, static_cast<const int32_t *>(indptr), static_cast<const int32_t *>(indices), info, widths,
                   cbase, deltas);
  else if (itype == KRY_I64)
    pair_plan_host(n, nnz, static_cast<const int64_t *>(indptr), static_cast<const int64_t *>(indices), info, widths,
                   cbase, deltas);
  else
    throw Error{KRY_EINVAL, "bad itype"};
  KRY_API_END
}

int kry_cb_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t *info,
                int64_t *gptr) {
  KRY_API_BEGIN
  KRY_REQUIRE(indptr && info && n >= 0 && nnz >= 0 && (nnz == 0 || indices), KRY_EINVAL, "bad plan arguments");
  if (itype == KRY_I32)
    cb_plan_host(n, nnz, static_cast<const int32_t *>(indptr), static_cast<const int32_t *>(indices), info, gptr);
  else if (itype == KRY_I64)
    cb_plan_host(n, nnz, static_cast<const int64_t *>(indptr), static_cast<const int64_t *>(indices), info, gptr);
  else
    throw Error{KRY_EINVAL, "bad itype"};
  KRY_API_END
}

int kry_rcm_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t wlimit,
                 int64_t *info, int32_t *perm) {
  KRY_API_BEGIN
  KRY_REQUIRE(indptr && info && n >= 0 && nnz >= 0 && (nnz == 0 || indices), KRY_EINVAL, "bad plan arguments");
  const int64_t wl = wlimit > 0 ? wlimit : std::max<int64_t>(int64_t(1) << 16, n / 32);
  std::vector<int32_t> p;
  int64_t levels = 0;
  bool built = false;
  if (itype == KRY_I32) {
    check_csr(n, nnz, static_cast<const int32_t *>(indptr), static_cast<const int32_t *>(indices));
    built = rcm_order(n, static_cast<const int32_t *>(indptr), static_cast<const int32_t *>(indices), wl, p, &levels);
  } else if (itype == KRY_I64) {
    check_csr(n, nnz, static_cast<const int64_t *>(indptr), static_cast<const int64_t *>(indices));
    built = rcm_order(n, static_cast<const int64_t *>(indptr), static_cast<const int64_t *>(indices), wl, p, &levels);
  } else {
    throw Error{KRY_EINVAL, "bad itype"};
  }
  info[0] = built ? 1 : 0;
  info[1] = built ? levels : 0;
  if (built && perm) std::copy(p.begin(), p.end(), perm);
  KRY_API_END
}

int kry_rs_plan(int64_t n, int64_t nnz, const void *indptr, const void *indices, int itype, int64_t *info,
                int32_t *widths, uint32_t *colrank) {
  KRY_API_BEGIN
  KRY_REQUIRE(indptr && info && n >= 0 && nnz >= 0 && (nnz == 0 || indices), KRY_EINVAL, "bad plan arguments");
  if (itype == KRY_I32)
    rs_plan_host(n, nnz, static_cast<const int32_t *>(indptr), static_cast<const int32_t *>(indices), info, widths,
                 colrank);
  else if (itype == KRY_I64)
    rs_plan_host(n, nnz, static_cast<const int64_t *>(indptr), static_cast<const int64_t *>(indices), info, widths,
                 colrank);
  else
    throw Error{KRY_EINVAL, "bad itype"};
  KRY_API_END
}

}  // extern "C"
