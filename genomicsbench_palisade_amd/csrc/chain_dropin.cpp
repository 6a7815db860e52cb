// chain_dropin.cpp -- host_chain_kernel (tools/minimap2-acceleration/kernel/scalar/src/host_kernel.cpp,
// benchmarks/chain/src/host_kernel.cpp:481-501) over the C ABI of csrc/chain.hip.
// The calls are flattened to CSR, run as one device batch, and the return vectors are resized and
// filled like the reference's (ret[c].n = n, four vectors of n entries). The flatten and the fill
// are spread over host threads (calls balanced by anchors), into and out of page-locked staging
// buffers kept per calling thread, so the H2D / D2H copies run at DMA rate.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/gb.h"

#include "../../include/gb_chain.h"
#include "../../include/gb_compat/minimap2_chain.h"

static void die(const char *what, int st) {
  fprintf(stderr, "[gb chain] %s failed (%d): %s\n", what, st, gb_last_error());
  abort();
}

// HIP's current device is per host thread: every calling thread selects GB_DEVICE once.
static void ensure_device() {
  static const int dev = [] {
    const char *d = getenv("GB_DEVICE");
    return d ? atoi(d) : 0;
  }();
  thread_local bool done = false;
  if (done) return;
  const int st = gb_set_device(dev);
  if (st) die("gb_set_device", st);
  done = true;
}

namespace {

// grow-only page-locked buffer, kept per calling thread across calls (the reference's loop calls
// host_chain_kernel once per input batch) and freed when the thread ends (thread-storage objects of
// the main thread are destroyed before the HIP runtime's statics)
struct Pinned {
  void *p = nullptr;
  size_t cap = 0;
  Pinned() = default;
  Pinned(const Pinned &) = delete;
  Pinned &operator=(const Pinned &) = delete;
  ~Pinned() {
    if (p) gb_host_free(p);
  }
  template <typename T>
  T *get(size_t n) {
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    if (bytes > cap) {
      if (p) gb_host_free(p);
      p = nullptr;
      cap = 0;
      const int st = gb_host_alloc(&p, bytes + bytes / 4);
      if (st) die("gb_host_alloc", st);
      cap = bytes + bytes / 4;
    }
    return static_cast<T *>(p);
  }
};

// run f(lo, hi) over [0, ncalls) in up to `nt` contiguous pieces balanced by anchors
template <typename F>
void parallel_calls(int64_t ncalls, const int64_t *off, int nt, F f) {
  if (nt <= 1 || ncalls < 2) {
    f((int64_t)0, ncalls);
    return;
  }
  std::vector<int64_t> cut((size_t)nt + 1, ncalls);
  cut[0] = 0;
  for (int t = 1; t < nt; t++)
    cut[(size_t)t] = std::upper_bound(off, off + ncalls + 1, off[ncalls] * t / nt) - off - 1;
  for (int t = 1; t <= nt; t++) cut[(size_t)t] = std::max(cut[(size_t)t], cut[(size_t)t - 1]);
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back(f, cut[(size_t)t], cut[(size_t)t + 1]);
  f(cut[0], cut[1]);
  for (auto &x : th) x.join();
}

}  // namespace

void host_chain_kernel(std::vector<call_t> &arg, std::vector<return_t> &ret, int /*numThreads*/) {
  ensure_device();
  const auto t0 = std::chrono::steady_clock::now();
  thread_local Pinned bx, by, bout;
  const int64_t nc = (int64_t)arg.size();
  std::vector<int64_t> off((size_t)nc + 1, 0);
  for (int64_t c = 0; c < nc; c++) off[c + 1] = off[c] + (int64_t)arg[c].anchors.size();
  const int64_t na = off[nc];
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                                na / 250000 + 1}));
  uint64_t *x = bx.get<uint64_t>((size_t)na), *y = by.get<uint64_t>((size_t)na);
  int32_t *out = bout.get<int32_t>(4 * (size_t)std::max<int64_t>(na, 1));
  std::vector<float> aq((size_t)nc);
  std::vector<int32_t> p4((size_t)nc * 4);
  parallel_calls(nc, off.data(), nt, [&](int64_t lo, int64_t hi) {
    for (int64_t c = lo; c < hi; c++) {
      const call_t &a = arg[c];
      const anchor_t *an = a.anchors.data();
      for (size_t k = 0; k < a.anchors.size(); k++) {
        x[off[c] + k] = an[k].x;
        y[off[c] + k] = an[k].y;
      }
      aq[c] = a.avg_qspan;
      p4[4 * c] = a.max_dist_x;
      p4[4 * c + 1] = a.max_dist_y;
      p4[4 * c + 2] = a.bw;
      p4[4 * c + 3] = a.n_segs;
    }
  });
  const size_t nn = (size_t)std::max<int64_t>(na, 1);
  int32_t *sc = out, *par = out + nn, *tg = out + 2 * nn, *pk = out + 3 * nn;
  const auto t1 = std::chrono::steady_clock::now();
  int st = gb_chain(nc, off.data(), aq.data(), p4.data(), x, y, sc, par, tg, pk);
  const auto t2 = std::chrono::steady_clock::now();
  if (st) die("gb_chain", st);
  ret.resize((size_t)nc);
  parallel_calls(nc, off.data(), nt, [&](int64_t lo, int64_t hi) {
    for (int64_t c = lo; c < hi; c++) {
      return_t &r = ret[c];
      const int64_t a = off[c], b = off[c + 1];
      r.n = b - a;
      r.scores.assign(sc + a, sc + b);
      r.parents.assign(par + a, par + b);
      r.targets.assign(tg + a, tg + b);
      r.peak_scores.assign(pk + a, pk + b);
    }
  });
  if (getenv("GB_CHAIN_HOSTPROF")) {
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr, "[host_chain_kernel] flatten %.2f ms, gb_chain %.2f ms, return vectors %.2f ms (%d threads)\n",
            ms(t0, t1), ms(t1, t2), ms(t2, std::chrono::steady_clock::now()), nt);
  }
}
