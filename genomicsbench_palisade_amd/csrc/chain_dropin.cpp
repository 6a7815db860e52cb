// chain_dropin.cpp -- host_chain_kernel (tools/minimap2-acceleration/kernel/scalar/src/host_kernel.cpp,
// benchmarks/chain/src/host_kernel.cpp:481-501) over the C ABI of csrc/chain.hip.
// The calls are flattened to CSR, run as one device batch, and the return vectors are resized and
// filled like the reference's (ret[c].n = n, four vectors of n entries).
#include <cstdio>
#include <cstdlib>
#include <vector>

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

void host_chain_kernel(std::vector<call_t> &arg, std::vector<return_t> &ret, int /*numThreads*/) {
  ensure_device();
  const int64_t nc = (int64_t)arg.size();
  std::vector<int64_t> off((size_t)nc + 1, 0);
  for (int64_t c = 0; c < nc; c++) off[c + 1] = off[c] + (int64_t)arg[c].anchors.size();
  const int64_t na = off[nc];
  std::vector<uint64_t> x((size_t)na), y((size_t)na);
  std::vector<float> aq((size_t)nc);
  std::vector<int32_t> p4((size_t)nc * 4);
  for (int64_t c = 0; c < nc; c++) {
    const call_t &a = arg[c];
    for (size_t k = 0; k < a.anchors.size(); k++) {
      x[off[c] + k] = a.anchors[k].x;
      y[off[c] + k] = a.anchors[k].y;
    }
    aq[c] = a.avg_qspan;
    p4[4 * c] = a.max_dist_x;
    p4[4 * c + 1] = a.max_dist_y;
    p4[4 * c + 2] = a.bw;
    p4[4 * c + 3] = a.n_segs;
  }
  std::vector<int32_t> sc((size_t)na), par((size_t)na), tg((size_t)na), pk((size_t)na);
  int st = gb_chain(nc, off.data(), aq.data(), p4.data(), x.data(), y.data(), sc.data(), par.data(),
                    tg.data(), pk.data());
  if (st) die("gb_chain", st);
  ret.resize((size_t)nc);
  for (int64_t c = 0; c < nc; c++) {
    return_t &r = ret[c];
    const int64_t n = off[c + 1] - off[c];
    r.n = n;
    r.scores.assign(sc.begin() + off[c], sc.begin() + off[c + 1]);
    r.parents.assign(par.begin() + off[c], par.begin() + off[c + 1]);
    r.targets.assign(tg.begin() + off[c], tg.begin() + off[c + 1]);
    r.peak_scores.assign(pk.begin() + off[c], pk.begin() + off[c + 1]);
  }
}
