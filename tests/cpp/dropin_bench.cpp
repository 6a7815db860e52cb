// dropin_bench.cpp -- BENCH/TEST HARNESS (bench.py dropin legs): calls the C++ drop-ins exactly the way
// the reference benchmarks do, from plain arrays handed over by ctypes.
//   bench_host_chain_kernel: builds std::vector<call_t> (outside the timed region) and times one
//     host_chain_kernel call, as tools/minimap2-acceleration/kernel/scalar/src/main.cpp:80-91 does.
//   bench_bsw_batches: one BandedPairWiseSW per thread; threads take 512-pair batches dynamically and
//     call getScores16 on each, as benchmarks/bsw/main_banded.cpp:896-924 does (OpenMP
//     schedule(dynamic, 1)); each batch's SeqPair.idr/idq index that batch's own buffers (loadPairs
//     restarts them per batch, main_banded.cpp:177-189).
// Both return the timed seconds and write the results out for the caller's parity check.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/gb_compat/bandedSWA.h"
#include "../../include/gb_compat/minimap2_chain.h"

extern "C" double bench_host_chain_kernel(int64_t ncalls, const int64_t *offsets, const float *avg_qspan,
                                          const int32_t *params4, const uint64_t *x, const uint64_t *y,
                                          int threads, int32_t *scores, int32_t *parents, int32_t *targets,
                                          int32_t *peaks) {
  std::vector<call_t> calls((size_t)ncalls);
  for (int64_t c = 0; c < ncalls; c++) {
    call_t &a = calls[(size_t)c];
    a.n = offsets[c + 1] - offsets[c];
    a.avg_qspan = avg_qspan[c];
    a.max_dist_x = params4[4 * c];
    a.max_dist_y = params4[4 * c + 1];
    a.bw = params4[4 * c + 2];
    a.n_segs = params4[4 * c + 3];
    a.anchors.resize((size_t)a.n);
    for (int64_t k = 0; k < a.n; k++) a.anchors[(size_t)k] = {x[offsets[c] + k], y[offsets[c] + k]};
  }
  std::vector<return_t> rets(calls.size());
  const auto t0 = std::chrono::steady_clock::now();
  host_chain_kernel(calls, rets, threads);
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (int64_t c = 0; c < ncalls; c++) {
    const return_t &r = rets[(size_t)c];
    const int64_t o = offsets[c];
    for (int64_t k = 0; k < r.n; k++) {
      scores[o + k] = r.scores[(size_t)k];
      parents[o + k] = r.parents[(size_t)k];
      targets[o + k] = r.targets[(size_t)k];
      peaks[o + k] = r.peak_scores[(size_t)k];
    }
  }
  return s;
}

// pairs: n SeqPair records whose idr/idq index the packed buffers tgt/qry (global offsets); out6 =
// score, qle, tle, gtle, gscore, max_off per pair.
extern "C" double bench_bsw_batches(const int32_t *par7, const int8_t *mat, int64_t n, const SeqPair *pairs,
                                    const uint8_t *tgt, const uint8_t *qry, int batch, int threads, int32_t *out6) {
  // per batch: its SeqPair slice re-based to the batch's first bytes, as loadPairs lays them out
  std::vector<SeqPair> sp(pairs, pairs + n);
  const int64_t nb = (n + batch - 1) / batch;
  std::vector<int64_t> rbase((size_t)nb), qbase((size_t)nb);
  for (int64_t b = 0; b < nb; b++) {
    const int64_t lo = b * batch, hi = std::min<int64_t>(n, lo + batch);
    int64_t r0 = INT64_MAX, q0 = INT64_MAX;
    for (int64_t k = lo; k < hi; k++) {
      r0 = std::min<int64_t>(r0, sp[(size_t)k].idr);
      q0 = std::min<int64_t>(q0, sp[(size_t)k].idq);
    }
    for (int64_t k = lo; k < hi; k++) {
      sp[(size_t)k].idr -= r0;
      sp[(size_t)k].idq -= q0;
    }
    rbase[(size_t)b] = r0;
    qbase[(size_t)b] = q0;
  }
  std::atomic<int64_t> next{0};
  auto worker = [&] {
    BandedPairWiseSW bsw(par7[0], par7[1], par7[2], par7[3], par7[4], par7[5], mat, 1, 4, 1);
    for (int64_t b; (b = next++) < nb;) {
      const int64_t lo = b * batch;
      const int32_t cnt = (int32_t)std::min<int64_t>(batch, n - lo);
      bsw.getScores16(sp.data() + lo, const_cast<uint8_t *>(tgt) + rbase[(size_t)b],
                      const_cast<uint8_t *>(qry) + qbase[(size_t)b], cnt, 1, par7[6]);
    }
  };
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++) th.emplace_back(worker);
  for (auto &t : th) t.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (int64_t k = 0; k < n; k++) {
    const SeqPair &p = sp[(size_t)k];
    int32_t *o = out6 + 6 * k;
    o[0] = p.score;
    o[1] = p.qle;
    o[2] = p.tle;
    o[3] = p.gtle;
    o[4] = p.gscore;
    o[5] = p.max_off;
  }
  return s;
}
