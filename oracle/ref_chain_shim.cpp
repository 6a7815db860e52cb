// oracle/ref_chain_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// Our own C entry point over the reference's UNMODIFIED scalar chaining kernel
// (tools/minimap2-acceleration/kernel/scalar/src/host_kernel.cpp, chain_dp :30-94 and
// host_chain_kernel :97-108), compiled by oracle/Makefile into oracle/_ref/libref_chain.so.
// Packs CSR arrays into the reference's call_t (host_data.h:19-39) and unpacks return_t.
#include <cstdint>
#include <cstddef>
#include <vector>

#include "host_data.h"
#include "host_kernel.h"

extern "C" void ref_chain_batch(int64_t ncalls, const int64_t *offsets, const float *avg_qspan,
                                const int32_t *params4, const uint64_t *ax, const uint64_t *ay,
                                int32_t *scores, int32_t *parents, int32_t *targets, int32_t *peaks,
                                int nthreads) {
  std::vector<call_t> calls((size_t)ncalls);
  std::vector<return_t> rets((size_t)ncalls);
  for (int64_t c = 0; c < ncalls; c++) {
    call_t &a = calls[(size_t)c];
    a.n = offsets[c + 1] - offsets[c];
    a.avg_qspan = avg_qspan[c];
    a.max_dist_x = params4[4 * c];
    a.max_dist_y = params4[4 * c + 1];
    a.bw = params4[4 * c + 2];
    a.n_segs = params4[4 * c + 3];
    a.anchors.resize((size_t)a.n);
    for (int64_t k = 0; k < a.n; k++) {
      a.anchors[(size_t)k].x = ax[offsets[c] + k];
      a.anchors[(size_t)k].y = ay[offsets[c] + k];
    }
  }
  host_chain_kernel(calls, rets, nthreads > 0 ? nthreads : 1);
  for (int64_t c = 0; c < ncalls; c++) {
    const return_t &r = rets[(size_t)c];
    for (int64_t k = 0; k < r.n; k++) {
      scores[offsets[c] + k] = r.scores[(size_t)k];
      parents[offsets[c] + k] = r.parents[(size_t)k];
      targets[offsets[c] + k] = r.targets[(size_t)k];
      peaks[offsets[c] + k] = r.peak_scores[(size_t)k];
    }
  }
}
