/*
 * gb_compat/minimap2_chain.h -- source-compatible declarations of the reference chaining interface
 * for relinking the reference's chain driver against the MI355X implementation.
 *
 * Mirrors (same member names, types and order; written here, not copied):
 *   anchor_t / call_t / return_t   tools/minimap2-acceleration/kernel/scalar/src/host_data.h:7-37
 *                                  (== benchmarks/chain/src/host_data.h:19-46 minus the HE members)
 *   host_chain_kernel              tools/minimap2-acceleration/kernel/scalar/src/host_kernel.h
 *                                  (== benchmarks/chain/src/host_kernel.h:6)
 * Implemented by genomicsbench_palisade_amd/lib/libgb_chain_dropin.so (csrc/chain_dropin.cpp) on
 * the device selected by $GB_DEVICE (default 0); numThreads is accepted and ignored.
 */
#ifndef GB_COMPAT_MINIMAP2_CHAIN_H
#define GB_COMPAT_MINIMAP2_CHAIN_H

#include <cstdint>
#include <vector>

typedef int64_t anchor_idx_t;
typedef uint32_t tag_t;
typedef int32_t loc_t;
typedef int32_t loc_dist_t;
typedef int32_t score_t;
typedef int32_t parent_t;
typedef int32_t target_t;
typedef int32_t peak_score_t;

#define ANCHOR_NULL (anchor_idx_t)(-1)

struct anchor_t {
  uint64_t x;
  uint64_t y;
};

struct call_t {
  anchor_idx_t n;
  float avg_qspan;
  int max_dist_x, max_dist_y, bw, n_segs;
  std::vector<anchor_t> anchors;
};

struct return_t {
  anchor_idx_t n;
  std::vector<score_t> scores;
  std::vector<parent_t> parents;
  std::vector<target_t> targets;
  std::vector<peak_score_t> peak_scores;
};

void host_chain_kernel(std::vector<call_t> &arg, std::vector<return_t> &ret, int numThreads);

#endif
