/*
 * gb_chain.h -- C ABI of the MI355X minimap2 anchor-chaining DP (drop-in boundary for benchmarks/chain).
 *
 * Reference interface this replaces (paths relative to the reference repo):
 *   void host_chain_kernel(std::vector<call_t>&, std::vector<return_t>&, int numThreads);
 *        benchmarks/chain/src/host_kernel.h:6, host_kernel.cpp:481-501 -> chain_dp :58-479 (plaintext
 *        branch :405-472 == tools/minimap2-acceleration/kernel/scalar/src/host_kernel.cpp:30-94)
 *   call_t / return_t / anchor_t: benchmarks/chain/src/host_data.h:19-46
 * The calls are flattened to CSR: anchors of call c are x[offsets[c] .. offsets[c+1]), same for y and
 * for the four outputs. params4[4c..4c+3] = {max_dist_x, max_dist_y, bw, n_segs}.
 * 0 on success, negative gb_status on failure (gb_last_error()).
 */
#ifndef GB_CHAIN_H
#define GB_CHAIN_H

#include <stdint.h>

#include "gb.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gb_chain_batch gb_chain_batch;

/* Upload a set of calls (anchors sorted by x within each call, as minimap2 produces them; each call
 * below 2^30 anchors, else GB_ERR_ARG). */
int gb_chain_batch_create(int64_t ncalls, const int64_t *offsets, const float *avg_qspan,
                          const int32_t *params4, const uint64_t *x, const uint64_t *y,
                          gb_chain_batch **out);
/* chain_dp for every call (asynchronous on the batch's stream). */
int gb_chain_batch_run(gb_chain_batch *b);
int gb_chain_batch_sync(gb_chain_batch *b);
/* scores/parents/targets/peak_scores per anchor (any may be NULL); visited = total (i, j) pairs the
 * reference loop visits (work accounting). */
int gb_chain_batch_results(gb_chain_batch *b, int32_t *scores, int32_t *parents, int32_t *targets,
                           int32_t *peak_scores, int64_t *visited);
int gb_chain_batch_timing(gb_chain_batch *b, float *kernel_ms);
/* Diagnostics of the last run: calls run as speculative segments (long calls with sorted x, see
 * csrc/chain_split.hip), guess/verify rounds, and fix-up blocks (anchors whose guess failed the
 * verification and were recomputed sequentially). Environment (development aids, read when a batch
 * is filled): GB_CHAIN_SPLIT = "0" (no splitting) or "SEG[,WARM[,1]]" (1: warm-up from the
 * segment start, not its window); GB_CHAIN_SPLIT_FAULT = k makes the guess of every k-th anchor
 * wrong (read at run time), to exercise the verification; GB_CHAIN_ROWS=0 runs every block on the
 * 64-lane sequential kernel instead of chain_rows (two calls per wave), GB_CHAIN_VLANES=0 verifies
 * every split anchor with the 64-lane verification instead of one anchor per lane (A/B, tests). */
int gb_chain_batch_split_stats(gb_chain_batch *b, int64_t *split_calls, int64_t *rounds, int64_t *fixups);
int gb_chain_batch_destroy(gb_chain_batch *b);

/* Chain backtrack on the batch's chain_dp outputs (asynchronous): minimap2's consumer of score /
 * parent / peak (tools/minimap2-acceleration/testbed/chain.c:140-219 == tools/minimap2/chain.c):
 * chain ends -> peaks, ordered by score, claimed greedily, kept if >= min_cnt anchors and (when
 * stopped by an earlier chain) score gain >= min_sc, reordered by the x of their first anchor.
 * minimap2's defaults are min_cnt 3, min_sc 40. */
int gb_chain_batch_backtrack(gb_chain_batch *b, int32_t min_cnt, int32_t min_sc);
/* Results of the last backtrack (synchronous), CSR by the batch's offsets: call c's chains
 * (score << 32 | anchor count, mm_chain_dp's u[]) at u[offsets[c] .. + n_chains[c]) and their anchors
 * concatenated in chain order at ax/ay[2*offsets[c] .. + n_anchors[c]) (capacity 2n per call: a
 * start that an earlier chain owns can be kept again as a one-anchor chain when min_cnt <= 1).
 * Any output may be NULL; totals are over all calls. */
int gb_chain_batch_chains(gb_chain_batch *b, int64_t *n_chains, uint64_t *u, int64_t *n_anchors,
                          uint64_t *ax, uint64_t *ay, int64_t *total_chains, int64_t *total_anchors);
int gb_chain_batch_backtrack_timing(gb_chain_batch *b, float *ms);

/* One-shot form of host_chain_kernel over CSR arrays. */
int gb_chain(int64_t ncalls, const int64_t *offsets, const float *avg_qspan, const int32_t *params4,
             const uint64_t *x, const uint64_t *y, int32_t *scores, int32_t *parents,
             int32_t *targets, int32_t *peak_scores);

#ifdef __cplusplus
}
#endif
#endif /* GB_CHAIN_H */
