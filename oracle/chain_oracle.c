/*
 * oracle/chain_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU checker, never the product path).
 *
 * Plain-C restatement of minimap2's chaining DP as the reference's chain benchmark computes it:
 * the plaintext branch of benchmarks/chain/src/host_kernel.cpp:405-472, identical to
 * tools/minimap2-acceleration/kernel/scalar/src/host_kernel.cpp:30-94 (chain_dp), ilog2_32 :22-27.
 * The benchmark's HE branch (host_kernel.cpp:104-404) crashes and is not the parity target
 * (SURVEY.md section 0.3). Pinned against the reference scalar kernel compiled from
 * /root/reference (oracle/_ref/libref_chain.so) and the committed golden vectors.
 * C integer/double semantics follow the C++ source exactly (int64 dr, int32 truncations, the
 * double expression order of the gap cost).
 */
#include <stdint.h>
#include <stdlib.h>

static const char LogTable256[256] = {
#define LT(n) n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, n
    -1, 0, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3,
    LT(4), LT(5), LT(5), LT(6), LT(6), LT(6), LT(6),
    LT(7), LT(7), LT(7), LT(7), LT(7), LT(7), LT(7), LT(7)};

static inline int ilog2_32(uint32_t v) {
  uint32_t t, tt;
  if ((tt = v >> 16)) return (t = tt >> 8) ? 24 + LogTable256[t] : 16 + LogTable256[tt];
  return (t = v >> 8) ? 8 + LogTable256[t] : LogTable256[v];
}

#define SEG_SHIFT 48
#define SEG_MASK (0xffULL << SEG_SHIFT)

/* One call. Outputs have n entries; targets must be zero-initialized by the caller (the reference's
 * fresh std::vector). Returns the number of (i, j) pairs visited by the inner loop. */
int64_t chain_oracle_dp(int64_t n, float avg_qspan, int max_dist_x, int max_dist_y, int bw, int n_segs,
                        const uint64_t *ax, const uint64_t *ay, int32_t *scores, int32_t *parents,
                        int32_t *targets, int32_t *peak_scores) {
  int64_t i, j, st = 0, visited = 0;
  const int is_cdna = 0;
  const float gap_scale = 1.0f;
  const int max_iter = 5000, max_skip = 25;
  for (i = 0; i < n; ++i) {
    uint64_t ri = ax[i];
    int64_t max_j = -1;
    int32_t qi = (int32_t)ay[i], q_span = ay[i] >> 32 & 0xff;
    int32_t max_f = q_span, n_skip = 0, min_d;
    int32_t sidi = (int32_t)((ay[i] & SEG_MASK) >> SEG_SHIFT);
    while (st < i && ri > ax[st] + max_dist_x) ++st;
    if (i - st > max_iter) st = i - max_iter;
    for (j = i - 1; j >= st; --j) {
      visited++;
      int64_t dr = ri - ax[j];
      int32_t dq = qi - (int32_t)ay[j], dd, sc, log_dd, gap_cost;
      int32_t sidj = (int32_t)((ay[j] & SEG_MASK) >> SEG_SHIFT);
      if ((sidi == sidj && dr == 0) || dq <= 0) continue;
      if ((sidi == sidj && dq > max_dist_y) || dq > max_dist_x) continue;
      dd = (int32_t)(dr > dq ? dr - dq : dq - dr);
      if (sidi == sidj && dd > bw) continue;
      if (n_segs > 1 && !is_cdna && sidi == sidj && dr > max_dist_y) continue;
      min_d = (int32_t)(dq < dr ? (int64_t)dq : dr);
      sc = (int32_t)(min_d > q_span ? (int64_t)q_span : (dq < dr ? (int64_t)dq : dr));
      log_dd = dd ? ilog2_32((uint32_t)dd) : 0;
      gap_cost = 0;
      if (is_cdna || sidi != sidj) {
        int c_log, c_lin;
        c_lin = (int)(dd * .01 * avg_qspan);
        c_log = log_dd;
        if (sidi != sidj && dr == 0)
          ++sc;
        else if (dr > dq || sidi != sidj)
          gap_cost = c_lin < c_log ? c_lin : c_log;
        else
          gap_cost = c_lin + (c_log >> 1);
      } else
        gap_cost = (int)(dd * .01 * avg_qspan) + (log_dd >> 1);
      sc -= (int)((double)gap_cost * gap_scale + .499);
      sc += scores[j];
      if (sc > max_f) {
        max_f = sc, max_j = j;
        if (n_skip > 0) --n_skip;
      } else if (targets[j] == i) {
        if (++n_skip > max_skip) break;
      }
      if (parents[j] >= 0) targets[parents[j]] = (int32_t)i;
    }
    scores[i] = max_f, parents[i] = (int32_t)max_j;
    peak_scores[i] = max_j >= 0 && peak_scores[max_j] > max_f ? peak_scores[max_j] : max_f;
  }
  return visited;
}

/* Many calls in CSR form (offsets[c]..offsets[c+1]); returns total visited pairs. */
int64_t chain_oracle_batch(int64_t ncalls, const int64_t *offsets, const float *avg_qspan, const int32_t *params4,
                           const uint64_t *ax, const uint64_t *ay, int32_t *scores, int32_t *parents,
                           int32_t *targets, int32_t *peak_scores, int nthreads) {
  int64_t total = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total) num_threads(nthreads > 0 ? nthreads : 1)
#endif
  for (int64_t c = 0; c < ncalls; c++) {
    const int64_t o = offsets[c], n = offsets[c + 1] - offsets[c];
    for (int64_t k = 0; k < n; k++) targets[o + k] = 0;
    total += chain_oracle_dp(n, avg_qspan[c], params4[4 * c], params4[4 * c + 1], params4[4 * c + 2],
                             params4[4 * c + 3], ax + o, ay + o, scores + o, parents + o, targets + o,
                             peak_scores + o);
  }
  return total;
}
