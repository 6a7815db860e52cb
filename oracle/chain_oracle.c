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

/* ---------------------------------------------------------------------------------------------
 * Chain backtrack: the consumer of chain_dp's score f[], parent p[] and peak v[] arrays in minimap2
 * (tools/minimap2-acceleration/testbed/chain.c:140-219, the same code follows the DP in
 * tools/minimap2/chain.c): chain ends -> their peaks, sorted by (score, index) descending, claimed
 * greedily along parent links, then reordered by the x of each chain's first anchor. The two sorts
 * are ksort.h's in-place MSD radix sort (KRADIX_SORT_INIT, ksort.h:93-150; 8 bits per pass,
 * insertion sort below 64 elements), restated here because its order of equal keys is part of the
 * output.
 * --------------------------------------------------------------------------------------------- */
typedef struct { uint64_t x, y; } bt128_t;

#define BT_RS_MIN 64
#define BT_RS_BITS 8

#define BT_RADIX(name, T, KEY)                                                                       \
  static void rs_ins_##name(T *beg, T *end) {                                                        \
    for (T *i = beg + 1; i < end; ++i)                                                                \
      if (KEY(*i) < KEY(*(i - 1))) {                                                                  \
        T *j, tmp = *i;                                                                               \
        for (j = i; j > beg && KEY(tmp) < KEY(*(j - 1)); --j) *j = *(j - 1);                          \
        *j = tmp;                                                                                     \
      }                                                                                               \
  }                                                                                                   \
  static void rs_sort_##name(T *beg, T *end, int n_bits, int s) {                                     \
    const int size = 1 << n_bits, m = size - 1;                                                       \
    struct { T *b, *e; } b[1 << BT_RS_BITS], *k, *be = b + size;                                      \
    for (k = b; k != be; ++k) k->b = k->e = beg;                                                      \
    for (T *i = beg; i != end; ++i) ++b[KEY(*i) >> s & m].e;                                          \
    for (k = b + 1; k != be; ++k) k->e += (k - 1)->e - beg, k->b = (k - 1)->e;                       \
    for (k = b; k != be;) {                                                                           \
      if (k->b != k->e) {                                                                             \
        __typeof__(b[0]) *l;                                                                          \
        if ((l = b + (KEY(*k->b) >> s & m)) != k) {                                                   \
          T tmp = *k->b, swap;                                                                        \
          do {                                                                                        \
            swap = tmp;                                                                               \
            tmp = *l->b;                                                                              \
            *l->b++ = swap;                                                                           \
            l = b + (KEY(tmp) >> s & m);                                                              \
          } while (l != k);                                                                           \
          *k->b++ = tmp;                                                                              \
        } else                                                                                        \
          ++k->b;                                                                                     \
      } else                                                                                          \
        ++k;                                                                                          \
    }                                                                                                 \
    for (b->b = beg, k = b + 1; k != be; ++k) k->b = (k - 1)->e;                                      \
    if (s) {                                                                                          \
      s = s > n_bits ? s - n_bits : 0;                                                                \
      for (k = b; k != be; ++k)                                                                       \
        if (k->e - k->b > BT_RS_MIN)                                                                  \
          rs_sort_##name(k->b, k->e, n_bits, s);                                                      \
        else if (k->e - k->b > 1)                                                                     \
          rs_ins_##name(k->b, k->e);                                                                  \
    }                                                                                                 \
  }                                                                                                   \
  void bt_radix_sort_##name(T *beg, T *end) {                                                         \
    if (end - beg <= BT_RS_MIN)                                                                       \
      rs_ins_##name(beg, end);                                                                        \
    else                                                                                              \
      rs_sort_##name(beg, end, BT_RS_BITS, (8 - 1) * BT_RS_BITS);                                     \
  }

#define BT_KEY64(a) (a)
#define BT_KEY128(a) ((a).x)
BT_RADIX(64, uint64_t, BT_KEY64)
BT_RADIX(128x, bt128_t, BT_KEY128)

/* One call (testbed/chain.c:140-219). u_out gets the chains (score << 32 | anchor count) in output
 * order, bx/by their anchors concatenated (capacity 2n: a chain start that an earlier chain already
 * claimed can be emitted again as a one-anchor chain when min_cnt <= 1). Returns the chain count;
 * *n_anchors = anchors written. */
int64_t chain_oracle_backtrack(int64_t n, const int32_t *f, const int32_t *p, const int32_t *v,
                               const uint64_t *ax, const uint64_t *ay, int min_cnt, int min_sc,
                               uint64_t *u_out, uint64_t *bx, uint64_t *by, int64_t *n_anchors) {
  *n_anchors = 0;
  if (n <= 0) return 0;
  int32_t *t = (int32_t *)calloc((size_t)n, 4), *vv = (int32_t *)malloc((size_t)n * 8);
  int64_t i, j, n_u, n_v, k;
  for (i = 0; i < n; ++i)
    if (p[i] >= 0) t[p[i]] = 1;
  for (i = n_u = 0; i < n; ++i)
    if (t[i] == 0 && v[i] >= min_sc) ++n_u;
  if (n_u == 0) {
    free(t);
    free(vv);
    return 0;
  }
  uint64_t *u = (uint64_t *)malloc((size_t)n_u * 8);
  for (i = n_u = 0; i < n; ++i) {
    if (t[i] == 0 && v[i] >= min_sc) {
      j = i;
      while (j >= 0 && f[j] < v[j]) j = p[j];  // the peak that maximizes f[]
      if (j < 0) j = i;
      u[n_u++] = (uint64_t)f[j] << 32 | (uint64_t)j;
    }
  }
  bt_radix_sort_64(u, u + n_u);
  for (i = 0; i < n_u >> 1; ++i) {  // highest score first
    const uint64_t tmp = u[i];
    u[i] = u[n_u - i - 1], u[n_u - i - 1] = tmp;
  }
  for (i = 0; i < n; ++i) t[i] = 0;
  for (i = n_v = k = 0; i < n_u; ++i) {
    const int64_t n_v0 = n_v, k0 = k;
    j = (int32_t)u[i];
    do {
      vv[n_v++] = (int32_t)j;
      t[j] = 1;
      j = p[j];
    } while (j >= 0 && t[j] == 0);
    if (j < 0) {
      if (n_v - n_v0 >= min_cnt) u[k++] = u[i] >> 32 << 32 | (uint64_t)(n_v - n_v0);
    } else if ((int32_t)(u[i] >> 32) - f[j] >= min_sc) {
      if (n_v - n_v0 >= min_cnt) u[k++] = ((u[i] >> 32) - (uint64_t)f[j]) << 32 | (uint64_t)(n_v - n_v0);
    }
    if (k0 == k) n_v = n_v0;
  }
  n_u = k;
  bt128_t *b = (bt128_t *)malloc((size_t)(n_v > 0 ? n_v : 1) * sizeof(bt128_t));
  for (i = 0, k = 0; i < n_u; ++i) {
    const int64_t k0 = k, ni = (int32_t)u[i];
    for (j = 0; j < ni; ++j) {
      const int32_t a = vv[k0 + (ni - j - 1)];
      b[k].x = ax[a], b[k].y = ay[a], ++k;
    }
  }
  bt128_t *w = (bt128_t *)malloc((size_t)n_u * sizeof(bt128_t));
  for (i = k = 0; i < n_u; ++i) {
    w[i].x = b[k].x, w[i].y = (uint64_t)k << 32 | (uint64_t)i;
    k += (int32_t)u[i];
  }
  bt_radix_sort_128x(w, w + n_u);
  for (i = k = 0; i < n_u; ++i) {
    const int64_t jj = (int32_t)w[i].y, nn = (int32_t)u[jj];
    u_out[i] = u[jj];
    for (int64_t q = 0; q < nn; q++) {
      bx[k + q] = b[(w[i].y >> 32) + q].x;
      by[k + q] = b[(w[i].y >> 32) + q].y;
    }
    k += nn;
  }
  *n_anchors = k;
  free(t);
  free(vv);
  free(u);
  free(b);
  free(w);
  return n_u;
}

/* All calls (CSR): u_out[offsets[c] ..) and bx/by[2*offsets[c] ..) per call; n_chains[c],
 * n_anchor[c] counts. OpenMP over calls. */
void chain_oracle_backtrack_batch(int64_t ncalls, const int64_t *offsets, const int32_t *f, const int32_t *p,
                                  const int32_t *v, const uint64_t *ax, const uint64_t *ay, int min_cnt,
                                  int min_sc, uint64_t *u_out, uint64_t *bx, uint64_t *by, int64_t *n_chains,
                                  int64_t *n_anchor, int nthreads) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int64_t c = 0; c < ncalls; c++) {
    const int64_t o = offsets[c], n = offsets[c + 1] - o;
    n_chains[c] = chain_oracle_backtrack(n, f + o, p + o, v + o, ax + o, ay + o, min_cnt, min_sc, u_out + o,
                                         bx + 2 * o, by + 2 * o, n_anchor + c);
  }
}
