/*
 * oracle/bsw_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU checker, never the product path).
 *
 * Plain-C restatement of GenomicsBench bsw's banded Smith-Waterman extension, used by tests/ and
 * bench.py's cpu_baseline leg as the parity checker.
 * Parity is pinned against bwa v1's ksw_extend2 (tools/bwa/ksw.c:380-481), compiled from the
 * reference tree by oracle/Makefile into oracle/_ref/libref_bwa.so: the benchmark's scalar kernel
 * is that function up to formatting (the reference's own comment-out of the h0 > 0 assert aside).
 *
 * Followed reference code (paths relative to /root/reference):
 *   kernel    benchmarks/bsw/bandedSWA.cpp:130-251 (BandedPairWiseSW::scalarBandedSWA)
 *   matrix    benchmarks/bsw/main_banded.cpp:77-88 (bwa_fill_scmat) with the defaults :53-57
 *             (match 1, mismatch 4, open 6, extend 1, ambig -1) and zdrop 100, w 100,
 *             end_bonus 5 (:846)
 *   pairs     benchmarks/bsw/main_banded.cpp:160-202 (loadPairs: h0, ref = target, query)
 *   outputs   SeqPair fields score/tle/qle/gtle/gscore/max_off (bandedSWA.h:92-101)
 */
#include <stdint.h>
#include <stdlib.h>

typedef struct {
  int32_t h, e;
} bo_eh; /* eh_t, bandedSWA.h:110-112 */

/* bandedSWA.cpp:130-251. out6 = {score, qle, tle, gtle, gscore, max_off}; cells counts the
 * inner-loop iterations (the reference's commented SW_cells counter, :189). */
int bsw_oracle_extend(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                      const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                      int end_bonus, int zdrop, int h0, int32_t *out6, int64_t *cells) {
  int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
  int8_t *qp = (int8_t *)malloc((size_t)qlen * m + 1);
  bo_eh *eh = (bo_eh *)calloc((size_t)qlen + 1, sizeof(bo_eh));
  int64_t ncell = 0;
  /* query profile (:150-154) */
  for (int k = 0, i = 0; k < m; ++k)
    for (int j = 0; j < qlen; ++j) qp[i++] = mat[k * m + query[j]];
  /* first row (:157-159) */
  eh[0].h = h0;
  if (qlen >= 1) eh[1].h = h0 > oe_ins ? h0 - oe_ins : 0;
  for (int j = 2; j <= qlen && eh[j - 1].h > e_ins; ++j) eh[j].h = eh[j - 1].h - e_ins;
  /* band adjustment (:161-170) */
  int mx = 0;
  for (int i = 0; i < m * m; ++i) mx = mx > mat[i] ? mx : mat[i];
  int max_ins = (int)((double)(qlen * mx + end_bonus - o_ins) / e_ins + 1.);
  max_ins = max_ins > 1 ? max_ins : 1;
  w = w < max_ins ? w : max_ins;
  int max_del = (int)((double)(qlen * mx + end_bonus - o_del) / e_del + 1.);
  max_del = max_del > 1 ? max_del : 1;
  w = w < max_del ? w : max_del;
  /* DP (:173-240) */
  int max = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
  int beg = 0, end = qlen, i, j;
  for (i = 0; i < tlen; ++i) {
    int t, f = 0, h1, mrow = 0, mj = -1;
    const int8_t *q = &qp[target[i] * qlen];
    if (beg < i - w) beg = i - w;
    if (end > i + w + 1) end = i + w + 1;
    if (end > qlen) end = qlen;
    if (beg == 0) {
      h1 = h0 - (o_del + e_del * (i + 1));
      if (h1 < 0) h1 = 0;
    } else
      h1 = 0;
    for (j = beg; j < end; ++j) {
      bo_eh *p = &eh[j];
      int h, M = p->h, e = p->e;
      p->h = h1;
      M = M ? M + q[j] : 0;
      h = M > e ? M : e;
      h = h > f ? h : f;
      h1 = h;
      mj = mrow > h ? mj : j;
      mrow = mrow > h ? mrow : h;
      t = M - oe_del;
      t = t > 0 ? t : 0;
      e -= e_del;
      e = e > t ? e : t;
      p->e = e;
      t = M - oe_ins;
      t = t > 0 ? t : 0;
      f -= e_ins;
      f = f > t ? f : t;
      ++ncell;
    }
    eh[end].h = h1;
    eh[end].e = 0;
    if (j == qlen) {
      max_ie = gscore > h1 ? max_ie : i;
      gscore = gscore > h1 ? gscore : h1;
    }
    if (mrow == 0) break;
    if (mrow > max) {
      max = mrow, max_i = i, max_j = mj;
      max_off = max_off > abs(mj - i) ? max_off : abs(mj - i);
    } else if (zdrop > 0) {
      if (i - max_i > mj - max_j) {
        if (max - mrow - ((i - max_i) - (mj - max_j)) * e_del > zdrop) break;
      } else {
        if (max - mrow - ((mj - max_j) - (i - max_i)) * e_ins > zdrop) break;
      }
    }
    for (j = beg; j < end && eh[j].h == 0 && eh[j].e == 0; ++j)
      ;
    beg = j;
    for (j = end; j >= beg && eh[j].h == 0 && eh[j].e == 0; --j)
      ;
    end = j + 2 < qlen ? j + 2 : qlen;
  }
  free(eh);
  free(qp);
  out6[0] = max;
  out6[1] = max_j + 1;
  out6[2] = max_i + 1;
  out6[3] = max_ie + 1;
  out6[4] = gscore;
  out6[5] = max_off;
  if (cells) *cells = ncell;
  return max;
}

/* bwa_fill_scmat (main_banded.cpp:77-88). */
void bsw_oracle_fill_scmat(int a, int b, int ambig, int8_t mat[25]) {
  int k = 0;
  for (int i = 0; i < 4; ++i) {
    for (int j = 0; j < 4; ++j) mat[k++] = i == j ? a : -b;
    mat[k++] = ambig;
  }
  for (int j = 0; j < 5; ++j) mat[k++] = ambig;
}

/* Batch over the flattened pair layout the tests and the product share: pair p has target
 * tgt[toff[p] .. +tlen[p]) and query qry[qoff[p] .. +qlen[p]); out is 6 int32 per pair.
 * params = {o_del, e_del, o_ins, e_ins, zdrop, end_bonus, w}. Returns total cells. */
int64_t bsw_oracle_batch(int64_t n, const uint8_t *tgt, const int64_t *toff, const int32_t *tlen,
                         const uint8_t *qry, const int64_t *qoff, const int32_t *qlen,
                         const int32_t *h0, const int8_t *mat, const int32_t *params, int32_t *out,
                         int64_t *cells, int nthreads) {
  int64_t total = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : total) \
    num_threads(nthreads > 0 ? nthreads : 1) if (nthreads != 1)
#endif
  for (int64_t p = 0; p < n; ++p) {
    int64_t c = 0;
    bsw_oracle_extend(qlen[p], qry + qoff[p], tlen[p], tgt + toff[p], 5, mat, params[0],
                      params[1], params[2], params[3], params[6], params[5], params[4], h0[p],
                      out + 6 * p, &c);
    if (cells) cells[p] = c;
    total += c;
  }
  return total;
}
