/* oracle/ref_bwa_shim.c -- TEST INFRASTRUCTURE ONLY.
 * Our own thin C entry points over the reference tree's UNMODIFIED bwa v1 sources
 * (/root/reference/tools/bwa, compiled by oracle/Makefile into oracle/_ref/libref_bwa.so), used as
 * an independent cross-check of the bwa-mem2 SMEM restatement (oracle/fmi_oracle.c): bwa-mem2's
 * SMEM search reproduces bwa-mem's, on the same forward+reverse-complement text.
 *   index     bwa_idx_build (tools/bwa/bwtindex.c:256) -> .pac/.bwt; bwt_restore_bwt (bwt.c:443)
 *   SMEMs     mem_collect_intv (tools/bwa/bwamem.c:114-162) restated below over bwt_smem1
 *             (bwt.c:353) and bwt_seed_strategy1 (bwt.c:358), without the final sort.
 *   SA        bwt_restore_sa (bwt.c:421) + bwt_sa (bwt.c:86): SA value of BWT rows, the same row
 *             numbering as bwa-mem2's (cross-check of FMI_search.cpp:1714 get_sa_entry_compressed).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "bwt.h"
#include "kvec.h"

int bwa_idx_build(const char *fa, const char *prefix, int algo_type, int block_size);
extern int bwa_verbose;

int ref_bwa_build(const char *fasta, const char *prefix) {
  bwa_verbose = 1;
  return bwa_idx_build(fasta, prefix, 0, 10000000);
}

void *ref_bwa_load(const char *bwt_path) { return bwt_restore_bwt(bwt_path); }
void ref_bwa_free(void *bwt) { bwt_destroy((bwt_t *)bwt); }

/* SA[rows[i]] via bwa v1's own sampled suffix array (<prefix>.sa, interval 32). */
int ref_bwa_sa(void *bwtp, const char *sa_path, const int64_t *rows, int64_t n, int64_t *out) {
  bwt_t *bwt = (bwt_t *)bwtp;
  if (!bwt->sa) bwt_restore_sa(sa_path, bwt);
  for (int64_t i = 0; i < n; i++) out[i] = (int64_t)bwt_sa(bwt, (bwtint_t)rows[i]);
  return 0;
}

/* mem_collect_intv with opt = {min_seed_len, split_factor 1.5, split_width 10, max_mem_intv 20}.
 * Out: k, l, s, m (start), n (end, inclusive) for every interval; returns count or -1 on overflow. */
int64_t ref_bwa_collect(void *bwtp, const uint8_t *seq, int len, int min_seed_len, int64_t *k,
                        int64_t *l, int64_t *s, int32_t *m, int32_t *n, int64_t cap) {
  const bwt_t *bwt = (const bwt_t *)bwtp;
  bwtintv_v mem = {0, 0, 0}, mem1 = {0, 0, 0}, t0 = {0, 0, 0}, t1 = {0, 0, 0};
  bwtintv_v *tmpv[2] = {&t0, &t1};
  int i, x = 0, old_n, kk;
  int split_len = (int)(min_seed_len * 1.5 + .499);
  while (x < len) {
    if (seq[x] < 4) {
      x = bwt_smem1(bwt, len, seq, x, 1, &mem1, tmpv);
      for (i = 0; i < (int)mem1.n; ++i) {
        bwtintv_t *p = &mem1.a[i];
        int slen = (uint32_t)p->info - (p->info >> 32);
        if (slen >= min_seed_len) kv_push(bwtintv_t, mem, *p);
      }
    } else
      ++x;
  }
  old_n = (int)mem.n;
  for (kk = 0; kk < old_n; ++kk) {
    bwtintv_t *p = &mem.a[kk];
    int start = p->info >> 32, end = (int32_t)p->info;
    if (end - start < split_len || p->x[2] > 10) continue;
    bwt_smem1(bwt, len, seq, (start + end) >> 1, p->x[2] + 1, &mem1, tmpv);
    for (i = 0; i < (int)mem1.n; ++i)
      if ((uint32_t)mem1.a[i].info - (mem1.a[i].info >> 32) >= (uint32_t)min_seed_len)
        kv_push(bwtintv_t, mem, mem1.a[i]);
  }
  x = 0;
  while (x < len) {
    if (seq[x] < 4) {
      bwtintv_t mm;
      x = bwt_seed_strategy1(bwt, len, seq, x, min_seed_len, 20, &mm);
      if (mm.x[2] > 0) kv_push(bwtintv_t, mem, mm);
    } else
      ++x;
  }
  int64_t cnt = (int64_t)mem.n;
  if (cnt <= cap) {
    for (int64_t q = 0; q < cnt; q++) {
      k[q] = (int64_t)mem.a[q].x[0];
      l[q] = (int64_t)mem.a[q].x[1];
      s[q] = (int64_t)mem.a[q].x[2];
      m[q] = (int32_t)(mem.a[q].info >> 32);
      n[q] = (int32_t)((uint32_t)mem.a[q].info) - 1;
    }
  } else {
    cnt = -1;
  }
  free(mem.a);
  free(mem1.a);
  free(t0.a);
  free(t1.a);
  return cnt;
}

/* Banded SW extension: bwa v1 ksw_extend2 (tools/bwa/ksw.c:380-481), the function the bsw
 * benchmark's scalarBandedSWA (benchmarks/bsw/bandedSWA.cpp:130-251) restates. ksw.c is compiled
 * with -DNDEBUG so its h0 > 0 assert is off, matching the benchmark (bandedSWA.cpp:139).
 * Same flattened layout as bsw_oracle_batch; out6 = {score, qle, tle, gtle, gscore, max_off}. */
int ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle, int *gscore,
                int *max_off);

void ref_bwa_ksw_batch(int64_t n, const uint8_t *tgt, const int64_t *toff, const int32_t *tlen,
                       const uint8_t *qry, const int64_t *qoff, const int32_t *qlen,
                       const int32_t *h0, const int8_t *mat, const int32_t *params, int32_t *out) {
  for (int64_t p = 0; p < n; ++p) {
    int32_t *o = out + 6 * p;
    o[0] = ksw_extend2(qlen[p], qry + qoff[p], tlen[p], tgt + toff[p], 5, mat, params[0],
                       params[1], params[2], params[3], params[6], params[5], params[4], h0[p],
                       &o[1], &o[2], &o[3], &o[4], &o[5]);
  }
}

/* A bwa v1 bwt_t over the BWT of a bwa-mem2 .bwt.2bit.64 index (its CP_OCC one-hot words, rows 0..n-1,
 * one row without a base = the sentinel): the $-removed BWT packed 16 bases per word the way
 * bwt_B00 reads it, then bwa's own bwt_bwtupdate_core (tools/bwa/bwtindex.c:151) interleaves the
 * occurrence counts and bwt_gen_cnt_table (bwt.c:42) fills the popcount table. Row numbering is
 * unchanged (bwa v1's primary = the sentinel row), so intervals compare directly. */
void *ref_bwa_from_cp_occ(const int64_t *cp_occ, int64_t n, int64_t sentinel) {
  bwt_t *bwt = (bwt_t *)calloc(1, sizeof(bwt_t));
  bwtint_t seq_len = (bwtint_t)(n - 1), c[4] = {0, 0, 0, 0};
  bwt->primary = (bwtint_t)sentinel;
  bwt->seq_len = seq_len;
  bwt->bwt_size = (seq_len + 15) >> 4;
  /* word-level packing (a human-scale index has 6.4 G rows): per 64-row line the code bits
   * hi = G|T, lo = C|T, interleaved MSB-first into two 64-bit words = four bwt words of 16 bases;
   * the sentinel row (code 0 here) is then cut out by shifting the rest of the array left by one
   * base. Equal to the row-by-row packing (tests/test_fmi_oracle.py). */
  const int64_t nlines = (n + 63) >> 6, nw = nlines * 4 + 2;
  uint32_t *w = (uint32_t *)calloc((size_t)nw, 4);
  for (int64_t ln = 0; ln < nlines; ln++) {
    const uint64_t *line = (const uint64_t *)(cp_occ + ln * 8);
    uint64_t valid = ~0ull;
    if ((ln << 6) + 64 > n) valid = ~0ull << (64 - (n - (ln << 6)));
    const uint64_t m1 = line[5] & valid, m2 = line[6] & valid, m3 = line[7] & valid;
    const uint64_t hi = m2 | m3, lo = m1 | m3;
    for (int half = 0; half < 2; half++) {
      /* 32 rows: bits 63..32 (half 0) or 31..0 (half 1) of hi / lo, row order MSB-first */
      uint64_t h = (hi >> (32 * (1 - half))) & 0xffffffffull, l = (lo >> (32 * (1 - half))) & 0xffffffffull;
      /* spread 32 bits to the even positions of 64 */
      h = (h | (h << 16)) & 0x0000FFFF0000FFFFull; h = (h | (h << 8)) & 0x00FF00FF00FF00FFull;
      h = (h | (h << 4)) & 0x0F0F0F0F0F0F0F0Full; h = (h | (h << 2)) & 0x3333333333333333ull;
      h = (h | (h << 1)) & 0x5555555555555555ull;
      l = (l | (l << 16)) & 0x0000FFFF0000FFFFull; l = (l | (l << 8)) & 0x00FF00FF00FF00FFull;
      l = (l | (l << 4)) & 0x0F0F0F0F0F0F0F0Full; l = (l | (l << 2)) & 0x3333333333333333ull;
      l = (l | (l << 1)) & 0x5555555555555555ull;
      const uint64_t v = (h << 1) | l; /* row 32*half + j at bits 63-2j, 62-2j */
      w[ln * 4 + 2 * half] = (uint32_t)(v >> 32);
      w[ln * 4 + 2 * half + 1] = (uint32_t)v;
    }
    c[1] += (uint64_t)__builtin_popcountll(m1 & ~m2 & ~m3);
    c[2] += (uint64_t)__builtin_popcountll(m2 & ~m3);
    c[3] += (uint64_t)__builtin_popcountll(m3);
  }
  c[0] = (bwtint_t)(n - 1) - c[1] - c[2] - c[3];
  /* drop the sentinel's base: every base after it moves one place (2 bits) towards the front */
  {
    const int64_t wk = sentinel >> 4;
    const int sh = (int)(sentinel & 15);
    const uint32_t keep = sh ? ~0u << (32 - 2 * sh) : 0u; /* bases before the sentinel in its word */
    uint32_t cur = w[wk];
    w[wk] = (cur & keep) | ((cur << 2) & ~keep) | (w[wk + 1] >> 30);
    for (int64_t k = wk + 1; k + 1 < nw; k++) w[k] = (w[k] << 2) | (w[k + 1] >> 30);
  }
  bwt->bwt = (uint32_t *)calloc(bwt->bwt_size, 4);
  memcpy(bwt->bwt, w, (size_t)bwt->bwt_size * 4);
  free(w);
  /* the row-by-row form this replaces left every bit past seq_len zero */
  if (seq_len & 15) bwt->bwt[bwt->bwt_size - 1] &= ~0u << (32 - 2 * (seq_len & 15));
  bwt->L2[0] = 0;
  for (int x = 0; x < 4; x++) bwt->L2[x + 1] = bwt->L2[x] + c[x];
  bwt_bwtupdate_core(bwt);
  bwt_gen_cnt_table(bwt);
  return bwt;
}

/* mem_collect_intv (above) over reads [0, nreads) of a row-major code matrix; returns the total
 * number of intervals (or -1 when a read overflows `cap`). One call per host thread. */
int64_t ref_bwa_collect_batch(void *bwtp, const uint8_t *codes, const int32_t *lens, int64_t nreads,
                              int64_t stride, int min_seed_len) {
  const int64_t cap = 1 << 14;
  int64_t *k = (int64_t *)malloc(cap * 8), *l = (int64_t *)malloc(cap * 8), *s = (int64_t *)malloc(cap * 8);
  int32_t *m = (int32_t *)malloc(cap * 4), *nn = (int32_t *)malloc(cap * 4);
  int64_t tot = 0;
  for (int64_t r = 0; r < nreads && tot >= 0; r++) {
    int64_t c = ref_bwa_collect(bwtp, codes + r * stride, lens[r], min_seed_len, k, l, s, m, nn, cap);
    tot = c < 0 ? -1 : tot + c;
  }
  free(k); free(l); free(s); free(m); free(nn);
  return tot;
}
