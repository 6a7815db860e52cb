/*
 * oracle/fmi_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU checker, never the product path).
 *
 * Plain-C restatement of bwa-mem2's FM-index SMEM search exactly as the reference's fmi benchmark
 * runs it (the Palisade HE layer is numerically an identity), used by tests/,
 * bench.py's cpu_baseline leg (kind "port") and __graft_entry__.smoke() as the parity checker.
 * The reference FMI_search.cpp cannot be compiled here without stand-in Palisade headers (forbidden),
 * so parity of this restatement is cross-checked against bwa v1's own SMEM code (tools/bwa/bwt.c,
 * built by oracle/Makefile into oracle/_ref/) -- see tests/test_fmi_oracle.py.
 *
 * Followed reference code (paths relative to /root/reference/tools/bwa-mem2/src):
 *   index build   FMI_search.cpp:109-169 (pac2nt: forward + reverse complement text),
 *                 :358-434 (build_index: counts, SA of the text, SA[0] = n),
 *                 :171-356 (build_fm_index: BWT, CP_OCC every 64 rows, one-hot MSB-first, file)
 *   index load    FMI_search.cpp:469-984 (file layout; count[i] += 1 at :763-768;
 *                 one_hot_mask_array :473-481; sentinel_index from the file :923)
 *   Occ           FMI_search.h:81-89 (GET_OCC)
 *   backwardExt   FMI_search.cpp:1536-1565
 *   SMEM search   FMI_search.cpp:986-1180 (getSMEMsOnePosOneThread), :1182-1241 (AllPos),
 *                 :1243-1326 (bwtSeedStrategyAllPosOneThread), :1499-1534 (compare_smem, sortSMEMs)
 *   batch driver  benchmarks/fmi/fmi.cpp:239-348 (smem1, reseed with split_len/splitWidth, LAST with
 *                 maxMemIntv=20 and minSeedLen+1, rid offset, per-batch sort)
 *   SA lookup     FMI_search.cpp:1714-1807 (get_sa_entry_compressed: LF walk to a sampled row),
 *                 :1834-1893 (call_one_step) and :1895-2040 (get_sa_entries_prefetch, the variant
 *                 bwamem.cpp:737 calls), max_occ sampling of an SMEM's interval as in :1596-1619
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CP_BLOCK 64
#define CP_SHIFT 6
#define CP_MASK 63
#define SA_COMPX 3

typedef struct {
  int64_t cp_count[4];
  uint64_t one_hot_bwt_str[4];
} or_cp_occ; /* CP_OCC, FMI_search.h:59-63 */

typedef struct {
  uint32_t rid, m, n;
  int64_t k, l, s;
} or_smem; /* SMEM, FMI_search.h:91-99 (non-DEBUG layout, 40 bytes) */

typedef struct {
  int64_t n;        /* reference_seq_len in the file = |text| + 1 */
  int64_t count[5]; /* after the load-time +1 */
  int64_t sentinel_index;
  or_cp_occ *cp_occ;
  int64_t cp_occ_size;
  uint64_t one_hot_mask[64];
  int64_t bwt_calls; /* backwardExt counter (work accounting for the roofline) */
  int64_t sa_ns;     /* sampled SA (every 8th row): (n >> SA_COMPX) + 1 entries, or 0 */
  int8_t *sa_ms_byte;
  uint32_t *sa_ls_word;
  int64_t lf_steps;  /* SA-lookup LF steps (work accounting) */
  const int64_t *sa64; /* adopted packed samples (sa_ms_byte << 32 + sa_ls_word), or NULL */
} or_fmi;

/* ------------------------------------------------------------------------------------------ */
/* Suffix array of a small text (prefix doubling with radix sort; test-sized inputs only).     */
/* Suffix order = lexicographic with end-of-text smallest, i.e. that of saisxx over the text. */
/* ------------------------------------------------------------------------------------------ */
static void radix_by(int64_t *sa, int64_t *tmp, const int64_t *key, int64_t n, int64_t nkeys) {
  int64_t *cnt = (int64_t *)calloc((size_t)nkeys + 1, sizeof(int64_t));
  for (int64_t i = 0; i < n; i++) cnt[key[sa[i]] + 1]++;
  for (int64_t i = 0; i < nkeys; i++) cnt[i + 1] += cnt[i];
  for (int64_t i = 0; i < n; i++) tmp[cnt[key[sa[i]]]++] = sa[i];
  memcpy(sa, tmp, (size_t)n * sizeof(int64_t));
  free(cnt);
}

static void suffix_array(const uint8_t *t, int64_t n, int64_t *sa) {
  int64_t *rank = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
  int64_t *rank2 = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
  int64_t *tmp = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
  int64_t *key2 = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
  for (int64_t i = 0; i < n; i++) {
    sa[i] = i;
    rank[i] = t[i] + 1;
  }
  int64_t maxr = 5;
  for (int64_t h = 1;; h <<= 1) {
    for (int64_t i = 0; i < n; i++) key2[i] = (i + h < n) ? rank[i + h] : 0;
    radix_by(sa, tmp, key2, n, maxr + 1);
    radix_by(sa, tmp, rank, n, maxr + 1);
    int64_t r = 1;
    rank2[sa[0]] = 1;
    for (int64_t i = 1; i < n; i++) {
      int64_t a = sa[i - 1], b = sa[i];
      if (rank[a] != rank[b] || key2[a] != key2[b]) r++;
      rank2[b] = r;
    }
    memcpy(rank, rank2, (size_t)n * sizeof(int64_t));
    maxr = r;
    if (r == n) break;
  }
  free(rank);
  free(rank2);
  free(tmp);
  free(key2);
}

/* Build the .bwt.2bit.64 content from forward-strand codes (0..3 = A,C,G,T) exactly like
 * build_index + build_fm_index. Writes the file when path != NULL. Fills *idx like load_index. */
int fmi_oracle_build(const uint8_t *ref, int64_t ref_len, const char *path, or_fmi *idx) {
  const int64_t pac_len = 2 * ref_len;
  uint8_t *text = (uint8_t *)malloc((size_t)pac_len);
  memcpy(text, ref, (size_t)ref_len);
  for (int64_t i = 0; i < ref_len; i++) text[ref_len + i] = (uint8_t)(3 - ref[ref_len - 1 - i]);
  int64_t count[5] = {0, 0, 0, 0, 0}, c4[4] = {0, 0, 0, 0};
  for (int64_t i = 0; i < pac_len; i++) c4[text[i]]++;
  count[4] = c4[0] + c4[1] + c4[2] + c4[3];
  count[3] = c4[0] + c4[1] + c4[2];
  count[2] = c4[0] + c4[1];
  count[1] = c4[0];
  count[0] = 0;
  int64_t *sa = (int64_t *)malloc((size_t)(pac_len + 2) * sizeof(int64_t));
  suffix_array(text, pac_len, sa + 1);
  sa[0] = pac_len;
  const int64_t n = pac_len + 1; /* ref_seq_len++ (build_fm_index) */
  const int64_t n_al = ((n + CP_BLOCK - 1) / CP_BLOCK) * CP_BLOCK;
  uint8_t *bwt = (uint8_t *)malloc((size_t)n_al);
  int64_t sentinel = -1;
  for (int64_t i = 0; i < n; i++) {
    if (sa[i] == 0) {
      bwt[i] = 4;
      sentinel = i;
    } else {
      bwt[i] = text[sa[i] - 1];
    }
  }
  for (int64_t i = n; i < n_al; i++) bwt[i] = 6; /* DUMMY_CHAR */
  const int64_t cp_size = (n >> CP_SHIFT) + 1;
  or_cp_occ *cp = (or_cp_occ *)calloc((size_t)cp_size, sizeof(or_cp_occ));
  int64_t cc[16] = {0};
  for (int64_t i = 0; i < n; i++) {
    if ((i & CP_MASK) == 0) {
      or_cp_occ o;
      for (int b = 0; b < 4; b++) {
        o.cp_count[b] = cc[b];
        o.one_hot_bwt_str[b] = 0;
      }
      for (int j = 0; j < CP_BLOCK; j++) {
        for (int b = 0; b < 4; b++) o.one_hot_bwt_str[b] <<= 1;
        uint8_t c = bwt[i + j];
        if (c < 4) o.one_hot_bwt_str[c] += 1;
      }
      cp[i >> CP_SHIFT] = o;
    }
    cc[bwt[i]]++;
  }
  const int64_t ns = (n >> SA_COMPX) + 1;
  int8_t *ms = (int8_t *)calloc((size_t)ns, 1);
  uint32_t *ls = (uint32_t *)calloc((size_t)ns, 4);
  for (int64_t i = 0, pos = 0; i < n; i++)
    if ((i & ((1 << SA_COMPX) - 1)) == 0) {
      ls[pos] = (uint32_t)(sa[i] & 0xffffffff);
      ms[pos] = (int8_t)((sa[i] >> 32) & 0xff);
      pos++;
    }
  if (path) {
    FILE *fp = fopen(path, "wb");
    if (!fp) return -1;
    fwrite(&n, sizeof(int64_t), 1, fp);
    fwrite(count, sizeof(int64_t), 5, fp);
    fwrite(cp, sizeof(or_cp_occ), (size_t)cp_size, fp);
    fwrite(ms, 1, (size_t)ns, fp);
    fwrite(ls, 4, (size_t)ns, fp);
    fwrite(&sentinel, sizeof(int64_t), 1, fp);
    fclose(fp);
  }
  if (idx) {
    idx->n = n;
    for (int b = 0; b < 5; b++) idx->count[b] = count[b] + 1;
    idx->sentinel_index = sentinel;
    idx->cp_occ = cp;
    idx->cp_occ_size = cp_size;
    idx->bwt_calls = 0;
    idx->one_hot_mask[0] = 0;
    idx->one_hot_mask[1] = 0x8000000000000000ull;
    for (int i = 2; i < 64; i++) idx->one_hot_mask[i] = (idx->one_hot_mask[i - 1] >> 1) | 0x8000000000000000ull;
    idx->sa_ns = ns;
    idx->sa_ms_byte = ms;
    idx->sa_ls_word = ls;
    idx->lf_steps = 0;
  } else {
    free(cp);
    free(ms);
    free(ls);
  }
  free(bwt);
  free(sa);
  free(text);
  return 0;
}

/* load_index (FMI_search.cpp:469-984), the fields the SMEM search reads. */
int fmi_oracle_load(const char *path, or_fmi *idx) {
  FILE *fp = fopen(path, "rb");
  if (!fp) return -1;
  int64_t n, count[5];
  if (fread(&n, 8, 1, fp) != 1 || fread(count, 8, 5, fp) != 5) return -2;
  const int64_t cp_size = (n >> CP_SHIFT) + 1;
  or_cp_occ *cp = (or_cp_occ *)malloc((size_t)cp_size * sizeof(or_cp_occ));
  if (fread(cp, sizeof(or_cp_occ), (size_t)cp_size, fp) != (size_t)cp_size) return -3;
  const int64_t ns = (n >> SA_COMPX) + 1;
  int8_t *ms = (int8_t *)malloc((size_t)ns);
  uint32_t *ls = (uint32_t *)malloc((size_t)ns * 4);
  if (fread(ms, 1, (size_t)ns, fp) != (size_t)ns || fread(ls, 4, (size_t)ns, fp) != (size_t)ns) return -4;
  int64_t sentinel;
  if (fread(&sentinel, 8, 1, fp) != 1) return -5;
  fclose(fp);
  idx->n = n;
  for (int b = 0; b < 5; b++) idx->count[b] = count[b] + 1;
  idx->sentinel_index = sentinel;
  idx->cp_occ = cp;
  idx->cp_occ_size = cp_size;
  idx->bwt_calls = 0;
  idx->one_hot_mask[0] = 0;
  idx->one_hot_mask[1] = 0x8000000000000000ull;
  for (int i = 2; i < 64; i++) idx->one_hot_mask[i] = (idx->one_hot_mask[i - 1] >> 1) | 0x8000000000000000ull;
  idx->sa_ns = ns;
  idx->sa_ms_byte = ms;
  idx->sa_ls_word = ls;
  idx->lf_steps = 0;
  return 0;
}

/* Adopt tables produced elsewhere (e.g. the product's GPU builder, whose output is tested
 * bit-identical to fmi_oracle_build's): count5 as stored in the file (before the +1). The caller keeps
 * cp_occ alive; fmi_oracle_free must not be called on such a handle. */
void fmi_oracle_adopt(or_fmi *idx, int64_t n, const int64_t *count5_file, int64_t sentinel, void *cp_occ) {
  idx->n = n;
  for (int b = 0; b < 5; b++) idx->count[b] = count5_file[b] + 1;
  idx->sentinel_index = sentinel;
  idx->cp_occ = (or_cp_occ *)cp_occ;
  idx->cp_occ_size = (n >> CP_SHIFT) + 1;
  idx->bwt_calls = 0;
  idx->one_hot_mask[0] = 0;
  idx->one_hot_mask[1] = 0x8000000000000000ull;
  for (int i = 2; i < 64; i++) idx->one_hot_mask[i] = (idx->one_hot_mask[i - 1] >> 1) | 0x8000000000000000ull;
}

/* Adopt packed sampled-SA entries produced elsewhere (caller keeps them alive). */
void fmi_oracle_adopt_sa64(or_fmi *idx, int64_t ns, const int64_t *sa64) {
  idx->sa_ns = ns;
  idx->sa64 = sa64;
}

void fmi_oracle_free(or_fmi *idx) {
  free(idx->cp_occ);
  free(idx->sa_ms_byte);
  free(idx->sa_ls_word);
  idx->cp_occ = NULL;
  idx->sa_ms_byte = NULL;
  idx->sa_ls_word = NULL;
}

static inline int64_t get_occ(const or_fmi *f, int64_t pp, int c) {
  int64_t occ_id = pp >> CP_SHIFT, y = pp & CP_MASK;
  int64_t occ = f->cp_occ[occ_id].cp_count[c];
  uint64_t m = f->cp_occ[occ_id].one_hot_bwt_str[c] & f->one_hot_mask[y];
  return occ + __builtin_popcountll(m);
}

/* backwardExt, FMI_search.cpp:1536-1565 */
static or_smem backward_ext(or_fmi *f, or_smem smem, uint8_t a) {
  int64_t k[4], l[4], s[4];
  f->bwt_calls++;
  for (int b = 0; b < 4; b++) {
    int64_t sp = smem.k, ep = smem.k + smem.s;
    int64_t occ_sp = get_occ(f, sp, b), occ_ep = get_occ(f, ep, b);
    k[b] = f->count[b] + occ_sp;
    s[b] = occ_ep - occ_sp;
  }
  int64_t sentinel_offset = 0;
  if (smem.k <= f->sentinel_index && (smem.k + smem.s) > f->sentinel_index) sentinel_offset = 1;
  l[3] = smem.l + sentinel_offset;
  l[2] = l[3] + s[3];
  l[1] = l[2] + s[2];
  l[0] = l[1] + s[1];
  smem.k = k[a];
  smem.l = l[a];
  smem.s = s[a];
  return smem;
}

static or_smem forward_ext(or_fmi *f, or_smem smem, uint8_t a) {
  or_smem t = smem;
  t.k = smem.l;
  t.l = smem.k;
  or_smem r = backward_ext(f, t, (uint8_t)(3 - a));
  or_smem o = r;
  o.k = r.l;
  o.l = r.k;
  return o;
}

/* getSMEMsOnePosOneThread, FMI_search.cpp:986-1180. prev: scratch of max_readlength entries. */
static void smems_one_pos(or_fmi *f, const uint8_t *enc_qdb, int16_t *query_pos, const int32_t *min_intv,
                          const int32_t *rid_array, int32_t num, const int32_t *lens, const int32_t *cum,
                          int32_t minSeedLen, or_smem *match, int64_t *ntot, or_smem *prev) {
  int64_t nt = *ntot;
  for (int32_t i = 0; i < num; i++) {
    int x = query_pos[i];
    int32_t rid = rid_array[i];
    int next_x = x + 1;
    int readlength = lens[rid];
    int offset = cum[rid];
    uint8_t a = enc_qdb[offset + x];
    if (a < 4) {
      or_smem smem;
      smem.rid = (uint32_t)rid;
      smem.m = (uint32_t)x;
      smem.n = (uint32_t)x;
      smem.k = f->count[a];
      smem.l = f->count[3 - a];
      smem.s = f->count[a + 1] - f->count[a];
      int numPrev = 0;
      int j;
      for (j = x + 1; j < readlength; j++) {
        a = enc_qdb[offset + j];
        next_x = j + 1;
        if (a < 4) {
          or_smem ns = forward_ext(f, smem, a);
          ns.n = (uint32_t)j;
          int32_t s_neq = ns.s != smem.s;
          prev[numPrev] = smem;
          numPrev += s_neq;
          if (ns.s < min_intv[i]) {
            next_x = j;
            break;
          }
          smem = ns;
        } else {
          break;
        }
      }
      if (smem.s >= min_intv[i]) {
        prev[numPrev] = smem;
        numPrev++;
      }
      for (int p = 0; p < numPrev / 2; p++) {
        or_smem t = prev[p];
        prev[p] = prev[numPrev - p - 1];
        prev[numPrev - p - 1] = t;
      }
      for (j = x - 1; j >= 0; j--) {
        int numCurr = 0;
        int curr_s = -1; /* int, as in the reference: assigned from int64 (truncating) */
        a = enc_qdb[offset + j];
        if (a > 3) break;
        int p;
        for (p = 0; p < numPrev; p++) {
          or_smem sm = prev[p];
          or_smem ns = backward_ext(f, sm, a);
          ns.m = (uint32_t)j;
          if ((ns.s < min_intv[i]) && ((sm.n - sm.m + 1) >= (uint32_t)minSeedLen)) {
            match[nt++] = sm;
            break;
          }
          if ((ns.s >= min_intv[i]) && (ns.s != curr_s)) {
            curr_s = (int)ns.s;
            prev[numCurr++] = ns;
            break;
          }
        }
        p++;
        for (; p < numPrev; p++) {
          or_smem sm = prev[p];
          or_smem ns = backward_ext(f, sm, a);
          ns.m = (uint32_t)j;
          if ((ns.s >= min_intv[i]) && (ns.s != curr_s)) {
            curr_s = (int)ns.s;
            prev[numCurr++] = ns;
          }
        }
        numPrev = numCurr;
        if (numCurr == 0) break;
      }
      if (numPrev != 0) {
        or_smem sm = prev[0];
        if ((sm.n - sm.m + 1) >= (uint32_t)minSeedLen) match[nt++] = sm;
        numPrev = 0;
      }
    }
    query_pos[i] = (int16_t)next_x;
  }
  *ntot = nt;
}

/* getSMEMsAllPosOneThread, FMI_search.cpp:1182-1241 */
static void smems_all_pos(or_fmi *f, const uint8_t *enc_qdb, int32_t *min_intv, int32_t *rid_array,
                          int32_t numReads, const int32_t *lens, const int32_t *cum, int32_t minSeedLen,
                          or_smem *match, int64_t *ntot, or_smem *prev) {
  int16_t *qpos = (int16_t *)calloc((size_t)numReads + 1, sizeof(int16_t));
  int32_t numActive = numReads;
  *ntot = 0;
  do {
    int32_t tail = 0;
    for (int32_t head = 0; head < numActive; head++) {
      int readlength = lens[rid_array[head]];
      if (qpos[head] < readlength) {
        rid_array[tail] = rid_array[head];
        qpos[tail] = qpos[head];
        min_intv[tail] = min_intv[head];
        tail++;
      }
    }
    smems_one_pos(f, enc_qdb, qpos, min_intv, rid_array, tail, lens, cum, minSeedLen, match, ntot, prev);
    numActive = tail;
  } while (numActive > 0);
  free(qpos);
}

/* bwtSeedStrategyAllPosOneThread, FMI_search.cpp:1243-1326 */
static int64_t seed_strategy(or_fmi *f, const uint8_t *enc_qdb, const int32_t *max_intv, int32_t numReads,
                             const int32_t *lens, const int32_t *cum, int32_t minSeedLen, or_smem *match) {
  int64_t nt = 0;
  for (int32_t i = 0; i < numReads; i++) {
    int readlength = lens[i];
    int16_t x = 0;
    while (x < readlength) {
      int next_x = x + 1;
      or_smem smem;
      smem.rid = (uint32_t)i;
      smem.m = (uint32_t)x;
      smem.n = (uint32_t)x;
      int offset = cum[i];
      uint8_t a = enc_qdb[offset + x];
      if (a < 4) {
        smem.k = f->count[a];
        smem.l = f->count[3 - a];
        smem.s = f->count[a + 1] - f->count[a];
        for (int j = x + 1; j < readlength; j++) {
          next_x = j + 1;
          a = enc_qdb[offset + j];
          if (a < 4) {
            or_smem ns = forward_ext(f, smem, a);
            ns.n = (uint32_t)j;
            smem = ns;
            if ((smem.s < max_intv[i]) && ((smem.n - smem.m + 1) >= (uint32_t)minSeedLen)) {
              if (smem.s > 0) match[nt++] = smem;
              break;
            }
          } else {
            break;
          }
        }
      }
      x = (int16_t)next_x;
    }
  }
  return nt;
}

static int compare_smem(const void *a, const void *b) {
  const or_smem *pa = (const or_smem *)a, *pb = (const or_smem *)b;
  if (pa->rid < pb->rid) return -1;
  if (pa->rid > pb->rid) return 1;
  if (pa->m < pb->m) return -1;
  if (pa->m > pb->m) return 1;
  if (pa->n > pb->n) return -1;
  if (pa->n < pb->n) return 1;
  return 0;
}

/* The per-batch pipeline of benchmarks/fmi/fmi.cpp:253-348 for reads [0, numReads), batches of
 * batch_size. enc_qdb has stride max_readlength (fmi.cpp:141-177); lens[r] = read length.
 * out must hold numReads * (2*max_readlength + 8) SMEMs (returns -1 when it would overflow);
 * batch_counts[b] = numTotalSmem of batch b; phase_counts[3] += num_smem1/2/3.
 * Returns the total number of SMEMs (totalSmems, fmi.cpp:381). */
int64_t fmi_oracle_run(or_fmi *f, const uint8_t *enc_qdb, const int32_t *lens, int32_t numReads,
                       int32_t max_readlength, int32_t batch_size, int32_t minSeedLen, or_smem *out,
                       int64_t out_cap, int64_t *batch_counts, int64_t *phase_counts) {
  const int splitWidth = 10, maxMemIntv = 20;
  const double splitFactor = 1.5;
  const int split_len = (int)(minSeedLen * splitFactor + .499);
  int32_t *min_intv = (int32_t *)malloc((size_t)batch_size * 64 * sizeof(int32_t));
  int32_t *rid = (int32_t *)malloc((size_t)batch_size * 64 * sizeof(int32_t));
  int16_t *qpos = (int16_t *)malloc((size_t)batch_size * 64 * sizeof(int16_t));
  int32_t *cum = (int32_t *)malloc((size_t)batch_size * sizeof(int32_t));
  or_smem *prev = (or_smem *)malloc((size_t)(max_readlength + 1) * sizeof(or_smem));
  const int64_t per_batch_cap = (int64_t)batch_size * (8 * (int64_t)max_readlength + 64);
  or_smem *tmp = (or_smem *)malloc((size_t)per_batch_cap * sizeof(or_smem));
  int64_t total = 0;
  for (int32_t i = 0; i < numReads; i += batch_size) {
    int32_t bc = batch_size;
    if (i + bc > numReads) bc = numReads - i;
    for (int32_t j = 0; j < bc; j++) {
      min_intv[j] = 1;
      rid[j] = j;
      cum[j] = j * max_readlength;
    }
    const uint8_t *q = enc_qdb + (int64_t)i * max_readlength;
    const int32_t *bl = lens + i;
    int64_t n1 = 0, n2 = 0, n3 = 0;
    smems_all_pos(f, q, min_intv, rid, bc, bl, cum, minSeedLen, tmp, &n1, prev);
    int64_t pos = 0;
    for (int64_t j = 0; j < n1; j++) {
      or_smem *p = &tmp[j];
      int start = (int)p->m, end = (int)p->n + 1;
      if (end - start < split_len || p->s > splitWidth) continue;
      rid[pos] = (int32_t)p->rid;
      qpos[pos] = (int16_t)((end + start) >> 1);
      min_intv[pos] = (int32_t)(p->s + 1);
      pos++;
    }
    smems_one_pos(f, q, qpos, min_intv, rid, (int32_t)pos, bl, cum, minSeedLen, tmp + n1, &n2, prev);
    for (int32_t j = 0; j < bc; j++) min_intv[j] = maxMemIntv;
    n3 = seed_strategy(f, q, min_intv, bc, bl, cum, minSeedLen + 1, tmp + n1 + n2);
    int64_t tot = n1 + n2 + n3;
    for (int64_t j = 0; j < tot; j++) tmp[j].rid += (uint32_t)i;
    qsort(tmp, (size_t)tot, sizeof(or_smem), compare_smem);
    if (total + tot > out_cap) {
      total = -1;
      break;
    }
    memcpy(out + total, tmp, (size_t)tot * sizeof(or_smem));
    total += tot;
    if (batch_counts) batch_counts[i / batch_size] = tot;
    if (phase_counts) {
      phase_counts[0] += n1;
      phase_counts[1] += n2;
      phase_counts[2] += n3;
    }
  }
  free(min_intv);
  free(rid);
  free(qpos);
  free(cum);
  free(prev);
  free(tmp);
  return total;
}

/* One phase of the class API in the reference's own emission order (test infrastructure for the
 * FMI_search method adapter): phase 0 getSMEMsAllPosOneThread (rid/intv compacted in place like the
 * reference), 1 getSMEMsOnePosOneThread (qpos updated in place), 2 bwtSeedStrategyAllPosOneThread
 * (intv = max_intv, reads 0..num-1). Returns the number of SMEMs written to out. */
int64_t fmi_oracle_phase(or_fmi *f, int phase, const uint8_t *qdb, const int32_t *lens, const int32_t *cum,
                         int16_t *qpos, int32_t *intv, int32_t *rid, int32_t num, int32_t max_readlength,
                         int32_t minSeedLen, or_smem *out) {
  or_smem *prev = (or_smem *)malloc((size_t)(max_readlength + 1) * sizeof(or_smem));
  int64_t nt = 0;
  if (phase == 0)
    smems_all_pos(f, qdb, intv, rid, num, lens, cum, minSeedLen, out, &nt, prev);
  else if (phase == 1)
    smems_one_pos(f, qdb, qpos, intv, rid, num, lens, cum, minSeedLen, out, &nt, prev);
  else
    nt = seed_strategy(f, qdb, intv, num, lens, cum, minSeedLen, out);
  free(prev);
  return nt;
}

/* FMI_search::getSMEMs, FMI_search.cpp:1328-1497: right-to-left SMEMs over fixed-stride reads.
 * Restated with the reference's quirks, which are its behaviour: the OpenMP region is commented out
 * (tid = 0), so only the first ceil(numReads / nthreads) reads are searched and only numTotalSmem[0]
 * is written; myPrevArray and myCurrArray are the same buffer (:1345-1346), which the backward loop
 * uses as in-place compaction (a write never overtakes the entry being read); a forward extension
 * stopped by an N pushes the current SMEM twice (:1394-1401). prev needs readlength + 2 entries. */
void fmi_oracle_get_smems(or_fmi *f, const uint8_t *enc_qdb, int32_t numReads, int32_t readlength,
                          int32_t minSeedLen, int32_t nthreads, or_smem *matchArray, int64_t *numTotalSmem) {
  or_smem *prev = (or_smem *)malloc((size_t)(readlength + 2) * sizeof(or_smem));
  numTotalSmem[0] = 0;
  int32_t quota = (numReads + (nthreads - 1)) / nthreads;
  int32_t last = quota > numReads ? numReads : quota;
  for (int32_t i = 0; i < last; i++) {
    const uint8_t *q = enc_qdb + (int64_t)i * readlength;
    int x = readlength - 1, numPrev = 0, numSmem = 0;
    while (x >= 0) {
      uint8_t a = q[x];
      if (a > 3) {
        x--;
        continue;
      }
      or_smem smem;
      smem.rid = (uint32_t)i;
      smem.m = smem.n = (uint32_t)x;
      smem.k = f->count[a];
      smem.l = f->count[3 - a];
      smem.s = f->count[a + 1] - f->count[a];
      int j;
      for (j = x + 1; j < readlength; j++) {
        a = q[j];
        if (a < 4) {
          or_smem ns = forward_ext(f, smem, a);
          ns.n = (uint32_t)j;
          if (ns.s != smem.s) prev[numPrev++] = smem;
          smem = ns;
          if (ns.s == 0) break;
        } else {
          prev[numPrev++] = smem;
          break;
        }
      }
      if (smem.s != 0) prev[numPrev++] = smem;
      for (int p = 0; p < numPrev / 2; p++) {
        or_smem t = prev[p];
        prev[p] = prev[numPrev - p - 1];
        prev[numPrev - p - 1] = t;
      }
      int next_x = x - 1, cur_j = readlength;
      for (j = x - 1; j >= 0; j--) {
        int numCurr = 0, curr_s = -1;
        a = q[j];
        if (a > 3) {
          next_x = j - 1;
          break;
        }
        for (int p = 0; p < numPrev; p++) {
          or_smem sm = prev[p];
          or_smem ns = backward_ext(f, sm, a);
          ns.m = (uint32_t)j;
          if (ns.s == 0 && numCurr == 0 && j < cur_j) {
            cur_j = j;
            if ((sm.n - sm.m + 1) >= (uint32_t)minSeedLen) matchArray[numTotalSmem[0] + numSmem++] = sm;
          }
          if (ns.s != 0 && ns.s != curr_s) {
            curr_s = (int)ns.s;
            prev[numCurr++] = ns;
          }
        }
        numPrev = numCurr;
        if (numCurr == 0) {
          next_x = j;
          break;
        }
        next_x = j - 1;
      }
      if (numPrev != 0) {
        or_smem sm = prev[0];
        if ((sm.n - sm.m + 1) >= (uint32_t)minSeedLen) matchArray[numTotalSmem[0] + numSmem++] = sm;
        numPrev = 0;
      }
      x = next_x;
    }
    numTotalSmem[0] += numSmem;
  }
  free(prev);
}

/* ctypes-friendly handle API */
or_fmi *fmi_oracle_new(void) { return (or_fmi *)calloc(1, sizeof(or_fmi)); }
void fmi_oracle_delete(or_fmi *f) {
  if (f) {
    fmi_oracle_free(f);
    free(f);
  }
}
int64_t fmi_oracle_bwt_calls(const or_fmi *f) { return f->bwt_calls; }
/* A second handle over the same CP_OCC table (own work counter) for multi-threaded CPU runs. */
or_fmi *fmi_oracle_share(const or_fmi *f) {
  or_fmi *g = (or_fmi *)malloc(sizeof(or_fmi));
  *g = *f;
  g->bwt_calls = 0;
  g->lf_steps = 0;
  return g;
}
void fmi_oracle_unshare(or_fmi *g) { free(g); }
void fmi_oracle_info(const or_fmi *f, int64_t *n, int64_t *count5, int64_t *sentinel) {
  *n = f->n;
  for (int b = 0; b < 5; b++) count5[b] = f->count[b];
  *sentinel = f->sentinel_index;
}
const void *fmi_oracle_cp_occ(const or_fmi *f, int64_t *size) {
  *size = f->cp_occ_size;
  return f->cp_occ;
}

/* ------------------------------------------------------------------------------------------ */
/* SA lookup                                                                                   */
/* ------------------------------------------------------------------------------------------ */
static inline int64_t sa_sample(const or_fmi *f, int64_t sp) {
  if (f->sa64) return f->sa64[sp >> SA_COMPX];
  int64_t e = f->sa_ms_byte[sp >> SA_COMPX];
  return (e << 32) + f->sa_ls_word[sp >> SA_COMPX];
}

/* mode 0: get_sa_entry_compressed (FMI_search.cpp:1714-1807): walk LF from row pos until a sampled
 * row (pos % 8 == 0) and add the number of steps; reaching the sentinel row ('$' in the BWT, no base
 * bit in CP_OCC) returns the step count (SA[sentinel row] = 0).
 * mode 1: call_one_step repeated as get_sa_entries_prefetch does (:1834-1893, :1965-2035): identical
 * except that reaching the sentinel row yields 0 whatever the step count (:1865-1869). */
int64_t fmi_oracle_sa_entry(or_fmi *f, int64_t pos, int mode) {
  int64_t offset = 0, sp = pos;
  while (sp & ((1 << SA_COMPX) - 1)) {
    const int64_t occ_id = sp >> CP_SHIFT, y = CP_BLOCK - (sp & CP_MASK) - 1;
    const uint64_t *oh = f->cp_occ[occ_id].one_hot_bwt_str;
    int b = 4;
    for (int c = 0; c < 4; c++)
      if ((oh[c] >> y) & 1) {
        b = c;
        break;
      }
    if (b == 4) return mode ? 0 : offset;
    sp = f->count[b] + get_occ(f, sp, b);
    offset++;
    f->lf_steps++;
  }
  return sa_sample(f, sp) + offset;
}

/* SA coordinates of every SMEM (FMI_search.cpp:1596-1619 / :1895-1931): for SMEM i, rows
 * j = k, k+step, ... (j < k+s, at most max_occ of them), step = s > max_occ ? s / max_occ : 1;
 * coords are concatenated in SMEM order, counts[i] = number for SMEM i. Returns the total. */
int64_t fmi_oracle_sa_entries(or_fmi *f, const or_smem *smems, int64_t n, int32_t max_occ, int mode,
                              int64_t *coords, int32_t *counts) {
  int64_t tot = 0;
  for (int64_t i = 0; i < n; i++) {
    const int64_t hi = smems[i].k + smems[i].s;
    const int64_t step = smems[i].s > max_occ ? smems[i].s / max_occ : 1;
    int32_t c = 0;
    for (int64_t j = smems[i].k; j < hi && c < max_occ; j += step, c++) coords[tot + c] = fmi_oracle_sa_entry(f, j, mode);
    if (counts) counts[i] = c;
    tot += c;
  }
  return tot;
}

void fmi_oracle_sa_lookup(or_fmi *f, const int64_t *rows, int64_t n, int mode, int64_t *out) {
  for (int64_t i = 0; i < n; i++) out[i] = fmi_oracle_sa_entry(f, rows[i], mode);
}
int64_t fmi_oracle_lf_steps(const or_fmi *f) { return f->lf_steps; }
