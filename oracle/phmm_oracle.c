/*
 * oracle/phmm_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU checker, never the product path).
 *
 * Plain-C restatement of the GKL PairHMM forward algorithm exactly as the reference computes it,
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the parity checker.
 * Parity is pinned against (a) the reference's own known-answer test
 * (tools/GKL/src/test/java/com/intel/gkl/pairhmm/PairHmmUnitTest.java:23-56, -0.6022797 +- 1e-5)
 * and (b) golden vectors produced by the reference kernels themselves (compute_fp_avxs/avxd,
 * built from /root/reference by oracle/Makefile into oracle/_ref/, see tests/golden/make_golden.py).
 *
 * Followed reference code (paths relative to /root/reference):
 *   tables     tools/GKL/src/main/native/pairhmm/Context.h:42-61 (jacobian, matchToMatch),
 *              :101-155 (ph2pr, INITIAL_CONSTANT, set_mm_prob), :67-90 (approximateLog10SumLog10)
 *   per-row    tools/GKL/src/main/native/pairhmm/avx-pairhmm-template.h:83-128 (initializeVectors),
 *              :150-160 (distm / 1-distm / distm/3)
 *   recurrence avx-pairhmm-template.h:183-198 (computeMXY) restated row-major; boundary rows from
 *              :93-98 and :160-177; result = sumM + sumX over the last row (:299-344)
 *   matching   pairhmm_common.h:26-45 (ConvertChar) + avx-pairhmm-template.h:3-35 (masks: N matches all)
 *   final      tools/GKL/src/main/native/pairhmm/IntelPairHmmCSource.cpp:61-85 (float, then double
 *              fallback below MIN_ACCEPTED=1e-28f, log10 minus LOG10_INITIAL_CONSTANT)
 *
 * Must be compiled with -ffp-contract=off (no FMA contraction; the reference never fuses).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_MAX_QUAL 254
#define OR_JAC_TOL 8.0
#define OR_JAC_STEP 0.0001
#define OR_JAC_INV_STEP (1.0 / OR_JAC_STEP)
#define OR_JAC_SIZE 80001 /* JACOBIAN_LOG_TABLE_SIZE = (int)(8.0 / 0.0001) + 1 (Context.h:10) */
#define OR_M2M_SIZE (((OR_MAX_QUAL + 1) * (OR_MAX_QUAL + 2)) >> 1)

typedef struct {
  int rslen, haplen;
  const char *q, *i, *d, *c;
  const char *hap, *rs;
} or_testcase; /* layout of testcase, pairhmm_common.h:20-24 */

static float jac_f[OR_JAC_SIZE];
static double jac_d[OR_JAC_SIZE];
static float m2m_f[OR_M2M_SIZE];
static double m2m_d[OR_M2M_SIZE];
static float ph2pr_f[128];
static double ph2pr_d[128];
static float init_f, log10_init_f;
static double init_d, log10_init_d;
static uint8_t conv[256];
static int inited = 0;

static int fast_round_f(float d) { return (d > 0.0f) ? (int)(d + 0.5f) : (int)(d - 0.5f); }
static int fast_round_d(double d) { return (d > 0.0) ? (int)(d + 0.5) : (int)(d - 0.5); }

/* Context.h:67-90 (NUMBER = float). std::isinf(x) == -1 is never true in C++ (bool), so omitted. */
static float log10sum_f(float small, float big) {
  if (small > big) { float t = big; big = small; small = t; }
  float diff = big - small;
  if (diff >= (float)OR_JAC_TOL) return big;
  int ind = fast_round_f((float)(diff * (float)OR_JAC_INV_STEP));
  return big + jac_f[ind];
}
static double log10sum_d(double small, double big) {
  if (small > big) { double t = big; big = small; small = t; }
  double diff = big - small;
  if (diff >= (double)OR_JAC_TOL) return big;
  int ind = fast_round_d((double)(diff * (double)OR_JAC_INV_STEP));
  return big + jac_d[ind];
}

void phmm_oracle_init(void) {
  if (inited) return;
  for (int k = 0; k < OR_JAC_SIZE; k++) {
    double v = log10(1.0 + pow(10.0, -((double)k) * OR_JAC_STEP));
    jac_f[k] = (float)v;
    jac_d[k] = v;
  }
  double LN10 = log(10);
  double INV_LN10 = 1.0 / LN10;
  for (int i = 0, offset = 0; i <= OR_MAX_QUAL; offset += ++i)
    for (int j = 0; j <= i; j++) {
      /* float context: arguments are narrowed to float at the call (Context.h:56) */
      double s_f = log10sum_f((float)(-0.1 * i), (float)(-0.1 * j));
      double l_f = log1p(-fmin(1.0, pow(10, s_f))) * INV_LN10;
      m2m_f[offset + j] = (float)(pow(10, l_f));
      double s_d = log10sum_d(-0.1 * i, -0.1 * j);
      double l_d = log1p(-fmin(1.0, pow(10, s_d))) * INV_LN10;
      m2m_d[offset + j] = pow(10, l_d);
    }
  for (int x = 0; x < 128; x++) {
    ph2pr_f[x] = powf(10.f, -((float)x) / 10.f);
    ph2pr_d[x] = pow(10.0, -((double)x) / 10.0);
  }
  init_f = ldexpf(1.f, 120);
  log10_init_f = log10f(init_f);
  init_d = ldexp(1.0, 1020);
  log10_init_d = log10(init_d);
  memset(conv, 0, sizeof(conv));
  conv['A'] = 0; conv['C'] = 1; conv['T'] = 2; conv['G'] = 3; conv['N'] = 4;
  inited = 1;
}

static inline int qual(char x) { return ((int)x) & 127; }

static inline int is_match(char h, char r) {
  uint8_t hc = conv[(uint8_t)h], rc = conv[(uint8_t)r];
  return hc == rc || hc == 4 || rc == 4;
}

#define DEFINE_PROB(NAME, T, PH2PR, M2M, INIT)                                               \
  T NAME(const or_testcase *tc) {                                                             \
    const int R = tc->rslen, C = tc->haplen;                                                  \
    T *buf = (T *)calloc((size_t)6 * (C + 1), sizeof(T));                                     \
    T *Mp = buf, *Xp = buf + (C + 1), *Yp = buf + 2 * (C + 1);                                \
    T *Mc = buf + 3 * (C + 1), *Xc = buf + 4 * (C + 1), *Yc = buf + 5 * (C + 1);              \
    const T init_Y = INIT / (T)(tc->haplen);                                                  \
    for (int c = 0; c <= C; c++) { Mp[c] = 0; Xp[c] = 0; Yp[c] = init_Y; }                    \
    for (int r = 1; r <= R; r++) {                                                            \
      int _i = qual(tc->i[r - 1]), _d = qual(tc->d[r - 1]), _c = qual(tc->c[r - 1]);          \
      int _q = qual(tc->q[r - 1]);                                                            \
      int mn = _d, mx = _i;                                                                   \
      if (_i <= _d) { mn = _i; mx = _d; }                                                     \
      const T pMM = M2M[((mx * (mx + 1)) >> 1) + mn];                                         \
      const T pGAPM = (T)1.0 - PH2PR[_c];                                                     \
      const T pMX = PH2PR[_i], pXX = PH2PR[_c], pMY = PH2PR[_d], pYY = PH2PR[_c];             \
      const T distm = PH2PR[_q];                                                              \
      const T d_match = (T)1.0 - distm;                                                       \
      const T d_mis = distm / (T)3.0;                                                         \
      const char rch = tc->rs[r - 1];                                                         \
      Mc[0] = 0; Xc[0] = 0; Yc[0] = 0;                                                        \
      for (int c = 1; c <= C; c++) {                                                          \
        T dist = is_match(tc->hap[c - 1], rch) ? d_match : d_mis;                             \
        Mc[c] = ((Mp[c - 1] * pMM + Xp[c - 1] * pGAPM) + Yp[c - 1] * pGAPM) * dist;           \
        Xc[c] = Mp[c] * pMX + Xp[c] * pXX;                                                    \
        Yc[c] = Mc[c - 1] * pMY + Yc[c - 1] * pYY;                                            \
      }                                                                                       \
      T *t;                                                                                   \
      t = Mp; Mp = Mc; Mc = t;                                                                \
      t = Xp; Xp = Xc; Xc = t;                                                                \
      t = Yp; Yp = Yc; Yc = t;                                                                \
    }                                                                                         \
    T sumM = 0, sumX = 0;                                                                     \
    for (int c = 1; c <= C; c++) sumM = sumM + Mp[c];                                         \
    for (int c = 1; c <= C; c++) sumX = sumX + Xp[c];                                         \
    free(buf);                                                                                \
    return sumM + sumX;                                                                       \
  }

DEFINE_PROB(phmm_oracle_prob_f32, float, ph2pr_f, m2m_f, init_f)
DEFINE_PROB(phmm_oracle_prob_f64, double, ph2pr_d, m2m_d, init_d)

/* IntelPairHmmCSource.cpp:61-85 for one testcase; also returns the raw values. */
double phmm_oracle_likelihood(const or_testcase *tc, float *raw_f, double *raw_d, int *used_double) {
  phmm_oracle_init();
  float f = phmm_oracle_prob_f32(tc);
  double d = 0.0;
  double out;
  int ud = 0;
  if (f < 1e-28f) {
    d = phmm_oracle_prob_f64(tc);
    out = log10(d) - log10_init_d;
    ud = 1;
  } else {
    out = (double)(log10f(f) - log10_init_f);
  }
  if (raw_f) *raw_f = f;
  if (raw_d) *raw_d = d;
  if (used_double) *used_double = ud;
  return out;
}

/* Batch form of computelikelihoodsboth (IntelPairHmmCSource.cpp:61-85), OpenMP over testcases
 * like the reference (schedule(dynamic,1)); nthreads <= 0 keeps the OpenMP default. */
void phmm_oracle_batch(const or_testcase *tcs, int n, double *out, float *raw_f, double *raw_d,
                       int *used_double, int nthreads) {
  phmm_oracle_init();
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) if (nthreads != 1)
#endif
  for (int k = 0; k < n; k++)
    out[k] = phmm_oracle_likelihood(&tcs[k], raw_f ? &raw_f[k] : 0, raw_d ? &raw_d[k] : 0,
                                    used_double ? &used_double[k] : 0);
}

/* Table access for tests (the product restates the same tables in its own host code). */
float phmm_oracle_ph2pr_f(int x) { phmm_oracle_init(); return ph2pr_f[x & 127]; }
float phmm_oracle_m2m_f(int idx) { phmm_oracle_init(); return m2m_f[idx]; }
double phmm_oracle_m2m_d(int idx) { phmm_oracle_init(); return m2m_d[idx]; }
