// oracle/ref_phmm_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// Our own thin C entry points over the UNMODIFIED reference GKL PairHMM kernels, compiled from
// /root/reference by oracle/Makefile into oracle/_ref/ (never committed, never the product path).
// Binds: compute_fp_avxs/avxd (tools/GKL/src/main/native/pairhmm/avx_impl.cc:4-5),
//        compute_fp_avx512s/avx512d (avx512_impl.cc:7-8), ConvertChar::init (pairhmm_common.h:30),
//        and restates the per-testcase driver of computelikelihoodsboth
//        (IntelPairHmmCSource.cpp:61-85) without its printf.
#include <cmath>
#include "pairhmm_common.h"
#include "Context.h"
#include "avx_impl.h"
#include "avx512_impl.h"

static Context<float> g_f;
static Context<double> g_d;
static int g_inited = 0;

static void ensure_init() {
  if (!g_inited) { ConvertChar::init(); g_inited = 1; }
}

extern "C" {
int ref_phmm_has_avx512(void) { return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512dq") && __builtin_cpu_supports("avx512vl"); }
float ref_phmm_prob_f32(testcase* tc, int engine) { ensure_init(); return engine == 512 ? compute_fp_avx512s(tc) : compute_fp_avxs(tc); }
double ref_phmm_prob_f64(testcase* tc, int engine) { ensure_init(); return engine == 512 ? compute_fp_avx512d(tc) : compute_fp_avxd(tc); }

// computelikelihoodsboth semantics; engine 256 = AVX2 kernels, 512 = AVX-512 kernels.
void ref_phmm_batch(testcase* tcs, int n, double* out, float* raw_f, double* raw_d, int engine, int nthreads) {
  ensure_init();
  float (*pf)(testcase*) = engine == 512 ? compute_fp_avx512s : compute_fp_avxs;
  double (*pd)(testcase*) = engine == 512 ? compute_fp_avx512d : compute_fp_avxd;
  // warm the static tables on this thread before the parallel loop (Context ctors are not thread safe)
  if (n > 0) (void)pf(&tcs[0]);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int i = 0; i < n; i++) {
    float f = pf(&tcs[i]);
    double d = 0.0, r;
    if (f < MIN_ACCEPTED) {
      d = pd(&tcs[i]);
      r = log10(d) - g_d.LOG10_INITIAL_CONSTANT;
    } else {
      r = (double)(log10f(f) - g_f.LOG10_INITIAL_CONSTANT);
    }
    out[i] = r;
    if (raw_f) raw_f[i] = f;
    if (raw_d) raw_d[i] = d;
  }
}
}
