/*
 * gkl_pairhmm_c.h -- the reference-compatible PairHMM entry points exported by
 * genomicsbench_palisade_amd/lib/libgkl_pairhmm_c.so (drop-in for GKL's libgkl_pairhmm_c.so).
 *
 * Same names, C++ linkage and argument meaning as the reference:
 *   testcase                 tools/GKL/src/main/native/pairhmm/pairhmm_common.h:20-24
 *   initPairHMM              tools/GKL/src/main/native/pairhmm/IntelPairHmmCSource.cpp:29-51
 *   computelikelihoodsboth   IntelPairHmmCSource.cpp:61-85  (results[i] = log10 likelihood)
 *   computelikelihoodsfloat  IntelPairHmmCSource.cpp:89-99
 *   computelikelihoodsdouble IntelPairHmmCSource.cpp:103-115
 * as declared by the benchmark driver (benchmarks/phmm/PairHMMUnitTest.cpp:103-105).
 * The work runs on the current MI355X (gb_set_device / $GB_DEVICE); a HIP failure is fatal
 * (message on stderr, abort), since the reference signatures have no error channel.
 */
#ifndef GKL_PAIRHMM_C_H
#define GKL_PAIRHMM_C_H

typedef struct {
  int rslen, haplen;
  const char *q, *i, *d, *c;
  const char *hap, *rs;
} testcase;

#ifdef __cplusplus
void initPairHMM();
void computelikelihoodsboth(testcase *testcases, double *expected_results, int batch_size);
void computelikelihoodsfloat(testcase *testcases, float *expected_result);
void computelikelihoodsdouble(testcase *testcases, double *expected_result);
#endif

#endif
