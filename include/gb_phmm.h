/*
 * gb_phmm.h -- C ABI of the MI355X PairHMM forward path (drop-in boundary for benchmarks/phmm).
 *
 * Reference interface this replaces (paths relative to the reference repo):
 *   void initPairHMM();                                    tools/GKL/src/main/native/pairhmm/IntelPairHmmCSource.cpp:29-51
 *   void computelikelihoodsboth(testcase*, double*, int);  IntelPairHmmCSource.cpp:61-85
 *     (declared by the caller at benchmarks/phmm/PairHMMUnitTest.cpp:103-105, linked -lgkl_pairhmm_c,
 *      benchmarks/phmm/Makefile:34)
 *   void computelikelihoodsfloat(testcase*, float*);       IntelPairHmmCSource.cpp:89-99
 *   void computelikelihoodsdouble(testcase*, double*);     IntelPairHmmCSource.cpp:103-115
 * Those C++-linkage symbols are exported unchanged by libgkl_pairhmm_c.so (built from
 * genomicsbench_palisade_amd/csrc/gkl_dropin.cpp) on top of the functions below.
 *
 * Plain pointers and sizes only. Every function returns 0 on success or a negative gb_status;
 * gb_last_error() describes the last failure on the calling thread. Objects are bound to the HIP
 * device that was current (gb_set_device) when they were created.
 */
#ifndef GB_PHMM_H
#define GB_PHMM_H

#include <stddef.h>
#include <stdint.h>

#include "gb.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Layout-identical to the reference `testcase` (pairhmm_common.h:20-24). q/i/d/c are already
 * phred-normalized bytes (PairHMMUnitTest.cpp:107-113); only the low 7 bits are used (&127,
 * avx-pairhmm-template.h:111-124). Bases: 'A','C','T','G','N'; any other byte behaves like 'A'
 * (ConvertChar, pairhmm_common.h:26-45). */
typedef struct gb_testcase {
  int rslen, haplen;
  const char *q, *i, *d, *c;
  const char *hap, *rs;
} gb_testcase;

/* initPairHMM(): builds the probability tables (Context.h) on the host and uploads them. */
int gb_phmm_init(void);

/* Limits: 1 <= rslen <= 65535 and 1 <= haplen <= 65535 (the 16-bit fields of the packed testcase
 * descriptor). Haplotypes up to 9400 bases keep a stack's boundary records and codes (17 bytes per
 * column) in one CU's LDS; longer ones run on kernels that keep them in a global scratch area per
 * workgroup, with the same arithmetic. A testcase outside the limits fails the call with GB_ERR_ARG
 * before any device work (the reference GKL kernels have no cap; the GKL-named drop-in aborts on such
 * input).
 *
 * computelikelihoodsboth(): results[k] = log10-likelihood of tcs[k], bit-identical to the
 * reference. raw_f / raw_d / used_double may be NULL; when given they receive the raw f32
 * probability, the raw f64 probability (0 when the f64 pass was not needed) and the fallback flag.
 * The reference never exposes the raw f32 value of a testcase that falls back (result below
 * MIN_ACCEPTED = 1e-28f): for those, raw_f holds a value below MIN_ACCEPTED -- the reference's, or 0
 * when the f32 pass's early exit proved the fallback before the last row (GB_PHMM_EXIT=0 turns the
 * exit off). raw_f of every testcase that does not fall back is bit-identical to the reference. */
int gb_phmm_compute(const gb_testcase *tcs, int n, double *results, float *raw_f, double *raw_d,
                    uint8_t *used_double);

/* computelikelihoodsdouble(): raw f64 probability for every testcase (no f32 pass). */
int gb_phmm_compute_f64(const gb_testcase *tcs, int n, double *raw_d);

/* computelikelihoodsfloat() (IntelPairHmmCSource.cpp:89-99): raw f32 probability of every testcase
 * in full, also of those below MIN_ACCEPTED (no early exit). */
int gb_phmm_compute_f32(const gb_testcase *tcs, int n, float *raw_f);

/* Device-resident batches: pack + upload once, run many times (what bench.py times). */
typedef struct gb_phmm_batch gb_phmm_batch;
int gb_phmm_batch_create(const gb_testcase *tcs, int n, gb_phmm_batch **out);
/* Enqueue the forward pass (f32 kernel, f64 fallback kernel, device log10 epilogue) on the
 * batch's stream. Asynchronous. */
int gb_phmm_batch_run(gb_phmm_batch *b);
int gb_phmm_batch_sync(gb_phmm_batch *b);
/* Copies results back (synchronous). results are computed on the HOST from the raw device
 * probabilities exactly like IntelPairHmmCSource.cpp:70-79 (bit-identical). dev_results (optional)
 * receives the device-side log10 epilogue for the same testcases. */
int gb_phmm_batch_results(gb_phmm_batch *b, double *results, float *raw_f, double *raw_d,
                          uint8_t *used_double, double *dev_results);
/* Kernel durations of the last run (HIP events on the batch's stream), milliseconds. */
int gb_phmm_batch_timing(gb_phmm_batch *b, float *f32_ms, float *f64_ms, float *total_ms);
/* Batch statistics: testcases, cells = sum(rslen*haplen), f64 fallbacks of the last run. */
int gb_phmm_batch_stats(gb_phmm_batch *b, int64_t *testcases, int64_t *cells, int64_t *n_f64);
/* The f32 pass's early exit in the last run: testcases it dropped before their last row (their
 * raw f32 reads 0; they fall back to f64 as they would have) and the read-row x haplotype cells it
 * did not compute for them. */
int gb_phmm_batch_exit_stats(gb_phmm_batch *b, int64_t *dropped, int64_t *cells_skipped);
int gb_phmm_batch_destroy(gb_phmm_batch *b);

#ifdef __cplusplus
}
#endif
#endif /* GB_PHMM_H */
