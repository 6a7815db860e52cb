/*
 * gb_bsw.h -- C ABI of the MI355X banded Smith-Waterman extension (drop-in boundary for benchmarks/bsw).
 *
 * Reference interface this replaces (paths relative to the reference repo):
 *   BandedPairWiseSW::BandedPairWiseSW(o_del, e_del, o_ins, e_ins, zdrop, end_bonus, mat, w_match,
 *        w_mismatch, numThreads)                               benchmarks/bsw/bandedSWA.h:120-124
 *   void BandedPairWiseSW::getScores16(SeqPair *pairArray, uint8_t *seqBufRef, uint8_t *seqBufQer,
 *        int32_t numPairs, uint16_t numThreads, int32_t w)     bandedSWA.h:195-200, bandedSWA.cpp:3521
 *        semantics == scalarBandedSWA                          bandedSWA.cpp:130-251
 *   SeqPair                                                    bandedSWA.h:92-101
 *   bwa_fill_scmat                                             benchmarks/bsw/main_banded.cpp:77-88
 * Pair p's target (the reference's "ref", len1) is seqBufRef[idr .. idr+len1) and its query
 * (len2) is seqBufQer[idq .. idq+len2), codes 0..4 (main_banded.cpp:186-195). Results go into the
 * SeqPair fields score, tle, gtle, qle, gscore, max_off exactly as getScores16 writes them.
 * Limits: len2 <= GB_BSW_MAX_QLEN, len1 < 2^31. 0 on success, negative gb_status on failure.
 */
#ifndef GB_BSW_H
#define GB_BSW_H

#include <stdint.h>

#include "gb.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GB_BSW_MAX_QLEN 255 /* >= MAX_SEQ_LEN_QER - 1 (main_banded.cpp:61) */

/* Same layout as SeqPair (bandedSWA.h:92-101); 72 bytes. */
typedef struct gb_seqpair {
  int64_t idr, idq, id;
  int32_t len1, len2;
  int32_t h0;
  int32_t seqid, regid;
  int32_t score, tle, gtle, qle;
  int32_t gscore, max_off;
} gb_seqpair;

/* Constructor arguments of BandedPairWiseSW (bandedSWA.h:120-124) plus getScores16's w. */
typedef struct gb_bsw_params {
  int32_t o_del, e_del, o_ins, e_ins;
  int32_t zdrop, end_bonus;
  int32_t w;
  int8_t mat[25]; /* 5x5, row = target base, column = query base (bandedSWA.cpp:150-154, :180) */
} gb_bsw_params;

/* bwa_fill_scmat (main_banded.cpp:77-88) and the benchmark defaults (main_banded.cpp:53-57,846):
 * match 1, mismatch 4, ambig -1, gap open 6, extend 1, zdrop 100, end_bonus 5, w 100. */
void gb_bsw_fill_scmat(int a, int b, int ambig, int8_t mat[25]);
void gb_bsw_default_params(gb_bsw_params *p);

typedef struct gb_bsw_batch gb_bsw_batch;

/* Upload numPairs pairs and the two sequence buffers (ref_bytes / qer_bytes long) to the device. */
int gb_bsw_batch_create(const gb_bsw_params *params, const gb_seqpair *pairs, int64_t num_pairs,
                        const uint8_t *seq_buf_ref, int64_t ref_bytes, const uint8_t *seq_buf_qer,
                        int64_t qer_bytes, gb_bsw_batch **out);
/* Extend every pair (asynchronous on the batch's stream). */
int gb_bsw_batch_run(gb_bsw_batch *b);
int gb_bsw_batch_sync(gb_bsw_batch *b);
/* Write score/tle/gtle/qle/gscore/max_off into pairs[0..num_pairs) (other fields untouched; may be
 * NULL); out6 (may be NULL) receives {score, qle, tle, gtle, gscore, max_off} per pair; cells
 * (may be NULL) the DP cells each pair evaluated (the reference's inner-loop iterations,
 * bandedSWA.cpp:189); total_cells (may be NULL) their sum. */
int gb_bsw_batch_results(gb_bsw_batch *b, gb_seqpair *pairs, int32_t *out6, int32_t *cells,
                         int64_t *total_cells);
int gb_bsw_batch_timing(gb_bsw_batch *b, float *kernel_ms);
int gb_bsw_batch_destroy(gb_bsw_batch *b);

/* One-shot getScores16: results written into pairs in place. Reuses one cached device batch per
 * (calling thread, device), so calling it once per batch of pairs (main_banded.cpp:896-909) does
 * not create streams or buffers per call. */
int gb_bsw_get_scores16(const gb_bsw_params *params, gb_seqpair *pairs, int64_t num_pairs,
                        const uint8_t *seq_buf_ref, int64_t ref_bytes, const uint8_t *seq_buf_qer,
                        int64_t qer_bytes);
/* The same, also returning the DP cells evaluated (SW_cells accounting of BandedPairWiseSW). */
int gb_bsw_get_scores16_ex(const gb_bsw_params *params, gb_seqpair *pairs, int64_t num_pairs,
                           const uint8_t *seq_buf_ref, int64_t ref_bytes, const uint8_t *seq_buf_qer,
                           int64_t qer_bytes, int64_t *total_cells);
/* getScores8 (bandedSWA.cpp:426-725): the 8-bit kernel's domain is the one its bwa-mem2 caller
 * routes to it (bwamem.cpp:2152-2155): len1 < 128, len2 < 128, h0 + min(len1, len2) * w_match < 128.
 * Pairs in it get the exact (16-bit) results; any pair outside it fails the call with GB_ERR_ARG and
 * nothing is written. */
int gb_bsw_get_scores8(const gb_bsw_params *params, int32_t w_match, gb_seqpair *pairs, int64_t num_pairs,
                       const uint8_t *seq_buf_ref, int64_t ref_bytes, const uint8_t *seq_buf_qer,
                       int64_t qer_bytes, int64_t *total_cells);

#ifdef __cplusplus
}
#endif
#endif /* GB_BSW_H */
