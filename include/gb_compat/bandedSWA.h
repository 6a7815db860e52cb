/*
 * gb_compat/bandedSWA.h -- source-compatible declaration of the reference banded-SW class for
 * relinking benchmarks/bsw (plain, non-HE build) against the MI355X implementation.
 *
 * Mirrors (written here, not copied):
 *   SeqPair / OutScore / eh_t          benchmarks/bsw/bandedSWA.h:92-112 (SeqPair layout == gb_seqpair)
 *   BandedPairWiseSW ctor, dtor,       benchmarks/bsw/bandedSWA.h:120-131 (ctor / scalarBandedSWA),
 *   scalarBandedSWA, getScores16,      :195-200 (getScores16, plain overload), getScores8 (plain),
 *   getScores8, getTicks               getTicks (bandedSWA.cpp:110-124)
 * Implemented by genomicsbench_palisade_amd/lib/libgb_bsw_dropin.so (csrc/bsw_dropin.cpp): every
 * call runs csrc/bsw.hip on the device selected by $GB_DEVICE (default 0). numThreads is accepted
 * and ignored. getScores8 computes the pairs of the 8-bit kernel's domain (len1, len2 < 128 and
 * h0 + min(len1, len2) * w_match < 128, bwamem.cpp:2152-2155) exactly and aborts on any other pair.
 */
#ifndef GB_COMPAT_BANDEDSWA_H
#define GB_COMPAT_BANDEDSWA_H

#include <cstdint>

#include "../gb_bsw.h"

#define MAX_SEQ_LEN_REF 256
#define MAX_SEQ_LEN_QER 128

// same name, members and layout as the reference's SeqPair, so mangled names match
// (e.g. _ZN16BandedPairWiseSW11getScores16EP10dnaSeqPairPhS2_iti)
typedef struct dnaSeqPair {
  int64_t idr, idq, id;
  int32_t len1, len2;
  int32_t h0;
  int seqid, regid;
  int32_t score, tle, gtle, qle;
  int32_t gscore, max_off;
} SeqPair;
static_assert(sizeof(SeqPair) == sizeof(gb_seqpair), "SeqPair layout");

typedef struct dnaOutScore {
  int32_t score, tle, gtle, qle;
  int32_t gscore, max_off;
} OutScore;

typedef struct {
  int32_t h, e;
} eh_t;

class BandedPairWiseSW {
 public:
  uint64_t SW_cells;

  BandedPairWiseSW(const int o_del, const int e_del, const int o_ins, const int e_ins, const int zdrop,
                   const int end_bonus, const int8_t *mat_, const int8_t w_match, const int8_t w_mismatch,
                   int numThreads);
  ~BandedPairWiseSW();

  int scalarBandedSWA(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int32_t w, int h0,
                      int *_qle, int *_tle, int *_gtle, int *_gscore, int *_max_off);

  void getScores16(SeqPair *pairArray, uint8_t *seqBufRef, uint8_t *seqBufQer, int32_t numPairs,
                   uint16_t numThreads, int32_t w);
  void getScores8(SeqPair *pairArray, uint8_t *seqBufRef, uint8_t *seqBufQer, int32_t numPairs,
                  uint16_t numThreads, int32_t w);
  int64_t getTicks();

 private:
  gb_bsw_params p_;
  int64_t ticks_;
  int32_t w_match_;
};

#endif
