// bsw_dropin.cpp -- BandedPairWiseSW (benchmarks/bsw/bandedSWA.h:115-285, plain overloads) over the C
// ABI of csrc/bsw.hip. getScores16 uploads the caller's buffers as they are (SeqPair.idr/idq index
// them, as loadPairs sets them, main_banded.cpp:188-189) and writes score/tle/gtle/qle/gscore/max_off
// back into the SeqPair array in place, like the reference.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/gb_compat/bandedSWA.h"

#include <cstddef>
static_assert(offsetof(SeqPair, max_off) == offsetof(gb_seqpair, max_off) &&
                  offsetof(SeqPair, len1) == offsetof(gb_seqpair, len1),
              "SeqPair must overlay gb_seqpair");
static gb_seqpair *gbp(SeqPair *p) { return reinterpret_cast<gb_seqpair *>(p); }

static void die(const char *what, int st) {
  fprintf(stderr, "[gb bsw] %s failed (%d): %s\n", what, st, gb_last_error());
  abort();
}

// HIP's current device is per host thread and the reference calls getScores16 from an OpenMP
// team (main_banded.cpp:896-909): every calling thread selects GB_DEVICE once (thread_local flag).
static void ensure_device() {
  static const int dev = [] {
    const char *d = getenv("GB_DEVICE");
    return d ? atoi(d) : 0;
  }();
  thread_local bool done = false;
  if (done) return;
  const int st = gb_set_device(dev);
  if (st) die("gb_set_device", st);
  done = true;
}

BandedPairWiseSW::BandedPairWiseSW(const int o_del, const int e_del, const int o_ins, const int e_ins,
                                   const int zdrop, const int end_bonus, const int8_t *mat_,
                                   const int8_t w_match, const int8_t /*w_mismatch*/, int /*numThreads*/)
    : SW_cells(0), ticks_(0), w_match_(w_match) {
  std::memset(&p_, 0, sizeof(p_));
  p_.o_del = o_del;
  p_.e_del = e_del;
  p_.o_ins = o_ins;
  p_.e_ins = e_ins;
  p_.zdrop = zdrop;
  p_.end_bonus = end_bonus;
  p_.w = 100;
  std::memcpy(p_.mat, mat_, 25);
}

BandedPairWiseSW::~BandedPairWiseSW() {}

int64_t BandedPairWiseSW::getTicks() { return ticks_; }

static int64_t span_end(const SeqPair *a, int32_t n, bool ref) {
  int64_t e = 0;
  for (int32_t k = 0; k < n; k++) {
    const int64_t v = ref ? a[k].idr + a[k].len1 : a[k].idq + a[k].len2;
    if (v > e) e = v;
  }
  return e;
}

void BandedPairWiseSW::getScores16(SeqPair *pairArray, uint8_t *seqBufRef, uint8_t *seqBufQer, int32_t numPairs,
                                   uint16_t /*numThreads*/, int32_t w) {
  ensure_device();
  const auto t0 = std::chrono::steady_clock::now();
  gb_bsw_params p = p_;
  p.w = w;
  int64_t cells = 0;
  const int st = gb_bsw_get_scores16_ex(&p, gbp(pairArray), numPairs, seqBufRef, span_end(pairArray, numPairs, true),
                                        seqBufQer, span_end(pairArray, numPairs, false), &cells);
  if (st) die("gb_bsw_get_scores16", st);
  SW_cells += (uint64_t)cells;
  ticks_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

// getScores8: exact results for the pairs the 8-bit kernel is defined on (gb_bsw_get_scores8); a pair
// outside that domain aborts, as the reference's assert on len2 does (bandedSWA.cpp:607-608).
void BandedPairWiseSW::getScores8(SeqPair *pairArray, uint8_t *seqBufRef, uint8_t *seqBufQer, int32_t numPairs,
                                  uint16_t /*numThreads*/, int32_t w) {
  ensure_device();
  const auto t0 = std::chrono::steady_clock::now();
  gb_bsw_params p = p_;
  p.w = w;
  int64_t cells = 0;
  const int st = gb_bsw_get_scores8(&p, w_match_, gbp(pairArray), numPairs, seqBufRef,
                                    span_end(pairArray, numPairs, true), seqBufQer,
                                    span_end(pairArray, numPairs, false), &cells);
  if (st) die("gb_bsw_get_scores8", st);
  SW_cells += (uint64_t)cells;
  ticks_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

int BandedPairWiseSW::scalarBandedSWA(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int32_t w,
                                      int h0, int *_qle, int *_tle, int *_gtle, int *_gscore, int *_max_off) {
  ensure_device();
  SeqPair sp;
  std::memset(&sp, 0, sizeof(sp));
  sp.idr = 0;
  sp.idq = 0;
  sp.len1 = tlen;
  sp.len2 = qlen;
  sp.h0 = h0;
  gb_bsw_params p = p_;
  p.w = w;
  const int st = gb_bsw_get_scores16(&p, gbp(&sp), 1, target, tlen, query, qlen);
  if (st) die("gb_bsw_get_scores16", st);
  if (_qle) *_qle = sp.qle;
  if (_tle) *_tle = sp.tle;
  if (_gtle) *_gtle = sp.gtle;
  if (_gscore) *_gscore = sp.gscore;
  if (_max_off) *_max_off = sp.max_off;
  return sp.score;
}
