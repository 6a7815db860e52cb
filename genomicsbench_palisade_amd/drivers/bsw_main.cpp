// bsw_main.cpp -- CLI drop-in for the bsw benchmark driver (benchmarks/bsw/main_banded.cpp, plain
// build): bsw -pairs <file> [-t threads] [-b batch] [-match a] [-mismatch b] [-ambig c] [-gapo o]
// [-gape e] [-o results.tsv]
// Pair file = loadPairs format (main_banded.cpp:160-202): per pair "h0", target ("ref") and query
// lines of '0'..'4'. Scoring = bwa_fill_scmat(match, mismatch, ambig) (:77-88), zdrop 100, w 100,
// end_bonus 5 (:846), BandedPairWiseSW::getScores16 from libgb_bsw_dropin.so (MI355X).
// Sequences are packed back to back (SeqPair.idr/idq are offsets) instead of the reference's
// 2048/256-byte strides; results are identical. -b is accepted; the GPU takes the whole set per call
// (batching only distributed work over OpenMP threads in the reference). -o writes one line per
// pair: score qle tle gtle gscore max_off.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gb_compat/bandedSWA.h"

int main(int argc, char **argv) {
  int w_match = 1, w_mismatch = 4, w_open = 6, w_extend = 1, w_ambig = -1, threads = 1, batch = 0, bits = 16;
  const char *pair_file = nullptr, *out_file = nullptr;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "-match")) w_match = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-mismatch")) w_mismatch = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-ambig")) w_ambig = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-gapo")) w_open = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-gape")) w_extend = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-pairs")) pair_file = argv[i + 1];
    else if (!strcmp(argv[i], "-t")) threads = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-b")) batch = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-o")) out_file = argv[i + 1];
    else if (!strcmp(argv[i], "-bits")) bits = atoi(argv[i + 1]);  // 8: getScores8 (bwa-mem2's 8-bit path)
    // -h0 is parsed by the reference but unused: every pair carries its own h0 line
  }
  if (!pair_file) {
    fprintf(stderr, "usage: bsw -pairs <InSeqFile> -t <threads> -b <batch_size>\n");
    return 1;
  }
  FILE *f = fopen(pair_file, "r");
  if (!f) {
    fprintf(stderr, "Could not open file: %s\n", pair_file);
    return 1;
  }
  std::vector<SeqPair> pairs;
  std::vector<uint8_t> ref, qer;
  std::vector<char> line(1 << 16);
  auto getline = [&](std::string &s) -> bool {
    s.clear();
    while (fgets(line.data(), (int)line.size(), f)) {
      s += line.data();
      if (!s.empty() && s.back() == '\n') break;
    }
    if (s.empty()) return false;
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
    return true;
  };
  std::string h, r, q;
  const auto tl0 = std::chrono::steady_clock::now();
  while (getline(h)) {
    if (!getline(r) || !getline(q)) {
      fprintf(stderr, "WARNING! Odd number of sequences in %s\n", pair_file);
      break;
    }
    if (r.empty() || q.empty() || r.size() > 2047 || q.size() > 255) {
      fprintf(stderr, "pair %zu: target length %zu / query length %zu outside [1,2047] / [1,255]\n",
              pairs.size(), r.size(), q.size());
      return 1;
    }
    SeqPair sp;
    memset(&sp, 0, sizeof(sp));
    sp.id = (int64_t)pairs.size();
    sp.len1 = (int32_t)r.size();
    sp.len2 = (int32_t)q.size();
    sp.h0 = atoi(h.c_str());
    sp.idr = (int64_t)ref.size();
    sp.idq = (int64_t)qer.size();
    sp.seqid = sp.regid = sp.score = sp.tle = sp.gtle = sp.qle = -1;
    sp.gscore = sp.max_off = -1;
    for (char c : r) ref.push_back((uint8_t)(c - 48));
    for (char c : q) qer.push_back((uint8_t)(c - 48));
    pairs.push_back(sp);
  }
  fclose(f);
  const double read_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tl0).count();
  printf("Number of input pairs: %zu\n", pairs.size());
  printf("Read time = %0.2lf s\n", read_s);

  int8_t mat[25];
  gb_bsw_fill_scmat(w_match, w_mismatch, w_ambig, mat);
  const int zdrop = 100, w = 100, end_bonus = 5;
  BandedPairWiseSW bsw(w_open, w_extend, w_open, w_extend, zdrop, end_bonus, mat, (int8_t)w_match,
                       (int8_t)w_mismatch, threads);
  (void)batch;
  const auto t0 = std::chrono::steady_clock::now();
  if (!pairs.empty() && bits == 8)
    bsw.getScores8(pairs.data(), ref.data(), qer.data(), (int32_t)pairs.size(), (uint16_t)threads, w);
  else if (!pairs.empty())
    bsw.getScores16(pairs.data(), ref.data(), qer.data(), (int32_t)pairs.size(), (uint16_t)threads, w);
  const double sw_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("Executed MI355X banded SW (gfx950)...\n");
  printf("Overall SW time = %0.3f s (%llu cells, %.2f GCUPS incl. host<->device copies)\n", sw_s,
         (unsigned long long)bsw.SW_cells, sw_s > 0 ? bsw.SW_cells / sw_s / 1e9 : 0.0);
  printf("Total Pairs processed: %zu\n", pairs.size());
  if (out_file) {
    FILE *o = fopen(out_file, "w");
    if (!o) {
      fprintf(stderr, "Could not open file: %s\n", out_file);
      return 1;
    }
    for (const auto &p : pairs)
      fprintf(o, "%d\t%d\t%d\t%d\t%d\t%d\n", p.score, p.qle, p.tle, p.gtle, p.gscore, p.max_off);
    fclose(o);
  }
  return 0;
}
