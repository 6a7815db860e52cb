// fmi_class_driver.cpp -- TEST DRIVER (tests/test_fmi_dropin.py): benchmarks/fmi/fmi.cpp:253-348's
// per-batch loop written against the FMI_search class of include/gb_compat/FMI_search.h and linked
// with libgb_fmi_dropin.so, i.e. what the reference benchmark does through the same mangled methods.
//   fmi_class_driver <prefix> <reads.bin> <batch_size> <minSeedLen> <threads> <out.bin> [build]
// reads.bin: int32 numReads, int32 max_readlength, int32 lens[numReads], uint8 codes[numReads][max_readlength]
// out.bin:   int64 num_batches; per batch int64 n1, n2, n3 and the sorted SMEMs; then for batch 0 the raw
//            (unsorted) phase outputs and the caller-visible array side effects; SA method outputs;
//            int64 backwardExt calls.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/gb_compat/FMI_search.h"

template <class T>
static void wr(FILE *f, const T *p, size_t n) {
  if (n) fwrite(p, sizeof(T), n, f);
}
static void wr64(FILE *f, int64_t v) { fwrite(&v, 8, 1, f); }

int main(int argc, char **argv) {
  if (argc < 7) return 2;
  FILE *fi = fopen(argv[2], "rb");
  if (!fi) return 3;
  int32_t numReads = 0, maxlen = 0;
  if (fread(&numReads, 4, 1, fi) != 1 || fread(&maxlen, 4, 1, fi) != 1) return 3;
  std::vector<int32_t> lens(numReads);
  std::vector<uint8_t> enc_qdb((size_t)numReads * maxlen);
  if (fread(lens.data(), 4, numReads, fi) != (size_t)numReads) return 3;
  if (fread(enc_qdb.data(), 1, enc_qdb.size(), fi) != enc_qdb.size()) return 3;
  fclose(fi);
  const int batch_size = atoi(argv[3]), minSeedLen = atoi(argv[4]), numthreads = atoi(argv[5]);
  std::vector<bseq1_t> seqs(numReads);
  std::vector<int32_t> query_cum_len_ar(numReads);
  for (int32_t i = 0; i < numReads; i++) {
    std::memset(&seqs[i], 0, sizeof(bseq1_t));
    seqs[i].l_seq = lens[i];
    query_cum_len_ar[i] = i * maxlen;  // fmi.cpp:141-146
  }
  FMI_search *fmiSearch = new FMI_search(argv[1]);
  if (argc > 7 && !strcmp(argv[7], "build")) fmiSearch->build_index();
  fmiSearch->load_index();

  const int splitWidth = 10, maxMemIntv = 20;
  const double splitFactor = 1.5;
  const int split_len = (int)(minSeedLen * splitFactor + .499);
  const int64_t num_batches = (numReads + batch_size - 1) / batch_size;
  std::vector<std::vector<SMEM>> batch_out(num_batches);
  std::vector<int64_t> n123(3 * num_batches);
  // batch-0 raw phase outputs and side effects
  std::vector<SMEM> raw1, raw2, raw3;
  std::vector<int32_t> rid_after, intv_after;
  std::vector<int16_t> qpos_after;
  std::atomic<int64_t> next{0};
  auto worker = [&]() {
    std::vector<SMEM> match((size_t)batch_size * maxlen * 4 + 64);
    std::vector<int32_t> min_intv(batch_size * (size_t)maxlen + 64), rid(batch_size * (size_t)maxlen + 64);
    std::vector<int16_t> qpos(batch_size * (size_t)maxlen + 64);
    for (int64_t b; (b = next++) < num_batches;) {
      const int64_t i = b * batch_size;
      int32_t bc = batch_size;
      if (i + bc > numReads) bc = (int32_t)(numReads - i);
      for (int32_t j = 0; j < bc; j++) {
        min_intv[j] = 1;
        rid[j] = j;
      }
      int64_t num_smem1 = 0, num_smem2 = 0, num_smem3 = 0;
      fmiSearch->getSMEMsAllPosOneThread(enc_qdb.data() + i * maxlen, min_intv.data(), rid.data(), bc, batch_size,
                                         seqs.data() + i, query_cum_len_ar.data(), maxlen, minSeedLen, match.data(),
                                         &num_smem1);
      if (b == 0) {
        raw1.assign(match.begin(), match.begin() + num_smem1);
        rid_after.assign(rid.begin(), rid.begin() + bc);
        intv_after.assign(min_intv.begin(), min_intv.begin() + bc);
      }
      int64_t pos = 0;
      for (int64_t j = 0; j < num_smem1; j++) {
        SMEM *p = &match[j];
        int start = p->m, end = p->n + 1;
        if (end - start < split_len || p->s > splitWidth) continue;
        rid[pos] = p->rid;
        qpos[pos] = (end + start) >> 1;
        min_intv[pos] = p->s + 1;
        pos++;
      }
      fmiSearch->getSMEMsOnePosOneThread(enc_qdb.data() + i * maxlen, qpos.data(), min_intv.data(), rid.data(),
                                         (int32_t)pos, (int32_t)pos, seqs.data() + i, query_cum_len_ar.data(), maxlen,
                                         minSeedLen, match.data() + num_smem1, &num_smem2);
      if (b == 0) {
        raw2.assign(match.begin() + num_smem1, match.begin() + num_smem1 + num_smem2);
        qpos_after.assign(qpos.begin(), qpos.begin() + pos);
      }
      for (int32_t j = 0; j < bc; j++) min_intv[j] = maxMemIntv;
      num_smem3 = fmiSearch->bwtSeedStrategyAllPosOneThread(enc_qdb.data() + i * maxlen, min_intv.data(), bc,
                                                             seqs.data() + i, query_cum_len_ar.data(), minSeedLen + 1,
                                                             match.data() + num_smem1 + num_smem2);
      if (b == 0) raw3.assign(match.begin() + num_smem1 + num_smem2, match.begin() + num_smem1 + num_smem2 + num_smem3);
      int64_t tot = num_smem1 + num_smem2 + num_smem3;
      for (int64_t j = 0; j < tot; j++) match[j].rid += (uint32_t)i;
      int64_t cnt = tot;
      fmiSearch->sortSMEMs(match.data(), &cnt, bc, maxlen, 1);
      batch_out[b].assign(match.begin(), match.begin() + tot);
      n123[3 * b] = num_smem1;
      n123[3 * b + 1] = num_smem2;
      n123[3 * b + 2] = num_smem3;
    }
  };
  // the SMEM phase of fmi.cpp (its batch loop over the class methods), timed like fmi.cpp's own
  // "SMEM" clock (bench.py's class drop-in leg reads this line)
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < numthreads; t++) th.emplace_back(worker);
  for (auto &t : th) t.join();
  fprintf(stderr, "SMEM phase: %.6f s\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());

  FILE *fo = fopen(argv[6], "wb");
  wr64(fo, num_batches);
  for (int64_t b = 0; b < num_batches; b++) {
    wr(fo, &n123[3 * b], 3);
    wr(fo, batch_out[b].data(), batch_out[b].size());
  }
  wr64(fo, (int64_t)raw1.size());
  wr(fo, raw1.data(), raw1.size());
  wr(fo, rid_after.data(), rid_after.size());
  wr(fo, intv_after.data(), intv_after.size());
  wr64(fo, (int64_t)qpos_after.size());
  wr(fo, qpos_after.data(), qpos_after.size());
  wr64(fo, (int64_t)raw2.size());
  wr(fo, raw2.data(), raw2.size());
  wr64(fo, (int64_t)raw3.size());
  wr(fo, raw3.data(), raw3.size());
  // SA methods over batch 0's sorted SMEMs (bwamem.cpp:737 calls get_sa_entries_prefetch)
  std::vector<SMEM> &s0 = batch_out[0];
  int64_t cap = 0;
  for (auto &s : s0) cap += s.s < 500 ? s.s : 500;
  std::vector<int64_t> coords(cap + 1);
  int64_t ccount = 0, id = 0;
  fmiSearch->get_sa_entries_prefetch(s0.data(), coords.data(), &ccount, (int64_t)s0.size(), 500, 0, id);
  wr64(fo, ccount);
  wr64(fo, id);
  wr(fo, coords.data(), (size_t)ccount);
  const int64_t nrows = 64, n = fmiSearch->reference_seq_len;
  for (int64_t r = 0; r < nrows; r++) wr64(fo, fmiSearch->get_sa_entry_compressed((r * 7919) % n, 0));
  for (int64_t r = 0; r < nrows; r++) {
    int64_t e = 0, off = 0;
    const int64_t done = fmiSearch->call_one_step((r * 104729) % n, e, off);
    wr64(fo, done);
    wr64(fo, e);
    wr64(fo, off);
  }
  for (int64_t r = 0; r < 16; r++) wr64(fo, fmiSearch->get_sa_entry(r));
  wr64(fo, fmiSearch->sentinel_index);
  wr64(fo, fmiSearch->reference_seq_len);
  wr64(fo, fmiSearch->bwt_calls());
  fclose(fo);
  delete fmiSearch;
  return 0;
}
