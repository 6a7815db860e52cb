// fmi_main.cpp -- CLI drop-in for the fmi benchmark driver (benchmarks/fmi/fmi.cpp, plain pipeline):
//   fmi <index_prefix> <reads.fastq[.gz] | reads.fa> <batch_size> <minSeedLen> <n_threads>
// Loads <index_prefix>.bwt.2bit.64 (FMI_search::load_index format), reads and 2-bit encodes the
// queries (A0 C1 G2 T3, anything else 4, stride max_readlength; fmi.cpp:139-177), runs the whole
// per-batch pipeline of fmi.cpp:253-348 (SMEMs, reseeding, LAST seeds, rid offset, per-read sort)
// on the MI355X through gb_fmi_search, and prints the reference's summary lines
// ("batch_id: %d, numTotalSmem[batch_id]: %d", "totalSmems = %ld"). GB_FMI_PRINT_OUTPUT=1 adds the
// PRINT_OUTPUT listing of fmi.cpp:383-415 ("<rid>:" headers and "[m,n+1]" per SMEM).
// n_threads is accepted (host parsing is single-threaded; the search runs on the GPU).
#include <zlib.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gb_fmi.h"

static void check(int st, const char *what) {
  if (st) {
    fprintf(stderr, "[gb fmi] %s failed (%d): %s\n", what, st, gb_last_error());
    exit(EXIT_FAILURE);
  }
}

// minimal FASTA/FASTQ reader over zlib (plain files pass through gzread unchanged)
struct Reader {
  gzFile f;
  std::vector<char> buf = std::vector<char>(1 << 20);
  std::string pending;
  bool has_pending = false;
  bool line(std::string &s) {
    if (has_pending) {
      s.swap(pending);
      has_pending = false;
      return true;
    }
    s.clear();
    while (gzgets(f, buf.data(), (int)buf.size())) {
      s += buf.data();
      if (!s.empty() && s.back() == '\n') break;
    }
    if (s.empty()) return false;
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
    return true;
  }
  void unread(std::string &s) {
    pending.swap(s);
    has_pending = true;
  }
};

int main(int argc, char **argv) {
  if (argc != 6) {
    printf("Need five arguments : ref_file query_set batch_size minSeedLen n_threads\n");
    return 1;
  }
  const std::string prefix = argv[1];
  const int batch_size = atoi(argv[3]);
  const int min_seed_len = atoi(argv[4]);
  if (batch_size <= 0 || min_seed_len <= 0) {
    fprintf(stderr, "batch_size and minSeedLen must be positive\n");
    return 1;
  }
  const char *dev = getenv("GB_DEVICE");
  check(gb_set_device(dev ? atoi(dev) : 0), "gb_set_device");

  Reader rd;
  rd.f = gzopen(argv[2], "r");
  if (!rd.f) {
    fprintf(stderr, "[E::%s] fail to open file `%s'.\n", __func__, argv[2]);
    return 1;
  }
  const auto t_read = std::chrono::steady_clock::now();
  std::vector<std::string> seqs;
  std::string l, s;
  while (rd.line(l)) {
    if (l.empty()) continue;
    const char tag = l[0];
    if (tag != '@' && tag != '>') {
      fprintf(stderr, "unexpected line in %s: %.40s\n", argv[2], l.c_str());
      return 1;
    }
    s.clear();
    while (rd.line(l)) {
      if (l.empty()) continue;
      if (l[0] == '>' || (tag == '@' && l[0] == '+')) {
        if (l[0] == '>') rd.unread(l);
        break;
      }
      s += l;
    }
    if (tag == '@') {  // skip the quality lines (same length as the sequence)
      size_t q = 0;
      while (q < s.size() && rd.line(l)) q += l.size();
    }
    seqs.push_back(s);
  }
  gzclose(rd.f);
  const int num_reads = (int)seqs.size();
  if (num_reads == 0) {
    printf("ERROR! seqs = NULL\n");
    return 1;
  }
  int max_len = 0, min_len = 1 << 30;
  for (const auto &q : seqs) {
    max_len = std::max(max_len, (int)q.size());
    min_len = std::min(min_len, (int)q.size());
  }
  if (max_len <= 0 || max_len >= 10000) {
    fprintf(stderr, "read lengths must be in [1, 10000)\n");
    return 1;
  }
  printf("Time taken by read: %lld microseconds\n",
         (long long)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t_read).count());
  printf("numReads = %d, max_readlength = %d, min_readlength = %d\n", num_reads, max_len, min_len);
  std::vector<uint8_t> enc((size_t)num_reads * max_len, 4);
  std::vector<int32_t> lens(num_reads);
  for (int r = 0; r < num_reads; r++) {
    lens[r] = (int32_t)seqs[r].size();
    uint8_t *e = enc.data() + (size_t)r * max_len;
    for (int k = 0; k < lens[r]; k++) {
      switch (seqs[r][k]) {
        case 'A': case 'a': e[k] = 0; break;
        case 'C': case 'c': e[k] = 1; break;
        case 'G': case 'g': e[k] = 2; break;
        case 'T': case 't': e[k] = 3; break;
        default: e[k] = 4;
      }
    }
  }
  seqs.clear();
  seqs.shrink_to_fit();

  gb_fmi_index *idx = nullptr;
  check(gb_fmi_index_load((prefix + ".bwt.2bit.64").c_str(), &idx), "gb_fmi_index_load");
  gb_fmi_reads *rs = nullptr;
  check(gb_fmi_reads_create(idx, enc.data(), lens.data(), num_reads, max_len, &rs), "gb_fmi_reads_create");
  const auto t0 = std::chrono::steady_clock::now();
  check(gb_fmi_search(rs, min_seed_len), "gb_fmi_search");
  check(gb_fmi_sync(rs), "gb_fmi_sync");
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const int64_t nb = (num_reads + batch_size - 1) / batch_size;
  std::vector<int64_t> bc((size_t)nb);
  int64_t total = 0, phases[3] = {0, 0, 0};
  const bool print = getenv("GB_FMI_PRINT_OUTPUT") && atoi(getenv("GB_FMI_PRINT_OUTPUT")) == 1;
  check(gb_fmi_results(rs, batch_size, nullptr, 0, &total, bc.data(), phases), "gb_fmi_results");
  std::vector<gb_smem> sm;
  if (print) {
    sm.resize((size_t)std::max<int64_t>(total, 1));
    check(gb_fmi_results(rs, batch_size, sm.data(), (int64_t)sm.size(), &total, bc.data(), phases),
          "gb_fmi_results");
  }
  float kms = 0, tms = 0;
  int64_t calls = 0;
  check(gb_fmi_timing(rs, &kms, &tms, &calls), "gb_fmi_timing");
  printf("Running on MI355X (gfx950): %d reads in %lld batches of %d\n", num_reads, (long long)nb, batch_size);
  printf("num_smem1: %lld, num_smem2: %lld, num_smem3: %lld\n", (long long)phases[0], (long long)phases[1],
         (long long)phases[2]);
  printf("Consumed: %0.4lf sec (kernels %0.4lf sec, %lld backwardExt)\n", secs, kms * 1e-3, (long long)calls);
  for (int64_t b = 0; b < nb; b++) printf("batch_id: %lld, numTotalSmem[batch_id]: %lld\n", (long long)b, (long long)bc[b]);
  printf("totalSmems = %lld\n", (long long)total);
  if (print) {
    int64_t prev = -1;
    for (int64_t i = 0; i < total; i++) {
      const gb_smem &m = sm[i];
      if ((int64_t)m.rid != prev)
        for (int64_t j = prev + 1; j <= (int64_t)m.rid; j++) printf("%lld:\n", (long long)j);
      prev = m.rid;
      printf("[%u,%u]\n", m.m, m.n + 1);
    }
  }
  gb_fmi_reads_destroy(rs);
  gb_fmi_index_destroy(idx);
  return 0;
}
