// fmi_dropin.cpp -- class FMI_search (tools/bwa-mem2/src/FMI_search.h:101-224, plain build) over the C
// ABI of csrc/fmi*.hip, so a plain (non-HE) build of benchmarks/fmi/fmi.cpp links against
// libgb_fmi_dropin.so (the shipped fmi.cpp is the HE build; see include/gb_compat/FMI_search.h).
// Every SMEM and SA method runs on the GPU that holds the index; each returns exactly what the
// reference writes, in the reference's order, including its caller-visible side effects on the
// input arrays (query_pos_array of OnePos, the in-place compaction of rid/min_intv by AllPos).
// Errors end the process like the reference's exit()/assert paths, with gb_last_error() printed.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gb_compat/FMI_search.h"

namespace {

[[noreturn]] void die(const char *what, int st) {
  fprintf(stderr, "[gb fmi] %s failed (%d): %s\n", what, st, gb_last_error());
  exit(EXIT_FAILURE);
}

int env_device() {
  const char *d = getenv("GB_DEVICE");
  return d ? atoi(d) : 0;
}

// HIP's current device is per host thread; fmi.cpp calls the methods from an OpenMP team.
void ensure_device(int dev) {
  thread_local int cur = -1;
  if (cur == dev) return;
  const int st = gb_set_device(dev);
  if (st) die("gb_set_device", st);
  cur = dev;
}

struct Lock {
  std::mutex m;
  std::atomic<int64_t> calls{0};
};

bool compare_smem(const SMEM &a, const SMEM &b) {  // compare_smem, FMI_search.cpp:1499-1518
  if (a.rid != b.rid) return a.rid < b.rid;
  if (a.m != b.m) return a.m < b.m;
  return a.n > b.n;
}

}  // namespace

FMI_search::FMI_search(const char *fname)
    : sentinel_index(0), reference_seq_len(0), idx_(nullptr), device_(env_device()), calls_(0),
      lock_(new Lock()) {
  std::snprintf(file_name, sizeof(file_name), "%s", fname);
}

FMI_search::~FMI_search() {
  if (idx_) gb_fmi_index_destroy(idx_);
  delete static_cast<Lock *>(lock_);
}

int64_t FMI_search::bwt_calls() const { return static_cast<Lock *>(lock_)->calls.load(); }

// build_index (FMI_search.cpp:358-434): <prefix>.pac -> text = forward + reverse complement
// (pac2nt :109-169) -> <prefix>.0123 and <prefix>.bwt.2bit.64, the suffix array built on the GPU.
int FMI_search::build_index() {
  ensure_device(device_);
  const std::string pac = std::string(file_name) + ".pac";
  FILE *fp = fopen(pac.c_str(), "rb");
  if (!fp) {
    fprintf(stderr, "[gb fmi] cannot open %s\n", pac.c_str());
    exit(EXIT_FAILURE);
  }
  fseek(fp, -1, SEEK_END);
  const int64_t pac_len = ftell(fp);
  uint8_t last = 0;
  if (fread(&last, 1, 1, fp) != 1) die("reading .pac", -1);
  const int64_t seq_len = (pac_len - 1) * 4 + (int)last;  // pac_seq_len, :96-107
  if (seq_len <= 0) die("empty .pac", -1);
  std::vector<uint8_t> buf((size_t)((seq_len >> 2) + ((seq_len & 3) ? 1 : 0)));
  fseek(fp, 0, SEEK_SET);
  if (fread(buf.data(), 1, buf.size(), fp) != buf.size()) die("reading .pac", -1);
  fclose(fp);
  std::vector<uint8_t> fwd((size_t)seq_len);
  for (int64_t i = 0; i < seq_len; i++) fwd[i] = buf[i >> 2] >> ((3 - (i & 3)) << 1) & 3;
  {  // the .0123 side file: the text as codes 0..3 (build_index :383-409)
    const std::string bin = std::string(file_name) + ".0123";
    FILE *fb = fopen(bin.c_str(), "wb");
    if (fb) {
      fwrite(fwd.data(), 1, fwd.size(), fb);
      std::vector<uint8_t> rc(fwd.rbegin(), fwd.rend());
      for (auto &c : rc) c = (uint8_t)(3 - c);
      fwrite(rc.data(), 1, rc.size(), fb);
      fclose(fb);
    }
  }
  gb_fmi_index *tmp = nullptr;
  const std::string out = std::string(file_name) + ".bwt.2bit.64";
  const int st = gb_fmi_index_build(fwd.data(), seq_len, out.c_str(), &tmp);
  if (st) die("gb_fmi_index_build", st);
  gb_fmi_index_destroy(tmp);
  return 0;
}

// load_index (FMI_search.cpp:469-984): <prefix>.bwt.2bit.64 into HBM
void FMI_search::load_index() {
  ensure_device(device_);
  const std::string path = std::string(file_name) + ".bwt.2bit.64";
  if (idx_) gb_fmi_index_destroy(idx_);
  idx_ = nullptr;
  int st = gb_fmi_index_load(path.c_str(), &idx_);
  if (st) die("gb_fmi_index_load", st);
  int64_t count5[5];
  st = gb_fmi_index_info(idx_, &reference_seq_len, count5, &sentinel_index);
  if (st) die("gb_fmi_index_info", st);
  // build the search-side tables now, single-threaded, before OpenMP threads share the object
  st = gb_fmi_index_prepare(idx_);
  if (st) die("gb_fmi_index_prepare", st);
}

namespace {
// lens[r] = seq_[r].l_seq for every rid a call can name; nrid = max named rid + 1
std::vector<int32_t> read_lengths(const bseq1_t *seq_, int32_t nrid) {
  std::vector<int32_t> lens((size_t)std::max(nrid, 0));
  for (int32_t r = 0; r < nrid; r++) lens[r] = seq_[r].l_seq;
  return lens;
}
}  // namespace

void FMI_search::getSMEMsOnePosOneThread(uint8_t *enc_qdb, int16_t *query_pos_array, int32_t *min_intv_array,
                                         int32_t *rid_array, int32_t numReads, int32_t /*batch_size*/,
                                         const bseq1_t *seq_, int32_t *query_cum_len_ar, int32_t /*max_readlength*/,
                                         int32_t minSeedLen, SMEM *matchArray, int64_t *__numTotalSmem) {
  if (numReads <= 0) return;
  ensure_device(device_);
  int32_t nrid = 0;
  for (int32_t i = 0; i < numReads; i++) nrid = std::max(nrid, rid_array[i] + 1);
  const std::vector<int32_t> lens = read_lengths(seq_, nrid);
  int64_t n = 0, calls = 0;
  // appends at matchArray[*__numTotalSmem] (FMI_search.cpp:1000, :1151)
  const int st = gb_fmi_smem_onepos(idx_, enc_qdb, lens.data(), query_cum_len_ar, nrid, query_pos_array,
                                    min_intv_array, rid_array, numReads, minSeedLen,
                                    reinterpret_cast<gb_smem *>(matchArray + *__numTotalSmem), INT64_MAX, &n,
                                    query_pos_array, &calls);
  if (st) die("getSMEMsOnePosOneThread", st);
  *__numTotalSmem += n;
  static_cast<Lock *>(lock_)->calls += calls;
}

void FMI_search::getSMEMsAllPosOneThread(uint8_t *enc_qdb, int32_t *min_intv_array, int32_t *rid_array,
                                         int32_t numReads, int32_t /*batch_size*/, const bseq1_t *seq_,
                                         int32_t *query_cum_len_ar, int32_t /*max_readlength*/, int32_t minSeedLen,
                                         SMEM *matchArray, int64_t *__numTotalSmem) {
  *__numTotalSmem = 0;
  if (numReads <= 0) return;
  ensure_device(device_);
  int32_t nrid = 0;
  for (int32_t i = 0; i < numReads; i++) nrid = std::max(nrid, rid_array[i] + 1);
  const std::vector<int32_t> lens = read_lengths(seq_, nrid);
  std::vector<int32_t> rounds((size_t)numReads);
  int64_t n = 0, calls = 0;
  const int st = gb_fmi_smem_allpos(idx_, enc_qdb, lens.data(), query_cum_len_ar, nrid, min_intv_array, rid_array,
                                    numReads, minSeedLen, reinterpret_cast<gb_smem *>(matchArray), INT64_MAX, &n,
                                    rounds.data(), &calls);
  if (st) die("getSMEMsAllPosOneThread", st);
  *__numTotalSmem = n;
  static_cast<Lock *>(lock_)->calls += calls;
  // The reference compacts rid_array / min_intv_array in place before every round (:1206-1223):
  // round r keeps, in order, the tasks with more than r x starts, written to the front. Slot k ends
  // up holding entry k of the last round that still had more than k active tasks.
  std::vector<int32_t> rid0(rid_array, rid_array + numReads), intv0(min_intv_array, min_intv_array + numReads);
  int32_t max_round = 0;
  for (int32_t r : rounds) max_round = std::max(max_round, r);
  std::vector<int32_t> active;
  for (int32_t r = 0; r < max_round; r++) {
    active.clear();
    for (int32_t t = 0; t < numReads; t++)
      if (rounds[t] > r) active.push_back(t);
    for (size_t k = 0; k < active.size(); k++) {
      rid_array[k] = rid0[active[k]];
      min_intv_array[k] = intv0[active[k]];
    }
  }
}

int64_t FMI_search::bwtSeedStrategyAllPosOneThread(uint8_t *enc_qdb, int32_t *max_intv_array, int32_t numReads,
                                                   const bseq1_t *seq_, int32_t *query_cum_len_ar,
                                                   int32_t minSeedLen, SMEM *matchArray) {
  if (numReads <= 0) return 0;
  ensure_device(device_);
  const std::vector<int32_t> lens = read_lengths(seq_, numReads);
  int64_t n = 0, calls = 0;
  const int st = gb_fmi_last_seeds(idx_, enc_qdb, lens.data(), query_cum_len_ar, numReads, max_intv_array,
                                   minSeedLen, reinterpret_cast<gb_smem *>(matchArray), INT64_MAX, &n, &calls);
  if (st) die("bwtSeedStrategyAllPosOneThread", st);
  static_cast<Lock *>(lock_)->calls += calls;
  return n;
}

// getSMEMs (FMI_search.cpp:1328-1497): matchArray from its start, numTotalSmem[0] = the count (the
// reference's commented-out OpenMP region leaves the other entries untouched); batch_size is unused
// there too
void FMI_search::getSMEMs(uint8_t *enc_qdb, int32_t numReads, int32_t batch_size, int32_t readlength,
                          int32_t minSeedLen, int32_t nthreads, SMEM *matchArray, int64_t *numTotalSmem) {
  (void)batch_size;
  ensure_device(device_);
  int64_t n = 0, calls = 0;
  const int st = gb_fmi_get_smems(idx_, enc_qdb, numReads, readlength, minSeedLen, nthreads,
                                  reinterpret_cast<gb_smem *>(matchArray), INT64_MAX, &n, &calls);
  if (st) die("getSMEMs", st);
  static_cast<Lock *>(lock_)->calls += calls;
  numTotalSmem[0] = n;
}

// sortSMEMs (FMI_search.cpp:1520-1534): per "thread" segment starting at first * readlength, a sort by
// compare_smem; glibc's qsort is a stable merge sort, so ties keep their order here too.
void FMI_search::sortSMEMs(SMEM *matchArray, int64_t numTotalSmem[], int32_t numReads, int32_t readlength,
                           int nthreads) {
  if (nthreads <= 0) return;
  const int32_t quota = (numReads + (nthreads - 1)) / nthreads;
  for (int tid = 0; tid < nthreads; tid++) {
    SMEM *a = matchArray + (int64_t)tid * quota * readlength;
    std::stable_sort(a, a + numTotalSmem[tid], compare_smem);
  }
}

int64_t FMI_search::get_sa_entry(int64_t pos) {
  ensure_device(device_);
  int64_t v = 0;
  const int st = gb_fmi_sa_raw(idx_, &pos, 1, &v);
  if (st) die("get_sa_entry", st);
  return v;
}

void FMI_search::get_sa_entries(int64_t *posArray, int64_t *coordArray, uint32_t count, int32_t /*nthreads*/) {
  if (!count) return;
  ensure_device(device_);
  const int st = gb_fmi_sa_raw(idx_, posArray, count, coordArray);
  if (st) die("get_sa_entries", st);
}

// The 5-argument overload (FMI_search.cpp:1588-1619) indexes the sampled arrays by row, as written.
void FMI_search::get_sa_entries(SMEM *smemArray, int64_t *coordArray, int32_t *coordCountArray, uint32_t count,
                                int32_t max_occ) {
  ensure_device(device_);
  std::vector<int64_t> pos;
  for (uint32_t i = 0; i < count; i++) {
    const SMEM &sm = smemArray[i];
    const int64_t hi = sm.k + sm.s, step = sm.s > max_occ ? sm.s / max_occ : 1;
    int32_t c = 0;
    for (int64_t j = sm.k; j < hi && c < max_occ; j += step, c++) pos.push_back(j);
    coordCountArray[i] = c;
  }
  if (pos.empty()) return;
  const int st = gb_fmi_sa_raw(idx_, pos.data(), (int64_t)pos.size(), coordArray);
  if (st) die("get_sa_entries", st);
}

int64_t FMI_search::get_sa_entry_compressed(int64_t pos, int /*tid*/) {
  ensure_device(device_);
  int64_t v = 0;
  const int st = gb_fmi_sa_lookup(idx_, &pos, 1, GB_FMI_SA_COMPRESSED, &v);
  if (st) die("get_sa_entry_compressed", st);
  return v;
}

// The 6-argument overload is declared but only present commented out in the reference
// (FMI_search.cpp:1808-1830); this follows that text: compressed lookups, one running total in
// *coordCountArray.
void FMI_search::get_sa_entries(SMEM *smemArray, int64_t *coordArray, int32_t *coordCountArray, uint32_t count,
                                int32_t max_occ, int /*tid*/) {
  ensure_device(device_);
  int64_t cap = 0, tot = 0;
  for (uint32_t i = 0; i < count; i++) cap += std::min<int64_t>(std::max<int64_t>(smemArray[i].s, 0), max_occ);
  const int st = gb_fmi_sa_entries(idx_, reinterpret_cast<const gb_smem *>(smemArray), count, max_occ,
                                   GB_FMI_SA_COMPRESSED, coordArray, std::max<int64_t>(cap, 1), nullptr, &tot);
  if (st) die("get_sa_entries", st);
  *coordCountArray += (int32_t)tot;
}

int64_t FMI_search::call_one_step(int64_t pos, int64_t &sa_entry, int64_t &offset) {
  ensure_device(device_);
  int32_t done = 0;
  const int st = gb_fmi_sa_one_step(idx_, pos, &sa_entry, &offset, &done);
  if (st) die("call_one_step", st);
  return done;
}

void FMI_search::get_sa_entries_prefetch(SMEM *smemArray, int64_t *coordArray, int64_t *coordCountArray,
                                         int64_t count, const int32_t max_occ, int /*tid*/, int64_t &id_) {
  ensure_device(device_);
  int64_t cap = 0, tot = 0;
  for (int64_t i = 0; i < count; i++) cap += std::min<int64_t>(std::max<int64_t>(smemArray[i].s, 0), max_occ);
  const int st = gb_fmi_sa_entries(idx_, reinterpret_cast<const gb_smem *>(smemArray), count, max_occ,
                                   GB_FMI_SA_PREFETCH, coordArray, std::max<int64_t>(cap, 1), nullptr, &tot);
  if (st) die("get_sa_entries_prefetch", st);
  *coordCountArray += tot;  // :1911 accumulates into one counter
  id_ += tot;               // :1913
}
