/*
 * gb_compat/FMI_search.h -- source-compatible declaration of bwa-mem2's FMI_search class for
 * building a plain (non-HE) variant of benchmarks/fmi/fmi.cpp against the MI355X implementation.
 * The shipped fmi.cpp is the HE build (it calls decrypt_ciphertext_to_plaintext_vector and reads
 * seqs[].enc_seq), so it does not compile against this header as is; tests/cpp/fmi_class_driver.cpp
 * is the plain variant (fmi.cpp's batch loop with the plaintext fields).
 *
 * Mirrors (written here, not copied):
 *   bseq1_t                          tools/bwa-mem2/src/bwa.h:60-69 (plain fields; methods read l_seq)
 *   SMEM (struct smem_struct)        tools/bwa-mem2/src/FMI_search.h:91-99 (non-DEBUG, == gb_smem)
 *   class FMI_search                 tools/bwa-mem2/src/FMI_search.h:101-224, public methods:
 *     FMI_search(fname), ~FMI_search, build_index, load_index            FMI_search.cpp:51-984
 *     getSMEMsOnePosOneThread / getSMEMsAllPosOneThread                  :986-1241
 *     bwtSeedStrategyAllPosOneThread, getSMEMs, sortSMEMs                :1243-1497, :1520-1534
 *     get_sa_entry, get_sa_entries (x3), get_sa_entry_compressed,        :1566-2040
 *     call_one_step, get_sa_entries_prefetch
 * Implemented by genomicsbench_palisade_amd/lib/libgb_fmi_dropin.so (csrc/fmi_dropin.cpp): the index
 * lives in HBM of the device selected by $GB_DEVICE (default 0) and every SMEM / SA method runs HIP
 * kernels there (csrc/fmi_tasks.hip, csrc/fmi_sa.hip), returning the reference's outputs in the
 * reference's order. One object may be shared by host threads, as fmi.cpp's OpenMP loop does.
 * Not provided: the HE members. (getSMEMs, which no benchmark calls, keeps its reference behaviour:
 * only the first ceil(numReads / nthreads) reads are searched, see gb_fmi_get_smems.)
 */
#ifndef GB_COMPAT_FMI_SEARCH_H
#define GB_COMPAT_FMI_SEARCH_H

#include <limits.h>
#include <stdint.h>

#include "../gb_fmi.h"

#ifndef PATH_MAX
#define PATH_MAX 4096
#endif

/* The plain bseq1_t. The reference's bwa.h:60-69 is the HE build's: it also carries five vecCT
 * members, so its stride differs and an object compiled against it must not call these methods --
 * the caller is a plain (non-HE) fmi.cpp compiled against this header. */
typedef struct {
  int l_seq, id;
  char *name, *comment, *seq, *qual, *sam;
} bseq1_t;
static_assert(sizeof(bseq1_t) == 2 * sizeof(int) + 5 * sizeof(char *), "plain bseq1_t (no HE vecCT members)");

typedef struct smem_struct {
  uint32_t rid;
  uint32_t m, n;
  int64_t k, l, s;
} SMEM;
static_assert(sizeof(SMEM) == sizeof(gb_smem), "SMEM layout");

class FMI_search {
 public:
  FMI_search(const char *fname);
  ~FMI_search();

  int build_index();
  void load_index();

  void getSMEMsOnePosOneThread(uint8_t *enc_qdb, int16_t *query_pos_array, int32_t *min_intv_array,
                               int32_t *rid_array, int32_t numReads, int32_t batch_size, const bseq1_t *seq_,
                               int32_t *query_cum_len_ar, int32_t max_readlength, int32_t minSeedLen,
                               SMEM *matchArray, int64_t *__numTotalSmem);

  void getSMEMsAllPosOneThread(uint8_t *enc_qdb, int32_t *min_intv_array, int32_t *rid_array, int32_t numReads,
                               int32_t batch_size, const bseq1_t *seq_, int32_t *query_cum_len_ar,
                               int32_t max_readlength, int32_t minSeedLen, SMEM *matchArray,
                               int64_t *__numTotalSmem);

  int64_t bwtSeedStrategyAllPosOneThread(uint8_t *enc_qdb, int32_t *max_intv_array, int32_t numReads,
                                         const bseq1_t *seq_, int32_t *query_cum_len_ar, int32_t minSeedLen,
                                         SMEM *matchArray);

  void getSMEMs(uint8_t *enc_qdb, int32_t numReads, int32_t batch_size, int32_t readlength, int32_t minSeedLen,
                int32_t nthreads, SMEM *matchArray, int64_t *numTotalSmem);

  void sortSMEMs(SMEM *matchArray, int64_t numTotalSmem[], int32_t numReads, int32_t readlength, int nthreads);

  int64_t get_sa_entry(int64_t pos);
  void get_sa_entries(int64_t *posArray, int64_t *coordArray, uint32_t count, int32_t nthreads);
  void get_sa_entries(SMEM *smemArray, int64_t *coordArray, int32_t *coordCountArray, uint32_t count,
                      int32_t max_occ);
  int64_t get_sa_entry_compressed(int64_t pos, int tid);
  void get_sa_entries(SMEM *smemArray, int64_t *coordArray, int32_t *coordCountArray, uint32_t count,
                      int32_t max_occ, int tid);
  int64_t call_one_step(int64_t pos, int64_t &sa_entry, int64_t &offset);
  void get_sa_entries_prefetch(SMEM *smemArray, int64_t *coordArray, int64_t *coordCountArray, int64_t count,
                               const int32_t max_occ, int tid, int64_t &id_);

  int64_t sentinel_index;
  int64_t reference_seq_len;

  /* MI355X extension: backwardExt calls made by this object's SMEM methods (all threads). */
  int64_t bwt_calls() const;

 private:
  char file_name[PATH_MAX];
  gb_fmi_index *idx_;
  int device_;
  int64_t calls_;
  void *lock_;
};

#endif /* GB_COMPAT_FMI_SEARCH_H */
