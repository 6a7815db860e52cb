/*
 * gb_fmi.h -- C ABI of the MI355X bwa-mem2 FM-index SMEM search (drop-in boundary for benchmarks/fmi).
 *
 * Reference interface this replaces (paths relative to the reference repo):
 *   class FMI_search (tools/bwa-mem2/src/FMI_search.h:101-224):
 *     FMI_search(const char *fname); load_index();                 FMI_search.cpp:469-984
 *     getSMEMsAllPosOneThread(...)                                  FMI_search.cpp:1182-1241
 *     getSMEMsOnePosOneThread(...)                                  FMI_search.cpp:986-1180
 *     bwtSeedStrategyAllPosOneThread(...)                           FMI_search.cpp:1243-1326
 *     sortSMEMs(...)                                                FMI_search.cpp:1520-1534
 *     build_index()                                                 FMI_search.cpp:358-434
 *   driven per batch by benchmarks/fmi/fmi.cpp:253-348 (smem1 -> reseed -> LAST -> rid offset -> sort).
 * gb_fmi_search() runs that whole per-batch pipeline for every read on the GPU (the CLI drop-in is
 * drivers/fmi_main.cpp -> bin/fmi).
 *
 * Plain pointers and sizes; 0 on success, negative gb_status on failure (gb_last_error()).
 */
#ifndef GB_FMI_H
#define GB_FMI_H

#include <stddef.h>
#include <stdint.h>

#include "gb.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Same 40-byte layout as the reference SMEM (FMI_search.h:91-99, non-DEBUG build). */
typedef struct gb_smem {
  uint32_t rid, m, n;
  int64_t k, l, s;
} gb_smem;

typedef struct gb_fmi_index gb_fmi_index;

/* load_index(): reads <prefix>.bwt.2bit.64 (reference file format) into HBM. */
int gb_fmi_index_load(const char *bwt_2bit_64_path, gb_fmi_index **out);
/* build_index() on the GPU from forward-strand codes (0..3 = A,C,G,T; pac2nt order): text =
 * ref + reverse complement, suffix array, BWT, CP_OCC checkpoints, sampled SA. out_path (nullable)
 * receives the reference-format .bwt.2bit.64 file. Text up to 2^34 - 2 rows (32-bit rows below 2^31,
 * 64-bit above); env GB_FMI_BUILD_WIDE=1 forces the 64-bit path, GB_FMI_BUILD_CHUNK=<rows> (64 ..
 * 2^30) caps the rows of one sort (tests). GB_ERR_ARG when more than that many suffixes share an
 * 8-base prefix or a tied group. */
int gb_fmi_index_build(const uint8_t *ref_codes, int64_t ref_len, const char *out_path,
                       gb_fmi_index **out);
/* Builds the search-side Occ32 table now (otherwise the first search does); call it before host
 * threads share the index. */
int gb_fmi_index_prepare(gb_fmi_index *idx);
/* n = reference_seq_len (|text|+1), count[5] as used by the search (load-time +1 applied). */
int gb_fmi_index_info(gb_fmi_index *idx, int64_t *n, int64_t *count5, int64_t *sentinel_index);
/* Copies the CP_OCC table (64 bytes per 64 BWT rows, reference layout) to host memory. */
int gb_fmi_index_cp_occ(gb_fmi_index *idx, void *dst, int64_t dst_bytes);
/* Copies the packed sampled SA ((n >> 3) + 1 int64 entries, sa_ms_byte << 32 + sa_ls_word) to host. */
int gb_fmi_index_sa(gb_fmi_index *idx, int64_t *dst, int64_t dst_entries);
int gb_fmi_index_destroy(gb_fmi_index *idx);

/* Device-resident read set: enc_qdb is numReads x max_readlength codes (A0 C1 G2 T3, else 4;
 * fmi.cpp:141-177), lens[r] = read length. */
typedef struct gb_fmi_reads gb_fmi_reads;
int gb_fmi_reads_create(gb_fmi_index *idx, const uint8_t *enc_qdb, const int32_t *lens,
                        int32_t num_reads, int32_t max_readlength, gb_fmi_reads **out);
int gb_fmi_reads_destroy(gb_fmi_reads *r);

/* The fmi.cpp per-batch pipeline over every read (asynchronous on the read set's stream):
 * SMEMs (min_intv 1), reseeding (split_len = (int)(min_seed_len*1.5+.499), split width 10),
 * LAST seeds (max_intv 20, min length min_seed_len+1), per-read sort by (m asc, n desc). */
int gb_fmi_search(gb_fmi_reads *r, int32_t min_seed_len);
/* Results of the last search: SMEMs in (rid, m, n desc) order with rid = read index, i.e. the
 * concatenation of the reference's sorted batches. batch_counts[b] = numTotalSmem of batch b
 * (batch_size reads per batch); phase_counts = {num_smem1, num_smem2, num_smem3} summed. */
int gb_fmi_results(gb_fmi_reads *r, int32_t batch_size, gb_smem *out, int64_t out_cap,
                   int64_t *total, int64_t *batch_counts, int64_t *phase_counts);
/* Kernel time of the last search (HIP events on the read set's stream), ms; backwardExt calls. */
int gb_fmi_timing(gb_fmi_reads *r, float *search_ms, float *total_ms, int64_t *bwt_calls);
int gb_fmi_sync(gb_fmi_reads *r);

/* ---- SA lookup: BWT rows -> reference coordinates (sampled SA every 8th row, SA_COMPX 3,
 *      macro.h:64-66; loaded from the index file / kept from gb_fmi_index_build).
 * GB_FMI_SA_COMPRESSED  FMI_search::get_sa_entry_compressed   FMI_search.cpp:1714-1807
 * GB_FMI_SA_PREFETCH    FMI_search::get_sa_entries_prefetch + call_one_step
 *                       FMI_search.cpp:1834-2040, the variant the aligner calls (bwamem.cpp:737);
 *                       differs from the above only when the LF walk reaches the sentinel row after
 *                       one or more steps: it answers 0 there (:1865-1869) instead of the step count. */
#define GB_FMI_SA_COMPRESSED 0
#define GB_FMI_SA_PREFETCH 1
/* SA value of each row rows[0..n) (0 <= row < n_index) into out[0..n). */
int gb_fmi_sa_lookup(gb_fmi_index *idx, const int64_t *rows, int64_t n, int32_t mode, int64_t *out);
/* get_sa_entries(_prefetch) (FMI_search.cpp:1596-1619 / :1895-1931) over n host SMEMs: SMEM i
 * contributes the SA values of rows k, k+step, ... (< k+s, at most max_occ of them), step =
 * s > max_occ ? s / max_occ : 1, concatenated in SMEM order into coords; counts[i] (nullable) = that
 * number; *total = sum. max_occ > 0 (bwa-mem2's default is 500). */
int gb_fmi_sa_entries(gb_fmi_index *idx, const gb_smem *smems, int64_t n, int32_t max_occ, int32_t mode,
                      int64_t *coords, int64_t coords_cap, int32_t *counts, int64_t *total);
/* The same over the last search of a read set, device-resident (the SMEMs in gb_fmi_results order,
 * i.e. bwamem.cpp:737 for every read): sizes its buffers (one host sync), then expands and walks
 * asynchronously on the read set's stream. */
int gb_fmi_reads_sa_run(gb_fmi_reads *r, int32_t max_occ, int32_t mode);
int gb_fmi_reads_sa_results(gb_fmi_reads *r, int64_t *coords, int64_t coords_cap, int32_t *counts,
                            int64_t *total);
/* Kernel time of the last SA run (row expansion + LF walks, HIP events), LF steps taken, coordinates. */
int gb_fmi_reads_sa_timing(gb_fmi_reads *r, float *ms, int64_t *lf_steps, int64_t *coords);

/* ---- Per-call phases (the FMI_search method adapter, include/gb_compat/FMI_search.h). Reads are
 * addressed like the reference: read r = enc_qdb[offs[r] .. offs[r] + lens[r]) (offs =
 * query_cum_len_ar, lens = seq_[r].l_seq) for r in [0, nrid). Output goes to out[0 .. *nout) in the
 * reference's emission order (out may be NULL to only count); bwt_calls (nullable) = backwardExt calls.
 * Synchronous; each host thread uses its own stream and device buffers on the index's device. */
/* getSMEMsOnePosOneThread (FMI_search.cpp:986-1180): task t = read rid[t] from query_pos[t] with
 * min_intv[t]; next_pos[t] (nullable) receives the updated query position. */
int gb_fmi_smem_onepos(gb_fmi_index *idx, const uint8_t *enc_qdb, const int32_t *lens, const int32_t *offs,
                       int32_t nrid, const int16_t *query_pos, const int32_t *min_intv, const int32_t *rid,
                       int32_t ntasks, int32_t min_seed_len, gb_smem *out, int64_t out_cap, int64_t *nout,
                       int16_t *next_pos, int64_t *bwt_calls);
/* getSMEMsAllPosOneThread (FMI_search.cpp:1182-1241): task t = read rid[t] at every x start with
 * min_intv[t], output round-major like the reference's do-while; rounds[t] (nullable) = the number of
 * x starts of task t (what the caller-visible compaction of rid/min_intv depends on). */
int gb_fmi_smem_allpos(gb_fmi_index *idx, const uint8_t *enc_qdb, const int32_t *lens, const int32_t *offs,
                       int32_t nrid, const int32_t *min_intv, const int32_t *rid, int32_t ntasks,
                       int32_t min_seed_len, gb_smem *out, int64_t out_cap, int64_t *nout, int32_t *rounds,
                       int64_t *bwt_calls);
/* bwtSeedStrategyAllPosOneThread (FMI_search.cpp:1243-1326): reads 0..nreads-1 with max_intv[i]; SMEM
 * rid = i. */
int gb_fmi_last_seeds(gb_fmi_index *idx, const uint8_t *enc_qdb, const int32_t *lens, const int32_t *offs,
                      int32_t nreads, const int32_t *max_intv, int32_t min_seed_len, gb_smem *out, int64_t out_cap,
                      int64_t *nout, int64_t *bwt_calls);
/* getSMEMs (FMI_search.cpp:1328-1497): right-to-left SMEMs of fixed-stride reads (read i =
 * enc_qdb[i * readlength ..], every base a position), with the reference's behaviour: its OpenMP region
 * is commented out, so only reads [0, ceil(num_reads / nthreads)) are searched, and *nout is what it
 * leaves in numTotalSmem[0]; SMEMs in read order, each read's in emission order (rid = i). */
int gb_fmi_get_smems(gb_fmi_index *idx, const uint8_t *enc_qdb, int32_t num_reads, int32_t readlength,
                     int32_t min_seed_len, int32_t nthreads, gb_smem *out, int64_t out_cap, int64_t *nout,
                     int64_t *bwt_calls);

/* get_sa_entry / get_sa_entries(pos[]) (FMI_search.cpp:1566-1586): the raw sampled-SA entries at
 * indices pos[i] (0 <= pos < (n >> 3) + 1, sa_ms_byte << 32 + sa_ls_word). */
int gb_fmi_sa_raw(gb_fmi_index *idx, const int64_t *pos, int64_t n, int64_t *out);
/* call_one_step (FMI_search.cpp:1834-1893): one LF step from row pos; *done = the reference's return
 * value (1: *sa_entry is final), *offset updated like the reference's reference argument. */
int gb_fmi_sa_one_step(gb_fmi_index *idx, int64_t pos, int64_t *sa_entry, int64_t *offset, int32_t *done);

/* Diagnostic: per-wave clock sums of the search kernel's phases when GB_FMI_FLAGS has bit 2 (value
 * 4) set -- out = {state machine, gather wait, consume, trips, lane state-loop iterations, trips in
 * which a lane took a new read, state-machine clocks of those trips, 0}; reset != 0 zeroes them. */
int gb_fmi_debug_prof(uint64_t out[8], int reset);
/* Diagnostic: after a search run with GB_FMI_FLAGS bit 3 (value 8) set, out[3 r .. 3 r + 2] = the
 * wall clock (100 MHz) at which read r was taken and finished, and its backwardExt calls. */
int gb_fmi_debug_trace(gb_fmi_reads *R, int64_t *out);
/* Diagnostic: the last search's control words -- out = {reads taken, big (kBigCap) slots taken,
 * reads past every slot (fatal), 0, reads handed to the wave pass, 0, 0, 0}. */
int gb_fmi_debug_ctl(gb_fmi_reads *R, int32_t out[8]);

/* Diagnostic, host only (no device work): round trips through the search's packed layouts, the
 * code the kernels run. ent: n entries of {k, l, s, m, n} (k, l, s < 2^34; m, n < 2^13) packed into
 * 16-byte `prev` entries and back into ent_out; cnt: n triples {A, C, G} (< 2^34) packed into an
 * Occ32 block's count words and back into cnt_out. */
int gb_fmi_debug_pack(int64_t n, const int64_t *ent, int64_t *ent_out, const int64_t *cnt, int64_t *cnt_out);

#ifdef __cplusplus
}
#endif
#endif /* GB_FMI_H */
