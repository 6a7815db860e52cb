// fmi_index.h -- device-side FM-index representation shared by the index builder and the search.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gbfmi {

// CP_OCC (tools/bwa-mem2/src/FMI_search.h:59-63): occurrence counts before row 64*i and one-hot
// bit planes (MSB = first row of the block) for BWT rows [64i, 64i+64).
struct __attribute__((aligned(64))) CpOcc {
  int64_t cp_count[4];
  uint64_t one_hot_bwt_str[4];
};
static_assert(sizeof(CpOcc) == 64, "CP_OCC is 64 bytes");

// Search-side layout, one 64-byte line per 128 BWT rows (half the reference table): the A, C and G
// one-hot planes of the two 64-row blocks (same bit order as CP_OCC) and the occurrence counts of
// A, C, G before the line packed as three 40-bit fields. T is derived: rows before p minus A, C, G
// minus the sentinel row (which carries no base bit).
struct __attribute__((aligned(64))) Occ2 {
  uint64_t a[2], c[2], g[2];
  uint64_t cnt[2];  // cA | cC << 40, cC >> 24 | cG << 16
};
static_assert(sizeof(Occ2) == 64, "Occ2 is 64 bytes");

}  // namespace gbfmi

// Index object behind the C ABI (one per device).
struct gb_fmi_index {
  int device = -1;
  int64_t n = 0;            // reference_seq_len = |text| + 1
  int64_t count[5] = {0};   // after the load-time +1 (FMI_search.cpp:763-768)
  int64_t sentinel = -1;
  int64_t cp_size = 0;      // (n >> 6) + 1 entries
  gbfmi::CpOcc *d_occ = nullptr;
  int64_t cp2_size = 0;     // (n >> 7) + 1 lines
  gbfmi::Occ2 *d_occ2 = nullptr;  // built from d_occ on first use
  int64_t sa_ns = 0;        // (n >> 3) + 1 sampled SA entries (SA_COMPX = 3, macro.h:64-66)
  int64_t *d_sa = nullptr;  // sa_ms_byte << 32 + sa_ls_word, one int64 per sampled row
};

struct gb_fmi_reads;
struct gb_smem;

namespace gbfmi {
// fmi.hip: the search-side Occ2 table (built once per index, on `s`).
int ensure_occ2(gb_fmi_index *ix, hipStream_t s);
// fmi.hip: the last search's SMEMs compacted on the device in (rid, m, n desc) order.
int reads_device_smems(gb_fmi_reads *R, const gb_smem **d_smems, int64_t *n);
hipStream_t reads_stream(gb_fmi_reads *R);
gb_fmi_index *reads_index(gb_fmi_reads *R);
// fmi_sa.hip: per-read-set SA-lookup state, released with the read set.
struct SaJob;
void sa_job_destroy(SaJob *j);
SaJob **reads_sa_job(gb_fmi_reads *R);
}  // namespace gbfmi
