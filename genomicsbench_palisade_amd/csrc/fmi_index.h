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

// Search-side layout, one 32-byte block per 64 BWT rows (the same bytes per row as half a CP_OCC):
// the 2-bit codes of rows [64b, 64b+64) (A0 C1 G2 T3, the sentinel row stored as 3; row r at bits
// 2*(r & 31) of word r >> 5) and the A, C, G counts before the block as three 34-bit fields. A lane
// reads one block with two 16-byte loads (a 64-byte line took four: the texture-address unit, which
// walks the 64 scattered lane addresses of each load, is what bounds the gathers). T is derived:
// rows before p minus A, C, G minus the sentinel row.
struct __attribute__((aligned(32))) Occ32 {
  uint64_t bwt[2];
  uint64_t cnt[2];  // cA | cC << 34, cC >> 30 | cG << 4
};
static_assert(sizeof(Occ32) == 32, "Occ32 is 32 bytes");

constexpr uint64_t kEven = 0x5555555555555555ull;

// The A, C, G counts of an Occ32 block: three 34-bit fields (rows < 2^34).
__host__ __device__ __forceinline__ void occ32_pack_counts(int64_t cA, int64_t cC, int64_t cG, uint64_t cnt[2]) {
  cnt[0] = (uint64_t)cA | ((uint64_t)cC << 34);
  cnt[1] = ((uint64_t)cC >> 30) | ((uint64_t)cG << 4);
}
__host__ __device__ __forceinline__ void occ32_unpack_counts(const uint64_t cnt[2], int64_t &cA, int64_t &cC,
                                                             int64_t &cG) {
  cA = (int64_t)(cnt[0] & ((1ull << 34) - 1));
  cC = (int64_t)((cnt[0] >> 34) | ((cnt[1] & 0xFull) << 30));
  cG = (int64_t)((cnt[1] >> 4) & ((1ull << 34) - 1));
}

// One `prev` entry of the search (an SMEM without rid), unpacked in registers and 16 bytes in
// memory: k, l, s < 2^34 rows and m, n < 2^13 read positions (checked on the host).
struct Ent {
  int64_t k, l, s;
  uint32_t m, n;
};
struct __attribute__((aligned(16))) PEnt {
  uint64_t w0, w1;
};
__host__ __device__ __forceinline__ PEnt pack_ent(const Ent &e) {
  PEnt p;
  p.w0 = (uint64_t)e.k | ((uint64_t)e.l << 34);
  p.w1 = ((uint64_t)e.l >> 30) | ((uint64_t)e.s << 4) | ((uint64_t)e.m << 38) | ((uint64_t)e.n << 51);
  return p;
}
__host__ __device__ __forceinline__ Ent unpack_ent(const PEnt &p) {
  constexpr uint64_t M34 = (1ull << 34) - 1, M13 = (1ull << 13) - 1;
  Ent e;
  e.k = (int64_t)(p.w0 & M34);
  e.l = (int64_t)((p.w0 >> 34) | ((p.w1 & 0xFull) << 30));
  e.s = (int64_t)((p.w1 >> 4) & M34);
  e.m = (uint32_t)((p.w1 >> 38) & M13);
  e.n = (uint32_t)((p.w1 >> 51) & M13);
  return e;
}

// A, C, G occurrences in rows [64b, p) of block b = p >> 6 plus the counts before the block.
__device__ __forceinline__ void occ32_acg(const Occ32 &L, int64_t p, int64_t &oA, int64_t &oC, int64_t &oG) {
  const int y = (int)(p & 63);
  const int y0 = y < 32 ? y : 32, y1 = y > 32 ? y - 32 : 0;
  const uint64_t m0 = y0 == 32 ? kEven : (((1ull << (2 * y0)) - 1) & kEven);
  const uint64_t m1 = (((1ull << (2 * y1)) - 1) & kEven);  // y1 <= 31
  const uint64_t lo0 = L.bwt[0] & kEven, hi0 = (L.bwt[0] >> 1) & kEven;
  const uint64_t lo1 = L.bwt[1] & kEven, hi1 = (L.bwt[1] >> 1) & kEven;
  int64_t cA, cC, cG;
  occ32_unpack_counts(L.cnt, cA, cC, cG);
  oA = cA + __popcll(m0 & ~(lo0 | hi0)) + __popcll(m1 & ~(lo1 | hi1));
  oC = cC + __popcll(m0 & lo0 & ~hi0) + __popcll(m1 & lo1 & ~hi1);
  oG = cG + __popcll(m0 & hi0 & ~lo0) + __popcll(m1 & hi1 & ~lo1);
}

// 2-bit code of row p (3 for both T and the sentinel row).
__device__ __forceinline__ int occ32_code(const Occ32 &L, int64_t p) {
  const int y = (int)(p & 63);
  return (int)((L.bwt[y >> 5] >> (2 * (y & 31))) & 3);
}

struct DevIndex {
  const Occ32 *occ;
  int64_t count[5];
  int64_t sentinel;
};

// Occ(b, p) for b = A, C, G, T from one Occ32 block (GET_OCC, FMI_search.h:81-89, over the same
// counts): T = p - A - C - G - [sentinel < p].
__device__ __forceinline__ void occ4(const Occ32 &L, int64_t p, int64_t sentinel, int64_t o[4]) {
  occ32_acg(L, p, o[0], o[1], o[2]);
  o[3] = p - o[0] - o[1] - o[2] - (sentinel < p ? 1 : 0);
}

// count[a] by selects over kernel-argument scalars: an indexed read would become a global load
// issued after the Occ gather (a second dependent memory round trip per backwardExt)
__device__ __forceinline__ int64_t count_of(const DevIndex &F, int a) {
  return a == 0 ? F.count[0] : a == 1 ? F.count[1] : a == 2 ? F.count[2] : a == 3 ? F.count[3] : F.count[4];
}

// backwardExt(smem{k,l,s}, a) -> {k', l', s'} (FMI_search.cpp:1536-1565). One 32-byte block covers
// 64 rows; when sp and ep share a block the second load is skipped.
__device__ __forceinline__ void bwt_ext(const DevIndex &F, int64_t k, int64_t l, int64_t s, int a,
                                        int64_t &ko, int64_t &lo, int64_t &so) {
  const int64_t sp = k, ep = k + s;
  const int64_t bs = sp >> 6, be = ep >> 6;
  // the second line only when sp and ep fall in different lines (a duplicate request for the same
  // line measured 10 % slower overall than the occasional wait for A)
  // (non-temporal loads, so the gathers would not evict the `prev` lists from L2, measured slower:
  // 130 -> 183 ms for 4 M reads, and FETCH / WRITE_SIZE up, 319 -> 338 / 69 -> 93 GB, r03g)
  const Occ32 A = F.occ[bs];
  Occ32 B;
  if (be != bs)
    B = F.occ[be];
  else
    B = A;
  int64_t os[4], oe[4];
  occ4(A, sp, F.sentinel, os);
  occ4(B, ep, F.sentinel, oe);
  const int64_t off = (k <= F.sentinel && k + s > F.sentinel) ? 1 : 0;
  const int64_t s3 = oe[3] - os[3], s2 = oe[2] - os[2], s1 = oe[1] - os[1], s0 = oe[0] - os[0];
  const int64_t l3 = l + off, l2 = l3 + s3, l1 = l2 + s2, l0 = l1 + s1;
  ko = a == 0 ? F.count[0] + os[0] : a == 1 ? F.count[1] + os[1] : a == 2 ? F.count[2] + os[2] : F.count[3] + os[3];
  so = a == 0 ? s0 : a == 1 ? s1 : a == 2 ? s2 : s3;
  lo = a == 0 ? l0 : a == 1 ? l1 : a == 2 ? l2 : l3;
}

}  // namespace gbfmi

// Index object behind the C ABI (one per device).
struct gb_fmi_index {
  int device = -1;
  int64_t n = 0;            // reference_seq_len = |text| + 1
  int64_t count[5] = {0};   // after the load-time +1 (FMI_search.cpp:763-768)
  int64_t sentinel = -1;
  int64_t cp_size = 0;      // (n >> 6) + 1 entries
  gbfmi::CpOcc *d_occ = nullptr;
  gbfmi::Occ32 *d_occ32 = nullptr;  // cp_size blocks, built from d_occ on first use
  int64_t sa_ns = 0;        // (n >> 3) + 1 sampled SA entries (SA_COMPX = 3, macro.h:64-66)
  int64_t *d_sa = nullptr;  // sa_ms_byte << 32 + sa_ls_word, one int64 per sampled row
};

struct gb_fmi_reads;
struct gb_smem;

namespace gbfmi {
// fmi.hip: the search-side Occ32 table (built once per index, on `s`).
int ensure_occ32(gb_fmi_index *ix, hipStream_t s);
// fmi.hip: the last search's SMEMs compacted on the device in (rid, m, n desc) order.
int reads_device_smems(gb_fmi_reads *R, const gb_smem **d_smems, int64_t *n);
hipStream_t reads_stream(gb_fmi_reads *R);
gb_fmi_index *reads_index(gb_fmi_reads *R);
// fmi_sa.hip: per-read-set SA-lookup state, released with the read set.
struct SaJob;
void sa_job_destroy(SaJob *j);
SaJob **reads_sa_job(gb_fmi_reads *R);
}  // namespace gbfmi
