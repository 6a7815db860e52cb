// phmm.hip -- MI355X (gfx950) PairHMM forward pass: host tables, batch packing, HIP kernels, C ABI.
//
// Arithmetic contract: the GKL recurrence
//   M[r][c] = ((M[r-1][c-1]*pMM + X[r-1][c-1]*pGAPM) + Y[r-1][c-1]*pGAPM) * dist(r,c)
//   X[r][c] = M[r-1][c]*pMX + X[r-1][c]*pXX
//   Y[r][c] = M[r][c-1]*pMY + Y[r][c-1]*pYY
// (tools/GKL/src/main/native/pairhmm/avx-pairhmm-template.h:183-198) with Y[0][*] = 2^120/haplen
// (f32) or 2^1020/haplen (f64), every other boundary 0, result = sum_c M[R][c] + sum_c X[R][c]
// (:299-344), f64 recomputation when the f32 result < 1e-28f (IntelPairHmmCSource.cpp:70-79).
// Must be built with -ffp-contract=off: no FMA anywhere, so every cell is bit-identical to the
// reference's AVX kernels.
//
// MI355X design: one stack of testcases sharing a haplotype per wave64 (phmm_stack: reads stacked
// vertically, each behind two virtual rows that reproduce the initial row); the stack is cut into
// stripes of 64 rows, lane k owns row r0+k and the wave sweeps anti-diagonals (step t: lane k is at
// column t-k+1). Values move one lane
// down per step with DPP wave_shr:1 (no LDS round trip); lane 0 takes the row above the stripe from
// one uniform LDS record per step, every lane reads the haplotype code of its own column from an
// LDS byte array, and lane 63 writes the stripe's last row back into the records (in place: the
// write index trails the read index by 63 columns). A second, persistent kernel recomputes in f64
// the testcases whose f32 result fell below MIN_ACCEPTED, stack by stack. Stacks are ordered by
// descending cost so the dispatcher balances waves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <functional>
#include <future>
#include <mutex>
#include <string>
#include <unordered_map>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/gb_phmm.h"
#include "gb_common.h"

namespace {

constexpr int kWave = 64;
// Longest haplotype a stack keeps in LDS: the f64 kernel's LDS (16-B boundary record + 1 code byte
// per column, plus kBndPad + kWave pad columns) must fit the 160 KB of one CU. Stacks of longer
// haplotypes (up to kMaxHaplen, the 16-bit field of TcDesc::dims) keep the same records in a global
// scratch area per workgroup instead (phmm_forward<.., kLong>): the reference GKL has no cap.
constexpr int kLdsHaplen = 9400;
constexpr int kMaxHaplen = 65535;
constexpr int kBndPad = 72;  // boundary records beyond column C (see phmm_stripe reads)
constexpr int kRecPad = 4;   // boundary records below column 0 (lane 63's writes start at column -2)
constexpr int kQualTab = 128;
constexpr int kStackRows = 2048;  // rows per stack (a testcase taller than this gets its own)
// the batch's device counter words (d_count): [0..7] the passes' counters, then the f64 plan's
// bucket counts, bucket cursors and its number of units with work (f64_plan)
constexpr int kPlanBuckets = 128;
constexpr int kPlanCount = 8, kPlanCursor = kPlanCount + kPlanBuckets, kPlanTotal = kPlanCursor + kPlanBuckets;
constexpr int kCountWords = kPlanTotal + 8;
constexpr int kMaxF64Parts = 8;
constexpr int kM2M = ((127 * 128) >> 1) + 128;  // set_mm_prob indices for quals < 128

// ---------------------------------------------------------------------------------------------
// Host tables: Context<float>/Context<double> (Context.h:13-190), restated.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxQual = 254;
constexpr double kJacTol = 8.0;
constexpr double kJacStep = 0.0001;
#define GB_JAC_INV_STEP (1.0 / kJacStep)
constexpr int kJacSize = (int)(kJacTol / kJacStep) + 1;

template <typename T>
struct HostTables {
  T ph2pr[kQualTab];
  T one_minus[kQualTab];  // 1 - ph2pr[x]: pGAPM (template.h:119) and 1-distm (template.h:152)
  T div3[kQualTab];       // ph2pr[x] / 3: mismatch distm (template.h:154)
  T m2m[kM2M];            // matchToMatchProb (Context.h:50-61) for quals < 128
  T init_const;           // INITIAL_CONSTANT
  T log10_init;           // LOG10_INITIAL_CONSTANT
};

template <typename T>
static int fast_round(T d) {
  return (d > (T)0.0) ? (int)(d + (T)0.5) : (int)(d - (T)0.5);
}

template <typename T>
static T log10sum(const std::vector<T> &jac, T small, T big) {
  if (small > big) std::swap(small, big);
  T diff = big - small;
  if (diff >= (T)kJacTol) return big;
  int ind = fast_round<T>((T)(diff * (T)GB_JAC_INV_STEP));
  return big + jac[ind];
}

template <typename T>
static void build_tables(HostTables<T> &t) {
  std::vector<T> jac(kJacSize);
  for (int k = 0; k < kJacSize; k++) jac[k] = (T)(log10(1.0 + pow(10.0, -((double)k) * kJacStep)));
  const double inv_ln10 = 1.0 / log(10);
  std::vector<T> m2m_full(((kMaxQual + 1) * (kMaxQual + 2)) >> 1);
  for (int i = 0, off = 0; i <= kMaxQual; off += ++i)
    for (int j = 0; j <= i; j++) {
      double s = log10sum<T>(jac, (T)(-0.1 * i), (T)(-0.1 * j));
      double l = log1p(-std::min(1.0, pow(10, s))) * inv_ln10;
      m2m_full[off + j] = (T)(pow(10, l));
    }
  for (int k = 0; k < kM2M; k++) t.m2m[k] = m2m_full[k];
  for (int x = 0; x < kQualTab; x++) {
    if constexpr (sizeof(T) == 4)
      t.ph2pr[x] = powf(10.f, -((float)x) / 10.f);
    else
      t.ph2pr[x] = pow(10.0, -((double)x) / 10.0);
    t.one_minus[x] = (T)1.0 - t.ph2pr[x];
    t.div3[x] = t.ph2pr[x] / (T)3.0;
  }
  if constexpr (sizeof(T) == 4) {
    t.init_const = ldexpf(1.f, 120);
    t.log10_init = log10f(t.init_const);
  } else {
    t.init_const = ldexp(1.0, 1020);
    t.log10_init = log10(t.init_const);
  }
}

// ConvertChar (pairhmm_common.h:30-39): A0 C1 T2 G3 N4, every other byte 0.
static uint8_t base_code(char ch) {
  switch ((uint8_t)ch) {
    case 'A': return 0;
    case 'C': return 1;
    case 'T': return 2;
    case 'G': return 3;
    case 'N': return 4;
    default: return 0;
  }
}
// Bit h set when a read base of this code matches a haplotype base of code h: equal codes, or
// either is N (mask construction in avx-pairhmm-template.h:5-27).
static uint8_t read_match_mask(uint8_t rc) { return rc == 4 ? 0x1F : (uint8_t)((1u << rc) | 0x10); }

// ---------------------------------------------------------------------------------------------
// Device side
// ---------------------------------------------------------------------------------------------
struct __attribute__((aligned(16))) TcDesc {
  uint32_t read_off;  // pool offset: rmatch[R] q[R] i[R] d[R] c[R]
  uint32_t hap_off;   // pool offset: hcode[C]
  uint32_t dims;      // rslen | haplen << 16
  uint32_t out_idx;   // position in the caller's testcase array
};

template <typename T>
struct DevTab {
  const T *ph2pr, *one_minus, *div3, *m2m;
  T init_const;
};

// Boundary record per column c (stripe above the current one): the two partial sums the first
// row of the current stripe needs from the row above, already multiplied by THAT first row's
// transition probabilities, plus the haplotype base code of column c:
//   z = (M*pMM + X*pGAPM) + Y*pGAPM   (the M recurrence's bracket, used one column later)
//   w = M*pMX + X*pXX                 (= X of the next row at the same column)
// Read by lane 0 with one uniform ds_read per step. The haplotype codes live in a separate byte
// array that every lane reads at its own column (no cross-lane traffic, no VALU).
template <typename T>
struct __attribute__((aligned(2 * sizeof(T)))) Brec {
  T z, w;
};

__device__ __forceinline__ int dpp_shr(int v, int lane0) {
  // wave_shr:1 (DPP ctrl 0x138); lane 0 has no source lane and keeps `lane0` (bound_ctrl off).
  return __builtin_amdgcn_update_dpp(lane0, v, 0x138, 0xF, 0xF, false);
}
template <int (*F)(int, int)>
__device__ __forceinline__ float dpp(float v, float keep) {
  return __builtin_bit_cast(float, F(__builtin_bit_cast(int, v), __builtin_bit_cast(int, keep)));
}
template <int (*F)(int, int)>
__device__ __forceinline__ double dpp(double v, double keep) {
  long long vb = __builtin_bit_cast(long long, v), kb = __builtin_bit_cast(long long, keep);
  int lo = F((int)(vb & 0xffffffffll), (int)(kb & 0xffffffffll));
  int hi = F((int)(vb >> 32), (int)(kb >> 32));
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
template <int (*F)(int, int)>
__device__ __forceinline__ uint32_t dpp(uint32_t v, uint32_t keep) {
  return (uint32_t)F((int)v, (int)keep);
}

// dist select without a compare: sign-extend bit `h` of the lane's match mask (0 or ~0) and
// bit-insert between the two candidates.
__device__ __forceinline__ float select_dist(uint32_t rmask, uint32_t h, float dmatch, float dmis) {
  uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)rmask, h, 1);
  uint32_t r = (m & __builtin_bit_cast(uint32_t, dmatch)) | (~m & __builtin_bit_cast(uint32_t, dmis));
  return __builtin_bit_cast(float, r);
}
// f64: the same mask applied to both halves. The mask comes from inline asm because hipcc 7.2
// mis-derives the high word of a sign-extended sbfe mask and constant-folds it; asm is opaque.
__device__ __forceinline__ double select_dist(uint32_t rmask, uint32_t h, double dmatch, double dmis) {
  uint32_t m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(rmask), "v"(h));
  const uint64_t a = __builtin_bit_cast(uint64_t, dmatch), b = __builtin_bit_cast(uint64_t, dmis);
  const uint32_t lo = (m & (uint32_t)a) | (~m & (uint32_t)b);
  const uint32_t hi = (m & (uint32_t)(a >> 32)) | (~m & (uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Per-lane constants of one stripe (initializeVectors, avx-pairhmm-template.h:83-128): the lane's
// own row (Y recurrence, emission) and the NEXT row's transitions (the partials z/w it hands down).
// nGAPMx is nGAPM for the X term of the bracket; a separate register so that the virtual row 0 of
// a stacked testcase (phmm_stack) can drop the X it receives from the testcase above it.
template <typename T>
struct RowParams {
  T pMY, pYY, dmatch, dmis;              // own row
  T nMM, nGAPM, nGAPMx, nMX, nXX;        // row below (lane+1; lane 63: first row of next stripe)
  uint32_t rmask;
};

// Lane state between steps. Row r = lane's row, column c = step - lane + 1:
//   Mp, Yp : M[r][c-1], Y[r][c-1]           zo, wo : this lane's z/w of column c-1
//   zd     : z of row r-1 at column c-1 (= the M bracket of this lane's next cell), shifted in
template <typename T>
struct LaneState {
  T Mp, Yp, zo, wo, zd;
};

// One anti-diagonal step. Arithmetic per cell is exactly the reference's (no FMA, same order):
//   X = M[r-1][c]*pMX + X[r-1][c]*pXX         computed by lane-1 as w, shifted in
//   M = ((M*pMM + X*pGAPM) + Y*pGAPM)[r-1][c-1] * dist    bracket computed by lane-1 as z
//   Y = M[r][c-1]*pMY + Y[r][c-1]*pYY
// kSum: accumulate the row sums (a testcase's last row is in the stripe); kWrite: lane 63 hands its
// row's partials to the next stripe through the LDS records.
template <typename T, bool kSum, bool kWrite>
__device__ __forceinline__ void phmm_step(const Brec<T> &rec, uint32_t h, LaneState<T> &st,
                                          const RowParams<T> &P, T &sumM, T &sumX, Brec<T> *wr, bool last_lane) {
  const T X = dpp<dpp_shr>(st.wo, rec.w);          // X[r][c]
  const T zdn = dpp<dpp_shr>(st.zo, rec.z);        // bracket for column c+1
  const T dist = select_dist(P.rmask, h, P.dmatch, P.dmis);
  const T M = st.zd * dist;
  const T Y = st.Mp * P.pMY + st.Yp * P.pYY;
  st.zo = (M * P.nMM + X * P.nGAPMx) + Y * P.nGAPM;
  st.wo = M * P.nMX + X * P.nXX;
  if constexpr (kSum) {
    sumM = sumM + M;
    sumX = sumX + X;
  }
  if constexpr (kWrite) {
    // lane 63 hands its row's z/w (the next stripe's brackets) to LDS; columns < 1 land in the pad
    if (last_lane) {
      Brec<T> b;
      b.z = st.zo;
      b.w = st.wo;
      *wr = b;
    }
  }
  st.zd = zdn;
  st.Mp = M;
  st.Yp = Y;
}

// Sweep `steps` anti-diagonals of one stripe, 4 per iteration, the boundary records of the next
// block prefetched before this block runs. Reads are at columns > t; lane 63 writes column t-62 of
// the row below at step t from step 60 on (bnd has kRecPad pad records below column 0).
// kSum: the lanes in `lastmask` hold the last row of a testcase; lane k reaches column C at step
// C + k - 1, where its row sum is final, so that step runs singly and lane k stores sumM + sumX
// (later steps add columns beyond C). The check is a uniform scalar compare per 4 steps.
template <typename T, bool kSum, bool kWrite>
__device__ __forceinline__ void phmm_stripe(int steps, LaneState<T> &st, const RowParams<T> &P,
                                            T &sumM, T &sumX, Brec<T> *__restrict__ bnd,
                                            const uint8_t *__restrict__ hcol, int C, int lane,
                                            uint64_t lastmask, T *__restrict__ out) {
  // hcol[c] = haplotype code of column c (valid for c in [-63, C+kBndPad)); lane's column at step
  // t is t - lane + 1.
  const uint8_t *hl = hcol + 1 - lane;
  const bool last_lane = lane == kWave - 1;
  constexpr int U = 4;
  // lane 63 reaches column 0 at step 62: its records for earlier (negative) columns are dropped by
  // running the first 60 steps without writes (the pad holds columns -2, -1)
  constexpr int kNoWrite = 60;
  uint64_t pend = lastmask;
  int target = (kSum && pend) ? C + __builtin_ctzll(pend) - 1 : INT_MAX;
  auto single = [&](int tt, auto wr_tag) {
    constexpr bool W = decltype(wr_tag)::value;
    phmm_step<T, kSum, W>(bnd[tt + 1], hl[tt], st, P, sumM, sumX, bnd + (tt - (kWave - 2)), last_lane);
    if (kSum && tt == target) {
      if (lane == __builtin_ctzll(pend)) *out = sumM + sumX;
      pend &= pend - 1;
      target = pend ? C + __builtin_ctzll(pend) - 1 : INT_MAX;
    }
  };
  // The block's record reads and writes go through one VGPR address with immediate offsets (an
  // SGPR base costs a v_mov per access); the asm zero keeps the compiler from rematerialising it.
  int vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  Brec<T> *wb = bnd - (kWave - 2) + vzero;
  auto run = [&](int t, int end, auto wr_tag) {
    constexpr bool W = decltype(wr_tag)::value;
    for (; t + U <= end; t += U) {
      if (kSum && target < t + U) {
        for (int u = 0; u < U; u++) single(t + u, wr_tag);
        continue;
      }
      // records land directly in the DPP "old" registers (no rotation copies); the LDS latency is
      // covered by the other waves on the SIMD
      Brec<T> *wr = wb + t;
      const Brec<T> c0 = wr[kWave - 1], c1 = wr[kWave], c2 = wr[kWave + 1], c3 = wr[kWave + 2];
      const uint32_t h0 = hl[t], h1 = hl[t + 1], h2 = hl[t + 2], h3 = hl[t + 3];
      phmm_step<T, kSum, W>(c0, h0, st, P, sumM, sumX, wr, last_lane);
      phmm_step<T, kSum, W>(c1, h1, st, P, sumM, sumX, wr + 1, last_lane);
      phmm_step<T, kSum, W>(c2, h2, st, P, sumM, sumX, wr + 2, last_lane);
      phmm_step<T, kSum, W>(c3, h3, st, P, sumM, sumX, wr + 3, last_lane);
    }
    for (; t < end; t++) single(t, wr_tag);
  };
  if constexpr (kWrite) {
    const int a = min(steps, kNoWrite);
    run(0, a, std::false_type{});
    run(a, steps, std::true_type{});
  } else {
    run(0, steps, std::false_type{});
  }
}

template <typename T>
__device__ __forceinline__ void load_row(const uint8_t *__restrict__ rbase, int R, int row,
                                         const DevTab<T> &tab, T &pMM, T &pGAPM, T &pMX, T &pXX,
                                         T &pMY, T &pYY, T &dmatch, T &dmis, uint32_t &rmask) {
  rmask = rbase[row];
  const int q = rbase[R + row] & 127, qi = rbase[2 * R + row] & 127;
  const int qd = rbase[3 * R + row] & 127, qc = rbase[4 * R + row] & 127;
  const int mn = qi <= qd ? qi : qd, mx = qi <= qd ? qd : qi;
  pMM = tab.m2m[((mx * (mx + 1)) >> 1) + mn];
  pGAPM = tab.one_minus[qc];
  pMX = tab.ph2pr[qi];
  pXX = tab.ph2pr[qc];
  pMY = tab.ph2pr[qd];
  pYY = tab.ph2pr[qc];
  dmatch = tab.one_minus[q];
  dmis = tab.div3[q];
}

// Stacks: testcases that share a haplotype are stacked into one tall matrix, so a wave sweeps
// 64-row stripes of the stack and a read's rows need not start at a stripe boundary: the partial
// last stripe of every testcase (a quarter of all lane steps for 100-250-row reads) disappears.
// Each read is preceded by two virtual rows, ordinary lanes whose constants make the shared step
// code produce the reference's initial row (M = X = 0, Y = INITIAL_CONSTANT / haplen) exactly, and
// zeros at the columns a lane sweeps before its column 1 (so nothing leaks into column 0):
//   va: dist = 0 (M = 0), Y = init_Y * 1 at every step, partials z = (0*0 + X*0) + init_Y*1 and
//       w = 0*0 + X*0 = 0, whatever the testcase above hands it;
//   v0: dist = 1 at columns >= 0 and 0 before (column codes 5 at column 0, 6 below it, matched by
//       v0's mask only up to 5), so M = init_Y from column 0 on, and its partials are
//       z = (M*pGAPM + X*0) + 0*0 = init_Y*pGAPM (the reference's (0*pMM + 0*pGAPM) + init_Y*pGAPM)
//       and w = 0 (its 0*pMX + 0*pXX), zero before column 0.
// Lanes beyond the stack's last row compute zeros.
struct __attribute__((aligned(16))) Stack {
  uint32_t first;  // first entry in the stack's testcase index list
  uint32_t count;  // testcases (<= 64)
  uint32_t hap_off;
  uint32_t C;
};
struct __attribute__((aligned(16))) StackEnt {
  int start;  // stacked row of the testcase's first virtual row
  int R;
  uint32_t read_off, out_idx;
};

__device__ __forceinline__ int scan_add(int v) {  // wave-wide inclusive prefix sum (DPP)
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
  return v;
}

// One stack. f32 pass: every testcase (kExit: with the early exit below); f64 pass: those whose f32
// result is below MIN_ACCEPTED (all of them when `force`). Returns the number of testcases computed.
template <typename T, bool kF64Pass, bool kExit = false>
__device__ __forceinline__ int phmm_stack(const Stack &S, const uint32_t *__restrict__ stk_tc, const TcDesc *__restrict__ descs,
                          const uint8_t *__restrict__ pool, const DevTab<T> &tab, T *__restrict__ raw_out,
                          const float *__restrict__ raw_f, bool force, uint8_t *smem_raw, int part = 0,
                          int parts = 1, unsigned long long *exit_stats = nullptr) {
  const int lane = threadIdx.x;
  const int C = (int)S.C;
  // LDS: boundary records for columns [-kRecPad, C+kBndPad) and the haplotype codes for columns
  // [-kWave, C+kBndPad). The stack's testcase table lives in lanes (lane a: entry a), read with
  // cross-lane shuffles.
  Brec<T> *bnd = reinterpret_cast<Brec<T> *>(smem_raw) + kRecPad;
  uint8_t *hcol = smem_raw + sizeof(Brec<T>) * (size_t)(C + kBndPad + kRecPad) + kWave;

  // the stack's testcases, compacted to those computed in this pass
  TcDesc d = {0, 0, 0, 0};
  // the f64 pass may take a stack in `parts` work units: unit `part` takes the stack's entries
  // [part * count / parts, (part + 1) * count / parts)
  bool act = lane < (int)S.count;
  if (parts > 1) act = act && lane >= part * (int)S.count / parts && lane < (part + 1) * (int)S.count / parts;
  if (act) {
    d = descs[stk_tc[S.first + lane]];
    if constexpr (kF64Pass) act = force || raw_f[d.out_idx] < 1e-28f;  // MIN_ACCEPTED, pairhmm_common.h:16
  }
  const uint64_t am = __builtin_amdgcn_ballot_w64(act);
  if (!am) return 0;
  const int na = __builtin_popcountll(am);
  const int rows = act ? (int)(d.dims & 0xffff) + 2 : 0;
  const int incl = scan_add(rows);
  const int T_rows = __builtin_amdgcn_readlane(incl, 63);
  // compaction: entry a = the a-th computed testcase (lane order), gathered into lane a
  int src = 0;
  {
    uint64_t m = am;
    for (int a = 0; a < lane && m; a++) m &= m - 1;  // drop the first `lane` active lanes
    src = m ? __builtin_ctzll(m) : 63;
  }
  const int e_start = __shfl(incl - rows, src), e_R = __shfl(rows - 2, src);
  const uint32_t e_read = (uint32_t)__shfl((int)d.read_off, src), e_out = (uint32_t)__shfl((int)d.out_idx, src);
  const T init_Y = tab.init_const / (T)C;
  const uint8_t *hcode = pool + S.hap_off;
  for (int c = lane; c < C + kBndPad; c += kWave) {
    Brec<T> b;
    b.z = (T)0;
    b.w = (T)0;
    bnd[c] = b;
  }
  // column codes: the haplotype's at 1..C, 5 at column 0 and 6 below it (see va / v0), 0 beyond C
  for (int c = lane - kWave; c < C + kBndPad; c += kWave)
    hcol[c] = (c >= 1 && c <= C) ? hcode[c - 1] : (c == 0 ? 5 : (c < 0 ? 6 : 0));
  __syncthreads();

  // the stripe loop walks stacked rows from `base`; an early exit (f32 pass, `force` set) can skip the
  // rest of a testcase, so the stripes are not at fixed multiples of 64
  for (int base = 0; base < T_rows;) {
    const int g = base + lane;
    // the lane's testcase: the last entry starting at or before row g
    int lo = 0, hi = na - 1;
    while (__builtin_amdgcn_ballot_w64(lo < hi)) {  // per-lane binary search over lanes' starts
      const int mid = (lo + hi + 1) >> 1;
      const int sm = __shfl(e_start, mid);
      if (lo < hi) {
        if (sm <= g) lo = mid; else hi = mid - 1;
      }
    }
    StackEnt e;
    e.start = __shfl(e_start, lo);
    e.R = __shfl(e_R, lo);
    e.read_off = (uint32_t)__shfl((int)e_read, lo);
    e.out_idx = (uint32_t)__shfl((int)e_out, lo);
    const int r = g - e.start;  // 0: va, 1: v0, 2..R+1: read row r-2
    const bool dead = g >= T_rows;
    const uint8_t *rbase = pool + e.read_off;
    RowParams<T> P;
    LaneState<T> st;
    st.Mp = st.zo = st.wo = (T)0;
    st.Yp = (T)0;
    // bracket at column 0 of the row above: lane 0 takes it from the record lane 63 wrote there
    st.zd = lane == 0 ? bnd[0].z : (T)0;
    {
      T pMM, pGAPM, pMX, pXX, a, b, dm, dx;
      uint32_t f;
      const T zero = (T)0, one = (T)1;
      P.nMM = P.nGAPM = P.nGAPMx = P.nMX = P.nXX = zero;
      if (dead) {
        P.pMY = P.pYY = P.dmatch = P.dmis = zero;
        P.rmask = 0;
      } else if (r == 0) {  // va
        P.pMY = zero;
        P.pYY = one;
        P.dmatch = P.dmis = zero;
        P.rmask = 0;
        P.nGAPM = one;
        st.Yp = init_Y;
        // the state of a lane that has swept the columns before its first one: va's outputs are
        // constant, so it hands init_Y down from its first step
        st.zo = (zero * zero + zero * zero) + init_Y * one;
      } else if (r == 1) {  // v0
        P.pMY = P.pYY = zero;
        P.dmatch = one;
        P.dmis = zero;
        P.rmask = 0x3F;
        load_row(rbase, e.R, 0, tab, pMM, pGAPM, pMX, pXX, a, b, dm, dx, f);
        P.nMM = pGAPM;
        st.zd = init_Y;  // va's output at the column before
        // lane 0 starts at column 1: the row below takes v0's column-0 bracket from its initial zo
        if (lane == 0) st.zo = (init_Y * P.nMM + zero * zero) + zero * zero;
      } else {
        load_row(rbase, e.R, r - 2, tab, pMM, pGAPM, pMX, pXX, P.pMY, P.pYY, P.dmatch, P.dmis, P.rmask);
        if (r - 1 < e.R) {
          load_row(rbase, e.R, r - 1, tab, P.nMM, P.nGAPM, P.nMX, P.nXX, a, b, dm, dx, f);
          P.nGAPMx = P.nGAPM;
        }  // the last row: nothing below it in this testcase (zero partials)
      }
    }
    const bool last_row = !dead && r == e.R + 1;
    const uint64_t lastmask = __builtin_amdgcn_ballot_w64(last_row);
    const bool more = base + kWave < T_rows;
    const int steps = more ? C + kWave - 1 : C + (T_rows - base) - 1;
    T sumM = (T)0, sumX = (T)0;
    T *out = raw_out + e.out_idx;
    // lane 63's row and testcase for the early exit below, taken before the sweep into scalars
    int r63 = 0, R63 = 0, start63 = 0, out63 = 0;
    if (kExit && more) {
      r63 = __builtin_amdgcn_readlane(r, 63);
      R63 = __builtin_amdgcn_readlane(e.R, 63);
      start63 = __builtin_amdgcn_readlane(e.start, 63);
      out63 = __builtin_amdgcn_readlane((int)e.out_idx, 63);
    }
    if (lastmask) {
      if (more)
        phmm_stripe<T, true, true>(steps, st, P, sumM, sumX, bnd, hcol, C, lane, lastmask, out);
      else
        phmm_stripe<T, true, false>(steps, st, P, sumM, sumX, bnd, hcol, C, lane, lastmask, out);
    } else {
      phmm_stripe<T, false, true>(steps, st, P, sumM, sumX, bnd, hcol, C, lane, 0, out);
    }
    __syncthreads();
    int next = base + kWave;
    if constexpr (!kF64Pass && kExit) {
      // Early exit (GB_PHMM_EXIT): every path of a testcase crosses from its row r to row r+1 once,
      // and what follows multiplies by transitions and emissions <= 1, so its result is at most the
      // crossing mass sum_c (z + w) of row r -- the records lane 63 just wrote for the next stripe,
      // already multiplied by row r+1's transitions. Below MIN_ACCEPTED / 4 (margin for the f32
      // rounding of the sum and of the rows not computed) the testcase must fail the f32 test: its
      // remaining rows are skipped, its f32 result is written as 0, and the f64 pass computes it as
      // it would have anyway. Only rows with a row of the same testcase below them are tested.
      if (r63 >= 2 && r63 <= R63) {
        T acc = (T)0;
#pragma unroll 1
        for (int c = 1 + lane; c <= C; c += kWave) acc += bnd[c].z + bnd[c].w;
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        // the sum is the same in every lane; readfirstlane tells the compiler so (a divergent loop
        // bound would turn the whole stripe loop into per-lane control flow)
        if (__builtin_amdgcn_readfirstlane(acc < (T)0.25e-28f ? 1 : 0)) {
          next = start63 + R63 + 2;  // the next testcase's first (virtual) row
          if (lane == 0) {
            raw_out[(uint32_t)out63] = (T)0;
            // exit_stats[0] testcases dropped, [1] their cells not computed (real rows from the next
            // stripe's first row to the testcase's last)
            atomicAdd(exit_stats, 1ull);
            atomicAdd(exit_stats + 1, (unsigned long long)(next - (base + kWave)) * (unsigned long long)C);
          }
        }
        __syncthreads();
      }
    }
    base = next;
  }
  return na;
}

// ---------------------------------------------------------------------------------------------
// Two rows per lane (the f32 pass over LDS stacks). A stripe is 128 rows: lane k owns rows 2k (a)
// and 2k+1 (b), and row rho of the stripe is at column t - rho + 1 at step t, as before. Row b runs
// one column behind row a in the same lane, so its inputs from the row above (X = w and the bracket
// z of row a) are row a's previous-step values, carried in registers; only row a's inputs cross a
// lane (lane k-1's row b, DPP wave_shr). Per two cells: 24 FP ops, 2 DPP moves, 2 selects, one LDS
// code read (row b reuses row a's code of the step before) -- against 2 DPP moves and 2 code reads
// per two cells with one row per lane. The arithmetic of each cell is unchanged (same operands,
// same order), so the results are bit-identical.
constexpr int kRows2 = 2 * kWave;  // stripe height
constexpr int kBndPad2 = 136;      // records / codes beyond column C (lane 0 reads up to C + kRows2 + 2)
constexpr int kCodePad2 = kRows2;  // codes below column 0 (lane 63's row a starts at column -125)
constexpr int kNoWrite2 = kRows2 - 4;  // lane 63's row b writes from column -2 on (step 124)

// One row's constants and initial state (phmm_stack's per-lane set-up, for stripe row rho): r is the
// row's place in its testcase (0: va, 1: v0, 2..R+1: read row r-2); z_top the bracket lane 0's first
// row takes from the record at column 0.
template <typename T>
__device__ __forceinline__ void setup_row(int rho, bool dead, int r, int R, const uint8_t *__restrict__ rbase,
                                          const DevTab<T> &tab, T init_Y, T z_top, RowParams<T> &P,
                                          LaneState<T> &st) {
  st.Mp = st.zo = st.wo = (T)0;
  st.Yp = (T)0;
  st.zd = rho == 0 ? z_top : (T)0;
  T pMM, pGAPM, pMX, pXX, a, b, dm, dx;
  uint32_t f;
  const T zero = (T)0, one = (T)1;
  P.nMM = P.nGAPM = P.nGAPMx = P.nMX = P.nXX = zero;
  if (dead) {
    P.pMY = P.pYY = P.dmatch = P.dmis = zero;
    P.rmask = 0;
  } else if (r == 0) {  // va
    P.pMY = zero;
    P.pYY = one;
    P.dmatch = P.dmis = zero;
    P.rmask = 0;
    P.nGAPM = one;
    st.Yp = init_Y;
    st.zo = (zero * zero + zero * zero) + init_Y * one;
  } else if (r == 1) {  // v0
    P.pMY = P.pYY = zero;
    P.dmatch = one;
    P.dmis = zero;
    P.rmask = 0x3F;
    load_row(rbase, R, 0, tab, pMM, pGAPM, pMX, pXX, a, b, dm, dx, f);
    P.nMM = pGAPM;
    st.zd = init_Y;
    if (rho == 0) st.zo = (init_Y * P.nMM + zero * zero) + zero * zero;
  } else {
    load_row(rbase, R, r - 2, tab, pMM, pGAPM, pMX, pXX, P.pMY, P.pYY, P.dmatch, P.dmis, P.rmask);
    if (r - 1 < R) {
      load_row(rbase, R, r - 1, tab, P.nMM, P.nGAPM, P.nMX, P.nXX, a, b, dm, dx, f);
      P.nGAPMx = P.nGAPM;
    }
  }
}

// One step of both rows: row b (column c - 1) from row a's previous-step partials, row a (column c)
// from lane k-1's row b (previous step) or, in lane 0, the record of the stripe above.
template <typename T, bool kSum, bool kWrite>
__device__ __forceinline__ void phmm_step2(const Brec<T> &rec, uint32_t h, uint32_t &hb, LaneState<T> &A,
                                           LaneState<T> &B, const RowParams<T> &PA, const RowParams<T> &PB,
                                           T &sMa, T &sXa, T &sMb, T &sXb, Brec<T> *wr, bool last_lane) {
  const T Xb = A.wo;
  const T zdnb = A.zo;
  const T Xa = dpp<dpp_shr>(B.wo, rec.w);
  const T zdna = dpp<dpp_shr>(B.zo, rec.z);
  const T Mb = B.zd * select_dist(PB.rmask, hb, PB.dmatch, PB.dmis);
  const T Ma = A.zd * select_dist(PA.rmask, h, PA.dmatch, PA.dmis);
  const T Yb = B.Mp * PB.pMY + B.Yp * PB.pYY;
  const T Ya = A.Mp * PA.pMY + A.Yp * PA.pYY;
  B.zo = (Mb * PB.nMM + Xb * PB.nGAPMx) + Yb * PB.nGAPM;
  B.wo = Mb * PB.nMX + Xb * PB.nXX;
  A.zo = (Ma * PA.nMM + Xa * PA.nGAPMx) + Ya * PA.nGAPM;
  A.wo = Ma * PA.nMX + Xa * PA.nXX;
  if constexpr (kSum) {
    sMa = sMa + Ma;
    sXa = sXa + Xa;
    sMb = sMb + Mb;
    sXb = sXb + Xb;
  }
  if constexpr (kWrite) {
    if (last_lane) {
      Brec<T> r;
      r.z = B.zo;
      r.w = B.wo;
      *wr = r;
    }
  }
  A.zd = zdna;
  A.Mp = Ma;
  A.Yp = Ya;
  B.zd = zdnb;
  B.Mp = Mb;
  B.Yp = Yb;
  hb = h;
}

// Sweep `steps` anti-diagonals of a 128-row stripe, 4 per iteration. Last rows: row rho of the stripe
// reaches column C at step C + rho - 1, where its sum is final (pa: rows a by lane, pb: rows b).
template <typename T, bool kSum, bool kWrite>
__device__ __forceinline__ void phmm_stripe2(int steps, LaneState<T> &A, LaneState<T> &B, const RowParams<T> &PA,
                                             const RowParams<T> &PB, Brec<T> *__restrict__ bnd,
                                             const uint8_t *__restrict__ hcol, int C, int lane, uint64_t pa,
                                             uint64_t pb, T *__restrict__ outA, T *__restrict__ outB) {
  const uint8_t *hl = hcol + 1 - 2 * lane;
  const bool last_lane = lane == kWave - 1;
  constexpr int U = 4;
  T sMa = (T)0, sXa = (T)0, sMb = (T)0, sXb = (T)0;
  uint32_t hb = hl[-1];  // row b's code at its column before step 0
  auto next_target = [&]() -> int {
    if (!kSum || !(pa | pb)) return INT_MAX;
    const int ra = pa ? 2 * __builtin_ctzll(pa) : INT_MAX / 2;
    const int rb = pb ? 2 * __builtin_ctzll(pb) + 1 : INT_MAX / 2;
    return C + min(ra, rb) - 1;
  };
  int target = next_target();
  auto single = [&](int tt, auto wr_tag) {
    constexpr bool W = decltype(wr_tag)::value;
    phmm_step2<T, kSum, W>(bnd[tt + 1], hl[tt], hb, A, B, PA, PB, sMa, sXa, sMb, sXb, bnd + (tt - (kRows2 - 2)),
                           last_lane);
    if (kSum && tt == target) {
      const int rho = tt - C + 1;
      if (rho & 1) {
        if (lane == (rho >> 1)) *outB = sMb + sXb;
        pb &= pb - 1;
      } else {
        if (lane == (rho >> 1)) *outA = sMa + sXa;
        pa &= pa - 1;
      }
      target = next_target();
    }
  };
  int vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  Brec<T> *wb = bnd - (kRows2 - 2) + vzero;
  auto run = [&](int t, int end, auto wr_tag) {
    constexpr bool W = decltype(wr_tag)::value;
    for (; t + U <= end; t += U) {
      if (kSum && target < t + U) {
        for (int u = 0; u < U; u++) single(t + u, wr_tag);
        continue;
      }
      Brec<T> *wr = wb + t;
      const Brec<T> c0 = wr[kRows2 - 1], c1 = wr[kRows2], c2 = wr[kRows2 + 1], c3 = wr[kRows2 + 2];
      const uint32_t h0 = hl[t], h1 = hl[t + 1], h2 = hl[t + 2], h3 = hl[t + 3];
      phmm_step2<T, kSum, W>(c0, h0, hb, A, B, PA, PB, sMa, sXa, sMb, sXb, wr, last_lane);
      phmm_step2<T, kSum, W>(c1, h1, hb, A, B, PA, PB, sMa, sXa, sMb, sXb, wr + 1, last_lane);
      phmm_step2<T, kSum, W>(c2, h2, hb, A, B, PA, PB, sMa, sXa, sMb, sXb, wr + 2, last_lane);
      phmm_step2<T, kSum, W>(c3, h3, hb, A, B, PA, PB, sMa, sXa, sMb, sXb, wr + 3, last_lane);
    }
    for (; t < end; t++) single(t, wr_tag);
  };
  if constexpr (kWrite) {
    const int a = min(steps, kNoWrite2);
    run(0, a, std::false_type{});
    run(a, steps, std::true_type{});
  } else {
    run(0, steps, std::false_type{});
  }
}

// phmm_stack with two rows per lane (f32 pass, every testcase of the stack).
template <typename T>
__device__ __forceinline__ void phmm_stack2(const Stack &S, const uint32_t *__restrict__ stk_tc,
                                            const TcDesc *__restrict__ descs, const uint8_t *__restrict__ pool,
                                            const DevTab<T> &tab, T *__restrict__ raw_out, uint8_t *smem_raw) {
  const int lane = threadIdx.x;
  const int C = (int)S.C;
  Brec<T> *bnd = reinterpret_cast<Brec<T> *>(smem_raw) + kRecPad;
  uint8_t *hcol = smem_raw + sizeof(Brec<T>) * (size_t)(C + kBndPad2 + kRecPad) + kCodePad2;
  const int na = (int)S.count;
  TcDesc d = {0, 0, 0, 0};
  if (lane < na) d = descs[stk_tc[S.first + lane]];
  const int rows = lane < na ? (int)(d.dims & 0xffff) + 2 : 0;
  const int incl = scan_add(rows);
  const int T_rows = __builtin_amdgcn_readlane(incl, 63);
  const int e_start = incl - rows, e_R = rows - 2;  // entry a in lane a
  const T init_Y = tab.init_const / (T)C;
  const uint8_t *hcode = pool + S.hap_off;
  for (int c = lane; c < C + kBndPad2; c += kWave) {
    Brec<T> b;
    b.z = (T)0;
    b.w = (T)0;
    bnd[c] = b;
  }
  for (int c = lane - kCodePad2; c < C + kBndPad2; c += kWave)
    hcol[c] = (c >= 1 && c <= C) ? hcode[c - 1] : (c == 0 ? 5 : (c < 0 ? 6 : 0));
  __syncthreads();

  const int nstripes = (T_rows + kRows2 - 1) / kRows2;
  for (int s = 0; s < nstripes; s++) {
    const int g0 = s * kRows2 + 2 * lane, g1 = g0 + 1;
    int lo = 0, hi = na - 1;
    while (__builtin_amdgcn_ballot_w64(lo < hi)) {
      const int mid = (lo + hi + 1) >> 1;
      const int sm = __shfl(e_start, mid);
      if (lo < hi) {
        if (sm <= g0) lo = mid; else hi = mid - 1;
      }
    }
    // row b: the same testcase, or the next one when it starts at g1
    const int nxt = __shfl(e_start, min(lo + 1, kWave - 1));
    const int lob = (lo + 1 < na && nxt <= g1) ? lo + 1 : lo;
    const int sa = __shfl(e_start, lo), Ra = __shfl(e_R, lo);
    const uint32_t rda = (uint32_t)__shfl((int)d.read_off, lo), oa = (uint32_t)__shfl((int)d.out_idx, lo);
    const int sb = __shfl(e_start, lob), Rb = __shfl(e_R, lob);
    const uint32_t rdb = (uint32_t)__shfl((int)d.read_off, lob), ob = (uint32_t)__shfl((int)d.out_idx, lob);
    const int ra = g0 - sa, rb = g1 - sb;
    const bool deadA = g0 >= T_rows, deadB = g1 >= T_rows;
    RowParams<T> PA, PB;
    LaneState<T> A, B;
    const T z_top = lane == 0 ? bnd[0].z : (T)0;
    setup_row<T>(2 * lane, deadA, ra, Ra, pool + rda, tab, init_Y, z_top, PA, A);
    setup_row<T>(2 * lane + 1, deadB, rb, Rb, pool + rdb, tab, init_Y, (T)0, PB, B);
    const uint64_t pa = __builtin_amdgcn_ballot_w64(!deadA && ra == Ra + 1);
    const uint64_t pb = __builtin_amdgcn_ballot_w64(!deadB && rb == Rb + 1);
    const bool more = s < nstripes - 1;
    const int steps = more ? C + kRows2 - 1 : C + (T_rows - s * kRows2) - 1;
    T *outA = raw_out + oa, *outB = raw_out + ob;
    if (pa | pb) {
      if (more)
        phmm_stripe2<T, true, true>(steps, A, B, PA, PB, bnd, hcol, C, lane, pa, pb, outA, outB);
      else
        phmm_stripe2<T, true, false>(steps, A, B, PA, PB, bnd, hcol, C, lane, pa, pb, outA, outB);
    } else {
      phmm_stripe2<T, false, true>(steps, A, B, PA, PB, bnd, hcol, C, lane, 0, 0, outA, outB);
    }
    __syncthreads();
  }
}

// W: the waves per SIMD the register allocation is held to (0: the compiler's own choice)
template <int W>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W ? W : 1, 8))) void phmm_forward2(
                                                     const Stack *__restrict__ stacks,
                                                     const uint32_t *__restrict__ stk_tc,
                                                     const TcDesc *__restrict__ descs,
                                                     const uint8_t *__restrict__ pool, DevTab<float> tab,
                                                     float *__restrict__ raw_out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  phmm_stack2<float>(stacks[blockIdx.x], stk_tc, descs, pool, tab, raw_out, smem_raw);
}

// f32 pass: one stack per workgroup (LPT order). f64 pass: a persistent grid takes stacks through
// counter[1] and recomputes their testcases whose f32 result fell below MIN_ACCEPTED; counter[0]
// counts them.
// kLong: stacks whose haplotype is longer than kLdsHaplen; their boundary records and codes live in
// `scratch` (scratch_stride bytes per workgroup, global memory: lane 63's record stores and lane 0's
// loads of the next stripe are ordered by the stripe's __syncthreads), and both passes take the
// stacks through a persistent grid (counter[2] f32, counter[3] f64).
template <typename T, bool kF64Pass, bool kLong = false, bool kExit = false>
__global__ __launch_bounds__(64) void phmm_forward(const Stack *__restrict__ stacks, int nstacks,
                                                    const uint32_t *__restrict__ stk_tc,
                                                    const TcDesc *__restrict__ descs,
                                                    const uint8_t *__restrict__ pool, DevTab<T> tab,
                                                    T *__restrict__ raw_out, const float *__restrict__ raw_f,
                                                    int *__restrict__ counter, int force, uint8_t *scratch,
                                                    size_t scratch_stride, const uint32_t *__restrict__ units) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  uint8_t *rec = kLong ? scratch + (size_t)blockIdx.x * scratch_stride : smem_raw;
  if constexpr (kF64Pass || kLong) {
    int done = 0;
    int *next = counter + (kLong ? (kF64Pass ? 3 : 2) : 1);
    // f64 pass over the LDS stacks: `parts` work units per stack (the top byte of `force`), so a job
    // of few stacks per worker balances its fallback work finer
    const int parts = (kF64Pass && !kLong) ? max(1, (force >> 8) & 0xFF) : 1;
    // with a plan (f64_plan / f64_plan_order): only the units that have work, costliest first
    const int nwork = units ? __builtin_amdgcn_readfirstlane(counter[kPlanTotal]) : nstacks * parts;
    while (true) {
      int k = 0;
      if (threadIdx.x == 0) k = atomicAdd(next, 1);
      k = __builtin_amdgcn_readfirstlane(__shfl(k, 0));
      if (k >= nwork) break;
      if (units) k = __builtin_amdgcn_readfirstlane((int)units[k]);
      done += phmm_stack<T, kF64Pass>(stacks[k / parts], stk_tc, descs, pool, tab, raw_out, raw_f, (force & 0xFF) != 0,
                                      rec, k % parts, parts);
      __syncthreads();  // the next stack re-initialises the records
    }
    if (kF64Pass && threadIdx.x == 0 && done) atomicAdd(counter, done);
  } else {
    phmm_stack<T, false, kExit>(stacks[blockIdx.x], stk_tc, descs, pool, tab, raw_out, nullptr, false, rec, 0, 1,
                                reinterpret_cast<unsigned long long *>(counter + 4));
  }
}

// f64 pass plan: the persistent grid's units (stack parts) ordered by their cost, costliest first, so
// the grid's tail is its cheapest units -- a 1/8 shard's f64 pass has only ~8 units per resident
// wave, and ordered by the f32 pass's stack order (its rows, not the fallback's) its last units were
// as long as any. f64_plan: per unit the stripes of its fallback rows times the columns a stripe
// sweeps, as a bucket key (0: no fallback row), and the buckets' counts; f64_plan_order: the units
// with work into `units`, by descending key (any order inside a bucket: a unit's outputs do not
// depend on when it runs).
__global__ __launch_bounds__(256) void f64_plan(const Stack *__restrict__ stacks, int nunits, int parts,
                                                const uint32_t *__restrict__ stk_tc, const TcDesc *__restrict__ descs,
                                                const float *__restrict__ raw_f, int force, uint8_t *__restrict__ ukey,
                                                int *__restrict__ counter) {
  __shared__ int hist[kPlanBuckets];
  for (int i = threadIdx.x; i < kPlanBuckets; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < nunits) {
    const Stack S = stacks[u / parts];
    const int part = u % parts, lo = part * (int)S.count / parts, hi = (part + 1) * (int)S.count / parts;
    int rows = 0;
    for (int a = lo; a < hi; a++) {
      const TcDesc d = descs[stk_tc[S.first + a]];
      if (force || raw_f[d.out_idx] < 1e-28f) rows += (int)(d.dims & 0xffff) + 2;  // as phmm_stack's `act`
    }
    int key = 0;
    if (rows) {
      key = (((rows + kWave - 1) / kWave) * ((int)S.C + kWave) + 63) / 64;
      key = key < 1 ? 1 : (key > kPlanBuckets - 1 ? kPlanBuckets - 1 : key);
      atomicAdd(&hist[key], 1);
    }
    ukey[u] = (uint8_t)key;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kPlanBuckets; i += blockDim.x)
    if (hist[i]) atomicAdd(&counter[kPlanCount + i], hist[i]);
}

__global__ __launch_bounds__(256) void f64_plan_order(int nunits, const uint8_t *__restrict__ ukey,
                                                      int *__restrict__ counter, uint32_t *__restrict__ units) {
  __shared__ int cnt[kPlanBuckets], off[kPlanBuckets], hist[kPlanBuckets], base[kPlanBuckets];
  for (int i = threadIdx.x; i < kPlanBuckets; i += blockDim.x) {
    cnt[i] = counter[kPlanCount + i];
    hist[i] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // bucket offsets, descending key
    int sum = 0;
    for (int k = kPlanBuckets - 1; k >= 1; k--) {
      off[k] = sum;
      sum += cnt[k];
    }
    if (blockIdx.x == 0) counter[kPlanTotal] = sum;
  }
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  const int key = u < nunits ? ukey[u] : 0;
  int rank = 0;
  if (key) rank = atomicAdd(&hist[key], 1);
  __syncthreads();
  for (int i = threadIdx.x; i < kPlanBuckets; i += blockDim.x)
    if (hist[i]) base[i] = atomicAdd(&counter[kPlanCursor + i], hist[i]);
  __syncthreads();
  if (key) units[off[key] + base[key] + rank] = (uint32_t)u;
}

// gb_phmm_init's warm-up launch (no work)
__global__ void phmm_warm(int *count) {
  if (threadIdx.x == 0 && blockIdx.x == 0) count[3] = 0;
}

// Device log10 epilogue (IntelPairHmmCSource.cpp:73-79); the host path recomputes it bit-exactly.
__global__ void phmm_finalize(const float *__restrict__ rf, const double *__restrict__ rd,
                              const uint8_t *__restrict__ used, double *__restrict__ out, int n,
                              float log10_init_f, double log10_init_d) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (rf[i] < 1e-28f) ? (log10(rd[i]) - log10_init_d) : (double)(log10f(rf[i]) - log10_init_f);
}

// ---------------------------------------------------------------------------------------------
// Host state
// ---------------------------------------------------------------------------------------------
struct DeviceTables {
  int device = -1;
  float *f = nullptr;   // ph2pr | one_minus | div3 | m2m
  double *d = nullptr;
  HostTables<float> hf;
  HostTables<double> hd;
};

std::mutex g_mu;
HostTables<float> *g_hf = nullptr;
HostTables<double> *g_hd = nullptr;
std::unordered_map<int, DeviceTables *> g_dev;

int ensure_host_tables() {
  if (!g_hf) {
    auto *f = new HostTables<float>();
    auto *d = new HostTables<double>();
    build_tables(*f);
    build_tables(*d);
    g_hf = f;
    g_hd = d;
  }
  return GB_OK;
}

template <typename T>
int upload_tables(const HostTables<T> &h, T **dst) {
  const size_t nel = 3 * kQualTab + kM2M;
  std::vector<T> blob(nel);
  std::memcpy(blob.data(), h.ph2pr, sizeof(T) * kQualTab);
  std::memcpy(blob.data() + kQualTab, h.one_minus, sizeof(T) * kQualTab);
  std::memcpy(blob.data() + 2 * kQualTab, h.div3, sizeof(T) * kQualTab);
  std::memcpy(blob.data() + 3 * kQualTab, h.m2m, sizeof(T) * kM2M);
  GB_HIP(hipMalloc(dst, sizeof(T) * nel));
  GB_HIP(hipMemcpy(*dst, blob.data(), sizeof(T) * nel, hipMemcpyHostToDevice));
  return GB_OK;
}

int get_device_tables(DeviceTables **out) {
  std::lock_guard<std::mutex> lk(g_mu);
  ensure_host_tables();
  int dev = -1;
  GB_HIP(hipGetDevice(&dev));
  auto it = g_dev.find(dev);
  if (it != g_dev.end()) {
    *out = it->second;
    return GB_OK;
  }
  auto *t = new DeviceTables();
  t->device = dev;
  t->hf = *g_hf;
  t->hd = *g_hd;
  int st = upload_tables(*g_hf, &t->f);
  if (st) return st;
  st = upload_tables(*g_hd, &t->d);
  if (st) return st;
  for (auto fn : {(const void *)phmm_forward<float, false>, (const void *)phmm_forward<float, false, false, true>,
                  (const void *)phmm_forward<double, true>, (const void *)phmm_forward2<0>, (const void *)phmm_forward2<6>, (const void *)phmm_forward2<8>})
    GB_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  g_dev[dev] = t;
  *out = t;
  return GB_OK;
}

template <typename T>
DevTab<T> dev_tab(const T *base, T init_const) {
  DevTab<T> t;
  t.ph2pr = base;
  t.one_minus = base + kQualTab;
  t.div3 = base + 2 * kQualTab;
  t.m2m = base + 3 * kQualTab;
  t.init_const = init_const;
  return t;
}

// Deduplication keys: the caller shares read/haplotype buffers across the R x H cross product
// (PairHMMUnitTest.cpp:564-579); identical pointers + length => identical packed record.
struct ReadKey {
  const char *rs, *q, *i, *d, *c;
  int len;
  bool operator==(const ReadKey &o) const {
    return rs == o.rs && q == o.q && i == o.i && d == o.d && c == o.c && len == o.len;
  }
};
struct HapKey {
  const char *h;
  int len;
  bool operator==(const HapKey &o) const { return h == o.h && len == o.len; }
};
struct KeyHash {
  size_t mix(size_t a, size_t b) const { return a ^ (b + 0x9e3779b97f4a7c15ull + (a << 6) + (a >> 2)); }
  size_t operator()(const ReadKey &k) const {
    size_t h = std::hash<const void *>()(k.rs);
    for (const void *p : {(const void *)k.q, (const void *)k.i, (const void *)k.d, (const void *)k.c})
      h = mix(h, std::hash<const void *>()(p));
    return mix(h, (size_t)k.len);
  }
  size_t operator()(const HapKey &k) const { return mix(std::hash<const void *>()(k.h), (size_t)k.len); }
};

}  // namespace

struct gb_phmm_batch {
  DeviceTables *tabs = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  int n = 0;
  int max_haplen = 0;
  int64_t cells = 0;
  uint8_t *h_stage = nullptr;  // pinned upload staging (grow-only)
  size_t cap_stage = 0;
  void *d_arena = nullptr;  // holds d_desc, d_rf, d_rd, d_out, d_stk_tc, d_stacks
  TcDesc *d_desc = nullptr;
  uint8_t *d_pool = nullptr;
  float *d_rf = nullptr;
  double *d_rd = nullptr;
  double *d_out = nullptr;
  uint32_t *d_stk_tc = nullptr;  // testcase indices, stack by stack
  Stack *d_stacks = nullptr;     // LPT order
  int nstacks = 0;                 // stacks whose haplotype fits the LDS (the first nstacks)
  int n_long = 0;                  // stacks behind them whose haplotype does not (kLong kernels)
  int long_grid = 0;               // their persistent grid
  uint8_t *d_scratch = nullptr;    // their boundary records, scratch_stride bytes per workgroup
  size_t scratch_stride = 0, cap_scratch = 0;
  int *d_count = nullptr;  // [0] testcases recomputed by the f64 pass, [1] its stack counter,
                           // [4..7] the f32 early exit's two u64 counts (testcases, cells skipped),
                           // [2] / [3] the kLong f32 / f64 stack counters, then the f64 plan's words
                           // (kCountWords in all)
  uint32_t *d_units = nullptr;  // f64 plan: units with work, costliest first (kMaxF64Parts per testcase)
  uint8_t *d_ukey = nullptr;    // f64 plan: per unit its cost bucket
  size_t cap_n = 0, cap_pool = 0;  // allocated capacities (a cached workspace batch is refilled)
  int f64_grid = 0;                // persistent f64 grid: resident workgroups of the device
  int cus = 256;                   // compute units of the device (stack height rule)
  bool ran = false;
  bool force_f64 = false;
  int rpl = 1;  // rows per lane of the f32 pass over LDS stacks (GB_PHMM_RPL=2: two, for A/B probes)
  int w2 = 0;   // its register budget: waves per SIMD 0 (compiler), 6 or 8 (GB_PHMM_W2, probes)
  int f64_parts = 2;  // work units per stack in the f64 pass (GB_PHMM_F64_PARTS)
  bool f64_plan = true;  // the f64 pass's units by cost (f64_plan; GB_PHMM_F64_PLAN=0: stack order)
  bool f32_exit = true;  // the f32 pass's early exit (phmm_stack kExit; GB_PHMM_EXIT=0 turns it off)
  // host scratch of the fills (grow-only, host_reserve)
  std::vector<uint32_t> hid;
  std::vector<Stack> stacks;
  std::vector<uint64_t> skeys;
  std::vector<std::vector<uint8_t>> pools;
};

namespace {
int warm_up(DeviceTables *t);
}

extern "C" {

int gb_phmm_init(void) {
  DeviceTables *t = nullptr;
  int st = get_device_tables(&t);
  if (st) return st;
  return warm_up(t);
}

}  // extern "C"

namespace {

// GB_PHMM_HOSTPROF=1: host phase times of the drop-in path on stderr (development aid)
struct HostClock {
  bool on;
  std::chrono::steady_clock::time_point t0;
  HostClock() : on(getenv("GB_PHMM_HOSTPROF") != nullptr), t0(std::chrono::steady_clock::now()) {}
  void mark(const char *what) {
    if (!on) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[phmm host] %s %.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
    t0 = t;
  }
};

// Device buffers of a batch for n testcases and a pool of pool_bytes (grow-only). The pipelined path
// reserves every chunk's buffers before its first launch: an allocation that grows a buffer frees
// the old one, and hipFree waits for the device.
int batch_reserve(gb_phmm_batch *b, int n, size_t pool_bytes) {
  const size_t nn = std::max(n, 1);
  if (nn > b->cap_n) {
    // the six per-testcase arrays carved from one allocation (a cold process pays per hipMalloc)
    (void)hipFree(b->d_arena);
    b->d_arena = nullptr;
    b->d_desc = nullptr;
    b->d_rf = nullptr;
    b->d_rd = b->d_out = nullptr;
    b->d_stk_tc = nullptr;
    b->d_stacks = nullptr;
    b->d_units = nullptr;
    b->d_ukey = nullptr;
    b->cap_n = 0;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t sz[8] = {up(sizeof(TcDesc) * nn), up(sizeof(float) * nn), up(sizeof(double) * nn),
                          up(sizeof(double) * nn), up(sizeof(uint32_t) * nn),
                          up(sizeof(Stack) * nn),  // at most one stack per testcase
                          up(sizeof(uint32_t) * nn * kMaxF64Parts), up(nn * kMaxF64Parts)};
    GB_HIP(hipMalloc(&b->d_arena, sz[0] + sz[1] + sz[2] + sz[3] + sz[4] + sz[5] + sz[6] + sz[7]));
    uint8_t *a = (uint8_t *)b->d_arena;
    b->d_desc = (TcDesc *)a;
    a += sz[0];
    b->d_rf = (float *)a;
    a += sz[1];
    b->d_rd = (double *)a;
    a += sz[2];
    b->d_out = (double *)a;
    a += sz[3];
    b->d_stk_tc = (uint32_t *)a;
    a += sz[4];
    b->d_stacks = (Stack *)a;
    a += sz[5];
    b->d_units = (uint32_t *)a;
    a += sz[6];
    b->d_ukey = a;
    b->cap_n = nn;
  }
  if (pool_bytes > b->cap_pool) {
    (void)hipFree(b->d_pool);
    b->d_pool = nullptr;
    b->cap_pool = 0;
    GB_HIP(hipMalloc(&b->d_pool, pool_bytes));
    b->cap_pool = pool_bytes;
  }
  if (!b->d_count) GB_HIP(hipMalloc(&b->d_count, kCountWords * sizeof(int)));
  return GB_OK;
}

// grow-only pinned staging buffer of a batch (uploads, results); its first `keep` bytes survive a growth
int stage_reserve(gb_phmm_batch *b, size_t bytes, size_t keep = 0) {
  if (bytes <= b->cap_stage) return GB_OK;
  uint8_t *h = nullptr;
  GB_HIP(hipHostMalloc((void **)&h, bytes, hipHostMallocDefault));
  if (b->h_stage) {
    if (keep) std::memcpy(h, b->h_stage, std::min(keep, b->cap_stage));
    (void)hipHostFree(b->h_stage);
  }
  b->h_stage = h;
  b->cap_stage = bytes;
  return GB_OK;
}

// Host scratch of a batch's fills for n testcases and pack pools of pool_bytes in all, kept across
// fills and touched here: a fresh vector pays a page fault per 4 KiB at its first write, and several
// fills faulting at once serialise on the process's memory map.
void host_reserve(gb_phmm_batch *b, size_t n, size_t pool_bytes, int threads) {
  if (b->hid.size() < n) b->hid.assign(n, 0);
  if (b->stacks.size() < n) b->stacks.assign(n, Stack{});
  if (b->skeys.size() < 2 * n) b->skeys.assign(2 * n, 0);
  if ((int)b->pools.size() < threads) b->pools.resize(threads);
  for (int t = 0; t < threads; t++) {
    auto &P = b->pools[t];
    const size_t want = pool_bytes / threads + 4096;
    if (P.capacity() < want) {
      P.clear();
      P.shrink_to_fit();
      P.resize(want);  // touch
    }
    P.clear();
  }
}

// Staging layout of a fill of n testcases and a pool of pool_bytes: descriptors | stack testcase
// lists | stacks (at most one per testcase) | pool
struct StageLayout {
  size_t o_tc, o_stk, o_pool, total;
  StageLayout(size_t n, size_t pool_bytes) {
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    o_tc = up(sizeof(TcDesc) * n);
    o_stk = o_tc + up(sizeof(uint32_t) * n);
    o_pool = o_stk + up(sizeof(Stack) * n);
    total = o_pool + up(pool_bytes) + 256;
  }
};

// The limits of include/gb_phmm.h, checked before any device work; the error names the first bad
// testcase by its index in the caller's array.
int validate_testcases(const gb_testcase *tcs, int n) {
  for (int k = 0; k < n; k++) {
    const gb_testcase &t = tcs[k];
    GB_ARG(t.rslen >= 1 && t.rslen <= 65535, "testcase %d: rslen %d outside [1,65535]", k, t.rslen);
    GB_ARG(t.haplen >= 1 && t.haplen <= kMaxHaplen, "testcase %d: haplen %d outside [1,%d]", k,
           t.haplen, kMaxHaplen);
    GB_ARG(t.rs && t.q && t.i && t.d && t.c && t.hap, "testcase %d: null sequence pointer", k);
  }
  return GB_OK;
}

// Pack the testcases (deduplicated reads/haplotypes, stacks in LPT order) into b's pinned staging
// buffer and upload them, growing its buffers when they are too small; b's stream/events exist
// already. threads: host threads of the pack and merge phases (0: up to 8 from pack_min testcases).
// validated: the caller has run validate_testcases over the whole call (compute_pipelined, whose
// chunks would otherwise name a testcase by its index in the chunk).
int batch_fill(gb_phmm_batch *b, const gb_testcase *tcs, int n, int threads = 0, bool validated = false) {
  HostClock clk;
  // Pack: deduplicate reads and haplotypes by pointer (the driver shares them across the R x H
  // cross product, PairHMMUnitTest.cpp:564-579), convert bases to codes once. Inputs are validated
  // first (sequentially, so the error names the first bad testcase), then big jobs pack in
  // contiguous chunks on several threads, each with its own pool and maps; chunk pools are
  // concatenated and haplotype ids are made global in first-appearance order, which is the id order
  // a single pass gives (a read shared across a chunk edge is stored once per chunk). Descriptors,
  // stack lists, stacks and pool are written straight into the pinned staging buffer.
  if (!validated)
    if (int st = validate_testcases(tcs, n)) return st;
  clk.mark("validate");
  // calls from 8 K testcases pack on several threads (2 K testcases each at least): the reference's
  // per-batch calls (PairHMMUnitTest.cpp:549-593) are mostly 5-45 K testcases
  int pack_min = 1 << 13;  // GB_PHMM_PACK_MIN (probes): the smallest call packed on several threads
  if (const char *e = getenv("GB_PHMM_PACK_MIN")) pack_min = std::max(1, atoi(e));
  int nth = n >= pack_min ? (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency())) : 1;
  if (threads > 0) nth = std::max(1, std::min(threads, n / 4096));
  nth = std::max(1, std::min(nth, n / 2048));
  const size_t nn = std::max(n, 1);
  host_reserve(b, nn, 0, nth);
  // descriptors are written by the pack (a bigger pool than guessed grows the buffer after it)
  if (int st = stage_reserve(b, StageLayout(nn, 32 * nn).total)) return st;
  TcDesc *desc = (TcDesc *)b->h_stage;
  uint32_t *hid = b->hid.data();  // dense haplotype index of each testcase (stack grouping)
  struct Chunk {
    int lo = 0, hi = 0;
    std::vector<uint8_t> *pool = nullptr;
    std::vector<uint32_t> hap_off;  // local haplotype id -> offset in this chunk's pool
    std::vector<HapKey> hap_key;    // local haplotype id -> key
    int64_t cells = 0;
  };
  std::vector<Chunk> ch(nth);
  auto pack_chunk = [&](Chunk &C) {
    std::unordered_map<ReadKey, uint32_t, KeyHash> read_at;
    std::unordered_map<HapKey, uint32_t, KeyHash> hap_at;
    // the reference driver's r-major loop repeats a read for every haplotype and cycles the
    // haplotypes: a last-read check and a small direct-mapped haplotype cache skip most hash lookups
    ReadKey last_rk{nullptr, nullptr, nullptr, nullptr, nullptr, -1};
    uint32_t last_roff = 0;
    struct HapSlot {
      const char *h = nullptr;
      int len = -1;
      uint32_t id = 0;
    };
    HapSlot hcache[256];
    std::vector<uint8_t> &pool = *C.pool;
    for (int k = C.lo; k < C.hi; k++) {
      const gb_testcase &t = tcs[k];
      const ReadKey rk{t.rs, t.q, t.i, t.d, t.c, t.rslen};
      uint32_t roff;
      if (rk == last_rk) {
        roff = last_roff;
      } else {
        auto ri = read_at.find(rk);
        if (ri != read_at.end()) {
          roff = ri->second;
        } else {
          roff = (uint32_t)pool.size();
          pool.resize(pool.size() + 5 * (size_t)t.rslen);
          uint8_t *rec = pool.data() + roff;
          for (int r = 0; r < t.rslen; r++) {
            rec[r] = read_match_mask(base_code(t.rs[r]));
            rec[t.rslen + r] = (uint8_t)t.q[r];
            rec[2 * t.rslen + r] = (uint8_t)t.i[r];
            rec[3 * t.rslen + r] = (uint8_t)t.d[r];
            rec[4 * t.rslen + r] = (uint8_t)t.c[r];
          }
          read_at.emplace(rk, roff);
        }
      }
      last_rk = rk;
      last_roff = roff;
      const HapKey hk{t.hap, t.haplen};
      HapSlot &hs = hcache[(((uintptr_t)t.hap) >> 4) & 255];
      uint32_t id;
      if (hs.h == t.hap && hs.len == t.haplen) {
        id = hs.id;
      } else {
        auto hi = hap_at.find(hk);
        if (hi != hap_at.end()) {
          id = hi->second;
        } else {
          id = (uint32_t)C.hap_off.size();
          const uint32_t hoff = (uint32_t)pool.size();
          pool.resize(pool.size() + (size_t)t.haplen);
          for (int c = 0; c < t.haplen; c++) pool[hoff + c] = base_code(t.hap[c]);
          hap_at.emplace(hk, id);
          C.hap_off.push_back(hoff);
          C.hap_key.push_back(hk);
        }
        hs.h = t.hap;
        hs.len = t.haplen;
        hs.id = id;
      }
      hid[k] = id;  // local until the merge
      // read offset chunk-relative and the local haplotype id until the merge
      desc[k] = TcDesc{roff, 0, (uint32_t)t.rslen | ((uint32_t)t.haplen << 16), (uint32_t)k};
      C.cells += (int64_t)t.rslen * t.haplen;
    }
  };
  for (int t = 0; t < nth; t++) {
    ch[t].lo = (int)((int64_t)n * t / nth);
    ch[t].hi = (int)((int64_t)n * (t + 1) / nth);
    ch[t].pool = &b->pools[t];
    ch[t].pool->clear();
  }
  if (nth == 1) {
    pack_chunk(ch[0]);
  } else {
    std::vector<std::thread> th;
    for (int t = 1; t < nth; t++) th.emplace_back(pack_chunk, std::ref(ch[t]));
    pack_chunk(ch[0]);
    for (auto &x : th) x.join();
  }
  clk.mark("pack");
  // merge: chunk pool bases, global haplotype ids (first appearance), one pool in the staging buffer
  std::vector<size_t> base(nth + 1, 0);
  for (int t = 0; t < nth; t++) base[t + 1] = base[t] + ch[t].pool->size();
  GB_ARG(base[nth] < (1ull << 32), "batch pool exceeds 4 GiB");
  const size_t pool_bytes = std::max<size_t>((base[nth] + 15) & ~size_t(15), 16);
  const StageLayout L(nn, pool_bytes);
  if (int st = stage_reserve(b, L.total, sizeof(TcDesc) * nn)) return st;
  desc = (TcDesc *)b->h_stage;
  uint8_t *h_pool = b->h_stage + L.o_pool;
  std::vector<uint32_t> hap_off_of;
  std::vector<std::vector<uint32_t>> gid(nth);
  {
    std::unordered_map<HapKey, uint32_t, KeyHash> hap_at;
    for (int t = 0; t < nth; t++) {
      gid[t].resize(ch[t].hap_off.size());
      for (size_t h = 0; h < ch[t].hap_off.size(); h++) {
        auto it = hap_at.find(ch[t].hap_key[h]);
        if (it == hap_at.end()) {
          it = hap_at.emplace(ch[t].hap_key[h], (uint32_t)hap_off_of.size()).first;
          hap_off_of.push_back((uint32_t)(base[t] + ch[t].hap_off[h]));
        }
        gid[t][h] = it->second;
      }
    }
  }
  int64_t cells = 0;
  for (int t = 0; t < nth; t++) cells += ch[t].cells;
  auto merge_chunk = [&](int t) {
    if (!ch[t].pool->empty()) std::memcpy(h_pool + base[t], ch[t].pool->data(), ch[t].pool->size());
    for (int k = ch[t].lo; k < ch[t].hi; k++) {
      hid[k] = gid[t][hid[k]];
      desc[k].read_off += (uint32_t)base[t];
      desc[k].hap_off = hap_off_of[hid[k]];
    }
  };
  if (nth == 1) {
    merge_chunk(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 1; t < nth; t++) th.emplace_back(merge_chunk, t);
    merge_chunk(0);
    for (auto &x : th) x.join();
  }
  std::memset(h_pool + base[nth], 0, pool_bytes - base[nth]);
  clk.mark("merge");
  // Stacks (phmm_stack): testcases grouped by haplotype, stacked up to kStackRows rows (R + 2 per
  // testcase) and 64 testcases; longest-processing-time first (the dispatcher hands out workgroups
  // in grid order).
  uint32_t *order = (uint32_t *)(b->h_stage + L.o_tc);  // the stacks' testcase lists
  {  // counting sort by haplotype (stable: testcases keep their order within a haplotype)
    std::vector<int> first(hap_off_of.size() + 1, 0);
    for (int k = 0; k < n; k++) first[hid[k] + 1]++;
    for (size_t h = 0; h < hap_off_of.size(); h++) first[h + 1] += first[h];
    for (int k = 0; k < n; k++) order[first[hid[k]]++] = (uint32_t)k;
  }
  clk.mark("haplotype order");
  // Stack height adapts to the job: tall stacks waste the least on partial stripes, but a job of
  // few stacks per resident wave leaves the grid's tail -- one whole stack -- exposed, and the f64
  // pass's persistent grid balances finer pieces better. 2048 rows from 4 stacks per resident wave
  // (32 per CU) up, 512 below 16 stacks per CU, 1024 between. Measured (tools/phmm_shard_probe.py,
  // profiles/r05w_phmm_rows.log, r05x): the 'large' job 2048 / 1024 / 512 rows 32.3 / 32.6 / 33.6 ms,
  // its 1/2, 1/4 and 1/8 shards best at 1024 (1/4: 8.57 ms against 8.76-8.80 at 512 / 2048; 1/8:
  // 4.48 against 4.53 / 4.74), the 'small' job 1024 (4.27 against 4.41 at 512) and its 1/8 shard,
  // 2.75 M rows, 512 (0.83 ms against 0.90 at 1024).
  int64_t total_rows = 0;
  for (int k = 0; k < n; k++) total_rows += (int64_t)(desc[k].dims & 0xffff) + 2;
  // one row per lane: the two-row form (phmm_forward2) issues 125 VALU per 8 cells against 67 per 4
  // but measured slower at every register budget (f32 19.1 ms; two rows 19.8 / 20.6 / 20.9 ms at 5 /
  // 6 / 8 waves per SIMD, profiles/r05b_phmm_rpl_ab.log); GB_PHMM_RPL=2 selects it for A/B probes
  b->rpl = 1;
  if (const char *e = getenv("GB_PHMM_RPL")) b->rpl = atoi(e) == 2 ? 2 : 1;
  b->w2 = 0;
  if (const char *e = getenv("GB_PHMM_W2")) b->w2 = atoi(e);
  // work units per stack in the f64 pass: in stack order, two units per stack took the 1/8 shard's
  // f64 pass 2.28 -> 2.00 ms (profiles/r05e_phmm_f64_parts.log); ordered by cost (f64_plan) one unit
  // per stack is best: the shard 1.93 (stack order, two) -> 1.82 (plan, two) -> 1.78 ms (plan, one), the
  // whole job 13.19 -> 13.07 -> 12.95 ms (profiles/r06x_phmm_f64_plan.log)
  b->f64_parts = 1;
  if (const char *e = getenv("GB_PHMM_F64_PARTS")) b->f64_parts = std::max(1, std::min(kMaxF64Parts, atoi(e)));
  b->f64_plan = true;
  if (const char *e = getenv("GB_PHMM_F64_PLAN")) b->f64_plan = atoi(e) != 0;
  // the f32 pass drops a testcase's remaining rows once its crossing mass proves it falls back to f64
  // (phmm_stack kExit): f32 pass 19.05 -> 18.40 ms, step +2.0 % (profiles/r05zzi_phmm_exit_ab.log);
  // finals, raw f64 and the fallback choice unchanged, a dropped testcase's raw f32 reads 0
  b->f32_exit = true;
  if (const char *e = getenv("GB_PHMM_EXIT")) b->f32_exit = atoi(e) != 0;
  int stack_rows = kStackRows;
  if (total_rows / stack_rows < 4ll * 32 * b->cus) stack_rows = 1024;
  if (stack_rows == 1024 && total_rows / stack_rows < 16ll * b->cus) stack_rows = 512;
  // a small call (one of the reference's per-batch calls) is its longest stack: below 2 stacks per
  // SIMD the stacks shrink further, to 128 rows
  while (stack_rows > 128 && total_rows / stack_rows < 8ll * b->cus) stack_rows /= 2;
  if (const char *e = getenv("GB_PHMM_STACK_ROWS")) stack_rows = std::max(1, atoi(e));  // probes
  // sort keys: long-haplotype stacks last (they run on the kLong kernels), then decreasing cost,
  // then stack index (so the order is the stable one)
  Stack *stacks = b->stacks.data();
  uint64_t *key = b->skeys.data(), *key2 = key + nn;
  int ns_all = 0, n_long = 0, max_h_short = 0, max_h_long = 0;
  const int sh = b->rpl == 2 ? kRows2 : kWave;  // stripe height of the f32 pass
  for (int k = 0; k < n;) {
    const uint32_t h = desc[order[k]].hap_off;
    const int C = (int)(desc[order[k]].dims >> 16);
    Stack S{(uint32_t)k, 0, h, (uint32_t)C};
    int rows = 0;
    while (k < n && desc[order[k]].hap_off == h && S.count < (uint32_t)kWave &&
           (S.count == 0 || rows + (int)(desc[order[k]].dims & 0xffff) + 2 <= stack_rows)) {
      rows += (int)(desc[order[k]].dims & 0xffff) + 2;
      S.count++;
      k++;
    }
    const bool is_long = C > kLdsHaplen;
    if (is_long) {
      n_long++;
      max_h_long = std::max(max_h_long, C);
    } else {
      max_h_short = std::max(max_h_short, C);
    }
    const uint64_t cost = std::min<uint64_t>((uint64_t)((rows + sh - 1) / sh) * (uint64_t)(C + sh), 0x7fffffffu);
    key[ns_all] = ((uint64_t)is_long << 63) | ((0x7fffffffu - cost) << 32) | (uint32_t)ns_all;
    stacks[ns_all++] = S;
  }
  clk.mark("stack build");
  {  // LSD radix sort of the keys' upper 32 bits, 8 bits a pass (the low 32 bits are the index)
    uint32_t cnt[256];
    for (int shift = 32; shift < 64; shift += 8) {
      const uint64_t d0 = ns_all ? (key[0] >> shift) & 255 : 0;
      bool same = true;
      for (int k = 1; k < ns_all && same; k++) same = ((key[k] >> shift) & 255) == d0;
      if (same) continue;
      std::memset(cnt, 0, sizeof(cnt));
      for (int k = 0; k < ns_all; k++) cnt[(key[k] >> shift) & 255]++;
      for (uint32_t d = 0, sum = 0; d < 256; d++) {
        const uint32_t c = cnt[d];
        cnt[d] = sum;
        sum += c;
      }
      for (int k = 0; k < ns_all; k++) key2[cnt[(key[k] >> shift) & 255]++] = key[k];
      std::swap(key, key2);
    }
  }
  Stack *h_stacks = (Stack *)(b->h_stage + L.o_stk);
  for (int k = 0; k < ns_all; k++) h_stacks[k] = stacks[(uint32_t)key[k]];
  // Tail split: the stacks holding the last 10 % of the LPT order's cost are cut into stacks of at
  // most 512 rows (taller stacks waste less on the anti-diagonal fill; shorter ones let the grid's
  // last waves end together). Measured (tools/phmm_shard_probe.py, profiles/r06h/r06i): the 'large'
  // job 31.93-32.00 -> 31.65 ms, its 1/8 shard 4.47-4.49 -> 4.41-4.46 ms; 5 / 15 / 20 / 30 % and
  // 128 / 256 / 384-row pieces no better on the job. GB_PHMM_TAIL=frac:rows (0 = off) for probes.
  double frac = stack_rows > 512 ? 0.10 : 0.0;
  int trows = 512;
  if (const char *te = getenv("GB_PHMM_TAIL")) {
    frac = atof(te);
    const char *cm = strchr(te, ':');
    if (cm) trows = std::max(1, atoi(cm + 1));
  }
  if (frac > 0) {
    const int ns_short = ns_all - n_long;
    auto cost_of = [&](const Stack &S) -> uint64_t {
      int rows = 0;
      for (uint32_t t = 0; t < S.count; t++) rows += (int)(desc[order[S.first + t]].dims & 0xffff) + 2;
      return (uint64_t)((rows + sh - 1) / sh) * (uint64_t)(S.C + sh);
    };
    uint64_t total = 0;
    for (int k = 0; k < ns_short; k++) total += cost_of(h_stacks[k]);
    uint64_t acc = 0;
    int t0 = ns_short;
    while (t0 > 0 && (double)acc < frac * (double)total) acc += cost_of(h_stacks[--t0]);
    std::vector<std::pair<uint64_t, Stack>> pieces;
    for (int k = t0; k < ns_short; k++) {
      const Stack S = h_stacks[k];
      uint32_t t = 0;
      while (t < S.count) {
        Stack P{S.first + t, 0, S.hap_off, S.C};
        int rows = 0;
        while (t < S.count && (P.count == 0 || rows + (int)(desc[order[S.first + t]].dims & 0xffff) + 2 <= trows)) {
          rows += (int)(desc[order[S.first + t]].dims & 0xffff) + 2;
          P.count++;
          t++;
        }
        pieces.push_back({(uint64_t)((rows + sh - 1) / sh) * (uint64_t)(S.C + sh), P});
      }
    }
    std::stable_sort(pieces.begin(), pieces.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
    std::vector<Stack> longs(h_stacks + ns_short, h_stacks + ns_all);
    int k = t0;
    for (const auto &pc : pieces) h_stacks[k++] = pc.second;
    for (const auto &ls : longs) h_stacks[k++] = ls;
    ns_all = k;
  }
  clk.mark("stacks");
  if (int st = batch_reserve(b, n, pool_bytes)) return st;
  if (n_long) {
    // records + codes of one long stack per workgroup of the persistent kLong grid
    b->long_grid = std::min(n_long, b->f64_grid);
    b->scratch_stride = (sizeof(Brec<double>) * (size_t)(max_h_long + kBndPad + kRecPad) +
                         (size_t)(max_h_long + kBndPad + kWave) + 16 + 255) & ~(size_t)255;
    const size_t need = b->scratch_stride * (size_t)b->long_grid;
    if (need > b->cap_scratch) {
      (void)hipFree(b->d_scratch);
      b->d_scratch = nullptr;
      b->cap_scratch = 0;
      GB_HIP(hipMalloc(&b->d_scratch, need));
      b->cap_scratch = need;
    }
  }
  // the uploads go through the pinned staging buffer: a pageable copy is staged by the runtime, and
  // while an earlier chunk's kernels held the GPU one chunk's upload waited 10-15 ms for it
  // (profiles/r05j_phmm_cli.log); a pinned copy is a plain DMA
  if (n) {
    GB_HIP(hipMemcpyAsync(b->d_desc, desc, sizeof(TcDesc) * n, hipMemcpyHostToDevice, b->stream));
    GB_HIP(hipMemcpyAsync(b->d_stk_tc, order, sizeof(uint32_t) * n, hipMemcpyHostToDevice, b->stream));
    GB_HIP(hipMemcpyAsync(b->d_stacks, h_stacks, sizeof(Stack) * ns_all, hipMemcpyHostToDevice, b->stream));
  }
  GB_HIP(hipMemcpyAsync(b->d_pool, h_pool, pool_bytes, hipMemcpyHostToDevice, b->stream));
  GB_HIP(hipStreamSynchronize(b->stream));  // the staging buffer is reused by the next fill
  clk.mark("upload");
  b->n = n;
  b->nstacks = ns_all - n_long;
  b->n_long = n_long;
  b->max_haplen = max_h_short;
  b->cells = cells;
  b->ran = false;
  return GB_OK;
}

int batch_new(DeviceTables *tabs, gb_phmm_batch **out) {
  auto *b = new gb_phmm_batch();
  b->tabs = tabs;
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, tabs->device) != hipSuccess) cus = 256;
  b->f64_grid = cus * 16;
  if (const char *e = getenv("GB_PHMM_F64_GRID")) b->f64_grid = cus * std::max(1, std::min(32, atoi(e)));  // probe
  b->cus = cus;
  hipError_t e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
  for (auto &ev : b->ev)
    if (e == hipSuccess) e = hipEventCreate(&ev);
  if (e != hipSuccess) {
    gb::set_error("gb_phmm_batch_create: %s", hipGetErrorString(e));
    gb_phmm_batch_destroy(b);
    return GB_ERR_HIP;
  }
  *out = b;
  return GB_OK;
}

// gb_phmm_compute's workspace: one batch per (host thread, device), refilled on every call so the
// reference's once-per-batch computelikelihoodsboth does not create streams, events and buffers
// each time. Kept for the life of the thread's process (never freed: freeing at thread exit could
// run after the HIP runtime is torn down).
gb_phmm_batch *thread_workspace(DeviceTables *tabs, int *st, int slot = 0) {
  thread_local std::unordered_map<int, std::vector<gb_phmm_batch *>> ws;
  auto &v = ws[tabs->device];
  if ((int)v.size() <= slot) v.resize(slot + 1, nullptr);
  if (v[slot]) return v[slot];
  gb_phmm_batch *b = nullptr;
  *st = batch_new(tabs, &b);
  if (*st) return nullptr;
  v[slot] = b;
  return b;
}

constexpr int kPipeMinChunk = 65536;  // testcases per chunk from three chunks on
constexpr int kPipeMin2 = 16384;      // the smallest call pipelined (two chunks)
constexpr int kPipeMaxChunks = 4;

// gb_phmm_init (the reference's initPairHMM, called before its timed loop) also readies what the
// first computation would otherwise pay for inside it: the code objects of the kernels (loaded at
// their first launch: empty launches here) and this thread's pipeline workspaces (streams, events).
int warm_up(DeviceTables *t) {
  int st = GB_OK;
  gb_phmm_batch *b = thread_workspace(t, &st, 0);
  if (!b) return st;
  if ((st = batch_reserve(b, 1, 16))) return st;
  // one launch of a no-op kernel of this module loads the module's code object (every phmm kernel);
  // a no-op of its own keeps the profiles' per-kernel statistics free of empty dispatches
  hipLaunchKernelGGL(phmm_warm, dim3(1), dim3(kWave), 0, b->stream, b->d_count);
  GB_HIP(hipGetLastError());
  GB_HIP(hipStreamSynchronize(b->stream));
  // the runtime creates a stream's hardware queue at its first command (~10-15 ms, measured inside
  // bin/phmm's timed region as a chunk upload): give each workspace stream one here
  for (int c = 1; c < kPipeMaxChunks; c++) {
    gb_phmm_batch *w = thread_workspace(t, &st, c);
    if (!w) return st;
    if ((st = batch_reserve(w, 1, 16))) return st;
    GB_HIP(hipMemsetAsync(w->d_count, 0, 8 * sizeof(int), w->stream));
    GB_HIP(hipEventRecord(w->ev[0], w->stream));
  }
  for (int c = 1; c < kPipeMaxChunks; c++) GB_HIP(hipStreamSynchronize(thread_workspace(t, &st, c)->stream));
  // buffers for a job of GB_PHMM_PREALLOC testcases (default 1 M; 0: none) in the pipeline's chunk
  // proportions: allocating them inside the first call cost bin/phmm ~14 ms of its timed region
  // (device ~90 B, pinned ~70 B and host scratch ~70 B per testcase; all grow on demand past it)
  int64_t pre = 1 << 20;
  if (const char *e = getenv("GB_PHMM_PREALLOC")) pre = std::max(0ll, atoll(e));
  if (pre > 0) {
    const int64_t W = (int64_t)kPipeMaxChunks * (kPipeMaxChunks + 1) / 2;
    for (int c = 0; c < kPipeMaxChunks; c++) {
      gb_phmm_batch *w = thread_workspace(t, &st, c);
      const int64_t m = pre * (c + 1) / W + 1;
      const size_t pool = 32 * (size_t)m;
      if ((st = batch_reserve(w, (int)std::min<int64_t>(m, 1 << 30), pool))) return st;
      if ((st = stage_reserve(w, StageLayout((size_t)m, pool).total))) return st;
      host_reserve(w, (size_t)m, pool, 4);
    }
  }
  return GB_OK;
}

// Pipelined one-call path for big calls: the testcases are cut into contiguous chunks of growing size
// (weights 1, 2, .., k), each packed into its own workspace batch (own stream). The first, small
// chunk is packed on the calling thread and launched at once; the others are packed meanwhile on
// worker threads and launched in order as they become ready, so the host's packing hides behind the
// kernels, and chunk c's results (D2H + log10) overlap the kernels of the chunks after it. Chunks are
// independent jobs, so results are those of one job.
int compute_pipelined(DeviceTables *tabs, const gb_testcase *tcs, int n, double *results, float *raw_f,
                      double *raw_d, uint8_t *used_double) {
  const char *e = getenv("GB_PHMM_PIPE");  // probes: the chunk count (1 = one job, no overlap)
  // two chunks from kPipeMin2 testcases (the reference's bigger per-batch calls), up to four
  int k = std::min(kPipeMaxChunks, std::max(2, n / kPipeMinChunk));
  if (e) k = std::max(1, std::min(16, atoi(e)));
  std::vector<gb_phmm_batch *> B(k);
  std::vector<int> lo(k + 1);
  const int64_t W = (int64_t)k * (k + 1) / 2;
  for (int c = 0; c <= k; c++) lo[c] = (int)((int64_t)n * ((int64_t)c * (c + 1) / 2) / W);
  int st = GB_OK;
  for (int c = 0; c < k; c++) {
    B[c] = thread_workspace(tabs, &st, c);
    if (!B[c]) return st;
    B[c]->force_f64 = false;
  }
  HostClock clk;
  // the whole call is validated here, before any chunk is packed or launched: a bad testcase fails the
  // call with its index in the caller's array and nothing on the device
  if ((st = validate_testcases(tcs, n))) return st;
  // host threads: about 12 over the concurrent fills (GB_PHMM_FILL_THREADS: per fill)
  int fill_threads = std::max(1, 12 / k);
  if (const char *f = getenv("GB_PHMM_FILL_THREADS")) fill_threads = std::max(1, atoi(f));
  const int device = tabs->device;
  auto fill = [&, device](int c) -> std::pair<int, std::string> {
    if (hipSetDevice(device) != hipSuccess) return {GB_ERR_HIP, "gb_phmm_compute: hipSetDevice failed"};
    const int s = batch_fill(B[c], tcs + lo[c], lo[c + 1] - lo[c], fill_threads, true);
    return {s, s ? std::string(gb::last_error()) : std::string()};
  };
  // the workers' futures join on destruction, also on an early return
  std::vector<std::future<std::pair<int, std::string>>> ready;
  for (int c = 1; c < k; c++) ready.push_back(std::async(std::launch::async, fill, c));
  auto fetch = [&](int c) {
    const int o = lo[c];
    return gb_phmm_batch_results(B[c], results ? results + o : nullptr, raw_f ? raw_f + o : nullptr,
                                 raw_d ? raw_d + o : nullptr, used_double ? used_double + o : nullptr, nullptr);
  };
  // on an error, the chunks already launched are waited for before the call returns, so no kernel
  // of this call is left in flight (results are undefined on a nonzero status) and the next call
  // refills those workspaces behind nothing
  int launched = 0;
  auto fail = [&](int s) {
    const std::string msg = gb::last_error();
    for (int c = 0; c < launched; c++) (void)hipStreamSynchronize(B[c]->stream);
    for (size_t c = 0; c < ready.size(); c++)
      if (ready[c].valid()) ready[c].wait();
    gb::set_error("%s", msg.c_str());
    return s;
  };
  if ((st = batch_fill(B[0], tcs, lo[1], fill_threads, true))) return fail(st);
  clk.mark("chunk 0 filled");
  if ((st = gb_phmm_batch_run(B[0]))) return fail(st);
  launched = 1;
  // chunk c - 2's results are fetched after chunk c is launched: the host never waits on the chunk
  // the GPU has just started, only on one queued behind it
  int fetched = 0;
  for (int c = 1; c < k; c++) {
    const auto r = ready[c - 1].get();
    if (r.first) {
      gb::set_error("%s", r.second.c_str());
      return fail(r.first);
    }
    clk.mark("chunk ready");
    if ((st = gb_phmm_batch_run(B[c]))) return fail(st);
    launched = c + 1;
    if (c >= 2) {
      if ((st = fetch(fetched++))) return fail(st);
      clk.mark("chunk fetched");
    }
  }
  while (fetched < k)
    if ((st = fetch(fetched++))) return fail(st);
  clk.mark("last chunks fetched");
  return st;
}

}  // namespace

extern "C" {

int gb_phmm_batch_create(const gb_testcase *tcs, int n, gb_phmm_batch **out) {
  GB_ARG(out, "gb_phmm_batch_create: null out");
  GB_ARG(n >= 0 && (n == 0 || tcs), "gb_phmm_batch_create: bad testcase array (n=%d)", n);
  *out = nullptr;
  DeviceTables *tabs = nullptr;
  int st = get_device_tables(&tabs);
  if (st) return st;
  gb_phmm_batch *b = nullptr;
  if ((st = batch_new(tabs, &b))) return st;
  if ((st = batch_fill(b, tcs, n))) {
    gb_phmm_batch_destroy(b);
    return st;
  }
  *out = b;
  return GB_OK;
}

int gb_phmm_batch_run(gb_phmm_batch *b) {
  gb::Range range_("gb.phmm.batch_run");
  GB_ARG(b, "gb_phmm_batch_run: null batch");
  DeviceTables *t = b->tabs;
  GB_HIP(hipSetDevice(t->device));
  const int n = b->n;
  GB_HIP(hipEventRecord(b->ev[0], b->stream));
  GB_HIP(hipMemsetAsync(b->d_count, 0, kCountWords * sizeof(int), b->stream));
  GB_HIP(hipMemsetAsync(b->d_rd, 0, sizeof(double) * std::max(n, 1), b->stream));
  if (n > 0) {
    const size_t rec = (size_t)(b->max_haplen + kBndPad + kRecPad), codes = (size_t)(b->max_haplen + kBndPad + kWave);
    const size_t lds_f = sizeof(Brec<float>) * rec + codes + 16;
    const size_t lds_d = sizeof(Brec<double>) * rec + codes + 16;
    auto f32k = phmm_forward<float, false>;
    auto f64k = phmm_forward<double, true>;
    const int ns = b->nstacks, nl = b->n_long;
    const Stack *d_long = b->d_stacks + ns;
    if (b->f32_exit) f32k = phmm_forward<float, false, false, true>;
    if (!b->force_f64) {
      if (ns > 0 && b->rpl == 2) {
        const size_t lds_f2 = sizeof(Brec<float>) * (size_t)(b->max_haplen + kBndPad2 + kRecPad) +
                              (size_t)(b->max_haplen + kBndPad2 + kCodePad2) + 16;
        auto k2 = b->w2 == 8 ? phmm_forward2<8> : b->w2 == 6 ? phmm_forward2<6> : phmm_forward2<0>;
        hipLaunchKernelGGL(k2, dim3(ns), dim3(kWave), lds_f2, b->stream, b->d_stacks, b->d_stk_tc,
                           b->d_desc, b->d_pool, dev_tab<float>(t->f, t->hf.init_const), b->d_rf);
      } else if (ns > 0) {
        hipLaunchKernelGGL(f32k, dim3(ns), dim3(kWave), lds_f, b->stream, b->d_stacks, ns, b->d_stk_tc, b->d_desc,
                           b->d_pool, dev_tab<float>(t->f, t->hf.init_const), b->d_rf, (const float *)nullptr,
                           b->d_count, 0, (uint8_t *)nullptr, (size_t)0, (const uint32_t *)nullptr);
      }
      if (nl > 0)
        hipLaunchKernelGGL((phmm_forward<float, false, true>), dim3(b->long_grid), dim3(kWave), 0, b->stream, d_long,
                           nl, b->d_stk_tc, b->d_desc, b->d_pool, dev_tab<float>(t->f, t->hf.init_const), b->d_rf,
                           (const float *)nullptr, b->d_count, 0, b->d_scratch, b->scratch_stride,
                           (const uint32_t *)nullptr);
      GB_HIP(hipGetLastError());
    }
    GB_HIP(hipEventRecord(b->ev[1], b->stream));
    // f64 fallback: persistent grid over the stacks, each recomputing its flagged testcases
    if (ns > 0) {
      const int nunits = ns * b->f64_parts;
      const int g64 = std::min(nunits, b->f64_grid);
      if (b->f64_plan) {
        const dim3 pg((unsigned)((nunits + 255) / 256)), pb(256);
        hipLaunchKernelGGL(f64_plan, pg, pb, 0, b->stream, b->d_stacks, nunits, b->f64_parts, b->d_stk_tc, b->d_desc,
                           (const float *)b->d_rf, b->force_f64 ? 1 : 0, b->d_ukey, b->d_count);
        hipLaunchKernelGGL(f64_plan_order, pg, pb, 0, b->stream, nunits, (const uint8_t *)b->d_ukey, b->d_count,
                           b->d_units);
      }
      hipLaunchKernelGGL(f64k, dim3(g64), dim3(kWave), lds_d, b->stream, b->d_stacks, ns, b->d_stk_tc, b->d_desc,
                         b->d_pool, dev_tab<double>(t->d, t->hd.init_const), b->d_rd, (const float *)b->d_rf,
                         b->d_count, (b->force_f64 ? 1 : 0) | (b->f64_parts << 8), (uint8_t *)nullptr, (size_t)0,
                         b->f64_plan ? (const uint32_t *)b->d_units : nullptr);
    }
    if (nl > 0)
      hipLaunchKernelGGL((phmm_forward<double, true, true>), dim3(b->long_grid), dim3(kWave), 0, b->stream, d_long,
                         nl, b->d_stk_tc, b->d_desc, b->d_pool, dev_tab<double>(t->d, t->hd.init_const), b->d_rd,
                         (const float *)b->d_rf, b->d_count, b->force_f64 ? 1 : 0, b->d_scratch, b->scratch_stride,
                         (const uint32_t *)nullptr);
    GB_HIP(hipGetLastError());
    GB_HIP(hipEventRecord(b->ev[2], b->stream));
    hipLaunchKernelGGL(phmm_finalize, dim3((n + 255) / 256), dim3(256), 0, b->stream, b->d_rf,
                       b->d_rd, (const uint8_t *)nullptr, b->d_out, n, t->hf.log10_init,
                       t->hd.log10_init);
    GB_HIP(hipGetLastError());
  } else {
    GB_HIP(hipEventRecord(b->ev[1], b->stream));
    GB_HIP(hipEventRecord(b->ev[2], b->stream));
  }
  GB_HIP(hipEventRecord(b->ev[3], b->stream));
  b->ran = true;
  return GB_OK;
}

int gb_phmm_batch_sync(gb_phmm_batch *b) {
  GB_ARG(b, "gb_phmm_batch_sync: null batch");
  GB_HIP(hipStreamSynchronize(b->stream));
  return GB_OK;
}

int gb_phmm_batch_results(gb_phmm_batch *b, double *results, float *raw_f, double *raw_d,
                          uint8_t *used_double, double *dev_results) {
  GB_ARG(b, "gb_phmm_batch_results: null batch");
  if (!b->ran) {
    gb::set_error("gb_phmm_batch_results: batch has not been run");
    return GB_ERR_STATE;
  }
  GB_HIP(hipSetDevice(b->tabs->device));
  GB_HIP(hipStreamSynchronize(b->stream));
  const int n = b->n;
  if (n == 0) return GB_OK;
  // raw likelihoods back through the pinned staging buffer when it is big enough (a pageable copy is
  // staged by the runtime)
  std::vector<float> rf_v;
  std::vector<double> rd_v;
  const float *rf;
  const double *rd;
  const size_t off_d = (sizeof(float) * (size_t)n + 255) & ~(size_t)255;
  if (b->h_stage && b->cap_stage >= off_d + sizeof(double) * (size_t)n) {
    GB_HIP(hipMemcpyAsync(b->h_stage, b->d_rf, sizeof(float) * n, hipMemcpyDeviceToHost, b->stream));
    GB_HIP(hipMemcpyAsync(b->h_stage + off_d, b->d_rd, sizeof(double) * n, hipMemcpyDeviceToHost, b->stream));
    GB_HIP(hipStreamSynchronize(b->stream));
    rf = (const float *)b->h_stage;
    rd = (const double *)(b->h_stage + off_d);
  } else {
    rf_v.resize(n);
    rd_v.resize(n);
    GB_HIP(hipMemcpy(rf_v.data(), b->d_rf, sizeof(float) * n, hipMemcpyDeviceToHost));
    GB_HIP(hipMemcpy(rd_v.data(), b->d_rd, sizeof(double) * n, hipMemcpyDeviceToHost));
    rf = rf_v.data();
    rd = rd_v.data();
  }
  if (dev_results) GB_HIP(hipMemcpy(dev_results, b->d_out, sizeof(double) * n, hipMemcpyDeviceToHost));
  const float l10f = b->tabs->hf.log10_init;
  const double l10d = b->tabs->hd.log10_init;
  auto part = [&](int lo, int hi) {
    for (int k = lo; k < hi; k++) {
      const bool ud = rf[k] < 1e-28f;
      if (results) results[k] = ud ? (log10(rd[k]) - l10d) : (double)(log10f(rf[k]) - l10f);
      if (raw_f) raw_f[k] = rf[k];
      if (raw_d) raw_d[k] = rd[k];
      if (used_double) used_double[k] = ud ? 1 : 0;
    }
  };
  // the host log10 epilogue (bit-exact, unlike the device one) over a few threads for big jobs
  const int nt = n >= (1 << 16) ? (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency())) : 1;
  if (nt == 1) {
    part(0, n);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++) th.emplace_back(part, (int)((int64_t)n * t / nt), (int)((int64_t)n * (t + 1) / nt));
    for (auto &t : th) t.join();
  }
  return GB_OK;
}

int gb_phmm_batch_timing(gb_phmm_batch *b, float *f32_ms, float *f64_ms, float *total_ms) {
  GB_ARG(b && b->ran, "gb_phmm_batch_timing: batch has not been run");
  GB_HIP(hipEventSynchronize(b->ev[3]));
  float a = 0, c = 0, tot = 0;
  GB_HIP(hipEventElapsedTime(&a, b->ev[0], b->ev[1]));
  GB_HIP(hipEventElapsedTime(&c, b->ev[1], b->ev[2]));
  GB_HIP(hipEventElapsedTime(&tot, b->ev[0], b->ev[3]));
  if (f32_ms) *f32_ms = a;
  if (f64_ms) *f64_ms = c;
  if (total_ms) *total_ms = tot;
  return GB_OK;
}

int gb_phmm_batch_stats(gb_phmm_batch *b, int64_t *testcases, int64_t *cells, int64_t *n_f64) {
  GB_ARG(b, "gb_phmm_batch_stats: null batch");
  if (testcases) *testcases = b->n;
  if (cells) *cells = b->cells;
  if (n_f64) {
    int c = 0;
    if (b->ran) {
      GB_HIP(hipStreamSynchronize(b->stream));
      GB_HIP(hipMemcpy(&c, b->d_count, sizeof(int), hipMemcpyDeviceToHost));
    }
    *n_f64 = c;
  }
  return GB_OK;
}

int gb_phmm_batch_exit_stats(gb_phmm_batch *b, int64_t *dropped, int64_t *cells_skipped) {
  GB_ARG(b, "gb_phmm_batch_exit_stats: null batch");
  unsigned long long c[2] = {0, 0};
  if (b->ran) {
    GB_HIP(hipStreamSynchronize(b->stream));
    GB_HIP(hipMemcpy(c, b->d_count + 4, sizeof(c), hipMemcpyDeviceToHost));
  }
  if (dropped) *dropped = (int64_t)c[0];
  if (cells_skipped) *cells_skipped = (int64_t)c[1];
  return GB_OK;
}

int gb_phmm_batch_destroy(gb_phmm_batch *b) {
  if (!b) return GB_OK;
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  (void)hipFree(b->d_arena);
  (void)hipFree(b->d_pool);
  if (b->h_stage) (void)hipHostFree(b->h_stage);
  (void)hipFree(b->d_count);
  (void)hipFree(b->d_scratch);
  for (auto e : b->ev)
    if (e) (void)hipEventDestroy(e);
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
  return GB_OK;
}

int gb_phmm_compute(const gb_testcase *tcs, int n, double *results, float *raw_f, double *raw_d,
                    uint8_t *used_double) {
  gb::Range range_("gb.phmm.compute");
  GB_ARG(n >= 0 && (n == 0 || tcs), "gb_phmm_compute: bad testcase array (n=%d)", n);
  if (n == 0) return GB_OK;
  DeviceTables *tabs = nullptr;
  int st = get_device_tables(&tabs);
  if (st) return st;
  if (n >= kPipeMin2 || getenv("GB_PHMM_PIPE"))
    return compute_pipelined(tabs, tcs, n, results, raw_f, raw_d, used_double);
  gb_phmm_batch *b = thread_workspace(tabs, &st);
  if (!b) return st;
  b->force_f64 = false;
  if ((st = batch_fill(b, tcs, n))) return st;
  HostClock clk;
  st = gb_phmm_batch_run(b);
  if (!st) st = gb_phmm_batch_sync(b);
  clk.mark("kernels");
  if (!st) st = gb_phmm_batch_results(b, results, raw_f, raw_d, used_double, nullptr);
  clk.mark("results");
  return st;
}

int gb_phmm_compute_f64(const gb_testcase *tcs, int n, double *raw_d) {
  GB_ARG(n >= 0 && raw_d && (n == 0 || tcs), "gb_phmm_compute_f64: bad arguments");
  if (n == 0) return GB_OK;
  DeviceTables *tabs = nullptr;
  int st = get_device_tables(&tabs);
  if (st) return st;
  gb_phmm_batch *b = thread_workspace(tabs, &st);
  if (!b) return st;
  if ((st = batch_fill(b, tcs, n))) return st;
  b->force_f64 = true;
  st = gb_phmm_batch_run(b);
  b->force_f64 = false;
  if (!st) st = gb_phmm_batch_results(b, nullptr, nullptr, raw_d, nullptr, nullptr);
  return st;
}

int gb_phmm_compute_f32(const gb_testcase *tcs, int n, float *raw_f) {
  gb::Range range_("gb.phmm.compute_f32");
  GB_ARG(n >= 0 && raw_f && (n == 0 || tcs), "gb_phmm_compute_f32: bad arguments");
  if (n == 0) return GB_OK;
  DeviceTables *tabs = nullptr;
  int st = get_device_tables(&tabs);
  if (st) return st;
  gb_phmm_batch *b = thread_workspace(tabs, &st);
  if (!b) return st;
  b->force_f64 = false;
  if ((st = batch_fill(b, tcs, n))) return st;
  b->f32_exit = false;  // every testcase's f32 probability in full, also those that fall back
  st = gb_phmm_batch_run(b);
  if (!st) st = gb_phmm_batch_sync(b);
  if (!st) st = gb_phmm_batch_results(b, nullptr, raw_f, nullptr, nullptr, nullptr);
  return st;
}

}  // extern "C"
