// bsw.hip -- MI355X (gfx950) banded Smith-Waterman extension (GenomicsBench bsw): kernel and C ABI.
//
// Semantics: benchmarks/bsw/bandedSWA.cpp:130-251 (scalarBandedSWA == bwa ksw_extend2), which the
// benchmark's 16-bit SIMD getScores16 reproduces. Integer arithmetic
// throughout, so results are bit-exact by construction.
//
// MI355X design: one pair per wave64, lanes across the query, lane l owning the K = ceil((qlen+1)/64)
// consecutive DP columns j = l*K .. l*K+K-1 (the eh[] entries 0..qlen of the reference live in
// registers for the whole pair, so stale entries outside the band persist exactly as in the
// reference's array). Rows (target bases) are processed in order; within a row the only sequential
// dependency is F, and F(i, j) = max(0, max_{beg<=k<j} (max(M_k - oe_ins, 0) - e_ins (j-1-k)))
// depends on the previous row only (M_k = H(i-1,k-1) + S), so a row is one max-plus prefix scan:
// in-lane over the K columns, then across lanes with DPP (row_shr 1/2/4/8, row_bcast 15/31).
// Row control (band, row max / last argmax, gscore, zdrop, band narrowing) is wave-uniform scalar
// code fed by one DPP max-reduction and three ballots per row. Waves pull pairs from an atomic
// counter (persistent grid), so ragged pairs balance across the 256 CUs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <condition_variable>
#include <mutex>
#include <string>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/gb_bsw.h"
#include "gb_common.h"

static_assert(sizeof(gb_seqpair) == 72, "gb_seqpair must match SeqPair (bandedSWA.h:92-101)");

namespace gbbsw {

constexpr int kNeg = -(1 << 28);
constexpr int kWavesPerBlock = 4;
constexpr int kBlocksPerCU = 8;

struct Pair {  // device descriptor, 32 B
  int64_t t_off, q_off;
  int32_t tlen, qlen, h0, w;  // w: band after the max_ins / max_del adjustment (bandedSWA.cpp:161-170)
};

struct Args {
  const Pair *pairs;
  const uint32_t *list;  // pair indices this launch processes
  int64_t n;             // entries in list
  const uint8_t *tgt, *qry;
  int32_t *out6, *cells;
  unsigned long long *total_cells;
  unsigned int *next;
  int o_del, e_del, o_ins, e_ins, zdrop;
  int8_t mat[28];
};

// wave-wide inclusive max scan (Hillis-Steele in 16-lane rows, then row broadcasts)
__device__ __forceinline__ int scan_max(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x111, 0xF, 0xF, false));  // row_shr:1
  v = max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x112, 0xF, 0xF, false));  // row_shr:2
  v = max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x114, 0xF, 0xF, false));  // row_shr:4
  v = max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x118, 0xF, 0xF, false));  // row_shr:8
  v = max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}
__device__ __forceinline__ int shr1(int v, int lane0) {
  return __builtin_amdgcn_update_dpp(lane0, v, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ __forceinline__ uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }

template <int K>
__device__ __forceinline__ void extend(const Args &A, const Pair &P, const int8_t *smat, int lane,
                                       int32_t *o6, int &ncells) {
  const int qlen = P.qlen, tlen = P.tlen, h0 = P.h0, w = P.w;
  const int o_del = A.o_del, e_del = A.e_del, o_ins = A.o_ins, e_ins = A.e_ins;
  const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
  const uint8_t *qry = A.qry + P.q_off;
  const uint8_t *tgt = A.tgt + P.t_off;

  int H[K], E[K], plo[K], phi[K], ej[K];
  const int v1 = max(h0 - oe_ins, 0);
#pragma unroll
  for (int c = 0; c < K; ++c) {
    const int j = lane * K + c;
    int qb = 4;
    if (j < qlen) qb = min((int)qry[j], 4);
    plo[c] = (smat[qb] & 0xFF) | (smat[5 + qb] & 0xFF) << 8 | (smat[10 + qb] & 0xFF) << 16 |
             (smat[15 + qb] & 0xFF) << 24;
    phi[c] = smat[20 + qb];
    // first row (bandedSWA.cpp:157-159): h0, then h0 - oe_ins decreasing by e_ins down to 0
    H[c] = j == 0 ? h0 : (j <= qlen ? max(v1 - (j - 1) * e_ins, 0) : 0);
    E[c] = 0;
    ej[c] = e_ins * j;
  }

  int beg = 0, end = qlen, mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
  int tword = 0;
  int i;
  for (i = 0; i < tlen; ++i) {
    const int ir = i & 255;
    if (ir == 0) {  // 256 target bases per VGPR: lane l holds bases i+4l .. i+4l+3
      tword = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int t = i + 4 * lane + b;
        if (t < tlen) tword |= (int)tgt[t] << (8 * b);
      }
    }
    const int tb = min((__builtin_amdgcn_readlane(tword, ir >> 2) >> (8 * (ir & 3))) & 0xFF, 4);
    const int sh = 8 * (tb & 3);
    const bool hi = tb >= 4;
    // band (bandedSWA.cpp:180-182)
    if (beg < i - w) beg = i - w;
    if (end > i + w + 1) end = i + w + 1;
    if (end > qlen) end = qlen;
    const int h1init = beg == 0 ? max(h0 - (o_del + e_del * (i + 1)), 0) : 0;
    ncells += max(end - beg, 0);

    int M[K], g[K], lpx[K], h[K], En[K];
    bool inb[K];
    int lp = kNeg;
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const int j = lane * K + c;
      inb[c] = j >= beg && j < end;
      const int s = __builtin_amdgcn_sbfe(hi ? phi[c] : plo[c], sh, 8);
      const int Mv = H[c] ? H[c] + s : 0;  // M = H(i-1,j-1) ? H(i-1,j-1) + S : 0
      M[c] = Mv;
      g[c] = inb[c] ? max(Mv - oe_ins, 0) + ej[c] : kNeg;
      lpx[c] = lp;
      lp = max(lp, g[c]);
    }
    const int lex = shr1(scan_max(lp), kNeg);
    int hm = -1;
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const int f = max(max(lex, lpx[c]) - ej[c] + e_ins, 0);  // F(i,j)
      h[c] = max(max(M[c], E[c]), f);
      En[c] = max(max(E[c] - e_del, M[c] - oe_del), 0);  // E(i+1,j)
      if (inb[c]) hm = max(hm, h[c]);
    }
    const int m = max(__builtin_amdgcn_readlane(scan_max(hm), 63), 0);
    int mj = -1;
    if (m > 0) {  // last column reaching the row maximum (bandedSWA.cpp:203-204)
      int jl = -1;
#pragma unroll
      for (int c = 0; c < K; ++c)
        if (inb[c] && h[c] == m) jl = lane * K + c;
      const uint64_t bal = ballot(jl >= 0);
      mj = __builtin_amdgcn_readlane(jl, 63 - __builtin_clzll(bal));
    }
    // eh[j].h <- H(i,j-1) for j in (beg, end], eh[beg].h <- first column, eh[j].e <- E(i+1,j),
    // eh[end].e <- 0 (bandedSWA.cpp:195-197,217)
    const int wlo = min(beg, end);
    const int hprev = shr1(h[K - 1], 0);
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const int j = lane * K + c;
      const int hs = c ? h[c - 1] : hprev;
      if (j >= wlo && j <= end) {
        H[c] = j == wlo ? h1init : hs;
        E[c] = j == end ? 0 : En[c];
      }
    }
    const int ce = end % K;
    int hsel = H[0];
#pragma unroll
    for (int c = 1; c < K; ++c)
      if (ce == c) hsel = H[c];
    const int h1 = __builtin_amdgcn_readlane(hsel, end / K);
    if ((beg < end ? end : beg) == qlen) {  // bandedSWA.cpp:218-221
      max_ie = gscore > h1 ? max_ie : i;
      gscore = gscore > h1 ? gscore : h1;
    }
    if (m == 0) break;
    if (m > mx) {
      mx = m, max_i = i, max_j = mj;
      max_off = max(max_off, abs(mj - i));
    } else if (A.zdrop > 0) {
      if (i - max_i > mj - max_j) {
        if (mx - m - ((i - max_i) - (mj - max_j)) * e_del > A.zdrop) break;
      } else {
        if (mx - m - ((mj - max_j) - (i - max_i)) * e_ins > A.zdrop) break;
      }
    }
    // band narrowing (bandedSWA.cpp:235-239)
    int jf = INT_MAX;
#pragma unroll
    for (int c = K - 1; c >= 0; --c) {
      const int j = lane * K + c;
      if ((H[c] | E[c]) != 0 && j >= beg && j < end) jf = j;
    }
    const uint64_t bf = ballot(jf != INT_MAX);
    const int nb = bf ? __builtin_amdgcn_readlane(jf, __builtin_ctzll(bf)) : end;
    int jl = -1;
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const int j = lane * K + c;
      if ((H[c] | E[c]) != 0 && j >= nb && j <= end) jl = j;
    }
    const uint64_t bl = ballot(jl >= 0);
    const int je = bl ? __builtin_amdgcn_readlane(jl, 63 - __builtin_clzll(bl)) : nb - 1;
    beg = nb;
    end = je + 2 < qlen ? je + 2 : qlen;
  }
  if (lane == 0) {
    o6[0] = mx;
    o6[1] = max_j + 1;
    o6[2] = max_i + 1;
    o6[3] = max_ie + 1;
    o6[4] = gscore;
    o6[5] = max_off;
  }
}

__global__ __launch_bounds__(64 * kWavesPerBlock) void bsw_extend_kernel(Args A) {
  __shared__ int8_t smat[32];
  if (threadIdx.x < 25) smat[threadIdx.x] = A.mat[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  unsigned long long wave_cells = 0;
  for (;;) {
    unsigned int p = 0;
    if (lane == 0) p = atomicAdd(A.next, 1u);
    p = __builtin_amdgcn_readfirstlane(p);
    if ((int64_t)p >= A.n) break;
    p = A.list[p];
    const Pair P = A.pairs[p];
    int nc = 0;
    int32_t *o6 = A.out6 + 6 * (int64_t)p;
    const int K = (P.qlen + 64) >> 6;  // columns 0..qlen
    if (K <= 1)
      extend<1>(A, P, smat, lane, o6, nc);
    else if (K == 2)
      extend<2>(A, P, smat, lane, o6, nc);
    else if (K == 3)
      extend<3>(A, P, smat, lane, o6, nc);
    else
      extend<4>(A, P, smat, lane, o6, nc);
    if (lane == 0) A.cells[p] = nc;
    wave_cells += (unsigned)nc;
  }
  if (lane == 0 && wave_cells) atomicAdd(A.total_cells, wave_cells);
}


// ------------------------------------------------------------------------------------------------
// Pair-per-lane kernel (the reference's own inter-pair SIMD shape, getScores16): 64 pairs per wave,
// each lane runs scalarBandedSWA for its pair. The lane's eh[0..qlen] lives in VGPRs, one register
// per column packing e (bits 0-15) and h (bits 16-31: H + S is one SDWA add of the high word and
// the sign-extended score byte, H << 16 one AND), so every column index is a compile-time
// constant: columns are swept in lockstep over the union of the lanes' bands, each lane's own band
// [beg, end) selected by a bit-select mask, 8-column chunks outside every band skipped by a uniform
// branch. Pairs are grouped by query length (NCH chunks of 8 columns hold eh[0..8*NCH-1]) and
// sorted by target length so the 64 lanes of a wave run rows in near lockstep.
// Exactness notes: M = H ? H + S : 0 only matters through max(M, 0) (h = max(M, e, f) with
// e, f >= 0, and both gap openings clamp at 0), so M is formed as med3(H << 16, H + S, 0); all
// scores stay below 2^15 (checked on the host), so the 16-bit packing is lossless.

// v_med3_i32(a, b, 0) = max(min(a, b), 0) whenever a >= 0 (LLVM only forms med3 from constant
// clamps, so it is spelled out)
__device__ __forceinline__ int med3_0(int a, int b) {
  int r;
  asm("v_med3_i32 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// wave-wide OR, result uniform (DPP row shifts and row broadcasts leave it in lane 63)
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

struct LaneArgs {
  const Pair *pairs;
  const uint32_t *order;
  int64_t first, count;  // order[first .. first+count)
  const uint8_t *tgt, *qry;
  int32_t *out6, *cells;
  unsigned long long *total_cells;
  int o_del, e_del, o_ins, e_ins, zdrop;
  unsigned long long *prof;  // GB_BSW_PROF=1: {wave rows, chunk-columns swept, lane-rows active, cells,
                             //  chunk-columns inside every active lane's band}
  uint32_t tab[10];  // per target code t: score bytes (int8) of query codes 0..3 (tab[2t]) and 4 (tab[2t+1])
};

// SYM: insertions and deletions cost the same (the benchmark's 6/1, 6/1), so M - oe_del and
// M - oe_ins are one value and the compiler shares it (one op per column)
template <int NCH, bool SYM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NCH >= 16 ? 2 : 1))) void bsw_lane_kernel(LaneArgs A) {
  constexpr int NCOL = 8 * NCH;
  constexpr int NW = (NCOL + 31) / 32;
  const int lane = threadIdx.x;
  const int64_t k = A.first + (int64_t)blockIdx.x * 64 + lane;
  const bool valid = k < A.first + A.count;
  const uint32_t p = valid ? A.order[k] : 0u;
  Pair P;
  if (valid) {
    P = A.pairs[p];
  } else {
    P.t_off = P.q_off = 0;
    P.tlen = 0;
    P.qlen = 1;
    P.h0 = 0;
    P.w = 0;
  }
  const int qlen = P.qlen, tlen = P.tlen, h0 = P.h0, w = P.w;
  const int o_del = A.o_del, e_del = A.e_del;
  const int o_ins = SYM ? o_del : A.o_ins, e_ins = SYM ? e_del : A.e_ins;
  const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
  const uint8_t *qry = A.qry + P.q_off;
  const uint8_t *tgt = A.tgt + P.t_off;

  // query codes, 4 bits per column, 8 columns per word, staged in LDS (Qs[c][lane]) so they cost
  // no VGPRs; eh row 0 (bandedSWA.cpp:157-159) computed in registers
  __shared__ uint32_t Qs[NCH][64];
  uint32_t X[NCOL];
  const int v1 = max(h0 - oe_ins, 0);
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    uint32_t q = 0;
    const int j0 = 8 * c;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint32_t code = j0 + b < qlen ? min((uint32_t)qry[j0 + b], 4u) : 4u;
      q |= code << (4 * b);
    }
    Qs[c][lane] = q;
  }
#pragma unroll
  for (int j = 0; j < NCOL; ++j)
    X[j] = (j == 0 ? (uint32_t)h0 : (j <= qlen ? (uint32_t)max(v1 - (j - 1) * e_ins, 0) : 0u)) << 16;

  int beg = 0, end = qlen, mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
  int ncells = 0;
  bool active = valid && tlen > 0;
  unsigned long long pr_rows = 0, pr_cols = 0, pr_lrows = 0, pr_full = 0;
  // target bases: the next row's byte is loaded one row ahead (clamped in-bounds) into one register;
  // a row of sweeping hides its latency, and the 256-VGPR variants keep it out of scratch (a
  // four-row prefetch group spilled there and waited on each load)
  const int tmax = max(tlen - 1, 0);
  uint32_t tnext = tgt[0];
  // per-lane constants used once per row (target pointer, last row, band width) live in LDS and are
  // re-read each row: in the 256-VGPR variants they were spilled to scratch instead, and a scratch
  // reload's vmcnt wait also waited for the row-ahead target load
  __shared__ uint32_t Pc[4][64];
  Pc[0][lane] = (uint32_t)(uintptr_t)tgt;
  Pc[1][lane] = (uint32_t)((uint64_t)(uintptr_t)tgt >> 32);
  Pc[2][lane] = (uint32_t)tmax;
  Pc[3][lane] = (uint32_t)w;
  typedef volatile __attribute__((address_space(3))) uint32_t lds_u32;  // ds_read, never flat

#pragma unroll 1
  for (int i = 0;; ++i) {
    if (i >= tlen) active = false;
    if (__builtin_amdgcn_ballot_w64(active) == 0) break;
    const uint32_t tb = min(tnext, 4u);
    const int wr = (int)*(lds_u32 *)&Pc[3][lane];
    {
      // a global (not flat) pointer: a flat load would also count on lgkmcnt and the chunk loop's LDS
      // waits would wait for it
      typedef const __attribute__((address_space(1))) uint8_t glb_u8;
      glb_u8 *tg = (glb_u8 *)(uintptr_t)((uint64_t) * (lds_u32 *)&Pc[1][lane] << 32 | *(lds_u32 *)&Pc[0][lane]);
      tnext = tg[min(i + 1, (int)*(lds_u32 *)&Pc[2][lane])];
    }
    uint32_t tlo = A.tab[8], thi = A.tab[9];  // per-lane row of the score table (select chain, no scratch)
#pragma unroll
    for (int t = 3; t >= 0; --t)
      if (tb == (uint32_t)t) {
        tlo = A.tab[2 * t];
        thi = A.tab[2 * t + 1];
      }
    // band (bandedSWA.cpp:180-182)
    if (beg < i - wr) beg = i - wr;
    if (end > i + wr + 1) end = i + wr + 1;
    if (end > qlen) end = qlen;
    const int width = active ? max(end - beg, 0) : 0;
    ncells += width;
    if (A.prof) {
      ++pr_rows;
      pr_lrows += active ? 1 : 0;
    }
    int h1 = beg == 0 ? max(h0 - (o_del + e_del * (i + 1)), 0) : 0;
    int f = 0, mkey = -1;
    uint32_t nz[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) nz[q] = 0;
    // the lane's band [beg, beg + width) as a bitmap, one word per 32 columns: a column's select mask
    // is then one sign-extending bit extract (the compare of j - beg against width was two ops)
    uint32_t bw[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int lo = min(max(beg - 32 * q, 0), 32), hi = min(max(beg + width - 32 * q, 0), 32);
      const int nb = hi - lo;
      bw[q] = nb > 0 ? (0xFFFFFFFFu >> (32 - nb)) << lo : 0u;
    }
    uint32_t qn = Qs[0][lane];
    // chunks meeting some lane's band: the OR of every lane's chunk range [beg >> 3, (end - 1) >> 3]
    const uint32_t swm = wave_or(width > 0 ? (2u << ((end - 1) >> 3)) - (1u << (beg >> 3)) : 0u);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const uint32_t qc = qn;
      if (c + 1 < NCH) qn = Qs[c + 1][lane];  // prefetch the next chunk's codes
      // skip the chunk when it meets no lane's band
      if (((swm >> c) & 1u) == 0) continue;
      if (A.prof) {
        pr_cols += 8;
        if (__builtin_amdgcn_ballot_w64(active && (beg > 8 * c || end < 8 * c + 8)) == 0) pr_full += 8;
      }
      const uint32_t qe = qc & 0x0F0F0F0Fu, qo = (qc >> 4) & 0x0F0F0F0Fu;
      const uint32_t se = __builtin_amdgcn_perm(thi, tlo, qe);  // score bytes, columns 0,2,4,6
      const uint32_t so = __builtin_amdgcn_perm(thi, tlo, qo);  // columns 1,3,5,7
      // branch-free: every lane evaluates all 8 columns (one basic block, so the scheduler can overlap
      // column j+1's independent work with column j's f/h1 chain); out-of-band lanes keep their state
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int j = 8 * c + b;
        // lane mask of the band, used as a bit-select (kept arithmetic so no branches come back)
        uint32_t msk;  // bit j of the band bitmap, sign-extended (asm: the compiler turns the shift form
                       // back into an AND and a compare)
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(msk) : "v"(bw[j >> 5]), "i"(j & 31));
        const uint32_t x = X[j];
        const int sb = (int)(int8_t)(((b & 1) ? so : se) >> (8 * (b >> 1)));  // score, sign-extended
        const int y = (int)(x >> 16) + sb;                                    // H + S
        const int M = med3_0((int)(x & 0xFFFF0000u), y);  // H ? H + S : 0 (clamped); H << 16 >= 0 (H < 2^15)
        const int e = (int)(x & 0xFFFFu);
        // one max3 (asm: the compiler folds the mask into an SDWA max and then needs a second max,
        // two 4.2-cycle ops where the AND is a 2.5-cycle one)
        int h;
        asm("v_max3_i32 %0, %1, %2, %3" : "=v"(h) : "v"(M), "v"(e), "v"(f));
        const int en = max(max(e - e_del, M - oe_del), 0);                    // E(i+1,j)
        const int fn = max(max(f - e_ins, M - oe_ins), 0);                    // F(i,j+1)
        // eh[j] = {H(i,j-1), E}: h1 written into the high word of en's register (an SDWA move issues at
        // the full rate, a v_lshl_or at 4.27 cycles); en, h1 < 2^16
        uint32_t xn = (uint32_t)en;
        asm("v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0" : "+v"(xn) : "v"(h1));
        uint32_t nzb;  // xn != 0 as 0 / 1 (asm: kept out of the compiler's compare-and-select form)
        asm("v_min_u32 %0, %1, 1" : "=v"(nzb) : "v"(xn));
        nz[j >> 5] |= nzb << (j & 31);  // out-of-band bits are cleared after the sweep
        X[j] = (xn & msk) | (x & ~msk);
        f = (int)(((uint32_t)fn & msk) | ((uint32_t)f & ~msk));
        h1 = (int)(((uint32_t)h & msk) | ((uint32_t)h1 & ~msk));
        // last argmax over keys (H << 8 | j) built from h1 unmasked: outside the band h1 holds the
        // last in-band H (or 0 / the row-0 value before it), fixed up once per row below
        mkey = max(mkey, (int)((uint32_t)h1 << 8 | (uint32_t)j));
      }
    }
#pragma unroll
    for (int q = 0; q < NW; ++q) nz[q] &= bw[q];
    // eh[end] = {h1, 0} (bandedSWA.cpp:217), chunks holding no lane's end skipped
    const bool wend = active && end < NCOL;
    // chunks holding some lane's end: one wave OR of one-hot chunk bits (DPP row shifts + row
    // broadcasts, lane 63 holds the result), then scalar bit tests instead of a ballot per chunk
    const uint32_t endm = wave_or(wend ? 1u << (end >> 3) : 0u);
    // the lane's end column as a one-bit map per 32-column word: in a chunk holding some lane's end
    // a column costs a bit extract and a bit-select (a compare, a mask AND and two selects before,
    // and the compiler hoisted every column's nonzero bit out of the chunk test), and the nonzero
    // bitmap takes h1's bit at the end column once per word
    uint32_t ew[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) ew[q] = (wend && (end >> 5) == q) ? 1u << (end & 31) : 0u;
    const uint32_t h1s = (uint32_t)h1 << 16;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (((endm >> c) & 1u) == 0) continue;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int j = 8 * c + b;
        uint32_t m;
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(ew[j >> 5]), "i"(j & 31));
        X[j] = (h1s & m) | (X[j] & ~m);
      }
    }
#pragma unroll
    for (int q = 0; q < NW; ++q) nz[q] = (nz[q] & ~ew[q]) | (h1 ? ew[q] : 0u);
    if (!active) continue;
    // keys past the band end repeat H(end-1) at larger j, so a winner there is column end-1; an
    // empty band computed nothing (row max 0, bandedSWA.cpp:222)
    const int m = (mkey < 0 || width == 0) ? 0 : (mkey >> 8);
    const int mj = mkey < 0 ? -1 : min(mkey & 0xFF, end - 1);
    if ((beg < end ? end : beg) == qlen) {  // bandedSWA.cpp:218-221
      max_ie = gscore > h1 ? max_ie : i;
      gscore = gscore > h1 ? gscore : h1;
    }
    if (m == 0) {
      active = false;
      continue;
    }
    if (m > mx) {
      mx = m, max_i = i, max_j = mj;
      max_off = max(max_off, abs(mj - i));
    } else if (A.zdrop > 0) {
      const bool brk = (i - max_i > mj - max_j) ? (mx - m - ((i - max_i) - (mj - max_j)) * e_del > A.zdrop)
                                                : (mx - m - ((mj - max_j) - (i - max_i)) * e_ins > A.zdrop);
      if (brk) {
        active = false;
        continue;
      }
    }
    // band narrowing (bandedSWA.cpp:235-239): first nonzero eh in [beg, end), last in [beg', end]
    int first = INT_MAX, last = -1;
#pragma unroll
    for (int q = NW - 1; q >= 0; --q)
      if (nz[q]) first = 32 * q + __builtin_ctz(nz[q]);
#pragma unroll
    for (int q = 0; q < NW; ++q)
      if (nz[q]) last = 32 * q + 31 - __builtin_clz(nz[q]);
    const int nb = min(first, end);
    const int je = last >= nb ? last : nb - 1;
    beg = nb;
    end = je + 2 < qlen ? je + 2 : qlen;
  }
  if (valid) {
    int32_t *o6 = A.out6 + 6 * (int64_t)p;
    o6[0] = mx;
    o6[1] = max_j + 1;
    o6[2] = max_i + 1;
    o6[3] = max_ie + 1;
    o6[4] = gscore;
    o6[5] = max_off;
    A.cells[p] = ncells;
  }
  unsigned long long wc = (unsigned long long)ncells;
  for (int d = 32; d >= 1; d >>= 1) wc += __shfl_xor(wc, d);
  if (lane == 0 && wc) atomicAdd(A.total_cells, wc);
  if (A.prof) {
    for (int d = 32; d >= 1; d >>= 1) pr_lrows += __shfl_xor(pr_lrows, d);
    if (lane == 0) {
      atomicAdd(A.prof + 0, pr_rows);
      atomicAdd(A.prof + 1, pr_cols);
      atomicAdd(A.prof + 2, pr_lrows);
      atomicAdd(A.prof + 3, wc);
      atomicAdd(A.prof + 4, pr_full);
    }
  }
}

// band adjustment of bandedSWA.cpp:161-170, in the reference's double arithmetic
static int adjust_w(int w, int qlen, int mx, const gb_bsw_params &p) {
  int max_ins = (int)((double)(qlen * mx + p.end_bonus - p.o_ins) / p.e_ins + 1.);
  max_ins = max_ins > 1 ? max_ins : 1;
  w = w < max_ins ? w : max_ins;
  int max_del = (int)((double)(qlen * mx + p.end_bonus - p.o_del) / p.e_del + 1.);
  max_del = max_del > 1 ? max_del : 1;
  return w < max_del ? w : max_del;
}

}  // namespace gbbsw

struct gb_bsw_batch {
  int device = -1, num_cus = 0;
  // launch plan: order[seg[v] .. seg[v+1]) are the pairs of variant v (lane kernels NCH = 4, 8, 12,
  // 16, 20; v = 5: wave-per-pair kernel), each segment sorted by decreasing target length
  static constexpr int kVariants = 6;
  int64_t seg[kVariants + 1] = {0};
  uint32_t *d_order = nullptr;
  unsigned long long *d_prof = nullptr;  // GB_BSW_PROF=1 per-variant sweep counters (development aid)
  hipStream_t stream = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  // the variants' launches run side by side: each on its own stream, forked from and joined back
  // into `stream` (a small batch fills the chip only when its short launches overlap)
  hipStream_t side[kVariants] = {};
  hipEvent_t fork = nullptr, join[kVariants] = {};
  gb_bsw_params params{};
  int64_t n = 0;
  gbbsw::Pair *d_pairs = nullptr;
  uint8_t *d_tgt = nullptr, *d_qry = nullptr;
  int32_t *d_out6 = nullptr, *d_cells = nullptr;
  unsigned long long *d_total = nullptr;  // [0] total cells, [1] work counter
  static constexpr int kTotals = 2;
  size_t cap_n = 0, cap_tgt = 0, cap_qry = 0;  // allocated capacities (cached workspaces are refilled)
  bool ran = false;
};

extern "C" {

void gb_bsw_fill_scmat(int a, int b, int ambig, int8_t mat[25]) {
  int k = 0;
  for (int i = 0; i < 4; ++i) {
    for (int j = 0; j < 4; ++j) mat[k++] = (int8_t)(i == j ? a : -b);
    mat[k++] = (int8_t)ambig;
  }
  for (int j = 0; j < 5; ++j) mat[k++] = (int8_t)ambig;
}

void gb_bsw_default_params(gb_bsw_params *p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->o_del = p->o_ins = 6;
  p->e_del = p->e_ins = 1;
  p->zdrop = 100;
  p->end_bonus = 5;
  p->w = 100;
  gb_bsw_fill_scmat(1, 4, -1, p->mat);
}

int gb_bsw_batch_destroy(gb_bsw_batch *B) {
  if (!B) return GB_OK;
  if (B->device >= 0) (void)hipSetDevice(B->device);
  if (B->stream) (void)hipStreamSynchronize(B->stream);
  for (void *p : {(void *)B->d_prof, (void *)B->d_order, (void *)B->d_pairs, (void *)B->d_tgt, (void *)B->d_qry, (void *)B->d_out6, (void *)B->d_cells,
                  (void *)B->d_total})
    (void)hipFree(p);
  for (auto &e : B->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto &e : B->join)
    if (e) (void)hipEventDestroy(e);
  if (B->fork) (void)hipEventDestroy(B->fork);
  for (auto &s : B->side)
    if (s) (void)hipStreamDestroy(s);
  if (B->stream) (void)hipStreamDestroy(B->stream);
  delete B;
  return GB_OK;
}

}  // extern "C"

namespace {

int bsw_batch_new(gb_bsw_batch **out) {
  auto *B = new gb_bsw_batch();
  hipError_t e = hipGetDevice(&B->device);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&B->num_cus, hipDeviceAttributeMultiprocessorCount, B->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&B->stream, hipStreamNonBlocking);
  for (auto &ev : B->ev)
    if (e == hipSuccess) e = hipEventCreate(&ev);
  for (auto &s : B->side)
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (auto &ev : B->join)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&B->fork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc(&B->d_total, gb_bsw_batch::kTotals * sizeof(unsigned long long));
  if (e != hipSuccess) {
    gb::set_error("gb_bsw_batch_create: %s", hipGetErrorString(e));
    gb_bsw_batch_destroy(B);
    return GB_ERR_HIP;
  }
  *out = B;
  return GB_OK;
}

// grow-only device buffer
template <typename T>
int bsw_reserve(T **p, size_t &cap, size_t want) {
  if (want <= cap) return GB_OK;
  (void)hipFree(*p);
  *p = nullptr;
  cap = 0;
  GB_HIP(hipMalloc(p, want * sizeof(T)));
  cap = want;
  return GB_OK;
}

// Validate, classify and order the pairs (launch plan), then upload them and the sequence buffers
// into B (buffers grow when too small).
int bsw_batch_fill(gb_bsw_batch *B, const gb_bsw_params *params, const gb_seqpair *pairs, int64_t n,
                   const uint8_t *ref, int64_t ref_bytes, const uint8_t *qer, int64_t qer_bytes) {
  GB_ARG(params && n >= 0 && (n == 0 || pairs), "gb_bsw_batch_create: bad arguments");
  GB_ARG(n < (1ll << 32) - 1, "gb_bsw_batch_create: too many pairs");
  GB_ARG(params->e_del > 0 && params->e_ins > 0, "gb_bsw_batch_create: gap extension must be > 0");
  GB_ARG(ref_bytes >= 0 && qer_bytes >= 0 && (ref_bytes == 0 || ref) && (qer_bytes == 0 || qer),
         "gb_bsw_batch_create: bad sequence buffers");
  int st0 = GB_OK;
  int mx = 0, mn = 0;
  for (int k = 0; k < 25; ++k) {
    mx = std::max(mx, (int)params->mat[k]);
    mn = std::min(mn, (int)params->mat[k]);
  }
  // The sequence buffers (the bulk of the bytes) go up on a helper thread while this one builds
  // the launch plan; the helper is joined on every return path.
  if ((st0 = bsw_reserve(&B->d_tgt, B->cap_tgt, (size_t)std::max<int64_t>(ref_bytes, 1)))) return st0;
  if ((st0 = bsw_reserve(&B->d_qry, B->cap_qry, (size_t)std::max<int64_t>(qer_bytes, 1)))) return st0;
  hipError_t up_err = hipSuccess;
  struct Joiner {
    std::thread t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } up;
  auto upload = [&, dev = B->device, dt = B->d_tgt, dq = B->d_qry] {
    up_err = hipSetDevice(dev);
    if (up_err == hipSuccess && ref_bytes) up_err = hipMemcpy(dt, ref, (size_t)ref_bytes, hipMemcpyHostToDevice);
    if (up_err == hipSuccess && qer_bytes) up_err = hipMemcpy(dq, qer, (size_t)qer_bytes, hipMemcpyHostToDevice);
  };
  if (ref_bytes + qer_bytes >= (16ll << 20))
    up.t = std::thread(upload);
  else
    upload();  // small calls (the reference's 512-pair batches): no thread start-up
  // per pair: descriptor, kernel variant and sort key -- in parallel chunks for big batches; a bad
  // pair is reported by the sequential check below (first offending index)
  // variant: the pair-per-lane kernel needs qlen < 8*NCH (NCH <= 20) and scores that fit the 16-bit
  // eh packing; everything else goes to the wave-per-pair kernel. A pair with h0 = 0 ends after its
  // first row (every H of row 0 is 0, so its row maximum is 0, bandedSWA.cpp:222-223): mixed into a
  // wave it leaves its lane idle for the wave's whole run, so those pairs get waves of their own.
  // The sort key is (high, low): high = variant, h0 == 0, h0 in steps of 8 (the first rows' band of
  // nonzero cells is ~h0 - o_ins wide, so it sets how far the early rows sweep), query length in
  // steps of 8 (similar band ends per wave); low = decreasing target length (similar row counts).
  constexpr int kQB = 64, kHB = 8, kTB = 4096;
  const char *ke = getenv("GB_BSW_H0STEP");  // probes: the h0 step (0: h0 not in the key)
  const int h0step = ke ? atoi(ke) : 8;
  const char *qe = getenv("GB_BSW_QSHIFT");  // probes: query-length step 1 << QSHIFT (default 8)
  const int qshift = qe ? std::min(std::max(atoi(qe), 0), 6) : 3;
  const char *oe = getenv("GB_BSW_KEYORD");  // probes: 0 = query length before the h0 step
  const bool h0first = !(oe && atoi(oe) == 0);
  auto key_hi = [h0step, qshift, h0first](int v, const gbbsw::Pair &q) {
    const uint32_t z = q.h0 == 0 ? 1 : 0, qb = (uint32_t)(kQB - 1 - std::min(q.qlen >> qshift, kQB - 1));
    const uint32_t hb = h0step > 0 ? (uint32_t)std::min(std::max(q.h0, 0) / h0step, kHB - 1) : 0;
    if (h0first) return (((uint32_t)v * 2 + z) * kHB + hb) * kQB + qb;
    return (((uint32_t)v * 2 + z) * kQB + qb) * kHB + hb;
  };
  auto key_lo = [](const gbbsw::Pair &q) { return (uint32_t)(kTB - 1 - std::min(q.tlen, kTB - 1)); };
  auto sort_key = [&](int v, const gbbsw::Pair &q) { return key_hi(v, q) * (uint32_t)kTB + key_lo(q); };
  const bool lane_ok = params->o_del >= 0 && params->o_ins >= 0 && mn >= -128 && mx <= 127;
  std::vector<gbbsw::Pair> P((size_t)n);
  std::vector<uint8_t> var((size_t)n);
  std::vector<uint32_t> keys((size_t)n);
  std::atomic<int64_t> bad{n};
  auto plan = [&](int64_t lo, int64_t hi) {
    for (int64_t p = lo; p < hi; ++p) {
      const gb_seqpair &s = pairs[p];
      if (!(s.len2 >= 1 && s.len2 <= GB_BSW_MAX_QLEN && s.len1 >= 0 && s.idr >= 0 && s.idr + s.len1 <= ref_bytes &&
            s.idq >= 0 && s.idq + s.len2 <= qer_bytes)) {
        int64_t b = bad.load();
        while (p < b && !bad.compare_exchange_weak(b, p)) {
        }
        return;
      }
      const gbbsw::Pair q{s.idr, s.idq, s.len1, s.len2, s.h0, gbbsw::adjust_w(params->w, s.len2, mx, *params)};
      P[p] = q;
      int v = 5;
      if (lane_ok && q.h0 >= 0 && (int64_t)q.h0 + (int64_t)q.qlen * mx < 30000) {
        const int nch = (q.qlen + 8) / 8;  // columns 0..qlen
        v = nch <= 4 ? 0 : nch <= 8 ? 1 : nch <= 12 ? 2 : nch <= 16 ? 3 : nch <= 20 ? 4 : 5;
      }
      var[p] = (uint8_t)v;
      keys[p] = sort_key(v, q);
    }
  };
  const int nth = n >= (1 << 17) ? (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency())) : 1;
  if (nth == 1) {
    plan(0, n);
  } else {
    std::vector<std::thread> th;
    for (int t = 1; t < nth; t++) th.emplace_back(plan, n * t / nth, n * (t + 1) / nth);
    plan(0, n / nth);
    for (auto &x : th) x.join();
  }
  if (bad.load() < n) {
    const int64_t p = bad.load();
    const gb_seqpair &s = pairs[p];
    GB_ARG(s.len2 >= 1 && s.len2 <= GB_BSW_MAX_QLEN && s.len1 >= 0,
           "gb_bsw_batch_create: pair %lld has len1=%d len2=%d (need len2 in [1,%d])", (long long)p,
           s.len1, s.len2, GB_BSW_MAX_QLEN);
    GB_ARG(false, "gb_bsw_batch_create: pair %lld lies outside the sequence buffers", (long long)p);
  }
  // Tail balance for batches that fill the chip only about once with lane waves: then the step is
  // the slowest lane wave, a wave of the longest pairs of the widest variants (~rows x chunks x
  // 0.28 us: ~1.4 ms for 250 rows at NCH 20), while the wave-per-pair kernel takes such a pair in
  // tens of microseconds. The fraction GB_BSW_TAIL (default 0.1) of the lane pairs with the
  // largest rows x chunks moves to the wave-per-pair kernel, which runs beside the lane kernels.
  {
    const char *te = getenv("GB_BSW_TAIL");
    // r03ab, 100 k pairs: 0 228, 0.05 234, 0.1 258, 0.2 243 GCUPS. A batch of fewer lane waves than
    // SIMDs (the 1/8 shard of the 'small' set: 12.5 k pairs, 195 waves on 1 024 SIMDs) is one wave's
    // critical path long: every lane pair goes to the wave-per-pair kernel (1.30 -> 0.56 ms,
    // profiles/r05b_bsw_small.log). The crossover against the 0.1 split, swept on the 'large' pair
    // distribution (profiles/r06j/r06k_bsw_tail_*.txt, 256 CUs): all-to-wave wins from 8 K to 65 536
    // pairs (49 152: 1.19 vs 1.79 ms; 65 536: 1.52 vs 1.65) and loses from 80 000 (1.79 vs 1.64 ms),
    // so the rule is n < 64 x 4.5 x CUs (73 728 pairs)
    const double frac = te ? atof(te) : (2 * n < (int64_t)64 * 9 * std::max(B->num_cus, 1) ? 1.0 : 0.1);
    const int64_t fill = (int64_t)64 * 8 * std::max(B->num_cus, 1);  // lane waves of 64 pairs, 2 per SIMD
    if (frac > 0 && (n >= 1024 || frac >= 1.0) && n <= 2 * fill) {
      std::vector<uint32_t> cost;
      cost.reserve((size_t)n);
      for (int64_t p = 0; p < n; ++p)
        if (var[p] < 5 && P[p].h0 != 0) cost.push_back((uint32_t)P[p].tlen * (uint32_t)(4 * (var[p] + 1)));
      const size_t k = std::min(cost.size(), (size_t)((double)cost.size() * std::min(1.0, frac)));
      if (k > 0) {
        std::nth_element(cost.begin(), cost.end() - (ptrdiff_t)k, cost.end());
        const uint32_t cut = *(cost.end() - (ptrdiff_t)k);
        for (int64_t p = 0; p < n; ++p)
          if (var[p] < 5 && P[p].h0 != 0 && (uint32_t)P[p].tlen * (uint32_t)(4 * (var[p] + 1)) >= cut) {
            var[p] = 5;
            keys[p] = sort_key(5, P[p]);
          }
      }
    }
  }
  std::vector<uint32_t> order((size_t)n);
  if (n < (1 << 16)) {
    // small batches: a stable comparison sort (the counting sort's 1.3 M-entry histogram would cost
    // more than the call)
    for (int64_t p = 0; p < n; ++p) order[(size_t)p] = (uint32_t)p;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return keys[a] < keys[b]; });
  } else {
    // two stable counting passes (least significant first): by the low key, then the high key
    // (the first pass carries each pair's high key along, so the second reads it sequentially)
    std::vector<uint32_t> tmp((size_t)n), thi((size_t)n);
    {
      std::vector<int64_t> cnt((size_t)kTB + 1, 0);
      for (int64_t p = 0; p < n; ++p) cnt[keys[p] % kTB]++;
      int64_t acc = 0;
      for (auto &c : cnt) {
        const int64_t t = c;
        c = acc;
        acc += t;
      }
      for (int64_t p = 0; p < n; ++p) {
        const int64_t at = cnt[keys[p] % kTB]++;
        tmp[(size_t)at] = (uint32_t)p;
        thi[(size_t)at] = keys[p] / kTB;
      }
    }
    {
      std::vector<int64_t> cnt((size_t)gb_bsw_batch::kVariants * 2 * kQB * kHB + 1, 0);
      for (int64_t k = 0; k < n; ++k) cnt[thi[k]]++;
      int64_t acc = 0;
      for (auto &c : cnt) {
        const int64_t t = c;
        c = acc;
        acc += t;
      }
      for (int64_t k = 0; k < n; ++k) order[cnt[thi[k]]++] = tmp[k];
    }
  }
  for (int v = 0; v <= gb_bsw_batch::kVariants; ++v) B->seg[v] = 0;
  for (int64_t p = 0; p < n; ++p) B->seg[var[p] + 1]++;
  for (int v = 0; v < gb_bsw_batch::kVariants; ++v) B->seg[v + 1] += B->seg[v];
  B->params = *params;
  B->n = n;
  B->ran = false;
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  size_t cap_pairs = B->cap_n, cap_order = B->cap_n, cap_out = B->cap_n * 6, cap_cells = B->cap_n;
  int st = bsw_reserve(&B->d_pairs, cap_pairs, nn);
  if (!st) st = bsw_reserve(&B->d_order, cap_order, nn);
  if (!st) st = bsw_reserve(&B->d_out6, cap_out, nn * 6);
  if (!st) st = bsw_reserve(&B->d_cells, cap_cells, nn);
  if (st) {
    // one of the four shares cap_n and may now be freed or smaller: the next fill reallocates all
    B->cap_n = 0;
    return st;
  }
  B->cap_n = std::max(B->cap_n, nn);
  if (n) GB_HIP(hipMemcpyAsync(B->d_order, order.data(), (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice, B->stream));
  if (n) GB_HIP(hipMemcpyAsync(B->d_pairs, P.data(), (size_t)n * sizeof(gbbsw::Pair), hipMemcpyHostToDevice, B->stream));
  GB_HIP(hipStreamSynchronize(B->stream));  // the host vectors die on return
  if (up.t.joinable()) up.t.join();
  GB_HIP(up_err);
  return GB_OK;
}

}  // namespace

extern "C" {

int gb_bsw_batch_create(const gb_bsw_params *params, const gb_seqpair *pairs, int64_t n,
                        const uint8_t *ref, int64_t ref_bytes, const uint8_t *qer, int64_t qer_bytes,
                        gb_bsw_batch **out) {
  GB_ARG(out, "gb_bsw_batch_create: null out");
  *out = nullptr;
  gb_bsw_batch *B = nullptr;
  int st = bsw_batch_new(&B);
  if (st) return st;
  if ((st = bsw_batch_fill(B, params, pairs, n, ref, ref_bytes, qer, qer_bytes))) {
    gb_bsw_batch_destroy(B);
    return st;
  }
  *out = B;
  return GB_OK;
}

int gb_bsw_batch_run(gb_bsw_batch *B) {
  gb::Range range_("gb.bsw.batch_run");
  GB_ARG(B, "gb_bsw_batch_run: null batch");
  GB_HIP(hipSetDevice(B->device));
  GB_HIP(hipMemsetAsync(B->d_total, 0, gb_bsw_batch::kTotals * sizeof(unsigned long long), B->stream));
  GB_HIP(hipEventRecord(B->ev[0], B->stream));
  bool forked[gb_bsw_batch::kVariants] = {};
  if (B->n > 0) {
    gbbsw::LaneArgs L;
    L.pairs = B->d_pairs;
    L.order = B->d_order;
    L.tgt = B->d_tgt;
    L.qry = B->d_qry;
    L.out6 = B->d_out6;
    L.cells = B->d_cells;
    L.total_cells = B->d_total;
    L.o_del = B->params.o_del;
    L.e_del = B->params.e_del;
    L.o_ins = B->params.o_ins;
    L.e_ins = B->params.e_ins;
    L.zdrop = B->params.zdrop;
    for (int t = 0; t < 5; ++t) {  // score bytes of row t for query codes 0..3 and 4
      uint32_t lo = 0;
      for (int q = 0; q < 4; ++q) lo |= (uint32_t)(uint8_t)B->params.mat[t * 5 + q] << (8 * q);
      L.tab[2 * t] = lo;
      L.tab[2 * t + 1] = (uint32_t)(uint8_t)B->params.mat[t * 5 + 4];
    }
    const bool sym = B->params.o_del == B->params.o_ins && B->params.e_del == B->params.e_ins;
    void (*lane_kernels[2][5])(gbbsw::LaneArgs) = {
        {gbbsw::bsw_lane_kernel<4, false>, gbbsw::bsw_lane_kernel<8, false>, gbbsw::bsw_lane_kernel<12, false>,
         gbbsw::bsw_lane_kernel<16, false>, gbbsw::bsw_lane_kernel<20, false>},
        {gbbsw::bsw_lane_kernel<4, true>, gbbsw::bsw_lane_kernel<8, true>, gbbsw::bsw_lane_kernel<12, true>,
         gbbsw::bsw_lane_kernel<16, true>, gbbsw::bsw_lane_kernel<20, true>}};
    L.prof = nullptr;
    const char *pe = getenv("GB_BSW_PROF");
    const bool prof = pe && *pe == '1';
    if (prof) {
      if (!B->d_prof) GB_HIP(hipMalloc(&B->d_prof, 25 * sizeof(unsigned long long)));
      GB_HIP(hipMemsetAsync(B->d_prof, 0, 25 * sizeof(unsigned long long), B->stream));
    }
    // variant v launches on side stream v, forked from `stream` here and joined back below
    GB_HIP(hipEventRecord(B->fork, B->stream));
    for (int v = 0; v < gb_bsw_batch::kVariants; ++v)
      if (B->seg[v + 1] > B->seg[v]) {
        GB_HIP(hipStreamWaitEvent(B->side[v], B->fork, 0));
        forked[v] = true;
      }
    for (int v = 0; v < 5; ++v) {
      if (prof) L.prof = B->d_prof + 5 * v;
      L.first = B->seg[v];
      L.count = B->seg[v + 1] - B->seg[v];
      if (L.count == 0) continue;
      hipLaunchKernelGGL(lane_kernels[sym ? 1 : 0][v], dim3((unsigned)((L.count + 63) / 64)), dim3(64), 0, B->side[v],
                         L);
      GB_HIP(hipGetLastError());
    }
    const int64_t nw = B->seg[6] - B->seg[5];
    if (nw > 0) {
      gbbsw::Args A;
      A.pairs = B->d_pairs;
      A.list = B->d_order + B->seg[5];
      A.n = nw;
      A.tgt = B->d_tgt;
      A.qry = B->d_qry;
      A.out6 = B->d_out6;
      A.cells = B->d_cells;
      A.total_cells = B->d_total;
      A.next = reinterpret_cast<unsigned int *>(B->d_total + 1);
      A.o_del = B->params.o_del;
      A.e_del = B->params.e_del;
      A.o_ins = B->params.o_ins;
      A.e_ins = B->params.e_ins;
      A.zdrop = B->params.zdrop;
      std::memset(A.mat, 0, sizeof(A.mat));
      std::memcpy(A.mat, B->params.mat, 25);
      const int64_t cap = (int64_t)B->num_cus * gbbsw::kBlocksPerCU;
      const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(cap, (nw + gbbsw::kWavesPerBlock - 1) / gbbsw::kWavesPerBlock));
      hipLaunchKernelGGL(gbbsw::bsw_extend_kernel, dim3((unsigned)blocks), dim3(64 * gbbsw::kWavesPerBlock), 0,
                         B->side[5], A);
      GB_HIP(hipGetLastError());
    }
  }
  for (int v = 0; v < gb_bsw_batch::kVariants; ++v)
    if (forked[v]) {
      GB_HIP(hipEventRecord(B->join[v], B->side[v]));
      GB_HIP(hipStreamWaitEvent(B->stream, B->join[v], 0));
    }
  GB_HIP(hipEventRecord(B->ev[1], B->stream));
  B->ran = true;
  if (B->d_prof && getenv("GB_BSW_PROF")) {
    unsigned long long h[25];
    GB_HIP(hipMemcpyAsync(h, B->d_prof, sizeof(h), hipMemcpyDeviceToHost, B->stream));
    GB_HIP(hipStreamSynchronize(B->stream));
    for (int v = 0; v < 5; ++v)
      if (h[5 * v])
        fprintf(stderr,
                "[bsw prof] NCH=%d pairs %lld: wave rows %llu, lane-row use %.3f, column use %.3f (cells %llu / "
                "lane-column slots %llu), chunk-columns inside every band %.3f\n",
                4 * (v + 1), (long long)(B->seg[v + 1] - B->seg[v]), h[5 * v], h[5 * v + 2] / (64.0 * h[5 * v]),
                h[5 * v + 3] / (64.0 * h[5 * v + 1]), h[5 * v + 3], 64 * h[5 * v + 1], (double)h[5 * v + 4] / h[5 * v + 1]);
  }
  return GB_OK;
}

int gb_bsw_batch_sync(gb_bsw_batch *B) {
  GB_ARG(B, "gb_bsw_batch_sync: null batch");
  GB_HIP(hipStreamSynchronize(B->stream));
  return GB_OK;
}

int gb_bsw_batch_results(gb_bsw_batch *B, gb_seqpair *pairs, int32_t *out6, int32_t *cells,
                         int64_t *total_cells) {
  GB_ARG(B, "gb_bsw_batch_results: null batch");
  if (!B->ran) {
    gb::set_error("gb_bsw_batch_results: batch has not been run");
    return GB_ERR_STATE;
  }
  GB_HIP(hipSetDevice(B->device));
  GB_HIP(hipStreamSynchronize(B->stream));
  const size_t n = (size_t)B->n;
  std::vector<int32_t> o;
  if (n && (pairs || out6)) {
    int32_t *dst = out6;
    if (!dst) {
      o.resize(6 * n);
      dst = o.data();
    }
    GB_HIP(hipMemcpy(dst, B->d_out6, n * 6 * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (pairs) {
      auto scatter = [&](size_t lo, size_t hi) {
        for (size_t p = lo; p < hi; ++p) {
          const int32_t *r = dst + 6 * p;
          pairs[p].score = r[0];
          pairs[p].qle = r[1];
          pairs[p].tle = r[2];
          pairs[p].gtle = r[3];
          pairs[p].gscore = r[4];
          pairs[p].max_off = r[5];
        }
      };
      const size_t nth = n >= (1u << 17) ? std::max(1u, std::min(8u, std::thread::hardware_concurrency())) : 1;
      std::vector<std::thread> th;
      for (size_t t = 1; t < nth; t++) th.emplace_back(scatter, n * t / nth, n * (t + 1) / nth);
      scatter(0, n / nth);
      for (auto &x : th) x.join();
    }
  }
  if (n && cells) GB_HIP(hipMemcpy(cells, B->d_cells, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (total_cells) {
    unsigned long long t = 0;
    GB_HIP(hipMemcpy(&t, B->d_total, sizeof(t), hipMemcpyDeviceToHost));
    *total_cells = (int64_t)t;
  }
  return GB_OK;
}

int gb_bsw_batch_timing(gb_bsw_batch *B, float *kernel_ms) {
  GB_ARG(B && kernel_ms, "gb_bsw_batch_timing: bad arguments");
  if (!B->ran) {
    gb::set_error("gb_bsw_batch_timing: batch has not been run");
    return GB_ERR_STATE;
  }
  GB_HIP(hipEventSynchronize(B->ev[1]));
  GB_HIP(hipEventElapsedTime(kernel_ms, B->ev[0], B->ev[1]));
  return GB_OK;
}

}  // extern "C"

namespace {

// ---- small calls (the reference's 512-pair getScores16 batches, main_banded.cpp:896-924) ----------
// A pair-per-lane launch lasts as long as its slowest pair's whole DP (~0.5 ms), so a call of a few
// hundred pairs is latency-bound. Small calls instead run every pair on the wave-per-pair kernel
// (rows are wave-wide scans: a pair takes tens of microseconds), with the call's bytes packed on the
// host into one pinned staging buffer -- descriptors, the pairs' own target and query bytes (the
// caller's fixed-stride buffers are mostly padding), zeroed counters -- moved by one H2D copy, and
// the results back by one D2H copy on the calling thread's stream.
constexpr int64_t kSmallCall = 16384;  // pairs; GB_BSW_SMALL overrides (0 = never)

struct SmallWs {
  int device = -1, num_cus = 256;
  hipStream_t stream = nullptr;
  uint8_t *h = nullptr, *d = nullptr;
  size_t hcap = 0, dcap = 0;
};

int64_t small_call_limit() {
  const char *e = getenv("GB_BSW_SMALL");  // read per call: tests switch paths inside one process
  return e ? (int64_t)atoll(e) : kSmallCall;
}

size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

struct SmallReq {
  const gb_bsw_params *params;
  gb_seqpair *pairs;
  int64_t n;
  const uint8_t *ref, *qer;
  int64_t *total_cells;
  int status = GB_OK;
  bool done = false;
};

SmallWs *small_ws(int dev, int *st) {
  // one workspace per (host thread, device); never freed (see gb_bsw_get_scores16_ex)
  thread_local std::vector<SmallWs *> wss;
  for (auto *w : wss)
    if (w->device == dev) return w;
  auto *W = new SmallWs();
  W->device = dev;
  hipError_t e = hipDeviceGetAttribute(&W->num_cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&W->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    gb::set_error("getScores16 workspace: %s", hipGetErrorString(e));
    *st = GB_ERR_HIP;
    return nullptr;
  }
  wss.push_back(W);
  return W;
}

// One launch for a group of requests with the same parameters: their pairs are concatenated (and
// their sequences packed) into W's staging buffer, run on the wave-per-pair kernel, and each
// request's SeqPair fields and cell total written back.
int small_group(SmallWs *W, const std::vector<SmallReq *> &g) {
  const gb_bsw_params *params = g[0]->params;
  int mx = 0;
  for (int k = 0; k < 25; ++k) mx = std::max(mx, (int)params->mat[k]);
  int64_t n = 0, tb = 0, qb = 0;
  for (const SmallReq *r : g) {
    n += r->n;
    for (int64_t p = 0; p < r->n; ++p) {
      tb += r->pairs[p].len1;
      qb += r->pairs[p].len2;
    }
  }
  // staging / device layout: [Pair n | list n | ctl 16 B | tgt | qry] (uploaded) [out6 n | cells n]
  const size_t o_list = up16(sizeof(gbbsw::Pair) * (size_t)n), o_ctl = o_list + up16(4 * (size_t)n),
               o_tgt = o_ctl + 16, o_qry = o_tgt + up16((size_t)tb), up_bytes = o_qry + up16((size_t)qb),
               o_out = up_bytes, o_cells = o_out + up16(24 * (size_t)n), d_bytes = o_cells + up16(4 * (size_t)n);
  if (std::max(up_bytes, d_bytes - o_out) > W->hcap) {
    if (W->h) (void)hipHostFree(W->h);
    W->h = nullptr;
    W->hcap = 0;
    const size_t want = std::max<size_t>(2 * std::max(up_bytes, d_bytes - o_out), 1 << 20);
    GB_HIP(hipHostMalloc(&W->h, want, hipHostMallocDefault));
    W->hcap = want;
  }
  if (d_bytes > W->dcap) {
    (void)hipFree(W->d);
    W->d = nullptr;
    W->dcap = 0;
    const size_t want = std::max<size_t>(2 * d_bytes, 1 << 20);
    GB_HIP(hipMalloc(&W->d, want));
    W->dcap = want;
  }
  uint8_t *h = W->h;
  auto *P = reinterpret_cast<gbbsw::Pair *>(h);
  auto *list = reinterpret_cast<uint32_t *>(h + o_list);
  int64_t to = 0, qo = 0, k = 0;
  for (const SmallReq *r : g)
    for (int64_t p = 0; p < r->n; ++p, ++k) {
      const gb_seqpair &sp = r->pairs[p];
      std::memcpy(h + o_tgt + to, r->ref + sp.idr, (size_t)sp.len1);
      std::memcpy(h + o_qry + qo, r->qer + sp.idq, (size_t)sp.len2);
      P[k] = gbbsw::Pair{to, qo, sp.len1, sp.len2, sp.h0, gbbsw::adjust_w(params->w, sp.len2, mx, *params)};
      list[k] = (uint32_t)k;
      to += sp.len1;
      qo += sp.len2;
    }
  std::memset(h + o_ctl, 0, 16);
  GB_HIP(hipMemcpyAsync(W->d, h, up_bytes, hipMemcpyHostToDevice, W->stream));
  gbbsw::Args A;
  A.pairs = reinterpret_cast<const gbbsw::Pair *>(W->d);
  A.list = reinterpret_cast<const uint32_t *>(W->d + o_list);
  A.n = n;
  A.tgt = W->d + o_tgt;
  A.qry = W->d + o_qry;
  A.out6 = reinterpret_cast<int32_t *>(W->d + o_out);
  A.cells = reinterpret_cast<int32_t *>(W->d + o_cells);
  A.total_cells = reinterpret_cast<unsigned long long *>(W->d + o_ctl);
  A.next = reinterpret_cast<unsigned int *>(W->d + o_ctl + 8);
  A.o_del = params->o_del;
  A.e_del = params->e_del;
  A.o_ins = params->o_ins;
  A.e_ins = params->e_ins;
  A.zdrop = params->zdrop;
  std::memset(A.mat, 0, sizeof(A.mat));
  std::memcpy(A.mat, params->mat, 25);
  const int64_t blocks = std::max<int64_t>(
      1, std::min<int64_t>((int64_t)W->num_cus * gbbsw::kBlocksPerCU, (n + gbbsw::kWavesPerBlock - 1) / gbbsw::kWavesPerBlock));
  hipLaunchKernelGGL(gbbsw::bsw_extend_kernel, dim3((unsigned)blocks), dim3(64 * gbbsw::kWavesPerBlock), 0, W->stream, A);
  GB_HIP(hipGetLastError());
  // out6 and the per-pair cell counts back in one copy (they are adjacent on the device)
  GB_HIP(hipMemcpyAsync(h, W->d + o_out, d_bytes - o_out, hipMemcpyDeviceToHost, W->stream));
  GB_HIP(hipStreamSynchronize(W->stream));
  const auto *r6 = reinterpret_cast<const int32_t *>(h);
  const auto *cells = reinterpret_cast<const int32_t *>(h + (o_cells - o_out));
  k = 0;
  for (SmallReq *r : g) {
    int64_t c = 0;
    for (int64_t p = 0; p < r->n; ++p, ++k) {
      const int32_t *o = r6 + 6 * k;
      gb_seqpair &sp = r->pairs[p];
      sp.score = o[0];
      sp.qle = o[1];
      sp.tle = o[2];
      sp.gtle = o[3];
      sp.gscore = o[4];
      sp.max_off = o[5];
      c += cells[k];
    }
    if (r->total_cells) *r->total_cells = c;
  }
  return GB_OK;
}

// Flat combining across host threads: the reference calls getScores16 on 512-pair batches from an
// OpenMP team, each call synchronous. A calling thread queues its request; whichever thread finds
// fewer than kLeaders groups in flight takes every queued request with the same parameters and runs
// them as one launch, the others wait for their request to be marked done. While one group runs, the
// next one accumulates, so groups grow to about one call per waiting thread.
// groups in flight per device (packing / copying while others compute): getScores16 per 512 pairs
// from 16 threads, 2 M pairs: 1 / 2 / 3 / 4 / 6 groups 40.3 / 48.6 / 52.4 / 52.9 / 49.1 GCUPS
// (profiles/r06u_bsw_leaders.txt)
constexpr int kLeaders = 4;
int leaders_limit() {  // GB_BSW_LEADERS (probes)
  static const int v = [] {
    const char *e = getenv("GB_BSW_LEADERS");
    return e ? std::max(1, atoi(e)) : kLeaders;
  }();
  return v;
}

struct Combiner {
  std::mutex m;
  std::condition_variable cv;
  std::vector<SmallReq *> pending;
  int leaders = 0;
};

Combiner &combiner(int dev) {
  static std::mutex gm;
  static std::vector<std::pair<int, Combiner *>> all;
  std::lock_guard<std::mutex> lk(gm);
  for (auto &c : all)
    if (c.first == dev) return *c.second;
  all.emplace_back(dev, new Combiner());  // never freed, like the workspaces
  return *all.back().second;
}

int small_call(const gb_bsw_params *params, gb_seqpair *pairs, int64_t n, const uint8_t *ref, int64_t ref_bytes,
               const uint8_t *qer, int64_t qer_bytes, int64_t *total_cells) {
  for (int64_t p = 0; p < n; ++p) {
    const gb_seqpair &sp = pairs[p];
    GB_ARG(sp.len2 >= 1 && sp.len2 <= GB_BSW_MAX_QLEN && sp.len1 >= 0,
           "gb_bsw_get_scores16: pair %lld has len1=%d len2=%d (need len2 in [1,%d])", (long long)p, sp.len1,
           sp.len2, GB_BSW_MAX_QLEN);
    GB_ARG(sp.idr >= 0 && sp.idr + sp.len1 <= ref_bytes && sp.idq >= 0 && sp.idq + sp.len2 <= qer_bytes,
           "gb_bsw_get_scores16: pair %lld lies outside the sequence buffers", (long long)p);
  }
  int dev = 0;
  GB_HIP(hipGetDevice(&dev));
  int st = GB_OK;
  SmallWs *W = small_ws(dev, &st);
  if (!W) return st;
  SmallReq me{params, pairs, n, ref, qer, total_cells};
  Combiner &C = combiner(dev);
  std::unique_lock<std::mutex> lk(C.m);
  C.pending.push_back(&me);
  while (!me.done) {
    if (C.leaders < leaders_limit() && !C.pending.empty()) {
      // lead: take the queued requests with the first one's parameters (up to kSmallCall pairs)
      std::vector<SmallReq *> g, rest;
      int64_t np = 0;
      for (SmallReq *r : C.pending)
        if ((g.empty() || (!std::memcmp(r->params, g[0]->params, sizeof(gb_bsw_params)) && np + r->n <= kSmallCall)))
          g.push_back(r), np += r->n;
        else
          rest.push_back(r);
      C.pending.swap(rest);
      C.leaders++;
      lk.unlock();
      const int gst = small_group(W, g);
      std::string err = gst ? gb_last_error() : std::string();
      lk.lock();
      for (SmallReq *r : g) {
        r->status = gst;
        r->done = true;
      }
      C.leaders--;
      C.cv.notify_all();
      if (gst && !me.done) gb::set_error("%s", err.c_str());
    } else {
      C.cv.wait(lk);
    }
  }
  lk.unlock();
  if (me.status && me.status != GB_OK) gb::set_error("gb_bsw_get_scores16: a combined getScores16 launch failed");
  return me.status;
}

}  // namespace

extern "C" {

int gb_bsw_get_scores16_ex(const gb_bsw_params *params, gb_seqpair *pairs, int64_t n, const uint8_t *ref,
                           int64_t ref_bytes, const uint8_t *qer, int64_t qer_bytes, int64_t *total_cells) {
  gb::Range range_("gb.bsw.get_scores16");
  GB_ARG(params && n >= 0 && (n == 0 || pairs), "gb_bsw_get_scores16: bad arguments");
  GB_ARG(params->e_del > 0 && params->e_ins > 0, "gb_bsw_get_scores16: gap extension must be > 0");
  GB_ARG(ref_bytes >= 0 && qer_bytes >= 0 && (ref_bytes == 0 || ref) && (qer_bytes == 0 || qer),
         "gb_bsw_get_scores16: bad sequence buffers");
  if (n > 0 && n <= small_call_limit()) return small_call(params, pairs, n, ref, ref_bytes, qer, qer_bytes, total_cells);
  // one cached batch per (host thread, device): the reference calls getScores16 once per batch of
  // 512 pairs (main_banded.cpp:896-909), so streams, events and buffers are reused across calls.
  // Never freed (freeing at thread exit could run after the HIP runtime is torn down).
  thread_local std::vector<std::pair<int, gb_bsw_batch *>> ws;
  int dev = 0;
  GB_HIP(hipGetDevice(&dev));
  gb_bsw_batch *B = nullptr;
  for (auto &w : ws)
    if (w.first == dev) B = w.second;
  int st = GB_OK;
  if (!B) {
    if ((st = bsw_batch_new(&B))) return st;
    ws.emplace_back(dev, B);
  }
  if ((st = bsw_batch_fill(B, params, pairs, n, ref, ref_bytes, qer, qer_bytes))) return st;
  st = gb_bsw_batch_run(B);
  if (!st) st = gb_bsw_batch_results(B, pairs, nullptr, nullptr, total_cells);
  return st;
}

int gb_bsw_get_scores16(const gb_bsw_params *params, gb_seqpair *pairs, int64_t n, const uint8_t *ref,
                        int64_t ref_bytes, const uint8_t *qer, int64_t qer_bytes) {
  return gb_bsw_get_scores16_ex(params, pairs, n, ref, ref_bytes, qer, qer_bytes, nullptr);
}

// getScores8 (bandedSWA.cpp:426-725, smithWaterman256_8 :727-1123): the reference's 8-bit kernel
// keeps every score in int8 lanes and is only defined where nothing wraps; its own caller in bwa-mem2
// sends a pair to it iff len1 < 128, len2 < 128 and h0 + min(len1, len2) * a < 128
// (tools/bwa-mem2/src/bwamem.cpp:2152-2155, MAX_SEQ_LEN8 = 128). Inside that domain the 8-bit kernel
// is the 16-bit DP, so those pairs run the exact kernel; a pair outside it is refused loudly (the
// reference asserts on len2, bandedSWA.cpp:607-608, and wraps silently otherwise).
int gb_bsw_get_scores8(const gb_bsw_params *params, int32_t w_match, gb_seqpair *pairs, int64_t n, const uint8_t *ref,
                       int64_t ref_bytes, const uint8_t *qer, int64_t qer_bytes, int64_t *total_cells) {
  GB_ARG(params && (n == 0 || pairs), "gb_bsw_get_scores8: null argument");
  for (int64_t i = 0; i < n; i++) {
    const gb_seqpair &p = pairs[i];
    const int64_t minval = (int64_t)p.h0 + (int64_t)std::min(p.len1, p.len2) * w_match;
    GB_ARG(p.len1 < 128 && p.len2 < 128 && p.len1 >= 0 && p.len2 >= 0 && minval < 128,
           "gb_bsw_get_scores8: pair %lld (len1 %d, len2 %d, h0 %d) is outside the 8-bit kernel's domain "
           "(len1 < 128, len2 < 128, h0 + min(len1, len2) * %d < 128; bwamem.cpp:2152-2155): use getScores16",
           (long long)i, p.len1, p.len2, p.h0, w_match);
  }
  return gb_bsw_get_scores16_ex(params, pairs, n, ref, ref_bytes, qer, qer_bytes, total_cells);
}

}  // extern "C"
