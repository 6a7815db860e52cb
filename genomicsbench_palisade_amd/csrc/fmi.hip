// fmi.hip -- MI355X (gfx950) bwa-mem2 SMEM search: index upload, search kernel, compaction, C ABI.
//
// Semantics (the reference's plaintext arithmetic; HE layer is an identity):
//   backwardExt           tools/bwa-mem2/src/FMI_search.cpp:1536-1565 (Occ = GET_OCC, FMI_search.h:81-89)
//   SMEMs at one position FMI_search.cpp:986-1180   (getSMEMsOnePosOneThread)
//   all positions         FMI_search.cpp:1182-1241  (getSMEMsAllPosOneThread)
//   LAST seeds            FMI_search.cpp:1243-1326  (bwtSeedStrategyAllPosOneThread)
//   batch pipeline        benchmarks/fmi/fmi.cpp:253-348 (smem1, reseed, LAST, rid offset, sort)
//
// MI355X design: the work is a chain of dependent random 64-byte gathers (two CP_OCC lines per
// backwardExt) with data-dependent control flow. One read per lane, and every lane runs a state
// machine that issues exactly one backwardExt per loop trip, so the divergent bookkeeping between
// extensions is short and the gathers of all 64 lanes issue together; thousands of waves keep the
// HBM/Infinity-Cache latency covered. A lane that finishes a read takes the next one from a
// device-wide counter (per-wave aggregated atomic), so long and short reads balance. Each lane's
// `prev` list lives in a private scratch slice (L2-resident in practice); each read's SMEMs go to a
// fixed-capacity slot, are insertion-sorted by (m asc, n desc) in place, then compacted by an
// exclusive scan + scatter into the reference's (rid, m, n desc) order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/gb_fmi.h"
#include "../../include/gb.h"
#include "gb_common.h"
#include "fmi_index.h"
#include "fmi_wave.h"

namespace gbfmi {

constexpr int kCap = 40;       // first-pass SMEM slots per read (~8 on average on the synthetic sets)
constexpr int kBigCap = 2048;  // second pass, for the rare reads that overflow the first
constexpr int kMaxOvf = 16384; // reads the second pass can take

// `prev` entries (Ent / PEnt, fmi_index.h) are laid out wave-interleaved (entry e of lane t of
// wave w at [(w * stride + e) * 64 + t]) so the lanes of a wave touching the same list depth hit the
// same lines.
struct PList {  // one lane's view of its wave-interleaved scratch
  PEnt *base;   // &scratch[(wave * stride) * 64 + lane]
  __device__ __forceinline__ Ent get(int e) const { return unpack_ent(base[(size_t)e * 64]); }
  __device__ __forceinline__ void put(int e, const Ent &v) const { base[(size_t)e * 64] = pack_ent(v); }
};

// byte codes -> 4-bit codes, 8 per word (base b of word w at bits 4*(b))
__global__ void pack_q4(const uint8_t *__restrict__ qdb, int32_t stride, int32_t nreads, int32_t q4_stride,
                        uint32_t *__restrict__ q4) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = t / q4_stride, w = t % q4_stride;
  if (r >= nreads) return;
  uint32_t v = 0;
  for (int b = 0; b < 8; b++) {
    const int64_t j = w * 8 + b;
    const uint32_t c = j < stride ? min((uint32_t)qdb[r * stride + j], 15u) : 4u;
    v |= c << (4 * b);
  }
  q4[r * q4_stride + w] = v;
}

// byte codes -> 2-bit codes, 16 per word (base b of word w at bits 2*(b); an N or any code >= 4 reads
// 0 here), and per read its N positions: up to four, one per byte (in any order: the search only
// tests membership), 0xFF = none (kNOverflow: more than four; the search hands such a read to the
// heavy pass). npos starts all ones and ncnt zero; an N (rare) takes a byte by an atomic count and
// writes it with one atomic AND; npos_finish marks the reads with more than four.
constexpr uint32_t kNOverflow = 0xFEFEFEFEu;
__global__ void pack_q2(const uint8_t *__restrict__ qdb, int32_t stride, const int32_t *__restrict__ lens,
                        int32_t nreads, int32_t q2_stride, uint32_t *__restrict__ q2, uint32_t *__restrict__ npos,
                        int32_t *__restrict__ ncnt) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = t / q2_stride, w = t % q2_stride;
  if (r >= nreads) return;
  const int L = lens[r];
  uint32_t v = 0;
  for (int b = 0; b < 16; b++) {
    const int64_t j = w * 16 + b;
    const uint32_t c = j < stride ? (uint32_t)qdb[r * stride + j] : 0u;
    v |= (c < 4 ? c : 0u) << (2 * b);
    if (c >= 4 && j < L) {
      const int k = atomicAdd(&ncnt[r], 1);
      if (k < 4) atomicAnd(&npos[r], ~(0xFFu << (8 * k)) | ((uint32_t)j << (8 * k)));
    }
  }
  q2[r * q2_stride + w] = v;
}
__global__ void npos_finish(const int32_t *__restrict__ ncnt, int32_t nreads, uint32_t *__restrict__ npos) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < nreads && ncnt[r] > 4) npos[r] = kNOverflow;
}

// CP_OCC (one-hot planes, MSB = first row) -> Occ32 (2-bit codes, LSB = first row), one per block
__global__ void compress_occ(const CpOcc *__restrict__ occ, int64_t cp_size, Occ32 *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cp_size) return;
  const CpOcc &b = occ[i];
  uint64_t w[2] = {0, 0};
  for (int r = 0; r < 64; r++) {
    const int bit = 63 - r;
    const uint64_t code = ((b.one_hot_bwt_str[0] >> bit) & 1)   ? 0
                          : ((b.one_hot_bwt_str[1] >> bit) & 1) ? 1
                          : ((b.one_hot_bwt_str[2] >> bit) & 1) ? 2
                                                                 : 3;
    w[r >> 5] |= code << (2 * (r & 31));
  }
  Occ32 L;
  L.bwt[0] = w[0];
  L.bwt[1] = w[1];
  occ32_pack_counts(b.cp_count[0], b.cp_count[1], b.cp_count[2], L.cnt);
  out[i] = L;
}

enum State : int {
  NEXT_READ,
  OP_START,   // getSMEMsOnePosOneThread at x
  FWD_NEXT,   // forward extension loop
  FWD_END,
  BWD_ITER,   // backward search, one j
  BWD_P,      // ... one prev entry
  BWD_FINAL,
  OP_END,
  P2_NEXT,    // reseeding over this read's phase-1 SMEMs
  P3_X,       // LAST seeds
  P3_NEXT,
  FINISH,
  DONE,
};

struct SearchArgs {
  DevIndex F;
  const uint8_t *qdb;
  const uint32_t *q4;    // nibble-packed copy of qdb (8 bases per word), q4_stride words per read
  int32_t q4_stride;
  const uint32_t *q2;    // 2-bit copy of qdb (16 bases per word), q2_stride words per read (pack_q2)
  int32_t q2_stride;
  const uint32_t *npos;  // per read: its N positions (pack_npos)
  const int32_t *lens;
  int32_t nreads, stride, min_seed_len, split_len;
  PEnt *scratch;         // per wave: stride x 64 entries, wave-interleaved
  gb_smem *slots;        // per read: cap entries
  gb_smem *big;          // kMaxOvf promoted slots of kBigCap entries
  int32_t cap;
  const int32_t *list;   // pass 2: reads to redo (null in pass 1)
  const int32_t *list_n; // pass 2: number of reads in `list`
  int32_t *counts;       // per read: total SMEMs
  int32_t *phase;        // per read: num_smem1, num_smem2, num_smem3
  int32_t *next_read;    // work counter
  int32_t *ovf_list;     // promoted reads, by big-slot index
  int32_t *ovf_n;
  int32_t *fatal;        // pass 2 overflow / list overflow
  unsigned long long *bwt_calls;
  int32_t budget;        // a read still running after this many backwardExt calls is handed to the
                         // wave-cooperative pass (smem_heavy); INT32_MAX = never
  int32_t *heavy;        // reads handed over, (read, big slot or -1) pairs (capacity nreads), and their count
  int32_t *heavy_n;
  int32_t prefetch;      // claim the next read when taking one (GB_FMI_PREFETCH, default off)
  int32_t flags;         // GB_FMI_FLAGS probe switches: 4 = phase clocks into g_fmi_prof,
                         // 8 = per-read trace (start / end wall clock, backwardExt calls) into `trace`
  int64_t *trace;
};

// Diagnostic phase clocks (GB_FMI_FLAGS & 4): per-wave s_memtime sums of [state machine, gather
// wait, consume] and the trip count; read with gb_fmi_debug_prof().
__device__ unsigned long long g_fmi_prof[8];

__device__ __forceinline__ bool smem_less(const gb_smem &a, const gb_smem &b) {
  return a.m < b.m || (a.m == b.m && a.n > b.n);  // compare_smem, FMI_search.cpp:1499-1518
}

__device__ void heap_sort(gb_smem *a, int n) {
  auto sift = [&](int root, int end) {
    while (true) {
      int child = 2 * root + 1;
      if (child >= end) return;
      if (child + 1 < end && smem_less(a[child], a[child + 1])) child++;
      if (!smem_less(a[root], a[child])) return;
      const gb_smem t = a[root];
      a[root] = a[child];
      a[child] = t;
      root = child;
    }
  };
  for (int start = n / 2 - 1; start >= 0; start--) sift(start, n);
  for (int end = n - 1; end > 0; end--) {
    const gb_smem t = a[0];
    a[0] = a[end];
    a[end] = t;
    sift(0, end);
  }
}

// Reads up to kQBases bases are staged, 4 bits per base, in the lane's LDS row when the lane takes
// the read (one pass of dword loads from the nibble-packed copy d_q4), so the base lookups of the
// state machine are LDS reads instead of dependent global byte loads. Longer reads read d_qdb.
// 152 bases (the reference's 151-bp reads): 19 words per lane row, odd, so same-word reads are
// conflict-free, and with the 8 KB `prev` list head (kTop) a wave's LDS is 13 056 B, of which 12
// fit a CU's 160 KB (the grid runs 11 per CU, lanes_for_device)
constexpr int kQBases = 152;
constexpr int kQW = kQBases / 8;
static_assert(kQW % 2 == 1, "odd row stride (LDS banks)");
// kQ 2: the same reads staged at 2 bits per base (11 words per lane row, odd; 2.75 KB per wave
// instead of 4.75) with the read's N positions in one register (pack_npos): the 2 KB saved hold two
// more `prev` head entries at the same 16 waves per CU. A read with more than four N's reads its
// bases from qdb instead.
constexpr int kQW2 = 11;
static_assert(kQW2 * 16 >= kQBases && kQW2 % 2 == 1, "2-bit rows: every base, odd stride");
// kQ 3 (default): the first 128 bases' 2-bit codes in LDS (8 words, 2 KB per wave) and bases
// 128..159 in two registers, so eight head entries fit 16 waves per CU (10 KB). (64 bases in LDS and
// six registers for nine entries pushed the kernel past 128 VGPRs into scratch spills: 382 ms.)
constexpr int kQW3 = 8;
static_assert(kQW3 * 16 + 32 >= kQBases, "2-bit split rows: every base");

// kTop: the first entries of every `prev` list (list indices p < kTop, where the backward loop's
// reads and its in-place compaction concentrate as the lists shrink) live in LDS, the rest in the
// wave-interleaved scratch. List index p of a list whose forward phase pushed n entries is push
// k = n - 1 - p, kept in LDS slot k & (kTop - 1) = (c - p) & (kTop - 1) with c = n - 1: during the
// forward phase the slots hold the last kTop pushes (a push evicts the one kTop before it to its
// scratch position), and the compaction writes r'[q] into r[q]'s slot, already read. 8 KB per wave
// beside the 5.25 KB of staged read codes: 12 waves per CU still fit.
// slot of a ring of N entries (N a power of two: a mask; 6: an unsigned modulo, x >= 0)
template <int N>
__device__ __forceinline__ int ring_slot(int x) {
  if constexpr ((N & (N - 1)) == 0)
    return x & (N - 1);
  else
    return (int)((unsigned)x % (unsigned)N);
}

template <int kQ, int kTop>  // kQ: read codes 0 from qdb, 1 staged 4-bit, 2 staged 2-bit; kTop 0: every entry in the scratch
__global__ __launch_bounds__(64) void smem_search(SearchArgs A) {
  constexpr bool kTopLds = kTop > 0;
  constexpr bool kLdsQ = kQ > 0;
  constexpr int kRowW = kQ == 3 ? kQW3 : kQ == 2 ? kQW2 : kQW;
  __shared__ uint32_t Qs[kLdsQ ? 64 * kRowW : 1];
  __shared__ PEnt Ltop[kTopLds ? kTop * 64 : 1];
  const DevIndex F = A.F;
  const int gid = blockIdx.x * 64 + threadIdx.x;
  PList prev;
  prev.base = A.scratch + (size_t)(gid >> 6) * A.stride * 64 + (gid & 63);
  PEnt *const top = Ltop + (kTopLds ? threadIdx.x : 0);
  int tc = 0;  // c of the current list (kTopLds)
  uint32_t calls = 0, calls_read = 0;  // backwardExt calls (all reads / this read)

  int st = NEXT_READ;
  int rd = 0, L = 0, mode = 0, nslot = -1;
  const uint8_t *q = nullptr;
  uint32_t *const qrow = Qs + (kLdsQ ? threadIdx.x * kRowW : 0);
  uint32_t nw = 0xFFFFFFFFu;  // kQ 2 / 3: the read's N positions (pack_q2)
  uint32_t qh0 = 0, qh1 = 0;  // kQ 3: the code words of bases 128..143 and 144..159
  auto base_at = [&](int idx) -> int {
    if constexpr (kQ >= 2) {
      uint32_t w;
      if constexpr (kQ >= 3) {
        const uint32_t lw = qrow[min(idx >> 4, kRowW - 1)];
        w = idx < 16 * kQW3 ? lw : (idx < 16 * kQW3 + 16 ? qh0 : qh1);
      } else {
        w = qrow[idx >> 4];
      }
      const int c = (int)((w >> (2 * (idx & 15))) & 3u);
      // idx is an N position iff some byte of nw ^ (idx in every byte) is zero
      const uint32_t x = nw ^ __builtin_amdgcn_perm(0u, (uint32_t)idx, 0u);
      return ((x - 0x01010101u) & ~x & 0x80808080u) ? 4 : c;
    } else if constexpr (kQ == 1) {
      return (int)((qrow[idx >> 3] >> (4 * (idx & 7))) & 15u);
    } else {
      return q[idx];
    }
  };
  gb_smem *o = nullptr;
  int nout = 0, n1 = 0, n2 = 0, ridx = 0;
  bool ovf = false;
  int x = 0, min_intv = 1, j = 0, next_x = 0, numPrev = 0, numCurr = 0, p = 0, curr_s = -1, a = 0;
  bool first = true;
  int64_t ck = 0, cl = 0, cs = 0;  // current SMEM of a forward extension
  uint32_t cm = 0;
  int r0 = 0;                      // reversed prev list: r[p] = prev[r0 + p] (r[0] = last pushed)
  PEnt cur{};                      // the prev entry of the pending BWD_P request (packed)
  // r[0] of the current list in registers, and r[p+1] loaded while r[p]'s backwardExt is in
  // flight: the backward loop never waits on a scratch read before its gather. (Entries are
  // compacted in place behind the read position, so a prefetched entry is never overwritten
  // before it is used.)
  PEnt head{};
  // forward push of e (push index k = numPrev): scratch position L - 1 - k, or with kTopLds the LDS
  // ring of the last kTop pushes
  auto push_fwd = [&](const Ent &e) {
    const PEnt pe = pack_ent(e);
    if constexpr (kTopLds) {
      const int k = numPrev;
      PEnt *slot = top + (size_t)ring_slot<kTop>(k) * 64;
      if (k >= kTop) prev.base[(size_t)(L - 1 - (k - kTop)) * 64] = *slot;
      *slot = pe;
    } else {
      prev.base[(size_t)(L - 1 - numPrev) * 64] = pe;
    }
    numPrev++;
    head = pe;
  };
  // list index p of the current reversed list (p >= 1; r[0] is `head`)
  auto get_r = [&](int p_) -> PEnt {
    if constexpr (kTopLds)
      if (p_ < kTop) return top[(size_t)ring_slot<kTop>(tc - p_) * 64];
    return prev.base[(size_t)(r0 + p_) * 64];
  };
  auto put_r = [&](int q_, const PEnt &pe) {
    if constexpr (kTopLds)
      if (q_ < kTop) {
        top[(size_t)ring_slot<kTop>(tc - q_) * 64] = pe;
        return;
      }
    prev.base[(size_t)(r0 + q_) * 64] = pe;
  };

  int cap = A.cap;  // slots of the current output area (kCap, or kBigCap once promoted)
  int kb_cur = -1;  // the big slot of the current read, if promoted
  auto emit = [&](int64_t k, int64_t l, int64_t s, uint32_t m, uint32_t n) {
    if (nout == cap && cap == kCap) {
      // promote the read to a big slot (first pass only, rare): copy what it has and carry on there
      const int kb = atomicAdd(A.ovf_n, 1);
      if (kb < kMaxOvf) {
        gb_smem *big = A.big + (size_t)kb * kBigCap;
        for (int t = 0; t < kCap; t++) big[t] = o[t];
        o = big;
        cap = kBigCap;
        kb_cur = kb;
        A.ovf_list[kb] = rd;
      }
    }
    if (nout < cap) {
      gb_smem e{};  // zeroed: the 4 padding bytes after n are part of the output records
      e.rid = (uint32_t)rd;
      e.m = m;
      e.n = n;
      e.k = k;
      e.l = l;
      e.s = s;
      o[nout] = e;
    } else {
      ovf = true;
    }
    nout++;
  };

  const bool prof = A.flags & 4;
  int64_t t_read = 0;
  unsigned long long p_sm = 0, p_mem = 0, p_cons = 0, p_trips = 0, p_iter = 0, p_nr_trips = 0, p_nr_clk = 0;
  // next backwardExt request; `pend` = already prepared by the previous consume step (the common
  // continuation of a forward, backward or LAST extension), which skips the state machine
  int64_t rk = 0, rl = 0, rs = 0;
  int rb = 0;
  bool pend = false;
  while (true) {
    const unsigned long long tA = prof ? clock64() : 0;
    if (calls_read >= (uint32_t)A.budget && st != NEXT_READ && st != DONE) {
      // a heavy read (a few per thousand, up to ~25x the median's backwardExt calls in repeats)
      // would hold its wave, and at the end of the grid the whole step, for its full length: drop
      // what it did (its calls are not counted, a big slot it took is released) and hand it to
      // smem_heavy, which spreads each backward step's independent extensions over a wave
      // (a big slot it took goes with it: smem_heavy promotes the read into that same slot, so a
      // handed-over read never holds two of the kMaxOvf slots)
      if (kb_cur >= 0) A.ovf_list[kb_cur] = -1;
      const int h = atomicAdd(A.heavy_n, 1);
      A.heavy[2 * h] = rd;
      A.heavy[2 * h + 1] = kb_cur;
      pend = false;
      st = NEXT_READ;
    }
    // ---- advance this lane's state machine to its next backwardExt request --------------------
    bool req = pend;
    pend = false;
    bool took_read = false;
    while (!req && st != DONE) {
      if (prof) p_iter++;
      if (st == NEXT_READ) took_read = true;
      switch (st) {
        case NEXT_READ: {
          // the slot of the following read is taken now and arrives while this read runs
          const int slot = nslot >= 0 ? nslot : atomicAdd(A.next_read, 1);
          if (slot >= (A.list ? *A.list_n : A.nreads)) {
            st = DONE;
            break;
          }
          // prefetch: claim the following read now so its atomic's latency hides behind this read;
          // but a claimed read waits behind the current one, which lengthens the grid's tail
          if (A.prefetch) nslot = atomicAdd(A.next_read, 1);
          rd = A.list ? A.list[slot] : slot;
          q = A.qdb + (size_t)rd * A.stride;
          if constexpr (kQ >= 2) {
            nw = A.npos[rd];
            if (nw == kNOverflow) {
              // more than four N's: the read goes to smem_heavy (which reads qdb) before it starts,
              // so the lookups here need no byte-load path
              const int h = atomicAdd(A.heavy_n, 1);
              A.heavy[2 * h] = rd;
              A.heavy[2 * h + 1] = -1;
              break;  // st stays NEXT_READ
            }
          }
          // L is loaded after that branch: loaded before it, the hand-over path left the load
          // outstanding as far as the compiler's wait analysis could tell, and every later use of L
          // in the state machine got a vmcnt(0) wait -- which also waited for the trip's stores
          L = A.lens[rd];
          if constexpr (kQ >= 3) {
            // words 0..7 to the LDS row, 8 and 9 to registers (q2_stride covers every word of the
            // longest read; a word past the read is never looked at)
            const uint4 *src = reinterpret_cast<const uint4 *>(A.q2 + (size_t)rd * A.q2_stride);
            const int n4 = (L + 63) >> 6;
            const uint4 v0 = src[0];
            const uint4 v1 = n4 > 1 ? src[1] : make_uint4(0, 0, 0, 0);
            const uint4 v2 = n4 > 2 ? src[2] : make_uint4(0, 0, 0, 0);
            qrow[0] = v0.x;
            qrow[1] = v0.y;
            qrow[2] = v0.z;
            qrow[3] = v0.w;
            qrow[4] = v1.x;
            qrow[5] = v1.y;
            qrow[6] = v1.z;
            qrow[7] = v1.w;
            qh0 = v2.x;
            qh1 = v2.y;
          } else if constexpr (kQ == 2) {
            // rows are q2_stride (a multiple of 4) words: all 16-byte loads issue together
            const uint4 *src = reinterpret_cast<const uint4 *>(A.q2 + (size_t)rd * A.q2_stride);
            const int n4 = (L + 63) >> 6;
            for (int w = 0; w < n4; w++) {
              const uint4 v = src[w];
              if (4 * w < kQW2) qrow[4 * w] = v.x;
              if (4 * w + 1 < kQW2) qrow[4 * w + 1] = v.y;
              if (4 * w + 2 < kQW2) qrow[4 * w + 2] = v.z;
              if (4 * w + 3 < kQW2) qrow[4 * w + 3] = v.w;
            }
          } else if constexpr (kQ == 1) {
            // rows are q4_stride (a multiple of 4) words: all 16-byte loads issue together
            const uint4 *src = reinterpret_cast<const uint4 *>(A.q4 + (size_t)rd * A.q4_stride);
            const int n4 = (L + 31) >> 5;
            for (int w = 0; w < n4; w++) {
              const uint4 v = src[w];
              // the row holds kQW words: the last 16-byte chunk's words past it are beyond the read
              if (4 * w < kQW) qrow[4 * w] = v.x;
              if (4 * w + 1 < kQW) qrow[4 * w + 1] = v.y;
              if (4 * w + 2 < kQW) qrow[4 * w + 2] = v.z;
              if (4 * w + 3 < kQW) qrow[4 * w + 3] = v.w;
            }
          }
          o = A.slots + (size_t)slot * A.cap;
          if (A.flags & 8) t_read = (int64_t)wall_clock64();
          cap = A.cap;
          kb_cur = -1;
          nout = 0;
          ovf = false;
          calls_read = 0;
          mode = 1;
          x = 0;
          min_intv = 1;
          st = OP_START;
          break;
        }
        case OP_START:
          if (mode == 1 && x >= L) {  // getSMEMsAllPosOneThread done: reseed next
            n1 = nout;
            ridx = 0;
            mode = 2;
            st = P2_NEXT;
            break;
          }
          next_x = x + 1;
          a = base_at(x);
          if (a >= 4) {
            st = OP_END;
            break;
          }
          ck = count_of(F, a);
          cl = count_of(F, 3 - a);
          cs = count_of(F, a + 1) - ck;
          cm = (uint32_t)x;
          numPrev = 0;
          j = x + 1;
          st = FWD_NEXT;
          break;
        case FWD_NEXT:
          if (j >= L) {
            st = FWD_END;
            break;
          }
          next_x = j + 1;
          a = base_at(j);
          if (a >= 4) {
            st = FWD_END;
            break;
          }
          // forward extension = backward extension on the reverse complement (k <-> l, 3 - a)
          rk = cl;
          rl = ck;
          rs = cs;
          rb = 3 - a;
          req = true;
          break;
        case FWD_END:
          if (cs >= min_intv) {
            Ent e;
            e.k = ck; e.l = cl; e.s = cs; e.m = cm; e.n = (uint32_t)(j - 1);  // current n = j-1
            push_fwd(e);
          }
          r0 = L - numPrev;
          tc = numPrev - 1;
          j = x - 1;
          st = BWD_ITER;
          break;
        case BWD_ITER:
          if (j < 0) {
            st = BWD_FINAL;
            break;
          }
          a = base_at(j);
          if (a > 3) {
            st = BWD_FINAL;
            break;
          }
          numCurr = 0;
          curr_s = -1;
          first = true;
          p = 0;
          st = BWD_P;
          break;
        case BWD_P:
          if (p >= numPrev) {
            numPrev = numCurr;
            if (numCurr == 0) {
              st = OP_END;
            } else {
              j--;
              st = BWD_ITER;
            }
            break;
          }
          cur = p == 0 ? head : get_r(p);
          {
            const Ent ce = unpack_ent(cur);
            rk = ce.k;
            rl = ce.l;
            rs = ce.s;
          }
          rb = a;
          req = true;
          break;
        case BWD_FINAL:
          if (numPrev != 0) {
            const Ent e = unpack_ent(head);  // r[0]
            if ((e.n - e.m + 1) >= (uint32_t)A.min_seed_len) emit(e.k, e.l, e.s, e.m, e.n);
          }
          st = OP_END;
          break;
        case OP_END:
          if (mode == 1) {
            x = next_x;
            st = OP_START;
          } else {
            ridx++;
            st = P2_NEXT;
          }
          break;
        case P2_NEXT: {
          // fmi.cpp:293-302: SMEMs of length >= split_len with s <= splitWidth(10) restart at
          // the midpoint with min_intv = s + 1
          bool found = false;
          while (ridx < n1 && ridx < cap) {
            const gb_smem e = o[ridx];
            const int start = (int)e.m, end = (int)e.n + 1;
            if (!(end - start < A.split_len || e.s > 10)) {
              x = (end + start) >> 1;
              min_intv = (int)(e.s + 1);
              found = true;
              break;
            }
            ridx++;
          }
          if (found) {
            st = OP_START;
          } else {
            n2 = nout - n1;
            mode = 3;
            x = 0;
            st = P3_X;
          }
          break;
        }
        case P3_X:
          if (x >= L) {
            st = FINISH;
            break;
          }
          next_x = x + 1;
          a = base_at(x);
          if (a >= 4) {
            x = next_x;
            break;
          }
          ck = count_of(F, a);
          cl = count_of(F, 3 - a);
          cs = count_of(F, a + 1) - ck;
          cm = (uint32_t)x;
          j = x + 1;
          st = P3_NEXT;
          break;
        case P3_NEXT:
          if (j >= L) {
            x = next_x;
            st = P3_X;
            break;
          }
          next_x = j + 1;
          a = base_at(j);
          if (a >= 4) {
            x = next_x;
            st = P3_X;
            break;
          }
          rk = cl;
          rl = ck;
          rs = cs;
          rb = 3 - a;
          req = true;
          break;
        case FINISH: {
          // the slot is sorted by (m asc, n desc) afterwards by sort_slots (an in-place sort here
          // would be a chain of dependent global loads that stalls the whole wave)
          A.counts[rd] = nout;
          A.phase[3 * rd + 0] = n1;
          A.phase[3 * rd + 1] = n2;
          A.phase[3 * rd + 2] = nout - n1 - n2;
          calls += calls_read;
          if (A.flags & 8) {
            A.trace[3 * (size_t)rd] = t_read;
            A.trace[3 * (size_t)rd + 1] = (int64_t)wall_clock64();
            A.trace[3 * (size_t)rd + 2] = calls_read;
          }
          if (ovf) atomicAdd(A.fatal, 1);  // more than kBigCap SMEMs, or the big-slot pool was exhausted
          st = NEXT_READ;
          break;
        }
        default:
          st = DONE;
          break;
      }
    }
    if (st == DONE) break;

    // ---- one backwardExt per lane per trip --------------------------------------------------
    int64_t ko, lo, so;
    const unsigned long long tB = prof ? clock64() : 0;
    bwt_ext(F, rk, rl, rs, rb, ko, lo, so);
    calls_read++;
    unsigned long long tC = 0;
    if (prof) {
      asm volatile("" ::"v"(ko), "v"(lo), "v"(so));
      tC = clock64();
    }

    // ---- consume ------------------------------------------------------------------------------
    if (st == FWD_NEXT) {
      // newSmem = swap(result); n = j (FMI_search.cpp:1044-1056)
      const int64_t nk = lo, nl = ko, ns = so;
      if (ns != cs) {  // push the current SMEM (prevArray[numPrev] = smem; numPrev += s_neq)
        Ent e;
        e.k = ck; e.l = cl; e.s = cs; e.m = cm; e.n = (uint32_t)(j - 1);
        push_fwd(e);
      }
      if (ns < min_intv) {
        next_x = j;
        st = FWD_END;
      } else {
        ck = nk;
        cl = nl;
        cs = ns;
        j++;
        if (j < L) {  // FWD_NEXT's request for the next base, inline
          const int na = base_at(j);
          if (na < 4) {
            next_x = j + 1;
            a = na;
            rk = cl;
            rl = ck;
            rs = cs;
            rb = 3 - na;
            pend = true;
          }
        }
      }
    } else if (st == BWD_P) {
      const Ent e = unpack_ent(cur);
      if (first) {
        if (so < min_intv && (e.n - e.m + 1) >= (uint32_t)A.min_seed_len) {
          emit(e.k, e.l, e.s, e.m, e.n);
          first = false;
        } else if (so >= min_intv && so != (int64_t)curr_s) {
          curr_s = (int)so;
          Ent ne;
          ne.k = ko; ne.l = lo; ne.s = so; ne.m = (uint32_t)j; ne.n = e.n;
          const PEnt pne = pack_ent(ne);
          if (numCurr == 0) head = pne;  // r[0] of the next j
          put_r(numCurr++, pne);
          first = false;
        }
      } else if (so >= min_intv && so != (int64_t)curr_s) {
        curr_s = (int)so;
        Ent ne;
        ne.k = ko; ne.l = lo; ne.s = so; ne.m = (uint32_t)j; ne.n = e.n;
        const PEnt pne = pack_ent(ne);
        if (numCurr == 0) head = pne;
        put_r(numCurr++, pne);
      }
      p++;
      if (p < numPrev) {  // BWD_P's request for the next list entry, inline
        cur = get_r(p);
        const Ent ce = unpack_ent(cur);
        rk = ce.k;
        rl = ce.l;
        rs = ce.s;
        rb = a;
        pend = true;
      }
    } else {  // P3_NEXT (bwtSeedStrategyAllPosOneThread)
      ck = lo;
      cl = ko;
      cs = so;
      if (cs < 20 && (uint32_t)(j - (int)cm + 1) >= (uint32_t)(A.min_seed_len + 1)) {
        if (cs > 0) emit(ck, cl, cs, cm, (uint32_t)j);
        x = j + 1;
        st = P3_X;
      } else {
        j++;
        if (j < L) {  // P3_NEXT's request for the next base, inline
          const int na = base_at(j);
          if (na < 4) {
            next_x = j + 1;
            a = na;
            rk = cl;
            rl = ck;
            rs = cs;
            rb = 3 - na;
            pend = true;
          }
        }
      }
    }
    if (prof) {
      const unsigned long long tD = clock64();
      p_sm += tB - tA;
      p_mem += tC - tB;
      p_cons += tD - tC;
      p_trips++;
      if (__ballot(took_read)) {
        p_nr_trips++;
        p_nr_clk += tB - tA;
      }
    }
  }
  atomicAdd(A.bwt_calls, (unsigned long long)calls);
  if (prof && (threadIdx.x & 63) == 0) {
    atomicAdd(&g_fmi_prof[0], p_sm);
    atomicAdd(&g_fmi_prof[1], p_mem);
    atomicAdd(&g_fmi_prof[2], p_cons);
    atomicAdd(&g_fmi_prof[3], p_trips);
    atomicAdd(&g_fmi_prof[5], p_nr_trips);
    atomicAdd(&g_fmi_prof[6], p_nr_clk);
  }
  if (prof) {
    // while-loop iterations: max over lanes per trip ~ wave iterations; sum of lane iterations here
    atomicAdd(&g_fmi_prof[4], p_iter);
  }
}

// ---- heavy reads: one wave per read ------------------------------------------------------------
// In a repeat a read's `prev` lists grow long and its backward search makes numPrev extensions per
// position j (FMI_search.cpp:1103-1160): a few reads per thousand make 2.5-25x the median's calls.
// Those extensions are independent of each other -- only the bookkeeping after them is sequential
// -- so here a wave takes one read: the forward and LAST extensions run wave-uniform (every lane
// computes the same one), each backward step extends up to 64 list entries at once, and the
// reference's sequential scan over the results becomes ballots:
//   * the first loop stops at the first entry f with s' >= min_intv (push) or with s' < min_intv and
//     a long enough SMEM (emit it);
//   * from f on, an entry with s' >= min_intv is pushed iff its s' differs from curr_s, the s' of
//     the last push -- which is always the s' of the previous entry with s' >= min_intv (an entry
//     not pushed had the same s' as that push), so the test is against the nearest lower such lane.
// The lists live in LDS (reads up to kHeavyMaxLen bases). Per read the SMEM set, the per-phase
// counts and the backwardExt count are the lane kernel's; only the order inside the read's slot
// differs, which sort_slots makes canonical (equal (m, n) keys are identical SMEMs).
// Measured and dropped in round 3 (r03o-r03w, same-box A/B against this version): resuming a
// handed-over read from its last position boundary instead of from scratch, with a list-length
// trigger; the search's own waves taking handed-over reads once their lanes were done (each XCD has
// its own L2, not coherent with the others inside a kernel, so the records had to stay per XCD); and
// handing over ordinary reads in the grid's tail. The extra state in the lane loop cost more
// (3-12 %) than the post-pass time they saved.
constexpr int kHeavyMaxLen = 256;
constexpr int kHeavyBudget = 2000;  // backwardExt calls before a lane hands its read over

struct HeavyArgs {
  DevIndex F;
  const uint8_t *qdb;
  const int32_t *lens;
  int32_t stride, min_seed_len, split_len;
  const int32_t *heavy;
  const int32_t *heavy_n;
  gb_smem *slots;  // kCap per read
  gb_smem *big;
  int32_t *counts, *phase, *ovf_list, *ovf_n, *fatal;
  unsigned long long *bwt_calls;
  int64_t *trace;  // GB_FMI_FLAGS & 8 (as SearchArgs::trace), or null
};

__global__ __launch_bounds__(64) void smem_heavy(HeavyArgs A) {
  __shared__ PEnt La[kHeavyMaxLen + 1], Lb[kHeavyMaxLen + 1];
  __shared__ uint8_t Q[kHeavyMaxLen];
  const DevIndex F = A.F;
  const int lane = threadIdx.x;
  const int nh = *(volatile const int32_t *)A.heavy_n;
  for (int t = blockIdx.x; t < nh; t += gridDim.x) {
    const int rd = A.heavy[2 * t];
    const int kb_pre = A.heavy[2 * t + 1];  // the big slot the lane kernel had promoted it to, or -1
    const int L = A.lens[rd];
    const int64_t t_read = A.trace ? (int64_t)wall_clock64() : 0;
    for (int i = lane; i < L; i += 64) Q[i] = A.qdb[(size_t)rd * A.stride + i];
    __syncthreads();
    // ---- output slot (lane 0 writes; every lane keeps the same counters) ----------------------
    gb_smem *o = A.slots + (size_t)rd * kCap;
    int cap = kCap, nout = 0;
    bool ovf = false;
    uint32_t calls = 0;
    // wave-uniform: o, cap and nout are the same in every lane (the reseed loop below reads them)
    auto emit = [&](int64_t k, int64_t l, int64_t s, uint32_t m, uint32_t n) {
      if (nout == cap && cap == kCap) {
        int kb = kb_pre;
        if (kb < 0) {
          if (lane == 0) kb = atomicAdd(A.ovf_n, 1);
          kb = __shfl(kb, 0);
        }
        if (kb < kMaxOvf) {
          gb_smem *big = A.big + (size_t)kb * kBigCap;
          if (lane == 0) {
            for (int i = 0; i < kCap; i++) big[i] = o[i];
            A.ovf_list[kb] = rd;
          }
          o = big;
          cap = kBigCap;
        }
      }
      if (nout < cap) {
        if (lane == 0) {
          gb_smem e{};  // zeroed: the 4 padding bytes after n are part of the output records
          e.rid = (uint32_t)rd;
          e.m = m;
          e.n = n;
          e.k = k;
          e.l = l;
          e.s = s;
          o[nout] = e;
        }
      } else {
        ovf = true;
      }
      nout++;
    };

    uint32_t *const calls_p = &calls;
    auto one_pos = [&](int x, int min_intv) -> int {
      return wave_one_pos(F, Q, L, x, min_intv, A.min_seed_len, La, Lb, lane, *calls_p, emit);
    };

    // getSMEMsAllPosOneThread (min_intv 1)
    for (int x = 0; x < L;) x = one_pos(x, 1);
    const int n1 = nout;
    // reseeding (fmi.cpp:293-302) over this read's phase-1 SMEMs
    for (int ridx = 0; ridx < n1 && ridx < cap; ridx++) {
      int mm = 0, nn = 0, ss = 0;
      if (lane == 0) {
        const gb_smem e = o[ridx];
        mm = (int)e.m;
        nn = (int)e.n;
        ss = (int)min<int64_t>(e.s, 1 << 30);
      }
      mm = __shfl(mm, 0);
      nn = __shfl(nn, 0);
      ss = __shfl(ss, 0);
      const int start = mm, end = nn + 1;
      if (!(end - start < A.split_len || ss > 10)) one_pos((end + start) >> 1, ss + 1);
    }
    const int n2 = nout - n1;
    // bwtSeedStrategyAllPosOneThread (FMI_search.cpp:1243-1326), max_intv 20
    wave_last_seeds(F, Q, L, 20, A.min_seed_len + 1, calls, emit);  // fmi.cpp passes minSeedLen + 1
    if (lane == 0) {
      A.counts[rd] = nout;
      A.phase[3 * rd + 0] = n1;
      A.phase[3 * rd + 1] = n2;
      A.phase[3 * rd + 2] = nout - n1 - n2;
      atomicAdd(A.bwt_calls, (unsigned long long)calls);
      if (ovf) atomicAdd(A.fatal, 1);
      if (A.trace) {
        A.trace[3 * (size_t)rd] = t_read;
        A.trace[3 * (size_t)rd + 1] = (int64_t)wall_clock64();
        A.trace[3 * (size_t)rd + 2] = -(int64_t)calls;  // negative: done by smem_heavy
      }
    }
    __syncthreads();
  }
}

// Reads with count <= kCap are in their pass-1 slot; the rest in the pass-2 slot at the position of
// the read in the overflow list (ovf_pos, filled by mark_overflow).
__global__ void mark_overflow(const int32_t *__restrict__ ovf_list, const int32_t *__restrict__ ovf_n,
                              int32_t *__restrict__ ovf_pos) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = min(*ovf_n, kMaxOvf);
  if (t < n && ovf_list[t] >= 0) ovf_pos[ovf_list[t]] = t;  // -1: released by a read handed to smem_heavy
}

// Sort every read's slot by (m asc, n desc) (sortSMEMs / compare_smem, FMI_search.cpp:1499-1534).
// Keys: m << 13 | (8191 - n) (m, n < 2^13, checked on the host; equal keys are identical SMEMs).
// A wave takes four reads at a time, 16 lanes each: the counts and the first 16 entries of the four
// slots are loaded together (one memory round trip; a slot holds kCap >= 16), and a lane's rank is
// the number of smaller (key, lane) pairs in its row of 16, rotated past it with DPP. Reads with
// 17 .. kCap SMEMs are ranked by the whole wave from readlane broadcasts, promoted reads (> kCap)
// heap-sorted by one lane.
template <int R>
__device__ __forceinline__ int rank_row(uint32_t kk) {
  const int rot = __builtin_amdgcn_mov_dpp((int)kk, 0x120 + R, 0xf, 0xf, false);  // row_ror:R
  return ((uint32_t)rot < kk ? 1 : 0) + rank_row<R - 1>(kk);
}
template <>
__device__ __forceinline__ int rank_row<0>(uint32_t) {
  return 0;
}
static_assert(kCap >= 16, "the first 16 entries of a slot are loaded unconditionally");

__global__ __launch_bounds__(256) void sort_slots(gb_smem *__restrict__ slots, gb_smem *__restrict__ big,
                                                  const int32_t *__restrict__ ovf_pos,
                                                  const int32_t *__restrict__ counts, int32_t nreads) {
  const int lane = threadIdx.x & 63, g = lane >> 4, sl = lane & 15;
  const int nwaves = gridDim.x * (blockDim.x >> 6);
  for (int base = 4 * ((blockIdx.x * blockDim.x + threadIdx.x) >> 6); base < nreads; base += 4 * nwaves) {
    const int rd = min(base + g, nreads - 1);
    const int n = base + g < nreads ? counts[rd] : 0;
    gb_smem *src = slots + (size_t)rd * kCap;
    const gb_smem e = src[sl];
    const bool mine = n > 1 && n <= 16 && sl < n;
    const uint32_t kk = mine ? ((((e.m << 13) | (8191u - e.n)) << 4) | (uint32_t)sl) : 0xffffffffu;
    const int rank = rank_row<15>(kk);
    if (mine) src[rank] = e;
    // the reads with more than 16 SMEMs, one at a time
    uint64_t wide = __ballot(sl == 0 && n > 16);
    while (wide) {
      const int gl = __builtin_ctzll(wide);
      wide &= wide - 1;
      const int rw = base + (gl >> 4);
      const int nw = __builtin_amdgcn_readlane(n, gl);
      if (nw <= kCap) {
        gb_smem *sw = slots + (size_t)rw * kCap;
        gb_smem ew{};
        uint32_t key = 0xffffffffu;
        if (lane < nw) {
          ew = sw[lane];
          key = (ew.m << 13) | (8191u - ew.n);
        }
        int rk = 0;
        for (int j = 0; j < nw; j++) {
          const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)key, j);
          rk += (kj < key || (kj == key && j < lane)) ? 1 : 0;
        }
        if (lane < nw) sw[rk] = ew;
      } else if (lane == 0) {
        heap_sort(big + (size_t)ovf_pos[rw] * kBigCap, min(nw, kBigCap));
      }
    }
  }
}

__global__ void scatter_smems(const gb_smem *__restrict__ slots, const gb_smem *__restrict__ big,
                              const int32_t *__restrict__ ovf_pos, const int32_t *__restrict__ counts,
                              const int64_t *__restrict__ offsets, gb_smem *__restrict__ out,
                              int32_t nreads) {
  const int rd = blockIdx.x * blockDim.x + threadIdx.x;
  if (rd >= nreads) return;
  const int n = counts[rd];
  const int64_t o = offsets[rd];
  const gb_smem *src = n <= kCap ? slots + (size_t)rd * kCap : big + (size_t)ovf_pos[rd] * kBigCap;
  for (int i = 0; i < n; i++) out[o + i] = src[i];
}

}  // namespace gbfmi

// ---------------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------------
struct gb_fmi_reads {
  gb_fmi_index *idx = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  int32_t nreads = 0, stride = 0;
  int lanes = 0;  // resident lanes of the persistent search grid
  int cus = 256;
  uint8_t *d_qdb = nullptr;
  uint32_t *d_q4 = nullptr;
  int32_t q4_stride = 0;
  uint32_t *d_q2 = nullptr;    // 2-bit codes (smem_search<2, ...>)
  int32_t q2_stride = 0;
  uint32_t *d_npos = nullptr;  // per read: N positions
  int32_t *d_lens = nullptr;
  gbfmi::PEnt *d_scratch = nullptr;
  gb_smem *d_slots = nullptr;
  int32_t *d_counts = nullptr;
  int32_t *d_phase = nullptr;
  int64_t *d_offsets = nullptr;
  gb_smem *d_out = nullptr;
  int64_t out_cap = 0;
  int32_t *d_ctl = nullptr;  // [0] next_read, [1] overflow count, [2] fatal, [3] unused, [4] heavy reads
  int32_t *d_heavy = nullptr;  // reads handed to smem_heavy (capacity nreads)
  int32_t *d_ovf_list = nullptr;
  int32_t *d_ovf_pos = nullptr;
  gb_smem *d_big = nullptr;
  unsigned long long *d_calls = nullptr;
  void *d_temp = nullptr;
  size_t temp_bytes = 0;
  bool ran = false;
  bool complete = false;   // every buffer allocated: only such a read set is recycled on destroy
  bool scattered = false;  // d_out holds the last search's compacted SMEMs
  int64_t total = 0;
  gbfmi::SaJob *sa = nullptr;
  int64_t *d_trace = nullptr;  // GB_FMI_FLAGS & 8 diagnostic (3 x nreads), allocated on demand
  size_t cap_trace = 0;
  // grow-only capacities (bytes): a destroyed read set goes back to its thread's free list with its
  // stream and buffers, and the next create reuses them (no hipMalloc / hipFree per batch)
  int device = -1;
  size_t cap_q2 = 0, cap_npos = 0;
  size_t cap_qdb = 0, cap_q4 = 0, cap_lens = 0, cap_scratch = 0, cap_slots = 0, cap_ovf_pos = 0, cap_counts = 0,
         cap_phase = 0, cap_offsets = 0, cap_temp = 0, cap_heavy = 0;
};

namespace {

int device_cus() {
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  return cus;
}

// read codes staged at 2 bits per base: by default the split rows of smem_search<3, ...>
// (GB_FMI_Q2=3); GB_FMI_Q2=1: whole 11-word rows (smem_search<2, ...>); 0: 4 bits, the round-5 form
bool q2_codes() {
  const char *e = getenv("GB_FMI_Q2");
  return !(e && *e == '0');
}
bool q3_codes() {
  const char *e = getenv("GB_FMI_Q2");
  return !e || !*e || *e == '3';
}

// `prev` list head entries kept in LDS (GB_FMI_TOP: 0, 4-8). With 4-bit codes five (9.9 KB per wave,
// 16 waves per CU still fit): 10 M reads 243.9 -> 232.7 ms, the 1/8 shard 35.2 -> 34.0 ms against
// four; six at 14 / 15 waves 233.8, seven at 13 249.7, eight at 11 259.6 (profiles/r05zi_fmi_top.log).
// With 2-bit codes (2.75 KB) seven fit at 16 waves (9.75 KB, five 2-KB granules); with the split rows
// (2 KB) eight (10 KB): 10 M reads 227.3 -> 222.0 ms (profiles/r06zt_fmi_split_rows_ab.log).
int top_entries() {
  const char *te = getenv("GB_FMI_TOP");
  return te ? atoi(te) : (q3_codes() ? 8 : q2_codes() ? 7 : 5);
}

int lanes_for_device(int cus) {
  const char *e = getenv("GB_FMI_WAVES_PER_CU");
  if (q2_codes() && !e) {
    // 2-bit codes: LDS per wave 2 816 B + 1 KB per head entry, allocated in 2 KB granules; 16 waves
    // per CU at most (116 VGPRs)
    const int lds = 64 * 4 * (q3_codes() ? gbfmi::kQW3 : gbfmi::kQW2) + 1024 * top_entries();
    const int gran = (lds + 2047) / 2048 * 2048;
    return cus * std::max(1, std::min(16, 160 * 1024 / gran)) * 64;
  }
  // Waves (workgroups) per CU of the persistent grid. LDS per wave is the staged read codes (4.9 KB)
  // plus the `prev` list head (1 KB per entry kept); 116 VGPRs allow 4 waves per SIMD. With an
  // 8-entry head (13 KB) 12 fit and 11 / 12 run alike; a 4- or 5-entry head (8.9 / 9.9 KB) lets the
  // VGPR limit, 16, bind, which hides more gather latency than extra LDS entries save (round 4: 10 M
  // reads 248 vs 260 ms at 4 / 8 entries, profiles/r04e_fmi_knobs.log; round 5: top_entries).
  const int top = top_entries();
  const int waves = e ? std::max(1, atoi(e)) : (top >= 8 ? 11 : top >= 7 ? 13 : top >= 6 ? 14 : 16);
  return cus * waves * 64;
}

}  // namespace

namespace gbfmi {

int ensure_occ32(gb_fmi_index *ix, hipStream_t s) {
  if (ix->d_occ32) return GB_OK;
  GB_ARG(ix->n < (1ll << 34), "FM index too large for 34-bit Occ32 counts (%lld rows)", (long long)ix->n);
  GB_HIP(hipMalloc(&ix->d_occ32, sizeof(Occ32) * (size_t)ix->cp_size));
  hipLaunchKernelGGL(compress_occ, dim3((unsigned)((ix->cp_size + 255) / 256)), dim3(256), 0, s, ix->d_occ,
                     ix->cp_size, ix->d_occ32);
  GB_HIP(hipGetLastError());
  GB_HIP(hipStreamSynchronize(s));  // other read sets of this index may use other streams
  return GB_OK;
}

hipStream_t reads_stream(gb_fmi_reads *R) { return R->stream; }
gb_fmi_index *reads_index(gb_fmi_reads *R) { return R->idx; }
SaJob **reads_sa_job(gb_fmi_reads *R) { return &R->sa; }

namespace {
int check_fatal(gb_fmi_reads *R, const char *who) {
  int32_t ctl[4];
  GB_HIP(hipMemcpy(ctl, R->d_ctl, sizeof(ctl), hipMemcpyDeviceToHost));
  if (ctl[2] != 0) {
    gb::set_error("%s: %d reads exceeded %d SMEM slots (or more than %d reads exceeded %d)", who, ctl[2], kBigCap,
                  kMaxOvf, kCap);
    return GB_ERR_STATE;
  }
  return GB_OK;
}

// Compact the slots into d_out (exclusive scan already in d_offsets); tot = total SMEMs.
int scatter_out(gb_fmi_reads *R, int64_t tot) {
  if (!R->scattered) {
    if (tot > R->out_cap) {
      (void)hipFree(R->d_out);
      R->d_out = nullptr;
      GB_HIP(hipMalloc(&R->d_out, sizeof(gb_smem) * (size_t)tot));
      R->out_cap = tot;
    }
    if (tot) {
      hipLaunchKernelGGL(scatter_smems, dim3((R->nreads + 255) / 256), dim3(256), 0, R->stream, R->d_slots, R->d_big,
                         R->d_ovf_pos, R->d_counts, R->d_offsets, R->d_out, R->nreads);
      GB_HIP(hipGetLastError());
    }
    R->scattered = true;
    R->total = tot;
  }
  return GB_OK;
}
}  // namespace

int reads_device_smems(gb_fmi_reads *R, const gb_smem **d_smems, int64_t *n) {
  GB_ARG(R && R->ran, "SA lookup: the read set has not been searched");
  GB_HIP(hipSetDevice(R->idx->device));
  GB_HIP(hipStreamSynchronize(R->stream));
  int st = check_fatal(R, "SA lookup");
  if (st) return st;
  int64_t tot = 0;
  if (R->nreads > 0) {
    int64_t last_off = 0;
    int32_t last_cnt = 0;
    GB_HIP(hipMemcpy(&last_off, R->d_offsets + (R->nreads - 1), sizeof(int64_t), hipMemcpyDeviceToHost));
    GB_HIP(hipMemcpy(&last_cnt, R->d_counts + (R->nreads - 1), sizeof(int32_t), hipMemcpyDeviceToHost));
    tot = last_off + last_cnt;
  }
  if ((st = scatter_out(R, tot))) return st;
  GB_HIP(hipStreamSynchronize(R->stream));
  *d_smems = R->d_out;
  *n = R->total;
  return GB_OK;
}

}  // namespace gbfmi

extern "C" {

int gb_fmi_debug_pack(int64_t n, const int64_t *ent, int64_t *ent_out, const int64_t *cnt, int64_t *cnt_out) {
  GB_ARG(n >= 0 && (n == 0 || (ent && ent_out && cnt && cnt_out)), "gb_fmi_debug_pack: bad arguments");
  for (int64_t i = 0; i < n; i++) {
    gbfmi::Ent e;
    e.k = ent[5 * i];
    e.l = ent[5 * i + 1];
    e.s = ent[5 * i + 2];
    e.m = (uint32_t)ent[5 * i + 3];
    e.n = (uint32_t)ent[5 * i + 4];
    const gbfmi::Ent r = gbfmi::unpack_ent(gbfmi::pack_ent(e));
    ent_out[5 * i] = r.k;
    ent_out[5 * i + 1] = r.l;
    ent_out[5 * i + 2] = r.s;
    ent_out[5 * i + 3] = r.m;
    ent_out[5 * i + 4] = r.n;
    uint64_t w[2];
    gbfmi::occ32_pack_counts(cnt[3 * i], cnt[3 * i + 1], cnt[3 * i + 2], w);
    gbfmi::occ32_unpack_counts(w, cnt_out[3 * i], cnt_out[3 * i + 1], cnt_out[3 * i + 2]);
  }
  return GB_OK;
}

int gb_fmi_debug_trace(gb_fmi_reads *R, int64_t *out) {
  GB_ARG(R && out && R->ran, "gb_fmi_debug_trace: bad arguments");
  GB_ARG(R->d_trace && R->cap_trace >= (size_t)R->nreads * 3 * sizeof(int64_t),
         "gb_fmi_debug_trace: the last search ran without GB_FMI_FLAGS & 8");
  GB_HIP(hipStreamSynchronize(R->stream));
  GB_HIP(hipMemcpy(out, R->d_trace, (size_t)R->nreads * 3 * sizeof(int64_t), hipMemcpyDeviceToHost));
  return GB_OK;
}

int gb_fmi_debug_ctl(gb_fmi_reads *R, int32_t out[8]) {
  GB_ARG(R && out && R->ran, "gb_fmi_debug_ctl: bad arguments");
  GB_HIP(hipSetDevice(R->idx->device));
  GB_HIP(hipStreamSynchronize(R->stream));
  GB_HIP(hipMemcpy(out, R->d_ctl, 8 * sizeof(int32_t), hipMemcpyDeviceToHost));
  return GB_OK;
}

int gb_fmi_debug_prof(uint64_t out[8], int reset) {
  GB_ARG(out, "gb_fmi_debug_prof: null out");
  GB_HIP(hipDeviceSynchronize());
  GB_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(gbfmi::g_fmi_prof), sizeof(uint64_t) * 8));
  if (reset) {
    const uint64_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    GB_HIP(hipMemcpyToSymbol(HIP_SYMBOL(gbfmi::g_fmi_prof), z, sizeof(z)));
  }
  return GB_OK;
}


int gb_fmi_index_load(const char *path, gb_fmi_index **out) {
  GB_ARG(path && out, "gb_fmi_index_load: null argument");
  *out = nullptr;
  FILE *fp = fopen(path, "rb");
  if (!fp) {
    gb::set_error("gb_fmi_index_load: cannot open %s", path);
    return GB_ERR_ARG;
  }
  int64_t n = 0, count[5];
  if (fread(&n, 8, 1, fp) != 1 || fread(count, 8, 5, fp) != 5 || n <= 1) {
    fclose(fp);
    gb::set_error("gb_fmi_index_load: %s: bad header", path);
    return GB_ERR_ARG;
  }
  const int64_t cp_size = (n >> 6) + 1;
  std::vector<gbfmi::CpOcc> occ((size_t)cp_size);
  if (fread(occ.data(), sizeof(gbfmi::CpOcc), (size_t)cp_size, fp) != (size_t)cp_size) {
    fclose(fp);
    gb::set_error("gb_fmi_index_load: %s: truncated CP_OCC table", path);
    return GB_ERR_ARG;
  }
  const int64_t ns = (n >> 3) + 1;  // SA_COMPRESSION with SA_COMPX = 3 (macro.h:64-66)
  int64_t sentinel = -1;
  std::vector<int8_t> ms((size_t)ns);
  std::vector<uint32_t> ls((size_t)ns);
  if (fread(ms.data(), 1, (size_t)ns, fp) != (size_t)ns || fread(ls.data(), 4, (size_t)ns, fp) != (size_t)ns ||
      fread(&sentinel, 8, 1, fp) != 1) {
    fclose(fp);
    gb::set_error("gb_fmi_index_load: %s: truncated (sampled SA / sentinel)", path);
    return GB_ERR_ARG;
  }
  fclose(fp);
  // sa_entry = sa_ms_byte << 32 + sa_ls_word (FMI_search.cpp:1790-1802), packed once at load
  std::vector<int64_t> sa((size_t)ns);
  for (int64_t i = 0; i < ns; i++) sa[i] = ((int64_t)ms[i] << 32) + (int64_t)ls[i];
  std::vector<int8_t>().swap(ms);
  std::vector<uint32_t>().swap(ls);
  auto *idx = new gb_fmi_index();
  GB_HIP(hipGetDevice(&idx->device));
  idx->n = n;
  for (int b = 0; b < 5; b++) idx->count[b] = count[b] + 1;  // FMI_search.cpp:763-768
  idx->sentinel = sentinel;
  idx->cp_size = cp_size;
  idx->sa_ns = ns;
  hipError_t e = hipMalloc(&idx->d_occ, sizeof(gbfmi::CpOcc) * (size_t)cp_size);
  if (e == hipSuccess)
    e = gb::memcpy_big(idx->d_occ, occ.data(), sizeof(gbfmi::CpOcc) * (size_t)cp_size, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&idx->d_sa, sizeof(int64_t) * (size_t)ns);
  if (e == hipSuccess) e = gb::memcpy_big(idx->d_sa, sa.data(), sizeof(int64_t) * (size_t)ns, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    gb::set_error("gb_fmi_index_load: %s", hipGetErrorString(e));
    gb_fmi_index_destroy(idx);
    return GB_ERR_HIP;
  }
  *out = idx;
  return GB_OK;
}

int gb_fmi_index_prepare(gb_fmi_index *idx) {
  GB_ARG(idx, "gb_fmi_index_prepare: null index");
  if (idx->d_occ32) return GB_OK;
  GB_HIP(hipSetDevice(idx->device));
  hipStream_t s;
  GB_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int st = gbfmi::ensure_occ32(idx, s);
  (void)hipStreamDestroy(s);
  return st;
}

int gb_fmi_index_info(gb_fmi_index *idx, int64_t *n, int64_t *count5, int64_t *sentinel) {
  GB_ARG(idx, "gb_fmi_index_info: null index");
  if (n) *n = idx->n;
  if (count5)
    for (int b = 0; b < 5; b++) count5[b] = idx->count[b];
  if (sentinel) *sentinel = idx->sentinel;
  return GB_OK;
}

int gb_fmi_index_cp_occ(gb_fmi_index *idx, void *dst, int64_t dst_bytes) {
  GB_ARG(idx && dst, "gb_fmi_index_cp_occ: null argument");
  const int64_t bytes = idx->cp_size * (int64_t)sizeof(gbfmi::CpOcc);
  GB_ARG(dst_bytes >= bytes, "gb_fmi_index_cp_occ: need %lld bytes", (long long)bytes);
  GB_HIP(gb::memcpy_big(dst, idx->d_occ, (size_t)bytes, hipMemcpyDeviceToHost));
  return GB_OK;
}

int gb_fmi_index_sa(gb_fmi_index *idx, int64_t *dst, int64_t dst_entries) {
  GB_ARG(idx && dst, "gb_fmi_index_sa: null argument");
  GB_ARG(idx->d_sa, "gb_fmi_index_sa: index has no sampled suffix array");
  GB_ARG(dst_entries >= idx->sa_ns, "gb_fmi_index_sa: need %lld entries", (long long)idx->sa_ns);
  GB_HIP(gb::memcpy_big(dst, idx->d_sa, sizeof(int64_t) * (size_t)idx->sa_ns, hipMemcpyDeviceToHost));
  return GB_OK;
}

int gb_fmi_index_destroy(gb_fmi_index *idx) {
  if (!idx) return GB_OK;
  (void)hipFree(idx->d_occ);
  (void)hipFree(idx->d_occ32);
  (void)hipFree(idx->d_sa);
  delete idx;
  return GB_OK;
}

}  // extern "C"

// Destroyed read sets of this thread, kept for reuse (never freed: freeing at thread exit could
// run after the HIP runtime is torn down).
static std::vector<gb_fmi_reads *> &free_reads() {
  thread_local std::vector<gb_fmi_reads *> fl;
  return fl;
}

extern "C" {

int gb_fmi_reads_create(gb_fmi_index *idx, const uint8_t *enc_qdb, const int32_t *lens,
                        int32_t num_reads, int32_t max_readlength, gb_fmi_reads **out) {
  GB_ARG(idx && out && (num_reads == 0 || (enc_qdb && lens)), "gb_fmi_reads_create: null argument");
  GB_ARG(num_reads >= 0 && max_readlength > 0 && max_readlength < 8192,
         "gb_fmi_reads_create: bad sizes (reads %d, max_readlength %d; need < 8192)", num_reads, max_readlength);
  GB_ARG(idx && idx->n < (1ll << 34), "gb_fmi_reads_create: index too large for 34-bit list entries");
  for (int32_t r = 0; r < num_reads; r++)
    GB_ARG(lens[r] >= 0 && lens[r] <= max_readlength, "read %d: length %d > max_readlength %d", r,
           lens[r], max_readlength);
  *out = nullptr;
  int dev = 0;
  GB_HIP(hipGetDevice(&dev));
  gb_fmi_reads *R = nullptr;
  {
    auto &fl = free_reads();
    for (size_t k = 0; k < fl.size(); k++)
      if (fl[k]->device == dev) {
        R = fl[k];
        fl.erase(fl.begin() + (long)k);
        break;
      }
  }
  hipError_t e = hipSuccess;
  if (!R) {
    R = new gb_fmi_reads();
    R->device = dev;
    e = hipStreamCreateWithFlags(&R->stream, hipStreamNonBlocking);
    for (auto &ev : R->ev)
      if (e == hipSuccess) e = hipEventCreate(&ev);
    if (e == hipSuccess) e = hipMalloc(&R->d_ovf_list, gbfmi::kMaxOvf * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&R->d_big, (size_t)gbfmi::kMaxOvf * gbfmi::kBigCap * sizeof(gb_smem));
    if (e == hipSuccess) e = hipMalloc(&R->d_ctl, 8 * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&R->d_calls, 2 * sizeof(unsigned long long));
  }
  R->idx = idx;
  R->nreads = num_reads;
  R->stride = max_readlength;
  R->cus = device_cus();
  R->lanes = lanes_for_device(R->cus);
  R->ran = R->scattered = false;
  R->total = 0;
  const size_t nr = (size_t)std::max(num_reads, 1);
  auto reserve = [&](auto **p, size_t *cap, size_t bytes) {
    if (e != hipSuccess || bytes <= *cap) return;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    e = hipMalloc(p, std::max<size_t>(bytes, 16));
    if (e == hipSuccess) *cap = bytes;
  };
  reserve(&R->d_qdb, &R->cap_qdb, nr * (size_t)max_readlength);
  reserve(&R->d_lens, &R->cap_lens, nr * sizeof(int32_t));
  reserve(&R->d_scratch, &R->cap_scratch, (size_t)R->lanes * max_readlength * sizeof(gbfmi::PEnt));
  reserve(&R->d_slots, &R->cap_slots, nr * gbfmi::kCap * sizeof(gb_smem));
  reserve(&R->d_ovf_pos, &R->cap_ovf_pos, nr * sizeof(int32_t));
  reserve(&R->d_counts, &R->cap_counts, nr * sizeof(int32_t));
  reserve(&R->d_heavy, &R->cap_heavy, 2 * nr * sizeof(int32_t));
  reserve(&R->d_phase, &R->cap_phase, nr * 3 * sizeof(int32_t));
  reserve(&R->d_offsets, &R->cap_offsets, (nr + 1) * sizeof(int64_t));
  if (e == hipSuccess)
    e = hipcub::DeviceScan::ExclusiveSum(nullptr, R->temp_bytes, R->d_counts, R->d_offsets, (int)nr);
  reserve(&R->d_temp, &R->cap_temp, std::max<size_t>(R->temp_bytes, 16));
  if (e == hipSuccess && num_reads) e = gb::memcpy_big(R->d_qdb, enc_qdb, (size_t)num_reads * max_readlength, hipMemcpyHostToDevice);
  R->q4_stride = (((max_readlength + 7) / 8) + 3) & ~3;  // 16-byte rows (smem_search staging)
  reserve(&R->d_q4, &R->cap_q4, nr * (size_t)R->q4_stride * sizeof(uint32_t));
  R->q2_stride = (((max_readlength + 15) / 16) + 3) & ~3;
  reserve(&R->d_q2, &R->cap_q2, nr * (size_t)R->q2_stride * sizeof(uint32_t));
  reserve(&R->d_npos, &R->cap_npos, nr * sizeof(uint32_t));
  if (e == hipSuccess && num_reads) e = hipMemcpy(R->d_lens, lens, (size_t)num_reads * sizeof(int32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess && num_reads) {
    const int64_t nt = (int64_t)num_reads * R->q4_stride;
    hipLaunchKernelGGL(gbfmi::pack_q4, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, R->stream, R->d_qdb,
                       max_readlength, num_reads, R->q4_stride, R->d_q4);
    // N positions: npos all ones, the per-read N counts (d_counts, which the search rewrites) zero
    e = hipMemsetAsync(R->d_npos, 0xFF, (size_t)num_reads * sizeof(uint32_t), R->stream);
    if (e == hipSuccess) e = hipMemsetAsync(R->d_counts, 0, (size_t)num_reads * sizeof(int32_t), R->stream);
    const int64_t n2 = (int64_t)num_reads * R->q2_stride;
    hipLaunchKernelGGL(gbfmi::pack_q2, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, R->stream, R->d_qdb,
                       max_readlength, R->d_lens, num_reads, R->q2_stride, R->d_q2, R->d_npos, R->d_counts);
    hipLaunchKernelGGL(gbfmi::npos_finish, dim3((unsigned)((num_reads + 255) / 256)), dim3(256), 0, R->stream,
                       R->d_counts, num_reads, R->d_npos);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(R->stream);
  }
  if (e != hipSuccess) {
    gb::set_error("gb_fmi_reads_create: %s", hipGetErrorString(e));
    R->complete = false;  // a partly built read set is freed, never recycled
    gb_fmi_reads_destroy(R);
    return GB_ERR_HIP;
  }
  R->complete = true;
  *out = R;
  return GB_OK;
}

int gb_fmi_reads_destroy(gb_fmi_reads *R) {
  if (!R) return GB_OK;
  if (R->stream) (void)hipStreamSynchronize(R->stream);
  gbfmi::sa_job_destroy(R->sa);
  R->sa = nullptr;
  if (R->complete) {  // a complete read set: keep it for the next create on this thread
    free_reads().push_back(R);
    return GB_OK;
  }
  for (void *p : {(void *)R->d_qdb, (void *)R->d_q4, (void *)R->d_q2, (void *)R->d_npos, (void *)R->d_lens, (void *)R->d_scratch, (void *)R->d_slots,
                  (void *)R->d_counts, (void *)R->d_phase, (void *)R->d_offsets, (void *)R->d_out,
                  (void *)R->d_ctl, (void *)R->d_calls, R->d_temp, (void *)R->d_ovf_list,
                  (void *)R->d_ovf_pos, (void *)R->d_big, (void *)R->d_trace, (void *)R->d_heavy})
    (void)hipFree(p);
  for (auto ev : R->ev)
    if (ev) (void)hipEventDestroy(ev);
  if (R->stream) (void)hipStreamDestroy(R->stream);
  delete R;
  return GB_OK;
}

int gb_fmi_search(gb_fmi_reads *R, int32_t min_seed_len) {
  gb::Range range_("gb.fmi.search");
  GB_ARG(R, "gb_fmi_search: null read set");
  GB_ARG(min_seed_len > 0, "gb_fmi_search: min_seed_len %d", min_seed_len);
  GB_HIP(hipSetDevice(R->idx->device));
  if (int st = gbfmi::ensure_occ32(R->idx, R->stream)) return st;
  GB_HIP(hipEventRecord(R->ev[0], R->stream));
  GB_HIP(hipMemsetAsync(R->d_ctl, 0, 8 * sizeof(int32_t), R->stream));
  GB_HIP(hipMemsetAsync(R->d_calls, 0, 2 * sizeof(unsigned long long), R->stream));
  gbfmi::SearchArgs A;
  A.F.occ = R->idx->d_occ32;
  for (int b = 0; b < 5; b++) A.F.count[b] = R->idx->count[b];
  A.F.sentinel = R->idx->sentinel;
  A.qdb = R->d_qdb;
  A.q4 = R->d_q4;
  A.q4_stride = R->q4_stride;
  A.q2 = R->d_q2;
  A.q2_stride = R->q2_stride;
  A.npos = R->d_npos;
  A.lens = R->d_lens;
  A.nreads = R->nreads;
  A.stride = R->stride;
  A.min_seed_len = min_seed_len;
  A.split_len = (int)(min_seed_len * 1.5 + .499);  // fmi.cpp:239
  A.scratch = R->d_scratch;
  A.slots = R->d_slots;
  A.counts = R->d_counts;
  A.phase = R->d_phase;
  A.next_read = R->d_ctl;
  A.ovf_list = R->d_ovf_list;
  A.ovf_n = R->d_ctl + 1;
  A.fatal = R->d_ctl + 2;
  A.bwt_calls = R->d_calls;
  {
    const char *e = getenv("GB_FMI_FLAGS");
    A.flags = e ? atoi(e) : 0;
    // GB_FMI_HEAVY: the hand-over budget in backwardExt calls (0 = never hand over)
    const char *h = getenv("GB_FMI_HEAVY");
    const int budget = h ? atoi(h) : gbfmi::kHeavyBudget;
    A.budget = (budget > 0 && R->stride <= gbfmi::kHeavyMaxLen) ? budget : INT32_MAX;
    const char *pf = getenv("GB_FMI_PREFETCH");
    A.prefetch = pf && *pf == '1';
  }
  A.heavy = R->d_heavy;
  A.heavy_n = R->d_ctl + 4;
  A.trace = nullptr;
  if ((A.flags & 8) && R->nreads > 0) {
    const size_t bytes = (size_t)R->nreads * 3 * sizeof(int64_t);
    if (bytes > R->cap_trace) {
      (void)hipFree(R->d_trace);
      R->d_trace = nullptr;
      R->cap_trace = 0;
      GB_HIP(hipMalloc(&R->d_trace, bytes));
      R->cap_trace = bytes;
    }
    GB_HIP(hipMemsetAsync(R->d_trace, 0, bytes, R->stream));
    A.trace = R->d_trace;
  }
  if (R->nreads > 0) {
    // one pass: every read, kCap slots each; a read that outgrows them is promoted in place to a
    // kBigCap slot of the d_big pool
    A.slots = R->d_slots;
    A.big = R->d_big;
    A.cap = gbfmi::kCap;
    A.list = nullptr;
    A.list_n = nullptr;
    const int blocks = std::max(1, std::min(R->lanes / 64, (R->nreads + 63) / 64));
    // entries of the `prev` list head kept in LDS, 4 (default), 8 or 0
    const int top = top_entries();
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, R->stream, A); };
    const char *qe = getenv("GB_FMI_QLDS");  // 0: read codes from global memory, not staged in LDS
    // the 2-bit form hands reads with more than four N's to the heavy pass, so it needs that pass
    if (R->stride <= gbfmi::kQBases && !(qe && *qe == '0') && q3_codes() && A.budget != INT32_MAX) {
      if (top >= 8)
        launch(gbfmi::smem_search<3, 8>);
      else
        launch(gbfmi::smem_search<3, 7>);
    } else if (R->stride <= gbfmi::kQBases && !(qe && *qe == '0') && q2_codes() && A.budget != INT32_MAX) {
      if (top >= 8)
        launch(gbfmi::smem_search<2, 8>);
      else if (top >= 7)
        launch(gbfmi::smem_search<2, 7>);
      else if (top >= 6)
        launch(gbfmi::smem_search<2, 6>);
      else if (top >= 5)
        launch(gbfmi::smem_search<2, 5>);
      else
        launch(gbfmi::smem_search<2, 0>);
    } else if (R->stride <= gbfmi::kQBases && !(qe && *qe == '0')) {
      if (top >= 8)
        launch(gbfmi::smem_search<1, 8>);
      else if (top >= 7)
        launch(gbfmi::smem_search<1, 7>);
      else if (top >= 6)
        launch(gbfmi::smem_search<1, 6>);
      else if (top >= 5)
        launch(gbfmi::smem_search<1, 5>);
      else if (top >= 4)
        launch(gbfmi::smem_search<1, 4>);
      else
        launch(gbfmi::smem_search<1, 0>);
    } else {
      if (top >= 8)
        launch(gbfmi::smem_search<0, 8>);
      else if (top >= 4)
        launch(gbfmi::smem_search<0, 4>);
      else
        launch(gbfmi::smem_search<0, 0>);
    }
    GB_HIP(hipGetLastError());
    if (A.budget != INT32_MAX) {
      gbfmi::HeavyArgs H;
      H.F = A.F;
      H.qdb = A.qdb;
      H.lens = A.lens;
      H.stride = A.stride;
      H.min_seed_len = A.min_seed_len;
      H.split_len = A.split_len;
      H.heavy = A.heavy;
      H.heavy_n = A.heavy_n;
      H.slots = A.slots;
      H.big = A.big;
      H.counts = A.counts;
      H.phase = A.phase;
      H.ovf_list = A.ovf_list;
      H.ovf_n = A.ovf_n;
      H.fatal = A.fatal;
      H.bwt_calls = A.bwt_calls;
      H.trace = A.trace;
      // the heavy-read count is on the device: a grid of 16 waves per CU strides over the list
      hipLaunchKernelGGL(gbfmi::smem_heavy, dim3((unsigned)std::max(1, R->cus * 16)), dim3(64), 0,
                         R->stream, H);
      GB_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(gbfmi::mark_overflow, dim3((gbfmi::kMaxOvf + 255) / 256), dim3(256), 0, R->stream,
                       R->d_ovf_list, R->d_ctl + 1, R->d_ovf_pos);
    GB_HIP(hipGetLastError());
    const int sort_blocks = std::max(1, std::min(256 * 8, (R->nreads + 15) / 16));  // 4 waves x 4 reads
    hipLaunchKernelGGL(gbfmi::sort_slots, dim3(sort_blocks), dim3(256), 0, R->stream, R->d_slots, R->d_big,
                       R->d_ovf_pos, R->d_counts, R->nreads);
    GB_HIP(hipGetLastError());
  }
  GB_HIP(hipEventRecord(R->ev[1], R->stream));
  if (R->nreads > 0) {
    GB_HIP(hipcub::DeviceScan::ExclusiveSum(R->d_temp, R->temp_bytes, R->d_counts, R->d_offsets,
                                            R->nreads, R->stream));
  }
  GB_HIP(hipEventRecord(R->ev[2], R->stream));
  R->ran = true;
  R->scattered = false;
  return GB_OK;
}

int gb_fmi_sync(gb_fmi_reads *R) {
  GB_ARG(R, "gb_fmi_sync: null read set");
  GB_HIP(hipStreamSynchronize(R->stream));
  return GB_OK;
}

int gb_fmi_results(gb_fmi_reads *R, int32_t batch_size, gb_smem *out, int64_t out_cap,
                   int64_t *total, int64_t *batch_counts, int64_t *phase_counts) {
  GB_ARG(R && R->ran, "gb_fmi_results: search has not run");
  GB_ARG(batch_size > 0, "gb_fmi_results: batch_size %d", batch_size);
  GB_HIP(hipSetDevice(R->idx->device));
  GB_HIP(hipStreamSynchronize(R->stream));
  if (int st = gbfmi::check_fatal(R, "gb_fmi_results")) return st;
  const int32_t n = R->nreads;
  std::vector<int32_t> counts((size_t)std::max(n, 1)), phase((size_t)std::max(n, 1) * 3);
  if (n) {
    GB_HIP(hipMemcpy(counts.data(), R->d_counts, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    GB_HIP(hipMemcpy(phase.data(), R->d_phase, sizeof(int32_t) * 3 * n, hipMemcpyDeviceToHost));
  }
  int64_t tot = 0;
  for (int32_t r = 0; r < n; r++) tot += counts[r];
  if (total) *total = tot;
  if (batch_counts) {
    for (int32_t b = 0; b * (int64_t)batch_size < n; b++) {
      int64_t s = 0;
      for (int32_t r = b * batch_size; r < std::min<int64_t>(n, (int64_t)(b + 1) * batch_size); r++) s += counts[r];
      batch_counts[b] = s;
    }
  }
  if (phase_counts) {
    phase_counts[0] = phase_counts[1] = phase_counts[2] = 0;
    for (int32_t r = 0; r < n; r++)
      for (int k = 0; k < 3; k++) phase_counts[k] += phase[3 * r + k];
  }
  if (out) {
    GB_ARG(out_cap >= tot, "gb_fmi_results: out_cap %lld < %lld SMEMs", (long long)out_cap, (long long)tot);
    if (int st = gbfmi::scatter_out(R, tot)) return st;
    if (tot) {
      GB_HIP(hipStreamSynchronize(R->stream));
      GB_HIP(gb::memcpy_big(out, R->d_out, sizeof(gb_smem) * (size_t)tot, hipMemcpyDeviceToHost));
    }
  }
  return GB_OK;
}

int gb_fmi_timing(gb_fmi_reads *R, float *search_ms, float *total_ms, int64_t *bwt_calls) {
  GB_ARG(R && R->ran, "gb_fmi_timing: search has not run");
  GB_HIP(hipEventSynchronize(R->ev[2]));
  float a = 0, b = 0;
  GB_HIP(hipEventElapsedTime(&a, R->ev[0], R->ev[1]));
  GB_HIP(hipEventElapsedTime(&b, R->ev[0], R->ev[2]));
  if (search_ms) *search_ms = a;
  if (total_ms) *total_ms = b;
  if (bwt_calls) {
    unsigned long long c = 0;
    GB_HIP(hipMemcpy(&c, R->d_calls, sizeof(c), hipMemcpyDeviceToHost));
    *bwt_calls = (int64_t)c;
  }
  return GB_OK;
}

}  // extern "C"
