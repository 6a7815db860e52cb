// chain.hip -- MI355X (gfx950) minimap2 chaining DP (chain_dp): kernel and C ABI.
//
// Semantics: benchmarks/chain/src/host_kernel.cpp:405-472 (plaintext branch) ==
// tools/minimap2-acceleration/kernel/scalar/src/host_kernel.cpp:30-94, with the C integer / double
// semantics of that source (int64 dr, int32 truncations, (int)(dd * .01 * avg_qspan), no FMA).
//
// MI355X design: one call (read) per workgroup of two waves; anchors are processed in order i
// (score[i] depends on score[j < i]) and the predecessor loop j = i-1 .. st runs 64 candidates per
// step, lane l taking j = jtop - l, i.e. lanes in the reference's visiting order. A producer wave
// computes the score-independent pair geometry ahead; the consumer wave resolves the reference's
// loop, which is sequential only through three quantities, each a wave-wide operation:
//   max_f        running maximum of the candidate scores             (DPP max scan)
//   n_skip       max(n-1, 0) on an improvement, n+1 on a "targeted" non-improvement
//                -> a reflected walk n = max(N + D, D - min D)      (mbcnt chain + DPP min scan)
//   break        first lane where n_skip exceeds 25                   (ballot + ctz)
// "targets[j] == i" is decided by marks from earlier-visited j' (> j) of the same i, which are all
// visited before any break that could stop j: marks are i+1 stamps in an LDS ring indexed by j.
// The last 64 anchors (the first step of every i) live in registers, shifted one lane per i with
// DPP, so most anchors need no memory access at all; older candidates are read from global memory
// through L2 (sc1 loads) after a vmcnt drain that orders the wave's own stores before them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <numeric>
#include <vector>

#include "../../include/gb_chain.h"
#include "gb_common.h"
#include "chain_internal.h"
#include "chain_dev.h"

namespace gbchain {

struct Args {
  const VCall *vc;  // blocks, longest first
  const float *avg_qspan;
  const int32_t *params4;
  const uint64_t *x, *y;
  int32_t *score, *parent, *target, *peak;
  int32_t *s_score, *s_parent;  // segment scratch (kVScratch blocks)
  unsigned long long *visited;
  unsigned long long *prof;  // optional phase clocks (GB_CHAIN_PROF=1), see chain_kernel
  int32_t exp;               // PROF == 2 timing experiments (GB_CHAIN_EXP): 1 producer skips the pair
                             // geometry, 2 consumer only drains the slots (outputs are then garbage)
};

// Producer -> consumer hand-off, one slot per anchor i: the geometry of its first 64 candidates.
// seq = i + 1 is written last and read first, so a slot whose seq matches is complete.
constexpr int kSlots = 16;
struct Slot {
  int32_t sg[64];  // kNoCand for filtered candidates
  int32_t seq, st, q_span, pad;
};


// LDS counters are read by every lane; the count is uniform, so take it into an SGPR
__device__ __forceinline__ int32_t lds_count(int *p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}

// Two waves per call. The anchors' pair geometry (filters, gap costs; no scores involved) runs ahead
// in the producer wave and is handed over through an LDS ring; the consumer wave keeps only the
// score-dependent sequential part (max_f / n_skip scans, break, targets, outputs), so the critical
// path of a long call is roughly halved. The consumer reads slot i+1 during step i and validates it
// by its seq word at step i+1; the producer polls the consumer's `consumed` count with s_sleep.
// PROF (GB_CHAIN_PROF): 1 = start/end stamps (100 MHz) of the first/longest call and of the
// whole grid; 2 = also phase clocks: head, steps, tail, nsteps, slot misses, miss ticks.
// RING: the stamp ring (kRing for any window, kRingSmall for blocks whose windows are known to hold
// <= kRingSmall anchors: 12 KB less LDS, three times the blocks per CU).
template <int PROF, int RING>
__global__ __launch_bounds__(128) void chain_kernel(Args A) {
  __shared__ uint32_t S[RING + 64];
  __shared__ Slot ring[kSlots];
  __shared__ int consumed;
  const VCall &V = A.vc[blockIdx.x];
  const int c = V.call;
  const int lane = threadIdx.x & 63;
  const bool producer = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) != 0;  // wave-uniform role
  const int32_t n = V.n, known = V.known;
  const bool fin = (V.mode & kVFinal) != 0;
  // parents in memory relative to the call, in registers relative to this block; a parent before the
  // block (only a fix-up block's loaded anchors have one) lies before every window it computes, so
  // it reads as "none"
  const int32_t pbase = V.pbase;
  auto p_in = [&](int32_t p) { return p >= pbase ? p - pbase : -1; };
  const int max_dist_x = A.params4[4 * c], max_dist_y = A.params4[4 * c + 1];
  const int bw = A.params4[4 * c + 2], n_segs = A.params4[4 * c + 3];
  const double avg_qspan = (double)A.avg_qspan[c];
  const uint64_t *X = A.x + V.in, *Y = A.y + V.in;
  const bool scr = (V.mode & kVScratch) != 0;
  int32_t *score = (scr ? A.s_score : A.score) + V.out, *parent = (scr ? A.s_parent : A.parent) + V.out;
  int32_t *target = A.target + V.out, *peak = A.peak + V.out;  // written by kVFinal blocks only

  for (int k = threadIdx.x; k < RING + 64; k += 128) S[k] = 0;
  if (fin)
    for (int32_t k = threadIdx.x; k < n; k += 128) target[k] = 0;  // a fresh std::vector in the reference
  if (threadIdx.x < kSlots) ring[threadIdx.x].seq = 0;
  if (threadIdx.x == 0) consumed = 0;
  __builtin_amdgcn_s_waitcnt(0);  // zeroing stores complete before any later targets store
  __syncthreads();

  if (producer) {
    // ---------------- producer: geometry of anchor i against i-1-lane --------------------------
    uint64_t wx = 0, wy = 0;  // lane l: anchor i-1-l
    int32_t st = 0;
    const bool pc = PROF == 2 && blockIdx.x == 0;
    unsigned long long p_load = 0, p_wait = 0, t0 = 0;
    // Anchor blocks: bx/by hold X/Y[64b .. 64b+63] (lane k = anchor 64b+k) and the next block is
    // loaded one block ahead, so x[i], y[i] are register reads (readlane), not LDS round trips.
    uint64_t bx = X[min(lane, n - 1)], by = Y[min(lane, n - 1)];
    uint64_t nx = X[min(64 + lane, n - 1)], ny = Y[min(64 + lane, n - 1)];
    // The window start st: X[sb .. sb+63] (sb = st rounded down to 64) sits in a VGPR, the next
    // block is loaded one block ahead, and st advances by one ballot over the block instead of a
    // chain of dependent scalar loads (while (st < i && x[i] > x[st] + max_dist_x) ++st).
    int32_t sb = 0;
    uint64_t sx = bx, sxn = nx;
    const uint64_t mdx = (uint64_t)(int64_t)max_dist_x;
    // the consumer's progress, read one anchor ahead (a stale value only delays; it never lets the
    // producer overwrite an unread slot)
    int32_t cons_v = 0;
    for (int32_t iv = 0; iv < n; iv++) {
      // opaque to loop strength reduction, which otherwise derives i from the per-lane i-1-lane
      // (a VGPR induction variable) and turns every uniform value below into a vector one
      const int32_t i = __builtin_amdgcn_readfirstlane(iv);
      if (pc) t0 = __builtin_amdgcn_s_memtime();
      if ((i & 63) == 0 && i > 0) {
        bx = nx;
        by = ny;
        nx = X[min(i + 64 + lane, n - 1)];
        ny = Y[min(i + 64 + lane, n - 1)];
      }
      const uint64_t xi = rfl64_lane(bx, i & 63), yi = rfl64_lane(by, i & 63);
      while (true) {  // first j >= st that stops the scan (j == i, or x[i] <= x[j] + max_dist_x)
        const int32_t jl = sb + lane;
        const uint64_t stop = __builtin_amdgcn_ballot_w64((jl >= st) & ((jl >= i) | !(xi > sx + mdx)));
        if (stop) {
          st = sb + __builtin_ctzll(stop);
          break;
        }
        sb += 64;  // every candidate of the block passed: next block
        sx = sxn;
        sxn = X[min(sb + 64 + lane, n - 1)];
        st = sb;
      }
      if (i - st > kMaxIter) {  // rare: > max_iter candidates in range
        st = i - kMaxIter;
        if (st >= sb + 64) {
          sb = st & ~63;
          sx = X[min(sb + lane, n - 1)];
          sxn = X[min(sb + 64 + lane, n - 1)];
        }
      }
      if (pc) {
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        p_load += t1 - t0;
      }
      int32_t sg;
      bool ok;
      if (PROF >= 1 && (A.exp & 1)) {
        ok = i - 1 - lane >= st;
        sg = 1;
      } else {
        ok = geometry(xi, yi, wx, wy, i - 1 - lane >= st, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sg);
      }
      // wait for a free slot
      if (pc) t0 = __builtin_amdgcn_s_memtime();
      if (i - __builtin_amdgcn_readfirstlane(cons_v) >= kSlots)
        while (i - lds_count(&consumed) >= kSlots) __builtin_amdgcn_s_sleep(1);
      if (pc) p_wait += __builtin_amdgcn_s_memtime() - t0;
      Slot &sl = ring[i & (kSlots - 1)];
      sl.sg[lane] = ok ? sg : kNoCand;
      if (lane == 0) {
        sl.st = st;
        sl.q_span = (int32_t)(yi >> 32 & 0xff);
        // published after the contents: the LDS performs one wave's accesses in issue order
        __hip_atomic_store(&sl.seq, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      cons_v = __hip_atomic_load(&consumed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      wx = dpp_shr_u64(wx, xi);
      wy = dpp_shr_u64(wy, yi);
    }
    {  // slot n: no candidates (the consumer precomputes one anchor ahead and reads it last)
      while (n - lds_count(&consumed) >= kSlots) __builtin_amdgcn_s_sleep(1);
      Slot &sl = ring[n & (kSlots - 1)];
      sl.sg[lane] = kNoCand;
      if (lane == 0) {
        sl.st = n;
        sl.q_span = 0;
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if (lane == 0) __hip_atomic_store(&sl.seq, n + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (pc && lane == 0) {
      atomicAdd(A.prof + 14, p_load);
      atomicAdd(A.prof + 15, p_wait);
    }
    return;
  }

  // ---------------- consumer ---------------------------------------------------------------------
  // Anchor i's first 64 candidates (lane l = j = i-1-l) are resolved in two parts. Everything that
  // does not depend on anchor i-1's own result is prepared one iteration early, while anchor i-1 is
  // still open: the partial scores of lanes >= 1 (their scores are known), their exclusive running
  // maximum, and the LDS stamps of the parents of lanes >= 1 (read back in the next iteration, so
  // the LDS latency is hidden). Once f[i-1] and p[i-1] arrive, what is left is lane 0's score (a
  // scalar add), one max + compare per lane for the improvements, lane 0's mark (one bit), and the
  // n_skip walk, which runs in scalar registers over the improvement and target bitmasks.
  // targets of speculative / fix-up blocks are not written: a zero-sized buffer drops every store
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(target, (short)0, fin ? n * 4 : 0, 0x00020000);
  const int32_t neg_lane = -lane;
  int32_t ws = 0, wpar = -1, wpk = 0;  // lane l: score/parent/peak of anchor i-1-l (top of iteration i)
  unsigned long long vis = 0, n_mem = 0, n_miss = 0, c_pre = 0, c_crit = 0, c_tail = 0, n_walk = 0, c_um = 0, c_walk = 0;
  typedef int32_t v4i __attribute__((ext_vector_type(4)));
  typedef volatile __attribute__((address_space(3))) v4i lds_v4i;
  typedef volatile __attribute__((address_space(3))) int32_t lds_i32;
  // slot a is read ahead (header first: LDS executes a wave's reads in order, so a matching seq
  // means the sg read after it saw the complete slot); slot n is the producer's empty sentinel
  v4i hdr = *(lds_v4i *)&ring[0].seq;
  int32_t psg = *(lds_i32 *)&ring[0].sg[lane];
  auto take = [&](int32_t a, int32_t &st, int32_t &q_span, int32_t &sg) {
    if (__builtin_amdgcn_readfirstlane(hdr.x) == a + 1) {
      st = __builtin_amdgcn_readfirstlane(hdr.y);
      q_span = __builtin_amdgcn_readfirstlane(hdr.z);
      sg = psg;
    } else {  // the producer was behind when the slot was read ahead: wait for it, read again
      if (PROF) ++n_miss;
      Slot &sl = ring[a & (kSlots - 1)];
      while (lds_count(&sl.seq) != a + 1) __builtin_amdgcn_s_sleep(1);
      st = __builtin_amdgcn_readfirstlane(*(lds_i32 *)&sl.st);
      q_span = __builtin_amdgcn_readfirstlane(*(lds_i32 *)&sl.q_span);
      sg = *(lds_i32 *)&sl.sg[lane];
    }
    // free slot a (its reads were issued before this write, and LDS runs them in order), then
    // read slot a+1 ahead
    if (lane == 0) __hip_atomic_store(&consumed, a + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    Slot &nl = ring[(a + 1) & (kSlots - 1)];
    hdr = *(lds_v4i *)&nl.seq;
    psg = *(lds_i32 *)&nl.sg[lane];
  };
  // prepared state of the anchor about to be resolved (the names of anchor a, lanes >= 1):
  //   psc  sg + score[j] (INT_MIN when filtered)   pB  max(q_span, psc of lanes 1..l-1)
  //   ppj  parent[j]                               pt  stamp read back at j (targeted iff == a+1)
  int32_t psc, pB, ppj, pt, pok, pst, pq, psg0;
  auto prepare_math = [&](int32_t a, int32_t sg, int32_t ws1, int32_t wp1) {
    const bool ok = sg != kNoCand;
    pok = ok;
    psc = ok ? (int32_t)((uint32_t)sg + (uint32_t)ws1) : INT_MIN;
    if (PROF >= 1 && (A.exp & 4)) {
      pB = pq;
    } else {
      const int32_t mx = scan_max(lane == 0 ? INT_MIN : psc);
      pB = max(dpp_shr_i32(mx, INT_MIN), pq);
    }
    ppj = wp1;
    // "targets[j] == a" from the parents of lanes >= 1: a stamp a+1 at each parent (a parent is an
    // earlier anchor, so only later lanes can be hit); read back here, consumed one iteration later
    if (PROF >= 1 && (A.exp & 8)) {
      pt = 0;
    } else {
      S[(ok & (lane > 0) & (wp1 >= pst)) ? (wp1 & (RING - 1)) : RING + lane] = (uint32_t)(a + 1);
      pt = (int32_t)S[(a - 1 - lane) & (RING - 1)];
    }
    psg0 = __builtin_amdgcn_readfirstlane(sg);
  };
  unsigned long long rt0 = 0, clk0 = 0;
  if (PROF) {
    rt0 = __builtin_amdgcn_s_memrealtime();
    clk0 = __builtin_amdgcn_s_memtime();
  }
  const bool pc = PROF == 2 && blockIdx.x == 0;
  {
    int32_t sg;
    take(0, pst, pq, sg);
    prepare_math(0, sg, 0, -1);
  }
  int32_t Mprev = 0, Jprev = -1;
  for (int32_t base = 0; base < n; base += 64) {
    const int32_t cnt = min(64, n - base);
    // kVFixup: anchors < known are final already; their score and parent replace the resolution
    int32_t kf = 0, kp = -1;
    if (base < known && base + lane < known) {
      kf = score[base + lane];
      kp = p_in(parent[base + lane]);
    }
    for (int32_t k = 0; k < cnt; k++) {
      const int32_t i = __builtin_amdgcn_readfirstlane(base + k);
      if (PROF >= 1 && (A.exp & 2)) {
        int32_t a0, a1, a2;
        take(i + 1, a0, a1, a2);
        continue;
      }
      unsigned long long t0 = 0;
      if (pc) t0 = __builtin_amdgcn_s_memtime();
      // this anchor's prepared state
      const int32_t sc = psc, B = pB, pjv_hi = ppj, st = __builtin_amdgcn_readfirstlane(pst),
                    q_span = __builtin_amdgcn_readfirstlane(pq), sg0 = psg0;
      const uint64_t okm = __builtin_amdgcn_ballot_w64(pok != 0);
      const uint64_t tgtm = __builtin_amdgcn_ballot_w64(pt == i + 1) & ~1ull;
      // the next anchor's slot (the only branch before the resolve: a producer that fell behind)
      int32_t sgn;
      take(i + 1, pst, pq, sgn);
      // From here to the walk's result the code is one basic block: the next anchor's preparation
      // (independent of this anchor's result) and this anchor's resolution interleave.
      const int32_t ws1 = dpp_shr_i32(ws, 0), wp1 = dpp_shr_i32(wpar, -1);
      prepare_math(i + 1, sgn, ws1, wp1);
      // ---- anchor i: no candidate passes the filters when jtop < st (okm == 0) ----------------
      const int32_t jtop = i - 1;
      const bool ok0 = okm & 1;
      const int32_t sc0 = ok0 ? (int32_t)((uint32_t)sg0 + (uint32_t)Mprev) : INT_MIN;
      // improvements: lane 0 against q_span, lanes >= 1 against max(q_span, sc0, earlier lanes)
      const uint64_t um = (__builtin_amdgcn_ballot_w64(sc > max(B, sc0)) & ~1ull) | (uint64_t)(sc0 > q_span);
      const int32_t dl = jtop - Jprev;  // lane 0 marks p[i-1]
      const uint64_t tg = tgtm | ((ok0 & (Jprev >= 0) & (dl < 64)) ? (1ull << (dl & 63)) : 0ull);
      // n_skip walk (host_kernel.cpp:81-88) over the lanes in visiting order: n after lane l is the
      // reflected walk max(D_l, D_l - min_{k<=l} D_k) of D_l = targeted non-improving minus
      // improving lanes up to l (n starts at 0; lane 0 is never targeted); the break is the first
      // targeted non-improving lane where n exceeds max_skip
      const uint64_t pm = okm & ~um & tg;
      const bool plus = (pm >> lane) & 1, upd = (um >> lane) & 1;
      const uint64_t num = ~um;
      const int32_t d_ex = (int32_t)__builtin_amdgcn_mbcnt_hi(
          (uint32_t)(num >> 32),
          __builtin_amdgcn_mbcnt_lo((uint32_t)num, __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)pm, (uint32_t)neg_lane))));
      const int32_t D = d_ex + (plus ? 1 : (upd ? -1 : 0));
      const int32_t n_after = max(D, D - scan_min(D));
      const uint64_t bm = __builtin_amdgcn_ballot_w64(plus & (n_after > kMaxSkip));
      const int32_t b = bm ? __builtin_ctzll(bm) : 64;
      const uint64_t below = bm ? (bm - 1) & ~bm : ~0ull;
      const int32_t nvalid = max(0, min(64, jtop - st + 1));
      uint32_t vis_i = bm ? (uint32_t)b + 1 : (uint32_t)nvalid;
      const uint64_t ume = um & below;
      const int32_t lu = 63 - __builtin_clzll(ume | 1);
      const int32_t m_lu = __builtin_amdgcn_readlane(sc, lu);
      int32_t M = ume ? (lu == 0 ? sc0 : m_lu) : q_span;
      int32_t J = ume ? jtop - lu : -1;
      // targets[p[j]] = i for the visited lanes that passed the filters
      const int32_t pjv = lane == 0 ? Jprev : pjv_hi;
      const bool wt = (bool)((okm & below) >> lane & 1) & (pjv >= 0);
      if (!(PROF >= 1 && (A.exp & 32)))
        __builtin_amdgcn_raw_buffer_store_b32(i, trs, wt ? (uint32_t)pjv * 4u : 0xFFFFFFFFu, 0, 0);
      if (!bm && jtop - 64 >= st && i >= known) {  // rare: older candidates (j < i-64) from memory
        if (PROF) ++n_mem;
        // this anchor's own stamps first (the next anchor's preparation overwrote them)
        const uint32_t stamp = (uint32_t)(i + 1);
        const bool okl = (okm >> lane) & 1;
        S[(okl & (pjv >= st)) ? (pjv & (RING - 1)) : RING + lane] = stamp;
        // the wave's flushed score/parent stores reach L2 before these sc1 reads of them
        __builtin_amdgcn_s_waitcnt(0);
        const uint64_t xi = X[i], yi = Y[i];
        int32_t N = __builtin_amdgcn_readlane(n_after, 63);
        for (int32_t jt = jtop - 64; jt >= st; jt -= 64) {
          const int32_t jj = jt - lane;
          const bool v = jj >= st;
          uint64_t xj = 0, yj = 0;
          int32_t scj = 0, pj = -1;
          if (v) {
            xj = X[jj];
            yj = Y[jj];
            scj = load_l2(score + jj);
            pj = p_in(load_l2(parent + jj));
          }
          int32_t sgo;
          const bool oko = geometry(xi, yi, xj, yj, v, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sgo);
          if (resolve_step<kMarkStore, RING>(oko ? sgo + scj : INT_MIN, oko, pj, jt, st, stamp, lane, neg_lane, trs, i, S, M, J, N,
                           vis_i))
            break;
        }
      }
      if (i < known) {
        M = __builtin_amdgcn_readlane(kf, k);
        J = __builtin_amdgcn_readlane(kp, k);
      }
      vis += vis_i;
      unsigned long long t2 = 0;
      if (pc) {
        t2 = __builtin_amdgcn_s_memtime();
        c_crit += t2 - t0;
      }
      // peak of the parent: from the register window when J >= i-64, else (rare) from memory
      const int32_t dJ = i - 1 - J;
      int32_t pkJ = __builtin_amdgcn_readlane(wpk, dJ & 63);
      // (kVFinal only: other blocks keep no peaks, and their `out` is not an offset into `peak`)
      if (fin && J >= 0 && dJ > 63) pkJ = __builtin_amdgcn_readfirstlane(load_l2(peak + J));
      const int32_t pki = (PROF >= 1 && (A.exp & 64)) ? M : (J >= 0 && pkJ > M) ? pkJ : M;
      ws = lane == 0 ? M : ws1;
      wpar = lane == 0 ? J : wp1;
      wpk = dpp_shr_i32(wpk, pki);
      Mprev = M;
      Jprev = J;
      if (pc) c_tail += __builtin_amdgcn_s_memtime() - t2;
    }
    // flush the window: anchors base .. base+cnt-1 (lane l: base+cnt-1-l)
    if (lane < cnt && base + cnt - 1 - lane >= known) {
      score[base + cnt - 1 - lane] = ws;
      parent[base + cnt - 1 - lane] = wpar >= 0 ? wpar + pbase : -1;
      if (fin) peak[base + cnt - 1 - lane] = wpk;
    }
  }
  if (PROF && lane == 0) {
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
    atomicMin(A.prof + 8, rt0);
    atomicMax(A.prof + 11, rt1);
    if (blockIdx.x == 0) {
      atomicAdd(A.prof + 9, rt0);
      atomicAdd(A.prof + 10, rt1);
      atomicAdd(A.prof + 0, c_pre);
      atomicAdd(A.prof + 1, c_crit);
      atomicAdd(A.prof + 2, c_tail);
      atomicAdd(A.prof + 3, n_mem);
      atomicAdd(A.prof + 4, n_miss);
      atomicAdd(A.prof + 5, n_walk);
      atomicAdd(A.prof + 12, c_um);
      atomicAdd(A.prof + 13, c_walk);
      atomicAdd(A.prof + 6, __builtin_amdgcn_s_memtime() - clk0);
      atomicAdd(A.prof + 7, __builtin_amdgcn_s_memrealtime() - rt0);
    }
  }
  // every lane accumulated the same (uniform) count
  if (fin && lane == 0) atomicAdd(A.visited, vis);
}

}  // namespace gbchain


namespace {
// A CSR call set the kernel can take (checked before any device work).
int validate(int64_t ncalls, const int64_t *offsets, const float *avg_qspan, const int32_t *params4,
             const uint64_t *x, const uint64_t *y) {
  GB_ARG(ncalls >= 0 && offsets, "gb_chain: bad arguments");
  GB_ARG(ncalls < (1ll << 31), "gb_chain: too many calls");
  const int64_t na = offsets[ncalls];
  GB_ARG(offsets[0] == 0 && na >= 0 && (na == 0 || (x && y)), "gb_chain: bad offsets");
  for (int64_t c = 0; c < ncalls; c++)
    GB_ARG(offsets[c + 1] >= offsets[c] && offsets[c + 1] - offsets[c] < (1ll << 30),
           "gb_chain: call %lld has a bad anchor range", (long long)c);
  GB_ARG(ncalls == 0 || (avg_qspan && params4), "gb_chain: null parameters");
  return GB_OK;
}

// Uploads a validated call set into B, growing B's buffers only when they are too small.
int batch_fill(gb_chain_batch *B, int64_t ncalls, const int64_t *offsets, const float *avg_qspan,
               const int32_t *params4, const uint64_t *x, const uint64_t *y) {
  if (int st = validate(ncalls, offsets, avg_qspan, params4, x, y)) return st;
  const int64_t na = offsets[ncalls];
  GB_HIP(hipSetDevice(B->device));
  GB_HIP(hipStreamSynchronize(B->stream));  // the previous contents may still be in use
  gbchain::chain_bt_destroy(B->bt);
  B->bt = nullptr;
  B->ran = false;
  const int64_t nc = std::max<int64_t>(ncalls, 1), nn = std::max<int64_t>(na, 1);
  if (nc > B->cap_calls) {
    for (void *q : {(void *)B->d_off, (void *)B->d_aq, (void *)B->d_par4}) (void)hipFree(q);
    B->d_off = nullptr, B->d_aq = nullptr, B->d_par4 = nullptr;
    B->cap_calls = 0;
    GB_HIP(hipMalloc(&B->d_off, (size_t)(nc + 1) * sizeof(int64_t)));
    GB_HIP(hipMalloc(&B->d_aq, (size_t)nc * sizeof(float)));
    GB_HIP(hipMalloc(&B->d_par4, (size_t)nc * 4 * sizeof(int32_t)));
    B->cap_calls = nc;
  }
  if (nn > B->cap_anchors) {
    for (void *q : {(void *)B->d_x, (void *)B->d_y, (void *)B->d_out}) (void)hipFree(q);
    B->d_x = nullptr, B->d_y = nullptr, B->d_out = nullptr;
    B->cap_anchors = 0;
    GB_HIP(hipMalloc(&B->d_x, (size_t)nn * sizeof(uint64_t)));
    GB_HIP(hipMalloc(&B->d_y, (size_t)nn * sizeof(uint64_t)));
    GB_HIP(hipMalloc(&B->d_out, (size_t)nn * 4 * sizeof(int32_t)));
    B->cap_anchors = nn;
  }
  B->ncalls = ncalls;
  B->nanchors = na;
  GB_HIP(hipMemcpy(B->d_off, offsets, (size_t)(ncalls + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (ncalls) {
    GB_HIP(hipMemcpy(B->d_aq, avg_qspan, (size_t)ncalls * sizeof(float), hipMemcpyHostToDevice));
    GB_HIP(hipMemcpy(B->d_par4, params4, (size_t)ncalls * 16, hipMemcpyHostToDevice));
  }
  // the anchors go up on the batch stream while the host plans the block table (from page-locked
  // caller memory -- the host_chain_kernel drop-in stages there -- the copy runs beside the plan)
  if (na) {
    GB_HIP(hipMemcpyAsync(B->d_x, x, (size_t)na * 8, hipMemcpyHostToDevice, B->stream));
    GB_HIP(hipMemcpyAsync(B->d_y, y, (size_t)na * 8, hipMemcpyHostToDevice, B->stream));
  }
  // the block table: whole calls, or long calls as speculative segments (chain_split.hip)
  const int st = gbchain::split_plan(B, offsets, x, params4);
  GB_HIP(hipStreamSynchronize(B->stream));  // the caller may free x / y on return
  return st;
}

}  // namespace

namespace gbchain {
// One launch of the sequential kernel over nvc blocks of the block table d_vc, with the small stamp
// ring (small: every block's windows hold <= kRingSmall anchors) or the full one.
int launch_chain(gb_chain_batch *B, const VCall *d_vc, int nvc, int prof, bool small, hipStream_t stream) {
  if (nvc <= 0) return GB_OK;
  Args A;
  A.vc = d_vc;
  A.avg_qspan = B->d_aq;
  A.params4 = B->d_par4;
  A.x = B->d_x;
  A.y = B->d_y;
  const size_t nn = (size_t)std::max<int64_t>(B->nanchors, 1);
  A.score = B->d_out;
  A.parent = B->d_out + nn;
  A.target = B->d_out + 2 * nn;
  A.peak = B->d_out + 3 * nn;
  A.s_score = B->d_sscore;
  A.s_parent = B->d_sparent;
  A.visited = B->d_vis;
  A.prof = prof ? B->d_prof : nullptr;
  A.exp = getenv("GB_CHAIN_EXP") ? atoi(getenv("GB_CHAIN_EXP")) : 0;
  const dim3 g((unsigned)nvc), b(128);
  if (int st = once_per_device(1, [](const DevLimits &L) -> int {
        for (const void *f : {(const void *)chain_kernel<0, kRingSmall>, (const void *)chain_kernel<1, kRingSmall>,
                              (const void *)chain_kernel<2, kRingSmall>, (const void *)chain_kernel<0, kRing>,
                              (const void *)chain_kernel<1, kRing>, (const void *)chain_kernel<2, kRing>})
          GB_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.max_dyn));
        return GB_OK;
      }))
    return st;
  const size_t lds_small = sizeof(uint32_t) * (kRingSmall + 64) + sizeof(Slot) * kSlots + 16;
  const size_t lds_full = sizeof(uint32_t) * (kRing + 64) + sizeof(Slot) * kSlots + 16;
  const size_t dyn = spread_lds(nvc, 2, small ? lds_small : lds_full);
  if (small) {
    if (prof == 2)
      hipLaunchKernelGGL((chain_kernel<2, kRingSmall>), g, b, dyn, stream, A);
    else if (prof == 1)
      hipLaunchKernelGGL((chain_kernel<1, kRingSmall>), g, b, dyn, stream, A);
    else
      hipLaunchKernelGGL((chain_kernel<0, kRingSmall>), g, b, dyn, stream, A);
  } else {
    if (prof == 2)
      hipLaunchKernelGGL((chain_kernel<2, kRing>), g, b, dyn, stream, A);
    else if (prof == 1)
      hipLaunchKernelGGL((chain_kernel<1, kRing>), g, b, dyn, stream, A);
    else
      hipLaunchKernelGGL((chain_kernel<0, kRing>), g, b, dyn, stream, A);
  }
  GB_HIP(hipGetLastError());
  return GB_OK;
}

// The block table of a batch: small-ring blocks first (on the batch's stream), full-ring blocks
// concurrently on the second stream.
int launch_table(gb_chain_batch *B, int prof) {
  if (B->n_rows > 0) {
    // chain_rows blocks on the batch stream (their targets / scratch marks cleared first), the
    // rest (unsorted calls: rare) on the second stream beside them
    const int nr = B->n_rows, nvc = (int)B->vc.size(), ns = B->n_small;
    // (the targets output and the scratch marks were cleared by step_clear)
    if (nr < nvc) {
      GB_HIP(hipEventRecord(B->fj[0], B->stream));
      GB_HIP(hipStreamWaitEvent(B->stream2, B->fj[0], 0));
      if (int st = launch_chain(B, B->d_vc + nr, ns, prof, true, B->stream2)) return st;
      if (int st = launch_chain(B, B->d_vc + nr + ns, nvc - nr - ns, prof, false, B->stream2)) return st;
      GB_HIP(hipEventRecord(B->fj[1], B->stream2));
    }
    if (int st = launch_rows(B, B->d_vc, nr, B->stream)) return st;
    if (nr < nvc) GB_HIP(hipStreamWaitEvent(B->stream, B->fj[1], 0));
    return GB_OK;
  }
  const int nvc = (int)B->vc.size(), ns = B->n_small;
  if (ns < nvc && ns > 0) {
    GB_HIP(hipEventRecord(B->fj[0], B->stream));
    GB_HIP(hipStreamWaitEvent(B->stream2, B->fj[0], 0));
    if (int st = launch_chain(B, B->d_vc + ns, nvc - ns, prof, false, B->stream2)) return st;
    GB_HIP(hipEventRecord(B->fj[1], B->stream2));
    if (int st = launch_chain(B, B->d_vc, ns, prof, true, B->stream)) return st;
    GB_HIP(hipStreamWaitEvent(B->stream, B->fj[1], 0));
    return GB_OK;
  }
  return launch_chain(B, B->d_vc, nvc, prof, ns == nvc, B->stream);
}
}  // namespace gbchain

namespace {
int batch_new(gb_chain_batch **out) {
  auto *B = new gb_chain_batch();
  hipError_t e = hipGetDevice(&B->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&B->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&B->stream2, hipStreamNonBlocking);
  for (auto &ev : B->ev)
    if (e == hipSuccess) e = hipEventCreate(&ev);
  for (auto &ev : B->fj)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&B->fail_ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc(&B->d_vis, sizeof(unsigned long long));
  if (e != hipSuccess) {
    gb::set_error("gb_chain: %s", hipGetErrorString(e));
    gb_chain_batch_destroy(B);
    return GB_ERR_HIP;
  }
  *out = B;
  return GB_OK;
}
}  // namespace

extern "C" {

int gb_chain_batch_create(int64_t ncalls, const int64_t *offsets, const float *avg_qspan,
                          const int32_t *params4, const uint64_t *x, const uint64_t *y,
                          gb_chain_batch **out) {
  GB_ARG(out, "gb_chain_batch_create: null out");
  *out = nullptr;
  int st = validate(ncalls, offsets, avg_qspan, params4, x, y);
  if (st) return st;
  gb_chain_batch *B = nullptr;
  st = batch_new(&B);
  if (st) return st;
  st = batch_fill(B, ncalls, offsets, avg_qspan, params4, x, y);
  if (st) {
    gb_chain_batch_destroy(B);
    return st;
  }
  *out = B;
  return GB_OK;
}

int gb_chain_batch_run(gb_chain_batch *B) {
  gb::Range range_("gb.chain.batch_run");
  GB_ARG(B, "gb_chain_batch_run: null batch");
  GB_HIP(hipSetDevice(B->device));
  GB_HIP(hipEventRecord(B->ev[0], B->stream));
  if (B->n_rows > 0 || !B->split.empty()) {
    if (int st = gbchain::step_clear_launch(B)) return st;
  } else {
    GB_HIP(hipMemsetAsync(B->d_vis, 0, sizeof(unsigned long long), B->stream));
  }
  if (B->ncalls > 0) {
    const char *pe = getenv("GB_CHAIN_PROF");
    const int prof = (pe && (*pe == '1' || *pe == '2')) ? *pe - '0' : 0;
    if (prof) {
      if (!B->d_prof) GB_HIP(hipMalloc(&B->d_prof, 16 * sizeof(unsigned long long)));
      GB_HIP(hipMemsetAsync(B->d_prof, 0, 16 * sizeof(unsigned long long), B->stream));
      GB_HIP(hipMemsetAsync(B->d_prof + 8, 0xff, sizeof(unsigned long long), B->stream));
    }
    if (int st = gbchain::launch_table(B, prof)) return st;
    if (!B->split.empty())
      if (int st = gbchain::split_resolve(B)) return st;
  }
  GB_HIP(hipEventRecord(B->ev[1], B->stream));
  if (B->d_prof && getenv("GB_CHAIN_PROF")) {
    unsigned long long h[16];
    GB_HIP(hipMemcpyAsync(h, B->d_prof, sizeof(h), hipMemcpyDeviceToHost, B->stream));
    GB_HIP(hipStreamSynchronize(B->stream));
    fprintf(stderr, "[chain prof] longest call, memtime ticks: prepare %llu resolve %llu tail %llu; memory passes %llu; "
            "slot misses %llu; walk iterations %llu; total %llu clk / %llu rt ticks = %.0f MHz\n", h[0], h[1], h[2], h[3],
            h[4], h[5], h[6], h[7], h[7] ? 100.0 * (double)h[6] / (double)h[7] : 0.0);
    fprintf(stderr, "[chain prof] grid %.3f ms; longest call starts at %.3f ms, ends at %.3f ms; producer load %llu wait %llu; "
            "resolve: to um %llu, walk %llu\n", (double)(h[11] - h[8]) * 1e-5, (double)(h[9] - h[8]) * 1e-5,
            (double)(h[10] - h[8]) * 1e-5, h[14], h[15], h[12], h[13]);
  }
  B->ran = true;
  return GB_OK;
}

int gb_chain_batch_split_stats(gb_chain_batch *B, int64_t *split_calls, int64_t *rounds, int64_t *fixups) {
  GB_ARG(B, "gb_chain_batch_split_stats: null batch");
  if (split_calls) *split_calls = (int64_t)B->split.size();
  if (rounds) *rounds = B->spec_rounds;
  if (fixups) *fixups = B->fixups;
  return GB_OK;
}

int gb_chain_batch_sync(gb_chain_batch *B) {
  GB_ARG(B, "gb_chain_batch_sync: null batch");
  GB_HIP(hipStreamSynchronize(B->stream));
  return GB_OK;
}

int gb_chain_batch_results(gb_chain_batch *B, int32_t *scores, int32_t *parents, int32_t *targets,
                           int32_t *peak_scores, int64_t *visited) {
  GB_ARG(B && B->ran, "gb_chain_batch_results: batch has not run");
  GB_HIP(hipSetDevice(B->device));
  GB_HIP(hipStreamSynchronize(B->stream));
  const size_t na = (size_t)B->nanchors, nn = (size_t)std::max<int64_t>(B->nanchors, 1);
  int32_t *dst[4] = {scores, parents, targets, peak_scores};
  for (int k = 0; k < 4; k++)
    if (dst[k] && na) GB_HIP(hipMemcpy(dst[k], B->d_out + k * nn, na * 4, hipMemcpyDeviceToHost));
  if (visited) {
    unsigned long long v = 0;
    GB_HIP(hipMemcpy(&v, B->d_vis, sizeof(v), hipMemcpyDeviceToHost));
    *visited = (int64_t)v;
  }
  return GB_OK;
}

int gb_chain_batch_timing(gb_chain_batch *B, float *kernel_ms) {
  GB_ARG(B && B->ran, "gb_chain_batch_timing: batch has not run");
  GB_HIP(hipEventSynchronize(B->ev[1]));
  float ms = 0;
  GB_HIP(hipEventElapsedTime(&ms, B->ev[0], B->ev[1]));
  if (kernel_ms) *kernel_ms = ms;
  return GB_OK;
}

int gb_chain_batch_destroy(gb_chain_batch *B) {
  if (!B) return GB_OK;
  if (B->stream) (void)hipStreamSynchronize(B->stream);
  gbchain::chain_bt_destroy(B->bt);
  gbchain::split_free(B);
  for (void *p : {(void *)B->d_off, (void *)B->d_aq, (void *)B->d_par4, (void *)B->d_x,
                  (void *)B->d_y, (void *)B->d_out, (void *)B->d_vis, (void *)B->d_prof})
    (void)hipFree(p);
  for (auto ev : B->ev)
    if (ev) (void)hipEventDestroy(ev);
  for (auto ev : B->fj)
    if (ev) (void)hipEventDestroy(ev);
  if (B->fail_ev) (void)hipEventDestroy(B->fail_ev);
  if (B->h_fail) (void)hipHostFree(B->h_fail);
  if (B->stream2) (void)hipStreamDestroy(B->stream2);
  if (B->stream) (void)hipStreamDestroy(B->stream);
  delete B;
  return GB_OK;
}

int gb_chain(int64_t ncalls, const int64_t *offsets, const float *avg_qspan, const int32_t *params4,
             const uint64_t *x, const uint64_t *y, int32_t *scores, int32_t *parents, int32_t *targets,
             int32_t *peak_scores) {
  // one cached batch per (host thread, device): repeated host_chain_kernel calls reuse its stream,
  // events and grow-only buffers. Never freed (freeing at thread exit could run after the HIP
  // runtime is torn down).
  int st = validate(ncalls, offsets, avg_qspan, params4, x, y);
  if (st) return st;
  thread_local std::vector<std::pair<int, gb_chain_batch *>> ws;
  int dev = 0;
  GB_HIP(hipGetDevice(&dev));
  gb_chain_batch *B = nullptr;
  for (auto &w : ws)
    if (w.first == dev) B = w.second;
  if (!B) {
    if ((st = batch_new(&B))) return st;
    ws.emplace_back(dev, B);
  }
  const bool hp = getenv("GB_CHAIN_HOSTPROF") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  if ((st = batch_fill(B, ncalls, offsets, avg_qspan, params4, x, y))) return st;
  const auto t1 = std::chrono::steady_clock::now();
  st = gb_chain_batch_run(B);
  if (!st && hp) st = gb_chain_batch_sync(B);
  const auto t2 = std::chrono::steady_clock::now();
  if (!st) st = gb_chain_batch_results(B, scores, parents, targets, peak_scores, nullptr);
  if (hp) {
    const auto t3 = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr, "[gb_chain] fill (validate, H2D, plan) %.2f ms, run %.2f ms, results %.2f ms\n", ms(t0, t1),
            ms(t1, t2), ms(t2, t3));
  }
  return st;
}

}  // extern "C"
