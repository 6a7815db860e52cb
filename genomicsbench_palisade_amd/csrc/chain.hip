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
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <numeric>
#include <vector>

#include "../../include/gb_chain.h"
#include "gb_common.h"
#include "chain_internal.h"

namespace gbchain {

constexpr int kRing = 8192;     // stamp ring >= max_iter (5000) + 64 candidates
constexpr int kMaxIter = 5000;  // host_kernel.cpp:41
constexpr int kMaxSkip = 25;    // host_kernel.cpp:42

struct Args {
  const int64_t *offsets;
  const float *avg_qspan;
  const int32_t *params4;
  const uint64_t *x, *y;
  const int32_t *order;  // calls, longest first
  int32_t *score, *parent, *target, *peak;
  unsigned long long *visited;
  unsigned long long *prof;  // optional phase clocks (GB_CHAIN_PROF=1), see chain_kernel
  int32_t prof_call;         // the call whose consumer also records shader-clock and 100 MHz ticks
};

__device__ __forceinline__ int ilog2_32(uint32_t v) { return 31 - __clz((int)v); }  // v > 0 (LogTable256)

__device__ __forceinline__ int dpp_shr_i32(int v, int lane0) {
  return __builtin_amdgcn_update_dpp(lane0, v, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ __forceinline__ uint64_t dpp_shr_u64(uint64_t v, uint64_t lane0) {
  const int lo = dpp_shr_i32((int)(uint32_t)v, (int)(uint32_t)lane0);
  const int hi = dpp_shr_i32((int)(uint32_t)(v >> 32), (int)(uint32_t)(lane0 >> 32));
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// anchors are read-only for the whole kernel: the constant address space turns the uniform X[st]
// reads of the window-start loop into scalar loads (lgkmcnt), so they never wait behind the
// wave's outstanding score/parent/peak stores (vmcnt)
typedef const __attribute__((address_space(4))) uint64_t const_u64;

// wave-wide inclusive scans with DPP (row_shr 1/2/4/8 inside 16-lane rows, then row_bcast 15/31)
__device__ __forceinline__ int32_t scan_max(int32_t v) {
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x111, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x112, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x114, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x118, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x142, 0xA, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x143, 0xC, 0xF, false));
  return v;
}
__device__ __forceinline__ int32_t scan_min(int32_t v) {
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x111, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x112, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x114, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x118, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x142, 0xA, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x143, 0xC, 0xF, false));
  return v;
}
__device__ __forceinline__ int32_t load_l2(const int32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load sc1 (bypasses L1)
}

// Pair geometry of anchor i against candidate j (host_kernel.cpp:55-82 without score[j]): whether j
// passes the filters, and s = min(q_span, dq, dr) (+1 paired bonus) - gap_cost.
__device__ __forceinline__ bool geometry(uint64_t xi, uint64_t yi, uint64_t xj, uint64_t yj, bool valid,
                                         int max_dist_x, int max_dist_y, int bw, int n_segs, double avg_qspan,
                                         int32_t &sg) {
  const int32_t qi = (int32_t)yi, q_span = (int32_t)(yi >> 32 & 0xff);
  const int32_t sidi = (int32_t)((yi & (0xffull << 48)) >> 48);
  const int64_t dr = (int64_t)(xi - xj);
  const int32_t dq = qi - (int32_t)yj;
  const int32_t sidj = (int32_t)((yj & (0xffull << 48)) >> 48);
  const bool same = sidi == sidj;
  const int32_t dd = (int32_t)(dr > dq ? dr - dq : dq - dr);
  // bitwise predicates and selects throughout: per-lane branches would cost exec-mask regions
  const bool ok = valid & !((same & (dr == 0)) | (dq <= 0)) & !((same & (dq > max_dist_y)) | (dq > max_dist_x)) &
                  !(same & (dd > bw)) & !((n_segs > 1) & same & (dr > max_dist_y));  // is_cdna = 0
  const int32_t min_d = (int32_t)(dq < dr ? (int64_t)dq : dr);
  const int log_dd = dd ? ilog2_32((uint32_t)dd) : 0;
  const int c_lin = (int)((double)dd * .01 * avg_qspan);
  const int32_t s0 = min_d > q_span ? q_span : min_d;
  // different sequences: +1 on dr == 0 and gap min(c_lin, log_dd) unless dr == 0; same: c_lin + log_dd/2
  const int32_t gap_diff = dr == 0 ? 0 : (c_lin < log_dd ? c_lin : log_dd);
  const int32_t gap_same = c_lin + (log_dd >> 1);
  const int32_t bonus = (!same & (dr == 0)) ? 1 : 0;
  // (int)((double)gap_cost * gap_scale + .499) with gap_scale == 1.0f (host_kernel.cpp:36) is
  // gap_cost itself for 0 <= gap_cost < 2^31
  sg = s0 + bonus - (same ? gap_same : gap_diff);
  return ok;
}

constexpr int32_t kNoCand = INT_MIN;  // sg of a filtered candidate (producer -> consumer)

// One 64-candidate step in visiting order (lane l = j = jtop - l): running max_f, n_skip, the
// break and the targets/stamps. sc is INT_MIN on filtered lanes (ok false). Updates M, J, N;
// returns whether the step broke. Indices are int32 (calls hold < 2^30 anchors, checked at batch
// creation) so uniform compares stay on the SALU, and the step has no exec-mask branch: lanes with
// nothing to mark stamp a private dummy word S[kRing + lane], and the targets store is a buffer
// store whose disabled lanes carry an out-of-range offset.
__device__ __forceinline__ bool resolve_step(int32_t sc, bool ok, int32_t pj, int32_t jtop, int32_t st, uint32_t stamp,
                                             int lane, int32_t neg_lane, __amdgpu_buffer_rsrc_t trs, int32_t i,
                                             uint32_t *S, int32_t &M, int32_t &J, int32_t &N, uint32_t &vis) {
  // "targets[j] == i": stamps from visited j' > j with parents[j'] == j. A stamp can only match a
  // lane whose j >= st (|pj - j| < kRing, so equal ring slots mean pj == j), so no validity test
  S[(ok & (pj >= st)) ? (pj & (kRing - 1)) : kRing + lane] = stamp;
  const bool tgt = S[(jtop - lane) & (kRing - 1)] == stamp;
  const int32_t mx = scan_max(sc);  // inclusive max scan
  const int32_t before = max(dpp_shr_i32(mx, INT_MIN), M);
  const bool upd = sc > before;  // false on filtered lanes: before >= M >= 0 > INT_MIN
  const bool plus = ok & !upd & tgt;
  const uint64_t um_all = __builtin_amdgcn_ballot_w64(upd), pm = __builtin_amdgcn_ballot_w64(plus);
  // n_skip after lane l as a reflected walk: steps +1 (target, no update), -1 floored at 0 (update),
  // so n_l = max(N + D_l, D_l - min_{k<=l} D_k) with D_l the inclusive step sum. Exclusive part:
  // mbcnt(pm) - mbcnt(um) = mbcnt(pm) + mbcnt(~um) - lane, one mbcnt chain
  const uint64_t num = ~um_all;
  const int32_t d_ex = (int32_t)__builtin_amdgcn_mbcnt_hi(
      (uint32_t)(num >> 32),
      __builtin_amdgcn_mbcnt_lo((uint32_t)num, __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)pm, (uint32_t)neg_lane))));
  const int32_t D = d_ex + (plus ? 1 : (upd ? -1 : 0));
  const int32_t n_after = max(N + D, D - scan_min(D));
  const uint64_t bm = __builtin_amdgcn_ballot_w64(plus & (n_after > kMaxSkip));
  const uint64_t below = (bm - 1) & ~bm;  // lanes before the break (all lanes when none)
  const int32_t nvalid = min(64, jtop - st + 1);
  vis += bm ? (uint32_t)__builtin_ctzll(bm) + 1 : (uint32_t)nvalid;
  const uint64_t um = um_all & below;
  const int lu = 63 - __builtin_clzll(um | 1);  // last improving lane before the break (when um != 0)
  const int32_t m_lu = __builtin_amdgcn_readlane(mx, lu);
  J = um ? jtop - lu : J;
  M = um ? m_lu : M;
  const bool wt = ok & (bool)((below >> lane) & 1) & (pj >= 0);
  __builtin_amdgcn_raw_buffer_store_b32(i, trs, wt ? (uint32_t)pj * 4u : 0xFFFFFFFFu, 0, 0);
  N = __builtin_amdgcn_readlane(n_after, 63);
  return bm != 0;
}

// Producer -> consumer hand-off, one slot per anchor i: the geometry of its first 64 candidates.
// seq = i + 1 is written last and read first, so a slot whose seq matches is complete.
constexpr int kSlots = 16;
struct Slot {
  int32_t sg[64];  // kNoCand for filtered candidates
  int32_t seq, st, q_span, pad;
};

__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32;
}

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
template <int PROF>
__global__ __launch_bounds__(128) void chain_kernel(Args A) {
  __shared__ uint32_t S[kRing + 64];
  __shared__ Slot ring[kSlots];
  __shared__ uint64_t xyblk[2][2][64];  // producer's staged anchor blocks: [b & 1][x | y][k]
  __shared__ int consumed;
  const int c = A.order[blockIdx.x];
  const int lane = threadIdx.x & 63;
  const bool producer = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) != 0;  // wave-uniform role
  const int64_t o = A.offsets[c];
  const int32_t n = __builtin_amdgcn_readfirstlane((int32_t)(A.offsets[c + 1] - o));
  const int max_dist_x = A.params4[4 * c], max_dist_y = A.params4[4 * c + 1];
  const int bw = A.params4[4 * c + 2], n_segs = A.params4[4 * c + 3];
  const double avg_qspan = (double)A.avg_qspan[c];
  const uint64_t *X = A.x + o, *Y = A.y + o;
  const const_u64 *XC = (const const_u64 *)X;
  int32_t *score = A.score + o, *parent = A.parent + o, *target = A.target + o, *peak = A.peak + o;

  for (int k = threadIdx.x; k < kRing + 64; k += 128) S[k] = 0;
  for (int32_t k = threadIdx.x; k < n; k += 128) target[k] = 0;  // a fresh std::vector in the reference
  if (threadIdx.x < kSlots) ring[threadIdx.x].seq = 0;
  if (threadIdx.x == 0) consumed = 0;
  __builtin_amdgcn_s_waitcnt(0);  // zeroing stores complete before any later targets store
  __syncthreads();

  if (producer) {
    // ---------------- producer: geometry of anchor i against i-1-lane --------------------------
    uint64_t wx = 0, wy = 0;  // lane l: anchor i-1-l
    int32_t st = 0;
    const bool pc = PROF == 2 && c == A.prof_call;
    unsigned long long p_load = 0, p_wait = 0, t0 = 0;
    // Anchors x/y reach the producer through LDS, a 64-anchor block ahead: at the start of block
    // b the block loaded at the start of b-1 (one coalesced load per array; its only wait is here)
    // goes into xy[b & 1], and block b+1 is requested. No load sits on the per-anchor path, which
    // keeps the producer ahead when L2/HBM are busy with other calls. The window start's x is kept
    // in SGPRs and refreshed by a scalar load only when st advances.
    uint64_t nx = X[min(lane, n - 1)], ny = Y[min(lane, n - 1)];
    uint64_t xst = n > 0 ? XC[0] : 0;
    for (int32_t iv = 0; iv < n; iv++) {
      // opaque to loop strength reduction, which otherwise derives i from the per-lane i-1-lane
      // (a VGPR induction variable) and turns every uniform value below into a vector one
      const int32_t i = __builtin_amdgcn_readfirstlane(iv);
      if (pc) t0 = __builtin_amdgcn_s_memtime();
      if ((i & 63) == 0) {
        xyblk[(i >> 6) & 1][0][lane] = nx;
        xyblk[(i >> 6) & 1][1][lane] = ny;
        nx = X[min(i + 64 + lane, n - 1)];
        ny = Y[min(i + 64 + lane, n - 1)];
      }
      const uint64_t xi = rfl64(xyblk[(i >> 6) & 1][0][i & 63]), yi = rfl64(xyblk[(i >> 6) & 1][1][i & 63]);
      while (st < i && xi > xst + (uint64_t)(int64_t)max_dist_x) xst = XC[++st];
      if (i - st > kMaxIter) {  // rare: > max_iter candidates in range
        st = i - kMaxIter;
        xst = XC[st];
      }
      if (pc) {
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        p_load += t1 - t0;
      }
      int32_t sg;
      const bool ok = geometry(xi, yi, wx, wy, i - 1 - lane >= st, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sg);
      // wait for a free slot
      if (pc) t0 = __builtin_amdgcn_s_memtime();
      while (i - lds_count(&consumed) >= kSlots) __builtin_amdgcn_s_sleep(1);
      if (pc) p_wait += __builtin_amdgcn_s_memtime() - t0;
      Slot &sl = ring[i & (kSlots - 1)];
      sl.sg[lane] = ok ? sg : kNoCand;
      if (lane == 0) {
        sl.st = st;
        sl.q_span = (int32_t)(yi >> 32 & 0xff);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // slot contents land before the seq that publishes them
      if (lane == 0) __hip_atomic_store(&sl.seq, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      wx = dpp_shr_u64(wx, xi);
      wy = dpp_shr_u64(wy, yi);
    }
    if (pc && lane == 0) {
      atomicAdd(A.prof + 12, p_load);
      atomicAdd(A.prof + 13, p_wait);
    }
    return;
  }

  // ---------------- consumer ---------------------------------------------------------------------
  const bool pc = PROF == 2 && c == A.prof_call;  // phase clocks for the profiled call only
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(target, (short)0, n * 4, 0x00020000);
  const int32_t neg_lane = -lane;
  int32_t ws = 0, wpar = -1, wpk = 0;  // lane l: score/parent/peak of anchor i-1-l
  unsigned long long vis = 0;
  unsigned long long c_head = 0, c_step = 0, c_tail = 0, n_step = 0, n_miss = 0, c_miss = 0, t_0 = 0, t_1 = 0;
  // slot i is read during step i-1 (header first: LDS executes a wave's reads in order, so a
  // matching seq means the sg read after it saw the complete slot)
  // volatile LDS (address space 3) reads: kept in program order (seq before sg) and still ds_read
  typedef int32_t v4i __attribute__((ext_vector_type(4)));
  typedef volatile __attribute__((address_space(3))) v4i lds_v4i;
  typedef volatile __attribute__((address_space(3))) int32_t lds_i32;
  v4i hdr = *(lds_v4i *)&ring[0].seq;
  int32_t psg = *(lds_i32 *)&ring[0].sg[lane];
  unsigned long long clk0 = 0, rt0 = 0;
  if (PROF) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int32_t base = 0; base < n; base += 64) {
    const int32_t cnt = min(64, n - base);
    for (int32_t k = 0; k < cnt; k++) {
      const int32_t i = __builtin_amdgcn_readfirstlane(base + k);
      if (pc) t_0 = __builtin_amdgcn_s_memtime();
      int32_t st, q_span, sg;
      if (__builtin_amdgcn_readfirstlane(hdr.x) == i + 1) {
        st = __builtin_amdgcn_readfirstlane(hdr.y);
        q_span = __builtin_amdgcn_readfirstlane(hdr.z);
        sg = psg;
      } else {  // the producer was behind when the slot was read ahead: wait for it, read again
        if (pc) {
          ++n_miss;
          t_1 = __builtin_amdgcn_s_memtime();
        }
        Slot &sl = ring[i & (kSlots - 1)];
        while (lds_count(&sl.seq) != i + 1) __builtin_amdgcn_s_sleep(1);
        if (pc) c_miss += __builtin_amdgcn_s_memtime() - t_1;
        st = __builtin_amdgcn_readfirstlane(*(lds_i32 *)&sl.st);
        q_span = __builtin_amdgcn_readfirstlane(*(lds_i32 *)&sl.q_span);
        sg = *(lds_i32 *)&sl.sg[lane];
      }
      // free slot i (its reads were issued before this write, and LDS runs them in order), then
      // read slot i+1 ahead; its latency overlaps this step
      if (lane == 0) __hip_atomic_store(&consumed, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      {
        Slot &nl = ring[(i + 1) & (kSlots - 1)];
        hdr = *(lds_v4i *)&nl.seq;
        psg = *(lds_i32 *)&nl.sg[lane];
      }
      const bool ok = sg != kNoCand;
      int32_t M = q_span, N = 0, J = -1;
      const uint32_t stamp = (uint32_t)(i + 1);
      uint32_t vis_i = 0;
      if (pc) {
        t_1 = __builtin_amdgcn_s_memtime();
        c_head += t_1 - t_0;
        t_0 = t_1;
      }
      const int32_t jtop = i - 1;
      bool brk = false;
      if (jtop >= st) {
        if (pc) ++n_step;
        const int32_t sc = ok ? (int32_t)((uint32_t)sg + (uint32_t)ws) : INT_MIN;
        brk = resolve_step(sc, ok, wpar, jtop, st, stamp, lane, neg_lane, trs, i, S, M, J, N, vis_i);
      }
      if (!brk && jtop - 64 >= st) {  // rare: older candidates (j < i-64) from memory
        // the wave's flushed score/parent stores reach L2 before these sc1 reads of them (the
        // drain sits here, not at every flush, so the common path never waits on a store)
        __builtin_amdgcn_s_waitcnt(0);
        const uint64_t xi = X[i], yi = Y[i];
        for (int32_t jt = jtop - 64; jt >= st; jt -= 64) {
          if (pc) ++n_step;
          const int32_t jj = jt - lane;
          const bool v = jj >= st;
          uint64_t xj = 0, yj = 0;
          int32_t scj = 0, pj = -1;
          if (v) {
            xj = X[jj];
            yj = Y[jj];
            scj = load_l2(score + jj);
            pj = load_l2(parent + jj);
          }
          int32_t sgo;
          const bool oko = geometry(xi, yi, xj, yj, v, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sgo);
          if (resolve_step(oko ? sgo + scj : INT_MIN, oko, pj, jt, st, stamp, lane, neg_lane, trs, i, S, M, J, N,
                           vis_i))
            break;
        }
      }
      vis += vis_i;
      if (pc) {
        t_1 = __builtin_amdgcn_s_memtime();
        c_step += t_1 - t_0;
        t_0 = t_1;
      }
      // peak of the parent: from the register window when J >= i-64, else (rare) from memory
      const int32_t dJ = i - 1 - J;
      int32_t pkJ = __builtin_amdgcn_readlane(wpk, dJ & 63);
      if (J >= 0 && dJ > 63) pkJ = __builtin_amdgcn_readfirstlane(load_l2(peak + J));
      const int32_t pki = (J >= 0 && pkJ > M) ? pkJ : M;
      ws = dpp_shr_i32(ws, M);
      wpar = dpp_shr_i32(wpar, J);
      wpk = dpp_shr_i32(wpk, pki);
      if (pc) c_tail += __builtin_amdgcn_s_memtime() - t_0;
    }
    // flush the window: anchors base .. base+cnt-1 (lane l: base+cnt-1-l)
    if (lane < cnt) {
      score[base + cnt - 1 - lane] = ws;
      parent[base + cnt - 1 - lane] = wpar;
      peak[base + cnt - 1 - lane] = wpk;
    }
  }
  if (PROF && lane == 0) {
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
    atomicMin(A.prof + 8, rt0);
    atomicMax(A.prof + 11, rt1);
    if (c == A.prof_call) {
      atomicAdd(A.prof + 9, rt0);
      atomicAdd(A.prof + 10, rt1);
    }
  }
  if (pc && lane == 0) {
    atomicAdd(A.prof + 0, c_head);
    atomicAdd(A.prof + 1, c_step);
    atomicAdd(A.prof + 2, c_tail);
    atomicAdd(A.prof + 3, n_step);
    atomicAdd(A.prof + 4, n_miss);
    atomicAdd(A.prof + 5, c_miss);
    if (c == A.prof_call) {
      atomicAdd(A.prof + 6, __builtin_amdgcn_s_memtime() - clk0);
      atomicAdd(A.prof + 7, __builtin_amdgcn_s_memrealtime() - rt0);
    }
  }
  // every lane accumulated the same (uniform) count
  if (lane == 0) atomicAdd(A.visited, vis);
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
  // longest calls first: the grid is dispatched in order, so the critical path starts first
  std::vector<int32_t> order((size_t)ncalls);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    return offsets[a + 1] - offsets[a] > offsets[b + 1] - offsets[b];
  });
  GB_HIP(hipSetDevice(B->device));
  GB_HIP(hipStreamSynchronize(B->stream));  // the previous contents may still be in use
  gbchain::chain_bt_destroy(B->bt);
  B->bt = nullptr;
  B->ran = false;
  const int64_t nc = std::max<int64_t>(ncalls, 1), nn = std::max<int64_t>(na, 1);
  if (nc > B->cap_calls) {
    for (void *q : {(void *)B->d_off, (void *)B->d_aq, (void *)B->d_par4, (void *)B->d_order}) (void)hipFree(q);
    B->d_off = nullptr, B->d_aq = nullptr, B->d_par4 = nullptr, B->d_order = nullptr;
    B->cap_calls = 0;
    GB_HIP(hipMalloc(&B->d_off, (size_t)(nc + 1) * sizeof(int64_t)));
    GB_HIP(hipMalloc(&B->d_aq, (size_t)nc * sizeof(float)));
    GB_HIP(hipMalloc(&B->d_par4, (size_t)nc * 4 * sizeof(int32_t)));
    GB_HIP(hipMalloc(&B->d_order, (size_t)nc * sizeof(int32_t)));
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
    GB_HIP(hipMemcpy(B->d_order, order.data(), (size_t)ncalls * 4, hipMemcpyHostToDevice));
  }
  if (na) {
    GB_HIP(hipMemcpy(B->d_x, x, (size_t)na * 8, hipMemcpyHostToDevice));
    GB_HIP(hipMemcpy(B->d_y, y, (size_t)na * 8, hipMemcpyHostToDevice));
  }
  return GB_OK;
}

int batch_new(gb_chain_batch **out) {
  auto *B = new gb_chain_batch();
  hipError_t e = hipGetDevice(&B->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&B->stream, hipStreamNonBlocking);
  for (auto &ev : B->ev)
    if (e == hipSuccess) e = hipEventCreate(&ev);
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
  GB_HIP(hipMemsetAsync(B->d_vis, 0, sizeof(unsigned long long), B->stream));
  GB_HIP(hipEventRecord(B->ev[0], B->stream));
  if (B->ncalls > 0) {
    gbchain::Args A;
    A.offsets = B->d_off;
    A.avg_qspan = B->d_aq;
    A.params4 = B->d_par4;
    A.x = B->d_x;
    A.y = B->d_y;
    A.order = B->d_order;
    const size_t nn = (size_t)std::max<int64_t>(B->nanchors, 1);
    A.score = B->d_out;
    A.parent = B->d_out + nn;
    A.target = B->d_out + 2 * nn;
    A.peak = B->d_out + 3 * nn;
    A.visited = B->d_vis;
    A.prof = nullptr;
    A.prof_call = -1;
    const char *pe = getenv("GB_CHAIN_PROF");
    const int prof = (pe && (*pe == '1' || *pe == '2')) ? *pe - '0' : 0;
    if (prof) {
      if (!B->d_prof) GB_HIP(hipMalloc(&B->d_prof, 14 * sizeof(unsigned long long)));
      GB_HIP(hipMemsetAsync(B->d_prof, 0, 14 * sizeof(unsigned long long), B->stream));
      GB_HIP(hipMemsetAsync(B->d_prof + 8, 0xff, sizeof(unsigned long long), B->stream));
      A.prof = B->d_prof;
      int32_t c0 = 0;
      GB_HIP(hipMemcpy(&c0, B->d_order, sizeof(c0), hipMemcpyDeviceToHost));
      A.prof_call = c0;
    }
    if (prof == 2)
      hipLaunchKernelGGL(gbchain::chain_kernel<2>, dim3((unsigned)B->ncalls), dim3(128), 0, B->stream, A);
    else if (prof == 1)
      hipLaunchKernelGGL(gbchain::chain_kernel<1>, dim3((unsigned)B->ncalls), dim3(128), 0, B->stream, A);
    else
      hipLaunchKernelGGL(gbchain::chain_kernel<0>, dim3((unsigned)B->ncalls), dim3(128), 0, B->stream, A);
    GB_HIP(hipGetLastError());
  }
  GB_HIP(hipEventRecord(B->ev[1], B->stream));
  if (B->d_prof && getenv("GB_CHAIN_PROF")) {
    unsigned long long h[14];
    GB_HIP(hipMemcpyAsync(h, B->d_prof, sizeof(h), hipMemcpyDeviceToHost, B->stream));
    GB_HIP(hipStreamSynchronize(B->stream));
    fprintf(stderr, "[chain prof] memtime ticks: head %llu steps %llu tail %llu; steps %llu; slot misses %llu (%llu ticks); "
            "longest call %llu clk / %llu rt ticks = %.0f MHz\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7],
            h[7] ? 100.0 * (double)h[6] / (double)h[7] : 0.0);
    fprintf(stderr, "[chain prof] grid %.3f ms; longest call starts at %.3f ms, ends at %.3f ms; producer load %llu wait %llu\n",
            (double)(h[11] - h[8]) * 1e-5, (double)(h[9] - h[8]) * 1e-5, (double)(h[10] - h[8]) * 1e-5, h[12], h[13]);
  }
  B->ran = true;
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
  for (void *p : {(void *)B->d_off, (void *)B->d_aq, (void *)B->d_par4, (void *)B->d_order, (void *)B->d_x,
                  (void *)B->d_y, (void *)B->d_out, (void *)B->d_vis, (void *)B->d_prof})
    (void)hipFree(p);
  for (auto ev : B->ev)
    if (ev) (void)hipEventDestroy(ev);
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
  if ((st = batch_fill(B, ncalls, offsets, avg_qspan, params4, x, y))) return st;
  st = gb_chain_batch_run(B);
  if (!st) st = gb_chain_batch_results(B, scores, parents, targets, peak_scores, nullptr);
  return st;
}

}  // extern "C"
