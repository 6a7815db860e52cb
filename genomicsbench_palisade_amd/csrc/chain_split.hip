// chain_split.hip -- long chain_dp calls as speculative segments, resolved exactly.
//
// chain_dp (minimap2-acceleration kernel/scalar/src/host_kernel.cpp:30-94) is sequential in the
// anchors of a call: score[i] needs score[j] for j in i's window. One call per block makes the
// longest call the bound of a whole set (an 87 k-anchor call takes as long as 10 000 calls). A call
// of >= 2 * kSeg anchors whose x are sorted (minimap2 sorts them) is therefore cut into segments
// [c_s, e_s) of kSeg anchors, and segment s >= 1 runs as its own block from a warm-up anchor a_s
// before its window (a_s = st(c_s) - kWarm: with sorted x the window start st(i) is a function of
// i alone, max(first j with x_i <= x_j + max_dist_x, i - max_iter), so the segment's loops see
// exactly the reference's candidates). Its scores are then off by the unknown score of the chains
// it continues, so:
//
//  1. guess: score[i] ~ score[p] + (spec[i] - spec[p]) along the speculative parents p, resolved by
//     pointer jumping back to a known score (segment 0 is exact) or a chain start;
//  2. verify: every anchor's loop is re-run in parallel (one wave per 64 anchors) against the
//     guessed scores and parents of its window; by induction over i, an anchor whose loop yields
//     its own guess is exact as long as all earlier anchors are, so the first mismatch bounds what
//     is final;
//  3. fix-up: from a mismatch, kFix anchors are recomputed by the sequential kernel with the final
//     anchors before them loaded (kVFixup), and 1-2 repeat from there (rare: the chains of the
//     warm-up have converged to the reference's well before c_s on the data measured);
//  4. peaks by pointer jumping (peak[i] = max(score[i], peak[parent[i]])), then the targets marks
//     and visited counts of the split anchors by one more parallel pass (atomic max: the last
//     marker of an anchor is the largest i).
//
// The results are those of the sequential loop, bit for bit; tests/test_chain.py forces tiny
// segments and no warm-up to drive every fix-up path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/gb_chain.h"
#include "gb_common.h"
#include "chain_dev.h"
#include "chain_internal.h"

namespace gbchain {

constexpr int kSegDefault = 4096;   // longest segment
// warm-up anchors before the window of a segment's first anchor. Measured (tools/chain_knob_probe.py,
// profiles/r04zj_chain_warm_ab.log): 128 -> 32 takes the 1/8 shard from 1.47 to 1.37 ms and 'large'
// from 5.09 to 5.06 ms; 16 and 8 also guess right on both sets, 0 fails (3 fix-ups, shard 2.16 ms),
// so 32 keeps a margin for sets whose loops reach further back
constexpr int kWarmDefault = 32;
// A segment's block starts kWarm anchors before the window of its first anchor, but at most kWinCap
// anchors of that window: the window is every anchor within max_dist_x (up to max_iter = 5000 in
// dense regions, median ~500 on the bench's sets) while the reference loop stops after ~30
// candidates (it visits at most 586 on the 'large' set, tests/host walk), so the rest of a wide
// window only lengthened the block. A loop that does reach past the block start is caught by the
// verification like any other wrong guess. Measured (tools/chain_knob_probe.py, r04c): cap 512 takes
// the 1/8 shard from 1.62 to 1.53 ms and 'large' from 5.37 to 5.30 ms with no failed guess; 256 made
// guesses fail (2 fix-ups on both sets, 3.5 / 7.9 ms).
constexpr int kWinCapDefault = 512;
constexpr int kFix = 1024;          // anchors recomputed sequentially after a failed guess
constexpr int kTagRing = 1024;      // verification stamp ring (tagged, see resolve_tagged)

struct SplitArgs {
  const SplitCall *split;
  const Seg *segs;
  const Chunk *chunks;
  const int32_t *st;
  const int32_t *front;
  int32_t *fail;
  const float *avg_qspan;
  const int32_t *params4;
  const uint64_t *x, *y;
  int32_t *score, *parent, *target, *peak;
  const int32_t *s_score, *s_parent;
  unsigned long long *visited;
  int32_t *t2;                   // the split anchors' targets marks (atomic max), merged at the end
  unsigned long long *viscall;   // visited pairs per split call
  int32_t fault;  // GB_CHAIN_SPLIT_FAULT (tests): guesses of every fault-th anchor are made wrong
  int32_t *slow;  // [0]: chunks verify_lanes leaves anchors of to verify_kernel, [1..]: the chunks
  int32_t nch;    // chunks
};

__device__ __forceinline__ int32_t cidx(const SplitCall &S, int32_t i) { return 64 * S.cbase + (i - S.c1); }

// 1. guess: per split anchor i >= front, its speculative parent p and the link / value pair of
// g[i] = g[link] + val (link -1: val is g[i]).
__global__ __launch_bounds__(64) void guess_init(SplitArgs A, int32_t *link, int32_t *val) {
  const Chunk ch = A.chunks[blockIdx.x];
  const SplitCall S = A.split[ch.sc];
  const int32_t i = ch.start + (int32_t)threadIdx.x, j = 64 * blockIdx.x + threadIdx.x;
  const int32_t front = A.front[ch.sc];
  if (i >= S.n || i < front) {
    link[j] = -1;
    val[j] = 0;
    return;
  }
  const int32_t s = min(i / S.c1, S.nseg - 1);  // segments are c1 anchors long, the last one shorter
  const Seg G = A.segs[S.seg0 + s];
  const int32_t fs = A.s_score[G.soff + (i - G.as)], q = A.s_parent[G.soff + (i - G.as)];
  const int32_t p = q >= 0 ? q + G.as : -1;
  A.parent[S.off + i] = p;
  int32_t l = -1, v = fs;
  if (p >= 0) {
    const int32_t d = fs - A.s_score[G.soff + (p - G.as)];
    if (p < front) {
      v = A.score[S.off + p] + d;
    } else {
      l = cidx(S, p);
      v = d;
    }
  }
  // fault injection (tests only): a wrong guess must be caught by the verification and repaired
  // by the fix-up, whatever the spec run found
  if (A.fault > 0 && i % A.fault == A.fault / 2) v += 1;
  link[j] = l;
  val[j] = v;
}

// The clears of one step in one launch (each hipMemset is a dispatch of its own, ~5 us at the launch
// floor, and a step had eight of them): the targets output and chain_rows' scratch marks before the
// blocks run, and the split resolution's first-round state -- t2 marks, per-call visited counts,
// failure flags, verify_kernel's work-list count, front = c1 (was a host copy per step).
__global__ __launch_bounds__(256) void step_clear(SplitArgs A, int32_t *targets, int64_t nanchors, int32_t *smark,
                                                  int64_t scratch_n, unsigned long long *vis, int32_t ns,
                                                  int32_t *front) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
  for (int64_t i = t; i < nanchors; i += stride) {
    targets[i] = 0;
    if (ns > 0) A.t2[i] = 0;
  }
  for (int64_t i = t; i < scratch_n; i += stride) smark[i] = 0;
  for (int64_t k = t; k < ns; k += stride) {
    front[k] = A.split[k].c1;
    A.fail[k] = 0x7f7f7f7f;
    A.viscall[k] = 0;
  }
  if (t == 0) {
    *vis = 0;
    if (ns > 0) A.slow[0] = 0;
  }
}

// one pointer-jumping round: OP 0 adds (guesses), OP 1 takes the maximum (peaks)
template <int OP>
__global__ __launch_bounds__(256) void jump_round(int64_t n, const int32_t *li, const int32_t *vi, int32_t *lo,
                                                  int32_t *vo) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const int32_t l = li[j];
  int32_t v = vi[j];
  if (l >= 0) {
    v = OP == 0 ? v + vi[l] : max(v, vi[l]);
    lo[j] = li[l];
  } else {
    lo[j] = -1;
  }
  vo[j] = v;
}

// Links inside one kTile-entry tile of the chunk space first: doubling rounds in LDS (until no link
// stays inside the tile, at most log2(kTile)) leave every entry with its first link outside its tile
// (links point to earlier anchors of the same call) and the value folded up to it, so the global
// rounds that follow count hops between tiles, not anchors: a path of a call of n split anchors
// crosses at most n / kTile + 2 tiles. 4096-entry tiles (1024 threads, 4 entries each, 64 KB of
// LDS): 'large' needs 5 global rounds per direction instead of 8 with 1024-entry tiles.
constexpr int kTile = 4096, kTileLog = 12, kTileThreads = 1024, kTilePer = kTile / kTileThreads;
template <int OP>
__global__ __launch_bounds__(kTileThreads) void jump_local(int64_t nj, int32_t *link, int32_t *val) {
  __shared__ int32_t ll[2][kTile], lv[2][kTile];
  const int64_t base = (int64_t)kTile * blockIdx.x;
#pragma unroll
  for (int q = 0; q < kTilePer; q++) {
    const int32_t t = (int32_t)threadIdx.x + q * kTileThreads;
    const bool in = base + t < nj;
    ll[0][t] = in ? link[base + t] : -1;
    lv[0][t] = in ? val[base + t] : 0;
  }
  __syncthreads();
  int cur = 0;
  for (int r = 0; r < kTileLog; r++) {
    int inside = 0;
#pragma unroll
    for (int q = 0; q < kTilePer; q++) {
      const int32_t t = (int32_t)threadIdx.x + q * kTileThreads;
      const int32_t l = ll[cur][t];
      int32_t v = lv[cur][t], nl = l;
      if (l >= base && l < base + kTile) {
        const int32_t w = lv[cur][l - base];
        v = OP == 0 ? v + w : max(v, w);
        nl = ll[cur][l - base];
        inside |= nl >= base && nl < base + kTile;
      }
      ll[cur ^ 1][t] = nl;
      lv[cur ^ 1][t] = v;
    }
    cur ^= 1;
    if (!__syncthreads_or(inside)) break;
  }
#pragma unroll
  for (int q = 0; q < kTilePer; q++) {
    const int32_t t = (int32_t)threadIdx.x + q * kTileThreads;
    if (base + t < nj) {
      link[base + t] = ll[cur][t];
      val[base + t] = lv[cur][t];
    }
  }
}

__global__ __launch_bounds__(64) void guess_write(SplitArgs A, const int32_t *val) {
  const Chunk ch = A.chunks[blockIdx.x];
  const SplitCall S = A.split[ch.sc];
  const int32_t i = ch.start + (int32_t)threadIdx.x;
  if (i < S.n && i >= A.front[ch.sc]) A.score[S.off + i] = val[64 * blockIdx.x + threadIdx.x];
}

// 4. peaks: peak[i] = parent >= 0 && peak[parent] > score[i] ? peak[parent] : score[i]
// (host_kernel.cpp:92), i.e. the maximum score on i's parent path; segment 0's peaks are final.
__global__ __launch_bounds__(64) void peak_init(SplitArgs A, int32_t *link, int32_t *val) {
  const Chunk ch = A.chunks[blockIdx.x];
  const SplitCall S = A.split[ch.sc];
  const int32_t i = ch.start + (int32_t)threadIdx.x, j = 64 * blockIdx.x + threadIdx.x;
  if (i >= S.n) {
    link[j] = -1;
    val[j] = 0;
    return;
  }
  const int32_t f = A.score[S.off + i], p = A.parent[S.off + i];
  int32_t l = -1, v = f;
  if (p >= S.c1)
    l = cidx(S, p);
  else if (p >= 0)
    v = max(f, A.peak[S.off + p]);
  link[j] = l;
  val[j] = v;
}

// The verification ring: a mark is the anchor's index within the chunk (k + 1, 7 bits) tagged with
// the position's bits above the ring size, so positions that share a slot are told apart; a mark
// that would overwrite another mark of the same anchor at a different position (the ring is
// smaller than max_iter) is a conflict, and the anchor is not verified (it goes to the fix-up).
template <int RING>
__device__ __forceinline__ uint32_t ring_tag(int k, int32_t pos) {
  constexpr int kLog = RING == 1024 ? 10 : 13;
  static_assert(RING == (1 << kLog), "ring sizes: 1024 (tagged, may clash) or 8192 (> any window)");
  return (uint32_t)(k + 1) | ((uint32_t)pos >> kLog << 7);
}

template <int RING>
__device__ __forceinline__ bool resolve_tagged(int32_t sc, bool ok, int32_t pj, int32_t jtop, int32_t st, int k,
                                               int lane, int32_t neg_lane, uint32_t *S, int32_t &M, int32_t &J,
                                               int32_t &N, uint32_t &vis, bool &conflict, int32_t *tgt, int32_t i) {
  const bool writer = ok & (pj >= st);
  const uint32_t slot = writer ? (uint32_t)(pj & (RING - 1)) : (uint32_t)(RING + lane);
  const uint32_t tw = ring_tag<RING>(k, pj);
  const uint32_t prev = S[slot];
  conflict |= writer & ((prev & 127u) == (uint32_t)(k + 1)) & (prev != tw);
  S[slot] = tw;
  conflict |= writer & (S[slot] != tw);
  const int32_t j = jtop - lane;
  const bool tg = S[j & (RING - 1)] == ring_tag<RING>(k, j);
  const int32_t mx = scan_max(sc);
  const int32_t before = max(dpp_shr_i32(mx, INT_MIN), M);
  const bool upd = sc > before;
  const bool plus = ok & !upd & tg;
  const uint64_t um_all = __builtin_amdgcn_ballot_w64(upd), pm = __builtin_amdgcn_ballot_w64(plus);
  const uint64_t num = ~um_all;
  const int32_t d_ex = (int32_t)__builtin_amdgcn_mbcnt_hi(
      (uint32_t)(num >> 32),
      __builtin_amdgcn_mbcnt_lo((uint32_t)num, __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)pm, (uint32_t)neg_lane))));
  const int32_t D = d_ex + (plus ? 1 : (upd ? -1 : 0));
  const int32_t n_after = max(N + D, D - scan_min(D));
  const uint64_t bm = __builtin_amdgcn_ballot_w64(plus & (n_after > kMaxSkip));
  const uint64_t below = (bm - 1) & ~bm;
  const int32_t nvalid = min(64, jtop - st + 1);
  vis += bm ? (uint32_t)__builtin_ctzll(bm) + 1 : (uint32_t)max(nvalid, 0);
  const uint64_t um = um_all & below;
  const int lu = 63 - __builtin_clzll(um | 1);
  const int32_t m_lu = __builtin_amdgcn_readlane(mx, lu);
  J = um ? jtop - lu : J;
  M = um ? m_lu : M;
  if (ok && ((below >> lane) & 1) && pj >= 0) atomicMax(tgt + pj, i);
  N = __builtin_amdgcn_readlane(n_after, 63);
  return bm != 0;
}

// 2. verify (CHECK): re-run the loop of every split anchor i >= front against the guessed window;
// fail[sc] = the first i whose loop does not give its own guess. The loops also write their
// targets marks into t2 and count visited pairs per call: a call that passes in the first round has
// all of them right; one that ever failed is re-marked after convergence (CHECK false, front = c1).
// The check pass stamps into the 1 K tagged ring: a window wider than the ring can make an anchor's
// mark overwrite its own earlier one (a clash), which fails the anchor. The re-mark pass (whose
// marks and visited counts are final) uses an 8 K ring, wider than any window (max_iter 5000 + 64
// lanes), so no mark is ever lost there.
// need (from verify_lanes): only the anchors whose bit is set (null: all of them).
template <bool CHECK, int RING>
__device__ __forceinline__ void verify_chunk(SplitArgs A, const uint64_t *need, int32_t chunk, uint32_t *S) {
  const uint64_t nd = need ? need[chunk] : ~0ull;
  if (!nd) return;
  const Chunk ch = A.chunks[chunk];
  const SplitCall Sc = A.split[ch.sc];
  const int lane = threadIdx.x;
  const int32_t start = ch.start, n = Sc.n;
  const int32_t front = A.front[ch.sc];
  const int32_t cnt = min(64, n - start);
  if (start + cnt <= front) return;
  const int c = Sc.call;
  const int max_dist_x = A.params4[4 * c], max_dist_y = A.params4[4 * c + 1];
  const int bw = A.params4[4 * c + 2], n_segs = A.params4[4 * c + 3];
  const double avg_qspan = (double)A.avg_qspan[c];
  const uint64_t *X = A.x + Sc.off, *Y = A.y + Sc.off;
  const int32_t *score = A.score + Sc.off, *parent = A.parent + Sc.off;
  int32_t *tgt = A.t2 + Sc.off;
  for (int t = lane; t < RING + 64; t += 64) S[t] = 0;
  // window: lane l = anchor start-1-l; the chunk's anchors: lane l = start+l
  const int32_t j0 = start - 1 - lane;
  uint64_t wx = 0, wy = 0;
  int32_t wf = 0, wp = -1;
  if (j0 >= 0) {
    wx = X[j0];
    wy = Y[j0];
    wf = score[j0];
    wp = parent[j0];
  }
  const int32_t ci = min(start + lane, n - 1);
  const uint64_t bx = X[ci], by = Y[ci];
  const int32_t bf = score[ci], bp = parent[ci], bst = A.st[64 * chunk + lane];
  const int32_t neg_lane = -lane;
  uint32_t vis = 0;
  int32_t first_bad = INT_MAX;
  for (int k = 0; k < cnt; k++) {
    const int32_t i = start + k;
    const uint64_t xi = rfl64_lane(bx, k), yi = rfl64_lane(by, k);
    const int32_t fi = __builtin_amdgcn_readlane(bf, k), pi = __builtin_amdgcn_readlane(bp, k);
    if (i >= front && ((nd >> k) & 1)) {
      const int32_t st = __builtin_amdgcn_readlane(bst, k);
      int32_t sg;
      const bool ok = geometry(xi, yi, wx, wy, i - 1 - lane >= st, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sg);
      int32_t M = (int32_t)(yi >> 32 & 0xff), J = -1, N = 0;
      bool conflict = false;
      bool broke = resolve_tagged<RING>(ok ? sg + wf : INT_MIN, ok, wp, i - 1, st, k, lane, neg_lane, S, M, J, N,
                                        vis, conflict, tgt, i);
      for (int32_t jt = i - 65; !broke && jt >= st; jt -= 64) {  // older candidates from memory
        const int32_t jj = jt - lane;
        const bool v = jj >= st;
        uint64_t xj = 0, yj = 0;
        int32_t fj = 0, pj = -1;
        if (v) {
          xj = X[jj];
          yj = Y[jj];
          fj = score[jj];
          pj = parent[jj];
        }
        int32_t sgo;
        const bool oko = geometry(xi, yi, xj, yj, v, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sgo);
        broke = resolve_tagged<RING>(oko ? sgo + fj : INT_MIN, oko, pj, jt, st, k, lane, neg_lane, S, M, J, N, vis,
                                     conflict, tgt, i);
      }
      const bool clash = __builtin_amdgcn_ballot_w64(conflict) != 0;
      if (CHECK && (M != fi || J != pi || clash) && first_bad == INT_MAX) first_bad = i;
    }
    wx = dpp_shr_u64(wx, xi);
    wy = dpp_shr_u64(wy, yi);
    wf = dpp_shr_i32(wf, fi);
    wp = dpp_shr_i32(wp, pi);
  }
  if (lane == 0) {
    if (CHECK && first_bad != INT_MAX) atomicMin(A.fail + ch.sc, first_bad);
    atomicAdd(A.viscall + ch.sc, (unsigned long long)vis);
  }
}

// With need, the grid walks the work list verify_lanes built (A.slow) instead of one workgroup per
// chunk (a launch of every chunk's workgroup, nearly all exiting at once, cost 35-45 us a step).
template <bool CHECK, int RING = CHECK ? kTagRing : 8192>
__global__ __launch_bounds__(64) void verify_kernel(SplitArgs A, const uint64_t *need) {
  static_assert(CHECK || RING > kMaxIter + 64, "the re-mark ring must hold any window");
  __shared__ uint32_t S[RING + 64];
  const int32_t nwork = need ? A.slow[0] : A.nch;
  for (int32_t w = blockIdx.x; w < nwork; w += gridDim.x) {
    const int32_t chunk = need ? A.slow[1 + w] : w;
    verify_chunk<CHECK, RING>(A, need, chunk, S);
  }
}

// 2'. verify, one anchor per lane (the common case, ahead of verify_kernel): lane l re-runs the
// reference loop of anchor start + l over its first 64 candidates, reading the guessed window from
// memory (neighbouring lanes read neighbouring anchors), with the "targets[j] == i" marks of its own
// loop as bits of a 64-bit mask (bit d: position i-1-d; a mark further back matters only to a loop
// that visits more than 64 candidates). Such loops -- no break and a window wider than 64 -- are
// left to verify_kernel through need[chunk]; every other anchor is decided here, with the same
// outputs (fail, t2 marks, visited pairs). About one wave instruction per lane-candidate instead of
// a 64-lane step per candidate block of every anchor.
template <bool CHECK>
__global__ __launch_bounds__(64) void verify_lanes(SplitArgs A, uint64_t *need) {
  // targets marks of the wave's 64 loops, max-reduced in LDS over positions [start - 192, start + 64)
  // before they go to t2 (neighbouring anchors visit the same candidates: one global atomic per
  // position instead of one per visited candidate, which made the pass atomic-bound)
  constexpr int kMarkLo = 192, kMarkN = 256;
  __shared__ int32_t lm[kMarkN];
  // the candidates of the wave's 64 loops (their first 64 each) are anchors [start - 64, start + 63):
  // staged once into LDS, so each candidate is four LDS reads (consecutive lanes, consecutive
  // entries: conflict-free) instead of four global loads
  constexpr int kStage = 128;
  __shared__ uint64_t cx[kStage], cy[kStage];
  __shared__ int32_t cf[kStage], cp[kStage];
  const Chunk ch = A.chunks[blockIdx.x];
  const SplitCall Sc = A.split[ch.sc];
  const int lane = threadIdx.x;
  const int32_t start = ch.start, n = Sc.n;
  const int32_t front = A.front[ch.sc];
  const int32_t i = start + lane;
  const bool mine = (i < n) & (i >= front);
  if (!__builtin_amdgcn_ballot_w64(mine)) {
    if (lane == 0) need[blockIdx.x] = 0;
    return;
  }
  const int c = Sc.call;
  const int max_dist_x = A.params4[4 * c], max_dist_y = A.params4[4 * c + 1];
  const int bw = A.params4[4 * c + 2], n_segs = A.params4[4 * c + 3];
  const double avg_qspan = (double)A.avg_qspan[c];
  const uint64_t *X = A.x + Sc.off, *Y = A.y + Sc.off;
  const int32_t *score = A.score + Sc.off, *parent = A.parent + Sc.off;
  int32_t *tgt = A.t2 + Sc.off;
  const int32_t ii = min(i, n - 1);
  const uint64_t xi = X[ii], yi = Y[ii];
  const int32_t fi = score[ii], pi = parent[ii], st = A.st[64 * blockIdx.x + lane];
  const int32_t mbase = start - kMarkLo;
  for (int t = lane; t < kMarkN; t += 64) lm[t] = 0;
  const int32_t cbase = start - 64;
  for (int t = lane; t < kStage; t += 64) {
    const int32_t j = cbase + t;
    if (j >= 0 && j < n) {
      cx[t] = X[j];
      cy[t] = Y[j];
      cf[t] = score[j];
      cp[t] = parent[j];
    }
  }
  __syncthreads();
  int32_t M = (int32_t)(yi >> 32 & 0xff), J = -1, N = 0;
  uint64_t marks = 0;
  bool act = mine;
  uint32_t vis = 0;
  constexpr int U = 4;  // candidates loaded per batch (their loads overlap)
  for (int k0 = 0; k0 < 64; k0 += U) {
    if (!__builtin_amdgcn_ballot_w64(act & (i - 1 - k0 >= st))) break;
    uint64_t xj[U], yj[U];
    int32_t fj[U], pj[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t j = i - 1 - k0 - u;
      xj[u] = yj[u] = 0;
      fj[u] = 0;
      pj[u] = -1;
      if (act & (j >= st)) {
        const int t = j - cbase;  // in [0, 127): j >= i - 64 >= start - 64, j < i <= start + 63
        xj[u] = cx[t];
        yj[u] = cy[t];
        fj[u] = cf[t];
        pj[u] = cp[t];
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int k = k0 + u;
      const int32_t j = i - 1 - k;
      act = act & (j >= st);  // the window is exhausted: the loop ends
      int32_t sg;
      const bool ok = geometry(xi, yi, xj[u], yj[u], act, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sg);
      vis += act ? 1u : 0u;
      const int32_t sc = ok ? (int32_t)((uint32_t)sg + (uint32_t)fj[u]) : INT_MIN;
      const bool upd = sc > M;  // false when filtered (M >= 0 > INT_MIN)
      bool brk = false;
      if (upd) {
        M = sc;
        J = j;
        N = N > 0 ? N - 1 : 0;
      } else if (ok & (bool)((marks >> k) & 1)) {
        brk = ++N > kMaxSkip;  // host_kernel.cpp:84-88: the break skips the mark below
      }
      if (ok & !brk & (pj[u] >= 0)) {  // targets[parents[j]] = i (host_kernel.cpp:89)
        const int32_t d = i - 1 - pj[u];
        if (d < 64) marks |= 1ull << d;
        const uint32_t o = (uint32_t)(pj[u] - mbase);
        if (o < (uint32_t)kMarkN)
          atomicMax(&lm[o], i);
        else
          atomicMax(tgt + pj[u], i);
      }
      act = act & !brk;
    }
  }
  __syncthreads();
  for (int t = lane; t < kMarkN; t += 64) {
    const int32_t v = lm[t];
    if (v) atomicMax(tgt + mbase + t, v);
  }
  // still scanning after 64 candidates with more in the window: verify_kernel takes the anchor
  const bool unres = act & (i - 65 >= st);
  const uint64_t um = __builtin_amdgcn_ballot_w64(unres);
  const bool done = mine & !unres;
  const uint64_t bad = __builtin_amdgcn_ballot_w64(CHECK & done & ((M != fi) | (J != pi)));
  // visited pairs of the decided anchors (the undecided ones are counted by verify_kernel)
  uint32_t v = done ? vis : 0u;
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  if (lane == 0) {
    need[blockIdx.x] = um;
    if (um) A.slow[1 + atomicAdd(A.slow, 1)] = (int32_t)blockIdx.x;  // verify_kernel's work list
    if (CHECK && bad) atomicMin(A.fail + ch.sc, start + (int32_t)__builtin_ctzll(bad));
    if (v) atomicAdd(A.viscall + ch.sc, (unsigned long long)v);
  }
}

// peaks of the split anchors, and their targets marks (only split anchors mark them: t2)
__global__ __launch_bounds__(64) void peak_write(SplitArgs A, const int32_t *pv) {
  const Chunk ch = A.chunks[blockIdx.x];
  const SplitCall S = A.split[ch.sc];
  const int32_t i = ch.start + (int32_t)threadIdx.x;
  if (i < S.n) {
    A.peak[S.off + i] = pv[64 * blockIdx.x + threadIdx.x];
    A.target[S.off + i] = A.t2[S.off + i];
  }
}

// targets of a split call's segment 0 (anchors < c1): its own marks merged with the split anchors'
// marks by maximum (the last marker is the largest i); the call's visited pairs into the total
__global__ __launch_bounds__(256) void merge_targets(SplitArgs A) {
  const SplitCall S = A.split[blockIdx.x];
  int32_t *tg = A.target + S.off;
  const int32_t *t2 = A.t2 + S.off;
  for (int32_t x = threadIdx.x; x < S.c1; x += 256) tg[x] = max(tg[x], t2[x]);
  if (threadIdx.x == 0) atomicAdd(A.visited, A.viscall[blockIdx.x]);
}

namespace {

template <typename T>
int grow(T **p, int64_t *cap, int64_t need) {
  need = std::max<int64_t>(need, 1);
  if (need <= *cap) return GB_OK;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  GB_HIP(hipMalloc(p, (size_t)need * sizeof(T)));
  *cap = need;
  return GB_OK;
}

// Segment length: as long as the segment's sequential run (its window and warm-up included) stays
// under the batch's throughput time, so small batches get shorter segments; shorter ones cost more
// verification and warm-up work. GB_CHAIN_SPLIT: "0" runs every call whole; "SEG[,WARM]" sets the segment length and warm-up
// (tests force tiny segments without warm-up to exercise the fix-up path).
void split_knobs(int64_t total_anchors, int *seg, int *warm, int *trunc, int *wcap) {
  // the power of two in [512, 4096] nearest below total / 12 000 (measured with chain_rows,
  // tools/chain_rows_probe.py: 'large' 25.4 M anchors 2048 (7.76 ms; 4096 7.87, 1024 10.3), 'small'
  // 2.5 M and the 1/8 shard 3.2 M anchors 512 (2.06 / 2.20 ms; 1024 2.29 / 2.38)
  *seg = kSegDefault;
  while (*seg > 512 && (int64_t)*seg * 12000 > total_anchors) *seg /= 2;
  *warm = kWarmDefault;
  *trunc = 0;
  *wcap = kWinCapDefault;
  const char *e = getenv("GB_CHAIN_SPLIT");
  if (!e || !*e) return;
  int a = 0, b = -1, t = 0, w = -1;
  const int k = sscanf(e, "%d,%d,%d,%d", &a, &b, &t, &w);
  if (k >= 1 && a >= 0) *seg = a;  // -1: the adaptive length
  if (k >= 2 && b >= 0) *warm = b;
  if (k >= 3) *trunc = t;
  if (k >= 4 && w >= 0) *wcap = w;
}

SplitArgs split_args(gb_chain_batch *B) {
  SplitArgs A;
  const size_t nn = (size_t)std::max<int64_t>(B->nanchors, 1);
  A.split = B->d_split;
  A.segs = B->d_segs;
  A.chunks = B->d_chunks;
  A.st = B->d_st;
  A.front = B->d_front;
  A.fail = B->d_fail;
  A.avg_qspan = B->d_aq;
  A.params4 = B->d_par4;
  A.x = B->d_x;
  A.y = B->d_y;
  A.score = B->d_out;
  A.parent = B->d_out + nn;
  A.target = B->d_out + 2 * nn;
  A.peak = B->d_out + 3 * nn;
  A.s_score = B->d_sscore;
  A.s_parent = B->d_sparent;
  A.visited = B->d_vis;
  A.t2 = B->d_t2;
  A.viscall = B->d_viscall;
  const char *f = getenv("GB_CHAIN_SPLIT_FAULT");
  A.fault = f ? atoi(f) : 0;
  A.slow = B->d_slow;
  A.nch = (int32_t)B->chunks.size();
  return A;
}

// ceil(log2(n)) + 1 rounds resolve any parent path of n anchors
int jump_rounds(int n) {
  int r = 1;
  while ((1ll << (r - 1)) < (int64_t)n) r++;
  return r;
}

// pointer jumping from buffers 0; returns the buffer index holding the result
int jump(gb_chain_batch *B, int op, int rounds) {
  const int64_t nj = 64 * (int64_t)B->chunks.size();
  const unsigned g = (unsigned)((nj + 255) / 256);
  const unsigned nt = (unsigned)((nj + kTile - 1) / kTile);
  if (op == 0)
    hipLaunchKernelGGL(jump_local<0>, dim3(nt), dim3(kTileThreads), 0, B->stream, nj, B->d_link[0], B->d_val[0]);
  else
    hipLaunchKernelGGL(jump_local<1>, dim3(nt), dim3(kTileThreads), 0, B->stream, nj, B->d_link[0], B->d_val[0]);
  int cur = 0;
  for (int r = 0; r < rounds; r++) {
    if (op == 0)
      hipLaunchKernelGGL(jump_round<0>, dim3(g), dim3(256), 0, B->stream, nj, B->d_link[cur], B->d_val[cur],
                         B->d_link[cur ^ 1], B->d_val[cur ^ 1]);
    else
      hipLaunchKernelGGL(jump_round<1>, dim3(g), dim3(256), 0, B->stream, nj, B->d_link[cur], B->d_val[cur],
                         B->d_link[cur ^ 1], B->d_val[cur ^ 1]);
    cur ^= 1;
  }
  return cur;
}

}  // namespace

int split_plan(gb_chain_batch *B, const int64_t *offsets, const uint64_t *x, const int32_t *params4) {
  int seg, warm, trunc, wcap;
  split_knobs(B->ncalls ? offsets[B->ncalls] : 0, &seg, &warm, &trunc, &wcap);
  // A row target: the longest block a split tries to stay under (0: equal segments of seg). A batch
  // this small is its longest block: the 1/8 shard of the 'small' set (318 k anchors) 0.89 -> 0.68 ms
  // at 600 rows; bigger batches have the work to lose (the 'large' 1/8 shard, 3.2 M anchors: 1.37 ->
  // 1.42 ms at 900, 'large' 5.0 -> 8.9 ms; profiles/r05j_chain_target.log). GB_CHAIN_TARGET overrides.
  const int64_t total = B->ncalls ? offsets[B->ncalls] : 0;
  const char *te = getenv("GB_CHAIN_TARGET");
  const int32_t target = te ? std::max(0, atoi(te)) : (total < (1 << 20) ? 600 : 0);
  // Under a row target the block is warm-up + capped window (<= 512) + segment, so the window cap
  // bounds it from below; a shorter segment floor and warm-up take it under: the 'small' 1/8 shard
  // 0.678 -> 0.637 ms at a 64-anchor floor and a 16-anchor warm-up, no failed guess on the bench's or
  // the tests' sets (profiles/r05zz8_chain_knobs.log; a failed guess costs a fix-up, never a result).
  // GB_CHAIN_SEGMIN sets the floor; GB_CHAIN_SPLIT's warm-up, when given, wins.
  const char *sm = getenv("GB_CHAIN_SEGMIN");
  const int32_t seg_floor = sm ? std::max(16, atoi(sm)) : 64;
  {
    const char *se = getenv("GB_CHAIN_SPLIT");
    int a = 0, b = -1;
    const bool warm_given = se && sscanf(se, "%d,%d", &a, &b) >= 2 && b >= 0;
    if (target > 0 && !warm_given) warm = std::min(warm, 16);
  }
  const int64_t ncalls = B->ncalls;
  B->vc.clear();
  B->split.clear();
  B->segs.clear();
  B->chunks.clear();
  B->st.clear();
  B->scratch_n = 0;
  B->max_split_n = 0;
  // per call: the widest window (i - st(i), st as the reference's loop walks it,
  // host_kernel.cpp:57-58) and whether x is sorted; calls in parallel
  std::vector<int32_t> maxwin((size_t)ncalls, 0);
  std::vector<uint8_t> sorted((size_t)ncalls, 0);
  // chain_rows takes the blocks of calls whose window test is monotone in j: x sorted and
  // x + max_dist_x without wrap-around (GB_CHAIN_ROWS=0: chain_kernel for every block)
  std::vector<uint8_t> mono((size_t)ncalls, 0);
  const char *rows_env = getenv("GB_CHAIN_ROWS");
  const bool rows_on = !(rows_env && rows_env[0] == '0');
  // split candidates (>= 2 segments): st(i) kept, and per segment its warm-up start and widest
  // window, all computed in the parallel pass
  struct Cand {
    std::vector<int32_t> st, as, win;
    int32_t L = 0;  // segment length: n split into ceil(n / seg) equal segments (the last one shorter)
  };
  std::vector<Cand> cand((size_t)ncalls);
  auto walk = [&](int64_t c, int32_t *stw) {
    const int64_t off = offsets[c];
    const int32_t n = (int32_t)(offsets[c + 1] - off);
    const uint64_t mdx = (uint64_t)(int64_t)params4[4 * c];
    int32_t s = 0, mw = 0;
    bool srt = true;
    for (int32_t i = 0; i < n; i++) {
      while (s < i && x[off + i] > x[off + s] + mdx) ++s;
      if (i - s > kMaxIter) s = i - kMaxIter;
      if (stw) stw[i] = s;
      mw = std::max(mw, i - s);
      if (i) srt &= x[off + i] >= x[off + i - 1];
    }
    maxwin[(size_t)c] = mw;
    sorted[(size_t)c] = srt;
    mono[(size_t)c] = srt && (int64_t)mdx >= 0 && (n == 0 || x[off + n - 1] + mdx >= x[off + n - 1]);
  };
  {
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                                 offsets[ncalls] / 200000 + 1}));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
      th.emplace_back([&, t] {
        for (int64_t c = t; c < ncalls; c += nt) {
          const int32_t n = (int32_t)(offsets[c + 1] - offsets[c]);
          const bool maybe = seg >= 64 && (target > 0 ? (int64_t)n > std::min<int64_t>(target, 2 * (int64_t)seg)
                                                      : (int64_t)n >= 2 * (int64_t)seg);
          if (!maybe) {
            walk(c, nullptr);
            continue;
          }
          Cand &K = cand[(size_t)c];
          K.st.resize((size_t)n);
          walk(c, K.st.data());
          if (!sorted[(size_t)c]) {
            K.st = std::vector<int32_t>();
            continue;
          }
          // with a row target: a call's segments are as long as its window leaves room for under the
          // target (block = warm-up + capped window + segment), and a call no longer than the target
          // runs whole
          int32_t segc = seg;
          if (target > 0) {
            if (n <= target) {
              K.st = std::vector<int32_t>();
              continue;
            }
            const int32_t cw = std::min(maxwin[(size_t)c], wcap);
            segc = std::max(seg_floor, std::min(seg, target - cw - warm));
          }
          // equal segments of at most segc anchors: the longest block of the launch (a segment, its
          // window and its warm-up) is then bounded by segc, not by a last segment of up to 2 segc - 1
          const int32_t nseg = (n + segc - 1) / segc, L = (n + nseg - 1) / nseg;
          K.L = L;
          K.as.resize((size_t)nseg);
          K.win.resize((size_t)nseg);
          for (int32_t k = 0; k < nseg; k++) {
            const int32_t cs = k * L, es = k + 1 == nseg ? n : (k + 1) * L;
            // trunc: the warm-up starts `warm` anchors before c_s whatever the window (the first
            // anchors' spec loops then miss their oldest candidates, which only matters -- and is
            // then caught by the verification -- for loops that would have reached them)
            const int32_t a =
                k == 0 ? 0 : std::max(0, trunc ? cs - warm : std::max(K.st[(size_t)cs], cs - wcap) - warm);
            int32_t w = 0;
            for (int32_t i = a; i < es; i++) w = std::max(w, i - std::max(a, K.st[(size_t)i]));
            K.as[(size_t)k] = a;
            K.win[(size_t)k] = w;
          }
        }
      });
    for (auto &t : th) t.join();
  }
  auto vpush = [&](int64_t in, int64_t out, int32_t n, int64_t c, int32_t mode, int32_t win) {
    const int32_t cls = (rows_on && mono[(size_t)c]) ? 2 : (win <= kRingSmall ? 1 : 0);
    B->vc.push_back({in, out, n, (int32_t)c, 0, mode, 0, cls});
  };
  for (int64_t c = 0; c < ncalls; c++) {
    const int64_t off = offsets[c];
    const int32_t n = (int32_t)(offsets[c + 1] - off);
    const Cand &K = cand[(size_t)c];
    bool split = !K.as.empty();
    // the chunk space (64 * chunks) is indexed with int32
    if (split && 64 * ((int64_t)B->chunks.size() + n / 64 + 1) >= INT32_MAX) split = false;
    if (!split) {
      vpush(off, off, n, c, kVFinal, maxwin[(size_t)c]);
      continue;
    }
    SplitCall S;
    S.off = off;
    S.n = n;
    S.call = (int32_t)c;
    S.seg0 = (int32_t)B->segs.size();
    S.nseg = (int32_t)K.as.size();
    S.c1 = K.L;
    S.cbase = (int32_t)B->chunks.size();
    vpush(off, off, K.L, c, kVFinal, K.win[0]);  // segment 0: exact
    B->segs.push_back({0, K.L, 0, 0, -1});
    for (int32_t k = 1; k < S.nseg; k++) {
      Seg G;
      G.cs = k * K.L;
      G.es = k + 1 == S.nseg ? n : (k + 1) * K.L;
      G.as = K.as[(size_t)k];
      G.pad = 0;
      G.soff = B->scratch_n;
      B->scratch_n += G.es - G.as;
      vpush(off + G.as, G.soff, G.es - G.as, c, kVScratch, K.win[(size_t)k]);
      B->segs.push_back(G);
    }
    const int32_t sc = (int32_t)B->split.size();
    for (int32_t st0 = S.c1; st0 < n; st0 += 64) B->chunks.push_back({sc, st0});
    B->st.resize(64 * B->chunks.size(), 0);
    std::copy(K.st.begin() + S.c1, K.st.end(), B->st.begin() + (size_t)64 * S.cbase);
    B->split.push_back(S);
    B->max_split_n = std::max(B->max_split_n, n);
  }
  // chain_rows blocks, small-ring blocks, then the others (VCall::pad holds the class until here);
  // longest first in each: the grid is dispatched in order, so the critical paths start first (and
  // the two halves of a chain_rows wave get blocks of about the same length)
  std::stable_sort(B->vc.begin(), B->vc.end(), [](const VCall &a, const VCall &b) {
    return a.pad != b.pad ? a.pad > b.pad : a.n > b.n;
  });
  B->n_rows = 0;
  B->n_small = 0;
  for (auto &v : B->vc) {
    B->n_rows += v.pad == 2;
    B->n_small += v.pad == 1;
    v.pad = 0;
  }
  const int64_t nvc = (int64_t)B->vc.size();
  // room for one fix-up block per split call behind the table (split_resolve)
  if (int st = grow(&B->d_vc, &B->cap_vc, nvc + (int64_t)B->split.size())) return st;
  if (nvc) GB_HIP(hipMemcpy(B->d_vc, B->vc.data(), (size_t)nvc * sizeof(VCall), hipMemcpyHostToDevice));
  if (B->split.empty()) return GB_OK;
  const int64_t ns = (int64_t)B->split.size(), nch = (int64_t)B->chunks.size();
  int st = grow(&B->d_split, &B->cap_split, ns);
  if (!st) st = grow(&B->d_segs, &B->cap_segs, (int64_t)B->segs.size());
  if (!st) st = grow(&B->d_chunks, &B->cap_chunks, nch);
  if (!st) st = grow(&B->d_st, &B->cap_st, 64 * nch);
  if (!st) st = grow(&B->d_sscore, &B->cap_sscore, B->scratch_n);
  if (!st) st = grow(&B->d_sparent, &B->cap_sparent, B->scratch_n);
  if (!st) st = grow(&B->d_smark, &B->cap_smark, B->scratch_n);
  if (!st) st = grow(&B->d_front, &B->cap_front, 2 * ns);
  if (!st) st = grow(&B->d_viscall, &B->cap_viscall, ns);
  if (!st) st = grow(&B->d_t2, &B->cap_t2, B->nanchors);
  if (!st) st = grow(&B->d_need, &B->cap_need, nch);
  if (!st) st = grow(&B->d_slow, &B->cap_slow, nch + 1);
  if (st) return st;
  B->d_fail = B->d_front + ns;
  {
    const int64_t need = 64 * nch;
    if (need > B->cap_jump) {
      for (int k = 0; k < 2; k++) {
        (void)hipFree(B->d_link[k]);
        (void)hipFree(B->d_val[k]);
        B->d_link[k] = B->d_val[k] = nullptr;
      }
      B->cap_jump = 0;
      for (int k = 0; k < 2; k++) {
        GB_HIP(hipMalloc(&B->d_link[k], (size_t)need * sizeof(int32_t)));
        GB_HIP(hipMalloc(&B->d_val[k], (size_t)need * sizeof(int32_t)));
      }
      B->cap_jump = need;
    }
  }
  GB_HIP(hipMemcpy(B->d_split, B->split.data(), (size_t)ns * sizeof(SplitCall), hipMemcpyHostToDevice));
  GB_HIP(hipMemcpy(B->d_segs, B->segs.data(), B->segs.size() * sizeof(Seg), hipMemcpyHostToDevice));
  GB_HIP(hipMemcpy(B->d_chunks, B->chunks.data(), (size_t)nch * sizeof(Chunk), hipMemcpyHostToDevice));
  GB_HIP(hipMemcpy(B->d_st, B->st.data(), (size_t)64 * nch * sizeof(int32_t), hipMemcpyHostToDevice));
  return GB_OK;
}

int step_clear_launch(gb_chain_batch *B) {
  const int64_t ns = (int64_t)B->split.size();
  const SplitArgs A = ns ? split_args(B) : SplitArgs{};
  const int64_t work = std::max<int64_t>(std::max<int64_t>(B->nanchors, B->scratch_n), ns);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 4096));
  hipLaunchKernelGGL(step_clear, dim3(g), dim3(256), 0, B->stream, A, B->d_out + 2 * std::max<int64_t>(B->nanchors, 1),
                     B->nanchors, B->d_smark, B->scratch_n, B->d_vis, (int32_t)ns, B->d_front);
  GB_HIP(hipGetLastError());
  return GB_OK;
}

int split_resolve(gb_chain_batch *B) {
  gb::Range range_("gb.chain.split_resolve");
  const int64_t ns = (int64_t)B->split.size();
  const unsigned nch = (unsigned)B->chunks.size();
  std::vector<int32_t> front((size_t)ns);
  if (ns > B->cap_hfail) {
    if (B->h_fail) (void)hipHostFree(B->h_fail);
    B->h_fail = nullptr;
    B->cap_hfail = 0;
    GB_HIP(hipHostMalloc((void **)&B->h_fail, (size_t)ns * sizeof(int32_t), hipHostMallocDefault));
    B->cap_hfail = ns;
  }
  const int32_t *fail = B->h_fail;
  // front = c1, t2, viscall, fail and the work-list count were cleared by step_clear at the step's start
  for (int64_t k = 0; k < ns; k++) front[(size_t)k] = B->split[(size_t)k].c1;
  const SplitArgs A = split_args(B);
  // global rounds after jump_local: hops between tiles
  const int rounds = jump_rounds(B->max_split_n / kTile + 2);
  // GB_CHAIN_VLANES=0: verify_kernel alone (A/B and tests)
  const char *vl = getenv("GB_CHAIN_VLANES");
  const bool lanes = !(vl && vl[0] == '0');
  // verify_kernel's persistent grid over verify_lanes' work list: 4 waves per SIMD
  const unsigned slow_grid = std::max(1u, std::min(nch, (unsigned)(16 * dev_limits().cus)));
  std::vector<VCall> fix;
  std::vector<uint8_t> failed((size_t)ns, 0);
  B->spec_rounds = 0;
  B->fixups = 0;
  // the peak pass (4.) reads only scores, parents and segment-0 peaks, so it is queued right behind
  // the first verification, before the host has seen whether any segment failed: the GPU runs it
  // while the failure flags come back (the common case: none, and the pass is final). A failure
  // makes it run again at the end; peak_write overwrites every split anchor's peak and target.
  auto peak_pass = [&]() {
    hipLaunchKernelGGL(peak_init, dim3(nch), dim3(64), 0, B->stream, A, B->d_link[0], B->d_val[0]);
    const int r = jump(B, 1, rounds);
    hipLaunchKernelGGL(peak_write, dim3(nch), dim3(64), 0, B->stream, A, (const int32_t *)B->d_val[r]);
  };
  bool peaks_final = false;
  while (true) {
    B->spec_rounds++;
    hipLaunchKernelGGL(guess_init, dim3(nch), dim3(64), 0, B->stream, A, B->d_link[0], B->d_val[0]);
    const int r = jump(B, 0, rounds);
    hipLaunchKernelGGL(guess_write, dim3(nch), dim3(64), 0, B->stream, A, (const int32_t *)B->d_val[r]);
    if (B->spec_rounds > 1) GB_HIP(hipMemsetAsync(B->d_fail, 0x7f, (size_t)ns * 4, B->stream));
    if (lanes) {
      if (B->spec_rounds > 1) GB_HIP(hipMemsetAsync(B->d_slow, 0, sizeof(int32_t), B->stream));
      hipLaunchKernelGGL(verify_lanes<true>, dim3(nch), dim3(64), 0, B->stream, A, B->d_need);
      hipLaunchKernelGGL(verify_kernel<true>, dim3(slow_grid), dim3(64), 0, B->stream, A, (const uint64_t *)B->d_need);
    } else {
      hipLaunchKernelGGL(verify_kernel<true>, dim3(nch), dim3(64), 0, B->stream, A, (const uint64_t *)nullptr);
    }
    GB_HIP(hipGetLastError());
    GB_HIP(hipMemcpyAsync(B->h_fail, B->d_fail, (size_t)ns * 4, hipMemcpyDeviceToHost, B->stream));
    GB_HIP(hipEventRecord(B->fail_ev, B->stream));
    if (B->spec_rounds == 1) {
      peak_pass();
      peaks_final = true;
    }
    GB_HIP(hipEventSynchronize(B->fail_ev));  // the failure flags; the peak pass runs on meanwhile
    fix.clear();
    for (int64_t k = 0; k < ns; k++) {
      const int32_t f = fail[(size_t)k];
      if (f == 0x7f7f7f7f) {
        front[(size_t)k] = B->split[(size_t)k].n;
        continue;
      }
      const SplitCall &S = B->split[(size_t)k];
      failed[(size_t)k] = 1;
      const int32_t a0 = B->st[(size_t)64 * S.cbase + (size_t)(f - S.c1)];
      const int32_t e = std::min<int32_t>(S.n, f + kFix);
      fix.push_back({S.off + a0, S.off + a0, e - a0, S.call, f - a0, kVFixup, a0, 0});
      front[(size_t)k] = e;
    }
    if (fix.empty()) break;
    peaks_final = false;
    B->fixups += (int64_t)fix.size();
    // fix-up blocks go behind the block table (split_plan left room for one per split call)
    VCall *d_fix = B->d_vc + B->vc.size();
    GB_HIP(hipMemcpyAsync(d_fix, fix.data(), fix.size() * sizeof(VCall), hipMemcpyHostToDevice, B->stream));
    if (int st = launch_chain(B, d_fix, (int)fix.size(), 0, false, B->stream)) return st;
    GB_HIP(hipMemcpyAsync(B->d_front, front.data(), (size_t)ns * 4, hipMemcpyHostToDevice, B->stream));
    GB_HIP(hipStreamSynchronize(B->stream));  // the host vectors are reused next round
  }
  // calls that ever failed: their marks and visited counts include wrong loops; redo them whole
  bool redo = false;
  for (int64_t k = 0; k < ns; k++) {
    const SplitCall &S = B->split[(size_t)k];
    front[(size_t)k] = failed[(size_t)k] ? S.c1 : S.n;
    if (failed[(size_t)k]) {
      redo = true;
      GB_HIP(hipMemsetAsync(B->d_t2 + S.off, 0, (size_t)S.n * 4, B->stream));
      GB_HIP(hipMemsetAsync(B->d_viscall + k, 0, 8, B->stream));
    }
  }
  if (redo) {
    GB_HIP(hipMemcpyAsync(B->d_front, front.data(), (size_t)ns * 4, hipMemcpyHostToDevice, B->stream));
    if (lanes) {
      GB_HIP(hipMemsetAsync(B->d_slow, 0, sizeof(int32_t), B->stream));
      hipLaunchKernelGGL(verify_lanes<false>, dim3(nch), dim3(64), 0, B->stream, A, B->d_need);
      hipLaunchKernelGGL(verify_kernel<false>, dim3(slow_grid), dim3(64), 0, B->stream, A, (const uint64_t *)B->d_need);
    } else {
      hipLaunchKernelGGL(verify_kernel<false>, dim3(nch), dim3(64), 0, B->stream, A, (const uint64_t *)nullptr);
    }
    GB_HIP(hipStreamSynchronize(B->stream));  // `front` is a host vector about to go
  }
  if (!peaks_final) peak_pass();
  hipLaunchKernelGGL(merge_targets, dim3((unsigned)ns), dim3(256), 0, B->stream, A);
  GB_HIP(hipGetLastError());
  return GB_OK;
}

void split_free(gb_chain_batch *B) {
  for (void *p : {(void *)B->d_vc, (void *)B->d_split, (void *)B->d_segs, (void *)B->d_chunks, (void *)B->d_st,
                  (void *)B->d_sscore, (void *)B->d_sparent, (void *)B->d_front, (void *)B->d_link[0],
                  (void *)B->d_link[1], (void *)B->d_val[0], (void *)B->d_val[1], (void *)B->d_t2,
                  (void *)B->d_viscall, (void *)B->d_smark, (void *)B->d_need, (void *)B->d_slow})
    (void)hipFree(p);
  B->d_vc = nullptr;
}

}  // namespace gbchain
