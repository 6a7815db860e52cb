// chain_bt.hip -- MI355X (gfx950) chain backtrack: minimap2's consumer of the chaining DP's
// score f[], parent p[] and peak v[] arrays, run on the device-resident outputs of chain.hip.
//
// Semantics (tools/minimap2-acceleration/testbed/chain.c:140-219; the same code follows the DP in
// tools/minimap2/chain.c): every chain end i (no child, v[i] >= min_sc) is moved to the peak j of
// its parent path (f[j] == v[j]); the ends are sorted by (f[j] << 32 | j) descending; in that order
// each one claims nodes along its parent links until it meets a node claimed earlier (its start is
// always taken); a chain is kept if it has >= min_cnt anchors and, when it stopped on a claimed
// node j, f[start] - f[j] >= min_sc; the kept chains are finally reordered by the x of their first
// anchor with ksort's in-place MSD radix sort (ksort.h:93-150), whose order of equal keys is part
// of the output.
//
// MI355X design: the greedy claim loop is sequential in the reference, but its result has a closed
// form. Let first(x) be the smallest rank of a start in the subtree of x (x and its descendants
// along child links). Then chain r owns exactly the nodes with first(x) == r -- a parent path from
// its start up to a top node, ending at p[top] -- and a start already owned by an earlier chain
// forms a one-anchor chain that stops at its parent. first() is a subtree minimum; because every
// parent lies within kMaxIter (5000) anchors of its child (the DP's predecessor window), one wave
// per call computes it in a single descending sweep with the running minima in an 8192-entry LDS
// ring. Chain lengths and tops are then plain atomics over the anchors, acceptance is per chain,
// output offsets are device scans, and anchor positions come from one ascending wave sweep per call.
// Sorting the ends uses hipCUB's segmented radix sort (the keys are unique up to equal copies of the
// same end, so any correct sort gives the reference's order); the final reorder replays ksort's
// algorithm exactly, one wave per call, with the bucket tables in LDS (global scratch for very large sets).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <vector>

#include "../../include/gb_chain.h"
#include "chain_internal.h"
#include "gb_common.h"

namespace gbchain {

namespace {

constexpr int32_t kInf = 0x7f7f7f7f;  // "no start below" (the byte value the rank array is cleared to)
constexpr int kParentWindow = 5000;  // p[i] >= i - max_iter (host_kernel.cpp:41, testbed chain.c:44)
constexpr int kWin = 8192;           // LDS ring of running subtree minima, > kParentWindow + 64
constexpr int kRsMin = 64;           // RS_MIN_SIZE (ksort.h:98)
constexpr int kRsLevels = 8;         // 64-bit keys, 8 bits per pass

struct W128 {
  uint64_t x, y;
};

__global__ void k_cid(const int64_t *__restrict__ off, int32_t *__restrict__ cid) {
  const int c = blockIdx.x;
  for (int64_t k = off[c] + threadIdx.x; k < off[c + 1]; k += blockDim.x) cid[k] = c;
}

__global__ void k_mark(int64_t n, const int64_t *__restrict__ off, const int32_t *__restrict__ cid,
                       const int32_t *__restrict__ par, uint8_t *__restrict__ child) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const int32_t pp = par[g];
  if (pp >= 0) child[off[cid[g]] + pp] = 1;
}

// chain ends -> their peaks (testbed chain.c:150-158): key = f[j] << 32 | j, in anchor order
__global__ void k_ends(int64_t n, const int64_t *__restrict__ off, const int32_t *__restrict__ cid,
                       const int32_t *__restrict__ f, const int32_t *__restrict__ par,
                       const int32_t *__restrict__ v, const uint8_t *__restrict__ child, int32_t min_sc,
                       uint64_t *__restrict__ key, uint8_t *__restrict__ flag, int32_t *__restrict__ ecnt) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const int c = cid[g];
  const int64_t o = off[c];
  const int32_t i = (int32_t)(g - o);
  const bool end = child[g] == 0 && v[g] >= min_sc;
  flag[g] = end ? 1 : 0;
  if (!end) return;
  int32_t j = i;
  while (j >= 0 && f[o + j] < v[o + j]) j = par[o + j];
  if (j < 0) j = i;
  key[g] = (uint64_t)(uint32_t)f[o + j] << 32 | (uint32_t)j;
  atomicAdd(&ecnt[c], 1);
}

__device__ __forceinline__ int call_of_entry(const int32_t *__restrict__ eoff, int ncalls, int32_t e) {
  int lo = 0, hi = ncalls;  // largest c with eoff[c] <= e
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (eoff[mid] <= e) lo = mid; else hi = mid;
  }
  return lo;
}

// rank of each start node: the smallest rank among the sorted ends that name it
__global__ void k_rank(int32_t cap, const int32_t *__restrict__ eoff, int ncalls, const int64_t *__restrict__ off,
                       const uint64_t *__restrict__ skeys, int32_t *__restrict__ ecall, int32_t *__restrict__ rank) {
  const int32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cap || e >= eoff[ncalls]) return;
  const int c = call_of_entry(eoff, ncalls, e);
  ecall[e] = c;
  atomicMin(&rank[off[c] + (uint32_t)skeys[e]], e - eoff[c]);
}

// first(x) = min(rank(x), first of the children of x): one descending sweep per call, 64 anchors
// per step. ring[] holds the running minima of the open nodes (the parent window), already folded
// with every child beyond the current chunk; inside the chunk the subtree minima come from six
// doubling rounds (round k folds in the descendants 2^k links down, by LDS atomicMin on the 2^k-th
// ancestor), then each chunk node whose parent lies below the chunk folds its value into the ring.
// The parents of a step's chunk and the ranks entering the window with it are loaded kFirstBlk
// steps at a time, one block ahead (the sweep then waits on memory once per block, not twice per
// step); the first step fills the whole window below the top chunk itself.
constexpr int kFirstBlk = 16;
__global__ __launch_bounds__(64) void k_first(const int64_t *__restrict__ off, const int32_t *__restrict__ par,
                                              const int32_t *__restrict__ rank, int32_t *__restrict__ first) {
  __shared__ int32_t ring[kWin];
  __shared__ int32_t tm[64];
  const int c = blockIdx.x, lane = threadIdx.x;
  const int64_t o = off[c];
  const int32_t n = (int32_t)(off[c + 1] - o);
  if (n == 0) return;
  const int32_t nsteps = (n + 63) / 64;
  auto lo_of = [&](int32_t t) { return max(n - 64 * (t + 1), 0); };
  auto need_of = [&](int32_t t) { return max(lo_of(t) - kParentWindow, 0); };
  // step t's parents (lane: anchor lo + lane) and new window ranks (lane: anchor need_t + lane)
  auto load_block = [&](int32_t t0, int32_t *P, int32_t *R) {
#pragma unroll
    for (int s = 0; s < kFirstBlk; s++) {
      const int32_t t = t0 + s;
      P[s] = -1;
      R[s] = kInf;
      if (t < nsteps) {
        const int32_t lo = lo_of(t), hi = n - 1 - 64 * t, i = lo + lane;
        if (i <= hi) P[s] = par[o + i];
        if (t > 0) {
          const int32_t k = need_of(t) + lane;
          if (k < need_of(t - 1)) R[s] = rank[o + k];
        }
      }
    }
  };
  {  // step 0's window: [need_0, n)
    const int32_t need0 = need_of(0);
    for (int32_t k = n - 1 - lane; k >= need0; k -= 64) ring[k & (kWin - 1)] = rank[o + k];
  }
  int32_t cp[kFirstBlk], cr[kFirstBlk], np[kFirstBlk], nr[kFirstBlk];
  load_block(0, cp, cr);
  for (int32_t t0 = 0; t0 < nsteps; t0 += kFirstBlk) {
    load_block(t0 + kFirstBlk, np, nr);
#pragma unroll
    for (int s = 0; s < kFirstBlk; s++) {
    const int32_t t = t0 + s;
    if (t >= nsteps) break;
    const int32_t hi = n - 1 - 64 * t, lo = lo_of(t);
    if (t > 0) {
      const int32_t k = need_of(t) + lane;
      if (k < need_of(t - 1)) ring[k & (kWin - 1)] = cr[s];
    }
    __syncthreads();
    const int32_t i = lo + lane;
    const bool live = i <= hi;
    const int32_t pp = cp[s];
    int32_t m = live ? ring[i & (kWin - 1)] : kInf;
    int anc = (live && pp >= lo) ? pp - lo : -1;  // in-chunk parent (lane), or -1
#pragma unroll
    for (int k = 0; k < 6; k++) {
      tm[lane] = m;
      __syncthreads();
      if (anc >= 0) atomicMin(&tm[anc], m);
      __syncthreads();
      m = tm[lane];
      const int up = __shfl(anc, anc < 0 ? lane : anc);  // ancestor 2^(k+1) links up
      anc = anc < 0 ? -1 : up;
      __syncthreads();
    }
    if (live && pp >= 0 && pp < lo) atomicMin(&ring[pp & (kWin - 1)], m);
    if (live) first[o + i] = m;
    __syncthreads();
    }
#pragma unroll
    for (int s = 0; s < kFirstBlk; s++) {
      cp[s] = np[s];
      cr[s] = nr[s];
    }
  }
}

// chain lengths and top nodes (smallest index) of the owned paths; lanes of one chain aggregate
// (long chains would otherwise serialise their atomics on one address)
__global__ void k_count(int64_t n, const int64_t *__restrict__ off, const int32_t *__restrict__ cid,
                        const int32_t *__restrict__ eoff, const int32_t *__restrict__ first,
                        int32_t *__restrict__ clen, int32_t *__restrict__ ctop) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int32_t e = -1, idx = 0;
  if (g < n) {
    const int32_t fr = first[g];
    if (fr != kInf) {
      const int c = cid[g];
      e = eoff[c] + fr;
      idx = (int32_t)(g - off[c]);
    }
  }
  int gsize = 0, leader = lane;
  for (int l = 0; l < 64; l++) {
    if (__builtin_amdgcn_readlane(e, l) == e) {
      gsize++;
      if (l < leader) leader = l;
    }
  }
  if (e >= 0 && leader == lane) {  // lowest lane of the group = smallest index of the group
    atomicAdd(&clen[e], gsize);
    atomicMin(&ctop[e], idx);
  }
}

// keep / drop each chain (testbed chain.c:176-182)
__global__ void k_accept(int32_t cap, const int32_t *__restrict__ eoff, int ncalls, const int64_t *__restrict__ off,
                         const int32_t *__restrict__ ecall, const uint64_t *__restrict__ skeys,
                         const int32_t *__restrict__ f, const int32_t *__restrict__ par,
                         const int32_t *__restrict__ first, const int32_t *__restrict__ clen,
                         const int32_t *__restrict__ ctop, int32_t min_cnt, int32_t min_sc, uint64_t *__restrict__ u,
                         int32_t *__restrict__ acc, int32_t *__restrict__ alen, uint8_t *__restrict__ own) {
  const int32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cap || e >= eoff[ncalls]) return;
  const int c = ecall[e];
  const int64_t o = off[c];
  const int32_t s = (int32_t)(uint32_t)skeys[e], r = e - eoff[c];
  const bool owner = first[o + s] == r;
  const int32_t len = owner ? clen[e] : 1;
  const int32_t stop = owner ? par[o + ctop[e]] : par[o + s];
  const int32_t score = (int32_t)(skeys[e] >> 32);
  bool ok;
  int32_t sc;
  if (stop < 0) {
    sc = score;
    ok = len >= min_cnt;
  } else {
    sc = score - f[o + stop];
    ok = sc >= min_sc && len >= min_cnt;
  }
  u[e] = (uint64_t)(uint32_t)sc << 32 | (uint32_t)len;
  acc[e] = ok ? 1 : 0;
  alen[e] = ok ? len : 0;
  own[e] = owner ? 1 : 0;
}

// a kept chain whose start an earlier chain owns: its single anchor; kentry maps output chain slots
// (call order, rank order) back to entries
__global__ void k_special(int32_t cap, const int32_t *__restrict__ eoff, int ncalls, const int64_t *__restrict__ off,
                          const int32_t *__restrict__ ecall, const uint64_t *__restrict__ skeys,
                          const int32_t *__restrict__ acc, const uint8_t *__restrict__ own,
                          const int32_t *__restrict__ kidx, const int32_t *__restrict__ aoff,
                          int32_t *__restrict__ bidx, int32_t *__restrict__ bchain, int32_t *__restrict__ kentry) {
  const int32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= cap || e >= eoff[ncalls] || !acc[e]) return;
  kentry[kidx[e]] = e;
  if (own[e]) return;
  const int64_t o = off[ecall[e]];
  bidx[aoff[e]] = (int32_t)(o + (uint32_t)skeys[e]);
  bchain[aoff[e]] = e;
}

// the accepted chain owning each anchor (entry index), or -1: one thread per anchor, ahead of the
// sequential sweep of k_place (whose steps then read one staged word instead of two dependent loads)
__global__ void k_ent(int64_t n, const int32_t *__restrict__ cid, const int32_t *__restrict__ eoff,
                      const int32_t *__restrict__ first, const int32_t *__restrict__ acc, int32_t *__restrict__ ent) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const int32_t fr = first[g];
  int32_t e = -1;
  if (fr != kInf) {
    e = eoff[cid[g]] + fr;
    if (!acc[e]) e = -1;
  }
  ent[g] = e;
}

// anchor positions of the owned paths: one ascending sweep per call, 64 anchors per step; a
// chain's counter (LDS when the call has <= kLdsCtr chains, global otherwise) advances once per
// step by its group size, and lanes rank themselves inside their group. The owners (k_ent) are read
// kPlaceBlk steps at a time, one block ahead, so the sweep waits on memory once per block; groups
// are found one distinct owner at a time (ballot), not by a 64-lane scan per lane.
constexpr int kLdsCtr = 8192;
constexpr int kPlaceBlk = 16;
__global__ __launch_bounds__(64) void k_place(const int64_t *__restrict__ off, const int32_t *__restrict__ eoff,
                                              const int32_t *__restrict__ ent, const int32_t *__restrict__ aoff,
                                              int32_t *__restrict__ ctr, int32_t *__restrict__ bidx,
                                              int32_t *__restrict__ bchain) {
  __shared__ int32_t lctr[kLdsCtr];
  __shared__ int32_t base_of[64];
  const int c = blockIdx.x, lane = threadIdx.x;
  const int64_t o = off[c];
  const int32_t n = (int32_t)(off[c + 1] - o), e0 = eoff[c], ne = eoff[c + 1] - e0;
  const bool lds = ne <= kLdsCtr;
  if (lds)
    for (int k = lane; k < ne; k += 64) lctr[k] = 0;
  __syncthreads();
  int32_t cur[kPlaceBlk], nxt[kPlaceBlk];
#pragma unroll
  for (int s = 0; s < kPlaceBlk; s++) cur[s] = s * 64 + lane < n ? ent[o + s * 64 + lane] : -1;
  for (int32_t blo = 0; blo < n; blo += 64 * kPlaceBlk) {
#pragma unroll
    for (int s = 0; s < kPlaceBlk; s++) {
      const int32_t i = blo + 64 * kPlaceBlk + s * 64 + lane;
      nxt[s] = i < n ? ent[o + i] : -1;
    }
#pragma unroll
    for (int s = 0; s < kPlaceBlk; s++) {
      const int32_t lo = blo + 64 * s;
      if (lo >= n) break;
      const int32_t i = lo + lane;
      const int32_t e = cur[s];
      int rank = 0, gsize = 0, leader = lane;
      uint64_t rem = __builtin_amdgcn_ballot_w64(e >= 0);
      while (rem) {
        const int l0 = __builtin_ctzll(rem);
        const int32_t v = __builtin_amdgcn_readlane(e, l0);
        const uint64_t m = __builtin_amdgcn_ballot_w64(e == v);
        if (e == v) {
          rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          gsize = __builtin_popcountll(m);
          leader = l0;
        }
        rem &= ~m;
      }
      if (e >= 0 && leader == lane) {
        if (lds) {
          base_of[lane] = lctr[e - e0];
          lctr[e - e0] += gsize;
        } else {
          base_of[lane] = atomicAdd(&ctr[e], gsize);
        }
      }
      __syncthreads();
      if (e >= 0) {
        const int32_t pos = aoff[e] + base_of[leader] + rank;
        bidx[pos] = (int32_t)(o + i);
        bchain[pos] = e;
      }
      __syncthreads();
    }
#pragma unroll
    for (int s = 0; s < kPlaceBlk; s++) cur[s] = nxt[s];
  }
}

// ---- ksort's radix_sort_128x (ksort.h:93-150, key = .x), replayed exactly -----------------------
__device__ void rs_insert(W128 *beg, W128 *end) {
  for (W128 *i = beg + 1; i < end; ++i)
    if (i->x < (i - 1)->x) {
      W128 *j, tmp = *i;
      for (j = i; j > beg && tmp.x < (j - 1)->x; --j) *j = *(j - 1);
      *j = tmp;
    }
}

struct RsFrame {
  int32_t beg, end, s, k;  // range (indices into the call's array), shift, next bucket
};

// one rs_sort pass on [beg, end) at shift s; bucket bounds left in bb/be (indices)
__device__ void rs_pass(W128 *a, int32_t beg, int32_t end, int s, int32_t *bb, int32_t *be) {
  for (int k = 0; k < 256; k++) bb[k] = be[k] = beg;
  for (int32_t i = beg; i < end; i++) ++be[a[i].x >> s & 255];
  for (int k = 1; k < 256; k++) be[k] += be[k - 1] - beg, bb[k] = be[k - 1];
  for (int k = 0; k < 256;) {
    if (bb[k] != be[k]) {
      int l = (int)(a[bb[k]].x >> s & 255);
      if (l != k) {
        W128 tmp = a[bb[k]], swap;
        do {
          swap = tmp;
          tmp = a[bb[l]];
          a[bb[l]++] = swap;
          l = (int)(tmp.x >> s & 255);
        } while (l != k);
        a[bb[k]++] = tmp;
      } else {
        ++bb[k];
      }
    } else {
      ++k;
    }
  }
  bb[0] = beg;
  for (int k = 1; k < 256; k++) bb[k] = be[k - 1];
}

__device__ void radix_sort_128x(W128 *a, int32_t n, int32_t *scratch) {
  if (n <= kRsMin) {
    rs_insert(a, a + n);
    return;
  }
  // recursion of rs_sort as an explicit stack: level L keeps its frame and its bucket bounds
  RsFrame fr[kRsLevels];
  int lev = 0;
  fr[0] = RsFrame{0, n, 56, 0};
  rs_pass(a, 0, n, 56, scratch, scratch + 256);
  while (lev >= 0) {
    RsFrame &F = fr[lev];
    int32_t *bb = scratch + lev * 512, *be = bb + 256;
    if (F.s == 0 || F.k >= 256) {
      lev--;
      continue;
    }
    const int ns = F.s > 8 ? F.s - 8 : 0;
    const int k = F.k++;
    const int32_t sz = be[k] - bb[k];
    if (sz > kRsMin) {
      lev++;
      fr[lev] = RsFrame{bb[k], be[k], ns, 0};
      rs_pass(a, bb[k], be[k], ns, scratch + lev * 512, scratch + lev * 512 + 256);
    } else if (sz > 1) {
      rs_insert(a + bb[k], a + be[k]);
    }
  }
}

// per call: w[k] = {x of chain k's first anchor, anchor offset << 32 | k}, sorted; chains and their
// anchor offsets in the final order (testbed chain.c:200-213). One wave per call. ksort
// insertion-sorts up to 64 elements, i.e. sorts them stably: lanes rank themselves. Larger sets
// replay the MSD radix sort exactly (lane 0, in LDS up to kLdsW elements, else in global memory).
constexpr int kLdsW = 2048;
__global__ __launch_bounds__(64) void k_reorder(const int32_t *__restrict__ eoff, const int32_t *__restrict__ kidx,
                                                const int32_t *__restrict__ aoff, const int32_t *__restrict__ kentry,
                                                const int32_t *__restrict__ bidx, const uint64_t *__restrict__ x,
                                                const uint64_t *__restrict__ u, W128 *__restrict__ w,
                                                uint64_t *__restrict__ uout, int32_t *__restrict__ newoff,
                                                int32_t *__restrict__ scratch) {
  __shared__ W128 lw[kLdsW];
  __shared__ int32_t lsc[kRsLevels * 512];
  const int c = blockIdx.x, lane = threadIdx.x;
  const int32_t k0 = kidx[eoff[c]], nu = kidx[eoff[c + 1]] - k0;
  if (nu == 0) return;
  const int32_t a0 = aoff[eoff[c]];
  if (nu <= kRsMin) {
    int32_t e = -1;
    uint64_t key = 0;
    if (lane < nu) {
      e = kentry[k0 + lane];
      key = x[bidx[aoff[e]]];
    }
    int pos = 0;
    for (int l = 0; l < nu; l++) {
      const uint64_t kl = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(key >> 32), l) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, l);
      pos += (kl < key || (kl == key && l < lane)) ? 1 : 0;
    }
    // sorted slot `pos` holds chain lane; offsets are the exclusive sum of lengths in sorted order
    const int32_t len = e >= 0 ? (int32_t)(uint32_t)u[e] : 0;
    int32_t before = 0;
    for (int l = 0; l < nu; l++) {
      const int pl = __builtin_amdgcn_readlane(pos, l);
      const int32_t ll = __builtin_amdgcn_readlane(len, l);
      before += pl < pos ? ll : 0;
    }
    if (lane < nu) {
      uout[k0 + pos] = u[e];
      newoff[e] = a0 + before;
    }
    return;
  }
  W128 *wc = nu <= kLdsW ? lw : w + k0;
  int32_t *sc = nu <= kLdsW ? lsc : scratch + (size_t)c * kRsLevels * 512;  // the call's own slice
  auto fill = [&]() {
    for (int32_t k = lane; k < nu; k += 64) {
      const int32_t e = kentry[k0 + k];
      wc[k].x = x[bidx[aoff[e]]];
      wc[k].y = (uint64_t)(uint32_t)(aoff[e] - a0) << 32 | (uint32_t)k;
    }
  };
  fill();
  __syncthreads();
  // Distinct keys (the usual case): every sort gives ksort's order, so the wave sorts the LDS copy
  // with a bitonic network (pads of ~0 payload last) and checks the keys are distinct; with a
  // repeated key, ksort's tie order is its own, so the array is rebuilt and lane 0 replays it.
  bool sorted = false;
  if (nu <= kLdsW) {
    int32_t np = 1;
    while (np < nu) np <<= 1;
    for (int32_t k = nu + lane; k < np; k += 64) {
      lw[k].x = ~0ull;
      lw[k].y = ~0ull;
    }
    __syncthreads();
    for (int32_t kk = 2; kk <= np; kk <<= 1)
      for (int32_t jj = kk >> 1; jj > 0; jj >>= 1) {
        for (int32_t t = lane; t < (np >> 1); t += 64) {
          const int32_t a = ((t & ~(jj - 1)) << 1) | (t & (jj - 1)), b = a | jj;  // a has bit jj clear
          const W128 pa = lw[a], pb = lw[b];
          const bool gt = pa.x > pb.x || (pa.x == pb.x && pa.y > pb.y);
          const bool up = (a & kk) == 0;
          if (gt == up) {
            lw[a] = pb;
            lw[b] = pa;
          }
        }
        __syncthreads();
      }
    bool dup = false;
    for (int32_t i = 1 + lane; i < nu; i += 64) dup |= lw[i].x == lw[i - 1].x;
    sorted = __builtin_amdgcn_ballot_w64(dup) == 0;
    if (!sorted) {
      __syncthreads();
      fill();
      __syncthreads();
    }
  }
  if (!sorted && lane == 0) radix_sort_128x(wc, nu, sc);
  __syncthreads();
  // outputs in sorted order; offsets are the running sum of the chain lengths (a wave scan per 64)
  int32_t run = a0;
  for (int32_t i0 = 0; i0 < nu; i0 += 64) {
    const int32_t i = i0 + lane;
    int32_t e = 0, len = 0;
    uint64_t ue = 0;
    if (i < nu) {
      e = kentry[k0 + (int32_t)(uint32_t)wc[i].y];
      ue = u[e];
      len = (int32_t)(uint32_t)ue;
    }
    int32_t incl = len;
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t t = __shfl_up(incl, d);
      if (lane >= d) incl += t;
    }
    if (i < nu) {
      uout[k0 + i] = ue;
      newoff[e] = run + incl - len;
    }
    run += __shfl(incl, 63);
  }
}

__global__ void k_copy(int32_t cap, int ncalls, const int32_t *__restrict__ eoff, const int32_t *__restrict__ bidx,
                       const int32_t *__restrict__ bchain, const int32_t *__restrict__ aoff,
                       const int32_t *__restrict__ newoff,
                       const uint64_t *__restrict__ x, const uint64_t *__restrict__ y, uint64_t *__restrict__ ox,
                       uint64_t *__restrict__ oy) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cap || j >= aoff[eoff[ncalls]]) return;
  const int32_t e = bchain[j];
  const int32_t dst = newoff[e] + (j - aoff[e]);
  const int32_t g = bidx[j];
  ox[dst] = x[g];
  oy[dst] = y[g];
}

}  // namespace

struct ChainBt {
  int64_t n = 0;  // anchors the buffers are sized for
  int ncalls = 0;
  int32_t *cid = nullptr, *ecnt = nullptr, *eoff = nullptr, *nsel = nullptr, *rank = nullptr, *first = nullptr;
  int32_t *ecall = nullptr, *clen = nullptr, *ctop = nullptr, *acc = nullptr, *alen = nullptr, *kidx = nullptr;
  int32_t *aoff = nullptr, *kentry = nullptr, *ctr = nullptr, *bidx = nullptr, *bchain = nullptr;
  int32_t *newoff = nullptr, *scratch = nullptr;
  uint8_t *child = nullptr, *flag = nullptr, *own = nullptr;
  uint64_t *key = nullptr, *ekeys = nullptr, *skeys = nullptr, *u = nullptr, *uout = nullptr;
  uint64_t *ox = nullptr, *oy = nullptr;
  W128 *w = nullptr;
  void *temp = nullptr;
  size_t temp_bytes = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool ran = false;
};

void chain_bt_destroy(ChainBt *T) {
  if (!T) return;
  for (void *p : {(void *)T->cid, (void *)T->ecnt, (void *)T->eoff, (void *)T->nsel, (void *)T->rank,
                  (void *)T->first, (void *)T->ecall, (void *)T->clen, (void *)T->ctop, (void *)T->acc,
                  (void *)T->alen, (void *)T->kidx, (void *)T->aoff, (void *)T->kentry, (void *)T->ctr,
                  (void *)T->bidx, (void *)T->bchain, (void *)T->newoff, (void *)T->scratch, (void *)T->child,
                  (void *)T->flag, (void *)T->own, (void *)T->key, (void *)T->ekeys, (void *)T->skeys,
                  (void *)T->u, (void *)T->uout, (void *)T->ox, (void *)T->oy, (void *)T->w, T->temp})
    if (p) (void)hipFree(p);
  for (auto e : T->ev)
    if (e) (void)hipEventDestroy(e);
  delete T;
}

namespace {

int bt_alloc(gb_chain_batch *B) {
  if (B->bt) return GB_OK;
  auto *T = new ChainBt();
  B->bt = T;
  const int64_t n = std::max<int64_t>(B->nanchors, 1);
  GB_ARG(n < (1ll << 30), "gb_chain_batch_backtrack: too many anchors (%lld)", (long long)n);
  T->n = n;
  T->ncalls = (int)B->ncalls;
  const size_t nc1 = (size_t)B->ncalls + 1;
  for (auto &e : T->ev) GB_HIP(hipEventCreate(&e));
  GB_HIP(hipMalloc(&T->cid, n * 4));
  GB_HIP(hipMalloc(&T->ecnt, nc1 * 4));
  GB_HIP(hipMalloc(&T->eoff, nc1 * 4));
  GB_HIP(hipMalloc(&T->nsel, 4));
  for (int32_t **p : {&T->rank, &T->first, &T->ecall, &T->clen, &T->ctop, &T->kentry, &T->ctr, &T->newoff})
    GB_HIP(hipMalloc(p, n * 4));
  for (int32_t **p : {&T->acc, &T->alen, &T->kidx, &T->aoff}) GB_HIP(hipMalloc(p, (n + 1) * 4));
  GB_HIP(hipMalloc(&T->bidx, 2 * n * 4));
  GB_HIP(hipMalloc(&T->bchain, 2 * n * 4));
  GB_HIP(hipMalloc(&T->scratch, nc1 * kRsLevels * 512 * 4));  // bucket tables of the > kLdsW reorders
  GB_HIP(hipMalloc(&T->child, n));
  GB_HIP(hipMalloc(&T->flag, n));
  GB_HIP(hipMalloc(&T->own, n));
  for (uint64_t **p : {&T->key, &T->ekeys, &T->skeys, &T->u, &T->uout}) GB_HIP(hipMalloc(p, n * 8));
  GB_HIP(hipMalloc(&T->ox, 2 * n * 8));
  GB_HIP(hipMalloc(&T->oy, 2 * n * 8));
  GB_HIP(hipMalloc(&T->w, n * sizeof(W128)));
  // hipCUB temporary storage: the largest of the select, the segmented sort and the scans
  size_t a = 0, b = 0, c = 0, d = 0;
  GB_HIP(hipcub::DeviceSelect::Flagged(nullptr, a, T->key, T->flag, T->ekeys, T->nsel, (int)n));
  GB_HIP(hipcub::DeviceSegmentedRadixSort::SortKeysDescending(nullptr, b, T->ekeys, T->skeys, (int)n, T->ncalls,
                                                               T->eoff, T->eoff + 1));
  GB_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, c, T->acc, T->kidx, (int)n + 1));
  GB_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, d, T->ecnt, T->eoff, T->ncalls + 1));
  T->temp_bytes = std::max(std::max(a, b), std::max(c, d));
  GB_HIP(hipMalloc(&T->temp, std::max<size_t>(T->temp_bytes, 16)));
  return GB_OK;
}

}  // namespace
}  // namespace gbchain

extern "C" {

int gb_chain_batch_backtrack(gb_chain_batch *B, int32_t min_cnt, int32_t min_sc) {
  gb::Range range_("gb.chain.backtrack");
  GB_ARG(B && B->ran, "gb_chain_batch_backtrack: chain_dp has not run on this batch");
  GB_HIP(hipSetDevice(B->device));
  using namespace gbchain;
  if (int st = bt_alloc(B)) return st;
  ChainBt *T = B->bt;
  hipStream_t s = B->stream;
  const int64_t n = B->nanchors;
  const int nc = (int)B->ncalls;
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  const int32_t *f = B->d_out, *par = B->d_out + nn, *v = B->d_out + 3 * nn;
  GB_HIP(hipEventRecord(T->ev[0], s));
  if (n > 0 && nc > 0) {
    const int32_t cap = (int32_t)n;
    const unsigned ga = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_cid, dim3(nc), dim3(256), 0, s, B->d_off, T->cid);
    GB_HIP(hipMemsetAsync(T->child, 0, n, s));
    GB_HIP(hipMemsetAsync(T->ecnt, 0, (nc + 1) * 4, s));
    hipLaunchKernelGGL(k_mark, dim3(ga), dim3(256), 0, s, n, B->d_off, T->cid, par, T->child);
    hipLaunchKernelGGL(k_ends, dim3(ga), dim3(256), 0, s, n, B->d_off, T->cid, f, par, v, T->child, min_sc, T->key,
                       T->flag, T->ecnt);
    GB_HIP(hipGetLastError());
    size_t tb = T->temp_bytes;
    GB_HIP(hipcub::DeviceSelect::Flagged(T->temp, tb, T->key, T->flag, T->ekeys, T->nsel, (int)n, s));
    tb = T->temp_bytes;
    GB_HIP(hipcub::DeviceScan::ExclusiveSum(T->temp, tb, T->ecnt, T->eoff, nc + 1, s));
    tb = T->temp_bytes;
    GB_HIP(hipcub::DeviceSegmentedRadixSort::SortKeysDescending(T->temp, tb, T->ekeys, T->skeys, (int)n, nc, T->eoff,
                                                                 T->eoff + 1, 0, 64, s));
    // starts' ranks, subtree minima, chain lengths/tops
    GB_HIP(hipMemsetAsync(T->rank, 0x7f, n * 4, s));  // 0x7f7f7f7f > any rank; normalised below
    hipLaunchKernelGGL(k_rank, dim3(ga), dim3(256), 0, s, cap, T->eoff, nc, B->d_off, T->skeys, T->ecall, T->rank);
    hipLaunchKernelGGL(k_first, dim3(nc), dim3(64), 0, s, B->d_off, par, T->rank, T->first);
    GB_HIP(hipGetLastError());
    GB_HIP(hipMemsetAsync(T->clen, 0, n * 4, s));
    GB_HIP(hipMemsetAsync(T->ctop, 0x7f, n * 4, s));
    hipLaunchKernelGGL(k_count, dim3(ga), dim3(256), 0, s, n, B->d_off, T->cid, T->eoff, T->first, T->clen, T->ctop);
    GB_HIP(hipMemsetAsync(T->acc, 0, (n + 1) * 4, s));
    GB_HIP(hipMemsetAsync(T->alen, 0, (n + 1) * 4, s));
    hipLaunchKernelGGL(k_accept, dim3(ga), dim3(256), 0, s, cap, T->eoff, nc, B->d_off, T->ecall, T->skeys, f, par,
                       T->first, T->clen, T->ctop, min_cnt, min_sc, T->u, T->acc, T->alen, T->own);
    GB_HIP(hipGetLastError());
    tb = T->temp_bytes;
    GB_HIP(hipcub::DeviceScan::ExclusiveSum(T->temp, tb, T->acc, T->kidx, (int)n + 1, s));
    tb = T->temp_bytes;
    GB_HIP(hipcub::DeviceScan::ExclusiveSum(T->temp, tb, T->alen, T->aoff, (int)n + 1, s));
    hipLaunchKernelGGL(k_special, dim3(ga), dim3(256), 0, s, cap, T->eoff, nc, B->d_off, T->ecall, T->skeys, T->acc,
                       T->own, T->kidx, T->aoff, T->bidx, T->bchain, T->kentry);
    GB_HIP(hipMemsetAsync(T->ctr, 0, n * 4, s));
    // owners per anchor into clen (no longer read after k_accept)
    hipLaunchKernelGGL(k_ent, dim3(ga), dim3(256), 0, s, n, T->cid, T->eoff, T->first, T->acc, T->clen);
    hipLaunchKernelGGL(k_place, dim3(nc), dim3(64), 0, s, B->d_off, T->eoff, (const int32_t *)T->clen, T->aoff,
                       T->ctr, T->bidx, T->bchain);
    hipLaunchKernelGGL(k_reorder, dim3(nc), dim3(64), 0, s, T->eoff, T->kidx, T->aoff, T->kentry, T->bidx, B->d_x,
                       T->u, T->w, T->uout, T->newoff, T->scratch);
    const unsigned gb = (unsigned)((2 * n + 255) / 256);
    hipLaunchKernelGGL(k_copy, dim3(gb), dim3(256), 0, s, (int32_t)(2 * n), nc, T->eoff, T->bidx, T->bchain, T->aoff,
                       T->newoff, B->d_x, B->d_y, T->ox, T->oy);
    GB_HIP(hipGetLastError());
  }
  GB_HIP(hipEventRecord(T->ev[1], s));
  T->ran = true;
  return GB_OK;
}

int gb_chain_batch_chains(gb_chain_batch *B, int64_t *n_chains, uint64_t *u, int64_t *n_anchors, uint64_t *ax,
                          uint64_t *ay, int64_t *total_chains, int64_t *total_anchors) {
  GB_ARG(B && B->bt && B->bt->ran, "gb_chain_batch_chains: backtrack has not run");
  GB_HIP(hipSetDevice(B->device));
  GB_HIP(hipStreamSynchronize(B->stream));
  gbchain::ChainBt *T = B->bt;
  const int64_t n = B->nanchors, nc = B->ncalls;
  std::vector<int64_t> off((size_t)nc + 1);
  if (nc) GB_HIP(hipMemcpy(off.data(), B->d_off, (nc + 1) * 8, hipMemcpyDeviceToHost));
  std::vector<int32_t> eoff((size_t)nc + 1, 0), kidx((size_t)n + 1, 0), aoff((size_t)n + 1, 0);
  if (n > 0 && nc > 0) {
    GB_HIP(hipMemcpy(eoff.data(), T->eoff, (nc + 1) * 4, hipMemcpyDeviceToHost));
    GB_HIP(hipMemcpy(kidx.data(), T->kidx, (n + 1) * 4, hipMemcpyDeviceToHost));
    GB_HIP(hipMemcpy(aoff.data(), T->aoff, (n + 1) * 4, hipMemcpyDeviceToHost));
  }
  const int64_t tc = kidx[(size_t)eoff[(size_t)nc]], ta = aoff[(size_t)eoff[(size_t)nc]];
  if (total_chains) *total_chains = tc;
  if (total_anchors) *total_anchors = ta;
  std::vector<uint64_t> hu((size_t)std::max<int64_t>(tc, 1)), hx((size_t)std::max<int64_t>(ta, 1)),
      hy((size_t)std::max<int64_t>(ta, 1));
  if (tc && u) GB_HIP(hipMemcpy(hu.data(), T->uout, tc * 8, hipMemcpyDeviceToHost));
  if (ta && (ax || ay)) {
    GB_HIP(hipMemcpy(hx.data(), T->ox, ta * 8, hipMemcpyDeviceToHost));
    GB_HIP(hipMemcpy(hy.data(), T->oy, ta * 8, hipMemcpyDeviceToHost));
  }
  for (int64_t c = 0; c < nc; c++) {
    const int32_t e0 = eoff[(size_t)c], e1 = eoff[(size_t)c + 1];
    const int64_t k0 = kidx[(size_t)e0], k1 = kidx[(size_t)e1], a0 = aoff[(size_t)e0], a1 = aoff[(size_t)e1];
    if (n_chains) n_chains[c] = k1 - k0;
    if (n_anchors) n_anchors[c] = a1 - a0;
    if (u)
      for (int64_t k = k0; k < k1; k++) u[off[(size_t)c] + (k - k0)] = hu[(size_t)k];
    for (int64_t a = a0; a < a1; a++) {
      if (ax) ax[2 * off[(size_t)c] + (a - a0)] = hx[(size_t)a];
      if (ay) ay[2 * off[(size_t)c] + (a - a0)] = hy[(size_t)a];
    }
  }
  return GB_OK;
}

int gb_chain_batch_backtrack_timing(gb_chain_batch *B, float *ms) {
  GB_ARG(B && B->bt && B->bt->ran && ms, "gb_chain_batch_backtrack_timing: backtrack has not run");
  GB_HIP(hipEventSynchronize(B->bt->ev[1]));
  GB_HIP(hipEventElapsedTime(ms, B->bt->ev[0], B->bt->ev[1]));
  return GB_OK;
}

}  // extern "C"
