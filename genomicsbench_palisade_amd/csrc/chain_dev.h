// chain_dev.h -- device helpers shared by the chain_dp kernels: the sequential kernel (chain.hip)
// and the speculative-segment verification (chain_split.hip). Semantics: minimap2-acceleration
// kernel/scalar/src/host_kernel.cpp:30-94.
#pragma once
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdint>

namespace gbchain {

constexpr int kRing = 8192;      // stamp ring >= max_iter (5000) + 64 candidates: any window
constexpr int kRingSmall = 1024; // for blocks whose windows hold <= 1024 anchors (i - st(i))
constexpr int kMaxIter = 5000;  // host_kernel.cpp:41
constexpr int kMaxSkip = 25;    // host_kernel.cpp:42

__device__ __forceinline__ int ilog2_32(uint32_t v) { return 31 - __clz((int)v); }  // v > 0 (LogTable256)

__device__ __forceinline__ int dpp_shr_i32(int v, int lane0) {
  return __builtin_amdgcn_update_dpp(lane0, v, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ __forceinline__ uint64_t dpp_shr_u64(uint64_t v, uint64_t lane0) {
  const int lo = dpp_shr_i32((int)(uint32_t)v, (int)(uint32_t)lane0);
  const int hi = dpp_shr_i32((int)(uint32_t)(v >> 32), (int)(uint32_t)(lane0 >> 32));
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

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
// MARK selects how the targets marks are written: kMarkStore a buffer store (one sequential writer
// per call), kMarkNone not at all, kMarkMax an atomic max into `tgt` (anchors of one call resolved
// in parallel: the last marker is the largest i).
enum { kMarkStore = 0, kMarkNone = 1, kMarkMax = 2 };
// RING: stamp ring size; positions of one loop lie in [st, i-1], so i - st <= RING keeps them apart.
template <int MARK = kMarkStore, int RING = kRing>
__device__ __forceinline__ bool resolve_step(int32_t sc, bool ok, int32_t pj, int32_t jtop, int32_t st, uint32_t stamp,
                                             int lane, int32_t neg_lane, __amdgpu_buffer_rsrc_t trs, int32_t i,
                                             uint32_t *S, int32_t &M, int32_t &J, int32_t &N, uint32_t &vis,
                                             int32_t *tgt_out = nullptr) {
  // "targets[j] == i": stamps from visited j' > j with parents[j'] == j. A stamp can only match a
  // lane whose j >= st (|pj - j| < kRing, so equal ring slots mean pj == j), so no validity test
  S[(ok & (pj >= st)) ? (pj & (RING - 1)) : RING + lane] = stamp;
  const bool tgt = S[(jtop - lane) & (RING - 1)] == stamp;
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
  if (MARK == kMarkStore) __builtin_amdgcn_raw_buffer_store_b32(i, trs, wt ? (uint32_t)pj * 4u : 0xFFFFFFFFu, 0, 0);
  if (MARK == kMarkMax && wt) atomicMax(tgt_out + pj, i);
  N = __builtin_amdgcn_readlane(n_after, 63);
  return bm != 0;
}

__device__ __forceinline__ uint64_t rfl64_lane(uint64_t v, int l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32;
}

}  // namespace gbchain
