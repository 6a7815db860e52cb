// chain_rows.hip -- chain_dp with two calls per wave64 (32 lanes each): the main sequential kernel.
//
// Semantics: tools/minimap2-acceleration/kernel/scalar/src/host_kernel.cpp:30-94 (== the plaintext
// branch of benchmarks/chain/src/host_kernel.cpp:405-472), bit for bit: scores, parents, targets
// marks, peak scores and the visited (i, j) count.
//
// Why halves. chain_kernel (chain.hip) runs one block per wave pair and resolves an anchor with
// 64-lane steps, but an anchor visits ~26 candidates on the bench's sets (none above 48): most of
// every step is filtered lanes, and its per-anchor bookkeeping (~212 VALU + ~219 SALU instructions
// for producer and consumer together) made the 'large' set issue-bound. Here each 32-lane half of a
// wave runs its own block; both halves share every VALU instruction, and an anchor usually needs
// one 32-candidate step. The sequential quantities of the reference loop are resolved as before
// (running max_f by a max scan, n_skip as a reflected walk, the break by ballot), with DPP scans
// confined to the half (row_shr 1/2/4/8, then row_bcast:15 into the odd row) and the per-half
// scalars (max_f, max_j, n_skip, the visited count) in SGPR pairs.
//
// Window start without a walk. A block is routed here only when its x are sorted and x + max_dist_x
// cannot wrap (checked on the host per call): then "x_i > x_j + max_dist_x" is monotone in j and the
// reference's st(i) is the first j where it fails, clamped to i - max_iter, so candidate j is in the
// window iff !(x_i > x_j + max_dist_x) && j >= i - max_iter -- a per-lane predicate on data the lane
// loads anyway. Other blocks (unsorted calls, fix-ups) stay on chain_kernel.
//
// LDS per half: a 128-entry ring of anchors {x, y, score, parent, peak, stamp} (as five arrays). x and y of anchors
// [i, i+32) are staged from HBM one 32-anchor block ahead; score/parent/peak enter when an anchor
// is resolved and leave for HBM 32 anchors at a time; "targets[j] == i" marks of the current anchor are i+1 stamps at the parents' entries
// (positions >= i-64, the two ring steps). Candidates older than 64 anchors (rare: no break within
// 64 and a wider window) are read from HBM after a vmcnt drain, with the marks taken from the
// global marks array (every visited lane stores its mark there: the targets output for final
// blocks, a scratch array for speculative segments) plus a DPP OR-scan for marks inside the step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <mutex>
#include <set>
#include <utility>
#include <cstdlib>
#include <cstdint>

#include "../../include/gb_chain.h"
#include "gb_common.h"
#include "chain_dev.h"
#include "chain_internal.h"

namespace gbchain {

namespace {

struct RowArgs {
  const VCall *vc;
  int nvc;
  const float *avg_qspan;
  const int32_t *params4;
  const uint64_t *x, *y;
  int32_t *score, *parent, *target, *peak;
  int32_t *s_score, *s_parent, *s_mark;
  unsigned long long *visited;
  int32_t prio_n;  // the longest block's length (wave priorities), 0: no priorities
};

constexpr int kRowRing = 128;           // ring entries per half (anchors [i-64, i+64) are live)
// Per half the ring is five arrays (structure of arrays, word offsets): x and y (2 words per entry),
// {score, parent}, peak, stamp. Lanes read consecutive entries, so every array is read at its own
// stride and conflict-free; an interleaved 8-word entry put a step's 32 stamp reads in 4 banks and
// made 61 % of the kernel's LDS cycles bank conflicts (SQ_LDS_BANK_CONFLICT, profiles/r04b_lds.json).
constexpr int kXW = 0, kYW = 2 * kRowRing, kSW = 4 * kRowRing, kPW = 6 * kRowRing, kTW = 7 * kRowRing;
constexpr int kHalfWords = 8 * kRowRing;

// inclusive scans over each 32-lane half: row_shr 1/2/4/8 inside the 16-lane rows, then the even
// row's lane 15 into the odd row (row_bcast:15 with row_mask 0b1010)
__device__ __forceinline__ int32_t hmax(int32_t v) {
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x111, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x112, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x114, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x118, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x142, 0xA, 0xF, false));
  return v;
}
__device__ __forceinline__ int32_t hmin(int32_t v) {
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x111, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x112, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x114, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x118, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x142, 0xA, 0xF, false));
  return v;
}
__device__ __forceinline__ int32_t hadd(int32_t v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
  return v;
}
__device__ __forceinline__ uint32_t hor(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
  return v;
}

// geometry() (chain_dev.h) for the blocks chain_rows takes: x sorted and x + max_dist_x without
// wrap, so on a lane in the window 0 <= x_i - x_j <= max_dist_x < 2^31 and dr is exact in 32 bits
// (lanes outside the window are masked by `valid`, whatever their dr). Same filters, same C integer
// and double arithmetic otherwise (host_kernel.cpp:59-79).
__device__ __forceinline__ bool geometry32(uint32_t xi_lo, uint32_t yi_lo, uint32_t yi_hi, uint32_t xj_lo,
                                           uint32_t yj_lo, uint32_t yj_hi, bool valid, int max_dist_x,
                                           int max_dist_y, int bw, int n_segs, double avg_qspan, int32_t &sg) {
  const int32_t q_span = (int32_t)(yi_hi & 0xff);
  const bool same = ((yi_hi ^ yj_hi) & 0xff0000u) == 0;  // seed segment ids, bits 48-55 of y
  const int32_t dr = (int32_t)(xi_lo - xj_lo);
  const int32_t dq = (int32_t)yi_lo - (int32_t)yj_lo;
  const int32_t dd = dr > dq ? dr - dq : dq - dr;
  const bool ok = valid & !((same & (dr == 0)) | (dq <= 0)) & !((same & (dq > max_dist_y)) | (dq > max_dist_x)) &
                  !(same & (dd > bw)) & !((n_segs > 1) & same & (dr > max_dist_y));  // is_cdna = 0
  const int32_t min_d = dq < dr ? dq : dr;
  const int log_dd = dd ? ilog2_32((uint32_t)dd) : 0;
  const int c_lin = (int)((double)dd * .01 * avg_qspan);
  const int32_t s0 = min_d > q_span ? q_span : min_d;
  const int32_t gap_diff = dr == 0 ? 0 : (c_lin < log_dd ? c_lin : log_dd);
  const int32_t gap_same = c_lin + (log_dd >> 1);
  const int32_t bonus = (!same & (dr == 0)) ? 1 : 0;
  sg = s0 + bonus - (same ? gap_same : gap_diff);
  return ok;
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef int32_t v2i __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(64) void chain_rows(RowArgs A) {
  // two rings (one per half) and 64 dummy words for lanes with no stamp to write; one array, so the
  // compiler keeps every LDS access in program order
  __shared__ __attribute__((aligned(16))) uint32_t L[2 * kHalfWords + 64];
  const int lane = threadIdx.x, hl = lane & 31;
  const bool hi = lane >= 32;
  const int bi = 2 * blockIdx.x + (hi ? 1 : 0);
  // this half's block (n = 0 for the spare half of an odd table)
  VCall V;
  V.in = V.out = 0;
  V.n = 0;
  V.call = 0;
  V.mode = kVFinal;
  if (bi < A.nvc) V = A.vc[bi];
  const int32_t n = V.n;
  const int32_t n0 = __builtin_amdgcn_readlane(n, 0), n1 = __builtin_amdgcn_readlane(n, 32);
  const int32_t nmax = max(n0, n1);
  if (nmax <= 0) return;
  // the longest blocks are the critical path of the launch: their waves issue first on a busy SIMD
  // (priority 3 from half the longest block's length, 2 from a quarter, 1 from an eighth)
  if (A.prio_n > 0) {
    if (nmax * 2 >= A.prio_n)
      __builtin_amdgcn_s_setprio(3);
    else if (nmax * 4 >= A.prio_n)
      __builtin_amdgcn_s_setprio(2);
    else if (nmax * 8 >= A.prio_n)
      __builtin_amdgcn_s_setprio(1);
  }
  const bool fin = (V.mode & kVFinal) != 0;
  const bool fin0 = __builtin_amdgcn_readlane((int)fin, 0) != 0, fin1 = __builtin_amdgcn_readlane((int)fin, 32) != 0;
  const int c = V.call;
  const int max_dist_x = A.params4[4 * c], max_dist_y = A.params4[4 * c + 1];
  const int bw = A.params4[4 * c + 2], n_segs = A.params4[4 * c + 3];
  const double avg_qspan = (double)A.avg_qspan[c];
  const uint64_t mdx = (uint64_t)(int64_t)max_dist_x;
  const uint64_t *X = A.x + V.in, *Y = A.y + V.in;
  int32_t *score = (fin ? A.score : A.s_score) + V.out, *parent = (fin ? A.parent : A.s_parent) + V.out;
  int32_t *mark = (fin ? A.target : A.s_mark) + V.out;  // zeroed by the host before the launch
  int32_t *peak = A.peak + V.out;                         // final blocks only
  uint32_t *ring = L + (hi ? kHalfWords : 0);
  uint32_t *dummy = L + 2 * kHalfWords + lane;

  // staged anchors [i, i+32) (lane hl: anchor i + hl), loaded one block ahead
  uint64_t gx = 0, gy = 0;
  if (hl < n) {
    gx = X[hl];
    gy = Y[hl];
  }
  // stamps are i + 1 >= 1: clear the half's stamp array, which holds whatever the CU's previous
  // workgroup left in this LDS (a stale value equal to i + 1 read as a mark made results depend on
  // what ran before; seen as a flaky targets / visited mismatch)
  for (int t = hl; t < kRowRing; t += 32) ring[kTW + t] = 0u;
  // anchors [a0, a0+32) of this half (lane hl: a0 + hl) from the ring to the block's outputs
  auto flush = [&](int32_t a0) {
    const int32_t a = a0 + hl;
    if (a < n) {
      const int e = a & (kRowRing - 1);
      const v2u o = *(const v2u *)(ring + kSW + 2 * e);
      score[a] = (int32_t)o.x;
      parent[a] = (int32_t)o.y;  // row blocks have pbase 0: parents are block-relative in memory too
      if (fin) peak[a] = (int32_t)ring[kPW + e];
    }
  };
  // targets[p] = i marks: one buffer store per half (the other half's lanes and the lanes with no
  // mark carry an out-of-range offset, which the buffer drops), no exec-mask branch
  const uint64_t mp = (uint64_t)(uintptr_t)mark;
  const uint64_t mp0 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mp, 0) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mp >> 32), 0) << 32);
  const uint64_t mp1 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mp, 32) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mp >> 32), 32) << 32);
  const __amdgpu_buffer_rsrc_t mr0 = __builtin_amdgcn_make_buffer_rsrc((void *)mp0, (short)0, n0 > 0 ? n0 * 4 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t mr1 = __builtin_amdgcn_make_buffer_rsrc((void *)mp1, (short)0, n1 > 0 ? n1 * 4 : 0, 0x00020000);
  auto store_mark = [&](bool w, int32_t pj, int32_t i) {
    const uint32_t off = (uint32_t)pj * 4u;
    __builtin_amdgcn_raw_buffer_store_b32(i, mr0, (w & !hi) ? off : 0xFFFFFFFFu, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(i, mr1, (w & hi) ? off : 0xFFFFFFFFu, 0, 0);
  };
  // per-half scalars (SGPR pairs): max_f, max_j, visited count
  uint32_t vis0 = 0, vis1 = 0;
  for (int32_t iv = 0; iv < nmax; iv++) {
    const int32_t i = __builtin_amdgcn_readfirstlane(iv);
    if ((i & 31) == 0) {
      // results of anchors [i-32, i) from the ring to HBM, 32 per store (the only vmcnt wait of the
      // common path is the one for the staged anchors below, once per 32 anchors)
      const int e = (i + hl) & (kRowRing - 1);
      v2u ex, ey;
      ex.x = (uint32_t)gx;
      ex.y = (uint32_t)(gx >> 32);
      ey.x = (uint32_t)gy;
      ey.y = (uint32_t)(gy >> 32);
      *(v2u *)(ring + kXW + 2 * e) = ex;
      *(v2u *)(ring + kYW + 2 * e) = ey;
      if (i > 0) flush(i - 32);
      const int32_t a = i + 32 + hl;
      if (a < n) {
        gx = X[a];
        gy = Y[a];
      }
    }
    const bool act0 = i < n0, act1 = i < n1;
    const bool act = hi ? act1 : act0;
    // own anchor (a broadcast read inside the half)
    v4u me;
    {
      const int e = i & (kRowRing - 1);
      const v2u mx_ = *(const v2u *)(ring + kXW + 2 * e), my_ = *(const v2u *)(ring + kYW + 2 * e);
      me.x = mx_.x;
      me.y = mx_.y;
      me.z = my_.x;
      me.w = my_.y;
    }
    const uint64_t xi = (uint64_t)me.x | ((uint64_t)me.y << 32);
    const int32_t q_span = (int32_t)(me.w & 0xff);
    int32_t M0 = __builtin_amdgcn_readlane(q_span, 0), M1 = __builtin_amdgcn_readlane(q_span, 32);
    int32_t J0 = -1, J1 = -1, N0 = 0, N1 = 0;
    bool go0 = act0, go1 = act1;
    const uint32_t stamp = (uint32_t)(i + 1);
    for (int32_t cs = 0;; cs++) {
      const int32_t jtop = i - 1 - 32 * cs;
      const int32_t j = jtop - hl;
      const bool go = hi ? go1 : go0;
      const bool inb = go & (j >= 0) & (j >= i - kMaxIter);
      uint64_t xj = 0, yj = 0;
      int32_t fj = 0, pj = -1;
      bool tgt;
      bool ok;
      int32_t sg;
      if (cs < 2) {
        // candidates in the ring
        const int ej = j & (kRowRing - 1);
        const v2u gx_ = *(const v2u *)(ring + kXW + 2 * ej), gy_ = *(const v2u *)(ring + kYW + 2 * ej);
        v4u g;
        g.x = gx_.x;
        g.y = gx_.y;
        g.z = gy_.x;
        g.w = gy_.y;
        const v2i r = *(const v2i *)(ring + kSW + 2 * ej);
        xj = (uint64_t)g.x | ((uint64_t)g.y << 32);
        yj = (uint64_t)g.z | ((uint64_t)g.w << 32);
        fj = r.x;
        pj = r.y;
        const bool valid = inb & !(xi > xj + mdx);
        ok = geometry32(me.x, me.z, me.w, g.x, g.z, g.w, valid, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sg);
        // "targets[j] == i": stamps at the parents of this anchor's visited candidates; lanes past
        // the break also stamp, but only positions after the break, which are never read
        const bool writer = ok & (pj >= i - 64) & (pj >= 0);
        uint32_t *sp = writer ? ring + kTW + (pj & (kRowRing - 1)) : dummy;
        *sp = stamp;
        tgt = ring[kTW + ej] == stamp;
        // (valid is needed below for the visited count)
        const uint64_t vm = __builtin_amdgcn_ballot_w64(valid);
        // ---- resolution (shared with the memory path below) ----
        const int32_t sc = ok ? (int32_t)((uint32_t)sg + (uint32_t)fj) : INT_MIN;
        const int32_t mx = hmax(sc);
        const int32_t Mh = hi ? M1 : M0, Nh = hi ? N1 : N0;
        const int32_t sh = dpp_shr_i32(mx, INT_MIN);
        const int32_t before = hl == 0 ? Mh : max(sh, Mh);
        const bool upd = sc > before;
        const bool plus = ok & !upd & tgt;
        const int32_t D = hadd(plus ? 1 : (upd ? -1 : 0));
        const int32_t na = max(Nh + D, D - hmin(D));
        const uint64_t bm = __builtin_amdgcn_ballot_w64(plus & (na > kMaxSkip));
        const uint64_t um = __builtin_amdgcn_ballot_w64(upd);
        const uint32_t bm0 = (uint32_t)bm, bm1 = (uint32_t)(bm >> 32);
        const uint32_t bl0 = (bm0 - 1) & ~bm0, bl1 = (bm1 - 1) & ~bm1;  // lanes before the break
        const uint32_t um0 = (uint32_t)um & bl0, um1 = (uint32_t)(um >> 32) & bl1;
        const uint32_t vm0 = (uint32_t)vm, vm1 = (uint32_t)(vm >> 32);
        const int lu0 = um0 ? 31 - __builtin_clz(um0) : 0, lu1 = um1 ? 31 - __builtin_clz(um1) : 0;
        const int32_t m0 = __builtin_amdgcn_readlane(mx, lu0), m1 = __builtin_amdgcn_readlane(mx, 32 + lu1);
        if (um0) {
          M0 = m0;
          J0 = jtop - lu0;
        }
        if (um1) {
          M1 = m1;
          J1 = jtop - lu1;
        }
        N0 = __builtin_amdgcn_readlane(na, 31);
        N1 = __builtin_amdgcn_readlane(na, 63);
        vis0 += bm0 ? (uint32_t)__builtin_ctz(bm0) + 1 : (uint32_t)__builtin_popcount(vm0);
        vis1 += bm1 ? (uint32_t)__builtin_ctz(bm1) + 1 : (uint32_t)__builtin_popcount(vm1);
        // the mark of every visited candidate: targets[parent[j]] = i
        const uint32_t blh = hi ? bl1 : bl0;
        store_mark(ok & (pj >= 0) & (bool)((blh >> hl) & 1), pj, i);
        go0 = go0 & (bm0 == 0) & (bool)(vm0 >> 31);
        go1 = go1 & (bm1 == 0) & (bool)(vm1 >> 31);
      } else {
        // rare: candidates older than the ring, from HBM. This wave's score/parent/mark stores must
        // have reached L2 before these sc1 loads read them.
        __builtin_amdgcn_s_waitcnt(0);
        bool valid = false;
        int32_t mk = 0;
        if (inb) {
          xj = X[j];
          yj = Y[j];
          valid = !(xi > xj + mdx);
          fj = load_l2(score + j);
          pj = load_l2(parent + j);
          mk = load_l2(mark + j);
        }
        ok = geometry32(me.x, me.z, me.w, (uint32_t)xj, (uint32_t)yj, (uint32_t)(yj >> 32), valid, max_dist_x,
                        max_dist_y, bw, n_segs, avg_qspan, sg);
        // marks from earlier steps of this anchor (in memory) and from earlier lanes of this step
        const int32_t dl = jtop - pj;  // the lane of position pj in this step
        const uint32_t oh = (ok & (pj >= 0) & (dl > hl) & (dl < 32)) ? (1u << (dl & 31)) : 0u;
        tgt = (mk == i) | (bool)((hor(oh) >> hl) & 1);
        const uint64_t vm = __builtin_amdgcn_ballot_w64(valid);
        const int32_t sc = ok ? (int32_t)((uint32_t)sg + (uint32_t)fj) : INT_MIN;
        const int32_t mx = hmax(sc);
        const int32_t Mh = hi ? M1 : M0, Nh = hi ? N1 : N0;
        const int32_t sh = dpp_shr_i32(mx, INT_MIN);
        const int32_t before = hl == 0 ? Mh : max(sh, Mh);
        const bool upd = sc > before;
        const bool plus = ok & !upd & tgt;
        const int32_t D = hadd(plus ? 1 : (upd ? -1 : 0));
        const int32_t na = max(Nh + D, D - hmin(D));
        const uint64_t bm = __builtin_amdgcn_ballot_w64(plus & (na > kMaxSkip));
        const uint64_t um = __builtin_amdgcn_ballot_w64(upd);
        const uint32_t bm0 = (uint32_t)bm, bm1 = (uint32_t)(bm >> 32);
        const uint32_t bl0 = (bm0 - 1) & ~bm0, bl1 = (bm1 - 1) & ~bm1;
        const uint32_t um0 = (uint32_t)um & bl0, um1 = (uint32_t)(um >> 32) & bl1;
        const uint32_t vm0 = (uint32_t)vm, vm1 = (uint32_t)(vm >> 32);
        const int lu0 = um0 ? 31 - __builtin_clz(um0) : 0, lu1 = um1 ? 31 - __builtin_clz(um1) : 0;
        const int32_t m0 = __builtin_amdgcn_readlane(mx, lu0), m1 = __builtin_amdgcn_readlane(mx, 32 + lu1);
        if (um0) {
          M0 = m0;
          J0 = jtop - lu0;
        }
        if (um1) {
          M1 = m1;
          J1 = jtop - lu1;
        }
        N0 = __builtin_amdgcn_readlane(na, 31);
        N1 = __builtin_amdgcn_readlane(na, 63);
        vis0 += bm0 ? (uint32_t)__builtin_ctz(bm0) + 1 : (uint32_t)__builtin_popcount(vm0);
        vis1 += bm1 ? (uint32_t)__builtin_ctz(bm1) + 1 : (uint32_t)__builtin_popcount(vm1);
        const uint32_t blh = hi ? bl1 : bl0;
        if (ok & (pj >= 0) & (bool)((blh >> hl) & 1)) mark[pj] = i;
        go0 = go0 & (bm0 == 0) & (bool)(vm0 >> 31);
        go1 = go1 & (bm1 == 0) & (bool)(vm1 >> 31);
      }
      if (!(go0 | go1)) break;
    }
    // ---- outputs of anchor i ------------------------------------------------------------------
    const int32_t M = hi ? M1 : M0, J = hi ? J1 : J0;
    int32_t pkJ = M;
    if (J >= 0) {
      if (J >= i - 64) {
        pkJ = (int32_t)ring[kPW + (J & (kRowRing - 1))];
      } else if (hi ? fin1 : fin0) {  // rare: the parent's peak from HBM (final blocks keep peaks)
        __builtin_amdgcn_s_waitcnt(0);
        pkJ = load_l2(peak + J);
        __builtin_amdgcn_s_waitcnt(0);  // nothing left pending into the common path
      }
    }
    const int32_t pki = (J >= 0 && pkJ > M) ? pkJ : M;
    if (hl == 0 && act) {
      const int e = i & (kRowRing - 1);
      v2u o;
      o.x = (uint32_t)M;
      o.y = (uint32_t)J;
      *(v2u *)(ring + kSW + 2 * e) = o;
      ring[kPW + e] = (uint32_t)pki;
    }
  }
  flush((nmax - 1) & ~31);
  if (hl == 0 && fin && n > 0) atomicAdd(A.visited, (unsigned long long)(hi ? vis1 : vis0));
}

}  // namespace

// Rows of the block table (sorted x, no fix-ups): two blocks per wave. The targets of final blocks
// and the scratch marks of speculative ones must be zero (launch_table clears them).
int launch_rows(gb_chain_batch *B, const VCall *d_vc, int nvc, hipStream_t stream) {
  if (nvc <= 0) return GB_OK;
  RowArgs A;
  A.vc = d_vc;
  A.nvc = nvc;
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
  A.s_mark = B->d_smark;
  A.visited = B->d_vis;
  // the table is sorted longest first within the class (split_plan)
  const char *pe = getenv("GB_CHAIN_PRIO");
  A.prio_n = (pe && pe[0] == '0') ? 0 : B->vc.empty() ? 0 : B->vc[0].n;
  const int nwg = (nvc + 1) / 2;
  if (int st = once_per_device(0, [](const DevLimits &L) -> int {
        GB_HIP(hipFuncSetAttribute((const void *)chain_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.max_dyn));
        return GB_OK;
      }))
    return st;
  hipLaunchKernelGGL(chain_rows, dim3((unsigned)nwg), dim3(64), spread_lds(nwg, 1, sizeof(uint32_t) * (2 * kHalfWords + 64)),
                     stream, A);
  GB_HIP(hipGetLastError());
  return GB_OK;
}

size_t spread_lds(int nwg, int waves_per_wg, size_t static_lds) {
  const char *e = getenv("GB_CHAIN_SPREAD");
  if (e && e[0] == '0') return 0;
  const DevLimits &L = dev_limits();
  // waves per SIMD one round needs, then the workgroups per CU that gives
  const int64_t waves = (int64_t)nwg * waves_per_wg;
  const int64_t per_simd = std::max<int64_t>(1, (waves + 4ll * L.cus - 1) / (4ll * L.cus));
  const int64_t wg_per_cu = std::max<int64_t>(1, per_simd * 4 / waves_per_wg);
  const size_t budget = L.lds_per_cu / (size_t)wg_per_cu;
  if (budget <= static_lds + 1024) return 0;
  return std::min<size_t>(budget - static_lds - 512, L.max_dyn);
}

namespace {
constexpr int kMaxDevices = 64;
std::once_flag g_lim_once[kMaxDevices];
DevLimits g_lim[kMaxDevices];
std::mutex g_attr_mu;
std::set<std::pair<int, int>> g_attr_done;

int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  return std::min(std::max(dev, 0), kMaxDevices - 1);
}
}  // namespace

const DevLimits &dev_limits() {
  const int dev = current_device();
  std::call_once(g_lim_once[dev], [dev] {
    DevLimits L;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) {
      if (prop.multiProcessorCount > 0) L.cus = prop.multiProcessorCount;
      if (prop.maxSharedMemoryPerMultiProcessor > 0) L.lds_per_cu = prop.maxSharedMemoryPerMultiProcessor;
    }
    L.max_dyn = L.lds_per_cu > 64 * 1024 ? std::min<size_t>(96 * 1024, L.lds_per_cu - 32 * 1024) : L.lds_per_cu / 2;
    g_lim[dev] = L;
  });
  return g_lim[dev];
}

int once_per_device(int slot, int (*set)(const DevLimits &)) {
  const int dev = current_device();
  std::lock_guard<std::mutex> lk(g_attr_mu);
  if (g_attr_done.count({dev, slot})) return GB_OK;
  if (int st = set(dev_limits())) return st;
  g_attr_done.insert({dev, slot});
  return GB_OK;
}

}  // namespace gbchain
