// chain.hip -- MI355X (gfx950) minimap2 chaining DP (chain_dp): kernel and C ABI.
//
// Semantics: benchmarks/chain/src/host_kernel.cpp:405-472 (plaintext branch) ==
// tools/minimap2-acceleration/kernel/scalar/src/host_kernel.cpp:30-94, with the C integer / double
// semantics of that source (int64 dr, int32 truncations, (int)(dd * .01 * avg_qspan), no FMA).
//
// MI355X design: one call (read) per wave64; anchors are processed in order i (score[i] depends on
// score[j < i]) and the predecessor loop j = i-1 .. st runs 64 candidates per step, lane l taking
// j = jtop - l, i.e. lanes in the reference's visiting order. The reference loop is sequential only
// through three quantities, each turned into a wave-wide prefix scan:
//   max_f        running maximum of the candidate scores             (max scan)
//   n_skip       max(n-1, 0) on an improvement, n+1 on a "targeted" non-improvement
//                -> compositions of n -> max(n + a, b), closed under composition (pair scan)
//   break        first lane where n_skip exceeds 25                   (ballot + ctz)
// "targets[j] == i" is decided by marks from earlier-visited j' (> j) of the same i, which are all
// visited before any break that could stop j: marks are i+1 stamps in an LDS ring indexed by j.
// The last 64 anchors (the first step of every i) live in registers, shifted one lane per i with
// DPP, so most anchors need no memory access at all; older candidates are read from global memory
// through L2 (sc1 loads) after a periodic vmcnt drain that orders the wave's own stores before them.
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
  unsigned long long *prof;  // optional phase clocks (GB_CHAIN_PROF=1): head, steps, tail, nsteps
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

constexpr int32_t kNegB = -(1 << 28);

// anchors are read-only for the whole kernel: the constant address space turns the uniform X[st]
// reads of the window-start loop into scalar loads (lgkmcnt), so they never wait behind the
// wave's outstanding score/parent/peak stores (vmcnt)
typedef const __attribute__((address_space(4))) uint64_t const_u64;  // identity of the n_skip composition scan

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
// (a, b) represents n -> max(n + a, b); earlier lanes apply first: (a1,b1) then (a2,b2) =
// (a1 + a2, max(b1 + a2, b2)). Identity (0, kNegB).
template <int CTRL, int ROWS>
__device__ __forceinline__ void compose_step(int32_t &a, int32_t &b) {
  const int32_t ua = __builtin_amdgcn_update_dpp(0, a, CTRL, ROWS, 0xF, false);
  const int32_t ub = __builtin_amdgcn_update_dpp(kNegB, b, CTRL, ROWS, 0xF, false);
  b = max(ub + a, b);
  a = ua + a;
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
// number of set bits of m in lanes 0..lane (inclusive)
__device__ __forceinline__ int32_t incl_count(uint64_t m, int lane) {
  const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  return below + (int)((m >> lane) & 1);
}
__device__ __forceinline__ void scan_compose(int32_t &a, int32_t &b) {
  compose_step<0x111, 0xF>(a, b);
  compose_step<0x112, 0xF>(a, b);
  compose_step<0x114, 0xF>(a, b);
  compose_step<0x118, 0xF>(a, b);
  compose_step<0x142, 0xA>(a, b);
  compose_step<0x143, 0xC>(a, b);
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
  const bool ok = valid && !((same && dr == 0) || dq <= 0) && !((same && dq > max_dist_y) || dq > max_dist_x) &&
                  !(same && dd > bw) && !(n_segs > 1 && same && dr > max_dist_y);  // is_cdna = 0
  const int32_t min_d = (int32_t)(dq < dr ? (int64_t)dq : dr);
  const int log_dd = dd ? ilog2_32((uint32_t)dd) : 0;
  const int c_lin = (int)((double)dd * .01 * avg_qspan);
  int32_t s0 = min_d > q_span ? q_span : min_d;
  int gap_cost;
  if (!same) {
    s0 += dr == 0 ? 1 : 0;
    gap_cost = dr == 0 ? 0 : (c_lin < log_dd ? c_lin : log_dd);
  } else {
    gap_cost = c_lin + (log_dd >> 1);
  }
  // (int)((double)gap_cost * gap_scale + .499) with gap_scale == 1.0f (host_kernel.cpp:36) is
  // gap_cost itself for 0 <= gap_cost < 2^31
  sg = s0 - gap_cost;
  return ok;
}

// One 64-candidate step in visiting order (lane l = j = jtop - l): running max_f, n_skip, the
// break and the targets/stamps. Updates M, J, N; returns the break lane (64 = none).
__device__ __forceinline__ int resolve_step(int32_t sc, bool ok, bool valid, int32_t pj, int64_t j, int64_t jtop,
                                            int64_t st, uint32_t stamp, int lane, int32_t *__restrict__ target,
                                            int64_t i, uint32_t *S, int32_t &M, int64_t &J, int32_t &N,
                                            unsigned long long &vis) {
  // "targets[j] == i": stamps from visited j' > j with parents[j'] == j
  if (ok && pj >= st) S[pj & (kRing - 1)] = stamp;
  const bool tgt = valid && S[j & (kRing - 1)] == stamp;
  const int32_t mx = scan_max(ok ? sc : INT_MIN);  // inclusive max scan
  const int32_t before = max(dpp_shr_i32(mx, INT_MIN), M);
  const bool upd = ok && sc > before;
  // n_skip after lane l as a reflected walk: steps +1 (target, no update), -1 floored at 0 (update),
  // so n_l = max(N + D_l, D_l - min_{k<=l} D_k) with D_l the inclusive step sum -- D from two
  // ballots and mbcnt, the running minimum from one DPP scan
  const bool plus = ok && !upd && tgt;
  const uint64_t pm = __ballot(plus), um_all = __ballot(upd);
  const int32_t D = incl_count(pm, lane) - incl_count(um_all, lane);
  const int32_t n_after = max(N + D, D - scan_min(D));
  const bool brk = plus && n_after > kMaxSkip;
  const uint64_t bm = __ballot(brk);
  const int bl = bm ? __builtin_ctzll(bm) : 64;
  const int64_t nvalid = min((int64_t)64, jtop - st + 1);
  vis += (bl < 64) ? (unsigned long long)(bl + 1) : (unsigned long long)nvalid;
  const uint64_t low = bl >= 64 ? ~0ull : ((1ull << bl) - 1);
  const uint64_t um = um_all & low;
  if (um) {
    const int lu = 63 - __builtin_clzll(um);
    J = jtop - lu;
    M = __builtin_amdgcn_readlane(mx, lu);
  }
  if (ok && lane < bl && pj >= 0) target[pj] = (int32_t)i;
  N = __builtin_amdgcn_readlane(n_after, 63);
  return bl;
}

// Producer -> consumer hand-off, one slot per anchor i: the geometry of its first 64 candidates.
constexpr int kSlots = 16;
struct Slot {
  int32_t sg[64];
  uint64_t okmask;
  int64_t st;
  uint64_t xi, yi;
};

// Two waves per call. The anchors' pair geometry (filters, gap costs; no scores involved) runs ahead
// in the producer wave and is handed over through an LDS ring; the consumer wave keeps only the
// score-dependent sequential part (max_f / n_skip scans, break, targets, outputs), so the critical
// path of a long call is roughly halved. Hand-off words are LDS counters polled with s_sleep.
__global__ __launch_bounds__(128) void chain_kernel(Args A) {
  __shared__ uint32_t S[kRing];
  __shared__ Slot ring[kSlots];
  __shared__ int produced, consumed;
  const int c = A.order[blockIdx.x];
  const int lane = threadIdx.x & 63;
  const bool producer = threadIdx.x >= 64;
  const int64_t o = A.offsets[c];
  const int64_t n = A.offsets[c + 1] - o;
  const int max_dist_x = A.params4[4 * c], max_dist_y = A.params4[4 * c + 1];
  const int bw = A.params4[4 * c + 2], n_segs = A.params4[4 * c + 3];
  const double avg_qspan = (double)A.avg_qspan[c];
  const uint64_t *X = A.x + o, *Y = A.y + o;
  const const_u64 *XC = (const const_u64 *)X, *YC = (const const_u64 *)Y;
  int32_t *score = A.score + o, *parent = A.parent + o, *target = A.target + o, *peak = A.peak + o;

  for (int k = threadIdx.x; k < kRing; k += 128) S[k] = 0;
  for (int64_t k = threadIdx.x; k < n; k += 128) target[k] = 0;  // a fresh std::vector in the reference
  if (threadIdx.x == 0) produced = consumed = 0;
  __builtin_amdgcn_s_waitcnt(0);  // zeroing stores complete before any later targets store
  __syncthreads();

  if (producer) {
    // ---------------- producer: geometry of anchor i against i-1-lane --------------------------
    uint64_t wx = 0, wy = 0;  // lane l: anchor i-1-l
    int64_t st = 0;
    for (int64_t i = 0; i < n; i++) {
      const uint64_t xi = XC[i], yi = YC[i];
      while (st < i && xi > XC[st] + (uint64_t)(int64_t)max_dist_x) ++st;
      if (i - st > kMaxIter) st = i - kMaxIter;
      int32_t sg;
      const bool ok = geometry(xi, yi, wx, wy, i - 1 - lane >= st, max_dist_x, max_dist_y, bw, n_segs, avg_qspan, sg);
      const uint64_t okm = __ballot(ok);
      // wait for a free slot
      while (i - (int64_t)__hip_atomic_load(&consumed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= kSlots)
        __builtin_amdgcn_s_sleep(1);
      Slot &sl = ring[i & (kSlots - 1)];
      sl.sg[lane] = sg;
      if (lane == 0) {
        sl.okmask = okm;
        sl.st = st;
        sl.xi = xi;
        sl.yi = yi;
      }
      __builtin_amdgcn_s_waitcnt(0);  // slot contents land before the count that publishes them
      if (lane == 0) __hip_atomic_store(&produced, (int)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      wx = dpp_shr_u64(wx, xi);
      wy = dpp_shr_u64(wy, yi);
    }
    return;
  }

  // ---------------- consumer ---------------------------------------------------------------------
  int32_t ws = 0, wpar = -1, wpk = 0;  // lane l: score/parent/peak of anchor i-1-l
  unsigned long long vis = 0;
  unsigned long long c_head = 0, c_step = 0, c_tail = 0, n_step = 0, t_0 = 0, t_1 = 0;
  const bool prof = A.prof != nullptr;
  for (int64_t i = 0; i < n; i++) {
    if (prof) t_0 = __builtin_amdgcn_s_memtime();
    if ((i & 63) == 0 && i > 0) {  // flush the window: anchors i-64 .. i-1 (lane l: i-1-l)
      score[i - 1 - lane] = ws;
      parent[i - 1 - lane] = wpar;
      peak[i - 1 - lane] = wpk;
      __builtin_amdgcn_s_waitcnt(0);  // flushed anchors are in L2 before any older-candidate read
    }
    while ((int64_t)__hip_atomic_load(&produced, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= i)
      __builtin_amdgcn_s_sleep(1);
    const Slot &sl = ring[i & (kSlots - 1)];
    const int32_t sg = sl.sg[lane];
    const bool ok = (sl.okmask >> lane) & 1;
    const int64_t st = sl.st;
    const uint64_t xi = sl.xi, yi = sl.yi;
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0) __hip_atomic_store(&consumed, (int)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int32_t q_span = (int32_t)(yi >> 32 & 0xff);
    int32_t M = q_span, N = 0;
    int64_t J = -1;
    const uint32_t stamp = (uint32_t)(i + 1);
    if (prof) {
      t_1 = __builtin_amdgcn_s_memtime();
      c_head += t_1 - t_0;
      t_0 = t_1;
    }
    const int64_t jtop = i - 1;
    int bl = 64;
    if (jtop >= st) {
      if (prof) ++n_step;
      const int64_t j = jtop - lane;
      bl = resolve_step(ok ? sg + ws : INT_MIN, ok, j >= st, wpar, j, jtop, st, stamp, lane, target, i, S, M, J, N, vis);
    }
    if (bl == 64 && jtop - 64 >= st) {  // rare: older candidates (j < i-64) from memory
      for (int64_t jt = jtop - 64; jt >= st; jt -= 64) {
        if (prof) ++n_step;
        const int64_t jj = jt - lane;
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
        if (resolve_step(oko ? sgo + scj : INT_MIN, oko, v, pj, jj, jt, st, stamp, lane, target, i, S, M, J, N,
                         vis) < 64)
          break;
      }
    }
    if (prof) {
      t_1 = __builtin_amdgcn_s_memtime();
      c_step += t_1 - t_0;
      t_0 = t_1;
    }
    int32_t pkJ = 0;
    if (J >= 0) {
      if (J >= i - 64)
        pkJ = __builtin_amdgcn_readlane(wpk, (int)(i - 1 - J));
      else  // rare: consume the load inside the branch so the common path carries no vmcnt wait
        pkJ = __builtin_amdgcn_readfirstlane(load_l2(peak + J));
    }
    const int32_t pki = (J >= 0 && pkJ > M) ? pkJ : M;
    ws = dpp_shr_i32(ws, M);
    wpar = dpp_shr_i32(wpar, (int32_t)J);
    wpk = dpp_shr_i32(wpk, pki);
    if (prof) c_tail += __builtin_amdgcn_s_memtime() - t_0;
  }
  // final flush: anchors max(0, n - r) .. n-1 with r = n mod 64 (or 64)
  {
    const int64_t r = ((n - 1) & 63) + 1;
    if (lane < r) {
      score[n - 1 - lane] = ws;
      parent[n - 1 - lane] = wpar;
      peak[n - 1 - lane] = wpk;
    }
  }
  // wave-reduce the visited count
  if (prof && lane == 0) {
    atomicAdd(A.prof + 0, c_head);
    atomicAdd(A.prof + 1, c_step);
    atomicAdd(A.prof + 2, c_tail);
    atomicAdd(A.prof + 3, n_step);
  }
  for (int d = 32; d >= 1; d >>= 1) vis += __shfl_xor(vis, d);
  if (lane == 0) atomicAdd(A.visited, vis / 64);
}

}  // namespace gbchain

extern "C" {

int gb_chain_batch_create(int64_t ncalls, const int64_t *offsets, const float *avg_qspan,
                          const int32_t *params4, const uint64_t *x, const uint64_t *y,
                          gb_chain_batch **out) {
  GB_ARG(out && ncalls >= 0 && offsets, "gb_chain_batch_create: bad arguments");
  GB_ARG(ncalls < (1ll << 31), "gb_chain_batch_create: too many calls");
  *out = nullptr;
  const int64_t na = offsets[ncalls];
  GB_ARG(offsets[0] == 0 && na >= 0 && (na == 0 || (x && y)), "gb_chain_batch_create: bad offsets");
  for (int64_t c = 0; c < ncalls; c++)
    GB_ARG(offsets[c + 1] >= offsets[c] && offsets[c + 1] - offsets[c] < (1ll << 31),
           "gb_chain_batch_create: call %lld has a bad anchor range", (long long)c);
  GB_ARG(ncalls == 0 || (avg_qspan && params4), "gb_chain_batch_create: null parameters");
  // longest calls first: the grid is dispatched in order, so the critical path starts first
  std::vector<int32_t> order((size_t)ncalls);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    return offsets[a + 1] - offsets[a] > offsets[b + 1] - offsets[b];
  });
  auto *B = new gb_chain_batch();
  B->ncalls = ncalls;
  B->nanchors = na;
  hipError_t e = hipGetDevice(&B->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&B->stream, hipStreamNonBlocking);
  for (auto &ev : B->ev)
    if (e == hipSuccess) e = hipEventCreate(&ev);
  const size_t nc = (size_t)std::max<int64_t>(ncalls, 1), nn = (size_t)std::max<int64_t>(na, 1);
  if (e == hipSuccess) e = hipMalloc(&B->d_off, (nc + 1) * sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc(&B->d_aq, nc * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&B->d_par4, nc * 4 * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&B->d_order, nc * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&B->d_x, nn * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMalloc(&B->d_y, nn * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMalloc(&B->d_out, nn * 4 * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&B->d_vis, sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpy(B->d_off, offsets, (size_t)(ncalls + 1) * sizeof(int64_t), hipMemcpyHostToDevice);
  if (e == hipSuccess && ncalls) e = hipMemcpy(B->d_aq, avg_qspan, (size_t)ncalls * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess && ncalls) e = hipMemcpy(B->d_par4, params4, (size_t)ncalls * 16, hipMemcpyHostToDevice);
  if (e == hipSuccess && ncalls) e = hipMemcpy(B->d_order, order.data(), (size_t)ncalls * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && na) e = hipMemcpy(B->d_x, x, (size_t)na * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess && na) e = hipMemcpy(B->d_y, y, (size_t)na * 8, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    gb::set_error("gb_chain_batch_create: %s", hipGetErrorString(e));
    gb_chain_batch_destroy(B);
    return GB_ERR_HIP;
  }
  *out = B;
  return GB_OK;
}

int gb_chain_batch_run(gb_chain_batch *B) {
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
    const char *pe = getenv("GB_CHAIN_PROF");
    if (pe && *pe == '1') {
      if (!B->d_prof) GB_HIP(hipMalloc(&B->d_prof, 4 * sizeof(unsigned long long)));
      GB_HIP(hipMemsetAsync(B->d_prof, 0, 4 * sizeof(unsigned long long), B->stream));
      A.prof = B->d_prof;
    }
    hipLaunchKernelGGL(gbchain::chain_kernel, dim3((unsigned)B->ncalls), dim3(128), 0, B->stream, A);
    GB_HIP(hipGetLastError());
  }
  GB_HIP(hipEventRecord(B->ev[1], B->stream));
  if (B->d_prof && getenv("GB_CHAIN_PROF")) {
    unsigned long long h[4];
    GB_HIP(hipMemcpyAsync(h, B->d_prof, sizeof(h), hipMemcpyDeviceToHost, B->stream));
    GB_HIP(hipStreamSynchronize(B->stream));
    fprintf(stderr, "[chain prof] memtime ticks: head %llu steps %llu tail %llu; steps %llu\n", h[0], h[1],
            h[2], h[3]);
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
  gb_chain_batch *B = nullptr;
  int st = gb_chain_batch_create(ncalls, offsets, avg_qspan, params4, x, y, &B);
  if (st) return st;
  st = gb_chain_batch_run(B);
  if (!st) st = gb_chain_batch_results(B, scores, parents, targets, peak_scores, nullptr);
  gb_chain_batch_destroy(B);
  return st;
}

}  // extern "C"
