// chain_step_probe.hip -- latency of the chain consumer's per-anchor step on gfx950 (MI355X), one
// wave alone on the GPU: the first-window step of csrc/chain.hip (resolve_step + the window tail)
// in a dependent loop on synthetic candidates, in variants that drop one piece each, so the
// cycles a piece adds to the critical path can be read off. Timing only; results are discarded.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o chain_step_probe \
//          chain_step_probe.hip ../../genomicsbench_palisade_amd/csrc/gb_common.cpp
#include "../../genomicsbench_palisade_amd/csrc/chain.hip"

namespace gbchain {
void chain_bt_destroy(ChainBt *) {}  // chain.hip's batch destructor references it
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)

using namespace gbchain;

enum : int {
  kNoStamp = 1,   // no LDS stamp write/read (targets from a register hash)
  kNoMax = 2,     // no max scan (mx = sc)
  kNoWalk = 4,    // no n_skip walk (never breaks)
  kNoStore = 8,   // no targets store
  kNoTail = 16,   // no parent-peak readlane (pkJ = 0)
  kWalkAll = 32,  // always run the n_skip walk (as when another step follows)
  kOrRed = 64,    // first-window marks from a register OR-reduction instead of the LDS stamps
};

// wave-wide OR of a 32-bit value, result in lane 63 (row_shr scan, then row broadcasts)
__device__ __forceinline__ uint32_t or_scan(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
  return v;
}

template <int V>
__global__ __launch_bounds__(64) void step_probe(int32_t *target, int n, int iters, int density,
                                                 unsigned long long *out) {
  __shared__ uint32_t S[kRing + 64];
  const int lane = threadIdx.x;
  for (int k = lane; k < kRing + 64; k += 64) S[k] = 0;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(target, (short)0, n * 4, 0x00020000);
  const int32_t neg_lane = -lane;
  int32_t ws = 0, wpar = -1, wpk = 0;
  uint32_t vis = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int32_t k = 0; k < iters; k++) {
    const int32_t i = __builtin_amdgcn_readfirstlane(k + 128);
    const uint32_t h = (uint32_t)i * 2654435761u ^ (uint32_t)lane * 40503u;
    const bool ok = (int)((h >> 8) & 15) < density;
    const int32_t sg = (int32_t)((h >> 20) & 31) - 6;
    const int32_t st = i - 64, jtop = i - 1;
    int32_t M = 15, N = 0, J = -1;
    const uint32_t stamp = (uint32_t)(i + 1);
    const int32_t sc = ok ? sg + ws : INT_MIN;
    const int32_t pj = wpar;
    // ---- replica of resolve_step (csrc/chain.hip) with switches ----
    uint64_t tgm;
    if (V & kNoStamp) {
      tgm = __builtin_amdgcn_ballot_w64((h & 3) == 0);
    } else if (V & kOrRed) {
      // bit (jtop - pj) for marking lanes whose parent falls inside this window
      const int32_t d = jtop - pj;
      const bool in = ok & (pj >= st) & (d >= 0) & (d < 64);
      const uint64_t one = in ? 1ull << (d & 63) : 0ull;
      const uint32_t lo = or_scan((uint32_t)one), hi = or_scan((uint32_t)(one >> 32));
      tgm = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, 63) |
            (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 32;
    } else {
      S[(ok & (pj >= st)) ? (pj & (kRing - 1)) : kRing + lane] = stamp;
      tgm = __builtin_amdgcn_ballot_w64(S[(jtop - lane) & (kRing - 1)] == stamp);
    }
    const uint64_t okm = __builtin_amdgcn_ballot_w64(ok);
    const int32_t mx = (V & kNoMax) ? sc : scan_max(sc);
    const int32_t before = max(dpp_shr_i32(mx, INT_MIN), M);
    const uint64_t um_all = __builtin_amdgcn_ballot_w64(sc > before);
    const uint64_t pm = okm & ~um_all & tgm;
    uint64_t bm = 0;
    if (!(V & kNoWalk) && ((V & kWalkAll) || (int32_t)__builtin_popcountll(pm) + N > kMaxSkip)) {
      const uint64_t num = ~um_all;
      const int32_t d_ex = (int32_t)__builtin_amdgcn_mbcnt_hi(
          (uint32_t)(num >> 32),
          __builtin_amdgcn_mbcnt_lo((uint32_t)num, __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)pm, (uint32_t)neg_lane))));
      const int32_t D = d_ex + (__builtin_amdgcn_inverse_ballot_w64(pm) ? 1 : (__builtin_amdgcn_inverse_ballot_w64(um_all) ? -1 : 0));
      const int32_t n_after = max(N + D, D - scan_min(D));
      bm = pm & __builtin_amdgcn_ballot_w64(n_after > kMaxSkip);
      N = __builtin_amdgcn_readlane(n_after, 63);
    }
    const uint64_t below = (bm - 1) & ~bm;
    vis += bm ? (uint32_t)__builtin_ctzll(bm) + 1 : 64u;
    const uint64_t um = um_all & below;
    const int lu = 63 - __builtin_clzll(um | 1);
    const int32_t m_lu = __builtin_amdgcn_readlane(mx, lu);
    J = um ? jtop - lu : J;
    M = um ? m_lu : M;
    if (!(V & kNoStore)) {
      const bool wt = __builtin_amdgcn_inverse_ballot_w64(okm & below) & (pj >= 0);
      __builtin_amdgcn_raw_buffer_store_b32(i, trs, wt ? (uint32_t)pj * 4u : 0xFFFFFFFFu, 0, 0);
    }
    // ---- the window tail ----
    const int32_t dJ = i - 1 - J;
    const int32_t pkJ = (V & kNoTail) ? 0 : __builtin_amdgcn_readlane(wpk, dJ & 63);
    const int32_t pki = (J >= 0 && pkJ > M) ? pkJ : M;
    ws = dpp_shr_i32(ws, M);
    wpar = dpp_shr_i32(wpar, J);
    wpk = dpp_shr_i32(wpk, pki);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = vis;
  }
  target[lane] = ws ^ wpar ^ wpk;
}

template <int V>
int run(const char *name, int32_t *d_t, unsigned long long *d_o, int density) {
  const int iters = 200000;
  unsigned long long h[2];
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(step_probe<V>, dim3(1), dim3(64), 0, 0, d_t, 1 << 20, iters, density, d_o);
    CK(hipDeviceSynchronize());
  }
  CK(hipMemcpy(h, d_o, sizeof(h), hipMemcpyDeviceToHost));
  printf("%-34s density %2d/16: %7.1f cycles per step (visited/step %.1f)\n", name, density, (double)h[0] / iters,
         (double)h[1] / iters);
  return 0;
}

int main() {
  int32_t *d_t;
  unsigned long long *d_o;
  CK(hipMalloc(&d_t, (1 << 20) * 4));
  CK(hipMalloc(&d_o, 16));
  for (int density : {4, 14}) {
    if (run<0>("full step", d_t, d_o, density)) return 1;
    if (run<kWalkAll>("full step, walk always", d_t, d_o, density)) return 1;
    if (run<kNoStamp>("- LDS stamp round trip", d_t, d_o, density)) return 1;
    if (run<kOrRed>("stamps -> register OR-reduction", d_t, d_o, density)) return 1;
    if (run<kNoMax>("- max scan", d_t, d_o, density)) return 1;
    if (run<kNoWalk>("- n_skip walk", d_t, d_o, density)) return 1;
    if (run<kNoStore>("- targets store", d_t, d_o, density)) return 1;
    if (run<kNoTail>("- parent-peak readlane", d_t, d_o, density)) return 1;
    if (run<kNoStamp | kNoMax | kNoWalk | kNoStore | kNoTail>("skeleton (tail shifts + M/J only)", d_t, d_o, density))
      return 1;
  }
  return 0;
}
