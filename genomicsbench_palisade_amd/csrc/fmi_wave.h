// fmi_wave.h -- one read per wave64: the SMEM routines of the wave-cooperative kernels (fmi.hip's
// smem_heavy for reads the lane kernel hands over, fmi_tasks.hip's per-call kernels of the FMI_search
// class drop-in). Every lane runs the same control flow with the same scalars; the forward and LAST
// extensions are wave-uniform (all lanes compute the same backwardExt), and each backward step of
// getSMEMsOnePosOneThread extends up to 64 `prev` entries at once -- they are independent of each
// other (FMI_search.cpp:1103-1160), only the bookkeeping after them is sequential, and it becomes
// ballots:
//   * the reference's first loop stops at the first entry f with s' >= min_intv (push) or with
//     s' < min_intv and a long enough SMEM (emit it);
//   * from f on, an entry with s' >= min_intv is pushed iff s' differs from curr_s, the s' of the
//     last push -- which is always the s' of the previous entry with s' >= min_intv (an entry not
//     pushed had the same s' as that push), so each lane compares with its nearest lower such lane.
//     curr_s is an int in the reference (assigned from the int64 s, FMI_search.cpp:1103-1160), so the
//     comparison is against that s' truncated to 32 bits, as there.
// The emission order of one OnePos call is the reference's (one possible emit per j, descending, then
// the final prev[0]). emit(k, l, s, m, n) is called by every lane with the same arguments.
// The `prev` lists live in LDS: La, Lb of (max read length + 1) entries.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "fmi_index.h"

namespace gbfmi {

__device__ __forceinline__ int64_t wave_shfl64(int64_t v, int src) {
  const int lo = __shfl((int)(uint32_t)v, src), hi = __shfl((int)(v >> 32), src);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// getSMEMsOnePosOneThread for one position x of the read Q[0, L) (FMI_search.cpp:1015-1176);
// returns next_x; `calls` counts backwardExt calls (the same in every lane).
template <class Emit>
__device__ int wave_one_pos(const DevIndex &F, const uint8_t *Q, int L, int x, int min_intv, int min_seed_len,
                            PEnt *La, PEnt *Lb, int lane, uint32_t &calls, Emit &&emit) {
  const uint64_t below = (1ull << lane) - 1;
  int next_x = x + 1;
  int a = Q[x];
  if (a >= 4) return next_x;
  int64_t ck = count_of(F, a), cl = count_of(F, 3 - a), cs = count_of(F, a + 1) - ck;
  const uint32_t cm = (uint32_t)x;
  int numPrev = 0, j;
  for (j = x + 1; j < L; j++) {  // forward extension, wave-uniform
    next_x = j + 1;
    a = Q[j];
    if (a >= 4) break;
    int64_t ko, lo, so;
    bwt_ext(F, cl, ck, cs, 3 - a, ko, lo, so);
    calls++;
    if (so != cs) {
      if (lane == 0) La[numPrev] = pack_ent(Ent{ck, cl, cs, cm, (uint32_t)(j - 1)});
      numPrev++;
    }
    if (so < min_intv) {
      next_x = j;
      break;
    }
    ck = lo;
    cl = ko;
    cs = so;
  }
  if (cs >= min_intv) {
    if (lane == 0) La[numPrev] = pack_ent(Ent{ck, cl, cs, cm, (uint32_t)(j - 1)});
    numPrev++;
  }
  __syncthreads();
  // backward search: r[p] = La[numPrev - 1 - p] at first (the reversed prev array), then each step's
  // pushes in order
  PEnt *in = La, *out = Lb;
  bool rev = true;
  for (j = x - 1; j >= 0; j--) {
    a = Q[j];
    if (a > 3) break;
    int numCurr = 0;
    bool found = false;
    int64_t carry_s = -1;  // s' of the last entry with s' >= min_intv so far (the last push's)
    for (int c0 = 0; c0 < numPrev; c0 += 64) {
      const int p = c0 + lane;
      const bool valid = p < numPrev;
      PEnt pe{};
      Ent e{};
      int64_t ko = 0, lo = 0, so = 0;
      if (valid) {
        pe = in[rev ? numPrev - 1 - p : p];
        e = unpack_ent(pe);
        bwt_ext(F, e.k, e.l, e.s, a, ko, lo, so);
      }
      const bool v = valid && so >= min_intv;
      const bool em = valid && so < min_intv && (e.n - e.m + 1) >= (uint32_t)min_seed_len;
      const uint64_t vm = __ballot(v);
      if (!found) {
        const uint64_t bm = __ballot(v || em);
        if (bm == 0) continue;  // the first loop has not stopped yet: nothing pushed
        found = true;
        const int f = __builtin_ctzll(bm);
        if (!((vm >> f) & 1)) {  // the first loop stops on an emit (lanes before f have neither)
          PEnt fe;
          fe.w0 = (uint64_t)wave_shfl64((int64_t)pe.w0, f);
          fe.w1 = (uint64_t)wave_shfl64((int64_t)pe.w1, f);
          const Ent ee = unpack_ent(fe);
          emit(ee.k, ee.l, ee.s, ee.m, ee.n);
        }
      }
      const uint64_t lowv = vm & below;
      const int64_t sp = wave_shfl64(so, lowv ? 63 - __builtin_clzll(lowv) : lane);
      const int64_t curr_s = (int64_t)(int32_t)(lowv ? sp : carry_s);  // the reference's int curr_s
      const bool push = v && so != curr_s;
      const uint64_t pm = __ballot(push);
      if (push) out[numCurr + __popcll(pm & below)] = pack_ent(Ent{ko, lo, so, (uint32_t)j, e.n});
      numCurr += __popcll(pm);
      if (vm) carry_s = wave_shfl64(so, 63 - __builtin_clzll(vm));
    }
    calls += numPrev;
    __syncthreads();
    PEnt *tmp = in;
    in = out;
    out = tmp;
    rev = false;
    numPrev = numCurr;
    if (numCurr == 0) break;
  }
  if (numPrev != 0) {
    const Ent e = unpack_ent(in[rev ? numPrev - 1 : 0]);
    if ((e.n - e.m + 1) >= (uint32_t)min_seed_len) emit(e.k, e.l, e.s, e.m, e.n);
  }
  __syncthreads();
  return next_x;
}

// bwtSeedStrategyAllPosOneThread for one read (FMI_search.cpp:1256-1323), wave-uniform;
// min_seed_len as the caller passes it (fmi.cpp passes minSeedLen + 1). x0: the position to start
// from (the loop carries nothing else from one x to the next, so a read handed over at x resumes there).
template <class Emit>
__device__ void wave_last_seeds(const DevIndex &F, const uint8_t *Q, int L, int max_intv, int min_seed_len,
                                uint32_t &calls, Emit &&emit, int x0 = 0) {
  for (int x = x0; x < L;) {
    int next_x = x + 1;
    int a = Q[x];
    if (a >= 4) {
      x = next_x;
      continue;
    }
    int64_t ck = count_of(F, a), cl = count_of(F, 3 - a), cs = count_of(F, a + 1) - ck;
    const uint32_t cm = (uint32_t)x;
    bool done = false;
    for (int j = x + 1; j < L; j++) {
      next_x = j + 1;
      a = Q[j];
      if (a >= 4) break;
      int64_t ko, lo, so;
      bwt_ext(F, cl, ck, cs, 3 - a, ko, lo, so);
      calls++;
      ck = lo;
      cl = ko;
      cs = so;
      if (cs < max_intv && (uint32_t)(j - (int)cm + 1) >= (uint32_t)min_seed_len) {
        if (cs > 0) emit(ck, cl, cs, cm, (uint32_t)j);
        x = j + 1;
        done = true;
        break;
      }
    }
    if (!done) x = (int16_t)next_x;
  }
}

}  // namespace gbfmi
