// phmm.hip -- MI355X (gfx950) PairHMM forward pass: host tables, batch packing, HIP kernels, C ABI.
//
// Arithmetic contract: the GKL recurrence
//   M[r][c] = ((M[r-1][c-1]*pMM + X[r-1][c-1]*pGAPM) + Y[r-1][c-1]*pGAPM) * dist(r,c)
//   X[r][c] = M[r-1][c]*pMX + X[r-1][c]*pXX
//   Y[r][c] = M[r][c-1]*pMY + Y[r][c-1]*pYY
// (tools/GKL/src/main/native/pairhmm/avx-pairhmm-template.h:183-198) with Y[0][*] = 2^120/haplen
// (f32) or 2^1020/haplen (f64), every other boundary 0, result = sum_c M[R][c] + sum_c X[R][c]
// (:299-344), f64 recomputation when the f32 result < 1e-28f (IntelPairHmmCSource.cpp:70-79).
// Must be built with -ffp-contract=off: no FMA anywhere, so every cell is bit-identical to the
// reference's AVX kernels.
//
// MI355X design: one testcase per wave64; the read is cut into stripes of 64 rows, lane k owns row
// r0+k and the wave sweeps anti-diagonals (step t: lane k is at column t-k+1). Values move one lane
// down per step with DPP wave_shr:1 (no LDS round trip); lane 0 takes the row above the stripe from
// one uniform LDS record per step, every lane reads the haplotype code of its own column from an
// LDS byte array, and lane 63 writes the stripe's last row back into the records (in place: the
// write index trails the read index by 63 columns). The f32 pass appends testcases that need f64 to a device list; a second kernel
// recomputes them in f64. Testcases are ordered by descending cost so the dispatcher balances waves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/gb_phmm.h"
#include "gb_common.h"

namespace {

constexpr int kWave = 64;
// Longest haplotype: the f64 kernel's LDS (16-B boundary record + 1 code byte per column, plus
// kBndPad + kWave pad columns) must fit the 160 KB of one CU.
constexpr int kMaxHaplen = 9400;
constexpr int kBndPad = 72;  // boundary records beyond column C (see phmm_stripe reads)
constexpr int kQualTab = 128;
constexpr int kM2M = ((127 * 128) >> 1) + 128;  // set_mm_prob indices for quals < 128

// ---------------------------------------------------------------------------------------------
// Host tables: Context<float>/Context<double> (Context.h:13-190), restated.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxQual = 254;
constexpr double kJacTol = 8.0;
constexpr double kJacStep = 0.0001;
#define GB_JAC_INV_STEP (1.0 / kJacStep)
constexpr int kJacSize = (int)(kJacTol / kJacStep) + 1;

template <typename T>
struct HostTables {
  T ph2pr[kQualTab];
  T one_minus[kQualTab];  // 1 - ph2pr[x]: pGAPM (template.h:119) and 1-distm (template.h:152)
  T div3[kQualTab];       // ph2pr[x] / 3: mismatch distm (template.h:154)
  T m2m[kM2M];            // matchToMatchProb (Context.h:50-61) for quals < 128
  T init_const;           // INITIAL_CONSTANT
  T log10_init;           // LOG10_INITIAL_CONSTANT
};

template <typename T>
static int fast_round(T d) {
  return (d > (T)0.0) ? (int)(d + (T)0.5) : (int)(d - (T)0.5);
}

template <typename T>
static T log10sum(const std::vector<T> &jac, T small, T big) {
  if (small > big) std::swap(small, big);
  T diff = big - small;
  if (diff >= (T)kJacTol) return big;
  int ind = fast_round<T>((T)(diff * (T)GB_JAC_INV_STEP));
  return big + jac[ind];
}

template <typename T>
static void build_tables(HostTables<T> &t) {
  std::vector<T> jac(kJacSize);
  for (int k = 0; k < kJacSize; k++) jac[k] = (T)(log10(1.0 + pow(10.0, -((double)k) * kJacStep)));
  const double inv_ln10 = 1.0 / log(10);
  std::vector<T> m2m_full(((kMaxQual + 1) * (kMaxQual + 2)) >> 1);
  for (int i = 0, off = 0; i <= kMaxQual; off += ++i)
    for (int j = 0; j <= i; j++) {
      double s = log10sum<T>(jac, (T)(-0.1 * i), (T)(-0.1 * j));
      double l = log1p(-std::min(1.0, pow(10, s))) * inv_ln10;
      m2m_full[off + j] = (T)(pow(10, l));
    }
  for (int k = 0; k < kM2M; k++) t.m2m[k] = m2m_full[k];
  for (int x = 0; x < kQualTab; x++) {
    if constexpr (sizeof(T) == 4)
      t.ph2pr[x] = powf(10.f, -((float)x) / 10.f);
    else
      t.ph2pr[x] = pow(10.0, -((double)x) / 10.0);
    t.one_minus[x] = (T)1.0 - t.ph2pr[x];
    t.div3[x] = t.ph2pr[x] / (T)3.0;
  }
  if constexpr (sizeof(T) == 4) {
    t.init_const = ldexpf(1.f, 120);
    t.log10_init = log10f(t.init_const);
  } else {
    t.init_const = ldexp(1.0, 1020);
    t.log10_init = log10(t.init_const);
  }
}

// ConvertChar (pairhmm_common.h:30-39): A0 C1 T2 G3 N4, every other byte 0.
static uint8_t base_code(char ch) {
  switch ((uint8_t)ch) {
    case 'A': return 0;
    case 'C': return 1;
    case 'T': return 2;
    case 'G': return 3;
    case 'N': return 4;
    default: return 0;
  }
}
// Bit h set when a read base of this code matches a haplotype base of code h: equal codes, or
// either is N (mask construction in avx-pairhmm-template.h:5-27).
static uint8_t read_match_mask(uint8_t rc) { return rc == 4 ? 0x1F : (uint8_t)((1u << rc) | 0x10); }

// ---------------------------------------------------------------------------------------------
// Device side
// ---------------------------------------------------------------------------------------------
struct __attribute__((aligned(16))) TcDesc {
  uint32_t read_off;  // pool offset: rmatch[R] q[R] i[R] d[R] c[R]
  uint32_t hap_off;   // pool offset: hcode[C]
  uint32_t dims;      // rslen | haplen << 16
  uint32_t out_idx;   // position in the caller's testcase array
};

template <typename T>
struct DevTab {
  const T *ph2pr, *one_minus, *div3, *m2m;
  T init_const;
};

// Boundary record per column c (stripe above the current one): the two partial sums the first
// row of the current stripe needs from the row above, already multiplied by THAT first row's
// transition probabilities, plus the haplotype base code of column c:
//   z = (M*pMM + X*pGAPM) + Y*pGAPM   (the M recurrence's bracket, used one column later)
//   w = M*pMX + X*pXX                 (= X of the next row at the same column)
// Read by lane 0 with one uniform ds_read per step. The haplotype codes live in a separate byte
// array that every lane reads at its own column (no cross-lane traffic, no VALU).
template <typename T>
struct __attribute__((aligned(2 * sizeof(T)))) Brec {
  T z, w;
};

__device__ __forceinline__ int dpp_shr(int v, int lane0) {
  // wave_shr:1 (DPP ctrl 0x138); lane 0 has no source lane and keeps `lane0` (bound_ctrl off).
  return __builtin_amdgcn_update_dpp(lane0, v, 0x138, 0xF, 0xF, false);
}
template <int (*F)(int, int)>
__device__ __forceinline__ float dpp(float v, float keep) {
  return __builtin_bit_cast(float, F(__builtin_bit_cast(int, v), __builtin_bit_cast(int, keep)));
}
template <int (*F)(int, int)>
__device__ __forceinline__ double dpp(double v, double keep) {
  long long vb = __builtin_bit_cast(long long, v), kb = __builtin_bit_cast(long long, keep);
  int lo = F((int)(vb & 0xffffffffll), (int)(kb & 0xffffffffll));
  int hi = F((int)(vb >> 32), (int)(kb >> 32));
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
template <int (*F)(int, int)>
__device__ __forceinline__ uint32_t dpp(uint32_t v, uint32_t keep) {
  return (uint32_t)F((int)v, (int)keep);
}

// dist select without a compare: sign-extend bit `h` of the lane's match mask (0 or ~0) and
// bit-insert between the two candidates.
__device__ __forceinline__ float select_dist(uint32_t rmask, uint32_t h, float dmatch, float dmis) {
  uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)rmask, h, 1);
  uint32_t r = (m & __builtin_bit_cast(uint32_t, dmatch)) | (~m & __builtin_bit_cast(uint32_t, dmis));
  return __builtin_bit_cast(float, r);
}
// f64: the same mask applied to both halves. The mask comes from inline asm because hipcc 7.2
// mis-derives the high word of a sign-extended sbfe mask and constant-folds it; asm is opaque.
__device__ __forceinline__ double select_dist(uint32_t rmask, uint32_t h, double dmatch, double dmis) {
  uint32_t m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(rmask), "v"(h));
  const uint64_t a = __builtin_bit_cast(uint64_t, dmatch), b = __builtin_bit_cast(uint64_t, dmis);
  const uint32_t lo = (m & (uint32_t)a) | (~m & (uint32_t)b);
  const uint32_t hi = (m & (uint32_t)(a >> 32)) | (~m & (uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Per-lane constants of one stripe (initializeVectors, avx-pairhmm-template.h:83-128): the lane's
// own row (Y recurrence, emission) and the NEXT row's transitions (the partials z/w it hands down).
template <typename T>
struct RowParams {
  T pMY, pYY, dmatch, dmis;              // own row
  T nMM, nGAPM, nMX, nXX;                // row below (lane+1; lane 63: first row of next stripe)
  uint32_t rmask;
};

// Lane state between steps. Row r = lane's row, column c = step - lane + 1:
//   Mp, Yp : M[r][c-1], Y[r][c-1]           zo, wo : this lane's z/w of column c-1
//   zd     : z of row r-1 at column c-1 (= the M bracket of this lane's next cell), shifted in
template <typename T>
struct LaneState {
  T Mp, Yp, zo, wo, zd;
};

// One anti-diagonal step. Arithmetic per cell is exactly the reference's (no FMA, same order):
//   X = M[r-1][c]*pMX + X[r-1][c]*pXX         computed by lane-1 as w, shifted in
//   M = ((M*pMM + X*pGAPM) + Y*pGAPM)[r-1][c-1] * dist    bracket computed by lane-1 as z
//   Y = M[r][c-1]*pMY + Y[r][c-1]*pYY
template <typename T, bool kLast>
__device__ __forceinline__ void phmm_step(const Brec<T> &rec, uint32_t h, LaneState<T> &st,
                                          const RowParams<T> &P, T &sumM, T &sumX, Brec<T> *wr, bool last_lane) {
  const T X = dpp<dpp_shr>(st.wo, rec.w);          // X[r][c]
  const T zdn = dpp<dpp_shr>(st.zo, rec.z);        // bracket for column c+1
  const T dist = select_dist(P.rmask, h, P.dmatch, P.dmis);
  const T M = st.zd * dist;
  const T Y = st.Mp * P.pMY + st.Yp * P.pYY;
  st.zo = (M * P.nMM + X * P.nGAPM) + Y * P.nGAPM;
  st.wo = M * P.nMX + X * P.nXX;
  if constexpr (kLast) {
    sumM = sumM + M;
    sumX = sumX + X;
  } else {
    // lane 63 hands its row's z/w (the next stripe's brackets) to LDS; columns < 1 land in the pad
    if (last_lane) {
      Brec<T> b;
      b.z = st.zo;
      b.w = st.wo;
      *wr = b;
    }
  }
  st.zd = zdn;
  st.Mp = M;
  st.Yp = Y;
}

// Sweep `steps` anti-diagonals of one stripe, 4 per iteration, the boundary records of the next
// block prefetched before this block runs. Reads are at columns > t; lane 63 writes column t-62 of
// the row below at step t (bnd has kWave pad records below column 0 for the first 62 steps).
template <typename T, bool kLast>
__device__ __forceinline__ void phmm_stripe(int steps, LaneState<T> &st, const RowParams<T> &P,
                                            T &sumM, T &sumX, Brec<T> *__restrict__ bnd,
                                            const uint8_t *__restrict__ hcol, int C, int lane) {
  // hcol[c] = haplotype code of column c (valid for c in [-63, C+kBndPad)); lane's column at step
  // t is t - lane + 1.
  const uint8_t *hl = hcol + 1 - lane;
  const bool last_lane = lane == kWave - 1;
  constexpr int U = 4;
  int t = 0;
  // The block's record reads and writes go through one VGPR address with immediate offsets (an
  // SGPR base costs a v_mov per access); the asm zero keeps the compiler from rematerialising it.
  int vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  Brec<T> *wb = bnd - (kWave - 2) + vzero;
  for (; t + U <= steps; t += U) {
    // records land directly in the DPP "old" registers (no rotation copies); the LDS latency is
    // covered by the other waves on the SIMD
    Brec<T> *wr = wb + t;
    const Brec<T> c0 = wr[kWave - 1], c1 = wr[kWave], c2 = wr[kWave + 1], c3 = wr[kWave + 2];
    const uint32_t h0 = hl[t], h1 = hl[t + 1], h2 = hl[t + 2], h3 = hl[t + 3];
    phmm_step<T, kLast>(c0, h0, st, P, sumM, sumX, wr, last_lane);
    phmm_step<T, kLast>(c1, h1, st, P, sumM, sumX, wr + 1, last_lane);
    phmm_step<T, kLast>(c2, h2, st, P, sumM, sumX, wr + 2, last_lane);
    phmm_step<T, kLast>(c3, h3, st, P, sumM, sumX, wr + 3, last_lane);
  }
  for (; t < steps; t++)
    phmm_step<T, kLast>(bnd[t + 1], hl[t], st, P, sumM, sumX, bnd + (t - (kWave - 2)), last_lane);
}

template <typename T>
__device__ __forceinline__ void load_row(const uint8_t *__restrict__ rbase, int R, int row,
                                         const DevTab<T> &tab, T &pMM, T &pGAPM, T &pMX, T &pXX,
                                         T &pMY, T &pYY, T &dmatch, T &dmis, uint32_t &rmask) {
  rmask = rbase[row];
  const int q = rbase[R + row] & 127, qi = rbase[2 * R + row] & 127;
  const int qd = rbase[3 * R + row] & 127, qc = rbase[4 * R + row] & 127;
  const int mn = qi <= qd ? qi : qd, mx = qi <= qd ? qd : qi;
  pMM = tab.m2m[((mx * (mx + 1)) >> 1) + mn];
  pGAPM = tab.one_minus[qc];
  pMX = tab.ph2pr[qi];
  pXX = tab.ph2pr[qc];
  pMY = tab.ph2pr[qd];
  pYY = tab.ph2pr[qc];
  dmatch = tab.one_minus[q];
  dmis = tab.div3[q];
}

// One testcase per 64-lane workgroup (f32 pass: blockIdx = testcase; f64 pass over every testcase
// when `f64_list` is null). The f64 fallback pass is persistent instead: a grid sized to the
// resident capacity takes the testcases the f32 pass flagged from `f64_list` through the counter
// f64_count[1], so no workgroup is launched for the ~70 % of testcases that need no fallback.
template <typename T, bool kF64Pass>
__device__ __forceinline__ void phmm_testcase(int w, const TcDesc *__restrict__ descs,
                                              const uint8_t *__restrict__ pool, const DevTab<T> &tab,
                                              T *__restrict__ raw_out, int *__restrict__ f64_list,
                                              int *__restrict__ f64_count, uint8_t *smem_raw);

template <typename T, bool kF64Pass>
__global__ __launch_bounds__(64) void phmm_forward(const TcDesc *__restrict__ descs,
                                                    const uint8_t *__restrict__ pool,
                                                    DevTab<T> tab, T *__restrict__ raw_out,
                                                    int *__restrict__ f64_list,
                                                    int *__restrict__ f64_count) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  if constexpr (kF64Pass) {
    if (f64_list) {
      const int total = __builtin_amdgcn_readfirstlane(__hip_atomic_load(f64_count, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT));
      while (true) {
        int k = 0;
        if (threadIdx.x == 0) k = atomicAdd(f64_count + 1, 1);
        k = __builtin_amdgcn_readfirstlane(__shfl(k, 0));
        if (k >= total) return;
        phmm_testcase<T, true>(f64_list[k], descs, pool, tab, raw_out, nullptr, nullptr, smem_raw);
        __syncthreads();  // the next testcase re-initialises the LDS records
      }
    }
  }
  phmm_testcase<T, kF64Pass>(blockIdx.x, descs, pool, tab, raw_out, f64_list, f64_count, smem_raw);
}

template <typename T, bool kF64Pass>
__device__ __forceinline__ void phmm_testcase(int w, const TcDesc *__restrict__ descs,
                                              const uint8_t *__restrict__ pool, const DevTab<T> &tab,
                                              T *__restrict__ raw_out, int *__restrict__ f64_list,
                                              int *__restrict__ f64_count, uint8_t *smem_raw) {
  const TcDesc desc = descs[w];
  const int R = (int)(desc.dims & 0xffff);
  const int C = (int)(desc.dims >> 16);
  const int lane = threadIdx.x;
  const T init_Y = tab.init_const / (T)C;
  const uint8_t *rbase = pool + desc.read_off;
  // LDS: boundary records for columns [0, C+kBndPad), then haplotype codes for columns
  // [-kWave, C+kBndPad) (codes 0 outside 1..C; cells outside the matrix never feed real cells).
  Brec<T> *bnd = reinterpret_cast<Brec<T> *>(smem_raw) + kWave;  // kWave pad records below column 0
  uint8_t *hcol = smem_raw + sizeof(Brec<T>) * (size_t)(C + kBndPad + kWave) + kWave;

  // Row 0 -> first row's partials: M = X = 0, Y = init_Y, so z = (0*pMM + 0*pGAPM) + init_Y*pGAPM
  // (evaluated, not simplified, to keep the reference's operation order) and w = 0*pMX + 0*pXX.
  T z0, w0;
  {
    T pMM, pGAPM, pMX, pXX, pMY, pYY, dm, dx;
    uint32_t rm;
    load_row(rbase, R, 0, tab, pMM, pGAPM, pMX, pXX, pMY, pYY, dm, dx, rm);
    const T zero = (T)0;
    z0 = (zero * pMM + zero * pGAPM) + init_Y * pGAPM;
    w0 = zero * pMX + zero * pXX;
  }
  const uint8_t *hcode = pool + desc.hap_off;
  for (int c = lane; c < C + kBndPad; c += kWave) {
    Brec<T> b;
    b.z = z0;
    b.w = w0;
    bnd[c] = b;
  }
  for (int c = lane - kWave; c < C + kBndPad; c += kWave) hcol[c] = (c >= 1 && c <= C) ? hcode[c - 1] : 0;
  __syncthreads();

  const int nstripes = (R + kWave - 1) / kWave;
  T result = (T)0;
  for (int s = 0; s < nstripes; s++) {
    const int r0 = s * kWave;
    const int nrows = min(kWave, R - r0);
    RowParams<T> P;
    {
      T pMM, pGAPM, pMX, pXX;
      load_row(rbase, R, min(r0 + lane, R - 1), tab, pMM, pGAPM, pMX, pXX, P.pMY, P.pYY, P.dmatch,
               P.dmis, P.rmask);
      T a, b, d, e;
      uint32_t f;
      load_row(rbase, R, min(r0 + lane + 1, R - 1), tab, P.nMM, P.nGAPM, P.nMX, P.nXX, a, b, d, e, f);
    }
    LaneState<T> st;
    st.Mp = st.Yp = st.zo = st.wo = (T)0;
    st.zd = (lane == 0) ? bnd[0].z : (T)0;  // bracket at column 0: z0 for stripe 0, 0 below
    T sumM = (T)0, sumX = (T)0;
    if (s == nstripes - 1) {
      phmm_stripe<T, true>(C + nrows - 1, st, P, sumM, sumX, bnd, hcol, C, lane);
      result = sumM + sumX;
    } else {
      phmm_stripe<T, false>(C + kWave - 1, st, P, sumM, sumX, bnd, hcol, C, lane);
      if (lane == 0) bnd[0].z = (T)0;  // rows >= 1 have M = X = Y = 0 at column 0
    }
    __syncthreads();
  }
  if (lane == ((R - 1) & (kWave - 1))) {
    raw_out[desc.out_idx] = result;
    if constexpr (!kF64Pass) {
      if (result < 1e-28f) {  // MIN_ACCEPTED, pairhmm_common.h:16
        int slot = atomicAdd(f64_count, 1);
        f64_list[slot] = w;
      }
    }
  }
}

// Device log10 epilogue (IntelPairHmmCSource.cpp:73-79); the host path recomputes it bit-exactly.
__global__ void phmm_finalize(const float *__restrict__ rf, const double *__restrict__ rd,
                              const uint8_t *__restrict__ used, double *__restrict__ out, int n,
                              float log10_init_f, double log10_init_d) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (rf[i] < 1e-28f) ? (log10(rd[i]) - log10_init_d) : (double)(log10f(rf[i]) - log10_init_f);
}

// ---------------------------------------------------------------------------------------------
// Host state
// ---------------------------------------------------------------------------------------------
struct DeviceTables {
  int device = -1;
  float *f = nullptr;   // ph2pr | one_minus | div3 | m2m
  double *d = nullptr;
  HostTables<float> hf;
  HostTables<double> hd;
};

std::mutex g_mu;
HostTables<float> *g_hf = nullptr;
HostTables<double> *g_hd = nullptr;
std::unordered_map<int, DeviceTables *> g_dev;

int ensure_host_tables() {
  if (!g_hf) {
    auto *f = new HostTables<float>();
    auto *d = new HostTables<double>();
    build_tables(*f);
    build_tables(*d);
    g_hf = f;
    g_hd = d;
  }
  return GB_OK;
}

template <typename T>
int upload_tables(const HostTables<T> &h, T **dst) {
  const size_t nel = 3 * kQualTab + kM2M;
  std::vector<T> blob(nel);
  std::memcpy(blob.data(), h.ph2pr, sizeof(T) * kQualTab);
  std::memcpy(blob.data() + kQualTab, h.one_minus, sizeof(T) * kQualTab);
  std::memcpy(blob.data() + 2 * kQualTab, h.div3, sizeof(T) * kQualTab);
  std::memcpy(blob.data() + 3 * kQualTab, h.m2m, sizeof(T) * kM2M);
  GB_HIP(hipMalloc(dst, sizeof(T) * nel));
  GB_HIP(hipMemcpy(*dst, blob.data(), sizeof(T) * nel, hipMemcpyHostToDevice));
  return GB_OK;
}

int get_device_tables(DeviceTables **out) {
  std::lock_guard<std::mutex> lk(g_mu);
  ensure_host_tables();
  int dev = -1;
  GB_HIP(hipGetDevice(&dev));
  auto it = g_dev.find(dev);
  if (it != g_dev.end()) {
    *out = it->second;
    return GB_OK;
  }
  auto *t = new DeviceTables();
  t->device = dev;
  t->hf = *g_hf;
  t->hd = *g_hd;
  int st = upload_tables(*g_hf, &t->f);
  if (st) return st;
  st = upload_tables(*g_hd, &t->d);
  if (st) return st;
  for (auto fn : {(const void *)phmm_forward<float, false>, (const void *)phmm_forward<double, true>})
    GB_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  g_dev[dev] = t;
  *out = t;
  return GB_OK;
}

template <typename T>
DevTab<T> dev_tab(const T *base, T init_const) {
  DevTab<T> t;
  t.ph2pr = base;
  t.one_minus = base + kQualTab;
  t.div3 = base + 2 * kQualTab;
  t.m2m = base + 3 * kQualTab;
  t.init_const = init_const;
  return t;
}

// Deduplication keys: the caller shares read/haplotype buffers across the R x H cross product
// (PairHMMUnitTest.cpp:564-579); identical pointers + length => identical packed record.
struct ReadKey {
  const char *rs, *q, *i, *d, *c;
  int len;
  bool operator==(const ReadKey &o) const {
    return rs == o.rs && q == o.q && i == o.i && d == o.d && c == o.c && len == o.len;
  }
};
struct HapKey {
  const char *h;
  int len;
  bool operator==(const HapKey &o) const { return h == o.h && len == o.len; }
};
struct KeyHash {
  size_t mix(size_t a, size_t b) const { return a ^ (b + 0x9e3779b97f4a7c15ull + (a << 6) + (a >> 2)); }
  size_t operator()(const ReadKey &k) const {
    size_t h = std::hash<const void *>()(k.rs);
    for (const void *p : {(const void *)k.q, (const void *)k.i, (const void *)k.d, (const void *)k.c})
      h = mix(h, std::hash<const void *>()(p));
    return mix(h, (size_t)k.len);
  }
  size_t operator()(const HapKey &k) const { return mix(std::hash<const void *>()(k.h), (size_t)k.len); }
};

}  // namespace

struct gb_phmm_batch {
  DeviceTables *tabs = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  int n = 0;
  int max_haplen = 0;
  int64_t cells = 0;
  TcDesc *d_desc = nullptr;
  uint8_t *d_pool = nullptr;
  float *d_rf = nullptr;
  double *d_rd = nullptr;
  double *d_out = nullptr;
  int *d_list = nullptr;
  int *d_count = nullptr;  // [0] f64 fallbacks flagged by the f32 pass, [1] f64 work counter
  size_t cap_n = 0, cap_pool = 0;  // allocated capacities (a cached workspace batch is refilled)
  int f64_grid = 0;                // persistent f64 grid: resident workgroups of the device
  bool ran = false;
  bool force_f64 = false;
};

extern "C" {

int gb_phmm_init(void) {
  DeviceTables *t = nullptr;
  return get_device_tables(&t);
}

}  // extern "C"

namespace {

// Pack the testcases (deduplicated reads/haplotypes, LPT order) and upload them into b, growing its
// device buffers when they are too small. b's stream/events exist already.
int batch_fill(gb_phmm_batch *b, const gb_testcase *tcs, int n) {
  // Pack: deduplicate reads and haplotypes by pointer (the driver shares them across the R x H
  // cross product, PairHMMUnitTest.cpp:564-579), convert bases to codes once.
  std::vector<uint8_t> pool;
  std::unordered_map<ReadKey, uint32_t, KeyHash> read_at;
  std::unordered_map<HapKey, uint32_t, KeyHash> hap_at;
  std::vector<TcDesc> desc(n);
  std::vector<uint64_t> cost(n);
  int max_h = 0;
  int64_t cells = 0;
  for (int k = 0; k < n; k++) {
    const gb_testcase &t = tcs[k];
    GB_ARG(t.rslen >= 1 && t.rslen <= 65535, "testcase %d: rslen %d outside [1,65535]", k, t.rslen);
    GB_ARG(t.haplen >= 1 && t.haplen <= kMaxHaplen, "testcase %d: haplen %d outside [1,%d]", k,
           t.haplen, kMaxHaplen);
    GB_ARG(t.rs && t.q && t.i && t.d && t.c && t.hap, "testcase %d: null sequence pointer", k);
    const ReadKey rk{t.rs, t.q, t.i, t.d, t.c, t.rslen};
    auto ri = read_at.find(rk);
    uint32_t roff;
    if (ri != read_at.end()) {
      roff = ri->second;
    } else {
      roff = (uint32_t)pool.size();
      pool.resize(pool.size() + 5 * (size_t)t.rslen);
      uint8_t *rec = pool.data() + roff;
      for (int r = 0; r < t.rslen; r++) {
        rec[r] = read_match_mask(base_code(t.rs[r]));
        rec[t.rslen + r] = (uint8_t)t.q[r];
        rec[2 * t.rslen + r] = (uint8_t)t.i[r];
        rec[3 * t.rslen + r] = (uint8_t)t.d[r];
        rec[4 * t.rslen + r] = (uint8_t)t.c[r];
      }
      read_at.emplace(rk, roff);
    }
    const HapKey hk{t.hap, t.haplen};
    auto hi = hap_at.find(hk);
    uint32_t hoff;
    if (hi != hap_at.end()) {
      hoff = hi->second;
    } else {
      hoff = (uint32_t)pool.size();
      pool.resize(pool.size() + (size_t)t.haplen);
      for (int c = 0; c < t.haplen; c++) pool[hoff + c] = base_code(t.hap[c]);
      hap_at.emplace(hk, hoff);
    }
    GB_ARG(pool.size() < (1ull << 32), "batch pool exceeds 4 GiB");
    desc[k].read_off = roff;
    desc[k].hap_off = hoff;
    desc[k].dims = (uint32_t)t.rslen | ((uint32_t)t.haplen << 16);
    desc[k].out_idx = (uint32_t)k;
    cost[k] = (uint64_t)((t.rslen + kWave - 1) / kWave) * (uint64_t)(t.haplen + kWave);
    max_h = std::max(max_h, t.haplen);
    cells += (int64_t)t.rslen * t.haplen;
  }
  // Longest-processing-time-first order (the dispatcher hands out workgroups in grid order).
  std::vector<int> order(n);
  for (int k = 0; k < n; k++) order[k] = k;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
  std::vector<TcDesc> sorted(n);
  for (int k = 0; k < n; k++) sorted[k] = desc[order[k]];
  if (pool.empty()) pool.resize(4);
  pool.resize((pool.size() + 15) & ~size_t(15));

  const size_t nn = std::max(n, 1);
  if (nn > b->cap_n) {
    for (void *p : {(void *)b->d_desc, (void *)b->d_rf, (void *)b->d_rd, (void *)b->d_out, (void *)b->d_list})
      (void)hipFree(p);
    b->d_desc = nullptr;
    b->d_rf = nullptr;
    b->d_rd = b->d_out = nullptr;
    b->d_list = nullptr;
    b->cap_n = 0;
    GB_HIP(hipMalloc(&b->d_desc, sizeof(TcDesc) * nn));
    GB_HIP(hipMalloc(&b->d_rf, sizeof(float) * nn));
    GB_HIP(hipMalloc(&b->d_rd, sizeof(double) * nn));
    GB_HIP(hipMalloc(&b->d_out, sizeof(double) * nn));
    GB_HIP(hipMalloc(&b->d_list, sizeof(int) * nn));
    b->cap_n = nn;
  }
  if (pool.size() > b->cap_pool) {
    (void)hipFree(b->d_pool);
    b->d_pool = nullptr;
    b->cap_pool = 0;
    GB_HIP(hipMalloc(&b->d_pool, pool.size()));
    b->cap_pool = pool.size();
  }
  if (!b->d_count) GB_HIP(hipMalloc(&b->d_count, 2 * sizeof(int)));
  if (n) GB_HIP(hipMemcpyAsync(b->d_desc, sorted.data(), sizeof(TcDesc) * n, hipMemcpyHostToDevice, b->stream));
  GB_HIP(hipMemcpyAsync(b->d_pool, pool.data(), pool.size(), hipMemcpyHostToDevice, b->stream));
  GB_HIP(hipStreamSynchronize(b->stream));  // the host vectors die on return
  b->n = n;
  b->max_haplen = max_h;
  b->cells = cells;
  b->ran = false;
  return GB_OK;
}

int batch_new(DeviceTables *tabs, gb_phmm_batch **out) {
  auto *b = new gb_phmm_batch();
  b->tabs = tabs;
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, tabs->device) == hipSuccess) cus = prop.multiProcessorCount;
  b->f64_grid = cus * 16;
  hipError_t e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
  for (auto &ev : b->ev)
    if (e == hipSuccess) e = hipEventCreate(&ev);
  if (e != hipSuccess) {
    gb::set_error("gb_phmm_batch_create: %s", hipGetErrorString(e));
    gb_phmm_batch_destroy(b);
    return GB_ERR_HIP;
  }
  *out = b;
  return GB_OK;
}

// gb_phmm_compute's workspace: one batch per (host thread, device), refilled on every call so the
// reference's once-per-batch computelikelihoodsboth does not create streams, events and buffers
// each time. Kept for the life of the thread's process (never freed: freeing at thread exit could
// run after the HIP runtime is torn down).
gb_phmm_batch *thread_workspace(DeviceTables *tabs, int *st) {
  thread_local std::unordered_map<int, gb_phmm_batch *> ws;
  auto it = ws.find(tabs->device);
  if (it != ws.end()) return it->second;
  gb_phmm_batch *b = nullptr;
  *st = batch_new(tabs, &b);
  if (*st) return nullptr;
  ws[tabs->device] = b;
  return b;
}

}  // namespace

extern "C" {

int gb_phmm_batch_create(const gb_testcase *tcs, int n, gb_phmm_batch **out) {
  GB_ARG(out, "gb_phmm_batch_create: null out");
  GB_ARG(n >= 0 && (n == 0 || tcs), "gb_phmm_batch_create: bad testcase array (n=%d)", n);
  *out = nullptr;
  DeviceTables *tabs = nullptr;
  int st = get_device_tables(&tabs);
  if (st) return st;
  gb_phmm_batch *b = nullptr;
  if ((st = batch_new(tabs, &b))) return st;
  if ((st = batch_fill(b, tcs, n))) {
    gb_phmm_batch_destroy(b);
    return st;
  }
  *out = b;
  return GB_OK;
}

int gb_phmm_batch_run(gb_phmm_batch *b) {
  gb::Range range_("gb.phmm.batch_run");
  GB_ARG(b, "gb_phmm_batch_run: null batch");
  DeviceTables *t = b->tabs;
  GB_HIP(hipSetDevice(t->device));
  const int n = b->n;
  GB_HIP(hipEventRecord(b->ev[0], b->stream));
  GB_HIP(hipMemsetAsync(b->d_count, 0, 2 * sizeof(int), b->stream));
  GB_HIP(hipMemsetAsync(b->d_rd, 0, sizeof(double) * std::max(n, 1), b->stream));
  if (n > 0) {
    const size_t span = (size_t)(b->max_haplen + kBndPad + kWave);  // records and code bytes
    const size_t lds_f = (sizeof(Brec<float>) + 1) * span + 16;
    const size_t lds_d = (sizeof(Brec<double>) + 1) * span + 16;
    auto f32k = phmm_forward<float, false>;
    auto f64k = phmm_forward<double, true>;
    if (!b->force_f64) {
      hipLaunchKernelGGL(f32k, dim3(n), dim3(kWave), lds_f, b->stream, b->d_desc, b->d_pool,
                         dev_tab<float>(t->f, t->hf.init_const), b->d_rf, b->d_list, b->d_count);
      GB_HIP(hipGetLastError());
    }
    GB_HIP(hipEventRecord(b->ev[1], b->stream));
    // f64 fallback: persistent grid over the flagged list (every testcase when forced)
    const int g64 = b->force_f64 ? n : std::min(n, b->f64_grid);
    hipLaunchKernelGGL(f64k, dim3(g64), dim3(kWave), lds_d, b->stream, b->d_desc, b->d_pool,
                       dev_tab<double>(t->d, t->hd.init_const), b->d_rd,
                       b->force_f64 ? nullptr : b->d_list, b->force_f64 ? nullptr : b->d_count);
    GB_HIP(hipGetLastError());
    GB_HIP(hipEventRecord(b->ev[2], b->stream));
    hipLaunchKernelGGL(phmm_finalize, dim3((n + 255) / 256), dim3(256), 0, b->stream, b->d_rf,
                       b->d_rd, (const uint8_t *)nullptr, b->d_out, n, t->hf.log10_init,
                       t->hd.log10_init);
    GB_HIP(hipGetLastError());
  } else {
    GB_HIP(hipEventRecord(b->ev[1], b->stream));
    GB_HIP(hipEventRecord(b->ev[2], b->stream));
  }
  GB_HIP(hipEventRecord(b->ev[3], b->stream));
  b->ran = true;
  return GB_OK;
}

int gb_phmm_batch_sync(gb_phmm_batch *b) {
  GB_ARG(b, "gb_phmm_batch_sync: null batch");
  GB_HIP(hipStreamSynchronize(b->stream));
  return GB_OK;
}

int gb_phmm_batch_results(gb_phmm_batch *b, double *results, float *raw_f, double *raw_d,
                          uint8_t *used_double, double *dev_results) {
  GB_ARG(b, "gb_phmm_batch_results: null batch");
  if (!b->ran) {
    gb::set_error("gb_phmm_batch_results: batch has not been run");
    return GB_ERR_STATE;
  }
  GB_HIP(hipSetDevice(b->tabs->device));
  GB_HIP(hipStreamSynchronize(b->stream));
  const int n = b->n;
  if (n == 0) return GB_OK;
  std::vector<float> rf(n);
  std::vector<double> rd(n);
  GB_HIP(hipMemcpy(rf.data(), b->d_rf, sizeof(float) * n, hipMemcpyDeviceToHost));
  GB_HIP(hipMemcpy(rd.data(), b->d_rd, sizeof(double) * n, hipMemcpyDeviceToHost));
  if (dev_results) GB_HIP(hipMemcpy(dev_results, b->d_out, sizeof(double) * n, hipMemcpyDeviceToHost));
  const float l10f = b->tabs->hf.log10_init;
  const double l10d = b->tabs->hd.log10_init;
  for (int k = 0; k < n; k++) {
    const bool ud = rf[k] < 1e-28f;
    if (results) results[k] = ud ? (log10(rd[k]) - l10d) : (double)(log10f(rf[k]) - l10f);
    if (raw_f) raw_f[k] = rf[k];
    if (raw_d) raw_d[k] = rd[k];
    if (used_double) used_double[k] = ud ? 1 : 0;
  }
  return GB_OK;
}

int gb_phmm_batch_timing(gb_phmm_batch *b, float *f32_ms, float *f64_ms, float *total_ms) {
  GB_ARG(b && b->ran, "gb_phmm_batch_timing: batch has not been run");
  GB_HIP(hipEventSynchronize(b->ev[3]));
  float a = 0, c = 0, tot = 0;
  GB_HIP(hipEventElapsedTime(&a, b->ev[0], b->ev[1]));
  GB_HIP(hipEventElapsedTime(&c, b->ev[1], b->ev[2]));
  GB_HIP(hipEventElapsedTime(&tot, b->ev[0], b->ev[3]));
  if (f32_ms) *f32_ms = a;
  if (f64_ms) *f64_ms = c;
  if (total_ms) *total_ms = tot;
  return GB_OK;
}

int gb_phmm_batch_stats(gb_phmm_batch *b, int64_t *testcases, int64_t *cells, int64_t *n_f64) {
  GB_ARG(b, "gb_phmm_batch_stats: null batch");
  if (testcases) *testcases = b->n;
  if (cells) *cells = b->cells;
  if (n_f64) {
    int c = 0;
    if (b->ran) {
      GB_HIP(hipStreamSynchronize(b->stream));
      GB_HIP(hipMemcpy(&c, b->d_count, sizeof(int), hipMemcpyDeviceToHost));
    }
    *n_f64 = c;
  }
  return GB_OK;
}

int gb_phmm_batch_destroy(gb_phmm_batch *b) {
  if (!b) return GB_OK;
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  (void)hipFree(b->d_desc);
  (void)hipFree(b->d_pool);
  (void)hipFree(b->d_rf);
  (void)hipFree(b->d_rd);
  (void)hipFree(b->d_out);
  (void)hipFree(b->d_list);
  (void)hipFree(b->d_count);
  for (auto e : b->ev)
    if (e) (void)hipEventDestroy(e);
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
  return GB_OK;
}

int gb_phmm_compute(const gb_testcase *tcs, int n, double *results, float *raw_f, double *raw_d,
                    uint8_t *used_double) {
  gb::Range range_("gb.phmm.compute");
  GB_ARG(n >= 0 && (n == 0 || tcs), "gb_phmm_compute: bad testcase array (n=%d)", n);
  if (n == 0) return GB_OK;
  DeviceTables *tabs = nullptr;
  int st = get_device_tables(&tabs);
  if (st) return st;
  gb_phmm_batch *b = thread_workspace(tabs, &st);
  if (!b) return st;
  b->force_f64 = false;
  if ((st = batch_fill(b, tcs, n))) return st;
  st = gb_phmm_batch_run(b);
  if (!st) st = gb_phmm_batch_results(b, results, raw_f, raw_d, used_double, nullptr);
  return st;
}

int gb_phmm_compute_f64(const gb_testcase *tcs, int n, double *raw_d) {
  GB_ARG(n >= 0 && raw_d && (n == 0 || tcs), "gb_phmm_compute_f64: bad arguments");
  if (n == 0) return GB_OK;
  DeviceTables *tabs = nullptr;
  int st = get_device_tables(&tabs);
  if (st) return st;
  gb_phmm_batch *b = thread_workspace(tabs, &st);
  if (!b) return st;
  if ((st = batch_fill(b, tcs, n))) return st;
  b->force_f64 = true;
  st = gb_phmm_batch_run(b);
  b->force_f64 = false;
  if (!st) st = gb_phmm_batch_results(b, nullptr, nullptr, raw_d, nullptr, nullptr);
  return st;
}

}  // extern "C"
