// fmi_build.hip -- build_index() on the MI355X: suffix array, BWT, CP_OCC, sampled SA, file writer.
//
// Reference (tools/bwa-mem2/src/FMI_search.cpp): pac2nt :109-169 (text = forward + reverse
// complement), build_index :358-434 (counts; SA of the text with SA[0] = |text|), build_fm_index
// :171-356 (BWT with '$' = 4 at the sentinel row, CP_OCC every 64 rows with one-hot bit planes MSB
// first, sampled SA every 8 rows as ms byte + ls word, file layout). The suffix order is that of
// saisxx over the text (end of text sorts first).
//
// MI355X design: prefix doubling on the GPU. Suffixes are first radix-sorted by their first 21
// bases (3-bit symbols, 0 past the end -> a 63-bit key), then only the still-tied groups are
// re-sorted by (rank[i], rank[i+h]) with h doubling, until every group is a singleton. For a
// genome-like text almost everything is resolved by the first sort, so the doubling rounds run on
// small subsets. Sorting uses hipCUB's device radix sort; the rest are streaming kernels.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../include/gb_fmi.h"
#include "gb_common.h"
#include "fmi_index.h"

namespace gbfmi {
namespace {

constexpr int kKmer = 21;
constexpr int kPrefixBits = 24;                        // bucket key: the first 8 symbols of the 21-mer key
constexpr int kPrefixShift = 3 * kKmer - kPrefixBits;  // 63-bit key >> 39
constexpr int kRelBits = 30;                           // doubling key: group ordinal in the chunk << 34 | rank2 + 1
constexpr int64_t kMaxChunk = 1ll << kRelBits;

// Kernels over every text position loop over the grid: an AQL dispatch's grid size is counted in
// 32-bit work-items, so a launch of one thread per position stops at 2^32 positions.
#define GRID_LOOP(i, n)                                                                             \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, _step = (int64_t)gridDim.x * blockDim.x; \
       i < (n); i += _step)

__global__ void make_text(const uint8_t *__restrict__ ref, int64_t G, uint8_t *__restrict__ text) {
  GRID_LOOP(i, G) {
    const uint8_t c = ref[i];
    text[i] = c;
    text[2 * G - 1 - i] = (uint8_t)(3 - c);  // reverse complement appended (pac2nt)
  }
}

__device__ __forceinline__ uint64_t kmer_key(const uint8_t *__restrict__ text, int64_t N, int64_t i) {
  uint64_t k = 0;
#pragma unroll
  for (int j = 0; j < kKmer; j++) {
    const int64_t p = i + j;
    const uint64_t sym = p < N ? (uint64_t)text[p] + 1 : 0;
    k = (k << 3) | sym;
  }
  return k;
}

// suffixes per 8-symbol prefix (the buckets of the first sort are runs of consecutive prefixes)
__global__ void prefix_hist(const uint8_t *__restrict__ text, int64_t N, unsigned long long *__restrict__ hist) {
  GRID_LOOP(i, N) {
    uint32_t p = 0;
#pragma unroll
    for (int j = 0; j < kPrefixBits / 3; j++) {
      const int64_t q = i + j;
      p = (p << 3) | (q < N ? (uint32_t)text[q] + 1 : 0u);
    }
    atomicAdd(&hist[p], 1ull);
  }
}

// the suffixes whose prefix lies in [p0, p1), in arbitrary order (the sort that follows decides it;
// equal 21-mer keys are tied and re-sorted by doubling, so the final order is deterministic)
template <typename I>
__global__ void bucket_keys(const uint8_t *__restrict__ text, int64_t N, uint32_t p0, uint32_t p1,
                            uint64_t *__restrict__ key, I *__restrict__ val, unsigned long long *__restrict__ cnt) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int lane = (int)__lane_id();
  // the loop bound is tested on the wave's first position, so every lane runs every ballot
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); w < N; w += step) {
    const int64_t i = w + lane;
    const uint64_t k = i < N ? kmer_key(text, N, i) : 0;
    const uint32_t p = (uint32_t)(k >> kPrefixShift);
    const bool take = i < N && p >= p0 && p < p1;
    // one atomic per wave: the wave's takers get consecutive slots
    const uint64_t mask = __ballot(take);
    if (!mask) continue;
    const int leader = __ffsll((unsigned long long)mask) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(cnt, (unsigned long long)__popcll(mask));
    base = __shfl(base, leader);
    if (take) {
      const unsigned long long slot = base + (unsigned long long)__popcll(mask & ((1ull << lane) - 1));
      key[slot] = k;
      val[slot] = (I)i;
    }
  }
}

// head of each element's group (scan input): base + t, or pos[t], where the key differs from its predecessor
template <typename I>
__global__ void group_heads(const uint64_t *__restrict__ key, int64_t n, const I *__restrict__ pos, int64_t base,
                            I *__restrict__ head) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const bool h = (t == 0) || key[t] != key[t - 1];
  head[t] = h ? (pos ? pos[t] : (I)(base + t)) : (I)0;
}

// rank[text position] = group head; unresolved flag (chunk-local) for members of groups larger than one
template <typename I>
__global__ void scatter_rank(const uint64_t *__restrict__ key, int64_t n, const I *__restrict__ sa_vals,
                             const I *__restrict__ headscan, I *__restrict__ rank, uint8_t *__restrict__ tied) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  rank[sa_vals[t]] = headscan[t];
  const bool prev_eq = t > 0 && key[t] == key[t - 1];
  const bool next_eq = t + 1 < n && key[t + 1] == key[t];
  tied[t] = (prev_eq || next_eq) ? 1 : 0;
}

template <typename I>
__global__ void copy_vals(const I *__restrict__ src, int64_t n, I *__restrict__ dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) dst[t] = src[t];
}

template <typename I>
__global__ void iota_from(I *__restrict__ p, int64_t n, int64_t base) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) p[t] = (I)(base + t);
}

// 1 where U[t] starts a group (it is its group's head row), for the group ordinals of a chunk
template <typename I>
__global__ void group_start_flags(const I *__restrict__ U, int64_t nu, const I *__restrict__ sa,
                                  const I *__restrict__ rank, I *__restrict__ flag) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nu) return;
  flag[t] = rank[sa[U[t]]] == U[t] ? (I)1 : (I)0;
}

// doubling key of a tied suffix: its group's ordinal in the chunk (inclusive count of group starts,
// < 2^30 since a chunk holds at most 2^30 rows), then the rank h symbols on (0 past the end of the
// text, else rank + 1 < 2^34)
template <typename I>
__global__ void doubling_keys(const I *__restrict__ U, int64_t nu, const I *__restrict__ sa,
                              const I *__restrict__ rank, int64_t N, int64_t h, const I *__restrict__ gord,
                              uint64_t *__restrict__ key2, I *__restrict__ val2) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nu) return;
  const I i = sa[U[t]];
  const uint64_t second = (int64_t)i + h < N ? (uint64_t)rank[(int64_t)i + h] + 1 : 0;
  key2[t] = ((uint64_t)(gord[t] - 1) << 34) | second;
  val2[t] = i;
}

template <typename I>
__global__ void write_back(const I *__restrict__ U, int64_t nu, const I *__restrict__ vals, I *__restrict__ sa) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nu) return;
  sa[U[t]] = vals[t];
}

// the last group start in U(t0, t1]: U[t] starts a group when it is its group's head row
template <typename I>
__global__ void last_group_start(const I *__restrict__ U, int64_t t0, int64_t t1, const I *__restrict__ sa,
                                 const I *__restrict__ rank, unsigned long long *__restrict__ cut) {
  const int64_t t = t0 + 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > t1) return;
  if (rank[sa[U[t]]] == U[t]) atomicMax(cut, (unsigned long long)t);
}

// BWT rows r in [0, n): r = 0 is the '$' suffix (SA[0] = N), row r >= 1 is sa[r-1].
template <typename I>
__device__ __forceinline__ int bwt_sym(const uint8_t *text, const I *sa, int64_t N, int64_t r) {
  if (r == 0) return text[N - 1];
  const int64_t s = (int64_t)sa[r - 1];
  return s == 0 ? 4 : text[s - 1];
}

template <typename I>
__global__ void occ_blocks(const uint8_t *__restrict__ text, const I *__restrict__ sa, int64_t N,
                           int64_t nblocks, CpOcc *__restrict__ occ, int64_t *__restrict__ cnt4) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const int64_t n = N + 1;
  uint64_t bits[4] = {0, 0, 0, 0};
  int64_t c[4] = {0, 0, 0, 0};
  for (int t = 0; t < 64; t++) {
    const int64_t r = b * 64 + t;
    for (int q = 0; q < 4; q++) bits[q] <<= 1;
    if (r < n) {
      const int s = bwt_sym(text, sa, N, r);
      if (s < 4) {
        bits[s] |= 1;
        c[s]++;
      }
    }
  }
  CpOcc o;
  for (int q = 0; q < 4; q++) {
    o.one_hot_bwt_str[q] = bits[q];
    o.cp_count[q] = 0;
    cnt4[q * nblocks + b] = c[q];
  }
  occ[b] = o;
}

__global__ void occ_counts(CpOcc *__restrict__ occ, const int64_t *__restrict__ scan4, int64_t nblocks,
                           int64_t n) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  // a block starting at or past row n is never written by build_fm_index (stays calloc-zero)
  for (int q = 0; q < 4; q++) occ[b].cp_count[q] = (b * 64 < n) ? scan4[q * nblocks + b] : 0;
}

template <typename I>
__global__ void find_sentinel(const I *__restrict__ sa, int64_t N, int64_t *__restrict__ out) {
  GRID_LOOP(j, N) {
    if (sa[j] == 0) *out = j + 1;
  }
}

// sampled SA every 8th row (SA_COMPX = 3): file layout (ms byte, ls word) and the packed search copy
template <typename I>
__global__ void sample_sa(const I *__restrict__ sa, int64_t N, int64_t ns, int8_t *__restrict__ ms,
                          uint32_t *__restrict__ ls, int64_t *__restrict__ sa64) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ns) return;
  const int64_t r = p << 3;
  int64_t v = 0;
  if (r == 0)
    v = N;
  else if (r <= N)
    v = (int64_t)sa[r - 1];
  const int8_t hi = (int8_t)((v >> 32) & 0xff);
  const uint32_t lo = (uint32_t)(v & 0xffffffff);
  if (ms) {
    ls[p] = lo;
    ms[p] = hi;
  }
  sa64[p] = ((int64_t)hi << 32) + (int64_t)lo;
}

inline unsigned grid(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }
// grid of the GRID_LOOP kernels: at most 2^20 blocks of 256 (2^28 work-items)
inline unsigned grid_loop(int64_t n) { return std::min<unsigned>(grid(n), 1u << 20); }

struct DevBuf {
  void *p = nullptr;
  ~DevBuf() { (void)hipFree(p); }
  template <typename T>
  T *as() { return static_cast<T *>(p); }
};

#define GB_HIPX(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) {                                                                   \
      gb::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
      return GB_ERR_HIP;                                                                      \
    }                                                                                         \
  } while (0)

template <typename T>
int dalloc(DevBuf &b, int64_t n) {
  GB_HIPX(hipMalloc(&b.p, sizeof(T) * (size_t)std::max<int64_t>(n, 1)));
  return GB_OK;
}

// rows of one sort (the first sort's buckets, the doubling chunks): GB_FMI_BUILD_CHUNK, default and
// maximum 2^30 (the doubling key's relative-rank field); tests lower it to exercise the chunking
int64_t chunk_cap() {
  const char *e = getenv("GB_FMI_BUILD_CHUNK");
  int64_t c = e && *e ? atoll(e) : kMaxChunk;
  return std::min<int64_t>(std::max<int64_t>(c, 64), kMaxChunk);
}

struct Bucket {
  uint32_t p0, p1;
  int64_t off, size;
};

// Suffix array of the text, then the index. I = uint32_t below 2^31 rows, uint64_t above (or with
// GB_FMI_BUILD_WIDE=1).
template <typename I>
int build_impl(const uint8_t *ref_codes, int64_t G, const char *out_path, gb_fmi_index **out) {
  const int64_t N = 2 * G;
  const int64_t C = std::min<int64_t>(chunk_cap(), N);
  hipStream_t s = 0;
  DevBuf d_ref, d_text, d_sa, d_rank, d_U, d_U2, d_hist, d_cnt, d_key, d_key_alt, d_val, d_val_alt, d_head, d_iota,
      d_tied, d_tmp;
  constexpr int64_t kBins = 1ll << kPrefixBits;
  int st;
  if ((st = dalloc<uint8_t>(d_ref, G)) || (st = dalloc<uint8_t>(d_text, N)) || (st = dalloc<I>(d_sa, N)) ||
      (st = dalloc<I>(d_rank, N)) || (st = dalloc<I>(d_U, N)) || (st = dalloc<unsigned long long>(d_hist, kBins)) ||
      (st = dalloc<unsigned long long>(d_cnt, 2)) || (st = dalloc<uint64_t>(d_key, C)) ||
      (st = dalloc<uint64_t>(d_key_alt, C)) || (st = dalloc<I>(d_val, C)) || (st = dalloc<I>(d_val_alt, C)) ||
      (st = dalloc<I>(d_head, C)) || (st = dalloc<I>(d_iota, C)) || (st = dalloc<uint8_t>(d_tied, C)))
    return st;
  I *const sa = d_sa.as<I>();
  I *const rank = d_rank.as<I>();
  unsigned long long *const cnt = d_cnt.as<unsigned long long>();
  GB_HIPX(gb::memcpy_big(d_ref.p, ref_codes, (size_t)G, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(make_text, dim3(grid_loop(G)), dim3(256), 0, s, d_ref.as<uint8_t>(), G, d_text.as<uint8_t>());
  GB_HIPX(hipMemsetAsync(d_hist.p, 0, sizeof(unsigned long long) * kBins, s));
  hipLaunchKernelGGL(prefix_hist, dim3(grid_loop(N)), dim3(256), 0, s, d_text.as<uint8_t>(), N,
                     d_hist.as<unsigned long long>());
  GB_HIPX(hipGetLastError());
  std::vector<unsigned long long> hist((size_t)kBins);
  GB_HIPX(hipMemcpy(hist.data(), d_hist.p, sizeof(unsigned long long) * kBins, hipMemcpyDeviceToHost));

  // buckets: runs of consecutive prefixes of at most C suffixes, in suffix order
  std::vector<Bucket> buckets;
  {
    Bucket cur{0, 0, 0, 0};
    for (int64_t p = 0; p < kBins; p++) {
      const int64_t c = (int64_t)hist[(size_t)p];
      if (c > C) {
        gb::set_error("gb_fmi_index_build: %lld suffixes share one 8-base prefix (chunk limit %lld)", (long long)c,
                      (long long)C);
        return GB_ERR_ARG;
      }
      if (cur.size + c > C) {
        cur.p1 = (uint32_t)p;
        buckets.push_back(cur);
        cur = Bucket{(uint32_t)p, 0, cur.off + cur.size, 0};
      }
      cur.size += c;
    }
    cur.p1 = (uint32_t)kBins;
    if (cur.size) buckets.push_back(cur);
  }

  // temp storage sized for the largest operation over C elements
  size_t tb_sort = 0, tb_scan = 0, tb_sum = 0, tb_sel = 0;
  {
    hipcub::DoubleBuffer<uint64_t> kb(d_key.as<uint64_t>(), d_key_alt.as<uint64_t>());
    hipcub::DoubleBuffer<I> vb(d_val.as<I>(), d_val_alt.as<I>());
    GB_HIPX(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, kb, vb, (int)C, 0, 64, s));
    GB_HIPX(hipcub::DeviceScan::InclusiveScan(nullptr, tb_scan, d_head.as<I>(), d_head.as<I>(), hipcub::Max(),
                                              (int)C, s));
    GB_HIPX(hipcub::DeviceScan::InclusiveSum(nullptr, tb_sum, d_head.as<I>(), d_head.as<I>(), (int)C, s));
    GB_HIPX(hipcub::DeviceSelect::Flagged(nullptr, tb_sel, d_iota.as<I>(), d_tied.as<uint8_t>(), d_U.as<I>(),
                                          cnt + 1, (int)C, s));
  }
  const size_t tb = std::max({tb_sort, tb_scan, tb_sum, tb_sel, (size_t)16});
  if ((st = dalloc<uint8_t>(d_tmp, (int64_t)tb))) return st;
  size_t tbv = tb;

  // (1) each bucket sorted by the suffixes' first 21 bases into its rows of the SA; ranks = group
  //     heads; tied rows listed in U (in row order)
  int64_t nu = 0;
  for (const Bucket &b : buckets) {
    const int64_t m = b.size;
    GB_HIPX(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(bucket_keys<I>, dim3(grid_loop(N)), dim3(256), 0, s, d_text.as<uint8_t>(), N, b.p0, b.p1,
                       d_key.as<uint64_t>(), d_val.as<I>(), cnt);
    hipcub::DoubleBuffer<uint64_t> kb(d_key.as<uint64_t>(), d_key_alt.as<uint64_t>());
    hipcub::DoubleBuffer<I> vb(d_val.as<I>(), d_val_alt.as<I>());
    tbv = tb;
    GB_HIPX(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, tbv, kb, vb, (int)m, 0, 63, s));
    const uint64_t *ks = kb.Current();
    const I *vs = vb.Current();
    hipLaunchKernelGGL(copy_vals<I>, dim3(grid(m)), dim3(256), 0, s, vs, m, sa + b.off);
    hipLaunchKernelGGL(group_heads<I>, dim3(grid(m)), dim3(256), 0, s, ks, m, (const I *)nullptr, b.off,
                       d_head.as<I>());
    tbv = tb;
    GB_HIPX(hipcub::DeviceScan::InclusiveScan(d_tmp.p, tbv, d_head.as<I>(), d_head.as<I>(), hipcub::Max(), (int)m, s));
    hipLaunchKernelGGL(scatter_rank<I>, dim3(grid(m)), dim3(256), 0, s, ks, m, vs, (const I *)d_head.as<I>(), rank,
                       d_tied.as<uint8_t>());
    hipLaunchKernelGGL(iota_from<I>, dim3(grid(m)), dim3(256), 0, s, d_iota.as<I>(), m, b.off);
    tbv = tb;
    GB_HIPX(hipcub::DeviceSelect::Flagged(d_tmp.p, tbv, d_iota.as<I>(), d_tied.as<uint8_t>(), d_U.as<I>() + nu,
                                          cnt + 1, (int)m, s));
    GB_HIPX(hipGetLastError());
    unsigned long long got[2] = {0, 0};
    GB_HIPX(hipMemcpy(got, cnt, sizeof(got), hipMemcpyDeviceToHost));
    if ((int64_t)got[0] != m) {
      gb::set_error("gb_fmi_index_build: bucket holds %llu suffixes, histogram said %lld", got[0], (long long)m);
      return GB_ERR_HIP;
    }
    nu += (int64_t)got[1];
  }
  if (nu > 0 && (st = dalloc<I>(d_U2, nu))) return st;

  // (2) prefix doubling on the tied rows only, in chunks of whole groups (a chunk's ranks are
  //     refined before the next chunk reads them, which only sharpens its keys: Larsson-Sadakane)
  for (int64_t h = kKmer; nu > 0; h *= 2) {
    GB_ARG(h < 2 * N, "gb_fmi_index_build: doubling did not converge");
    I *U = d_U.as<I>(), *U2 = d_U2.as<I>();
    int64_t nu2 = 0;
    for (int64_t t0 = 0; t0 < nu;) {
      int64_t t1 = std::min(t0 + C, nu);
      if (t1 < nu) {  // end the chunk at the last group start in (t0, t1]
        GB_HIPX(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), s));
        hipLaunchKernelGGL(last_group_start<I>, dim3(grid(t1 - t0)), dim3(256), 0, s, U, t0, t1, (const I *)sa,
                           (const I *)rank, cnt);
        unsigned long long cut = 0;
        GB_HIPX(hipMemcpy(&cut, cnt, sizeof(cut), hipMemcpyDeviceToHost));
        if (cut == 0) {
          gb::set_error("gb_fmi_index_build: a tied group exceeds the chunk limit %lld", (long long)C);
          return GB_ERR_ARG;
        }
        t1 = (int64_t)cut;
      }
      const int64_t m = t1 - t0;
      hipLaunchKernelGGL(group_start_flags<I>, dim3(grid(m)), dim3(256), 0, s, (const I *)(U + t0), m, (const I *)sa,
                         (const I *)rank, d_head.as<I>());
      tbv = tb;
      GB_HIPX(hipcub::DeviceScan::InclusiveSum(d_tmp.p, tbv, d_head.as<I>(), d_head.as<I>(), (int)m, s));
      hipLaunchKernelGGL(doubling_keys<I>, dim3(grid(m)), dim3(256), 0, s, U + t0, m, (const I *)sa, (const I *)rank,
                         N, h, (const I *)d_head.as<I>(), d_key.as<uint64_t>(), d_val.as<I>());
      hipcub::DoubleBuffer<uint64_t> kb(d_key.as<uint64_t>(), d_key_alt.as<uint64_t>());
      hipcub::DoubleBuffer<I> vb(d_val.as<I>(), d_val_alt.as<I>());
      tbv = tb;
      GB_HIPX(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, tbv, kb, vb, (int)m, 0, 64, s));
      const uint64_t *ks = kb.Current();
      const I *vs = vb.Current();
      hipLaunchKernelGGL(write_back<I>, dim3(grid(m)), dim3(256), 0, s, (const I *)(U + t0), m, vs, sa);
      hipLaunchKernelGGL(group_heads<I>, dim3(grid(m)), dim3(256), 0, s, ks, m, (const I *)(U + t0), (int64_t)0,
                         d_head.as<I>());
      tbv = tb;
      GB_HIPX(hipcub::DeviceScan::InclusiveScan(d_tmp.p, tbv, d_head.as<I>(), d_head.as<I>(), hipcub::Max(), (int)m,
                                                s));
      hipLaunchKernelGGL(scatter_rank<I>, dim3(grid(m)), dim3(256), 0, s, ks, m, vs, (const I *)d_head.as<I>(), rank,
                         d_tied.as<uint8_t>());
      tbv = tb;
      GB_HIPX(hipcub::DeviceSelect::Flagged(d_tmp.p, tbv, U + t0, d_tied.as<uint8_t>(), U2 + nu2, cnt + 1, (int)m, s));
      GB_HIPX(hipGetLastError());
      unsigned long long got = 0;
      GB_HIPX(hipMemcpy(&got, cnt + 1, sizeof(got), hipMemcpyDeviceToHost));
      nu2 += (int64_t)got;
      t0 = t1;
    }
    std::swap(d_U.p, d_U2.p);
    nu = nu2;
  }

  // (3) BWT -> CP_OCC (counts = exclusive scan of per-block base counts), sentinel row
  const int64_t n = N + 1;
  const int64_t nblocks = (n >> 6) + 1;
  // every return below (error or not) goes through the guard: an unfinished index is destroyed
  struct IdxGuard {
    gb_fmi_index *p;
    ~IdxGuard() {
      if (p) gb_fmi_index_destroy(p);
    }
  } guard{new gb_fmi_index()};
  gb_fmi_index *const idx = guard.p;
  GB_HIPX(hipGetDevice(&idx->device));
  hipError_t e = hipMalloc(&idx->d_occ, sizeof(CpOcc) * (size_t)nblocks);
  if (e != hipSuccess) {
    gb::set_error("gb_fmi_index_build: %s", hipGetErrorString(e));
    return GB_ERR_HIP;
  }
  // the sort buffers are dead now: free them before the per-block count arrays
  for (DevBuf *b : {&d_U, &d_U2, &d_key, &d_key_alt, &d_val, &d_val_alt, &d_head, &d_iota, &d_rank}) {
    (void)hipFree(b->p);
    b->p = nullptr;
  }
  DevBuf d_cnt4, d_scan;
  if ((st = dalloc<int64_t>(d_cnt4, 4 * nblocks)) || (st = dalloc<int64_t>(d_scan, 4 * nblocks))) {
    return st;
  }
  hipLaunchKernelGGL(occ_blocks<I>, dim3(grid(nblocks)), dim3(256), 0, s, d_text.as<uint8_t>(), (const I *)sa, N,
                     nblocks, idx->d_occ, d_cnt4.as<int64_t>());
  size_t tb64 = 0;
  GB_HIPX(hipcub::DeviceScan::ExclusiveSum(nullptr, tb64, d_cnt4.as<int64_t>(), d_scan.as<int64_t>(), (int)nblocks, s));
  DevBuf d_tmp64;
  if ((st = dalloc<uint8_t>(d_tmp64, (int64_t)tb64 + 16))) {
    return st;
  }
  for (int q = 0; q < 4; q++) {
    size_t t2 = tb64;
    GB_HIPX(hipcub::DeviceScan::ExclusiveSum(d_tmp64.p, t2, d_cnt4.as<int64_t>() + q * nblocks,
                                             d_scan.as<int64_t>() + q * nblocks, (int)nblocks, s));
  }
  hipLaunchKernelGGL(occ_counts, dim3(grid(nblocks)), dim3(256), 0, s, idx->d_occ, d_scan.as<int64_t>(), nblocks, n);
  int64_t *const d_sent = d_scan.as<int64_t>();  // the scans are consumed by occ_counts above (same stream)
  GB_HIPX(hipMemsetAsync(d_sent, 0xff, sizeof(int64_t), s));
  hipLaunchKernelGGL(find_sentinel<I>, dim3(grid_loop(N)), dim3(256), 0, s, (const I *)sa, N, d_sent);
  GB_HIPX(hipGetLastError());
  GB_HIPX(hipDeviceSynchronize());
  int64_t sentinel = -1;
  GB_HIPX(hipMemcpy(&sentinel, d_sent, sizeof(int64_t), hipMemcpyDeviceToHost));
  // base totals from the text (the BWT is a permutation of it plus '$')
  int64_t c4[4] = {0, 0, 0, 0};
  for (int64_t i = 0; i < G; i++) {
    c4[ref_codes[i]]++;
    c4[3 - ref_codes[i]]++;
  }
  int64_t count[5];
  count[0] = 0;
  count[1] = c4[0];
  count[2] = c4[0] + c4[1];
  count[3] = c4[0] + c4[1] + c4[2];
  count[4] = N;
  idx->n = n;
  for (int q = 0; q < 5; q++) idx->count[q] = count[q] + 1;
  idx->sentinel = sentinel;
  idx->cp_size = nblocks;

  // (4) sampled SA kept on the device for SA lookups; optional reference-format file
  //     (build_fm_index, FMI_search.cpp:206-347)
  const int64_t ns = (n >> 3) + 1;
  idx->sa_ns = ns;
  if (hipMalloc(&idx->d_sa, sizeof(int64_t) * (size_t)ns) != hipSuccess) {
    gb::set_error("gb_fmi_index_build: out of device memory (sampled SA)");
    return GB_ERR_HIP;
  }
  if (!out_path) {
    hipLaunchKernelGGL(sample_sa<I>, dim3(grid(ns)), dim3(256), 0, s, (const I *)sa, N, ns, (int8_t *)nullptr,
                       (uint32_t *)nullptr, idx->d_sa);
    GB_HIPX(hipGetLastError());
    GB_HIPX(hipDeviceSynchronize());
  } else {
    DevBuf d_ms, d_ls;
    if ((st = dalloc<int8_t>(d_ms, ns)) || (st = dalloc<uint32_t>(d_ls, ns))) {
      return st;
    }
    hipLaunchKernelGGL(sample_sa<I>, dim3(grid(ns)), dim3(256), 0, s, (const I *)sa, N, ns, d_ms.as<int8_t>(),
                       d_ls.as<uint32_t>(), idx->d_sa);
    std::vector<CpOcc> occ((size_t)nblocks);
    std::vector<int8_t> ms((size_t)ns);
    std::vector<uint32_t> ls((size_t)ns);
    GB_HIPX(gb::memcpy_big(occ.data(), idx->d_occ, sizeof(CpOcc) * (size_t)nblocks, hipMemcpyDeviceToHost));
    GB_HIPX(gb::memcpy_big(ms.data(), d_ms.p, (size_t)ns, hipMemcpyDeviceToHost));
    GB_HIPX(gb::memcpy_big(ls.data(), d_ls.p, 4 * (size_t)ns, hipMemcpyDeviceToHost));
    FILE *fp = fopen(out_path, "wb");
    if (!fp) {
      gb::set_error("gb_fmi_index_build: cannot write %s", out_path);
      return GB_ERR_ARG;
    }
    fwrite(&n, 8, 1, fp);
    fwrite(count, 8, 5, fp);
    fwrite(occ.data(), sizeof(CpOcc), (size_t)nblocks, fp);
    fwrite(ms.data(), 1, (size_t)ns, fp);
    fwrite(ls.data(), 4, (size_t)ns, fp);
    fwrite(&sentinel, 8, 1, fp);
    fclose(fp);
  }
  *out = idx;
  guard.p = nullptr;  // handed to the caller
  return GB_OK;
}

}  // namespace
}  // namespace gbfmi

extern "C" int gb_fmi_index_build(const uint8_t *ref_codes, int64_t ref_len, const char *out_path,
                                  gb_fmi_index **out) {
  using namespace gbfmi;
  GB_ARG(ref_codes && out && ref_len > 0, "gb_fmi_index_build: bad arguments");
  const int64_t N = 2 * ref_len;
  // rank + 1 of the doubling key and the search's Occ32 counts / list entries are 34-bit fields
  GB_ARG(N + 1 < (1ll << 34), "gb_fmi_index_build: text of %lld bases exceeds the 2^34-row limit", (long long)N);
  for (int64_t i = 0; i < ref_len; i++)
    if (ref_codes[i] > 3) {
      gb::set_error("gb_fmi_index_build: code %d at %lld (expected 0..3)", ref_codes[i], (long long)i);
      return GB_ERR_ARG;
    }
  *out = nullptr;
  const char *w = getenv("GB_FMI_BUILD_WIDE");
  const bool wide = (w && *w && atoi(w) != 0) || N >= (1ll << 31) - 1;
  return wide ? build_impl<uint64_t>(ref_codes, ref_len, out_path, out)
              : build_impl<uint32_t>(ref_codes, ref_len, out_path, out);
}
