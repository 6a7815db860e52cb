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

__global__ void make_text(const uint8_t *__restrict__ ref, int64_t G, uint8_t *__restrict__ text) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G) return;
  const uint8_t c = ref[i];
  text[i] = c;
  text[2 * G - 1 - i] = (uint8_t)(3 - c);  // reverse complement appended (pac2nt)
}

__global__ void kmer_keys(const uint8_t *__restrict__ text, int64_t N, uint64_t *__restrict__ key,
                          uint32_t *__restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  uint64_t k = 0;
#pragma unroll
  for (int j = 0; j < kKmer; j++) {
    const int64_t p = i + j;
    const uint64_t sym = p < N ? (uint64_t)text[p] + 1 : 0;
    k = (k << 3) | sym;
  }
  key[i] = k;
  idx[i] = (uint32_t)i;
}

// head index of each element's group (scan input): j if key differs from its predecessor
__global__ void group_heads(const uint64_t *__restrict__ key, int64_t n, const uint32_t *__restrict__ pos,
                            uint32_t *__restrict__ head) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const bool h = (t == 0) || key[t] != key[t - 1];
  head[t] = h ? (pos ? pos[t] : (uint32_t)t) : 0u;
}

// rank[text position] = group head; unresolved flag for members of groups larger than one
__global__ void scatter_rank(const uint64_t *__restrict__ key, int64_t n, const uint32_t *__restrict__ sa_vals,
                             const uint32_t *__restrict__ headscan, uint32_t *__restrict__ rank,
                             uint8_t *__restrict__ tied) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  rank[sa_vals[t]] = headscan[t];
  const bool prev_eq = t > 0 && key[t] == key[t - 1];
  const bool next_eq = t + 1 < n && key[t + 1] == key[t];
  tied[t] = (prev_eq || next_eq) ? 1 : 0;
}

__global__ void doubling_keys(const uint32_t *__restrict__ U, int64_t nu, const uint32_t *__restrict__ sa,
                              const uint32_t *__restrict__ rank, int64_t N, int64_t h,
                              uint64_t *__restrict__ key2, uint32_t *__restrict__ val2) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nu) return;
  const uint32_t i = sa[U[t]];
  const uint64_t second = (int64_t)i + h < N ? (uint64_t)rank[i + h] + 1 : 0;
  key2[t] = ((uint64_t)rank[i] << 32) | second;
  val2[t] = i;
}

__global__ void write_back(const uint32_t *__restrict__ U, int64_t nu, const uint32_t *__restrict__ vals,
                           uint32_t *__restrict__ sa) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nu) return;
  sa[U[t]] = vals[t];
}

__global__ void iota_u32(uint32_t *p, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) p[t] = (uint32_t)t;
}

// BWT rows r in [0, n): r = 0 is the '$' suffix (SA[0] = N), row r >= 1 is sa[r-1].
__device__ __forceinline__ int bwt_sym(const uint8_t *text, const uint32_t *sa, int64_t N, int64_t r) {
  if (r == 0) return text[N - 1];
  const uint32_t s = sa[r - 1];
  return s == 0 ? 4 : text[s - 1];
}

__global__ void occ_blocks(const uint8_t *__restrict__ text, const uint32_t *__restrict__ sa, int64_t N,
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

__global__ void find_sentinel(const uint32_t *__restrict__ sa, int64_t N, int64_t *__restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < N && sa[j] == 0) *out = j + 1;
}

// sampled SA every 8th row (SA_COMPX = 3): file layout (ms byte, ls word) and the packed search copy
__global__ void sample_sa(const uint32_t *__restrict__ sa, int64_t N, int64_t ns, int8_t *__restrict__ ms,
                          uint32_t *__restrict__ ls, int64_t *__restrict__ sa64) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ns) return;
  const int64_t r = p << 3;
  int64_t v = 0;
  if (r == 0)
    v = N;
  else if (r <= N)
    v = sa[r - 1];
  const int8_t hi = (int8_t)((v >> 32) & 0xff);
  const uint32_t lo = (uint32_t)(v & 0xffffffff);
  if (ms) {
    ls[p] = lo;
    ms[p] = hi;
  }
  sa64[p] = ((int64_t)hi << 32) + (int64_t)lo;
}

inline unsigned grid(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

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

}  // namespace
}  // namespace gbfmi

extern "C" int gb_fmi_index_build(const uint8_t *ref_codes, int64_t ref_len, const char *out_path,
                                  gb_fmi_index **out) {
  using namespace gbfmi;
  GB_ARG(ref_codes && out && ref_len > 0, "gb_fmi_index_build: bad arguments");
  const int64_t G = ref_len, N = 2 * ref_len;
  GB_ARG(N < (1ll << 31) - 1, "gb_fmi_index_build: text of %lld bases exceeds the 2^31 limit of the "
         "GPU builder (load a prebuilt .bwt.2bit.64 instead)", (long long)N);
  for (int64_t i = 0; i < G; i++)
    if (ref_codes[i] > 3) {
      gb::set_error("gb_fmi_index_build: code %d at %lld (expected 0..3)", ref_codes[i], (long long)i);
      return GB_ERR_ARG;
    }
  *out = nullptr;
  hipStream_t s = 0;
  DevBuf d_ref, d_text, d_key, d_key_alt, d_val, d_val_alt, d_rank, d_head, d_tied, d_U, d_U2, d_tmp, d_nsel;
  int st;
  if ((st = dalloc<uint8_t>(d_ref, G)) || (st = dalloc<uint8_t>(d_text, N)) ||
      (st = dalloc<uint64_t>(d_key, N)) || (st = dalloc<uint64_t>(d_key_alt, N)) ||
      (st = dalloc<uint32_t>(d_val, N)) || (st = dalloc<uint32_t>(d_val_alt, N)) ||
      (st = dalloc<uint32_t>(d_rank, N)) || (st = dalloc<uint32_t>(d_head, N)) ||
      (st = dalloc<uint8_t>(d_tied, N)) || (st = dalloc<uint32_t>(d_U, N)) ||
      (st = dalloc<uint32_t>(d_U2, N)) || (st = dalloc<int64_t>(d_nsel, 2)))
    return st;
  GB_HIPX(hipMemcpy(d_ref.p, ref_codes, (size_t)G, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(make_text, dim3(grid(G)), dim3(256), 0, s, d_ref.as<uint8_t>(), G, d_text.as<uint8_t>());
  hipLaunchKernelGGL(kmer_keys, dim3(grid(N)), dim3(256), 0, s, d_text.as<uint8_t>(), N,
                     d_key.as<uint64_t>(), d_val.as<uint32_t>());
  GB_HIPX(hipGetLastError());

  // temp storage sized for the largest operation (full sort of N pairs)
  size_t tb_sort = 0, tb_scan = 0, tb_sel = 0;
  {
    hipcub::DoubleBuffer<uint64_t> kb(d_key.as<uint64_t>(), d_key_alt.as<uint64_t>());
    hipcub::DoubleBuffer<uint32_t> vb(d_val.as<uint32_t>(), d_val_alt.as<uint32_t>());
    GB_HIPX(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, kb, vb, (int)N, 0, 63, s));
    GB_HIPX(hipcub::DeviceScan::InclusiveScan(nullptr, tb_scan, d_head.as<uint32_t>(), d_head.as<uint32_t>(),
                                              hipcub::Max(), (int)N, s));
    GB_HIPX(hipcub::DeviceSelect::Flagged(nullptr, tb_sel, d_U.as<uint32_t>(), d_tied.as<uint8_t>(),
                                          d_U2.as<uint32_t>(), d_nsel.as<int64_t>(), (int)N, s));
  }
  const size_t tb = std::max({tb_sort, tb_scan, tb_sel, (size_t)16});
  if ((st = dalloc<uint8_t>(d_tmp, (int64_t)tb))) return st;
  size_t tbv = tb;

  // (1) sort all suffixes by their first 21 bases
  uint32_t *sa = nullptr;
  uint64_t *skey = nullptr;
  {
    hipcub::DoubleBuffer<uint64_t> kb(d_key.as<uint64_t>(), d_key_alt.as<uint64_t>());
    hipcub::DoubleBuffer<uint32_t> vb(d_val.as<uint32_t>(), d_val_alt.as<uint32_t>());
    tbv = tb;
    GB_HIPX(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, tbv, kb, vb, (int)N, 0, 63, s));
    sa = vb.Current();
    skey = kb.Current();
  }
  uint32_t *const sa_alt = (sa == d_val.as<uint32_t>()) ? d_val_alt.as<uint32_t>() : d_val.as<uint32_t>();
  uint64_t *const key_alt = (skey == d_key.as<uint64_t>()) ? d_key_alt.as<uint64_t>() : d_key.as<uint64_t>();
  hipLaunchKernelGGL(group_heads, dim3(grid(N)), dim3(256), 0, s, skey, N, (const uint32_t *)nullptr,
                     d_head.as<uint32_t>());
  tbv = tb;
  GB_HIPX(hipcub::DeviceScan::InclusiveScan(d_tmp.p, tbv, d_head.as<uint32_t>(), d_head.as<uint32_t>(),
                                            hipcub::Max(), (int)N, s));
  hipLaunchKernelGGL(scatter_rank, dim3(grid(N)), dim3(256), 0, s, skey, N, sa, d_head.as<uint32_t>(),
                     d_rank.as<uint32_t>(), d_tied.as<uint8_t>());
  hipLaunchKernelGGL(iota_u32, dim3(grid(N)), dim3(256), 0, s, d_U2.as<uint32_t>(), N);
  tbv = tb;
  GB_HIPX(hipcub::DeviceSelect::Flagged(d_tmp.p, tbv, d_U2.as<uint32_t>(), d_tied.as<uint8_t>(),
                                        d_U.as<uint32_t>(), d_nsel.as<int64_t>(), (int)N, s));
  int64_t nu = 0;
  GB_HIPX(hipMemcpy(&nu, d_nsel.p, sizeof(int64_t), hipMemcpyDeviceToHost));

  // (2) prefix doubling on the tied suffixes only
  int rounds = 0;
  for (int64_t h = kKmer; nu > 0; h *= 2, rounds++) {
    GB_ARG(h < 2 * N, "gb_fmi_index_build: doubling did not converge");
    uint64_t *k2 = skey, *k2b = key_alt;  // reuse the key buffers (the 21-mer keys are dead now)
    uint32_t *v2 = d_head.as<uint32_t>(), *v2b = sa_alt;
    hipLaunchKernelGGL(doubling_keys, dim3(grid(nu)), dim3(256), 0, s, d_U.as<uint32_t>(), nu, sa,
                       d_rank.as<uint32_t>(), N, h, k2, v2);
    hipcub::DoubleBuffer<uint64_t> kb(k2, k2b);
    hipcub::DoubleBuffer<uint32_t> vb(v2, v2b);
    tbv = tb;
    GB_HIPX(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, tbv, kb, vb, (int)nu, 0, 64, s));
    uint64_t *ks = kb.Current();
    uint32_t *vs = vb.Current();
    hipLaunchKernelGGL(write_back, dim3(grid(nu)), dim3(256), 0, s, d_U.as<uint32_t>(), nu, vs, sa);
    uint32_t *hd = (vs == v2) ? v2b : v2;  // free 32-bit buffer of >= nu entries
    hipLaunchKernelGGL(group_heads, dim3(grid(nu)), dim3(256), 0, s, ks, nu, d_U.as<uint32_t>(), hd);
    tbv = tb;
    GB_HIPX(hipcub::DeviceScan::InclusiveScan(d_tmp.p, tbv, hd, hd, hipcub::Max(), (int)nu, s));
    hipLaunchKernelGGL(scatter_rank, dim3(grid(nu)), dim3(256), 0, s, ks, nu, vs, hd,
                       d_rank.as<uint32_t>(), d_tied.as<uint8_t>());
    tbv = tb;
    GB_HIPX(hipcub::DeviceSelect::Flagged(d_tmp.p, tbv, d_U.as<uint32_t>(), d_tied.as<uint8_t>(),
                                          d_U2.as<uint32_t>(), d_nsel.as<int64_t>(), (int)nu, s));
    GB_HIPX(hipMemcpy(&nu, d_nsel.p, sizeof(int64_t), hipMemcpyDeviceToHost));
    std::swap(d_U.p, d_U2.p);
    // keep `skey`/`key_alt` roles stable for the next round
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
  DevBuf d_cnt, d_scan;
  if ((st = dalloc<int64_t>(d_cnt, 4 * nblocks)) || (st = dalloc<int64_t>(d_scan, 4 * nblocks))) {
    return st;
  }
  hipLaunchKernelGGL(occ_blocks, dim3(grid(nblocks)), dim3(256), 0, s, d_text.as<uint8_t>(), sa, N, nblocks,
                     idx->d_occ, d_cnt.as<int64_t>());
  size_t tb64 = 0;
  GB_HIPX(hipcub::DeviceScan::ExclusiveSum(nullptr, tb64, d_cnt.as<int64_t>(), d_scan.as<int64_t>(), (int)nblocks, s));
  DevBuf d_tmp64;
  if ((st = dalloc<uint8_t>(d_tmp64, (int64_t)tb64 + 16))) {
    return st;
  }
  for (int q = 0; q < 4; q++) {
    size_t t2 = tb64;
    GB_HIPX(hipcub::DeviceScan::ExclusiveSum(d_tmp64.p, t2, d_cnt.as<int64_t>() + q * nblocks,
                                             d_scan.as<int64_t>() + q * nblocks, (int)nblocks, s));
  }
  hipLaunchKernelGGL(occ_counts, dim3(grid(nblocks)), dim3(256), 0, s, idx->d_occ, d_scan.as<int64_t>(), nblocks, n);
  GB_HIPX(hipMemset(d_nsel.p, 0xff, sizeof(int64_t)));
  hipLaunchKernelGGL(find_sentinel, dim3(grid(N)), dim3(256), 0, s, sa, N, d_nsel.as<int64_t>());
  GB_HIPX(hipGetLastError());
  GB_HIPX(hipDeviceSynchronize());
  int64_t sentinel = -1;
  GB_HIPX(hipMemcpy(&sentinel, d_nsel.p, sizeof(int64_t), hipMemcpyDeviceToHost));
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
    hipLaunchKernelGGL(sample_sa, dim3(grid(ns)), dim3(256), 0, s, sa, N, ns, (int8_t *)nullptr, (uint32_t *)nullptr,
                       idx->d_sa);
    GB_HIPX(hipGetLastError());
    GB_HIPX(hipDeviceSynchronize());
  } else {
    DevBuf d_ms, d_ls;
    if ((st = dalloc<int8_t>(d_ms, ns)) || (st = dalloc<uint32_t>(d_ls, ns))) {
        return st;
    }
    hipLaunchKernelGGL(sample_sa, dim3(grid(ns)), dim3(256), 0, s, sa, N, ns, d_ms.as<int8_t>(), d_ls.as<uint32_t>(),
                       idx->d_sa);
    std::vector<CpOcc> occ((size_t)nblocks);
    std::vector<int8_t> ms((size_t)ns);
    std::vector<uint32_t> ls((size_t)ns);
    GB_HIPX(hipMemcpy(occ.data(), idx->d_occ, sizeof(CpOcc) * (size_t)nblocks, hipMemcpyDeviceToHost));
    GB_HIPX(hipMemcpy(ms.data(), d_ms.p, (size_t)ns, hipMemcpyDeviceToHost));
    GB_HIPX(hipMemcpy(ls.data(), d_ls.p, 4 * (size_t)ns, hipMemcpyDeviceToHost));
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
