// fmi_sa.hip -- MI355X (gfx950) SA lookup for the bwa-mem2 FM index: BWT rows -> reference coordinates.
//
// Semantics (tools/bwa-mem2/src, SA_COMPRESSION 1 / SA_COMPX 3, macro.h:64-66):
//   get_sa_entry_compressed  FMI_search.cpp:1714-1807  walk LF (sp = count[b] + Occ(b, sp)) from the row
//                            until a sampled row (sp % 8 == 0), answer = sample + steps; the sentinel
//                            row ('$', no base bit) answers the step count
//   get_sa_entries_prefetch  FMI_search.cpp:1895-2040 over call_one_step :1834-1893 -- the variant the
//                            aligner calls (bwamem.cpp:737); same walk, but reaching the sentinel row
//                            answers 0 whatever the step count (:1865-1869)
//   max_occ sampling         FMI_search.cpp:1906-1924: SMEM {k, s} contributes rows k, k+step, ...
//                            (< k+s, at most max_occ), step = s > max_occ ? s / max_occ : 1
//
// MI355X design: every coordinate is an independent chain of dependent random 64-byte gathers (one
// Occ32 block per LF step, ~8-14 steps) ended by one 8-byte sampled-SA gather -- pure HBM/Infinity-Cache
// latency work with no arithmetic to speak of. The reference keeps 20 walks in flight per CPU thread
// and prefetches; here every lane of every resident wave owns one walk and issues one gather per loop
// trip, so ~500k gathers are in flight. Walk lengths are geometric, so a lane that finishes takes the
// next row at once from a wave-private pool of 256 rows (one device-wide atomic per pool), instead of
// idling until the wave's longest walk ends. The row list itself is expanded on the device from the
// SMEM intervals (count -> scan -> expand), in the reference's coordinate order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/gb.h"
#include "../../include/gb_fmi.h"
#include "fmi_index.h"
#include "gb_common.h"

namespace gbfmi {

constexpr int kSaChunk = 256;  // rows a wave takes from the device-wide counter at a time

struct SaJob {
  int device = -1;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipEvent_t ev[2] = {nullptr, nullptr};
  int64_t nsmem = 0, ncoords = 0;
  int32_t max_occ = 0;
  const gb_smem *d_smems = nullptr;  // borrowed (read set) or d_smems_own
  gb_smem *d_smems_own = nullptr;
  int64_t smem_own_cap = 0;
  int64_t *d_cnt = nullptr;   // per SMEM
  int64_t *d_coff = nullptr;  // nsmem + 1 (coff[0] = 0)
  int64_t cnt_cap = 0;
  int64_t *d_rows = nullptr, *d_coords = nullptr;
  int64_t coord_cap = 0;
  unsigned long long *d_ctl = nullptr;  // [0] next row, [1] LF steps
  void *d_temp = nullptr;
  size_t temp_cap = 0;
  bool ran = false;
};

struct WalkArgs {
  const Occ32 *occ;
  const int64_t *sa;
  int64_t c0, c1, c2, c3;  // count[] after the load-time +1
  int64_t sentinel;
  const int64_t *rows;
  int64_t *out;
  int64_t n;
  unsigned long long *ctl;
  int mode;  // GB_FMI_SA_COMPRESSED / GB_FMI_SA_PREFETCH
};

__device__ __forceinline__ int64_t bcast64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__global__ __launch_bounds__(256) void sa_walk(WalkArgs A) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  int64_t pb = 0, pe = 0;  // this wave's row pool [pb, pe) -- wave-uniform
  bool dry = false;        // device-wide counter exhausted -- wave-uniform
  bool busy = false;
  int64_t t = 0, sp = 0, off = 0;
  uint32_t steps = 0;
  for (;;) {
    const uint64_t need = __ballot(!busy);
    if (need) {
      const int cnt = __popcll(need);
      const int64_t rem = pe - pb;
      int64_t nb = 0, ne = 0;
      bool got = false;
      if (rem < cnt && !dry) {
        unsigned long long v = 0;
        if (lane == 0) v = atomicAdd(A.ctl, (unsigned long long)kSaChunk);
        nb = bcast64((int64_t)v);
        if (nb >= A.n)
          dry = true;
        else {
          got = true;
          ne = min(nb + kSaChunk, A.n);
        }
      }
      if (!busy) {
        const int64_t rank = __popcll(need & below);
        int64_t tt = -1;
        if (rank < rem)
          tt = pb + rank;
        else if (got && nb + (rank - rem) < ne)
          tt = nb + (rank - rem);
        if (tt >= 0) {
          t = tt;
          sp = A.rows[t];
          off = 0;
          busy = true;
        }
      }
      if (rem >= cnt) {
        pb += cnt;
      } else if (got) {
        pb = min(nb + (cnt - rem), ne);
        pe = ne;
      } else {
        pb = pe;
      }
    }
    if (!__ballot(busy)) break;  // nobody busy => pool empty and counter exhausted
    if (busy) {
      if ((sp & 7) == 0) {
        A.out[t] = A.sa[sp >> 3] + off;
        busy = false;
      } else {
        const Occ32 L = A.occ[sp >> 6];
        int b = occ32_code(L, sp);
        if (b == 3 && sp == A.sentinel) b = 4;
        if (b == 4) {
          A.out[t] = A.mode ? 0 : off;
          busy = false;
        } else {
          // Occ(b, sp): rows before sp carrying b (GET_OCC, FMI_search.h:81-89)
          int64_t oA, oC, oG;
          occ32_acg(L, sp, oA, oC, oG);
          const int64_t oT = sp - oA - oC - oG - (A.sentinel < sp ? 1 : 0);
          sp = b == 0 ? A.c0 + oA : b == 1 ? A.c1 + oC : b == 2 ? A.c2 + oG : A.c3 + oT;
          off++;
          steps++;
        }
      }
    }
  }
  for (int o = 32; o; o >>= 1) steps += __shfl_xor(steps, o);
  if (lane == 0 && steps) atomicAdd(A.ctl + 1, (unsigned long long)steps);
}

__global__ void sa_counts(const gb_smem *__restrict__ sm, int64_t n, int32_t max_occ, int64_t *__restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s = sm[i].s;
  cnt[i] = s <= 0 ? 0 : std::min<int64_t>(s, max_occ);  // loop bound of FMI_search.cpp:1918
}

__global__ void sa_expand(const gb_smem *__restrict__ sm, int64_t n, int32_t max_occ, const int64_t *__restrict__ coff,
                          int64_t *__restrict__ rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t k = sm[i].k, s = sm[i].s;
  const int64_t step = s > max_occ ? s / max_occ : 1;
  const int64_t c0 = coff[i], c = coff[i + 1] - c0;
  for (int64_t j = 0; j < c; j++) rows[c0 + j] = k + j * step;
}

inline unsigned grid1(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

void sa_job_destroy(SaJob *J) {
  if (!J) return;
  if (J->stream) (void)hipStreamSynchronize(J->stream);
  for (void *p : {(void *)J->d_smems_own, (void *)J->d_cnt, (void *)J->d_coff, (void *)J->d_rows,
                  (void *)J->d_coords, (void *)J->d_ctl, J->d_temp})
    (void)hipFree(p);
  for (auto e : J->ev)
    if (e) (void)hipEventDestroy(e);
  if (J->own_stream && J->stream) (void)hipStreamDestroy(J->stream);
  delete J;
}

namespace {

int job_create(hipStream_t borrowed, SaJob **out) {
  auto *J = new SaJob();
  GB_HIP(hipGetDevice(&J->device));
  hipError_t e = hipSuccess;
  if (borrowed) {
    J->stream = borrowed;
  } else {
    e = hipStreamCreateWithFlags(&J->stream, hipStreamNonBlocking);
    J->own_stream = true;
  }
  for (auto &ev : J->ev)
    if (e == hipSuccess) e = hipEventCreate(&ev);
  if (e == hipSuccess) e = hipMalloc(&J->d_ctl, 2 * sizeof(unsigned long long));
  if (e != hipSuccess) {
    gb::set_error("SA lookup: %s", hipGetErrorString(e));
    sa_job_destroy(J);
    return GB_ERR_HIP;
  }
  *out = J;
  return GB_OK;
}

template <typename T>
int grow(T *&p, int64_t &cap, int64_t need) {
  if (need <= cap) return GB_OK;
  (void)hipFree(p);
  p = nullptr;
  cap = 0;
  GB_HIP(hipMalloc(&p, sizeof(T) * (size_t)std::max<int64_t>(need, 1)));
  cap = need;
  return GB_OK;
}

int grow_coords(SaJob *J, int64_t need) {
  if (need <= J->coord_cap) return GB_OK;
  (void)hipFree(J->d_rows);
  (void)hipFree(J->d_coords);
  J->d_rows = J->d_coords = nullptr;
  J->coord_cap = 0;
  GB_HIP(hipMalloc(&J->d_rows, sizeof(int64_t) * (size_t)std::max<int64_t>(need, 1)));
  GB_HIP(hipMalloc(&J->d_coords, sizeof(int64_t) * (size_t)std::max<int64_t>(need, 1)));
  J->coord_cap = need;
  return GB_OK;
}

// per-SMEM coordinate counts and their offsets; sizes the row/coord buffers (one host sync)
int prepare(SaJob *J, const gb_smem *d_smems, int64_t nsmem, int32_t max_occ) {
  J->d_smems = d_smems;
  J->nsmem = nsmem;
  J->max_occ = max_occ;
  int64_t cap = J->cnt_cap;
  if (nsmem + 1 > cap) {
    int st = grow(J->d_cnt, J->cnt_cap, nsmem + 1);
    if (st) return st;
    (void)hipFree(J->d_coff);
    J->d_coff = nullptr;
    GB_HIP(hipMalloc(&J->d_coff, sizeof(int64_t) * (size_t)(nsmem + 1)));
  }
  GB_HIP(hipMemsetAsync(J->d_coff, 0, sizeof(int64_t), J->stream));
  J->ncoords = 0;
  if (nsmem > 0) {
    hipLaunchKernelGGL(sa_counts, dim3(grid1(nsmem)), dim3(256), 0, J->stream, d_smems, nsmem, max_occ, J->d_cnt);
    GB_HIP(hipGetLastError());
    size_t tb = 0;
    GB_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, J->d_cnt, J->d_coff + 1, (int)nsmem, J->stream));
    if (tb > J->temp_cap) {
      (void)hipFree(J->d_temp);
      J->d_temp = nullptr;
      GB_HIP(hipMalloc(&J->d_temp, tb));
      J->temp_cap = tb;
    }
    GB_HIP(hipcub::DeviceScan::InclusiveSum(J->d_temp, tb, J->d_cnt, J->d_coff + 1, (int)nsmem, J->stream));
    GB_HIP(hipMemcpyAsync(&J->ncoords, J->d_coff + nsmem, sizeof(int64_t), hipMemcpyDeviceToHost, J->stream));
    GB_HIP(hipStreamSynchronize(J->stream));
  }
  return grow_coords(J, J->ncoords);
}

int launch_walk(SaJob *J, gb_fmi_index *ix, int64_t n, int32_t mode) {
  GB_HIP(hipMemsetAsync(J->d_ctl, 0, 2 * sizeof(unsigned long long), J->stream));
  if (n == 0) return GB_OK;
  WalkArgs A;
  A.occ = ix->d_occ32;
  A.sa = ix->d_sa;
  A.c0 = ix->count[0];
  A.c1 = ix->count[1];
  A.c2 = ix->count[2];
  A.c3 = ix->count[3];
  A.sentinel = ix->sentinel;
  A.rows = J->d_rows;
  A.out = J->d_coords;
  A.n = n;
  A.ctl = J->d_ctl;
  A.mode = mode;
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, J->device) == hipSuccess) cus = prop.multiProcessorCount;
  const char *e = getenv("GB_SA_BLOCKS_PER_CU");
  const int64_t per_cu = e ? std::max(1, atoi(e)) : 4;  // 16 waves per CU: best of 2..16 (tools/sa_probe.py)
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(cus * per_cu, (n + 255) / 256));
  hipLaunchKernelGGL(sa_walk, dim3((unsigned)blocks), dim3(256), 0, J->stream, A);
  GB_HIP(hipGetLastError());
  return GB_OK;
}

int check_index(gb_fmi_index *ix, hipStream_t s) {
  GB_ARG(ix->d_sa && ix->sa_ns == (ix->n >> 3) + 1, "SA lookup: index has no sampled suffix array");
  return ensure_occ32(ix, s);
}

int download(SaJob *J, int64_t *coords, int64_t coords_cap, int32_t *counts, int64_t *total) {
  GB_HIP(hipStreamSynchronize(J->stream));
  if (total) *total = J->ncoords;
  if (coords) {
    GB_ARG(coords_cap >= J->ncoords, "SA lookup: coords_cap %lld < %lld coordinates", (long long)coords_cap,
           (long long)J->ncoords);
    if (J->ncoords)
      GB_HIP(gb::memcpy_big(coords, J->d_coords, sizeof(int64_t) * (size_t)J->ncoords, hipMemcpyDeviceToHost));
  }
  if (counts && J->nsmem) {
    std::vector<int64_t> c((size_t)J->nsmem);
    GB_HIP(hipMemcpy(c.data(), J->d_cnt, sizeof(int64_t) * (size_t)J->nsmem, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < J->nsmem; i++) counts[i] = (int32_t)c[i];
  }
  return GB_OK;
}

}  // namespace
}  // namespace gbfmi

extern "C" {

int gb_fmi_sa_lookup(gb_fmi_index *idx, const int64_t *rows, int64_t n, int32_t mode, int64_t *out) {
  using namespace gbfmi;
  GB_ARG(idx && (n == 0 || (rows && out)) && n >= 0, "gb_fmi_sa_lookup: bad arguments");
  GB_ARG(mode == GB_FMI_SA_COMPRESSED || mode == GB_FMI_SA_PREFETCH, "gb_fmi_sa_lookup: mode %d", mode);
  for (int64_t i = 0; i < n; i++)
    GB_ARG(rows[i] >= 0 && rows[i] < idx->n, "gb_fmi_sa_lookup: row %lld outside [0, %lld)", (long long)rows[i],
           (long long)idx->n);
  GB_HIP(hipSetDevice(idx->device));
  SaJob *J = nullptr;
  int st = job_create(nullptr, &J);
  if (!st) st = check_index(idx, J->stream);
  if (!st) st = grow_coords(J, n);
  if (!st && n) {
    if (hipMemcpy(J->d_rows, rows, sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) {
      gb::set_error("gb_fmi_sa_lookup: upload failed");
      st = GB_ERR_HIP;
    }
  }
  if (!st) st = launch_walk(J, idx, n, mode);
  if (!st) {
    J->ncoords = n;
    st = download(J, out, n, nullptr, nullptr);
  }
  sa_job_destroy(J);
  return st;
}

int gb_fmi_sa_entries(gb_fmi_index *idx, const gb_smem *smems, int64_t n, int32_t max_occ, int32_t mode,
                      int64_t *coords, int64_t coords_cap, int32_t *counts, int64_t *total) {
  using namespace gbfmi;
  GB_ARG(idx && n >= 0 && (n == 0 || smems), "gb_fmi_sa_entries: bad arguments");
  GB_ARG(max_occ > 0, "gb_fmi_sa_entries: max_occ %d", max_occ);
  GB_ARG(mode == GB_FMI_SA_COMPRESSED || mode == GB_FMI_SA_PREFETCH, "gb_fmi_sa_entries: mode %d", mode);
  for (int64_t i = 0; i < n; i++)
    GB_ARG(smems[i].k >= 0 && smems[i].s >= 0 && smems[i].k + smems[i].s <= idx->n,
           "gb_fmi_sa_entries: SMEM %lld interval [%lld, +%lld) outside the index", (long long)i,
           (long long)smems[i].k, (long long)smems[i].s);
  GB_HIP(hipSetDevice(idx->device));
  SaJob *J = nullptr;
  int st = job_create(nullptr, &J);
  if (!st) st = check_index(idx, J->stream);
  if (!st) st = grow(J->d_smems_own, J->smem_own_cap, n);
  if (!st && n && gb::memcpy_big(J->d_smems_own, smems, sizeof(gb_smem) * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) {
    gb::set_error("gb_fmi_sa_entries: upload failed");
    st = GB_ERR_HIP;
  }
  if (!st) st = prepare(J, J->d_smems_own, n, max_occ);
  if (!st && J->ncoords) {
    hipLaunchKernelGGL(sa_expand, dim3(grid1(n)), dim3(256), 0, J->stream, J->d_smems, n, max_occ, J->d_coff,
                       J->d_rows);
    if (hipGetLastError() != hipSuccess) {
      gb::set_error("gb_fmi_sa_entries: expand launch failed");
      st = GB_ERR_HIP;
    }
  }
  if (!st) st = launch_walk(J, idx, J->ncoords, mode);
  if (!st) st = download(J, coords, coords_cap, counts, total);
  sa_job_destroy(J);
  return st;
}

int gb_fmi_reads_sa_run(gb_fmi_reads *r, int32_t max_occ, int32_t mode) {
  gb::Range range_("gb.fmi.sa_run");
  using namespace gbfmi;
  GB_ARG(r, "gb_fmi_reads_sa_run: null read set");
  GB_ARG(max_occ > 0, "gb_fmi_reads_sa_run: max_occ %d", max_occ);
  GB_ARG(mode == GB_FMI_SA_COMPRESSED || mode == GB_FMI_SA_PREFETCH, "gb_fmi_reads_sa_run: mode %d", mode);
  const gb_smem *d_smems = nullptr;
  int64_t nsmem = 0;
  int st = reads_device_smems(r, &d_smems, &nsmem);
  if (st) return st;
  SaJob **slot = reads_sa_job(r);
  if (!*slot && (st = job_create(reads_stream(r), slot))) return st;
  SaJob *J = *slot;
  gb_fmi_index *ix = reads_index(r);
  if ((st = check_index(ix, J->stream))) return st;
  if ((st = prepare(J, d_smems, nsmem, max_occ))) return st;
  GB_HIP(hipEventRecord(J->ev[0], J->stream));
  if (J->ncoords) {
    hipLaunchKernelGGL(sa_expand, dim3(grid1(nsmem)), dim3(256), 0, J->stream, J->d_smems, nsmem, max_occ, J->d_coff,
                       J->d_rows);
    GB_HIP(hipGetLastError());
  }
  if ((st = launch_walk(J, ix, J->ncoords, mode))) return st;
  GB_HIP(hipEventRecord(J->ev[1], J->stream));
  J->ran = true;
  return GB_OK;
}

int gb_fmi_reads_sa_results(gb_fmi_reads *r, int64_t *coords, int64_t coords_cap, int32_t *counts, int64_t *total) {
  using namespace gbfmi;
  GB_ARG(r, "gb_fmi_reads_sa_results: null read set");
  SaJob *J = *reads_sa_job(r);
  GB_ARG(J && J->ran, "gb_fmi_reads_sa_results: gb_fmi_reads_sa_run has not run");
  return download(J, coords, coords_cap, counts, total);
}

int gb_fmi_reads_sa_timing(gb_fmi_reads *r, float *ms, int64_t *lf_steps, int64_t *coords) {
  using namespace gbfmi;
  GB_ARG(r, "gb_fmi_reads_sa_timing: null read set");
  SaJob *J = *reads_sa_job(r);
  GB_ARG(J && J->ran, "gb_fmi_reads_sa_timing: gb_fmi_reads_sa_run has not run");
  GB_HIP(hipEventSynchronize(J->ev[1]));
  float a = 0;
  GB_HIP(hipEventElapsedTime(&a, J->ev[0], J->ev[1]));
  if (ms) *ms = a;
  if (lf_steps) {
    unsigned long long c[2];
    GB_HIP(hipMemcpy(c, J->d_ctl, sizeof(c), hipMemcpyDeviceToHost));
    *lf_steps = (int64_t)c[1];
  }
  if (coords) *coords = J->ncoords;
  return GB_OK;
}

}  // extern "C"
