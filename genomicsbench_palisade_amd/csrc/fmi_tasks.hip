// fmi_tasks.hip -- MI355X (gfx950) per-call SMEM kernels behind the FMI_search method adapter
// (include/gb_compat/FMI_search.h, csrc/fmi_dropin.cpp).
//
// The fused search (fmi.hip) runs the whole fmi.cpp batch pipeline for a device-resident read set.
// The reference's class API instead hands over one phase at a time, with caller-chosen inputs:
//   getSMEMsOnePosOneThread          FMI_search.cpp:986-1180   task = (rid, x, min_intv)
//   getSMEMsAllPosOneThread          FMI_search.cpp:1182-1241  task = (rid, min_intv), every x start
//   bwtSeedStrategyAllPosOneThread   FMI_search.cpp:1243-1326  task = (read i, max_intv)
//   getSMEMs                         FMI_search.cpp:1328-1497  task = read i (right-to-left search
//                                    over fixed-stride reads; no caller in the benchmarks)
// and expects the matchArray in the reference's emission order. One task per lane: the lane runs the
// reference loop for its task (backwardExt over the same Occ32 blocks as the fused kernel, `prev` list
// in a private global scratch row) and appends (SMEM, round) records to its slot; the host adapter
// lays the slots out in reference order: OnePos and LAST in task order, AllPos round-major (each
// round visits the still-active reads in rid_array order, FMI_search.cpp:1203-1236), which is a
// stable merge of the per-task lists by round. Tasks whose output overflows the slot are re-run with
// a slot sized to their count (the kernels are deterministic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "../../include/gb.h"
#include "../../include/gb_fmi.h"
#include "fmi_index.h"
#include "fmi_wave.h"
#include "gb_common.h"

namespace gbfmi {
namespace {

enum TaskMode { kOnePos = 0, kAllPos = 1, kLast = 2, kRight = 3 };

struct TSmem {  // gb_smem with the round in the padding word
  uint32_t rid, m, n, round;
  int64_t k, l, s;
};
static_assert(sizeof(TSmem) == sizeof(gb_smem), "TSmem mirrors gb_smem");

struct TEnt {  // one `prev` entry
  int64_t k, l, s;
  uint32_t m, n;
};

struct TaskArgs {
  DevIndex F;
  const uint8_t *qdb;
  const int32_t *lens, *offs;  // per rid
  const int32_t *rid;          // per task
  const int16_t *qpos;         // per task (OnePos)
  const int32_t *intv;         // per task: min_intv (OnePos / AllPos) or max_intv (LAST)
  int32_t ntasks, min_seed_len, cap, maxlen;
  TSmem *out;                  // task t: out[t * cap ...]
  int32_t *counts;             // per task: records emitted (may exceed cap)
  int16_t *next_pos;           // per task (OnePos)
  int32_t *rounds;             // per task (AllPos)
  TEnt *prev;                  // per task: maxlen + 2 entries
  uint32_t *tcalls;            // per task: backwardExt calls (work counter)
  // the records of every task that fits its slot, packed: task t's at compact[toff[t]], in any task
  // order (one atomic per task on *cursor), so the host copies back only what was emitted
  TSmem *compact;
  int32_t *toff;
  unsigned long long *cursor;
};

// a task's records from its slot to the packed array (by the thread that wrote them)
__device__ __forceinline__ void pack_task(const TaskArgs &A, int t, int cnt) {
  const int c = cnt > A.cap ? 0 : cnt;  // an overflowing task is re-run with a bigger slot
  const int32_t off = (int32_t)atomicAdd(A.cursor, (unsigned long long)c);
  A.toff[t] = off;
  for (int k = 0; k < c; k++) A.compact[off + k] = A.out[(size_t)t * A.cap + k];
}

__device__ __forceinline__ void emit(const TaskArgs &A, int t, int &cnt, uint32_t rid, const TEnt &e, uint32_t round) {
  if (cnt < A.cap) {
    TSmem o;
    o.rid = rid;
    o.m = e.m;
    o.n = e.n;
    o.round = round;
    o.k = e.k;
    o.l = e.l;
    o.s = e.s;
    A.out[(size_t)t * A.cap + cnt] = o;
  }
  cnt++;
}

// forward extension = backwardExt on the reverse-complement BWT with k/l swapped (FMI_search.cpp:1044-1056)
__device__ __forceinline__ TEnt fwd_ext(const DevIndex &F, const TEnt &sm, int a, unsigned &calls) {
  TEnt o = sm;
  int64_t ko, lo, so;
  bwt_ext(F, sm.l, sm.k, sm.s, 3 - a, ko, lo, so);
  calls++;
  o.k = lo;
  o.l = ko;
  o.s = so;
  return o;
}

__device__ __forceinline__ TEnt bwd_ext(const DevIndex &F, const TEnt &sm, int a, unsigned &calls) {
  TEnt o = sm;
  bwt_ext(F, sm.k, sm.l, sm.s, a, o.k, o.l, o.s);
  calls++;
  return o;
}

// getSMEMsOnePosOneThread for one (rid, x) (FMI_search.cpp:1004-1178); returns next_x.
__device__ int one_pos(const TaskArgs &A, int t, uint32_t rid, int x, int32_t min_intv, uint32_t round, int &cnt,
                       unsigned &calls) {
  const DevIndex &F = A.F;
  const uint8_t *q = A.qdb + A.offs[rid];
  const int len = A.lens[rid];
  TEnt *prev = A.prev + (size_t)t * (A.maxlen + 2);
  int next_x = x + 1;
  int a = q[x];
  if (a >= 4) return next_x;
  TEnt sm;
  sm.m = sm.n = (uint32_t)x;
  sm.k = count_of(F, a);
  sm.l = count_of(F, 3 - a);
  sm.s = count_of(F, a + 1) - count_of(F, a);
  int numPrev = 0;
  for (int j = x + 1; j < len; j++) {
    a = q[j];
    next_x = j + 1;
    if (a >= 4) break;
    TEnt ns = fwd_ext(F, sm, a, calls);
    ns.n = (uint32_t)j;
    prev[numPrev] = sm;
    numPrev += ns.s != sm.s ? 1 : 0;
    if (ns.s < min_intv) {
      next_x = j;
      break;
    }
    sm = ns;
  }
  if (sm.s >= min_intv) prev[numPrev++] = sm;
  for (int p = 0; p < numPrev / 2; p++) {
    const TEnt tmp = prev[p];
    prev[p] = prev[numPrev - p - 1];
    prev[numPrev - p - 1] = tmp;
  }
  for (int j = x - 1; j >= 0; j--) {
    int numCurr = 0;
    int curr_s = -1;  // int in the reference: assigned from the int64 s (truncating)
    a = q[j];
    if (a > 3) break;
    int p;
    for (p = 0; p < numPrev; p++) {
      const TEnt s0 = prev[p];
      TEnt ns = bwd_ext(F, s0, a, calls);
      ns.m = (uint32_t)j;
      if (ns.s < min_intv && (s0.n - s0.m + 1) >= (uint32_t)A.min_seed_len) {
        emit(A, t, cnt, rid, s0, round);
        break;
      }
      if (ns.s >= min_intv && ns.s != (int64_t)curr_s) {
        curr_s = (int)ns.s;
        prev[numCurr++] = ns;
        break;
      }
    }
    p++;
    for (; p < numPrev; p++) {
      const TEnt s0 = prev[p];
      TEnt ns = bwd_ext(F, s0, a, calls);
      ns.m = (uint32_t)j;
      if (ns.s >= min_intv && ns.s != (int64_t)curr_s) {
        curr_s = (int)ns.s;
        prev[numCurr++] = ns;
      }
    }
    numPrev = numCurr;
    if (numCurr == 0) break;
  }
  if (numPrev != 0 && (prev[0].n - prev[0].m + 1) >= (uint32_t)A.min_seed_len) emit(A, t, cnt, rid, prev[0], round);
  return next_x;
}

// bwtSeedStrategyAllPosOneThread for read i (FMI_search.cpp:1256-1323)
__device__ void last_seeds(const TaskArgs &A, int t, uint32_t i, int32_t max_intv, int &cnt, unsigned &calls) {
  const DevIndex &F = A.F;
  const uint8_t *q = A.qdb + A.offs[i];
  const int len = A.lens[i];
  int x = 0;
  while (x < len) {
    int next_x = x + 1;
    int a = q[x];
    if (a < 4) {
      TEnt sm;
      sm.m = sm.n = (uint32_t)x;
      sm.k = count_of(F, a);
      sm.l = count_of(F, 3 - a);
      sm.s = count_of(F, a + 1) - count_of(F, a);
      for (int j = x + 1; j < len; j++) {
        next_x = j + 1;
        a = q[j];
        if (a >= 4) break;
        TEnt ns = fwd_ext(F, sm, a, calls);
        ns.n = (uint32_t)j;
        sm = ns;
        if (sm.s < max_intv && (sm.n - sm.m + 1) >= (uint32_t)A.min_seed_len) {
          if (sm.s > 0) emit(A, t, cnt, i, sm, 0);
          break;
        }
      }
    }
    x = (int16_t)next_x;
  }
}

// getSMEMs for read i (FMI_search.cpp:1328-1497), with the reference's own behaviour: SMEMs are found
// right to left (forward extension from x, then backward from x - 1); a forward extension stopped by
// an ambiguous base pushes the current SMEM twice (:1394-1401); the aliased prev/curr arrays
// (:1345-1346) are in-place compaction, as here. Emits in the reference's order.
__device__ void right_smems(const TaskArgs &A, int t, uint32_t i, int &cnt, unsigned &calls) {
  const DevIndex &F = A.F;
  const uint8_t *q = A.qdb + A.offs[i];
  const int len = A.lens[i];
  TEnt *prev = A.prev + (size_t)t * (A.maxlen + 2);
  int x = len - 1, numPrev = 0;
  while (x >= 0) {
    int a = q[x];
    if (a > 3) {
      x--;
      continue;
    }
    TEnt sm;
    sm.m = sm.n = (uint32_t)x;
    sm.k = count_of(F, a);
    sm.l = count_of(F, 3 - a);
    sm.s = count_of(F, a + 1) - count_of(F, a);
    for (int j = x + 1; j < len; j++) {
      a = q[j];
      if (a < 4) {
        TEnt ns = fwd_ext(F, sm, a, calls);
        ns.n = (uint32_t)j;
        if (ns.s != sm.s) prev[numPrev++] = sm;
        sm = ns;
        if (ns.s == 0) break;
      } else {
        prev[numPrev++] = sm;
        break;
      }
    }
    if (sm.s != 0) prev[numPrev++] = sm;
    for (int p = 0; p < numPrev / 2; p++) {
      const TEnt tmp = prev[p];
      prev[p] = prev[numPrev - p - 1];
      prev[numPrev - p - 1] = tmp;
    }
    int next_x = x - 1, cur_j = len;
    for (int j = x - 1; j >= 0; j--) {
      int numCurr = 0;
      int curr_s = -1;  // int in the reference
      a = q[j];
      if (a > 3) {
        next_x = j - 1;
        break;
      }
      for (int p = 0; p < numPrev; p++) {
        const TEnt s0 = prev[p];
        TEnt ns = bwd_ext(F, s0, a, calls);
        ns.m = (uint32_t)j;
        if (ns.s == 0 && numCurr == 0 && j < cur_j) {
          cur_j = j;
          if ((s0.n - s0.m + 1) >= (uint32_t)A.min_seed_len) emit(A, t, cnt, i, s0, 0);
        }
        if (ns.s != 0 && ns.s != (int64_t)curr_s) {
          curr_s = (int)ns.s;
          prev[numCurr++] = ns;
        }
      }
      numPrev = numCurr;
      if (numCurr == 0) {
        next_x = j;
        break;
      }
      next_x = j - 1;
    }
    if (numPrev != 0) {
      if ((prev[0].n - prev[0].m + 1) >= (uint32_t)A.min_seed_len) emit(A, t, cnt, i, prev[0], 0);
      numPrev = 0;
    }
    x = next_x;
  }
}

template <int kMode>
__global__ __launch_bounds__(64) void fmi_task_kernel(TaskArgs A) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned calls = 0;
  if (t < A.ntasks) {
    const uint32_t rid = (uint32_t)A.rid[t];
    int cnt = 0;
    if (kMode == kOnePos) {
      A.next_pos[t] = (int16_t)one_pos(A, t, rid, A.qpos[t], A.intv[t], 0, cnt, calls);
    } else if (kMode == kAllPos) {
      const int len = A.lens[rid];
      int x = 0;
      uint32_t round = 0;
      while (x < len) {  // the do-while of FMI_search.cpp:1203-1236 as seen by this read
        x = (int16_t)one_pos(A, t, rid, x, A.intv[t], round, cnt, calls);
        round++;
      }
      A.rounds[t] = (int32_t)round;
    } else if (kMode == kLast) {
      last_seeds(A, t, rid, A.intv[t], cnt, calls);
    } else {
      right_smems(A, t, rid, cnt, calls);
    }
    A.counts[t] = cnt;
    A.tcalls[t] = calls;
    pack_task(A, t, cnt);
  }
}

// The same tasks, one wave per task (fmi_wave.h): a call of a few hundred tasks is latency-bound --
// one lane per task lasts as long as its longest task's chain of dependent gathers, where a wave runs
// each backward step's extensions in parallel. Records and their order per task are those of
// fmi_task_kernel. Reads up to kWaveMaxLen bases (the `prev` lists live in LDS).
constexpr int kWaveMaxLen = 256;

// LDS: the read, then (OnePos / AllPos) two `prev` lists of maxlen + 1 entries, sized per launch
// (wave_lds): 151-base reads take 5 KB instead of the 8.5 KB of 256-base lists, so LDS no longer caps
// the waves per CU below what the registers allow.
__host__ __device__ inline size_t wave_lds(int mode, int maxlen) {
  const size_t q = ((size_t)maxlen + 15) & ~(size_t)15;
  return mode == kLast ? q : q + 2 * sizeof(PEnt) * ((size_t)maxlen + 1);
}

template <int kMode>
__global__ __launch_bounds__(64) void fmi_task_wave(TaskArgs A) {
  extern __shared__ uint8_t lds[];
  uint8_t *Q = lds;
  PEnt *La = reinterpret_cast<PEnt *>(lds + (((size_t)A.maxlen + 15) & ~(size_t)15)), *Lb = La + A.maxlen + 1;
  const int lane = threadIdx.x;
  for (int t = blockIdx.x; t < A.ntasks; t += gridDim.x) {
    const uint32_t rid = (uint32_t)A.rid[t];
    const int L = A.lens[rid];
    const uint8_t *q = A.qdb + A.offs[rid];
    for (int i = lane; i < L; i += 64) Q[i] = q[i];
    __syncthreads();
    int cnt = 0;
    uint32_t calls = 0, round = 0;
    auto emit = [&](int64_t k, int64_t l, int64_t s, uint32_t m, uint32_t n) {
      if (lane == 0 && cnt < A.cap) {
        TSmem o;
        o.rid = rid;
        o.m = m;
        o.n = n;
        o.round = round;
        o.k = k;
        o.l = l;
        o.s = s;
        A.out[(size_t)t * A.cap + cnt] = o;
      }
      cnt++;
    };
    if (kMode == kOnePos) {
      const int nx = wave_one_pos(A.F, Q, L, A.qpos[t], A.intv[t], A.min_seed_len, La, Lb, lane, calls, emit);
      if (lane == 0) A.next_pos[t] = (int16_t)nx;
    } else if (kMode == kAllPos) {
      for (int x = 0; x < L; round++)  // the do-while of FMI_search.cpp:1203-1236 as seen by this read
        x = (int16_t)wave_one_pos(A.F, Q, L, x, A.intv[t], A.min_seed_len, La, Lb, lane, calls, emit);
      if (lane == 0) A.rounds[t] = (int32_t)round;
    } else {
      wave_last_seeds(A.F, Q, L, A.intv[t], A.min_seed_len, calls, emit);
    }
    if (lane == 0) {
      A.counts[t] = cnt;
      A.tcalls[t] = calls;
      pack_task(A, t, cnt);
    }
    __syncthreads();
  }
}

// Per host thread and device: stream, grow-only device buffers and a pinned staging buffer (the
// reference's methods are called from OpenMP threads sharing one FMI_search object).
struct Workspace {
  int device = -1;
  hipStream_t stream = nullptr;
  void *buf[10] = {nullptr};
  size_t cap[10] = {0};
  uint8_t *h = nullptr;  // pinned: uploads are packed here, downloads land here
  size_t hcap = 0;
  ~Workspace() {
    if (device < 0) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    for (void *p : buf) (void)hipFree(p);
    if (h) (void)hipHostFree(h);
    if (stream) (void)hipStreamDestroy(stream);
    (void)hipSetDevice(cur);
  }
  hipError_t ensure(int slot, size_t bytes) {
    bytes = std::max<size_t>(bytes, 64);
    if (cap[slot] >= bytes) return hipSuccess;
    (void)hipFree(buf[slot]);
    buf[slot] = nullptr;
    cap[slot] = 0;
    hipError_t e = hipMalloc(&buf[slot], bytes + bytes / 2);
    if (e == hipSuccess) cap[slot] = bytes + bytes / 2;
    return e;
  }
  hipError_t ensure_host(size_t bytes) {
    bytes = std::max<size_t>(bytes, 1 << 20);
    if (hcap >= bytes) return hipSuccess;
    if (h) (void)hipHostFree(h);
    h = nullptr;
    hcap = 0;
    hipError_t e = hipHostMalloc((void **)&h, bytes + bytes / 2, hipHostMallocDefault);
    if (e == hipSuccess) hcap = bytes + bytes / 2;
    return e;
  }
};

Workspace &workspace(int device) {
  static thread_local std::vector<Workspace *> ws;
  if ((int)ws.size() <= device) ws.resize(device + 1, nullptr);
  if (!ws[device]) {
    ws[device] = new Workspace();
    ws[device]->device = device;
  }
  return *ws[device];
}

struct HostTasks {
  std::vector<int32_t> rid, intv;
  std::vector<int16_t> qpos;
};

inline size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }

// The checks of one call's tasks (the reads they name, their lengths and query positions); the
// extent of enc_qdb they read and their longest read.
int check_tasks(int mode, const int32_t *lens, const int32_t *offs, int32_t nrid, const HostTasks &T,
                int64_t *extent, int32_t *maxlen) {
  const int32_t ntasks = (int32_t)T.rid.size();
  *extent = 0;
  *maxlen = 1;
  for (int32_t t = 0; t < ntasks; t++) {
    const int32_t r = T.rid[t];
    GB_ARG(r >= 0 && r < nrid, "FMI_search: task %d names read %d outside [0, %d)", t, r, nrid);
    GB_ARG(lens[r] >= 0 && (lens[r] < 32768 || mode == kRight) && offs[r] >= 0, "FMI_search: read %d has length %d / offset %d", r,
           lens[r], offs[r]);
    if (mode == kOnePos)
      GB_ARG(T.qpos[t] >= 0 && T.qpos[t] < lens[r], "FMI_search: query position %d outside read %d (length %d)",
             T.qpos[t], r, lens[r]);
    *extent = std::max<int64_t>(*extent, (int64_t)offs[r] + lens[r]);
    *maxlen = std::max(*maxlen, lens[r]);
  }
  return GB_OK;
}

// Runs `mode` over the given tasks; fills per-task record lists (reference emission order within a
// task) and per-task next_pos / rounds, and counts backwardExt calls. Overflowing tasks are re-run
// with a larger slot. Per launch: one upload of the task inputs from pinned staging, the kernel
// (which packs the records of the tasks that fit), one download of the per-task control words and
// the packed count, one download of the packed records.
int run_tasks(gb_fmi_index *idx, int mode, const uint8_t *qdb, const int32_t *lens, const int32_t *offs, int32_t nrid,
              const HostTasks &T, int32_t min_seed_len, std::vector<std::vector<TSmem>> &recs,
              std::vector<int16_t> *next_pos, std::vector<int32_t> *rounds, int64_t *calls_out) {
  gb::Range range_(mode == kOnePos ? "gb.fmi.onepos"
                   : mode == kAllPos ? "gb.fmi.allpos"
                   : mode == kLast   ? "gb.fmi.last"
                                     : "gb.fmi.get_smems");
  const int32_t ntasks = (int32_t)T.rid.size();
  recs.assign(ntasks, {});
  if (next_pos) next_pos->assign(ntasks, 0);
  if (rounds) rounds->assign(ntasks, 0);
  if (calls_out) *calls_out = 0;
  if (ntasks == 0) return GB_OK;
  int64_t extent = 0;
  int32_t maxlen = 1;
  if (int st = check_tasks(mode, lens, offs, nrid, T, &extent, &maxlen)) return st;
  GB_HIP(hipSetDevice(idx->device));
  Workspace &W = workspace(idx->device);
  if (!W.stream) GB_HIP(hipStreamCreateWithFlags(&W.stream, hipStreamNonBlocking));
  if (int st = ensure_occ32(idx, W.stream)) return st;
  hipStream_t s = W.stream;

  TaskArgs A;
  A.F.occ = idx->d_occ32;
  for (int b = 0; b < 5; b++) A.F.count[b] = idx->count[b];
  A.F.sentinel = idx->sentinel;
  A.min_seed_len = min_seed_len;
  A.maxlen = maxlen;

  // the reads, once per call: [qdb extent | lens | offs]
  {
    const size_t o_lens = up256((size_t)extent), o_offs = o_lens + up256(4 * (size_t)nrid),
                 bytes = o_offs + 4 * (size_t)nrid;
    GB_HIP(W.ensure(0, bytes));
    GB_HIP(W.ensure_host(bytes));
    std::memcpy(W.h, qdb, (size_t)extent);
    std::memcpy(W.h + o_lens, lens, 4 * (size_t)nrid);
    std::memcpy(W.h + o_offs, offs, 4 * (size_t)nrid);
    GB_HIP(hipMemcpyAsync(W.buf[0], W.h, bytes, hipMemcpyHostToDevice, s));
    A.qdb = (const uint8_t *)W.buf[0];
    A.lens = (const int32_t *)((uint8_t *)W.buf[0] + o_lens);
    A.offs = (const int32_t *)((uint8_t *)W.buf[0] + o_offs);
    GB_HIP(hipStreamSynchronize(s));  // W.h is reused below
  }

  // Tiles of at most ~256 MB of `prev` scratch ((maxlen + 1) entries per task): the per-thread
  // workspace stays bounded whatever the batch. Per tile: the whole tile, then its overflowing
  // subset with a slot sized to its largest count.
  // (getSMEMs takes reads of any length: for ~Mb reads the tile falls below a wave's 64 tasks rather
  // than the scratch growing past the bound)
  int64_t tile = std::max<int64_t>(1, (256ll << 20) / ((int64_t)(maxlen + 2) * (int64_t)sizeof(TEnt)));
  if (tile >= 64) tile &= ~63ll;
  if (const char *te = getenv("GB_FMI_TASK_TILE")) tile = std::max(1, atoi(te));  // tests: force many tiles
  int64_t calls_sum = 0;
  for (int32_t t0 = 0; t0 < ntasks; t0 = (int32_t)std::min<int64_t>(ntasks, t0 + tile)) {
  const int32_t t1 = (int32_t)std::min<int64_t>(ntasks, t0 + tile);
  std::vector<int32_t> todo(t1 - t0);
  for (int32_t t = t0; t < t1; t++) todo[t - t0] = t;
  int32_t cap = mode == kLast ? 48 : mode == kRight ? 64 : 32;
  for (int pass = 0; pass < 2 && !todo.empty(); pass++) {
    const int32_t n = (int32_t)todo.size();
    // task inputs (uploaded): [cursor 8 B | rid n | intv n | qpos n]
    const size_t i_rid = 256, i_intv = i_rid + up256(4 * (size_t)n), i_qpos = i_intv + up256(4 * (size_t)n),
                 in_bytes = i_qpos + 2 * (size_t)n;
    // control words (downloaded): [counts n | rounds n | tcalls n | toff n | next_pos n]
    const size_t c_rounds = up256(4 * (size_t)n), c_tcalls = c_rounds + up256(4 * (size_t)n),
                 c_toff = c_tcalls + up256(4 * (size_t)n), c_np = c_toff + up256(4 * (size_t)n),
                 ctl_bytes = c_np + 2 * (size_t)n;
    const size_t rec_bytes = sizeof(TSmem) * (size_t)n * cap;
    hipError_t e = W.ensure(3, in_bytes);
    if (e == hipSuccess) e = W.ensure(6, rec_bytes);
    if (e == hipSuccess) e = W.ensure(7, ctl_bytes);
    if (e == hipSuccess) e = W.ensure(8, sizeof(TEnt) * (size_t)n * (maxlen + 2));
    if (e == hipSuccess) e = W.ensure(9, rec_bytes);
    if (e == hipSuccess) e = W.ensure_host(std::max(std::max(in_bytes, up256(ctl_bytes) + 256), rec_bytes));
    GB_HIP(e);
    uint8_t *h = W.h;
    std::memset(h, 0, 8);
    auto *hrid = reinterpret_cast<int32_t *>(h + i_rid);
    auto *hintv = reinterpret_cast<int32_t *>(h + i_intv);
    auto *hqpos = reinterpret_cast<int16_t *>(h + i_qpos);
    for (int32_t i = 0; i < n; i++) {
      hrid[i] = T.rid[todo[i]];
      hintv[i] = T.intv[todo[i]];
      hqpos[i] = mode == kOnePos ? T.qpos[todo[i]] : 0;
    }
    uint8_t *din = (uint8_t *)W.buf[3], *dctl = (uint8_t *)W.buf[7];
    GB_HIP(hipMemcpyAsync(din, h, in_bytes, hipMemcpyHostToDevice, s));
    A.cursor = (unsigned long long *)din;
    A.rid = (const int32_t *)(din + i_rid);
    A.intv = (const int32_t *)(din + i_intv);
    A.qpos = (const int16_t *)(din + i_qpos);
    A.out = (TSmem *)W.buf[6];
    A.compact = (TSmem *)W.buf[9];
    A.counts = (int32_t *)dctl;
    A.rounds = (int32_t *)(dctl + c_rounds);
    A.tcalls = (uint32_t *)(dctl + c_tcalls);
    A.toff = (int32_t *)(dctl + c_toff);
    A.next_pos = (int16_t *)(dctl + c_np);
    A.prev = (TEnt *)W.buf[8];
    A.ntasks = n;
    A.cap = cap;
    // a wave per task when the reads fit its LDS lists (GB_FMI_TASK_WAVE=0: a lane per task)
    const char *we = getenv("GB_FMI_TASK_WAVE");
    if (mode != kRight && maxlen <= kWaveMaxLen && !(we && *we == '0')) {
      const dim3 grid((unsigned)std::min<int64_t>(n, 65535)), block(64);
      const size_t lds = wave_lds(mode, maxlen);
      if (mode == kOnePos)
        hipLaunchKernelGGL(fmi_task_wave<kOnePos>, grid, block, lds, s, A);
      else if (mode == kAllPos)
        hipLaunchKernelGGL(fmi_task_wave<kAllPos>, grid, block, lds, s, A);
      else
        hipLaunchKernelGGL(fmi_task_wave<kLast>, grid, block, lds, s, A);
    } else {
      const dim3 grid((unsigned)((n + 63) / 64)), block(64);
      if (mode == kOnePos)
        hipLaunchKernelGGL(fmi_task_kernel<kOnePos>, grid, block, 0, s, A);
      else if (mode == kAllPos)
        hipLaunchKernelGGL(fmi_task_kernel<kAllPos>, grid, block, 0, s, A);
      else if (mode == kLast)
        hipLaunchKernelGGL(fmi_task_kernel<kLast>, grid, block, 0, s, A);
      else
        hipLaunchKernelGGL(fmi_task_kernel<kRight>, grid, block, 0, s, A);
    }
    GB_HIP(hipGetLastError());
    // the control words and the packed count (the input block's first word) in one download each
    GB_HIP(hipMemcpyAsync(h, dctl, ctl_bytes, hipMemcpyDeviceToHost, s));
    unsigned long long packed = 0;
    GB_HIP(hipMemcpyAsync(h + up256(ctl_bytes), din, 8, hipMemcpyDeviceToHost, s));
    GB_HIP(hipStreamSynchronize(s));
    std::memcpy(&packed, h + up256(ctl_bytes), 8);
    GB_ARG(packed <= (unsigned long long)n * cap, "FMI_search: %llu packed records exceed the %lld slots", packed,
           (long long)n * cap);
    const int32_t *hc = reinterpret_cast<const int32_t *>(h);
    const std::vector<int32_t> cnt(hc, hc + n), rnd(reinterpret_cast<const int32_t *>(h + c_rounds),
                                                    reinterpret_cast<const int32_t *>(h + c_rounds) + n),
        toff(reinterpret_cast<const int32_t *>(h + c_toff), reinterpret_cast<const int32_t *>(h + c_toff) + n);
    const std::vector<uint32_t> tc(reinterpret_cast<const uint32_t *>(h + c_tcalls),
                                   reinterpret_cast<const uint32_t *>(h + c_tcalls) + n);
    const std::vector<int16_t> np(reinterpret_cast<const int16_t *>(h + c_np),
                                  reinterpret_cast<const int16_t *>(h + c_np) + n);
    if (packed) {
      GB_HIP(hipMemcpyAsync(h, A.compact, sizeof(TSmem) * (size_t)packed, hipMemcpyDeviceToHost, s));
      GB_HIP(hipStreamSynchronize(s));
    }
    const TSmem *rec = reinterpret_cast<const TSmem *>(h);
    std::vector<int32_t> again;
    int32_t need = 0;
    for (int32_t i = 0; i < n; i++) {
      const int32_t t = todo[i], c = cnt[i];
      if (pass == 0) calls_sum += tc[i];
      if (c > cap) {
        again.push_back(t);
        need = std::max(need, c);
        continue;
      }
      recs[t].assign(rec + toff[i], rec + toff[i] + c);
      if (next_pos) (*next_pos)[t] = np[i];
      if (rounds) (*rounds)[t] = rnd[i];
    }
    todo.swap(again);
    cap = need;
  }
  GB_ARG(todo.empty(), "FMI_search: SMEM output of %zu tasks could not be sized", todo.size());
  }
  if (calls_out) *calls_out = calls_sum;
  return GB_OK;
}

// raw sampled-SA entries (get_sa_entry / get_sa_entries, FMI_search.cpp:1566-1619: sa_ms_byte << 32
// + sa_ls_word at the given index of the sampled arrays)
__global__ void sa_raw_kernel(const int64_t *__restrict__ sa, const int64_t *__restrict__ pos, int64_t n,
                              int64_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = sa[pos[i]];
}

// call_one_step (FMI_search.cpp:1834-1893) on the reference CP_OCC lines
__global__ void sa_one_step_kernel(const CpOcc *__restrict__ occ, const int64_t *__restrict__ sa, DevIndex F,
                                   int64_t pos, int64_t offset, int64_t *out3) {
  int64_t ret, entry;
  if ((pos & 7) == 0) {
    entry = sa[pos >> 3];
    ret = 1;
  } else {
    const CpOcc &L = occ[pos >> 6];
    const int y = 63 - (int)(pos & 63);
    int b = 4;
    for (int c = 3; c >= 0; c--)
      if ((L.one_hot_bwt_str[c] >> y) & 1) b = c;
    if (b == 4) {
      entry = 0;
      ret = 1;
    } else {
      const uint64_t mask = (pos & 63) ? ~0ull << (64 - (pos & 63)) : 0ull;
      const int64_t sp = count_of(F, b) + L.cp_count[b] + __popcll(L.one_hot_bwt_str[b] & mask);
      offset++;
      if ((sp & 7) == 0) {
        entry = sa[sp >> 3] + offset;
        ret = 1;
      } else {
        entry = sp;
        ret = 0;
      }
    }
  }
  out3[0] = ret;
  out3[1] = entry;
  out3[2] = offset;
}

void put(gb_smem *dst, const TSmem &r) {
  gb_smem o;
  std::memset(&o, 0, sizeof(o));
  o.rid = r.rid;
  o.m = r.m;
  o.n = r.n;
  o.k = r.k;
  o.l = r.l;
  o.s = r.s;
  *dst = o;
}

}  // namespace
}  // namespace gbfmi

using namespace gbfmi;

extern "C" {

int gb_fmi_smem_onepos(gb_fmi_index *idx, const uint8_t *enc_qdb, const int32_t *lens, const int32_t *offs,
                       int32_t nrid, const int16_t *query_pos, const int32_t *min_intv, const int32_t *rid,
                       int32_t ntasks, int32_t min_seed_len, gb_smem *out, int64_t out_cap, int64_t *nout,
                       int16_t *next_pos, int64_t *bwt_calls) {
  GB_ARG(idx && nout && ntasks >= 0 && nrid >= 0, "gb_fmi_smem_onepos: bad arguments");
  GB_ARG(ntasks == 0 || (enc_qdb && lens && offs && query_pos && min_intv && rid), "gb_fmi_smem_onepos: null array");
  HostTasks T;
  T.rid.assign(rid, rid + ntasks);
  T.intv.assign(min_intv, min_intv + ntasks);
  T.qpos.assign(query_pos, query_pos + ntasks);
  std::vector<std::vector<TSmem>> recs;
  std::vector<int16_t> np;
  int st = run_tasks(idx, kOnePos, enc_qdb, lens, offs, nrid, T, min_seed_len, recs, &np, nullptr, bwt_calls);
  if (st) return st;
  int64_t tot = 0;
  for (auto &v : recs) tot += (int64_t)v.size();
  *nout = tot;
  if (next_pos) std::copy(np.begin(), np.end(), next_pos);
  if (!out) return GB_OK;
  GB_ARG(tot <= out_cap, "gb_fmi_smem_onepos: %lld SMEMs exceed out_cap %lld", (long long)tot, (long long)out_cap);
  int64_t o = 0;
  for (auto &v : recs)
    for (auto &r : v) put(out + o++, r);
  return GB_OK;
}

int gb_fmi_smem_allpos(gb_fmi_index *idx, const uint8_t *enc_qdb, const int32_t *lens, const int32_t *offs,
                       int32_t nrid, const int32_t *min_intv, const int32_t *rid, int32_t ntasks,
                       int32_t min_seed_len, gb_smem *out, int64_t out_cap, int64_t *nout, int32_t *rounds,
                       int64_t *bwt_calls) {
  GB_ARG(idx && nout && ntasks >= 0 && nrid >= 0, "gb_fmi_smem_allpos: bad arguments");
  GB_ARG(ntasks == 0 || (enc_qdb && lens && offs && min_intv && rid), "gb_fmi_smem_allpos: null array");
  HostTasks T;
  T.rid.assign(rid, rid + ntasks);
  T.intv.assign(min_intv, min_intv + ntasks);
  std::vector<std::vector<TSmem>> recs;
  std::vector<int32_t> rn;
  int st = run_tasks(idx, kAllPos, enc_qdb, lens, offs, nrid, T, min_seed_len, recs, nullptr, &rn, bwt_calls);
  if (st) return st;
  int64_t tot = 0;
  int32_t max_round = 0;
  for (int32_t t = 0; t < ntasks; t++) {
    tot += (int64_t)recs[t].size();
    max_round = std::max(max_round, rn[t]);
  }
  *nout = tot;
  if (rounds) std::copy(rn.begin(), rn.end(), rounds);
  if (!out) return GB_OK;
  GB_ARG(tot <= out_cap, "gb_fmi_smem_allpos: %lld SMEMs exceed out_cap %lld", (long long)tot, (long long)out_cap);
  // round-major, tasks in order within a round: a merge of the per-task lists (rounds ascending)
  std::vector<size_t> cur(ntasks, 0);
  std::vector<int32_t> live;
  for (int32_t t = 0; t < ntasks; t++)
    if (!recs[t].empty()) live.push_back(t);
  int64_t o = 0;
  for (uint32_t r = 0; r < (uint32_t)max_round && !live.empty(); r++) {
    size_t w = 0;
    for (int32_t t : live) {
      auto &v = recs[t];
      size_t &c = cur[t];
      while (c < v.size() && v[c].round == r) put(out + o++, v[c++]);
      if (c < v.size()) live[w++] = t;
    }
    live.resize(w);
  }
  return o == tot ? GB_OK : (gb::set_error("gb_fmi_smem_allpos: round merge lost records"), GB_ERR_STATE);
}

int gb_fmi_last_seeds(gb_fmi_index *idx, const uint8_t *enc_qdb, const int32_t *lens, const int32_t *offs,
                      int32_t nreads, const int32_t *max_intv, int32_t min_seed_len, gb_smem *out, int64_t out_cap,
                      int64_t *nout, int64_t *bwt_calls) {
  GB_ARG(idx && nout && nreads >= 0, "gb_fmi_last_seeds: bad arguments");
  GB_ARG(nreads == 0 || (enc_qdb && lens && offs && max_intv), "gb_fmi_last_seeds: null array");
  HostTasks T;
  T.rid.resize(nreads);
  for (int32_t i = 0; i < nreads; i++) T.rid[i] = i;
  T.intv.assign(max_intv, max_intv + nreads);
  std::vector<std::vector<TSmem>> recs;
  int st = run_tasks(idx, kLast, enc_qdb, lens, offs, nreads, T, min_seed_len, recs, nullptr, nullptr, bwt_calls);
  if (st) return st;
  int64_t tot = 0;
  for (auto &v : recs) tot += (int64_t)v.size();
  *nout = tot;
  if (!out) return GB_OK;
  GB_ARG(tot <= out_cap, "gb_fmi_last_seeds: %lld SMEMs exceed out_cap %lld", (long long)tot, (long long)out_cap);
  int64_t o = 0;
  for (auto &v : recs)
    for (auto &r : v) put(out + o++, r);
  return GB_OK;
}

int gb_fmi_get_smems(gb_fmi_index *idx, const uint8_t *enc_qdb, int32_t num_reads, int32_t readlength,
                     int32_t min_seed_len, int32_t nthreads, gb_smem *out, int64_t out_cap, int64_t *nout,
                     int64_t *bwt_calls) {
  GB_ARG(idx && nout && num_reads >= 0 && readlength >= 0 && nthreads >= 1, "gb_fmi_get_smems: bad arguments");
  GB_ARG(num_reads == 0 || readlength == 0 || enc_qdb, "gb_fmi_get_smems: null enc_qdb");
  // the reference's omp region is commented out (tid 0): only the first thread's quota of reads
  const int32_t last = std::min<int64_t>(num_reads, ((int64_t)num_reads + nthreads - 1) / nthreads);
  *nout = 0;
  if (bwt_calls) *bwt_calls = 0;
  if (last == 0 || readlength == 0) return GB_OK;
  GB_ARG((int64_t)last * readlength < INT32_MAX, "gb_fmi_get_smems: %d reads x %d bases exceed 2^31", last, readlength);
  HostTasks T;
  T.rid.resize(last);
  T.intv.assign(last, 0);
  std::vector<int32_t> lens(last, readlength), offs(last);
  for (int32_t i = 0; i < last; i++) {
    T.rid[i] = i;
    offs[i] = (int32_t)((int64_t)i * readlength);
  }
  std::vector<std::vector<TSmem>> recs;
  int st = run_tasks(idx, kRight, enc_qdb, lens.data(), offs.data(), last, T, min_seed_len, recs, nullptr, nullptr,
                     bwt_calls);
  if (st) return st;
  int64_t tot = 0;
  for (auto &v : recs) tot += (int64_t)v.size();
  *nout = tot;
  if (!out) return GB_OK;
  GB_ARG(tot <= out_cap, "gb_fmi_get_smems: %lld SMEMs exceed out_cap %lld", (long long)tot, (long long)out_cap);
  int64_t o = 0;
  for (auto &v : recs)
    for (auto &r : v) put(out + o++, r);
  return GB_OK;
}

int gb_fmi_sa_raw(gb_fmi_index *idx, const int64_t *pos, int64_t n, int64_t *out) {
  GB_ARG(idx && n >= 0 && (n == 0 || (pos && out)), "gb_fmi_sa_raw: bad arguments");
  for (int64_t i = 0; i < n; i++)
    GB_ARG(pos[i] >= 0 && pos[i] < idx->sa_ns, "gb_fmi_sa_raw: index %lld outside the %lld sampled entries",
           (long long)pos[i], (long long)idx->sa_ns);
  if (n == 0) return GB_OK;
  GB_HIP(hipSetDevice(idx->device));
  Workspace &W = workspace(idx->device);
  if (!W.stream) GB_HIP(hipStreamCreateWithFlags(&W.stream, hipStreamNonBlocking));
  GB_HIP(W.ensure(3, sizeof(int64_t) * 2 * (size_t)n));
  int64_t *d = (int64_t *)W.buf[3];
  GB_HIP(hipMemcpyAsync(d, pos, sizeof(int64_t) * n, hipMemcpyHostToDevice, W.stream));
  hipLaunchKernelGGL(sa_raw_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, W.stream, idx->d_sa, d, n, d + n);
  GB_HIP(hipGetLastError());
  GB_HIP(hipMemcpyAsync(out, d + n, sizeof(int64_t) * n, hipMemcpyDeviceToHost, W.stream));
  GB_HIP(hipStreamSynchronize(W.stream));
  return GB_OK;
}

int gb_fmi_sa_one_step(gb_fmi_index *idx, int64_t pos, int64_t *sa_entry, int64_t *offset, int32_t *done) {
  GB_ARG(idx && sa_entry && offset && done, "gb_fmi_sa_one_step: null argument");
  GB_ARG(pos >= 0 && pos < idx->n, "gb_fmi_sa_one_step: row %lld outside [0, %lld)", (long long)pos, (long long)idx->n);
  GB_HIP(hipSetDevice(idx->device));
  Workspace &W = workspace(idx->device);
  if (!W.stream) GB_HIP(hipStreamCreateWithFlags(&W.stream, hipStreamNonBlocking));
  GB_HIP(W.ensure(9, 4 * sizeof(int64_t)));
  DevIndex F;
  F.occ = nullptr;
  for (int b = 0; b < 5; b++) F.count[b] = idx->count[b];
  F.sentinel = idx->sentinel;
  int64_t *d = (int64_t *)W.buf[9];
  hipLaunchKernelGGL(sa_one_step_kernel, dim3(1), dim3(1), 0, W.stream, idx->d_occ, idx->d_sa, F, pos, *offset, d);
  GB_HIP(hipGetLastError());
  int64_t r[3];
  GB_HIP(hipMemcpyAsync(r, d, sizeof(r), hipMemcpyDeviceToHost, W.stream));
  GB_HIP(hipStreamSynchronize(W.stream));
  *done = (int32_t)r[0];
  *sa_entry = r[1];
  *offset = r[2];
  return GB_OK;
}

}  // extern "C"
