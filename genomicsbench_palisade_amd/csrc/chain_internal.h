// chain_internal.h -- the device-resident chain batch shared by chain.hip (chain_dp), chain_split.hip
// (long calls as speculative segments) and chain_bt.hip (the backtrack that consumes the outputs).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

namespace gbchain {
struct ChainBt;                   // chain_bt.hip
void chain_bt_destroy(ChainBt *);

// One block of the sequential kernel: anchors [in, in + n) of call `call` (x/y offsets), outputs at
// `out` in the final arrays (kVFinal: scores, parents, targets, peaks, visited count) or in the
// segment scratch (kVScratch: scores and parents only), or in the final arrays for anchors
// [known, n) only (kVFixup: the first `known` anchors are already final and are read, not computed;
// the block works with indices relative to its first anchor, memory holds call-relative parents).
enum { kVFinal = 1, kVScratch = 2, kVFixup = 4 };
struct VCall {
  int64_t in, out;
  int32_t n, call, known, mode;
  int32_t pbase, pad;  // kVFixup: parents in memory are call-relative, pbase = the block's first anchor
};

// A call run as speculative segments (chain_split.hip): segment s covers anchors [c_s, e_s) of the
// call, its speculative run starts at the warm-up anchor a_s and its outputs for [a_s, e_s) sit at
// scratch offset soff.
struct Seg {
  int32_t cs, es, as, pad;
  int64_t soff;
};
struct SplitCall {
  int64_t off;         // the call's first anchor in the batch
  int32_t n, call;     // anchors, call index
  int32_t seg0, nseg;  // its segments in the segment table
  int32_t c1;          // first anchor of segment 1 (anchors before it are final after the first run)
  int32_t cbase;       // first chunk: anchor i >= c1 has chunk-space index 64 * cbase + (i - c1)
};
// 64-anchor chunks of the split calls' anchors [c_1, n) (verification, marks, pointer jumping)
struct Chunk {
  int32_t sc, start;  // split-call index, first anchor (call-relative)
};
}  // namespace gbchain

struct gb_chain_batch {
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipStream_t stream2 = nullptr;            // full-ring blocks run here, beside the small-ring ones
  hipEvent_t fj[2] = {nullptr, nullptr};    // fork / join of the two streams
  int64_t ncalls = 0, nanchors = 0;
  int64_t cap_calls = 0, cap_anchors = 0;  // allocated sizes (a refilled batch reuses its buffers)
  int64_t *d_off = nullptr;
  float *d_aq = nullptr;
  int32_t *d_par4 = nullptr;
  uint64_t *d_x = nullptr, *d_y = nullptr;
  int32_t *d_out = nullptr;  // score | parent | target | peak, nanchors (>= 1) each
  unsigned long long *d_vis = nullptr;
  unsigned long long *d_prof = nullptr;  // GB_CHAIN_PROF=1 phase clocks (development aid)
  bool ran = false;
  gbchain::ChainBt *bt = nullptr;  // backtrack state (gb_chain_batch_backtrack)

  // the block table: n_rows blocks for chain_rows (sorted x, chain_rows.hip), then n_small
  // small-ring blocks and the full-ring ones for chain_kernel, each class longest first
  std::vector<gbchain::VCall> vc;
  int n_rows = 0;
  int n_small = 0;
  gbchain::VCall *d_vc = nullptr;
  int64_t cap_vc = 0;
  // long calls as speculative segments (chain_split.hip); empty when no call is split
  std::vector<gbchain::SplitCall> split;
  std::vector<gbchain::Seg> segs;
  std::vector<gbchain::Chunk> chunks;
  std::vector<int32_t> st;  // window start st(i) of the split calls' anchors >= c1, chunk-space index
  int64_t scratch_n = 0;
  int max_split_n = 0;
  gbchain::SplitCall *d_split = nullptr;
  gbchain::Seg *d_segs = nullptr;
  gbchain::Chunk *d_chunks = nullptr;
  int32_t *d_st = nullptr;        // st, chunk-space index
  int32_t *d_sscore = nullptr, *d_sparent = nullptr;  // segment scratch
  int32_t *d_smark = nullptr;     // segment scratch: targets marks of chain_rows' speculative blocks
  uint64_t *d_need = nullptr;     // per chunk: anchors verify_lanes leaves to verify_kernel
  int32_t *d_slow = nullptr;      // [0]: chunks with such anchors, then their indices (verify_kernel's work list)
  int32_t *d_front = nullptr;     // per split call: first anchor not known to be final
  int32_t *d_fail = nullptr;      // per split call: first anchor whose guess failed verification
  int32_t *d_link[2] = {nullptr, nullptr};  // pointer jumping (chunk-space index or -1)
  int32_t *d_val[2] = {nullptr, nullptr};
  int32_t *d_t2 = nullptr;                 // split anchors' targets marks, merged at the end
  unsigned long long *d_viscall = nullptr; // visited pairs per split call
  int64_t cap_split = 0, cap_segs = 0, cap_chunks = 0, cap_st = 0, cap_sscore = 0, cap_sparent = 0, cap_smark = 0, cap_need = 0, cap_slow = 0, cap_front = 0,
          cap_jump = 0, cap_t2 = 0, cap_viscall = 0;
  int64_t spec_rounds = 0, fixups = 0;  // statistics of the last run
  int32_t *h_fail = nullptr;   // pinned copy of d_fail (the host reads it mid-step)
  int64_t cap_hfail = 0;
  hipEvent_t fail_ev = nullptr;  // recorded behind the d_fail copy
};

namespace gbchain {
// chain_split.hip
int split_plan(gb_chain_batch *B, const int64_t *offsets, const uint64_t *x, const int32_t *params4);
int split_resolve(gb_chain_batch *B);
int step_clear_launch(gb_chain_batch *B);  // every per-step clear in one launch (before the blocks)
void split_free(gb_chain_batch *B);
int launch_chain(gb_chain_batch *B, const VCall *d_vc, int nvc, int prof, bool small, hipStream_t stream);
int launch_table(gb_chain_batch *B, int prof);
// chain_rows.hip
int launch_rows(gb_chain_batch *B, const VCall *d_vc, int nvc, hipStream_t stream);
// Dynamic LDS that spreads a launch of nwg workgroups (waves_per_wg waves each, static_lds bytes of
// LDS each) over every SIMD: a launch with fewer waves than SIMD slots is latency-bound, and the
// dispatcher otherwise stacks its workgroups on few CUs. 0 when the launch fills the chip anyway.
size_t spread_lds(int nwg, int waves_per_wg, size_t static_lds);
// The current device's CU count and LDS per CU (queried once per device, thread-safe), and the
// dynamic LDS the chain kernels may request on it (96 KB, less on a device with less LDS).
struct DevLimits {
  int cus = 256;
  size_t lds_per_cu = 160 * 1024;
  size_t max_dyn = 96 * 1024;
};
const DevLimits &dev_limits();
// Runs set() once per (current device, slot), e.g. hipFuncSetAttribute for a kernel; thread-safe.
int once_per_device(int slot, int (*set)(const DevLimits &));
}  // namespace gbchain
