// chain_internal.h -- the device-resident chain batch shared by chain.hip (chain_dp) and
// chain_bt.hip (the backtrack that consumes its outputs).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gbchain {
struct ChainBt;                   // chain_bt.hip
void chain_bt_destroy(ChainBt *);
}  // namespace gbchain

struct gb_chain_batch {
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  int64_t ncalls = 0, nanchors = 0;
  int64_t cap_calls = 0, cap_anchors = 0;  // allocated sizes (a refilled batch reuses its buffers)
  int64_t *d_off = nullptr;
  float *d_aq = nullptr;
  int32_t *d_par4 = nullptr, *d_order = nullptr;
  uint64_t *d_x = nullptr, *d_y = nullptr;
  int32_t *d_out = nullptr;  // score | parent | target | peak, nanchors (>= 1) each
  unsigned long long *d_vis = nullptr;
  unsigned long long *d_prof = nullptr;  // GB_CHAIN_PROF=1 phase clocks (development aid)
  bool ran = false;
  gbchain::ChainBt *bt = nullptr;  // backtrack state (gb_chain_batch_backtrack)
};
