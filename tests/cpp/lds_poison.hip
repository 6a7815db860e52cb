// lds_poison.hip -- TEST INFRASTRUCTURE (tests/test_lds_poison.py): fill every CU's LDS with an
// adversarial pattern before a product kernel runs, so a kernel that reads LDS words it never wrote
// in this workgroup (stale state from the CU's previous workgroup, as chain_rows' stamp ring did
// before commit 1da81ef) produces wrong results deterministically instead of occasionally.
// A workgroup may declare all 160 KiB of a CU's LDS, so each workgroup owns a whole CU's LDS while it
// runs; the grid holds many workgroups per CU so every CU runs at least one.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kLdsBytes = 160 * 1024;
constexpr int kWords = kLdsBytes / 4;

__global__ __launch_bounds__(256) void lds_poison_kernel(uint32_t mode, uint32_t value, uint32_t seed,
                                                         uint32_t *sink) {
  extern __shared__ uint32_t lds[];
  for (int w = threadIdx.x; w < kWords; w += blockDim.x) {
    uint32_t v;
    switch (mode) {
      case 0: v = 0xFFFFFFFFu; break;                 // all ones
      case 1: v = (uint32_t)w + 1u; break;            // word index + 1 (an i + 1 stamp at its own slot)
      case 2: v = value; break;                       // one constant everywhere
      case 3: v = (uint32_t)w + value; break;         // word index + offset
      default: {                                      // hashed
        uint32_t x = (uint32_t)w * 0x9E3779B9u ^ seed ^ (blockIdx.x * 0x85EBCA6Bu);
        x ^= x >> 16;
        x *= 0x7FEB352Du;
        x ^= x >> 15;
        v = x;
      }
    }
    lds[w] = v;
  }
  __syncthreads();
  // keep the stores: one word of the block's LDS goes out (never read back)
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = lds[(blockIdx.x * 977u) % kWords];
}

}  // namespace

extern "C" {

// Fill the LDS of every CU of `device` with the pattern (mode, value, seed) and wait for it. Returns
// 0, or the HIP error code.
int lds_poison(int device, uint32_t mode, uint32_t value, uint32_t seed) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  hipDeviceProp_t prop;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return (int)e;
  const int blocks = 8 * prop.multiProcessorCount;
  static uint32_t *sink = nullptr;
  if (!sink && (e = hipMalloc(&sink, sizeof(uint32_t) * (size_t)blocks)) != hipSuccess) return (int)e;
  if ((e = hipFuncSetAttribute((const void *)lds_poison_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               kLdsBytes)) != hipSuccess)
    return (int)e;
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(256), kLdsBytes, 0, mode, value, seed, sink);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  return (int)hipDeviceSynchronize();
}

}  // extern "C"
