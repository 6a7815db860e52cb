// rewrite_probe.hip -- does WRITE_SIZE on gfx950 (MI355X) count every store to a small, repeatedly
// rewritten per-wave region (write-through-like), or only the region once (L2 write-back)?
// This is the access class of fmi smem_search's `prev` lists (16 B per lane, wave-interleaved,
// rewritten in place, a few KB hot per wave). Each wave owns `depth` KB (depth x 64 lanes x 16 B);
// every lane stores `iters` times, cycling through its depth slots, with 16 waves per CU.
// Store bytes and region bytes are printed; compare with rocprofv3 --pmc WRITE_SIZE (KiB):
//   rocprofv3 --pmc WRITE_SIZE --output-format csv -d DIR -o run -- ./rewrite_probe
//   build: hipcc --offload-arch=gfx950 -O3 -o rewrite_probe rewrite_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// mode 0: every lane stores each trip (full 1 KB rows); mode 1: one lane in 8 active per trip
// (divergent partial rows, like lanes of a wave at different list depths)
__global__ __launch_bounds__(64) void rewrite(uint4 *scratch, int depth, int iters, int mode) {
  uint4 *base = scratch + (size_t)blockIdx.x * depth * 64 + threadIdx.x;
  uint32_t v = threadIdx.x * 2654435761u + blockIdx.x;
  for (int i = 0; i < iters; ++i) {
    const int e = (i + (mode ? (int)(threadIdx.x >> 3) : 0)) % depth;
    if (mode == 0 || ((threadIdx.x + i) & 7) == 0) base[(size_t)e * 64] = make_uint4(v, v + i, v ^ i, e);
    v = v * 1664525u + 1013904223u;
  }
}

int main() {
  int cus = 256;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  cus = prop.multiProcessorCount;
  const int waves = cus * 16, iters = 4096;
  uint4 *d = nullptr;
  CK(hipMalloc(&d, (size_t)waves * 64 * 64 * sizeof(uint4)));
  for (int mode = 0; mode < 2; ++mode)
    for (int depth : {1, 4, 8, 16, 64}) {
      hipLaunchKernelGGL(rewrite, dim3(waves), dim3(64), 0, 0, d, depth, iters, mode);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      const double stores = (double)waves * 64 * iters * 16 / (mode ? 8 : 1);
      const double region = (double)waves * depth * 1024;
      printf("mode %d depth %2d KB/wave: store bytes %.3f GB, region %.1f MB (%.1f MB per XCD)\n", mode, depth,
             stores / 1e9, region / 1e6, region / 8e6);
    }
  CK(hipFree(d));
  return 0;
}
