// gather_probe.hip -- random 64-byte line gather ceiling on MI355X (the fmi roofline calibration).
// Every lane runs CH independent pointer chases; each hop loads one random 64-B line (4 x 16 B,
// like one Occ2 line) and derives the next line index from the loaded data, so the hops of a chain
// are dependent exactly like backwardExt calls. Reports G lines/s and GB/s (64 B per hop).
//   build: hipcc --offload-arch=gfx950 -O3 -o gather_probe gather_probe.hip
//   run:   ./gather_probe  (sweeps table size x waves per CU x chains per lane)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void fill(uint4 *t, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h = i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
    t[i] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)(h * 3), (uint32_t)(h >> 17));
  }
}

template <int CH>
__global__ __launch_bounds__(64) void chase(const uint4 *__restrict__ t, uint64_t mask, int hops, uint32_t *out) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  uint64_t x[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) x[c] = ((uint64_t)(gid * 2654435761u) * (c + 1) * 0x9E3779B97F4A7C15ull >> 11) & mask;
  uint32_t acc = 0;
  for (int h = 0; h < hops; h++) {
    uint4 a[CH], b[CH], c2[CH], d[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) {
      const uint4 *p = t + x[c] * 4;
      a[c] = p[0]; b[c] = p[1]; c2[c] = p[2]; d[c] = p[3];
    }
#pragma unroll
    for (int c = 0; c < CH; c++) {
      const uint64_t v = ((uint64_t)(a[c].x ^ b[c].y ^ c2[c].z ^ d[c].w) << 32) | (a[c].y ^ d[c].x);
      x[c] = (v * 0x9E3779B97F4A7C15ull + x[c]) >> 7 & mask;
      acc += a[c].z;
    }
  }
  out[gid] = acc + (uint32_t)x[0];
}

template <int CH>
double run(const uint4 *t, uint64_t lines, int waves_per_cu, int hops, uint32_t *out) {
  const int blocks = 256 * waves_per_cu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(chase<CH>, dim3(blocks), dim3(64), 0, 0, t, lines - 1, 8, out);  // warm
  hipEventRecord(e0);
  hipLaunchKernelGGL(chase<CH>, dim3(blocks), dim3(64), 0, 0, t, lines - 1, hops, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0); hipEventDestroy(e1);
  return (double)blocks * 64 * CH * hops / (ms * 1e-3) / 1e9;  // G lines/s
}

int main() {
  const uint64_t max_bytes = 4ull << 30;
  uint4 *t;
  uint32_t *out;
  CK(hipMalloc(&t, max_bytes));
  CK(hipMalloc(&out, 256 * 64 * 64 * sizeof(uint32_t)));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, t, max_bytes / 16);
  CK(hipDeviceSynchronize());
  for (uint64_t mb : {64ull, 512ull, 4096ull}) {
    const uint64_t lines = (mb << 20) / 64;
    for (int w : {8, 16, 32}) {
      for (int ch : {1, 2, 4}) {
        double g = ch == 1 ? run<1>(t, lines, w, 256, out) : ch == 2 ? run<2>(t, lines, w, 128, out) : run<4>(t, lines, w, 64, out);
        printf("table %5llu MB  waves/CU %2d  chains/lane %d : %6.1f G lines/s = %7.0f GB/s (64 B/line)\n",
               (unsigned long long)mb, w, ch, g, g * 64);
        fflush(stdout);
      }
    }
  }
  CK(hipFree(t));
  CK(hipFree(out));
  return 0;
}
