// pmc_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 (MI355X) for the access
// classes this repo's kernels use, against known byte counts (MI355X_MICROARCH.md, HBM section:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access
// pattern"). One kernel per class, each touching every byte of its region once, regions far past
// the 256 MiB Infinity Cache and streamed over in between so nothing is served on-die:
//   gather64  random 64-B lines, 4 x 16 B per lane (one full line per lane)
//   gather32  random 32-B blocks, 2 x 16 B per lane (the Occ32 gather of fmi / SA)
//   gather8   random 8-B words, one per 64-B line (the sampled-SA lookup)
//   stream16  coalesced 16 B per lane read (the guide's calibrated case: FETCH_SIZE = 1/2)
//   write16   coalesced 16 B per lane store
// Known bytes are printed; run each counter in its own pass:
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d DIR -o run -- ./pmc_calib
//   build: hipcc --offload-arch=gfx950 -O3 -o pmc_calib pmc_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void fill(uint4 *t, uint64_t n, uint32_t salt) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = make_uint4((uint32_t)i ^ salt, (uint32_t)(i >> 32), salt, (uint32_t)i * 3u);
}

// a random visit order that reads every unit exactly once: odd multiplies mod 2^k and xorshifts
// are both invertible on k-bit integers
__device__ __forceinline__ uint64_t perm(uint64_t i, int k) {
  const uint64_t m = (1ull << k) - 1;
  uint64_t x = (i * 0x9E3779B97F4A7C15ull) & m;
  x ^= x >> (k / 2);
  x = (x * 0xBF58476D1CE4E5B9ull) & m;
  x ^= x >> (k / 3 + 1);
  return x;
}

__global__ void gather64(const uint4 *t, int k, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << k); i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 *p = t + perm(i, k) * 4;
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    acc += a.x ^ b.y ^ c.z ^ d.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void gather32(const uint4 *t, int k, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << k); i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 *p = t + perm(i, k) * 2;
    const uint4 a = p[0], b = p[1];
    acc += a.x ^ b.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// 8-B words, one per 64-B line (every line of the region once): known useful bytes = lines * 8
__global__ void gather8(const uint64_t *t, int k, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << k); i += (uint64_t)gridDim.x * blockDim.x)
    acc += (uint32_t)t[perm(i, k) * 8 + (i & 7)];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void stream16(const uint4 *t, uint64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 a = t[i];
    acc += a.x ^ a.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void write16(uint4 *t, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main() {
  const int kb = 31;  // 2 GiB per region: 8x the Infinity Cache
  const uint64_t bytes = 1ull << kb;
  uint4 *a, *b;
  uint32_t *out;
  const int grid = 256 * 16, block = 256;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&out, (size_t)grid * block * 4));
  auto evict = [&](uint32_t salt) {  // stream the other region through L2 and the Infinity Cache
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, b, bytes / 16, salt);
    return hipDeviceSynchronize();
  };
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, a, bytes / 16, 7u);
  CK(evict(1));
  printf("gather64 known read bytes %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(gather64, dim3(grid), dim3(block), 0, 0, a, kb - 6, out);
  CK(hipDeviceSynchronize());
  CK(evict(2));
  printf("gather32 known read bytes %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(gather32, dim3(grid), dim3(block), 0, 0, a, kb - 5, out);
  CK(hipDeviceSynchronize());
  CK(evict(3));
  printf("gather8 known read bytes %llu (8 B from each 64-B line; %llu as whole lines)\n",
         (unsigned long long)(bytes / 8), (unsigned long long)bytes);
  hipLaunchKernelGGL(gather8, dim3(grid), dim3(block), 0, 0, (const uint64_t *)a, kb - 6, out);
  CK(hipDeviceSynchronize());
  CK(evict(4));
  printf("stream16 known read bytes %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(stream16, dim3(grid), dim3(block), 0, 0, a, bytes / 16, out);
  CK(hipDeviceSynchronize());
  printf("write16 known write bytes %llu\n", (unsigned long long)bytes);
  hipLaunchKernelGGL(write16, dim3(grid), dim3(block), 0, 0, a, bytes / 16);
  CK(hipDeviceSynchronize());
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(out));
  return 0;
}
