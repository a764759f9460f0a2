// calib_fetch.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE against known byte
// counts for the access shapes the hot path uses (MI355X_MICROARCH.md §HBM: only wide
// streaming reads are calibrated by the guide; "calibrate on a known byte count in your
// own access pattern").  Measurement tool, not product code.
//
//   k_stream    16 B per lane, fully coalesced, N bytes            (known: N)
//   k_gather64  4 lanes x 16 B = one 64-B record at a random index (known: M x 64)
//   k_gather16  one 16-B record per lane at a random index          (known: M x 16 requested)
//   k_gather4   one 4-B word per lane at a random index             (known: M x 4 requested)
//   k_write8    8 B per lane, scattered                             (known: M x 8 written)
//
// Tables are 2 GiB so that random reads miss L2 and the 256 MiB Infinity Cache.
// Run:  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d DIR -- ./calib_fetch
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__device__ inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__global__ void k_stream(const uint4* __restrict__ a, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_gather64(const uint4* __restrict__ a, uint64_t n_rec, uint64_t m, uint32_t* out) {
  const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (uint64_t i = tid >> 2; i < m; i += ((uint64_t)gridDim.x * blockDim.x) >> 2) {
    const uint64_t r = mix64(i) % n_rec;
    const uint4 v = a[r * 4 + (threadIdx.x & 3)];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_gather16(const uint4* __restrict__ a, uint64_t n16, uint64_t m, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[mix64(i) % n16];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_gather4(const uint32_t* __restrict__ a, uint64_t n4, uint64_t m, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= a[mix64(i) % n4];
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_write8(uint64_t* __restrict__ a, uint64_t n8, uint64_t m) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
    a[mix64(i) % n8] = i;
}

int main() {
  const uint64_t bytes = 2ull << 30;
  void* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 1, bytes));
  const uint64_t m = 16ull << 20;  // random accesses per gather launch
  const dim3 grid(8192), block(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_stream, grid, block, 0, 0, (const uint4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_gather64, grid, block, 0, 0, (const uint4*)buf, bytes / 64, m, out);
    hipLaunchKernelGGL(k_gather16, grid, block, 0, 0, (const uint4*)buf, bytes / 16, m, out);
    hipLaunchKernelGGL(k_gather4, grid, block, 0, 0, (const uint32_t*)buf, bytes / 4, m, out);
    hipLaunchKernelGGL(k_write8, grid, block, 0, 0, (uint64_t*)buf, bytes / 8, m);
  }
  CK(hipDeviceSynchronize());
  printf("{\"stream_bytes\": %llu, \"gather64_bytes\": %llu, \"gather16_bytes\": %llu, "
         "\"gather4_bytes\": %llu, \"write8_bytes\": %llu}\n",
         (unsigned long long)bytes, (unsigned long long)(m * 64), (unsigned long long)(m * 16),
         (unsigned long long)(m * 4), (unsigned long long)(m * 8));
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
