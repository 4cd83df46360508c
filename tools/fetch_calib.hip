// fetch_calib — calibrates rocprofv3 FETCH_SIZE on gfx950 for the access
// widths the decode kernels use (MI355X_MICROARCH.md: only 16-byte streaming
// reads are calibrated; "calibrate on a known byte count in your own access
// pattern").  Each kernel reads a known number of bytes; run it under
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o calib -- ./fetch_calib
// and divide each dispatch's FETCH_SIZE by the byte count printed here.
//   k_stream16   16 B per lane, coalesced, over 1 GiB (the guide's ½ case)
//   k_stream4    4 B per lane, coalesced, over 1 GiB
//   k_gather4_T  4-byte random gathers (k_dict4's b = 16 / 20 dictionary
//                reads) from a T-byte table: 256 KiB and 4 MiB, 2^28 gathers
// Diagnostic tool only (not part of libpqgpu).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void k_stream16(const uint4* __restrict__ p, size_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads
}

__global__ void k_stream4(const uint32_t* __restrict__ p, size_t n4, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// 4-byte gathers at pseudo-random indices (splitmix-like hash of the index)
__global__ void k_gather4(const uint32_t* __restrict__ table, uint32_t mask, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9e3779b9u;
    x ^= x >> 16;
    x *= 0x85ebca6bu;
    x ^= x >> 13;
    acc ^= table[x & mask];
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

int main() {
  const size_t big = (size_t)1 << 30;  // 1 GiB: past the 256 MiB Infinity Cache
  uint8_t* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, big));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, big));
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  const dim3 grid(cus * 8), block(256);
  // warm-up of every kernel, then the measured dispatches (printed in order)
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_stream16, grid, block, 0, 0, (const uint4*)buf, big / 16, sink);
    hipLaunchKernelGGL(k_stream4, grid, block, 0, 0, (const uint32_t*)buf, big / 4, sink);
    const size_t ng = (size_t)1 << 28;
    hipLaunchKernelGGL(k_gather4, grid, block, 0, 0, (const uint32_t*)buf, (uint32_t)((256u << 10) / 4 - 1), ng, sink);
    hipLaunchKernelGGL(k_gather4, grid, block, 0, 0, (const uint32_t*)buf, (uint32_t)((4u << 20) / 4 - 1), ng, sink);
    CK(hipDeviceSynchronize());
  }
  printf("dispatch order (x2, the second set is the measurement):\n");
  printf("k_stream16 bytes=%zu\n", big);
  printf("k_stream4 bytes=%zu\n", big);
  printf("k_gather4 table=262144 gathers=%zu useful_bytes=%zu\n", (size_t)1 << 28, ((size_t)1 << 28) * 4);
  printf("k_gather4 table=4194304 gathers=%zu useful_bytes=%zu\n", (size_t)1 << 28, ((size_t)1 << 28) * 4);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
