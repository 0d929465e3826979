// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE for the align path's access patterns on gfx950.
//
// MI355X_MICROARCH.md (§HBM) calibrates FETCH_SIZE only for wide coalesced streaming reads
// (reported at 1/2 of the bytes) and asks for a calibration of any other pattern on a known byte
// count.  The search kernels read random 64-B Occ blocks (4 x 16-B nontemporal loads per lane,
// loadBlock in bsf_core.h), random 8-B words (k-mer table, text) and random 4-B suffix-array values.
// Each kernel here issues exactly one such access per lane at a pseudo-random, distinct, aligned
// address of a 16 GiB buffer (far beyond the 256 MiB Infinity Cache), so the DRAM bytes are known:
// lanes x access size (or x 64 / 128 B if the fabric moves whole half / full lines).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d gpurun_out/calib -- tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {  // splitmix64
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// one random 64-B block per lane, read as 4 x 16 B (the Occ block gather)
__global__ void calib_block64(const u32x4 *buf, uint64_t nblocks, uint32_t *out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t b = mix(g) % nblocks;
  const u32x4 *p = buf + b * 4;
  u32x4 a = __builtin_nontemporal_load(p + 0), c = __builtin_nontemporal_load(p + 1);
  u32x4 d = __builtin_nontemporal_load(p + 2), e = __builtin_nontemporal_load(p + 3);
  const uint32_t v = a.x ^ a.y ^ a.z ^ a.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w ^ e.x ^ e.y ^ e.z ^ e.w;
  if (v == 0x12345678u) out[0] = (uint32_t)g;  // keeps the loads alive (never true: the buffer is 0x5A bytes)
}

// one random 8-B word per lane (k-mer table entry, 2-bit text word)
__global__ void calib_word8(const uint64_t *buf, uint64_t nwords, uint32_t *out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t w = buf[mix(g ^ 0xABCDEFULL) % nwords];
  if ((uint32_t)(w ^ (w >> 32)) == 0x12345678u) out[0] = (uint32_t)g;
}

// one random 4-B value per lane (suffix-array gather)
__global__ void calib_word4(const uint32_t *buf, uint64_t nwords, uint32_t *out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w = buf[mix(g ^ 0x5555ULL) % nwords];
  if (w == 0x12345678u) out[0] = (uint32_t)g;
}

// coalesced streaming 16 B per lane (the guide's calibrated case, as a control)
__global__ void calib_stream16(const u32x4 *buf, uint32_t *out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const u32x4 a = __builtin_nontemporal_load(buf + g);
  if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678u) out[0] = (uint32_t)g;
}

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main() {
  const uint64_t bytes = 16ULL << 30;  // 16 GiB
  void *buf = nullptr;
  uint32_t *out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 0x5A, bytes));
  CK(hipDeviceSynchronize());
  const uint32_t lanes = 1u << 24;  // 16M accesses per kernel: distinct with high probability
  const dim3 grid(lanes / 256), blk(256);
  hipLaunchKernelGGL(calib_block64, grid, blk, 0, 0, (const u32x4 *)buf, bytes / 64, out);
  hipLaunchKernelGGL(calib_word8, grid, blk, 0, 0, (const uint64_t *)buf, bytes / 8, out);
  hipLaunchKernelGGL(calib_word4, grid, blk, 0, 0, (const uint32_t *)buf, bytes / 4, out);
  hipLaunchKernelGGL(calib_stream16, grid, blk, 0, 0, (const u32x4 *)buf, out);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("{\"lanes\": %u, \"block64_bytes\": %llu, \"word8_bytes\": %llu, \"word4_bytes\": %llu, \"stream16_bytes\": %llu}\n",
         lanes, (unsigned long long)lanes * 64ULL, (unsigned long long)lanes * 8ULL, (unsigned long long)lanes * 4ULL,
         (unsigned long long)lanes * 16ULL);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
