// gather_roof.hip -- the random-gather ceiling of one MI355X, the roofline the rank kernels live under.
//
// fm_quickscan and bsf_search read HBM as independent random gathers (64-B Occ blocks, 8-B k-mer
// and text words, 4-B suffix-array values), not as streams, so the 8 TB/s streaming peak is not
// the ceiling they can reach: every gather moves at least one 64-B fabric request
// (profiles/r01_fetch_calibration.json) and DRAM pages are opened at random.  This tool measures
// the ceiling directly: every lane issues D independent random accesses of one kind per round
// (D = 1, 2, 4, 8 in flight per lane), over a 32 GiB buffer (beyond the 256 MiB Infinity Cache),
// with the grid sized to fill the chip, timed with HIP events.  Addresses come from a per-lane
// LCG fed by the loaded data (a power-of-two mask, no 64-bit modulo: the kernel must not be ALU-bound).  It prints one JSON object:
// accesses/s and fabric bytes/s (64 B per access; 128 B for two-line blocks) per kind and depth.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/gather_roof tools/gather_roof.hip && tools/gather_roof
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

// D random 64-B blocks per lane per round (4 x 16-B loads each, as loadBlock), `rounds` rounds;
// each round's addresses depend on the previous round's data, so a lane has exactly D blocks in
// flight, as a read's dependent FM-step chain has
template <int D>
__global__ void __launch_bounds__(256) g_block64(const u32x4 *buf, uint64_t nblocks, int rounds, uint32_t *out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t st[D];
#pragma unroll
  for (int d = 0; d < D; ++d) st[d] = mix(g * D + d);
  uint32_t acc = 0;
  for (int r = 0; r < rounds; ++r) {
    u32x4 v[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const u32x4 *p = buf + ((st[d] >> 20) & (nblocks - 1)) * 4;  // nblocks: a power of two
#pragma unroll
      for (int j = 0; j < 4; ++j) v[d][j] = __builtin_nontemporal_load(p + j);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const uint32_t x = v[d][0].x ^ v[d][1].y ^ v[d][2].z ^ v[d][3].w;
      acc += x;
      st[d] = st[d] * 6364136223846793005ULL + (1442695040888963407ULL ^ x);  // LCG step, data-dependent
    }
  }
  if (acc == 0x12345678u) out[0] = (uint32_t)g;
}

// The same random 64-B blocks, loaded cooperatively by the 4 lanes of a quad: for each of the
// quad's 4 blocks in turn, lane q of the quad loads bytes [16q, 16q + 16) of it, so one load
// instruction covers 16 whole blocks (one 64-B line each) instead of 64 quarter blocks.  The owner
// gets its block back through 12 quad permutes (__shfl within the quad).
template <int D>
__global__ void __launch_bounds__(256) g_block64_quad(const u32x4 *buf, uint64_t nblocks, int rounds, uint32_t *out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = (int)(threadIdx.x & 63), q = lane & 3, qb = lane & ~3;
  uint64_t st[D];
#pragma unroll
  for (int d = 0; d < D; ++d) st[d] = mix(g * D + d);
  uint32_t acc = 0;
  for (int r = 0; r < rounds; ++r) {
    u32x4 v[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const uint64_t mine = (st[d] >> 20) & (nblocks - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint64_t bj = (uint64_t)__shfl((long long)mine, qb + j);
        v[d][j] = __builtin_nontemporal_load(buf + bj * 4 + q);  // part q of block j
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      // owner q needs part p of its block from lane qb + p, which holds it in v[d][q]
      uint32_t x = 0;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        u32x4 w = v[d][0];
#pragma unroll
        for (int j = 1; j < 4; ++j) w = ((lane & 3) == j) ? v[d][j] : w;  // what this lane sends: v[q'] for owner q'...
        const uint32_t y = (uint32_t)__shfl((int)(p == 0 ? w.x : p == 1 ? w.y : p == 2 ? w.z : w.w), qb + p);
        x ^= y;
      }
      acc += x;
      st[d] = st[d] * 6364136223846793005ULL + (1442695040888963407ULL ^ x);
    }
  }
  if (acc == 0x12345678u) out[0] = (uint32_t)g;
}

// D random 8-B words per lane per round (k-mer entries, text words)
template <int D>
__global__ void __launch_bounds__(256) g_word8(const uint64_t *buf, uint64_t nwords, int rounds, uint32_t *out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t st[D];
#pragma unroll
  for (int d = 0; d < D; ++d) st[d] = mix(g * D + d + 0x777);
  uint32_t acc = 0;
  for (int r = 0; r < rounds; ++r) {
    uint64_t v[D];
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = buf[(st[d] >> 20) & (nwords - 1)];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc += (uint32_t)v[d];
      st[d] = st[d] * 6364136223846793005ULL + (1442695040888963407ULL ^ v[d]);
    }
  }
  if (acc == 0x12345678u) out[0] = (uint32_t)g;
}

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

template <typename F>
static int timeIt(F launch, float *ms) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();  // warm-up
  CK(hipEventRecord(a, 0));
  launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  CK(hipEventElapsedTime(ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main() {
  const uint64_t bytes = 32ULL << 30;  // 32 GiB
  void *buf = nullptr;
  uint32_t *out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 0x5A, bytes));
  CK(hipDeviceSynchronize());
  // 256 CUs x 8 waves x 64 lanes resident; 4x that in the grid
  const uint32_t lanes = 256u * 8u * 64u * 4u;
  const int rounds = 64;
  const dim3 grid(lanes / 256), blk(256);
  printf("{\"tool\": \"tools/gather_roof.hip\", \"buffer_GiB\": 32, \"lanes\": %u, \"rounds\": %d", lanes, rounds);
#define RUN(KIND, D, EXPR, FABRIC)                                                                   \
  {                                                                                                  \
    float ms = 0;                                                                                    \
    if (timeIt([&] { EXPR; }, &ms)) return 1;                                                        \
    const double acc = (double)lanes * rounds * D;                                                   \
    printf(", \"%s_d%d\": {\"ms\": %.3f, \"Gaccess_per_s\": %.2f, \"fabric_GBs\": %.1f}", KIND, D, ms, \
           acc / ms / 1e6, acc * FABRIC / ms / 1e6);                                                 \
    fflush(stdout);                                                                                  \
  }
  RUN("block64", 1, hipLaunchKernelGGL(g_block64<1>, grid, blk, 0, 0, (const u32x4 *)buf, bytes / 64, rounds, out), 64.0)
  RUN("block64", 2, hipLaunchKernelGGL(g_block64<2>, grid, blk, 0, 0, (const u32x4 *)buf, bytes / 64, rounds, out), 64.0)
  RUN("block64", 4, hipLaunchKernelGGL(g_block64<4>, grid, blk, 0, 0, (const u32x4 *)buf, bytes / 64, rounds, out), 64.0)
  RUN("block64quad", 1, hipLaunchKernelGGL(g_block64_quad<1>, grid, blk, 0, 0, (const u32x4 *)buf, bytes / 64, rounds, out), 64.0)
  RUN("block64quad", 2, hipLaunchKernelGGL(g_block64_quad<2>, grid, blk, 0, 0, (const u32x4 *)buf, bytes / 64, rounds, out), 64.0)
  RUN("word8", 1, hipLaunchKernelGGL(g_word8<1>, grid, blk, 0, 0, (const uint64_t *)buf, bytes / 8, rounds, out), 64.0)
  RUN("word8", 2, hipLaunchKernelGGL(g_word8<2>, grid, blk, 0, 0, (const uint64_t *)buf, bytes / 8, rounds, out), 64.0)
  RUN("word8", 4, hipLaunchKernelGGL(g_word8<4>, grid, blk, 0, 0, (const uint64_t *)buf, bytes / 8, rounds, out), 64.0)
  RUN("word8", 8, hipLaunchKernelGGL(g_word8<8>, grid, blk, 0, 0, (const uint64_t *)buf, bytes / 8, rounds, out), 64.0)
  printf("}\n");
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
