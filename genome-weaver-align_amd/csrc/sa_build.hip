// sa_build.hip -- MI355X index construction: cyclic suffix array by prefix doubling on the GPU
// (rocPRIM onesweep radix sort over 64-bit keys, 64-bit problem sizes), then BWT Occ blocks,
// 2-bit text and the reversed text, all built in HBM.
//
// The reference builds the same arrays on the CPU (PackFasta + CyclicSAIS + BWTransform,
// A/BWTransform.java:111-179, A/sais/CyclicSAIS.java:223-431).  The cyclic SA of a text that is
// not a power of a shorter string is unique, so any correct construction yields the identical
// index; tests/ compare this builder with the oracle's independent one.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <stdexcept>
#include <string>

#include "gwa_layout.h"

namespace gwa {

#define SCHK(x)                                                                                       \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("sa_build: ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)

static inline unsigned gridFor(uint64_t n, unsigned bs = 256) {
  uint64_t g = (n + bs - 1) / bs;
  return (unsigned)(g > 0x7FFFFFFFull ? 0x7FFFFFFF : g);
}

// key[i] = the first K symbols of rotation i, `bits` bits apiece (cyclic)
__global__ void saInitKeys(const uint8_t *__restrict__ T, uint64_t N, int K, int bits, uint64_t *__restrict__ key,
                           uint32_t *__restrict__ val) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = 0;
    uint64_t p = i;
    for (int j = 0; j < K; ++j) {
      k = (k << bits) | T[p];
      if (++p == N) p = 0;
    }
    key[i] = k;
    val[i] = (uint32_t)i;
  }
}

// head[j] = j if key[j] starts a new group else 0 ; dup counts positions equal to their predecessor
__global__ void saHeads(const uint64_t *__restrict__ key, uint64_t N, uint32_t *__restrict__ head,
                        unsigned long long *__restrict__ dup) {
  unsigned long long local = 0;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < N; j += (uint64_t)gridDim.x * blockDim.x) {
    bool start = j == 0 || key[j] != key[j - 1];
    head[j] = start ? (uint32_t)j : 0u;
    local += start ? 0 : 1;
  }
  if (local) atomicAdd(dup, local);
}

// rank[val[j]] = group start of position j
__global__ void saScatterRank(const uint32_t *__restrict__ grp, const uint32_t *__restrict__ val, uint64_t N,
                              uint32_t *__restrict__ rank) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < N; j += (uint64_t)gridDim.x * blockDim.x)
    rank[val[j]] = grp[j];
}

// doubling key in the current sorted order: (rank[i], rank[(i+h) mod N])
__global__ void saDoublingKeys(const uint32_t *__restrict__ rank, const uint32_t *__restrict__ val, uint64_t N, uint64_t h,
                               uint64_t *__restrict__ key) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < N; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i = val[j];
    uint64_t i2 = i + h;
    i2 %= N;
    key[j] = ((uint64_t)rank[i] << 32) | rank[i2];
  }
}

__global__ void reverseText(const uint8_t *__restrict__ T, uint64_t N, uint8_t *__restrict__ R) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x)
    R[i] = T[N - 1 - i];
}

struct Cnt4 {
  uint32_t c[4];
};
struct Cnt4Plus {
  __host__ __device__ Cnt4 operator()(const Cnt4 &a, const Cnt4 &b) const {
    Cnt4 r;
    for (int i = 0; i < 4; ++i) r.c[i] = a.c[i] + b.c[i];
    return r;
  }
};

// One lane per 128 BWT positions: BWT[p] = T[(SA[p]-1) mod N] (A/BWTransform.java:172-179)
__global__ void occLocal(const uint8_t *__restrict__ T, const uint32_t *__restrict__ SA, uint64_t N, uint64_t nb,
                         OccBlock *__restrict__ occ, Cnt4 *__restrict__ local) {
  for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t lo[2] = {0, 0}, hi[2] = {0, 0}, nm[2] = {0, 0};
    Cnt4 c = {{0, 0, 0, 0}};
    const uint64_t p0 = b * 128;
    for (int r = 0; r < 128; ++r) {
      uint64_t p = p0 + r;
      if (p >= N) break;
      uint64_t s = SA[p];
      uint8_t ch = T[s == 0 ? N - 1 : s - 1];
      if (ch >= 4) {
        nm[r >> 6] |= 1ULL << (r & 63);
      } else {
        if (ch & 1) lo[r >> 6] |= 1ULL << (r & 63);
        if (ch & 2) hi[r >> 6] |= 1ULL << (r & 63);
        c.c[ch]++;
      }
    }
    OccBlock &B = occ[b];
    B.lo[0] = lo[0]; B.lo[1] = lo[1]; B.hi[0] = hi[0]; B.hi[1] = hi[1]; B.nmask[0] = nm[0]; B.nmask[1] = nm[1];
    local[b] = c;
  }
}

__global__ void occCounts(const Cnt4 *__restrict__ excl, uint64_t nb, OccBlock *__restrict__ occ) {
  for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x)
    for (int i = 0; i < 4; ++i) occ[b].cnt[i] = excl[b].c[i];
}

// 2-bit text (32 codes per word, LSB-first) + N bitmap (64 per word)
__global__ void packText(const uint8_t *__restrict__ T, uint64_t N, uint64_t *__restrict__ text2, uint64_t *__restrict__ textN,
                         uint64_t nw) {
  for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t v2a = 0, v2b = 0, vn = 0;
    for (int r = 0; r < 64; ++r) {
      uint64_t p = w * 64 + r;
      if (p >= N) break;
      uint8_t c = T[p];
      if (c >= 4) vn |= 1ULL << r;
      else if (r < 32) v2a |= (uint64_t)c << (2 * r);
      else v2b |= (uint64_t)c << (2 * (r - 32));
    }
    text2[2 * w] = v2a;
    text2[2 * w + 1] = v2b;
    textN[w] = vn;
  }
}

// inverse of packText: codes 0..4 from the 2-bit text + N bitmap (a saved index, gwa_index_save)
__global__ void unpackText(const uint64_t *__restrict__ text2, const uint64_t *__restrict__ textN, uint64_t N,
                           uint8_t *__restrict__ T) {
  for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < N; p += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t w = text2[p >> 5];
    const uint8_t c = (uint8_t)((w >> (2 * (p & 31))) & 3);
    T[p] = ((textN[p >> 6] >> (p & 63)) & 1) ? (uint8_t)4 : c;
  }
}

// CharacterCount (A/CharacterCount.java:41-50): occurrences of codes 0..4, one atomic per workgroup
// and code
__global__ void countCodes(const uint8_t *__restrict__ T, uint64_t N, unsigned long long *__restrict__ cnt) {
  __shared__ unsigned long long c[5];
  if (threadIdx.x < 5) c[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long m[5] = {0, 0, 0, 0, 0};
  for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < N; p += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t x = T[p];
    m[x > 4 ? 4 : x]++;
  }
  for (int i = 0; i < 5; ++i) atomicAdd(&c[i], m[i]);
  __syncthreads();
  if (threadIdx.x < 5) atomicAdd(&cnt[threadIdx.x], c[threadIdx.x]);
}

// Cyclic suffix array of d_T[0,N) into d_sa (both device).  alphabetBits 3 for codes 0..4.
// Returns false when the text is periodic (rotations tie).
bool cyclicSAGpu(const uint8_t *d_T, uint64_t N, uint32_t *d_sa, int alphabetBits, hipStream_t s) {
  if (N == 0) return true;
  if (N >= 0xFFFFFFFFull) throw std::runtime_error("text too long for 32-bit suffix array");
  const int K = 63 / alphabetBits;
  uint64_t *k0 = nullptr, *k1 = nullptr;
  uint32_t *v1 = nullptr, *rank = nullptr, *head = nullptr;
  unsigned long long *dup = nullptr;
  void *tmp = nullptr;
  size_t tmpBytes = 0;
  SCHK(hipMalloc(&k0, N * 8));
  SCHK(hipMalloc(&k1, N * 8));
  SCHK(hipMalloc(&v1, N * 4));
  SCHK(hipMalloc(&rank, N * 4));
  SCHK(hipMalloc(&head, N * 4));
  SCHK(hipMalloc(&dup, 8));
  uint32_t *v0 = d_sa;  // values ping-pong with the output buffer
  const unsigned g = gridFor(N);
  const unsigned gg = g > 65536 ? 65536 : g;
  hipLaunchKernelGGL(saInitKeys, dim3(gg), dim3(256), 0, s, d_T, N, K, alphabetBits, k0, v0);
  SCHK(hipGetLastError());
  rocprim::double_buffer<uint64_t> kb(k0, k1);
  rocprim::double_buffer<uint32_t> vb(v0, v1);
  SCHK(rocprim::radix_sort_pairs(nullptr, tmpBytes, kb, vb, (size_t)N, 0, 64, s));
  SCHK(hipMalloc(&tmp, tmpBytes));
  bool ok = true;
  uint64_t h = (uint64_t)K;
  for (int iter = 0;; ++iter) {
    SCHK(rocprim::radix_sort_pairs(tmp, tmpBytes, kb, vb, (size_t)N, 0, iter == 0 ? 63 : 64, s));
    SCHK(hipMemsetAsync(dup, 0, 8, s));
    hipLaunchKernelGGL(saHeads, dim3(gg), dim3(256), 0, s, kb.current(), N, head, dup);
    unsigned long long nd = 0;
    SCHK(hipMemcpyAsync(&nd, dup, 8, hipMemcpyDeviceToHost, s));
    SCHK(hipStreamSynchronize(s));
    if (nd == 0) break;
    if (h >= N) { ok = false; break; }
    // group start via inclusive max-scan of heads
    size_t scanBytes = 0;
    SCHK(rocprim::inclusive_scan(nullptr, scanBytes, head, head, (size_t)N, rocprim::maximum<uint32_t>(), s));
    void *stmp = nullptr;
    SCHK(hipMalloc(&stmp, scanBytes));
    SCHK(rocprim::inclusive_scan(stmp, scanBytes, head, head, (size_t)N, rocprim::maximum<uint32_t>(), s));
    hipLaunchKernelGGL(saScatterRank, dim3(gg), dim3(256), 0, s, head, vb.current(), N, rank);
    hipLaunchKernelGGL(saDoublingKeys, dim3(gg), dim3(256), 0, s, rank, vb.current(), N, h, kb.current());
    SCHK(hipStreamSynchronize(s));
    SCHK(hipFree(stmp));
    h *= 2;
  }
  if (vb.current() != d_sa) SCHK(hipMemcpyAsync(d_sa, vb.current(), N * 4, hipMemcpyDeviceToDevice, s));
  SCHK(hipStreamSynchronize(s));
  (void)hipFree(k0);
  (void)hipFree(k1);
  (void)hipFree(v1);
  (void)hipFree(rank);
  (void)hipFree(head);
  (void)hipFree(dup);
  (void)hipFree(tmp);
  return ok;
}

void reverseTextGpu(const uint8_t *d_T, uint64_t N, uint8_t *d_R, hipStream_t s) {
  const unsigned g = gridFor(N);
  hipLaunchKernelGGL(reverseText, dim3(g > 65536 ? 65536 : g), dim3(256), 0, s, d_T, N, d_R);
  SCHK(hipGetLastError());
}

// Occ blocks of the BWT of d_T under d_sa; fills d_occ[0 .. N/128]
void buildOccGpu(const uint8_t *d_T, const uint32_t *d_sa, uint64_t N, OccBlock *d_occ, hipStream_t s) {
  const uint64_t nb = N / 128 + 1;
  Cnt4 *local = nullptr;
  SCHK(hipMalloc(&local, nb * sizeof(Cnt4)));
  const unsigned g = gridFor(nb);
  hipLaunchKernelGGL(occLocal, dim3(g > 65536 ? 65536 : g), dim3(256), 0, s, d_T, d_sa, N, nb, d_occ, local);
  SCHK(hipGetLastError());
  size_t bytes = 0;
  Cnt4 zero = {{0, 0, 0, 0}};
  SCHK(rocprim::exclusive_scan(nullptr, bytes, local, local, zero, (size_t)nb, Cnt4Plus(), s));
  void *tmp = nullptr;
  SCHK(hipMalloc(&tmp, bytes));
  SCHK(rocprim::exclusive_scan(tmp, bytes, local, local, zero, (size_t)nb, Cnt4Plus(), s));
  hipLaunchKernelGGL(occCounts, dim3(g > 65536 ? 65536 : g), dim3(256), 0, s, local, nb, d_occ);
  SCHK(hipGetLastError());
  SCHK(hipStreamSynchronize(s));
  (void)hipFree(tmp);
  (void)hipFree(local);
}

void unpackTextGpu(const uint64_t *d_text2, const uint64_t *d_textN, uint64_t N, uint8_t *d_T, hipStream_t s) {
  const unsigned g = gridFor(N);
  hipLaunchKernelGGL(unpackText, dim3(g > 65536 ? 65536 : g), dim3(256), 0, s, d_text2, d_textN, N, d_T);
  SCHK(hipGetLastError());
}

void countCodesGpu(const uint8_t *d_T, uint64_t N, unsigned long long *d_cnt5, hipStream_t s) {
  SCHK(hipMemsetAsync(d_cnt5, 0, 5 * sizeof(unsigned long long), s));
  const unsigned g = gridFor(N);
  hipLaunchKernelGGL(countCodes, dim3(g > 4096 ? 4096 : g), dim3(256), 0, s, d_T, N, d_cnt5);
  SCHK(hipGetLastError());
}

void packTextGpu(const uint8_t *d_T, uint64_t N, uint64_t *d_text2, uint64_t *d_textN, hipStream_t s) {
  const uint64_t nw = N / 64 + 1;
  const unsigned g = gridFor(nw);
  hipLaunchKernelGGL(packText, dim3(g > 65536 ? 65536 : g), dim3(256), 0, s, d_T, N, d_text2, d_textN, nw);
  SCHK(hipGetLastError());
}

}  // namespace gwa
