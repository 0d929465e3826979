// repro_flag.hip -- an attempt at a small model of the gfx950 flag-form fault: each lane
// runs a best-first search over a synthetic interval tree whose step expands four children in a loop,
// once with an early `return` out of the loop (the product's form) and once with a loop-carried `ok`
// flag (the form that loses reads in the -m sf kernel).  Both forms are the same program, so every
// lane's (children, result) must agree; lanes are made to diverge (different seeds), as in the batch
// where the loss shows.  Tools only.
//   hipcc --offload-arch=gfx950 -O3 -o tools/repro_flag tools/repro_flag.hip && tools/repro_flag
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int R = 8, CAP = 512;
struct St {
  uint32_t lb, ub;
  int idx, score;
  uint64_t nfa[R];
};

struct Lane {
  St *arena;
  int *heap;
  int heapSize, created, children, status, best;
  uint32_t seed;
  const uint32_t *occ;
  uint32_t n;

  __device__ bool stairOk(const St &c, int ch) const { return ((uint32_t)(c.idx * 7 + ch) ^ seed) % 53u != 0u; }
  __device__ void push(int id) {
    int i = heapSize++;
    const int sc = arena[id].score;
    while (i > 0) {  // sift up, break flag form as the kernels had it
      const int p = (i - 1) / 2;
      if (arena[heap[p]].score >= sc) break;
      heap[i] = heap[p];
      i = p;
    }
    heap[i] = id;
    if (heapSize > CAP / 2) status = 2;
  }
  __device__ int pop() {
    const int top = heap[0];
    const int last = heap[--heapSize];
    int i = 0;
    for (;;) {
      int l = 2 * i + 1;
      if (l >= heapSize) break;
      if (l + 1 < heapSize && arena[heap[l + 1]].score > arena[heap[l]].score) ++l;
      if (arena[heap[l]].score <= arena[last].score) break;
      heap[i] = heap[l];
      i = l;
    }
    if (heapSize > 0) heap[i] = last;
    return top;
  }
  __device__ bool child(const St &c, int ch, uint32_t lb, uint32_t ub) {
    if (!stairOk(c, ch)) return false;
    ++children;
    uint64_t rows[R];
    uint64_t eq = (uint64_t)occ[(lb * 4u + (uint32_t)ch) % n] << 32 | occ[(ub + (uint32_t)ch) % n];
    int alive = 0, nk = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t prev = r ? rows[r - 1] : 0ULL;
      rows[r] = ((c.nfa[r] << 1) & eq) | (prev << 1) | (r ? c.nfa[r - 1] : 0ULL);
      if (rows[r]) { ++alive; if (!nk) nk = r + 1; }
    }
    if (!alive) return true;  // filtered
    if (created >= CAP) return false;
    const int id = created++;
    St &s = arena[id];
    s.lb = lb; s.ub = ub; s.idx = c.idx + 1; s.score = c.score + (nk == 1 ? 1 : -3 * (nk - 1));
#pragma unroll
    for (int r = 0; r < R; ++r) s.nfa[r] = rows[r];
    if (s.idx >= 24 || ub - lb == 1) best = max(best, s.score);
    push(id);
    return status != 2;
  }
  template <bool FLAG>
  __device__ int step() {
    if (heapSize == 0 || status) return 0;
    const St c = arena[pop()];
    if (c.idx >= 24 || c.ub - c.lb <= 1 || c.score < best - 6) return 1;
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
      const uint32_t w = c.ub - c.lb;
      lo[ch] = (uint32_t)ch * (w / 4u) + occ[(c.lb * 5u + (uint32_t)ch + seed) % n] % (w / 16u + 1u);
      hi[ch] = lo[ch] + w / 4u - occ[(c.ub * 3u + (uint32_t)ch) % n] % (w / 6u + 1u);
    }
    if (FLAG) {
      int ok = 1;
      for (int ch = 0; ch < 4; ++ch) {
        const uint64_t l = c.lb + lo[ch], u = c.lb + hi[ch];
        if (ok && l < u && !child(c, ch, (uint32_t)l, (uint32_t)u)) ok = 0;
      }
      return ok ? 1 : 0;
    } else {
      for (int ch = 0; ch < 4; ++ch) {
        const uint64_t l = c.lb + lo[ch], u = c.lb + hi[ch];
        if (l < u && !child(c, ch, (uint32_t)l, (uint32_t)u)) return 0;
      }
      return 1;
    }
  }
};

template <bool FLAG>
__global__ void __launch_bounds__(256) search(const uint32_t *occ, uint32_t n, St *arenas, int *heaps, int *out, int lanes) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= lanes) return;
  Lane L;
  L.arena = arenas + (size_t)g * CAP;
  L.heap = heaps + (size_t)g * CAP;
  L.heapSize = 0; L.created = 1; L.children = 0; L.status = 0; L.best = -1000;
  L.seed = (uint32_t)g * 2654435761u;
  L.occ = occ; L.n = n;
  St &root = L.arena[0];
  root.lb = 0; root.ub = 1u << 20; root.idx = 0; root.score = 0;
  for (int r = 0; r < R; ++r) root.nfa[r] = ~0ULL >> r;
  L.push(0);
  while (L.template step<FLAG>()) {}
  out[3 * g] = L.children;
  out[3 * g + 1] = L.best;
  out[3 * g + 2] = L.status;
}

int main() {
  const int lanes = 64 * 1024;
  const uint32_t n = 1u << 20;
  std::vector<uint32_t> occ(n);
  uint64_t x = 88172645463325252ull;
  for (auto &v : occ) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)x; }
  uint32_t *dOcc; St *dA; int *dH, *dOut[2];
  if (hipMalloc(&dOcc, n * 4) || hipMalloc(&dA, (size_t)lanes * CAP * sizeof(St)) ||
      hipMalloc(&dH, (size_t)lanes * CAP * 4) || hipMalloc(&dOut[0], lanes * 12) || hipMalloc(&dOut[1], lanes * 12))
    return 2;
  if (hipMemcpy(dOcc, occ.data(), n * 4, hipMemcpyHostToDevice)) return 2;
  hipLaunchKernelGGL(search<false>, dim3(lanes / 256), dim3(256), 0, 0, dOcc, n, dA, dH, dOut[0], lanes);
  hipLaunchKernelGGL(search<true>, dim3(lanes / 256), dim3(256), 0, 0, dOcc, n, dA, dH, dOut[1], lanes);
  if (hipDeviceSynchronize()) return 3;
  std::vector<int> a(3 * lanes), b(3 * lanes);
  if (hipMemcpy(a.data(), dOut[0], lanes * 12, hipMemcpyDeviceToHost) ||
      hipMemcpy(b.data(), dOut[1], lanes * 12, hipMemcpyDeviceToHost))
    return 3;
  long diff = 0, ch = 0;
  for (int i = 0; i < lanes; ++i) {
    ch += a[3 * i];
    if (a[3 * i] != b[3 * i] || a[3 * i + 1] != b[3 * i + 1] || a[3 * i + 2] != b[3 * i + 2]) {
      if (diff < 5) printf("lane %d: return form (%d, %d, %d), flag form (%d, %d, %d)\n", i, a[3 * i], a[3 * i + 1],
                           a[3 * i + 2], b[3 * i], b[3 * i + 1], b[3 * i + 2]);
      ++diff;
    }
  }
  printf("{\"lanes\": %d, \"children_return_form\": %ld, \"lanes_differing\": %ld}\n", lanes, ch, diff);
  return 0;
}
