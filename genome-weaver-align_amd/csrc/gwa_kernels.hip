// gwa_kernels.hip -- CDNA4 (gfx950) kernels of the align path.
//
//   fm_quickscan  : one read per lane; N check + FMQuickScan on both strands + exact-hit SA gather
//                   (S/FMQuickScan.java:66-94, S/BidirectionalSuffixFilter.java:281-316).
//                   Reads that need the best-first search are appended to a work list with one
//                   wave-aggregated atomic per wavefront (ballot + mbcnt).
//   bsf_search<R> : one read per lane, persistent grid-stride over the work list; each lane owns a
//                   slice of HBM scratch for its state arena / heap / hits / DP history
//                   (S/BidirectionalSuffixFilter.java:318-477).  R = NFA row capacity >= k+1.
//                   Reads that exceed a capacity tier are appended to an overflow list and rerun
//                   on a larger tier (fewer lanes, bigger slices): no CPU fallback exists.
#include <hip/hip_runtime.h>

#include "bsf_core.h"
#include "kernels.h"

namespace gwa {

__device__ __forceinline__ void waveAppend(bool need, uint32_t value, uint32_t *list, uint32_t *count) {
  const uint64_t mask = __ballot(need);
  if (mask == 0) return;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(mask));
  base = __shfl(base, leader);
  if (need) {
    const uint64_t below = lane == 0 ? 0ULL : (mask & ((~0ULL) >> (64 - lane)));
    list[base + __popcll(below)] = value;
  }
}

__global__ void __launch_bounds__(256) fm_quickscan_kernel(IndexView ix, SearchConfig cfg, ReadsView reads, ScanRes *sres,
                                                           OutHeader *oh, OutHit *ohits, uint16_t *ocig, int hitCap, int cigCap,
                                                           uint32_t *searchList, uint32_t *searchCount, uint32_t *trace,
                                                           int traceRead) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  bool need = false;
  if (r < reads.n) {
    const uint32_t o = reads.off[r];
    const int m = (int)(reads.off[r + 1] - o);
    OutHeader *h = oh + r;
    if (m > 255) {
      h->status = ST_TOO_LONG;
      h->nChains = h->nHits = h->nCigar = 0;
    } else {
      StairTables st{};
      LaneMem<4> L{};
      Caps caps{};
      BsfLane<4> lane(ix, cfg, st, L, caps);
      if (trace && (int)r == traceRead) { lane.trace = trace + 1; lane.traceCap = 65536; }
      lane.initRead(reads.codes + o, m);
      need = lane.quickPhase(sres + r, h, ohits + (size_t)r * hitCap, ocig + (size_t)r * cigCap) != 0;
      if (lane.trace) trace[0] = (uint32_t)lane.traceN;
    }
  }
  waveAppend(need, r, searchList, searchCount);
}

template <int R>
__global__ void __launch_bounds__(256) bsf_search_kernel(IndexView ix, SearchConfig cfg, StairTables st, ReadsView reads,
                                                         const ScanRes *sres, const uint32_t *list, uint32_t n, uint8_t *scratch,
                                                         uint64_t laneStride, Caps caps, OutHeader *oh, OutHit *ohits,
                                                         uint16_t *ocig, int hitCap, int cigCap, const int32_t *chrRank,
                                                         uint32_t *ovfList, uint32_t *ovfCount, uint32_t *trace, int traceRead) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t total = gridDim.x * blockDim.x;
  LaneMem<R> L = laneMem<R>(scratch + (size_t)gid * laneStride, caps);
  // uniform trip count across the wave so the ballot in waveAppend sees every lane
  const uint32_t rounds = (n + total - 1) / total;
  for (uint32_t it = 0; it < rounds; ++it) {
    const uint32_t i = gid + it * total;
    bool ovf = false;
    uint32_t r = 0;
    if (i < n) {
      r = list[i];
      const uint32_t o = reads.off[r];
      const int m = (int)(reads.off[r + 1] - o);
      BsfLane<R> lane(ix, cfg, st, L, caps);
      lane.chrRank = chrRank;
      if (trace && (int)r == traceRead) { lane.trace = trace + 1; lane.traceCap = 65536; }
      lane.initRead(reads.codes + o, m);
      lane.searchPhase(sres[r]);
      lane.writeSearchOutput(oh + r, ohits + (size_t)r * hitCap, ocig + (size_t)r * cigCap, hitCap, cigCap);
      if (lane.trace) trace[0] = (uint32_t)lane.traceN;
      ovf = oh[r].status == ST_OVERFLOW;
    }
    waveAppend(ovf, r, ovfList, ovfCount);
  }
}

void launchQuickscan(const IndexView &ix, const SearchConfig &cfg, const ReadsView &reads, ScanRes *sres, OutHeader *oh,
                     OutHit *ohits, uint16_t *ocig, int hitCap, int cigCap, uint32_t *searchList, uint32_t *searchCount,
                     hipStream_t s, uint32_t *trace, int traceRead) {
  if (reads.n == 0) return;
  dim3 grid((reads.n + 255) / 256);
  hipLaunchKernelGGL(fm_quickscan_kernel, grid, dim3(256), 0, s, ix, cfg, reads, sres, oh, ohits, ocig, hitCap, cigCap,
                     searchList, searchCount, trace, traceRead);
}

void launchSearch(int R, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                  const ReadsView &reads, const ScanRes *sres, const uint32_t *list, uint32_t n, uint8_t *scratch,
                  uint64_t laneStride, const Caps &caps, OutHeader *oh, OutHit *ohits, uint16_t *ocig, int hitCap, int cigCap,
                  const int32_t *chrRank, uint32_t *ovfList, uint32_t *ovfCount, hipStream_t s, uint32_t *trace,
                  int traceRead) {
  if (n == 0) return;
  dim3 grid((lanes + 255) / 256);
  switch (R) {
#define GWA_CASE(RR)                                                                                                  \
  case RR:                                                                                                            \
    hipLaunchKernelGGL(bsf_search_kernel<RR>, grid, dim3(256), 0, s, ix, cfg, st, reads, sres, list, n, scratch,     \
                       laneStride, caps, oh, ohits, ocig, hitCap, cigCap, chrRank, ovfList, ovfCount, trace, traceRead);                \
    break;
    GWA_CASE(4)
    GWA_CASE(8)
    GWA_CASE(16)
    GWA_CASE(32)
#undef GWA_CASE
    default: break;
  }
}

size_t laneBytesFor(int R, const Caps &c) {
  switch (R) {
    case 4: return laneBytes<4>(c);
    case 8: return laneBytes<8>(c);
    case 16: return laneBytes<16>(c);
    default: return laneBytes<32>(c);
  }
}

}  // namespace gwa
