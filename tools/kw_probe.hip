#include <hip/hip_runtime.h>
#include "../genome-weaver-align_amd/csrc/bsf_core.h"
using namespace gwa;
template <int V>
__global__ void __launch_bounds__(256) probe(IndexView ix, SearchConfig cfg, StairTables st, ReadsView reads, const ScanRes *sres,
                                             uint8_t *scratch, Caps caps, const int32_t *chrRank, int *out) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  LaneMem<4> L = laneMem<4>(scratch + gid * 4096, scratch, (int)(gid & 63), 64, caps);
  BsfLane<4, 4> lane(ix, cfg, st, L, caps);
  lane.chrRank = chrRank;
  lane.initRead(reads.codes + reads.off[gid], 100);
  int r = 0;
  if (V == 0) { r = lane.searchStart(sres[gid]); }
  if (V == 1) { lane.searchStart(sres[gid]); r = lane.searchStep(); }
  if (V == 2) { lane.searchStart(sres[gid]); r = lane.searchReport(); }
  if (V == 3) { lane.searchStart(sres[gid]); for (int i = 0; i < 100; ++i) r += lane.searchStep(); }
  if (V == 4) { lane.searchStart(sres[gid]); int p = 0, q = 0; r = lane.alignBlockDetailed(0, 0, 100, 1000, 1104, &p, &q, &p, &q); r += p + q; }
  if (V == 5) { lane.searchStart(sres[gid]); r = lane.nextStateLocal(0, lane.S(0), 1); }
  if (V == 6) { lane.searchStart(sres[gid]); uint64_t rows[4]; int a, b; bool h; r = lane.nfaNext(lane.S(0), 1, 0, rows, &a, &b, &h); r += (int)rows[1]; }
  if (V == 7) { lane.searchStart(sres[gid]); DState<4> d; lane.nextSi(lane.S(0), 1, d); r = d.lb[1] + d.ub[2]; }
  if (V == 8) { lane.searchStart(sres[gid]); r = lane.queuePoll(); lane.queueAdd(3); }
  if (V == 9) { lane.searchStart(sres[gid]); r = (int)lane.patternMask64(0, gid & 1, gid & 63, 40, gid & 31, 2, 2); }
  if (V == 10) { lane.searchStart(sres[gid]); r = (int)lane.stairMask(gid & 3, gid & 7); }
  if (V == 11) { lane.searchStart(sres[gid]); r = (int)lane.eqWindow(0, 2, gid & 63); }
  if (V == 12) { lane.searchStart(sres[gid]); r = (int)lane.qword(gid & 1, gid & 7); }
  if (V == 13) { lane.searchStart(sres[gid]); r = lane.queuePoll(); DState<4> d; lane.loadState(r, d); r += d.lb[2] + (int)d.nfa[1]; }
  if (V == 14) { lane.searchStart(sres[gid]); r = lane.chainScore(gid & 7, true); }
  if (V == 15) { lane.searchStart(sres[gid]); r = lane.nextStateAfterSplit(gid & 7, gid & 1); }
  if (V == 16) { lane.searchStart(sres[gid]); r = lane.update(gid & 7, 1, 2); }
  if (V == 17) { lane.searchStart(sres[gid]); lane.refreshKeys(); }
  if (V == 18) { lane.searchStart(sres[gid]); r = lane.verify(gid & 7); }
  if (V == 19) { lane.searchStart(sres[gid]); r = lane.sortSplits(gid & 7); lane.resultAdd(r); }
  if (V == 20) { lane.searchStart(sres[gid]); r = lane.reportAlignment(gid & 7); }
  out[gid] = r + lane.status + lane.nStates;
}
template __global__ void probe<0>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<1>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<2>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<3>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<4>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<5>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<6>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<7>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<8>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<9>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<10>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<11>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<12>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<13>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<14>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<15>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<16>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<17>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<18>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<19>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
template __global__ void probe<20>(IndexView, SearchConfig, StairTables, ReadsView, const ScanRes *, uint8_t *, Caps, const int32_t *, int *);
