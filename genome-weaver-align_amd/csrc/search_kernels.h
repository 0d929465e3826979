// search_kernels.h -- the per-read search kernels of the align path, as templates instantiated by
// search_inst.hip once per (query words QW = 4, 8, 16: reads <= 128, 256, 512 bp; NFA rows R), each
// pair in its own translation unit; gwa_kernels.hip dispatches to them.
#pragma once
#include <hip/hip_runtime.h>

#include "bsf_core.h"
#include "sf_core.h"
#include "kernels.h"

namespace gwa {


// appends value to list (one atomic per wavefront); returns the lane's position (needing lanes)
__device__ __forceinline__ uint32_t waveAppend(bool need, uint32_t value, uint32_t *list, uint32_t *count) {
  const uint64_t mask = __ballot(need);
  if (mask == 0) return 0;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(mask));
  base = __shfl(base, leader);
  const uint64_t below = lane == 0 ? 0ULL : (mask & ((~0ULL) >> (64 - lane)));
  const uint32_t pos = base + (uint32_t)__popcll(below);
  if (need) list[pos] = value;
  return pos;
}

template <int QW>
__global__ void __launch_bounds__(256) fm_quickscan_kernel(IndexView ix, SearchConfig cfg, ReadsView reads, ScanRes *sres,
                                                           OutHeader *oh, OutSlots os,
                                                           uint32_t *searchList, uint32_t *searchCount,
                                                           uint32_t *trace, int traceRead) {
  // lane r scans read r
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  bool need = false;
  if (r < reads.n) {
    const uint32_t o = reads.off[r];
    const int m = (int)reads.len[r];
    OutHeader *h = oh + r;
    if (m > 32 * QW) {
      *h = OutHeader{};
      h->status = ST_TOO_LONG;
    } else {
      StairTables st{};
      LaneMem<4> L{};
      Caps caps{};
      BsfLane<4, QW> lane(ix, cfg, st, L, caps);
      if (trace && (int)r == traceRead) { lane.trace = trace + 1; lane.traceCap = 65536; }
      lane.initRead(reads.codes + o, m);
      need = lane.quickPhase(sres + r, h, os, r) != 0;
      if (lane.trace) trace[0] = (uint32_t)lane.traceN;
    }
  }
  waveAppend(need, r, searchList, searchCount);
}

// -m sf: the quick scan's per-strand result of every read, for the search-list key only (no output is
// written: the SuffixFilter search decides every read).  Reads too long or with more N than k keep a
// key of zeros.
template <int QW>
__global__ void __launch_bounds__(256) fm_keyscan_kernel(IndexView ix, SearchConfig cfg, ReadsView reads, ScanRes *sres) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= reads.n) return;
  ScanRes q{};
  const int m = (int)reads.len[r];
  if (m <= 32 * QW) {
    StairTables st{};
    LaneMem<4> L{};
    Caps caps{};
    BsfLane<4, QW> lane(ix, cfg, st, L, caps);
    lane.initRead(reads.codes + reads.off[r], m);
    if (lane.loadWords(lane.pw0, lane.pw1) <= lane.k) {
      const auto sF = lane.quickScan(0);
      const auto sR = lane.quickScan(1);
      q.nmF = sF.numMismatches; q.lmF = sF.lmStart; q.feF = sF.firstEmpty;
      q.nmR = sR.numMismatches; q.lmR = sR.lmStart; q.feR = sR.firstEmpty;
    }
  }
  sres[r] = q;
}

#ifndef GWA_SEARCH_WAVES
#define GWA_SEARCH_WAVES 2
#endif
// RES: 0 = the first tier (no suspension, no resume: BsfLane DPM 1), 1 = suspends and resumes reads
// from records, 2 = suspends only (a tier whose input has no records: the second, after a first tier
// that does not suspend).  The suspend / resume paths' register pressure is kept out of the kernels
// that run most reads (C4 first tier 172 -> 107 ms without them).
template <int R, int QW, int LH, int RES>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GWA_SEARCH_WAVES))) bsf_search_kernel(IndexView ix, SearchConfig cfg, StairTables st, ReadsView reads,
                                                         const ScanRes *sres, const uint32_t *list, uint32_t n, uint8_t *scratch,
                                                         uint64_t laneStride, Caps caps, OutHeader *oh, OutSlots os,
                                                         const int32_t *chrRank,
                                                         uint32_t *work, uint32_t *ovfList, uint32_t *ovfCount,
                                                         uint32_t *ovfBits, ResumeBufs res, uint32_t *trace, int traceRead) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t total = gridDim.x * blockDim.x;
  // scratch = [active lanes][laneStride] slices, then [lanes / 64][64-lane interleaved DP block]; a
  // sparse tier (caps.sparse = s > 1: every s-th lane takes reads) has total / s active lanes
  const uint32_t sp = caps.sparse > 1 ? (uint32_t)caps.sparse : 1u;
  const uint32_t act = (gid >> 6) * (64u / sp) + (gid & 63) / sp;
  uint8_t *chunk = scratch + (size_t)(total / sp) * laneStride + (size_t)(gid >> 6) * 64 * ilvBytes(caps);
  LaneMem<R> L = laneMem<R>(scratch + (size_t)act * laneStride, chunk, (int)(gid & 63), 64, caps);
  // first tier: the priority queue lives in LDS, entry i of thread t at heapLds[i * 256 + t]
  // (heap high-water marks are ~5 entries for k <= 2, 100 bp; larger heaps overflow to tier 1)
  // LH 2: a sparse deep tier (caps.sparse >= 8, a few long searches, one workgroup per CU): each
  // active lane holds the top kDeepLdsHeap * sparse / 256 entries of its queue in LDS, contiguous,
  // and the rest in its slice -- the sift of a queue of thousands of states then waits on HBM for
  // its lowest levels only
  __shared__ uint64_t heapLds[LH == 2 ? kDeepLdsHeap : LH ? kLdsHeap * 256 : 1];
  if (LH == 1) {
    L.heapP = heapLds + threadIdx.x;
    L.hs = 256;
    L.heapL = heapLds + threadIdx.x;  // hybrid heap (k >= 4): LDS for the top slots, the slice beyond
    L.heapH = kLdsHeap;
  } else if (LH == 2) {
    const int per = kDeepLdsHeap / 256 * caps.sparse;
    L.heapL = heapLds + (threadIdx.x / caps.sparse) * per;
    L.hsL = 1;
    L.heapH = per;
  }
#ifdef GWA_PROF
  // profiling build: `trace` is a [lanes][PR_N] cycle-counter array, slot PR_N-1 = wave lifetime
  uint64_t *prof = (uint64_t *)trace + (size_t)gid * PR_N;
  const uint64_t tk = clock64();
  trace = nullptr;
#endif
  __shared__ uint64_t stairLds[kStairLdsWords];
  if (st.ldsM >= 0) {
    for (uint32_t i = threadIdx.x; i < st.ldsCount; i += blockDim.x) stairLds[i] = st.tab[st.ldsBase + i];
    __syncthreads();
  }
  // hybrid heap: k >= 4 with the LDS heap, sparse tiers; the first tier's kernel (LH 1 without resume)
  // keeps the DP slice (BsfLane DPM)
  typedef BsfLane<R, QW, (LH == 2 || (LH != 0 && R >= 8)), 24, RES == 0 ? 1 : 0> Lane;
  Lane lane(ix, cfg, st, L, caps);
#ifdef GWA_PROF
  lane.profG = prof;
#endif
  lane.chrRank = chrRank;
  if (st.ldsM >= 0) lane.stairLds = (lds_cu64 *)stairLds;
  __shared__ uint64_t qwLds[2 * QW * 256];  // the lanes' 2-bit read words (BsfLane::qword)
  lane.qwL = (lds_u64 *)(qwLds + threadIdx.x);
  lane.qwS = 256;
  // the lanes' QueryMask rows (BsfLane::pmL), m <= 128 only (LDS budget: 2 workgroups per CU)
  __shared__ uint64_t pmLds[QW == 4 ? 2 * 4 * (QW / 2) * 256 : 1];
  if (QW == 4) {
    lane.pmL = (lds_u64 *)(pmLds + threadIdx.x);
    lane.pmS = 256;
  }
  // Persistent lanes with a shared read counter.  A lane whose search reaches a report parks (WAIT);
  // the wavefront runs the parked reports (DP verification + traceback) together once they are at
  // least half of its live lanes, instead of once per lane on a divergent path.
  enum { IDLE, RUN, WAIT, FINISH, EXHAUSTED, SUSPEND, RESUME };
  uint32_t resIdx = 0;
  int phase = IDLE;
  uint32_t r = 0;
  // deep tiers with few reads (caps.sparse > 1): only every caps.sparse-th lane takes reads, so the
  // long searches of a tier spread over more wavefronts instead of diverging inside few
  if (caps.sparse > 1 && ((gid & 63) % (uint32_t)caps.sparse) != 0) phase = EXHAUSTED;
  for (;;) {
    const bool need = phase == IDLE;
    const uint64_t needMask = __ballot(need);
    // (cfg.refillMin > 1: the idle lanes wait until that many are idle or every live lane is)
    if (needMask && (cfg.refillMin <= 1 || __popcll(needMask) >= cfg.refillMin ||
                     needMask == __ballot(phase != EXHAUSTED))) {
      const int lid = __lane_id();
      const int leader = __ffsll((long long)needMask) - 1;
      uint32_t base = 0;
      if (lid == leader) base = atomicAdd(work, (uint32_t)__popcll(needMask));
      base = __shfl(base, leader);
      if (need) {
        const uint64_t below = lid == 0 ? 0ULL : (needMask & ((~0ULL) >> (64 - lid)));
        const uint32_t i = base + (uint32_t)__popcll(below);
        if (i < n) {
          r = list[i];
          const uint32_t o = reads.off[r];
          const int m = (int)reads.len[r];
          lane.trace = nullptr;
          if (trace && (int)r == traceRead) { lane.trace = trace + 1; lane.traceCap = 65536; lane.traceN = 0; }
          lane.initRead(reads.codes + o, m);
          // a read the previous tier suspended continues from its record (Lane::resumeFrom, below)
          lane.buildMasks();
          const bool rec = RES == 1 && res.in && i < res.inCap && lane.resumeValid(res.in + (size_t)i * res.inStride, r);
          if (rec) {
            resIdx = i;
            phase = RESUME;
          } else {
            phase = lane.searchStart(sres[r], false) ? RUN : FINISH;
          }
        } else {
          phase = EXHAUSTED;
        }
      }
    }
    if (__ballot(phase != EXHAUSTED) == 0) break;
    if (RES == 1 && phase == RESUME) {
      int rp = 0;
      lane.resumeFrom(res.in + (size_t)resIdx * res.inStride, r, &rp, false);
      phase = rp == Lane::LP_WAIT ? WAIT : RUN;
    }
    const int nWait = __popcll(__ballot(phase == WAIT));
    const int nRun = __popcll(__ballot(phase == RUN));
#ifdef GWA_PROF
    if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) lane.prof[PR_NWAIT] += (uint64_t)nWait;
#endif
    if (nWait > 0 && nWait * 16 >= cfg.waitQ16 * (nWait + nRun)) {
#ifdef GWA_PROF
      const uint64_t trp = clock64();
#endif
      if (phase == WAIT) {
        const int lp = lane.laneReport();
        phase = lp == Lane::LP_RUN ? RUN : lp == Lane::LP_SUSPEND ? SUSPEND : FINISH;
      }
#ifdef GWA_PROF
      if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) lane.prof[PR_REPORT] += clock64() - trp;
#endif
    } else if (phase == RUN) {
      const int lp = lane.laneStep();
      phase = lp == Lane::LP_WAIT ? WAIT : lp == Lane::LP_FINISH ? FINISH : lp == Lane::LP_SUSPEND ? SUSPEND : RUN;
    }
    bool ovf = false;
    if (phase == FINISH) {
      lane.writeSearchOutput(oh + r, os, r);
      if (lane.trace) trace[0] = (uint32_t)lane.traceN;
      ovf = oh[r].status == ST_OVERFLOW;
      if (ovf) atomicOr(ovfBits, (uint32_t)oh[r].ovfWhat);
    } else if (phase == SUSPEND) {  // the next tier resumes it from its record
      lane.status = ST_OVERFLOW;
      lane.writeSearchOutput(oh + r, os, r);
      atomicOr(ovfBits, (uint32_t)lane.ovfWhat);
      ovf = true;
    }
    const uint32_t pos = waveAppend(ovf, r, ovfList, ovfCount);
    if (ovf && res.out && pos < res.outCap) {
      uint8_t *rec = res.out + (size_t)pos * res.outStride;
      if (phase == SUSPEND) lane.suspendTo(rec, r);
      else Lane::resumeInvalidate(rec);
    }
    if (phase == FINISH || phase == SUSPEND) phase = IDLE;
  }
#ifdef GWA_PROF
  for (int q = 0; q < PR_N - 1; ++q) prof[q] += lane.prof[q];
  if (__lane_id() == 0) prof[PR_N - 1] += clock64() - tk;
#endif
}

// sf_search<R, QW>: persistent lanes over the read list, one read per lane per iteration (lanes take
// reads from a shared counter, one atomic per wavefront); overflowing reads go to the next tier.
// COOP (the sparse last tier, caps.sparse = 64): one read per wavefront, lane 0 searching and
// deferring its verifications, lanes 1-63 running them in passes of up to 63 (SfLane: deferred
// verification, roll-back when a result would lower minMismatches); its queue top in LDS,
// whole-column DP history (a lone traceback of tens of edits would recompute a column per edit), one
// wave per SIMD (the few wavefronts need no occupancy).
template <int R, int QW, bool WRAP, bool COOP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(COOP ? 1 : GWA_SEARCH_WAVES)))
sf_search_kernel(IndexView ix, SearchConfig cfg, StairTables st, ReadsView reads, const uint32_t *list, uint32_t n,
                 uint8_t *scratch, uint64_t laneStride, Caps caps, OutHeader *oh, OutSlots os,
                 const int32_t *chrRank, uint32_t *work, uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits,
                 uint32_t *trace) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t total = gridDim.x * blockDim.x;
  // scratch = [active lanes][laneStride] slices, then [lanes / 64][64-lane interleaved DP block]; a
  // sparse tier (caps.sparse = s > 1: every s-th lane takes reads) has total / s active lanes
  const uint32_t sp = caps.sparse > 1 ? (uint32_t)caps.sparse : 1u;
  const uint32_t act = (gid >> 6) * (64u / sp) + (gid & 63) / sp;
  uint8_t *chunk = scratch + (size_t)(total / sp) * laneStride + (size_t)(gid >> 6) * 64 * ilvBytes(caps);
  LaneMem<R> L = laneMem<R>(scratch + (size_t)act * laneStride, chunk, (int)(gid & 63), 64, caps);
  __shared__ uint64_t stairLds[kStairLdsWords];
  if (st.ldsM >= 0) {
    for (uint32_t i = threadIdx.x; i < st.ldsCount; i += blockDim.x) stairLds[i] = st.tab[st.ldsBase + i];
    __syncthreads();
  }
  __shared__ uint64_t qwLds[2 * QW * 256];
  // COOP: each wavefront's (one read's) queue entries [0, kSfLdsHeap) in LDS
  __shared__ uint64_t sfHeapLds[COOP ? 4 * kSfLdsHeap : 1];
  if (COOP) {
    L.heapL = sfHeapLds + (threadIdx.x >> 6) * kSfLdsHeap;
    L.hsL = 1;
    L.heapH = kSfLdsHeap;
  }
  SfLane<R, QW, WRAP, COOP ? 2 : 0> lane(ix, cfg, st, L, caps);
  lane.chrRank = chrRank;
#ifdef GWA_PROF
  // profiling build: the same [lanes][PR_N] slots as bsf_search_kernel (regions: SfLane::sfStep)
  uint64_t *prof = (uint64_t *)trace + (size_t)gid * PR_N;
  const uint64_t tk = clock64();
  lane.profG = prof;
#else
  (void)trace;
#endif
  if (st.ldsM >= 0) lane.stairLds = (lds_cu64 *)stairLds;
  lane.qwL = (lds_u64 *)(qwLds + threadIdx.x);
  lane.qwS = 256;
  __shared__ uint64_t pmLds[QW == 4 ? 2 * 4 * (QW / 2) * 256 : 1];
  if (QW == 4) {
    lane.pmL = (lds_u64 *)(pmLds + threadIdx.x);
    lane.pmS = 256;
  }
  if constexpr (COOP) {
    const int lid = (int)(gid & 63);
    // a helper's CIGAR area: its share of the wavefront's (otherwise unused) path plane
    const int hcap = caps.path / 2;
    uint16_t *hcg = (uint16_t *)(chunk + L.oPath) + (size_t)lid * hcap;
    for (;;) {
      uint32_t i = 0;
      if (lid == 0) i = atomicAdd(work, 1u);
      i = __shfl(i, 0);
      if (i >= n) break;
      const uint32_t r = list[i];
      const int m = (int)reads.len[r];
      OutHeader *h = oh + r;
      bool ovf = false;
      if (m > 32 * QW) {
        if (lid == 0) {
          OutHeader z{};
          z.status = ST_TOO_LONG;
          *h = z;
        }
      } else {
        lane.initRead(reads.codes + reads.off[r], m);
        lane.coopClear(lid);
        __threadfence_block();
        int run = 0;
        if (lid == 0) run = lane.sfBegin(false) ? 1 : 0;
        else lane.buildMasks();  // (the helpers' DPs read the query words from their LDS rows)
        decltype(lane) snap = lane;  // lane 0: its registers where the current deferral began
        for (;;) {
          int need = 0;
          if (lid == 0 && run) {
            int stp = 1;
            while (stp == 1 || stp == 3) {
              stp = lane.template sfStepT<true>();
              if (stp == 3) {
                laneCopy(snap, lane);
                lane.dMode = 1;
                lane.uOn = 1;
                stp = 1;
              }
            }
            need = stp == 2 ? 1 : 0;
            run = need;
          }
          need = __shfl(need, 0);
          if (!need) break;
          __threadfence_block();
          // the pass: lane j (1..63) runs queued job j - 1 into the result table
          const int qn = __shfl(lane.dN, 0);
#ifdef GWA_PROF
          const uint64_t tpass = clock64();
          if (lid == 0) prof[PR_NVW] += 1;
#endif
          if (lid != 0 && lane.djobLoad(lid - 1, qn)) {
#ifdef GWA_PROF
            prof[PR_NVL] += 1;
#endif
            int pos = 0, diff = 0, co = 0, cl = 0;
            lane.nCigar = 0;
            lane.status = ST_UNMAPPED;
            const int rr = lane.alignBlockDetailed(lane.jStrand, 0, m, lane.jRefStart, lane.jRefEnd, &pos, &diff, &co, &cl,
                                                   hcg, hcap);
            lane.specPut(rr, pos, diff, co, cl, hcg);
          }
          __threadfence_block();
#ifdef GWA_PROF
          if (lid == 0) prof[PR_REPORT] += clock64() - tpass;
#endif
          if (lid == 0) {
            bool go = true;
            if (lane.dCommit(&go) >= 0) {  // a result lowers minMismatches: back to the deferral's start
#ifdef GWA_PROF
              prof[PR_NBW] += 1;
#endif
              lane.undoApply();
              laneCopy(lane, snap);
              lane.dN = 0;
              go = lane.candFinish();  // (its job: the first deferred one, now in the table)
            }
            run = go ? 1 : 0;
          }
        }
        if (lid == 0) {
          lane.writeSearchOutput(h, os, r);
          h->states = lane.created;
          h->quickSteps = lane.quickSteps;
          h->blocks = 0;
          h->kmerLookups = lane.kmerLookups;
          h->quickShort = lane.shortSteps;
          h->quickSa = 0;
          h->quickText = 0;
          ovf = h->status == ST_OVERFLOW;
          if (ovf) atomicOr(ovfBits, (uint32_t)h->ovfWhat);
        }
      }
      waveAppend(ovf, r, ovfList, ovfCount);
    }
#ifdef GWA_PROF
    for (int q = 0; q < PR_N - 1; ++q) prof[q] += lane.prof[q];
    if (__lane_id() == 0) prof[PR_N - 1] += clock64() - tk;
#endif
    return;
  }
  // the grown last tier (few reads, long searches): every caps.sparse-th lane only, so the searches
  // run on separate wavefronts instead of serialising inside one (bsf_search_kernel's sparse tiers)
  if (caps.sparse > 1 && ((gid & 63) % (uint32_t)caps.sparse) != 0) return;
  for (;;) {
    const uint64_t act = __ballot(1);
    const int lid = __lane_id();
    const int leader = __ffsll((long long)act) - 1;
    uint32_t base = 0;
    if (lid == leader) base = atomicAdd(work, (uint32_t)__popcll(act));
    base = __shfl(base, leader);
    const uint32_t i = base + (uint32_t)__popcll(act & ((1ULL << lid) - 1ULL));
    if (i >= n) break;
    const uint32_t r = list[i];
    const int m = (int)reads.len[r];
    OutHeader *h = oh + r;
    bool ovf = false;
    if (m > 32 * QW) {
      OutHeader z{};
      z.status = ST_TOO_LONG;
      *h = z;
    } else {
      lane.initRead(reads.codes + reads.off[r], m);
      lane.sfSearch();
      lane.writeSearchOutput(h, os, r);
      h->states = lane.created;  // (nStates is the arena's high-water mark: slots are recycled)
      h->quickSteps = lane.quickSteps;
      h->blocks = 0;  // (all Occ blocks are in searchBlocks on this path)
      h->kmerLookups = lane.kmerLookups;
      h->quickShort = lane.shortSteps;
      h->quickSa = 0;
      h->quickText = 0;
      ovf = h->status == ST_OVERFLOW;
      if (ovf) atomicOr(ovfBits, (uint32_t)h->ovfWhat);
    }
    waveAppend(ovf, r, ovfList, ovfCount);
  }
#ifdef GWA_PROF
  for (int q = 0; q < PR_N - 1; ++q) prof[q] += lane.prof[q];
  if (__lane_id() == 0) prof[PR_N - 1] += clock64() - tk;
#endif
}


template <int QW>
void launchKeyscanT(const IndexView &ix, const SearchConfig &cfg, const ReadsView &reads, ScanRes *sres, hipStream_t s) {
  hipLaunchKernelGGL(fm_keyscan_kernel<QW>, dim3((reads.n + 255) / 256), dim3(256), 0, s, ix, cfg, reads, sres);
}

template <int QW>
void launchQuickscanT(const IndexView &ix, const SearchConfig &cfg, const ReadsView &reads, ScanRes *sres, OutHeader *oh,
                      const OutSlots &os, uint32_t *searchList, uint32_t *searchCount, hipStream_t s, uint32_t *trace,
                      int traceRead) {
  hipLaunchKernelGGL(fm_quickscan_kernel<QW>, dim3((reads.n + 255) / 256), dim3(256), 0, s, ix, cfg, reads, sres, oh, os,
                     searchList, searchCount, trace, traceRead);
}

// one (QW, R) instance set per translation unit (search_inst.hip, built once per pair by the
// Makefile): the bsf_search kernels of the three heap kinds and the sf_search kernels
template <int QW, int R>
void launchSearchQR(int ldsHeap, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                    const ReadsView &reads, const ScanRes *sres, const uint32_t *list, uint32_t n, uint8_t *scratch,
                    uint64_t laneStride, const Caps &caps, OutHeader *oh, const OutSlots &os, const int32_t *chrRank,
                    uint32_t *work, uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits, const ResumeBufs &res,
                    hipStream_t s, uint32_t *trace, int traceRead) {
  dim3 grid((lanes + 255) / 256);
#define GWA_CASE(LL, RR)                                                                                               \
  hipLaunchKernelGGL((bsf_search_kernel<R, QW, LL, RR>), grid, dim3(256), 0, s, ix, cfg, st, reads, sres, list, n,     \
                     scratch, laneStride, caps, oh, os, chrRank, work, ovfList, ovfCount, ovfBits, res, trace, traceRead)
  if (ldsHeap == 2) GWA_CASE(2, 1);
  else if (ldsHeap && caps.dpSlice) GWA_CASE(1, 0);  // the first tier
  else if (ldsHeap && res.in) GWA_CASE(1, 1);
  else if (ldsHeap) GWA_CASE(1, 2);
  else GWA_CASE(0, 1);
#undef GWA_CASE
}

// wrap: the batch has reads whose prefix-scan chunks wrap (sfChunksWrap: some lengths of 129-256 bp,
// and reads of <= 31 bp at a large k); QW = 16 reads are always run with the WRAP path
template <int QW, int R>
void launchSfSearchQR(bool wrap, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                      const ReadsView &reads, const uint32_t *list, uint32_t n, uint8_t *scratch, uint64_t laneStride,
                      const Caps &caps, OutHeader *oh, const OutSlots &os, const int32_t *chrRank, uint32_t *work,
                      uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits, hipStream_t s, uint32_t *trace) {
  dim3 grid((lanes + 255) / 256);
  // the cooperative kernel for the sparse last tier (one read per wavefront, caps.spec > 0)
  const bool coop = caps.sparse == 64 && caps.spec > 0;
#define GWA_SF(WW, CC)                                                                                                 \
  hipLaunchKernelGGL((sf_search_kernel<R, QW, WW, CC>), grid, dim3(256), 0, s, ix, cfg, st, reads, list, n, scratch,  \
                     laneStride, caps, oh, os, chrRank, work, ovfList, ovfCount, ovfBits, trace)
  if (wrap || QW == 16) {
    if (coop) GWA_SF(true, true);
    else GWA_SF(true, false);
  } else if (QW != 16) {
    if (coop) GWA_SF(QW == 16, true);
    else GWA_SF(QW == 16, false);
  }
#undef GWA_SF
}

// explicit instantiation (search_inst.hip: `template`) or declaration (`extern template`) of one
// (QW, R) instance set
#define GWA_SEARCH_INSTANCE(KW, QW_, R_)                                                                           \
  KW void launchSearchQR<QW_, R_>(int, uint32_t, const IndexView &, const SearchConfig &, const StairTables &,     \
                                  const ReadsView &, const ScanRes *, const uint32_t *, uint32_t, uint8_t *, uint64_t, \
                                  const Caps &, OutHeader *, const OutSlots &, const int32_t *, uint32_t *,        \
                                  uint32_t *, uint32_t *, uint32_t *, const ResumeBufs &, hipStream_t, uint32_t *, \
                                  int);                                                                            \
  KW void launchSfSearchQR<QW_, R_>(bool, uint32_t, const IndexView &, const SearchConfig &, const StairTables &,  \
                                    const ReadsView &, const uint32_t *, uint32_t, uint8_t *, uint64_t,           \
                                    const Caps &, OutHeader *, const OutSlots &, const int32_t *, uint32_t *,      \
                                    uint32_t *, uint32_t *, uint32_t *, hipStream_t, uint32_t *);
#define GWA_SEARCH_EXTERN_QW(QW_)                                                                                  \
  GWA_SEARCH_INSTANCE(extern template, QW_, 4)                                                                    \
  GWA_SEARCH_INSTANCE(extern template, QW_, 8)                                                                    \
  GWA_SEARCH_INSTANCE(extern template, QW_, 16)                                                                   \
  GWA_SEARCH_INSTANCE(extern template, QW_, 32)                                                                   \
  extern template void launchKeyscanT<QW_>(const IndexView &, const SearchConfig &, const ReadsView &, ScanRes *,     \
                                           hipStream_t);                                                             \
  extern template void launchQuickscanT<QW_>(const IndexView &, const SearchConfig &, const ReadsView &, ScanRes *, \
                                             OutHeader *, const OutSlots &, uint32_t *, uint32_t *, hipStream_t,   \
                                             uint32_t *, int);

}  // namespace gwa
