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
//   sf_search<R>  : `-m sf` (S/SuffixFilter.java), one read per lane over all reads: PrefixScan
//                   seeds, the SFState queue and whole-read DP verification (sf_core.h); same
//                   scratch slices and capacity tiers.
#include <hip/hip_runtime.h>

#include "sam_core.h"

#include "search_kernels.h"

namespace gwa {

// Paired-end pair choice and mate rescue (orc_align_pairs rules 1-3, oracle/gwa_oracle.cpp
// orc_align_pairs / peRescue; the build's own design -- the reference has no paired-end path).
// Per pair: the proper pair with the fewest differences (ties: first in mate-1, then mate-2 report
// order) and each mate's first candidate go to out[i]; pairs with more than kPairQuad candidate
// combinations are appended to `heavy` for pair_choose_kernel instead of the all-pairs loop.  For a
// pair whose mates are one with and one without candidates, the mate without is aligned by the
// search's own DP (BsfLane::alignBlockDetailed, full history) inside the window the insert range
// allows next to the anchor; a hit with at most max(k, m / 10) differences is the rescue.
// Persistent lanes over the pairs, 64 per workgroup (the query words of each lane's mate in LDS).
__global__ void __launch_bounds__(64) pair_rescue_kernel(IndexView ix, SearchConfig cfg, StairTables st, ReadsView reads,
                                                         SamText t, const OutHeader *oh, const OutHit *hits,
                                                         const uint16_t *cig, uint32_t np, int32_t minIns, int32_t maxIns,
                                                         uint8_t *scratch, uint64_t laneStride, Caps caps, RescueOut *out,
                                                         int64_t quad, uint32_t *heavy, uint32_t *heavyCount) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t total = gridDim.x * blockDim.x;
  uint8_t *chunk = scratch + (size_t)total * laneStride + (size_t)(gid >> 6) * 64 * ilvBytes(caps);
  const LaneMem<4> L = laneMem<4>(scratch + (size_t)gid * laneStride, chunk, (int)(gid & 63), 64, caps);
  __shared__ uint64_t qwLds[2 * 8 * 64];
  for (uint32_t i = gid; i < np; i += total) {
    RescueOut &R = out[i];
    int status = 0;
    int32_t ca = -1, cb = -1, fa = -1, fb = -1;
    bool isHeavy = false;
    const OutHeader &A = oh[i], &B = oh[np + i];
    if (pairStatusOk(A, B)) {
      const int na = pairCandidates(A, hits, &fa), nb = pairCandidates(B, hits, &fb);
      if ((int64_t)na * nb > quad) {
        isHeavy = true;  // both mates have candidates: no rescue
      } else {
        const PairChoice P = pairChoose(t, i, np, oh, hits, cig, minIns, maxIns);
        ca = P.a ? (int32_t)(P.a - hits) : -1;
        cb = P.b ? (int32_t)(P.b - hits) : -1;
        if (!P.a && ((P.fa != nullptr) != (P.fb != nullptr))) {
          const OutHit &an = P.fa ? *P.fa : *P.fb;
          const uint16_t *anc = P.fa ? P.ca : P.cb;
          const uint32_t r = P.fa ? np + i : i;  // the mate without candidates
          const int m = (int)reads.len[r];
          BsfLane<4, 8> lane(ix, cfg, st, L, caps);
          lane.qwL = (lds_u64 *)(qwLds + threadIdx.x);
          lane.qwS = 64;
          lane.initRead(reads.codes + reads.off[r], m);
          if (m > 256) atomicAdd(heavyCount + 1, 1u);  // rule 3 not tried: mates over 256 bp (gwa.h)
          const int countN = m > 0 && m <= 256 ? lane.buildMasks() : 0x7FFF;
          const int k = lane.k;
          if (m > 0 && m <= 256 && k >= 0 && countN <= k) {  // (QW = 8: mates up to 256 bp are rescued)
            const int kr = k > m / 10 ? k : m / 10;
            const int64_t off = ix.contigOff[an.chr];
            const int64_t clen = (an.chr + 1 < ix.nContig ? ix.contigOff[an.chr + 1] : (int64_t)ix.N) - off;
            const int64_t s0 = off + (int64_t)an.pos - 1;
            int64_t ws, we;
            int strand;
            if (an.strand == 0) {
              strand = 1;
              ws = s0 + minIns - m - kr;
              we = s0 + maxIns + kr;
            } else {
              strand = 0;
              const int64_t e0 = s0 + samRefLen(anc, an) - 1;
              ws = e0 - maxIns + 1 - kr;
              we = e0 - minIns + 1 + m + kr;
            }
            ws = ws > off ? ws : off;
            we = we < off + clen ? we : off + clen;
            if (we - ws > kRescueWindow) atomicAdd(heavyCount + 1, 1u);  // rule 3 not applied (gwa.h)
            if (we - ws >= m && we - ws <= kRescueWindow) {
              int pos = 0, diff = 0, co = 0, cl = 0;
              const int res = lane.alignBlockDetailed(strand, 0, m, ws, we, &pos, &diff, &co, &cl);
              int32_t chr = 0, p = 0;
              if (res == 0 && diff <= kr && cl <= kRescueCig && lane.translate(ws + pos + 1, &chr, &p) == 0) {
                R.hit.chr = chr; R.hit.pos = p; R.hit.matchLength = m; R.hit.qStart = 0; R.hit.qEnd = m;
                R.hit.diff = diff; R.hit.strand = strand; R.hit.numHits = 1; R.hit.next = -1;
                R.hit.cigarOff = 0; R.hit.cigarLen = (uint32_t)cl;
                for (int j = 0; j < cl; ++j) R.cig[j] = lane.L.cigar()[co + j];
                status = P.fa ? 2 : 1;
              }
            }
          }
        }
      }
    }
    R.status = status;
    R.a = ca; R.b = cb; R.fa = fa; R.fb = fb;
    waveAppend(isHeavy, i, heavy, heavyCount);
  }
}

// One workgroup per heavy pair (rules 1-2 over many candidates): the candidates of both mates are
// keyed (mate, contig, strand, anchor) -- anchor = start on the forward strand, end on the reverse --
// and bitonic-sorted in LDS; a sliding-window minimum of (diff, report order) over the opposite
// mate's opposite-strand candidates then gives each candidate its best proper partner in one pass:
// a proper pair has forward start <= reverse end and template length reverse end - forward start + 1
// in [max(minIns, 1), maxIns].  Ties resolve as in the all-pairs loop (report order of mate 1, then
// mate 2).  More than kPairSortCap candidates: the all-pairs loop spread over the workgroup.
__device__ __forceinline__ bool tupleLess(uint32_t t0, int32_t a0, int32_t b0, uint32_t t1, int32_t a1, int32_t b1) {
  return t0 != t1 ? t0 < t1 : a0 != a1 ? a0 < a1 : b0 < b1;
}
__global__ void __launch_bounds__(256) pair_choose_kernel(SamText t, const OutHeader *oh, const OutHit *hits,
                                                          const uint16_t *cig, uint32_t np, int32_t minIns, int32_t maxIns,
                                                          const uint32_t *heavy, int sortCap, RescueOut *out) {
  __shared__ uint64_t key[kPairSortCap], pay[kPairSortCap];
  __shared__ uint16_t dq[kPairSortCap];
  __shared__ uint32_t redT[256];
  __shared__ int32_t redA[256], redB[256];
  __shared__ int cnt[2];
  const uint32_t i = heavy[blockIdx.x];
  const int tid = threadIdx.x;
  const OutHeader *H[2] = {oh + i, oh + np + i};
  const int32_t lo = minIns > 1 ? minIns : 1, hi = maxIns;
  if (tid == 0) {  // the chain walk is sequential (linked fragments)
    int c = 0;
    for (int mate = 0; mate < 2; ++mate) {
      const OutHeader &Hm = *H[mate];
      const OutHit *h = hits + Hm.hitOff;
      const uint16_t *cb = cig + Hm.cigOff;
      const int nc = (int)Hm.nChains;
      int nm = 0;
      for (int x = 0, hx = 0; x < nc; ++x) {
        const OutHit &u = h[hx];
        int e = hx;
        while (h[e].next >= 0) e = h[e].next;
        if (u.next < 0 && u.chr >= 0) {
          if (c < sortCap) {
            const int64_t anchor = u.strand == 0 ? (int64_t)u.pos : (int64_t)u.pos + samRefLen(cb, u) - 1;
            key[c] = ((uint64_t)mate << 63) | ((uint64_t)(uint32_t)t.chrKey[u.chr] << 33) |
                     ((uint64_t)(u.strand & 1) << 32) | (uint64_t)(uint32_t)(anchor < 0 ? 0 : anchor);
            pay[c] = ((uint64_t)(uint32_t)u.diff << 32) | (uint32_t)(Hm.hitOff + hx);
          }
          ++c;
          ++nm;
        }
        hx = e + 1;
      }
      cnt[mate] = nm;
    }
  }
  __syncthreads();
  const int na = cnt[0], nb = cnt[1];
  uint32_t bestT = 0xFFFFFFFFu;
  int32_t bestA = -1, bestB = -1;
  if (na + nb <= sortCap) {
    int P = 2;
    while (P < na + nb) P <<= 1;
    for (int x = na + nb + tid; x < P; x += 256) { key[x] = ~0ULL; pay[x] = ~0ULL; }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int x = tid; x < P; x += 256) {
          const int y = x ^ j;
          if (y > x) {
            const uint64_t kx = key[x], ky = key[y];
            if ((kx > ky) == ((x & k) == 0)) {
              key[x] = ky; key[y] = kx;
              const uint64_t px = pay[x];
              pay[x] = pay[y]; pay[y] = px;
            }
          }
        }
        __syncthreads();
      }
    }
    if (tid == 0 && lo <= hi) {
      const int end = na + nb;
      for (int u = 0; u < na;) {
        const uint64_t g = key[u] >> 32;  // (mate 0, contig, strand)
        int ue = u;
        while (ue < na && (key[ue] >> 32) == g) ++ue;
        const uint64_t gv = (1ULL << 31) | (g ^ 1);  // mate 1, same contig, the other strand
        int vs = na, ve;
        {  // [vs, ve) = mate-2 candidates of group gv
          int l = na, h2 = end;
          while (l < h2) { const int md = (l + h2) >> 1; if ((key[md] >> 32) < gv) l = md + 1; else h2 = md; }
          vs = l;
          h2 = end;
          while (l < h2) { const int md = (l + h2) >> 1; if ((key[md] >> 32) <= gv) l = md + 1; else h2 = md; }
          ve = l;
        }
        const bool fwd = (g & 1) == 0;
        int head = 0, tail = 0, add = vs;
        for (int x = u; x < ue && vs < ve; ++x) {
          const int64_t kx = (int64_t)(key[x] & 0xFFFFFFFFULL);
          const int64_t wl = fwd ? kx + lo - 1 : kx - hi + 1, wh = fwd ? kx + hi - 1 : kx - lo + 1;
          while (add < ve && (int64_t)(key[add] & 0xFFFFFFFFULL) <= wh) {
            while (tail > head && pay[dq[tail - 1]] > pay[add]) --tail;
            dq[tail++] = (uint16_t)add;
            ++add;
          }
          while (head < tail && (int64_t)(key[dq[head]] & 0xFFFFFFFFULL) < wl) ++head;
          if (head < tail) {
            const uint64_t pu = pay[x], pv = pay[dq[head]];
            const uint32_t tt = (uint32_t)(pu >> 32) + (uint32_t)(pv >> 32);
            const int32_t ia = (int32_t)(uint32_t)pu, ib = (int32_t)(uint32_t)pv;
            if (tupleLess(tt, ia, ib, bestT, bestA, bestB)) { bestT = tt; bestA = ia; bestB = ib; }
          }
        }
        u = ue;
      }
    }
  } else {
    // all pairs, mate-1 candidates dealt round-robin over the threads
    const OutHit *ha = hits + H[0]->hitOff, *hb = hits + H[1]->hitOff;
    const uint16_t *ca = cig + H[0]->cigOff, *cb = cig + H[1]->cigOff;
    for (int x = 0, hx = 0, ord = 0; x < (int)H[0]->nChains; ++x) {
      const OutHit &u = ha[hx];
      int e = hx;
      while (ha[e].next >= 0) e = ha[e].next;
      if (u.next < 0 && u.chr >= 0 && (ord++ & 255) == tid) {
        for (int y = 0, hy = 0; y < (int)H[1]->nChains; ++y) {
          const OutHit &v = hb[hy];
          int f = hy;
          while (hb[f].next >= 0) f = hb[f].next;
          if (v.next < 0 && v.chr >= 0) {
            const uint32_t tt = (uint32_t)(u.diff + v.diff);
            const int32_t ia = (int32_t)(H[0]->hitOff + hx), ib = (int32_t)(H[1]->hitOff + hy);
            if (tupleLess(tt, ia, ib, bestT, bestA, bestB) && pairProper(t, u, ca, v, cb, minIns, maxIns)) {
              bestT = tt; bestA = ia; bestB = ib;
            }
          }
          hy = f + 1;
        }
      }
      hx = e + 1;
    }
  }
  redT[tid] = bestT; redA[tid] = bestA; redB[tid] = bestB;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w && tupleLess(redT[tid + w], redA[tid + w], redB[tid + w], redT[tid], redA[tid], redB[tid])) {
      redT[tid] = redT[tid + w]; redA[tid] = redA[tid + w]; redB[tid] = redB[tid + w];
    }
    __syncthreads();
  }
  if (tid == 0) {
    RescueOut &R = out[i];
    const bool found = redT[0] != 0xFFFFFFFFu;
    R.a = found ? redA[0] : -1;
    R.b = found ? redB[0] : -1;
  }
}

void launchPairRescue(uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                      const ReadsView &reads, const SamText &t, const OutHeader *oh, const OutHit *hits,
                      const uint16_t *cig, uint32_t np, int32_t minIns, int32_t maxIns, uint8_t *scratch,
                      uint64_t laneStride, const Caps &caps, RescueOut *out, int64_t quad, uint32_t *heavy,
                      uint32_t *heavyCount, hipStream_t s) {
  if (np == 0) return;
  hipLaunchKernelGGL(pair_rescue_kernel, dim3((lanes + 63) / 64), dim3(64), 0, s, ix, cfg, st, reads, t, oh, hits, cig, np,
                     minIns, maxIns, scratch, laneStride, caps, out, quad, heavy, heavyCount);
}

void launchPairChoose(uint32_t nHeavy, const SamText &t, const OutHeader *oh, const OutHit *hits, const uint16_t *cig,
                      uint32_t np, int32_t minIns, int32_t maxIns, const uint32_t *heavy, int sortCap, RescueOut *out,
                      hipStream_t s) {
  if (nHeavy == 0) return;
  if (sortCap < 0 || sortCap > kPairSortCap) sortCap = kPairSortCap;
  hipLaunchKernelGGL(pair_choose_kernel, dim3(nHeavy), dim3(256), 0, s, t, oh, hits, cig, np, minIns, maxIns, heavy, sortCap,
                     out);
}

// one thread per k-mer (IndexView::kmer)
__global__ void __launch_bounds__(256) kmer_table_kernel(const OccBlock *occ, IndexView ix, int K, uint64_t *out) {
  const uint64_t key = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (key >> (2 * K)) return;
  out[key] = kmerInterval(occ, ix.C, ix.N, (uint32_t)key, K);
}

void buildKmerTable(const IndexView &ix, int fm, int K, uint64_t *out, hipStream_t s) {
  const uint64_t n = 1ULL << (2 * K);
  hipLaunchKernelGGL(kmer_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ix.occ[fm], ix, K, out);
}

// the search instances live in search_inst.hip (one translation unit per (QW, R))
GWA_SEARCH_EXTERN_QW(4)
GWA_SEARCH_EXTERN_QW(8)
GWA_SEARCH_EXTERN_QW(16)

void launchQuickscan(int QW, const IndexView &ix, const SearchConfig &cfg, const ReadsView &reads, ScanRes *sres, OutHeader *oh,
                     const OutSlots &os, uint32_t *searchList, uint32_t *searchCount,
                     hipStream_t s, uint32_t *trace, int traceRead) {
  if (reads.n == 0) return;
  if (QW == 4) launchQuickscanT<4>(ix, cfg, reads, sres, oh, os, searchList, searchCount, s, trace, traceRead);
  else if (QW == 8) launchQuickscanT<8>(ix, cfg, reads, sres, oh, os, searchList, searchCount, s, trace, traceRead);
  else launchQuickscanT<16>(ix, cfg, reads, sres, oh, os, searchList, searchCount, s, trace, traceRead);
}

void launchKeyscan(int QW, const IndexView &ix, const SearchConfig &cfg, const ReadsView &reads, ScanRes *sres,
                   hipStream_t s) {
  if (reads.n == 0) return;
  if (QW == 4) launchKeyscanT<4>(ix, cfg, reads, sres, s);
  else if (QW == 8) launchKeyscanT<8>(ix, cfg, reads, sres, s);
  else launchKeyscanT<16>(ix, cfg, reads, sres, s);
}

void launchSearch(int R, int QW, int ldsHeap, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg,
                  const StairTables &st, const ReadsView &reads, const ScanRes *sres, const uint32_t *list, uint32_t n,
                  uint8_t *scratch, uint64_t laneStride, const Caps &caps, OutHeader *oh, const OutSlots &os,
                  const int32_t *chrRank, uint32_t *work, uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits,
                  const ResumeBufs &res, hipStream_t s, uint32_t *trace, int traceRead) {
  if (n == 0) return;
#define GWA_L(Q, RR)                                                                                                   \
  if (QW == Q && R == RR) {                                                                                            \
    launchSearchQR<Q, RR>(ldsHeap, lanes, ix, cfg, st, reads, sres, list, n, scratch, laneStride, caps, oh, os, chrRank, \
                          work, ovfList, ovfCount, ovfBits, res, s, trace, traceRead);                                 \
    return;                                                                                                            \
  }
#define GWA_LQ(Q) GWA_L(Q, 4) GWA_L(Q, 8) GWA_L(Q, 16) GWA_L(Q, 32)
  GWA_LQ(4) GWA_LQ(8) GWA_LQ(16)
#undef GWA_LQ
#undef GWA_L
}

void launchSfSearch(int R, int QW, bool wrap, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                    const ReadsView &reads, const uint32_t *list, uint32_t n, uint8_t *scratch, uint64_t laneStride,
                    const Caps &caps, OutHeader *oh, const OutSlots &os,
                    const int32_t *chrRank, uint32_t *work, uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits,
                    hipStream_t s, uint32_t *trace) {
  if (n == 0) return;
#define GWA_L(Q, RR)                                                                                                   \
  if (QW == Q && R == RR) {                                                                                            \
    launchSfSearchQR<Q, RR>(wrap, lanes, ix, cfg, st, reads, list, n, scratch, laneStride, caps, oh, os, chrRank, work, \
                            ovfList, ovfCount, ovfBits, s, trace);                                                            \
    return;                                                                                                            \
  }
#define GWA_LQ(Q) GWA_L(Q, 4) GWA_L(Q, 8) GWA_L(Q, 16) GWA_L(Q, 32)
  GWA_LQ(4) GWA_LQ(8) GWA_LQ(16)
#undef GWA_LQ
#undef GWA_L
}

size_t laneBytesFor(int R, const Caps &c) {
  switch (R) {
    case 4: return laneBytes<4>(c);
    case 8: return laneBytes<8>(c);
    case 16: return laneBytes<16>(c);
    default: return laneBytes<32>(c);
  }
}
size_t ilvBytesFor(const Caps &c) { return ilvBytes(c); }
size_t resumeBytesFor(int R, const Caps &c) {
  switch (R) {
    case 4: return BsfLane<4>::resumeBytes(c);
    case 8: return BsfLane<8>::resumeBytes(c);
    case 16: return BsfLane<16>::resumeBytes(c);
    default: return BsfLane<32>::resumeBytes(c);
  }
}

}  // namespace gwa
