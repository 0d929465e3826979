// sf_core.h -- per-lane SuffixFilter search (`align -m sf`, S/SuffixFilter.java), MI355X device code.
//
// One read per lane, as the BSF path (bsf_core.h), whose primitives it reuses: the 2-bit read
// words in LDS, the Occ-block rank, the k-mer interval tables, single-row text mode, the
// staircase tables, the NFA step, the keyed java.util.PriorityQueue, Myers DP verification and the
// hit list.  The operation order is the reference's:
//   PrefixScan.scanRead per strand (S/PrefixScan.java:66-92), initQueue (S/SuffixFilter.java:144-158),
//   the queue loop of align_internal (:229-292), addCandidate (:298-343), reportResult (:345-353),
//   AlignmentResultHolder.add (:369-389); the report selection of align (:165-222) is
//   BsfLane::writeSearchOutput (the same code in the reference).
#pragma once
#include "bsf_core.h"

namespace gwa {

// SFState (S/SuffixFilter.java:414-471).  si: rows [lb, ub) of the forward-extension index
// (FMIndexOnGenome.forwardSearch, A/FMIndexOnGenome.java:138-141,203-209); with M_TEXT in meta the
// interval is one row and lb holds that row's suffix-array value instead (prefix scan in text mode).
template <int R>
struct SfState {
  uint32_t lb, ub;
  int32_t score;
  int16_t offset, index;  // read positions (reads up to 512 bp; negative after a wrapped (byte) chunk start)
  uint8_t strand, nrows, kOffset, hasHit;
  uint8_t meta, pad[3];
  uint64_t nfa[R];
};
static_assert(sizeof(SfState<4>) == 24 + 8 * 4 && sizeof(SfState<8>) == 24 + 8 * 8 && sizeof(SfState<32>) == 24 + 8 * 32,
              "SfState size must match stateBytes (bsf_core.h)");

// StaircaseFilter(m, kk) chunk i with the reference's (byte) arithmetic (S/StaircaseFilter.java:47-67);
// kk >= 1 here (the prefix scan runs at minMismatches = k + 1)
GWA_HD void sfChunk(int m_, int kk, int i, int *start, int *len) {
  const int lastChunkSize = (m_ - kk >= 6) ? m_ * 2 / (kk + 2) : m_ - kk;
  const int rest = (int)(int8_t)(uint8_t)(m_ - lastChunkSize);
  const int s0 = (int)(int8_t)(uint8_t)(rest * i / kk);
  const int s1 = i + 1 <= kk ? (int)(int8_t)(uint8_t)(rest * (i + 1) / kk) : (int)(int8_t)(uint8_t)m_;
  *start = s0;
  *len = (int)(int8_t)(uint8_t)(s1 - s0);
}
// true when some prefix-scan chunk of an m-base read at minMismatches kk starts outside [0, m] or
// ends past m: only then can an SFState offset leave the staircase table's range (the automaton's
// masks then come from SfLane's WRAP path); the host picks the kernel instance from this
GWA_HD bool sfChunksWrap(int m_, int kk) {
  int wrap = 0;
  for (int c = 0; c <= kk; ++c) {
    int cs = 0, w = 0;
    sfChunk(m_, kk, c, &cs, &w);
    wrap |= (cs < 0 || cs > m_ || cs + (w > 0 ? w : 0) > m_) ? 1 : 0;
  }
  return wrap != 0;
}

// WRAP: the batch has reads whose chunk starts wrap (sfChunksWrap); without them the automaton's
// out-of-table mask path is compiled out (it cost the R = 8 kernel ~35 spilled VGPRs)
template <int R, int QW, bool WRAP = true>
struct SfLane : BsfLane<R, QW, false, 24> {
  typedef BsfLane<R, QW, false, 24> B;
  using B::ix;
  using B::cfg;
  using B::L;
  using B::caps;
  using B::m;
  using B::k;
  using B::minMismatches;
  using B::maxMatchLength;
  using B::bestScore;
  using B::numFMIndexSearches;
  using B::heapSize;
  using B::listSize;
  using B::status;
  using B::quickSteps;
  using B::blocks;
  using B::saReads;
  using B::kmerLookups;
  using B::shortSteps;

  GWA_HD SfLane(const IndexView &ix_, const SearchConfig &c_, const StairTables &s_, LaneMem<R> L_, Caps caps_)
      : B(ix_, c_, s_, L_, caps_) {}

  GWA_HD SfState<R> *arena() const { return (SfState<R> *)L.slice; }
  int nCand = 0;  // candidates (TreeSet<Long>[2], :295) as start << 1 | strand in L.cand()

  // A polled SFState is never read again (the loop works on its register copy; SF has no split
  // chains), so its arena slot is recycled: the arena holds the queued states only, and its size
  // bounds the live queue, not the states created.  Free slots are linked through SfState::lb.
  // The newest free slot is kept in a register (spare): a step frees the polled state and then
  // allocates its children, and taking the spare costs no memory round trip, where popping the list
  // waits on a load of the link.
  int freeHead = -1, spare = -1, created = 0;
  GWA_HD int sfAlloc() {
    if (spare >= 0) {
      const int id = spare;
      spare = -1;
      return id;
    }
    if (freeHead >= 0) {
      const int id = freeHead;
      freeHead = (int)arena()[id].lb;
      return id;
    }
    return B::allocState();
  }
  GWA_HD void sfFree(int id) {
    if (spare >= 0) {
      arena()[spare].lb = (uint32_t)freeHead;
      freeHead = spare;
    }
    spare = id;
  }

  // candidates[strand].contains(start) / add: a linear scan of L.cand() for the small sets of the
  // first tiers; an open-addressing hash table (caps.cand slots, a power of two, at most half full)
  // when caps.cand >= kCandHash -- the deep tiers hold reads with tens of thousands of candidates,
  // where a scan per candidate would be quadratic.  Only membership is used (:304-306), so the
  // table's order does not matter.
  static constexpr int kCandHash = 4096;
  static constexpr int64_t kCandEmpty = (int64_t)0x8000000000000000LL;
  GWA_HD void candClear() {
    nCand = 0;
    if (caps.cand >= kCandHash)
      for (int i = 0; i < caps.cand; ++i) L.cand()[i] = kCandEmpty;
  }
  // 1 = newly added, 0 = already present, -1 = the set is full (overflow)
  GWA_HD int candInsert(int64_t key) {
    int64_t *c = L.cand();
    if (caps.cand < kCandHash) {
      for (int i = 0; i < nCand; ++i)
        if (c[i] == key) return 0;
      if (nCand >= caps.cand) return -1;
      c[nCand++] = key;
      return 1;
    }
    const uint32_t mask = (uint32_t)caps.cand - 1u;
    uint32_t h = (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ULL) >> 40) & mask;
    for (;;) {
      const int64_t v = c[h];
      if (v == key) return 0;
      if (v == kCandEmpty) break;
      h = (h + 1u) & mask;
    }
    if (2 * (nCand + 1) > caps.cand) return -1;
    c[h] = key;
    ++nCand;
    return 1;
  }

  // SFState.compareTo (:463-469) as a heap key: kOffset ascending, then score descending
  GWA_HD static uint64_t keyOf(int kOffset, int score) {
    return ((uint64_t)(kOffset & 0xFF) << 32) | ((uint64_t)((int64_t)0x7FFFFFFF - (int64_t)score) & 0xFFFFFFFFULL);
  }
  GWA_HD void push(int idx, int kOffset, int score) { B::queueAddKeyed((keyOf(kOffset, score) << 24) | (uint64_t)idx); }

  GWA_HD int newState(int strand, int offset, int index, int score, uint32_t lb, uint32_t ub, uint8_t meta,
                      const uint64_t (&rows)[R], int nrows, int kOffset, bool hasHit) {
    const int id = sfAlloc();
    if (id < 0) return -1;
    ++created;
    SfState<R> d;
    d.lb = lb; d.ub = ub; d.score = score;
    d.strand = (uint8_t)strand; d.offset = (int16_t)offset; d.index = (int16_t)index; d.nrows = (uint8_t)nrows;
    d.kOffset = (uint8_t)kOffset; d.hasHit = hasHit ? 1 : 0; d.meta = meta;
#pragma unroll
    for (int i = 0; i < R; ++i) d.nfa[i] = i < nrows ? rows[i] : 0ULL;
    arena()[id] = d;
    return id;
  }

  GWA_HD static void chunk(int m_, int kk, int i, int *start, int *len) { sfChunk(m_, kk, i, start, len); }

  // PrefixScan.scanRead for one chunk: exact forward search of q[strand][cs, cs + w) from [0, N).
  // Returns 0 = mismatch (null si), 1 = rows [lb, ub), 2 = one row whose SA value is *lb.
  // The k-mer table answers the first K steps (an empty step anywhere in them = a mismatch, the
  // only outcome the reference keeps), and a one-row interval continues in text mode
  // (BsfLane::textBefore).
  GWA_HD int scanChunk(int strand, int cs, int w, uint32_t *olb, uint32_t *oub) {
    const int fm = strand == 0 ? 1 : 0;  // forwardSearch on FORWARD uses the reverse index (:138-141)
    uint64_t lb = 0, ub = ix.N, tp = 0;
    int uniq = 0, x = cs;
    const int end = cs + w;
    const int K = ix.kmerK;
    if (K > 0 && w >= K) {
      const uint64_t e = ix.kmer[fm][B::qWindowL(strand, cs, K)];
      ++kmerLookups;
      if (e == 0) return 0;
      lb = e & 0xFFFFFFFFULL;
      ub = e >> 32;
      quickSteps += K;
      shortSteps += K;
      x += K;
      if (ub - lb == 1) {
        tp = ix.sa[fm][lb];
        ++saReads;
        uniq = 1;
      }
    }
    typename B::TextWalk tw;
    int miss = 0;
    for (; x < end && miss == 0; ++x) {
      const int ch = B::qcode(strand, x);
      ++quickSteps;
      if (uniq) {
        ++shortSteps;
        const int tc = B::textBefore(fm, tp, tw);
        miss = tc != ch ? 1 : 0;
        tp = tp == 0 ? ix.N - 1 : tp - 1;
      } else {
        // backwardSearch(ch, si) = C[ch] + getOcc(ch, lb|ub) (A/FMIndexOnOccTable.java:47-51)
        Block B0, B1;
        loadBlock(ix.occ[fm], lb >> 7, B0);
        loadBlock(ix.occ[fm], ub >> 7, B1);
        blocks += 1 + ((lb >> 7) != (ub >> 7) ? 1 : 0);
        const uint64_t nlb = ix.C[ch] + rankOne(B0, lb, ch), nub = ix.C[ch] + rankOne(B1, ub, ch);
        miss = nlb >= nub ? 1 : 0;
        lb = nlb;
        ub = nub;
        if (miss == 0 && nub - nlb == 1) {
          tp = ix.sa[fm][nlb];
          ++saReads;
          uniq = 1;
        }
      }
    }
    if (miss) return 0;
    if (uniq) {
      *olb = (uint32_t)tp;
      *oub = (uint32_t)tp + 1;
      return 2;
    }
    *olb = (uint32_t)lb;
    *oub = (uint32_t)ub;
    return 1;
  }

  // align_internal up to the loop (:229-256): N check, prefix scans, initQueue.  false = done.
  GWA_HD bool sfStart() {
    const int countN = B::buildMasks();
    if (countN > k) return false;  // reported unmapped (:232-236)
    if (!B::stairOk()) return false;  // StaircaseFilter(m, k + 1) throws (PrefixScan.scanRead's filter, :244)
    const int kk = minMismatches;  // k + 1
    const int nch = kk + 1;
    const int mCap = (m + 63) / 64 * 64;  // ACGTSequence storage: positions past it throw
    uint64_t init[R];
#pragma unroll
    for (int i = 0; i < R; ++i) init[i] = i <= k ? (uint64_t)jshl(1, k + i) : 0ULL;  // activateDiagonalStates
    for (int strand = 0; strand < 2; ++strand) {
      for (int c = 0; c < nch; ++c) {
        int cs = 0, w = 0;
        chunk(m, kk, c, &cs, &w);
        // getACGT outside the read's storage throws ArrayIndexOutOfBounds when the scan reaches it:
        // at once below 0, at mCap unless a mismatch ends the chunk first.  A chunk of width <= 0
        // (the reference's (byte) chunk starts wrap for long reads) scans nothing.
        if (w > 0 && cs < 0) {
          status = ST_ERROR;
          return false;
        }
        const bool past = w > 0 && cs + w > mCap;
        uint32_t lb = 0, ub = (uint32_t)ix.N;  // an empty chunk keeps wholeSARange
        const int r = w > 0 ? scanChunk(strand, cs, past ? mCap - cs : w, &lb, &ub) : 1;
        if (past && r != 0) {
          status = ST_ERROR;
          return false;
        }
        if (r == 0) continue;  // chunkWithMismatch
        const int score = cfg.matchScore * w;
        const int id = newState(strand, cs, cs + w, score, lb, ub, r == 2 ? M_TEXT : 0, init, k + 1, 0, false);
        if (id < 0) return false;
        push(id, 0, score);
        if (status == ST_OVERFLOW) return false;
      }
    }
    return true;
  }

  // AlignmentResultHolder.add (:369-389) for a single-hit chain (no splits on this path)
  GWA_HD void sfResultAdd(int hit, int diff) {
    if (m > 0 && diff < minMismatches) {
      minMismatches = diff;
      bestScore = m * cfg.matchScore - diff * cfg.mismatchPenalty;
    }
    if (maxMatchLength < m) maxMatchLength = m;
    int n = 0;
    for (int i = 0; i < listSize; ++i) {
      const int e = L.list()[i];
      if (L.hits()[e].diff <= minMismatches) L.list()[n++] = e;
    }
    if (n >= caps.list) {
      B::ovf(OV_LIST);
      listSize = n;
      return;
    }
    L.list()[n++] = hit;
    listSize = n;
  }

  // addCandidate (:298-343); false = the search ends (overflow / error)
  GWA_HD bool addCandidate(const SfState<R> &c) {
    if (c.ub - c.lb != 1) return true;  // multi hit: nothing (:339-342)
    const int strand = c.strand;
    // toCoordinate(si.lowerBound, strand, Forward) (A/FMIndexOnGenome.java:227-238), full SA
    const int fm = strand == 0 ? 1 : 0;
    int64_t v;
    if (c.meta & M_TEXT) {
      v = (int64_t)c.lb;
    } else {
      v = (int64_t)ix.sa[fm][c.lb];
      ++saReads;
    }
    const int64_t seqIndex = fm == 0 ? v : (int64_t)ix.N - v;
    const int offsetFromSearchHead = strand == 0 ? c.index : m - c.index;
    const int64_t start = seqIndex - offsetFromSearchHead;
    const int64_t key = (int64_t)((uint64_t)start << 1) | strand;
    const int ins = candInsert(key);
    if (ins == 0) return true;  // candidates[strand].contains(start)
    if (ins < 0) {
      B::ovf(OV_CAND);
      return false;
    }
    const int64_t refStart = start - k > 0 ? start - k : 0;
    const int64_t refEnd = start + m + k < (int64_t)ix.N ? start + m + k : (int64_t)ix.N;
    if (refStart > refEnd) {  // ACGTSequence.subString throws
      status = ST_ERROR;
      return false;
    }
    int pos = 0, diff = 0, co = 0, cl = 0;
    // the whole read, reversed on strand 1 (:317-321)
    const int r = B::alignBlockDetailed(strand, 0, m, refStart, refEnd, &pos, &diff, &co, &cl);
    if (r < 0) return false;
    if (r == 1) return true;  // alignment == null
    // a dropped hit's CIGAR ops are released (the lane's CIGAR area then holds the listed hits' ops
    // only: reads on repeats verify millions of candidates)
    int32_t chr, p;
    if (B::translate(refStart + pos + 1, &chr, &p) != 0) {  // UTGBException is logged
      B::nCigar = co;
      return true;
    }
    // reportResult (:345-353): total match length m; a hit above minMismatches is dropped
    if (m == 0 || diff > minMismatches) {
      B::nCigar = co;
      return true;
    }
    const int h = B::newHit(chr, p, m, 0, m, diff, strand, co, cl, 1);
    if (h < 0) return false;
    sfResultAdd(h, diff);
    return status != ST_OVERFLOW;
  }

  // SFState.nextState (:448-460) + ReadAlignmentNFA.nextState(nextACGTIndex, progress, m, ...)
  // (S/ReadAlignmentNFA.java:136-144); pushes the child; false = the search ends
  GWA_HD bool child(const SfState<R> &c, int ch, uint32_t lb, uint32_t ub) {
    if (!B::stairOk()) return false;  // c.nextState(..., getStairCaseFilter(m)) (:282)
    const int nextIndex = c.index + 1;
    const int kr = c.nrows - 1;
    const int64_t qeq = B::patternMask64(c.strand, true, nextIndex, 0, nextIndex, ch, kr);
    uint64_t rows[R];
    int nh = 0, nko = 0;
    bool hm = false;
    if (!B::template nfaCore<WRAP>(c.nfa, c.nrows, c.kOffset, qeq, nextIndex - c.offset, m - c.offset, rows, &nh, &nko, &hm))
      return true;  // null: numFiltered++
    const int diff = nko - c.kOffset;
    int newScore = c.score - diff * cfg.mismatchPenalty;
    if (diff == 0) newScore++;
    const int id = newState(c.strand, c.offset, nextIndex, newScore, lb, ub, 0, rows, nh, nko, hm);
    if (id < 0) return false;
    push(id, nko, newScore);
    return status != ST_OVERFLOW;
  }

  // one iteration of the queue loop (:257-290); false = the loop ended
  GWA_HD bool sfStep() {
    if (heapSize == 0 || status == ST_OVERFLOW || status == ST_ERROR) return false;
    const int idx = B::queuePoll();
    const SfState<R> c = arena()[idx];
    sfFree(idx);
    const int ubScore = c.score + (c.offset + (m - c.index)) * cfg.matchScore;  // scoreUpperBound (:444-446)
    if ((int)c.kOffset > minMismatches || ubScore < bestScore) return true;    // numCutOff++
    if (c.hasHit || c.index >= m || c.ub - c.lb == 1) return addCandidate(c);
    // fmIndex.forwardSearch(strand, si) (A/FMIndexOnGenome.java:203-225): the four base extensions
    const int fm = c.strand == 0 ? 1 : 0;
    uint64_t lo[5], hi[5];
    B::rank2(fm, c.lb, c.ub, lo, hi);
    ++numFMIndexSearches;
    for (int ch = 0; ch < 4; ++ch) {  // ACGT.exceptN
      const uint64_t l = ix.C[ch] + lo[ch], u = ix.C[ch] + hi[ch];
      if (l < u && !child(c, ch, (uint32_t)l, (uint32_t)u)) return false;
    }
    return true;
  }

  GWA_HD void sfSearch() {
    candClear();
    freeHead = spare = -1;
    created = 0;
    if (!sfStart()) return;
    while (sfStep()) {
    }
  }
};

}  // namespace gwa
