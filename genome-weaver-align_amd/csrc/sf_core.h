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
#include <new>
#include "bsf_core.h"

namespace gwa {

// dst = src for lane objects (their IndexView / SearchConfig / StairTables members are references,
// the same objects in both: copy-construction in place; the cooperative kernel's register snapshot)
template <class T>
GWA_HD void laneCopy(T &dst, const T &src) {
  dst.~T();
  ::new (static_cast<void *>(&dst)) T(src);
}

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
// DPM: the DP history mode (BsfLane); the cooperative sparse kernel keeps whole columns (2) and the
// top of its queue in LDS (BsfLane's hybrid heap: L.heapL / heapH, set by the kernel)
template <int R, int QW, bool WRAP = true, int DPM = 0>
struct SfLane : BsfLane<R, QW, DPM == 2, 24, DPM> {
  typedef BsfLane<R, QW, DPM == 2, 24, DPM> B;
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
  using B::nCigar;
  using B::numSW;
  using B::verifyBytes;
  using B::ovfWhat;
#ifdef GWA_PROF
  using B::prof;
  using B::profG;
#endif

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
      if (DPM == 2 && B::uOn) B::ulogPut(kUArena | (uint32_t)id, (uint64_t)(uint32_t)freeHead);  // (its free link)
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
  // first tier; an open-addressing hash table (caps.cand slots, a power of two, at most half full)
  // when caps.cand >= kCandHash -- the deeper tiers hold reads with up to hundreds of thousands of
  // candidates, where a scan per candidate (one dependent load per entry) would be quadratic.  Only
  // membership is used (:304-306), so the table's order does not matter.
  static constexpr int kCandHash = 64;
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
      c[nCand++] = key;  // (past the restored nCand: no undo entry)
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
    if (DPM == 2 && B::uOn) B::ulogPut(kUCand | h, (uint64_t)kCandEmpty);
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

  // AlignmentResultHolder.add (:369-389) for a single-hit chain (no splits on this path).  After
  // every add each listed hit has diff <= minMismatches (reportResult drops the others, :349-350),
  // so the rebuild of the list (:381-388) can only drop entries when this add lowers minMismatches:
  // only then is the list scanned (at most k + 1 times per read; reads on repeats list thousands of
  // hits, and a scan per add was quadratic in them)
  GWA_HD void sfResultAdd(int hit, int diff) {
    const bool lower = m > 0 && diff < minMismatches;
    if (lower) {
      minMismatches = diff;
      bestScore = m * cfg.matchScore - diff * cfg.mismatchPenalty;
    }
    if (maxMatchLength < m) maxMatchLength = m;
    int n = listSize;
    if (lower) {  // (the scan in a branch of its own: a loop whose condition also tests the loop-invariant
                  // flag lost hits on gfx950 -- tests/test_gpu_parity.py::test_long_reads_on_gpu, -m sf 400 bp)
      n = 0;
      for (int i = 0; i < listSize; ++i) {
        const int e = L.list()[i];
        if (L.hits()[e].diff <= minMismatches) L.list()[n++] = e;
      }
    }
    if (n >= caps.list) {
      B::ovf(OV_LIST);
      listSize = n;
      return;
    }
    L.list()[n++] = hit;
    listSize = n;
  }

  // The verification job of a candidate: alignBlockDetailed(jStrand, 0, m, jRefStart, jRefEnd), a pure
  // function of (start, strand) = jKey
  int jStrand = 0;
  int64_t jRefStart = 0, jRefEnd = 0, jKey = 0;
  // toCoordinate(si.lowerBound, strand, Forward) (A/FMIndexOnGenome.java:227-238) of a single-row
  // state, as the candidate's start position (:301-303) and its set key start << 1 | strand
  GWA_HD int64_t candStart(uint32_t lb, int strand, int index, uint8_t meta, int64_t *key) {
    const int fm = strand == 0 ? 1 : 0;
    int64_t v;
    if (meta & M_TEXT) {
      v = (int64_t)lb;
    } else {
      v = (int64_t)ix.sa[fm][lb];
      ++saReads;
    }
    const int64_t seqIndex = fm == 0 ? v : (int64_t)ix.N - v;
    const int offsetFromSearchHead = strand == 0 ? index : m - index;
    const int64_t start = seqIndex - offsetFromSearchHead;
    *key = (int64_t)((uint64_t)start << 1) | strand;
    return start;
  }
  // addCandidate (:298-343) up to the verification: 0 = done (*go: false = the search ends, overflow /
  // error), 1 = the job (jStrand, jRefStart, jRefEnd) is to be verified, then candEnd
  GWA_HD int candBegin(const SfState<R> &c, bool *go) {
    *go = true;
    if (c.ub - c.lb != 1) return 0;  // multi hit: nothing (:339-342)
    int64_t key;
    const int64_t start = candStart(c.lb, c.strand, c.index, c.meta, &key);
    GWA_PT(tci);
    const int ins = candInsert(key);
    GWA_PA(PR_SPLIT, tci);
    if (ins == 0) return 0;  // candidates[strand].contains(start)
    if (ins < 0) {
      B::ovf(OV_CAND);
      *go = false;
      return 0;
    }
    const int64_t refStart = start - k > 0 ? start - k : 0;
    const int64_t refEnd = start + m + k < (int64_t)ix.N ? start + m + k : (int64_t)ix.N;
    if (refStart > refEnd) {  // ACGTSequence.subString throws
      status = ST_ERROR;
      *go = false;
      return 0;
    }
    jStrand = c.strand;  // the whole read, reversed on strand 1 (:317-321)
    jRefStart = refStart;
    jRefEnd = refEnd;
    jKey = key;
    return 1;
  }
  // addCandidate after the verification r (0 alignment, 1 null, < 0 overflow); false = the search ends
  GWA_HD bool candEnd(int r, int pos, int diff, int co, int cl) {
    if (r < 0) return false;
    if (r == 1) return true;  // alignment == null
    // a dropped hit's CIGAR ops are released (the lane's CIGAR area then holds the listed hits' ops
    // only: reads on repeats verify millions of candidates)
    int32_t chr, p;
    if (B::translate(jRefStart + pos + 1, &chr, &p) != 0) {  // UTGBException is logged
      nCigar = co;
      return true;
    }
    // reportResult (:345-353): total match length m; a hit above minMismatches is dropped
    if (m == 0 || diff > minMismatches) {
      nCigar = co;
      return true;
    }
    const int h = B::newHit(chr, p, m, 0, m, diff, jStrand, co, cl, 1);
    if (h < 0) return false;
    sfResultAdd(h, diff);
    return status != ST_OVERFLOW;
  }
  // addCandidate (:298-343) in one piece (the per-lane kernels: locals, not the job fields)
  GWA_HD bool addCandidate(const SfState<R> &c) {
    if (c.ub - c.lb != 1) return true;  // multi hit: nothing (:339-342)
    const int strand = c.strand;
    int64_t key;
    const int64_t start = candStart(c.lb, strand, c.index, c.meta, &key);
    GWA_PT(tci);
    const int ins = candInsert(key);
    GWA_PA(PR_SPLIT, tci);
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
    GWA_PC(PR_NVW, PR_NVL);
    const int r = B::alignBlockDetailed(strand, 0, m, refStart, refEnd, &pos, &diff, &co, &cl);
    if (r < 0) return false;
    if (r == 1) return true;  // alignment == null
    int32_t chr, p;
    if (B::translate(refStart + pos + 1, &chr, &p) != 0) {  // UTGBException is logged
      nCigar = co;
      return true;
    }
    if (m == 0 || diff > minMismatches) {  // reportResult (:345-353)
      nCigar = co;
      return true;
    }
    const int h = B::newHit(chr, p, m, 0, m, diff, strand, co, cl, 1);
    if (h < 0) return false;
    sfResultAdd(h, diff);
    return status != ST_OVERFLOW;
  }

  // ---- deferred verification (the cooperative kernel of the sparse last tier, DPM 2) ----
  // Lane 0 of a wavefront runs the read's search.  A verification whose result is not in the result
  // table is not waited for: it is queued -- with every later one, in poll order -- and the search
  // goes on with its writes to the queue, the arena's free links and the candidate set logged (undo
  // log).  At kSfDJobs queued jobs, at the search's end or when the log is nearly full, lanes 1-63
  // run the queued DPs into the table and lane 0 commits the jobs in order (candEnd).  A
  // verification acts on the search only through minMismatches / bestScore (the cutoff, :261): if a
  // committed result would lower them while something was polled after its job, the search is put
  // back to where the deferral began (the undo log, and the copy of the lane's registers the kernel
  // took there) and goes on from that point, taking every result it meets from the table.
  // minMismatches only decreases, so a read rolls back at most k + 1 times.  A DP result is a pure
  // function of (start, strand): taking it from the table changes nothing but the time.
  // Table entry: the key, the result and a CIGAR of up to kSpecOps ops (a longer one is recomputed
  // by lane 0 when it commits); open addressing, <= kSpecProbe probes, slots claimed by CAS.
  struct SpecEntry {
    int64_t key;
    int32_t r, diff, pos;
    uint16_t ncig, pad;
    uint16_t ops[20];
  };
  struct DJob {
    int64_t key, refStart, refEnd;
    int32_t strand;
    uint32_t popsAt;  // polls of the read when the job was queued
  };
  static constexpr int kSpecOps = 20, kSpecProbe = 32;
  // undo-log tags: 0 a queue slot, kUArena a free link, kUCand a candidate-set slot, kUWord an arena word
  static constexpr uint64_t kUArena = 1ULL << 62, kUCand = 2ULL << 62, kUWord = 3ULL << 62;
  int dMode = 0, dN = 0;  // deferring; jobs queued
  uint32_t dPops = 0;     // polls so far
  GWA_HD SpecEntry *spec() const { return (SpecEntry *)(L.slice + L.oSpec); }
  GWA_HD DJob *djobs() const { return (DJob *)(L.slice + L.oSpec + 64 * (size_t)caps.spec); }
  GWA_HD uint64_t *ulogBase() const {
    return (uint64_t *)(L.slice + L.oSpec + 64 * (size_t)caps.spec + sizeof(DJob) * (size_t)kSfDJobs);
  }
  GWA_HD uint32_t specSlot(int64_t key) const {
    return (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ULL) >> 40) & ((uint32_t)caps.spec - 1u);
  }
  // the table slot holding key, or -1
  GWA_HD int specFind(int64_t key) const {
    uint32_t h = specSlot(key);
    int at = -1, go = 1;
    for (int q = 0; go && q < kSpecProbe; ++q) {
      const int64_t v = spec()[h].key;
      at = v == key ? (int)h : -1;
      go = (at < 0 && v != kCandEmpty) ? 1 : 0;
      h = (h + 1u) & ((uint32_t)caps.spec - 1u);
    }
    return at;
  }
  // the job's verification from table slot at, with alignBlockDetailed's effects (counters, CIGAR
  // ops appended); *r as alignBlockDetailed returns it
  GWA_HD void specApply(int at, int *r, int *pos, int *diff, int *co, int *cl) {
    const SpecEntry &e = spec()[at];
    const int N = (int)(jRefEnd - jRefStart), bMax = (m + 63) / 64 > 0 ? (m + 63) / 64 : 1;
    ++numSW;
    verifyBytes += (2 * N + 7) / 8 + (N + 7) / 8 + 32 * bMax;
    *r = e.r;
    if (e.r != 0) return;
    const int n = e.ncig;
    if (nCigar + n + 4 > caps.cigar) {
      B::ovf(OV_CIGAR);
      *r = -1;
      return;
    }
    for (int i = 0; i < n; ++i) L.cigar()[nCigar + i] = e.ops[i];
    *co = nCigar;
    *cl = n;
    nCigar += n;
    *pos = e.pos;
    *diff = e.diff;
  }
  // the job (jKey ...): its result from the table, or its DP run here; then candEnd
  GWA_HD bool candFinish() {
    int r = 0, pos = 0, diff = 0, co = 0, cl = 0;
    const int at = specFind(jKey);
    if (at >= 0) specApply(at, &r, &pos, &diff, &co, &cl);
    else r = B::alignBlockDetailed(jStrand, 0, m, jRefStart, jRefEnd, &pos, &diff, &co, &cl);
    return candEnd(r, pos, diff, co, cl);
  }
  // a helper lane: keep its result (r >= 0; a CIGAR of <= kSpecOps ops, from its own area cg)
  GWA_HD void specPut(int r, int pos, int diff, int co, int cl, const uint16_t *cg) {
    if (r < 0 || (r == 0 && cl > kSpecOps)) return;
    uint32_t h = specSlot(jKey);
    int at = -1, go = 1;
    for (int q = 0; go && q < kSpecProbe; ++q) {
#ifdef __HIP_DEVICE_COMPILE__
      const unsigned long long old = atomicCAS((unsigned long long *)&spec()[h].key, (unsigned long long)kCandEmpty,
                                               (unsigned long long)jKey);
#else
      const unsigned long long old = (unsigned long long)spec()[h].key;
      if (old == (unsigned long long)kCandEmpty) spec()[h].key = jKey;
#endif
      at = old == (unsigned long long)kCandEmpty ? (int)h : -1;
      go = (at < 0 && old != (unsigned long long)jKey) ? 1 : 0;  // (another lane holds this key: done)
      h = (h + 1u) & ((uint32_t)caps.spec - 1u);
    }
    if (at < 0) return;
    SpecEntry &e = spec()[at];
    e.r = r;
    e.diff = diff;
    e.pos = pos;
    e.ncig = (uint16_t)(r == 0 ? cl : 0);
    for (int i = 0; r == 0 && i < cl; ++i) e.ops[i] = cg[co + i];
  }
  // a helper lane (1..63): load queued job lid - 1 of the owner (sharing its slice); false = none, or
  // its result is already in the table
  GWA_HD bool djobLoad(int j, int qn) {
    if (j >= qn) return false;
    const DJob jb = djobs()[j];
    jKey = jb.key;
    jStrand = jb.strand;
    jRefStart = jb.refStart;
    jRefEnd = jb.refEnd;
    return specFind(jKey) < 0;
  }
  // the candidate set and the result table emptied by the 64 lanes of the wavefront together
  GWA_HD void coopClear(int lid) {
    nCand = 0;
    dMode = dN = 0;
    dPops = 0;
    B::uN = B::uOn = 0;
    B::ulogP = ulogBase();
    if (caps.cand >= kCandHash)
      for (int i = lid; i < caps.cand; i += 64) L.cand()[i] = kCandEmpty;
    for (int i = lid; i < caps.spec; i += 64) spec()[i].key = kCandEmpty;
  }
  // lane 0 after a pass: commit the queued jobs in order.  Returns -1 when all were committed (*go
  // false: the search ended), else the job at which the search must roll back.
  GWA_HD int dCommit(bool *go) {
    *go = true;
    int rb = -1;
    for (int i = 0; i < dN && rb < 0 && *go; ++i) {
      const DJob jb = djobs()[i];
      jKey = jb.key;
      jStrand = jb.strand;
      jRefStart = jb.refStart;
      jRefEnd = jb.refEnd;
      const int at = specFind(jKey);
      int r = 0, pos = 0, diff = 0, co = 0, cl = 0;
      if (at >= 0) {
        r = spec()[at].r;
        pos = spec()[at].pos;
        diff = spec()[at].diff;
      } else {  // (not kept: its DP here, in order; rolled back below if need be)
        r = B::alignBlockDetailed(jStrand, 0, m, jRefStart, jRefEnd, &pos, &diff, &co, &cl);
      }
      int32_t chr, p;
      const bool lower = r == 0 && m > 0 && diff < minMismatches && B::translate(jRefStart + pos + 1, &chr, &p) == 0;
      if (lower && (i + 1 < dN || dPops > jb.popsAt)) {
        rb = i;
      } else {
        if (at >= 0) specApply(at, &r, &pos, &diff, &co, &cl);
        *go = candEnd(r, pos, diff, co, cl);
      }
    }
    B::uOn = 0;  // (a roll-back then replays the log: undoApply)
    if (rb < 0) dMode = dN = B::uN = 0;
    return rb;
  }
  // the logged writes undone, newest first (the kernel then restores the registers)
  GWA_HD void undoApply() {
    for (int i = B::uN - 1; i >= 0; --i) {
      const uint64_t tag = B::ulogP[2 * (size_t)i], old = B::ulogP[2 * (size_t)i + 1];
      const uint32_t at = (uint32_t)tag;
      const uint64_t kind = tag >> 62;
      if (kind == 0) B::hslot((int)at) = old;
      else if (kind == 1) arena()[at].lb = (uint32_t)old;
      else if (kind == 2) L.cand()[at] = (int64_t)old;
      else ((uint64_t *)arena())[tag & ((1ULL << 62) - 1ULL)] = old;
    }
    B::uN = 0;
  }

  // SFState.nextState (:448-460) + ReadAlignmentNFA.nextState(nextACGTIndex, progress, m, ...)
  // (S/ReadAlignmentNFA.java:136-144); pushes the child; false = the search ends
  GWA_HD bool child(const SfState<R> &c, int ch, uint32_t lb, uint32_t ub) {
    if (!B::stairOk()) return false;  // c.nextState(..., getStairCaseFilter(m)) (:282)
    const int nextIndex = c.index + 1;
    const int kr = c.nrows - 1;
    GWA_PT(tq);
    const int64_t qeq = B::patternMask64(c.strand, true, nextIndex, 0, nextIndex, ch, kr);
    uint64_t rows[R];
    int nh = 0, nko = 0;
    bool hm = false;
    if (!B::template nfaCore<WRAP>(c.nfa, c.nrows, c.kOffset, qeq, nextIndex - c.offset, m - c.offset, rows, &nh, &nko, &hm))
      return true;  // null: numFiltered++
    GWA_PA(PR_NFA, tq);
    GWA_PT(ta);
    const int diff = nko - c.kOffset;
    int newScore = c.score - diff * cfg.mismatchPenalty;
    if (diff == 0) newScore++;
    const int id = newState(c.strand, c.offset, nextIndex, newScore, lb, ub, 0, rows, nh, nko, hm);
    if (id < 0) return false;
    push(id, nko, newScore);
    GWA_PA(PR_ADD1, ta);
    return status != ST_OVERFLOW;
  }

  // one iteration of the queue loop (:257-290): 0 = the loop ended, 1 = go on.  COOP (lane 0 of the
  // cooperative kernel): 2 = run a pass over the queued jobs and commit them (dCommit); 3 = a job was
  // queued and deferral begins here (the kernel copies the lane's registers, then sets dMode / uOn)
  template <bool COOP>
  GWA_HD int sfStepT() {
    const int end = COOP && dMode ? 2 : 0;
    if (heapSize == 0 || status == ST_OVERFLOW || status == ST_ERROR) return end;
    if (COOP && dMode && B::uN + 512 > kSfULog) return 2;  // (a step logs < 512 writes)
    GWA_PT(tp);
    int idx;
    SfState<R> c;
    if (COOP) {  // the root's state is loaded while the sift runs (its registers are free in that kernel)
      idx = (int)(B::hslot(0) & ((1ULL << 24) - 1ULL));
      c = arena()[idx];
      B::queuePoll();
      ++dPops;
      if (DPM == 2 && B::uOn) {  // the polled state's words: its slot may be reused before a roll-back
        const uint64_t *w = (const uint64_t *)&c;
#pragma unroll
        for (int q = 0; q < (int)(sizeof(SfState<R>) / 8); ++q)
          B::ulogPut(kUWord | ((uint64_t)idx * (sizeof(SfState<R>) / 8) + q), w[q]);
      }
    } else {
      idx = B::queuePoll();
      c = arena()[idx];
    }
    sfFree(idx);
    GWA_PC(PR_NSW, PR_NSL);
    GWA_PA(PR_POLL, tp);
    const int ubScore = c.score + (c.offset + (m - c.index)) * cfg.matchScore;  // scoreUpperBound (:444-446)
    if ((int)c.kOffset > minMismatches || ubScore < bestScore) return 1;    // numCutOff++
    if (c.hasHit || c.index >= m || c.ub - c.lb == 1) {
      GWA_PT(tv);
      int res;
      if (COOP) {
        bool go;
        if (!candBegin(c, &go)) {
          res = go ? 1 : end;
        } else if (!dMode && specFind(jKey) >= 0) {
#ifdef GWA_PROF
          if (profG) profG[PR_NBL] += 1;  // (results taken from the table outside a deferral)
#endif
          res = candFinish() ? 1 : 0;
        } else {
          djobs()[dN] = DJob{jKey, jRefStart, jRefEnd, jStrand, dPops};
          ++dN;
          res = !dMode ? 3 : dN >= kSfDJobs ? 2 : 1;
        }
      } else {
        res = addCandidate(c) ? 1 : 0;
      }
      GWA_PA(PR_VERIFY, tv);
      return res;
    }
    // fmIndex.forwardSearch(strand, si) (A/FMIndexOnGenome.java:203-225): the four base extensions
    const int fm = c.strand == 0 ? 1 : 0;
    uint64_t lo[5], hi[5];
    GWA_PT(tf);
    B::rank2(fm, c.lb, c.ub, lo, hi);
    GWA_PA(PR_FM, tf);
    ++numFMIndexSearches;
    for (int ch = 0; ch < 4; ++ch) {  // ACGT.exceptN
      const uint64_t l = ix.C[ch] + lo[ch], u = ix.C[ch] + hi[ch];
      if (l < u && !child(c, ch, (uint32_t)l, (uint32_t)u)) return end;
    }
    return 1;
  }
  GWA_HD bool sfStep() { return sfStepT<false>() != 0; }

  // align_internal's start (candidate set emptied by the caller in the cooperative kernel)
  GWA_HD bool sfBegin(bool clear) {
    if (clear) candClear();
    freeHead = spare = -1;
    created = 0;
    GWA_PT(tsd);
    const bool go = sfStart();
    GWA_PA(PR_SEED, tsd);
    return go;
  }
  GWA_HD void sfSearch() {
    if (!sfBegin(true)) return;
    while (sfStep()) {
    }
  }
};

}  // namespace gwa
