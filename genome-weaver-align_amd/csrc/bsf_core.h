// bsf_core.h -- per-lane bidirectional suffix-filter search (BSF, `align -m bsf`), MI355X device code.
//
// One read per lane.  Each lane owns a slice of HBM scratch (state arena, binary heap, hit arena,
// DP history) and runs the reference's best-first search with the exact operation order of
//   S/BidirectionalSuffixFilter.java:278-477 (AlignmentProcess.align_internal)
// so that results are bit-identical to the reference (and to the CPU oracle in oracle/).
// Data layouts are MI355X-native (gwa_layout.h): 64-B Occ blocks, full SA, 96..320-B states.
//
// The same source is compiled by hipcc for gfx950 (the product) and, for CPU-side debugging of
// the kernel logic only, by g++ in tests/ (never a product fallback: the C-ABI requires a GPU).
#pragma once
#include <math.h>
#include <string.h>

#include "gwa_layout.h"

namespace gwa {

// ---- Java arithmetic (JLS 15.19: shift counts masked to 6 bits for long) ----
GWA_HD int64_t jshl(int64_t x, int64_t s) { return (int64_t)((uint64_t)x << (s & 63)); }
GWA_HD int64_t jushr(int64_t x, int64_t s) { return (int64_t)((uint64_t)x >> (s & 63)); }
GWA_HD int popc64(uint64_t x) { return __builtin_popcountll(x); }

// a[i] for a runtime i through unrolled selects: small arrays stay in VGPRs instead of scratch
// (the empty asm pins each element as a VGPR value, so the select chain is not folded back into
// a load from a runtime address, which would force the array into scratch memory)
template <class T>
GWA_HD T pinv(T x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x));
#endif
  return x;
}
// true when c holds on any active lane of the wavefront (the lane's own c on host builds): a
// uniform branch around work that only some lanes need
GWA_HD bool anyLane(bool c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(c) != 0;
#else
  return c;
#endif
}
#if defined(GWA_VERIFY_LOG) && !defined(__HIP_DEVICE_COMPILE__)
// host test builds only: one line per DP verification, to the file $GWA_VERIFY_LOG
inline FILE *gwaVerifyLog() {
  static FILE *f = getenv("GWA_VERIFY_LOG") ? fopen(getenv("GWA_VERIFY_LOG"), "w") : nullptr;
  return f;
}
#endif
// Region timers of the search loop (profiling builds only, -DGWA_PROF): the delta of the
// shader clock across a region is charged once per wavefront (first active lane), so summing over
// lanes gives wavefront cycles spent per region.
#if defined(GWA_PROF) && defined(__HIP_DEVICE_COMPILE__)
#define GWA_PT(v) const uint64_t v = clock64()
#define GWA_PA(r, v)                                                            \
  do {                                                                          \
    const uint64_t d_ = clock64() - (v);                                        \
    if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) prof[r] += d_;      \
  } while (0)
// GWA_PC(w, l): count one wavefront execution in slot w and one lane execution in slot l (counters
// in the lane's global profile slots, profG: a register array of them broke the gfx950 backend)
#define GWA_PC(w, l)                                                            \
  do {                                                                          \
    if (profG) {                                                                \
      if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) profG[w] += 1;    \
      profG[l] += 1;                                                            \
    }                                                                           \
  } while (0)
// GWA_PW(w, e, b): a store of b bytes at one site: bytes in slot w, one lane event in slot e
#define GWA_PW(w, e, b)                                                         \
  do {                                                                          \
    if (profG) {                                                                \
      profG[w] += (uint64_t)(b);                                                \
      profG[e] += 1;                                                            \
    }                                                                           \
  } while (0)
#else
#define GWA_PT(v)
#define GWA_PA(r, v)
#define GWA_PC(w, l)
#define GWA_PW(w, e, b)
#endif

// LDS-typed pointers on the device (plain pointers on host builds)
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) const uint64_t lds_cu64;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
#else
typedef const uint64_t lds_cu64;
typedef uint64_t lds_u64;
#endif

template <class T, int N>
GWA_HD T pick(const T (&a)[N], int i) {
  T v = pinv(a[0]);
#pragma unroll
  for (int j = 1; j < N; ++j) {
    // every element is pinned, then chosen: a select (v_cndmask), not a branch around the asm
    // (measured: bsf_search 100.8 -> 97.4 ms, hg19 C2)
    const T x = pinv(a[j]);
    v = (i == j) ? x : v;
  }
  return v;
}

// ---------------------------------------------------------------------------------------------
// Rank on one 64-B Occ block (A/OccurrenceCountTable.java:80-107, A/ACGTSequence.java:456-549)
// ---------------------------------------------------------------------------------------------
struct Block {
  uint32_t cnt[4];
  uint64_t lo0, lo1, hi0, hi1, n0, n1;
};

GWA_HD void loadBlock(const OccBlock *occ, uint64_t b, Block &o) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 *p = reinterpret_cast<const u32x4 *>(occ + b);
  u32x4 a = __builtin_nontemporal_load(p + 0);
  u32x4 l = __builtin_nontemporal_load(p + 1);
  u32x4 h = __builtin_nontemporal_load(p + 2);
  u32x4 n = __builtin_nontemporal_load(p + 3);
  o.cnt[0] = a.x; o.cnt[1] = a.y; o.cnt[2] = a.z; o.cnt[3] = a.w;
  o.lo0 = ((uint64_t)l.y << 32) | l.x; o.lo1 = ((uint64_t)l.w << 32) | l.z;
  o.hi0 = ((uint64_t)h.y << 32) | h.x; o.hi1 = ((uint64_t)h.w << 32) | h.z;
  o.n0 = ((uint64_t)n.y << 32) | n.x; o.n1 = ((uint64_t)n.w << 32) | n.z;
#else
  const OccBlock &B = occ[b];
  for (int i = 0; i < 4; ++i) o.cnt[i] = B.cnt[i];
  o.lo0 = B.lo[0]; o.lo1 = B.lo[1]; o.hi0 = B.hi[0]; o.hi1 = B.hi[1]; o.n0 = B.nmask[0]; o.n1 = B.nmask[1];
#endif
}

// counts of A,C,G,T,N in bwt[0, i) where i lies in block B (i>>7 == block index)
GWA_HD void rankAll(const Block &B, uint64_t i, uint64_t out[5]) {
  const uint32_t r = (uint32_t)(i & 127);
  const uint64_t m0 = r >= 64 ? ~0ULL : ((1ULL << r) - 1ULL);
  const uint64_t m1 = r > 64 ? ((1ULL << (r - 64)) - 1ULL) : 0ULL;
  const uint32_t pLo = popc64(B.lo0 & m0) + popc64(B.lo1 & m1);
  const uint32_t pHi = popc64(B.hi0 & m0) + popc64(B.hi1 & m1);
  const uint32_t pT = popc64(B.lo0 & B.hi0 & m0) + popc64(B.lo1 & B.hi1 & m1);
  const uint32_t pN = popc64(B.n0 & m0) + popc64(B.n1 & m1);
  const uint32_t cC = pLo - pT, cG = pHi - pT;
  const uint32_t cA = r - cC - cG - pT - pN;
  out[0] = (uint64_t)B.cnt[0] + cA;
  out[1] = (uint64_t)B.cnt[1] + cC;
  out[2] = (uint64_t)B.cnt[2] + cG;
  out[3] = (uint64_t)B.cnt[3] + pT;
  out[4] = i - out[0] - out[1] - out[2] - out[3];
}

GWA_HD uint64_t rankOne(const Block &B, uint64_t i, int ch) {
  const uint32_t r = (uint32_t)(i & 127);
  const uint64_t m0 = r >= 64 ? ~0ULL : ((1ULL << r) - 1ULL);
  const uint64_t m1 = r > 64 ? ((1ULL << (r - 64)) - 1ULL) : 0ULL;
  switch (ch) {
    case 1: return (uint64_t)B.cnt[1] + popc64(B.lo0 & ~B.hi0 & m0) + popc64(B.lo1 & ~B.hi1 & m1);
    case 2: return (uint64_t)B.cnt[2] + popc64(B.hi0 & ~B.lo0 & m0) + popc64(B.hi1 & ~B.lo1 & m1);
    case 3: return (uint64_t)B.cnt[3] + popc64(B.hi0 & B.lo0 & m0) + popc64(B.hi1 & B.lo1 & m1);
    case 0: {
      uint32_t any = popc64((B.lo0 | B.hi0 | B.n0) & m0) + popc64((B.lo1 | B.hi1 | B.n1) & m1);
      return (uint64_t)B.cnt[0] + (r - any);
    }
    default: {
      uint64_t o[5];
      rankAll(B, i, o);
      return o[4];
    }
  }
}

// One entry of the k-mer interval table (IndexView::kmer): K backward-search steps
// (A/FMIndexOnOccTable.java:47-51) from [0, N) over `key`, first-processed base in the low bits
// (the order of the 2-bit packed read words, so a key is a shifted window of them).
GWA_HD uint64_t kmerInterval(const OccBlock *occ, const uint64_t C[5], uint64_t N, uint32_t key, int K) {
  uint64_t lb = 0, ub = N;
  for (int j = 0; j < K; ++j) {
    const int ch = (int)((key >> (2 * j)) & 3);
    Block B0, B1;
    loadBlock(occ, lb >> 7, B0);
    loadBlock(occ, ub >> 7, B1);
    const uint64_t nlb = C[ch] + rankOne(B0, lb, ch), nub = C[ch] + rankOne(B1, ub, ch);
    if (nlb >= nub) return 0;
    lb = nlb;
    ub = nub;
  }
  return (ub << 32) | lb;
}

// ---------------------------------------------------------------------------------------------
// Per-lane search state (SearchState, S/BidirectionalSuffixFilter.java:658-877)
// ---------------------------------------------------------------------------------------------
enum : uint8_t { SI_FWD = 0, SI_BWD = 1, SI_BID = 2, SI_EMPTY = 3 };
enum : uint8_t { M_SIVALID = 4, M_CURVALID = 8, M_NFAVALID = 16, M_TEXT = 32 };
// Text mode (M_TEXT, BsfLane::nextSi): the state's pattern P occurs exactly once in the cyclic text,
// so every interval of its SiSet is one row or empty and is decided by one text character.  The
// SiSet then holds lb[0] = t, the text start of P (strand 0) or of reverse(P) (strand 1; the read
// complement is matched reversed, A/FMIndexOnGenome.java:134-146), lb[1] = |P|, lb[2] = the one
// character c whose SiSet entry is non-empty (4 = none).
enum : int { D_FORWARD = 0, D_BACKWARD = 1, D_BIFWD = 2 };

template <int R>
struct DState {
  uint32_t lb[4], ub[4];  // SiSet primary intervals: F for SI_FWD/SI_BID, B for SI_BWD (valid iff lb<ub)
  uint32_t curLb, curUb;  // currentSi
  uint32_t bBase;         // SI_BID: B interval of ch = bBase + sum_{j<ch} width_j + [0, width_ch)
  int32_t state;          // flags(5) | base(3) | minK(8) | priority(8) | hasHit(1) | clipped(1)  (:664)
  int32_t nextSplit;      // arena index, -1 = null
  uint8_t flag, nrows, kOffset, meta;
  uint16_t start, end, cursor, pivot;  // Cursor (S/Cursor.java:42-47); reads up to 512 bp
  uint64_t nfa[R];        // ReadAlignmentNFA rows (S/ReadAlignmentNFA.java:60-61)
};

struct DHit {
  int32_t chr, pos, matchLength, qStart, qEnd, diff, strand, numHits, next;
  int32_t cigarOff, cigarLen;
  int32_t pad;
};

// per-lane scratch capacities (entries)
struct Caps {
  int32_t arena, heap, hits, list, cigar, dpWords, path;
  int32_t dpSlice;  // 1: the DP history keeps a 32-row slice around the read's diagonal (first tier)
  int32_t cand;  // SuffixFilter candidate set (sf_core.h); 0 on the BSF path
  int32_t sparse;  // > 1: only every sparse-th lane of a wavefront takes reads (deep tiers, bsf_search_kernel)
  int32_t sf;      // 1: the arena holds SfState<R> (sf_core.h), else DState<R>
  int32_t spec;    // -m sf sparse last tier: verification result table entries (SfLane::SpecEntry, a power of two)
};
// bytes of one arena slot: SfState<R> is 24 + 8 R bytes (static_assert in sf_core.h)
template <int R>
GWA_HD size_t stateBytes(const Caps &c) { return c.sf ? (size_t)(24 + 8 * R) : sizeof(DState<R>); }

// Per-lane scratch.  The search structures (arena/heap/hits/list/cigar) sit in a per-lane slice;
// the DP history, the per-column DP flags and the traceback path are "interleaved": element e of
// this lane lives at ptr[e * is].  On the GPU is = 64 and a wavefront's 64 lanes are adjacent, so
// the lock-step DP column stores of a wavefront coalesce into one contiguous line per store.
template <int R>
struct LaneMem {
  // two base pointers + uniform offsets (kept in SGPRs), not eight per-lane pointers
  uint8_t *slice;          // this lane's slice: arena | heap | hits | list | cigar
  uint8_t *chunk;          // interleaved block (the wavefront's on the GPU, the lane's on the host)
  uint32_t oHeap, oCand, oHits, oList, oCigar, oSpec;  // byte offsets in the slice
  uint32_t oPath;          // byte offset of the path plane in the chunk
  int lane, is;            // lane in the interleaved block, interleave stride (elements)
  // PriorityQueue array of (key << KS | state index): entry i at heapP[i * hs].  In the slice
  // (hs = 1) or, for the first tier, in LDS interleaved across the workgroup (hs = 256).
  // Hybrid heap (HY kernels: k >= 4, and the sparse deep tiers): entries [0, heapH) in LDS at
  // heapL[i * hsL], the rest in the slice at heapG[i] (heapH = 0: all in the slice)
  uint64_t *heapP;
  int hs;
  uint64_t *heapL = nullptr, *heapG = nullptr;
  int heapH = 0, hsL = 256;
  GWA_HD DState<R> *arena() const { return (DState<R> *)slice; }
  GWA_HD uint64_t *heap() const { return heapP; }
  GWA_HD int64_t *cand() const { return (int64_t *)(slice + oCand); }
  GWA_HD DHit *hits() const { return (DHit *)(slice + oHits); }
  GWA_HD int32_t *list() const { return (int32_t *)(slice + oList); }
  GWA_HD uint16_t *cigar() const { return (uint16_t *)(slice + oCigar); }
  GWA_HD uint64_t *dp() const { return (uint64_t *)chunk + lane; }   // [2][col 0..N][block] vp / vn history
  GWA_HD uint8_t *path() const { return chunk + oPath + lane; }      // traceback path
};

template <int R>
GWA_HD size_t laneBytes(const Caps &c) {  // per-lane slice
  size_t b = 0;
  b += stateBytes<R>(c) * (size_t)c.arena;
  b += 8 * (size_t)c.heap;
  b += 8 * (size_t)c.cand;
  b += sizeof(DHit) * (size_t)c.hits;
  b += 4 * (size_t)c.list;
  b += 2 * (size_t)c.cigar;
  // (-m sf cooperative kernel: result table, deferred jobs, undo log; SfLane)
  if (c.spec > 0) b = ((b + 63) & ~(size_t)63) + 64 * (size_t)c.spec + 32 * (size_t)kSfDJobs + 16 * (size_t)kSfULog;
  return (b + 255) & ~(size_t)255;
}
GWA_HD size_t ilvBytes(const Caps &c) {  // interleaved bytes per lane
  return (8 * (size_t)c.dpWords + (size_t)c.path + 7) & ~(size_t)7;
}

// slice = this lane's slice; chunk = its wavefront's interleaved block (64 lanes, is = 64), or the
// lane's own interleaved block (is = 1, host builds)
template <int R>
GWA_HD LaneMem<R> laneMem(uint8_t *slice, uint8_t *chunk, int laneInWave, int is, const Caps &c) {
  LaneMem<R> L;
  size_t b = stateBytes<R>(c) * (size_t)c.arena;
  L.slice = slice;
  L.oHeap = (uint32_t)b; b += 8 * (size_t)c.heap;
  L.oCand = (uint32_t)b; b += 8 * (size_t)c.cand;
  L.oHits = (uint32_t)b; b += sizeof(DHit) * (size_t)c.hits;
  L.oList = (uint32_t)b; b += 4 * (size_t)c.list;
  L.oCigar = (uint32_t)b; b += 2 * (size_t)c.cigar;
  L.oSpec = (uint32_t)((b + 63) & ~(size_t)63);
  L.chunk = chunk;
  L.oPath = (uint32_t)((size_t)is * 8 * (size_t)c.dpWords);
  L.lane = laneInWave;
  L.is = is;
  L.heapP = (uint64_t *)(slice + L.oHeap);
  L.hs = 1;
  L.heapG = L.heapP;
  L.heapH = 0;
  return L;
}
template <int R>
GWA_HD LaneMem<R> laneMem(uint8_t *base, const Caps &c) {  // host: one lane, is = 1
  return laneMem<R>(base, base + laneBytes<R>(c), 0, 1, c);
}

// Streaming reader of reference codes (0-3, 4 = N) over the 2-bit text + N bitmap.  The word after
// (fwd) or before (back) the current one is loaded one word ahead, so a column walk waits on HBM
// once per 32 columns at most instead of once per column.
struct RefCursor {
  const uint64_t *t2, *tn;
  int64_t last2, lastN;                 // last valid word indices
  int64_t a2 = -4, an = -4;             // word indices held in c2 / cn
  uint64_t c2 = 0, cn = 0, x2 = 0, xn = 0;  // current words, prefetched neighbours
  int64_t xa2 = -4, xan = -4;           // indices of the prefetched neighbours
  GWA_HD RefCursor(const uint64_t *t2_, const uint64_t *tn_, uint64_t N)
      : t2(t2_), tn(tn_), last2(N ? (int64_t)((N - 1) >> 5) : 0), lastN(N ? (int64_t)((N - 1) >> 6) : 0) {}
  GWA_HD int code(int64_t p, int dir) {
    const int64_t a = p >> 5, b = p >> 6;
    if (a != a2) {
      c2 = a == xa2 ? x2 : t2[a];
      a2 = a;
      int64_t na = a + dir;
      na = na < 0 ? 0 : na > last2 ? last2 : na;
      xa2 = na;
      x2 = t2[na];
    }
    if (b != an) {
      cn = b == xan ? xn : tn[b];
      an = b;
      int64_t nb = b + dir;
      nb = nb < 0 ? 0 : nb > lastN ? lastN : nb;
      xan = nb;
      xn = tn[nb];
    }
    return ((cn >> (p & 63)) & 1) ? 4 : (int)((c2 >> ((p & 31) * 2)) & 3);
  }
};

// The DP's reference window [p0, p0 + n) held in registers: 2-bit codes as W2 words of 32 bases and
// the N bitmap as WN words of 64, each re-aligned to p0 (funnel shift).  All 2 (W2 + WN + 2) loads are
// issued together before the DP, so the window costs one memory wait; RefCursor's per-column
// prefetch made every column of a wavefront wait on whichever lane crossed a word boundary.
template <int W2, int WN>
struct RefWindow {
  uint64_t c2[W2], cn[WN];
  GWA_HD void load(const uint64_t *t2, const uint64_t *tn, uint64_t N, int64_t p0) {
    const int64_t last2 = N ? (int64_t)((N - 1) >> 5) : 0, lastN = N ? (int64_t)((N - 1) >> 6) : 0;
    const int64_t a = p0 >> 5, b = p0 >> 6;
    uint64_t r2[W2 + 1], rn[WN + 1];
#pragma unroll
    for (int i = 0; i <= W2; ++i) r2[i] = t2[a + i < last2 ? a + i : last2];
#pragma unroll
    for (int i = 0; i <= WN; ++i) rn[i] = tn[b + i < lastN ? b + i : lastN];
    const int s2 = (int)(p0 & 31) * 2, sn = (int)(p0 & 63);
#pragma unroll
    for (int i = 0; i < W2; ++i) c2[i] = s2 ? (r2[i] >> s2) | (r2[i + 1] << (64 - s2)) : r2[i];
#pragma unroll
    for (int i = 0; i < WN; ++i) cn[i] = sn ? (rn[i] >> sn) | (rn[i + 1] << (64 - sn)) : rn[i];
  }
  // codes (2-bit fields) and N flags of window positions [p, p + 32), -31 <= p; positions below 0
  // read as code 0, no N
  GWA_HD void window32(int p, uint64_t *c, uint32_t *nb) const {
    if (p < 0) {
      *c = c2[0] << (2 * -p);
      *nb = (uint32_t)(cn[0] << -p);
      return;
    }
    const int w = p >> 5, sh = 2 * (p & 31), wn = p >> 6, sn = p & 63;
    const uint64_t a = pick(c2, w), b = w + 1 < W2 ? pick(c2, w + 1) : 0ULL;
    const uint64_t an = pick(cn, wn), bn = wn + 1 < WN ? pick(cn, wn + 1) : 0ULL;
    *c = sh ? (a >> sh) | (b << (64 - sh)) : a;
    *nb = (uint32_t)(sn ? (an >> sn) | (bn << (64 - sn)) : an);
  }
  // code (0-3, 4 = N) of window position j (0 <= j < 32 * W2)
  GWA_HD int code(int j) const {
    if ((pick(cn, j >> 6) >> (j & 63)) & 1) return 4;
    return (int)((pick(c2, j >> 5) >> ((j & 31) * 2)) & 3);
  }
};

struct Overflow {};  // thrown only on host test builds; device uses status codes

// QW = 2-bit query words per strand held in registers (4: reads <= 128 bp, 8: <= 255 bp); the
// DP then needs at most DB = QW / 2 blocks of 64 rows.  HY: hybrid heap (hslot).
// KS: bits of the state index in a queue entry (key << KS | index).  Both paths' keys are 40 bits
// (packKey here, SfLane::keyOf), so an arena holds up to 2^24 states.
// DPM: the DP traceback's history (alignBlockDetailed): 0 = column checkpoints, recomputed on
// demand; 1 = the first tier's kernel, whose reads of more than two 64-row blocks keep a 32-row
// slice of every column instead (the recompute of a 4-block column costs the k >= 4 first tier more
// than the slice's 8 B per column); 2 = every column's blocks (16 B per block per column: the -m sf
// verification of a lone lane, whose tracebacks take tens of edits and would recompute a column
// per edit)
template <int R, int QW = 8, bool HY = false, int KS = 24, int DPM = 0>
struct BsfLane {
  static constexpr int DB = QW / 2;
  static constexpr uint64_t IDXM = (1ULL << KS) - 1ULL;
  const IndexView &ix;
  const SearchConfig &cfg;
  const StairTables &st;
  LaneMem<R> L;
  Caps caps;
  // read
  const uint8_t *rd;  // original codes 0..4
  int m, k;
  bool nReplaced;
  // search bookkeeping (AlignmentProcess fields, :175-187, :588-592)
  int minMismatches, maxMatchLength, bestScore;
  int numFMIndexSearches;
  int nStates, heapSize, nHits, listSize, nCigar;
  int status;  // ST_*
  int ovfWhat = 0;  // OV_* bits: which per-lane capacity a ST_OVERFLOW exceeded (the host grows it)
  GWA_HD void ovf(int what) {
    status = ST_OVERFLOW;
    ovfWhat |= what;
  }
  // instrumentation
  int quickSteps, blocks, saReads, maxHeap, kmerLookups, shortSteps, textSteps, textRuns;
  int numSW, verifyBytes;  // DP verifications and their §8d bytes (instrumentation)
  // debug trace (nullptr in production launches): 4 words per event
  uint32_t *trace = nullptr;
  int traceCap = 0, traceN = 0;
#ifdef GWA_PROF
  uint64_t prof[PR_N] = {};  // cycle regions (GWA_PA)
  uint64_t *profG = nullptr; // this lane's global profile slots (GWA_PC / GWA_PW counters)
#endif
  GWA_HD void tr(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    if (!trace || traceN + 4 > traceCap) return;
    trace[traceN++] = a; trace[traceN++] = b; trace[traceN++] = c; trace[traceN++] = d;
  }
  GWA_HD uint32_t curWord(const DState<R> &d) const {
    return (uint32_t)d.flag | ((uint32_t)d.start << 8) | ((uint32_t)d.end << 16) | ((uint32_t)d.cursor << 24);
  }

  GWA_HD BsfLane(const IndexView &ix_, const SearchConfig &c_, const StairTables &s_, LaneMem<R> L_, Caps caps_)
      : ix(ix_), cfg(c_), st(s_), L(L_), caps(caps_) {}

  // The read, 2-bit packed for both strands after replaceN_withA (S/BidirectionalSuffixFilter.java:
  // 281-291): q[1] is the complement (not the reverse complement) of q[0] (:193); N -> A on both.
  // Word w of strand s holds positions 32w..32w+31, position p at bits 2(p&31); positions >= m are 0.
  // The codes are read 16 bytes at a time (reads start 16-B aligned in HBM, ReadsView); returns the
  // number of N codes (fastCount(N), A/ACGTSequence.java:456-477).
  GWA_HD static uint32_t pack4(uint32_t v) {  // 4 byte codes -> 4 two-bit fields
    uint32_t x = v & 0x03030303u;
    x = (x | (x >> 6)) & 0x000F000Fu;
    return (x | (x >> 12)) & 0xFFu;
  }
  GWA_HD static uint32_t nbits4(uint32_t v) {  // 4 byte codes -> 4 N flags
    uint32_t x = (v >> 2) & 0x01010101u;
    return (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xFu;
  }
  GWA_HD int loadWords(uint64_t (&w0)[QW], uint64_t (&w1)[QW]) const {
    int countN = 0;
#pragma unroll
    for (int w = 0; w < QW; ++w) {
      uint64_t a0 = 0, a1 = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // 16 codes per half word
        const int p0 = 32 * w + 16 * h;
        if (p0 < m) {
          uint32_t v[4];
#if defined(__HIP_DEVICE_COMPILE__)
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 c = *reinterpret_cast<const u32x4 *>(rd + p0);
          v[0] = c.x; v[1] = c.y; v[2] = c.z; v[3] = c.w;
#else
          memcpy(v, rd + p0, 16);
#endif
          uint32_t lo = 0, nb = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            lo |= pack4(v[j]) << (8 * j);
            nb |= nbits4(v[j]) << (4 * j);
          }
          const int valid = m - p0;  // positions p0 + [0, valid) belong to the read
          const uint32_t vm = valid >= 16 ? 0xFFFFu : ((1u << valid) - 1u);
          nb &= vm;
          // 2-bit field mask of the valid, non-N positions
          uint32_t keep = 0;
#pragma unroll
          for (int j = 0; j < 16; ++j) keep |= (((vm & ~nb) >> j) & 1u) * (3u << (2 * j));
          countN += popc64(nb);
          a0 |= (uint64_t)(lo & keep) << (32 * h);
          a1 |= (uint64_t)((lo ^ 0xFFFFFFFFu) & keep) << (32 * h);
        }
      }
      w0[w] = a0;
      w1[w] = a1;
    }
    return countN;
  }
  // quick-scan kernel: the read words in registers
  uint64_t pw0[QW], pw1[QW];
  GWA_HD int q(int strand, int i) const {
    const uint64_t x = strand ? pick(pw1, i >> 5) : pick(pw0, i >> 5);
    return (int)((x >> (2 * (i & 31))) & 3);
  }
  // bits [2i, 2i + 2K) of strand `strand` (K <= 16): q(i + j) at bits 2j
  GWA_HD uint32_t qWindow(int strand, int i, int K) const {
    const int w = i >> 5, sh = 2 * (i & 31);
    const uint64_t a = strand ? pick(pw1, w) : pick(pw0, w);
    const uint64_t b = (w + 1 < QW) ? (strand ? pick(pw1, w + 1) : pick(pw0, w + 1)) : 0ULL;
    const uint64_t x = sh ? (a >> sh) | (b << (64 - sh)) : a;
    return (uint32_t)(x & ((1ULL << (2 * K)) - 1ULL));
  }

  // ---- FM index primitives (A/FMIndexOnGenome.java:121-225) ----
  GWA_HD uint64_t occOne(int fm, int ch, uint64_t i) {
    if (i > ix.N) i = ix.N;
    Block B;
    loadBlock(ix.occ[fm], i >> 7, B);
    ++blocks;
    return rankOne(B, i, ch);
  }
  // two rankACGTN calls; block shared when lb and ub fall in the same 128-position window
  GWA_HD void rank2(int fm, uint64_t lb, uint64_t ub, uint64_t lo[5], uint64_t hi[5]) {
    if (lb > ix.N) lb = ix.N;
    if (ub > ix.N) ub = ix.N;
    // both blocks are requested before either is used: one memory round trip, not two
    const int two = (ub >> 7) != (lb >> 7);
    Block B0, B1;
    loadBlock(ix.occ[fm], lb >> 7, B0);
    loadBlock(ix.occ[fm], ub >> 7, B1);  // same line when !two (an L2 hit)
    blocks += 1 + two;
    rankAll(B0, lb, lo);
    rankAll(B1, ub, hi);
  }

  // ---- SequenceBoundary.translate (A/SequenceBoundary.java:104-121): last offset < textIndex ----
  GWA_HD int translate(int64_t textIndex, int32_t *chr, int32_t *pos) const {
    int lo = 0, hi = ix.nContig;  // count of offsets < textIndex
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (ix.contigOff[mid] < textIndex) lo = mid + 1;
      else hi = mid;
    }
    if (lo == 0) return -1;  // UTGBException
    *chr = lo - 1;
    *pos = (int32_t)(textIndex - ix.contigOff[lo - 1]);
    return 0;
  }

  // ---- QueryMask (A/QueryMask.java:41-97), computed on the fly ----
  // The read (after replaceN_withA) is kept 2-bit packed for both strands: word (s, w) holds
  // positions 32w..32w+31 of strand s.  A 64-bit pattern window is a funnel shift of three words,
  // a 2-bit compare and an even-bit compress (no per-read mask arrays).  On the device the words
  // live in LDS, interleaved across the workgroup (word e of thread t at qwL[e * qwS], qwS = 256):
  // a runtime word index is then one ds_read instead of a select chain over registers.
  lds_u64 *qwL = nullptr;
  int qwS = 1;
  // QueryMask rows P[strand][ch] (A/QueryMask.java:41-67: bit p = (q[strand][p] == ch), p < m) as
  // PW 64-bit words per row, precomputed once per read into LDS (interleaved like qwL) when the
  // kernel provides room (pmL != nullptr; m <= 128 kernels); eqWindow is then a two-word funnel
  // shift instead of a 2-bit compare and two even-bit compresses per NFA step.
  static constexpr int PW = QW / 2;
  lds_u64 *pmL = nullptr;
  int pmS = 1;
#if !defined(__HIP_DEVICE_COMPILE__)
  uint64_t qwH[2 * QW];
  uint64_t pmH[2 * 4 * PW];
  GWA_HD void hostWords() { qwL = qwH; qwS = 1; pmL = pmH; pmS = 1; }
#endif
  GWA_HD int buildMasks() {  // returns the read's N count
#if !defined(__HIP_DEVICE_COMPILE__)
    hostWords();
#endif
    uint64_t v0[QW], v1[QW];
    const int countN = loadWords(v0, v1);
#pragma unroll
    for (int w = 0; w < QW; ++w) {
      qwL[(size_t)w * qwS] = v0[w];
      qwL[(size_t)(QW + w) * qwS] = v1[w];
    }
    if (pmL) {
      // each 32-base word split once into its two bit planes (code bit 0, code bit 1); the four
      // rows are then plane combinations (A = 00, C = 01, G = 10, T = 11), A masked to p < m
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int w = 0; w < PW; ++w) {
          uint64_t rA = 0, rC = 0, rG = 0, rT = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint64_t v = st ? v1[2 * w + h] : v0[2 * w + h];
            const uint64_t p0 = compressEven(v), p1 = compressEven(v >> 1);
            const int valid = m - (64 * w + 32 * h);
            const uint64_t vm = valid >= 32 ? 0xFFFFFFFFULL : valid <= 0 ? 0ULL : (1ULL << valid) - 1ULL;
            rA |= (~p0 & ~p1 & vm) << (32 * h);
            rC |= (p0 & ~p1) << (32 * h);
            rG |= (~p0 & p1 & 0xFFFFFFFFULL) << (32 * h);
            rT |= (p0 & p1) << (32 * h);
          }
          pmL[(size_t)((st * 4 + 0) * PW + w) * pmS] = rA;
          pmL[(size_t)((st * 4 + 1) * PW + w) * pmS] = rC;
          pmL[(size_t)((st * 4 + 2) * PW + w) * pmS] = rG;
          pmL[(size_t)((st * 4 + 3) * PW + w) * pmS] = rT;
        }
      }
    }
    return countN;
  }
  // qWindow over the LDS words (search kernels)
  GWA_HD uint32_t qWindowL(int strand, int i, int K) const {
    const int w = i >> 5, sh = 2 * (i & 31);
    const uint64_t a = qword(strand, w), b = qword(strand, w + 1);
    const uint64_t x = sh ? (a >> sh) | (b << (64 - sh)) : a;
    return (uint32_t)(x & ((1ULL << (2 * K)) - 1ULL));
  }
  GWA_HD uint64_t qword(int strand, int w) const {
    return (unsigned)w < (unsigned)QW ? (uint64_t)qwL[(size_t)(strand * QW + w) * qwS] : 0ULL;
  }
  // 2-bit codes of strand `strand`'s read words at positions [p, p + 32); positions below 0 read as 0
  GWA_HD uint64_t qcodes32(int strand, int p) const {
    if (p < 0) return p <= -32 ? 0ULL : qword(strand, 0) << (2 * -p);
    const int w = p >> 5, sh = 2 * (p & 31);
    const uint64_t a = qword(strand, w), b = qword(strand, w + 1);
    return sh ? (a >> sh) | (b << (64 - sh)) : a;
  }
  GWA_HD static uint64_t compressEven(uint64_t x) {
    x &= 0x5555555555555555ULL;
    x = (x | (x >> 1)) & 0x3333333333333333ULL;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0FULL;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFULL;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFULL;
    x = (x | (x >> 16)) & 0x00000000FFFFFFFFULL;
    return x;
  }
  GWA_HD static uint64_t bitrev64(uint64_t x) {
#if defined(__clang__)
    return __builtin_bitreverse64(x);
#else
    x = ((x >> 1) & 0x5555555555555555ULL) | ((x & 0x5555555555555555ULL) << 1);
    x = ((x >> 2) & 0x3333333333333333ULL) | ((x & 0x3333333333333333ULL) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL) | ((x & 0x0F0F0F0F0F0F0F0FULL) << 4);
    x = ((x >> 8) & 0x00FF00FF00FF00FFULL) | ((x & 0x00FF00FF00FF00FFULL) << 8);
    x = ((x >> 16) & 0x0000FFFF0000FFFFULL) | ((x & 0x0000FFFF0000FFFFULL) << 16);
    return (x >> 32) | (x << 32);
#endif
  }
  // bit j = (q[strand][start + j] == ch) for start + j < m, else 0   (start >= 0)
  GWA_HD uint64_t eqWindow(int strand, int ch, int start) const {
    if (start >= m) return 0;
    if (pmL) {  // from the precomputed rows (bits at positions >= m are 0 there)
      const int w = start >> 6, sh = start & 63;
      const size_t row = (size_t)(strand * 4 + ch) * PW;
      const uint64_t a = (uint64_t)pmL[(row + w) * pmS];
      const uint64_t b = w + 1 < PW ? (uint64_t)pmL[(row + w + 1) * pmS] : 0ULL;
      return sh ? (a >> sh) | (b << (64 - sh)) : a;
    }
    const int w = start >> 5, sh = 2 * (start & 31);
    const uint64_t a = qword(strand, w), b = qword(strand, w + 1), c = qword(strand, w + 2);
    const uint64_t lo = sh ? (a >> sh) | (b << (64 - sh)) : a;
    const uint64_t hi = sh ? (b >> sh) | (c << (64 - sh)) : b;
    const uint64_t pat = 0x5555555555555555ULL * (uint64_t)ch;
    const uint64_t xl = lo ^ pat, xh = hi ^ pat;
    uint64_t r = compressEven(~(xl | (xl >> 1))) | (compressEven(~(xh | (xh >> 1))) << 32);
    const int range = m - start;
    if (range < 64) r &= (1ULL << range) - 1ULL;
    return r;
  }
  // QueryMask.getBidirectionalPatternMask64 (A/QueryMask.java:73-97): forward = patternMaskF window,
  // backward = patternMaskR window = the reversed forward window ending at the pivot.
  GWA_HD int64_t patternMask64(int strand, bool isForward, int nextIdx, int pivot, int cursor, int ch, int margin) {
    int64_t p;
    if (isForward) {
      int pos = nextIdx - margin;
      if (pos < 0) p = jshl((int64_t)eqWindow(strand, ch, 0), -pos);
      else p = (int64_t)eqWindow(strand, ch, pos);
    } else {
      uint64_t f;
      if (pivot <= 0) f = 0;
      else if (pivot >= 64) f = bitrev64(eqWindow(strand, ch, pivot - 64));
      else f = bitrev64((eqWindow(strand, ch, 0) & ((1ULL << pivot) - 1ULL)) << (64 - pivot));
      p = (int64_t)f;
      int rshift = pivot - cursor - margin;
      if (rshift >= 0) p = jushr(p, rshift);
      else p = jshl(p, -rshift);
    }
    return p;
  }
  // StaircaseFilter.getStairCaseMask64bit via the host-built table (S/StaircaseFilter.java:91-102)
  // this read's table (resolved once per read in initRead): the LDS copy when the kernel staged
  // the table of this length, else global memory.  The LDS pointer is typed address_space(3) so
  // the two loads are never merged into one flat load (which would wait on every outstanding
  // global access).
  lds_cu64 *stairLds = nullptr;
  const uint64_t *stairTab = nullptr;
  uint64_t stairBad = 0;  // bit kk: StaircaseFilter(m, kk) throws (the reference's (byte) chunk starts)
  int stairInLds = 0;
  // getStairCaseFilter(m) (S/BidirectionalSuffixFilter.java:206-208, S/SuffixFilter.java:140-142) at
  // the reference's call sites: the filter of the current minMismatches is built there, and a length
  // whose filter constructor throws aborts the run (ST_ERROR) at that point and no earlier
  GWA_HD bool stairOk() {
    if ((stairBad >> (minMismatches & 63)) & 1) {
      status = ST_ERROR;
      return false;
    }
    return true;
  }
  // getStairCaseMask64bit from the mask words behind the table (offsets outside [-kmax, m]):
  // offset >= 0: (~0L << (m - offset)) | mask.substring64(offset, offset + 64), else
  // mask.substring64(0, 64) << -offset (S/StaircaseFilter.java:91-102, A/BitVector.java:106-116)
  // (a static function of plain values, not inlined for R >= 8: the path is rare -- reads whose
  // (byte) chunk starts wrap, > ~223 bp -- and inlined into the automaton step's unrolled rows it
  // cost the R = 8 kernels 40-45 spilled VGPRs; the R = 4 kernels spill more with the call)
  GWA_HDNI static int64_t stairMaskRawNI(const uint64_t *tab, int km, int m, int kk, int row, int offset) {
    return stairMaskRaw(tab, km, m, kk, row, offset);
  }
  GWA_HD static int64_t stairMaskRaw(const uint64_t *tab, int km, int m, int kk, int row, int offset) {
    const int W = (m + 63) / 64;
    const uint64_t *v = tab + (size_t)(km + 2) * (km + 1) * (size_t)(m + km + 1) + (size_t)(kk * (km + 1) + row) * W;
    auto sub64 = [&](int64_t start, int64_t end) -> int64_t {  // start >= 0
      const int pos = (int)(start / 64);
      if (pos >= W) return 0;
      const int64_t range = end - start, off = start % 64;
      const int64_t mask = range >= 64 ? ~0LL : ~jshl(~0LL, range);
      const int64_t low = jushr((int64_t)v[pos], off);
      const int64_t high = pos + 1 < W ? jshl((int64_t)v[pos + 1] & ~jshl(~0LL, off), 64 - off) : 0LL;
      return (high | low) & mask;
    };
    if (offset >= 0) return jshl(~0LL, m - offset) | sub64(offset, (int64_t)offset + 64);
    return jshl(sub64(0, 64), -offset);
  }
  // WRAP: offsets outside the table are possible -- -m sf reads whose (byte) chunk starts wrap (a
  // negative SFState offset); the BSF automaton's offsets (processed bases - rows) never leave it
  template <bool WRAP>
  GWA_HD int64_t stairMask(int row, int offset) {
    const int kk = minMismatches;
    if (row >= kk + 1) return 0;
    const int km = st.kmax;
    // (a length whose filter throws never gets here: stairOk ran at the reference's call site)
#if !defined(__HIP_DEVICE_COMPILE__)
    if (!WRAP && (offset < -km || offset > m)) abort();  // host builds check the claim above
#endif
    if (WRAP && (offset < -km || offset > m))
      return R >= 8 ? stairMaskRawNI(stairTab, km, m, kk, row, offset) : stairMaskRaw(stairTab, km, m, kk, row, offset);
    const uint32_t i = (uint32_t)((kk * (km + 1) + row) * (m + km + 1) + offset + km);  // (tables < 2^32 words)
    if (stairInLds) return (int64_t)stairLds[i];
    return (int64_t)stairTab[i];
  }

  // ---- Cursor (S/Cursor.java) ----
  GWA_HD static int cDir(const DState<R> &s) { int d = (s.flag >> 1) & 3; return d == 3 ? D_FORWARD : d; }
  GWA_HD static bool cFwd(const DState<R> &s) { return cDir(s) != D_BACKWARD; }
  GWA_HD static int cStrand(const DState<R> &s) { return s.flag & 1; }
  GWA_HD static int cFrag(const DState<R> &s) { return (int)s.end - (int)s.start; }
  GWA_HD static int cProcessed(const DState<R> &s) { return cFwd(s) ? (int)s.cursor - (int)s.pivot : (int)s.end - (int)s.cursor; }
  GWA_HD static int cRemaining(const DState<R> &s) { return cFrag(s) - cProcessed(s); }
  GWA_HD static int cNextIdx(const DState<R> &s) { return cFwd(s) ? (int)s.cursor : (int)s.cursor - 1; }
  GWA_HD static int cOffsetOfSearchHead(const DState<R> &s) {
    int off = (int)s.cursor - (int)s.start;
    if (cStrand(s) == 1) off = cFrag(s) - off;
    return off;
  }
  GWA_HD static void setCursor(DState<R> &d, int strand, int dir, int start, int end, int cur, int piv) {
    d.flag = (uint8_t)(strand | (dir << 1));
    d.start = (uint16_t)start; d.end = (uint16_t)end; d.cursor = (uint16_t)cur; d.pivot = (uint16_t)piv;
  }

  // ---- SiSet accessors (A/SiSet.java) ----
  GWA_HD static uint8_t siType(const DState<R> &s) { return s.meta & 3; }
  GWA_HD static bool siValid(const DState<R> &s) { return (s.meta & M_SIVALID) != 0; }
  // getForward(ch): returns false for null
  GWA_HD static bool siText(const DState<R> &s) { return (s.meta & M_TEXT) != 0; }
  // (in text mode the returned interval is the dummy one-row [0, 1): its rows are never read)
  GWA_HD static bool siGetF(const DState<R> &s, int ch, uint32_t *lb, uint32_t *ub) {
    uint8_t t = siType(s);
    if (!siValid(s) || (t != SI_FWD && t != SI_BID)) return false;
    if (siText(s)) {
      if ((int)s.lb[2] != ch) return false;
      *lb = 0; *ub = 1;
      return true;
    }
    const uint32_t l = pick(s.lb, ch), u = pick(s.ub, ch);
    if (l >= u) return false;
    *lb = l; *ub = u;
    return true;
  }
  GWA_HD static bool siGetB(const DState<R> &s, int ch, uint32_t *lb, uint32_t *ub) {
    uint8_t t = siType(s);
    if (!siValid(s)) return false;
    if (siText(s)) {  // SI_BWD: c.P occurs; SI_BID: the B side of P.c, which occurs iff P.c does
      if ((t != SI_BWD && t != SI_BID) || (int)s.lb[2] != ch) return false;
      *lb = 0; *ub = 1;
      return true;
    }
    const uint32_t l = pick(s.lb, ch), u = pick(s.ub, ch);
    if (t == SI_BWD) {
      if (l >= u) return false;
      *lb = l; *ub = u;
      return true;
    }
    if (t != SI_BID) return false;
    if (l >= u) return false;
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) x += j < ch ? s.ub[j] - s.lb[j] : 0u;
    *lb = s.bBase + x;
    *ub = s.bBase + x + (u - l);
    return true;
  }
  GWA_HD static bool siIsEmpty(const DState<R> &s, int ch) {
    if (!siValid(s)) return true;  // NullPointerException in the reference; never reached (clipped tails)
    if (siType(s) == SI_EMPTY) return true;
    if (siText(s)) return (int)s.lb[2] != ch;
    return pick(s.lb, ch) >= pick(s.ub, ch);
  }
  GWA_HD void siInit(DState<R> &d, int dir) {  // FMIndexOnGenome.initSet (:117-128)
    d.meta = (uint8_t)((d.meta & ~(3 | M_TEXT)) | M_SIVALID | (dir == D_FORWARD ? SI_FWD : dir == D_BACKWARD ? SI_BWD : SI_BID));
    for (int c = 0; c < 4; ++c) {
      d.lb[c] = (uint32_t)ix.C[c];
      d.ub[c] = (uint32_t)ix.C[c + 1];
    }
    d.bBase = 0;
  }

  // ---- state flags ----
  GWA_HD DState<R> &S(int i) { return L.arena()[i]; }
  GWA_HD int minK(int s) { return (int)(((uint32_t)S(s).state >> 8) & 0xFF); }
  GWA_HD void setMinK(int s, int d) {
    invalidateCache();
    GWA_PW(PR_WS, PR_ES, 4);
    S(s).state &= ~(0xFF << 8);
    S(s).state |= (d & 0xFF) << 8;
  }
  GWA_HD int prio(int s) { return (int)(((uint32_t)S(s).state >> 16) & 0xFF); }
  GWA_HD bool hasHit(int s) { return (((uint32_t)S(s).state >> 24) & 1) != 0; }
  GWA_HD bool isClipped(int s) { return (((uint32_t)S(s).state >> 25) & 1) != 0; }
  GWA_HD bool isFinished(int s) { return (S(s).state & 0x1F) == 0x1F; }
  GWA_HD int curACGT(int s) { int c = ((uint32_t)S(s).state >> 5) & 7; return c > 4 ? 4 : c; }
  GWA_HD bool isChecked(int s, int ch) { return (S(s).state & (1 << ch)) != 0; }
  GWA_HD void updateFlag(int s, int ch) { S(s).state |= 1 << ch; }
  GWA_HD void updateSplitFlag(int s) { S(s).state |= 1 << 4; }
  GWA_HD int numSplit(int s) {
    int n = 0;
    for (int t = S(s).nextSplit; t >= 0; t = S(t).nextSplit) ++n;
    return n;
  }

  GWA_HD int allocState() {
    if (nStates >= caps.arena) { ovf(OV_ARENA); return -1; }
    return nStates++;
  }
  // state word bit 26 (not a reference field): some state's nextSplit is, or was, this state -- it
  // is a later member of a split chain (set by nextStateAfterSplit and update, never cleared)
  static constexpr int32_t kStRef = 1 << 26;
  GWA_HD void markRef(int s) {
    if (s == cacheIdx) flushCache();  // a referenced state is never a deferred one
    GWA_PW(PR_WS, PR_ES, 4);
    S(s).state |= kStRef;
    if (s == cacheIdx) cache.state |= kStRef;
  }
  GWA_HD static int32_t packState(int ch, int mk, int pr, bool hm) {
    return ((ch & 7) << 5) | ((mk & 0xFF) << 8) | ((pr & 0xFF) << 16) | ((hm ? 1 : 0) << 24);
  }
  // new SearchState(k, null, cursor, priority) (:753-757)
  GWA_HD int newInitial(int strand, int dir, int start, int end, int cur, int piv, int priority) {
    int id = allocState();
    if (id < 0) return -1;
    GWA_PW(PR_WA, PR_EA, sizeof(DState<R>));
    DState<R> &d = S(id);
    d.meta = 0;
    setCursor(d, strand, dir, start, end, cur, piv);
    siInit(d, dir);
    d.curLb = d.curUb = 0;
    d.state = packState(4, 0, priority, false);
    d.nextSplit = -1;
    d.nrows = (uint8_t)(k + 1);
    d.kOffset = 0;
    d.meta |= M_NFAVALID;
    for (int i = 0; i < R; ++i) d.nfa[i] = 0;
    for (int i = 0; i <= k; ++i) d.nfa[i] = (uint64_t)jshl(1, k + i);  // activateDiagonalStates (:77-84)
    return id;
  }

  // SearchState.score / upperBoundOfScore (:781-801), iterative over the split chain
  GWA_HD int chainScore(int s, bool upper) {
    // sum over members i of mm_i*M - nm_i*N - ns_i*S with ns_i = len-1-i, nm_i = minK_i - ns_i,
    // mm_i = processed_i (+ remaining_i) - nm_i, regrouped so one walk of the chain suffices
    int len = 0, sumPR = 0, sumK = 0;
    for (int t = s; t >= 0;) {
      const DState<R> &x = S(t);
      sumPR += cProcessed(x) + (upper ? cRemaining(x) : 0);
      sumK += (int)(((uint32_t)x.state >> 8) & 0xFF);
      ++len;
      t = x.nextSplit;
    }
    const int T = len * (len - 1) / 2;
    const int M = cfg.matchScore;
    return M * sumPR - (M + cfg.mismatchPenalty) * (sumK - T) - cfg.splitOpenPenalty * T;
  }
  // The queue order (SearchState comparator, :141-150: priority ascending, then score() descending,
  // then processed bases descending) as one unsigned 40-bit key: priority (6 bits; <= k + 1 <= 32) |
  // 2^23 - 1 - score (24 bits; the host bounds |score| < 2^23 for the batch's scoring and read
  // lengths, gwa_api.cpp batchTail) | 1023 - processed (10 bits; reads <= 512 bp)
  GWA_HD static uint64_t packKey(int pr, int sc, int proc) {
    return ((uint64_t)(pr & 63) << 34) | ((uint64_t)((int64_t)0x7FFFFF - (int64_t)sc) & 0xFFFFFFULL) << 10 |
           (uint64_t)(1023 - proc);
  }
  GWA_HD uint64_t keyOf(int s) {
    if (s == cacheIdx && cache.nextSplit < 0)
      return packKey((int)(((uint32_t)cache.state >> 16) & 0xFF), stateScore(cache, 0, false), cProcessed(cache));
    return packKey(prio(s), chainScore(s, false), cProcessed(S(s)));
  }
  // Heap slot i: the LDS / slice array of the kernel instance (first tier: LDS), or, with the hybrid
  // heap (HY; k >= 4 kernels: their heaps outgrow a small LDS array, deep heaps are rare), LDS for the
  // top slots and the slice beyond them -- one flat address either way
  // Undo log of the queue's writes (DPM 2: the cooperative -m sf kernel's deferred verification,
  // SfLane): while uOn, every queue slot written is logged first as (slot, old entry), so the
  // queue can be put back as it was when the deferral began.  The old entries are values the sifts
  // hold anyway (no extra loads); a poll logs its vacated last slot, so an offer's new slot needs none.
  uint64_t *ulogP = nullptr;
  int uN = 0, uOn = 0;
  GWA_HD void ulogPut(uint64_t tag, uint64_t old) {
    ulogP[2 * (size_t)uN] = tag;
    ulogP[2 * (size_t)uN + 1] = old;
    ++uN;
  }
  GWA_HD void ulogHeap(int i, uint64_t old) {
    if (DPM == 2 && uOn) ulogPut((uint64_t)(uint32_t)i, old);
  }
  GWA_HD uint64_t &hslot(int i) const {
    if (HY) return i < L.heapH ? L.heapL[(size_t)i * L.hsL] : L.heapG[i];
    return L.heap()[(size_t)i * L.hs];
  }
  // Re-key the queued entries whose split chain passes through state `changed` (its minK or its
  // nextSplit changed, so their score(), S/BidirectionalSuffixFilter.java:781-801, did; Java's queue
  // sees the new value at its next comparison, the cached key must show it).  The others keep their
  // keys.  Entries are scanned 8 at a time with their loads issued together (deep tiers keep the
  // heap and the arena in HBM scratch; a refresh per report was a long dependent walk).
  GWA_HD void refreshKeysFor(int changed) {
    if (!(S(changed).state & kStRef)) {
      // no state holds `changed` as its nextSplit: the chains through it are its own queue entries
      // (duplicates), found by index alone -- no arena reads, no chain walks
      uint64_t key = 0;
      int have = 0;
      for (int i = 0; i < heapSize; ++i) {
        const uint64_t e = hslot(i);
        if ((int)(e & IDXM) == changed) {
          if (!have) { key = keyOf(changed); have = 1; }
          hslot(i) = (key << KS) | (uint64_t)changed;
        }
      }
      return;
    }
    constexpr int U = 8;
    for (int i0 = 0; i0 < heapSize; i0 += U) {
      uint64_t e[U];
      int nx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) e[u] = i0 + u < heapSize ? hslot(i0 + u) : 0ULL;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = (int)(e[u] & IDXM);
        nx[u] = (i0 + u < heapSize && idx != changed) ? S(idx).nextSplit : -1;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i0 + u >= heapSize) continue;
        const int idx = (int)(e[u] & IDXM);
        int hit = idx == changed ? 1 : 0, t = nx[u];
        while (hit == 0 && t >= 0) {  // (single-exit loop: see quickScan)
          hit = t == changed ? 1 : 0;
          t = hit ? t : S(t).nextSplit;
        }
        if (hit) hslot(i0 + u) = (keyOf(idx) << KS) | (uint64_t)idx;
      }
    }
  }
  GWA_HD void refreshKeys() {
    for (int i = 0; i < heapSize; ++i) {
      const int idx = (int)(hslot(i) & IDXM);
      hslot(i) = (keyOf(idx) << KS) | (uint64_t)idx;
    }
  }
  // java.util.PriorityQueue.offer / poll on cached keys.  The element moves are exactly Java's
  // siftUp / siftDown; only the loads are reordered: offer reads the whole ancestor path (up to
  // 8 levels) at once, poll reads children and grandchildren together, so a heap operation waits
  // on memory once per 8 (offer) or 2 (poll) levels instead of once per level.
  GWA_HD void queueAddKeyed(uint64_t e) {
    if (heapSize >= caps.heap) { ovf(OV_HEAP); return; }
#ifdef GWA_HEAP_STATS
    maxHeap = heapSize + 1 > maxHeap ? heapSize + 1 : maxHeap;
#endif
    const int kk = heapSize++;
    const uint64_t ek = e >> KS;
    constexpr int MAXD = 8;
    uint64_t av[MAXD];
    int ai[MAXD];
    {
      int idx = kk;
#pragma unroll
      for (int d = 0; d < MAXD; ++d) {
        const int p = idx > 0 ? (idx - 1) >> 1 : 0;
        ai[d] = p;
        av[d] = hslot(p);
        idx = p;
      }
    }
    // Java's siftUp stops at the first ancestor d with ek >= key (the cached keys need not be
    // heap-ordered after a refresh, so this is a first-match, not a count).  Selects only: no
    // loop-carried flag (see quickScan).
    const int depth = 31 - __builtin_clz((unsigned)kk + 1u);
    int t = MAXD;
#pragma unroll
    for (int d = MAXD - 1; d >= 0; --d) t = (d >= depth || ek >= (av[d] >> KS)) ? d : t;
#pragma unroll
    for (int d = 0; d < MAXD; ++d)
      if (d < t) {
        const int w = d == 0 ? kk : ai[d - 1];
        if (d > 0) ulogHeap(w, av[d - 1]);
        hslot(w) = av[d];
      }
    int pos = t == 0 ? kk : pick(ai, t - 1);
    uint64_t cur = t == 0 ? 0ULL : pick(av, t - 1);  // the entry at pos (t > 0)
    if (t == MAXD) {  // deeper than MAXD levels (large tiers only): Java's loop from there
      while (pos > 0) {
        const int parent = (pos - 1) >> 1;
        const uint64_t p = hslot(parent);
        if (ek >= (p >> KS)) break;
        ulogHeap(pos, cur);
        hslot(pos) = p;
        pos = parent;
        cur = p;
      }
    }
    if (t > 0) ulogHeap(pos, cur);
    hslot(pos) = e;
    tr(9, (uint32_t)(e & IDXM), (uint32_t)kk, (uint32_t)pos);
  }
  GWA_HD int queuePoll() {
    if (heapSize == 0) return -1;
    int s = --heapSize;
    const uint64_t result = hslot(0);
    const uint64_t x = hslot(s);
    ulogHeap(s, x);  // (a later offer reuses the vacated slot)
    if (s != 0) {
      const int n = heapSize, half = n >> 1, capm1 = caps.heap - 1;
      int kk = 0;
      uint64_t cur = result;  // the entry at kk (the undo log's old value)
      const uint64_t xk = x >> KS;
      int go = kk < half;  // single-exit loop (no break): see quickScan
      while (go) {
        // children c0,c1 and grandchildren g0..g3 of kk (indices clamped into the array; entries
        // at or past n are never selected)
        const int c = (kk << 1) + 1;
        const int g = (kk << 2) + 3;
        const uint64_t c0 = hslot(c), c1 = hslot(c + 1 <= capm1 ? c + 1 : capm1);
        const uint64_t g0 = hslot(g <= capm1 ? g : capm1), g1 = hslot(g + 1 <= capm1 ? g + 1 : capm1);
        const uint64_t g2 = hslot(g + 2 <= capm1 ? g + 2 : capm1), g3 = hslot(g + 3 <= capm1 ? g + 3 : capm1);
        // level 1
        const int right = (c + 1 < n && (c0 >> KS) > (c1 >> KS)) ? 1 : 0;
        const uint64_t cv = right ? c1 : c0;
        if (xk <= (cv >> KS)) {
          go = 0;
        } else {
          ulogHeap(kk, cur);
          hslot(kk) = cv;
          cur = cv;
          kk = c + right;
          go = kk < half;
        }
        // level 2: the children of c are g0,g1, those of c+1 are g2,g3
        if (go) {
          const int c2 = (kk << 1) + 1;
          const uint64_t d0 = right ? g2 : g0, d1 = right ? g3 : g1;
          const int right2 = (c2 + 1 < n && (d0 >> KS) > (d1 >> KS)) ? 1 : 0;
          const uint64_t dv = right2 ? d1 : d0;
          if (xk <= (dv >> KS)) {
            go = 0;
          } else {
            ulogHeap(kk, cur);
            hslot(kk) = dv;
            cur = dv;
            kk = c2 + right2;
            go = kk < half;
          }
        }
      }
      ulogHeap(kk, cur);
      hslot(kk) = x;
    }
    tr(10, (uint32_t)(result & IDXM), (uint32_t)heapSize, (uint32_t)(x & IDXM));
    return (int)(result & IDXM);
  }
  GWA_HD void queueAdd(int e) {
    if (e < 0) return;
    queueAddKeyed((keyOf(e) << KS) | (uint64_t)e);
  }

  // ---- FMQuickScan.scanMismatchLocations (S/FMQuickScan.java:66-94) ----
  // uniq != 0: [lb, ub) is one row whose suffix-array value is tp (the FM steps ran in text mode)
  struct Scan { uint64_t lb, ub, tp; int numMismatches, lmStart, uniq, firstEmpty; };

  // One reference FM step from a single-row interval, read off the text instead of the Occ blocks.
  // For a one-row interval [l, l+1) with SA value p, backwardSearch(c) (A/FMIndexOnOccTable.java:47-51)
  // is non-empty iff BWT[l] == c, i.e. iff the cyclic text character before rotation p is c
  // (A/BWTransform.java:172-179), and the extended interval is again one row, with SA value p-1.
  // fm 0 indexes T, fm 1 indexes R = reverse(T), whose character R[p-1] is T[N-p]; both are
  // read from the 2-bit forward text (+ N bitmap), one word per 32 (64) steps.
  struct TextWalk {
    int64_t w2 = -1, wN = -1;
    uint64_t c2 = 0, cN = 0;
  };
  GWA_HD int textBefore(int fm, uint64_t p, TextWalk &tw) {
    const uint64_t N = ix.N;
    const uint64_t t = fm ? (p == 0 ? 0 : N - p) : (p == 0 ? N - 1 : p - 1);
    const int64_t a = (int64_t)(t >> 5), b = (int64_t)(t >> 6);
    if (a != tw.w2) { tw.c2 = ix.text2[a]; tw.w2 = a; }
    if (b != tw.wN) { tw.cN = ix.textN[b]; tw.wN = b; }
    return ((tw.cN >> (t & 63)) & 1) ? 4 : (int)((tw.c2 >> ((t & 31) * 2)) & 3);
  }

  // Up to 32 text-mode steps at once: the number of leading matches between the read's bases
  // q[strand][i, i + L) and the text characters the steps from SA value tp would read
  // (textBefore(fm, tp), textBefore(fm, tp - 1), ...), compared as 2-bit words (N never matches).
  // L is capped so the text positions do not wrap around the cyclic text.
  GWA_HD static uint64_t rev2(uint64_t x) {  // reverse the order of the 32 two-bit fields
    x = bitrev64(x);
    return ((x >> 1) & 0x5555555555555555ULL) | ((x & 0x5555555555555555ULL) << 1);
  }
  GWA_HD static uint32_t rev32(uint32_t x) {
#if defined(__clang__)
    return __builtin_bitreverse32(x);
#else
    return (uint32_t)(bitrev64((uint64_t)x) >> 32);
#endif
  }
  // 32 text codes from position s (2-bit fields) and their N flags; positions >= N read as 0
  GWA_HD void textWin(int64_t s, uint64_t *codes, uint32_t *nb) const {
    const int64_t last2 = (int64_t)((ix.N - 1) >> 5), lastN = (int64_t)((ix.N - 1) >> 6);
    const int64_t a = s >> 5, b = s >> 6;
    const int sa = (int)(s & 31) * 2, sn = (int)(s & 63);
    // the second N word only when the 32 flags cross into it (sn > 32): its bits land above bit 31
    // otherwise and the cast drops them
    const uint64_t a0 = ix.text2[a], a1 = (sa != 0 && a + 1 <= last2) ? ix.text2[a + 1] : 0ULL;
    const uint64_t n0 = ix.textN[b], n1 = (sn > 32 && b + 1 <= lastN) ? ix.textN[b + 1] : 0ULL;
    *codes = sa ? (a0 >> sa) | (a1 << (64 - sa)) : a0;
    *nb = (uint32_t)(sn ? (n0 >> sn) | (n1 << (64 - sn)) : n0);
  }
  GWA_HD int textRun(int fm, uint64_t tp, int strand, int i, int L) {
    const int64_t N = (int64_t)ix.N;
    uint64_t tw;
    uint32_t tn;
    if (fm) {  // T[N - tp], T[N - tp + 1], ...
      const int64_t t0 = tp == 0 ? 0 : N - (int64_t)tp;
      if (L > N - t0) L = (int)(N - t0);
      textWin(t0, &tw, &tn);
    } else {   // T[tp - 1], T[tp - 2], ...
      const int64_t t0 = tp == 0 ? N - 1 : (int64_t)tp - 1;
      if (L > t0 + 1) L = (int)(t0 + 1);
      if (t0 >= 31) {
        textWin(t0 - 31, &tw, &tn);
        tw = rev2(tw);
        tn = rev32(tn);
      } else {
        textWin(0, &tw, &tn);
        tw = rev2(tw << (2 * (31 - t0)));
        tn = rev32(tn << (31 - t0));
      }
    }
    const int w = i >> 5, sh = 2 * (i & 31);
    const uint64_t qa = strand ? pick(pw1, w) : pick(pw0, w);
    const uint64_t qb = (w + 1 < QW) ? (strand ? pick(pw1, w + 1) : pick(pw0, w + 1)) : 0ULL;
    const uint64_t rw = sh ? (qa >> sh) | (qb << (64 - sh)) : qa;
    const uint64_t x = tw ^ rw;
    const uint64_t nz = (x | (x >> 1)) & 0x5555555555555555ULL;
    const int j1 = nz ? __builtin_ctzll(nz) >> 1 : 32;
    const int j2 = tn ? __builtin_ctz(tn) : 32;
    const int j = j1 < j2 ? j1 : j2;
    return j < L ? j : L;
  }

  // One strand's FMQuickScan as a resumable loop: quickScan runs qsStep until qsMore is false; the
  // persistent quick-scan kernel runs one qsStep per lane per iteration, so a lane whose read is done
  // takes the next read instead of waiting for its wavefront's slowest scan (search_kernels.h).
  struct QS {
    uint64_t lb, ub, tp;
    // fe: the first empty step (the search-list sort key).  longestMatch bookkeeping kept branch-free
    // (loop-carried i1 flags in this divergent loop were mis-lowered by the gfx950 backend in our
    // tests); `have` is an int 0/1.  Text mode: once the interval is a single row [lb, lb + 1) with SA
    // value tp, each further step is one text character compare (textBefore), run 32 at a time by
    // textRun; uniq is an int 0/1 for the same reason as have.
    int i, mark, nmm, fe, have, lmS, lmE, uniq, strand;
  };
  GWA_HD void qsBegin(QS &s, int strand) const {
    s.lb = 0; s.ub = ix.N; s.tp = 0;
    s.i = 0; s.mark = 0; s.nmm = 0; s.fe = m; s.have = 0; s.lmS = 0; s.lmE = 0; s.uniq = 0; s.strand = strand;
  }
  // The scan stops at its (k+1)-th empty interval: the caller only reads numMismatches <= k and,
  // under that condition, longestMatch (S/BidirectionalSuffixFilter.java:324-345), so a scan past
  // k + 1 mismatches cannot change the result (the wrong strand of a read stops after ~3 restarts).
  GWA_HD bool qsMore(const QS &s) const { return s.i < m && s.nmm <= k; }
  GWA_HD void qsStep(QS &s) {
    const int strand = s.strand;
    const int fm = strand == 0 ? 1 : 0;  // forwardSearch on FORWARD uses the reverse index (:134-137)
    const uint64_t N = ix.N;
    const int K = ix.kmerK;
    // at a restart from [0, N) (mark == i), the k-mer table answers the next K steps at once
    // when none of them is empty; otherwise the steps below run one by one
    if (K > 0 && s.i == s.mark && s.i + K <= m) {
      const uint32_t key = qWindow(strand, s.i, K);
      const uint64_t e = ix.kmer[fm][key];
      ++kmerLookups;
      if (e != 0) {
        s.lb = e & 0xFFFFFFFFULL;
        s.ub = e >> 32;
        quickSteps += K;
        shortSteps += K;
        s.i += K;
        const int u = s.ub - s.lb == 1 ? 1 : 0;
        if (u) { s.tp = ix.sa[fm][s.lb]; ++saReads; }
        s.uniq = u;
        return;
      }
    }
    const int i = s.i;
    uint64_t nlb = s.lb, nub = s.ub;
    int empty;
    if (s.uniq) {
      const int L = m - i < 32 ? m - i : 32;
      const int j = textRun(fm, s.tp, strand, i, L);
      ++textRuns;
      s.tp = s.tp >= (uint64_t)j ? s.tp - j : s.tp + N - j;  // j hits, each moving to SA value tp - 1 (cyclic)
      s.i += j;
      quickSteps += j;
      shortSteps += j;
      if (j == L) return;
      ++quickSteps;  // the step at i: BWT character != read base, empty interval
      ++shortSteps;
      empty = 1;
    } else {
      const int ch = q(strand, i);
      // backwardSearch(ch, si) = C[ch] + getOcc(ch, lb|ub) (A/FMIndexOnOccTable.java:47-51);
      // one 64-B block when lb and ub share a 128-position window
      Block B;
      loadBlock(ix.occ[fm], s.lb >> 7, B);
      ++blocks;
      nlb = ix.C[ch] + rankOne(B, s.lb, ch);
      if ((s.ub >> 7) != (s.lb >> 7)) {
        loadBlock(ix.occ[fm], s.ub >> 7, B);
        ++blocks;
      }
      nub = ix.C[ch] + rankOne(B, s.ub, ch);
      ++quickSteps;
      tr(16 + strand, (uint32_t)(i | (ch << 16)), (uint32_t)nlb, (uint32_t)nub);
      empty = nlb >= nub ? 1 : 0;
      if (!empty && nub - nlb == 1) { s.tp = ix.sa[fm][nlb]; ++saReads; s.uniq = 1; }
    }
    const int ii = s.i;  // (the text branch moved i past its matches to the empty step)
    const int better = empty & ((s.have ^ 1) | ((s.lmE - s.lmS) < (ii - s.mark) ? 1 : 0));
    s.lmS = better ? s.mark : s.lmS;
    s.lmE = better ? ii : s.lmE;
    s.have |= empty;
    s.fe = (empty && s.nmm == 0) ? ii : s.fe;
    s.nmm += empty;
    s.lb = empty ? 0 : nlb;
    s.ub = empty ? N : nub;
    s.mark = empty ? ii + 1 : s.mark;
    s.uniq = empty ? 0 : s.uniq;
    s.i = ii + 1;
  }
  GWA_HD Scan qsEnd(const QS &s) const {
    const int better = (s.have ^ 1) | ((s.lmE - s.lmS) < (s.i - s.mark) ? 1 : 0);
    Scan r;
    r.lb = s.lb; r.ub = s.ub; r.tp = s.tp; r.numMismatches = s.nmm; r.lmStart = better ? s.mark : s.lmS; r.uniq = s.uniq;
    r.firstEmpty = s.fe;
    return r;
  }
  GWA_HD Scan quickScan(int strand) {
    QS s;
    qsBegin(s, strand);
    while (qsMore(s)) qsStep(s);
    return qsEnd(s);
  }

  // ---- hits (R/ReadHit.java) ----
  GWA_HD int newHit(int32_t chr, int32_t pos, int ml, int qs, int qe, int diff, int strand, int cigOff, int cigLen, int numHits) {
    if (nHits >= caps.hits) { ovf(OV_HITS); return -1; }
    GWA_PW(PR_WH, PR_EH, sizeof(DHit));
    DHit &h = L.hits()[nHits];
    h.chr = chr; h.pos = pos; h.matchLength = ml; h.qStart = qs; h.qEnd = qe; h.diff = diff; h.strand = strand;
    h.numHits = numHits; h.next = -1; h.cigarOff = cigOff; h.cigarLen = cigLen; h.pad = 0;
    return nHits++;
  }
  GWA_HD int putCigarOp(int type, int len) {
    if (nCigar >= caps.cigar) { ovf(OV_CIGAR); return -1; }
    GWA_PW(PR_WH, PR_EH, 2);
    L.cigar()[nCigar++] = (uint16_t)((len << 3) | type);
    return 0;
  }
  GWA_HD int hitTotalDiff(int h) {
    int d = 0;
    for (int t = h; t >= 0; t = L.hits()[t].next) d += L.hits()[t].diff + (L.hits()[t].next >= 0 ? 1 : 0);
    return d;
  }
  GWA_HD int hitTotalMatch(int h) {
    int d = 0;
    for (int t = h; t >= 0; t = L.hits()[t].next) d += L.hits()[t].matchLength;
    return d;
  }
  GWA_HD int hitTotalScore(int h) {
    int sc = 0;
    for (int t = h; t >= 0; t = L.hits()[t].next) {
      const DHit &x = L.hits()[t];
      sc += x.matchLength * cfg.matchScore - x.diff * cfg.mismatchPenalty;
      if (x.next >= 0) sc -= cfg.splitOpenPenalty;
    }
    return sc;
  }
  // AlignmentResultHolder.add (:606-628).  The filter keeps the entries with totalDifferences <=
  // minMismatches and totalMatchLength >= maxMatchLength; both thresholds only tighten and a listed
  // chain never changes, so when neither moved since the last add, the entries that passed then
  // (the first listOk) pass again and only the ones appended after it are tested: the same list,
  // without a chain walk per entry per report (lists of equal hits in repeats reach thousands).
  int listOk = 0;
  GWA_HD void resultAdd(int hit) {
    int newK = hitTotalDiff(hit);
    int matchLen = hitTotalMatch(hit);
    int newScore = hitTotalScore(hit);
    const int mm0 = minMismatches, ml0 = maxMatchLength;
    if (newScore > bestScore) {
      if (matchLen > 0 && newK <= minMismatches) minMismatches = newK;
      bestScore = newScore;
    }
    if (maxMatchLength < matchLen) maxMatchLength = matchLen;
    const int keep = (minMismatches == mm0 && maxMatchLength == ml0) ? listOk : 0;
    int n = keep;
    for (int i = keep; i < listSize; ++i) {
      int e = L.list()[i];
      if (hitTotalDiff(e) <= minMismatches && hitTotalMatch(e) >= maxMatchLength) { GWA_PW(PR_WH, PR_EH, 4); L.list()[n++] = e; }
    }
    listOk = n;
    if (n >= caps.list) { ovf(OV_LIST); listSize = n; return; }
    GWA_PW(PR_WH, PR_EH, 4);
    L.list()[n++] = hit;
    listSize = n;
  }

  // ReadHit.sortSplits (R/ReadHit.java:148-182): stable insertion sort of the chain
  GWA_HD int sortSplits(int head) {
    if (L.hits()[head].next < 0) return head;
    int arr[8];
    int n = 0;
    for (int t = head; t >= 0; t = L.hits()[t].next) {
      if (n >= 8) { ovf(OV_CHAIN); return head; }
      arr[n++] = t;
    }
    const int headStrand = L.hits()[head].strand;
    for (int i = 1; i < n; ++i) {
      int x = arr[i];
      int j = i - 1;
      while (j >= 0) {
        int c = cmpHit(arr[j], x, headStrand);
        if (status == ST_ERROR) return head;
        if (c <= 0) break;
        arr[j + 1] = arr[j];
        --j;
      }
      arr[j + 1] = x;
    }
    GWA_PW(PR_WH, PR_EH, 4 * n);
    for (int i = 0; i + 1 < n; ++i) L.hits()[arr[i]].next = arr[i + 1];
    L.hits()[arr[n - 1]].next = -1;
    return arr[0];
  }
  GWA_HD int cmpHit(int a, int b, int headStrand) {
    const DHit &o1 = L.hits()[a];
    const DHit &o2 = L.hits()[b];
    int diff = 0;
    if (o1.chr == CHR_NULL || o2.chr == CHR_NULL) {
      diff = o1.qStart - o2.qStart;
      if (headStrand != 0) diff = -diff;
    }
    if (diff != 0) return diff;
    if (o1.chr == CHR_NULL || o2.chr == CHR_NULL) { status = ST_ERROR; return 0; }  // NullPointerException
    // chr.compareTo: contig names are compared through their precomputed lexicographic rank
    diff = chrRankCmp(o1.chr, o2.chr);
    if (diff != 0) return diff;
    return (int)((int64_t)o1.pos - (int64_t)o2.pos);
  }
  const int32_t *chrRank = nullptr;  // lexicographic (String.compareTo) rank of each contig name
  GWA_HD int chrRankCmp(int a, int b) const {
    auto rk = [&](int c) -> int { return c >= 0 ? chrRank[c] : (c == CHR_EMPTY ? -1 : -2); };
    return rk(a) - rk(b);
  }

  // ---- BitParallelSmithWaterman.alignBlockDetailed (A/BitParallelSmithWaterman.java:141-147,335-644) ----
  // query = q[strand][qs,qe) (reversed for strand 1), ref = T[refStart, refEnd)
  // a one-word cache of the 2-bit text and of the N bitmap for the text-mode FM steps (nextSi)
  int64_t tcW2 = -1, tcWN = -1;
  uint64_t tcC2 = 0, tcCN = 0;
  GWA_HD int refCode(int64_t p) const {
    uint64_t nb = ix.textN[p >> 6];
    if ((nb >> (p & 63)) & 1) return 4;
    return (int)((ix.text2[p >> 5] >> ((p & 31) * 2)) & 3);
  }

  // One Myers/Hyyro block step (A/BitParallelSmithWaterman.java:476-504); vp/vn in/out
  GWA_HD static int dpBlock(uint64_t x, int hin, uint64_t &vp, uint64_t &vn) {
    if (hin < 0) x |= 1ULL;
    const uint64_t d0 = (((x & vp) + vp) ^ vp) | x | vn;
    const uint64_t hp = vn | ~(d0 | vp);
    const uint64_t hn = d0 & vp;
    const int hout = (int)((hp >> 63) & 1ULL) - (int)((hn >> 63) & 1ULL);
    uint64_t hp2 = hp << 1, hn2 = hn << 1;
    if (hin < 0) hn2 |= 1ULL;
    if (hin > 0) hp2 |= 1ULL;
    vp = hn2 | ~(d0 | hp2);
    vn = d0 & hp2;
    return hout;
  }

  // BitParallelSmithWaterman.alignBlockDetailed (A/BitParallelSmithWaterman.java:141-147,394-644).
  // The live column (<= DB blocks of 64 rows) stays in VGPRs; the history the traceback reads is
  // kept in the lane's interleaved DP area (64 lanes of a wavefront adjacent per word) as column
  // checkpoints or, in the first tier's k >= 4 kernel, a 32-row slice per column (DPM, below).
  // bits [lo, lo + 32) of a DP column of DB blocks (rows outside [0, 64 DB) read as 0)
  GWA_HD static uint32_t rows32(const uint64_t (&E)[DB], int lo) {
    const int w = lo >> 6, sh = lo & 63;  // lo < 0: w = -1
    const uint64_t a = w >= 0 && w < DB ? pick(E, w) : 0ULL;
    const uint64_t b = w + 1 >= 0 && w + 1 < DB ? pick(E, w + 1) : 0ULL;
    return (uint32_t)((a >> sh) | (sh ? b << (64 - sh) : 0ULL));
  }
  // Peq of the DP query (the fragment q[strand][qs, qe), reversed on strand 1, :532-534) for block r
  // and base ch: bit j = (query[64 r + j] == ch), from the 2-bit read words (eqWindow), not per base
  GWA_HD uint64_t dpPeq(int strand, int qs, int qe, int r, int ch) const {
    const int mq = qe - qs, rows = mq - 64 * r;
    uint64_t x;
    if (strand == 0) {
      x = eqWindow(0, ch, qs + 64 * r);
    } else {
      const int len = qe - 64 * r;  // positions [0, len) of strand 1 precede this block's first row
      x = len >= 64 ? bitrev64(eqWindow(1, ch, len - 64)) : bitrev64(eqWindow(1, ch, 0) << (64 - len));
    }
    return rows >= 64 ? x : (x & ((1ULL << rows) - 1ULL));
  }
  // returns 0 ok, 1 null (no alignment), <0 overflow
  // cgOver / capOver: the CIGAR area and its capacity, when not the lane's own (the helper lanes of
  // the cooperative -m sf kernel, whose slice is the owner's)
  GWA_HD int alignBlockDetailed(int strand, int qs, int qe, int64_t refStart, int64_t refEnd, int *outPos, int *outDiff,
                                int *cigOff, int *cigLen, uint16_t *cgOver = nullptr, int capOver = 0) {
    const int w = 64;
    const int mq = qe - qs;
    const int kb = cfg.bandWidth;
    const int bMax = mq + w - 1 >= w ? (mq + w - 1) / w : 1;
    const int N = (int)(refEnd - refStart);
    ++numSW;
    verifyBytes += (2 * N + 7) / 8 + (N + 7) / 8 + 32 * bMax;
#if defined(GWA_VERIFY_LOG) && !defined(__HIP_DEVICE_COMPILE__)
    if (FILE *vf = gwaVerifyLog()) { fprintf(vf, "V %d %d %d %d %lld %lld\n", caps.hits, strand, qs, qe, (long long)refStart, (long long)refEnd); fflush(vf); }
#endif
    if (bMax > DB || (size_t)2 * bMax * (N + 1) > (size_t)caps.dpWords) { ovf(OV_DP); return -1; }
    uint64_t pA[DB], pC[DB], pG[DB], pT[DB];
#pragma unroll
    for (int r = 0; r < DB; ++r) {
      const bool on = r < bMax;
      pA[r] = on ? dpPeq(strand, qs, qe, r, 0) : 0ULL;
      pC[r] = on ? dpPeq(strand, qs, qe, r, 1) : 0ULL;
      pG[r] = on ? dpPeq(strand, qs, qe, r, 2) : 0ULL;
      pT[r] = on ? dpPeq(strand, qs, qe, r, 3) : 0ULL;
    }
    const size_t is = (size_t)L.is;
    uint64_t vp[DB], vn[DB];
    int D[DB] = {}, sb[DB];
#pragma unroll
    for (int r = 0; r < DB; ++r) {
      vp[r] = ~0ULL;
      vn[r] = 0;
      const int v = mq - ((r + 1) * w) + kb;
      sb[r] = v > 0 ? v : 0;
    }
    D[0] = mq;
    int bCeil = (kb + w - 1) / w;
    if (bCeil < 1) bCeil = 1;
    int have = 0;  // int, not bool: see quickScan
    int bestTail = 0, bestDiff = 0;
    // the window: N <= m + 2k + 2 <= 32 QW + 64 bases
    RefWindow<QW + 2, QW / 2 + 1> rw;
    if (N > 32 * (QW + 2)) { ovf(OV_DP); return -1; }
    rw.load(ix.text2, ix.textN, ix.N, refStart);
    // One column of the pass (:420-473) for reference code ch: the blocks are computed with selects,
    // not divergent branches; blocks past bCeil give values nobody reads, except block bCeil, whose
    // input is set to ~0 / 0 first -- if it is activated at this column (:427-428) its carry-in is
    // that of the active blocks above it, as there.  Blocks from 2 on are skipped (uniform branch) when
    // no lane of the wavefront needs them.  Afterwards the blocks not computed here are zeroed (what
    // the reference's zero-initialised history holds for them).  Returns the block activated with
    // this column as its input, or -1.
    auto column = [&](int ch, uint64_t (&cp)[DB], uint64_t (&cn)[DB], int (&cD)[DB], int &cb) -> int {
      int carry = 0, cIn = 0, nsC = 0;
      uint64_t nextPeq = 0;
#pragma unroll
      for (int r = 0; r < DB; ++r) {
        int ns = 0;
        if (r < 2 || anyLane(r <= cb && r < bMax)) {
          if (r == cb) { cp[r] = ~0ULL; cn[r] = 0ULL; }
          const uint64_t xr = ch == 0 ? pA[r] : ch == 1 ? pC[r] : ch == 2 ? pG[r] : ch == 3 ? pT[r] : 0ULL;
          const int hin = carry;
          ns = dpBlock(xr, hin, cp[r], cn[r]);
          if (r < cb) cD[r] += ns;
          if (r == cb) { cIn = hin; nsC = ns; nextPeq = xr; }  // hin = ns of block cb - 1
        }
        carry = ns;
      }
      const int bOld = cb;
      const int dPrev = pick(cD, cb - 1);
      const int act = cb < bMax && dPrev - cIn <= pick(sb, cb - 1) && (((nextPeq & 1ULL) != 0ULL) || cIn < 0);
      const int actBlock = act ? cb : -1;
#pragma unroll
      for (int r = 0; r < DB; ++r) {
        if (r == actBlock) cD[r] = dPrev - cIn + nsC;
        if (!(r < bOld || r == actBlock)) { cp[r] = 0ULL; cn[r] = 0ULL; }  // not computed at this column
      }
      if (act) {
        cb++;
      } else {
#pragma unroll
        for (int q = 0; q < DB - 1; ++q)
          if (cb > 1 && pick(cD, cb - 1) > pick(sb, cb - 1) + w) --cb;
      }
      return actBlock;
    };
    // No per-column history: every kCk columns the pass keeps its state (vp / vn of every block, the
    // block scores, the active block count) as a checkpoint, element e of this lane's interleaved area
    // at chunk[e * is + lane]; the traceback recomputes the column an edit needs from the checkpoint at
    // or before it (below).  ~6 words per 16 columns instead of one word per column (first tier) or
    // 16 B per block per column (deeper tiers), and no traceback ever leaves the kept rows.
    // DPM 1 with more than two blocks: one word per column instead, rows [lo, lo + 32) of column j + 1
    // with lo = j - c0 - 16 -- the diagonal band a k <= 15 traceback of a first-tier read stays in;
    // one that leaves it overflows (OV_SLICE: laneReport rolls the report back and the read resumes
    // on the next tier, whose kernel keeps checkpoints).  Activated rows (~0 / 0) are patched into
    // the previous column's word.
    constexpr bool kSlice = DPM == 1 && DB > 2;
    constexpr bool kHist = DPM == 2;
    struct alignas(16) VpVn { uint64_t vp, vn; };
    VpVn *hist = (VpVn *)L.chunk + L.lane;  // DPM 2: {vp, vn} of block b of column c at [(c * bMax + b) * is]
    const int c0 = ((N - mq) >> 1) + (caps.dpSlice > 0 ? caps.dpSlice - 1 : 0);
    uint64_t *h8 = (uint64_t *)L.chunk + L.lane;
    uint64_t lastWord = 0;
    constexpr int kCk = 16, kCw = 2 * DB + (DB + 2) / 2;  // checkpoint words
    uint64_t *ckBase = (uint64_t *)L.chunk + L.lane;
    if (!kSlice && !kHist && (size_t)((N + kCk - 1) / kCk + 1) * kCw > (size_t)caps.dpWords) { ovf(OV_DP); return -1; }
    auto ckStore = [&](int t) {
      uint64_t *e = ckBase + (size_t)t * kCw * is;
#pragma unroll
      for (int r = 0; r < DB; ++r)
        if (r < bMax) { e[(2 * r) * is] = vp[r]; e[(2 * r + 1) * is] = vn[r]; }
#pragma unroll
      for (int r = 0; r <= DB; r += 2) {
        const uint32_t a = (uint32_t)(r < DB ? D[r] : bCeil);
        const uint32_t b2 = (uint32_t)(r + 1 < DB ? D[r + 1] : r + 1 == DB ? bCeil : 0);
        e[(2 * DB + r / 2) * is] = (uint64_t)a | ((uint64_t)b2 << 32);
      }
      GWA_PW(PR_WD, PR_ED, 8 * (2 * bMax + (DB + 2) / 2));
      GWA_PC(PR_EDW, PR_N - 2);
    };
    GWA_PT(tdf);
    uint64_t run2 = 0, runN = 0;  // the window's codes from column j on (the loop index is uniform)
    for (int j = 0; j < N; ++j) {
      if ((j & 31) == 0) run2 = pick(rw.c2, j >> 5);
      if ((j & 63) == 0) runN = pick(rw.cn, j >> 6);
      const int ch = (runN & 1ULL) ? 4 : (int)(run2 & 3ULL);
      run2 >>= 2;
      runN >>= 1;
      if (!kSlice && !kHist && (j & (kCk - 1)) == 0) ckStore(j / kCk);  // the state entering column j
      const int actBlock = column(ch, vp, vn, D, bCeil);
      if (kHist) {  // column j + 1; a block activated with input column j reads ~0 / 0 there
        VpVn *hc = hist + (size_t)j * bMax * is;
        if (actBlock >= 0) hc[(size_t)actBlock * is] = VpVn{~0ULL, 0ULL};
#pragma unroll
        for (int r = 0; r < DB; ++r)
          if (r < bMax) hc[((size_t)bMax + r) * is] = VpVn{vp[r], vn[r]};
        GWA_PW(PR_WD, PR_ED, 16 * bMax);
      }
      if (kSlice) {
        uint64_t *hc8 = h8 + (size_t)j * is;
        if (actBlock >= 0) {
          const int lo = j - c0 - 17, r0 = 64 * actBlock - lo, r1 = r0 + 64;
          const int s0 = r0 < 0 ? 0 : r0 > 32 ? 32 : r0, s1 = r1 < 0 ? 0 : r1 > 32 ? 32 : r1;
          const uint64_t msk = ((s1 >= 32 ? 0xFFFFFFFFULL : (1ULL << s1) - 1ULL) & ~((1ULL << s0) - 1ULL));
          *hc8 = (lastWord | msk) & ~(msk << 32);
        }
        const int lo1 = j - c0 - 16;
        lastWord = (uint64_t)rows32(vp, lo1) | ((uint64_t)rows32(vn, lo1) << 32);
        hc8[is] = lastWord;
        GWA_PW(PR_WD, PR_ED, 8);
      }
      if (bCeil == bMax) {
        const int dl = pick(D, bCeil - 1);
        if (!have) { have = 1; bestTail = j; bestDiff = dl; continue; }
        if (bestDiff > dl) { bestTail = j; bestDiff = dl; }
      }
    }
    GWA_PA(PR_DPF, tdf);
    (void)bestDiff;
    if (!have) return 1;
    GWA_PT(tdt);
    // Traceback (:515-643).  A match decides the step from the codes alone (:547), so the history is
    // read only at edits: each round walks a lane's run of matches up its diagonal, then takes one
    // edit step, so the lanes of a wavefront issue their history reads together (one memory latency
    // per round, not per step).  The path is generated backwards (CIGAR end first) and run-length
    // encoded as it goes -- no path array: S/I/D before the first M are the trailing soft clip
    // (`right`), S/I/D after the last M the leading one (`left`); the runs in between are kept
    // (generation order) at the top of this read's CIGAR area, CIGAR entry cap-1-i = run i.  The ops
    // then come out as cigarStr = reverse(path) + CIGAR.add merging would make them (:599-643).
    uint16_t *cg = cgOver ? cgOver : L.cigar();
    const int cap = cgOver ? capOver : caps.cigar;
    int row = mq - 1, col = bestTail;
    int diff = 0, leftMostPos = 0;
    int right = 0, adj = 0;  // trailing S/I/D count, of which I/D
    int seenM = 0, curT = 0, curL = 0, nRuns = 0, lastM = 0, pendL = 0, pendAdj = 0;
    int bad = 0;
    // path char t (0 M, 1 I, 2 D, 4 S), cnt of them
    auto emit = [&](int t, int cnt) {
      if (cnt <= 0) return;
      if (!seenM) {
        if (t == 0) { seenM = 1; curT = 0; curL = cnt; lastM = 0; }
        else { right += cnt; adj += (t == 1 || t == 2) ? 1 : 0; }
      } else {
        if (t == curT) {
          curL += cnt;
        } else {
          if (nCigar + 2 * nRuns + 4 > cap) bad = 1;
          else { GWA_PW(PR_WH, PR_EH, 2); cg[cap - 1 - nRuns] = (uint16_t)((curL << 3) | curT); }
          ++nRuns;
          curT = t;
          curL = cnt;
        }
        if (t == 0) { lastM = nRuns; pendL = 0; pendAdj = 0; }
        else { pendL += cnt; pendAdj += (t == 1 || t == 2) ? 1 : 0; }
      }
    };
    for (;;) {
      // the run of matches up the diagonal, 32 cells per pass: the reference codes at col - t and
      // the query codes at row - t (t = 0..31) as 2-bit words, XOR, first nonzero field (a
      // reference N never matches).  Query row i is read position qs + i on strand 0 and qe - 1 - i
      // on strand 1 (dpPeq).
      int runLen = 0;
      int go = col >= 0 && row >= 0;
      while (go) {
        uint64_t rc;
        uint32_t rn;
        rw.window32(col - 31, &rc, &rn);
        rc = rev2(rc);
        rn = rev32(rn);
        const uint64_t qc = strand == 0 ? rev2(qcodes32(0, qs + row - 31)) : qcodes32(1, qe - 1 - row);
        const uint64_t x = rc ^ qc;
        const uint64_t nz = (x | (x >> 1)) & 0x5555555555555555ULL;
        const int t1 = nz ? __builtin_ctzll(nz) >> 1 : 32;
        const int t2 = rn ? __builtin_ctz(rn) : 32;
        const int lim = (row < col ? row : col) + 1;
        int t = t1 < t2 ? t1 : t2;
        t = t < lim ? t : lim;
        runLen += t;
        col -= t;
        row -= t;
        go = t == 32 && col >= 0 && row >= 0;
      }
      if (runLen > 0) {
        leftMostPos = col + 1;
        emit(0, runLen);
      }
      if (col >= 0 && row >= 0) {
        // the history the reference holds for column c = col + 1 (:532-546), recomputed: the value
        // column c - 1 computed, unless the block of this row was activated with input column c
        // (then ~0 / 0), from the checkpoint at or before column c - 1
        int bp = 0, bn = 0;
        if (kSlice) {
          const int rr = row - (col + 1 - c0 - 17);
          if (rr < 0 || rr >= 32) { ovf(OV_SLICE); return -1; }
          const uint64_t h = h8[(size_t)(col + 1) * is];
          bp = (int)(h >> rr) & 1;
          bn = (int)(h >> (32 + rr)) & 1;
        } else if (kHist) {
          const VpVn h = hist[((size_t)(col + 1) * bMax + (row >> 6)) * is];
          bp = (int)(h.vp >> (row & 63)) & 1;
          bn = (int)(h.vn >> (row & 63)) & 1;
        } else {
          const int c = col + 1, block = row >> 6, offset = row & 63;
          const int t = (c - 1) / kCk;
          uint64_t rp[DB], rn[DB];
          int rD[DB], rb;
          const uint64_t *e = ckBase + (size_t)t * kCw * is;
#pragma unroll
          for (int r = 0; r < DB; ++r) {
            rp[r] = r < bMax ? e[(2 * r) * is] : 0ULL;
            rn[r] = r < bMax ? e[(2 * r + 1) * is] : 0ULL;
          }
#pragma unroll
          for (int r = 0; r <= DB; r += 2) {
            const uint64_t x = e[(2 * DB + r / 2) * is];
            if (r < DB) rD[r] = (int)(uint32_t)x;
            else rb = (int)(uint32_t)x;
            if (r + 1 < DB) rD[r + 1] = (int)(uint32_t)(x >> 32);
            else if (r + 1 == DB) rb = (int)(uint32_t)(x >> 32);
          }
          for (int j = t * kCk; j < c; ++j) column(rw.code(j), rp, rn, rD, rb);
          uint64_t hp = pick(rp, block), hn = pick(rn, block);
          if (c < N && column(rw.code(c), rp, rn, rD, rb) == block) { hp = ~0ULL; hn = 0ULL; }
          bp = (int)(hp >> offset) & 1;
          bn = (int)(hn >> offset) & 1;
        }
        const int t = bp ? 1 : bn == 0 ? 0 : 2;
        diff++;
        if (t == 0) { leftMostPos = col; col--; row--; }
        else if (t == 1) { leftMostPos = col + 1; row--; }
        else { col--; }
        emit(t, 1);
      } else {
        // NONE: the remaining rows become S (:588-597)
        emit(4, row >= 0 ? row + 1 : 0);
        break;
      }
    }
    if (bad) { ovf(OV_CIGAR); return -1; }
    GWA_PA(PR_DPT, tdt);
    const int off = nCigar;
    auto put = [&](int type, int len) -> int {  // putCigarOp on this DP's CIGAR area
      if (nCigar >= cap) { ovf(OV_CIGAR); return -1; }
      GWA_PW(PR_WH, PR_EH, 2);
      cg[nCigar++] = (uint16_t)((len << 3) | type);
      return 0;
    };
    if (!seenM) {
      diff -= adj;  // the whole path is the leading clip (left = plen, right = 0)
      if (right > 0 && put(4, right) < 0) return -1;
    } else {
      if (nCigar + 2 * nRuns + 4 > cap) { ovf(OV_CIGAR); return -1; }
      cg[cap - 1 - nRuns] = (uint16_t)((curL << 3) | curT);
      GWA_PW(PR_WH, PR_EH, 2 * (lastM + 2));
      diff -= adj + pendAdj;
      if (pendL > 0 && put(4, pendL) < 0) return -1;
      for (int i = lastM; i >= 0; --i) cg[nCigar++] = cg[cap - 1 - i];
      if (right > 0 && put(4, right) < 0) return -1;
    }
    *cigOff = off;
    *cigLen = nCigar - off;
    *outPos = leftMostPos;
    *outDiff = diff;
    return 0;
  }

  // ---- verify (:496-560); returns hit index, -1 = Java null, -2 = overflow ----
  GWA_HD int verify(int s) {
    const DState<R> d = S(s);
    const int strand = cStrand(d);
    if (isClipped(s)) {
      int off = nCigar;
      if (putCigarOp(4, cFrag(d)) < 0) return -2;
      int h = newHit(CHR_NULL, -1, 0, d.start, d.end, 0, strand, off, 1, 0);
      return h < 0 ? -2 : h;
    }
    if (!(d.meta & M_CURVALID)) {
      int h = newHit(CHR_EMPTY, 0, 0, 0, 0, 0, strand, nCigar, 0, 0);  // ReadHit.noHit
      return h < 0 ? -2 : h;
    }
    // FMIndexOnGenome.toCoordinate (A/FMIndexOnGenome.java:227-238) via the full SA; in text mode
    // the SA value of the one row on side fm follows from the occurrence (t, |P|) directly
    const int fm = ~(strand ^ (cFwd(d) ? 0 : 1)) & 1;
    int64_t seqIndex;
    if (siText(d)) {
      const int64_t N = (int64_t)ix.N;
      int64_t v = (int64_t)d.lb[0];
      if (fm == 1) {
        v = N - v - (int64_t)d.lb[1];
        v = v < 0 ? v + N : v;
      }
      seqIndex = fm == 0 ? v : N - v;
    } else {
      seqIndex = fm == 0 ? (int64_t)ix.sa[0][d.curLb] : (int64_t)ix.N - (int64_t)ix.sa[1][d.curLb];
      ++saReads;
    }
    int64_t x = seqIndex - cOffsetOfSearchHead(d);
    const int frag = cFrag(d);
    int64_t refStart = x - k > 0 ? x - k : 0;
    int64_t refEnd = x + frag + k < (int64_t)ix.N ? x + frag + k : (int64_t)ix.N;
    if (refStart > refEnd) { status = ST_ERROR; return -2; }  // IllegalArgumentException in subString
    // Verification memo (caps.cand > 0: the k >= 4 kernels).  The DP's result -- position, edit
    // count, CIGAR -- is a function of (strand, query fragment, reference window) alone, and a read
    // with indels verifies the same window again and again through different split chains (C4: 37 %
    // of the verifications repeat one of the same read).  A hit made from an unclamped window keeps
    // refStart + 1 in its pad word, and a small direct-mapped table of the lane's slice points at
    // the newest such hit per slot; a repeat copies that hit (sharing its CIGAR ops, which are never
    // changed once written) instead of running the DP again.  Stale slots from earlier reads are
    // harmless: a slot counts only if its hit index is below nHits and the hit's key matches, and
    // then it IS this read's result for that window.  numSW / verifyBytes count every call, as the
    // reference runs the DP every time.  (The key refStart + 1 is exact: the host refuses texts of
    // 2^32 - 1 bases or more, gwa_api.cpp checkSize, so refStart + 1 < 2^32.)
    const bool memo = caps.cand > 0 && refStart > 0 && refEnd < (int64_t)ix.N;
    const uint32_t mkey = (uint32_t)refStart + 1u;
    uint32_t mslot = 0;
    if (memo) {
      mslot = ((mkey * 0x9E3779B1u) ^ ((uint32_t)d.start * 0x85EBCA6Bu) ^ ((uint32_t)d.end << 7) ^ (uint32_t)strand) &
              (uint32_t)(caps.cand - 1);
      const int hi = (int)(uint32_t)L.cand()[mslot] - 1;
      if (hi >= 0 && hi < nHits) {
        const DHit hh = L.hits()[hi];
        if ((uint32_t)hh.pad == mkey && hh.strand == strand && hh.qStart == (int)d.start && hh.qEnd == (int)d.end) {
          const int N = (int)(refEnd - refStart), mq = (int)d.end - (int)d.start;
          const int bMax = mq + 63 >= 64 ? (mq + 63) / 64 : 1;
          ++numSW;
          verifyBytes += (2 * N + 7) / 8 + (N + 7) / 8 + 32 * bMax;
          const int h = newHit(hh.chr, hh.pos, frag, d.start, d.end, hh.diff, strand, hh.cigarOff, hh.cigarLen,
                               (int)(d.curUb - d.curLb));
          if (h < 0) return -2;
          L.hits()[h].pad = (int32_t)mkey;
          return h;
        }
      }
    }
    int pos = 0, diff = 0, co = 0, cl = 0;
    GWA_PT(tv);
    GWA_PC(PR_NVW, PR_NVL);
    int r = alignBlockDetailed(strand, d.start, d.end, refStart, refEnd, &pos, &diff, &co, &cl);
    GWA_PA(PR_VERIFY, tv);
    tr(7, (uint32_t)refStart, (uint32_t)(r == 0 ? pos : -1), (uint32_t)(diff | (cl << 16)));
    if (r < 0) return -2;
    if (r == 1) {
      int h = newHit(CHR_EMPTY, 0, 0, 0, 0, 0, strand, nCigar, 0, 0);
      return h < 0 ? -2 : h;
    }
    int32_t chr, p;
    if (translate(refStart + pos + 1, &chr, &p) != 0) return -1;
    int h = newHit(chr, p, frag, d.start, d.end, diff, strand, co, cl, (int)(d.curUb - d.curLb));
    if (h < 0) return -2;
    if (memo) {
      GWA_PW(PR_WH, PR_EH, 12);
      L.hits()[h].pad = (int32_t)mkey;
      L.cand()[mslot] = (int64_t)(h + 1);
    }
    return h;
  }

  // reportAlignment (:562-586); returns false on overflow/error
  GWA_HD bool reportAlignment(int c) {
    // one verify call site (the DP is large): member 0 is the chain head, the rest hang off it
    int al = -1;
    for (int nx = c, first = 1; nx >= 0; nx = S(nx).nextSplit, first = 0) {
      const int res = verify(nx);
      if (res == -2) return false;
      if (first) { al = res; continue; }
      if (al < 0) { status = ST_ERROR; return false; }
      GWA_PW(PR_WH, PR_EH, 4);
      L.hits()[al].next = res;  // nextHit is never advanced (:567-571)
    }
    if (al < 0) { status = ST_ERROR; return false; }
    tr(8, (uint32_t)c, (uint32_t)hitTotalMatch(al), (uint32_t)hitTotalDiff(al));
    if (hitTotalMatch(al) == 0) return true;
    int newK = hitTotalDiff(al);
    if (newK > k) return true;
    setMinK(c, newK);
    refreshKeysFor(c);  // c may still be queued (duplicate references), and chains through it
    int head = sortSplits(al);
    if (status == ST_ERROR || status == ST_OVERFLOW) return false;
    resultAdd(head);
    return status != ST_OVERFLOW;
  }

  // ---- ReadAlignmentNFA.nextState (S/ReadAlignmentNFA.java:127-203) ----
  // returns: -1 null, else (hasMatch, new rows/kOffset written into out)
  GWA_HD bool nfaNext(const DState<R> &s, int ch, int strand, uint64_t (&outRows)[R], int *outH, int *outKOff, bool *hasMatch) {
    const int height = s.nrows;
    const int kOff = s.kOffset;
    const int kr = height - 1;
    const int64_t qeq = patternMask64(strand, cFwd(s), cNextIdx(s), s.pivot, s.cursor, ch, kr);
    return nfaCore(s.nfa, height, kOff, qeq, cProcessed(s), cFrag(s), outRows, outH, outKOff, hasMatch);
  }
  // ReadAlignmentNFA.nextState(qeq, progressIndex, fragmentLength, ...) (S/ReadAlignmentNFA.java:146-203)
  template <bool WRAP = false>
  GWA_HD bool nfaCore(const uint64_t (&nfa)[R], int height, int kOff, int64_t qeq, int progress, int frag,
                      uint64_t (&outRows)[R], int *outH, int *outKOff, bool *hasMatch) {
    const int kk = kOff + height - 1;
    const int soff = progress - kk;
    int64_t next[R];
    int minKwithMatch = kk + 1, minKwithProgress = kk + 1;
    int64_t prevRow = 0, prevNext = 0;
    // R'_0 = ((R_0 & P[ch]) << 1) & staircase;  R'_i = ((R_i & P[ch]) << 1) | R_{i-1} | R_{i-1} << 1 | R'_{i-1} << 1
#pragma unroll
    for (int i = 0; i < R; ++i) {
      next[i] = 0;
      if (i < height) {
        const int64_t a = (int64_t)nfa[i];
        int64_t nx = jshl(a & qeq, 1);
        if (i == 0) {
          if (nx != 0) { minKwithMatch = 0; minKwithProgress = 0; }
          nx &= stairMask<WRAP>(kOff, soff);
        } else {
          if (minKwithMatch > kk && nx != 0) minKwithMatch = i;
          nx |= prevRow | jshl(prevRow, 1) | jshl(prevNext, 1);
          nx &= stairMask<WRAP>(kOff + i, soff);
          if (minKwithProgress > kk && (nx & jshl(1, height)) != 0) minKwithProgress = i;
        }
        next[i] = nx;
        prevRow = a;
        prevNext = nx;
      }
    }
    const int mPos = kk + frag - progress;
    int rem = -1;
    int hm = 0;
    if (mPos < 64) {
      const int64_t bit = jshl(1, mPos);
#pragma unroll
      for (int nm = 0; nm < R; ++nm)
        if (nm < height && rem < 0 && (next[nm] & bit) != 0) { rem = nm; hm = 1; }
    }
    if (!hm) {
      int mk = minKwithMatch < minKwithProgress ? minKwithMatch : minKwithProgress;
      if (mk < kk) rem = mk;
      else return false;
    }
    // removeLayersFromAutomaton (:205-215): the OLD rows when nothing is trimmed
    if (rem == 0) {
#pragma unroll
      for (int i = 0; i < R; ++i) outRows[i] = nfa[i];
      *outH = height;
    } else {
      const int nh = height - rem;
#pragma unroll
      for (int h = 0; h < R; ++h) outRows[h] = (uint64_t)next[h];
      // outRows[h] = next[h + rem]: a log2(R)-stage barrel shift with static indices only
#pragma unroll
      for (int b = 1; b < R; b <<= 1) {
        const int on = (rem & b) != 0;
#pragma unroll
        for (int h = 0; h < R; ++h) outRows[h] = on ? (h + b < R ? outRows[h + b] : 0ULL) : outRows[h];
      }
#pragma unroll
      for (int h = 0; h < R; ++h) outRows[h] = h < nh ? (uint64_t)jushr((int64_t)outRows[h], 1) : 0ULL;
      *outH = nh;
    }
    *outKOff = kOff + rem;
    *hasMatch = hm != 0;
    return true;
  }

  // Cursor.nextSi + FMIndexOnGenome.bidirectionalSearch (S/Cursor.java:182-196, A/FMIndexOnGenome.java:162-191)
  // writes the resulting SiSet into d (lb/ub/bBase/meta-type)
  // `between` runs after the FM step's reads are issued and before their values are used: the
  // caller puts independent work there (the automaton step), so it overlaps the read latency
  template <class F>
  GWA_HD void nextSi(const DState<R> &c, int ch, DState<R> &d, F &&between) {
    uint32_t fl = 0, fu = 0, bl = 0, bu = 0;
    bool hasF = siGetF(c, ch, &fl, &fu);
    bool hasB = siGetB(c, ch, &bl, &bu);
    if (cDir(c) == D_BIFWD && (int)c.cursor >= (int)c.end - 1) hasF = false;
    const int strand = cStrand(c);
    d.meta = (uint8_t)((d.meta & ~(3 | M_TEXT)) | M_SIVALID);
    // Text mode: the child's pattern P' (P.ch when c's cursor moves forward, ch.P backward; |P'| =
    // processed bases of c + 1) occurs once, either because P does (c in text mode) or because the
    // interval just reached is one row (its SA value gives the occurrence).  The SiSet of P' is then
    // the one text character next to the occurrence in the SiSet's direction.
    enum { K_EMPTY, K_TEXT, K_RANK };
    const int kind = !(hasF || hasB) ? K_EMPTY
                     : (siText(c) || (cfg.textSearch && (hasF ? fu - fl : bu - bl) == 1)) ? K_TEXT : K_RANK;
    const int64_t N = (int64_t)ix.N;
    int64_t t = 0, p = 0;
    int len = 0;
    if (kind == K_TEXT) {
      if (siText(c)) {
        len = (int)c.lb[1] + 1;
        t = (int64_t)c.lb[0];
        // strand 0 prepends (backward) and strand 1 appends (forward) at the text start
        if ((strand == 0) != cFwd(c)) t = t == 0 ? N - 1 : t - 1;
      } else {
        len = cProcessed(c) + 1;
        const int fm = hasF ? (strand == 0 ? 1 : 0) : (strand == 0 ? 0 : 1);
        const int64_t v = (int64_t)ix.sa[fm][hasF ? fl : bl];
        ++saReads;
        // fm 0 (T) rows start at t; fm 1 (reverse(T)) rows start at N - t - |P'|
        t = fm == 0 ? v : N - v - len;
        t = t < 0 ? t + N : t;
      }
      // the next character: after the occurrence for a forward SiSet on strand 0 / a backward one
      // on strand 1, before it otherwise
      const bool after = (strand == 0) == hasF;
      p = after ? t + len : t - 1;
      p = p >= N ? p - N : p < 0 ? p + N : p;
    }
    // The memory reads of this FM step -- the text words (text mode) or the two Occ blocks of the
    // interval (rankACGTN at lb and ub, A/FMIndexOnOccTable.java:53-55; shared when both fall in one
    // 128-position window) -- are issued for all lanes of the wavefront before any is used, so a
    // wavefront mixing text-mode and Occ lanes waits once, not once per kind.
    const int fmR = hasF ? (strand == 0 ? 1 : 0) : (strand == 0 ? 0 : 1);
    uint64_t rl = hasF ? fl : bl, ru = hasF ? fu : bu;
    rl = rl > ix.N ? ix.N : rl;
    ru = ru > ix.N ? ix.N : ru;
    Block B0, B1;
    // text words through the lane's one-word cache (a text-mode run moves one position per step: one
    // load per 32 / 64 steps), the loads issued here, before `between`
    if (kind == K_TEXT) {
      const int64_t a = p >> 5, b = p >> 6;
      if (a != tcW2) { tcC2 = ix.text2[a]; tcW2 = a; }
      if (b != tcWN) { tcCN = ix.textN[b]; tcWN = b; }
    }
    if (kind == K_RANK) {
      loadBlock(ix.occ[fmR], rl >> 7, B0);
      loadBlock(ix.occ[fmR], ru >> 7, B1);  // same line when both share a window (an L2 hit)
      blocks += 1 + ((ru >> 7) != (rl >> 7) ? 1 : 0);
    }
    between();
    if (kind == K_TEXT) {
      ++textSteps;
      d.meta |= M_TEXT | (hasF ? (hasB ? SI_BID : SI_FWD) : SI_BWD);
      d.lb[0] = (uint32_t)t;
      d.lb[1] = (uint32_t)len;
      d.lb[2] = (uint32_t)(((tcCN >> (p & 63)) & 1) ? 4 : (int)((tcC2 >> ((p & 31) * 2)) & 3));
      d.lb[3] = 0;
      for (int i = 0; i < 4; ++i) d.ub[i] = 0;
      d.bBase = 0;
      return;
    }
    if (kind == K_RANK) {
      uint64_t lo[5], hi[5];
      rankAll(B0, rl, lo);
      rankAll(B1, ru, hi);
      for (int i = 0; i < 4; ++i) {
        d.lb[i] = (uint32_t)(ix.C[i] + lo[i]);
        d.ub[i] = (uint32_t)(ix.C[i] + hi[i]);
      }
      d.meta |= hasF ? (hasB ? SI_BID : SI_FWD) : SI_BWD;
      d.bBase = hasF && hasB ? bl : 0;
      return;
    }
    d.meta |= SI_EMPTY;
    for (int i = 0; i < 4; ++i) d.lb[i] = d.ub[i] = 0;
    d.bBase = 0;
  }

  // nextStateAfterSplit / nextStateAfterClipping (:803-838); -1 null, -2 overflow
  GWA_HD int nextStateAfterSplit(const DState<R> &cs, bool clip, uint64_t *key) {
    // cs = register copy of the expanded state, its split flag already stored by the caller
    const int mk = (int)(((uint32_t)cs.state >> 8) & 0xFF);
    if (!(mk < k)) return -1;
    const int pr = (int)(((uint32_t)cs.state >> 16) & 0xFF);
    // Cursor.split (S/Cursor.java:130-156)
    int strand = cStrand(cs), dir = cDir(cs);
    int ld, ls, le, lc, lp, rdr, rs, re, rc, rp;
    if (dir == D_FORWARD) {
      ld = dir; ls = cs.start; le = cs.cursor; lc = cs.cursor; lp = cs.pivot;
      rdr = D_FORWARD; rs = cs.cursor; re = cs.end; rc = cs.cursor; rp = cs.cursor;
    } else if (dir == D_BACKWARD) {
      ld = dir; ls = cs.cursor; le = cs.end; lc = cs.cursor; lp = cs.pivot;
      rdr = D_BACKWARD; rs = cs.start; re = cs.cursor; rc = cs.cursor; rp = cs.start;
    } else {
      if (cs.cursor + 1 < cs.end) {
        ld = dir; ls = cs.start; le = cs.cursor; lc = cs.cursor; lp = cs.pivot;
        rdr = dir; rs = cs.cursor; re = cs.end; rc = cs.cursor; rp = cs.cursor;
      } else {
        ld = D_BACKWARD; ls = cs.start; le = cs.cursor; lc = cs.cursor; lp = cs.pivot;
        rdr = dir; rs = cs.cursor; re = cs.end; rc = cs.cursor; rp = cs.cursor;
      }
    }
    const int a = allocState();
    if (a < 0) return -2;
    const int b = allocState();
    if (b < 0) return -2;
    DState<R> d = cs;  // currentSi, siTable carried over
    setCursor(d, strand, ld, ls, le, lc, lp);
    {
      // ReadAlignmentNFA.nextStateAfterSplit (S/ReadAlignmentNFA.java:107-114)
      int height = cs.nrows - 1;
      d.nrows = (uint8_t)(height < 0 ? 0 : height);
      d.kOffset = (uint8_t)(cs.kOffset + 1);
      for (int i = 0; i < R; ++i) d.nfa[i] = i < height ? (uint64_t)jshl(1, height + i - 1) : 0;
      const int cur = ((uint32_t)cs.state >> 5) & 7;
      d.state = packState(cur > 4 ? 4 : cur, mk, pr, (((uint32_t)cs.state >> 24) & 1) != 0);
      d.nextSplit = b;
    }
    DState<R> t;
    t.meta = 0;
    setCursor(t, strand, rdr, rs, re, rc, rp);
    t.curLb = t.curUb = 0;
    t.nextSplit = -1;
    t.state = packState(4, mk, pr, false);
    if (!clip) {
      siInit(t, rdr);
      t.meta |= M_NFAVALID;
      t.nrows = (uint8_t)(k + 1);
      t.kOffset = 0;
      for (int i = 0; i < R; ++i) t.nfa[i] = i <= k ? (uint64_t)jshl(1, k + i) : 0;
    } else {
      for (int i = 0; i < 4; ++i) t.lb[i] = t.ub[i] = 0;
      t.bBase = 0;
      t.nrows = 0;
      t.kOffset = 0;
      for (int i = 0; i < R; ++i) t.nfa[i] = 0;
      t.state |= 1 << 25;  // updateClippedFlag
    }
    t.state |= kStRef;  // a's nextSplit
    GWA_PW(PR_WA, PR_EA, 2 * sizeof(DState<R>));
    S(a) = d;
    S(b) = t;
    // keyOf(a) for the chain [a -> b] from the registers (chainScore with one split)
    const int M = cfg.matchScore;
    const int sc = M * (cProcessed(d) + cProcessed(t)) - (M + cfg.mismatchPenalty) * (2 * mk - 1) - cfg.splitOpenPenalty;
    *key = packKey(pr, sc, cProcessed(d));
    return a;
  }

  // SearchState.update (:861-875); -1 = null
  GWA_HD int update(int self, int oldS, int newS) {
    if (oldS == self) return newS;
    invalidateCache();
    int prev = self;
    while (S(prev).nextSplit != oldS) {
      prev = S(prev).nextSplit;
      if (prev < 0) return -1;
    }
    GWA_PW(PR_WS, PR_ES, 4);
    S(prev).nextSplit = newS;
    if (newS >= 0) markRef(newS);
    refreshKeysFor(prev);  // score() of every chain through prev changed
    return self;
  }

  // ---- AlignmentProcess.align_internal (:278-477), split at the quick scan ----
  // Phase 1 (fm_quickscan kernel): N check, FMQuickScan on both strands, exact hits.
  // Returns 1 when the read needs the best-first search; otherwise the result is final.
  GWA_HD int quickPhase(ScanRes *sr, OutHeader *oh, const OutSlots &os, uint32_t rd_) {
    if (!quickOpen(oh)) return 0;
    Scan sF = quickScan(0);
    if (sF.numMismatches == 0) { reportExact(sF, 0, oh, os, rd_); return 0; }
    Scan sR = quickScan(1);
    return quickClose(sF.numMismatches, sF.lmStart, sF.firstEmpty, sR, sr, oh, os, rd_);
  }
  // quickPhase's opening: the header's search fields cleared, the read words loaded; false = the read
  // has more N than k mismatches (its result is final)
  GWA_HD bool quickOpen(OutHeader *oh) {
    oh->fmSearches = 0;
    oh->states = 0;
    oh->searchBlocks = 0;
    oh->saReads = 0;
    oh->searchShort = 0;
    oh->numSW = oh->verifyBytes = 0;
    oh->poolFail = 0;
    oh->ovfWhat = 0;
    oh->nChains = oh->nHits = oh->nCigar = 0;
    oh->status = ST_UNMAPPED;
    const int countN = loadWords(pw0, pw1);
    if (countN > k) { finishQuick(oh); return false; }
    return true;
  }
  // quickPhase's close after both strands (strand 0 inexact: its numMismatches, longest-match start,
  // first empty step); 1 = the read needs the best-first search
  GWA_HD int quickClose(int nmF, int lmF, int feF, const Scan &sR, ScanRes *sr, OutHeader *oh, const OutSlots &os,
                        uint32_t rd_) {
    if (sR.numMismatches == 0) { reportExact(sR, 1, oh, os, rd_); return 0; }
    if (k == 0) { finishQuick(oh); return 0; }
    sr->nmF = nmF; sr->lmF = lmF;
    sr->nmR = sR.numMismatches; sr->lmR = sR.lmStart;
    sr->feF = feF; sr->feR = sR.firstEmpty;
    finishQuick(oh);
    return 1;
  }
  GWA_HD void finishQuick(OutHeader *oh) {
    oh->quickSteps = quickSteps;
    oh->blocks = blocks;
    oh->kmerLookups = kmerLookups;
    oh->quickSa = saReads;
    oh->quickShort = shortSteps;
    oh->quickText = textRuns;
  }
  // reportExactMatchAlignment (:490-494) + FMIndexOnGenome.toGenomeCoordinate (:258-269):
  // the single exact ReadHit is the reported BESTHIT/ALLHITS/TOPL result.
  GWA_HD void reportExact(const Scan &s, int strand, OutHeader *oh, const OutSlots &os, uint32_t rd_) {
    int64_t sav = s.uniq ? (int64_t)s.tp : (int64_t)ix.sa[strand == 0 ? 1 : 0][s.lb];
    if (!s.uniq) ++saReads;
    finishQuick(oh);
    int64_t pos = strand == 0 ? (int64_t)ix.N - sav : sav;
    if (strand == 0) pos -= m;
    pos += 1;
    int32_t chr, p;
    if (pos < 0 || translate(pos, &chr, &p) != 0) { oh->status = ST_ERROR; return; }
    oh->hitOff = rd_ * os.hitCap;
    oh->cigOff = rd_ * os.cigCap;
    OutHit &o = os.hits[oh->hitOff];
    o.chr = chr; o.pos = p; o.matchLength = m; o.qStart = 0; o.qEnd = m; o.diff = 0; o.strand = strand;
    o.numHits = (int32_t)(s.ub - s.lb); o.next = -1; o.cigarOff = 0; o.cigarLen = 1;
    os.cig[oh->cigOff] = (uint16_t)((m << 3) | 0);
    oh->nChains = 1; oh->nHits = 1; oh->nCigar = 1;
    oh->status = ST_MAPPED;
  }

  // Phase 2 (bsf_search kernel): seeds from the quick scans (:318-349) and the queue loop (:352-475)
  // The best-first loop of searchPhase as a resumable step machine, so a wavefront can hold lanes
  // that reached a report (the DP verification) and run those together:
  //   searchStart: seeds (:318-341); false = nothing to search
  //   searchStep : one loop iteration (:343-477); SS_CONTINUE, SS_REPORT (run searchReport next)
  //                or SS_DONE
  //   searchReport: reportAlignment of the pending chain; false = the search ended (error/overflow)
  enum { SS_CONTINUE = 0, SS_REPORT = 1, SS_DONE = 2, SS_SUSPEND = 3 };
  int pendingBase = -1, upperSearches = 0;
  GWA_HD bool searchReport() { return reportAlignment(pendingBase); }

  // ---- suspend / resume across capacity tiers ----
  // A read about to outgrow one of its lane's capacities is suspended between micro-steps -- its lane
  // fields and the used part of its slice (arena, queue, hits, report list, CIGAR ops) copied to a
  // record -- and resumed on the next, larger tier from that record instead of rerunning its search
  // from the seeds.  Exactness: a micro-step is started only when it cannot overflow the arena or the
  // queue (at most 9 states and 5 queue entries per step: two control rounds of split + clip children,
  // then one child), and a report that overflows the hits, the CIGAR area or the first tier's DP slice
  // is rolled back to its start (verify only appends) and suspended before it; a report also needs a
  // free report-list entry (AlignmentResultHolder.add keeps at most listSize + 1).  Everything else a
  // step or report touches is as it would be without the suspension.
  enum { LP_RUN = 0, LP_WAIT = 1, LP_FINISH = 2, LP_SUSPEND = 3 };
  int susPhase = LP_RUN;  // the phase a suspended read resumes in (LP_RUN or LP_WAIT: a report pending)
  // room for one micro-step (searchStep), by where it starts: at most 5 new states (a child, then the
  // split and clip children's 4 when it was the last candidate; or a first child and its run-ahead's
  // last state) and, net of a poll (xMode 0), 2 more queue entries; 3 from the next child (1).  0 when
  // there is room, else the OV_* capacity that may run out.
  // (DPM 1, the first tier's kernel: no suspension at all -- its overflows restart on the next tier,
  // as the suspend paths cost that kernel's register budget more than its few overflows' reruns)
  GWA_HD int passRoom() const {
    if (DPM == 1) return 0;
    const int q = xMode == 1 ? 3 : 2;
    return nStates + 5 > caps.arena ? OV_ARENA : heapSize + q > caps.heap ? OV_HEAP : 0;
  }
  GWA_HD int laneStep() {
    const int st = searchStep();
    if (st == SS_SUSPEND) {
      susPhase = LP_RUN;
      return LP_SUSPEND;
    }
    return st == SS_REPORT ? LP_WAIT : st == SS_DONE ? LP_FINISH : LP_RUN;
  }
  GWA_HD int laneReport() {
    if (DPM != 1 && listSize >= caps.list) {
      ovfWhat |= OV_LIST;
      susPhase = LP_WAIT;
      return LP_SUSPEND;
    }
    const int h0 = nHits, c0 = nCigar, sw0 = numSW, vb0 = verifyBytes, sa0 = saReads, st0 = status;
    if (searchReport()) return LP_RUN;
    if (DPM != 1 && status == ST_OVERFLOW && (ovfWhat & ~(OV_HITS | OV_CIGAR | OV_SLICE)) == 0) {
      nHits = h0;  // (verify appended hits and CIGAR ops only; nothing else changed yet)
      nCigar = c0;
      numSW = sw0;
      verifyBytes = vb0;
      saReads = sa0;
      status = st0;
      susPhase = LP_WAIT;
      return LP_SUSPEND;
    }
    return LP_FINISH;
  }
  // record layout: header (lane fields, the cached state), then arena | queue | hits | list | CIGAR
  static constexpr uint32_t kResumeMagic = 0x52534D31u;
  static constexpr int kResumeInts = 48;
  GWA_HD static size_t resumeHdrBytes() { return ((size_t)kResumeInts * 4 + 8 + sizeof(DState<R>) + 63) & ~(size_t)63; }
  GWA_HD static size_t resumeBytes(const Caps &c) {
    return resumeHdrBytes() + sizeof(DState<R>) * (size_t)c.arena + 8 * (size_t)c.heap + sizeof(DHit) * (size_t)c.hits +
           4 * (size_t)c.list + 2 * (size_t)c.cigar + 64;
  }
  // no record for read r at rec (restart on the next tier)
  GWA_HD static void resumeInvalidate(uint8_t *rec) { ((uint32_t *)rec)[0] = 0; }
  GWA_HD void suspendTo(uint8_t *rec, uint32_t r) {
    int32_t *h = (int32_t *)rec;
    int q = 1;  // (h[0]: the magic word, written last)
    h[q++] = (int32_t)r;
    h[q++] = minMismatches; h[q++] = maxMatchLength; h[q++] = bestScore; h[q++] = numFMIndexSearches;
    h[q++] = nStates; h[q++] = heapSize; h[q++] = nHits; h[q++] = listSize; h[q++] = nCigar; h[q++] = listOk;
    h[q++] = pendingBase; h[q++] = upperSearches; h[q++] = xMode; h[q++] = xT; h[q++] = xBase; h[q++] = xC;
    h[q++] = xNm; h[q++] = xNextBase;
    h[q++] = cacheIdx; h[q++] = cacheDirty; h[q++] = susPhase;
    h[q++] = quickSteps; h[q++] = blocks; h[q++] = saReads; h[q++] = maxHeap; h[q++] = kmerLookups;
    h[q++] = shortSteps; h[q++] = textSteps; h[q++] = textRuns; h[q++] = numSW; h[q++] = verifyBytes;
    *(DState<R> *)(rec + kResumeInts * 4 + 8) = cache;
    uint8_t *o = rec + resumeHdrBytes();
    copyOut(o, (const uint8_t *)L.arena(), sizeof(DState<R>) * (size_t)nStates);
    o += (sizeof(DState<R>) * (size_t)nStates + 15) & ~(size_t)15;
    uint64_t *hq = (uint64_t *)o;
    for (int i = 0; i < heapSize; ++i) hq[i] = hslot(i);
    o += ((size_t)heapSize * 8 + 15) & ~(size_t)15;
    copyOut(o, (const uint8_t *)L.hits(), sizeof(DHit) * (size_t)nHits);
    o += (sizeof(DHit) * (size_t)nHits + 15) & ~(size_t)15;
    int32_t *lo = (int32_t *)o;
    for (int i = 0; i < listSize; ++i) lo[i] = L.list()[i];
    o += ((size_t)listSize * 4 + 15) & ~(size_t)15;
    uint16_t *co = (uint16_t *)o;
    for (int i = 0; i < nCigar; ++i) co[i] = L.cigar()[i];
    h[0] = (int32_t)kResumeMagic;  // (written last: the record is complete)
  }
  GWA_HD static bool resumeValid(const uint8_t *rec, uint32_t r) {
    const int32_t *h = (const int32_t *)rec;
    return (uint32_t)h[0] == kResumeMagic && (uint32_t)h[1] == r;
  }
  // true when rec holds read r's suspended search; then the lane continues it (phase in *phase)
  GWA_HD bool resumeFrom(const uint8_t *rec, uint32_t r, int *phase, bool masks = true) {
    const int32_t *h = (const int32_t *)rec;
    if (!resumeValid(rec, r)) return false;
    int q = 2;
    minMismatches = h[q++]; maxMatchLength = h[q++]; bestScore = h[q++]; numFMIndexSearches = h[q++];
    nStates = h[q++]; heapSize = h[q++]; nHits = h[q++]; listSize = h[q++]; nCigar = h[q++]; listOk = h[q++];
    pendingBase = h[q++]; upperSearches = h[q++]; xMode = h[q++]; xT = h[q++]; xBase = h[q++]; xC = h[q++];
    xNm = h[q++]; xNextBase = h[q++];
    cacheIdx = h[q++]; cacheDirty = h[q++]; *phase = h[q++];
    quickSteps = h[q++]; blocks = h[q++]; saReads = h[q++]; maxHeap = h[q++]; kmerLookups = h[q++];
    shortSteps = h[q++]; textSteps = h[q++]; textRuns = h[q++]; numSW = h[q++]; verifyBytes = h[q++];
    cache = *(const DState<R> *)(rec + kResumeInts * 4 + 8);
    const uint8_t *o = rec + resumeHdrBytes();
    copyOut((uint8_t *)L.arena(), o, sizeof(DState<R>) * (size_t)nStates);
    o += (sizeof(DState<R>) * (size_t)nStates + 15) & ~(size_t)15;
    const uint64_t *hq = (const uint64_t *)o;
    for (int i = 0; i < heapSize; ++i) hslot(i) = hq[i];
    o += ((size_t)heapSize * 8 + 15) & ~(size_t)15;
    copyOut((uint8_t *)L.hits(), o, sizeof(DHit) * (size_t)nHits);
    o += (sizeof(DHit) * (size_t)nHits + 15) & ~(size_t)15;
    const int32_t *lo = (const int32_t *)o;
    for (int i = 0; i < listSize; ++i) L.list()[i] = lo[i];
    o += ((size_t)listSize * 4 + 15) & ~(size_t)15;
    const uint16_t *co = (const uint16_t *)o;
    for (int i = 0; i < nCigar; ++i) L.cigar()[i] = co[i];
    if (masks) buildMasks();  // the read words / QueryMask rows in LDS (searchStart builds them on a fresh start)
    status = ST_UNMAPPED;
    ovfWhat = 0;
    return true;
  }
  // n bytes (a multiple of 8, both ends 8-B aligned) 8 B at a time
  GWA_HD static void copyOut(uint8_t *dst, const uint8_t *src, size_t n) {
    for (size_t i = 0; i < n / 8; ++i) ((uint64_t *)dst)[i] = ((const uint64_t *)src)[i];
  }
  GWA_HD bool searchStart(const ScanRes &sr, bool masks = true) {
    GWA_PT(tsd);
    if (masks) buildMasks();
    int a = -1, b = -1;
    if (sr.nmF <= k) {
      if (sr.lmF != 0 && sr.lmF < m) a = newInitial(0, D_BIFWD, 0, m, sr.lmF, sr.lmF, sr.nmF);
      else a = newInitial(0, D_FORWARD, 0, m, 0, 0, sr.nmF);
      if (a < 0) return false;
    }
    if (sr.nmR <= k) {
      if (sr.lmR != 0 && sr.lmR < m) b = newInitial(1, D_BIFWD, 0, m, sr.lmR, sr.lmR, sr.nmR);
      else b = newInitial(1, D_FORWARD, 0, m, 0, 0, sr.nmR);
      if (b < 0) return false;
    }
    queueAdd(a);
    queueAdd(b);
    GWA_PA(PR_SEED, tsd);
    upperSearches = m * 20;
    return true;
  }
  // One call = one micro-step of the loop of align_internal (:343-477).  A poll is followed by at
  // most ONE child expansion (an FM step); the remaining children of the same poll and the split /
  // clip children come in later calls (xMode 1 / 2), so every lane of a wavefront performs about
  // one FM step per call instead of the wavefront looping until its slowest lane has tried all
  // four bases.  Nothing else touches a lane between its micro-steps, so the order of operations
  // on its heap and arena is exactly the reference's.
  // (the expanded state xC is re-read from the arena / cache at each micro-step rather than kept
  // in the lane object: its flag word is always stored, so the arena copy is current)
  int xMode = 0, xT = 0, xBase = 0, xC = 0, xNm = 0, xNextBase = 0;
  GWA_HD int searchStep() {
    // a micro-step starts only when it cannot overflow the arena or the queue (passRoom); else the
    // read is suspended here, before it (suspend / resume below)
    if (const int ov = passRoom()) {
      ovfWhat |= ov;
      return SS_SUSPEND;
    }
    DState<R> xCS;
    if (xMode == 0) {
      GWA_PC(PR_NSW, PR_NSL);
      if (!(heapSize > 0 && status != ST_OVERFLOW && status != ST_ERROR)) return SS_DONE;
      if (numFMIndexSearches > upperSearches) return SS_DONE;
      GWA_PT(tp);
      const int base = queuePoll();
      if (base != cacheIdx) flushCache();  // the deferred state stays queued
      // the polled state and its split chain are read once into registers
      DState<R> C;
      loadState(base, C);
      tr(1, (uint32_t)base, curWord(C), (uint32_t)(C.state & ~kStRef));
      // upperBoundOfScore of the polled chain (:380), taken before the walk (which only reads)
      const int ubScore = C.nextSplit < 0 ? stateScore(C, 0, true) : chainScore(base, true);
      int c = base;
      // skip finished members (hasHit | isClipped | done); a chain with none left is reported
      // (single-exit loop: no break / loop-carried flag, see quickScan)
      while (((((uint32_t)C.state >> 24) & 3) != 0 || cRemaining(C) == 0) && C.nextSplit >= 0) {
        c = C.nextSplit;
        loadState(c, C);
      }
      GWA_PA(PR_POLL, tp);
      if ((((uint32_t)C.state >> 24) & 3) != 0 || cRemaining(C) == 0) {
        flushCache();  // verify reads the chain from the arena
        pendingBase = base;
        return SS_REPORT;
      }
      // the checks below drop the polled state (a deferred one is chain-free: dead from here)
      const int nm = (int)(((uint32_t)C.state >> 8) & 0xFF);
      if ((C.state & 0x1F) == 0x1F || nm > minMismatches || minMismatches - nm < 0 || ubScore < 0 ||
          ubScore < bestScore) {  // isFinished / pruned
        dropIfCached(base);
        return SS_CONTINUE;
      }
      xBase = base;
      xC = c;
      xCS = C;
      xNm = nm;
      xNextBase = qcode(cStrand(C), cNextIdx(C));
      xT = -1;
      xMode = 1;
    } else {
      loadState(xC, xCS);
    }
    if (xMode == 1) {
      // children (:386-410): nextBase first -- a state from it ends the iteration -- then every
      // base still unchecked; one FM step per call
      GWA_PT(te);
      // (the checked flags are stored once, with the child taken below or with the split flag: nothing
      // reads the arena copy of xC in between, siIsEmpty reads the register copy)
      int ch = -1, tt = xT, zero = 0;
      for (; tt < 4 && ch < 0; ++tt) {
        zero |= tt == 0 ? 1 : 0;  // (single-exit loop, integer state: see quickScan)
        const int cand = tt < 0 ? xNextBase : tt;
        if (xCS.state & (1 << cand)) continue;  // isChecked
        xCS.state |= 1 << cand;                 // updateFlag
        if (siIsEmpty(xCS, cand)) continue;
        ch = cand;
      }
      // StaircaseFilter sf = getStairCaseFilter(m) where the loop over every base begins (:439); this
      // micro-step entered it if it ran the loop at tt = 0
      if (zero && !stairOk()) return SS_DONE;
      const int first = (xT < 0 && tt == 0) ? 1 : 0;  // the child taken is nextBase
      xT = tt;
      if (ch >= 0) {
        storeStateWord(xC, xCS.state);
        GWA_PT(tn);
        int ns = nextStateLocal(xC, xCS, ch, first && xC == xBase && deferrable(xCS));
        GWA_PA(PR_LOOP, tn);
        if (ns == -2) return SS_DONE;
        if (ns >= 0) {
          if (first && xC == xBase) {
            GWA_PT(tra);
            ns = runAhead(ns);
            GWA_PA(PR_BOUND, tra);
            if (ns == -2) return SS_DONE;
          }
          GWA_PT(tad);
          queueAdd(update(xBase, xC, ns));
          GWA_PA(PR_ADD1, tad);
          if (first) {
            xMode = 0;
            GWA_PA(PR_EXP1, te);
            return SS_CONTINUE;
          }
        }
        GWA_PA(PR_EXPN, te);
        if (xT < 4) return SS_CONTINUE;  // more candidates: next call
      }
      xMode = 2;
    }
    // split / clip children (:412-475)
    GWA_PT(ts);
    xMode = 0;
    xCS.state |= 1 << 4;  // updateSplitFlag
    storeStateWord(xC, xCS.state);
    const int nsplit = (xC == xBase && xCS.nextSplit < 0) ? 0 : numSplit(xBase);
    if (nsplit < cfg.numSplit && xNm + 1 <= minMismatches) {
      const int index = cNextIdx(xCS);
      if (index > cfg.indelEndSkip && m - index >= cfg.indelEndSkip) {
        for (int clip = 0; clip < 2; ++clip) {  // split, then clip (:414-425)
          uint64_t key = 0;
          const int ns = nextStateAfterSplit(xCS, clip != 0, &key);
          if (ns == -2) return SS_DONE;
          if (ns >= 0) {
            if (xC == xBase) queueAddKeyed((key << KS) | (uint64_t)ns);  // update(base, base, ns) == ns
            else queueAdd(update(xBase, xC, ns));
          }
        }
      }
    }
    if (xC == xBase && deferrable(xCS)) dropIfCached(xC);  // the expanded chain-free state is done
    GWA_PA(PR_SPLIT, ts);
    return SS_CONTINUE;
  }

  // ---- register cache of the most recently created state (the usual next poll) ----
  // Write-back deferral: a new state that no split chain holds (nextSplit < 0, no kStRef) stays
  // only in the cache (cacheDirty) until it is evicted.  The usual next poll returns it, and when
  // its own next base is accepted the reference drops it (:386-396: the child is pushed, the parent
  // is not) -- its arena copy would never be read, so it is never written.  Every other path writes
  // it back first (flushCache): a poll of another state, a report, a chain operation, an eviction
  // by a state other than its accepted first child.
  int cacheIdx = -1, cacheDirty = 0;
  DState<R> cache;
  GWA_HD void flushCache() {
    if (cacheDirty) {
      GWA_PW(PR_WA, PR_EA, sizeof(DState<R>));
      L.arena()[cacheIdx] = cache;
      cacheDirty = 0;
    }
  }
  GWA_HD static bool deferrable(const DState<R> &d) { return d.nextSplit < 0 && !(d.state & kStRef); }
  GWA_HD void loadState(int idx, DState<R> &d) {
#ifdef GWA_NO_CACHE
    d = L.arena()[idx];
#else
    if (idx == cacheIdx) d = cache;
    else d = L.arena()[idx];
#endif
  }
  GWA_HD void storeStateWord(int idx, int32_t w) {
    if (!(idx == cacheIdx && cacheDirty)) { GWA_PW(PR_WS, PR_ES, 4); L.arena()[idx].state = w; }
    if (idx == cacheIdx) cache.state = w;
  }
  GWA_HD void invalidateCache() {
    flushCache();
    cacheIdx = -1;
  }
  // the polled state `base` (the cache, chain-free) is dead: the reference drops it here
  GWA_HD void dropIfCached(int base) {
    if (base == cacheIdx && cacheDirty) cacheDirty = 0;
  }
  GWA_HD int qcode(int strand, int i) const { return (int)((qword(strand, i >> 5) >> (2 * (i & 31))) & 3); }
  // one chain member's term of score()/upperBoundOfScore() with ns splits after it
  GWA_HD int stateScore(const DState<R> &d, int ns, bool upper) const {
    const int nm = (int)(((uint32_t)d.state >> 8) & 0xFF) - ns;
    const int mm = cProcessed(d) + (upper ? cRemaining(d) : 0) - nm;
    return mm * cfg.matchScore - nm * cfg.mismatchPenalty - ns * cfg.splitOpenPenalty;
  }
  // SearchState.nextState (:840-852) from a register copy of the parent, into d; false = null
  GWA_HD bool buildChild(const DState<R> &cs, int ch, DState<R> &d) {
    // c.nextState(ch, nextSi, queryMask, getStairCaseFilter(m)) (:423-425, :445-447)
    if (!stairOk()) return false;
    const int strand = cStrand(cs);
    uint64_t rows[R];
    int nh = 0, nko = 0;
    bool hm = false;
    d.meta = 0;
    // The FM step (next(c, ch)) precedes the automaton in the reference (:422-425); the two are
    // independent (both read only the parent), so the automaton step runs while the FM step's
    // reads are in flight.  Counts and results are those of the reference order.
    bool nfaOk = false;
    GWA_PC(PR_NBW, PR_NBL);
    GWA_PT(tf);
    nextSi(cs, ch, d, [&] {
      GWA_PT(tq);
      nfaOk = nfaNext(cs, ch, strand, rows, &nh, &nko, &hm);
      GWA_PA(PR_NFA, tq);
    });
    GWA_PA(PR_FM, tf);
    ++numFMIndexSearches;
    tr(2, (uint32_t)ch, d.lb[0] ^ (d.ub[1] * 3u) ^ (d.lb[2] * 7u) ^ (d.ub[3] * 11u) ^ d.bBase, (uint32_t)(d.meta & 3));
    if (!nfaOk) { tr(3, 0, 0, 0); return false; }
    tr(4, (uint32_t)nh | ((uint32_t)nko << 8) | ((uint32_t)hm << 16), (uint32_t)rows[0], (uint32_t)(nh > 1 ? rows[1] : 0));
    int nc = cs.cursor, dir = cDir(cs);
    if (dir == D_FORWARD) ++nc;
    else if (dir == D_BACKWARD) --nc;
    else {
      if (nc + 1 < cs.end) ++nc;
      else { dir = D_BACKWARD; nc = cs.pivot; }
    }
    setCursor(d, strand, dir, cs.start, cs.end, nc, cs.pivot);
    uint32_t sl = 0, su = 0;
    bool sv = dir != D_BACKWARD ? siGetF(cs, ch, &sl, &su) : siGetB(cs, ch, &sl, &su);
    d.curLb = sv ? sl : 0;
    d.curUb = sv ? su : 0;
    if (sv) d.meta |= M_CURVALID;
    d.meta |= M_NFAVALID;
    d.state = packState(ch, nko, (int)(((uint32_t)cs.state >> 16) & 0xFF), hm);
    d.nextSplit = cs.nextSplit;
    d.nrows = (uint8_t)nh;
    d.kOffset = (uint8_t)nko;
#pragma unroll
    for (int i = 0; i < R; ++i) d.nfa[i] = i < nh ? rows[i] : 0;
    return true;
  }
  // the child in a new arena slot (stays cached); -1 null, -2 overflow.  parentDead: c is the
  // polled chain-free state and this child is its accepted next base (the reference drops c), so a
  // deferred c is not written back
  GWA_HD int nextStateLocal(int c, const DState<R> &cs, int ch, bool parentDead) {
    DState<R> d;
    if (!buildChild(cs, ch, d)) return -1;
    int id = allocState();
    if (id < 0) return -2;
#ifndef GWA_NO_CACHE
    if (parentDead && c == cacheIdx) cacheDirty = 0;
    flushCache();
    cache = d;
    cacheIdx = id;
    if (deferrable(d)) cacheDirty = 1;
    else { GWA_PW(PR_WA, PR_EA, sizeof(DState<R>)); L.arena()[id] = d; }
#else
    L.arena()[id] = d;
#endif
    return id;
  }

  // ---- run-ahead over text-mode match runs ----
  // When the polled state's first child (its own next base, :386-396) is accepted, the reference
  // pushes it and ends the iteration; the next poll usually returns that child, whose first child
  // is tried next, and so on, one FM step per loop iteration.  In text mode (one occurrence) while
  // the text continues with the read's bases, such a run lasts tens of steps.  If the queue array
  // provably comes back unchanged from every push + poll of the run (heapNoop: the child sifts up to
  // the root and the displaced last element sifts back down to its slot), the iterations are run
  // here back to back in registers: the same FM steps (counted), automaton steps and loop checks
  // (:352-396) in the same order, without the heap round trips and without arena copies of the
  // intermediate states, which nothing references (chain-free, not queued, not reported).  The run
  // stops before any state that the loop would treat otherwise -- report, prune, empty or rejected
  // first child, non-text interval -- and that state is pushed as the reference pushes it.
  GWA_HD uint64_t heapKeyAt(int i) const { return hslot(i) >> KS; }
  GWA_HD bool heapNoop(uint64_t *bound) const {
    const int kk = heapSize;
    *bound = ~0ULL;
    if (kk == 0) return true;
    const int depth = 31 - __builtin_clz((unsigned)kk + 1u);  // levels above slot kk
    const uint64_t x = heapKeyAt((kk - 1) >> 1);              // P0's element, displaced to slot kk
    uint64_t mn = ~0ULL;
    int ok = 1;
    for (int j = depth; j >= 1; --j) {
      const int node = ((kk + 1) >> j) - 1;  // path node, root first; node(1) = P0
      const uint64_t v = heapKeyAt(node);
      mn = v < mn ? v : mn;
      const int lc = 2 * node + 1, rc = lc + 1;
      if (j >= 2) {
        // siftDown at node must pick the path child (holding v after the push) and move x below it
        const int nxt = ((kk + 1) >> (j - 1)) - 1;
        if (nxt == lc) ok &= (rc < kk && v > heapKeyAt(rc)) ? 0 : 1;
        else ok &= heapKeyAt(lc) > v ? 1 : 0;
        ok &= x > v ? 1 : 0;
      } else if (kk == rc) {
        ok &= x > heapKeyAt(lc) ? 0 : 1;  // siftDown must stop at P0
      }
    }
    *bound = mn;
    return ok != 0;
  }
  GWA_HD uint64_t keyOfLocal(const DState<R> &c) const {  // keyOf of a chain-free state
    return packKey((int)(((uint32_t)c.state >> 16) & 0xFF), stateScore(c, 0, false), cProcessed(c));
  }
  GWA_HD int runAhead(int ns) {
#ifdef GWA_NO_RA
    return ns;
#endif
    if (cfg.runAheadMax <= 0 || cacheIdx != ns || cache.nextSplit >= 0 || !siText(cache)) return ns;
    uint64_t bound;
    if (!heapNoop(&bound)) return ns;
    // the run works on the register copy `cache` (the state to be polled next) in place
    int moved = 0;
    for (int it = 0; it < cfg.runAheadMax; ++it) {
      // loop top (:352-356) and the poll checks (:358-385) for the cached state
      if (numFMIndexSearches > upperSearches || status == ST_OVERFLOW || status == ST_ERROR) break;
      if (keyOfLocal(cache) >= bound) break;
      if ((((uint32_t)cache.state >> 24) & 3) != 0 || cRemaining(cache) == 0) break;
      if ((cache.state & 0x1F) == 0x1F) break;
      const int nm = (int)(((uint32_t)cache.state >> 8) & 0xFF);
      if (nm > minMismatches) break;
      const int ubs = stateScore(cache, 0, true);
      if (ubs < 0 || ubs < bestScore) break;
      if (!siText(cache)) break;
      const int nb = qcode(cStrand(cache), cNextIdx(cache));
      if ((cache.state & (1 << nb)) != 0 || siIsEmpty(cache, nb)) break;
      // (the parent's checked flag for nb is not recorded: the parent is never read again, and the
      // child takes only the priority bits of the parent's state word)
      DState<R> d;
      const int fm0 = numFMIndexSearches, ts0 = textSteps;
      const bool ok = buildChild(cache, nb, d);
      if (!ok) {  // a rejected first child: the state goes through the loop as the reference runs it
        numFMIndexSearches = fm0;
        textSteps = ts0;
        break;
      }
      cache = d;
      moved = 1;
    }
    if (!moved) return ns;
    // ns (the run's first state, deferred or written) is never referenced: the run's last state
    // takes its place in the queue
    const int id = allocState();
    if (id < 0) return -2;
    cacheDirty = 0;
    cacheIdx = id;
    if (deferrable(cache)) cacheDirty = 1;
    else { GWA_PW(PR_WA, PR_EA, sizeof(DState<R>)); L.arena()[id] = cache; }
    return id;
  }

  // AlignmentProcess.align (:210-268) minus the record conversion (host side, sam.cpp)
  GWA_HD void initRead(const uint8_t *codes, int m_) {
    rd = codes;
    m = m_;
    k = getMaximumEditDistance(m);
    minMismatches = k + 1;
    maxMatchLength = 0;
    bestScore = -1;
    numFMIndexSearches = 0;
    nStates = heapSize = nHits = listSize = nCigar = listOk = 0;
    cacheIdx = -1;
    cacheDirty = 0;
    xMode = 0;
    status = ST_UNMAPPED;
    ovfWhat = 0;
    stairBad = 0;
    stairInLds = 0;
    stairTab = nullptr;
    if (st.base) {
      const uint32_t b = st.base[m];
      stairBad = b >= 0xFFFFFFFEu ? ~0ULL : st.bad[m];
      stairInLds = (stairLds != nullptr && m == st.ldsM) ? 1 : 0;
      stairTab = st.tab + (b >= 0xFFFFFFFEu ? 0 : b);
    }
    quickSteps = blocks = saReads = maxHeap = kmerLookups = shortSteps = textSteps = textRuns = 0;
    tcW2 = tcWN = -1;
    numSW = verifyBytes = 0;
  }
  // AlignmentProcess.align (:210-268) after the search: pick the reported chains
  GWA_HD void writeSearchOutput(OutHeader *oh, const OutSlots &os, uint32_t rd_) {
    GWA_PW(PR_WO, PR_EO, 16 * 4);
    oh->fmSearches = numFMIndexSearches;
    oh->searchBlocks = blocks;
    oh->saReads = saReads;
    oh->searchShort = textSteps;
    oh->states = nStates;
    oh->maxHeap = maxHeap;
    oh->numSW = numSW;
    oh->verifyBytes = verifyBytes;
    oh->nChains = 0;
    oh->nHits = 0;
    oh->nCigar = 0;
    oh->poolFail = 0;
    oh->ovfWhat = ovfWhat;
    if (status == ST_OVERFLOW || status == ST_ERROR) { oh->status = status; return; }
    bool hasHitF = minMismatches <= k && listSize > 0;
    if (!hasHitF) { oh->status = ST_UNMAPPED; return; }
    int nRep = cfg.reportType == 0 ? 1 : cfg.reportType == 1 ? listSize : (cfg.topL < listSize ? cfg.topL : listSize);
    // room: the read's fixed slot, or a reservation in the shared pool (OutSlots)
    uint32_t needH = 0, needC = 0;
    for (int r = 0; r < nRep; ++r)
      for (int t = L.list()[r]; t >= 0; t = L.hits()[t].next) {
        ++needH;
        needC += (uint32_t)L.hits()[t].cigarLen;
      }
    uint64_t hb = (uint64_t)rd_ * os.hitCap, cb = (uint64_t)rd_ * os.cigCap;
    if (needH > os.hitCap || needC > os.cigCap) {
      hb = os.poolHit0 + outReserve(os.poolUsed, needH);
      cb = os.poolCig0 + outReserve(os.poolUsed + 1, needC);
      if (hb + needH > os.poolHitEnd || cb + needC > os.poolCigEnd) {
        outReserve(os.poolUsed + 2, 1);
        oh->status = ST_OVERFLOW;
        oh->poolFail = 1;
        return;
      }
    }
    OutHit *oHits = os.hits + hb;
    uint16_t *oCig = os.cig + cb;
    uint32_t nh = 0, ncg = 0;
    for (int r = 0; r < nRep; ++r) {
      int prevOut = -1;
      for (int t = L.list()[r]; t >= 0; t = L.hits()[t].next) {
        const DHit &h = L.hits()[t];
        OutHit &o = oHits[nh];
        o.chr = h.chr; o.pos = h.pos; o.matchLength = h.matchLength; o.qStart = h.qStart; o.qEnd = h.qEnd;
        o.diff = h.diff; o.strand = h.strand; o.numHits = h.numHits; o.next = -1;
        o.cigarOff = ncg;
        o.cigarLen = (uint32_t)h.cigarLen;
        GWA_PW(PR_WO, PR_EO, sizeof(OutHit) + 2 * h.cigarLen);
        for (int i = 0; i < h.cigarLen; ++i) oCig[ncg++] = L.cigar()[h.cigarOff + i];
        if (prevOut >= 0) oHits[prevOut].next = (int32_t)nh;
        prevOut = (int)nh;
        ++nh;
      }
    }
    oh->hitOff = (uint32_t)hb;
    oh->cigOff = (uint32_t)cb;
    oh->nChains = nRep;
    oh->nHits = (int32_t)nh;
    oh->nCigar = (int32_t)ncg;
    oh->status = ST_MAPPED;
  }

  // AlignmentScoreConfig.getMaximumEditDistance (A/AlignmentScoreConfig.java:40-47)
  GWA_HD int getMaximumEditDistance(int readLength) const {
    if (cfg.k > 0 && cfg.k < 1) return (int)floor((double)((float)readLength * cfg.k));
    return (int)cfg.k;
  }
};

}  // namespace gwa
