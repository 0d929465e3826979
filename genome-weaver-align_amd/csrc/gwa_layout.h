// gwa_layout.h -- device data layouts of the MI355X-native aligner.
//
// HBM layout (one replica per GPU, built once by index_build.cpp):
//   OccBlock occ[2][N/128+1]   forward-text BWT (fm 0) and reverse-text BWT (fm 1);
//                               one 64-B block per 128 BWT positions = one HBM burst
//   uint32_t sa[2][N]          FULL suffix arrays (the reference samples every 32nd entry and
//                               LF-walks up to 31 steps, A/SparseSuffixArray.java:141-158; with
//                               288 GB of HBM we keep every entry: 1 gather instead of <=31)
//   uint64_t text2[N/32+1]     forward text, 2-bit codes (N stored as A) ...
//   uint64_t textN[N/64+1]     ... plus its N bitmap  (verification windows)
//   int64_t  contigOff[n]      contig start offsets (SequenceBoundary)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GWA_HD __host__ __device__ __forceinline__
#define GWA_HDNI __host__ __device__ __noinline__
#else
#define GWA_HD inline
#define GWA_HDNI
#endif

namespace gwa {

// One Occ block: counts of A,C,G,T in bwt[0, 128*b), then the 128 codes of the block as two
// bit planes (lo = code&1, hi = code>>1; position p at bit p%64 of word p/64) and the N bitmap.
// N positions carry code 0 in the planes; occ(A) subtracts them, occ(N) = i - sum(ACGT).
// Reproduces OccurrenceCountTable.getOcc/getOccACGTN (A/OccurrenceCountTable.java:80-107)
// with W = 128 (A/FMIndexOnGenome.java:46).
struct alignas(64) OccBlock {
  uint32_t cnt[4];
  uint64_t lo[2];
  uint64_t hi[2];
  uint64_t nmask[2];
};
static_assert(sizeof(OccBlock) == 64, "OccBlock must be one 64-byte burst");

struct IndexView {
  const OccBlock *occ[2];  // [0] forward index (BWT of T), [1] reverse index (BWT of reverse(T))
  const uint32_t *sa[2];   // full cyclic suffix arrays of T and reverse(T)
  const uint64_t *text2;   // T, 2-bit codes, 32 per word, LSB-first
  const uint64_t *textN;   // T, N bitmap, 64 per word
  const int64_t *contigOff;
  int32_t nContig;
  int32_t kmerK;           // k of the k-mer interval tables (0 = none)
  uint64_t N;
  uint64_t C[5];  // CharacterCount.C (A/CharacterCount.java:41-50); identical for both strands
  // Per index: the suffix interval reached by kmerK backward-search steps from [0, N) over each
  // k-mer (first-processed base in the high bits), packed ub << 32 | lb; 0 = a step was empty.
  // FMQuickScan restarts from [0, N) (S/FMQuickScan.java:80-89), so one lookup replaces its next
  // kmerK steps whenever the k-mer occurs.
  const uint64_t *kmer[2];
};

// k of the k-mer tables for a text of n bases: about log4(n) - 1, in [6, 14] (0 below 4^7)
inline int kmerKFor(uint64_t n) {
  int l = 0;
  while (l < 31 && (1ULL << (2 * (l + 1))) <= n) ++l;  // l = floor(log4 n)
  const int k = l - 1;
  return k < 6 ? 0 : k > 14 ? 14 : k;
}

// AlignmentConfig + AlignmentScoreConfig fields read on the BSF path
// (S/BidirectionalSuffixFilter.java:250,461,539,785; A/AlignmentScoreConfig.java:37-77)
struct SearchConfig {
  float k;
  int32_t reportType;  // 0 BESTHIT, 1 ALLHITS, 2 TOPL
  int32_t topL;
  int32_t numSplit;
  int32_t matchScore, mismatchPenalty, splitOpenPenalty;
  int32_t indelEndSkip, bandWidth;
  // scheduler (not a reference option): a wavefront runs its parked reports once they are at least
  // waitQ16/16 of its live lanes
  int32_t waitQ16;
  // 1: search states whose pattern occurs once step by text compares (M_TEXT).  Exact for
  // numSplit <= 1, where no split changes a state's search direction (BsfLane::nextSi)
  int32_t textSearch;
  // BsfLane::runAhead: at most this many text-mode match steps run back to back per search step
  // (0 = off).  A lane running ahead holds its wavefront, so long runs cost the other lanes time.
  int32_t runAheadMax;
  // 1: every text-mode FM step reads the text through the lane's one-word cache (BsfLane::refCodeCached),
  // kept across search steps (the states of one read mostly walk one text neighbourhood)
  int32_t textCache;
  // scheduler: a wavefront's idle lanes take new reads once at least this many are idle (or all its
  // live lanes are); 1 = each lane as soon as it is idle
  int32_t refillMin;
};

// Read batch as resident in HBM: one byte code (0..4) per base; every read starts at a 16-B
// aligned offset and is zero-padded to a multiple of 16 B, so a lane loads it 16 codes at a time.
struct ReadsView {
  const uint8_t *codes;
  const uint32_t *off;  // n offsets into codes (multiples of 16)
  const uint32_t *len;  // n read lengths
  uint32_t n;
};

// Staircase-mask tables (StaircaseFilter.getStairCaseMask64bit, S/StaircaseFilter.java:91-102),
// precomputed on the host per read length m for every minMismatches value kk in [0, kmax+1],
// row in [0, kmax], offset in [-kmax, m]:  tab[base(m) + ((kk*(kmax+1) + row)*(m+kmax+1) + offset+kmax)]
struct StairTables {
  const uint64_t *tab;
  const uint32_t *base;  // per m (0..kMaxReadLen), index into tab; 0xFFFFFFFF = no table
  int32_t kmax;
  int32_t ldsM;          // reads of this length use a copy of their table staged in LDS (-1 = none)
  uint32_t ldsBase, ldsCount;  // that table: tab[ldsBase, ldsBase + ldsCount)
  const uint64_t *bad;   // per m: bit kk set when StaircaseFilter(m, kk) throws (S/StaircaseFilter.java:47-72)
};
constexpr int kStairLdsWords = 2048;  // 16 KiB of LDS per workgroup
// Longest read of the device path: 16 two-bit query words per strand (QW = 16), 10-bit read positions
// in the queue key (BsfLane::packKey), 16-bit cursor fields (DState)
constexpr int kMaxReadLen = 512;
constexpr int kLdsHeap = 8;           // first-tier priority-queue capacity (entries, in LDS)
constexpr int kDeepLdsHeap = 8192;    // LDS queue entries per workgroup of a sparse deep tier (64 KiB)
constexpr int kSfLdsHeap = 2048;      // -m sf cooperative kernel: LDS queue entries per wavefront (4 per workgroup)
constexpr int kSfDJobs = 63;          // -m sf cooperative kernel: deferred verifications per pass (lanes 1-63)
constexpr int kSfULog = 32768;        // -m sf cooperative kernel: undo-log entries (16 B) per read

// ---- per-read output ----
enum : int32_t {
  ST_UNMAPPED = 0,  // emitted "*" record
  ST_MAPPED = 1,
  ST_OVERFLOW = 2,  // a per-lane capacity was exceeded: rerun on a larger tier
  ST_ERROR = 3,     // the reference would abort with an exception (ReadHit null/NPE etc)
  ST_TOO_LONG = 4,  // read longer than the device path supports
};

// OutHeader.ovfWhat: the per-lane capacities a ST_OVERFLOW read exceeded (Caps fields)
enum : int32_t {
  OV_ARENA = 1, OV_HEAP = 2, OV_HITS = 4, OV_CIGAR = 8, OV_LIST = 16, OV_CAND = 32,
  OV_CHAIN = 64,   // a split chain of more than 8 pieces (sortSplits)
  OV_DP = 128,     // a DP window / history larger than the lane's (fixed by the read length)
  OV_SLICE = 256,  // a traceback left the first tier's DP slice (any later tier keeps whole columns)
};

// chr codes in OutHit.chr
enum : int32_t { CHR_NULL = -1, CHR_EMPTY = -2, CHR_STAR = -3 };

struct OutHit {           // one ReadHit (R/ReadHit.java:42-53)
  int32_t chr;            // contig index or CHR_*
  int32_t pos;
  int32_t matchLength, qStart, qEnd, diff;
  int32_t strand, numHits;
  int32_t next;           // index of nextSplit within the record's hits, -1 = none
  uint32_t cigarOff, cigarLen;  // ops [cigarOff, cigarOff + cigarLen) of the record's CIGAR area
};

// Per-read output header.  A read's hits are OutHit[hitOff, hitOff + nHits) and its CIGAR ops
// cig[cigOff, cigOff + nCigar); the reported chains lie back to back in report order (chain c + 1
// starts after the last hit of chain c), so no per-chain index is stored and the number of reported
// chains is not bounded (-R allhits reports every hit, S/BidirectionalSuffixFilter.java:240-255).
struct OutHeader {
  int32_t status;
  int32_t nChains;   // reported ReadHit chains (BESTHIT: 1)
  int32_t nHits;     // OutHit entries used
  int32_t nCigar;    // cigar ops used
  uint32_t hitOff, cigOff;
  int32_t poolFail;  // 1: ST_OVERFLOW came from a full output pool, not from a search capacity
  int32_t numSW;     // DP verifications (alignBlockDetailed calls, the reference's numSW)
  // instrumentation: FM steps, quick-scan steps, rank block loads
  int32_t fmSearches, quickSteps, blocks, states;
  int32_t searchBlocks, saReads, maxHeap, kmerLookups;  // maxHeap: heap high-water mark (instrumentation)
  // quick-scan steps answered without Occ blocks (k-mer table or single-row text compare)
  int32_t quickShort, quickSa, searchShort;  // quickSa: SA gathers of the quick scan; searchShort:
  // search FM steps answered by one text character (M_TEXT)
  int32_t verifyBytes;  // SURVEY.md §8d verify bytes: ceil(2n/8) + ceil(n/8) of each n-base window + 32 B Peq per block
  int32_t quickText;    // text-mode runs of the quick scan (each reads one 32-base text window: textWin)
  int32_t ovfWhat;      // ST_OVERFLOW: OV_* bits of the capacities exceeded
};

// Where reads write their reported hits: read r owns the fixed slot hits[r * hitCap, + hitCap) and
// cig[r * cigCap, + cigCap); a read reporting more (-R allhits / topL with many equal hits, long
// split chains) reserves room in the shared pool behind the slots with one atomic bump per array.
// A reservation past the pool end marks the read ST_OVERFLOW with poolFail = 1; the host grows the
// pool and reruns it (gwa_batch_run).
struct OutSlots {
  OutHit *hits;
  uint16_t *cig;
  uint32_t hitCap, cigCap;
  uint32_t *poolUsed;            // [0] hits, [1] cigar ops reserved so far, [2] reads refused
  uint64_t poolHit0, poolHitEnd; // pool = hits[poolHit0, poolHitEnd)
  uint64_t poolCig0, poolCigEnd; //        cig[poolCig0, poolCigEnd)
};

GWA_HD uint32_t outReserve(uint32_t *ctr, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAdd(ctr, v);
#else
  const uint32_t o = *ctr;  // host replay (tests/hostcore) is one read at a time
  *ctr = o + v;
  return o;
#endif
}

// Paired-end mate rescue (orc_align_pairs rule 3, the build's own design): per pair, the rescued
// mate's hit when the pair had no proper pair and only one mate had candidates
constexpr int kRescueCig = 64;     // CIGAR ops of a rescued hit (at most 2 kr + 3 <= 53 for m <= 255)
constexpr int kRescueWindow = 320; // longest rescue window (bases)
struct RescueOut {
  int32_t status;  // 0 none, 1 mate 1 rescued, 2 mate 2 rescued
  // the pair choice (rules 1-2), hit indices into the batch's hit pool, -1 = none: a / b = the proper
  // pair with the fewest differences, fa / fb = each mate's first candidate
  int32_t a, b, fa, fb;
  OutHit hit;      // cigarOff 0 into cig
  uint16_t cig[kRescueCig];
};
// pairs whose candidate counts multiply past kPairQuad are chosen by pair_choose_kernel (sorted
// sweep, O(na log na + nb log nb)) instead of the all-pairs loop (tests lower both limits with
// GWA_PAIR_QUAD / GWA_PAIR_SORT_CAP to drive every pair through the sweep or its fallback)
constexpr int64_t kPairQuad = 64;
constexpr int kPairSortCap = 4096;  // candidates of both mates one workgroup sorts in LDS

// Resume records of the reads a search tier suspends (BsfLane::suspendTo / resumeFrom): record i
// belongs to entry i of the tier's overflow list (= the next tier's read list); a tier reads `in`
// (the previous tier's records) and writes `out` (null: none kept, the reads restart)
struct ResumeBufs {
  const uint8_t *in;
  uint8_t *out;
  uint64_t inStride, outStride;
  uint32_t inCap, outCap;
};

// quick-scan outcome carried from fm_quickscan to bsf_search (FMQuickScan fields used at
// S/BidirectionalSuffixFilter.java:324-346)
struct ScanRes {
  int32_t nmF, lmF, nmR, lmR;
  int32_t feF, feR;  // each strand's first empty step (m: none): the search-list sort key only
};

// CIGAR op = (len << 3) | type ; type: M0 I1 D2 N3 S4 H5 P6 X7  (A/CIGAR.java:39-47)
// search-loop profiling regions (-DGWA_PROF builds)
// (cycle regions, then wave / lane execution counts; PR_W* / PR_E*: bytes / lane store events of
// each HBM store site of the search -- arena states, state words, DP history, hit/list/CIGAR/memo
// slices, the output slots; PR_EDW: wave store instructions of the DP history)
enum {
  PR_POLL, PR_REPORT, PR_BOUND, PR_EXP1, PR_ADD1, PR_EXPN, PR_SPLIT, PR_LOOP, PR_VERIFY, PR_NFA, PR_FM, PR_SEED,
  PR_NVW, PR_NVL, PR_NSW, PR_NSL, PR_DPF, PR_DPT, PR_NWAIT, PR_NBW, PR_NBL,
  PR_WA, PR_EA, PR_WS, PR_ES, PR_WD, PR_ED, PR_EDW, PR_WH, PR_EH, PR_WO, PR_EO,
  PR_N = 34
};

}  // namespace gwa
