// gwa_api.cpp -- C-ABI implementation (include/gwa.h): index residency in HBM, batch
// orchestration (quick-scan kernel -> work list -> search kernel tiers), SAM formatting.
#include "../../include/gwa.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "bsf_core.h"
#include "sf_core.h"
#include "host_index.h"
#include "kernels.h"
#include "sam.h"
#include "sam_core.h"

using namespace gwa;

static thread_local std::string g_err;

namespace {

struct HipError : std::runtime_error {
  explicit HipError(const std::string &m) : std::runtime_error(m) {}
};
#define HIPCHK(x)                                                                                          \
  do {                                                                                                     \
    hipError_t e_ = (x);                                                                                   \
    if (e_ != hipSuccess) throw HipError(std::string(#x) + ": " + hipGetErrorString(e_));                  \
  } while (0)

template <class T>
T *devAlloc(size_t n, size_t *acc = nullptr) {
  void *p = nullptr;
  size_t b = std::max<size_t>(n * sizeof(T), 64);
  HIPCHK(hipMalloc(&p, b));
  if (acc) *acc += b;
  return (T *)p;
}
template <class T>
T *devUpload(const std::vector<T> &v, hipStream_t s, size_t *acc) {
  T *p = devAlloc<T>(v.size(), acc);
  if (!v.empty()) HIPCHK(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return p;
}

// Device memory and streams of batches, kept per device for reuse: a pipeline creates and frees one
// batch per chunk of a read file, and hipFree / hipStreamDestroy wait for the whole device, so each
// free would stall the kernels other host threads' batches have in flight.  A freed buffer goes back
// only after the stream that used it is drained (that stream alone).
struct DevCache {
  std::mutex mu;
  std::multimap<size_t, void *> free;         // cached blocks by size
  std::unordered_map<void *, size_t> size;    // every block handed out or cached -> its size
  std::vector<hipStream_t> streams;           // idle streams
  size_t cached = 0;
};
DevCache g_devCache[64];
const size_t kDevCacheCap = (size_t)24 << 30;  // cached bytes per device at most

DevCache &devCache() {
  int d = 0;
  (void)hipGetDevice(&d);
  return g_devCache[d & 63];
}
size_t cacheRound(size_t b) {
  b = std::max<size_t>(b, 256);
  int e = 63 - __builtin_clzll(b);
  const size_t step = std::max<size_t>(256, ((size_t)1 << e) / 8);
  return (b + step - 1) / step * step;
}
// give every idle cached block of the current device back to the driver (index close, allocation
// failures): blocks idle in the cache are invisible to hipMemGetInfo
void devCacheTrim() {
  DevCache &c = devCache();
  std::lock_guard<std::mutex> g(c.mu);
  for (auto &kv : c.free) {
    (void)hipFree(kv.second);
    c.size.erase(kv.second);
  }
  c.free.clear();
  c.cached = 0;
}
size_t devCacheIdle() {
  DevCache &c = devCache();
  std::lock_guard<std::mutex> g(c.mu);
  return c.cached;
}
// Per device: reading the free memory and allocating the search scratch it sizes are one step, so
// batches of several host threads (gwa_pipeline workers) cannot each size their scratch from the
// same free memory (gwa_batch_run holds it from scratchBudget to the tier's last allocation).
std::mutex g_allocMu[64];
void *batchMalloc(size_t bytes) {
  DevCache &c = devCache();
  const size_t r = cacheRound(bytes);
  {
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.free.lower_bound(r);
    if (it != c.free.end() && it->first <= r + r / 4) {
      void *p = it->second;
      c.cached -= it->first;
      c.free.erase(it);
      return p;
    }
  }
  void *p = nullptr;
  if (hipMalloc(&p, r) != hipSuccess) {  // give the cached blocks back and try once more
    (void)hipGetLastError();
    devCacheTrim();
    HIPCHK(hipMalloc(&p, r));
  }
  std::lock_guard<std::mutex> g(c.mu);
  c.size[p] = r;
  return p;
}
// p back to the cache once stream s (the last user of p; nullptr: none pending) has drained
void batchFree(void *p, hipStream_t s) {
  if (!p) return;
  if (s) (void)hipStreamSynchronize(s);
  DevCache &c = devCache();
  std::unique_lock<std::mutex> g(c.mu);
  auto it = c.size.find(p);
  if (it == c.size.end()) {  // (not a cached block)
    g.unlock();
    (void)hipFree(p);
    return;
  }
  if (c.cached + it->second > kDevCacheCap) {
    c.size.erase(it);
    g.unlock();
    (void)hipFree(p);
    return;
  }
  c.cached += it->second;
  c.free.insert({it->second, p});
}
template <class T>
T *bAlloc(size_t n) {
  return (T *)batchMalloc(std::max<size_t>(n * sizeof(T), 64));
}
template <class T>
T *bUpload(const std::vector<T> &v, hipStream_t s) {
  T *p = bAlloc<T>(v.size());
  if (!v.empty()) HIPCHK(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return p;
}
hipStream_t batchStream() {
  DevCache &c = devCache();
  {
    std::lock_guard<std::mutex> g(c.mu);
    if (!c.streams.empty()) {
      hipStream_t s = c.streams.back();
      c.streams.pop_back();
      return s;
    }
  }
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return s;
}
void batchStreamDone(hipStream_t s) {
  if (!s) return;
  (void)hipStreamSynchronize(s);
  DevCache &c = devCache();
  std::lock_guard<std::mutex> g(c.mu);
  c.streams.push_back(s);
}

int fail(const std::string &m) {
  g_err = m;
  return -1;
}

}  // namespace

// error path shared with reads_io.cpp (sets gwa_last_error)
extern "C" int gwa_fail_message(const char *msg) { return fail(msg); }

struct gwa_index {
  int device = 0;
  hipStream_t stream = nullptr;
  HostIndex host;
  OccBlock *d_occ[2] = {nullptr, nullptr};
  uint32_t *d_sa[2] = {nullptr, nullptr};
  uint64_t *d_text2 = nullptr, *d_textN = nullptr;
  uint64_t *d_kmer[2] = {nullptr, nullptr};
  int64_t *d_contig = nullptr;
  int32_t *d_chrRank = nullptr;  // String.compareTo rank of each contig name (also its SAM name key)
  char *d_ctg = nullptr;         // contig names (SAM RNAME / RNEXT text)
  uint64_t *d_ctgOff = nullptr;
  int32_t starKey = -3, emptyKey = -2;  // name keys of "*" and "" (SamText)
  size_t bytes = 0;
  IndexView view{};
  // Search scratch buffers, reused across batches: a running batch takes one from the pool and puts
  // it back after its tiers, so batches of several host threads run their kernels concurrently on
  // the device (each on its own stream and scratch; gwa_pipeline), one buffer per concurrent batch.
  std::mutex scratchMu;
  std::vector<std::pair<uint8_t *, size_t>> scratchFree;
  size_t scratchHeld = 0;  // bytes of every buffer, in the pool or taken
};

namespace {
// a scratch buffer of the index's pool for the duration of one gwa_batch_run
struct Scratch {
  gwa_index *ix;
  hipStream_t s;  // the batch's stream: drained before the buffer goes back to the pool
  uint8_t *p = nullptr;
  size_t bytes = 0;
  Scratch(gwa_index *x, hipStream_t st) : ix(x), s(st) {
    std::lock_guard<std::mutex> g(ix->scratchMu);
    if (!ix->scratchFree.empty()) {  // the largest free one
      size_t best = 0;
      for (size_t i = 1; i < ix->scratchFree.size(); ++i)
        if (ix->scratchFree[i].second > ix->scratchFree[best].second) best = i;
      p = ix->scratchFree[best].first;
      bytes = ix->scratchFree[best].second;
      ix->scratchFree.erase(ix->scratchFree.begin() + (long)best);
    }
  }
  // at least `need` bytes (the old contents are not kept)
  void ensure(size_t need) {
    if (need <= bytes) return;
    release();
    if (hipMalloc(&p, need) != hipSuccess) {
      // memory held idle elsewhere in this process: the device cache's blocks and the index's
      // idle scratch buffers (other batches' are in use) -- given back, then one more try
      (void)hipGetLastError();
      p = nullptr;
      devCacheTrim();
      {
        std::lock_guard<std::mutex> g(ix->scratchMu);
        for (auto &f : ix->scratchFree) {
          (void)hipFree(f.first);
          ix->scratchHeld -= f.second;
        }
        ix->scratchFree.clear();
      }
      HIPCHK(hipMalloc(&p, need));
    }
    bytes = need;
    std::lock_guard<std::mutex> g(ix->scratchMu);
    ix->scratchHeld += need;
  }
  // give the memory back to the device (a grown tier's tens of GiB for a few reads)
  void release() {
    if (!p) return;
    (void)hipStreamSynchronize(s);
    (void)hipFree(p);
    std::lock_guard<std::mutex> g(ix->scratchMu);
    ix->scratchHeld -= bytes;
    p = nullptr;
    bytes = 0;
  }
  ~Scratch() {
    if (!p) return;
    (void)hipStreamSynchronize(s);  // (an error path may leave a kernel of this batch running)
    std::lock_guard<std::mutex> g(ix->scratchMu);
    ix->scratchFree.push_back({p, bytes});
  }
};
}  // namespace

struct gwa_batch {
  gwa_index *ix = nullptr;
  hipStream_t stream = nullptr;
  gwa_config_t cfg{};
  SearchConfig scfg{};
  uint32_t n = 0;
  bool hasQual = false;
  int maxM = 0, kmax = 0, R = 4;
  bool sfWrap = false;  // some read's -m sf prefix-scan chunks wrap (sfChunksWrap): the WRAP kernel instance
  // the read text in HBM: bases (encoded on the device into d_codes), names and qualities (read by
  // the SAM writer).  Read r's bases are d_seqText[d_seqB[r], d_seqE[r]) etc.: SoA blobs (E = B + 1)
  // or, from the pipeline, the fields of FASTQ records inside one copy of the file text.
  char *d_seqText = nullptr, *d_nameText = nullptr, *d_qualText = nullptr;
  const uint64_t *d_seqB = nullptr, *d_seqE = nullptr, *d_nameB = nullptr, *d_nameE = nullptr;
  const uint64_t *d_qualB = nullptr, *d_qualE = nullptr;
  uint8_t *d_qualNull = nullptr;  // per read: nonzero = no quality (gwa_reads_t.qual_null), or nullptr
  uint64_t *d_fieldOwn[3] = {nullptr, nullptr, nullptr};  // the allocations behind the field arrays
  // SAM formatting buffers (grown on demand) and the statistics accumulator
  uint64_t *d_fmtLen = nullptr, *d_fmtOff = nullptr;
  uint32_t *d_fmtIdx = nullptr, *d_fmtErr = nullptr;
  void *d_fmtTmp = nullptr;
  char *d_fmtText = nullptr;
  size_t fmtCap = 0, fmtTmpBytes = 0, fmtTextCap = 0;
  uint64_t fmtBytes = 0;  // the text of the last formatting, and whether it was the whole batch
  bool fmtWhole = false;
  unsigned long long *d_stats = nullptr;
  bool statsDone = false;
  // device encoding of the read text (gwa_batch_run re-encodes every run: the timed path starts
  // from the text in HBM, as the reference's per-read call starts from the Read's String)
  uint32_t *d_row = nullptr, *d_seen = nullptr;
  void *d_encTmp = nullptr;
  size_t encTmpBytes = 0;
  // device
  uint8_t *d_codes = nullptr;
  uint32_t *d_off = nullptr, *d_len = nullptr;
  ScanRes *d_sres = nullptr;
  OutHeader *d_oh = nullptr;
  OutHit *d_hits = nullptr;
  uint16_t *d_cig = nullptr;
  uint32_t *d_list[2] = {nullptr, nullptr};
  uint32_t *d_all = nullptr;    // -m sf: every read (0..n-1) is searched
  uint32_t *d_count = nullptr;  // [0] search list, [1 + t] overflow list of tier t, [8 + t] tier t work counter
  uint64_t *d_stair = nullptr;
  uint32_t *d_stairBase = nullptr;
  uint64_t *d_stairBad = nullptr;
  uint32_t hitCap = 4, cigCap = 64;
  uint64_t poolHits = 0, poolCig = 0;  // OutSlots pool behind the fixed slots (grown on demand)
  uint64_t poolUsedH = 0, poolUsedC = 0;
  StairTables st{};
  gwa_batch_stats_t stats{};
  bool ran = false;
  bool headerOnly = false;  // -m bd / -m bwa: the reference emits no SAM records (see gwa_batch_create)
  uint32_t pairs = 0;       // paired-end batch: mate 1 of pair i = read i, mate 2 = read pairs + i
  int32_t minIns = 0, maxIns = 0;
  RescueOut *d_rescue = nullptr;  // paired-end: per pair, the pair choice and mate rescue (pair_rescue_kernel)
  uint32_t *d_heavy = nullptr;     // paired-end: [pairs] heavy-pair list + its count (pair_choose_kernel)
  std::vector<std::pair<uint32_t, int>> deep;  // (read, tier) of every read rerun on a tier >= 1
};

static void freeIndexDev(gwa_index *ix) {
  for (int s = 0; s < 2; ++s) {
    if (ix->d_occ[s]) (void)hipFree(ix->d_occ[s]);
    if (ix->d_sa[s]) (void)hipFree(ix->d_sa[s]);
  }
  if (ix->d_text2) (void)hipFree(ix->d_text2);
  for (int f = 0; f < 2; ++f)
    if (ix->d_kmer[f]) (void)hipFree(ix->d_kmer[f]);
  if (ix->d_textN) (void)hipFree(ix->d_textN);
  if (ix->d_contig) (void)hipFree(ix->d_contig);
  if (ix->d_chrRank) (void)hipFree(ix->d_chrRank);
  if (ix->d_ctg) (void)hipFree(ix->d_ctg);
  if (ix->d_ctgOff) (void)hipFree(ix->d_ctgOff);
  for (auto &f : ix->scratchFree) (void)hipFree(f.first);
  ix->scratchFree.clear();
  if (ix->stream) (void)hipStreamDestroy(ix->stream);
  devCacheTrim();  // (the device's idle batch buffers: no batch of a closed index reuses them)
}

namespace gwa {
bool cyclicSAGpu(const uint8_t *d_T, uint64_t N, uint32_t *d_sa, int alphabetBits, hipStream_t s);
void reverseTextGpu(const uint8_t *d_T, uint64_t N, uint8_t *d_R, hipStream_t s);
void buildOccGpu(const uint8_t *d_T, const uint32_t *d_sa, uint64_t N, OccBlock *d_occ, hipStream_t s);
void packTextGpu(const uint8_t *d_T, uint64_t N, uint64_t *d_text2, uint64_t *d_textN, hipStream_t s);
void unpackTextGpu(const uint64_t *d_text2, const uint64_t *d_textN, uint64_t N, uint8_t *d_T, hipStream_t s);
void countCodesGpu(const uint8_t *d_T, uint64_t N, unsigned long long *d_cnt5, hipStream_t s);
}  // namespace gwa

// Index construction in HBM (the `bwt` command's work, A/BWTransform.java:72-179) from the text
// codes already on the device (dT, N bytes; freed here): the reversed text, both cyclic SAs, both
// Occ-block arrays, the 2-bit text (unless a saved index supplied it), the symbol counts, the contig
// table and the k-mer tables.
static void buildFromDeviceText(gwa_index *ix, uint8_t *dT) {
  HostIndex &h = ix->host;
  hipStream_t s = ix->stream;
  const uint64_t N = h.N;
  uint8_t *dR = nullptr;
  try {
    dR = devAlloc<uint8_t>(N);
    reverseTextGpu(dT, N, dR, s);
    ix->d_sa[0] = devAlloc<uint32_t>(N, &ix->bytes);
    ix->d_sa[1] = devAlloc<uint32_t>(N, &ix->bytes);
    // cyclic suffix arrays (A/sais/CyclicSAIS.java:223-431 computes the same unique order)
    if (!cyclicSAGpu(dT, N, ix->d_sa[0], 3, s) || !cyclicSAGpu(dR, N, ix->d_sa[1], 3, s))
      throw std::runtime_error("reference text is periodic (cyclic rotations tie): unsupported");
    const uint64_t nb = N / 128 + 1;
    ix->d_occ[0] = devAlloc<OccBlock>(nb, &ix->bytes);
    ix->d_occ[1] = devAlloc<OccBlock>(nb, &ix->bytes);
    buildOccGpu(dT, ix->d_sa[0], N, ix->d_occ[0], s);
    buildOccGpu(dR, ix->d_sa[1], N, ix->d_occ[1], s);
    if (!ix->d_text2) {
      const uint64_t nw = N / 64 + 1;
      ix->d_text2 = devAlloc<uint64_t>(2 * nw, &ix->bytes);
      ix->d_textN = devAlloc<uint64_t>(nw, &ix->bytes);
      packTextGpu(dT, N, ix->d_text2, ix->d_textN, s);
    }
    // CharacterCount.C (A/CharacterCount.java:41-50)
    unsigned long long *dCnt = devAlloc<unsigned long long>(5);
    countCodesGpu(dT, N, dCnt, s);
    unsigned long long count[5];
    HIPCHK(hipMemcpyAsync(count, dCnt, sizeof(count), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    (void)hipFree(dCnt);
    uint64_t sum = 0;
    for (int c = 0; c < 5; ++c) { h.C[c] = sum; sum += count[c]; }
  } catch (...) {
    (void)hipFree(dT);
    if (dR) (void)hipFree(dR);
    throw;
  }
  (void)hipFree(dT);
  (void)hipFree(dR);
  rankNames(h);
  ix->d_contig = devUpload(h.offsets, s, &ix->bytes);
  ix->d_chrRank = devUpload(h.chrRank, s, &ix->bytes);
  {  // contig names for the SAM writer
    const SamNames sn = samNames(h);
    std::vector<char> blob(sn.blob.begin(), sn.blob.end());
    blob.push_back(0);
    ix->d_ctg = devUpload(blob, s, &ix->bytes);
    ix->d_ctgOff = devUpload(sn.off, s, &ix->bytes);
    ix->starKey = sn.starKey;
    ix->emptyKey = sn.emptyKey;
  }
  HIPCHK(hipStreamSynchronize(s));
  IndexView &v = ix->view;
  v.occ[0] = ix->d_occ[0]; v.occ[1] = ix->d_occ[1];
  v.sa[0] = ix->d_sa[0]; v.sa[1] = ix->d_sa[1];
  v.text2 = ix->d_text2; v.textN = ix->d_textN;
  v.contigOff = ix->d_contig;
  v.nContig = (int32_t)h.names.size();
  v.N = N;
  for (int c = 0; c < 5; ++c) v.C[c] = h.C[c];
  // k-mer interval tables for FMQuickScan restarts (IndexView::kmer)
  v.kmerK = kmerKFor(N);
  if (const char *e = getenv("GWA_KMER_K")) {  // tuning runs: a larger table, up to log4(N) and 16
    int l = 0;
    while (l < 31 && (1ULL << (2 * (l + 1))) <= N) ++l;
    v.kmerK = std::max(0, std::min({atoi(e), l, 16}));
  }
  if (v.kmerK > 0) {
    const uint64_t nk = 1ULL << (2 * v.kmerK);
    for (int f = 0; f < 2; ++f) {
      ix->d_kmer[f] = devAlloc<uint64_t>(nk, &ix->bytes);
      v.kmer[f] = ix->d_kmer[f];
      buildKmerTable(v, f, v.kmerK, ix->d_kmer[f], s);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
  }
}

static void checkSize(const HostIndex &h) {
  if (h.N == 0) throw std::runtime_error("empty reference");
  if (h.N >= 0xFFFFFFFFull) throw std::runtime_error("reference longer than 2^32-2 bases is not supported");
}

// from the host text codes (h.T, released afterwards: the text lives in HBM from here on)
static void finishAndUpload(gwa_index *ix) {
  HostIndex &h = ix->host;
  checkSize(h);
  HIPCHK(hipSetDevice(ix->device));
  HIPCHK(hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking));
  uint8_t *dT = devAlloc<uint8_t>(h.N);
  HIPCHK(hipMemcpyAsync(dT, h.T.data(), h.N, hipMemcpyHostToDevice, ix->stream));
  buildFromDeviceText(ix, dT);
  std::vector<uint8_t>().swap(h.T);
}

// from a saved index's 2-bit text + N bitmap (gwa_index_save)
static void loadPacked(gwa_index *ix, const std::vector<uint64_t> &text2, const std::vector<uint64_t> &textN) {
  HostIndex &h = ix->host;
  checkSize(h);
  HIPCHK(hipSetDevice(ix->device));
  HIPCHK(hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking));
  ix->d_text2 = devUpload(text2, ix->stream, &ix->bytes);
  ix->d_textN = devUpload(textN, ix->stream, &ix->bytes);
  uint8_t *dT = devAlloc<uint8_t>(h.N);
  unpackTextGpu(ix->d_text2, ix->d_textN, h.N, dT, ix->stream);
  buildFromDeviceText(ix, dT);
}

extern "C" {

void gwa_config_default(gwa_config_t *c) {
  c->k = 0.1f; c->strategy = 0; c->report_type = 0; c->top_l = 5;
  c->num_gap_open = 1; c->num_gap_ext = 4; c->num_split = 1;
  c->match = 1; c->mismatch = 3; c->gap_open = 11; c->gap_ext = 4; c->split_open = 11;
  c->indel_end_skip = 5; c->band_width = 31;
}

const char *gwa_last_error(void) { return g_err.c_str(); }

int gwa_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static int buildCommon(gwa_index *ix, int device, gwa_index_t **out) {
  try {
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) throw std::runtime_error("no HIP device: the gwa align path requires an MI355X GPU");
    if (device < 0 || device >= nd) throw std::runtime_error("invalid device " + std::to_string(device));
    ix->device = device;
    finishAndUpload(ix);
    *out = ix;
    return 0;
  } catch (std::exception &e) {
    freeIndexDev(ix);
    delete ix;
    return fail(e.what());
  }
}

int gwa_index_build_fasta(const char *text, uint64_t len, int device, gwa_index_t **out) {
  auto *ix = new gwa_index();
  packFasta(text, (size_t)len, ix->host);
  return buildCommon(ix, device, out);
}

// Saved index (gwa_index_save): the text as 2-bit words + N bitmap and the contig table; loading
// rebuilds the suffix arrays, Occ blocks and k-mer tables on the GPU (seconds at hg19 size), which is
// faster than reading their 30 GB from storage.  Layout (little endian):
//   "GWAIDX1\n"  u64 N  u32 nContigs  u32 0  { u32 nameLen, name, i64 length } x nContigs
//   u64 nw  u64 text2[2 * nw]  u64 textN[nw]          (nw = N / 64 + 1)
static const char kIdxMagic[8] = {'G', 'W', 'A', 'I', 'D', 'X', '1', '\n'};

static std::string readWholeFile(const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) throw std::runtime_error(std::string("cannot open ") + path);
  std::string t;
  if (fseek(f, 0, SEEK_END) == 0) {
    const long sz = ftell(f);
    if (sz > 0) t.resize((size_t)sz);
    fseek(f, 0, SEEK_SET);
  }
  size_t got = t.empty() ? 0 : fread(&t[0], 1, t.size(), f);
  t.resize(got);
  char buf[1 << 16];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) t.append(buf, r);  // (non-seekable input)
  fclose(f);
  return t;
}

int gwa_index_open(const char *path, int device, gwa_index_t **out) {
  gwa_index *ix = nullptr;
  try {
    const std::string t = readWholeFile(path);
    if (t.size() < 8 || memcmp(t.data(), kIdxMagic, 8) != 0)
      return gwa_index_build_fasta(t.data(), t.size(), device, out);
    ix = new gwa_index();
    HostIndex &h = ix->host;
    size_t pos = 8;
    auto get = [&](void *dst, size_t n) {
      if (pos + n > t.size()) throw std::runtime_error(std::string("truncated index file ") + path);
      memcpy(dst, t.data() + pos, n);
      pos += n;
    };
    uint64_t N = 0;
    uint32_t nc = 0, zero = 0;
    get(&N, 8);
    get(&nc, 4);
    get(&zero, 4);
    int64_t off = 0;
    for (uint32_t i = 0; i < nc; ++i) {
      uint32_t ln = 0;
      get(&ln, 4);
      std::string nm(ln, '\0');
      if (ln) get(&nm[0], ln);
      int64_t L = 0;
      get(&L, 8);
      h.names.push_back(nm);
      h.offsets.push_back(off);
      h.lengths.push_back(L);
      off += L;
    }
    if ((uint64_t)off != N) throw std::runtime_error(std::string("corrupt index file (contig lengths) ") + path);
    uint64_t nw = 0;
    get(&nw, 8);
    if (nw != N / 64 + 1) throw std::runtime_error(std::string("corrupt index file (text size) ") + path);
    std::vector<uint64_t> text2(2 * nw), textN(nw);
    get(text2.data(), text2.size() * 8);
    get(textN.data(), textN.size() * 8);
    h.N = N;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) throw std::runtime_error("no HIP device: the gwa align path requires an MI355X GPU");
    if (device < 0 || device >= nd) throw std::runtime_error("invalid device " + std::to_string(device));
    ix->device = device;
    loadPacked(ix, text2, textN);
    *out = ix;
    return 0;
  } catch (std::exception &e) {
    if (ix) {
      freeIndexDev(ix);
      delete ix;
    }
    return fail(e.what());
  }
}

int gwa_index_save(const gwa_index_t *ix, const char *path) {
  FILE *f = nullptr;
  try {
    const HostIndex &h = ix->host;
    const uint64_t N = h.N, nw = N / 64 + 1;
    std::vector<uint64_t> text2(2 * nw), textN(nw);
    HIPCHK(hipSetDevice(ix->device));
    HIPCHK(hipMemcpy(text2.data(), ix->d_text2, text2.size() * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(textN.data(), ix->d_textN, textN.size() * 8, hipMemcpyDeviceToHost));
    f = fopen(path, "wb");
    if (!f) throw std::runtime_error(std::string("cannot create ") + path);
    auto put = [&](const void *p, size_t n) {
      if (n && fwrite(p, 1, n, f) != n) throw std::runtime_error(std::string("write failed: ") + path);
    };
    const uint32_t nc = (uint32_t)h.names.size(), zero = 0;
    put(kIdxMagic, 8);
    put(&N, 8);
    put(&nc, 4);
    put(&zero, 4);
    for (uint32_t i = 0; i < nc; ++i) {
      const uint32_t ln = (uint32_t)h.names[i].size();
      put(&ln, 4);
      put(h.names[i].data(), ln);
      put(&h.lengths[i], 8);
    }
    put(&nw, 8);
    put(text2.data(), text2.size() * 8);
    put(textN.data(), textN.size() * 8);
    if (fclose(f) != 0) { f = nullptr; throw std::runtime_error(std::string("write failed: ") + path); }
    return 0;
  } catch (std::exception &e) {
    if (f) fclose(f);
    return fail(e.what());
  }
}

int gwa_index_build_codes(const uint8_t *codes, uint64_t n, int32_t n_contigs, const char *const *names,
                          const int64_t *lengths, int device, gwa_index_t **out) {
  auto *ix = new gwa_index();
  HostIndex &h = ix->host;
  h.T.assign(codes, codes + n);
  int64_t off = 0;
  for (int i = 0; i < n_contigs; ++i) {
    h.names.push_back(names[i]);
    h.offsets.push_back(off);
    h.lengths.push_back(lengths[i]);
    off += lengths[i];
  }
  if ((uint64_t)off != n) {
    delete ix;
    return fail("contig lengths do not sum to n");
  }
  h.N = n;
  return buildCommon(ix, device, out);
}

uint64_t gwa_index_text_size(const gwa_index_t *ix) { return ix->host.N; }
uint64_t gwa_index_device_bytes(const gwa_index_t *ix) { return ix->bytes; }

int gwa_index_export_sa(const gwa_index_t *ix, int strand, uint32_t *out) {
  if (strand < 0 || strand > 1) return fail("strand must be 0 or 1");
  try {
    HIPCHK(hipSetDevice(ix->device));
    HIPCHK(hipMemcpy(out, ix->d_sa[strand], ix->host.N * sizeof(uint32_t), hipMemcpyDeviceToHost));
  } catch (std::exception &e) {
    return fail(e.what());
  }
  return 0;
}

int gwa_sam_header(const gwa_index_t *ix, char **text, uint64_t *len) {
  std::string h = samHeader(ix->host);
  *text = (char *)malloc(h.size() + 1);
  memcpy(*text, h.c_str(), h.size() + 1);
  *len = h.size();
  return 0;
}

void gwa_index_close(gwa_index_t *ix) {
  if (!ix) return;
  (void)hipSetDevice(ix->device);
  freeIndexDev(ix);
  delete ix;
}

void gwa_free(void *p) { free(p); }

static void freeBatchDev(gwa_batch *b) {
  void *ps[] = {b->d_codes, b->d_off, b->d_len, b->d_sres, b->d_oh, b->d_hits, b->d_cig, b->d_list[0], b->d_list[1], b->d_all, b->d_count,
                b->d_stair, b->d_stairBase, b->d_stairBad, b->d_fieldOwn[0], b->d_fieldOwn[1], b->d_fieldOwn[2],
                b->d_fmtLen, b->d_fmtOff, b->d_fmtIdx, b->d_fmtErr, b->d_fmtTmp, b->d_fmtText, b->d_stats,
                b->d_row, b->d_seen, b->d_encTmp, b->d_qualNull, b->d_rescue, b->d_heavy};
  if (b->stream) (void)hipStreamSynchronize(b->stream);  // (then every buffer below is idle)
  for (void *p : ps) batchFree(p, nullptr);
  // the text blobs (one allocation may back several of them)
  char *tx[3] = {b->d_seqText, b->d_nameText, b->d_qualText};
  for (int i = 0; i < 3; ++i) {
    bool dup = false;
    for (int j = 0; j < i; ++j) dup = dup || tx[j] == tx[i];
    if (tx[i] && !dup) batchFree(tx[i], nullptr);
  }
  batchStreamDone(b->stream);
  b->stream = nullptr;
}

}  // extern "C"

// Batch set-up shared by every way reads arrive: config, stream; true for -m bd / -m bwa
static bool batchHead(gwa_index *ix, const gwa_config_t *cfg, uint32_t n, gwa_batch *b) {
  if (cfg->strategy < 0 || cfg->strategy > 3) throw std::runtime_error("unknown strategy (-m bsf, sf, bd, bwa)");
  HIPCHK(hipSetDevice(ix->device));
  b->ix = ix;
  b->cfg = *cfg;
  b->n = n;
  if (cfg->strategy >= 2) {
    // -m bd / -m bwa (A/Align.java:124-132): BidirectionalBWT reports BWAState / AlignmentSA objects,
    // which SAMOutput.emit drops (it prints AlignmentRecord only, A/SAMOutput.java:73-82), so the
    // reference's SAM is the header alone.  Same output here, without a search whose results no one
    // reads.
    b->headerOnly = true;
    return true;
  }
  SearchConfig &sc = b->scfg;
  sc.k = cfg->k; sc.reportType = cfg->report_type; sc.topL = cfg->top_l; sc.numSplit = cfg->num_split;
  sc.matchScore = cfg->match; sc.mismatchPenalty = cfg->mismatch; sc.splitOpenPenalty = cfg->split_open;
  sc.indelEndSkip = cfg->indel_end_skip; sc.bandWidth = cfg->band_width;
  // a wavefront runs its parked reports once they are waitQ16/16 of its live lanes; the default is
  // set with the NFA size in batchTail (DESIGN.md §4 sweeps)
  sc.waitQ16 = getenv("GWA_WAITQ16") ? atoi(getenv("GWA_WAITQ16")) : 0;
  sc.refillMin = 1;  // (per tier: gwa_batch_run)
  sc.textSearch = (cfg->num_split <= 1 && !getenv("GWA_NO_TEXT")) ? 1 : 0;
  sc.runAheadMax = getenv("GWA_RUNAHEAD") ? atoi(getenv("GWA_RUNAHEAD")) : 4;
  sc.textCache = getenv("GWA_TEXT_CACHE") ? atoi(getenv("GWA_TEXT_CACHE")) : 0;
  b->stream = batchStream();
  return false;
}

// Once the read text is in HBM (b->d_seqText with d_seqB / d_seqE, names, qualities): encode the
// bases on the device (batch_io.hip: ACGTSequence(String), A/ACGTSequence.java:86-97), build the
// staircase tables of the batch's read lengths and allocate the search and output buffers.
static void batchTail(gwa_batch *b, uint64_t seqBytes) {
  const uint32_t n = b->n;
  const gwa_config_t *cfg = &b->cfg;
  hipStream_t s = b->stream;
  const uint64_t codeBound = seqBytes + 16ull * n + 32;
  if (codeBound > 0xFFFFFFFFull) throw std::runtime_error("read batch too large (> 4 GiB of codes): use fewer reads per batch");
  b->d_codes = bAlloc<uint8_t>(codeBound);
  b->d_off = bAlloc<uint32_t>((size_t)n + 1);
  b->d_len = bAlloc<uint32_t>((size_t)n + 1);
  b->d_row = bAlloc<uint32_t>((size_t)n + 1);
  b->d_seen = bAlloc<uint32_t>(kLenSeen);
  b->encTmpBytes = encodeScanTempBytes(n);
  b->d_encTmp = bAlloc<uint8_t>(b->encTmpBytes);
  // the length pass (read lengths, code offsets, the lengths present); gwa_batch_run encodes
  std::vector<uint32_t> seen(kLenSeen);
  HIPCHK(hipMemsetAsync(b->d_seen, 0, kLenSeen * sizeof(uint32_t), s));
  launchEncode(b->d_seqText, b->d_seqB, b->d_seqE, n, b->d_len, b->d_row, b->d_off, b->d_seen, b->d_codes, b->d_encTmp,
               b->encTmpBytes, 0, s);
  HIPCHK(hipMemcpyAsync(seen.data(), b->d_seen, kLenSeen * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  // the distinct read lengths: maximum length, k per length (AlignmentScoreConfig
  // .getMaximumEditDistance) and the staircase tables
  std::vector<int> lens;
  for (uint32_t m = 0; m < kLenSeen; ++m)
    if (seen[m]) {
      b->maxM = (int)m;
      if ((int)m <= kMaxReadLen) lens.push_back((int)m);
    }
  if (b->maxM > kMaxReadLen)  // 16 query words per strand, 10-bit positions in the queue keys; DESIGN.md §1
    throw std::runtime_error("read longer than " + std::to_string(kMaxReadLen) + " bp in this batch (" +
                             std::to_string(b->maxM) + " bp): the device path aligns reads of at most " +
                             std::to_string(kMaxReadLen) + " bp");
  b->sfWrap = false;
  for (int m : lens) {
    int k = (cfg->k > 0 && cfg->k < 1) ? (int)floor((double)((float)m * cfg->k)) : (int)cfg->k;
    b->kmax = std::max(b->kmax, k);
    if (m > 0 && k >= 0 && k <= 31 && sfChunksWrap(m, k + 1)) b->sfWrap = true;  // -m sf kernel instance
  }
  if (b->kmax > 31) throw std::runtime_error("k > 31 is not supported on the device path");
  {  // the -m bsf queue keys hold score() in 24 bits (BsfLane::packKey): |score| < 2^23 for these
     // scores; the -m sf keys (SfLane::keyOf) hold it in 32 bits and have no split chains
    const bool sfPath = cfg->strategy == 1;
    const int64_t s = sfPath ? 0 : std::max(1, cfg->num_split), T = (s + 1) * s / 2;
    const int64_t M = std::llabs((int64_t)cfg->match), Nn = std::llabs((int64_t)cfg->mismatch);
    const int64_t S = std::llabs((int64_t)cfg->split_open);
    const int64_t bound = M * b->maxM + (M + Nn) * (255 * (s + 1) + T) + S * T;
    const int lim = sfPath ? 31 : 23;
    if ((!sfPath && cfg->num_split > 64) || bound >= (1LL << lim))
      throw std::runtime_error("scoring parameters too large for the device's queue keys (|score| may reach " +
                               std::to_string(bound) + ", limit 2^" + std::to_string(lim) + ")");
  }
  b->R = b->kmax + 1 <= 4 ? 4 : b->kmax + 1 <= 8 ? 8 : b->kmax + 1 <= 16 ? 16 : 32;
  // report-batch threshold: 14/16 for k <= 3 (C2: 14-16 tie, 12 is 2 % slower; hg19r favours 14),
  // 8/16 for k >= 4 (C4 -m bsf, round-4 tiers: 6 / 8 / 10 / 12 -> 323-330 / 315-316 / 320-330 / 346 ms
  // per 1M reads, tier 0 109 ms at 8 against 113-114 at 10)
  if (b->scfg.waitQ16 <= 0) b->scfg.waitQ16 = b->R >= 8 ? 8 : 14;
  std::vector<uint64_t> tab, bad;
  std::vector<uint32_t> base;
  buildStairTables(lens, std::max(b->kmax, 0), tab, base, bad);
  b->d_stair = bUpload(tab, s);
  b->d_stairBase = bUpload(base, s);
  b->d_stairBad = bUpload(bad, s);
  b->st.tab = b->d_stair;
  b->st.base = b->d_stairBase;
  b->st.bad = b->d_stairBad;
  b->st.kmax = std::max(b->kmax, 0);
  b->st.ldsM = -1;
  {  // stage the table of the longest length in LDS when it fits (all reads share it in the usual case)
    const int km = std::max(b->kmax, 0), m0 = b->maxM;
    const uint64_t cnt = (uint64_t)(km + 2) * (km + 1) * (uint64_t)(m0 + km + 1);
    if (m0 >= 1 && m0 <= kMaxReadLen && base[(size_t)m0] < 0xFFFFFFFEu && cnt <= (uint64_t)kStairLdsWords) {
      b->st.ldsM = m0;
      b->st.ldsBase = base[(size_t)m0];
      b->st.ldsCount = (uint32_t)cnt;
    }
  }
  // fixed output slot per read: the chains besthit / a small -L report; more go to the pool
  const int chains = cfg->report_type == 0 ? 1 : cfg->report_type == 2 ? std::max(1, std::min(cfg->top_l, 4)) : 2;
  b->hitCap = (uint32_t)(chains * std::max(1, cfg->num_split + 1));
  b->cigCap = (uint32_t)(64 * chains);
  b->poolHits = std::max<uint64_t>(1 << 16, (uint64_t)n * b->hitCap / 16);
  b->poolCig = std::max<uint64_t>(1 << 20, (uint64_t)n * b->cigCap / 16);
  if (const char *e = getenv("GWA_OUT_POOL")) {  // initial pool size in hits (tests: force growth)
    b->poolHits = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    b->poolCig = 64 * b->poolHits;
  }
  if ((uint64_t)n * b->cigCap + b->poolCig >= 0xFFFFFFFFull)
    throw std::runtime_error("read batch too large for 32-bit output offsets: use fewer reads per batch");
  b->d_sres = bAlloc<ScanRes>(n);
  b->d_oh = bAlloc<OutHeader>(n);
  b->d_hits = bAlloc<OutHit>((size_t)n * b->hitCap + b->poolHits);
  b->d_cig = bAlloc<uint16_t>((size_t)n * b->cigCap + b->poolCig);
  b->d_list[0] = bAlloc<uint32_t>(n);
  b->d_list[1] = bAlloc<uint32_t>(n);
  b->d_count = bAlloc<uint32_t>(16);
  if (cfg->strategy == 1) {
    std::vector<uint32_t> all(n);
    for (uint32_t i = 0; i < n; ++i) all[i] = i;
    b->d_all = bUpload(all, s);
  }
  HIPCHK(hipStreamSynchronize(s));
}

extern "C" {

int gwa_batch_create(gwa_index_t *ix, const gwa_config_t *cfg, const gwa_reads_t *reads, gwa_batch_t **out) {
  auto *b = new gwa_batch();
  try {
    const uint32_t n = reads->n;
    if (batchHead(ix, cfg, n, b)) {
      *out = b;
      return 0;
    }
    b->hasQual = reads->qual != nullptr;
    hipStream_t s = b->stream;
    // the read text goes to HBM as it is (offsets rebased to the blob starts)
    auto blob = [&](const char *base, const uint64_t *off, char **dText, uint64_t **dOff) {
      std::vector<uint64_t> o(off, off + n + 1);
      const uint64_t o0 = o[0];
      for (auto &x : o) x -= o0;
      *dText = bAlloc<char>(o[n] + 32);  // (+32: the device reads the text in aligned 16-B chunks)
      if (o[n]) HIPCHK(hipMemcpyAsync(*dText, base + o0, o[n], hipMemcpyHostToDevice, s));
      *dOff = bUpload(o, s);
      HIPCHK(hipStreamSynchronize(s));  // (o is a local vector)
      return o[n];
    };
    uint64_t *off = nullptr;
    const uint64_t seqBytes = blob(reads->seq, reads->seq_off, &b->d_seqText, &off);
    b->d_fieldOwn[0] = off;
    b->d_seqB = off;
    b->d_seqE = off + 1;
    blob(reads->name, reads->name_off, &b->d_nameText, &off);
    b->d_fieldOwn[1] = off;
    b->d_nameB = off;
    b->d_nameE = off + 1;
    if (b->hasQual) {
      blob(reads->qual, reads->qual_off, &b->d_qualText, &off);
      b->d_fieldOwn[2] = off;
      b->d_qualB = off;
      b->d_qualE = off + 1;
      if (reads->qual_null) {  // reads without a quality among reads with one
        b->d_qualNull = bAlloc<uint8_t>(n);
        if (n) HIPCHK(hipMemcpyAsync(b->d_qualNull, reads->qual_null, n, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
      }
    }
    batchTail(b, seqBytes);
    *out = b;
    return 0;
  } catch (std::exception &e) {
    freeBatchDev(b);
    delete b;
    return fail(e.what());
  }
}

}  // extern "C"

namespace gwa {
// Pipeline use (pipeline.cpp): a batch from FASTQ text holding n complete records, record r's header
// line at start[r] (reads_io.cpp frameRecords).  The text goes to HBM as it is and the record fields
// are located there (batch_io.hip fastqFieldsKernel); names and qualities are read by the SAM writer
// in place.  A malformed record fails with the host parser's message.
int batchCreateFastq(gwa_index_t *ix, const gwa_config_t *cfg, const char *text, uint64_t len, const uint64_t *start,
                     uint32_t n, gwa_batch_t **out) {
  auto *b = new gwa_batch();
  try {
    if (batchHead(ix, cfg, n, b)) {
      *out = b;
      return 0;
    }
    b->hasQual = true;
    hipStream_t s = b->stream;
    char *dText = bAlloc<char>(len + 32);  // (+32: the device reads the text in aligned 16-B chunks)
    b->d_seqText = dText;
    HIPCHK(hipMemcpyAsync(dText, text, len, hipMemcpyHostToDevice, s));
    uint64_t *dStart = bAlloc<uint64_t>(n);
    HIPCHK(hipMemcpyAsync(dStart, start, (size_t)n * 8, hipMemcpyHostToDevice, s));
    uint64_t *f = bAlloc<uint64_t>(6 * (size_t)n);
    b->d_fieldOwn[0] = f;
    uint32_t *dErr = bAlloc<uint32_t>(1);
    uint32_t err = 0;
    HIPCHK(hipMemsetAsync(dErr, 0xFF, 4, s));
    launchFastqFields(dText, len, dStart, n, f, dErr, s);
    HIPCHK(hipMemcpyAsync(&err, dErr, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    batchFree(dStart, nullptr);  // (the stream was synchronised above)
    batchFree(dErr, nullptr);
    if (err != 0xFFFFFFFFu) {  // the host parser words the error
      gwa_read_buf_t pb{};
      uint64_t used = 0;
      if (gwa_reads_parse(text, len, 1, 1, &pb, &used) != 0) throw std::runtime_error(gwa_last_error());
      gwa_reads_free(&pb);
      throw std::runtime_error("malformed FASTQ record " + std::to_string(err));
    }
    b->d_nameText = dText;
    b->d_qualText = dText;
    b->d_nameB = f;
    b->d_nameE = f + n;
    b->d_seqB = f + 2 * (size_t)n;
    b->d_seqE = f + 3 * (size_t)n;
    b->d_qualB = f + 4 * (size_t)n;
    b->d_qualE = f + 5 * (size_t)n;
    uint64_t seqBytes = len;  // (an upper bound of the bases: the codes buffer is sized from it)
    batchTail(b, seqBytes);
    *out = b;
    return 0;
  } catch (std::exception &e) {
    freeBatchDev(b);
    delete b;
    return fail(e.what());
  }
}
}  // namespace gwa

extern "C" {

// capacity tiers: (arena, heap, hits, list, cigar, candidates) and the lane budget of each tier
struct Tier {
  int arena, heap, hits, list, cigar, cand;
  uint32_t maxLanes;
};
static const int kNumTiers = 4;
static const Tier kTiers[kNumTiers] = {
    {256, kLdsHeap, 32, 32, 512, 0, 256u * 1024u},  // heap in LDS
    // every resident lane of the chip (256 CUs x 8 waves x 64) on the next tier: the reads that
    // outgrow the LDS heap are many at k >= 4 (C4: ~57 % of 150 bp reads at k 5)
    {1024, 1024, 64, 64, 1024, 0, 128u * 1024u},
    {4096, 4096, 256, 256, 4096, 0, 65536u},  // 65536 lanes: C4 -m bsf tier 2 737 -> 494 ms (32768 / 131072: 737 / 601)
    {65536, 65536, 4096, 4096, 65536, 0, 1024u},
};
// -m sf: no quick-scan exit, every read starts with up to 2 (k + 2) seeds; heap in the slice
// (candidate sets of >= 64 slots are hash tables at most half full, SfLane::candInsert)
static const Tier kSfTiers[kNumTiers] = {
    {512, 512, 32, 32, 512, 32, 128u * 1024u},
    {2048, 2048, 64, 64, 2048, 512, 128u * 1024u},
    {8192, 8192, 256, 256, 4096, 2048, 16384u},
    {65536, 65536, 4096, 4096, 65536, 16384, 1024u},
};

// value t of a comma-separated tuning list in env variable `var`, or def
static uint32_t tierValue(const char *var, int t, uint32_t def) {
  const char *e = getenv(var);
  if (!e) return def;
  for (int i = 0; i < t && e; ++i) {
    e = strchr(e, ',');
    if (e) ++e;
  }
  const long v = e ? atol(e) : 0;
  return v > 0 ? (uint32_t)v : def;
}

// Search scratch one batch's tiers may hold: half of what is free on the device plus the buffer the
// batch already holds, at most 64 GiB (the index replica and the other batches keep the rest).
// Idle blocks of the device cache count as free (Scratch::ensure gives them back when it needs
// them).  Called under g_allocMu of the device, with the allocations it sizes.
static uint64_t scratchBudget(size_t held) {
  size_t freeB = 0, totalB = 0;
  if (hipMemGetInfo(&freeB, &totalB) != hipSuccess) return 16ull << 30;
  uint64_t cap = 64ull << 30;
  if (const char *e = getenv("GWA_SCRATCH_BUDGET_MB"))  // tests: concurrent batches under a small budget
    if (atoll(e) > 0) cap = std::min<uint64_t>(cap, (uint64_t)atoll(e) << 20);
  return std::min<uint64_t>(cap, ((uint64_t)freeB + held + devCacheIdle()) / 2);
}

// the batch's output slots + pool (gwa_layout.h OutSlots); pool counters at d_count[12..14]
static OutSlots outSlots(const gwa_batch *b) {
  OutSlots o;
  o.hits = b->d_hits;
  o.cig = b->d_cig;
  o.hitCap = b->hitCap;
  o.cigCap = b->cigCap;
  o.poolUsed = b->d_count + 12;
  o.poolHit0 = (uint64_t)b->n * b->hitCap;
  o.poolHitEnd = o.poolHit0 + b->poolHits;
  o.poolCig0 = (uint64_t)b->n * b->cigCap;
  o.poolCigEnd = o.poolCig0 + b->poolCig;
  return o;
}

// Grow the output pool to hold at least twice what has been reserved so far.  Offsets are absolute
// indices into the hit / CIGAR arrays, so what the kernels already wrote is copied as it lies.
static void growPool(gwa_batch *b, uint64_t usedH, uint64_t usedC, hipStream_t s) {
  const uint64_t nh = std::max<uint64_t>(2 * b->poolHits, 2 * usedH), nc = std::max<uint64_t>(2 * b->poolCig, 2 * usedC);
  const uint64_t fh = (uint64_t)b->n * b->hitCap, fc = (uint64_t)b->n * b->cigCap;
  if (fc + nc >= 0xFFFFFFFFull || fh + nh >= 0xFFFFFFFFull)
    throw std::runtime_error("reported hits exceed the 32-bit output offsets: use fewer reads per batch");
  OutHit *h = bAlloc<OutHit>(fh + nh);
  uint16_t *c = bAlloc<uint16_t>(fc + nc);
  HIPCHK(hipMemcpyAsync(h, b->d_hits, (fh + b->poolHits) * sizeof(OutHit), hipMemcpyDeviceToDevice, s));
  HIPCHK(hipMemcpyAsync(c, b->d_cig, (fc + b->poolCig) * sizeof(uint16_t), hipMemcpyDeviceToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  batchFree(b->d_hits, nullptr);  // (the stream was synchronised above)
  batchFree(b->d_cig, nullptr);
  b->d_hits = h;
  b->d_cig = c;
  b->poolHits = nh;
  b->poolCig = nc;
}

namespace {
struct Events {  // destroyed on every path out of gwa_batch_run
  hipEvent_t e[3] = {nullptr, nullptr, nullptr};
  Events() {
    for (auto &x : e) HIPCHK(hipEventCreate(&x));
  }
  ~Events() {
    for (auto &x : e)
      if (x) (void)hipEventDestroy(x);
  }
};
}  // namespace

static SamText samText(const gwa_batch *b);

// 2-bit query words per strand the kernels keep for reads of up to m bases (QW = 4, 8 or 16)
static int qwFor(int m) { return m <= 128 ? 4 : m <= 256 ? 8 : 16; }

int gwa_batch_run(gwa_batch_t *b) {
  try {
    gwa_index *ix = b->ix;
    HIPCHK(hipSetDevice(ix->device));
    hipStream_t s = b->stream;
    memset(&b->stats, 0, sizeof(b->stats));
    if (b->headerOnly) {
      b->ran = true;
      return 0;
    }
    b->ran = b->statsDone = false;
    b->poolUsedH = b->poolUsedC = 0;
    b->deep.clear();
    ReadsView rv{b->d_codes, b->d_off, b->d_len, b->n};
    Scratch scr(ix, s);  // this run's search scratch (from the index's pool, back to it at the end)
    Events ev;
    hipEvent_t e0 = ev.e[0], e1 = ev.e[1], e2 = ev.e[2];
    // encode the read text in HBM (ACGTSequence(String), A/ACGTSequence.java:86-97): lengths and
    // code offsets, then the code rows
    HIPCHK(hipEventRecord(e2, s));
    launchEncode(b->d_seqText, b->d_seqB, b->d_seqE, b->n, b->d_len, b->d_row, b->d_off, b->d_seen, b->d_codes,
                 b->d_encTmp, b->encTmpBytes, 0, s);
    launchEncode(b->d_seqText, b->d_seqB, b->d_seqE, b->n, b->d_len, b->d_row, b->d_off, b->d_seen, b->d_codes,
                 b->d_encTmp, b->encTmpBytes, 1, s);
    HIPCHK(hipMemsetAsync(b->d_count, 0, 16 * sizeof(uint32_t), s));
    HIPCHK(hipEventRecord(e0, s));
    const bool sf = b->cfg.strategy == 1;
    if (!sf)
      launchQuickscan(qwFor(b->maxM), ix->view, b->scfg, rv, b->d_sres, b->d_oh, outSlots(b), b->d_list[0],
                      b->d_count, s);
    // -m sf, k >= 4 (R >= 8): the quick scan of every read for the search-list key only (see sortLists
    // below).  C4 (1M reads): search 17.8 -> 13.7 ms for a 1.6 ms scan; at k = 2 (C2 -m sf, 2M reads)
    // 9.8 -> 9.4 ms for a 1.8 ms scan, so k <= 3 batches keep input order.
    const bool sfSort = sf && b->R >= 8 && !(getenv("GWA_SEARCH_SORT") && atoi(getenv("GWA_SEARCH_SORT")) == 0);
    if (sfSort) launchKeyscan(qwFor(b->maxM), ix->view, b->scfg, rv, b->d_sres, s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e1, s));
    uint32_t nSearch = b->n;
    if (!sf) HIPCHK(hipMemcpyAsync(&nSearch, b->d_count, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    float qms = 0, ems = 0;
    HIPCHK(hipEventElapsedTime(&qms, e0, e1));
    HIPCHK(hipEventElapsedTime(&ems, e2, e0));
    b->stats.quickscan_ms = qms;
    b->stats.encode_ms = ems;
    double searchMs = 0;
    int cur = 0;
    uint32_t n = nSearch;
    // The first tier takes the searched reads in quick-scan key order (launchSortSearchList: reads
    // with the same seeds share wavefronts), and the second tier takes the first tier's overflows in
    // input order (in the first tier's completion order, i.e. key order, the heavy reads of one key
    // would crowd the same wavefronts: C4 tier 1 158 ms against 112 ms).  -m sf searches every read in
    // input order.  GWA_SEARCH_SORT=0: no sorting (A/B runs).
    // -m sf (round 6): every read is searched, and a wavefront takes 64 reads at a time and runs each
    // to its end (sf_search_kernel), so the first tier's list of all reads is sorted by the same key,
    // from a quick scan that only computes it (launchKeyscan).
    const bool sortLists = !(getenv("GWA_SEARCH_SORT") && atoi(getenv("GWA_SEARCH_SORT")) == 0);
    bool sfSorted = false;  // (-m sf: the first tier reads the sorted list, not d_all)
    const int m = std::max(b->maxM, 1);
    int t = 0, regrow = 0, launches = 0;
    // Reads that overflow the last tier rerun on it with the exceeded capacities doubled (OV_* bits
    // the kernel ORs into d_count[15]), as often as needed: no read the reference would finish is
    // refused for capacity.  The hard limits are the state index of a queue entry (2^24 states,
    // BsfLane KS) and the scratch budget; past them the batch fails with the read count and the
    // limit.  (BSF arenas are bounded by the search itself: <= 20m + 5 FM steps each create <= 1
    // state and, with num_split = 1, <= 2 split states per state expanded: ~31k states for m = 512.
    // The SF search has no such bound, S/SuffixFilter.java:257-290.)
    int gArena = 0, gHits = 0, gList = 0, gCigar = 0, gCand = 0;
    int arenaMaxLog = 24;
    if (const char *e = getenv("GWA_MAX_STATES_LOG2"))  // diagnostics (tools/diag_sf.py): a lower state limit
      arenaMaxLog = std::max(16, std::min(24, atoi(e)));
    const bool hybrid = !sf && b->R >= 8;
    // resume records (-m bsf): a tier writes those of the reads it suspends into resOut (entry i of its
    // overflow list), the next tier reads them from resIn (bsf_search_kernel, BsfLane::suspendTo)
    struct ResBuf {
      uint8_t *p = nullptr;
      size_t bytes = 0;
      uint64_t stride = 0;
      uint32_t cap = 0;
    } resIn, resOut;
    struct ResFree {  // (the batch's stream is drained before the buffers go back)
      ResBuf *a, *b;
      hipStream_t s;
      ~ResFree() {
        batchFree(a->p, s);
        batchFree(b->p, nullptr);
      }
    } resFree{&resIn, &resOut, s};
    // the capacities of tier tb (the last one grown by the g* shifts)
    auto capsFor = [&](int tb) {
      const Tier &T = sf ? kSfTiers[tb] : kTiers[tb];
      Caps caps;
      caps.sparse = 0;
      caps.arena = T.arena; caps.heap = T.heap; caps.hits = T.hits; caps.list = T.list; caps.cigar = T.cigar;
      // GWA_TIER_ARENA="a0,a1,a2,a3": arena / heap states of tiers >= 1, and of tier 0 for the
      // hybrid-heap (k >= 4) kernels, whose heap is not bounded by the LDS array (tuning runs)
      if ((tb > 0 || b->R >= 8) && !sf) {
        // k >= 4: hit lists of 128 / 256 entries in tiers 0 / 1 (C4: 32 / 64 sent 241k / 108k of 833k
        // reads to a rerun, 128 / 256 151k / 5k; search 457 -> 409 ms per 1M reads)
        const bool wide = b->R >= 8 && tb < 2;
        const uint32_t dh = wide ? (tb == 0 ? 128u : 256u) : (uint32_t)T.hits;
        const uint32_t dc = wide ? (tb == 0 ? 2048u : 4096u) : (uint32_t)T.cigar;
        const int a = (int)std::min<uint32_t>(tierValue("GWA_TIER_ARENA", tb, (uint32_t)T.arena), 1u << 24);
        caps.arena = caps.heap = a;
        caps.hits = caps.list = (int)tierValue("GWA_TIER_HITS", tb, dh);  // hit list / report list
        caps.cigar = (int)tierValue("GWA_TIER_CIGAR", tb, dc);
      }
      caps.cand = T.cand;
      caps.sf = sf ? 1 : 0;
      caps.spec = 0;
      if (tb == kNumTiers - 1) {  // the grown last tier
        caps.arena <<= gArena;
        caps.heap <<= gArena;
        caps.hits <<= gHits;
        caps.list <<= gList;
        caps.cigar <<= gCigar;
        caps.cand <<= gCand;
        // -m sf: the result table of the cooperative kernel (run when the tier is sparse, 64);
        // GWA_SF_COOP=0 runs the per-lane kernel there instead (A/B and diagnostics)
        if (sf && !(getenv("GWA_SF_COOP") && atoi(getenv("GWA_SF_COOP")) == 0)) caps.spec = caps.cand;
      }
      // -m bsf, k >= 4 (R >= 8): the verification memo (bsf_core.h verify), twice the hit list's
      // entries, a power of two; k <= 3 reads do not repeat verifications (C2: 1431 of 1431 unique)
      // and skip the lookup.  GWA_VERIFY_MEMO=0 turns it off (A/B runs).
      if (!sf) {
        caps.cand = 0;
        const char *vm = getenv("GWA_VERIFY_MEMO");
        if (b->R >= 8 && !(vm && atoi(vm) == 0)) {
          int c = 64;
          while (c < 2 * caps.hits && c < (1 << 22)) c <<= 1;
          caps.cand = c;
        }
      }
      // k >= 4 (R >= 8): a hybrid heap, its top slots in LDS and the rest in the slice, holding as
      // many entries as the arena has states (k >= 4 heaps outgrow the 8-slot LDS heap of tier 0)
      if (hybrid) caps.heap = caps.arena;
      const int bMax = std::max(1, (m + 63) / 64);
      const int nref = m + 2 * b->kmax + 2;
      caps.dpWords = 2 * bMax * (nref + 1);
      caps.path = m + nref + 8;
      caps.dpSlice = tb == 0 ? 1 : 0;  // the first tier's DP keeps the diagonal slice (bsf_core.h)
      return caps;
    };
    // the search-list sort (tier 0: by quick-scan key; the second tier: input order)
    auto sortList = [&](bool byKey, const uint32_t *in) {
      const size_t tb = sortSearchListTmpBytes(n);
      uint32_t *keys = bAlloc<uint32_t>(2 * (size_t)n);
      void *tmp = batchMalloc(std::max<size_t>(tb, 64));
      HIPCHK(hipEventRecord(e1, s));
      launchSortSearchList(in, b->d_list[cur ^ 1], keys, keys + n, n, b->d_sres, byKey, tmp, tb, s);
      HIPCHK(hipEventRecord(e2, s));
      HIPCHK(hipStreamSynchronize(s));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, e1, e2));
      searchMs += ms;
      batchFree(keys, nullptr);
      batchFree(tmp, nullptr);
      cur ^= 1;
    };
    while (n > 0) {
      if (++launches > 96) throw std::runtime_error("search capacity growth did not converge");
      // (the second tier's input has no resume records -- the first tier does not suspend -- so its
      // list may be reordered; deeper tiers find their records by list position)
      // (key order for the second tier too: C4 tier 1 184 ms against 117 ms, 178-193 ms with
      // wavefront-wide refills as well; hg19r's 21.9 against 23.5 ms)
      if (sfSort && n > 1 && t == 0 && regrow == 0) {
        sortList(true, b->d_all);
        sfSorted = true;
      } else if (sortLists && n > 1 && ((t == 0 && !sf) || (t == 1 && resIn.cap == 0))) {
        sortList(t == 0, b->d_list[cur]);
      }
      // the budget and this tier's scratch / resume allocations as one step per device (released
      // before the launch: the memory is allocated by then, so the next batch's budget sees it)
      std::unique_lock<std::mutex> allocLock(g_allocMu[ix->device & 63]);
      const uint64_t budget = scratchBudget(scr.bytes);
      // Few reads left after the first tier: straight to the largest tier whose capacities give every
      // one of them a slice within the scratch budget.  A rerun restarts a search from its seeds, and
      // the reads still overflowing here are the heaviest (C4 -m bsf: 5k reads in tier 2, of which 2
      // then reran on tier 3 for 65 ms).  GWA_TIER_JUMP=0 turns it off.
      if (t >= 1 && t < kNumTiers - 1 && !(getenv("GWA_TIER_JUMP") && atoi(getenv("GWA_TIER_JUMP")) == 0)) {
        for (int u = kNumTiers - 1; u > t; --u) {
          const Caps lc = capsFor(u);
          if ((uint64_t)n * (laneBytesFor(b->R, lc) + ilvBytesFor(lc)) <= budget) {
            t = u;
            break;
          }
        }
      }
      const int tb = std::min(t, kNumTiers - 1);  // t > kNumTiers - 1: the last tier, grown
      const Tier &T = sf ? kSfTiers[tb] : kTiers[tb];
      Caps caps = capsFor(tb);
      const uint64_t stride = laneBytesFor(b->R, caps), ilv = ilvBytesFor(caps);
      const uint64_t maxSparse = tierValue("GWA_SPARSE_LANES", 0, 262144u);
      // scratch of `ln` lanes of which every sp-th takes reads: slices for the active ones, the
      // interleaved DP block for all (bsf_search_kernel / sf_search_kernel addressing)
      auto mem = [&](uint64_t st, uint64_t ln, uint64_t sp) { return st * (ln / sp) + ilv * ln; };
      uint32_t lanes = std::min<uint32_t>(n, tierValue("GWA_TIER_LANES", tb, T.maxLanes));
      lanes = (lanes + 255) / 256 * 256;
      // deep tiers: as many lanes as the scratch budget allows (at least one workgroup)
      lanes = (uint32_t)std::min<uint64_t>(lanes, std::max<uint64_t>(256, budget / (stride + ilv) / 256 * 256));
      if (tb > 0 && (!sf || tb == kNumTiers - 1)) {
        // a deep tier with few reads: 64 / s reads per wavefront (every s-th lane), the largest s
        // whose n x s lanes stay within GWA_SPARSE_LANES (default 262144) and the scratch budget
        for (uint32_t sp = 64; sp >= 2; sp /= 2) {
          const uint64_t sl = ((uint64_t)n * sp + 255) / 256 * 256;
          if (sl <= maxSparse && mem(stride, sl, sp) <= budget) {
            lanes = (uint32_t)sl;
            caps.sparse = (int32_t)sp;
            break;
          }
        }
      }
      uint64_t spUsed = caps.sparse > 1 ? (uint64_t)caps.sparse : 1;
      if (mem(stride, lanes, spUsed) > budget) {
        // fewer active lanes than reads: the persistent lanes take the reads from the shared counter,
        // as many at once as the budget holds (deep tiers: one read per wavefront)
        if (tb > 0 && spUsed == 1) {
          caps.sparse = 64;
          spUsed = 64;
        }
        lanes = (uint32_t)std::min<uint64_t>(lanes, budget / (stride + ilv * spUsed) * spUsed / 256 * 256);
        if (lanes < 256)
          throw std::runtime_error(std::to_string(n) + " reads need more than the " + std::to_string(budget >> 20) +
                                   " MiB search scratch budget (" + std::to_string(caps.arena) +
                                   " states per lane): the device memory is exhausted");
      }
      // a very sparse tier whose lanes fit one round of one workgroup per CU (256 CUs x 4 waves):
      // its queue tops go to LDS (bsf_search_kernel LH 2; the 64 KiB array leaves one workgroup per CU)
      const bool deepLds = !sf && tb > 0 && caps.sparse >= 8 && lanes <= 65536u;
      scr.ensure((size_t)mem(stride, lanes, spUsed));
      uint32_t *ovfCount = b->d_count + 1 + tb;
      uint32_t *ovfBits = b->d_count + 15;
      HIPCHK(hipMemsetAsync(ovfCount, 0, 4, s));
      HIPCHK(hipMemsetAsync(b->d_count + 8 + tb, 0, 4, s));
      HIPCHK(hipMemsetAsync(ovfBits, 0, 4, s));
      ResumeBufs rb{};
      if (!sf) {
        const uint64_t rstride = resumeBytesFor(b->R, caps);
        // (the first tier's kernel does not suspend: its overflows restart on the next tier)
        const uint64_t cap = tb == 0 ? 0 : std::min<uint64_t>(n, std::min<uint64_t>(8ull << 30, budget / 4) / rstride);
        if (resOut.bytes < cap * rstride) {
          batchFree(resOut.p, s);
          resOut.p = nullptr;
          resOut.bytes = 0;
          resOut.p = bAlloc<uint8_t>(cap * rstride);
          resOut.bytes = cap * rstride;
        }
        resOut.stride = rstride;
        resOut.cap = (uint32_t)cap;
        rb.out = cap ? resOut.p : nullptr;
        rb.outStride = rstride;
        rb.outCap = (uint32_t)cap;
        rb.in = resIn.cap ? resIn.p : nullptr;
        rb.inStride = resIn.stride;
        rb.inCap = resIn.cap;
      }
      allocLock.unlock();
      HIPCHK(hipEventRecord(e1, s));
      const OutSlots os = outSlots(b);
      // The first tier's wavefronts take new reads for their idle lanes only once most of their lanes
      // are idle (SearchConfig::refillMin), as a run of consecutive reads of the key-sorted list: the
      // lanes of a wavefront then hold reads of one key and step together, and they run their reports
      // later, when more of them are parked (waitQ16).  First-tier search ms (hg19 / hg19r / C4 per 1M):
      // lane by lane, waitQ16 14 (8): 65.0 / 110.9 / 100.3; refill 48 (C4 32): 46.2 / 80.9 / 90.5;
      // with waitQ16 16: 41.7 / 89.8 / 99.7; 15 and refill 56 (kept): 44.0 / 84.6; C4 waitQ16 12:
      // 84.9.  Deeper tiers keep lane-by-lane refills and their thresholds (C4 tier 1: 114.7 ms; 120.2
      // at refill 32; 172 at waitQ16 16).  SAM identical throughout.  GWA_REFILL sets the first tier's
      // threshold (1: lane by lane, A/B runs); GWA_WAITQ16 still sets every tier's.
      SearchConfig tcfg = b->scfg;
      if (tb == 0 && !sf) {
        tcfg.refillMin = getenv("GWA_REFILL") ? atoi(getenv("GWA_REFILL")) : b->R >= 8 ? 32 : 56;
        if (!getenv("GWA_WAITQ16")) tcfg.waitQ16 = b->R >= 8 ? 12 : 15;
      }

#ifdef GWA_PROF
      uint64_t *d_prof = nullptr;
      HIPCHK(hipMalloc(&d_prof, (size_t)lanes * PR_N * 8));
      HIPCHK(hipMemsetAsync(d_prof, 0, (size_t)lanes * PR_N * 8, s));
      if (sf)
        launchSfSearch(b->R, qwFor(b->maxM), b->sfWrap, lanes, ix->view, b->scfg, b->st, rv,
                       (t == 0 && regrow == 0 && !sfSorted) ? b->d_all : b->d_list[cur], n, scr.p, stride, caps, b->d_oh, os,
                       ix->d_chrRank, b->d_count + 8 + tb, b->d_list[cur ^ 1], ovfCount, ovfBits, s, (uint32_t *)d_prof);
      else
        launchSearch(b->R, qwFor(b->maxM), deepLds ? 2 : (tb == 0 || hybrid) ? 1 : 0, lanes, ix->view, tcfg, b->st, rv, b->d_sres,
                     b->d_list[cur], n, scr.p, stride, caps, b->d_oh, os, ix->d_chrRank, b->d_count + 8 + tb,
                     b->d_list[cur ^ 1], ovfCount, ovfBits, rb, s, (uint32_t *)d_prof, -1);
      {
        std::vector<uint64_t> pv((size_t)lanes * PR_N);
        HIPCHK(hipMemcpyAsync(pv.data(), d_prof, pv.size() * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipFree(d_prof));
        double sum[PR_N] = {};
        for (size_t i = 0; i < pv.size(); ++i) sum[i % PR_N] += (double)pv[i];
        static const char *nm[PR_N] = {"poll", "report", "runahead", "exp1", "add1", "expN", "split", "newstate",
                                       "verify", "nfa", "fm", "seed", "nVerifyWave", "nVerifyLane", "nStepWave",
                                       "nStepLane", "dpFwd", "dpTrace", "sumWait", "nBuildWave", "nBuildLane",
                                       "wArenaGB", "eArena", "wWordGB", "eWord", "wDpGB", "eDp", "eDpWave",
                                       "wHitGB", "eHit", "wOutGB", "eOut", "-", "wave"};
        // -m sf (SfLane::sfStep): poll = queuePoll + state load, fm = rank2, nfa = the children's
        // automaton steps, add1 = newState + offer, verify = addCandidate (dpFwd / dpTrace inside it),
        // split = the candidate-set probe, seed = sfStart; nStep = polls, nVerify = DP verifications
        fprintf(stderr, "[gwa-prof] %s", sf ? "-m sf " : "");
        fprintf(stderr, "tier %d reads %u lanes %u (Gcycles summed over waves; counts in M; bytes in GB):", t, n, lanes);
        for (int q = 0; q < PR_N; ++q) {
          if (nm[q][0] == '-') continue;
          const bool count = (q >= PR_NVW && q <= PR_NSL) || q == PR_NWAIT || q == PR_NBW || q == PR_NBL ||
                             (q >= PR_WA && q <= PR_EO && nm[q][0] == 'e');
          fprintf(stderr, " %s=%.3f", nm[q], sum[q] / (count ? 1e6 : 1e9));
        }
        fprintf(stderr, "\n");
      }
#else
      if (sf)
        launchSfSearch(b->R, qwFor(b->maxM), b->sfWrap, lanes, ix->view, b->scfg, b->st, rv,
                       (t == 0 && regrow == 0 && !sfSorted) ? b->d_all : b->d_list[cur], n, scr.p, stride, caps, b->d_oh, os,
                       ix->d_chrRank, b->d_count + 8 + tb, b->d_list[cur ^ 1], ovfCount, ovfBits, s);
      else
        launchSearch(b->R, qwFor(b->maxM), deepLds ? 2 : (tb == 0 || hybrid) ? 1 : 0, lanes, ix->view, tcfg, b->st, rv, b->d_sres, b->d_list[cur], n,
                     scr.p, stride, caps, b->d_oh, os, ix->d_chrRank, b->d_count + 8 + tb, b->d_list[cur ^ 1],
                     ovfCount, ovfBits, rb, s);
#endif
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(e2, s));
      uint32_t ctr[16];
      HIPCHK(hipMemcpyAsync(ctr, b->d_count, sizeof(ctr), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, e1, e2));
      searchMs += ms;
      b->stats.tier_reads[tb] += n;
      b->stats.tier_ms[tb] += ms;
      if (getenv("GWA_VERBOSE"))
        fprintf(stderr, "[gwa] tier %d: %u reads on %u lanes (sparse %d; arena %d hits %d list %d cigar %d cand %d): %.1f ms, %u overflow (bits 0x%x)\n",
                t, n, lanes, caps.sparse, caps.arena, caps.hits, caps.list, caps.cigar, caps.cand, ms, ctr[1 + tb], ctr[15]);
      n = ctr[1 + tb];
      const uint32_t bits = ctr[15];
      cur ^= 1;
      if (!sf) std::swap(resIn, resOut);  // this tier's records are the next one's input
      if (n > 0) {  // the reads rerun on the next tier (instrumentation, gwa_batch_read_counters)
        std::vector<uint32_t> ids(n);
        HIPCHK(hipMemcpyAsync(ids.data(), b->d_list[cur], n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (uint32_t r : ids) b->deep.push_back({r, t + 1});
      }
      b->poolUsedH = std::min<uint64_t>(ctr[12], b->poolHits);
      b->poolUsedC = std::min<uint64_t>(ctr[13], b->poolCig);
      const bool refused = ctr[14] > 0;
      if (refused) {  // reads whose reported hits did not fit the pool: grow it, rerun them
        if (++regrow > 8) throw std::runtime_error("output pool growth did not converge");
        growPool(b, ctr[12], ctr[13], s);
        HIPCHK(hipMemsetAsync(b->d_count + 14, 0, 4, s));
      }
      if (n > 0 && t >= kNumTiers - 1) {  // overflow of the last tier: grow what was exceeded
        if (bits & (OV_CHAIN | OV_DP))
          throw std::runtime_error(std::to_string(n) + (bits & OV_CHAIN ? " reads with a split chain of more than 8 pieces"
                                                                        : " reads with a DP window beyond the read-length limit"));
        if (bits & (OV_ARENA | OV_HEAP)) {
          int lg = 0;
          while ((1 << lg) < caps.arena) ++lg;
          if (lg >= arenaMaxLog)
            throw std::runtime_error(std::to_string(n) + " reads need more than 2^" + std::to_string(arenaMaxLog) +
                                     " search states (the queue-entry state index)");
          // straight to the largest arena the scratch budget gives these reads (one read per
          // wavefront when they are few), not one doubling per rerun: every rerun restarts the
          // searches, and the -m sf searches on repeats queue up to millions of states
          ++gArena;
          ++lg;
          const uint64_t conc = std::min<uint64_t>(n, 256);  // reads searching at once, at least
          const uint64_t ln = (conc * 64 + 255) / 256 * 256;
          for (; lg < arenaMaxLog; ++lg, ++gArena) {
            Caps c2 = caps;
            c2.arena = c2.heap = 1 << (lg + 1);
            if (mem(laneBytesFor(b->R, c2), ln, 64) > budget / 2) break;
          }
        }
        // (x4 per rerun: every rerun restarts the searches, and the reads still growing here are the
        // heaviest; -m sf reads on repeats verify millions of candidates)
        if (bits & OV_HITS) gHits += 2;
        if (bits & OV_LIST) gList += 2;
        if (bits & OV_CIGAR) gCigar += 2;
        // the candidate set straight to >= 2^20 slots (8 MiB per read; half may fill): the reads that
        // outgrow 16384 candidates on repeats verify hundreds of thousands
        if (bits & OV_CAND) gCand = std::max(gCand + 2, 6);
        if (!(bits & (OV_ARENA | OV_HEAP | OV_HITS | OV_LIST | OV_CIGAR | OV_CAND)) && !refused)
          throw std::runtime_error(std::to_string(n) + " reads exceeded the largest search tier (overflow bits " +
                                   std::to_string(bits) + ")");
      }
      ++t;
    }
    b->stats.search_ms = searchMs;
    double rescueMs = 0;
    if (b->pairs) {  // paired-end: mate rescue (orc_align_pairs rule 3), part of the alignment
      Caps rc{};
      rc.cigar = 512;
      rc.dpWords = 2 * 4 * (kRescueWindow + 1);  // QW = 8: up to 4 blocks of 64 rows, full history
      rc.path = 256 + kRescueWindow + 8;
      rc.dpSlice = 0;
      const uint64_t stride = laneBytesFor(4, rc);
      uint32_t lanes = std::min<uint32_t>(b->pairs, 65536u);
      lanes = (lanes + 63) / 64 * 64;
      scr.ensure((size_t)(stride + ilvBytesFor(rc)) * lanes);
      uint32_t *heavyCount = b->d_heavy + b->pairs;
      HIPCHK(hipEventRecord(e1, s));
      HIPCHK(hipMemsetAsync(heavyCount, 0, 8, s));
      launchPairRescue(lanes, ix->view, b->scfg, b->st, rv, samText(b), b->d_oh, b->d_hits, b->d_cig, b->pairs, b->minIns,
                       b->maxIns, scr.p, stride, rc, b->d_rescue,
                       getenv("GWA_PAIR_QUAD") ? atol(getenv("GWA_PAIR_QUAD")) : kPairQuad, b->d_heavy, heavyCount, s);
      HIPCHK(hipGetLastError());
      uint32_t hc[2] = {0, 0};
      HIPCHK(hipMemcpyAsync(hc, heavyCount, 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));  // (hc is read only after the copy has landed)
      const uint32_t nHeavy = hc[0];
      b->stats.rescue_window_skipped = hc[1];
      if (nHeavy > b->pairs) throw std::runtime_error("pair choice: heavy-pair count out of range");
      launchPairChoose(nHeavy, samText(b), b->d_oh, b->d_hits, b->d_cig, b->pairs, b->minIns, b->maxIns, b->d_heavy,
                       getenv("GWA_PAIR_SORT_CAP") ? atoi(getenv("GWA_PAIR_SORT_CAP")) : kPairSortCap, b->d_rescue, s);
      HIPCHK(hipGetLastError());
      b->stats.heavy_pairs = nHeavy;
      HIPCHK(hipEventRecord(e2, s));
      HIPCHK(hipEventSynchronize(e2));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, e1, e2));
      rescueMs = ms;
    }
    b->stats.rescue_ms = rescueMs;
    b->stats.kernel_ms = ems + qms + searchMs + rescueMs;
    // a grown last tier may have taken tens of GiB of scratch for a few reads: give it back rather
    // than hold it for the index's life (the next batch allocates what its tiers need)
    if (t > kNumTiers) {
      HIPCHK(hipStreamSynchronize(s));
      scr.release();
    }
    b->ran = true;
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

}  // extern "C"

// the batch statistics (gwa_batch_stats_t sums) as one device reduction over the output headers
static void ensureStats(gwa_batch *b) {
  if (b->statsDone || b->headerOnly || !b->ran) return;
  HIPCHK(hipSetDevice(b->ix->device));
  hipStream_t s = b->stream;
  if (!b->d_stats) b->d_stats = bAlloc<unsigned long long>(kStatFields);
  launchStats(b->d_oh, b->n, b->d_stats, s);
  unsigned long long v[kStatFields];
  HIPCHK(hipMemcpyAsync(v, b->d_stats, sizeof(v), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  gwa_batch_stats_t &st = b->stats;
  st.fm_searches = v[0];
  st.quick_steps = v[1];
  st.quick_blocks = v[2];
  st.blocks = v[2] + v[3];
  st.kmer_lookups = v[4];
  st.quick_sa_reads = v[6];
  st.sa_reads = v[5] + v[6];
  st.quick_short_steps = v[7];
  st.search_short_steps = v[8];
  st.states = v[9];
  st.num_sw = v[10];
  st.verify_bytes = v[11];
  st.quick_text_runs = v[14];
  st.n_mapped = (uint32_t)v[12];
  st.n_unmapped = (uint32_t)v[13];
  b->statsDone = true;
}

static SamText samText(const gwa_batch *b) {
  SamText t;
  t.name = b->d_nameText;
  t.nameB = b->d_nameB;
  t.nameE = b->d_nameE;
  t.qual = b->hasQual ? b->d_qualText : nullptr;
  t.qualB = b->d_qualB;
  t.qualE = b->d_qualE;
  t.qualNull = b->d_qualNull;
  t.codes = b->d_codes;
  t.codeOff = b->d_off;
  t.codeLen = b->d_len;
  t.ctg = b->ix->d_ctg;
  t.ctgOff = b->ix->d_ctgOff;
  t.chrKey = b->ix->d_chrRank;
  t.starKey = b->ix->starKey;
  t.emptyKey = b->ix->emptyKey;
  return t;
}

template <class T>
static void growDev(T **p, size_t *cap, size_t need, hipStream_t s) {
  if (*p && *cap >= need) return;
  batchFree(*p, s);
  *p = nullptr;
  *p = bAlloc<T>(need);
  *cap = need;
}

// SAM text of the reads idx[0..count) (or first .. first + count - 1) written on the device
// (batch_io.hip) into d_fmtText, line offsets in d_fmtOff; returns the text size in bytes
static uint64_t formatOnDevice(gwa_batch *b, const uint32_t *hostIdx, uint32_t first, uint32_t count) {
  if (!b->ran) throw std::runtime_error("gwa_batch_run has not completed");
  const uint32_t n = count;
  HIPCHK(hipSetDevice(b->ix->device));
  hipStream_t s = b->stream;
  if (!b->d_fmtLen || b->fmtCap < (size_t)n + 1) {
    void *ps[] = {b->d_fmtLen, b->d_fmtOff, b->d_fmtIdx, b->d_fmtTmp};
    for (void *p : ps) batchFree(p, s);
    b->d_fmtLen = b->d_fmtOff = nullptr;
    b->d_fmtIdx = nullptr;
    b->d_fmtTmp = nullptr;
    b->d_fmtLen = bAlloc<uint64_t>((size_t)n + 1);
    b->d_fmtOff = bAlloc<uint64_t>((size_t)n + 1);
    b->d_fmtIdx = bAlloc<uint32_t>((size_t)n + 1);
    b->fmtTmpBytes = samScanTempBytes(n);
    b->d_fmtTmp = bAlloc<uint8_t>(b->fmtTmpBytes);
    b->fmtCap = (size_t)n + 1;
  }
  if (!b->d_fmtErr) b->d_fmtErr = bAlloc<uint32_t>(1);
  const uint32_t *dIdx = nullptr;
  if (hostIdx) {
    HIPCHK(hipMemcpyAsync(b->d_fmtIdx, hostIdx, (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    dIdx = b->d_fmtIdx;
  }
  HIPCHK(hipMemsetAsync(b->d_fmtErr, 0xFF, sizeof(uint32_t), s));
  Events ev;
  HIPCHK(hipEventRecord(ev.e[0], s));
  const SamText t = samText(b);
  const PairSpec ps{b->pairs, b->minIns, b->maxIns, b->pairs ? b->d_rescue : nullptr};
  size_t tmpBytes = b->fmtTmpBytes;
  launchSamFormat(t, b->d_oh, b->d_hits, b->d_cig, dIdx, first, n, b->d_fmtLen, b->d_fmtOff, b->d_fmtTmp, &tmpBytes,
                  b->d_fmtErr, nullptr, 0, s, ps);
  launchSamFormat(t, b->d_oh, b->d_hits, b->d_cig, dIdx, first, n, b->d_fmtLen, b->d_fmtOff, b->d_fmtTmp, &tmpBytes,
                  b->d_fmtErr, nullptr, 1, s, ps);
  uint64_t total = 0;
  uint32_t err = 0;
  HIPCHK(hipMemcpyAsync(&total, b->d_fmtOff + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&err, b->d_fmtErr, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (err != 0xFFFFFFFFu) {  // a read the reference would abort on, or whose search failed
    uint32_t r = hostIdx ? hostIdx[err] : first + err;
    if (b->pairs) {  // the failing mate of pair r
      OutHeader h1;
      HIPCHK(hipMemcpy(&h1, b->d_oh + r, sizeof(h1), hipMemcpyDeviceToHost));
      if (h1.status == ST_MAPPED || h1.status == ST_UNMAPPED) r += b->pairs;
    }
    OutHeader h;
    uint64_t no[2];
    HIPCHK(hipMemcpy(&h, b->d_oh + r, sizeof(h), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&no[0], b->d_nameB + r, 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&no[1], b->d_nameE + r, 8, hipMemcpyDeviceToHost));
    std::string nm(no[1] - no[0], '\0');
    if (!nm.empty()) HIPCHK(hipMemcpy(&nm[0], b->d_nameText + no[0], nm.size(), hipMemcpyDeviceToHost));
    const int stt = h.status;
    throw std::runtime_error(std::string(stt == ST_TOO_LONG ? "read longer than the device path supports: "
                                         : stt == ST_OVERFLOW ? "output slot overflow at read "
                                         : stt == ST_ERROR ? "reference would abort (exception) at read "
                                                           : "reference would abort (exception in AlignmentRecord.convert) at read ") + nm);
  }
  growDev(&b->d_fmtText, &b->fmtTextCap, (size_t)total + 1, s);
  launchSamFormat(t, b->d_oh, b->d_hits, b->d_cig, dIdx, first, n, b->d_fmtLen, b->d_fmtOff, b->d_fmtTmp, &tmpBytes,
                  b->d_fmtErr, b->d_fmtText, 2, s, ps, total);
  HIPCHK(hipEventRecord(ev.e[1], s));
  HIPCHK(hipEventSynchronize(ev.e[1]));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, ev.e[0], ev.e[1]));
  b->stats.format_ms = ms;
  b->fmtBytes = total;
  b->fmtWhole = false;
  return total;
}

// formatOnDevice into library-owned host memory (gwa_results_t)
static void formatResults(gwa_batch *b, const uint32_t *hostIdx, uint32_t first, uint32_t count, gwa_results_t *out) {
  const uint32_t n = count;
  out->n_reads = n;
  out->sam = nullptr;
  out->line_off = nullptr;
  out->records = nullptr;
  out->n_records = 0;
  out->paired = b->pairs ? 1 : 0;
  if (b->headerOnly) {
    if (!b->ran) throw std::runtime_error("gwa_batch_run has not completed");
    out->sam = (char *)calloc(1, 1);
    out->sam_len = 0;
    out->line_off = (uint64_t *)calloc((size_t)n + 1, sizeof(uint64_t));
    return;
  }
  const uint64_t total = formatOnDevice(b, hostIdx, first, count);
  hipStream_t s = b->stream;
  out->sam = (char *)malloc(total + 1);
  out->line_off = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)n + 1));
  if (!out->sam || !out->line_off) {
    free(out->sam);
    free(out->line_off);
    out->sam = nullptr;
    out->line_off = nullptr;
    throw std::runtime_error("out of host memory for the SAM text");
  }
  if (total) HIPCHK(hipMemcpyAsync(out->sam, b->d_fmtText, total, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(out->line_off, b->d_fmtOff, sizeof(uint64_t) * ((size_t)n + 1), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  out->sam[total] = 0;
  out->sam_len = total;
}

namespace gwa {
// Pipeline use (pipeline.cpp): the whole batch's SAM text into a caller buffer (pinned host memory,
// grown with hipHostMalloc as needed); returns its size.  Throws on a failing read.
uint64_t batchSamInto(gwa_batch_t *b, char **buf, uint64_t *cap) {
  if (b->headerOnly) {
    if (!b->ran) throw std::runtime_error("gwa_batch_run has not completed");
    return 0;
  }
  const uint64_t total = formatOnDevice(b, nullptr, 0, b->pairs ? b->pairs : b->n);
  if (*cap < total) {
    if (*buf) (void)hipHostFree(*buf);
    *buf = nullptr;
    *cap = 0;
    const uint64_t want = total + total / 8 + (1 << 20);
    HIPCHK(hipHostMalloc((void **)buf, want, hipHostMallocDefault));
    *cap = want;
  }
  if (total) HIPCHK(hipMemcpyAsync(*buf, b->d_fmtText, total, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return total;
}
void pinnedFree(char *p) {
  if (p) (void)hipHostFree(p);
}
char *pinnedAlloc(uint64_t bytes) {
  char *p = nullptr;
  HIPCHK(hipHostMalloc((void **)&p, bytes, hipHostMallocDefault));
  return p;
}
}  // namespace gwa

extern "C" {

int gwa_batch_stats(gwa_batch_t *b, gwa_batch_stats_t *st) {
  try {
    ensureStats(b);
    *st = b->stats;
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

int gwa_batch_format(gwa_batch_t *b, uint64_t *sam_bytes) {
  try {
    *sam_bytes = b->headerOnly ? 0 : formatOnDevice(b, nullptr, 0, b->pairs ? b->pairs : b->n);
    b->fmtWhole = true;
    if (b->headerOnly) b->fmtBytes = 0;
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

int gwa_batch_sam_copy(gwa_batch_t *b, void *dst, uint64_t *len) {
  try {
    if (!b->fmtWhole) throw std::runtime_error("gwa_batch_sam_copy: the batch's SAM text was not formatted by gwa_batch_format");
    *len = b->fmtBytes;
    if (dst && b->fmtBytes) {
      HIPCHK(hipSetDevice(b->ix->device));
      HIPCHK(hipMemcpyAsync(dst, b->d_fmtText, b->fmtBytes, hipMemcpyDeviceToDevice, b->stream));
      HIPCHK(hipStreamSynchronize(b->stream));
    }
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

int gwa_batch_results(gwa_batch_t *b, gwa_results_t *out) {
  return gwa_batch_results_range(b, 0, b->pairs ? b->pairs : b->n, out);
}

int gwa_batch_create_pairs(gwa_index_t *ix, const gwa_config_t *cfg, const gwa_reads_t *mate1, const gwa_reads_t *mate2,
                           int32_t min_insert, int32_t max_insert, gwa_batch_t **out) {
  try {
    if (mate1->n != mate2->n) throw std::runtime_error("paired-end: the mate files hold different numbers of reads");
    if (cfg->strategy != 0) throw std::runtime_error("paired-end alignment runs the -m bsf search");
    if (min_insert < 0 || max_insert < min_insert) throw std::runtime_error("bad insert-size range");
    // one batch of 2n single-end reads: mate 1 of every pair, then mate 2
    const uint32_t n = mate1->n;
    std::string blob[3];
    std::vector<uint64_t> off[3];
    const gwa_reads_t *ms[2] = {mate1, mate2};
    const bool anyQual = mate1->qual || mate2->qual;
    std::vector<uint8_t> qnull;  // per read of the combined batch: no quality
    for (int f = 0; f < 3; ++f) {
      if (f == 2 && !anyQual) break;
      off[f].reserve(2 * (size_t)n + 1);
      off[f].push_back(0);
      for (int k = 0; k < 2; ++k) {
        const gwa_reads_t *r = ms[k];
        if (f == 2 && !r->qual) {  // this mate set has no qualities: empty ranges, marked null
          for (uint32_t i = 1; i <= n; ++i) off[f].push_back(off[f].back());
          continue;
        }
        const char *base = f == 0 ? r->name : f == 1 ? r->seq : r->qual;
        const uint64_t *o = f == 0 ? r->name_off : f == 1 ? r->seq_off : r->qual_off;
        blob[f].append(base + o[0], o[n] - o[0]);
        const uint64_t at = off[f].back();
        for (uint32_t i = 1; i <= n; ++i) off[f].push_back(at + (o[i] - o[0]));
      }
    }
    if (anyQual && (!mate1->qual || !mate2->qual || mate1->qual_null || mate2->qual_null)) {
      qnull.assign(2 * (size_t)n, 0);
      for (int k = 0; k < 2; ++k)
        for (uint32_t i = 0; i < n; ++i)
          qnull[(size_t)k * n + i] = !ms[k]->qual ? 1 : (ms[k]->qual_null && ms[k]->qual_null[i]) ? 1 : 0;
    }
    gwa_reads_t both{2 * n, blob[0].data(), blob[1].data(), anyQual ? blob[2].data() : nullptr, off[0].data(),
                     off[1].data(), anyQual ? off[2].data() : nullptr, qnull.empty() ? nullptr : qnull.data()};
    gwa_config_t c = *cfg;
    c.report_type = 1;  // every best hit of a mate is a pairing candidate
    if (gwa_batch_create(ix, &c, &both, out) != 0) return -1;
    (*out)->pairs = n;
    (*out)->minIns = min_insert;
    (*out)->maxIns = max_insert;
    (*out)->d_rescue = bAlloc<RescueOut>(n);
    (*out)->d_heavy = bAlloc<uint32_t>((size_t)n + 2);  // list, its count, rescues skipped (window)
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

int gwa_batch_results_range(gwa_batch_t *b, uint32_t first, uint32_t count, gwa_results_t *out) {
  try {
    if ((uint64_t)first + count > (b->pairs ? b->pairs : b->n)) throw std::runtime_error("result range out of bounds");
    formatResults(b, nullptr, first, count, out);
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

int gwa_batch_results_select(gwa_batch_t *b, const uint32_t *idx, uint32_t count, gwa_results_t *out) {
  try {
    for (uint32_t j = 0; j < count; ++j)
      if (idx[j] >= (b->pairs ? b->pairs : b->n)) throw std::runtime_error("result index out of bounds");
    formatResults(b, idx, 0, count, out);
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

int gwa_batch_read_counters(gwa_batch_t *b, int32_t *out) {
  try {
    if (!b->ran) throw std::runtime_error("gwa_batch_run has not completed");
    if (b->headerOnly) throw std::runtime_error("-m bd / -m bwa batches have no device counters");
    HIPCHK(hipSetDevice(b->ix->device));
    std::vector<OutHeader> oh(b->n);
    std::vector<ScanRes> sr(b->n);
    HIPCHK(hipMemcpy(oh.data(), b->d_oh, b->n * sizeof(OutHeader), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(sr.data(), b->d_sres, b->n * sizeof(ScanRes), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < b->n; ++i) {
      const OutHeader &h = oh[i];
      int32_t *o = out + (size_t)i * GWA_READ_COUNTERS;
      o[8] = sr[i].nmF; o[9] = sr[i].lmF; o[10] = sr[i].nmR; o[11] = sr[i].lmR;
      o[0] = h.status; o[1] = h.fmSearches; o[2] = h.quickSteps; o[3] = h.blocks; o[4] = h.searchBlocks;
      o[5] = h.states; o[6] = h.saReads; o[7] = h.nHits;
      o[12] = (b->cfg.strategy == 0 && h.states == 0) ? -1 : 0;
      o[13] = h.kmerLookups; o[14] = h.quickShort; o[15] = h.searchShort;
      o[16] = h.numSW; o[17] = h.verifyBytes; o[18] = o[19] = 0;
    }
    for (auto &d : b->deep) {
      int32_t &t = out[(size_t)d.first * GWA_READ_COUNTERS + 12];
      t = std::max(t, (int32_t)d.second);
    }
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

void gwa_batch_free(gwa_batch_t *b) {
  if (!b) return;
  (void)hipSetDevice(b->ix->device);
  freeBatchDev(b);
  delete b;
}

void gwa_results_free(gwa_results_t *r) {
  if (!r) return;
  free(r->sam);
  free(r->line_off);
  free(r->records);
  r->sam = nullptr;
  r->line_off = nullptr;
  r->records = nullptr;
  r->n_records = 0;
}

int gwa_results_records(const gwa_index_t *ix, gwa_results_t *r) {
  try {
    free(r->records);
    r->records = nullptr;
    r->n_records = 0;
    std::vector<gwa_record_t> recs;
    const HostIndex &h = ix->host;
    // contig name -> index (the first contig of that name, as String.equals lookups would find)
    std::vector<std::pair<std::string, int>> byName;
    for (size_t i = 0; i < h.names.size(); ++i) byName.push_back({h.names[i], (int)i});
    std::stable_sort(byName.begin(), byName.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    auto refOf = [&](const char *p, size_t n) -> int {
      if (n == 1 && p[0] == '*') return -1;
      const std::string k(p, n);
      auto it = std::lower_bound(byName.begin(), byName.end(), k, [](const auto &a, const std::string &x) { return a.first < x; });
      if (it == byName.end() || it->first != k) throw std::runtime_error("SAM record names an unknown contig: " + k);
      return it->second;
    };
    const char *t = r->sam;
    for (uint32_t i = 0; i < r->n_reads; ++i) {
      uint64_t a = r->line_off[i];
      const uint64_t e = r->line_off[i + 1];
      while (a < e) {
        const char *nl = (const char *)memchr(t + a, '\n', e - a);
        const uint64_t le = nl ? (uint64_t)(nl - t) : e;
        // the tab-separated fields of the line
        std::vector<std::pair<uint64_t, uint64_t>> f;
        uint64_t b = a;
        for (uint64_t x = a; x <= le; ++x)
          if (x == le || t[x] == '\t') {
            f.push_back({b, x - b});
            b = x + 1;
          }
        if (f.size() < 11) throw std::runtime_error("malformed SAM line in results");
        gwa_record_t g{};
        g.read = i;
        g.flag = (uint32_t)strtoul(std::string(t + f[1].first, f[1].second).c_str(), nullptr, 10);
        g.ref = refOf(t + f[2].first, f[2].second);
        g.pos = (int32_t)strtol(std::string(t + f[3].first, f[3].second).c_str(), nullptr, 10);
        g.end = g.pos;
        g.strand = (g.flag & 0x10) ? 1 : 0;
        g.nm = -1;
        g.x0 = 0;
        g.split = -1;
        g.line_off = a; g.line_len = (uint32_t)(le - a);
        g.name_off = f[0].first; g.name_len = (uint32_t)f[0].second;
        g.cigar_off = f[5].first; g.cigar_len = (uint32_t)f[5].second;
        g.seq_off = f[9].first; g.seq_len = (uint32_t)f[9].second;
        g.qual_off = f[10].first; g.qual_len = (uint32_t)f[10].second;
        g.qual_null = (f[10].second == 1 && t[f[10].first] == '*') ? 1 : 0;
        for (size_t k = 11; k < f.size(); ++k) {
          const char *p = t + f[k].first;
          if (f[k].second >= 5 && !memcmp(p, "NM:i:", 5)) g.nm = (int32_t)strtol(std::string(p + 5, f[k].second - 5).c_str(), nullptr, 10);
          else if (f[k].second >= 5 && !memcmp(p, "X0:i:", 5)) g.x0 = (int32_t)strtol(std::string(p + 5, f[k].second - 5).c_str(), nullptr, 10);
          else if (f[k].second >= 5 && !memcmp(p, "XP:Z:", 5)) { g.state_off = f[k].first + 5; g.state_len = (uint32_t)(f[k].second - 5); }
        }
        // single-end results: a first line with FLAG 0x1 and without 0x80 is followed by its split
        // record (AlignmentRecord.toSAMLine, R/AlignmentRecord.java:109-170); paired-end results have
        // two mate lines per unit and no split records
        if (!r->paired && !recs.empty() && recs.back().split == -2) {
          gwa_record_t &first = recs.back();
          first.split = (int32_t)recs.size();
          g.is_split = 1;
        }
        if (!r->paired && (g.flag & 0x1) && !(g.flag & 0x80) && !g.is_split) {
          g.split = -2;  // (resolved by the next line)
          g.end = g.pos;
        }
        recs.push_back(g);
        a = le + 1;
      }
    }
    // the split record's end = POS + TLEN of its first line (AlignmentRecord.toSAMLine prints
    // split.end - start as TLEN)
    for (size_t k = 0; k < recs.size(); ++k) {
      if (recs[k].split == -2) throw std::runtime_error("SAM results end inside a split record pair");
      if (recs[k].split >= 0) {
        const gwa_record_t &g = recs[k];
        const char *p = t + g.line_off;
        // TLEN is field 9 (index 8)
        int tab = 0;
        uint64_t x = 0;
        while (x < g.line_len && tab < 8) tab += p[x++] == '\t';
        recs[(size_t)g.split].end = g.pos + (int32_t)strtol(p + x, nullptr, 10);
      }
    }
    r->records = (gwa_record_t *)malloc(sizeof(gwa_record_t) * std::max<size_t>(1, recs.size()));
    if (!r->records) throw std::runtime_error("out of host memory for the records");
    if (!recs.empty()) memcpy(r->records, recs.data(), sizeof(gwa_record_t) * recs.size());
    r->n_records = recs.size();
    return 0;
  } catch (std::exception &e) {
    return fail(e.what());
  }
}

int gwa_align_pairs(gwa_index_t *ix, const gwa_config_t *cfg, const gwa_reads_t *mate1, const gwa_reads_t *mate2,
                    int32_t min_insert, int32_t max_insert, gwa_results_t *out) {
  gwa_batch_t *b = nullptr;
  if (gwa_batch_create_pairs(ix, cfg, mate1, mate2, min_insert, max_insert, &b) != 0) return -1;
  int rc = gwa_batch_run(b);
  if (rc == 0) rc = gwa_batch_results(b, out);
  gwa_batch_free(b);
  return rc;
}

int gwa_align_batch(gwa_index_t *ix, const gwa_config_t *cfg, const gwa_reads_t *reads, gwa_results_t *out) {
  gwa_batch_t *b = nullptr;
  if (gwa_batch_create(ix, cfg, reads, &b) != 0) return -1;
  int rc = gwa_batch_run(b);
  if (rc == 0) rc = gwa_batch_results(b, out);
  gwa_batch_free(b);
  return rc;
}

}  // extern "C"
