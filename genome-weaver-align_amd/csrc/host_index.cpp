// host_index.cpp -- host half of index construction: FASTA packing, host cyclic SA (small and
// mid-size texts; large texts use the GPU builder in sa_build.hip), Occ-block layout, 2-bit text,
// staircase-filter tables.
#include "host_index.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <parallel/algorithm>
#include <stdexcept>

namespace gwa {

void addSequence(const std::string &name, const char *seq, size_t len, HostIndex &ix) {
  int64_t off = (int64_t)ix.T.size();
  for (size_t i = 0; i < len; ++i)
    if (seq[i] != ' ') ix.T.push_back(to3bit((unsigned char)seq[i]));
  ix.names.push_back(name);
  ix.offsets.push_back(off);
  ix.lengths.push_back((int64_t)ix.T.size() - off);
  ix.N = ix.T.size();
}

void packFasta(const char *text, size_t len, HostIndex &ix) {
  // one pass, lines found with memchr, codes written through a 256-entry table
  uint8_t lut[256];
  for (int c = 0; c < 256; ++c) lut[c] = to3bit((unsigned char)c);
  const char *p = text, *end = text + len;
  bool inSeq = false;
  std::string name;
  int64_t off = (int64_t)ix.T.size();
  size_t n = ix.T.size();
  ix.T.resize(n + len);  // upper bound, trimmed at the end
  uint8_t *o = ix.T.data();
  auto finish = [&]() {
    if (!inSeq) return;
    ix.names.push_back(name);
    ix.offsets.push_back(off);
    ix.lengths.push_back((int64_t)n - off);
    off = (int64_t)n;
  };
  while (p < end) {
    const char *e = (const char *)memchr(p, '\n', (size_t)(end - p));
    if (!e) e = end;
    const char *le = e;
    if (le > p && le[-1] == '\r') le--;
    if (le > p && *p == '>') {
      finish();
      const char *a = p + 1;
      while (a < le && isspace((unsigned char)*a)) a++;
      const char *b = a;
      while (b < le && !isspace((unsigned char)*b) && *b != '|') b++;
      name.assign(a, b);
      inSeq = true;
    } else if (inSeq) {
      // the line trimmed of chars <= ' ' at both ends (Java String.trim), every char through to3bit
      const char *a = p, *b = le;
      while (a < b && (unsigned char)*a <= ' ') a++;
      while (b > a && (unsigned char)b[-1] <= ' ') b--;
      for (; a < b; ++a) o[n++] = lut[(unsigned char)*a];
    }
    p = e + 1;
  }
  finish();
  ix.T.resize(n);
  ix.N = n;
}

void rankNames(HostIndex &ix) {
  // Java String.compareTo over ASCII names == byte-wise lexicographic order
  std::vector<std::string> u = ix.names;
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  ix.chrRank.resize(ix.names.size());
  for (size_t i = 0; i < ix.names.size(); ++i)
    ix.chrRank[i] = (int32_t)(std::lower_bound(u.begin(), u.end(), ix.names[i]) - u.begin());
}

// Prefix doubling over cyclic rotations.  Initial key: the first K symbols of each rotation
// packed `alphabetBits` bits apiece; then (rank[i], rank[i+h]) pairs with h doubling.
bool cyclicSAHost(const uint8_t *codes, uint64_t n, std::vector<uint32_t> &sa, int alphabetBits) {
  sa.resize(n);
  if (n == 0) return true;
  if (n >= (1ULL << 32)) throw std::runtime_error("text longer than 2^32-1 is not supported");
  const int K = 63 / alphabetBits;
  struct KV { uint64_t key; uint32_t idx; };
  std::vector<KV> kv(n);
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t key = 0;
    uint64_t p = i;
    for (int j = 0; j < K; ++j) {
      key = (key << alphabetBits) | codes[p];
      if (++p == n) p = 0;
    }
    kv[i] = {key, (uint32_t)i};
  }
  auto lessKV = [](const KV &a, const KV &b) { return a.key < b.key || (a.key == b.key && a.idx < b.idx); };
  __gnu_parallel::sort(kv.begin(), kv.end(), lessKV);
  std::vector<uint32_t> rank(n);
  auto assign = [&](bool *allUnique) {
    uint64_t groupStart = 0;
    bool uniq = true;
    for (uint64_t j = 0; j < n; ++j) {
      if (j > 0 && kv[j].key != kv[j - 1].key) groupStart = j;
      else if (j > 0) uniq = false;
      rank[kv[j].idx] = (uint32_t)groupStart;
    }
    *allUnique = uniq;
  };
  bool uniq;
  assign(&uniq);
  uint64_t h = (uint64_t)K;
  while (!uniq) {
    if (h >= n) return false;  // periodic text: rotations tie
    for (uint64_t j = 0; j < n; ++j) {
      uint32_t i = kv[j].idx;
      uint64_t i2 = (i + h) % n;
      kv[j].key = ((uint64_t)rank[i] << 32) | rank[i2];
    }
    __gnu_parallel::sort(kv.begin(), kv.end(), lessKV);
    assign(&uniq);
    h *= 2;
  }
  for (uint64_t j = 0; j < n; ++j) sa[j] = kv[j].idx;
  return true;
}

static void buildOcc(const std::vector<uint8_t> &T, const std::vector<uint32_t> &SA, std::vector<OccBlock> &occ) {
  const uint64_t n = T.size();
  const uint64_t nb = n / 128 + 1;
  occ.assign(nb, OccBlock());
  memset(occ.data(), 0, nb * sizeof(OccBlock));
  uint32_t cnt[4] = {0, 0, 0, 0};
  for (uint64_t b = 0; b < nb; ++b) {
    OccBlock &B = occ[b];
    for (int c = 0; c < 4; ++c) B.cnt[c] = cnt[c];
    for (uint64_t p = b * 128; p < std::min<uint64_t>(n, (b + 1) * 128); ++p) {
      // BWT[p] = T[(SA[p] - 1 + n) % n]   (A/BWTransform.java:172-179)
      uint64_t src = SA[p] == 0 ? n - 1 : SA[p] - 1;
      uint8_t c = T[src];
      int r = (int)(p - b * 128);
      if (c >= 4) {
        B.nmask[r >> 6] |= 1ULL << (r & 63);
      } else {
        if (c & 1) B.lo[r >> 6] |= 1ULL << (r & 63);
        if (c & 2) B.hi[r >> 6] |= 1ULL << (r & 63);
        cnt[c]++;
      }
    }
  }
}

void finishIndex(HostIndex &ix) {
  const uint64_t n = ix.N;
  std::vector<uint8_t> R(n);
  for (uint64_t i = 0; i < n; ++i) R[i] = ix.T[n - 1 - i];
  buildOcc(ix.T, ix.sa[0], ix.occ[0]);
  buildOcc(R, ix.sa[1], ix.occ[1]);
  uint64_t count[5] = {0, 0, 0, 0, 0};
  for (uint64_t i = 0; i < n; ++i) count[ix.T[i] > 4 ? 4 : ix.T[i]]++;
  uint64_t sum = 0;
  for (int c = 0; c < 5; ++c) { ix.C[c] = sum; sum += count[c]; }
  ix.text2.assign(n / 32 + 2, 0);
  ix.textN.assign(n / 64 + 2, 0);
  for (uint64_t i = 0; i < n; ++i) {
    uint8_t c = ix.T[i];
    if (c >= 4) ix.textN[i >> 6] |= 1ULL << (i & 63);
    else ix.text2[i >> 5] |= (uint64_t)c << ((i & 31) * 2);
  }
  rankNames(ix);
}

// ---------------------------------------------------------------------------------------------
// StaircaseFilter (S/StaircaseFilter.java:47-102) with BitVector (A/BitVector.java) semantics,
// evaluated once per (read length, minMismatches) on the host.
// ---------------------------------------------------------------------------------------------
namespace {
inline int64_t jl(int64_t x, int64_t s) { return (int64_t)((uint64_t)x << (s & 63)); }
inline int64_t jr(int64_t x, int64_t s) { return (int64_t)((uint64_t)x >> (s & 63)); }
struct JavaThrow {};
struct BV {
  int64_t size;
  std::vector<int64_t> b;
  explicit BV(int64_t s) : size(s), b((size_t)((s + 63) / 64), 0) {}
  void notInPlace() {
    if (b.empty()) throw JavaThrow();
    for (size_t i = 0; i + 1 < b.size(); ++i) b[i] = ~b[i];
    int off = (int)size % 64;
    b.back() = (~b.back()) & ~jl(~0LL, off);
  }
  void lshiftInPlace(int len) {
    int bo = len / 64;
    int64_t off = len % 64;
    int64_t lowMask = ~jr(~0LL, off);
    int nb = (int)b.size();
    for (int i = nb - 1; i >= 0; --i) {
      int x = i - bo;
      if (x >= nb || x - 1 >= nb) throw JavaThrow();
      int64_t high = x >= 0 ? jl(b[(size_t)x], off) : 0;
      int64_t low = (x - 1 >= 0) ? jr(b[(size_t)x - 1] & lowMask, 64 - off) : 0;
      b[(size_t)i] = high | low;
    }
  }
  int64_t sub64(int64_t start, int64_t end) const {
    int pos = (int)(start / 64);
    if (pos >= (int)b.size()) return 0;
    if (pos < 0) throw JavaThrow();
    int64_t range = end - start;
    int64_t mask = range >= 64 ? ~0LL : ~jl(~0LL, range);
    int64_t off = start % 64;
    int64_t low = jr(b[(size_t)pos], off);
    int64_t high = pos + 1 < (int)b.size() ? jl(b[(size_t)pos + 1] & ~jl(~0LL, off), 64 - off) : 0;
    return (high | low) & mask;
  }
};
inline int8_t jb(int x) { return (int8_t)(uint8_t)(uint32_t)x; }
}  // namespace

// words of the table block of one read length (the offsets table, then the raw masks)
static size_t stairBlockWords(int m, int kmax) {
  const size_t W = (size_t)(m + 63) / 64;
  return (size_t)(kmax + 2) * (size_t)(kmax + 1) * ((size_t)(m + kmax + 1) + W);
}

namespace {
// Blocks already built, per (read length, kmax): a pipeline creates one batch per chunk of a file
// and the chunks share their read lengths, so each block is built once per process, not per batch.
struct StairBlock {
  std::vector<uint64_t> words;
  uint64_t threw = 0;
};
std::mutex g_stairMu;
std::map<std::pair<int, int>, std::shared_ptr<const StairBlock>> g_stairCache;
size_t g_stairCacheWords = 0;
const size_t kStairCacheWords = (size_t)64 << 20;  // 512 MiB of cached blocks at most
}  // namespace

void buildStairTables(const std::vector<int> &lengths, int kmax, std::vector<uint64_t> &tab, std::vector<uint32_t> &base,
                      std::vector<uint64_t> &bad) {
  base.assign(kMaxReadLen + 1, 0xFFFFFFFFu);
  bad.assign(kMaxReadLen + 1, 0);
  tab.clear();
  {  // every block indexes rows and offsets by the batch's kmax: refuse a table too large to stage
    size_t words = 0;
    for (int m : lengths)
      if (m >= 0 && m <= kMaxReadLen) words += stairBlockWords(m, kmax);
    if (words > kStairMaxWords)
      throw std::runtime_error("staircase tables of this batch's read lengths at k " + std::to_string(kmax) + " need " +
                               std::to_string(words * 8 >> 20) + " MiB (limit " + std::to_string(kStairMaxWords * 8 >> 20) +
                               " MiB): align reads of very different lengths in separate batches");
    tab.reserve(words);
  }
  for (int m : lengths) {
    if (m < 0 || m > kMaxReadLen || base[(size_t)m] != 0xFFFFFFFFu) continue;
    std::shared_ptr<const StairBlock> blk;
    {
      std::lock_guard<std::mutex> g(g_stairMu);
      auto it = g_stairCache.find({m, kmax});
      if (it != g_stairCache.end()) blk = it->second;
    }
    if (!blk) {
      auto nb = std::make_shared<StairBlock>();
      nb->threw = buildStairBlock(m, kmax, nb->words);
      blk = nb;
      std::lock_guard<std::mutex> g(g_stairMu);
      if (g_stairCacheWords + blk->words.size() <= kStairCacheWords) {
        g_stairCache[{m, kmax}] = blk;
        g_stairCacheWords += blk->words.size();
      }
    }
    base[(size_t)m] = (uint32_t)tab.size();
    bad[(size_t)m] = blk->threw;
    tab.insert(tab.end(), blk->words.begin(), blk->words.end());
  }
  if (tab.empty()) tab.push_back(0);
}

// one read length's block (layout in BsfLane::stairMask / stairMaskRaw); returns bit kk set when
// StaircaseFilter(m, kk) throws
uint64_t buildStairBlock(int m, int kmax, std::vector<uint64_t> &tab) {
  tab.assign(stairBlockWords(m, kmax), 0);
  {
    const size_t perRow = (size_t)(m + kmax + 1);
    const size_t start = 0;
    const size_t W = (size_t)(m + 63) / 64, rawAt = start + (size_t)(kmax + 2) * (size_t)(kmax + 1) * perRow;
    uint64_t threw = 0;  // bit kk: StaircaseFilter(m, kk) throws
    for (int kk = 0; kk <= kmax + 1; ++kk) {
      try {
        int lastChunkSize = (m - kk >= 6) ? m * 2 / (kk + 2) : m - kk;
        std::vector<int8_t> cs((size_t)kk + 2, 0);
        int8_t rest = jb(m - lastChunkSize);
        if (kk == 0) cs[0] = rest;
        else for (int i = 0; i <= kk; ++i) cs[(size_t)i] = jb((int)rest * i / kk);
        cs[(size_t)kk + 1] = jb(m);
        std::vector<BV> masks;
        for (int i = 0; i <= kk; ++i) {
          BV v(m);
          v.notInPlace();
          v.lshiftInPlace(cs[(size_t)i]);
          masks.push_back(v);
        }
        for (int row = 0; row <= kmax; ++row)
          for (int off = -kmax; off <= m; ++off) {
            int64_t val;
            if (row >= (int)masks.size()) val = 0;
            else if (off >= 0) val = jl(~0LL, m - off) | masks[(size_t)row].sub64(off, off + 64);
            else val = jl(masks[(size_t)row].sub64(0, 64), -off);
            tab[start + ((size_t)kk * (size_t)(kmax + 1) + (size_t)row) * perRow + (size_t)(off + kmax)] = (uint64_t)val;
          }
        // the masks themselves, for offsets outside [-kmax, m] (BsfLane::stairMask)
        for (int row = 0; row < (int)masks.size() && row <= kmax; ++row)
          for (size_t w = 0; w < W && w < masks[(size_t)row].b.size(); ++w)
            tab[rawAt + ((size_t)kk * (size_t)(kmax + 1) + (size_t)row) * W + w] = (uint64_t)masks[(size_t)row].b[w];
      } catch (JavaThrow &) {
        threw |= 1ULL << kk;
      }
    }
    return threw;
  }
}

}  // namespace gwa
