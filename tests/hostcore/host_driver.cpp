// host_driver.cpp -- TEST-ONLY: runs the device kernel logic (bsf_core.h) on the CPU so the
// kernel's control flow can be debugged against the oracle without a GPU.  Never linked into
// libgwa.so and never used as a product fallback (the product C-ABI requires a GPU).
#include <cstdio>
#include <cstring>
#include <cmath>
#include <algorithm>
#include <string>
#include <type_traits>
#include <vector>

#include "../../genome-weaver-align_amd/csrc/bsf_core.h"
#include "../../genome-weaver-align_amd/csrc/sf_core.h"
#include "../../genome-weaver-align_amd/csrc/host_index.h"
#include "../../genome-weaver-align_amd/csrc/sam.h"
#include "../../genome-weaver-align_amd/csrc/sam_core.h"
#include "../../genome-weaver-align_amd/csrc/text_core.h"

using namespace gwa;

struct HC {
  HostIndex h;
  IndexView v{};
  std::vector<uint64_t> kmer[2];
};

static uint64_t g_suspends = 0;  // reads suspended (and resumed on the next tier), all calls
static uint64_t g_specJobs = 0, g_specMiss = 0, g_specTaken = 0;  // HC_SF_COOP: helper verifications, passes, roll-backs

// the GPU's capacity tiers (gwa_api.cpp kTiers) replayed on the CPU
template <int R, int QW>
static int runAll(HC *x, int strategy, const SearchConfig &cfg, const StairTables &st, int maxM, int kmax, uint32_t n,
                  const char *const *names, const char *const *seqs, const char *const *quals, std::string &sam,
                  int32_t *stats) {
  const int bMax = std::max(1, (maxM + 63) / 64), nref = maxM + 2 * kmax + 2;
  const int dpw = 2 * bMax * (nref + 1), path = maxM + nref + 8;
  // GWA_TEST_SLICE_SHIFT moves the first tier's DP slice off the diagonal (every edit then
  // overflows into the next tier): the slice fallback path gives the same SAM
  const int sl = 1 + (getenv("GWA_TEST_SLICE_SHIFT") ? atoi(getenv("GWA_TEST_SLICE_SHIFT")) : 0);
  // (k >= 4, R >= 8: the GPU's hybrid heap holds as many entries as the arena, gwa_batch_run)
  // (k >= 4: hit lists of 128 / 256 in tiers 0 / 1, gwa_batch_run)
  const bool w = R >= 8;
  const Caps tiers[4] = {{256, w ? 256 : kLdsHeap, w ? 128 : 32, w ? 128 : 32, w ? 2048 : 512, dpw, path, sl, 0},
                         {1024, 1024, w ? 256 : 64, w ? 256 : 64, w ? 4096 : 1024, dpw, path, 0, 0},
                         {4096, 4096, 256, 256, 4096, dpw, path, 0, 0}, {65536, 65536, 4096, 4096, 65536, dpw, path, 0, 0}};
  // -m sf tiers (gwa_api.cpp kSfTiers)
  const Caps sfTiers[4] = {{512, 512, 32, 32, 512, dpw, path, sl, 32, 0, 1}, {2048, 2048, 64, 64, 2048, dpw, path, 0, 512, 0, 1},
                           {8192, 8192, 256, 256, 4096, dpw, path, 0, 2048, 0, 1},
                           {65536, 65536, 4096, 4096, 65536, dpw, path, 0, 16384, 0, 1}};
  std::vector<uint8_t> scratch(std::max(laneBytes<R>(tiers[3]), laneBytes<R>(sfTiers[3])) + ilvBytes(tiers[3]) + 4096);
  // one read at a time: a one-slot OutSlots whose pool is large enough for any report
  const int chains = cfg.reportType == 0 ? 1 : 2;
  const uint32_t hitCap = chains * (cfg.numSplit + 1), cigCap = 64 * chains;
  const uint64_t poolH = 1 << 16, poolC = 1 << 20;
  std::vector<OutHit> oh(hitCap + poolH);
  std::vector<uint16_t> oc(cigCap + poolC);
  uint32_t used[3];
  OutSlots os{oh.data(), oc.data(), hitCap, cigCap, used, hitCap, hitCap + poolH, cigCap, cigCap + poolC};
  std::vector<int32_t> rk = x->h.chrRank;
  const SamNames sn = samNames(x->h);
  for (uint32_t i = 0; i < n; ++i) {
    std::vector<uint8_t> codes;
    for (const char *c = seqs[i]; *c; ++c)
      if (*c != ' ') codes.push_back(to3bit((unsigned char)*c));
    const size_t mlen = codes.size();
    codes.resize(((mlen + 15) & ~(size_t)15) + 16, 0);  // 16-B padded, as ReadsView
    OutHeader hd{};
    std::vector<uint32_t> tv(65537, 0);
    bool traced = false;
    std::vector<uint8_t> rec;  // the read's resume record from the tier that suspended it
    bool haveRec = false, quickDone = false;
    ScanRes sr{};
    // tiers 0-3, then the last tier with every capacity doubled per rerun (gwa_batch_run grows the
    // exceeded ones; doubling all of them gives the same results, capacities only decide overflow)
    for (int t = 0; t < 14; ++t) {
      Caps sc = sfTiers[t < 4 ? t : 3], bc = tiers[t < 4 ? t : 3];
      if (t == 0 && getenv("HC_T0_HITS")) { bc.hits = bc.list = atoi(getenv("HC_T0_HITS")); bc.cigar = 16 * bc.hits; }  // experiments
      if (t == 1 && getenv("HC_T1_HITS")) { bc.hits = bc.list = atoi(getenv("HC_T1_HITS")); bc.cigar = 16 * bc.hits; }
      if (t == 0 && getenv("HC_T0_ARENA")) { bc.arena = bc.heap = atoi(getenv("HC_T0_ARENA")); }
      if (t == 1 && getenv("HC_T1_ARENA")) { bc.arena = bc.heap = atoi(getenv("HC_T1_ARENA")); }
      if (t >= 4) {
        const int g = t - 3;
        for (Caps *c : {&sc, &bc}) {
          c->arena <<= g; c->heap <<= g; c->hits <<= g; c->list <<= g; c->cigar <<= g; c->cand <<= g;
        }
      }
      // the k >= 4 verification memo, as gwa_batch_run sizes it (GWA_VERIFY_MEMO=0: off)
      bc.cand = 0;
      if (R >= 8 && !(getenv("GWA_VERIFY_MEMO") && atoi(getenv("GWA_VERIFY_MEMO")) == 0)) {
        bc.cand = 64;
        while (bc.cand < 2 * bc.hits && bc.cand < (1 << 22)) bc.cand <<= 1;
      }
      // HC_SF_COOP=1: -m sf through the cooperative kernel's algorithm (search_kernels.h sf_search_kernel
      // COOP: deferred verification, 63 helper lanes sharing the slice) on every tier
      const bool coop = strategy == 1 && getenv("HC_SF_COOP") && atoi(getenv("HC_SF_COOP")) != 0;
      if (coop) {
        sc.spec = 64;
        while (sc.spec < sc.cand) sc.spec <<= 1;
      }
      {
        const size_t need = std::max(laneBytes<R>(sc), laneBytes<R>(bc)) + ilvBytes(bc) + 4096;
        if (scratch.size() < need) scratch.resize(need);
      }
      if (coop) {
        typedef SfLane<R, QW, true, 2> CL;
        LaneMem<R> L = laneMem<R>(scratch.data(), sc);
        const int hcap = sc.path / 2;
        static std::vector<uint8_t> hchunk;
        static std::vector<uint16_t> hcig;
        // (each helper's interleaved block 64-B aligned, as a wavefront's block is on the GPU: the
        // DP history is read and written as 16-B {vp, vn} pairs)
        const size_t hstride = (ilvBytes(sc) + 64 + 63) & ~(size_t)63;
        hchunk.assign((size_t)64 * hstride + 64, 0);
        uint8_t *hbase = (uint8_t *)(((uintptr_t)hchunk.data() + 63) & ~(uintptr_t)63);
        hcig.assign((size_t)64 * hcap, 0);
        std::vector<CL> ln;
        ln.reserve(64);
        for (int h = 0; h < 64; ++h) {
          LaneMem<R> Lh = laneMem<R>(scratch.data(), hbase + (size_t)h * hstride, 0, 1, sc);
          ln.emplace_back(x->v, cfg, st, h == 0 ? L : Lh, sc);
          ln[h].chrRank = rk.data();
          ln[h].initRead(codes.data(), (int)mlen);
        }
        for (int h = 0; h < 64; ++h) ln[h].coopClear(h);
        for (int h = 1; h < 64; ++h) ln[h].buildMasks();
        CL &o = ln[0];
        hd = OutHeader{};
        int run = o.sfBegin(false) ? 1 : 0;
        CL snap = o;  // (the kernel's copy of lane 0's registers where a deferral began)
        for (;;) {
          int need = 0;
          if (run) {
            int stp = 1;
            while (stp == 1 || stp == 3) {
              stp = o.template sfStepT<true>();
              if (stp == 3) {
                laneCopy(snap, o);
                o.dMode = 1;
                o.uOn = 1;
                stp = 1;
              }
            }
            need = stp == 2 ? 1 : 0;
            run = need;
          }
          if (!need) break;
          ++g_specMiss;  // (passes)
          const int qn = o.dN;
          for (int h = 1; h < 64; ++h) {
            if (!ln[h].djobLoad(h - 1, qn)) continue;
            int pos = 0, diff = 0, co = 0, cl = 0;
            ln[h].nCigar = 0;
            ln[h].status = ST_UNMAPPED;
            uint16_t *cg = hcig.data() + (size_t)h * hcap;
            const int r = ln[h].alignBlockDetailed(ln[h].jStrand, 0, (int)mlen, ln[h].jRefStart, ln[h].jRefEnd, &pos, &diff,
                                                   &co, &cl, cg, hcap);
            ln[h].specPut(r, pos, diff, co, cl, cg);
            ++g_specJobs;
          }
          bool go = true;
          if (o.dCommit(&go) >= 0) {
            ++g_specTaken;  // (roll-backs)
            o.undoApply();
            laneCopy(o, snap);
            o.dN = 0;
            go = o.candFinish();
          }
          run = go ? 1 : 0;
        }
        used[0] = used[1] = used[2] = 0;
        o.writeSearchOutput(&hd, os, 0);
        hd.quickSteps = o.quickSteps;
        if (hd.status != ST_OVERFLOW) break;
        continue;
      }
      if (strategy == 1) {
        LaneMem<R> L = laneMem<R>(scratch.data(), sc);
        SfLane<R, QW> lane(x->v, cfg, st, L, sc);
        lane.chrRank = rk.data();
        lane.initRead(codes.data(), (int)mlen);
        hd = OutHeader{};
        lane.sfSearch();
        used[0] = used[1] = used[2] = 0;
        lane.writeSearchOutput(&hd, os, 0);
        hd.quickSteps = lane.quickSteps;
        if (hd.status != ST_OVERFLOW) break;
        continue;
      }
      // the first tier's kernel keeps the DP slice (BsfLane DPM 1, search_kernels.h), the others checkpoints
      auto tier = [&](auto dpm) -> bool {  // false: the read is done
      typedef BsfLane<R, QW, false, 24, decltype(dpm)::value> Lane;
      LaneMem<R> L = laneMem<R>(scratch.data(), bc);
      Lane lane(x->v, cfg, st, L, bc);
      lane.chrRank = rk.data();
      const char *tre = getenv("GWA_TRACE_READ");
      const char *qtre = getenv("GWA_QTRACE_READ");
      if ((tre && atoi(tre) == (int)i) || (qtre && atoi(qtre) == (int)i)) { lane.trace = tv.data() + 1; lane.traceCap = 65536; traced = true; }
      lane.initRead(codes.data(), (int)mlen);
      used[0] = used[1] = used[2] = 0;
      // the kernel's lane loop (search_kernels.h bsf_search_kernel): steps and reports until the read
      // finishes or is suspended; a suspended read resumes on the next tier from its record, as there
      // (HC_NO_RESUME=1: every overflow restarts from the seeds, the pre-resume behaviour)
      int phase = Lane::LP_FINISH;
      int rp = 0;
      if (haveRec && lane.resumeFrom(rec.data(), i, &rp)) {
        phase = rp;
      } else if (t == 0 || !quickDone) {
        quickDone = true;
        phase = lane.quickPhase(&sr, &hd, os, 0) ? (lane.searchStart(sr) ? Lane::LP_RUN : Lane::LP_FINISH) : -1;
      } else {
        phase = lane.searchStart(sr) ? Lane::LP_RUN : Lane::LP_FINISH;
      }
      haveRec = false;
      if (phase == -1) {  // the quick scan finished the read
        if (traced) tv[0] = (uint32_t)lane.traceN;
        return false;
      }
      while (phase == Lane::LP_RUN || phase == Lane::LP_WAIT) phase = phase == Lane::LP_RUN ? lane.laneStep() : lane.laneReport();
      if (phase == Lane::LP_SUSPEND) {
        lane.status = ST_OVERFLOW;
        lane.writeSearchOutput(&hd, os, 0);
        if (!getenv("HC_NO_RESUME")) {
          rec.assign(Lane::resumeBytes(bc), 0);
          lane.suspendTo(rec.data(), i);
          haveRec = true;
        }
        ++g_suspends;
      } else {
        lane.writeSearchOutput(&hd, os, 0);
      }
      if (traced) tv[0] = (uint32_t)lane.traceN;
      if (hd.status == ST_OVERFLOW && getenv("HC_OVF_LOG")) fprintf(stderr, "[hc] read %u tier %d overflow 0x%x\n", i, t, hd.ovfWhat);
      return hd.status == ST_OVERFLOW;
      };
      const bool more = t == 0 ? tier(std::integral_constant<int, 1>()) : tier(std::integral_constant<int, 0>());
      if (!more) break;
    }
    if (traced) {
      FILE *tf = fopen("hc_trace.bin", "wb");
      if (tf) { fwrite(tv.data(), 4, 1 + tv[0], tf); fclose(tf); }
    }
    if (stats) { stats[i * 4] = hd.fmSearches; stats[i * 4 + 1] = hd.quickSteps; stats[i * 4 + 2] = hd.maxHeap; stats[i * 4 + 3] = hd.states; }
    // the device SAM writer (sam_core.h) on the host, for this one read
    const char *qv = quals ? quals[i] : nullptr;
    const uint64_t nameOff[2] = {0, strlen(names[i])}, qualOff[2] = {0, qv ? strlen(qv) : 0};
    const uint32_t codeOff[1] = {0}, codeLen[1] = {(uint32_t)mlen};
    const SamText t{names[i], nameOff, nameOff + 1, qv, qualOff, qualOff + 1, nullptr, codes.data(), codeOff, codeLen,
                    sn.blob.data(), sn.off.data(), rk.data(), sn.starKey, sn.emptyKey};
    if (hd.status == ST_MAPPED || hd.status == ST_UNMAPPED) {
      SamOut cnt{nullptr, 0};
      if (samRead(cnt, t, 0, hd, oh.data(), oc.data()) != 0) return -2;
      const size_t at = sam.size();
      sam.resize(at + cnt.n);
      SamOut o{&sam[at], 0};
      samRead(o, t, 0, hd, oh.data(), oc.data());
    } else {
      fprintf(stderr, "hc: status %d at read %u\n", hd.status, i);
      return -1 - hd.status;
    }
  }
  return 0;
}

extern "C" {

void *hc_index_codes(const uint8_t *codes, uint64_t n, int32_t nc, const char *const *names, const int64_t *lengths) {
  auto *x = new HC();
  x->h.T.assign(codes, codes + n);
  int64_t off = 0;
  for (int i = 0; i < nc; ++i) { x->h.names.push_back(names[i]); x->h.offsets.push_back(off); x->h.lengths.push_back(lengths[i]); off += lengths[i]; }
  x->h.N = n;
  std::vector<uint8_t> R(n);
  for (uint64_t i = 0; i < n; ++i) R[i] = codes[n - 1 - i];
  if (!cyclicSAHost(x->h.T.data(), n, x->h.sa[0]) || !cyclicSAHost(R.data(), n, x->h.sa[1])) { delete x; return nullptr; }
  finishIndex(x->h);
  IndexView &v = x->v;
  v.occ[0] = x->h.occ[0].data(); v.occ[1] = x->h.occ[1].data();
  v.sa[0] = x->h.sa[0].data(); v.sa[1] = x->h.sa[1].data();
  v.text2 = x->h.text2.data(); v.textN = x->h.textN.data();
  v.contigOff = x->h.offsets.data();
  v.nContig = (int32_t)x->h.names.size();
  v.N = n;
  for (int c = 0; c < 5; ++c) v.C[c] = x->h.C[c];
  // the k-mer tables, as gwa_api.cpp builds them on the GPU (GWA_KMER_K overrides k for tests)
  v.kmerK = getenv("GWA_KMER_K") ? atoi(getenv("GWA_KMER_K")) : kmerKFor(n);
  if (v.kmerK > 0) {
    const uint64_t nk = 1ULL << (2 * v.kmerK);
    for (int f = 0; f < 2; ++f) {
      x->kmer[f].resize(nk);
#pragma omp parallel for schedule(static)
      for (int64_t key = 0; key < (int64_t)nk; ++key) x->kmer[f][key] = kmerInterval(v.occ[f], v.C, n, (uint32_t)key, v.kmerK);
      v.kmer[f] = x->kmer[f].data();
    }
  }
  return x;
}

void *hc_index_fasta(const char *text, uint64_t len) {
  HostIndex tmp;
  packFasta(text, len, tmp);
  std::vector<const char *> nm;
  for (auto &s : tmp.names) nm.push_back(s.c_str());
  return hc_index_codes(tmp.T.data(), tmp.N, (int32_t)nm.size(), nm.data(), tmp.lengths.data());
}

void hc_index_free(void *p) { delete (HC *)p; }

uint64_t hc_suspends(void) { return g_suspends; }
void hc_spec_stats(uint64_t *out) { out[0] = g_specJobs; out[1] = g_specMiss; out[2] = g_specTaken; }

int hc_sa(void *p, int strand, uint32_t *out) {
  auto *x = (HC *)p;
  memcpy(out, x->h.sa[strand].data(), x->h.N * 4);
  return 0;
}

// Align with the kernel logic on the CPU; output SAM text (malloc'd).  stats[i*4..] = fm, quick, max heap, states
int hc_align(void *p, float k, int reportType, int numSplit, int strategy, uint32_t n, const char *const *names, const char *const *seqs,
             const char *const *quals, char **out, uint64_t *outLen, int32_t *stats) {
  auto *x = (HC *)p;
  SearchConfig cfg{};
  cfg.k = k; cfg.reportType = reportType; cfg.topL = 5; cfg.numSplit = numSplit;
  cfg.matchScore = 1; cfg.mismatchPenalty = 3; cfg.splitOpenPenalty = 11; cfg.indelEndSkip = 5; cfg.bandWidth = 31;
  cfg.waitQ16 = 16;
  cfg.textSearch = (numSplit <= 1 && !getenv("GWA_NO_TEXT")) ? 1 : 0;  // as gwa_batch_create
  cfg.runAheadMax = getenv("GWA_RUNAHEAD") ? atoi(getenv("GWA_RUNAHEAD")) : 1000;  // long runs on the CPU
  cfg.textCache = getenv("GWA_TEXT_CACHE") ? atoi(getenv("GWA_TEXT_CACHE")) : 1;
  std::vector<int> lens;
  int kmax = 0;
  for (uint32_t i = 0; i < n; ++i) {
    int m = 0;
    for (const char *c = seqs[i]; *c; ++c) m += *c != ' ';
    lens.push_back(m);
    int kk = (k > 0 && k < 1) ? (int)floor((double)((float)m * k)) : (int)k;
    kmax = std::max(kmax, kk);
  }
  std::vector<uint64_t> tab, bad;
  std::vector<uint32_t> base;
  buildStairTables(lens, kmax, tab, base, bad);
  StairTables st{tab.data(), base.data(), kmax, -1, 0, 0, bad.data()};
  std::string sam;
  int maxM = 1;
  for (int m : lens) maxM = std::max(maxM, m);
  int R = kmax + 1 <= 4 ? 4 : kmax + 1 <= 8 ? 8 : kmax + 1 <= 16 ? 16 : 32;
  int rc = 0;
  if (maxM > kMaxReadLen) return -9;
  // QW as gwa_api.cpp qwFor
#define HC_RUN(RR) (maxM <= 128 ? runAll<RR, 4> : maxM <= 256 ? runAll<RR, 8> : runAll<RR, 16>)
  switch (R) {
    case 4: rc = HC_RUN(4)(x, strategy, cfg, st, maxM, kmax, n, names, seqs, quals, sam, stats); break;
    case 8: rc = HC_RUN(8)(x, strategy, cfg, st, maxM, kmax, n, names, seqs, quals, sam, stats); break;
    case 16: rc = HC_RUN(16)(x, strategy, cfg, st, maxM, kmax, n, names, seqs, quals, sam, stats); break;
    default: rc = HC_RUN(32)(x, strategy, cfg, st, maxM, kmax, n, names, seqs, quals, sam, stats); break;
  }
#undef HC_RUN
  if (rc != 0) return rc;
  *out = (char *)malloc(sam.size() + 1);
  memcpy(*out, sam.c_str(), sam.size() + 1);
  *outLen = sam.size();
  return 0;
}
}

// the encode kernels' byte-parallel ACGT.to3bitCode (text_core.h)
extern "C" uint32_t hc_to3bit4(uint32_t x) { return to3bit4(x); }

// the -m sf kernel-instance rule (sf_core.h sfChunksWrap; search_kernels.h launchSfSearchT)
extern "C" int hc_sf_chunks_wrap(int m, int kk) { return sfChunksWrap(m, kk) ? 1 : 0; }
