// kernels.h -- host-callable launchers of the HIP kernels (gwa_kernels.hip, sa_build.hip)
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "gwa_layout.h"

namespace gwa {

struct Caps;

void launchQuickscan(int QW, const IndexView &ix, const SearchConfig &cfg, const ReadsView &reads, ScanRes *sres, OutHeader *oh,
                     const OutSlots &os, uint32_t *searchList, uint32_t *searchCount,
                     hipStream_t s, uint32_t *trace = nullptr, int traceRead = -1);
// -m sf: every read's quick-scan result into sres (the search-list key), nothing else written
void launchKeyscan(int QW, const IndexView &ix, const SearchConfig &cfg, const ReadsView &reads, ScanRes *sres,
                   hipStream_t s);
void launchSearch(int R, int QW, int ldsHeap, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                  const ReadsView &reads, const ScanRes *sres, const uint32_t *list, uint32_t n, uint8_t *scratch,
                  uint64_t laneStride, const Caps &caps, OutHeader *oh, const OutSlots &os,
                  const int32_t *chrRank, uint32_t *work, uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits,
                  const ResumeBufs &res, hipStream_t s, uint32_t *trace = nullptr, int traceRead = -1);
size_t resumeBytesFor(int R, const Caps &c);  // one resume record of a tier with capacities c
void launchSfSearch(int R, int QW, bool wrap, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                    const ReadsView &reads, const uint32_t *list, uint32_t n, uint8_t *scratch, uint64_t laneStride,
                    const Caps &caps, OutHeader *oh, const OutSlots &os,
                    const int32_t *chrRank, uint32_t *work, uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits,
                    hipStream_t s, uint32_t *trace = nullptr);
void buildKmerTable(const IndexView &ix, int fm, int K, uint64_t *out, hipStream_t s);

// batch_io.hip: reads in (encode on the device), SAM out (two-pass formatting), batch statistics
struct SamText;
constexpr uint32_t kLenSeen = 65536;  // read-length presence table (lengths >= 65535 share the last slot)
constexpr int kStatFields = 15;
void launchEncode(const char *seq, const uint64_t *seqB, const uint64_t *seqE, uint32_t n, uint32_t *codeLen,
                  uint32_t *rowLen, uint32_t *codeOff, uint32_t *lenSeen, uint8_t *codes, void *scanTmp,
                  size_t scanTmpBytes, int pass, hipStream_t s);
void launchFastqFields(const char *text, uint64_t len, const uint64_t *start, uint32_t n, uint64_t *fields,
                       uint32_t *err, hipStream_t s);
size_t encodeScanTempBytes(uint32_t n);
struct PairSpec {  // paired-end formatting: np pairs (mate 1 = read i, mate 2 = read np + i); np = 0: single-end
  uint32_t np;
  int32_t minIns, maxIns;
  const RescueOut *resc;  // pair_rescue_kernel's output (or nullptr)
};
// paired-end mate rescue (orc_align_pairs rule 3) over np pairs, `lanes` persistent lanes
void launchPairRescue(uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                      const ReadsView &reads, const SamText &t, const OutHeader *oh, const OutHit *hits,
                      const uint16_t *cig, uint32_t np, int32_t minIns, int32_t maxIns, uint8_t *scratch,
                      uint64_t laneStride, const Caps &caps, RescueOut *out, int64_t quad, uint32_t *heavy,
                      uint32_t *heavyCount, hipStream_t s);
// the pair choice of the heavy pairs pair_rescue_kernel listed (one workgroup each)
void launchPairChoose(uint32_t nHeavy, const SamText &t, const OutHeader *oh, const OutHit *hits, const uint16_t *cig,
                      uint32_t np, int32_t minIns, int32_t maxIns, const uint32_t *heavy, int sortCap, RescueOut *out,
                      hipStream_t s);
void launchSamFormat(const SamText &t, const OutHeader *oh, const OutHit *hits, const uint16_t *cig, const uint32_t *idx,
                     uint32_t first, uint32_t n, uint64_t *len, uint64_t *off, void *scanTmp, size_t *scanTmpBytes,
                     uint32_t *err, char *out, int pass, hipStream_t s, const PairSpec &ps, uint64_t totalBytes = 0);
size_t samScanTempBytes(uint32_t n);
size_t sortSearchListTmpBytes(uint32_t n);
void launchSortSearchList(const uint32_t *listIn, uint32_t *listOut, uint32_t *keysIn, uint32_t *keysOut, uint32_t n,
                          const ScanRes *sres, bool byKey, void *tmp, size_t tmpBytes, hipStream_t s);
void launchStats(const OutHeader *oh, uint32_t n, unsigned long long *acc, hipStream_t s);
size_t laneBytesFor(int R, const Caps &c);  // per-lane slice
size_t ilvBytesFor(const Caps &c);          // per-lane share of the interleaved DP block

}  // namespace gwa
