// gwa_kernels_long.hip -- the QW = 16 instances of the search kernels (search_kernels.h): reads of
// 257..512 bp (16 two-bit query words per strand, up to 8 DP blocks of 64 rows).  Their own translation
// unit, so they build in parallel with gwa_kernels.hip.
#include "search_kernels.h"

namespace gwa {

void launchQuickscan16(const IndexView &ix, const SearchConfig &cfg, const ReadsView &reads, ScanRes *sres, OutHeader *oh,
                       const OutSlots &os, uint32_t *searchList, uint32_t *searchCount, const uint32_t *order,
                       hipStream_t s, uint32_t *trace, int traceRead) {
  launchQuickscanT<16>(ix, cfg, reads, sres, oh, os, searchList, searchCount, order, s, trace, traceRead);
}

void launchSearch16(int R, int ldsHeap, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                    const ReadsView &reads, const ScanRes *sres, const uint32_t *list, uint32_t n, uint8_t *scratch,
                    uint64_t laneStride, const Caps &caps, OutHeader *oh, const OutSlots &os, const int32_t *chrRank,
                    uint32_t *work, uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits, hipStream_t s,
                    uint32_t *trace, int traceRead) {
  launchSearchT<16>(R, ldsHeap, lanes, ix, cfg, st, reads, sres, list, n, scratch, laneStride, caps, oh, os, chrRank, work,
                    ovfList, ovfCount, ovfBits, s, trace, traceRead);
}

void launchSfSearch16(int R, uint32_t lanes, const IndexView &ix, const SearchConfig &cfg, const StairTables &st,
                      const ReadsView &reads, const uint32_t *list, uint32_t n, uint8_t *scratch, uint64_t laneStride,
                      const Caps &caps, OutHeader *oh, const OutSlots &os, const int32_t *chrRank, uint32_t *work,
                      uint32_t *ovfList, uint32_t *ovfCount, uint32_t *ovfBits, hipStream_t s) {
  launchSfSearchT<16>(R, true, lanes, ix, cfg, st, reads, list, n, scratch, laneStride, caps, oh, os, chrRank, work, ovfList,
                      ovfCount, ovfBits, s);
}

}  // namespace gwa
