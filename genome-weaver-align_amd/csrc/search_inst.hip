// search_inst.hip -- one (query words QW, NFA rows R) instance set of the search kernels
// (search_kernels.h), compiled once per pair by the Makefile (-DGWA_QW=.. -DGWA_R=..): the 12
// translation units build in parallel instead of one unit holding every instance.
#include "search_kernels.h"

#if !defined(GWA_QW) || !defined(GWA_R)
#error "search_inst.hip is built with -DGWA_QW=<4|8|16> -DGWA_R=<4|8|16|32>"
#endif

namespace gwa {
GWA_SEARCH_INSTANCE(template, GWA_QW, GWA_R)
#if GWA_R == 4
template void launchKeyscanT<GWA_QW>(const IndexView &, const SearchConfig &, const ReadsView &, ScanRes *, hipStream_t);
template void launchQuickscanT<GWA_QW>(const IndexView &, const SearchConfig &, const ReadsView &, ScanRes *, OutHeader *,
                                       const OutSlots &, uint32_t *, uint32_t *, hipStream_t, uint32_t *, int);
#endif
}  // namespace gwa
