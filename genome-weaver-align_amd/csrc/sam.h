// sam.h -- host-side AlignmentRecord conversion + SAM text
#pragma once
#include <string>
#include <vector>

#include "host_index.h"

namespace gwa {

std::string samHeader(const HostIndex &ix);

// Contig names as the SAM writer (sam_core.h SamText) reads them: one blob + offsets, and the keys
// of the names "*" and "" (the contig's chrRank when a contig carries that name)
struct SamNames {
  std::string blob;
  std::vector<uint64_t> off;
  int32_t starKey, emptyKey;
};
SamNames samNames(const HostIndex &ix);

}  // namespace gwa
