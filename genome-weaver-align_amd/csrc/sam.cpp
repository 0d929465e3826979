// sam.cpp -- the SAM header (SequenceBoundary.toSAMHeader, A/SequenceBoundary.java:81-87) and the
// contig-name table the device SAM writer reads (the records themselves: sam_core.h, batch_io.hip).
#include "sam.h"

#include <algorithm>
#include <cstring>

namespace gwa {

std::string samHeader(const HostIndex &ix) {
  std::string h;
  for (size_t i = 0; i < ix.names.size(); ++i) {
    h += "@SQ\tSN:";
    h += ix.names[i];
    h += "\tLN:";
    h += std::to_string(ix.lengths[i]);
    h += '\n';
  }
  return h;
}

SamNames samNames(const HostIndex &ix) {
  SamNames o;
  o.off.push_back(0);
  o.starKey = -3;
  o.emptyKey = -2;
  for (size_t i = 0; i < ix.names.size(); ++i) {
    o.blob += ix.names[i];
    o.off.push_back(o.blob.size());
    if (ix.names[i] == "*") o.starKey = ix.chrRank[i];
    if (ix.names[i].empty()) o.emptyKey = ix.chrRank[i];
  }
  return o;
}

}  // namespace gwa
