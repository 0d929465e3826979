// sam.h -- host-side AlignmentRecord conversion + SAM text
#pragma once
#include <string>

#include "host_index.h"

namespace gwa {

struct ReadText {
  const char *name;
  size_t nameLen;
  const char *seq;
  size_t seqLen;
  const char *qual;  // nullptr == no quality (Java null -> "*")
  size_t qualLen;
};

std::string samHeader(const HostIndex &ix);
int formatChain(const HostIndex &ix, const ReadText &rt, const OutHit *hits, const uint16_t *cig, int head, std::string &out);
void formatUnmapped(const ReadText &rt, std::string &out);
// every reported chain of a mapped read (OutHeader: hits and CIGAR ops at hitOff / cigOff, chains
// back to back); 0, or -1 where the reference would throw
int formatRead(const HostIndex &ix, const ReadText &rt, const OutHeader &h, const OutHit *hits, const uint16_t *cig,
               std::string &out);

}  // namespace gwa
