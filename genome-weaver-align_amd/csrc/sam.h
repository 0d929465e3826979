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

}  // namespace gwa
