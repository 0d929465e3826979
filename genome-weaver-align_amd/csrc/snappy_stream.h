// snappy_stream.h -- snappy-java streams (`.snap` read files, snappy_stream.cpp)
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>

namespace gwa {

// one Snappy block appended to out (throws on corrupt input)
void snappyBlock(const unsigned char *in, size_t n, std::string &out);
// a whole SnappyOutputStream stream (or one bare Snappy block) appended to out
void snappyJavaDecode(const unsigned char *in, size_t n, std::string &out);

// sequential reader of a `.snap` file: read() returns the decompressed bytes in order, 0 at the end
class SnapReader {
 public:
  explicit SnapReader(const char *path);
  ~SnapReader();
  SnapReader(const SnapReader &) = delete;
  SnapReader &operator=(const SnapReader &) = delete;
  size_t read(char *dst, size_t n);

 private:
  bool fill();
  std::string path_, comp_, buf_;
  FILE *f_ = nullptr;
  size_t pos_ = 0;
  uint64_t fileSize_ = 0;  // (a chunk length is checked against the bytes left before any allocation)
  bool stream_ = false, eof_ = false;
};

}  // namespace gwa
