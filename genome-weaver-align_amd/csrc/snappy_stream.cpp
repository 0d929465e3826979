// snappy_stream.cpp -- `.snap` read files (R/ReadReaderFactory.java:126-151: a file whose name ends in
// ".snap" is read through org.xerial.snappy.SnappyInputStream).  snappy-java is not vendored with the
// reference (project/Build.scala:142-146 comments it out) and no snappy library exists
// in this image, so its published stream format and the Snappy block format are restated here:
//
//   SnappyOutputStream stream: the 8-byte magic 0x82 'S' 'N' 'A' 'P' 'P' 'Y' 0x00, a big-endian int32
//   version and a big-endian int32 minimum compatible version (both 1), then chunks, each a
//   big-endian int32 compressed length followed by one Snappy block; a stream without the magic is
//   one whole Snappy block (SnappyInputStream's fallback for data from Snappy.compress(byte[])).
//   Snappy block: the uncompressed length as a little-endian base-128 varint, then elements whose
//   tag byte's low 2 bits give the kind: 00 literal (length - 1 in the upper 6 bits, or 60..63 = that
//   many minus 59 following little-endian length bytes), 01 copy of 4 + ((tag >> 2) & 7) bytes at
//   offset ((tag >> 5) << 8) | next byte, 10 copy of (tag >> 2) + 1 bytes at a 2-byte offset, 11 the
//   same with a 4-byte offset.  Copies may overlap their output (offset < length: a repeat).
//
// SnapReader streams a file chunk by chunk (the pipeline's IO thread, pipeline.cpp);
// gwa_snappy_decompress decodes a whole buffer (the CLI's small-file paths, tests).
#include "snappy_stream.h"

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/gwa.h"

namespace gwa {

namespace {
const unsigned char kMagic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};

uint32_t be32(const unsigned char *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
}  // namespace

// one Snappy block [in, in + n) appended to out
void snappyBlock(const unsigned char *in, size_t n, std::string &out) {
  size_t p = 0;
  uint64_t ulen = 0;
  for (int shift = 0;; shift += 7) {
    // (Snappy's length is a uint32: at most 5 varint bytes)
    if (p >= n || shift > 28) throw std::runtime_error("corrupt snappy block (length)");
    const unsigned char b = in[p++];
    ulen |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) break;
  }
  // checked before the output is sized: no element expands more than 22x (a 3-byte copy of 64
  // bytes), so a larger claimed length is corrupt, not a reason to allocate it
  if (ulen > 0xFFFFFFFFull || ulen > 64 * (uint64_t)n + 64) throw std::runtime_error("corrupt snappy block (length)");
  const size_t base = out.size();
  out.resize(base + ulen);
  char *o = &out[0] + base;
  size_t w = 0;
  while (p < n) {
    const unsigned char tag = in[p++];
    size_t len, off = 0;
    switch (tag & 3) {
      case 0: {  // literal
        len = tag >> 2;
        if (len >= 60) {
          const int nb = (int)len - 59;
          if (p + nb > n) throw std::runtime_error("corrupt snappy block (literal length)");
          len = 0;
          for (int i = 0; i < nb; ++i) len |= (size_t)in[p + i] << (8 * i);
          p += nb;
        }
        len += 1;
        if (p + len > n || w + len > ulen) throw std::runtime_error("corrupt snappy block (literal)");
        memcpy(o + w, in + p, len);
        p += len;
        w += len;
        continue;
      }
      case 1:
        if (p + 1 > n) throw std::runtime_error("corrupt snappy block (copy)");
        len = 4 + ((tag >> 2) & 7);
        off = ((size_t)(tag >> 5) << 8) | in[p];
        p += 1;
        break;
      case 2:
        if (p + 2 > n) throw std::runtime_error("corrupt snappy block (copy)");
        len = (tag >> 2) + 1;
        off = (size_t)in[p] | ((size_t)in[p + 1] << 8);
        p += 2;
        break;
      default:
        if (p + 4 > n) throw std::runtime_error("corrupt snappy block (copy)");
        len = (tag >> 2) + 1;
        off = (size_t)in[p] | ((size_t)in[p + 1] << 8) | ((size_t)in[p + 2] << 16) | ((size_t)in[p + 3] << 24);
        p += 4;
        break;
    }
    if (off == 0 || off > w || w + len > ulen) throw std::runtime_error("corrupt snappy block (copy offset)");
    // byte by byte when the copy overlaps its own output (a repeated pattern)
    if (off >= len) memcpy(o + w, o + w - off, len);
    else for (size_t i = 0; i < len; ++i) o[w + i] = o[w - off + i];
    w += len;
  }
  if (w != ulen) throw std::runtime_error("corrupt snappy block (length mismatch)");
}

void snappyJavaDecode(const unsigned char *in, size_t n, std::string &out) {
  if (n < 16 || memcmp(in, kMagic, 8) != 0) {  // Snappy.compress(byte[]) output: one block
    snappyBlock(in, n, out);
    return;
  }
  size_t p = 16;
  while (p < n) {
    if (p + 4 > n) throw std::runtime_error("truncated snappy stream (chunk length)");
    const uint32_t c = be32(in + p);
    p += 4;
    if (p + c > n) throw std::runtime_error("truncated snappy stream (chunk)");
    snappyBlock(in + p, c, out);
    p += c;
  }
}

SnapReader::SnapReader(const char *path) : path_(path) {
  f_ = fopen(path, "rb");
  if (!f_) throw std::runtime_error(std::string("cannot open ") + path);
  if (fseeko(f_, 0, SEEK_END) == 0) {
    const off_t e = ftello(f_);
    fileSize_ = e > 0 ? (uint64_t)e : 0;
  }
  if (fseeko(f_, 0, SEEK_SET) != 0) throw std::runtime_error(std::string("cannot read ") + path);
  unsigned char h[16];
  const size_t got = fread(h, 1, 16, f_);
  if (got == 16 && memcmp(h, kMagic, 8) == 0) {
    stream_ = true;
  } else {  // no header: the whole file is one Snappy block
    std::string raw((const char *)h, got);
    char b[1 << 16];
    size_t r;
    while ((r = fread(b, 1, sizeof b, f_)) > 0) raw.append(b, r);
    snappyBlock((const unsigned char *)raw.data(), raw.size(), buf_);
    eof_ = true;
  }
}

SnapReader::~SnapReader() {
  if (f_) fclose(f_);
}

bool SnapReader::fill() {
  if (eof_) return false;
  unsigned char lb[4];
  const size_t g = fread(lb, 1, 4, f_);
  if (g == 0) {
    eof_ = true;
    return false;
  }
  if (g != 4) throw std::runtime_error(std::string("truncated snappy stream: ") + path_);
  const uint32_t c = be32(lb);
  const off_t at = ftello(f_);
  if (at < 0 || (uint64_t)at + c > fileSize_) throw std::runtime_error(std::string("truncated snappy stream: ") + path_);
  comp_.resize(c);
  if (c && fread(&comp_[0], 1, c, f_) != c) throw std::runtime_error(std::string("truncated snappy stream: ") + path_);
  buf_.clear();
  pos_ = 0;
  snappyBlock((const unsigned char *)comp_.data(), comp_.size(), buf_);
  return true;
}

size_t SnapReader::read(char *dst, size_t n) {
  size_t w = 0;
  while (w < n) {
    if (pos_ >= buf_.size()) {
      buf_.clear();
      pos_ = 0;
      if (!stream_ || !fill()) break;
      continue;
    }
    const size_t k = std::min(n - w, buf_.size() - pos_);
    memcpy(dst + w, buf_.data() + pos_, k);
    pos_ += k;
    w += k;
  }
  return w;
}

}  // namespace gwa

extern "C" int gwa_fail_message(const char *msg);

extern "C" int gwa_snappy_decompress(const uint8_t *in, uint64_t n, char **out, uint64_t *out_len) {
  try {
    std::string s;
    gwa::snappyJavaDecode(in, (size_t)n, s);
    *out = (char *)malloc(s.size() + 1);
    if (!*out) throw std::runtime_error("out of memory");
    memcpy(*out, s.data(), s.size());
    (*out)[s.size()] = 0;
    *out_len = s.size();
    return 0;
  } catch (std::exception &e) {
    return gwa_fail_message(e.what());
  }
}
