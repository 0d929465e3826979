// jsem.h -- Java-semantics helpers for the CPU oracle (TEST INFRASTRUCTURE ONLY).
//
// The oracle restates the reference's Java `align` path literally; every place
// where Java arithmetic differs from C++ goes through these helpers
// (SURVEY.md Appendix A):
//   * long shift counts are masked to 6 bits (JLS 15.19), int to 5 bits;
//   * `>>>` is a logical shift;
//   * int arithmetic wraps; `(byte)` casts truncate to int8.
// Used by the reference at e.g. StaircaseFilter.java:96,100,
// QueryMask.java:81,92,94, BitVector.java:111-114.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>

namespace orc {

// Java `long << s`
static inline int64_t jshl(int64_t x, int64_t s) { return (int64_t)((uint64_t)x << (s & 63)); }
// Java `long >>> s`
static inline int64_t jushr(int64_t x, int64_t s) { return (int64_t)((uint64_t)x >> (s & 63)); }
// Java `long >> s`
static inline int64_t jshr(int64_t x, int64_t s) { return x >> (s & 63); }
// Java `int << s`
static inline int32_t jishl(int32_t x, int32_t s) { return (int32_t)((uint32_t)x << (s & 31)); }
// Java `int >>> s`
static inline int32_t jiushr(int32_t x, int32_t s) { return (int32_t)((uint32_t)x >> (s & 31)); }
// Java `(byte) x`
static inline int8_t jbyte(int32_t x) { return (int8_t)(uint8_t)(uint32_t)x; }
// Java Long.bitCount
static inline int jbitcount(int64_t x) { return __builtin_popcountll((uint64_t)x); }

// Any Java exception that would abort the reference run (the reference
// rethrows per-read exceptions: BidirectionalSuffixFilter.java:264-267).
struct JavaException : std::runtime_error {
  explicit JavaException(const std::string &m) : std::runtime_error(m) {}
};

}  // namespace orc
