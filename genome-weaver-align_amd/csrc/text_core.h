// text_core.h -- byte-parallel read-text helpers shared by the encode kernels (batch_io.hip) and
// the host test harness (tests/hostcore): four text bytes per 32-bit word.
#pragma once
#include "gwa_layout.h"

namespace gwa {

// 0x80 in every byte of x that equals b, else 0 (exact: no carries cross bytes)
GWA_HD uint32_t bytesEq(uint32_t x, uint32_t b) {
  const uint32_t y = x ^ (b * 0x01010101u);
  const uint32_t t = (y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(t | y | 0x7F7F7F7Fu);
}

// ACGT.to3bitCode (A/ACGT.java:36-43) of the 4 bytes of x: A/a 0, C/c 1, G/g 2, T/t/U/u 3, else 4
GWA_HD uint32_t to3bit4(uint32_t x) {
  const uint32_t u = x & 0xDFDFDFDFu;  // clears bit 5 only: a letter and its lower case meet
  const uint32_t isA = bytesEq(u, 'A'), isC = bytesEq(u, 'C'), isG = bytesEq(u, 'G');
  const uint32_t isT = bytesEq(u, 'T') | bytesEq(u, 'U');
  const uint32_t any = (isA | isC | isG | isT) >> 7;  // 0x01 in every byte that is a base letter
  uint32_t c = 0x04040404u & ~(any * 0x07u);
  c |= (isC >> 7) | ((isG >> 7) * 2u) | ((isT >> 7) * 3u);
  return c;
}

}  // namespace gwa
