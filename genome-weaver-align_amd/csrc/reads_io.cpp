// reads_io.cpp -- the align CLI's read-file parser on the host, native: FASTA / FASTQ text ->
// gwa_reads_t SoA blobs (include/gwa.h gwa_reads_parse).
//
// The reference reads files through utgb's FastqReader / its FASTA reader
// (R/ReadReaderFactory.java:126-151), which are not vendored (read-name parsing is
// parity unpinned).  The record rules are therefore this repository's own, stated once in
// gwa_cli.read_fasta / read_fastq (Python, text mode with universal newlines) and restated here
// byte for byte (tests/test_cli.py compares the two):
//   lines end at "\n", "\r\n" or "\r";
//   FASTA: a '>' line starts a record named by the first whitespace-separated token of the rest of
//          the line ("" if none); the following lines, each stripped of surrounding whitespace,
//          are concatenated into the sequence; lines before the first header are ignored;
//   FASTQ: 4-line records; blank lines where a header is expected are skipped; the header must
//          start with '@', the third line with '+', and the quality must be as long as the sequence.
// Whitespace is the ASCII set Python's str.split() / str.strip() use: " \t\n\r\v\f\x1c\x1d\x1e\x1f".
#include <immintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/gwa.h"

namespace {

struct Buf {
  std::string name, seq, qual;
  std::vector<uint64_t> nameOff{0}, seqOff{0}, qualOff{0};
};

inline bool isWs(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r') || (c >= 0x1c && c <= 0x1f); }

// one line [b, e) of text[pos, len); returns false when no complete line is available (the
// terminator is missing, or is a "\r" at the buffer end that a "\n" may follow, unless final)
struct Lines {
  const char *t;
  uint64_t len, pos;
  bool final;
  bool next(uint64_t *b, uint64_t *e) {
    if (pos >= len) return false;
    // the first "\n" or "\r" from pos: memchr over growing windows, so a text with "\r" line ends
    // only is scanned once (a "\n" search to the end of the text per line would be quadratic)
    uint64_t i = pos;
    for (uint64_t w = 256;; w *= 2) {
      const uint64_t end = std::min<uint64_t>(len, i + w);
      const char *nl = (const char *)memchr(t + i, '\n', end - i);
      const uint64_t lim = nl ? (uint64_t)(nl - t) : end;
      if (const char *cr = (const char *)memchr(t + i, '\r', lim - i)) { i = (uint64_t)(cr - t); break; }
      if (nl || end == len) { i = lim; break; }
      i = end;
    }
    if (i == len) {
      if (!final) return false;
      *b = pos; *e = len; pos = len;
      return true;
    }
    uint64_t nx = i + 1;
    if (t[i] == '\r') {
      if (nx == len && !final) return false;
      if (nx < len && t[nx] == '\n') ++nx;
    }
    *b = pos; *e = i; pos = nx;
    return true;
  }
};

void firstToken(const char *t, uint64_t b, uint64_t e, std::string &out) {
  while (b < e && isWs((unsigned char)t[b])) ++b;
  uint64_t x = b;
  while (x < e && !isWs((unsigned char)t[x])) ++x;
  out.append(t + b, x - b);
}

std::string excerpt(const char *t, uint64_t b, uint64_t e) {
  return std::string(t + b, (size_t)std::min<uint64_t>(e - b, 80));
}

// FASTA: records complete up to the last header when !final
uint64_t parseFasta(const char *t, uint64_t len, bool final, Buf &o) {
  Lines L{t, len, 0, final};
  uint64_t b, e, done = 0;
  bool inRec = false;
  uint64_t recStart = 0;
  while (true) {
    const uint64_t lineStart = L.pos;
    if (!L.next(&b, &e)) break;
    if (e > b && t[b] == '>') {
      if (inRec) {  // close the previous record
        o.nameOff.push_back(o.name.size());
        o.seqOff.push_back(o.seq.size());
      }
      done = lineStart;  // (text before the first header is ignored, i.e. consumed)
      inRec = true;
      recStart = lineStart;
      firstToken(t, b + 1, e, o.name);
    } else if (inRec) {
      while (b < e && isWs((unsigned char)t[b])) ++b;
      while (e > b && isWs((unsigned char)t[e - 1])) --e;
      o.seq.append(t + b, e - b);
    } else {
      done = L.pos;
    }
  }
  if (inRec) {
    if (final) {
      o.nameOff.push_back(o.name.size());
      o.seqOff.push_back(o.seq.size());
      done = len;
    } else {  // the last record may continue in the next chunk: drop it
      o.name.resize(o.nameOff.back());
      o.seq.resize(o.seqOff.back());
      done = recStart;
    }
  } else if (final) {
    done = len;
  }
  return done;
}

uint64_t parseFastq(const char *t, uint64_t len, bool final, Buf &o) {
  Lines L{t, len, 0, final};
  uint64_t done = 0;
  while (true) {
    uint64_t hb, he;
    const uint64_t recStart = L.pos;
    if (!L.next(&hb, &he)) break;
    if (he == hb) { done = L.pos; continue; }  // blank line where a header is expected
    if (t[hb] != '@') throw std::runtime_error("malformed FASTQ header: " + excerpt(t, hb, he));
    uint64_t sb = 0, se = 0, pb = 0, pe = 0, qb = 0, qe = 0;
    const bool hs = L.next(&sb, &se), hp = hs && L.next(&pb, &pe), hq = hp && L.next(&qb, &qe);
    if (!hq && !final) { L.pos = recStart; break; }
    // at the end of the text a missing line reads as "" (Python readline)
    if (!hs) { sb = se = len; }
    if (!hp) { pb = pe = len; }
    if (!hq) { qb = qe = len; }
    if (pe == pb || t[pb] != '+' || qe - qb != se - sb)
      throw std::runtime_error("malformed FASTQ record: " + excerpt(t, hb, he));
    firstToken(t, hb + 1, he, o.name);
    o.seq.append(t + sb, se - sb);
    o.qual.append(t + qb, qe - qb);
    o.nameOff.push_back(o.name.size());
    o.seqOff.push_back(o.seq.size());
    o.qualOff.push_back(o.qual.size());
    done = L.pos;
  }
  return done;
}

}  // namespace

namespace gwa {
// Positions of every '\n' in t[a, b), appended in order (SSE2: 16 bytes per compare).
void newlinePositions(const char *t, uint64_t a, uint64_t b, std::vector<uint64_t> &out) {
  uint64_t i = a;
  const __m128i nl = _mm_set1_epi8('\n');
  for (; i < b && (i & 15); ++i)
    if (t[i] == '\n') out.push_back(i);
  for (; i + 16 <= b; i += 16) {
    unsigned m = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(t + i)), nl));
    while (m) {
      out.push_back(i + (uint64_t)__builtin_ctz(m));
      m &= m - 1;
    }
  }
  for (; i < b; ++i)
    if (t[i] == '\n') out.push_back(i);
}

// Count of '\n' in t[a, b) and whether the range holds a "\n\n" or a '\r'.  AVX2 (32 bytes per
// compare) where the CPU has it, a byte loop otherwise.
__attribute__((target("avx2,popcnt"))) static void newlineCountAvx2(const char *t, uint64_t a, uint64_t b, uint64_t *count,
                                                                     bool *blank, bool *cr) {
  uint64_t c = 0;
  bool bl = false, r = false;
  uint64_t i = a;
  char prev = i > 0 ? t[i - 1] : 0;
  for (; i < b && (i & 31); ++i) {
    c += t[i] == '\n';
    bl |= t[i] == '\n' && prev == '\n';
    r |= t[i] == '\r';
    prev = t[i];
  }
  const __m256i nl = _mm256_set1_epi8('\n'), crv = _mm256_set1_epi8('\r');
  uint32_t carry = prev == '\n' ? 1u : 0u;  // the byte before the block was a newline
  uint32_t blm = 0, crm = 0;
  for (; i + 32 <= b; i += 32) {
    const __m256i v = _mm256_loadu_si256((const __m256i *)(t + i));
    const uint32_t m = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, nl));
    c += (uint64_t)_mm_popcnt_u32(m);
    blm |= m & ((m << 1) | carry);
    crm |= (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, crv));
    carry = m >> 31;
  }
  bl |= blm != 0;
  r |= crm != 0;
  prev = i > a ? t[i - 1] : (a > 0 ? t[a - 1] : 0);
  for (; i < b; ++i) {
    c += t[i] == '\n';
    bl |= t[i] == '\n' && prev == '\n';
    r |= t[i] == '\r';
    prev = t[i];
  }
  *count = c;
  *blank = bl;
  *cr = r;
}

static void newlineCountScalar(const char *t, uint64_t a, uint64_t b, uint64_t *count, bool *blank, bool *cr) {
  uint64_t c = 0;
  bool bl = false, r = false;
  char prev = a > 0 ? t[a - 1] : 0;
  for (uint64_t i = a; i < b; ++i) {
    c += t[i] == '\n';
    bl |= t[i] == '\n' && prev == '\n';
    r |= t[i] == '\r';
    prev = t[i];
  }
  *count = c;
  *blank = bl;
  *cr = r;
}

void newlineCount(const char *t, uint64_t a, uint64_t b, uint64_t *count, bool *blank, bool *cr) {
  static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("popcnt");
  if (avx2) newlineCountAvx2(t, a, b, count, blank, cr);
  else newlineCountScalar(t, a, b, count, blank, cr);
}

// Record starts of t[a, b) for text without blank lines or '\r' (every record = 4 lines): the line
// after the g-th newline of the text (g counted from 0 over the whole text, g0 = newlines before a)
// starts record (g + 1) / 4 when (g + 1) % 4 == 0; starts[rec] = its offset, for rec < cap.
template <bool Avx2>
__attribute__((target("avx2,popcnt,bmi"))) static void recordStartsImpl(const char *t, uint64_t a, uint64_t b, uint64_t g0,
                                                                          uint64_t *starts, uint64_t cap) {
  uint64_t g = g0;
  uint64_t i = a;
  auto hit = [&](uint64_t pos) {
    if (((g + 1) & 3) == 0 && (g + 1) / 4 < cap) starts[(g + 1) / 4] = pos + 1;
    ++g;
  };
  if (Avx2) {
    for (; i < b && (i & 31); ++i)
      if (t[i] == '\n') hit(i);
    const __m256i nl = _mm256_set1_epi8('\n');
    for (; i + 32 <= b; i += 32) {
      uint32_t m = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_loadu_si256((const __m256i *)(t + i)), nl));
      while (m) {
        hit(i + (uint64_t)__builtin_ctz(m));
        m &= m - 1;
      }
    }
  }
  for (; i < b; ++i)
    if (t[i] == '\n') hit(i);
}

void recordStartsFromNewlines(const char *t, uint64_t a, uint64_t b, uint64_t g0, uint64_t *starts, uint64_t cap) {
  static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("popcnt");
  if (avx2) recordStartsImpl<true>(t, a, b, g0, starts, cap);
  else recordStartsImpl<false>(t, a, b, g0, starts, cap);
}

// FASTQ framing over precomputed newline positions (text without '\r'): the same records as
// frameRecords -- blank lines where a header is expected are skipped, a record is 4 lines, the last
// line of a final text may lack its terminator.  nl = the '\n' offsets of t[0, len) in order.
uint64_t frameFastqLines(const char *t, uint64_t len, const std::vector<uint64_t> &nl, bool final, uint64_t maxRec,
                         uint64_t *nRec, std::vector<uint64_t> *starts) {
  (void)t;
  const size_t L = nl.size();
  // line j is [S(j), E(j)); after the last '\n' a final text has one more line when bytes remain
  auto S = [&](size_t j) -> uint64_t { return j == 0 ? 0 : nl[j - 1] + 1; };
  auto E = [&](size_t j) -> uint64_t { return j < L ? nl[j] : len; };
  const size_t lines = L + ((final && S(L) < len) ? 1 : 0);
  auto nextStart = [&](size_t j) -> uint64_t { return j < L ? nl[j] + 1 : len; };  // after line j
  uint64_t done = 0, n = 0;
  size_t j = 0;
  while (n < maxRec && j < lines) {
    if (E(j) == S(j)) {  // blank line where a header is expected
      done = nextStart(j);
      ++j;
      continue;
    }
    if (j + 3 < lines) {
      if (starts) starts->push_back(S(j));
      ++n;
      j += 4;
      done = nextStart(j - 1);
    } else if (final) {  // the missing lines of the last record read as ""
      if (starts) starts->push_back(S(j));
      ++n;
      j = lines;
      done = len;
    } else {
      break;
    }
  }
  if (final && n < maxRec && j >= lines) done = len;
  *nRec = n;
  return done;
}

// Record framing for the pipeline reader: the end offset of the first `maxRec` complete records of
// text[0, len) (fewer when the text ends first) under the same rules as parseFasta / parseFastq, and
// their count; for FASTQ optionally the offset of each record's header line (`starts`, appended).  Only line ends are scanned (memchr); the parse itself runs later, in parallel, on each
// framed slice.  Malformed records are left to that parse to report.
uint64_t frameRecords(const char *t, uint64_t len, int format, bool final, uint64_t maxRec, uint64_t *nRec,
                      std::vector<uint64_t> *starts) {
  Lines L{t, len, 0, final};
  uint64_t done = 0, n = 0, b, e;
  if (format == 1) {
    while (n < maxRec) {
      const uint64_t recStart = L.pos;
      if (!L.next(&b, &e)) break;
      if (e == b) { done = L.pos; continue; }
      uint64_t x0, x1;
      const bool ok = L.next(&x0, &x1) && L.next(&x0, &x1) && L.next(&x0, &x1);
      if (!ok && !final) { L.pos = recStart; break; }
      if (starts) starts->push_back(b);
      ++n;
      done = L.pos;
    }
  } else {
    bool inRec = false;
    while (true) {
      const uint64_t lineStart = L.pos;
      if (!L.next(&b, &e)) break;
      if (e > b && t[b] == '>') {
        if (inRec && ++n == maxRec) { done = lineStart; inRec = false; break; }
        inRec = true;
        done = lineStart;
      } else if (!inRec) {
        done = L.pos;
      }
    }
    if (inRec && final) { ++n; done = len; }
    if (!inRec && n < maxRec && final) done = len;
  }
  *nRec = n;
  return done;
}
}  // namespace gwa

extern "C" int gwa_fail_message(const char *msg);  // gwa_api.cpp: sets gwa_last_error, returns -1

extern "C" int gwa_reads_parse(const char *text, uint64_t len, int format, int final, gwa_read_buf_t *out,
                               uint64_t *consumed) {
  try {
    if (format != 0 && format != 1) throw std::runtime_error("read format must be 0 (FASTA) or 1 (FASTQ)");
    auto *b = new Buf();
    // FASTQ is about 45 % bases and 45 % qualities; FASTA mostly bases (one allocation each)
    b->seq.reserve(format == 1 ? len / 2 + 64 : len + 64);
    if (format == 1) b->qual.reserve(len / 2 + 64);
    b->name.reserve(len / 8 + 64);
    uint64_t done = 0;
    try {
      done = format == 0 ? parseFasta(text, len, final != 0, *b) : parseFastq(text, len, final != 0, *b);
    } catch (...) {
      delete b;
      throw;
    }
    out->priv = b;
    out->reads.n = (uint32_t)(b->nameOff.size() - 1);
    out->reads.name = b->name.data();
    out->reads.seq = b->seq.data();
    out->reads.name_off = b->nameOff.data();
    out->reads.seq_off = b->seqOff.data();
    out->reads.qual = format == 1 ? b->qual.data() : nullptr;
    out->reads.qual_off = format == 1 ? b->qualOff.data() : nullptr;
    out->reads.qual_null = nullptr;
    *consumed = done;
    return 0;
  } catch (std::exception &e) {
    return gwa_fail_message(e.what());
  }
}

extern "C" void gwa_reads_free(gwa_read_buf_t *b) {
  if (!b || !b->priv) return;
  delete (Buf *)b->priv;
  b->priv = nullptr;
  b->reads.n = 0;
}
