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
    // the next "\n" (memchr), unless a "\r" comes first
    const char *nl = (const char *)memchr(t + pos, '\n', len - pos);
    uint64_t i = nl ? (uint64_t)(nl - t) : len;
    if (const char *cr = (const char *)memchr(t + pos, '\r', i - pos)) i = (uint64_t)(cr - t);
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
// Record framing for the pipeline reader: the end offset of the first `maxRec` complete records of
// text[0, len) (fewer when the text ends first) under the same rules as parseFasta / parseFastq, and
// their count.  Only line ends are scanned (memchr); the parse itself runs later, in parallel, on each
// framed slice.  Malformed records are left to that parse to report.
uint64_t frameRecords(const char *t, uint64_t len, int format, bool final, uint64_t maxRec, uint64_t *nRec) {
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
