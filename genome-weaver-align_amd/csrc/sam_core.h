// sam_core.h -- the SAM records of one read, written by one GPU lane (or by the host test harness):
//   AlignmentRecord.convert   (R/AlignmentRecord.java:181-276)
//   AlignmentRecord.toSAMLine (R/AlignmentRecord.java:109-170)
//   SAMOutput.emit            (A/SAMOutput.java:73-82)
// The same function measures a record (SamOut with p == nullptr counts bytes) and writes it, so the
// device formats a batch in two passes: lengths, an exclusive scan, then every read's text at its
// offset (sam_format.hip).  SAM flag values follow the SAM spec (utgb SAMReadFlag is unvendored;
// SURVEY.md §8c).
#pragma once
#include "gwa_layout.h"

namespace gwa {

// Read text and contig names as the formatter reads them (device or host memory).  Read r's name
// is name[nameB[r], nameE[r]) and its quality qual[qualB[r], qualE[r]): SoA blobs (nameE = nameB + 1)
// or the fields of FASTQ records inside the file text itself.
struct SamText {
  const char *name;
  const uint64_t *nameB, *nameE;
  const char *qual;          // nullptr: no qualities (SAM "*", as for FASTA input)
  const uint64_t *qualB, *qualE;
  const uint8_t *qualNull;   // nullptr, or per read: nonzero = this read's quality is null ("*")
  const uint8_t *codes;      // ReadsView: the read as codes 0..4 (spaces skipped)
  const uint32_t *codeOff, *codeLen;
  const char *ctg;           // contig names
  const uint64_t *ctgOff;    // nContig + 1
  const int32_t *chrKey;     // per contig: equal names <=> equal keys (String.equals)
  int32_t starKey, emptyKey; // the keys of the names "*" and "" (a contig may be called that)
};

// byte sink: counts when p == nullptr
struct SamOut {
  char *p;
  uint64_t n;
  GWA_HD void ch(char c) {
    if (p) p[n] = c;
    ++n;
  }
  // Text copies run 16 bytes per pass with the 16 loads issued before any store: a record's name,
  // sequence and quality (~250 B) then wait on memory ~16 times, not once per byte (the SAM writer is
  // latency-bound: a few workgroups per CU, each lane formatting one record)
  GWA_HD void bytes(const char *s, uint64_t len) {
    if (p) {
      for (uint64_t i = 0; i < len; i += 16) {
        char b[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) b[k] = i + k < len ? s[i + k] : 0;
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (i + k < len) p[n + i + k] = b[k];
      }
    }
    n += len;
  }
  template <unsigned long L>
  GWA_HD void lit(const char (&s)[L]) {  // a string literal (without its terminating 0)
    bytes(s, L - 1);
  }
  GWA_HD void num(int64_t v) {  // Integer.toString
    // the digits, least significant first, packed 8 per register (no runtime-indexed array, which
    // would live in scratch memory on the device)
    const bool neg = v < 0;
    uint64_t u = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    uint64_t d0 = 0, d1 = 0, d2 = 0;
    int k = 0;
    do {
      const uint64_t q = u / 10, dig = u - q * 10;
      if (k < 8) d0 |= dig << (8 * k);
      else if (k < 16) d1 |= dig << (8 * (k - 8));
      else d2 |= dig << (8 * (k - 16));
      ++k;
      u = q;
    } while (u);
    if (neg) ch('-');
    for (int i = k - 1; i >= 0; --i) {
      const uint64_t w = i < 8 ? d0 : i < 16 ? d1 : d2;
      ch((char)('0' + (int)((w >> (8 * (i & 7))) & 0xFF)));
    }
  }
};

// Read.getQual(0) == null for read r: the batch has no qualities or this read has none
GWA_HD bool qualAbsent(const SamText &t, uint32_t r) { return t.qual == nullptr || (t.qualNull && t.qualNull[r]); }

namespace samfmt {

constexpr char kSym[5] = {'A', 'C', 'G', 'T', 'N'};
// kSym[x] as a shift of one packed constant (a table lookup is a memory load per base on the device)
GWA_HD char sym(unsigned x) { return (char)((0x4E54474341ULL >> (8 * x)) & 0xFF); }
constexpr char kOp[8] = {'M', 'I', 'D', 'N', 'S', 'H', 'P', 'X'};

GWA_HD char stateCh(int numHits) { return numHits > 0 ? (numHits == 1 ? 'U' : 'R') : 'N'; }

// CIGAR of a record as items: elements copied from a hit's list keep that list as it is (a fresh
// CIGAR built from an element list), later add() calls merge with the last element
// (CIGAR.add, A/CIGAR.java:158-170)
struct CigSpec {
  const uint16_t *a;  // first element list (raw), or nullptr
  int na;
  int preS;           // -1, or add(S, preS) first (on an empty CIGAR)
  int postS;          // -1, or add(S, postS) after list a
  const uint16_t *b;  // elements added one by one after list a (merged), or nullptr
  int nb;
};

struct CigEmit {
  SamOut &o;
  int pt = -1;
  int64_t pl = 0;
  GWA_HD explicit CigEmit(SamOut &o_) : o(o_) {}
  GWA_HD void flush() {
    if (pt >= 0) {
      o.num(pl);
      o.ch(kOp[pt & 7]);
    }
  }
  GWA_HD void raw(int t, int64_t l) {
    flush();
    pt = t;
    pl = l;
  }
  GWA_HD void add(int t, int64_t l) {
    if (pt == t) pl += l;
    else raw(t, l);
  }
};

GWA_HD void emitCigar(SamOut &o, const CigSpec &c) {
  CigEmit e(o);
  if (c.preS >= 0) e.add(4, c.preS);
  for (int i = 0; i < c.na; ++i) e.raw(c.a[i] & 7, c.a[i] >> 3);
  if (c.postS >= 0) e.add(4, c.postS);
  for (int i = 0; i < c.nb; ++i) e.add(c.b[i] & 7, c.b[i] >> 3);
  e.flush();
}

// one AlignmentRecord to print
struct Rec {
  int chr, strand, start, end, nm, numBestHits;
  CigSpec cig;
  int seqA, seqB;       // SEQ = the strand-oriented query [seqA, seqB)
  int qualA, qualB;     // QUAL = the strand-oriented quality [qualA, qualB)
  int stateHead, stateSelf;  // XP = ReadHit.getAlignmentState over the chain from stateHead
  bool hasSplit;
};

struct Ctx {
  const SamText &t;
  uint32_t r;
  const OutHit *hits;   // the read's hits (chain indices are relative to this)
  int m;
  int strand;           // of the chain head: orientation of SEQ / QUAL
  bool qualNull;
  uint64_t q0, qn;      // quality text [q0, q0 + qn)
  bool npe = false;     // the reference would throw
};

GWA_HD int32_t nameKey(const Ctx &cx, int chr) {
  if (chr >= 0) return cx.t.chrKey[chr];
  if (chr == CHR_STAR) return cx.t.starKey;
  if (chr == CHR_EMPTY) return cx.t.emptyKey;
  return -2147483647 - 1;
}

GWA_HD void chrName(SamOut &o, Ctx &cx, int chr) {
  if (chr >= 0) o.bytes(cx.t.ctg + cx.t.ctgOff[chr], cx.t.ctgOff[chr + 1] - cx.t.ctgOff[chr]);
  else if (chr == CHR_STAR) o.ch('*');
  else if (chr == CHR_EMPTY) {
  } else cx.npe = true;  // null chr
}

// (16 positions per pass, loads first: SamOut::bytes)
GWA_HD void emitSeq(SamOut &o, const Ctx &cx, int a, int b) {
  const uint8_t *c = cx.t.codes + cx.t.codeOff[cx.r];
  for (int j0 = a; j0 < b; j0 += 16) {
    uint8_t x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int j = j0 + k;
      x[k] = j < b ? (cx.strand == 0 ? c[j] : c[cx.m - 1 - j]) : 0;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (j0 + k < b) o.ch(sym(cx.strand == 0 ? x[k] : (x[k] < 4 ? 3 - x[k] : 4)));
  }
}

GWA_HD void emitQual(SamOut &o, const Ctx &cx, int a, int b) {
  if (cx.qualNull) {
    o.ch('*');
    return;
  }
  const char *q = cx.t.qual + cx.q0;
  for (int j0 = a; j0 < b; j0 += 16) {
    char x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int j = j0 + k;
      x[k] = j < b ? (cx.strand == 0 ? q[j] : q[cx.qn - 1 - j]) : 0;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (j0 + k < b) o.ch(x[k]);
  }
}

GWA_HD void emitState(SamOut &o, const Ctx &cx, int head, int self) {
  for (int t = head; t >= 0; t = cx.hits[t].next) {
    const char c = stateCh(cx.hits[t].numHits);
    o.ch(t == self ? c : (char)(c - 'A' + 'a'));
  }
}

// AlignmentRecord.toSAMLine (R/AlignmentRecord.java:109-170) of one record; returns the
// eachFragmentIsMapped value handed on to the split record's line
GWA_HD bool lineOne(SamOut &o, Ctx &cx, const Rec &r, const Rec *split, bool hasSegments, bool isFirst, bool eachMapped) {
  int flag = 0;
  if (hasSegments) flag |= 0x1;
  if (r.strand == 1) flag |= 0x10;
  if (isFirst) {
    flag |= 0x40;
    if (r.numBestHits <= 0 || (split && split->numBestHits <= 0)) eachMapped = false;
  } else if (!split) {
    flag |= 0x80;
  }
  if (eachMapped) flag |= 0x2;
  if (r.numBestHits <= 0) flag |= 0x4;
  if (split && split->numBestHits <= 0) flag |= 0x8;
  o.bytes(cx.t.name + cx.t.nameB[cx.r], cx.t.nameE[cx.r] - cx.t.nameB[cx.r]);
  o.ch('\t');
  o.num(flag);
  o.ch('\t');
  chrName(o, cx, r.chr);
  o.ch('\t');
  o.num(r.start);
  o.lit("\t1\t");  // MAPQ column = AlignmentRecord.score, always 1 (:199)
  emitCigar(o, r.cig);
  if (!split) {
    o.lit("\t*\t0\t0");
  } else {
    const int32_t ck = nameKey(cx, r.chr), sk = nameKey(cx, split->chr);
    if (r.chr != CHR_NULL && split->chr != CHR_NULL && ck != cx.t.starKey && ck == sk) {
      o.lit("\t=");
    } else {
      o.ch('\t');
      chrName(o, cx, split->chr);
    }
    o.ch('\t');
    o.num(split->start);
    o.ch('\t');
    o.num((int64_t)split->end - r.start);
  }
  o.ch('\t');
  emitSeq(o, cx, r.seqA, r.seqB);
  o.ch('\t');
  emitQual(o, cx, r.qualA, r.qualB);
  if (r.numBestHits > 0) {
    if (r.nm >= 0) {
      o.lit("\tNM:i:");
      o.num(r.nm);
    }
    o.lit("\tXP:Z:");
    emitState(o, cx, r.stateHead, r.stateSelf);
    o.lit("\tX0:i:");
    o.num(r.numBestHits);
  }
  return eachMapped;
}

// a record and, when it has one, its split record on the next line
GWA_HD void emitRec(SamOut &o, Ctx &cx, const Rec &r, const Rec *split, bool hasSegments) {
  const bool em = lineOne(o, cx, r, split, hasSegments, true, true);
  if (split) {
    o.ch('\n');
    lineOne(o, cx, *split, nullptr, hasSegments, false, em);
  }
}

}  // namespace samfmt

// One reported ReadHit chain (head = index into hits) -> SAM text, '\n' terminated.  Returns 0, or
// -1 where the reference would throw (the run aborts, S/BidirectionalSuffixFilter.java:264-267).
GWA_HD int samChain(SamOut &o, const SamText &t, uint32_t r, const OutHit *hits, const uint16_t *cig, int head) {
  using namespace samfmt;
  const OutHit &h = hits[head];
  Ctx cx{t, r, hits, (int)t.codeLen[r], h.strand != 0 ? 1 : 0, qualAbsent(t, r), 0, 0};
  if (!cx.qualNull) {
    cx.q0 = t.qualB[r];
    cx.qn = t.qualE[r] - t.qualB[r];
  }
  const int m = cx.m;
  const int fullQual = cx.qualNull ? 0 : (int)cx.qn;
  Rec rec{};
  rec.cig = CigSpec{cig + h.cigarOff, (int)h.cigarLen, -1, -1, nullptr, 0};
  rec.seqA = 0; rec.seqB = m;
  rec.qualA = 0; rec.qualB = fullQual;
  rec.stateHead = head;
  rec.stateSelf = head;
  if (h.next < 0) {
    rec.chr = h.chr; rec.strand = h.strand; rec.start = h.pos; rec.end = h.pos + h.matchLength; rec.nm = h.diff;
    rec.numBestHits = h.numHits;
    emitRec(o, cx, rec, nullptr, false);
  } else {
    // the head and its first split are converted; later fragments of a longer chain are dropped
    // (R/AlignmentRecord.java:201-206 reads hit.nextSplit only), but still named in XP
    const OutHit &s = hits[h.next];
    const int numHits = h.numHits;
    const int qualLen = !cx.qualNull ? (int)cx.qn : h.matchLength;
    const bool hU = h.numHits == 1, sU = s.numHits == 1;
    // substrings taken by convert (:187-196): a bad range is a Java exception
    auto bad = [](int a, int b, int size) { return a < 0 || b > size || a > b; };
    const int b1 = qualLen < h.matchLength ? qualLen : h.matchLength;
    const int b2 = qualLen < m ? qualLen : m;
    if (bad(h.qStart, h.qEnd, m) || bad(s.qStart, s.qEnd, m)) return -1;
    if (!cx.qualNull && (bad(0, b1, (int)cx.qn) || bad(b1, b2, (int)cx.qn))) return -1;
    if (hU) {
      if (sU) {
        if (h.chr == CHR_NULL) return -1;
        bool same = (h.chr >= 0 && s.chr >= 0) ? t.chrKey[h.chr] == t.chrKey[s.chr] : h.chr == s.chr;
        if (s.chr == CHR_NULL) same = false;
        if (same) {
          Rec srec{};
          rec.chr = h.chr; rec.strand = h.strand; rec.start = h.pos; rec.end = h.pos + h.matchLength; rec.nm = h.diff;
          rec.seqA = h.qStart; rec.seqB = h.qEnd; rec.qualA = 0; rec.qualB = b1; rec.numBestHits = 1;
          srec.chr = s.chr; srec.strand = s.strand; srec.start = s.pos; srec.end = s.pos + s.matchLength; srec.nm = s.diff;
          srec.cig = CigSpec{cig + s.cigarOff, (int)s.cigarLen, -1, -1, nullptr, 0};
          srec.seqA = s.qStart; srec.seqB = s.qEnd; srec.qualA = b1; srec.qualB = b2; srec.numBestHits = 1;
          srec.stateHead = head;
          srec.stateSelf = h.next;
          if (cx.qualNull) { rec.qualB = srec.qualB = 0; }
          emitRec(o, cx, rec, &srec, true);
        } else if (h.matchLength >= s.matchLength) {
          rec.cig.postS = s.matchLength;
          rec.chr = h.chr; rec.strand = h.strand; rec.start = h.pos; rec.end = h.pos + m; rec.nm = h.diff;
          rec.numBestHits = numHits;
          emitRec(o, cx, rec, nullptr, false);
        } else {
          if (s.chr == CHR_NULL) return -1;
          rec.cig.b = cig + s.cigarOff;
          rec.cig.nb = (int)s.cigarLen;
          rec.chr = s.chr; rec.strand = s.strand; rec.start = s.pos - h.matchLength; rec.end = s.pos - h.matchLength + m;
          rec.nm = s.diff; rec.numBestHits = numHits; rec.stateSelf = h.next;
          emitRec(o, cx, rec, nullptr, false);
        }
      } else {
        if (h.chr == CHR_NULL) return -1;
        rec.cig.postS = s.qEnd - s.qStart;
        rec.chr = h.chr; rec.strand = h.strand; rec.start = h.pos; rec.end = h.pos; rec.nm = h.diff;
        rec.numBestHits = numHits;
        emitRec(o, cx, rec, nullptr, false);
      }
    } else {
      if (!sU) return 0;  // convert returns null: SAMOutput.emit prints nothing (:78-81)
      if (s.chr == CHR_NULL) return -1;
      rec.cig = CigSpec{nullptr, 0, h.matchLength, -1, cig + s.cigarOff, (int)s.cigarLen};
      rec.chr = s.chr; rec.strand = s.strand; rec.start = s.pos - h.matchLength; rec.end = s.pos - h.matchLength + m;
      rec.nm = s.diff; rec.numBestHits = numHits; rec.stateSelf = h.next;
      emitRec(o, cx, rec, nullptr, false);
    }
  }
  o.ch('\n');
  return cx.npe ? -1 : 0;
}

// The unmapped record: ReadHit("*", 0, 0, 0, 0, -1, FORWARD, CIGAR(), 0)
// (S/BidirectionalSuffixFilter.java:258-261)
GWA_HD void samUnmapped(SamOut &o, const SamText &t, uint32_t r) {
  o.bytes(t.name + t.nameB[r], t.nameE[r] - t.nameB[r]);
  o.lit("\t68\t*\t0\t1\t\t*\t0\t0\t");
  const uint8_t *c = t.codes + t.codeOff[r];
  const uint32_t len = t.codeLen[r];
  for (uint32_t j0 = 0; j0 < len; j0 += 16) {
    uint8_t x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = j0 + k < len ? c[j0 + k] : 0;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (j0 + k < len) o.ch(samfmt::sym(x[k] > 4 ? 4 : x[k]));
  }
  o.ch('\t');
  if (!qualAbsent(t, r)) o.bytes(t.qual + t.qualB[r], t.qualE[r] - t.qualB[r]);
  else o.ch('*');
  o.ch('\n');
}

// Every record of read r: its reported chains (OutHeader: hits at hitOff, CIGAR ops at cigOff,
// chains back to back) or the unmapped record.  0, or -1 where the reference would throw.
GWA_HD int samRead(SamOut &o, const SamText &t, uint32_t r, const OutHeader &h, const OutHit *hits, const uint16_t *cig) {
  if (h.status == ST_UNMAPPED) {
    samUnmapped(o, t, r);
    return 0;
  }
  if (h.status != ST_MAPPED) return -1;
  const OutHit *hb = hits + h.hitOff;
  const uint16_t *cb = cig + h.cigOff;
  int head = 0;
  for (int c = 0; c < h.nChains; ++c) {
    if (samChain(o, t, r, hb, cb, head) != 0) return -1;
    int x = head;
    while (hb[x].next >= 0) x = hb[x].next;
    head = x + 1;
  }
  return 0;
}

// ---- paired-end (config C5): the build's own design, the reference has none
// (R/ReadReaderFactory.java:60-84); the rules are stated with their CPU restatement, oracle/
// gwa_oracle.cpp orc_align_pairs.  Mate 1 of pair i is read i, mate 2 is read np + i; each mate was
// aligned as a single-end read with every best hit reported (ALLHITS). ----

// unclipped size of a hit's CIGAR (CIGAR.getUnclippedSize: M X D P N, A/CIGAR.java:115-131)
GWA_HD int samRefLen(const uint16_t *cig, const OutHit &h) {
  int l = 0;
  for (uint32_t i = 0; i < h.cigarLen; ++i) {
    const int t = cig[h.cigarOff + i] & 7;
    if (t == 0 || t == 7 || t == 2 || t == 6 || t == 3) l += cig[h.cigarOff + i] >> 3;
  }
  return l;
}

// one mate's SAM line; h / mate = its chosen hit and its mate's (nullptr: unmapped)
GWA_HD void samMateLine(SamOut &o, const SamText &t, uint32_t r, const OutHit *h, const uint16_t *hc, const OutHit *mate,
                        bool first, bool proper, bool leftmost, int64_t tlenAbs, bool sameChr) {
  int flag = 0x1 | (first ? 0x40 : 0x80);
  if (proper) flag |= 0x2;
  if (!h) flag |= 0x4;
  if (!mate) flag |= 0x8;
  if (h && h->strand == 1) flag |= 0x10;
  if (mate && mate->strand == 1) flag |= 0x20;
  o.bytes(t.name + t.nameB[r], t.nameE[r] - t.nameB[r]);
  o.ch('\t');
  o.num(flag);
  o.ch('\t');
  if (h) {
    o.bytes(t.ctg + t.ctgOff[h->chr], t.ctgOff[h->chr + 1] - t.ctgOff[h->chr]);
    o.ch('\t');
    o.num(h->pos);
    o.lit("\t1\t");
    for (uint32_t i = 0; i < h->cigarLen; ++i) {
      o.num(hc[h->cigarOff + i] >> 3);
      o.ch(samfmt::kOp[hc[h->cigarOff + i] & 7]);
    }
    o.ch('\t');
  } else {
    o.lit("*\t0\t1\t*\t");
  }
  if (mate) {
    if (h && sameChr) o.ch('=');
    else o.bytes(t.ctg + t.ctgOff[mate->chr], t.ctgOff[mate->chr + 1] - t.ctgOff[mate->chr]);
    o.ch('\t');
    o.num(mate->pos);
    o.ch('\t');
  } else {
    o.lit("*\t0\t");
  }
  o.num(h && mate && sameChr ? (leftmost ? tlenAbs : -tlenAbs) : 0);
  o.ch('\t');
  const bool rev = h && h->strand == 1;
  const uint8_t *c = t.codes + t.codeOff[r];
  const int m = (int)t.codeLen[r];
  for (int j = 0; j < m; ++j) {
    const uint8_t x = rev ? c[m - 1 - j] : c[j];
    o.ch(samfmt::sym(!rev ? (x > 4 ? 4 : x) : (x < 4 ? 3 - x : 4)));
  }
  o.ch('\t');
  if (qualAbsent(t, r)) {
    o.ch('*');
  } else {
    const uint64_t q0 = t.qualB[r], qn = t.qualE[r] - t.qualB[r];
    for (uint64_t j = 0; j < qn; ++j) o.ch(rev ? t.qual[q0 + qn - 1 - j] : t.qual[q0 + j]);
  }
  if (h) {
    o.lit("\tNM:i:");
    o.num(h->diff);
    o.lit("\tXP:Z:");
    o.ch(h->numHits == 1 ? 'U' : 'R');
    o.lit("\tX0:i:");
    o.num(h->numHits);
  }
  o.ch('\n');
}

// The mates' candidates and the best proper pair of pair i (orc_align_pairs rules 1-2): fa / fb = each
// mate's first candidate (a chain head without a split and with a contig, in report order), a / b =
// the proper pair with the fewest differences (ties: the first in mate-1, then mate-2 order), or null.
// ok = false where a mate's search failed.
struct PairChoice {
  const OutHit *a = nullptr, *b = nullptr, *fa = nullptr, *fb = nullptr;
  const uint16_t *ca = nullptr, *cb = nullptr;  // the CIGAR bases of mate 1's / mate 2's hits
  bool ok = true;
};

// rule 2's test: one contig, opposite strands, forward start <= reverse end, template length in range
GWA_HD bool pairProper(const SamText &t, const OutHit &u, const uint16_t *cu, const OutHit &v, const uint16_t *cv,
                       int32_t minIns, int32_t maxIns) {
  if (t.chrKey[u.chr] != t.chrKey[v.chr] || u.strand == v.strand) return false;
  const OutHit &fw = u.strand == 0 ? u : v, &rv = u.strand == 0 ? v : u;
  const uint16_t *rc = u.strand == 0 ? cv : cu;
  const int64_t fs = fw.pos, re = (int64_t)rv.pos + samRefLen(rc, rv) - 1;
  const int64_t tl = re - fs + 1;
  return !(fs > re || tl < minIns || tl > maxIns);
}

GWA_HD bool pairStatusOk(const OutHeader &A, const OutHeader &B) {
  return (A.status == ST_MAPPED || A.status == ST_UNMAPPED) && (B.status == ST_MAPPED || B.status == ST_UNMAPPED);
}
// a mate's pairing candidates (chain heads without a split and with a contig): their count, and the
// pool index of the first one in report order (-1 = none)
GWA_HD int pairCandidates(const OutHeader &H, const OutHit *hits, int32_t *first) {
  *first = -1;
  const int nc = H.status == ST_MAPPED ? (int)H.nChains : 0;
  const OutHit *h = hits + H.hitOff;
  int count = 0;
  for (int x = 0, hx = 0; x < nc; ++x) {
    const OutHit &u = h[hx];
    int e = hx;
    while (h[e].next >= 0) e = h[e].next;
    if (u.next < 0 && u.chr >= 0) {
      if (*first < 0) *first = (int32_t)(H.hitOff + hx);
      ++count;
    }
    hx = e + 1;
  }
  return count;
}

GWA_HD PairChoice pairChoose(const SamText &t, uint32_t i, uint32_t np, const OutHeader *oh, const OutHit *hits,
                             const uint16_t *cig, int32_t minIns, int32_t maxIns) {
  PairChoice P;
  const OutHeader &A = oh[i], &B = oh[np + i];
  if ((A.status != ST_MAPPED && A.status != ST_UNMAPPED) || (B.status != ST_MAPPED && B.status != ST_UNMAPPED)) {
    P.ok = false;
    return P;
  }
  const OutHit *ha = hits + A.hitOff, *hb = hits + B.hitOff;
  P.ca = cig + A.cigOff;
  P.cb = cig + B.cigOff;
  const int na = A.status == ST_MAPPED ? A.nChains : 0, nb = B.status == ST_MAPPED ? B.nChains : 0;
  int best = 0x7FFFFFFF;
  for (int x = 0, hx = 0; x < na; ++x) {
    const OutHit &u = ha[hx];
    int e = hx;
    while (ha[e].next >= 0) e = ha[e].next;
    const int next = e + 1;
    if (u.next < 0 && u.chr >= 0) {
      if (!P.fa) P.fa = &u;
      for (int y = 0, hy = 0; y < nb; ++y) {
        const OutHit &v = hb[hy];
        int f = hy;
        while (hb[f].next >= 0) f = hb[f].next;
        const int nextB = f + 1;
        if (v.next < 0 && v.chr >= 0 && u.diff + v.diff < best && pairProper(t, u, P.ca, v, P.cb, minIns, maxIns)) {
          best = u.diff + v.diff;
          P.a = &u;
          P.b = &v;
        }
        hy = nextB;
      }
    }
    hx = next;
  }
  for (int y = 0, hy = 0; y < nb && !P.fb; ++y) {
    const OutHit &v = hb[hy];
    if (v.next < 0 && v.chr >= 0) P.fb = &v;
    int f = hy;
    while (hb[f].next >= 0) f = hb[f].next;
    hy = f + 1;
  }
  return P;
}

// Pair i: choose the mates' hits (orc_align_pairs rules 1-3; rule 3's rescued hit from `resc`, the
// pair_rescue kernel's output) and write both lines.  -1 where a mate's search failed.
GWA_HD int samPair(SamOut &o, const SamText &t, uint32_t i, uint32_t np, const OutHeader *oh, const OutHit *hits,
                   const uint16_t *cig, int32_t minIns, int32_t maxIns, const RescueOut *resc) {
  PairChoice P;
  if (resc) {  // the choice made by pair_rescue_kernel / pair_choose_kernel
    if (!pairStatusOk(oh[i], oh[np + i])) return -1;
    const RescueOut &R = resc[i];
    P.a = R.a >= 0 ? hits + R.a : nullptr;
    P.b = R.b >= 0 ? hits + R.b : nullptr;
    P.fa = R.fa >= 0 ? hits + R.fa : nullptr;
    P.fb = R.fb >= 0 ? hits + R.fb : nullptr;
    P.ca = cig + oh[i].cigOff;
    P.cb = cig + oh[np + i].cigOff;
  } else {
    P = pairChoose(t, i, np, oh, hits, cig, minIns, maxIns);
    if (!P.ok) return -1;
  }
  const OutHit *a = P.a, *b = P.b;
  const uint16_t *ca = P.ca, *cb = P.cb;
  bool proper = a != nullptr;
  if (!proper) {
    a = P.fa;
    b = P.fb;
    if (resc && resc[i].status != 0) {  // rule 3: the rescued mate is that mate's only candidate
      const RescueOut &R = resc[i];
      if (R.status == 1) { a = &R.hit; ca = R.cig; }
      else { b = &R.hit; cb = R.cig; }
      proper = a && b && pairProper(t, *a, ca, *b, cb, minIns, maxIns);
    }
  }
  const bool sameChr = a && b && t.chrKey[a->chr] == t.chrKey[b->chr];
  int64_t tlen = 0;
  bool aLeft = true;
  if (sameChr) {
    const int64_t ea = (int64_t)a->pos + samRefLen(ca, *a) - 1, eb = (int64_t)b->pos + samRefLen(cb, *b) - 1;
    tlen = (ea > eb ? ea : eb) - (a->pos < b->pos ? a->pos : b->pos) + 1;
    aLeft = a->pos <= b->pos;
  }
  samMateLine(o, t, i, a, ca, b, true, proper, aLeft, tlen, sameChr);
  samMateLine(o, t, np + i, b, cb, a, false, proper, !aLeft, tlen, sameChr);
  return 0;
}

}  // namespace gwa
