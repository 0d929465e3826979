// sam.cpp -- host-side record conversion and SAM text (the reporting tail of the align path):
//   AlignmentRecord.convert   (R/AlignmentRecord.java:181-276)
//   AlignmentRecord.toSAMLine (R/AlignmentRecord.java:109-170)
//   SAMOutput.emit            (A/SAMOutput.java:73-82)
//   SequenceBoundary.toSAMHeader (A/SequenceBoundary.java:81-87)
// SAM flag values follow the SAM spec (utgb SAMReadFlag is unvendored).
#include "sam.h"

#include <algorithm>
#include <cstring>

namespace gwa {

static const char kSym[5] = {'A', 'C', 'G', 'T', 'N'};
static const char kOp[8] = {'M', 'I', 'D', 'N', 'S', 'H', 'P', 'X'};

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

namespace {
struct Cig {
  std::vector<std::pair<int, int>> e;  // (type, len)
  void add(int t, int len) {  // CIGAR.add(Element) merges equal adjacent types (A/CIGAR.java:158-170)
    if (!e.empty() && e.back().first == t) e.back().second += len;
    else e.push_back({t, len});
  }
  void add(const Cig &o) { for (auto &x : o.e) add(x.first, x.second); }
  int unclipped() const {
    int l = 0;
    for (auto &x : e)
      if (x.first == 0 || x.first == 7 || x.first == 2 || x.first == 6 || x.first == 3) l += x.second;
    return l;
  }
  void str(std::string &o) const {
    for (auto &x : e) { o += std::to_string(x.second); o += kOp[x.first & 7]; }
  }
};

struct Rec {
  int chr;  // contig or CHR_STAR
  int strand, start, end, nm;
  Cig cigar;
  std::string seq;
  bool qualNull;
  std::string qual;
  int numBestHits;
  std::string state;
  Rec *split = nullptr;
};

struct Ctx {
  const HostIndex &ix;
  const char *name;
  size_t nameLen;
};

const std::string &chrName(const HostIndex &ix, int c, bool *npe) {
  static const std::string star = "*", empty = "";
  if (c >= 0) return ix.names[(size_t)c];
  if (c == CHR_STAR) return star;
  if (c == CHR_EMPTY) return empty;
  *npe = true;
  return empty;
}

void line(const Ctx &cx, const Rec &r, bool hasSegments, bool isFirst, bool eachMapped, std::string &o, bool *npe) {
  int flag = 0;
  if (hasSegments) flag |= 0x1;
  if (r.strand == 1) flag |= 0x10;
  if (isFirst) {
    flag |= 0x40;
    for (const Rec *x = &r; x; x = x->split)
      if (x->numBestHits <= 0) { eachMapped = false; break; }
  } else if (!r.split) {
    flag |= 0x80;
  }
  if (eachMapped) flag |= 0x2;
  if (r.numBestHits <= 0) flag |= 0x4;
  if (r.split && r.split->numBestHits <= 0) flag |= 0x8;
  o.append(cx.name, cx.nameLen);
  o += '\t';
  o += std::to_string(flag);
  o += '\t';
  const std::string &cn = chrName(cx.ix, r.chr, npe);
  o += cn;
  o += '\t';
  o += std::to_string(r.start);
  o += "\t1\t";  // MAPQ column = AlignmentRecord.score, always 1 (:199)
  r.cigar.str(o);
  if (!r.split) {
    o += "\t*\t0\t0";
  } else {
    const std::string &sn = chrName(cx.ix, r.split->chr, npe);
    if (cn != "*" && cn == sn) o += "\t=";
    else { o += '\t'; o += sn; }
    o += '\t';
    o += std::to_string(r.split->start);
    o += '\t';
    o += std::to_string(r.split->end - r.start);
  }
  o += '\t';
  o += r.seq;
  o += '\t';
  if (r.qualNull) o += '*';
  else o += r.qual;
  if (r.numBestHits > 0) {
    if (r.nm >= 0) { o += "\tNM:i:"; o += std::to_string(r.nm); }
    o += "\tXP:Z:";
    o += r.state;
    o += "\tX0:i:";
    o += std::to_string(r.numBestHits);
  }
  if (r.split) {
    o += '\n';
    line(cx, *r.split, hasSegments, false, eachMapped, o, npe);
  }
}

inline const char *stateSingle(int numHits) { return numHits > 0 ? (numHits == 1 ? "U" : "R") : "N"; }
}  // namespace

// Convert one reported ReadHit chain into SAM text (appended to `out`, '\n' terminated).
// Returns 0, or -1 for a Java exception in the reference (the whole run would abort).
int formatChain(const HostIndex &ix, const ReadText &rt, const OutHit *hits, const uint16_t *cig, int head, std::string &out) {
  bool npe = false;
  Ctx cx{ix, rt.name, rt.nameLen};
  // the read as an ACGTSequence (spaces skipped, A/ACGTSequence.java:86-97)
  std::string fwd;
  fwd.reserve(rt.seqLen);
  for (size_t i = 0; i < rt.seqLen; ++i)
    if (rt.seq[i] != ' ') fwd += kSym[to3bit((unsigned char)rt.seq[i])];
  const int m = (int)fwd.size();
  const OutHit &h = hits[head];
  std::string query = fwd;
  bool qualNull = rt.qual == nullptr;
  std::string qual = qualNull ? std::string() : std::string(rt.qual, rt.qualLen);
  if (h.strand != 0) {  // reverseComplement + reversed qual (:187-191)
    std::string rc(query.rbegin(), query.rend());
    for (auto &c : rc) c = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
    query.swap(rc);
    if (!qualNull) std::reverse(qual.begin(), qual.end());
  }
  auto cigOf = [&](const OutHit &x) {
    Cig c;
    for (int i = 0; i < x.cigarLen; ++i) {
      uint16_t v = cig[x.cigarOff + i];
      c.e.push_back({v & 7, v >> 3});  // a fresh CIGAR keeps its own element list
    }
    return c;
  };
  auto chainState = [&](int self) {  // ReadHit.getAlignmentState(head) (R/ReadHit.java:121-131)
    std::string s;
    for (int t = head; t >= 0; t = hits[t].next) {
      std::string x = stateSingle(hits[t].numHits);
      if (t != self) x[0] = (char)(x[0] - 'A' + 'a');
      s += x;
    }
    return s;
  };
  Rec rec, srec;
  if (h.next < 0) {
    int totalDiff = h.diff;
    std::string st = stateSingle(h.numHits);
    rec.chr = h.chr; rec.strand = h.strand; rec.start = h.pos; rec.end = h.pos + h.matchLength; rec.nm = totalDiff;
    rec.cigar = cigOf(h); rec.seq = query; rec.qualNull = qualNull; rec.qual = qual; rec.numBestHits = h.numHits;
    rec.state = st;
  } else {
    // the head and its first split are converted; later fragments of a longer chain are dropped
    // (R/AlignmentRecord.java:201-206 reads hit.nextSplit only), but still named in XP (chainState)
    const OutHit &s = hits[h.next];
    const int numHits = h.numHits;
    int qualLen = !qualNull ? (int)qual.size() : h.matchLength;
    auto sub = [&](const std::string &x, int a, int b) -> std::string {
      if (a < 0 || b > (int)x.size() || a > b) { npe = true; return std::string(); }
      return x.substr((size_t)a, (size_t)(b - a));
    };
    std::string s1 = sub(query, h.qStart, h.qEnd);
    std::string s2 = sub(query, s.qStart, s.qEnd);
    int b1 = std::min(qualLen, h.matchLength);
    int b2 = std::min(qualLen, m);
    std::string q1, q2;
    if (!qualNull) { q1 = sub(qual, 0, b1); q2 = sub(qual, b1, b2); }
    if (npe) return -1;
    bool hU = h.numHits == 1, sU = s.numHits == 1;
    if (hU) {
      if (sU) {
        if (h.chr == CHR_NULL) return -1;
        bool same = (h.chr >= 0 && s.chr >= 0) ? ix.names[(size_t)h.chr] == ix.names[(size_t)s.chr] : h.chr == s.chr;
        if (s.chr == CHR_NULL) same = false;
        if (same) {
          rec.chr = h.chr; rec.strand = h.strand; rec.start = h.pos; rec.end = h.pos + h.matchLength; rec.nm = h.diff;
          rec.cigar = cigOf(h); rec.seq = s1; rec.qualNull = qualNull; rec.qual = q1; rec.numBestHits = 1;
          rec.state = chainState(head);
          srec.chr = s.chr; srec.strand = s.strand; srec.start = s.pos; srec.end = s.pos + s.matchLength; srec.nm = s.diff;
          srec.cigar = cigOf(s); srec.seq = s2; srec.qualNull = qualNull; srec.qual = q2; srec.numBestHits = 1;
          srec.state = chainState(h.next);
          rec.split = &srec;
        } else if (h.matchLength >= s.matchLength) {
          Cig c = cigOf(h);
          c.add(4, s.matchLength);
          rec.chr = h.chr; rec.strand = h.strand; rec.start = h.pos; rec.end = h.pos + m; rec.nm = h.diff;
          rec.cigar = c; rec.seq = query; rec.qualNull = qualNull; rec.qual = qual; rec.numBestHits = numHits;
          rec.state = chainState(head);
        } else {
          Cig c = cigOf(h);
          c.add(cigOf(s));
          if (s.chr == CHR_NULL) return -1;
          rec.chr = s.chr; rec.strand = s.strand; rec.start = s.pos - h.matchLength; rec.end = s.pos - h.matchLength + m;
          rec.nm = s.diff; rec.cigar = c; rec.seq = query; rec.qualNull = qualNull; rec.qual = qual;
          rec.numBestHits = numHits; rec.state = chainState(h.next);
        }
      } else {
        Cig c = cigOf(h);
        c.add(4, s.qEnd - s.qStart);
        if (h.chr == CHR_NULL) return -1;
        rec.chr = h.chr; rec.strand = h.strand; rec.start = h.pos; rec.end = h.pos + c.unclipped(); rec.nm = h.diff;
        rec.cigar = c; rec.seq = query; rec.qualNull = qualNull; rec.qual = qual; rec.numBestHits = numHits;
        rec.state = chainState(head);
      }
    } else {
      if (!sU) return 0;  // convert returns null: SAMOutput.emit prints nothing (:78-81)
      Cig c;
      c.add(4, h.matchLength);
      c.add(cigOf(s));
      if (s.chr == CHR_NULL) return -1;
      rec.chr = s.chr; rec.strand = s.strand; rec.start = s.pos - h.matchLength; rec.end = s.pos - h.matchLength + m;
      rec.nm = s.diff; rec.cigar = c; rec.seq = query; rec.qualNull = qualNull; rec.qual = qual;
      rec.numBestHits = numHits; rec.state = chainState(h.next);
    }
  }
  line(cx, rec, rec.split != nullptr, true, true, out, &npe);
  out += '\n';
  return npe ? -1 : 0;
}

int formatRead(const HostIndex &ix, const ReadText &rt, const OutHeader &h, const OutHit *hits, const uint16_t *cig,
               std::string &out) {
  const OutHit *hb = hits + h.hitOff;
  const uint16_t *cb = cig + h.cigOff;
  int head = 0;
  for (int c = 0; c < h.nChains; ++c) {
    if (formatChain(ix, rt, hb, cb, head, out) != 0) return -1;
    int t = head;
    while (hb[t].next >= 0) t = hb[t].next;
    head = t + 1;
  }
  return 0;
}

// The unmapped record: ReadHit("*", 0, 0, 0, 0, -1, FORWARD, CIGAR(), 0) (S/BidirectionalSuffixFilter.java:258-261)
void formatUnmapped(const ReadText &rt, std::string &out) {
  out.append(rt.name, rt.nameLen);
  out += "\t68\t*\t0\t1\t\t*\t0\t0\t";
  for (size_t i = 0; i < rt.seqLen; ++i)
    if (rt.seq[i] != ' ') out += kSym[to3bit((unsigned char)rt.seq[i])];
  out += '\t';
  if (rt.qual) out.append(rt.qual, rt.qualLen);
  else out += '*';
  out += '\n';
}

}  // namespace gwa
