// host_index.h -- host-side index construction and the host half of the align path
// (FASTA packing, cyclic SA, Occ blocks, staircase tables, SAM records).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "gwa_layout.h"

namespace gwa {

struct HostIndex {
  uint64_t N = 0;
  std::vector<uint8_t> T;  // forward text, codes 0..4
  std::vector<std::string> names;
  std::vector<int64_t> lengths, offsets;
  std::vector<int32_t> chrRank;  // String.compareTo rank of each contig name
  std::vector<uint32_t> sa[2];   // cyclic SA of T and of reverse(T)
  std::vector<OccBlock> occ[2];
  std::vector<uint64_t> text2, textN;
  uint64_t C[5] = {0, 0, 0, 0, 0};
};

// PackFasta.encodeFASTA (A/PackFasta.java:81-108): sequence lines trimmed, every char through
// ACGT.to3bitCode; contig name = first token of the description line.
void packFasta(const char *text, size_t len, HostIndex &ix);
// Add a contig from a plain sequence string (FMIndexOnGenome.buildFromSequence, A/FMIndexOnGenome.java:105-115)
void addSequence(const std::string &name, const char *seq, size_t len, HostIndex &ix);
// Cyclic suffix array of codes[0,n) (sorted rotations, A<C<G<T<N; CyclicSAIS's answer for
// non-periodic texts).  Host prefix doubling; returns false for a periodic text.
bool cyclicSAHost(const uint8_t *codes, uint64_t n, std::vector<uint32_t> &sa, int alphabetBits = 3);
// Derive BWT Occ blocks, 2-bit text, C[] from T and the two SAs.
void finishIndex(HostIndex &ix);
// Staircase tables for read lengths in `lengths` and k up to kmax.
// per read length m <= kMaxReadLen: the tables of every kk in [0, kmax + 1] (base[m]) and the kk whose
// StaircaseFilter(m, kk) constructor throws in the reference (bit kk of bad[m]; its table is zeros).
// Behind each length's table: the staircase masks themselves, ceil(m / 64) words per (kk, row)
// (offsets outside [-kmax, m], which only chunks with wrapped (byte) starts reach)
// Blocks are cached per (m, kmax) across batches; a batch whose tables exceed kStairMaxWords fails
// with an error naming the size (reads of many lengths at a large k: split the batch by length).
void buildStairTables(const std::vector<int> &lengths, int kmax, std::vector<uint64_t> &tab, std::vector<uint32_t> &base,
                      std::vector<uint64_t> &bad);
// one length's block (offsets table, then raw masks) into tab; bit kk set: StaircaseFilter(m, kk) throws
uint64_t buildStairBlock(int m, int kmax, std::vector<uint64_t> &tab);
static const size_t kStairMaxWords = (size_t)128 << 20;  // 1 GiB of tables per batch at most

// Java-String.compareTo-consistent ranks of contig names
void rankNames(HostIndex &ix);

// to3bitCode (A/ACGT.java:36-43)
static inline uint8_t to3bit(unsigned char c) {
  switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 4;
  }
}

}  // namespace gwa
