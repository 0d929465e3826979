// batch_io.hip -- a batch's reads in and SAM text out, on the GPU.
//
// Reads in: the caller's read text (names, bases, qualities) is copied to HBM as it is and encoded
// there -- ACGTSequence(String) (A/ACGTSequence.java:86-97: spaces skipped, ACGT.to3bitCode,
// A/ACGT.java:36-43) into 16-B aligned, zero-padded code rows (ReadsView).
//
// SAM out: the text of a batch is written on the GPU (the reporting tail of the align path:
// AlignmentRecord.convert / toSAMLine and SAMOutput.emit, R/AlignmentRecord.java:109-276,
// A/SAMOutput.java:73-82; the per-read logic is sam_core.h).
//
// The reference formats one record at a time on the host thread that aligned it.  Here one lane
// formats one read: a length pass (the writer in counting mode), an exclusive scan of the lengths
// (rocPRIM), and a write pass that puts every read's records at its offset.  The host receives
// the finished text of the batch in one copy, in input order.  A read on which the reference
// would throw (or whose search failed) is reported through `err` (lowest failing position).
//
// Also here: the batch statistics as a device reduction over the per-read output headers.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "kernels.h"
#include "sam_core.h"
#include "text_core.h"

namespace gwa {

#define FCHK(x)                                                                                         \
  do {                                                                                                  \
    hipError_t e_ = (x);                                                                                \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("sam_format: ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)

// ---- reads in ----

__device__ __forceinline__ uint8_t to3bitDev(unsigned char c) {
  switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 4;
  }
}

// Read text loads: 16-B aligned chunks (the text allocations are padded by 32 bytes, so the chunk
// holding a field's last byte is always inside the allocation) funnel-shifted to the field start.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 loadChunk(const char *__restrict__ base, uint64_t a16) {
  return *reinterpret_cast<const u32x4 *>(base + a16);
}
// bytes [p, p + 16) of the text as 4 dwords (p any alignment)
__device__ __forceinline__ void load16(const char *__restrict__ t, uint64_t p, uint32_t (&w)[4]) {
  const uint64_t a = p & ~(uint64_t)15;
  const int sh = (int)(p & 15);
  const u32x4 c0 = loadChunk(t, a);
  uint32_t x[8] = {c0.x, c0.y, c0.z, c0.w, 0, 0, 0, 0};
  if (sh) {
    const u32x4 c1 = loadChunk(t, a + 16);
    x[4] = c1.x; x[5] = c1.y; x[6] = c1.z; x[7] = c1.w;
  }
  const int q = sh >> 2, r = (sh & 3) * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // dwords q + i and q + i + 1 (q = 0..3) through selects
    uint32_t lo = x[i], hi = x[i + 1];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      lo = q == k ? x[k + i] : lo;
      hi = q == k ? x[k + i + 1] : hi;
    }
    w[i] = r ? (lo >> r) | (hi << (32 - r)) : lo;
  }
}
// per read: bases after skipping spaces, its padded row size, and a mark in the length table
__global__ void __launch_bounds__(256) encodeLenKernel(const char *__restrict__ seq, const uint64_t *__restrict__ seqB,
                                                       const uint64_t *__restrict__ seqE, uint32_t n, uint32_t *__restrict__ codeLen,
                                                       uint32_t *__restrict__ rowLen, uint32_t *__restrict__ lenSeen) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n) return;
  if (r == n) {  // the scan's tail: 16 zero bytes after the last row
    rowLen[n] = 16;
    return;
  }
  const uint64_t b = seqB[r], e = seqE[r];
  uint32_t spaces = 0;
  // aligned 16-B chunks over [b, e); bytes outside the field are masked off
  for (uint64_t a = b & ~(uint64_t)15; a < e; a += 16) {
    const u32x4 c = loadChunk(seq, a);
    const uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t p = a + 4 * i;
      uint32_t m = bytesEq(w[i], ' ');
      // keep bytes p + j with b <= p + j < e
      const int64_t lo = (int64_t)b - (int64_t)p, hi = (int64_t)e - (int64_t)p;
      const uint32_t keepLo = lo <= 0 ? 0xFFFFFFFFu : lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo));
      const uint32_t keepHi = hi >= 4 ? 0xFFFFFFFFu : hi <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - hi)));
      spaces += __builtin_popcount(m & keepLo & keepHi);
    }
  }
  const uint32_t m = (uint32_t)(e - b) - spaces;
  codeLen[r] = m;
  rowLen[r] = (m + 15) & ~15u;
  lenSeen[m < kLenSeen - 1 ? m : kLenSeen - 1] = 1;
}

// one read's code row: 16 codes per store (rows are 16-B aligned and zero-padded); a read with
// spaces in its text (skipped, A/ACGTSequence.java:86-97) takes the byte loop
__global__ void __launch_bounds__(256) encodeWriteKernel(const char *__restrict__ seq, const uint64_t *__restrict__ seqB,
                                                         const uint64_t *__restrict__ seqE, uint32_t n,
                                                         const uint32_t *__restrict__ codeOff,
                                                         const uint32_t *__restrict__ codeLen,
                                                         uint8_t *__restrict__ codes) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  uint8_t *o = codes + codeOff[r];
  const uint64_t b = seqB[r], e = seqE[r];
  const uint32_t m = codeLen[r], row = codeOff[r + 1] - codeOff[r];
  if (m == e - b) {
    for (uint32_t k = 0; k < row; k += 16) {
      uint32_t w[4];
      load16(seq, b + k, w);
      u32x4 v;
      uint32_t c[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int valid = (int)m - (int)(k + 4 * i);  // bytes of this dword inside the read
        const uint32_t keep = valid >= 4 ? 0xFFFFFFFFu : valid <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - valid)));
        c[i] = to3bit4(w[i]) & keep;
      }
      v.x = c[0]; v.y = c[1]; v.z = c[2]; v.w = c[3];
      *reinterpret_cast<u32x4 *>(o + k) = v;
    }
    return;
  }
  uint32_t k = 0;
  for (uint64_t i = b; i < e; ++i)
    if (seq[i] != ' ') o[k++] = to3bitDev((unsigned char)seq[i]);
  for (; k < row; ++k) o[k] = 0;
}

void launchEncode(const char *seq, const uint64_t *seqB, const uint64_t *seqE, uint32_t n, uint32_t *codeLen, uint32_t *rowLen,
                  uint32_t *codeOff, uint32_t *lenSeen, uint8_t *codes, void *scanTmp, size_t scanTmpBytes, int pass,
                  hipStream_t s) {
  const dim3 grid((n + 1 + 255) / 256);
  if (pass == 0) {
    hipLaunchKernelGGL(encodeLenKernel, grid, dim3(256), 0, s, seq, seqB, seqE, n, codeLen, rowLen, lenSeen);
    FCHK(hipGetLastError());
    size_t b = scanTmpBytes;
    FCHK(rocprim::exclusive_scan(scanTmp, b, rowLen, codeOff, (uint32_t)0, (size_t)n + 1, rocprim::plus<uint32_t>(), s));
  } else {
    hipLaunchKernelGGL(encodeWriteKernel, grid, dim3(256), 0, s, seq, seqB, seqE, n, codeOff, codeLen, codes);
    FCHK(hipGetLastError());
  }
}

size_t encodeScanTempBytes(uint32_t n) {
  size_t b = 0;
  FCHK(rocprim::exclusive_scan(nullptr, b, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t)0, (size_t)n + 1,
                               rocprim::plus<uint32_t>(), (hipStream_t)0));
  return b;
}

// FASTQ records straight from the file text (the pipeline's zero-copy path): record r starts at
// start[r] (its header line; the host framed the text into complete records, reads_io.cpp
// frameRecords).  The fields are located under the record rules of reads_io.cpp parseFastq: lines
// end at "\n", "\r\n" or "\r"; a line missing at the end of the text reads as ""; the name is the
// first whitespace-delimited token after '@'; the third line must start with '+' and the quality
// must be as long as the sequence.  A malformed record sets err (lowest record index); the host
// then re-parses the text to report it as the host parser words it.
__device__ __forceinline__ bool isWsDev(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r') || (c >= 0x1c && c <= 0x1f); }

__device__ __forceinline__ uint64_t lineAt(const char *__restrict__ t, uint64_t len, uint64_t pos, uint64_t *e) {
  if (pos >= len) {
    *e = len;
    return len;
  }
  uint64_t i = pos;
  while (i < len && t[i] != '\n' && t[i] != '\r') ++i;
  *e = i;
  if (i == len) return len;
  if (t[i] == '\r' && i + 1 < len && t[i + 1] == '\n') return i + 2;
  return i + 1;
}

__global__ void __launch_bounds__(256) fastqFieldsKernel(const char *__restrict__ t, uint64_t len, const uint64_t *__restrict__ start,
                                                         uint32_t n, uint64_t *__restrict__ f, uint32_t *__restrict__ err) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  uint64_t he, se, pe, qe;
  const uint64_t hb = start[r];
  const uint64_t sb = lineAt(t, len, hb, &he);
  const uint64_t pb = lineAt(t, len, sb, &se);
  const uint64_t qb = lineAt(t, len, pb, &pe);
  (void)lineAt(t, len, qb, &qe);
  if (he == hb || t[hb] != '@' || pe == pb || t[pb] != '+' || qe - qb != se - sb) atomicMin(err, r);
  uint64_t nb = hb + 1;
  while (nb < he && isWsDev((unsigned char)t[nb])) ++nb;
  uint64_t ne = nb;
  while (ne < he && !isWsDev((unsigned char)t[ne])) ++ne;
  // six field arrays of n: name [b, e), sequence [b, e), quality [b, e)
  f[r] = nb;
  f[(size_t)n + r] = ne;
  f[2 * (size_t)n + r] = sb;
  f[3 * (size_t)n + r] = se;
  f[4 * (size_t)n + r] = qb;
  f[5 * (size_t)n + r] = qe;
}

void launchFastqFields(const char *text, uint64_t len, const uint64_t *start, uint32_t n, uint64_t *fields,
                       uint32_t *err, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(fastqFieldsKernel, dim3((n + 255) / 256), dim3(256), 0, s, text, len, start, n, fields, err);
  FCHK(hipGetLastError());
}

// ---- SAM out ----

// one read's records, or (pairs mode, ps.np > 0) pair r's two mate lines
__device__ __forceinline__ int samUnit(SamOut &o, const SamText &t, uint32_t r, const OutHeader *oh, const OutHit *hits,
                                       const uint16_t *cig, const PairSpec &ps) {
  if (ps.np) return samPair(o, t, r, ps.np, oh, hits, cig, ps.minIns, ps.maxIns, ps.resc);
  return samRead(o, t, r, oh[r], hits, cig);
}

__global__ void __launch_bounds__(256) samLenKernel(SamText t, const OutHeader *__restrict__ oh, const OutHit *__restrict__ hits,
                                                    const uint16_t *__restrict__ cig, const uint32_t *__restrict__ idx,
                                                    uint32_t first, uint32_t n, uint64_t *__restrict__ len,
                                                    uint32_t *__restrict__ err, PairSpec ps) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j > n) return;
  if (j == n) {  // the scan's total
    len[n] = 0;
    return;
  }
  const uint32_t r = idx ? idx[j] : first + j;
  SamOut o{nullptr, 0};
  if (samUnit(o, t, r, oh, hits, cig, ps) != 0) {
    atomicMin(err, j);
    o.n = 0;
  }
  len[j] = o.n;
}

// Write pass.  The text of a workgroup's 64 units is one contiguous range of the output
// [off[j0], off[j0 + 64]); it is formatted into LDS (byte stores that stay on the CU) at the
// position it has relative to the 16-B aligned start of that range, then copied out with coalesced
// 16-B stores (the two partial chunks at the range's ends are written bytewise, the neighbouring
// workgroups own their other bytes).  A range larger than the staging buffer (many reported lines)
// is written directly to HBM.
template <int STAGE>
__global__ void __launch_bounds__(64) samWriteKernel(SamText t, const OutHeader *__restrict__ oh, const OutHit *__restrict__ hits,
                                                     const uint16_t *__restrict__ cig, const uint32_t *__restrict__ idx,
                                                     uint32_t first, uint32_t n, const uint64_t *__restrict__ off,
                                                     char *__restrict__ out, PairSpec ps) {
  __shared__ u32x4 stage[STAGE / 16];
  const uint32_t j0 = blockIdx.x * 64, j = j0 + threadIdx.x;
  const uint32_t jEnd = j0 + 64 < n ? j0 + 64 : n;
  const uint64_t gBeg = off[j0], gEnd = off[jEnd];
  const uint64_t base = gBeg & ~(uint64_t)15;
  if (gEnd - base > (uint64_t)STAGE) {
    if (j < n) {
      SamOut o{out + off[j], 0};
      (void)samUnit(o, t, idx ? idx[j] : first + j, oh, hits, cig, ps);
    }
    return;
  }
  if (j < n) {
    SamOut o{reinterpret_cast<char *>(stage) + (off[j] - base), 0};
    (void)samUnit(o, t, idx ? idx[j] : first + j, oh, hits, cig, ps);
  }
  __syncthreads();
  const uint32_t chunks = (uint32_t)((gEnd - base + 15) >> 4);
  for (uint32_t c = threadIdx.x; c < chunks; c += 64) {
    const uint64_t a = base + 16ull * c;
    if (a >= gBeg && a + 16 <= gEnd) {
      *reinterpret_cast<u32x4 *>(out + a) = stage[c];
    } else {
      const char *sb = reinterpret_cast<const char *>(stage) + 16ull * c;
      for (int i = 0; i < 16; ++i)
        if (a + i >= gBeg && a + i < gEnd) out[a + i] = sb[i];
    }
  }
}

void launchSamFormat(const SamText &t, const OutHeader *oh, const OutHit *hits, const uint16_t *cig, const uint32_t *idx,
                     uint32_t first, uint32_t n, uint64_t *len, uint64_t *off, void *scanTmp, size_t *scanTmpBytes,
                     uint32_t *err, char *out, int pass, hipStream_t s, const PairSpec &ps, uint64_t totalBytes) {
  const dim3 grid((n + 1 + 255) / 256);
  if (pass == 0) {
    hipLaunchKernelGGL(samLenKernel, grid, dim3(256), 0, s, t, oh, hits, cig, idx, first, n, len, err, ps);
    FCHK(hipGetLastError());
  } else if (pass == 1) {  // exclusive scan of n + 1 lengths: off[n] = total bytes
    FCHK(rocprim::exclusive_scan(scanTmp, *scanTmpBytes, len, off, (uint64_t)0, (size_t)n + 1, rocprim::plus<uint64_t>(), s));
  } else {
    if (n == 0) return;
    const dim3 g64((n + 63) / 64);
    // Staging for 64 records: the smallest size that holds 64 records of the batch's average length
    // with 3 % to spare (a workgroup whose records do not fit writes them directly, correct but
    // uncoalesced), so more workgroups fit a CU: 20 KiB (8 per CU) for 100 bp, 24 KiB (6) for 150 bp
    // single-end records; pairs 48 KiB
    const uint64_t need = n ? totalBytes * 64 * 103 / 100 / n + 16 : 0;
    // GWA_SAM_STAGE (tests): a small staging buffer, so that workgroups whose records do not fit
    // take the direct-write path next to workgroups that stage theirs
    const char *stg = getenv("GWA_SAM_STAGE");
    if (stg && atoi(stg) > 0) {
      if (atoi(stg) <= 1024)
        hipLaunchKernelGGL(samWriteKernel<1024>, g64, dim3(64), 0, s, t, oh, hits, cig, idx, first, n, off, out, ps);
      else
        hipLaunchKernelGGL(samWriteKernel<4096>, g64, dim3(64), 0, s, t, oh, hits, cig, idx, first, n, off, out, ps);
    } else if (ps.np || need > 32768)
      hipLaunchKernelGGL(samWriteKernel<49152>, g64, dim3(64), 0, s, t, oh, hits, cig, idx, first, n, off, out, ps);
    else if (need > 24576)
      hipLaunchKernelGGL(samWriteKernel<32768>, g64, dim3(64), 0, s, t, oh, hits, cig, idx, first, n, off, out, ps);
    else if (need > 20480 || totalBytes == 0)
      hipLaunchKernelGGL(samWriteKernel<24576>, g64, dim3(64), 0, s, t, oh, hits, cig, idx, first, n, off, out, ps);
    else
      hipLaunchKernelGGL(samWriteKernel<20480>, g64, dim3(64), 0, s, t, oh, hits, cig, idx, first, n, off, out, ps);
    FCHK(hipGetLastError());
  }
}

size_t samScanTempBytes(uint32_t n) {
  size_t b = 0;
  FCHK(rocprim::exclusive_scan(nullptr, b, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint64_t)0, (size_t)n + 1,
                               rocprim::plus<uint64_t>(), (hipStream_t)0));
  return b;
}

// Batch statistics: sums of the per-read instrumentation (gwa_batch_stats_t), one atomic per
// workgroup and field.
__global__ void __launch_bounds__(256) statsKernel(const OutHeader *__restrict__ oh, uint32_t n,
                                                   unsigned long long *__restrict__ acc) {
  __shared__ unsigned long long sh[kStatFields];
  if (threadIdx.x < kStatFields) sh[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long v[kStatFields];
  for (int f = 0; f < kStatFields; ++f) v[f] = 0;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const OutHeader &h = oh[r];
    v[0] += (unsigned)h.fmSearches;
    v[1] += (unsigned)h.quickSteps;
    v[2] += (unsigned)h.blocks;
    v[3] += (unsigned)h.searchBlocks;
    v[4] += (unsigned)h.kmerLookups;
    v[5] += (unsigned)h.saReads;
    v[6] += (unsigned)h.quickSa;
    v[7] += (unsigned)h.quickShort;
    v[8] += (unsigned)h.searchShort;
    v[9] += (unsigned)h.states;
    v[10] += (unsigned)h.numSW;
    v[11] += (unsigned)h.verifyBytes;
    v[12] += h.status == ST_MAPPED;
    v[13] += h.status == ST_UNMAPPED;
    v[14] += (unsigned)h.quickText;
  }
  for (int f = 0; f < kStatFields; ++f) atomicAdd(&sh[f], v[f]);
  __syncthreads();
  if (threadIdx.x < kStatFields) atomicAdd(&acc[threadIdx.x], sh[threadIdx.x]);
}

void launchStats(const OutHeader *oh, uint32_t n, unsigned long long *acc, hipStream_t s) {
  FCHK(hipMemsetAsync(acc, 0, kStatFields * sizeof(unsigned long long), s));
  if (n == 0) return;
  const uint32_t g = (n + 255) / 256;
  hipLaunchKernelGGL(statsKernel, dim3(g > 2048 ? 2048 : g), dim3(256), 0, s, oh, n, acc);
  FCHK(hipGetLastError());
}

// ---- the first tier's search list in quick-scan order (gwa_batch_run) ----
// The searched reads' order does not change any result (each lane runs its own reads to the end), but
// it decides which reads share a wavefront.  A read's best-first search starts from seeds given by its
// quick scan (each strand's numMismatches and longest-match start, S/BidirectionalSuffixFilter.java:
// 318-341), so reads whose scans match alike walk search trees of a similar shape: they reach their
// reports and finish at similar times, and the lanes of a wavefront take the same paths through a
// micro-step together.  Key (byKey), of the strand with fewer mismatches ("lo"; forward on a tie): its
// longest-match start, then both strands' mismatch counts, then its first empty step (2-base buckets).
// !byKey: the read index (a deep tier's list back in input order).  A stable radix sort keeps input
// order inside a key.  Measured per 10M C2 reads (first-tier search ms, hg19 / hg19r): unsorted
// 89.0 / 132.0, this key 65.3 / 111.1; DESIGN.md §4 lists the keys tried.
__global__ void searchKeyKernel(const uint32_t *list, uint32_t n, const ScanRes *sres, int byKey, uint32_t *keys) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = list[i];
  if (!byKey) {
    keys[i] = r;
    return;
  }
  const ScanRes q = sres[r];
  const bool f = q.nmF <= q.nmR;
  const uint32_t lo = (uint32_t)(f ? q.nmF : q.nmR) & 15, hi = (uint32_t)(f ? q.nmR : q.nmF) & 15;
  const uint32_t lm = (uint32_t)(f ? q.lmF : q.lmR) & 511, fe = (uint32_t)(f ? q.feF : q.feR) & 511;
  keys[i] = (((lm >> 1) << 4 | lo) << 4 | hi) << 8 | fe >> 1;
}

size_t sortSearchListTmpBytes(uint32_t n) {
  size_t b = 0;
  FCHK(rocprim::radix_sort_pairs(nullptr, b, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                 (uint32_t *)nullptr, (size_t)n, 0, 32, (hipStream_t)0));
  return b;
}

void launchSortSearchList(const uint32_t *listIn, uint32_t *listOut, uint32_t *keysIn, uint32_t *keysOut, uint32_t n,
                          const ScanRes *sres, bool byKey, void *tmp, size_t tmpBytes, hipStream_t s) {
  hipLaunchKernelGGL(searchKeyKernel, dim3((n + 255) / 256), dim3(256), 0, s, listIn, n, sres, byKey ? 1 : 0, keysIn);
  FCHK(hipGetLastError());
  size_t b = tmpBytes;
  FCHK(rocprim::radix_sort_pairs(tmp, b, keysIn, keysOut, listIn, listOut, (size_t)n, 0, byKey ? 24 : 32, s));
}

}  // namespace gwa
