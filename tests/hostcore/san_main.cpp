// san_main.cpp -- TEST-ONLY: the host build of the kernel logic (host_driver.cpp: bsf_core.h,
// sf_core.h, sam_core.h) as a standalone program, so it can run under AddressSanitizer +
// UndefinedBehaviorSanitizer (g++) and MemorySanitizer (clang++) without instrumenting Python.
// tests/test_hostcore_sanitize.py drives it.  Never part of libgwa.so.
//
//   hc_san GENOME READS K REPORT_TYPE NUM_SPLIT STRATEGY > SAM
//   GENOME: "<n_contigs>\n" then "<name> <length>\n" per contig, then the codes (0..4) as raw bytes
//   READS:  one read per line, "name\tsequence\tquality" (quality "*" = none)
// Exit status: 0 aligned (SAM on stdout), 3 the batch failed as the reference would throw,
// 2 bad input.  A sanitizer report aborts the program (-fno-sanitize-recover).
#include "host_driver.cpp"

#include <fstream>
#include <sstream>

#ifdef HC_OMP_STUBS
// the MemorySanitizer build has no OpenMP runtime (an uninstrumented libomp would report false
// positives); host_index.cpp's __gnu_parallel sort then runs on one thread
extern "C" int omp_get_max_threads(void) { return 1; }
extern "C" int omp_get_num_threads(void) { return 1; }
extern "C" int omp_get_thread_num(void) { return 0; }
#endif

int main(int argc, char **argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s GENOME READS K REPORT_TYPE NUM_SPLIT STRATEGY\n", argv[0]);
    return 2;
  }
  std::ifstream g(argv[1], std::ios::binary);
  int nc = 0;
  g >> nc;
  if (!g || nc <= 0) return 2;
  std::vector<std::string> names(nc);
  std::vector<int64_t> lengths(nc);
  int64_t total = 0;
  for (int i = 0; i < nc; ++i) {
    g >> names[i] >> lengths[i];
    total += lengths[i];
  }
  g.get();  // the newline after the last contig line
  std::vector<uint8_t> codes((size_t)total);
  g.read((char *)codes.data(), total);
  if (g.gcount() != total) return 2;
  std::vector<const char *> nm;
  for (auto &s : names) nm.push_back(s.c_str());
  void *ix = hc_index_codes(codes.data(), (uint64_t)total, nc, nm.data(), lengths.data());
  if (!ix) return 2;

  std::ifstream rf(argv[2]);
  std::vector<std::string> rn, rs, rq;
  std::vector<char> hasQ;
  for (std::string line; std::getline(rf, line);) {
    std::istringstream ls(line);
    std::string a, b, c;
    std::getline(ls, a, '\t');
    std::getline(ls, b, '\t');
    std::getline(ls, c, '\t');
    rn.push_back(a);
    rs.push_back(b);
    rq.push_back(c);
    hasQ.push_back(c != "*");
  }
  const uint32_t n = (uint32_t)rn.size();
  std::vector<const char *> pn(n), ps(n), pq(n);
  for (uint32_t i = 0; i < n; ++i) {
    pn[i] = rn[i].c_str();
    ps[i] = rs[i].c_str();
    pq[i] = hasQ[i] ? rq[i].c_str() : nullptr;
  }
  char *out = nullptr;
  uint64_t outLen = 0;
  std::vector<int32_t> stats(4 * (size_t)std::max<uint32_t>(n, 1));
  const int rc = hc_align(ix, (float)atof(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), n, pn.data(), ps.data(),
                          pq.data(), &out, &outLen, stats.data());
  hc_index_free(ix);
  if (rc != 0) return 3;
  fwrite(out, 1, outLen, stdout);
  free(out);
  return 0;
}
