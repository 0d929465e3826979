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

#ifdef HC_OMP_STUBS
// the MemorySanitizer build has no OpenMP runtime (an uninstrumented libomp would report false
// positives); host_index.cpp's __gnu_parallel sort then runs on one thread
extern "C" int omp_get_max_threads(void) { return 1; }
extern "C" int omp_get_num_threads(void) { return 1; }
extern "C" int omp_get_thread_num(void) { return 0; }
#endif

// (input through C stdio, which the sanitizers intercept; libstdc++'s iostreams are not
// instrumented and would read as uninitialised under MemorySanitizer)
int main(int argc, char **argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s GENOME READS K REPORT_TYPE NUM_SPLIT STRATEGY\n", argv[0]);
    return 2;
  }
  FILE *g = fopen(argv[1], "rb");
  if (!g) return 2;
  char line[4096];
  if (!fgets(line, sizeof line, g)) return 2;
  const int nc = atoi(line);
  if (nc <= 0) return 2;
  std::vector<std::string> names(nc);
  std::vector<int64_t> lengths(nc);
  int64_t total = 0;
  for (int i = 0; i < nc; ++i) {
    if (!fgets(line, sizeof line, g)) return 2;
    char *sp = strchr(line, ' ');
    if (!sp) return 2;
    names[i].assign(line, (size_t)(sp - line));
    lengths[i] = atoll(sp + 1);
    total += lengths[i];
  }
  std::vector<uint8_t> codes((size_t)total);
  if (fread(codes.data(), 1, (size_t)total, g) != (size_t)total) return 2;
  fclose(g);
  std::vector<const char *> nm;
  for (auto &s : names) nm.push_back(s.c_str());
  void *ix = hc_index_codes(codes.data(), (uint64_t)total, nc, nm.data(), lengths.data());
  if (!ix) return 2;

  FILE *rf = fopen(argv[2], "rb");
  if (!rf) return 2;
  std::vector<std::string> rn, rs, rq;
  std::vector<char> hasQ;
  char *buf = nullptr;
  size_t cap = 0;
  ssize_t got;
  while ((got = getline(&buf, &cap, rf)) > 0) {
    std::string l(buf, (size_t)got);
    if (!l.empty() && l.back() == '\n') l.pop_back();
    const size_t a = l.find('\t'), b = a == std::string::npos ? a : l.find('\t', a + 1);
    if (b == std::string::npos) return 2;
    rn.push_back(l.substr(0, a));
    rs.push_back(l.substr(a + 1, b - a - 1));
    rq.push_back(l.substr(b + 1));
    hasQ.push_back(rq.back() != "*");
  }
  free(buf);
  fclose(rf);
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
