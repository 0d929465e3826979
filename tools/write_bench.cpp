// write_bench.cpp -- what bounds the pipeline's SAM sink: write `gb` GiB of text
// from memory into files with T threads, each thread writing its own 64 MiB batches (as the pipeline's
// workers do, tools only; nothing here is part of libgwa).
//   write_bench DIR GB THREADS MODE
//   MODE: one     -- buffered pwrite, all threads into one file at disjoint offsets (the pipeline)
//         sep     -- buffered write, one file per thread (the --shard processes)
//         direct  -- O_DIRECT pwrite into one preallocated file (fallocate), 4 KiB-aligned batches
//         mem     -- memcpy into a private buffer (the copy alone, no file system)
//         mmap    -- one file sized up front (ftruncate), mapped MAP_SHARED; threads memcpy their batches
//         mmappop -- the same with each batch's pages populated first (MADV_POPULATE_WRITE)
// Prints one JSON line: GB/s over the wall time.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

int main(int argc, char **argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s DIR GB THREADS one|sep|direct|mem\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1], mode = argv[4];
  const size_t total = (size_t)(atof(argv[2]) * (1ull << 30));
  const int T = atoi(argv[3]);
  const size_t batch = 64ull << 20;
  const size_t nb = (total + batch - 1) / batch;
  std::vector<char *> src(T);
  for (int t = 0; t < T; ++t) {
    if (posix_memalign((void **)&src[t], 4096, batch)) return 3;
    for (size_t i = 0; i < batch; ++i) src[t][i] = (char)('A' + (i * 7 + t) % 26);
  }
  std::vector<int> fds;
  const int flags = O_WRONLY | O_CREAT | O_TRUNC | (mode == "direct" ? O_DIRECT : 0);
  if (mode == "sep") {
    for (int t = 0; t < T; ++t) fds.push_back(open((dir + "/wb_" + std::to_string(t)).c_str(), flags, 0644));
  } else if (mode != "mem" && mode != "mmap" && mode != "mmappop") {
    fds.push_back(open((dir + "/wb_one").c_str(), flags, 0644));
    if (mode == "direct" && fallocate(fds[0], 0, 0, (off_t)(nb * batch)) != 0) perror("fallocate");
  }
  for (int fd : fds)
    if (fd < 0) { perror("open"); return 4; }
  char *map = nullptr;
  if (mode == "mmap" || mode == "mmappop") {
    fds.push_back(open((dir + "/wb_one").c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644));
    if (fds[0] < 0 || ftruncate(fds[0], (off_t)(nb * batch)) != 0) { perror("ftruncate"); return 4; }
    map = (char *)mmap(nullptr, nb * batch, PROT_READ | PROT_WRITE, MAP_SHARED, fds[0], 0);
    if (map == MAP_FAILED) { perror("mmap"); return 4; }
  }
  std::vector<char *> dst;
  if (mode == "mem")
    for (int t = 0; t < T; ++t) dst.push_back((char *)malloc(batch));
  std::atomic<size_t> next{0};
  std::atomic<bool> bad{false};
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      for (size_t b; (b = next.fetch_add(1)) < nb;) {
        if (mode == "mem") {
          memcpy(dst[t], src[t], batch);
          continue;
        }
        if (map) {
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
          if (mode == "mmappop" && madvise(map + b * batch, batch, MADV_POPULATE_WRITE) != 0) { bad = true; return; }
          memcpy(map + b * batch, src[t], batch);
          continue;
        }
        const int fd = mode == "sep" ? fds[t] : fds[0];
        size_t done = 0;
        while (done < batch) {
          const ssize_t w = mode == "sep" ? write(fd, src[t] + done, batch - done)
                                          : pwrite(fd, src[t] + done, batch - done, (off_t)(b * batch + done));
          if (w <= 0) { bad = true; return; }
          done += (size_t)w;
        }
      }
    });
  for (auto &x : th) x.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (map) munmap(map, nb * batch);
  for (int fd : fds) close(fd);
  printf("{\"mode\": \"%s\", \"threads\": %d, \"gib\": %.2f, \"seconds\": %.4f, \"GBps\": %.3f, \"ok\": %s}\n", mode.c_str(), T,
         (double)nb * batch / (1ull << 30), s, (double)nb * batch / s / 1e9, bad ? "false" : "true");
  if (mode == "sep")
    for (int t = 0; t < T; ++t) unlink((dir + "/wb_" + std::to_string(t)).c_str());
  else if (mode != "mem")
    unlink((dir + "/wb_one").c_str());
  return bad ? 1 : 0;
}
