// pipeline.cpp -- the multi-device, overlapped host driver of the align path (include/gwa.h
// gwa_pipeline_*).
//
// The reference aligns one read at a time on one thread and emits each SAM line as it goes
// (A/Align.java:174-196, PassReadToAligner; A/SAMOutput.java:53 autoflush).  Here reads are cut into
// batches that are dealt to every device handle as it becomes free -- each handle is a full index
// replica on its own GPU, so there is no exchange between devices (reads shard embarrassingly) --
// and the SAM of the batches is written back in input order, byte-identical to a one-device run.
//
// Threads: one reader (the file: framing of complete records only, no parsing), W workers per
// device (parse a framed slice, set the batch up on the device, run the kernels, format the SAM),
// and the caller, which writes the results in batch order.  The workers of one device run their
// batches' kernels concurrently, each batch on its own stream and search scratch (gwa_api.cpp
// Scratch), so one batch's set-up, deep-tier tail and SAM formatting overlap another's kernels.  At
// most `depth` batches are in flight, which bounds memory.
#include <hip/hip_runtime.h>
#include <zlib.h>

#include "snappy_stream.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

#include "../../include/gwa.h"

extern "C" int gwa_fail_message(const char *msg);  // gwa_api.cpp

namespace gwa {
uint64_t frameRecords(const char *t, uint64_t len, int format, bool final, uint64_t maxRec, uint64_t *nRec,
                      std::vector<uint64_t> *starts);
void newlinePositions(const char *t, uint64_t a, uint64_t b, std::vector<uint64_t> &out);
void newlineCount(const char *t, uint64_t a, uint64_t b, uint64_t *count, bool *blank, bool *cr);
void recordStartsFromNewlines(const char *t, uint64_t a, uint64_t b, uint64_t g0, uint64_t *starts, uint64_t cap);
uint64_t frameFastqLines(const char *t, uint64_t len, const std::vector<uint64_t> &nl, bool final, uint64_t maxRec,
                         uint64_t *nRec, std::vector<uint64_t> *starts);
int batchCreateFastq(gwa_index_t *ix, const gwa_config_t *cfg, const char *text, uint64_t len, const uint64_t *start,
                     uint32_t n, gwa_batch_t **out);
uint64_t batchSamInto(gwa_batch_t *b, char **buf, uint64_t *cap);  // gwa_api.cpp
void pinnedFree(char *p);
char *pinnedAlloc(uint64_t bytes);
}

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// A buffer of read-file text.  Pinned host memory makes the batch's H2D copy one DMA instead of a
// staged pageable copy, which the runtime serialises across worker threads (measured: set-up 0.36 s
// -> 0.21 s and 11 -> 22 M reads/s FASTQ -> SAM for 10M reads).  Pinning takes about a second per
// 5 GB; gwa_pipeline_open pins the buffers a run keeps in flight, and the pool falls back to pageable
// buffers beyond them.  Buffers are recycled when the last job that references one is done, and kept
// across align_file calls.
struct TextBuf {
  char *p = nullptr;
  size_t cap = 0, size = 0;
  bool pinned = false;
  const char *data() const { return p; }
};

class BufPool {
  std::mutex mu;
  std::vector<TextBuf *> free_, freePageable_;
  std::shared_ptr<bool> alive = std::make_shared<bool>(true);  // buffers out at destruction free themselves

  static void release(TextBuf *b) {
    if (b->pinned) gwa::pinnedFree(b->p);
    else ::free(b->p);
    delete b;
  }
  static TextBuf *take(std::vector<TextBuf *> &v, size_t cap) {
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i]->cap >= cap) {
        TextBuf *b = v[i];
        v.erase(v.begin() + (long)i);
        return b;
      }
    return nullptr;
  }

 public:
  ~BufPool() {
    std::lock_guard<std::mutex> g(mu);
    *alive = false;
    for (auto *b : free_) release(b);
    for (auto *b : freePageable_) release(b);
    free_.clear();
    freePageable_.clear();
  }
  // a pinned buffer for the free list (the background pinning thread)
  void addPinned(size_t cap) {
    TextBuf *b = new TextBuf();
    try {
      b->p = gwa::pinnedAlloc(cap);
    } catch (...) {
      delete b;
      throw;
    }
    b->cap = cap;
    b->pinned = true;
    std::lock_guard<std::mutex> g(mu);
    if (!*alive) { release(b); return; }
    free_.push_back(b);
    // a pageable buffer is dropped for each pinned one that arrives
    if (!freePageable_.empty()) {
      release(freePageable_.back());
      freePageable_.pop_back();
    }
  }
  // free pinned buffers of at least `cap` bytes
  uint64_t countPinned(size_t cap) {
    std::lock_guard<std::mutex> g(mu);
    uint64_t n = 0;
    for (auto *b : free_) n += b->cap >= cap ? 1 : 0;
    return n;
  }
  // unpin the free pinned buffers smaller than `cap` (they can never serve a request of that size);
  // returns how many and their bytes
  void releasePinnedBelow(size_t cap, uint64_t *n, uint64_t *bytes) {
    std::lock_guard<std::mutex> g(mu);
    *n = *bytes = 0;
    for (size_t i = 0; i < free_.size();)
      if (free_[i]->cap < cap) {
        ++*n;
        *bytes += free_[i]->cap;
        release(free_[i]);
        free_.erase(free_.begin() + (long)i);
      } else {
        ++i;
      }
  }
  std::shared_ptr<TextBuf> get(size_t cap) {
    TextBuf *b = nullptr;
    {
      std::lock_guard<std::mutex> g(mu);
      b = take(free_, cap);
      if (!b) b = take(freePageable_, cap);
    }
    if (!b) {
      b = new TextBuf();
      b->p = (char *)::malloc(cap);
      if (!b->p) {
        delete b;
        throw std::runtime_error("out of host memory for the read text");
      }
      b->cap = cap;
    }
    b->size = 0;
    std::shared_ptr<bool> live = alive;
    return std::shared_ptr<TextBuf>(b, [this, live](TextBuf *x) {
      if (!*live) { release(x); return; }
      std::lock_guard<std::mutex> g(mu);
      (x->pinned ? free_ : freePageable_).push_back(x);
    });
  }
};

// One unit of work: either reads already in memory (a gwa_reads_t slice) or a framed slice of file
// text that the worker parses itself.
struct Job {
  uint64_t id = 0;
  gwa_reads_t reads{};                 // in-memory reads (text == nullptr)
  std::shared_ptr<TextBuf> text;       // or: file text holding complete records [tb, te)
  uint64_t tb = 0, te = 0;
  int format = 1;
  std::vector<uint64_t> starts;  // FASTQ: each record's header line, relative to tb
};

struct Result {
  gwa_results_t r{};
  uint32_t n = 0;
};

}  // namespace

// read-file chunks (and the room before each for the records carried over from the previous one);
// a smaller file reads in one chunk of its own size
constexpr uint64_t kChunk = 256ull << 20, kReserve = 512ull << 20;

namespace {
// MemAvailable of /proc/meminfo in bytes (0 = unknown)
uint64_t memAvailable() {
  FILE *f = fopen("/proc/meminfo", "r");
  if (!f) return 0;
  char line[256];
  uint64_t kb = 0;
  while (fgets(line, sizeof line, f))
    if (sscanf(line, "MemAvailable: %lu kB", (unsigned long *)&kb) == 1) break;
  fclose(f);
  return kb * 1024;
}
}  // namespace

struct gwa_pipeline {
  std::vector<gwa_index_t *> ix;
  gwa_config_t cfg{};
  uint32_t batchReads = 1u << 20;
  int workersPerDevice = 2;
  gwa_pipeline_stats_t stats{};
  BufPool pool;  // pinned read-text buffers, kept across align_file calls
  uint64_t pinnedBufs = 0, pinnedBytes = 0;  // pinned so far (lazily, by align_file)
  std::mutex samMu;
  std::vector<std::pair<char *, uint64_t>> samBufs;  // pinned SAM buffers, one per file worker, kept too
  ~gwa_pipeline() {
    for (auto &b : samBufs) gwa::pinnedFree(b.first);
  }
};

namespace {

// Shared state of one run (align or align_file).
struct Run {
  gwa_pipeline *p;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Job> jobs;
  std::map<uint64_t, Result> done;
  bool noMoreJobs = false, failed = false;
  std::string err;
  size_t inflight = 0, depth;
  std::vector<std::thread> workers;
  std::atomic<uint64_t> reads{0};
  std::vector<double> devBusy;  // per device: seconds of kernels
  double parseS = 0, setupS = 0, formatS = 0, writeS = 0, waitS = 0;  // summed over worker threads
  // file mode: each worker writes its own batch's SAM from its pinned buffer -- at its offset with
  // pwrite when the output is a regular file (offsets fixed in batch order as sizes become known),
  // else in batch order with write
  int fd = -1;
  bool seekable = false;
  uint64_t base = 0;                        // file position of the first record
  std::map<uint64_t, uint64_t> sizes, offs; // batch -> SAM bytes / offset
  uint64_t cursor = 0, nextOff = 0;         // first batch whose offset is not fixed yet, its offset
  uint64_t turn = 0;                        // non-seekable output: the batch that writes next
  std::atomic<uint64_t> fileReads{0}, fileBatches{0};

  explicit Run(gwa_pipeline *p_) : p(p_) {
    depth = std::max<size_t>(4, 2 * p->ix.size() * p->workersPerDevice);
    devBusy.assign(p->ix.size(), 0.0);
  }

  void fail(const std::string &m) {
    std::lock_guard<std::mutex> g(mu);
    if (!failed) { failed = true; err = m; }
    cv.notify_all();
  }

  // producer side: blocks while `depth` batches are in flight; false once the run has failed
  bool push(Job &&j) {
    std::unique_lock<std::mutex> g(mu);
    cv.wait(g, [&] { return failed || inflight < depth; });
    if (failed) return false;
    ++inflight;
    jobs.push_back(std::move(j));
    cv.notify_all();
    return true;
  }
  void finishJobs() {
    std::lock_guard<std::mutex> g(mu);
    noMoreJobs = true;
    cv.notify_all();
  }

  void worker(int d) {
    gwa_index_t *ix = p->ix[(size_t)d];
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return failed || !jobs.empty() || noMoreJobs; });
        if (failed || jobs.empty()) return;
        j = std::move(jobs.front());
        jobs.pop_front();
      }
      Result res;
      gwa_read_buf_t parsed{};
      const gwa_reads_t *rd = &j.reads;
      int rc = 0;
      if (j.text) {
        uint64_t used = 0;
        rc = gwa_reads_parse(j.text->data() + j.tb, j.te - j.tb, j.format, 1, &parsed, &used);
        rd = &parsed.reads;
      }
      if (rc == 0) {
        res.n = rd->n;
        gwa_batch_t *b = nullptr;
        rc = gwa_batch_create(ix, &p->cfg, rd, &b);
        if (rc == 0) {
          const auto t0 = Clock::now();
          rc = gwa_batch_run(b);
          const double kt = secs(t0, Clock::now());
          if (rc == 0) rc = gwa_batch_results(b, &res.r);
          {
            std::lock_guard<std::mutex> g(mu);
            devBusy[(size_t)d] += kt;
          }
        }
        gwa_batch_free(b);
      }
      const std::string msg = rc != 0 ? std::string(gwa_last_error()) : std::string();
      if (j.text) gwa_reads_free(&parsed);
      if (rc != 0) {
        gwa_results_free(&res.r);
        fail("batch " + std::to_string(j.id) + " on device handle " + std::to_string(d) + ": " + msg);
        return;
      }
      reads += res.n;
      std::lock_guard<std::mutex> g(mu);
      done.emplace(j.id, std::move(res));
      cv.notify_all();
    }
  }

  // file mode: put batch `id`'s SAM (size bytes at p) into the output in batch order
  void output(uint64_t id, const char *p, uint64_t size) {
    const auto w0 = Clock::now();
    uint64_t off = 0;
    {
      std::unique_lock<std::mutex> g(mu);
      if (seekable) {
        sizes[id] = size;
        for (auto it = sizes.find(cursor); it != sizes.end(); it = sizes.find(cursor)) {
          offs[cursor] = nextOff;
          nextOff += it->second;
          sizes.erase(it);
          ++cursor;
        }
        cv.notify_all();
        cv.wait(g, [&] { return failed || offs.count(id) != 0; });
        if (failed) return;
        off = offs[id];
        offs.erase(id);
      } else {
        cv.wait(g, [&] { return failed || turn == id; });
        if (failed) return;
      }
    }
    const auto w1 = Clock::now();
    uint64_t done = 0;
    while (done < size) {
      const size_t chunk = (size_t)std::min<uint64_t>(size - done, 1ull << 30);
      const ssize_t w = seekable ? ::pwrite(fd, p + done, chunk, (off_t)(base + off + done)) : ::write(fd, p + done, chunk);
      if (w <= 0) throw std::runtime_error("write to the SAM output failed");
      done += (uint64_t)w;
    }
    const auto w2 = Clock::now();
    std::lock_guard<std::mutex> g(mu);
    if (!seekable) ++turn;
    waitS += secs(w0, w1);
    writeS += secs(w1, w2);
    cv.notify_all();
  }

  // file mode worker: parse its framed slice, align it on device d, write its SAM
  void fileWorker(int d) {
    gwa_index_t *ix = p->ix[(size_t)d];
    char *pinned = nullptr;
    uint64_t cap = 0;
    {
      std::lock_guard<std::mutex> g(p->samMu);
      if (!p->samBufs.empty()) {
        pinned = p->samBufs.back().first;
        cap = p->samBufs.back().second;
        p->samBufs.pop_back();
      }
    }
    try {
      for (;;) {
        Job j;
        {
          std::unique_lock<std::mutex> g(mu);
          cv.wait(g, [&] { return failed || !jobs.empty() || noMoreJobs; });
          if (failed || jobs.empty()) break;
          j = std::move(jobs.front());
          jobs.pop_front();
        }
        const auto t0 = Clock::now();
        gwa_batch_t *b = nullptr;
        int rc = 0;
        uint32_t nr = 0;
        auto t1 = t0;
        if (j.format == 1) {  // FASTQ: the text itself goes to the device, fields located there
          nr = (uint32_t)j.starts.size();
          rc = gwa::batchCreateFastq(ix, &p->cfg, j.text->data() + j.tb, j.te - j.tb, j.starts.data(), nr, &b);
        } else {  // FASTA reads (multi-line records): parsed on the host
          gwa_read_buf_t parsed{};
          uint64_t used = 0;
          if (gwa_reads_parse(j.text->data() + j.tb, j.te - j.tb, j.format, 1, &parsed, &used) != 0)
            throw std::runtime_error(gwa_last_error());
          t1 = Clock::now();
          nr = parsed.reads.n;
          rc = gwa_batch_create(ix, &p->cfg, &parsed.reads, &b);
          gwa_reads_free(&parsed);
        }
        j.text.reset();
        const auto t2 = Clock::now();
        if (rc == 0) rc = gwa_batch_run(b);
        const auto t3 = Clock::now();
        uint64_t size = 0;
        if (rc == 0) {
          try {
            size = gwa::batchSamInto(b, &pinned, &cap);
          } catch (...) {
            gwa_batch_free(b);
            throw;
          }
        }
        const std::string msg = rc != 0 ? std::string(gwa_last_error()) : std::string();
        gwa_batch_free(b);
        if (rc != 0) throw std::runtime_error("batch " + std::to_string(j.id) + ": " + msg);
        const auto t4 = Clock::now();
        output(j.id, pinned, size);
        fileReads += nr;
        ++fileBatches;
        std::lock_guard<std::mutex> g(mu);
        parseS += secs(t0, t1);
        setupS += secs(t1, t2);
        devBusy[(size_t)d] += secs(t2, t3);
        formatS += secs(t3, t4);
        --inflight;
        cv.notify_all();
      }
    } catch (std::exception &e) {
      fail(e.what());
    }
    if (pinned) {
      std::lock_guard<std::mutex> g(p->samMu);
      p->samBufs.emplace_back(pinned, cap);
    }
  }

  void startFile() {
    for (int w = 0; w < p->workersPerDevice; ++w)
      for (size_t d = 0; d < p->ix.size(); ++d) workers.emplace_back(&Run::fileWorker, this, (int)d);
  }

  void start() {
    for (int w = 0; w < p->workersPerDevice; ++w)
      for (size_t d = 0; d < p->ix.size(); ++d) workers.emplace_back(&Run::worker, this, (int)d);
  }

  // consumer side: the result of batch `id` (blocks); false once the run has failed
  bool take(uint64_t id, Result *out) {
    std::unique_lock<std::mutex> g(mu);
    cv.wait(g, [&] { return failed || done.count(id) != 0; });
    if (failed) return false;
    auto it = done.find(id);
    *out = std::move(it->second);
    done.erase(it);
    --inflight;
    cv.notify_all();
    return true;
  }

  void join() {
    finishJobs();
    for (auto &t : workers) t.join();
    workers.clear();
    for (auto &kv : done) gwa_results_free(&kv.second.r);
    done.clear();
  }
};

// 1: gzip (.gz), 2: snappy-java (.snap, R/ReadReaderFactory.java:130-139), 0: plain
int compressedKind(const char *path) {
  const size_t n = strlen(path);
  if (n > 3 && strcmp(path + n - 3, ".gz") == 0) return 1;
  if (n > 5 && strcmp(path + n - 5, ".snap") == 0) return 2;
  return 0;
}

int formatOf(const char *path) {
  std::string s(path);
  if (s.size() > 3 && s.compare(s.size() - 3, 3, ".gz") == 0) s.resize(s.size() - 3);
  else if (s.size() > 5 && s.compare(s.size() - 5, 5, ".snap") == 0) s.resize(s.size() - 5);
  auto ends = [&](const char *x) {
    const size_t n = strlen(x);
    return s.size() >= n && s.compare(s.size() - n, n, x) == 0;
  };
  if (ends(".fa") || ends(".fasta") || ends(".fan")) return 0;
  if (ends(".fastq") || ends(".fq")) return 1;
  throw std::runtime_error(std::string("Unsupported file type: ") + path);
}

// The first record start at or after byte x of a plain read file of `size` bytes (size when none):
// FASTA, a line starting with '>'; FASTQ, a line starting with '@' whose next-but-one line starts
// with '+'.  The FASTQ test is unique: a quality line may start with '@', but two lines below it is
// the next record's sequence line (or header), never a '+' line; sequence lines start with neither.
// A record found this way is one the sequential framing (frameRecords) starts as well.
uint64_t syncRecord(int fd, uint64_t size, uint64_t x, int fmt) {
  if (x == 0 || x >= size) return x >= size ? size : 0;
  uint64_t win = 1ull << 20;
  for (;;) {
    const uint64_t a = x - 1, b = std::min(size, a + win);
    std::string t(b - a, '\0');
    uint64_t got = 0;
    while (got < t.size()) {
      const ssize_t r = ::pread(fd, &t[got], t.size() - got, (off_t)(a + got));
      if (r <= 0) throw std::runtime_error("read error while locating a shard boundary");
      got += (uint64_t)r;
    }
    const bool atEnd = b == size;
    // line starts from x on: x itself when byte x - 1 ends a line
    size_t p = 1;
    if (t[0] != '\n') {
      const size_t nl = t.find('\n', 1);
      if (nl == std::string::npos) {
        if (atEnd) return size;
        win *= 4;
        continue;
      }
      p = nl + 1;
    }
    bool more = false;
    while (p < t.size()) {
      if (fmt == 0 ? t[p] == '>' : t[p] == '@') {
        if (fmt == 0) return a + p;
        const size_t n1 = t.find('\n', p), n2 = n1 == std::string::npos ? n1 : t.find('\n', n1 + 1);
        if (n2 == std::string::npos || n2 + 1 >= t.size()) {
          if (atEnd) return size;  // no complete record follows
          more = true;
          break;
        }
        if (t[n2 + 1] == '+') return a + p;
      }
      const size_t nl = t.find('\n', p);
      if (nl == std::string::npos) {
        if (atEnd) return size;
        more = true;
        break;
      }
      p = nl + 1;
    }
    if (!more && atEnd) return size;
    win *= 4;
  }
}

}  // namespace

extern "C" {

int gwa_pipeline_open(gwa_index_t *const *ix, int n_ix, const gwa_config_t *cfg, uint32_t batch_reads,
                      int workers_per_device, gwa_pipeline_t **out) {
  try {
    if (n_ix < 1) throw std::runtime_error("gwa_pipeline_open: no index handle");
    if (cfg->strategy < 0 || cfg->strategy > 3) throw std::runtime_error("unknown strategy");
    auto *p = new gwa_pipeline();
    p->ix.assign(ix, ix + n_ix);
    p->cfg = *cfg;
    p->batchReads = batch_reads ? batch_reads : (1u << 20);
    p->workersPerDevice = workers_per_device > 0 ? workers_per_device : 3;
    *out = p;
    return 0;
  } catch (std::exception &e) {
    return gwa_fail_message(e.what());
  }
}

void gwa_pipeline_close(gwa_pipeline_t *p) { delete p; }

int gwa_pipeline_stats(const gwa_pipeline_t *p, gwa_pipeline_stats_t *st) {
  *st = p->stats;
  return 0;
}

int gwa_pipeline_align(gwa_pipeline_t *p, const gwa_reads_t *reads, gwa_results_t *out) {
  Run run(p);
  std::thread feeder;
  try {
    const auto t0 = Clock::now();
    const uint32_t n = reads->n;
    const uint64_t nb = ((uint64_t)n + p->batchReads - 1) / p->batchReads;
    run.start();
    feeder = std::thread([&] {
      for (uint64_t i = 0; i < nb; ++i) {
        Job j;
        j.id = i;
        const uint32_t a = (uint32_t)(i * p->batchReads), c = (uint32_t)std::min<uint64_t>(p->batchReads, n - a);
        j.reads = *reads;
        j.reads.n = c;
        j.reads.name_off = reads->name_off + a;
        j.reads.seq_off = reads->seq_off + a;
        j.reads.qual_off = reads->qual ? reads->qual_off + a : nullptr;
        j.reads.qual_null = reads->qual && reads->qual_null ? reads->qual_null + a : nullptr;
        if (!run.push(std::move(j))) break;
      }
      run.finishJobs();
    });
    std::vector<Result> parts;
    bool ok = true;
    for (uint64_t i = 0; i < nb && ok; ++i) {
      Result r;
      ok = run.take(i, &r);
      if (ok) parts.push_back(std::move(r));
    }
    feeder.join();
    run.join();
    if (!ok) {
      for (auto &r : parts) gwa_results_free(&r.r);
      throw std::runtime_error(run.err);
    }
    uint64_t total = 0;
    for (auto &r : parts) total += r.r.sam_len;
    out->n_reads = n;
    out->records = nullptr;
    out->n_records = 0;
    out->paired = 0;
    out->sam = (char *)malloc(total + 1);
    out->sam_len = total;
    out->line_off = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)n + 1));
    uint64_t pos = 0, ri = 0;
    for (auto &r : parts) {
      memcpy(out->sam + pos, r.r.sam, r.r.sam_len);
      for (uint32_t k = 0; k < r.r.n_reads; ++k) out->line_off[ri++] = pos + r.r.line_off[k];
      pos += r.r.sam_len;
      gwa_results_free(&r.r);
    }
    out->line_off[n] = pos;
    out->sam[total] = 0;
    p->stats = gwa_pipeline_stats_t{};
    p->stats.reads = n;
    p->stats.batches = nb;
    p->stats.wall_s = secs(t0, Clock::now());
    p->stats.read_s = 0;
    for (size_t d = 0; d < p->ix.size() && d < 16; ++d) p->stats.device_kernel_s[d] = run.devBusy[d];
    return 0;
  } catch (std::exception &e) {
    run.fail(e.what());  // (wakes a feeder blocked in push)
    if (feeder.joinable()) feeder.join();
    run.join();
    return gwa_fail_message(e.what());
  }
}

int gwa_reads_shard_range(const char *path, uint32_t shard, uint32_t nshards, uint64_t *begin, uint64_t *end) {
  int in = -1;
  try {
    if (nshards == 0 || shard >= nshards) throw std::runtime_error("shard index out of range");
    const int fmt = formatOf(path);
    if (compressedKind(path))
      throw std::runtime_error(std::string("a sharded run needs an uncompressed read file (not .gz / .snap): ") + path);
    in = ::open(path, O_RDONLY);
    if (in < 0) throw std::runtime_error(std::string("cannot open ") + path);
    struct stat st;
    if (::fstat(in, &st) != 0 || !S_ISREG(st.st_mode))
      throw std::runtime_error(std::string("a sharded run needs a regular read file: ") + path);
    const uint64_t size = (uint64_t)st.st_size;
    auto cut = [&](uint64_t s) -> uint64_t {
      if (s == 0) return 0;
      if (s >= nshards) return size;
      return syncRecord(in, size, (uint64_t)((unsigned __int128)size * s / nshards), fmt);
    };
    *begin = cut(shard);
    *end = cut(shard + 1);
    ::close(in);
    return 0;
  } catch (std::exception &e) {
    if (in >= 0) ::close(in);
    return gwa_fail_message(e.what());
  }
}

int gwa_pipeline_align_file(gwa_pipeline_t *p, const char *path, int fd, uint64_t *n_reads) {
  return gwa_pipeline_align_file_range(p, path, fd, 0, ~0ull, n_reads);
}

int gwa_pipeline_align_file_range(gwa_pipeline_t *p, const char *path, int fd, uint64_t begin, uint64_t end,
                                  uint64_t *n_reads) {
  BufPool &pool = p->pool;
  Run run(p);
  gzFile f = nullptr;
  std::unique_ptr<gwa::SnapReader> snap;
  int in = -1;
  try {
    const int fmt = formatOf(path);
    const int ck = compressedKind(path);
    const bool gz = ck != 0;  // (a compressed stream: gzip or snappy-java)
    const bool whole = begin == 0 && end == ~0ull;
    if (gz) {
      if (!whole) throw std::runtime_error(std::string("a byte range needs an uncompressed read file: ") + path);
      if (ck == 1) {
        f = gzopen(path, "rb");
        if (!f) throw std::runtime_error(std::string("cannot open ") + path);
        gzbuffer(f, 1u << 20);
      } else {
        snap.reset(new gwa::SnapReader(path));
      }
    } else {
      in = ::open(path, O_RDONLY);
      if (in < 0) throw std::runtime_error(std::string("cannot open ") + path);
      struct stat st;
      if (::fstat(in, &st) == 0 && S_ISREG(st.st_mode)) end = std::min<uint64_t>(end, (uint64_t)st.st_size);
      if (begin > end) begin = end;
      if (::lseek(in, (off_t)begin, SEEK_SET) < 0) throw std::runtime_error(std::string("cannot seek in ") + path);
    }
    struct stat sb;
    const off_t pos0 = ::lseek(fd, 0, SEEK_CUR);
    run.fd = fd;
    // batches are written at their offsets (pwrite) only to a regular file opened without O_APPEND:
    // pwrite ignores the offset under O_APPEND (Linux) and would append in completion order
    const int fl = ::fcntl(fd, F_GETFL);
    run.seekable = pos0 >= 0 && fl >= 0 && !(fl & O_APPEND) && ::fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode);
    run.base = run.seekable ? (uint64_t)pos0 : 0;
    // chunk size: the whole file when it is smaller than kChunk (plain files; .gz sizes are unknown)
    uint64_t fileBytes = 0;
    {
      struct stat st;
      if (!gz && ::fstat(in, &st) == 0 && S_ISREG(st.st_mode)) fileBytes = end - begin;
    }
    const uint64_t chunk = fileBytes ? std::min<uint64_t>(kChunk, ((fileBytes >> 20) + 1) << 20) : kChunk;
    const uint64_t reserve = std::min<uint64_t>(kReserve, 2 * chunk);
    // Pin the read-text buffers this run keeps in flight (read-ahead, the chunk being framed, the
    // batches in the workers) before it starts -- pinning while batches run stalls their copies in
    // the runtime (measured: FASTQ -> SAM 8 M reads/s with background pinning, 20-25 M with the
    // buffers pinned first) -- as many as the file needs, at most a quarter of the available host
    // memory, kept for later calls.  Beyond them runs use pageable buffers.
    uint64_t pinnedUsable = 0;
    // Buffers pinned by an earlier call for a smaller file cannot hold this file's chunks: they are
    // unpinned, and only the pinned buffers of at least reserve + chunk bytes count.
    {
      const uint64_t nbuf = 4 + (uint64_t)p->ix.size() * (uint64_t)p->workersPerDevice;
      const uint64_t need = fileBytes ? std::min<uint64_t>(nbuf, fileBytes / chunk + 3) : nbuf;
      const uint64_t avail = memAvailable(), capB = avail ? avail / 4 : (8ull << 30);
      const uint64_t bufCap = reserve + chunk;
      uint64_t relN = 0, relB = 0;
      p->pool.releasePinnedBelow(bufCap, &relN, &relB);
      p->pinnedBufs -= std::min(p->pinnedBufs, relN);
      p->pinnedBytes -= std::min(p->pinnedBytes, relB);
      uint64_t usable = p->pool.countPinned(bufCap);
      try {
        while (usable < need && p->pinnedBytes + bufCap <= capB) {
          p->pool.addPinned(bufCap);
          ++p->pinnedBufs;
          ++usable;
          p->pinnedBytes += bufCap;
        }
      } catch (std::exception &) {  // (pinning failed: pageable buffers)
      }
      pinnedUsable = usable;
    }
    const auto t0 = Clock::now();
    double readS = 0, frameS = 0;
    run.startFile();
    // This thread reads the file and frames it into batches of complete records (FASTQ: every
    // record's header offset, from the '\n' positions found on several threads); the workers do the
    // rest.  Only full batches leave a chunk unless the file has ended; the rest carries over.
    // An IO thread reads the file in chunks into pooled pinned buffers, behind `reserve` bytes of
    // room where this thread puts the records carried over from the previous chunk; this thread frames
    // each chunk into batches of complete records (FASTQ: every record's header offset) while the IO
    // thread reads the next.  Only full batches leave a chunk unless the file has ended.
    const unsigned nth = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    struct Chunk {
      std::shared_ptr<TextBuf> buf;
      uint64_t got = 0;
      bool final = false;
    };
    std::mutex qmu;
    std::condition_variable qcv;
    std::deque<Chunk> q;
    bool ioDone = false, stop = false;
    std::string ioErr;
    std::thread io([&] {
      try {
        for (;;) {
          {
            std::unique_lock<std::mutex> g(qmu);
            qcv.wait(g, [&] { return stop || q.size() < 2; });
            if (stop) break;
          }
          Chunk c;
          c.buf = pool.get(reserve + chunk);
          const auto r0 = Clock::now();
          char *dst = c.buf->p + reserve;
          if (snap) {
            c.got = snap->read(dst, chunk);
          } else if (gz) {
            while (c.got < chunk) {
              const int r = gzread(f, dst + c.got, (unsigned)(chunk - c.got));
              if (r < 0) throw std::runtime_error(std::string("read error: ") + path);
              if (r == 0) break;
              c.got += (uint64_t)r;
            }
          } else {  // four preads at a time (the page cache copies in parallel), up to `end`
            const off_t at = ::lseek(in, 0, SEEK_CUR);
            const uint64_t want = std::min<uint64_t>(chunk, end > (uint64_t)at ? end - (uint64_t)at : 0);
            std::atomic<bool> bad{false};
            std::vector<std::thread> th;
            std::vector<uint64_t> gotk(4, 0);
            auto lo = [&](int k) { return want * (uint64_t)k / 4; };
            for (int k = 0; k < 4; ++k)
              th.emplace_back([&, k] {
                const uint64_t part = lo(k + 1) - lo(k);
                uint64_t gk = 0;
                while (gk < part) {
                  const ssize_t r = ::pread(in, dst + lo(k) + gk, (size_t)(part - gk), at + (off_t)(lo(k) + gk));
                  if (r < 0) { bad = true; return; }
                  if (r == 0) break;
                  gk += (uint64_t)r;
                }
                gotk[(size_t)k] = gk;
              });
            for (auto &x : th) x.join();
            if (bad) throw std::runtime_error(std::string("read error: ") + path);
            // the bytes read are contiguous up to the first short part (end of file)
            for (int k = 0; k < 4; ++k) {
              c.got += gotk[(size_t)k];
              if (gotk[(size_t)k] < lo(k + 1) - lo(k)) break;
            }
            ::lseek(in, at + (off_t)c.got, SEEK_SET);
            if ((uint64_t)at + c.got >= end) c.got = std::min<uint64_t>(c.got, end - (uint64_t)at);
          }
          c.final = c.got < chunk || (!gz && (uint64_t)::lseek(in, 0, SEEK_CUR) >= end);
          const double rs = secs(r0, Clock::now());
          std::lock_guard<std::mutex> g(qmu);
          readS += rs;
          const bool fin = c.final;
          q.push_back(std::move(c));
          qcv.notify_all();
          if (fin) break;
        }
      } catch (std::exception &e) {
        std::lock_guard<std::mutex> g(qmu);
        ioErr = e.what();
      }
      std::lock_guard<std::mutex> g(qmu);
      ioDone = true;
      qcv.notify_all();
    });
    std::shared_ptr<TextBuf> prev;
    uint64_t carryFrom = 0, carryLen = 0, id = 0;
    bool ok = true;
    std::vector<uint64_t> starts;
    try {
      for (;;) {
        Chunk c;
        {
          std::unique_lock<std::mutex> g(qmu);
          qcv.wait(g, [&] { return !q.empty() || ioDone; });
          if (q.empty()) {
            if (!ioErr.empty()) throw std::runtime_error(ioErr);
            break;
          }
          c = std::move(q.front());
          q.pop_front();
          qcv.notify_all();
        }
        const auto f0 = Clock::now();
        // the text of this round: the carried records, then the chunk
        std::shared_ptr<TextBuf> buf = c.buf;
        uint64_t base = reserve - carryLen;
        if (carryLen > reserve) {  // more carry than room: one buffer holding both
          buf = pool.get(carryLen + c.got + 64);
          memcpy(buf->p + carryLen, c.buf->p + reserve, c.got);
          base = 0;
        }
        if (carryLen) memcpy(buf->p + base, prev->p + carryFrom, carryLen);
        prev.reset();
        const char *t = buf->p + base;
        const uint64_t len = carryLen + c.got;
        buf->size = base + len;
        const bool final = c.final;
        // all complete records of the text: their header offsets (FASTQ) and the end of the last
        starts.clear();
        uint64_t nrec = 0, done = 0;
        bool fast = false;
        if (fmt == 1 && !final) {  // no '\r', no blank line: record k starts after newline 4k - 1
          std::vector<uint64_t> cnt(nth);
          std::vector<char> bl(nth), cr(nth);
          std::vector<std::thread> th;
          for (unsigned k = 0; k < nth; ++k)
            th.emplace_back([&, k] {
              bool b0, c0;
              gwa::newlineCount(t, len * k / nth, len * (k + 1) / nth, &cnt[k], &b0, &c0);
              bl[k] = b0;
              cr[k] = c0;
            });
          for (auto &x : th) x.join();
          bool clean = len > 0 && t[0] != '\n';
          uint64_t tot = 0;
          std::vector<uint64_t> g0(nth);
          for (unsigned k = 0; k < nth; ++k) {
            clean = clean && !bl[k] && !cr[k];
            g0[k] = tot;
            tot += cnt[k];
          }
          if (clean) {
            fast = true;
            nrec = tot / 4;
            starts.resize(nrec + 1);
            starts[0] = 0;
            th.clear();
            for (unsigned k = 0; k < nth; ++k)
              th.emplace_back([&, k] {
                gwa::recordStartsFromNewlines(t, len * k / nth, len * (k + 1) / nth, g0[k], starts.data(), nrec + 1);
              });
            for (auto &x : th) x.join();
            done = starts[nrec];  // the start of the first incomplete record
            starts.resize(nrec);
          }
        }
        if (!fast) done = gwa::frameRecords(t, len, fmt, final, ~0ull, &nrec, fmt == 1 ? &starts : nullptr);
        frameS += secs(f0, Clock::now());
        // batches of batchReads records; the records after the last full batch carry over
        const uint64_t B = p->batchReads;
        const uint64_t full = final ? (nrec + B - 1) / B : nrec / B;
        uint64_t pos = 0;
        if (fmt == 1) {
          for (uint64_t k = 0; k < full && ok; ++k) {
            const uint64_t r0i = k * B, r1i = std::min(nrec, r0i + B);
            Job j;
            j.id = id++;
            j.text = buf;
            j.tb = base + starts[r0i];
            j.te = base + (r1i < nrec ? starts[r1i] : done);
            j.format = fmt;
            j.starts.assign(starts.begin() + (long)r0i, starts.begin() + (long)r1i);
            const uint64_t s0 = starts[r0i];
            for (auto &x : j.starts) x -= s0;
            if (!run.push(std::move(j))) ok = false;
          }
          pos = (full * B < nrec) ? starts[full * B] : done;
        } else {  // FASTA: frame again batch by batch (record starts are not kept)
          uint64_t left = full == 0 ? 0 : nrec;
          while (left > 0 && ok) {
            uint64_t nr = 0;
            const uint64_t e = pos + gwa::frameRecords(t + pos, len - pos, fmt, final, std::min<uint64_t>(B, left), &nr, nullptr);
            if (nr == 0) break;
            if (nr < B && !final) break;
            Job j;
            j.id = id++;
            j.text = buf;
            j.tb = base + pos;
            j.te = base + e;
            j.format = fmt;
            if (!run.push(std::move(j))) ok = false;
            pos = e;
            left -= nr;
          }
        }
        if (!ok || final) break;
        prev = buf;
        carryFrom = base + pos;
        carryLen = len - pos;
      }
    } catch (...) {
      {
        std::lock_guard<std::mutex> g(qmu);
        stop = true;
        qcv.notify_all();
      }
      io.join();
      throw;
    }
    {
      std::lock_guard<std::mutex> g(qmu);
      stop = true;
      qcv.notify_all();
    }
    io.join();
    q.clear();
    if (in >= 0) ::close(in);
    in = -1;
    run.finishJobs();
    for (auto &t : run.workers) t.join();
    run.workers.clear();
    if (f) gzclose(f);
    f = nullptr;
    if (run.failed) throw std::runtime_error(run.err);
    if (run.seekable) ::lseek(fd, (off_t)(run.base + run.nextOff), SEEK_SET);
    const uint64_t n = run.fileReads;
    if (n_reads) *n_reads = n;
    gwa_pipeline_stats_t &st = p->stats;
    st = gwa_pipeline_stats_t{};
    st.reads = n;
    st.batches = run.fileBatches;
    st.pinned_bufs = pinnedUsable;
    st.wall_s = secs(t0, Clock::now());
    st.read_s = readS;
    st.frame_s = frameS;
    for (size_t d = 0; d < p->ix.size() && d < 16; ++d) st.device_kernel_s[d] = run.devBusy[d];
    st.parse_s = run.parseS;
    st.setup_s = run.setupS;
    st.format_s = run.formatS;
    st.write_s = run.writeS;
    st.order_wait_s = run.waitS;
    return 0;
  } catch (std::exception &e) {
    run.fail(e.what());
    run.join();
    if (f) gzclose(f);
    if (in >= 0) ::close(in);
    return gwa_fail_message(e.what());
  }
}

}  // extern "C"
