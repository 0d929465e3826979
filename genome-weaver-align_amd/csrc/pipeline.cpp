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
// and the caller, which writes the results in batch order.  With two workers per device, one
// worker's set-up and SAM formatting overlap the other's kernels (gwa_index serialises the kernels
// of its batches, gwa_api.cpp runMu).  At most `depth` batches are in flight, which bounds memory.
#include <zlib.h>

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
#include <unistd.h>
#include <vector>

#include "../../include/gwa.h"

extern "C" int gwa_fail_message(const char *msg);  // gwa_api.cpp

namespace gwa {
uint64_t frameRecords(const char *t, uint64_t len, int format, bool final, uint64_t maxRec, uint64_t *nRec);
}

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// One unit of work: either reads already in memory (a gwa_reads_t slice) or a framed slice of file
// text that the worker parses itself.
struct Job {
  uint64_t id = 0;
  gwa_reads_t reads{};                 // in-memory reads (text == nullptr)
  std::shared_ptr<std::string> text;   // or: file text holding complete records [tb, te)
  uint64_t tb = 0, te = 0;
  int format = 1;
};

struct Result {
  gwa_results_t r{};
  uint32_t n = 0;
};

}  // namespace

struct gwa_pipeline {
  std::vector<gwa_index_t *> ix;
  gwa_config_t cfg{};
  uint32_t batchReads = 1u << 20;
  int workersPerDevice = 2;
  gwa_pipeline_stats_t stats{};
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

void writeAll(int fd, const char *p, uint64_t n) {
  while (n > 0) {
    const ssize_t w = ::write(fd, p, (size_t)std::min<uint64_t>(n, 1ull << 30));
    if (w < 0) throw std::runtime_error("write to the SAM output failed");
    p += w;
    n -= (uint64_t)w;
  }
}

int formatOf(const char *path) {
  std::string s(path);
  if (s.size() > 3 && s.compare(s.size() - 3, 3, ".gz") == 0) s.resize(s.size() - 3);
  auto ends = [&](const char *x) {
    const size_t n = strlen(x);
    return s.size() >= n && s.compare(s.size() - n, n, x) == 0;
  };
  if (ends(".fa") || ends(".fasta") || ends(".fan")) return 0;
  if (ends(".fastq") || ends(".fq")) return 1;
  throw std::runtime_error(std::string("Unsupported file type: ") + path);
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
    p->workersPerDevice = workers_per_device > 0 ? workers_per_device : 2;
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
  try {
    const auto t0 = Clock::now();
    const uint32_t n = reads->n;
    const uint64_t nb = ((uint64_t)n + p->batchReads - 1) / p->batchReads;
    run.start();
    std::thread feeder([&] {
      for (uint64_t i = 0; i < nb; ++i) {
        Job j;
        j.id = i;
        const uint32_t a = (uint32_t)(i * p->batchReads), c = (uint32_t)std::min<uint64_t>(p->batchReads, n - a);
        j.reads = *reads;
        j.reads.n = c;
        j.reads.name_off = reads->name_off + a;
        j.reads.seq_off = reads->seq_off + a;
        j.reads.qual_off = reads->qual ? reads->qual_off + a : nullptr;
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
    p->stats.reads = n;
    p->stats.batches = nb;
    p->stats.wall_s = secs(t0, Clock::now());
    p->stats.read_s = 0;
    for (size_t d = 0; d < p->ix.size() && d < 16; ++d) p->stats.device_kernel_s[d] = run.devBusy[d];
    return 0;
  } catch (std::exception &e) {
    run.fail(e.what());
    run.join();
    return gwa_fail_message(e.what());
  }
}

int gwa_pipeline_align_file(gwa_pipeline_t *p, const char *path, int fd, uint64_t *n_reads) {
  Run run(p);
  try {
    const int fmt = formatOf(path);
    gzFile f = gzopen(path, "rb");
    if (!f) throw std::runtime_error(std::string("cannot open ") + path);
    gzbuffer(f, 1u << 20);
    const auto t0 = Clock::now();
    double readS = 0;
    run.start();
    std::atomic<uint64_t> nJobs{0};
    std::atomic<bool> readerDone{false};
    std::string readErr;
    std::thread reader([&] {
      try {
        const uint64_t chunk = 256ull << 20;
        std::string carry;
        uint64_t id = 0;
        for (;;) {
          auto buf = std::make_shared<std::string>();
          buf->swap(carry);
          const size_t old = buf->size();
          buf->resize(old + chunk);
          const auto r0 = Clock::now();
          const int got = gzread(f, &(*buf)[old], (unsigned)chunk);
          readS += secs(r0, Clock::now());
          if (got < 0) throw std::runtime_error(std::string("read error: ") + path);
          buf->resize(old + (size_t)got);
          const bool final = got == 0;
          uint64_t pos = 0;
          while (pos < buf->size()) {
            uint64_t nrec = 0;
            const uint64_t e = pos + gwa::frameRecords(buf->data() + pos, buf->size() - pos, fmt, final, p->batchReads, &nrec);
            if (nrec == 0) {
              if (final) pos = buf->size();  // trailing text without records
              break;
            }
            if (nrec < p->batchReads && !final) break;  // wait for more text: full batches only
            Job j;
            j.id = id++;
            j.text = buf;
            j.tb = pos;
            j.te = e;
            j.format = fmt;
            if (!run.push(std::move(j))) return;
            nJobs = id;
            pos = e;
          }
          carry.assign(buf->data() + pos, buf->size() - pos);
          if (final) break;
        }
      } catch (std::exception &e) {
        readErr = e.what();
        run.fail(e.what());
      }
      readerDone = true;
      run.finishJobs();
      std::lock_guard<std::mutex> g(run.mu);
      run.cv.notify_all();
    });
    // write batch results in order as they complete
    uint64_t next = 0, n = 0;
    bool ok = true;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(run.mu);
        run.cv.wait(g, [&] { return run.failed || run.done.count(next) != 0 || (readerDone && next >= nJobs); });
        if (run.failed) { ok = false; break; }
        if (run.done.count(next) == 0) break;  // reader finished and every batch was written
      }
      Result r;
      if (!run.take(next, &r)) { ok = false; break; }
      try {
        writeAll(fd, r.r.sam, r.r.sam_len);
      } catch (std::exception &e) {
        gwa_results_free(&r.r);
        run.fail(e.what());
        ok = false;
        break;
      }
      n += r.n;
      gwa_results_free(&r.r);
      ++next;
    }
    reader.join();
    run.join();
    gzclose(f);
    if (!ok) throw std::runtime_error(run.err);
    if (n_reads) *n_reads = n;
    p->stats.reads = n;
    p->stats.batches = next;
    p->stats.wall_s = secs(t0, Clock::now());
    p->stats.read_s = readS;
    for (size_t d = 0; d < p->ix.size() && d < 16; ++d) p->stats.device_kernel_s[d] = run.devBusy[d];
    return 0;
  } catch (std::exception &e) {
    run.fail(e.what());
    run.join();
    return gwa_fail_message(e.what());
  }
}

}  // extern "C"
