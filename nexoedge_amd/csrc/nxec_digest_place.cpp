// Where nxec_encode_host_md5 computes its digests (include/nxec.h §2, §6b).
//
// The unmodified write path calls RSCode::encode once per stripe and then
// Chunk::computeMD5 on each of the n chunks (chunk_manager.cc:99 -> :175);
// the agent's repair hashes its outputs the same way (agent.cc:339 -> :342).
// Two places can hash those chunks, and each wins in its own regime:
//
//  * the GPU, in the coding pass itself (k_gather_md5, nxec_runtime.hip
//    "digest rounds"): one lane per chunk, and an MD5 chain is serial -- one
//    VALU op per 4 cycles on a wave alone, ~9-12 ms per MiB whatever else
//    runs -- so a call returns no sooner than that, but thousands of chains
//    run at once and they cost the host nothing;
//  * the host cores (OpenSSL, as the reference hashes): ~0.8 GB/s per core,
//    so the n chunks of one 1 MiB stripe spread over the pool finish in ~2 ms,
//    but the cores are few (the GPU box grants 16 CPUs' worth of time) and
//    the callers need them too (rs.cc:80's copy, page faults, the proxy).
//
// NXEC_DIGEST_PLACE=auto (the default) hashes on the host pool while the
// calling threads are no more than the CPUs the process may use (cgroup
// quota / affinity mask), and moves the calls onto the GPU as callers
// multiply beyond that (DigestHost::decide_auto): few callers get a stripe's
// digests in ~2 ms instead of a ~12 ms chain, many callers get the GPU's
// rate, which grows with them, instead of CPUs they would starve.
// `gpu` and `host` pin the placement (A/B, tests).  Whatever the placement
// the coding itself runs on the GPU, and the digests are RFC 1321 MD5 of the
// same bytes.
#include <openssl/evp.h>
#include <sched.h>
#include <unistd.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nxec.h"
#include "nxec_internal.h"

namespace nxec {
namespace {

std::atomic<int> g_mode{-1};
std::atomic<unsigned long long> g_host_calls{0}, g_gpu_calls{0};

int env_mode() {
  const char *e = std::getenv("NXEC_DIGEST_PLACE");
  if (!e || !e[0] || std::strcmp(e, "auto") == 0) return NXEC_DIGEST_AUTO;
  if (std::strcmp(e, "gpu") == 0 || std::strcmp(e, "1") == 0) return NXEC_DIGEST_GPU;
  if (std::strcmp(e, "host") == 0 || std::strcmp(e, "2") == 0) return NXEC_DIGEST_HOST;
  return NXEC_DIGEST_AUTO;
}

int mode() {
  int m = g_mode.load(std::memory_order_relaxed);
  if (m < 0) {
    int want = env_mode(), expected = -1;
    g_mode.compare_exchange_strong(expected, want);
    m = g_mode.load(std::memory_order_relaxed);
  }
  return m;
}

// the cgroup directories holding this process's CPU quota, innermost first:
// /proc/self/cgroup names the process's own (possibly nested) cgroup, and the
// effective limit is the smallest quota on the way up to the root
std::vector<std::string> cgroup_dirs(bool v2) {
  std::vector<std::string> dirs;
  FILE *f = std::fopen("/proc/self/cgroup", "r");
  if (!f) return dirs;
  char line[4096];
  std::string rel;
  while (std::fgets(line, sizeof(line), f)) {
    std::string l(line);
    while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
    const size_t a = l.find(':'), b = a == std::string::npos ? a : l.find(':', a + 1);
    if (b == std::string::npos) continue;
    const std::string ctrl = l.substr(a + 1, b - a - 1), path = l.substr(b + 1);
    if (v2 ? (l.compare(0, 2, "0:") == 0 && ctrl.empty())
           : (ctrl == "cpu" || ctrl.find("cpu,") == 0 || ctrl.find(",cpu,") != std::string::npos ||
              (ctrl.size() > 4 && ctrl.compare(ctrl.size() - 4, 4, ",cpu") == 0))) {
      rel = path;
      break;
    }
  }
  std::fclose(f);
  if (rel.empty() || rel[0] != '/') rel = "/";
  const std::string base = v2 ? "/sys/fs/cgroup" : "/sys/fs/cgroup/cpu";
  for (std::string r = rel;;) {
    dirs.push_back(base + (r == "/" ? "" : r));
    if (r == "/" || r.empty()) break;
    const size_t cut = r.find_last_of('/');
    r = cut == 0 ? "/" : r.substr(0, cut);
  }
  return dirs;
}

// quota / period of one cgroup directory, or 0 when it sets none
double cgroup_quota(const std::string &dir, bool v2) {
  double cpus = 0;
  if (v2) {
    if (FILE *f = std::fopen((dir + "/cpu.max").c_str(), "r")) {
      char q[32] = {0};
      long per = 0;
      if (std::fscanf(f, "%31s %ld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0)
        cpus = std::atof(q) / static_cast<double>(per);
      std::fclose(f);
    }
  } else if (FILE *g = std::fopen((dir + "/cpu.cfs_quota_us").c_str(), "r")) {
    long quota = -1, per = 0;
    if (std::fscanf(g, "%ld", &quota) == 1 && quota > 0)
      if (FILE *h = std::fopen((dir + "/cpu.cfs_period_us").c_str(), "r")) {
        if (std::fscanf(h, "%ld", &per) == 1 && per > 0) cpus = static_cast<double>(quota) / static_cast<double>(per);
        std::fclose(h);
      }
    std::fclose(g);
  }
  return cpus;
}

// CPUs this process may use: the smallest cgroup quota (cpu.max, v2; cfs
// quota, v1) from the process's own cgroup up to the root, capped by the
// affinity mask
double cpu_budget() {
  double cpus = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
  const bool v2 = access("/sys/fs/cgroup/cgroup.controllers", F_OK) == 0;
  for (const std::string &d : cgroup_dirs(v2)) {
    const double q = cgroup_quota(d, v2);
    if (q > 0) cpus = std::min(cpus > 0 ? cpus : 1e9, q);
  }
  return cpus > 0 ? cpus : 1;
}

double now_ns(clockid_t c) {
  timespec ts;
  clock_gettime(c, &ts);
  return static_cast<double>(ts.tv_sec) * 1e9 + static_cast<double>(ts.tv_nsec);
}

// Group of digests one call waits for.
struct Group {
  int left = 0;
};

struct Task {
  const unsigned char *p;
  size_t len;
  unsigned char *out;
  Group *g;
};

class DigestHost {
 public:
  static DigestHost &get() {
    static DigestHost h;
    return h;
  }

  int threads() const { return nthreads_; }
  double cpus() const { return cpus_; }
  double hostCallers() const { return host_callers_; }

  // Auto placement of a call hashing `bytes` in chunks of `len` (true: the
  // host pool, its bytes then reserved).  The pool is CPU-bound (~16 ms of
  // CPU per RS(10,4) 1 MiB stripe, ~1000 stripes/s on 16 CPUs) but quick
  // (~2 ms a stripe); the GPU's chains take ~12 ms a call whatever the load
  // but cost the host nothing, so the GPU's rate grows with the callers.
  // Measured on the box (profiles/r03_dropin_place.jsonl) the pool wins up
  // to about as many calling threads as CPUs and the GPU from about twice
  // that, because beyond the CPUs the pool's hashing starves the callers' own
  // host work (rs.cc:80's copy, the proxy).  So: the calling threads seen in
  // the last 200 ms are counted (N); up to H = the CPU budget
  // (NXEC_DIGEST_HOST_CALLERS) every call goes to the pool, from 2H on none,
  // in between the share (2H - N) / N, dithered.  A call also stays off the
  // pool while its queue would outlast the GPU's latency.
  bool decide_auto(int64_t bytes, int64_t len) {
    const double w = now_ns(CLOCK_MONOTONIC);
    std::lock_guard<std::mutex> lk(mu_);
    if (tl_slot_ < 0 && seen_.size() < 65536) {
      tl_slot_ = static_cast<int>(seen_.size());
      seen_.push_back(0);
    }
    if (tl_slot_ >= 0) seen_[tl_slot_] = w;
    if (w - win_w0_ >= 20e6) {
      int n = 0;
      for (double t : seen_) n += w - t < 200e6;
      callers_ = std::max(1, n);
      share_ = callers_ <= host_callers_ ? 1.0 : std::max(0.0, (2.0 * host_callers_ - callers_) / callers_);
      win_w0_ = w;
    }
    const double lg = (gpu_ms_per_mib_ * static_cast<double>(len) / (1 << 20) + 0.5) * 1e6;  // ns
    const double hashers = std::max(1.0, std::min(static_cast<double>(nthreads_ + 1), cpus_));
    if (static_cast<double>(backlog_ + bytes) / (rate_ * hashers) >= lg) return false;
    dither_ += share_;
    if (dither_ < 1.0) return false;
    dither_ -= 1.0;
    backlog_ += bytes;
    return true;
  }
  void reserve(int64_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    backlog_ += bytes;
  }
  void unreserve(int64_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    backlog_ -= bytes;
  }
  // a GPU-placed call's latency (the pool's queue guard)
  void gpu_observe(int64_t len, double ms) {
    if (len < (64 << 10)) return;  // launch-bound: says nothing of the chain rate
    std::lock_guard<std::mutex> lk(mu_);
    const double per_mib = std::max(0.0, ms - 0.5) * (1 << 20) / static_cast<double>(len);
    gpu_ms_per_mib_ += (per_mib - gpu_ms_per_mib_) * 0.125;
  }

  // queues one digest (its bytes already reserved)
  void submit(Group *g, const unsigned char *p, size_t len, unsigned char *out) {
    start();
    {
      std::lock_guard<std::mutex> lk(mu_);
      g->left++;
      q_.push_back({p, len, out, g});
    }
    cv_.notify_one();
  }

  // the caller hashes queued digests (its own or others') until its group is done
  void finish(Group *g) {
    std::unique_lock<std::mutex> lk(mu_);
    while (g->left > 0) {
      if (!q_.empty()) {
        Task t = q_.front();
        q_.pop_front();
        lk.unlock();
        run(t);
        lk.lock();
        continue;
      }
      done_cv_.wait(lk, [&] { return g->left == 0 || !q_.empty(); });
    }
  }

 private:
  DigestHost() {
    int nt = 16;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) nt = std::min(nt, CPU_COUNT(&set));
    if (const char *e = std::getenv("NXEC_DIGEST_THREADS")) nt = std::atoi(e);
    nthreads_ = std::max(0, std::min(nt, 256));
    cpus_ = cpu_budget();
    if (const char *e = std::getenv("NXEC_DIGEST_CPUS")) cpus_ = std::max(1.0, std::atof(e));
    host_callers_ = tuning().digest_host_callers > 0 ? tuning().digest_host_callers : cpus_;
    md_ = EVP_MD_fetch(nullptr, "MD5", nullptr);
  }
  ~DigestHost() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
    if (md_) EVP_MD_free(md_);
  }
  void start() {
    std::call_once(started_, [this] {
      for (int i = 0; i < nthreads_; i++) workers_.emplace_back([this] { loop(); });
    });
  }
  void run(const Task &t) {
    bool clean;  // no more hashers than CPUs: the measured time is the hash's own
    {
      std::lock_guard<std::mutex> lk(mu_);
      clean = ++hashing_ <= cpus_;
    }
    const auto t0 = std::chrono::steady_clock::now();
    unsigned int olen = 16;
    if (!md_ || EVP_Digest(t.p, t.len, t.out, &olen, md_, nullptr) != 1)
      EVP_Digest(t.p, t.len, t.out, &olen, EVP_md5(), nullptr);
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    {
      std::lock_guard<std::mutex> lk(mu_);
      clean = clean && hashing_ <= cpus_;
      hashing_--;
      backlog_ -= static_cast<int64_t>(t.len);
      if (clean && t.len >= (64 << 10) && ns > 0) rate_ += (static_cast<double>(t.len) / ns - rate_) * 0.0625;
      t.g->left--;
    }
    done_cv_.notify_all();
  }
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (stop_ && q_.empty()) return;
      Task t = q_.front();
      q_.pop_front();
      lk.unlock();
      run(t);
      lk.lock();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Task> q_;
  std::vector<std::thread> workers_;
  std::once_flag started_;
  EVP_MD *md_ = nullptr;
  int nthreads_ = 0;
  int hashing_ = 0;              // digests being computed right now
  double cpus_ = 1;              // the process's CPU budget
  double win_w0_ = 0;            // current window's start
  std::vector<double> seen_;     // per calling thread: its last call (ns)
  int callers_ = 1;              // calling threads seen in the last 200 ms
  double host_callers_ = 16;     // H (see decide_auto)
  double share_ = 1;             // share of the calls for the pool (last window)
  double dither_ = 0;
  static thread_local int tl_slot_;
  bool stop_ = false;
  int64_t backlog_ = 0;          // bytes reserved, queued or being hashed
  double rate_ = 0.8;            // bytes per ns per thread (EWMA of measured digests)
  double gpu_ms_per_mib_ = 12.0; // GPU digest-call latency per MiB of chunk length (EWMA)
};

thread_local int DigestHost::tl_slot_ = -1;

}  // namespace

bool digest_place_host(int64_t len, int nhash) {
  const int m = mode();
  if (m == NXEC_DIGEST_GPU) return false;
  DigestHost &h = DigestHost::get();
  const int64_t bytes = len * nhash;
  if (m == NXEC_DIGEST_AUTO) return h.decide_auto(bytes, len);
  h.reserve(bytes);
  return true;
}

double digest_clock_ns() { return now_ns(CLOCK_MONOTONIC); }


void digest_gpu_observe(int64_t len, double ms) {
  g_gpu_calls.fetch_add(1, std::memory_order_relaxed);
  DigestHost::get().gpu_observe(len, ms);
}

// the call of nxec_encode_host_md5 placed on the host: the inputs' digests
// start at once and overlap the GPU's coding pass, the outputs' follow it
int encode_host_md5_host_digests(int len, int k, int rows, const unsigned char *coeffs,
                                 const unsigned char *const *data, unsigned char *const *coding,
                                 unsigned char *md5_data, unsigned char *md5_code) {
  g_host_calls.fetch_add(1, std::memory_order_relaxed);
  DigestHost &h = DigestHost::get();
  Group g;
  for (int j = 0; md5_data && j < k; j++) h.submit(&g, data[j], static_cast<size_t>(len), md5_data + 16 * j);
  const int rc = nxec_encode_host(len, k, rows, coeffs, data, coding);
  if (md5_code) {
    if (rc == NXEC_OK)
      for (int r = 0; r < rows; r++) h.submit(&g, coding[r], static_cast<size_t>(len), md5_code + 16 * r);
    else
      h.unreserve(static_cast<int64_t>(len) * rows);
  }
  h.finish(&g);
  return rc;
}

}  // namespace nxec

extern "C" {

int nxec_set_digest_placement(int m) {
  if (m != NXEC_DIGEST_AUTO && m != NXEC_DIGEST_GPU && m != NXEC_DIGEST_HOST)
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_set_digest_placement: mode %d", m);
  const int prev = nxec::mode();
  nxec::g_mode.store(m);
  return prev;
}

int nxec_digest_placement(void) { return nxec::mode(); }

int nxec_digest_place_params(double *cpu_budget, double *host_callers) {
  nxec::DigestHost &h = nxec::DigestHost::get();
  if (cpu_budget) *cpu_budget = h.cpus();
  if (host_callers) *host_callers = h.hostCallers();
  return NXEC_OK;
}

int nxec_digest_place_stats(unsigned long long *host_calls, unsigned long long *gpu_calls, int *host_threads) {
  if (host_calls) *host_calls = nxec::g_host_calls.load();
  if (gpu_calls) *gpu_calls = nxec::g_gpu_calls.load();
  if (host_threads) *host_threads = nxec::DigestHost::get().threads();
  return NXEC_OK;
}

}  // extern "C"
