// libnxec's context and plumbing: the thread's last error, the deployment
// settings, the host worker pool and pinned-memory views, contexts with their
// staging slots, the library's own kernel timers, and the device / memory /
// stream helpers of include/nxec.h §2.
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include <sched.h>

#include "nxec_runtime.h"

namespace nxec {

namespace {
thread_local std::string g_last_error;
}  // namespace

const std::string &last_error() { return g_last_error; }
void restore_error(const std::string &msg) { g_last_error = msg; }

// Copy into pinned staging.  The NT-staging probe (nxec_tuning.h) uses
// streaming (non-temporal) stores: the staging lines are never read by the
// CPU, so skipping their read-for-ownership halves the DRAM traffic of a
// large gather (tools/microbench/host_copy.cc measures both on the box); it
// did not raise the measured rates, so the product copies plainly.
void stage_copy(void *dst, const void *src, size_t n) {
  uint8_t *d = static_cast<uint8_t *>(dst);
  const uint8_t *sp = static_cast<const uint8_t *>(src);
  if (!tuning().nt_staging || n < 4096) {
    std::memcpy(d, sp, n);
    return;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15;
  std::memcpy(d, sp, head);
  size_t i = head;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(sp + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(sp + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(sp + i + 32));
    const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i *>(sp + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 48), e);
  }
  _mm_sfence();  // streamed lines visible before the copy engine is told to read them
  std::memcpy(d + i, sp + i, n - i);
}

// Copy out of pinned staging into a caller's buffer.  With the NT-staging
// probe the caller's lines are written with streaming stores too (no
// read-for-ownership of a destination the CPU does not read next): the
// read pipeline's host DRAM traffic per byte drops from ~4 to ~3 passes.
void unstage_copy(void *dst, const void *src, size_t n) {
  uint8_t *d = static_cast<uint8_t *>(dst);
  const uint8_t *sp = static_cast<const uint8_t *>(src);
  if (!tuning().nt_staging || n < 4096) {
    std::memcpy(d, sp, n);
    return;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15;
  std::memcpy(d, sp, head);
  size_t i = head;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(sp + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(sp + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(sp + i + 32));
    const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i *>(sp + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 48), e);
  }
  _mm_sfence();
  std::memcpy(d + i, sp + i, n - i);
}

namespace {

// Host worker pool for staging copies (pageable <-> pinned) of the host entry
// points: one memcpy thread moves ~10 GB/s, so a 1 MiB RS(10,4) stripe spends
// most of a call copying.  parallel_for splits a call's copies over the pool;
// the calling thread works too, and concurrent callers share the pool.
class HostPool {
 public:
  // With the lanes probe on (nxec_tuning.h host_lanes) copies into pinned
  // staging and copies out of it have a worker set each, so a pipelined
  // caller's gather and scatter (nxec_decode_frames) do not queue behind each
  // other's helper tasks; otherwise one shared pool (rounds 1-5).
  // One pool per NUMA node of the GPUs served (round 6): its threads run on
  // that node's CPUs, next to the GPU's PCIe root and, by first touch, the
  // staging they fill, instead of wherever the scheduler puts them (the
  // pageable-frames read pipeline: 33 -> 39 GiB/s with its threads on the
  // GPU's node, profiles/r06_frames_ab.jsonl).  Pools are made on first use
  // and live for the process.
  static HostPool &get(HostLane lane, int node) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, HostPool *> pools;
    const int l = lane == HostLane::kOut && tuning().host_lanes ? 1 : 0;
    std::lock_guard<std::mutex> lk(mu);
    HostPool *&p = pools[{node, l}];
    if (!p) p = new HostPool(node);
    return *p;
  }
  // runs fn(i) for i in [0, n), returns when all are done.  The pool serves
  // two jobs at a time (a pipelined caller's gather and scatter,
  // nxec_decode_frames); a caller arriving while both run (many concurrent
  // callers already keep the cores busy) runs its items inline.
  void parallel_for(int n, const std::function<void(int)> &fn) {
    if (n <= 0) return;
    if (n == 1 || workers_.empty() || jobs_.fetch_add(1) >= kJobs) {
      if (n > 1 && !workers_.empty()) jobs_.fetch_sub(1);
      for (int i = 0; i < n; i++) fn(i);
      return;
    }
    struct Release {
      std::atomic<int> &j;
      ~Release() { j.fetch_sub(1); }
    } release{jobs_};
    struct Job {
      const std::function<void(int)> *fn;
      std::atomic<int> next{0}, done{0};
      int n;
    };
    auto job = std::make_shared<Job>();
    job->fn = &fn;
    job->n = n;
    auto work = [job] {
      int i;
      while ((i = job->next.fetch_add(1)) < job->n) {
        (*job->fn)(i);
        job->done.fetch_add(1, std::memory_order_release);
      }
    };
    {
      std::lock_guard<std::mutex> lk(mu_);
      const int helpers = std::min<int>(n - 1, static_cast<int>(workers_.size()));
      for (int h = 0; h < helpers; h++) tasks_.push_back(work);
    }
    cv_.notify_all();
    work();
    while (job->done.load(std::memory_order_acquire) < n) std::this_thread::yield();
  }

 private:
  explicit HostPool(int node) {
    int nt = 8;  // deployment setting NXEC_HOST_THREADS
    if (const char *e = std::getenv("NXEC_HOST_THREADS")) nt = std::max(0, std::atoi(e));
    const std::vector<int> cpus = node_cpus(node);
    for (int i = 0; i < nt; i++)
      workers_.emplace_back([this, cpus] {
        (void)bind_thread_cpus(cpus);  // within the process's affinity; unknown node: unbound
        loop();
      });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  void loop() {
    while (true) {
      std::function<void()> t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !tasks_.empty(); });
        if (stop_ && tasks_.empty()) return;
        t = std::move(tasks_.front());
        tasks_.pop_front();
      }
      t();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> tasks_;
  std::vector<std::thread> workers_;
  static constexpr int kJobs = 2;
  std::atomic<int> jobs_{0};
  bool stop_ = false;
};

}  // namespace

bool host_direct_enabled() {
  // deployment setting NXEC_HOST_DIRECT, read at every call:
  // a host may switch zero copy off and on between calls (bench.py times both)
  const char *e = std::getenv("NXEC_HOST_DIRECT");
  return !(e && e[0] == '0');
}

bool test_fault(const char *name) {
  static const std::string faults = [] {
    const char *e = std::getenv("NXEC_TEST_FAULT");
    return "," + std::string(e ? e : "") + ",";
  }();
  return faults.find("," + std::string(name) + ",") != std::string::npos;
}

void *host_device_view(const void *h) {
  if (!host_direct_enabled()) return nullptr;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, h) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}

// both ends in one mapping: the device addresses of the first and last byte
// differ by bytes - 1 (hipHostRegister on a sub-range, a frame running past the
// end of its registration take the staged path instead of faulting the GPU)
void *host_device_view_range(const void *h, size_t bytes) {
  void *d0 = host_device_view(h);
  if (!d0 || bytes <= 1) return d0;
  const void *last = static_cast<const uint8_t *>(h) + (bytes - 1);
  void *d1 = host_device_view(last);
  if (!d1 || static_cast<uint8_t *>(d1) - static_cast<uint8_t *>(d0) != static_cast<ptrdiff_t>(bytes - 1)) return nullptr;
  return d0;
}

void host_parallel_for(int n, const std::function<void(int)> &fn, HostLane lane, int node) {
  if (n <= 1) {  // nothing to spread: no pool (and no thread) needed
    if (n == 1) fn(0);
    return;
  }
  HostPool::get(lane, node).parallel_for(n, fn);
}

int set_error(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int hip_err(hipError_t e, const char *what) {
  return set_error(e == hipErrorNoDevice || e == hipErrorInvalidDevice ? NXEC_ERR_NODEV : NXEC_ERR_HIP, "%s: %s", what,
                   hipGetErrorString(e));
}

void ObjStage::release() {
  for (int i = 0; i < kObjSlots; i++) {
    if (streams[i]) {
      (void)hipStreamSynchronize(streams[i]);
      if (i > 0 || !borrowed0) (void)hipStreamDestroy(streams[i]);
    }
    if (h2d_done[i]) (void)hipEventDestroy(h2d_done[i]);
    streams[i] = nullptr;
    h2d_done[i] = nullptr;
  }
  if (aux) {
    (void)hipStreamSynchronize(aux);
    (void)hipStreamDestroy(aux);
    aux = nullptr;
  }
  if (d) (void)hipFree(d);
  d = nullptr;
  cap = 0;
}


namespace {
std::mutex g_prep_mu;
std::vector<bool> g_prepared;
}  // namespace

int ensure_device(int device) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0) return set_error(NXEC_ERR_NODEV, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= count) return set_error(NXEC_ERR_NODEV, "device %d out of range (%d devices)", device, count);
  NXEC_HIP(hipSetDevice(device));
  std::lock_guard<std::mutex> lk(g_prep_mu);
  if (g_prepared.size() < static_cast<size_t>(count)) g_prepared.resize(count, false);
  if (!g_prepared[device]) {
    hipDeviceProp_t prop;
    NXEC_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      return set_error(NXEC_ERR_NODEV, "device %d is %s; libnxec is built for gfx950 only", device, prop.gcnArchName);
    int rc = prepare_kernels();
    if (rc) return rc;
    g_prepared[device] = true;
  }
  return NXEC_OK;
}

int acquire_slot(nxec_ctx_t *ctx, size_t bytes, Slot **out, bool may_wait) {
  Slot *s = nullptr;
  {
    // best fit: the smallest free slot that holds `bytes`, else the largest
    // (grown below) -- so callers of different sizes do not keep re-pinning
    // each other's slots (hipHostMalloc of a GiB costs ~0.1 s).  Slots still
    // read by an asynchronous call's launches are taken only by an
    // asynchronous caller (may_wait), only when no idle one is free and the
    // context already has kAsyncSlots: the best of those, waited on below.
    // Everyone else gets an idle slot or a new one (never a wait on another
    // stream's queued work).
    std::lock_guard<std::mutex> lk(ctx->slot_mu);
    int best = -1;
    bool any_idle = false;
    for (Slot *f : ctx->free_slots) any_idle = any_idle || f->idle();
    const bool only_idle = !may_wait || any_idle || ctx->all_slots.size() < kAsyncSlots;
    for (int i = 0; i < static_cast<int>(ctx->free_slots.size()); i++) {
      if (only_idle && !ctx->free_slots[i]->idle()) continue;
      const size_t c = ctx->free_slots[i]->cap;
      if (best < 0) {
        best = i;
        continue;
      }
      const size_t b = ctx->free_slots[best]->cap;
      if ((c >= bytes && (b < bytes || c < b)) || (c < bytes && b < bytes && c > b)) best = i;
    }
    if (best >= 0) {
      s = ctx->free_slots[best];
      ctx->free_slots.erase(ctx->free_slots.begin() + best);
    }
  }
  if (!s) {
    s = new Slot();
    hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete s;
      return hip_err(e, "hipStreamCreate(slot)");
    }
    std::lock_guard<std::mutex> lk(ctx->slot_mu);
    ctx->all_slots.push_back(s);
  }
  if (s->busy_set) {  // an asynchronous call's launches may still read the staging
    (void)hipEventSynchronize(s->busy);
    s->busy_set = false;
  }
  if (s->cap < bytes) {
    if (s->h) (void)hipHostFree(s->h);
    if (s->d) (void)hipFree(s->d);
    s->h = nullptr;
    s->d = nullptr;
    s->cap = 0;
    hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&s->h), bytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s->d), bytes);
    if (e != hipSuccess) {
      std::lock_guard<std::mutex> lk(ctx->slot_mu);
      ctx->free_slots.push_back(s);
      return hip_err(e, "staging allocation");
    }
    s->cap = bytes;
  }
  *out = s;
  return NXEC_OK;
}

namespace {
// Idle slots keep their pinned + device staging for the next call, up to
// NXEC_SLOT_POOL_MAX bytes per context (deployment setting, default 2 GiB);
// past it a returned slot gives its buffers back (it keeps its stream), so
// one large round -- e.g. an agent round of many callers -- does not stay
// pinned for the process's lifetime.
size_t slot_pool_max() {
  static const size_t v = [] {
    const char *e = std::getenv("NXEC_SLOT_POOL_MAX");
    return e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : (size_t(2) << 30);
  }();
  return v;
}
}  // namespace

void release_slot(nxec_ctx_t *ctx, Slot *s) {
  bool drop = false;
  {
    std::lock_guard<std::mutex> lk(ctx->slot_mu);
    size_t pooled = s->cap;
    for (Slot *f : ctx->free_slots) pooled += f->cap;
    drop = pooled > slot_pool_max();
    if (!drop) {
      ctx->free_slots.push_back(s);
      return;
    }
  }
  (void)hipStreamSynchronize(s->stream);
  if (s->busy_set) (void)hipEventSynchronize(s->busy);
  s->busy_set = false;
  if (s->h) (void)hipHostFree(s->h);
  if (s->d) (void)hipFree(s->d);
  s->h = nullptr;
  s->d = nullptr;
  s->cap = 0;
  std::lock_guard<std::mutex> lk(ctx->slot_mu);
  ctx->free_slots.push_back(s);
}

int batch_stage(nxec_ctx_t *ctx, size_t slot_bytes, std::unique_lock<std::mutex> &lk, ObjStage &priv,
                ObjStage **out) {
  lk = std::unique_lock<std::mutex>(ctx->obj_mu, std::try_to_lock);
  ObjStage &stg = lk.owns_lock() ? ctx->obj : priv;
  slot_bytes = (slot_bytes + 255) / 256 * 256;
  if (stg.cap < slot_bytes) {
    stg.release();
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&stg.d), slot_bytes * kObjSlots);
    stg.borrowed0 = lk.owns_lock();
    for (int i = 0; i < kObjSlots && e == hipSuccess; i++) {
      if (i == 0 && stg.borrowed0)
        stg.streams[0] = ctx->stream;
      else
        e = hipStreamCreateWithFlags(&stg.streams[i], hipStreamNonBlocking);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&stg.h2d_done[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
      stg.release();
      return hip_err(e, "batch staging allocation");
    }
    stg.cap = slot_bytes;
  }
  *out = &stg;
  return NXEC_OK;
}

// ---- The default-context pool of the entry points that take no context ----
// The reference shares one RSCode across the proxy's worker threads
// (chunk_manager.cc:1779-1801, zmq.cc:83) and never selects a GPU, so the
// drop-in cannot follow "the caller's device": every stripe would go to
// device 0 over one PCIe link.  Instead each call leases a member of a pool --
// by default one context per visible device -- chosen per call by
// nxec_default_pick: the member with the fewest calls in flight, a device on
// the calling CPU's NUMA node winning ties against a remote one by one call
// (a remote device is taken only when it has fewer calls in flight than the
// local one), and on an exact tie the member this thread used last (its
// staging slots are warm).  NXEC_DEFAULT_DEVICES=current keeps the old rule
// (the calling thread's current device); a list ("0,0,1") names the members,
// a device listed twice getting two contexts.  Members' contexts live for the
// process: a reconfiguration (nxec_default_devices) only changes which serve.
namespace {

struct Member {
  int device = 0, ordinal = 0, node = -1;
  std::mutex mu;  // creation of ctx
  std::atomic<nxec_ctx_t *> ctx{nullptr};
  std::atomic<int> inflight{0};
  std::atomic<unsigned long long> calls{0};
};

struct PoolCfg {
  bool current = false;           // the calling thread's current device
  std::vector<Member *> members;  // list mode
  uint64_t gen = 0;
};

std::mutex g_pool_mu;
std::deque<Member> g_members;                 // every member ever made (stable addresses)
std::shared_ptr<const PoolCfg> g_pool;        // null: not resolved yet
std::vector<int> g_pool_request;              // nxec_default_devices' list (resolved at next use)
int g_pool_request_mode = -2;                 // -2 unset (environment), -1 current, 0 all, 1 list
uint64_t g_pool_gen = 0;
thread_local int t_prev_member = -1;
thread_local uint64_t t_prev_gen = 0;

// under g_pool_mu: the member for (device, ordinal), made on first use
Member *member_for(int device, int ordinal) {
  for (Member &m : g_members)
    if (m.device == device && m.ordinal == ordinal) return &m;
  g_members.emplace_back();
  Member &m = g_members.back();
  m.device = device;
  m.ordinal = ordinal;
  char bus[64] = {0};
  int node = -1;
  if (device_bus_id(device, bus, sizeof(bus)) == NXEC_OK) (void)pci_node_cpus(bus, &node);
  m.node = node;
  return &m;
}

// "all" | "current" | "0,0,1" -> mode (-1 current, 0 all, 1 list) and list; false when malformed
bool parse_devices(const char *text, int *mode, std::vector<int> *devs) {
  devs->clear();
  const std::string t(text);
  if (t.empty() || t == "all") {
    *mode = 0;
    return true;
  }
  if (t == "current") {
    *mode = -1;
    return true;
  }
  size_t i = 0;
  while (i < t.size()) {
    size_t j = t.find(',', i);
    if (j == std::string::npos) j = t.size();
    const std::string f = t.substr(i, j - i);
    char *end = nullptr;
    const long d = std::strtol(f.c_str(), &end, 10);
    if (f.empty() || *end != '\0' || d < 0 || d > 4095) return false;
    devs->push_back(static_cast<int>(d));
    i = j + 1;
  }
  *mode = 1;
  return !devs->empty();
}

// under g_pool_mu
int resolve_pool(std::shared_ptr<const PoolCfg> *out) {
  if (!g_pool) {
    int mode = g_pool_request_mode;
    std::vector<int> devs = g_pool_request;
    if (mode == -2) {  // deployment setting NXEC_DEFAULT_DEVICES
      const char *e = std::getenv("NXEC_DEFAULT_DEVICES");
      if (!parse_devices(e ? e : "all", &mode, &devs))
        return set_error(NXEC_ERR_INVALID, "NXEC_DEFAULT_DEVICES=%s: expected all, current or a device list", e);
    }
    auto cfg = std::make_shared<PoolCfg>();
    cfg->gen = ++g_pool_gen;
    cfg->current = mode == -1;
    if (mode == 0) {
      int count = 0;
      const hipError_t e = hipGetDeviceCount(&count);
      if (e != hipSuccess || count == 0) {
        (void)hipGetLastError();
        return set_error(NXEC_ERR_NODEV, "no HIP device available (%s)", hipGetErrorString(e));
      }
      for (int d = 0; d < count; d++) devs.push_back(d);
    }
    if (mode >= 0) {
      std::vector<int> seen;
      for (int d : devs) {
        const int ord = static_cast<int>(std::count(seen.begin(), seen.end(), d));
        seen.push_back(d);
        cfg->members.push_back(member_for(d, ord));
      }
    }
    g_pool = cfg;
  }
  *out = g_pool;
  return NXEC_OK;
}

int member_ctx(Member *m, nxec_ctx_t **out) {
  nxec_ctx_t *c = m->ctx.load(std::memory_order_acquire);
  if (!c) {
    std::lock_guard<std::mutex> lk(m->mu);
    c = m->ctx.load(std::memory_order_acquire);
    if (!c) {
      if (int rc = nxec_ctx_create(m->device, &c)) return rc;
      m->ctx.store(c, std::memory_order_release);
    }
  }
  *out = c;
  return NXEC_OK;
}

}  // namespace

namespace {
// Per-device admission (tuning().pool_admit, 8): at most that many drop-in
// calls run on a device at once; the rest wait here instead of piling staging
// slots, streams and host-pool copies onto one device (64 callers on one GPU:
// CodingUtils::encode 21 -> 64 GiB/s, RSCode::decode 14 -> 62; 16 callers
// 56 -> 67; profiles/r06_admit_ab.jsonl).  The pick above already counted
// this call, so later callers go to a less busy member while this one waits.
struct DeviceGate {
  std::mutex mu;
  std::condition_variable cv;
  int running = 0;
  int peak = 0;                 // most calls running at once (nxec_default_admission)
  unsigned long long waited = 0;  // calls that found the gate full
};
DeviceGate &device_gate(int device) {
  static std::mutex mu;
  static std::deque<DeviceGate> gates;  // stable addresses
  std::lock_guard<std::mutex> lk(mu);
  while (static_cast<int>(gates.size()) <= device) gates.emplace_back();
  return gates[device];
}
}  // namespace

DefaultLease::~DefaultLease() {
  if (gate_) {
    DeviceGate *g = static_cast<DeviceGate *>(gate_);
    {
      std::lock_guard<std::mutex> lk(g->mu);
      g->running--;
    }
    g->cv.notify_one();
  }
  if (member_) static_cast<Member *>(member_)->inflight.fetch_sub(1, std::memory_order_relaxed);
  int cur = -1;
  if (saved_device_ >= 0 && hipGetDevice(&cur) == hipSuccess && cur != saved_device_) (void)hipSetDevice(saved_device_);
}

int lease_admit(DefaultLease &lease) {
  const int cap = tuning().pool_admit;
  Member *m = static_cast<Member *>(lease.member_);
  if (cap <= 0 || !m || lease.gate_) return 0;
  DeviceGate &g = device_gate(m->device);
  int admitted = 0;
  {
    std::unique_lock<std::mutex> lk(g.mu);
    if (g.running >= cap) g.waited++;
    g.cv.wait(lk, [&] { return g.running < cap; });
    admitted = ++g.running;
    g.peak = std::max(g.peak, admitted);
    lease.gate_ = &g;
  }
  // testing (NXEC_TEST_FAULT=admit_stall): hold the place 30 ms so callers queue
  if (test_fault("admit_stall")) std::this_thread::sleep_for(std::chrono::milliseconds(30));
  lease.device_inflight = admitted;
  return admitted;
}

int default_ctx(DefaultLease &lease, bool admit) {
  std::shared_ptr<const PoolCfg> cfg;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (int rc = resolve_pool(&cfg)) return rc;
  }
  int saved = 0;
  hipError_t e = hipGetDevice(&saved);
  if (e != hipSuccess) return hip_err(e, "hipGetDevice");
  Member *m = nullptr;
  if (cfg->current) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    m = member_for(saved, 0);
  } else {
    const int n = static_cast<int>(cfg->members.size());
    std::vector<int> inflight(n), nodes(n);
    for (int i = 0; i < n; i++) {
      inflight[i] = cfg->members[i]->inflight.load(std::memory_order_relaxed);
      nodes[i] = cfg->members[i]->node;
    }
    const int prev = t_prev_gen == cfg->gen ? t_prev_member : -1;
    const int idx = nxec_default_pick(n, inflight.data(), nodes.data(), cpu_numa_node(sched_getcpu()), prev);
    m = cfg->members[idx];
    t_prev_member = idx;
    t_prev_gen = cfg->gen;
  }
  m->inflight.fetch_add(1, std::memory_order_relaxed);
  m->calls.fetch_add(1, std::memory_order_relaxed);
  lease.member_ = m;
  lease.saved_device_ = saved;
  const int admitted = admit ? lease_admit(lease) : 0;
  nxec_ctx_t *c = nullptr;
  if (int rc = member_ctx(m, &c)) return rc;
  lease.ctx = c;
  // this call runs on c's device (the lease restores the caller's on release)
  if (int rc = ensure_device(c->device)) return rc;
  // calls in flight on the device: its PCIe link's share (zero copy or DMA)
  int dev_inflight = 0;
  if (cfg->current) {
    dev_inflight = m->inflight.load(std::memory_order_relaxed);
  } else {
    for (Member *o : cfg->members)
      if (o->device == m->device) dev_inflight += o->inflight.load(std::memory_order_relaxed);
  }
  lease.device_inflight = std::max(1, admitted ? admitted : dev_inflight);
  return NXEC_OK;
}

int zero_line(nxec_ctx_t *ctx, size_t bytes, const uint8_t **out) {
  std::lock_guard<std::mutex> lk(ctx->zero_mu);
  if (ctx->zero_bytes < bytes) {
    // at least doubling, so a context retires few lines however its callers' sizes creep up
    const size_t want = std::max<size_t>({(bytes + 4095) / 4096 * 4096, size_t(1) << 20, 2 * ctx->zero_bytes});
    uint8_t *z = nullptr;
    NXEC_HIP(hipMalloc(reinterpret_cast<void **>(&z), want));
    hipError_t e = hipMemsetAsync(z, 0, want, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
      (void)hipFree(z);
      return hip_err(e, "zero line");
    }
    // Launches queued (or about to be queued: a caller that took the old line
    // and has not launched yet) may still read the old line, so it is retired,
    // never freed while the context lives (nxec_ctx_destroy frees it).  Lines
    // at least double, so a context holds about log2(M / 1 MiB) + 1 of them.
    if (ctx->zero) ctx->zero_retired.push_back(ctx->zero);
    ctx->zero = z;
    ctx->zero_bytes = want;
  }
  *out = ctx->zero;
  return NXEC_OK;
}

}  // namespace nxec

using namespace nxec;

extern "C" {

const char *nxec_last_error(void) { return last_error().c_str(); }
const char *nxec_version(void) { return "nxec 0.1.0 gfx950"; }

int nxec_ctx_create(int device, nxec_ctx_t **out) {
  if (!out) return set_error(NXEC_ERR_INVALID, "null out pointer");
  *out = nullptr;
  int rc = ensure_device(device);
  if (rc) return rc;
  std::unique_ptr<nxec_ctx_t> ctx(new nxec_ctx_t());
  ctx->device = device;
  hipDeviceProp_t prop;
  NXEC_HIP(hipGetDeviceProperties(&prop, device));
  ctx->num_cus = prop.multiProcessorCount;
  {
    char bus[64] = {0};
    if (device_bus_id(device, bus, sizeof(bus)) == NXEC_OK) (void)pci_node_cpus(bus, &ctx->numa_node);
  }
  NXEC_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  *out = ctx.release();
  return NXEC_OK;
}

void nxec_ctx_destroy(nxec_ctx_t *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  ctx->obj.release();  // before the context stream it borrows
  for (auto &pr : ctx->kt_pending) {
    (void)hipEventSynchronize(pr.second);
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  if (ctx->stream) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
  }
  // the zero lines last: launches on the context's streams have drained above
  // (hipFree itself waits for the device)
  if (ctx->zero) ctx->zero_retired.push_back(ctx->zero);
  for (uint8_t *z : ctx->zero_retired) (void)hipFree(z);
  for (Slot *s : ctx->all_slots) {
    if (s->stream) {
      (void)hipStreamSynchronize(s->stream);
      (void)hipStreamDestroy(s->stream);
    }
    for (hipEvent_t ev : s->events) (void)hipEventDestroy(ev);
    if (s->busy) {
      (void)hipEventSynchronize(s->busy);
      (void)hipEventDestroy(s->busy);
    }
    if (s->h) (void)hipHostFree(s->h);
    if (s->d) (void)hipFree(s->d);
    delete s;
  }
  delete ctx;
}

void *nxec_ctx_stream(nxec_ctx_t *ctx) { return ctx ? static_cast<void *>(ctx->stream) : nullptr; }

int nxec_default_pick(int n, const int *inflight, const int *nodes, int caller_node, int prev) {
  if (n < 1 || !inflight) return set_error(NXEC_ERR_INVALID, "nxec_default_pick: invalid arguments");
  int best = -1;
  long best_cost = 0;
  for (int i = 0; i < n; i++) {
    const bool remote = nodes && caller_node >= 0 && nodes[i] >= 0 && nodes[i] != caller_node;
    const long cost = 2L * std::max(0, inflight[i]) + (remote ? 1 : 0);
    if (best < 0 || cost < best_cost || (cost == best_cost && i == prev)) {
      best = i;
      best_cost = cost;
    }
  }
  return best;
}

int nxec_default_devices(const int *devices, int n) {
  if (n > 0 && !devices) return set_error(NXEC_ERR_INVALID, "nxec_default_devices: null device list");
  for (int i = 0; i < n; i++)
    if (devices[i] < 0) return set_error(NXEC_ERR_INVALID, "nxec_default_devices: device %d", devices[i]);
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool_request_mode = n < 0 ? -1 : (n == 0 ? 0 : 1);
  g_pool_request.clear();
  if (n > 0) g_pool_request.assign(devices, devices + n);
  g_pool.reset();  // resolved at the next call; calls in flight keep their snapshot
  return NXEC_OK;
}

int nxec_default_pool_stats(int *devices, int *nodes, unsigned long long *calls, int *inflight, int max, int *count) {
  if (!count || (max > 0 && (!devices || !nodes || !calls || !inflight)))
    return set_error(NXEC_ERR_INVALID, "nxec_default_pool_stats: invalid arguments");
  std::lock_guard<std::mutex> lk(g_pool_mu);
  std::vector<Member *> ms;
  if (g_pool && !g_pool->current) {
    ms = g_pool->members;
  } else {
    for (Member &m : g_members) ms.push_back(&m);  // current mode: every device used so far
  }
  *count = static_cast<int>(ms.size());
  for (int i = 0; i < max && i < *count; i++) {
    devices[i] = ms[i]->device;
    nodes[i] = ms[i]->node;
    calls[i] = ms[i]->calls.load(std::memory_order_relaxed);
    inflight[i] = ms[i]->inflight.load(std::memory_order_relaxed);
  }
  return NXEC_OK;
}

int nxec_default_admission(int device, int *limit, int *running, int *peak, unsigned long long *waited, int reset) {
  int count = 0;
  if (device < 0 || hipGetDeviceCount(&count) != hipSuccess || device >= count)
    return set_error(NXEC_ERR_INVALID, "nxec_default_admission: no device %d", device);
  DeviceGate &g = device_gate(device);
  std::lock_guard<std::mutex> lk(g.mu);
  if (limit) *limit = tuning().pool_admit;
  if (running) *running = g.running;
  if (peak) *peak = g.peak;
  if (waited) *waited = g.waited;
  if (reset) {
    g.peak = g.running;
    g.waited = 0;
  }
  return NXEC_OK;
}

}  // extern "C"

namespace nxec {

void kt_begin(nxec_ctx_t *ctx, hipStream_t st, hipEvent_t ev[2]) {
  ev[0] = ev[1] = nullptr;
  {
    std::lock_guard<std::mutex> lk(ctx->kt_mu);
    if (!ctx->kt_on) return;
  }
  if (hipEventCreate(&ev[0]) != hipSuccess) {
    ev[0] = nullptr;
    return;
  }
  if (hipEventCreate(&ev[1]) != hipSuccess) {
    (void)hipEventDestroy(ev[0]);
    ev[0] = ev[1] = nullptr;
    return;
  }
  (void)hipEventRecord(ev[0], st);
}

void kt_end(nxec_ctx_t *ctx, const hipEvent_t ev[2], hipStream_t st) {
  if (!ev[0]) return;
  (void)hipEventRecord(ev[1], st);
  std::lock_guard<std::mutex> lk(ctx->kt_mu);
  ctx->kt_pending.emplace_back(ev[0], ev[1]);
}

}  // namespace nxec

extern "C" {

int nxec_kernel_timing(nxec_ctx_t *ctx, int enable) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  double ms = 0;
  int64_t n = 0;
  int rc = nxec_kernel_time(ctx, &ms, &n);  // drains (and frees) the pending pairs
  std::lock_guard<std::mutex> lk(ctx->kt_mu);
  ctx->kt_on = enable != 0;
  ctx->kt_ms = 0;
  ctx->kt_launches = 0;
  return rc;
}

int nxec_kernel_time(nxec_ctx_t *ctx, double *ms, int64_t *launches) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pend;
  {
    std::lock_guard<std::mutex> lk(ctx->kt_mu);
    pend.swap(ctx->kt_pending);
  }
  double sum = 0;
  int64_t cnt = 0;
  int rc = NXEC_OK;
  for (auto &pr : pend) {
    float t = 0;
    hipError_t e = hipEventSynchronize(pr.second);
    if (e == hipSuccess) e = hipEventElapsedTime(&t, pr.first, pr.second);
    if (e == hipSuccess) {
      sum += t;
      cnt++;
    } else if (!rc) {
      rc = hip_err(e, "nxec_kernel_time");
    }
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  std::lock_guard<std::mutex> lk(ctx->kt_mu);
  ctx->kt_ms += sum;
  ctx->kt_launches += cnt;
  if (ms) *ms = ctx->kt_ms;
  if (launches) *launches = ctx->kt_launches;
  return rc;
}

// ---- plumbing ----

int nxec_device_count(int *count) {
  if (!count) return set_error(NXEC_ERR_INVALID, "null pointer");
  *count = 0;
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) {
    *count = 0;
    return hip_err(e, "hipGetDeviceCount");
  }
  return NXEC_OK;
}

int nxec_set_device(int device) { return ensure_device(device); }

int nxec_device_info(int device, char *name, int name_len, int *num_cus, int64_t *total_mem) {
  hipDeviceProp_t prop;
  NXEC_HIP(hipGetDeviceProperties(&prop, device));
  if (name && name_len > 0) std::snprintf(name, name_len, "%s", prop.gcnArchName);
  if (num_cus) *num_cus = prop.multiProcessorCount;
  if (total_mem) *total_mem = static_cast<int64_t>(prop.totalGlobalMem);
  return NXEC_OK;
}

int nxec_dev_malloc(void **p, size_t bytes) {
  if (!p) return set_error(NXEC_ERR_INVALID, "null pointer");
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory) return set_error(NXEC_ERR_NOMEM, "hipMalloc(%zu): out of memory", bytes);
  NXEC_HIP(e);
  return NXEC_OK;
}
int nxec_dev_free(void *p) {
  NXEC_HIP(hipFree(p));
  return NXEC_OK;
}
int nxec_host_malloc_pinned(void **p, size_t bytes) {
  if (!p) return set_error(NXEC_ERR_INVALID, "null pointer");
  NXEC_HIP(hipHostMalloc(p, bytes, hipHostMallocDefault));
  return NXEC_OK;
}
int nxec_host_free_pinned(void *p) {
  NXEC_HIP(hipHostFree(p));
  return NXEC_OK;
}
int nxec_host_register(void *p, size_t bytes) {
  NXEC_HIP(hipHostRegister(p, bytes, hipHostRegisterDefault));
  return NXEC_OK;
}
int nxec_host_unregister(void *p) {
  NXEC_HIP(hipHostUnregister(p));
  return NXEC_OK;
}
int nxec_memcpy_h2d(void *d_dst, const void *h_src, size_t bytes, void *stream) {
  NXEC_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, static_cast<hipStream_t>(stream)));
  return NXEC_OK;
}
int nxec_memcpy_d2h(void *h_dst, const void *d_src, size_t bytes, void *stream) {
  NXEC_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream)));
  return NXEC_OK;
}
int nxec_memcpy_d2d(void *d_dst, const void *d_src, size_t bytes, void *stream) {
  NXEC_HIP(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
  return NXEC_OK;
}
int nxec_memset(void *d_dst, int value, size_t bytes, void *stream) {
  NXEC_HIP(hipMemsetAsync(d_dst, value, bytes, static_cast<hipStream_t>(stream)));
  return NXEC_OK;
}
int nxec_memset2d(void *d_dst, size_t pitch, int value, size_t width, size_t height, void *stream) {
  if (!d_dst || width > pitch) return set_error(NXEC_ERR_INVALID, "nxec_memset2d: invalid arguments");
  if (!width || !height) return NXEC_OK;
  NXEC_HIP(hipMemset2DAsync(d_dst, pitch, value, width, height, static_cast<hipStream_t>(stream)));
  return NXEC_OK;
}
int nxec_stream_create(void **stream) {
  if (!stream) return set_error(NXEC_ERR_INVALID, "null pointer");
  hipStream_t s;
  NXEC_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = s;
  return NXEC_OK;
}
int nxec_stream_destroy(void *stream) {
  NXEC_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)));
  return NXEC_OK;
}
int nxec_stream_sync(void *stream) {
  NXEC_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  return NXEC_OK;
}
int nxec_device_sync(void) {
  NXEC_HIP(hipDeviceSynchronize());
  return NXEC_OK;
}
int nxec_event_create(void **event) {
  if (!event) return set_error(NXEC_ERR_INVALID, "null pointer");
  hipEvent_t ev;
  NXEC_HIP(hipEventCreate(&ev));
  *event = ev;
  return NXEC_OK;
}
int nxec_event_destroy(void *event) {
  NXEC_HIP(hipEventDestroy(static_cast<hipEvent_t>(event)));
  return NXEC_OK;
}
int nxec_event_record(void *event, void *stream) {
  NXEC_HIP(hipEventRecord(static_cast<hipEvent_t>(event), static_cast<hipStream_t>(stream)));
  return NXEC_OK;
}
int nxec_event_elapsed_ms(void *start, void *stop, float *ms) {
  if (!ms) return set_error(NXEC_ERR_INVALID, "null pointer");
  NXEC_HIP(hipEventSynchronize(static_cast<hipEvent_t>(stop)));
  NXEC_HIP(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)));
  return NXEC_OK;
}
int nxec_fill_random(void *d_dst, size_t bytes, uint64_t seed, void *stream) {
  return launch_fill(d_dst, bytes, seed, stream);
}
int nxec_checksum(const void *d_src, size_t bytes, uint64_t *out, void *stream) {
  if (!out) return set_error(NXEC_ERR_INVALID, "null pointer");
  uint64_t *d_acc = nullptr;
  NXEC_HIP(hipMalloc(reinterpret_cast<void **>(&d_acc), sizeof(uint64_t)));
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(d_acc, 0, sizeof(uint64_t), st);
  int rc = e == hipSuccess ? launch_checksum(d_src, bytes, d_acc, st) : hip_err(e, "hipMemsetAsync");
  if (rc == NXEC_OK) {
    e = hipMemcpyAsync(out, d_acc, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = hip_err(e, "checksum readback");
  }
  (void)hipFree(d_acc);
  return rc;
}

int nxec_host_range_mapped(const void *p, size_t bytes) {
  return p && host_device_view_range(p, bytes) != nullptr ? 1 : 0;
}

int nxec_reset_work_queues(void) {
  int dev = 0;
  NXEC_HIP(hipGetDevice(&dev));
  int rc = ensure_device(dev);
  return rc ? rc : reset_work_queues(nullptr);
}

int nxec_debug_poison_next_queue_slot(uint32_t next_tile) {
  int dev = 0;
  NXEC_HIP(hipGetDevice(&dev));
  int rc = ensure_device(dev);
  return rc ? rc : debug_poison_next_queue_slot(next_tile);
}

int nxec_describe_launch(nxec_ctx_t *ctx, int rows, int k, int64_t len, int64_t nstripes, char *buf, int buf_len) {
  if (!ctx || !buf || buf_len <= 0 || k < 1 || k > NXEC_MAX_K)
    return set_error(NXEC_ERR_INVALID, "invalid arguments");
  const int64_t nvec = len / 16;
  LaunchInfo li = plan_launch(k, std::min(rows, static_cast<int>(kMaxRowsPerPass)), nvec, nstripes, ctx->num_cus,
                              nvec % 1024 == 0, false, false);
  std::snprintf(buf, buf_len,
                "{\"kernel\":\"%s\",\"k\":%d,\"rows\":%d,\"passes\":%d,\"lds_copies\":%d,\"block\":%d,\"grid\":%d,"
                "\"lds_bytes\":%d,\"cus\":%d}",
                li.variant, k, rows, (rows + kMaxRowsPerPass - 1) / kMaxRowsPerPass, li.lds_copies, li.block, li.grid,
                li.lds_bytes, ctx->num_cus);
  return NXEC_OK;
}

}  // extern "C"
