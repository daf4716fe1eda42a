// Host runtime of libnxec: contexts, argument validation, the RS batch entry
// points and the drop-in host-buffer encode.  Compute always goes to the
// gfx950 kernels in nxec_kernels.hip; there is no CPU fallback.
#include <hip/hip_runtime.h>
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
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
#include <stdexcept>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "nxec.h"
#include "nxec_internal.h"

namespace nxec {

namespace {
thread_local std::string g_last_error;

// Copy into pinned staging.  NXEC_NT_STAGING=1 uses streaming (non-temporal)
// stores: the staging lines are never read by the CPU, so skipping their
// read-for-ownership halves the DRAM traffic of a large gather
// (tools/microbench/host_copy.cc measures both on the box).
bool nt_staging() {
  static const bool on = [] {
    const char *e = std::getenv("NXEC_NT_STAGING");
    return e && e[0] == '1';
  }();
  return on;
}
void stage_copy(void *dst, const void *src, size_t n) {
  uint8_t *d = static_cast<uint8_t *>(dst);
  const uint8_t *sp = static_cast<const uint8_t *>(src);
  if (!nt_staging() || n < 4096) {
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

// A host-staging slot: pinned + device buffers and a stream, used by the
// synchronous host-buffer entry points.  Slots are pooled per context so
// concurrent callers (proxy workers, agent threads) do not serialize.
struct Slot {
  hipStream_t stream = nullptr;
  uint8_t *h = nullptr;
  uint8_t *d = nullptr;
  size_t cap = 0;
  std::vector<hipEvent_t> events;  // per-piece completion (pipelined host path)
  // asynchronous calls (NXEC_OBJECTS_ASYNC) hand the slot back while their
  // launches still read its tables: recorded on the call's stream, waited on
  // before the next user writes the staging
  hipEvent_t busy = nullptr;
  bool busy_set = false;
  bool idle() const { return !busy_set || hipEventQuery(busy) == hipSuccess; }
};

// Host worker pool for staging copies (pageable <-> pinned) of the host entry
// points: one memcpy thread moves ~10 GB/s, so a 1 MiB RS(10,4) stripe spends
// most of a call copying.  parallel_for splits a call's copies over the pool;
// the calling thread works too, and concurrent callers share the pool.
class HostPool {
 public:
  static HostPool &get() {
    static HostPool pool;
    return pool;
  }
  // runs fn(i) for i in [0, n), returns when all are done.  The pool serves
  // one job at a time: a caller arriving while it is busy (many concurrent
  // callers already keep the cores busy) runs its items inline.
  void parallel_for(int n, const std::function<void(int)> &fn) {
    if (n <= 0) return;
    bool expected = false;
    if (n == 1 || workers_.empty() || !busy_.compare_exchange_strong(expected, true)) {
      for (int i = 0; i < n; i++) fn(i);
      return;
    }
    struct Release {
      std::atomic<bool> &b;
      ~Release() { b.store(false); }
    } release{busy_};
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
  HostPool() {
    int nt = 8;
    if (const char *e = std::getenv("NXEC_HOST_THREADS")) nt = std::max(0, std::atoi(e));
    for (int i = 0; i < nt; i++) workers_.emplace_back([this] { loop(); });
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
  std::atomic<bool> busy_{false};
  bool stop_ = false;
};

// Device address of pinned / registered host memory (kernels read and write
// it over PCIe: zero copy), or nullptr for pageable memory or when
// NXEC_HOST_DIRECT=0.
void *host_device_view(const void *h) {
  const char *env = std::getenv("NXEC_HOST_DIRECT");
  if (env && env[0] == '0') return nullptr;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, h) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}

// Device address of the whole host range [h, h + bytes): both ends must lie in
// pinned / registered memory of one mapping (the device addresses of the first
// and last byte differ by bytes - 1), else nullptr -- a buffer registered only
// in part (hipHostRegister on a sub-range, a frame running past the end of
// its registration) takes the staged path instead of faulting the GPU.
void *host_device_view_range(const void *h, size_t bytes) {
  void *d0 = host_device_view(h);
  if (!d0 || bytes <= 1) return d0;
  const void *last = static_cast<const uint8_t *>(h) + (bytes - 1);
  void *d1 = host_device_view(last);
  if (!d1 || static_cast<uint8_t *>(d1) - static_cast<uint8_t *>(d0) != static_cast<ptrdiff_t>(bytes - 1)) return nullptr;
  return d0;
}

// host entry-point calls in flight (the pipelined, pool-assisted form is for
// few callers; many concurrent callers are better served one piece each)
std::atomic<int> g_host_calls{0};
}  // namespace

void host_parallel_for(int n, const std::function<void(int)> &fn) { HostPool::get().parallel_for(n, fn); }

int set_error(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

static int hip_err(hipError_t e, const char *what) {
  return set_error(e == hipErrorNoDevice || e == hipErrorInvalidDevice ? NXEC_ERR_NODEV : NXEC_ERR_HIP, "%s: %s", what,
                   hipGetErrorString(e));
}

static int hip_check(hipError_t e, const char *what) { return e == hipSuccess ? NXEC_OK : hip_err(e, what); }

#define NXEC_HIP(call)                           \
  do {                                           \
    hipError_t e_ = (call);                      \
    if (e_ != hipSuccess) return hip_err(e_, #call); \
  } while (0)

}  // namespace nxec

using namespace nxec;

namespace {
// Device staging of the batched host entry points (nxec_encode_object_host,
// nxec_rs_encode_host_batch), kept across calls (allocating ~4 GiB per call
// cost ~12 ms of a 150 ms call): kObjSlots batches in flight, one stream and
// one H2D-done event each.  The context's own stream serves as slot 0: HIP
// has 4 hardware queues per process (GPU_MAX_HW_QUEUES), and a fifth stream
// shares one, serialising two slots' copies (object write 44 -> 34 GiB/s).
constexpr int kObjSlots = 3;
struct ObjStage {
  uint8_t *d = nullptr;
  size_t cap = 0;  // bytes per slot
  hipStream_t streams[kObjSlots] = {};
  hipEvent_t h2d_done[kObjSlots] = {};
  bool borrowed0 = false;  // streams[0] is the context's stream
  void release() {
    for (int i = 0; i < kObjSlots; i++) {
      if (streams[i]) {
        (void)hipStreamSynchronize(streams[i]);
        if (i > 0 || !borrowed0) (void)hipStreamDestroy(streams[i]);
      }
      if (h2d_done[i]) (void)hipEventDestroy(h2d_done[i]);
      streams[i] = nullptr;
      h2d_done[i] = nullptr;
    }
    if (d) (void)hipFree(d);
    d = nullptr;
    cap = 0;
  }
};
}  // namespace

struct nxec_ctx {
  int device = 0;
  int num_cus = 0;
  hipStream_t stream = nullptr;
  std::mutex slot_mu;
  std::vector<Slot *> free_slots;
  std::vector<Slot *> all_slots;
  std::mutex obj_mu;  // guards obj (one object host call at a time uses it)
  ObjStage obj;
  // agent-service aggregation (nxec_agent_encode_batch): concurrent callers'
  // requests join one round; one caller at a time leads and runs the round
  std::mutex agent_mu;
  std::condition_variable agent_cv;
  std::deque<struct AgentJob *> agent_pending;
  bool agent_leader = false;
  // nxec_encode_host_md5 rounds (zero copy): a leader launches every pending
  // call in one kernel and hands leadership on at once, so rounds overlap
  std::mutex dg_mu;
  std::condition_variable dg_cv;
  std::deque<struct DigestJob *> dg_pending;
  bool dg_leader = false;
  int dg_inflight = 0;
  // nxec_kernel_timing: event pairs around the coding launches, read by nxec_kernel_time
  std::mutex kt_mu;
  bool kt_on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> kt_pending;
  double kt_ms = 0;
  int64_t kt_launches = 0;
};

// one nxec_encode_host_md5 call whose buffers are all device-mapped
struct DigestJob {
  int len, k, rows;
  const unsigned char *coeffs;
  unsigned char *md5_data, *md5_code;
  std::vector<uintptr_t> in_dv, out_dv;  // device views of the inputs / outputs
  int rc = NXEC_OK;
  bool done = false;
  std::string error;
};

struct AgentJob {
  const nxec_agent_req *reqs;
  int nreqs;
  int64_t chunk_size, batch_bytes;
  int rc = NXEC_OK;
  bool done = false;
  std::string error;
};

namespace {

std::mutex g_prep_mu;
std::vector<bool> g_prepared;

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

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// staging slots a context grows to before an asynchronous caller waits for
// one of its earlier calls (two in flight keep the GPU fed: the host plans
// call i + 1 while call i runs)
constexpr size_t kAsyncSlots = 4;

int acquire_slot(nxec_ctx_t *ctx, size_t bytes, Slot **out) {
  Slot *s = nullptr;
  {
    // best fit: the smallest free slot that holds `bytes`, else the largest
    // (grown below) -- so callers of different sizes do not keep re-pinning
    // each other's slots (hipHostMalloc of a GiB costs ~0.1 s)
    // (slots still read by an asynchronous call's launches only when no idle
    // one is free and the context already has kAsyncSlots: then the best of
    // those, waited on below)
    std::lock_guard<std::mutex> lk(ctx->slot_mu);
    int best = -1;
    bool any_idle = false;
    for (Slot *f : ctx->free_slots) any_idle = any_idle || f->idle();
    const bool only_idle = any_idle || ctx->all_slots.size() < kAsyncSlots;
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

// Idle slots keep their pinned + device staging for the next call, up to
// NXEC_SLOT_POOL_MAX bytes per context (default 2 GiB); past it a returned
// slot gives its buffers back (it keeps its stream), so one large round --
// e.g. an agent round of many callers -- does not stay pinned for the
// process's lifetime.
size_t slot_pool_max() {
  static const size_t v = [] {
    const char *e = std::getenv("NXEC_SLOT_POOL_MAX");
    return e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : (size_t(2) << 30);
  }();
  return v;
}

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

// The context's persistent batch staging (kObjSlots slots of at least
// slot_bytes, grown on demand), or a private one in `priv` while another call
// holds the context's; the caller releases `priv` when it did not get the lock.
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

std::mutex g_default_mu;
std::vector<nxec_ctx_t *> g_default_ctx;

int default_ctx(nxec_ctx_t **out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_err(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_default_mu);
  if (g_default_ctx.size() <= static_cast<size_t>(dev)) g_default_ctx.resize(dev + 1, nullptr);
  if (!g_default_ctx[dev]) {
    int rc = nxec_ctx_create(dev, &g_default_ctx[dev]);
    if (rc) return rc;
  }
  *out = g_default_ctx[dev];
  return NXEC_OK;
}

hipStream_t pick_stream(nxec_ctx_t *ctx, void *stream) {
  return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}

// Shared implementation of the strided and gather forms.
int stripes_mul_impl(nxec_ctx_t *ctx, int rows, int k, const unsigned char *coeffs, const unsigned char *d_src,
                     const unsigned char *const *d_src_ptrs, const int32_t *src_idx, int64_t src_cs, int64_t src_ss,
                     unsigned char *d_dst, unsigned char *const *d_dst_ptrs, const int32_t *dst_idx, int64_t dst_cs,
                     int64_t dst_ss, const int32_t *copy_idx, int64_t len, int64_t nstripes, void *stream) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  const bool gather = d_src_ptrs != nullptr;
  bool any_copy = false;
  if (copy_idx)
    for (int j = 0; j < k; j++) any_copy |= copy_idx[j] >= 0;
  if (k < 1 || k > NXEC_MAX_K || rows < 0 || rows > NXEC_MAX_K || (rows == 0 && !any_copy))
    return set_error(NXEC_ERR_INVALID, "rows=%d k=%d out of range", rows, k);
  if (len < 0 || nstripes < 0) return set_error(NXEC_ERR_INVALID, "negative len or nstripes");
  if (rows > 0 && !coeffs) return set_error(NXEC_ERR_INVALID, "null coefficient matrix");
  if (len == 0 || nstripes == 0) return NXEC_OK;
  if (gather) {
    if (!d_dst_ptrs) return set_error(NXEC_ERR_INVALID, "gather form needs both pointer tables");
  } else if (!d_src || (!d_dst && (rows > 0 || any_copy))) {
    return set_error(NXEC_ERR_INVALID, "null stripe buffer");
  }
  int rc = ensure_device(ctx->device);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);

  MulArgs a;
  std::memset(&a, 0, sizeof(a));
  a.src = d_src;
  a.dst = d_dst;
  a.src_ptrs = d_src_ptrs;
  a.dst_ptrs = d_dst_ptrs;
  a.src_chunk_stride = src_cs;
  a.src_stripe_stride = src_ss;
  a.dst_chunk_stride = dst_cs;
  a.dst_stripe_stride = dst_ss;
  a.len = len;
  a.nstripes = nstripes;
  a.k = k;
  a.dst_ptr_rows = rows;
  if (gather && any_copy) return set_error(NXEC_ERR_INVALID, "copy_idx is only supported in the strided form");
  // chunk byte offsets inside a stripe (kept 32-bit for the kernels' scalar address math)
  auto chunk_off = [&](int32_t idx, int64_t stride, uint32_t *out) -> bool {
    if (idx < 0) return false;
    const int64_t off = static_cast<int64_t>(idx) * stride;
    if (stride < 0 || off + len > (int64_t(1) << 32) - 1) return false;
    *out = static_cast<uint32_t>(off);
    return true;
  };
  for (int j = 0; j < k && !gather; j++) {
    const int32_t si = src_idx ? src_idx[j] : j;
    if (!chunk_off(si, src_cs, &a.src_off[j]))
      return set_error(NXEC_ERR_INVALID, "src_idx[%d]=%d: offset out of range (chunks of a stripe must lie within 4 GiB)",
                       j, si);
    a.copy_off[j] = kNoCopy;
    if (copy_idx && copy_idx[j] >= 0 && !chunk_off(copy_idx[j], dst_cs, &a.copy_off[j]))
      return set_error(NXEC_ERR_INVALID, "copy_idx[%d]=%d: offset out of range", j, copy_idx[j]);
  }

  bool vec_ok = true;
  if (!gather) {
    vec_ok = aligned16(d_src) && aligned16(d_dst) && (src_cs % 16 == 0) && (src_ss % 16 == 0) &&
             (dst_cs % 16 == 0) && (dst_ss % 16 == 0);
  }
  // gather form: the kernels assume 16-byte aligned chunk pointers
  const int64_t vec_count = vec_ok ? len / 16 : 0;
  a.vec_count = vec_count;
  a.byte_begin = vec_count * 16;

  // split nstripes so one launch's tile count fits 32 bits
  const int64_t tps = std::max<int64_t>(1, (vec_count + 1023) / 1024);
  const int64_t max_stripes = std::max<int64_t>(1, ((int64_t(1) << 31) / tps));

  const int passes = rows == 0 ? 1 : (rows + kMaxRowsPerPass - 1) / kMaxRowsPerPass;
  for (int p = 0; p < passes; p++) {
    const int r0 = p * kMaxRowsPerPass;
    const int pr = std::min(kMaxRowsPerPass, rows - r0);
    a.rows = std::max(pr, 0);
    a.any_copy = (p == 0 && any_copy) ? 1 : 0;
    a.dst_ptr_row0 = r0;
    for (int r = 0; r < kMaxRowsPerPass; r++) {
      const int rr = r0 + r;
      a.dst_off[r] = 0;
      if (r < pr && !gather) {
        const int32_t di = dst_idx ? dst_idx[rr] : rr;
        if (!chunk_off(di, dst_cs, &a.dst_off[r]))
          return set_error(NXEC_ERR_INVALID, "dst_idx[%d]=%d: offset out of range", rr, di);
      }
      for (int j = 0; j < k; j++) a.coef[r * k + j] = r < pr ? coeffs[static_cast<size_t>(rr) * k + j] : 0;
    }
    for (int64_t s0 = 0; s0 < nstripes; s0 += max_stripes) {
      MulArgs b = a;
      b.nstripes = std::min(max_stripes, nstripes - s0);
      if (gather) {
        b.src_ptrs = d_src_ptrs + s0 * k;
        b.dst_ptrs = d_dst_ptrs + s0 * rows;
      } else {
        b.src = d_src + s0 * src_ss;
        b.dst = d_dst ? d_dst + s0 * dst_ss : nullptr;
      }
      rc = launch_mul(b, vec_ok, ctx->num_cus, st);
      if (rc) return rc;
    }
  }
  return NXEC_OK;
}

}  // namespace

extern "C" {

const char *nxec_last_error(void) { return g_last_error.c_str(); }
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

namespace {
// an event pair around a coding launch when nxec_kernel_timing is on (else nulls)
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
}  // namespace

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

int nxec_stripes_mul(nxec_ctx_t *ctx, int rows, int k, const unsigned char *coeffs, const unsigned char *d_src,
                     const int32_t *src_idx, int64_t src_chunk_stride, int64_t src_stripe_stride,
                     unsigned char *d_dst, const int32_t *dst_idx, int64_t dst_chunk_stride,
                     int64_t dst_stripe_stride, const int32_t *copy_idx, int64_t len, int64_t nstripes,
                     void *stream) {
  return stripes_mul_impl(ctx, rows, k, coeffs, d_src, nullptr, src_idx, src_chunk_stride, src_stripe_stride, d_dst,
                          nullptr, dst_idx, dst_chunk_stride, dst_stripe_stride, copy_idx, len, nstripes, stream);
}

int nxec_matmul_batch(nxec_ctx_t *ctx, int rows, int k, const unsigned char *coeffs, const unsigned char *d_src,
                      int64_t src_chunk_stride, int64_t src_stripe_stride, unsigned char *d_dst,
                      int64_t dst_chunk_stride, int64_t dst_stripe_stride, int64_t len, int64_t nstripes,
                      void *stream) {
  return nxec_stripes_mul(ctx, rows, k, coeffs, d_src, nullptr, src_chunk_stride, src_stripe_stride, d_dst, nullptr,
                          dst_chunk_stride, dst_stripe_stride, nullptr, len, nstripes, stream);
}

int nxec_encode_data(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *src,
                     unsigned char *const *dst) {
  return nxec_encode_host(len, k, rows, coeffs, src, dst);
}

int nxec_stripes_mul_ptrs(nxec_ctx_t *ctx, int rows, int k, const unsigned char *coeffs,
                          const unsigned char *const *d_src_ptrs, unsigned char *const *d_dst_ptrs, int64_t len,
                          int64_t nstripes, void *stream) {
  if (!d_src_ptrs) return set_error(NXEC_ERR_INVALID, "null source pointer table");
  if (rows < 1) return set_error(NXEC_ERR_INVALID, "rows must be >= 1");
  return stripes_mul_impl(ctx, rows, k, coeffs, nullptr, d_src_ptrs, nullptr, 0, 0, nullptr, d_dst_ptrs, nullptr, 0,
                          0, nullptr, len, nstripes, stream);
}

int nxec_rs_encode_stripes(nxec_ctx_t *ctx, int n, int k, unsigned char *d_stripes, int64_t chunk_stride,
                           int64_t stripe_stride, int64_t len, int64_t nstripes, void *stream) {
  if (!valid_nk(n, k)) return set_error(NXEC_ERR_INVALID, "invalid (n,k)=(%d,%d)", n, k);
  if (n == k) return NXEC_OK;
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
  nxec_gf_gen_rs_matrix(enc.data(), n, k);  // rs.cc:26
  std::vector<int32_t> dst(n - k);
  for (int i = k; i < n; i++) dst[i - k] = i;
  return nxec_stripes_mul(ctx, n - k, k, enc.data() + static_cast<size_t>(k) * k, d_stripes, nullptr, chunk_stride,
                          stripe_stride, d_stripes, dst.data(), chunk_stride, stripe_stride, nullptr, len, nstripes,
                          stream);
}

int nxec_rs_recover_stripes(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                            unsigned char *d_stripes, int64_t chunk_stride, int64_t stripe_stride, int64_t len,
                            int64_t nstripes, void *stream) {
  if (!valid_nk(n, k)) return set_error(NXEC_ERR_INVALID, "invalid (n,k)=(%d,%d)", n, k);
  if (nfailed == 0) return NXEC_OK;
  std::vector<int32_t> inputs(n);
  std::vector<uint8_t> rm(static_cast<size_t>(std::max(nfailed, 1)) * k);
  int ni = 0, mi = 0;
  int rc = nxec_rs_plan(n, k, failed, nfailed, 1, inputs.data(), &ni, &mi, rm.data());  // rs.cc:238-322
  if (rc) return rc;
  return nxec_stripes_mul(ctx, nfailed, k, rm.data(), d_stripes, inputs.data(), chunk_stride, stripe_stride,
                          d_stripes, failed, chunk_stride, stripe_stride, nullptr, len, nstripes, stream);
}

int nxec_rs_decode_stripes(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                           const unsigned char *d_stripes, int64_t chunk_stride, int64_t stripe_stride,
                           unsigned char *d_out, int64_t out_chunk_stride, int64_t out_stripe_stride, int64_t len,
                           int64_t nstripes, void *stream) {
  if (!valid_nk(n, k)) return set_error(NXEC_ERR_INVALID, "invalid (n,k)=(%d,%d)", n, k);
  std::vector<int32_t> inputs(n);
  int ni = 0, mi = 0;
  int rc = nxec_rs_plan(n, k, failed, nfailed, 0, inputs.data(), &ni, &mi, nullptr);  // rs.cc:252-265
  if (rc) return rc;
  // erased data chunks get inverse rows (rs.cc:196,228-230); surviving data
  // chunks are unit rows of the inverse, i.e. copies of their input.
  std::vector<int32_t> targets, copy(k, -1);
  for (int i = 0; i < nfailed; i++)
    if (failed[i] < k) targets.push_back(failed[i]);
  for (int j = 0; j < k; j++)
    if (inputs[j] < k) copy[j] = inputs[j];
  std::vector<uint8_t> m(std::max<size_t>(1, targets.size() * k));
  if (!targets.empty()) {
    rc = nxec_rs_decode_matrix(n, k, inputs.data(), targets.data(), static_cast<int>(targets.size()), m.data());
    if (rc) return rc;
  }
  return stripes_mul_impl(ctx, static_cast<int>(targets.size()), k, m.data(), d_stripes, nullptr, inputs.data(),
                          chunk_stride, stripe_stride, d_out, nullptr, targets.data(), out_chunk_stride,
                          out_stripe_stride, copy.data(), len, nstripes, stream);
}

int nxec_rs_car_repair_stripes(nxec_ctx_t *ctx, int n, int k, int failed, const int32_t *group_offsets,
                               const int32_t *group_chunks, int ngroups, unsigned char *d_stripes, int64_t chunk_stride,
                               int64_t stripe_stride, unsigned char *d_partials, int64_t partial_chunk_stride,
                               int64_t partial_stripe_stride, int64_t len, int64_t nstripes, void *stream) {
  if (!valid_nk(n, k)) return set_error(NXEC_ERR_INVALID, "invalid (n,k)=(%d,%d)", n, k);
  std::vector<int32_t> so(static_cast<size_t>(std::max(ngroups, 0)) + 2), sc(k);
  std::vector<unsigned char> cf(k);
  int ns = 0;
  int rc = nxec_car_plan(n, k, failed, group_offsets, group_chunks, ngroups, so.data(), sc.data(), cf.data(), &ns);
  if (rc) return rc;
  if (!d_partials || partial_chunk_stride < len || partial_stripe_stride < (ns - 1) * partial_chunk_stride + len)
    return set_error(NXEC_ERR_INVALID, "nxec_rs_car_repair_stripes: partials layout too small");
  for (int g = 0; g < ns; g++) {  // agent partial encodes (container_manager.cc:251)
    const int32_t dst = g;
    rc = nxec_stripes_mul(ctx, 1, so[g + 1] - so[g], cf.data() + so[g], d_stripes, sc.data() + so[g], chunk_stride,
                          stripe_stride, d_partials, &dst, partial_chunk_stride, partial_stripe_stride, nullptr, len,
                          nstripes, stream);
    if (rc) return rc;
  }
  std::vector<unsigned char> ones(ns, 1);  // CAR finalize: XOR of the partials (rs.cc:94-109)
  const int32_t tgt = failed;
  return nxec_stripes_mul(ctx, 1, ns, ones.data(), d_partials, nullptr, partial_chunk_stride, partial_stripe_stride, d_stripes, &tgt,
                          chunk_stride, stripe_stride, nullptr, len, nstripes, stream);
}

int nxec_md5_chunks(nxec_ctx_t *ctx, const unsigned char *d_base, int64_t chunk_stride, int64_t stripe_stride,
                    int nchunks, int64_t len, int64_t nstripes, unsigned char *d_digests, void *stream) {
  if (!ctx || nchunks < 0 || len < 0 || nstripes < 0 || ((nchunks > 0 && nstripes > 0) && (!d_base || !d_digests)))
    return set_error(NXEC_ERR_INVALID, "nxec_md5_chunks: invalid arguments");
  int rc = ensure_device(ctx->device);
  if (rc) return rc;
  const Md5Region r{d_base, chunk_stride, stripe_stride, len, nstripes, d_digests, int64_t(nchunks) * 16, nchunks};
  return launch_md5(&r, 1, pick_stream(ctx, stream));
}

int nxec_md5_verify_chunks(nxec_ctx_t *ctx, const unsigned char *d_base, int64_t chunk_stride, int64_t stripe_stride,
                           int nchunks, int64_t len, int64_t nstripes, const unsigned char *d_expected,
                           unsigned char *d_ok, unsigned long long *d_nbad, void *stream) {
  if (!ctx || nchunks < 0 || len < 0 || nstripes < 0 ||
      ((nchunks > 0 && nstripes > 0) && (!d_base || !d_expected || !d_ok)))
    return set_error(NXEC_ERR_INVALID, "nxec_md5_verify_chunks: invalid arguments");
  int rc = ensure_device(ctx->device);
  if (rc) return rc;
  // the kernel only reads the digests in verify mode
  const Md5Region r{d_base, chunk_stride, stripe_stride, len, nstripes, const_cast<unsigned char *>(d_expected),
                    int64_t(nchunks) * 16, nchunks, d_ok, nchunks};
  return launch_md5(&r, 1, pick_stream(ctx, stream), d_nbad);
}

}  // extern "C"

namespace {

// Fused write-path launch (encode + MD5 of all n chunks): data chunk j of
// stripe s at data + s*data_ss + j*data_cs, parity row r at parity + s*par_ss
// + r*par_cs, digests [s][n][16].  False when the fused kernel cannot take it.
bool encode_md5_args(int n, int k, const unsigned char *data, int64_t data_cs, int64_t data_ss, unsigned char *parity,
                     int64_t par_cs, int64_t par_ss, unsigned char *digests, int64_t len, int64_t nstripes,
                     MulMd5Args &a) {
  const int p = n - k;
  if (k > kEncMd5MaxK || p < 1 || p > kMaxRowsPerPass) return false;
  if (int64_t(k - 1) * data_cs >= (int64_t(1) << 32) || int64_t(p - 1) * par_cs >= (int64_t(1) << 32)) return false;
  a = MulMd5Args{};
  for (int j = 0; j < k; j++) a.src_off[j] = static_cast<uint32_t>(j * data_cs);
  for (int r = 0; r < p; r++) a.dst_off[r] = static_cast<uint32_t>(r * par_cs);
  if (!mul_md5_eligible(k, p, len, data, data_ss, a.src_off, parity, par_ss, a.dst_off)) return false;
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
  nxec_gf_gen_rs_matrix(enc.data(), n, k);  // rs.cc:26
  std::memcpy(a.coef, enc.data() + static_cast<size_t>(k) * k, static_cast<size_t>(p) * k);
  a.src = data;
  a.src_stripe_stride = data_ss;
  a.dst = parity;
  a.dst_stripe_stride = par_ss;
  a.digests = digests;
  a.digest_stripe_stride = int64_t(n) * 16;
  a.len = len;
  a.nstripes = nstripes;
  a.k = k;
  a.p = p;
  a.hash_src = a.hash_dst = 1;
  for (int c = 0; c < n; c++) a.digest_slot[c] = static_cast<uint8_t>(c);
  return true;
}

}  // namespace

extern "C" {

int nxec_rs_encode_md5_stripes(nxec_ctx_t *ctx, int n, int k, unsigned char *d_stripes, int64_t chunk_stride,
                               int64_t stripe_stride, int64_t len, int64_t nstripes, unsigned char *d_digests,
                               void *stream) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  if (!valid_nk(n, k)) return set_error(NXEC_ERR_INVALID, "invalid (n,k)=(%d,%d)", n, k);
  if (len < 0 || nstripes < 0 || ((len > 0 && nstripes > 0) && (!d_stripes || !d_digests)))
    return set_error(NXEC_ERR_INVALID, "nxec_rs_encode_md5_stripes: invalid arguments");
  if (nstripes == 0) return NXEC_OK;
  MulMd5Args ea;
  if (encode_md5_args(n, k, d_stripes, chunk_stride, stripe_stride, d_stripes + int64_t(k) * chunk_stride, chunk_stride,
                      stripe_stride, d_digests, len, nstripes, ea)) {
    int rc = ensure_device(ctx->device);
    if (rc) return rc;
    return launch_mul_md5(ea, ctx->num_cus, pick_stream(ctx, stream));
  }
  int rc = nxec_rs_encode_stripes(ctx, n, k, d_stripes, chunk_stride, stripe_stride, len, nstripes, stream);
  return rc ? rc : nxec_md5_chunks(ctx, d_stripes, chunk_stride, stripe_stride, n, len, nstripes, d_digests, stream);
}

int nxec_rs_recover_md5_stripes(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                                unsigned char *d_stripes, int64_t chunk_stride, int64_t stripe_stride, int64_t len,
                                int64_t nstripes, unsigned char *d_digests, void *stream) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  if (!valid_nk(n, k)) return set_error(NXEC_ERR_INVALID, "invalid (n,k)=(%d,%d)", n, k);
  if (nfailed < 0 || len < 0 || nstripes < 0 || (nfailed > 0 && !failed) ||
      ((nfailed > 0 && len > 0 && nstripes > 0) && (!d_stripes || !d_digests)))
    return set_error(NXEC_ERR_INVALID, "nxec_rs_recover_md5_stripes: invalid arguments");
  if (nfailed == 0 || nstripes == 0) return NXEC_OK;
  std::vector<int32_t> inputs(n);
  std::vector<uint8_t> rm(static_cast<size_t>(nfailed) * k);
  int ni = 0, mi = 0;
  int rc = nxec_rs_plan(n, k, failed, nfailed, 1, inputs.data(), &ni, &mi, rm.data());  // rs.cc:238-322
  if (rc) return rc;
  bool fused = k <= kEncMd5MaxK && nfailed <= kMaxRowsPerPass && int64_t(n - 1) * chunk_stride < (int64_t(1) << 32);
  MulMd5Args a{};
  if (fused) {
    for (int j = 0; j < k; j++) a.src_off[j] = static_cast<uint32_t>(inputs[j] * chunk_stride);
    for (int r = 0; r < nfailed; r++) a.dst_off[r] = static_cast<uint32_t>(failed[r] * chunk_stride);
    fused = mul_md5_eligible(k, nfailed, len, d_stripes, stripe_stride, a.src_off, d_stripes, stripe_stride, a.dst_off);
  }
  if (fused) {
    if ((rc = ensure_device(ctx->device))) return rc;
    a.src = d_stripes;
    a.src_stripe_stride = stripe_stride;
    a.dst = d_stripes;
    a.dst_stripe_stride = stripe_stride;
    a.digests = d_digests;
    a.digest_stripe_stride = int64_t(nfailed) * 16;
    a.len = len;
    a.nstripes = nstripes;
    a.k = k;
    a.p = nfailed;
    a.hash_src = 0;
    a.hash_dst = 1;
    for (int r = 0; r < nfailed; r++) a.digest_slot[r] = static_cast<uint8_t>(r);
    std::memcpy(a.coef, rm.data(), rm.size());
    return launch_mul_md5(a, ctx->num_cus, pick_stream(ctx, stream));
  }
  rc = nxec_rs_recover_stripes(ctx, n, k, failed, nfailed, d_stripes, chunk_stride, stripe_stride, len, nstripes, stream);
  if (rc) return rc;
  if ((rc = ensure_device(ctx->device))) return rc;
  for (int r0 = 0; r0 < nfailed; r0 += kMaxMd5Regions) {  // one MD5 launch per 4 rebuilt chunks
    Md5Region reg[kMaxMd5Regions];
    int nr = 0;
    for (int r = r0; r < nfailed && nr < kMaxMd5Regions; r++, nr++)
      reg[nr] = Md5Region{d_stripes + failed[r] * chunk_stride, chunk_stride, stripe_stride, len, nstripes,
                          d_digests + int64_t(r) * 16, int64_t(nfailed) * 16, 1};
    if ((rc = launch_md5(reg, nr, pick_stream(ctx, stream)))) return rc;
  }
  return NXEC_OK;
}

int nxec_batch_layout(int n, int64_t len, int flags, int64_t *chunk_stride, int64_t *stripe_stride) {
  if (n < 1 || n > NXEC_MAX_N || len < 0 || !chunk_stride || !stripe_stride)
    return set_error(NXEC_ERR_INVALID, "nxec_batch_layout: invalid arguments");
  constexpr int64_t kMiB = int64_t(1) << 20;
  int64_t cs = (len + 15) / 16 * 16;
  if (len >= 2 * kMiB) cs += 2048;  // break the power-of-two chunk stride (profiles/r02_layout_sweep.log)
  int64_t ss = cs * n;
  // stripes of a power-of-two number of MiB alias worst: an odd multiple of
  // the chunk wins for every op there ((16,12) 1 MiB: encode 0.798 -> 0.812,
  // single repairs 0.74 -> 0.79); elsewhere only scattered recovers gain
  if (cs % kMiB == 0 && (ss / kMiB) % 2 == 0) {
    const int64_t mib = ss / kMiB;
    if ((mib & (mib - 1)) == 0 || (flags & NXEC_LAYOUT_RECOVER_HEAVY)) ss += cs;
  }
  *chunk_stride = cs;
  *stripe_stride = ss;
  return NXEC_OK;
}

int nxec_object_layout(int n, int k, int64_t length, int64_t max_chunk_size, int64_t *nstripes,
                       int64_t *full_stripes, int64_t *last_chunk_size) {
  if (!valid_nk(n, k) || length < 0 || max_chunk_size <= 0 || !nstripes || !full_stripes || !last_chunk_size)
    return set_error(NXEC_ERR_INVALID, "nxec_object_layout: invalid arguments");
  const int64_t stripe_data = max_chunk_size * k;  // getMaxDataSizePerStripe (chunk_manager.cc:1395-1400)
  *full_stripes = length / stripe_data;
  const int64_t rem = length - *full_stripes * stripe_data;
  *nstripes = *full_stripes + (rem > 0 ? 1 : 0);
  *last_chunk_size = rem > 0 ? (rem + k - 1) / k : (*full_stripes > 0 ? max_chunk_size : 0);  // rs.cc:52-55
  return NXEC_OK;
}

int nxec_encode_object(nxec_ctx_t *ctx, int n, int k, const unsigned char *d_object, int64_t length,
                       int64_t max_chunk_size, unsigned char *d_parity, unsigned char *d_tail, unsigned char *d_md5,
                       void *stream) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  int64_t ns = 0, nf = 0, cs_last = 0;
  int rc = nxec_object_layout(n, k, length, max_chunk_size, &ns, &nf, &cs_last);
  if (rc) return rc;
  if (ns == 0) return NXEC_OK;
  const int p = n - k;
  const int64_t M = max_chunk_size;
  const bool tail = ns > nf;
  if (!d_object || (p > 0 && !d_parity) || (tail && !d_tail))
    return set_error(NXEC_ERR_INVALID, "nxec_encode_object: null buffer");
  rc = ensure_device(ctx->device);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
  nxec_gf_gen_rs_matrix(enc.data(), n, k);
  const uint8_t *prow = enc.data() + static_cast<size_t>(k) * k;
  // full stripes: data chunks are read in place from the object (no copy of
  // rs.cc:80), parity chunk (s, i) at d_parity + (s*p + i)*M; with digests
  // wanted, the encode and the MD5 of all n chunks run as one kernel
  const int64_t ds = int64_t(n) * 16;
  MulMd5Args ea;
  const bool fused = d_md5 && nf > 0 && encode_md5_args(n, k, d_object, M, k * M, d_parity, M, p * M, d_md5, M, nf, ea);
  if (fused) {
    rc = launch_mul_md5(ea, ctx->num_cus, st);
    if (rc) return rc;
  } else if (nf > 0 && p > 0) {
    rc = nxec_stripes_mul(ctx, p, k, prow, d_object, nullptr, M, k * M, d_parity, nullptr, M, p * M, nullptr, M, nf,
                          st);
    if (rc) return rc;
  }
  const unsigned char *tail_src = d_object + nf * k * M;
  const int64_t rem = length - nf * k * M;
  if (tail) {  // last stripe: zero-padded to k * cs_last (encodeFile's realloc+memset, chunk_manager.cc:390-399)
    rc = hip_check(hipMemcpyAsync(d_tail, tail_src, rem, hipMemcpyDeviceToDevice, st), "tail copy");
    if (!rc && k * cs_last > rem)
      rc = hip_check(hipMemsetAsync(d_tail + rem, 0, k * cs_last - rem, st), "tail pad");
    if (!rc && p > 0)
      rc = nxec_stripes_mul(ctx, p, k, prow, d_tail, nullptr, cs_last, k * cs_last, d_parity + nf * p * M, nullptr, M,
                            p * M, nullptr, cs_last, 1, st);
    if (rc) return rc;
  }
  if (!d_md5) return NXEC_OK;
  // per-chunk MD5 (writeFileStripe -> Chunk::computeMD5, chunk_manager.cc:175): one launch over
  // full-stripe data, full-stripe parity, tail data, tail parity; digests
  // [s][n][16] (the full stripes' are done when the fused kernel ran)
  const int64_t nfm = fused ? 0 : nf;
  const Md5Region r[4] = {
      {d_object, M, k * M, M, nfm, d_md5, ds, k},
      {d_parity, M, p * M, M, nfm, d_md5 + int64_t(k) * 16, ds, p},
      {d_tail, cs_last, k * cs_last, cs_last, tail ? 1 : 0, d_md5 + nf * ds, ds, k},
      {d_parity + nf * p * M, M, p * M, cs_last, tail ? 1 : 0, d_md5 + nf * ds + int64_t(k) * 16, ds, p},
  };
  return launch_md5(r, 4, st);
}

int nxec_objects_layout(int n, int k, int nobjects, const int64_t *lengths, int64_t max_chunk_size,
                        int64_t *total_stripes, int64_t *tail_bytes) {
  if (!valid_nk(n, k) || nobjects < 0 || (nobjects > 0 && !lengths) || max_chunk_size <= 0 || !total_stripes ||
      !tail_bytes)
    return set_error(NXEC_ERR_INVALID, "nxec_objects_layout: invalid arguments");
  *total_stripes = 0;
  *tail_bytes = 0;
  for (int o = 0; o < nobjects; o++) {
    int64_t ns = 0, nf = 0, cl = 0;
    int rc = nxec_object_layout(n, k, lengths[o], max_chunk_size, &ns, &nf, &cl);
    if (rc) return rc;
    *total_stripes += ns;
    if (ns > nf) *tail_bytes += int64_t(k) * ((cl + 15) / 16 * 16);
  }
  return NXEC_OK;
}

int nxec_encode_objects(nxec_ctx_t *ctx, int n, int k, int nobjects, const unsigned char *const *d_objects,
                        const int64_t *lengths, int64_t max_chunk_size, unsigned char *d_parity,
                        unsigned char *d_tail, unsigned char *d_md5, void *stream) {
  return nxec_encode_objects_ex(ctx, n, k, nobjects, d_objects, lengths, max_chunk_size, d_parity, d_tail, d_md5, 0,
                                stream);
}

int nxec_encode_objects_ex(nxec_ctx_t *ctx, int n, int k, int nobjects, const unsigned char *const *d_objects,
                           const int64_t *lengths, int64_t max_chunk_size, unsigned char *d_parity,
                           unsigned char *d_tail, unsigned char *d_md5, int flags, void *stream) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  if (flags & ~(NXEC_OBJECTS_TAIL_INPLACE | NXEC_OBJECTS_ASYNC))
    return set_error(NXEC_ERR_INVALID, "nxec_encode_objects_ex: flags %d", flags);
  const bool async = flags & NXEC_OBJECTS_ASYNC;
  // NXEC_TIMING=1: the host side's share of the call on stderr (planning, tables, launch, wait)
  static const bool timing = [] {
    const char *e = std::getenv("NXEC_TIMING");
    return e && e[0] == '1';
  }();
  const auto th0 = std::chrono::steady_clock::now();
  auto ms_since = [&](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  };
  int64_t total = 0, tail_total = 0;
  int rc = nxec_objects_layout(n, k, nobjects, lengths, max_chunk_size, &total, &tail_total);
  if (rc) return rc;
  if (total == 0) return NXEC_OK;
  const int p = n - k;
  const int64_t M = max_chunk_size;
  if (!d_objects || (p > 0 && !d_parity) || (tail_total > 0 && !d_tail))
    return set_error(NXEC_ERR_INVALID, "nxec_encode_objects: null buffer");
  for (int o = 0; o < nobjects; o++)
    if (lengths[o] > 0 && !d_objects[o]) return set_error(NXEC_ERR_INVALID, "nxec_encode_objects: object %d is NULL", o);
  rc = ensure_device(ctx->device);
  if (rc) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
  nxec_gf_gen_rs_matrix(enc.data(), n, k);
  const uint8_t *prow = enc.data() + static_cast<size_t>(k) * k;

  // Host plan, every table to the device in one copy:
  //  * full stripes of every object: gather pointer tables, one k_mul_vec launch
  //    (objects not 16-byte aligned: the byte-capable list kernel instead);
  //  * each object's last stripe: its k chunks copied zero-padded into the
  //    tail arena at 16-byte-aligned chunk strides (one k_pad_chunks launch),
  //    then coded as aligned ragged stripes (one k_mul_ragged launch; the list
  //    kernel when parity slots are not 16-byte aligned or k > 19);
  //  * every chunk an MD5 item (one launch).
  std::vector<const uint8_t *> fsrc;
  std::vector<uint8_t *> fdst;
  std::vector<PadChunks> pads;
  std::vector<uint32_t> pad_bstart;
  std::vector<ListStripe> ragged, ulist;
  std::vector<uint32_t> stripe_tile0, tile_stripe;
  std::vector<int64_t> uprefix(1, 0);
  std::vector<Md5Item> items, ritems;
  bool full_aligned = M % 16 == 0;
  // ragged stripes through the aligned work-queue kernel: parity slots must be
  // 16-byte aligned (else they join the byte-capable list kernel)
  const bool ragged_ok = p > 0 && M % 16 == 0 && (reinterpret_cast<uintptr_t>(d_parity) & 15) == 0 && k <= kMaxRaggedK;
  // one launch for every stripe's coding and every chunk's MD5 (k_files_md5):
  // full stripes in place, last stripes straight from their objects (the kernel
  // also writes their zero-padded data chunks to the tail arena; NXEC_FUSED_MD5=0:
  // pad copy + the separate launches, for A/B)
  // NXEC_FILES_TAIL=0: last stripes through the pad copy into the tail arena
  // first, then read from there (A/B of the in-kernel tail reads)
  const char *tenv = std::getenv("NXEC_FILES_TAIL");
  const bool tail_direct = !(tenv && tenv[0] == '0');
  const char *fenv = std::getenv("NXEC_FUSED_MD5");
  const bool want_fused = !(fenv && fenv[0] == '0') && d_md5 && ragged_ok && p <= kMaxRowsPerPass &&
                          k <= kFilesMd5MaxK;
  std::vector<const uint8_t *> q_src, q_tsrc;
  std::vector<uint8_t *> q_dst, q_dig;
  std::vector<int64_t> q_len, q_trem;
  // full stripes are read in place: 16-byte aligned objects (any object whose
  // only stripe is its last one is read byte-wise, or padded, either way)
  for (int o = 0; o < nobjects && full_aligned; o++)
    full_aligned = (reinterpret_cast<uintptr_t>(d_objects[o]) & 15) == 0 || lengths[o] < int64_t(k) * M;
  // the fused launch plans only its own tables; the separate launches only theirs
  const bool fused = want_fused && full_aligned;
  const bool sep = !fused;
  const bool need_pads = sep || !tail_direct;
  // NXEC_OBJECTS_TAIL_INPLACE on the one-launch path (NXEC_FILES_TAIL=0 keeps the whole-tail pad copy)
  // Without the flag (whole tail arena) last stripes are in-place requests
  // too, and the kernel also stores their whole data chunks to the tail
  // arena (tail_store); NXEC_FILES_COPY=kernel: the kernel's older last-stripe
  // path that reads the tail bytes itself (A/B)
  static const bool copy_in_kernel = [] {
    const char *e = std::getenv("NXEC_FILES_COPY");
    return e && e[0] == 'k';
  }();
  const bool tstore = !(flags & NXEC_OBJECTS_TAIL_INPLACE) && fused && tail_direct && !copy_in_kernel;
  const bool inplace = ((flags & NXEC_OBJECTS_TAIL_INPLACE) || tstore) && fused && tail_direct;
  int64_t g = 0, toff = 0, pad_blocks = 0;
  for (int o = 0; o < nobjects; o++) {
    int64_t ns = 0, nf = 0, cl = 0;
    nxec_object_layout(n, k, lengths[o], M, &ns, &nf, &cl);
    const uint8_t *obj = d_objects[o];
    for (int64_t s = 0; s < ns; s++, g++) {
      uint8_t *par = d_parity ? d_parity + g * p * M : nullptr;
      uint8_t *dig = d_md5 ? d_md5 + g * n * 16 : nullptr;
      if (s < nf) {
        if (sep) {
          for (int j = 0; j < k; j++) fsrc.push_back(obj + (s * k + j) * M);
          for (int i = 0; i < p; i++) fdst.push_back(par + i * M);
        }
        if (fused) {
          for (int j = 0; j < k; j++) q_src.push_back(obj + (s * k + j) * M);
          for (int i = 0; i < p; i++) q_dst.push_back(par + i * M);
          q_len.push_back(M);
          q_dig.push_back(dig);
          q_tsrc.push_back(nullptr);
          q_trem.push_back(0);
        }
        if (sep && dig) {
          for (int j = 0; j < k; j++) items.push_back({obj + (s * k + j) * M, M, dig + j * 16});
          for (int i = 0; i < p; i++) items.push_back({par + i * M, M, dig + (k + i) * 16});
        }
      } else {  // last stripe (chunk_manager.cc:390-399)
        const int64_t cls = (cl + 15) / 16 * 16;
        uint8_t *td = d_tail + toff;
        if (need_pads) {
          pads.push_back({obj + nf * k * M, td, lengths[o] - nf * k * M, cl, cls, k});
          pad_bstart.push_back(static_cast<uint32_t>(pad_blocks));
          pad_blocks += (cls / 16 * k + 256 * kPadVecs - 1) / (256 * kPadVecs);
        }
        if (sep && p > 0 && !ragged_ok) {
          ulist.push_back({td, par, cl, cls, M});
          uprefix.push_back(uprefix.back() + (cl + 15) / 16);
        } else if (sep && p > 0) {
          const uint32_t s_idx = static_cast<uint32_t>(ragged.size());
          ragged.push_back({td, par, cls, cls, M});
          stripe_tile0.push_back(static_cast<uint32_t>(tile_stripe.size()));
          const int64_t nt = (cls / 16 + 1023) / 1024;
          for (int64_t t = 0; t < nt; t++) tile_stripe.push_back(s_idx);
        }
        if (sep && dig) {
          for (int j = 0; j < k; j++) ritems.push_back({td + j * cls, cl, dig + j * 16});
          for (int i = 0; i < p; i++) ritems.push_back({par + i * M, cl, dig + (k + i) * 16});
        }
        if (fused && inplace) {
          // In place: the last stripe becomes an ordinary request.  Its data
          // chunks below j0 are read where they lie in the object (no byte of
          // theirs is zero padding, and their 16-byte column vectors stay
          // inside the tail's last 16-byte line); chunks j0.. -- the partial
          // one, the all-zero ones, and a whole one whose last vector would
          // run past that line -- are first written zero-padded to their
          // tail-arena slots by one small copy launch and read from there.
          // The kernel then needs none of its per-step last-stripe handling
          // (4.6 -> ~3.7 us per step of a last-stripe workgroup).
          const uint8_t *tb = obj + nf * k * M;
          const int64_t rem = lengths[o] - nf * k * M;
          const int64_t jf = std::min<int64_t>(rem / cl, k), last = jf < k ? rem - jf * cl : 0;  // r % cl
          const int64_t safe = static_cast<int64_t>(((reinterpret_cast<uintptr_t>(tb) + rem + 15) & ~uintptr_t(15)) -
                                                    reinterpret_cast<uintptr_t>(tb));
          (void)last;
          int64_t j0 = jf;  // the partial chunk (last > 0), else the first all-zero one (or k: none)
          const int64_t jov = safe >= cls ? (safe - cls) / cl + 1 : 0;  // first chunk reading past `safe`
          j0 = std::min(j0, jov);
          for (int j = 0; j < k; j++) q_src.push_back(j < j0 ? tb + j * cl : td + j * cls);
          if (j0 < k) {
            pads.push_back({tb + j0 * cl, td + j0 * cls, rem - j0 * cl, cl, cls, k - j0});
            pad_bstart.push_back(static_cast<uint32_t>(pad_blocks));
            pad_blocks += (cls / 16 * (k - j0) + 256 * kPadVecs - 1) / (256 * kPadVecs);
          }
          for (int i = 0; i < p; i++) q_dst.push_back(par + i * M);
          q_len.push_back(cl);
          q_dig.push_back(dig);
          // tail_store: the kernel writes chunks j < j0 (read in place) to their slots
          q_tsrc.push_back(tstore ? td : nullptr);
          q_trem.push_back(tstore ? (cls | (j0 << 40)) : 0);
        } else if (fused) {  // read from the object; the kernel writes the padded chunks to td
          for (int j = 0; j < k; j++) q_src.push_back(td + j * cls);
          for (int i = 0; i < p; i++) q_dst.push_back(par + i * M);
          q_len.push_back(cl);
          q_dig.push_back(dig);
          q_tsrc.push_back(tail_direct ? obj + nf * k * M : nullptr);
          q_trem.push_back(lengths[o] - nf * k * M);
        }
        toff += k * cls;
      }
    }
  }
  // MD5 lanes in descending chunk length: a wave lasts as long as its longest
  // chain, and the first waves dispatched get a SIMD to themselves, so full
  // chunks go first and the last-stripe chunks follow longest first (sorted by
  // object, k + p items per object share one length)
  {
    const size_t per = static_cast<size_t>(n);
    std::vector<size_t> order(ritems.size() / per);
    for (size_t i = 0; i < order.size(); i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](size_t x, size_t y) { return ritems[x * per].len > ritems[y * per].len; });
    for (size_t o : order) items.insert(items.end(), ritems.begin() + o * per, ritems.begin() + (o + 1) * per);
  }
  if (pad_blocks >= (int64_t(1) << 31) || tile_stripe.size() >= (size_t(1) << 32))
    return set_error(NXEC_ERR_INVALID, "nxec_encode_objects: batch too large (split it)");
  pad_bstart.push_back(static_cast<uint32_t>(pad_blocks));
  const int64_t nfs = static_cast<int64_t>(fsrc.size()) / k;
  if (!full_aligned && nfs > 0 && p > 0) {  // unaligned objects: full stripes through the list kernel too
    for (int64_t f = 0; f < nfs; f++) {
      ulist.push_back({fsrc[f * k], fdst[f * p], M, M, M});
      uprefix.push_back(uprefix.back() + (M + 15) / 16);
    }
  }
  // fused: requests longest first (the slot planner packs them in this order)
  std::vector<const uint8_t *> f_src, f_tsrc;
  std::vector<uint8_t *> f_dst, f_dig;
  std::vector<int64_t> f_len, f_trem;
  if (fused) {
    const size_t R = q_len.size();
    std::vector<size_t> order(R);
    for (size_t i = 0; i < R; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return q_len[x] > q_len[y]; });
    f_src.reserve(R * k);
    f_dst.reserve(R * p);
    for (size_t o : order) {
      f_src.insert(f_src.end(), q_src.begin() + o * k, q_src.begin() + (o + 1) * k);
      f_dst.insert(f_dst.end(), q_dst.begin() + o * p, q_dst.begin() + (o + 1) * p);
      f_len.push_back(q_len[o]);
      f_dig.push_back(q_dig[o]);
      f_tsrc.push_back(q_tsrc[o]);
      f_trem.push_back(q_trem[o]);
    }
  }
  const std::vector<uint8_t> scratch_pad(fused ? 4096 : 0, 0);  // idle lanes' device line
  // the fused launch's slots: requests packed so one wave of workgroups runs them all
  FilesMd5Args fa;
  std::memset(&fa, 0, sizeof(fa));
  std::vector<int32_t> slot_first, slot_reqs, wg_steps;
  if (fused) plan_files_slots(f_len, k, p, ctx->num_cus, slot_first, slot_reqs, wg_steps, fa);
  struct Tab {
    const void *h;
    size_t bytes;
  };
  const Tab tabs[] = {{f_src.data(), f_src.size() * sizeof(void *)},
                      {f_dst.data(), f_dst.size() * sizeof(void *)},
                      {f_len.data(), f_len.size() * sizeof(int64_t)},
                      {f_dig.data(), f_dig.size() * sizeof(void *)},
                      {scratch_pad.data(), scratch_pad.size()},
                      {slot_first.data(), slot_first.size() * sizeof(int32_t)},
                      {slot_reqs.data(), slot_reqs.size() * sizeof(int32_t)},
                      {wg_steps.data(), wg_steps.size() * sizeof(int32_t)},
                      {f_tsrc.data(), f_tsrc.size() * sizeof(void *)},
                      {f_trem.data(), f_trem.size() * sizeof(int64_t)},
                      {fsrc.data(), fsrc.size() * sizeof(void *)},
                      {fdst.data(), fdst.size() * sizeof(void *)},
                      {pads.data(), pads.size() * sizeof(PadChunks)},
                      {pad_bstart.data(), pad_bstart.size() * sizeof(uint32_t)},
                      {ragged.data(), ragged.size() * sizeof(ListStripe)},
                      {stripe_tile0.data(), stripe_tile0.size() * sizeof(uint32_t)},
                      {tile_stripe.data(), tile_stripe.size() * sizeof(uint32_t)},
                      {ulist.data(), ulist.size() * sizeof(ListStripe)},
                      {uprefix.data(), uprefix.size() * sizeof(int64_t)},
                      {items.data(), items.size() * sizeof(Md5Item)}};
  constexpr int kTabs = sizeof(tabs) / sizeof(tabs[0]);
  size_t off[kTabs + 1] = {0};
  for (int i = 0; i < kTabs; i++) off[i + 1] = off[i] + (tabs[i].bytes + 15) / 16 * 16;
  Slot *slot = nullptr;
  const double t_plan = timing ? ms_since(th0) : 0;
  rc = acquire_slot(ctx, std::max<size_t>(off[kTabs], 16), &slot);
  if (rc) return rc;
  // the slot's staging may still be in use by an earlier call on its own stream
  rc = hip_check(hipStreamSynchronize(slot->stream), "slot sync");
  if (!rc && async && !slot->busy) rc = hip_check(hipEventCreateWithFlags(&slot->busy, hipEventDisableTiming), "slot event");
  for (int i = 0; i < kTabs && !rc; i++)
    if (tabs[i].bytes) std::memcpy(slot->h + off[i], tabs[i].h, tabs[i].bytes);
  if (!rc) rc = hip_check(hipMemcpyAsync(slot->d, slot->h, off[kTabs], hipMemcpyHostToDevice, st), "tables H2D");
  const int T0 = 10;  // the first ten tables belong to the fused launch
  auto dptr = [&](int i) { return slot->d + off[i + T0]; };
  if (fused) {
    // the whole-tail pad copy (NXEC_FILES_TAIL=0) or, in place, the few chunks
    // of each last stripe that are not read from the object; otherwise last
    // stripes read their object and the kernel writes the tail arena itself
    if (!rc && !pads.empty())
      rc = launch_pad_chunks(reinterpret_cast<const PadChunks *>(dptr(2)), reinterpret_cast<const uint32_t *>(dptr(3)),
                             int64_t(pads.size()), pad_blocks, st);
    // no last stripe read from its object (in place: all ordinary requests):
    // null tables select the kernel without the tail handling
    const bool any_tail = std::any_of(f_tsrc.begin(), f_tsrc.end(), [](const uint8_t *t) { return t != nullptr; });
    fa.tail_src = any_tail ? reinterpret_cast<const uint8_t *const *>(slot->d + off[8]) : nullptr;
    fa.tail_rem = any_tail ? reinterpret_cast<const int64_t *>(slot->d + off[9]) : nullptr;
    fa.src_ptrs = reinterpret_cast<const uint8_t *const *>(slot->d + off[0]);
    fa.dst_ptrs = reinterpret_cast<uint8_t *const *>(slot->d + off[1]);
    fa.lens = reinterpret_cast<const int64_t *>(slot->d + off[2]);
    fa.dig_ptrs = reinterpret_cast<uint8_t *const *>(slot->d + off[3]);
    fa.scratch = slot->d + off[4];
    fa.slot_first = reinterpret_cast<const int32_t *>(slot->d + off[5]);
    fa.slot_reqs = reinterpret_cast<const int32_t *>(slot->d + off[6]);
    fa.wg_steps = reinterpret_cast<const int32_t *>(slot->d + off[7]);
    fa.k = k;
    fa.p = p;
    fa.tail_partial_only = 0;  // in place, last stripes reach the kernel as ordinary requests
    fa.tail_store = tstore && any_tail ? 1 : 0;
    std::memcpy(fa.coef, prow, size_t(p) * k);
    // NXEC_FILES_CLOCK=1: per-workgroup timestamps (diagnostics, stderr)
    static const bool wg_clock = [] {
      const char *e = std::getenv("NXEC_FILES_CLOCK");
      return e && e[0] == '1';
    }();
    const int64_t nwg = static_cast<int64_t>(wg_steps.size());
    unsigned long long *d_clock = nullptr;
    if (wg_clock && !rc && hipMalloc(&d_clock, size_t(nwg) * 3 * 8) == hipSuccess) {
      (void)hipMemsetAsync(d_clock, 0, size_t(nwg) * 3 * 8, st);
      fa.wg_clock = d_clock;
    }
    if (!rc) {
      hipEvent_t kt[2];
      kt_begin(ctx, st, kt);
      rc = launch_files_md5(fa, ctx->num_cus, st);
      kt_end(ctx, kt, st);
    }
    const double t_launch = timing ? ms_since(th0) : 0;
    if (async && !d_clock) {  // the tables stay in the slot until the stream gets past the launches
      if (!rc) rc = hip_check(hipEventRecord(slot->busy, st), "slot event record");
      slot->busy_set = !rc;
      if (rc) (void)hipStreamSynchronize(st);
      release_slot(ctx, slot);
      return rc;
    }
    const int rc2 = hip_check(hipStreamSynchronize(st), "nxec_encode_objects sync");
    if (d_clock) {  // per workgroup: start, code end, hash end (100 MHz), by slot composition
      std::vector<unsigned long long> c(size_t(nwg) * 3);
      if (hipMemcpy(c.data(), d_clock, c.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
        unsigned long long t0 = ~0ull;
        for (int64_t b = 0; b < nwg; b++) t0 = std::min(t0, c[size_t(b) * 3]);
        const int64_t S = fa.slots_per_group;
        for (int64_t b = 0; b < nwg; b++) {
          int nfull = 0, ntail = 0;
          for (int64_t g = b * S; g < std::min<int64_t>((b + 1) * S, fa.nslots); g++)
            for (int32_t i = slot_first[size_t(g)]; i < slot_first[size_t(g) + 1]; i++)
              (f_tsrc[size_t(slot_reqs[size_t(i)])] ? ntail : nfull)++;
          std::fprintf(stderr, "wg %lld steps %d full %d tail %d start %.1f code_end %.1f hash_end %.1f us\n",
                       static_cast<long long>(b), wg_steps[size_t(b)], nfull, ntail,
                       (c[size_t(b) * 3] - t0) * 0.01, (c[size_t(b) * 3 + 1] - t0) * 0.01,
                       (c[size_t(b) * 3 + 2] - t0) * 0.01);
        }
      }
      (void)hipFree(d_clock);
    }
    if (timing)
      std::fprintf(stderr, "nxec_encode_objects: %d objects, %zu requests: plan %.3f ms, tables + launch %.3f ms, "
                   "wait %.3f ms\n", nobjects, f_len.size(), t_plan, t_launch - t_plan, ms_since(th0) - t_launch);
    release_slot(ctx, slot);
    return rc ? rc : rc2;
  }
  hipEvent_t kt[2];
  kt_begin(ctx, st, kt);
  if (!rc && p > 0 && full_aligned && nfs > 0)
    rc = stripes_mul_impl(ctx, p, k, prow, nullptr, reinterpret_cast<const unsigned char *const *>(dptr(0)), nullptr,
                          0, 0, nullptr, reinterpret_cast<unsigned char *const *>(dptr(1)), nullptr, 0, 0, nullptr, M,
                          nfs, st);
  if (!rc)
    rc = launch_pad_chunks(reinterpret_cast<const PadChunks *>(dptr(2)), reinterpret_cast<const uint32_t *>(dptr(3)),
                           int64_t(pads.size()), pad_blocks, st);
  // after the pad copy on the same stream: the tail arena is complete
  if (!rc && !ragged.empty())
    rc = launch_mul_ragged(p, k, prow, reinterpret_cast<const ListStripe *>(dptr(4)),
                           reinterpret_cast<const uint32_t *>(dptr(6)), reinterpret_cast<const uint32_t *>(dptr(5)),
                           int64_t(tile_stripe.size()), ctx->num_cus, st);
  if (!rc && !ulist.empty())
    rc = launch_mul_list(p, k, prow, reinterpret_cast<const ListStripe *>(dptr(7)),
                         reinterpret_cast<const int64_t *>(dptr(8)), int64_t(ulist.size()), uprefix.back(),
                         ctx->num_cus, st);
  if (!rc && !items.empty()) rc = launch_md5_list(reinterpret_cast<const Md5Item *>(dptr(9)), int64_t(items.size()), st);
  kt_end(ctx, kt, st);
  if (async) {
    if (!rc) rc = hip_check(hipEventRecord(slot->busy, st), "slot event record");
    slot->busy_set = !rc;
    if (rc) (void)hipStreamSynchronize(st);
    release_slot(ctx, slot);
    return rc;
  }
  // the tables live in the slot: drain before handing it back (synchronous call)
  const int rc2 = hip_check(hipStreamSynchronize(st), "nxec_encode_objects sync");
  release_slot(ctx, slot);
  return rc ? rc : rc2;
}

int nxec_decode_object(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                       const unsigned char *d_chunks, int64_t length, int64_t max_chunk_size, unsigned char *d_object,
                       unsigned char *d_tail, void *stream) {
  return nxec_decode_object_ex(ctx, n, k, failed, nfailed, d_chunks, max_chunk_size, int64_t(n) * max_chunk_size,
                               length, max_chunk_size, d_object, d_tail, stream);
}

int nxec_decode_object_ex(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                          const unsigned char *d_chunks, int64_t chunk_stride, int64_t stripe_stride, int64_t length,
                          int64_t max_chunk_size, unsigned char *d_object, unsigned char *d_tail, void *stream) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  int64_t ns = 0, nf = 0, cs_last = 0;
  int rc = nxec_object_layout(n, k, length, max_chunk_size, &ns, &nf, &cs_last);
  if (rc) return rc;
  if (ns == 0) return NXEC_OK;
  const int64_t M = max_chunk_size;
  const bool tail = ns > nf;
  if (!d_chunks || !d_object || (tail && !d_tail)) return set_error(NXEC_ERR_INVALID, "nxec_decode_object: null buffer");
  if (chunk_stride < M || stripe_stride < int64_t(n) * chunk_stride)
    return set_error(NXEC_ERR_INVALID, "nxec_decode_object: strides smaller than the chunks");
  hipStream_t st = pick_stream(ctx, stream);
  // full stripes straight into the object: data chunk j of stripe s at s*k*M + j*M
  if (nf > 0) {
    rc = nxec_rs_decode_stripes(ctx, n, k, failed, nfailed, d_chunks, chunk_stride, stripe_stride, d_object, M, k * M,
                                M, nf, st);
    if (rc) return rc;
  }
  if (!tail) return NXEC_OK;
  // last stripe: chunks of cs_last bytes in the same slots; decode to scratch, keep the unpadded bytes
  rc = nxec_rs_decode_stripes(ctx, n, k, failed, nfailed, d_chunks + nf * stripe_stride, chunk_stride, stripe_stride,
                              d_tail, cs_last, k * cs_last, cs_last, 1, st);
  if (rc) return rc;
  const int64_t rem = length - nf * k * M;
  return hip_check(hipMemcpyAsync(d_object + nf * k * M, d_tail, rem, hipMemcpyDeviceToDevice, st), "tail copy");
}

int nxec_decode_object_verify(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                              const unsigned char *d_chunks, int64_t length, int64_t max_chunk_size,
                              const unsigned char *d_md5, unsigned char *d_object, unsigned char *d_tail,
                              unsigned char *d_ok, unsigned long long *d_nbad, void *stream) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  int64_t ns = 0, nf = 0, cs_last = 0;
  int rc = nxec_object_layout(n, k, length, max_chunk_size, &ns, &nf, &cs_last);
  if (rc) return rc;
  if (ns == 0) return NXEC_OK;
  const int64_t M = max_chunk_size;
  const bool tail = ns > nf;
  if (!d_chunks || !d_object || !d_md5 || !d_ok || (tail && !d_tail))
    return set_error(NXEC_ERR_INVALID, "nxec_decode_object_verify: null buffer");
  std::vector<int32_t> inputs(n);
  int ni = 0, mi = 0;
  if ((rc = nxec_rs_plan(n, k, failed, nfailed, 0, inputs.data(), &ni, &mi, nullptr))) return rc;  // rs.cc:252-265
  if ((rc = ensure_device(ctx->device))) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  std::vector<int32_t> targets;
  for (int i = 0; i < nfailed; i++)
    if (failed[i] < k) targets.push_back(failed[i]);
  const int e = static_cast<int>(targets.size());
  // verify the k inputs of `nst` stripes of `len`-byte chunks (MD5 launches, 4 chunks each)
  auto verify = [&](const unsigned char *chunks, int64_t len, int64_t nst, int64_t s0) -> int {
    for (int j0 = 0; j0 < k; j0 += kMaxMd5Regions) {
      Md5Region reg[kMaxMd5Regions];
      int nr = 0;
      for (int j = j0; j < k && nr < kMaxMd5Regions; j++, nr++) {
        const int id = inputs[j];
        reg[nr] = Md5Region{chunks + id * M, M, n * M, len, nst,
                            const_cast<unsigned char *>(d_md5) + (s0 * n + id) * 16, int64_t(n) * 16, 1,
                            d_ok + s0 * n + id, n};
      }
      if (int r = launch_md5(reg, nr, st, d_nbad)) return r;
    }
    return NXEC_OK;
  };
  if (nf > 0) {
    MulMd5Args a{};
    bool fused = e <= kMaxRowsPerPass && k <= kEncMd5MaxK && int64_t(n - 1) * M < (int64_t(1) << 32) &&
                 int64_t(k) * M < (int64_t(1) << 32);
    if (fused) {
      a.any_copy = 0;
      for (int j = 0; j < k; j++) {
        a.src_off[j] = static_cast<uint32_t>(inputs[j] * M);
        a.copy_off[j] = inputs[j] < k ? static_cast<uint32_t>(inputs[j] * M) : kNoCopy;
        a.any_copy |= inputs[j] < k;
        a.digest_slot[j] = static_cast<uint8_t>(inputs[j]);
      }
      for (int r = 0; r < e; r++) a.dst_off[r] = static_cast<uint32_t>(targets[r] * M);
      fused = mul_md5_eligible(k, e, M, d_chunks, n * M, a.src_off, d_object, k * M, a.dst_off, a.copy_off);
    }
    if (fused) {
      if (e > 0) {
        std::vector<uint8_t> m(static_cast<size_t>(e) * k);
        if ((rc = nxec_rs_decode_matrix(n, k, inputs.data(), targets.data(), e, m.data()))) return rc;  // rs.cc:196,228
        std::memcpy(a.coef, m.data(), m.size());
      }
      a.src = d_chunks;
      a.src_stripe_stride = n * M;
      a.dst = d_object;
      a.dst_stripe_stride = k * M;
      a.digests = const_cast<unsigned char *>(d_md5);
      a.digest_stripe_stride = int64_t(n) * 16;
      a.ok = d_ok;
      a.ok_stripe_stride = n;
      a.nbad = d_nbad;
      a.len = M;
      a.nstripes = nf;
      a.k = k;
      a.p = e;
      a.hash_src = 1;
      a.hash_dst = 0;
      if ((rc = launch_mul_md5(a, ctx->num_cus, st))) return rc;
    } else {
      if ((rc = verify(d_chunks, M, nf, 0))) return rc;
      if ((rc = nxec_rs_decode_stripes(ctx, n, k, failed, nfailed, d_chunks, M, n * M, d_object, M, k * M, M, nf, st)))
        return rc;
    }
  }
  if (!tail) return NXEC_OK;
  // last stripe (chunks of cs_last bytes in the same slots): verify, decode to scratch, keep the unpadded bytes
  if ((rc = verify(d_chunks + nf * n * M, cs_last, 1, nf))) return rc;
  if ((rc = nxec_rs_decode_stripes(ctx, n, k, failed, nfailed, d_chunks + nf * n * M, M, n * M, d_tail, cs_last,
                                   k * cs_last, cs_last, 1, st)))
    return rc;
  const int64_t rem = length - nf * k * M;
  return hip_check(hipMemcpyAsync(d_object + nf * k * M, d_tail, rem, hipMemcpyDeviceToDevice, st), "tail copy");
}

namespace {

// One batch of same-shape agent requests in a staging slot: [B][ninputs][stride]
// inputs, [B][noutputs][stride] outputs, [B][noutputs][16] digests.
struct AgentBatch {
  Slot *slot = nullptr;
  std::vector<int> reqs;  // request indices staged in this slot (outputs pending)
  size_t out_off = 0, md5_off = 0;
  int hsrc = 0;  // digests per request: [inputs (hsrc) ][outputs], (hsrc + noutputs) x 16 bytes
  int64_t stride = 0;
  size_t d2h_bytes = 0;  // outputs (+ digests) still to be queued device -> host
  // fused form (k_gather_md5 over pinned memory): the kernel wrote outputs
  // straight into mapped caller buffers; out_pos[i*no + o] >= 0 is the slot
  // offset of an output that went to the slot instead (pageable caller buffer)
  bool fused = false;
  std::vector<int64_t> out_pos;
};

// Queues a batch's D2H.  Held back until the next batch's H2D is queued: a
// D2H queued first (it waits for the batch's MD5, ~10 ms) blocked the next
// batch's H2D on the other stream behind it, so batches ran one after the
// other (tools/agent_probe.py timeline, profiles/r01_agent_timeline.txt).
// The outputs go back by a copy kernel writing the slot's device-mapped pinned
// staging over PCIe: SDMA copies run one after another on this box, so an
// SDMA D2H queued between two batches' H2Ds stalled the next H2D by its whole
// duration (rocprofv3 memory-copy trace, profiles/r02_agent_timeline.txt);
// the kernel's stores use the link's other direction while the H2Ds stream.
int agent_d2h(nxec_ctx_t *ctx, AgentBatch &b) {
  if (!b.d2h_bytes) return NXEC_OK;
  const size_t nb = b.d2h_bytes;
  b.d2h_bytes = 0;
  uint8_t *hv = static_cast<uint8_t *>(host_device_view(b.slot->h));
  if (hv && nb % 16 == 0 && b.out_off % 16 == 0)
    return launch_copy16(hv + b.out_off, b.slot->d + b.out_off, nb, ctx->num_cus, b.slot->stream);
  return hip_check(hipMemcpyAsync(b.slot->h + b.out_off, b.slot->d + b.out_off, nb, hipMemcpyDeviceToHost,
                                  b.slot->stream),
                   "agent D2H");
}

int agent_finish(nxec_ctx_t *ctx, const nxec_agent_req *reqs, int64_t cs, AgentBatch &b) {
  if (b.reqs.empty()) return NXEC_OK;
  if (int rc = agent_d2h(ctx, b)) return rc;
  NXEC_HIP(hipStreamSynchronize(b.slot->stream));
  const nxec_agent_req &r0 = reqs[b.reqs[0]];
  const int no = r0.noutputs, nh = b.hsrc + no;
  HostPool::get().parallel_for(static_cast<int>(b.reqs.size()) * no, [&](int item) {  // scatter the outputs
    const size_t i = static_cast<size_t>(item / no);
    const int o = item % no;
    const nxec_agent_req &r = reqs[b.reqs[i]];
    if (!b.fused)
      std::memcpy(r.outputs[o], b.slot->h + b.out_off + (i * no + o) * b.stride, cs);
    else if (b.out_pos[static_cast<size_t>(item)] >= 0)
      std::memcpy(r.outputs[o], b.slot->h + b.out_pos[static_cast<size_t>(item)], cs);
    const uint8_t *dg = b.slot->h + b.md5_off + i * size_t(nh) * 16;
    if (o == 0 && r.md5) std::memcpy(r.md5, dg + size_t(b.hsrc) * 16, size_t(no) * 16);
    if (o == 0 && r.md5_inputs && b.hsrc) std::memcpy(r.md5_inputs, dg, size_t(b.hsrc) * 16);
  });
  b.reqs.clear();
  return NXEC_OK;
}

}  // namespace

}  // extern "C"

static bool agent_trace() {
  static const bool t = std::getenv("NXEC_AGENT_TRACE") != nullptr;
  return t;
}

// testing hook: NXEC_TEST_AGENT_THROW=1 makes every round's leader throw
// before it runs (the round must still complete with an error, no waiter hangs)
static bool agent_test_throw() {
  static const bool t = [] {
    const char *e = std::getenv("NXEC_TEST_AGENT_THROW");
    return e && e[0] == '1';
  }();
  return t;
}

// three staging slots in rotation: batch b gathers into its slot while
// batch b-1's H2D runs and batch b-2's MD5 chains finish, so the link never
// waits for a gather (two slots left ~6 ms gaps per batch)
constexpr int kAgentSlots = 3;

// b's slot holds at least `bytes` (a larger one is taken when it does not)
static int agent_slot(nxec_ctx_t *ctx, AgentBatch &b, size_t bytes) {
  bytes = std::max<size_t>(bytes, 4096);
  if (b.slot && b.slot->cap < bytes) {
    release_slot(ctx, b.slot);
    b.slot = nullptr;
  }
  return b.slot ? NXEC_OK : acquire_slot(ctx, bytes, &b.slot);
}

// One matrix group through the fused kernel.  Every input and output is
// classified once: a pinned / registered caller buffer (an arena Chunk) is
// handed to the kernel as is, a pageable or misaligned one is gathered into
// (input) or collected from (output) the slot.  Batches are bounded by the
// staging they need, not by the bytes they code -- each batch pays one whole
// MD5 chain (~9 ms per 1 MiB chunk whatever its size), so requests in mapped
// buffers all go in one launch (64 MiB staging batches: 23 -> 11 GiB/s at one
// caller).  Slots rotate with the two-kernel form's.
// md5 = false (a group that wants no digests: ENC_CHUNK_REQ, whose
// getEncodedChunks computes none, container_manager.cc:221-258): when every
// input is mapped the same tables feed the gather form of the multiply
// kernel -- zero copy, no MD5 chain (64 x 4->1 arena requests: 1 caller 37 ->
// 50 GiB/s); with inputs to stage, *taken = false and the caller runs the
// H2D -> multiply -> D2H form, whose copy engines beat kernel reads of the
// staging slot when no MD5 chain hides them (pageable: 34 vs 29 GiB/s).
// hsrc: the inputs are hashed too (RSCode::encode through nxec_encode_host_md5).
static int agent_fused_group(nxec_ctx_t *ctx, const nxec_agent_req *reqs, const std::vector<int> &ids,
                             int64_t chunk_size, int64_t stride, int64_t batch_bytes, AgentBatch (&slots)[kAgentSlots],
                             int &cur, bool md5, bool hsrc, bool *taken) {
  *taken = true;
  const nxec_agent_req &r0 = reqs[ids[0]];
  const int ni = r0.ninputs, no = r0.noutputs, nh = (hsrc ? ni : 0) + no;
  const size_t nid = ids.size(), cs = size_t(chunk_size);
  std::vector<uintptr_t> in_dv(nid * ni), out_dv(nid * no);  // 0: not mapped
  const auto tc0 = std::chrono::steady_clock::now();
  HostPool::get().parallel_for(static_cast<int>(nid * (ni + no)), [&](int item) {
    const size_t q = static_cast<size_t>(item);
    if (q < nid * ni) {
      const unsigned char *p = reqs[ids[q / ni]].inputs[q % ni];
      in_dv[q] = aligned16(p) ? reinterpret_cast<uintptr_t>(host_device_view_range(p, cs)) : 0;
    } else {
      const size_t o = q - nid * ni;
      unsigned char *p = reqs[ids[o / no]].outputs[o % no];
      out_dv[o] = aligned16(p) ? reinterpret_cast<uintptr_t>(host_device_view_range(p, cs)) : 0;
    }
  });
  if (agent_trace())
    std::fprintf(stderr, "agent fused group of %zu: classify %zu buffers %.3f ms\n", nid, nid * (ni + no),
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc0).count());
  if (!md5 && std::find(in_dv.begin(), in_dv.end(), uintptr_t(0)) != in_dv.end()) {
    *taken = false;
    return NXEC_OK;
  }
  int rc = NXEC_OK;
  for (size_t first = 0; first < nid && rc == NXEC_OK;) {
    // [first, last): requests whose staging fits batch_bytes (at least one)
    size_t last = first;
    int64_t staged = 0;
    while (last < nid) {
      int64_t n_st = 0;
      for (int j = 0; j < ni; j++) n_st += in_dv[last * ni + j] == 0;
      for (int o = 0; o < no; o++) n_st += out_dv[last * no + o] == 0;
      const int64_t need = n_st * stride + (md5 ? int64_t(nh) * 16 : 0) + (int64_t(ni) + no) * 8;
      if (last > first && staged + need > batch_bytes) break;
      staged += need;
      last++;
    }
    const size_t nb = last - first;
    AgentBatch &b = slots[cur], &other = slots[(cur + kAgentSlots - 1) % kAgentSlots];
    cur = (cur + 1) % kAgentSlots;
    const auto tr0 = std::chrono::steady_clock::now();
    if ((rc = agent_finish(ctx, reqs, chunk_size, b))) break;  // this slot's previous batch
    const auto tr1 = std::chrono::steady_clock::now();
    if ((rc = agent_slot(ctx, b, size_t(staged)))) break;
    uint8_t *hv = static_cast<uint8_t *>(host_device_view(b.slot->h));
    if (!hv) {
      rc = set_error(NXEC_ERR_HIP, "agent staging slot is not device-mapped");
      break;
    }
    // slot: [staged chunks][digests nb x no x 16][source table nb x ni][output table nb x no]
    std::vector<int64_t> in_pos(nb * ni, -1);
    b.out_pos.assign(nb * no, -1);
    int64_t pos = 0;
    for (size_t q = 0; q < nb * ni; q++)
      if (!in_dv[first * ni + q]) in_pos[q] = pos, pos += stride;
    for (size_t q = 0; q < nb * no; q++)
      if (!out_dv[first * no + q]) b.out_pos[q] = pos, pos += stride;
    b.fused = true;
    b.stride = stride;
    b.hsrc = hsrc ? ni : 0;
    b.md5_off = size_t(pos);
    const size_t tab_off = b.md5_off + (md5 ? nb * size_t(nh) * 16 : 0);
    uint64_t *src_tab = reinterpret_cast<uint64_t *>(b.slot->h + tab_off);
    uint64_t *dst_tab = src_tab + nb * ni;
    HostPool::get().parallel_for(static_cast<int>(nb * (ni + no)), [&](int item) {
      const size_t q = static_cast<size_t>(item);
      if (q < nb * ni) {
        if (in_pos[q] < 0) {
          src_tab[q] = in_dv[first * ni + q];
        } else {
          stage_copy(b.slot->h + in_pos[q], reqs[ids[first + q / ni]].inputs[q % ni], cs);
          src_tab[q] = reinterpret_cast<uintptr_t>(hv + in_pos[q]);
        }
      } else {
        const size_t o = q - nb * ni;
        dst_tab[o] = b.out_pos[o] < 0 ? out_dv[first * no + o] : reinterpret_cast<uintptr_t>(hv + b.out_pos[o]);
      }
    });
    for (size_t i = first; i < last; i++) b.reqs.push_back(ids[i]);
    if (agent_trace()) {
      const auto tr2 = std::chrono::steady_clock::now();
      std::fprintf(stderr, "agent fused batch of %zu (%lld staged bytes): finish-previous %.2f ms, tables + gather %.2f ms\n",
                   nb, static_cast<long long>(pos), std::chrono::duration<double, std::milli>(tr1 - tr0).count(),
                   std::chrono::duration<double, std::milli>(tr2 - tr1).count());
    }
    if (!md5) {  // CodingUtils::encode of the batch over the pointer tables
      rc = stripes_mul_impl(ctx, no, ni, r0.matrix, nullptr,
                            reinterpret_cast<const unsigned char *const *>(hv + tab_off), nullptr, 0, 0, nullptr,
                            reinterpret_cast<unsigned char *const *>(hv + tab_off + nb * ni * 8), nullptr, 0, 0,
                            nullptr, chunk_size, int64_t(nb), b.slot->stream);
      if (rc) break;
      b.d2h_bytes = 0;
      rc = agent_d2h(ctx, other);
      first = last;
      continue;
    }
    GatherMd5Args ga;
    std::memset(&ga, 0, sizeof(ga));
    ga.src_ptrs = reinterpret_cast<const uint8_t *const *>(hv + tab_off);
    ga.dst_ptrs = reinterpret_cast<uint8_t *const *>(hv + tab_off + nb * ni * 8);
    ga.digests = hv + b.md5_off;
    ga.scratch = b.slot->d;
    ga.len = chunk_size;
    ga.nstripes = int64_t(nb);
    ga.k = ni;
    ga.p = no;
    ga.hash_src = hsrc ? 1 : 0;
    std::memcpy(ga.coef, r0.matrix, size_t(no) * ni);
    if ((rc = launch_gather_md5(ga, ctx->num_cus, b.slot->stream))) break;
    b.d2h_bytes = 0;
    rc = agent_d2h(ctx, other);  // a two-kernel previous batch's D2H, if any
    first = last;
  }
  return rc;
}

// One round of agent requests (validated): grouped by matrix, staged through
// two double-buffered pinned slots of up to batch_bytes each.
static int agent_encode_impl(nxec_ctx_t *ctx, const nxec_agent_req *reqs, int nreqs, int64_t chunk_size,
                             int64_t batch_bytes) {
  int rc = ensure_device(ctx->device);
  if (rc) return rc;
  // group requests by (ninputs, noutputs, matrix): one kernel pass per batch of a group
  std::map<std::string, std::vector<int>> groups;
  for (int i = 0; i < nreqs; i++) {
    const nxec_agent_req &r = reqs[i];
    std::string key(1, r.md5_inputs ? 'S' : '-');  // inputs hashed: its own kernel form
    key.append(reinterpret_cast<const char *>(&r.ninputs), sizeof(int));
    key.append(reinterpret_cast<const char *>(&r.noutputs), sizeof(int));
    key.append(reinterpret_cast<const char *>(r.matrix), size_t(r.ninputs) * r.noutputs);
    groups[key].push_back(i);
  }
  const int64_t stride = (chunk_size + 15) / 16 * 16;
  if (batch_bytes <= 0) batch_bytes = int64_t(256) << 20;
  if (const char *e = std::getenv("NXEC_AGENT_BATCH_MB")) batch_bytes = std::max<int64_t>(1, std::atoll(e)) << 20;  // tuning
  // fused form (any chunk size): one k_gather_md5 launch per batch codes and hashes the
  // requests straight from and into pinned host memory (mapped caller
  // buffers, e.g. arena Chunks, are used in place; pageable ones go through
  // the slot).  NXEC_AGENT_FUSED=0: H2D -> multiply -> MD5 -> D2H (A/B).
  static const bool fused_env = [] {
    const char *e = std::getenv("NXEC_AGENT_FUSED");
    return !(e && e[0] == '0');
  }();
  static const bool host_direct = [] {
    const char *e = std::getenv("NXEC_HOST_DIRECT");
    return !(e && e[0] == '0');
  }();
  AgentBatch slots[kAgentSlots];
  int cur = 0;
  rc = NXEC_OK;
  for (auto &kv : groups) {
    const std::vector<int> &ids = kv.second;
    const nxec_agent_req &r0 = reqs[ids[0]];
    const int ni = r0.ninputs, no = r0.noutputs;
    const bool hsrc = r0.md5_inputs != nullptr;  // the whole group (grouping key)
    bool group_md5 = hsrc;
    for (int id : ids) group_md5 |= reqs[id].md5 != nullptr;
    const int nh = (hsrc ? ni : 0) + no;
    if (fused_env && host_direct && ni <= kGatherMd5MaxK && no <= kMaxRowsPerPass) {
      bool taken = false;
      if ((rc = agent_fused_group(ctx, reqs, ids, chunk_size, stride, batch_bytes, slots, cur, group_md5, hsrc,
                                  &taken)))
        break;
      if (taken) continue;
    }
    const int64_t per = (int64_t(ni) + no) * stride + int64_t(nh) * 16;
    const int64_t B = std::max<int64_t>(1, std::min<int64_t>(int64_t(ids.size()), batch_bytes / per));
    const size_t slot_bytes = size_t(B * per);
    for (size_t first = 0; first < ids.size() && rc == NXEC_OK; first += B) {
      const int64_t nb = std::min<int64_t>(B, int64_t(ids.size() - first));
      AgentBatch &b = slots[cur], &other = slots[(cur + kAgentSlots - 1) % kAgentSlots];
      cur = (cur + 1) % kAgentSlots;
      const auto tr0 = std::chrono::steady_clock::now();
      if ((rc = agent_finish(ctx, reqs, chunk_size, b))) break;  // this slot's previous batch
      const auto tr1 = std::chrono::steady_clock::now();
      if ((rc = agent_slot(ctx, b, slot_bytes))) break;
      const size_t in_bytes = size_t(nb) * ni * stride;
      b.stride = stride;
      b.out_off = in_bytes;
      b.md5_off = in_bytes + size_t(nb) * no * stride;
      b.fused = false;
      b.hsrc = hsrc ? ni : 0;
      HostPool::get().parallel_for(static_cast<int>(nb) * ni, [&](int item) {  // gather into pinned staging
        const int64_t i = item / ni;
        const int j = item % ni;
        stage_copy(b.slot->h + (i * ni + j) * stride, reqs[ids[first + i]].inputs[j], chunk_size);
      });
      for (int64_t i = 0; i < nb; i++) b.reqs.push_back(ids[first + i]);
      if (agent_trace()) {
        const auto tr2 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "agent batch of %lld: finish-previous %.2f ms, gather %.2f ms (%.1f GB/s)\n",
                     static_cast<long long>(nb), std::chrono::duration<double, std::milli>(tr1 - tr0).count(),
                     std::chrono::duration<double, std::milli>(tr2 - tr1).count(),
                     double(nb) * ni * chunk_size / std::chrono::duration<double>(tr2 - tr1).count() / 1e9);
      }
      hipStream_t st = b.slot->stream;
      uint8_t *d_in = b.slot->d, *d_out = b.slot->d + b.out_off, *d_md5 = b.slot->d + b.md5_off;
      bool any_md5 = hsrc;
      for (int64_t i = 0; i < nb; i++) any_md5 |= reqs[ids[first + i]].md5 != nullptr;
      if ((rc = hip_check(hipMemcpyAsync(d_in, b.slot->h, in_bytes, hipMemcpyHostToDevice, st), "agent H2D"))) break;
      // CodingUtils::encode (container_manager.cc:251, agent.cc:339) for the whole batch
      rc = nxec_stripes_mul(ctx, no, ni, r0.matrix, d_in, nullptr, stride, ni * stride, d_out, nullptr, stride,
                            no * stride, nullptr, chunk_size, nb, st);
      if (rc) break;
      if (any_md5) {  // Chunk::computeMD5 of the outputs (agent.cc:342), and of the inputs for hsrc
        const int64_t ds = int64_t(nh) * 16;
        const Md5Region reg[2] = {{d_out, stride, no * stride, chunk_size, nb, d_md5 + (hsrc ? ni * 16 : 0), ds, no},
                                  {d_in, stride, ni * stride, chunk_size, nb, d_md5, ds, ni}};
        if ((rc = launch_md5(reg, hsrc ? 2 : 1, st))) break;
      }
      b.d2h_bytes = size_t(nb) * (no * stride + (any_md5 ? nh * 16 : 0));
      if ((rc = agent_d2h(ctx, other))) break;  // the previous batch's D2H, behind this batch's H2D
    }
    if (rc) break;
  }
  if (!rc) rc = agent_d2h(ctx, slots[(cur + kAgentSlots - 1) % kAgentSlots]);  // the last batch's D2H
  for (int i = 0; i < kAgentSlots; i++) {  // oldest batch first
    AgentBatch &b = slots[(cur + i) % kAgentSlots];
    if (b.slot) {
      int rc2 = rc ? NXEC_OK : agent_finish(ctx, reqs, chunk_size, b);
      if (rc) (void)hipStreamSynchronize(b.slot->stream);
      if (!rc) rc = rc2;
      release_slot(ctx, b.slot);
    }
  }
  return rc;
}

// Requests from concurrent callers are aggregated: a caller queues its job;
// whichever waiting caller finds no round in progress leads the next one,
// taking every queued job of the same chunk size, and runs them as ONE set of
// batches (one MD5 launch per batch covers all callers' outputs, so the ~10 ms
// MD5 chain of a 1 MiB chunk is paid once per round, not once per call).
// A round stages at most the smallest batch_bytes its callers asked for;
// when none asked, 512 MiB per slot for a merged round (4 pageable callers:
// 20 GiB/s at 1 GiB, 26 at 512 MiB) and 256 MiB for a lone call.
// NXEC_AGENT_AGGREGATE=0 runs every call on its own.
extern "C" int nxec_agent_encode_batch(nxec_ctx_t *ctx, const nxec_agent_req *reqs, int nreqs, int64_t chunk_size,
                                       int64_t batch_bytes) {
  if (!ctx || nreqs < 0 || chunk_size < 0 || (nreqs > 0 && !reqs))
    return set_error(NXEC_ERR_INVALID, "nxec_agent_encode_batch: invalid arguments");
  for (int i = 0; i < nreqs; i++) {
    const nxec_agent_req &r = reqs[i];
    if (r.ninputs < 1 || r.ninputs > NXEC_MAX_K || r.noutputs < 1 || r.noutputs > NXEC_MAX_N || !r.matrix ||
        !r.inputs || !r.outputs)
      return set_error(NXEC_ERR_INVALID, "nxec_agent_encode_batch: request %d malformed", i);
  }
  if (nreqs == 0 || chunk_size == 0) return NXEC_OK;
  static const bool aggregate = [] {
    const char *e = std::getenv("NXEC_AGENT_AGGREGATE");
    return !(e && e[0] == '0');
  }();
  if (!aggregate) return agent_encode_impl(ctx, reqs, nreqs, chunk_size, batch_bytes);
  AgentJob job;
  job.reqs = reqs;
  job.nreqs = nreqs;
  job.chunk_size = chunk_size;
  job.batch_bytes = batch_bytes;
  std::unique_lock<std::mutex> lk(ctx->agent_mu);
  ctx->agent_pending.push_back(&job);
  while (!job.done) {
    // wait while a round is being issued, or when this job is already in a
    // round that is still finishing (nothing left to lead)
    if (ctx->agent_leader || ctx->agent_pending.empty()) {
      ctx->agent_cv.wait(lk);
      continue;
    }
    ctx->agent_leader = true;
    std::vector<AgentJob *> round;
    const int64_t cs0 = ctx->agent_pending.front()->chunk_size;
    for (auto it = ctx->agent_pending.begin(); it != ctx->agent_pending.end();) {
      if ((*it)->chunk_size == cs0) {
        round.push_back(*it);
        it = ctx->agent_pending.erase(it);
      } else {
        ++it;
      }
    }
    lk.unlock();
    // (overlapping rounds -- leadership handed on once a round's batches are
    // queued -- measured worse: many small rounds, each paying a whole MD5
    // chain, and two rounds' gathers sharing the host pool; 16 callers 5-11
    // vs 27-29 GiB/s, profiles/r02_agent_nt_staging.log)
    int rc = NXEC_OK;
    std::string err;
    try {  // whatever happens, the round's jobs finish and leadership is released
      std::vector<nxec_agent_req> merged;
      int64_t bb = 0;  // the smallest staging bound any caller of the round asked for
      for (AgentJob *j : round) {
        merged.insert(merged.end(), j->reqs, j->reqs + j->nreqs);
        if (j->batch_bytes > 0) bb = bb > 0 ? std::min(bb, j->batch_bytes) : j->batch_bytes;
      }
      if (bb <= 0 && round.size() > 1) bb = int64_t(512) << 20;
      if (agent_test_throw()) throw std::bad_alloc();
      rc = agent_encode_impl(ctx, merged.data(), static_cast<int>(merged.size()), cs0, bb);
      if (rc) err = g_last_error;
    } catch (const std::exception &e) {
      rc = set_error(NXEC_ERR_NOMEM, "nxec_agent_encode_batch: %s", e.what());
      err = g_last_error;
    }
    lk.lock();
    for (AgentJob *j : round) {
      j->rc = rc;
      j->error = err;
      j->done = true;
    }
    ctx->agent_leader = false;
    ctx->agent_cv.notify_all();
  }
  if (job.rc != NXEC_OK) g_last_error = job.error;
  return job.rc;
}

extern "C" {

int nxec_rs_encode_host_batch(nxec_ctx_t *ctx, int n, int k, const unsigned char *h_data, unsigned char *h_parity,
                              int64_t len, int64_t nstripes, int64_t batch_stripes) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  if (!valid_nk(n, k) || len < 0 || nstripes < 0) return set_error(NXEC_ERR_INVALID, "invalid arguments");
  if (n == k || len == 0 || nstripes == 0) return NXEC_OK;
  if (!h_data || !h_parity) return set_error(NXEC_ERR_INVALID, "null host buffer");
  int rc = ensure_device(ctx->device);
  if (rc) return rc;
  const int p = n - k;
  // Pinned / registered buffers: zero copy.  The coding kernel reads the data
  // and writes the parity over PCIe itself; its ~1 KiB requests from every CU
  // keep more of the link busy than the copy engines do (RS(10,4) 1 MiB,
  // 512 stripes: 71.6 vs 48.7 GiB/s of (k+p)*cs, tools/zero_copy_probe.py).
  {
    const unsigned char *dd =
        static_cast<const unsigned char *>(host_device_view_range(h_data, static_cast<size_t>(nstripes * k * len)));
    unsigned char *dp = static_cast<unsigned char *>(host_device_view_range(h_parity, static_cast<size_t>(nstripes * p * len)));
    if (dd && dp) {
      std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
      nxec_gf_gen_rs_matrix(enc.data(), n, k);
      hipStream_t st = pick_stream(ctx, nullptr);
      rc = nxec_stripes_mul(ctx, p, k, enc.data() + static_cast<size_t>(k) * k, dd, nullptr, len, k * len, dp, nullptr,
                            len, p * len, nullptr, len, nstripes, st);
      if (rc) return rc;
      return hip_check(hipStreamSynchronize(st), "encode_host_batch (direct) sync");
    }
  }
  if (batch_stripes <= 0) batch_stripes = std::max<int64_t>(1, (int64_t(256) << 20) / (len * n));
  batch_stripes = std::min(batch_stripes, nstripes);
  const int64_t nbatches = (nstripes + batch_stripes - 1) / batch_stripes;
  batch_stripes = (nstripes + nbatches - 1) / nbatches;  // equal batches
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
  nxec_gf_gen_rs_matrix(enc.data(), n, k);
  const size_t dbytes = static_cast<size_t>(batch_stripes) * k * len, pbytes = static_cast<size_t>(batch_stripes) * p * len;
  std::unique_lock<std::mutex> lk;
  ObjStage priv, *pstg = nullptr;
  if ((rc = batch_stage(ctx, dbytes + pbytes, lk, priv, &pstg))) return rc;
  ObjStage &stg = *pstg;
  int prev = -1;
  for (int64_t b = 0; b < nbatches && rc == NXEC_OK; b++) {
    const int slot = static_cast<int>(b % kObjSlots);
    const int64_t s0 = b * batch_stripes, ns = std::min(batch_stripes, nstripes - s0);
    hipStream_t st = stg.streams[slot];
    uint8_t *dbuf = stg.d + slot * stg.cap, *pbuf = dbuf + dbytes;
    // H2D copies one batch after another, so the first batch's kernel starts early
    if (prev >= 0) rc = hip_check(hipStreamWaitEvent(st, stg.h2d_done[prev], 0), "H2D order");
    if (!rc)
      rc = hip_check(hipMemcpyAsync(dbuf, h_data + s0 * k * len, static_cast<size_t>(ns) * k * len,
                                    hipMemcpyHostToDevice, st),
                     "H2D");
    if (!rc) rc = hip_check(hipEventRecord(stg.h2d_done[slot], st), "H2D event");
    prev = slot;
    if (!rc)
      rc = nxec_stripes_mul(ctx, p, k, enc.data() + static_cast<size_t>(k) * k, dbuf, nullptr, len, k * len, pbuf,
                            nullptr, len, p * len, nullptr, len, ns, st);
    if (!rc)
      rc = hip_check(hipMemcpyAsync(h_parity + s0 * p * len, pbuf, static_cast<size_t>(ns) * p * len,
                                    hipMemcpyDeviceToHost, st),
                     "D2H");
  }
  for (int i = 0; i < kObjSlots; i++) {
    hipError_t e = hipStreamSynchronize(stg.streams[i]);
    if (!rc) rc = hip_check(e, "encode_host_batch sync");
  }
  if (!lk.owns_lock()) priv.release();
  return rc;
}

namespace {

// Chunk frames <-> device batch: item i of the plan is segment (i % segs) of
// chunk (i / segs); a piece is up to `per` items staged back to back in one
// pinned slot.  Chunks longer than a piece are cut into segments.
constexpr int64_t kFramePiece = int64_t(16) << 20;
// Pinned frames at least this long are DMA'd one copy per frame; shorter ones
// are staged too: per-copy overhead holds 1 MiB pinned frames to 34 GiB/s
// against 50 staged (tools/frames_rate.py).
constexpr int64_t kFrameDirect = int64_t(8) << 20;

struct FramePlan {
  int64_t len, seg, segs, per, items, npieces;
  FramePlan(int64_t nchunks, int64_t l) : len(l) {
    seg = std::min(len, kFramePiece);
    segs = (len + seg - 1) / seg;
    per = std::max<int64_t>(1, kFramePiece / seg);
    items = nchunks * segs;
    npieces = (items + per - 1) / per;
  }
  int64_t chunk(int64_t i) const { return i / segs; }
  int64_t off(int64_t i) const { return (i % segs) * seg; }
  int64_t bytes(int64_t i) const { return std::min(seg, len - off(i)); }
};

// host memcpy of items [first, first+count) between frames and staging, in
// jobs of at most 1 MiB spread over the host pool
void frame_copies(const FramePlan &fp, int64_t first, int64_t count, uint8_t *staging,
                  const std::function<void(int64_t item, int64_t off, int64_t n, uint8_t *stage)> &copy) {
  const int64_t job = int64_t(1) << 20;
  const int64_t jobs_per_item = (fp.seg + job - 1) / job;
  host_parallel_for(static_cast<int>(count * jobs_per_item), [&](int t) {
    const int64_t i = t / jobs_per_item, o = (t % jobs_per_item) * job;
    const int64_t b = fp.bytes(first + i);
    if (o < b) copy(first + i, o, std::min(job, b - o), staging + i * fp.seg + o);
  });
}

// whether every frame is pinned / registered host memory over its whole
// length (DMA reads it directly)
bool frames_pinned(const void *const *frames, int64_t n, int64_t len) {
  for (int64_t i = 0; i < n; i++)
    if (!host_device_view_range(frames[i], static_cast<size_t>(len))) return false;
  return true;
}

int frames_check(nxec_ctx_t *ctx, const void *frames, int64_t nchunks, int64_t len, const void *d, int64_t stride,
                 const char *what) {
  if (!ctx || nchunks < 0 || len < 0 || (nchunks > 0 && len > 0 && (!frames || !d || stride < len)))
    return set_error(NXEC_ERR_INVALID, "%s: invalid arguments", what);
  return NXEC_OK;
}

}  // namespace

int nxec_gather_chunks(nxec_ctx_t *ctx, const unsigned char *const *h_chunks, int64_t nchunks, int64_t len,
                       unsigned char *d_dst, int64_t dst_stride, void *stream) {
  int rc = frames_check(ctx, h_chunks, nchunks, len, d_dst, dst_stride, "nxec_gather_chunks");
  if (rc || nchunks == 0 || len == 0) return rc;
  if ((rc = ensure_device(ctx->device))) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  if (len >= kFrameDirect && frames_pinned(reinterpret_cast<const void *const *>(h_chunks), nchunks, len)) {
    for (int64_t i = 0; i < nchunks; i++)
      NXEC_HIP(hipMemcpyAsync(d_dst + i * dst_stride, h_chunks[i], size_t(len), hipMemcpyHostToDevice, st));
    NXEC_HIP(hipStreamSynchronize(st));
    return NXEC_OK;
  }
  // pageable frames: the pool packs piece p into one pinned slot while the
  // copy engine moves piece p-1 out of the other
  const FramePlan fp(nchunks, len);
  Slot *slots[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  const size_t cap = size_t(std::min(fp.per, fp.items) * fp.seg);
  for (int s = 0; s < 2 && rc == NXEC_OK; s++) {
    if ((rc = acquire_slot(ctx, cap, &slots[s]))) break;
    rc = hip_check(hipEventCreateWithFlags(&done[s], hipEventDisableTiming), "hipEventCreate");
  }
  for (int64_t p = 0; p < fp.npieces && rc == NXEC_OK; p++) {
    const int s = static_cast<int>(p & 1);
    const int64_t first = p * fp.per, count = std::min(fp.per, fp.items - first);
    if (p >= 2 && (rc = hip_check(hipEventSynchronize(done[s]), "gather piece sync"))) break;
    frame_copies(fp, first, count, slots[s]->h, [&](int64_t item, int64_t o, int64_t nb, uint8_t *stage) {
      stage_copy(stage, h_chunks[fp.chunk(item)] + fp.off(item) + o, size_t(nb));
    });
    hipError_t e = hipSuccess;
    if (fp.segs == 1) {  // whole chunks: one 2D copy scatters the piece to its strided rows
      e = hipMemcpy2DAsync(d_dst + fp.chunk(first) * dst_stride, size_t(dst_stride), slots[s]->h, size_t(fp.seg),
                           size_t(len), size_t(count), hipMemcpyHostToDevice, st);
    } else {
      for (int64_t i = first; i < first + count && e == hipSuccess; i++)
        e = hipMemcpyAsync(d_dst + fp.chunk(i) * dst_stride + fp.off(i), slots[s]->h + (i - first) * fp.seg,
                           size_t(fp.bytes(i)), hipMemcpyHostToDevice, st);
    }
    if (e == hipSuccess) e = hipEventRecord(done[s], st);
    rc = hip_check(e, "gather H2D");
  }
  hipError_t e = hipStreamSynchronize(st);  // the slots go back to the pool only once drained
  if (rc == NXEC_OK) rc = hip_check(e, "gather sync");
  for (int s = 0; s < 2; s++) {
    if (done[s]) (void)hipEventDestroy(done[s]);
    if (slots[s]) release_slot(ctx, slots[s]);
  }
  return rc;
}

int nxec_scatter_chunks(nxec_ctx_t *ctx, const unsigned char *d_src, int64_t src_stride, int64_t nchunks, int64_t len,
                        unsigned char *const *h_chunks, void *stream) {
  int rc = frames_check(ctx, h_chunks, nchunks, len, d_src, src_stride, "nxec_scatter_chunks");
  if (rc || nchunks == 0 || len == 0) return rc;
  if ((rc = ensure_device(ctx->device))) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  if (len >= kFrameDirect && frames_pinned(reinterpret_cast<const void *const *>(h_chunks), nchunks, len)) {
    for (int64_t i = 0; i < nchunks; i++)
      NXEC_HIP(hipMemcpyAsync(h_chunks[i], d_src + i * src_stride, size_t(len), hipMemcpyDeviceToHost, st));
    NXEC_HIP(hipStreamSynchronize(st));
    return NXEC_OK;
  }
  // the copy engine fills piece p+1 into one slot while the pool unpacks piece p
  const FramePlan fp(nchunks, len);
  Slot *slots[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  const size_t cap = size_t(std::min(fp.per, fp.items) * fp.seg);
  for (int s = 0; s < 2 && rc == NXEC_OK; s++) {
    if ((rc = acquire_slot(ctx, cap, &slots[s]))) break;
    rc = hip_check(hipEventCreateWithFlags(&done[s], hipEventDisableTiming), "hipEventCreate");
  }
  auto issue = [&](int64_t p) {
    const int s = static_cast<int>(p & 1);
    const int64_t first = p * fp.per, count = std::min(fp.per, fp.items - first);
    hipError_t e = hipSuccess;
    if (fp.segs == 1) {
      e = hipMemcpy2DAsync(slots[s]->h, size_t(fp.seg), d_src + fp.chunk(first) * src_stride, size_t(src_stride),
                           size_t(len), size_t(count), hipMemcpyDeviceToHost, st);
    } else {
      for (int64_t i = first; i < first + count && e == hipSuccess; i++)
        e = hipMemcpyAsync(slots[s]->h + (i - first) * fp.seg, d_src + fp.chunk(i) * src_stride + fp.off(i),
                           size_t(fp.bytes(i)), hipMemcpyDeviceToHost, st);
    }
    if (e == hipSuccess) e = hipEventRecord(done[s], st);
    return hip_check(e, "scatter D2H");
  };
  if (rc == NXEC_OK) rc = issue(0);
  for (int64_t p = 0; p < fp.npieces && rc == NXEC_OK; p++) {
    const int s = static_cast<int>(p & 1);
    if (p + 1 < fp.npieces && (rc = issue(p + 1))) break;
    if ((rc = hip_check(hipEventSynchronize(done[s]), "scatter piece sync"))) break;
    const int64_t first = p * fp.per, count = std::min(fp.per, fp.items - first);
    frame_copies(fp, first, count, slots[s]->h, [&](int64_t item, int64_t o, int64_t nb, uint8_t *stage) {
      std::memcpy(h_chunks[fp.chunk(item)] + fp.off(item) + o, stage, size_t(nb));
    });
  }
  hipError_t e = hipStreamSynchronize(st);
  if (rc == NXEC_OK) rc = hip_check(e, "scatter sync");
  for (int s = 0; s < 2; s++) {
    if (done[s]) (void)hipEventDestroy(done[s]);
    if (slots[s]) release_slot(ctx, slots[s]);
  }
  return rc;
}

}  // extern "C"

// One asynchronous frame copy: the synchronous call run on its own thread,
// its status and error message kept for nxec_request_wait.
struct nxec_request {
  std::vector<unsigned char *> frames;  // the caller's frame table, copied
  std::thread worker;
  int rc = NXEC_OK;
  std::string error;
};

namespace {
template <class Fn>
int start_request(const void *frames, int64_t nchunks, Fn &&fn, nxec_request_t **req) {
  auto *r = new (std::nothrow) nxec_request();
  if (!r) return set_error(NXEC_ERR_NOMEM, "nxec request: out of memory");
  const auto *f = static_cast<unsigned char *const *>(frames);
  r->frames.assign(f, f + nchunks);
  try {
    r->worker = std::thread([r, fn]() {
      r->rc = fn(r->frames.data());
      if (r->rc != NXEC_OK) r->error = g_last_error;
    });
  } catch (const std::system_error &) {
    delete r;
    return set_error(NXEC_ERR_HIP, "nxec request: cannot start a worker thread");
  }
  *req = r;
  return NXEC_OK;
}
}  // namespace

extern "C" {

int nxec_gather_chunks_async(nxec_ctx_t *ctx, const unsigned char *const *h_chunks, int64_t nchunks, int64_t len,
                             unsigned char *d_dst, int64_t dst_stride, void *stream, nxec_request_t **req) {
  if (!req) return set_error(NXEC_ERR_INVALID, "nxec_gather_chunks_async: null request pointer");
  *req = nullptr;
  int rc = frames_check(ctx, h_chunks, nchunks, len, d_dst, dst_stride, "nxec_gather_chunks_async");
  if (rc) return rc;
  return start_request(
      h_chunks, nchunks,
      [=](unsigned char *const *fr) {
        return nxec_gather_chunks(ctx, const_cast<const unsigned char *const *>(fr), nchunks, len, d_dst, dst_stride,
                                  stream);
      },
      req);
}

int nxec_scatter_chunks_async(nxec_ctx_t *ctx, const unsigned char *d_src, int64_t src_stride, int64_t nchunks,
                              int64_t len, unsigned char *const *h_chunks, void *stream, nxec_request_t **req) {
  if (!req) return set_error(NXEC_ERR_INVALID, "nxec_scatter_chunks_async: null request pointer");
  *req = nullptr;
  int rc = frames_check(ctx, h_chunks, nchunks, len, d_src, src_stride, "nxec_scatter_chunks_async");
  if (rc) return rc;
  return start_request(
      h_chunks, nchunks,
      [=](unsigned char *const *fr) { return nxec_scatter_chunks(ctx, d_src, src_stride, nchunks, len, fr, stream); },
      req);
}

int nxec_request_wait(nxec_request_t *req) {
  if (!req) return NXEC_OK;
  if (req->worker.joinable()) req->worker.join();
  const int rc = req->rc;
  if (rc != NXEC_OK) g_last_error = req->error;
  delete req;
  return rc;
}

int nxec_rs_recover_frames(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                           unsigned char *const *frames, int64_t len, int64_t nstripes) {
  if (!ctx || !valid_nk(n, k) || nfailed < 0 || len < 0 || nstripes < 0 || (nfailed > 0 && !failed) ||
      (nstripes > 0 && !frames))
    return set_error(NXEC_ERR_INVALID, "nxec_rs_recover_frames: invalid arguments");
  if (nfailed == 0 || len == 0 || nstripes == 0) return NXEC_OK;
  std::vector<int32_t> inputs(n);
  std::vector<uint8_t> rm(static_cast<size_t>(nfailed) * k);
  int ni = 0, mi = 0;
  int rc = nxec_rs_plan(n, k, failed, nfailed, 1, inputs.data(), &ni, &mi, rm.data());  // rs.cc:238-322
  if (rc) return rc;
  if ((rc = ensure_device(ctx->device))) return rc;
  const int e = nfailed, w = k + e;
  for (int64_t s = 0; s < nstripes; s++)
    for (int j = 0; j < w; j++) {
      const int c = j < k ? inputs[j] : failed[j - k];
      if (!frames[s * n + c])
        return set_error(NXEC_ERR_INVALID, "nxec_rs_recover_frames: stripe %lld chunk %d frame is null",
                         static_cast<long long>(s), c);
    }
  // Zero copy when every frame involved is pinned / registered: one kernel
  // reads the k survivors and writes the e recovered chunks over PCIe
  // through device pointer tables ([s][k] inputs, then [s][e] outputs).
  std::vector<uint64_t> tab(static_cast<size_t>(nstripes) * w);
  bool direct = true;
  for (int64_t s = 0; s < nstripes && direct; s++)
    for (int j = 0; j < w && direct; j++) {
      const int c = j < k ? inputs[j] : failed[j - k];
      void *dv = host_device_view_range(frames[s * n + c], static_cast<size_t>(len));
      direct = dv != nullptr;
      (j < k ? tab[s * k + j] : tab[nstripes * k + s * e + (j - k)]) = reinterpret_cast<uintptr_t>(dv);
    }
  if (direct) {
    Slot *slot = nullptr;
    if ((rc = acquire_slot(ctx, tab.size() * sizeof(uint64_t), &slot))) return rc;
    std::memcpy(slot->h, tab.data(), tab.size() * sizeof(uint64_t));
    rc = hip_check(hipMemcpyAsync(slot->d, slot->h, tab.size() * sizeof(uint64_t), hipMemcpyHostToDevice, slot->stream),
                   "pointer tables H2D");
    const auto *d_src = reinterpret_cast<const unsigned char *const *>(slot->d);
    auto *d_dst = reinterpret_cast<unsigned char *const *>(slot->d + size_t(nstripes) * k * sizeof(uint64_t));
    if (!rc) rc = nxec_stripes_mul_ptrs(ctx, e, k, rm.data(), d_src, d_dst, len, nstripes, slot->stream);
    hipError_t he = hipStreamSynchronize(slot->stream);
    if (!rc) rc = hip_check(he, "recover_frames sync");
    release_slot(ctx, slot);
    return rc;
  }
  // Otherwise staged through HBM in batches: gather the survivors' frames into
  // [B][k+e][stride], recover rows k.., scatter them to the failed frames.
  const int64_t stride = (len + 15) / 16 * 16;
  const int64_t B = std::max<int64_t>(1, std::min<int64_t>(nstripes, (int64_t(256) << 20) / (w * stride)));
  std::unique_lock<std::mutex> lk;
  ObjStage priv, *pstg = nullptr;
  if ((rc = batch_stage(ctx, size_t(B) * w * stride, lk, priv, &pstg))) return rc;
  uint8_t *d = pstg->d;
  hipStream_t st = pstg->streams[0];
  std::vector<int32_t> dst(e);
  for (int r = 0; r < e; r++) dst[r] = k + r;
  std::vector<const unsigned char *> in_f(B);
  std::vector<unsigned char *> out_f(B);
  for (int64_t s0 = 0; s0 < nstripes && rc == NXEC_OK; s0 += B) {
    const int64_t nb = std::min(B, nstripes - s0);
    for (int j = 0; j < k && rc == NXEC_OK; j++) {
      for (int64_t i = 0; i < nb; i++) in_f[i] = frames[(s0 + i) * n + inputs[j]];
      rc = nxec_gather_chunks(ctx, in_f.data(), nb, len, d + j * stride, w * stride, st);
    }
    if (!rc)
      rc = nxec_stripes_mul(ctx, e, k, rm.data(), d, nullptr, stride, w * stride, d, dst.data(), stride, w * stride,
                            nullptr, len, nb, st);
    for (int r = 0; r < e && rc == NXEC_OK; r++) {
      for (int64_t i = 0; i < nb; i++) out_f[i] = frames[(s0 + i) * n + failed[r]];
      rc = nxec_scatter_chunks(ctx, d + (k + r) * stride, w * stride, nb, len, out_f.data(), st);
    }
  }
  hipError_t he = hipStreamSynchronize(st);
  if (!rc) rc = hip_check(he, "recover_frames sync");
  if (!lk.owns_lock()) priv.release();
  return rc;
}

int nxec_encode_object_host(nxec_ctx_t *ctx, int n, int k, const unsigned char *h_object, int64_t length,
                            int64_t max_chunk_size, unsigned char *h_parity, unsigned char *h_md5,
                            int64_t batch_stripes) {
  if (!ctx) return set_error(NXEC_ERR_INVALID, "null context");
  int64_t nst = 0, nf = 0, cs_last = 0;
  int rc = nxec_object_layout(n, k, length, max_chunk_size, &nst, &nf, &cs_last);
  if (rc) return rc;
  if (nst == 0) return NXEC_OK;
  const int p = n - k;
  const int64_t M = max_chunk_size;
  if (!h_object || (p > 0 && !h_parity)) return set_error(NXEC_ERR_INVALID, "nxec_encode_object_host: null buffer");
  rc = ensure_device(ctx->device);
  if (rc) return rc;
  // MD5 is chain-bound (~one chunk's hash time per launch whatever the chunk
  // count), so batches are large and the slots' streams run concurrently
  if (batch_stripes <= 0) batch_stripes = std::max<int64_t>(1, (int64_t(1) << 30) / (M * n));
  batch_stripes = std::min(batch_stripes, nst);
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
  nxec_gf_gen_rs_matrix(enc.data(), n, k);
  const uint8_t *prow = enc.data() + static_cast<size_t>(k) * k;
  // equal batches: a short last batch would add one whole MD5 chain time
  // (~10 ms for 1 MiB chunks) after everything else has drained
  const int64_t nbatches = (nst + batch_stripes - 1) / batch_stripes;
  batch_stripes = (nst + nbatches - 1) / nbatches;
  const size_t dbytes = size_t(batch_stripes) * k * M, pbytes = size_t(batch_stripes) * std::max(p, 1) * M,
               mbytes = size_t(batch_stripes) * n * 16;
  std::unique_lock<std::mutex> lk;
  ObjStage priv, *pstg = nullptr;
  if ((rc = batch_stage(ctx, dbytes + pbytes + mbytes, lk, priv, &pstg))) return rc;
  ObjStage &stg = *pstg;
  const int64_t ds = int64_t(n) * 16;
  int prev = -1;
  for (int64_t b = 0; b < nbatches && rc == NXEC_OK; b++) {
    const int slot = static_cast<int>(b % kObjSlots);
    hipStream_t st = stg.streams[slot];
    uint8_t *dbuf = stg.d + slot * stg.cap, *pbuf = dbuf + dbytes, *mbuf = pbuf + pbytes;
    const int64_t s0 = b * batch_stripes, nb = std::min(batch_stripes, nst - s0);
    const int64_t nfull = std::max<int64_t>(0, std::min(nb, nf - s0));  // full stripes in this batch
    const bool tail = s0 + nb > nf;
    // H2D copies run one batch after another (concurrent ones share the link
    // and would delay the first batch's compute)
    if (prev >= 0) rc = hip_check(hipStreamWaitEvent(st, stg.h2d_done[prev], 0), "H2D order");
    // data: the full stripes are one contiguous run of the object
    if (!rc && nfull > 0)
      rc = hip_check(hipMemcpyAsync(dbuf, h_object + s0 * k * M, size_t(nfull) * k * M, hipMemcpyHostToDevice, st),
                     "H2D");
    uint8_t *dtail = dbuf + nfull * k * M;
    const int64_t rem = length - nf * k * M;
    if (!rc && tail) {
      rc = hip_check(hipMemsetAsync(dtail, 0, size_t(k) * cs_last, st), "tail pad");
      if (!rc) rc = hip_check(hipMemcpyAsync(dtail, h_object + nf * k * M, rem, hipMemcpyHostToDevice, st), "tail H2D");
    }
    if (!rc) rc = hip_check(hipEventRecord(stg.h2d_done[slot], st), "H2D event");
    prev = slot;
    if (!rc && p > 0 && nfull > 0)
      rc = nxec_stripes_mul(ctx, p, k, prow, dbuf, nullptr, M, k * M, pbuf, nullptr, M, p * M, nullptr, M, nfull, st);
    if (!rc && p > 0 && tail)
      rc = nxec_stripes_mul(ctx, p, k, prow, dtail, nullptr, cs_last, k * cs_last, pbuf + nfull * p * M, nullptr, M,
                            p * M, nullptr, cs_last, 1, st);
    if (!rc && h_md5) {
      const Md5Region r[4] = {
          {dbuf, M, k * M, M, nfull, mbuf, ds, k},
          {pbuf, M, p * M, M, p > 0 ? nfull : 0, mbuf + int64_t(k) * 16, ds, p},
          {dtail, cs_last, k * cs_last, cs_last, tail ? 1 : 0, mbuf + nfull * ds, ds, k},
          {pbuf + nfull * p * M, M, p * M, cs_last, (tail && p > 0) ? 1 : 0, mbuf + nfull * ds + int64_t(k) * 16, ds,
           p},
      };
      rc = launch_md5(r, 4, st);
    }
    if (!rc && p > 0 && nfull > 0)
      rc = hip_check(hipMemcpyAsync(h_parity + s0 * p * M, pbuf, size_t(nfull) * p * M, hipMemcpyDeviceToHost, st),
                     "D2H");
    if (!rc && p > 0 && tail)  // last stripe: first cs_last bytes of each parity slot
      rc = hip_check(hipMemcpy2DAsync(h_parity + nf * p * M, M, pbuf + nfull * p * M, M, cs_last, p,
                                      hipMemcpyDeviceToHost, st),
                     "tail D2H");
    if (!rc && h_md5)
      rc = hip_check(hipMemcpyAsync(h_md5 + s0 * ds, mbuf, size_t(nb) * ds, hipMemcpyDeviceToHost, st), "md5 D2H");
  }
  for (int i = 0; i < kObjSlots; i++) {
    hipError_t e = hipStreamSynchronize(stg.streams[i]);
    if (!rc) rc = hip_check(e, "encode_object_host sync");
  }
  if (!lk.owns_lock()) priv.release();
  return rc;
}

}  // extern "C"

namespace {

constexpr int kNotPinned = 1;  // encode_host_pinned: some input is not device-mapped

// nxec_encode_host whose inputs are all pinned / registered host memory
// (e.g. Chunk buffers from the pinned arena, chunk.hh): the inputs never pass
// through a host staging copy.  Outputs that are pinned too are written in
// place; pageable outputs (RSCode::decode's malloc'd result, rs.cc:164-173)
// come back through the call's pinned slot.  Few concurrent callers: one
// kernel reads the inputs and writes the outputs over PCIe through device
// pointer tables (zero copy).  Many callers: the copy engines DMA every input
// straight from its chunk into HBM and every output back, around the kernel
// (they share the link better than many zero-copy kernels).
// Returns kNotPinned (nothing done) when an input is pageable.
int encode_host_pinned(nxec_ctx_t *ctx, int len, int k, int rows, const unsigned char *coeffs,
                       const unsigned char *const *data, unsigned char *const *coding, int inflight) {
  std::vector<uint64_t> tab(static_cast<size_t>(k) + rows);
  std::vector<bool> out_mapped(rows);
  for (int j = 0; j < k; j++) {
    void *dv = aligned16(data[j]) ? host_device_view_range(data[j], static_cast<size_t>(len)) : nullptr;
    if (!dv) return kNotPinned;
    tab[j] = reinterpret_cast<uintptr_t>(dv);
  }
  int staged = 0;
  for (int r = 0; r < rows; r++) {
    void *dv = aligned16(coding[r]) ? host_device_view_range(coding[r], static_cast<size_t>(len)) : nullptr;
    out_mapped[r] = dv != nullptr;
    tab[k + r] = reinterpret_cast<uintptr_t>(dv);
    staged += dv == nullptr;
  }
  const bool zero_copy = inflight <= 2;
  const int64_t stride = (static_cast<int64_t>(len) + 15) / 16 * 16;
  const size_t tab_bytes = (tab.size() * sizeof(uint64_t) + 4095) / 4096 * 4096;
  // slot: [pointer table][k + rows chunk slots]; host side holds staged outputs
  // at the same chunk offsets, device side the DMA'd chunks
  const size_t need = tab_bytes + static_cast<size_t>(stride) * (k + rows);
  Slot *slot = nullptr;
  int rc = acquire_slot(ctx, need, &slot);
  if (rc) return rc;
  hipStream_t st = slot->stream;
  auto chunk_off = [&](int i) { return tab_bytes + static_cast<size_t>(stride) * i; };
  if (zero_copy) {
    uint8_t *hv = staged ? static_cast<uint8_t *>(host_device_view(slot->h)) : nullptr;
    if (staged && !hv) rc = set_error(NXEC_ERR_HIP, "encode_host: staging slot is not device-mapped");
    for (int r = 0; r < rows && !rc; r++)
      if (!out_mapped[r]) tab[k + r] = reinterpret_cast<uintptr_t>(hv + chunk_off(k + r));
    if (!rc) {
      std::memcpy(slot->h, tab.data(), tab.size() * sizeof(uint64_t));
      rc = hip_check(hipMemcpyAsync(slot->d, slot->h, tab.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st),
                     "pointer table H2D");
    }
    if (!rc)
      rc = nxec_stripes_mul_ptrs(ctx, rows, k, coeffs, reinterpret_cast<const unsigned char *const *>(slot->d),
                                 reinterpret_cast<unsigned char *const *>(slot->d + size_t(k) * sizeof(uint64_t)), len,
                                 1, st);
  } else {
    for (int j = 0; j < k && !rc; j++)
      rc = hip_check(hipMemcpyAsync(slot->d + chunk_off(j), data[j], size_t(len), hipMemcpyHostToDevice, st), "H2D");
    std::vector<int32_t> dst(rows);
    for (int r = 0; r < rows; r++) dst[r] = k + r;
    if (!rc)
      rc = nxec_stripes_mul(ctx, rows, k, coeffs, slot->d + tab_bytes, nullptr, stride, 0, slot->d + tab_bytes,
                            dst.data(), stride, 0, nullptr, len, 1, st);
    for (int r = 0; r < rows && !rc; r++)
      rc = hip_check(hipMemcpyAsync(out_mapped[r] ? coding[r] : slot->h + chunk_off(k + r),
                                    slot->d + chunk_off(k + r), size_t(len), hipMemcpyDeviceToHost, st),
                     "D2H");
  }
  const hipError_t e = hipStreamSynchronize(st);  // the slot goes back only once drained
  if (!rc) rc = hip_check(e, "encode_host (pinned) sync");
  if (!rc && staged)
    host_parallel_for(rows, [&](int r) {
      if (!out_mapped[r]) std::memcpy(coding[r], slot->h + chunk_off(k + r), size_t(len));
    });
  release_slot(ctx, slot);
  return rc;
}

}  // namespace

extern "C" {

int nxec_encode_host_ex(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *data,
                        unsigned char *const *coding, const int32_t *copy_idx, unsigned char *const *copy_out) {
  int ncopy = 0;
  if (copy_idx)
    for (int j = 0; j < k; j++) ncopy = std::max(ncopy, copy_idx[j] + 1);
  if (len < 0 || k < 1 || k > NXEC_MAX_K || rows < 0 || (rows == 0 && ncopy == 0) || !data ||
      (rows > 0 && (!coeffs || !coding)) || (ncopy > 0 && !copy_out))
    return set_error(NXEC_ERR_INVALID, "nxec_encode_host: invalid arguments");
  if (len == 0) return NXEC_OK;
  nxec_ctx_t *ctx = nullptr;
  int rc = default_ctx(&ctx);
  if (rc) return rc;
  struct InFlight {
    int n;
    InFlight() : n(g_host_calls.fetch_add(1) + 1) {}
    ~InFlight() { g_host_calls.fetch_sub(1); }
  } inflight;
  // chunk buffers that are already pinned (the chunk arena, registered
  // receive pools): straight to the GPU, no staging memcpy
  if (ncopy == 0) {
    rc = encode_host_pinned(ctx, len, k, rows, coeffs, data, coding, inflight.n);
    if (rc != kNotPinned) return rc;
  }
  const int64_t stride = (static_cast<int64_t>(len) + 15) / 16 * 16;  // keep chunks 16-B aligned in staging
  const int nout = rows + ncopy;
  const int nchunks = k + nout;
  Slot *slot = nullptr;
  rc = acquire_slot(ctx, static_cast<size_t>(stride) * nchunks, &slot);
  if (rc) return rc;
  // Pipelined in column pieces: the pool copies piece p of every input into
  // pinned staging while the copy engine and the kernel work on piece p-1;
  // outputs come back per piece.  Staging layout [k inputs][rows outputs]
  // [ncopy pass-through outputs], each chunk at a 16-byte stride.
  const int64_t piece = (len >= 2 * kHostPiece && inflight.n <= 2) ? kHostPiece : stride;
  const int npieces = static_cast<int>((len + piece - 1) / piece);
  while (static_cast<int>(slot->events.size()) < npieces) {
    hipEvent_t ev;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      release_slot(ctx, slot);
      return hip_err(e, "hipEventCreate");
    }
    slot->events.push_back(ev);
  }
  std::vector<int32_t> dst(std::max(rows, 1)), cpy(k, -1);
  for (int r = 0; r < rows; r++) dst[r] = k + r;
  for (int j = 0; j < k; j++)
    if (copy_idx && copy_idx[j] >= 0) cpy[j] = k + rows + copy_idx[j];
  HostPool &pool = HostPool::get();
  // Few callers: zero copy, the kernel works on the pinned staging itself over
  // PCIe (no copy-engine round trip: 1 caller 25.8 -> 33.6 GiB/s).  Many
  // callers: H2D -> kernel -> D2H per piece, whose copy engines share the link
  // better (4 callers 69.8 vs 52.0 GiB/s zero copy; profiles/r01_dropin*.jsonl).
  uint8_t *hv = inflight.n <= 2 ? static_cast<uint8_t *>(host_device_view(slot->h)) : nullptr;
  for (int pc = 0; pc < npieces && rc == NXEC_OK; pc++) {
    const int64_t off = pc * piece, pl = std::min<int64_t>(piece, len - off);
    pool.parallel_for(k, [&](int j) { stage_copy(slot->h + j * stride + off, data[j] + off, static_cast<size_t>(pl)); });
    hipError_t e = hipSuccess;
    uint8_t *base = hv ? hv : slot->d;
    if (!hv) {
      e = hipMemcpy2DAsync(slot->d + off, stride, slot->h + off, stride, static_cast<size_t>(pl), k,
                           hipMemcpyHostToDevice, slot->stream);
      if (e != hipSuccess) {
        rc = hip_err(e, "H2D");
        break;
      }
    }
    rc = nxec_stripes_mul(ctx, rows, k, coeffs, base + off, nullptr, stride, 0, base + off, dst.data(), stride, 0,
                          ncopy ? cpy.data() : nullptr, pl, 1, slot->stream);
    if (rc) break;
    if (!hv)
      e = hipMemcpy2DAsync(slot->h + stride * k + off, stride, slot->d + stride * k + off, stride,
                           static_cast<size_t>(pl), nout, hipMemcpyDeviceToHost, slot->stream);
    if (e == hipSuccess) e = hipEventRecord(slot->events[pc], slot->stream);
    if (e != hipSuccess) rc = hip_err(e, "D2H");
  }
  if (rc == NXEC_OK) {
    for (int pc = 0; pc < npieces && rc == NXEC_OK; pc++) {
      const int64_t off = pc * piece, pl = std::min<int64_t>(piece, len - off);
      hipError_t e = hipEventSynchronize(slot->events[pc]);
      if (e != hipSuccess) {
        rc = hip_err(e, "piece sync");
        break;
      }
      pool.parallel_for(nout, [&](int o) {
        unsigned char *to = nullptr;
        if (o < rows) {
          to = coding[o];
        } else {
          for (int j = 0; j < k; j++)
            if (copy_idx && copy_idx[j] == o - rows) to = copy_out[o - rows];
        }
        if (to) std::memcpy(to + off, slot->h + (k + o) * stride + off, static_cast<size_t>(pl));
      });
    }
  } else {
    (void)hipStreamSynchronize(slot->stream);
  }
  release_slot(ctx, slot);
  return rc;
}

int nxec_encode_host(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *data,
                     unsigned char *const *coding) {
  if (rows < 1) return set_error(NXEC_ERR_INVALID, "nxec_encode_host: rows must be >= 1");
  return nxec_encode_host_ex(len, k, rows, coeffs, data, coding, nullptr, nullptr);
}

}  // extern "C"

namespace {

int digest_rounds_max() {
  static const int v = [] {
    const char *e = std::getenv("NXEC_DIGEST_ROUNDS");
    return e ? std::max(1, std::atoi(e)) : 4;
  }();
  return v;
}

// One round of zero-copy digest calls: per group of equal (len, k, rows,
// inputs hashed, matrix) one k_gather_md5 launch over pointer tables in a
// pinned slot (device-mapped: no H2D), digests written back into the slot.
// Returns after the launches are queued; `wait` finishes the round.
struct DigestRound {
  struct Group {
    std::vector<DigestJob *> jobs;
    Slot *slot = nullptr;
    size_t md5_off = 0;
    int nh = 0;
    bool hsrc = false;
  };
  std::vector<Group> groups;
};

int digest_round_launch(nxec_ctx_t *ctx, const std::vector<DigestJob *> &jobs, DigestRound &round) {
  std::map<std::string, size_t> key_of;
  for (DigestJob *j : jobs) {
    std::string key(reinterpret_cast<const char *>(&j->len), sizeof(int));
    key.append(reinterpret_cast<const char *>(&j->k), sizeof(int));
    key.append(reinterpret_cast<const char *>(&j->rows), sizeof(int));
    key.append(1, j->md5_data ? 'S' : '-');
    key.append(reinterpret_cast<const char *>(j->coeffs), size_t(j->rows) * j->k);
    auto it = key_of.find(key);
    if (it == key_of.end()) {
      it = key_of.emplace(key, round.groups.size()).first;
      round.groups.emplace_back();
    }
    round.groups[it->second].jobs.push_back(j);
  }
  for (DigestRound::Group &g : round.groups) {
    const DigestJob &j0 = *g.jobs[0];
    const int k = j0.k, p = j0.rows;
    g.hsrc = j0.md5_data != nullptr;
    g.nh = (g.hsrc ? k : 0) + p;
    const size_t nb = g.jobs.size();
    const size_t tab_bytes = nb * size_t(k + p) * 8;
    g.md5_off = (tab_bytes + 255) / 256 * 256;
    const size_t need = std::max<size_t>(g.md5_off + nb * size_t(g.nh) * 16, 4096);
    if (int rc = acquire_slot(ctx, need, &g.slot)) return rc;
    uint8_t *hv = static_cast<uint8_t *>(host_device_view(g.slot->h));
    if (!hv) return set_error(NXEC_ERR_HIP, "encode_host_md5: staging slot is not device-mapped");
    uint64_t *src_tab = reinterpret_cast<uint64_t *>(g.slot->h);
    uint64_t *dst_tab = src_tab + nb * k;
    for (size_t i = 0; i < nb; i++) {
      for (int q = 0; q < k; q++) src_tab[i * k + q] = g.jobs[i]->in_dv[q];
      for (int r = 0; r < p; r++) dst_tab[i * p + r] = g.jobs[i]->out_dv[r];
    }
    GatherMd5Args ga;
    std::memset(&ga, 0, sizeof(ga));
    ga.src_ptrs = reinterpret_cast<const uint8_t *const *>(hv);
    ga.dst_ptrs = reinterpret_cast<uint8_t *const *>(hv + nb * k * 8);
    ga.digests = hv + g.md5_off;
    ga.scratch = g.slot->d;
    ga.len = j0.len;
    ga.nstripes = int64_t(nb);
    ga.k = k;
    ga.p = p;
    ga.hash_src = g.hsrc ? 1 : 0;
    std::memcpy(ga.coef, j0.coeffs, size_t(p) * k);
    if (int rc = launch_gather_md5(ga, ctx->num_cus, g.slot->stream)) return rc;
  }
  return NXEC_OK;
}

int digest_round_wait(nxec_ctx_t *ctx, DigestRound &round, int rc) {
  for (DigestRound::Group &g : round.groups) {
    if (!g.slot) continue;
    const hipError_t e = hipStreamSynchronize(g.slot->stream);
    if (!rc) rc = hip_check(e, "encode_host_md5 sync");
    if (!rc)
      for (size_t i = 0; i < g.jobs.size(); i++) {
        const uint8_t *dg = g.slot->h + g.md5_off + i * size_t(g.nh) * 16;
        DigestJob &j = *g.jobs[i];
        if (j.md5_data) std::memcpy(j.md5_data, dg, size_t(j.k) * 16);
        if (j.md5_code) std::memcpy(j.md5_code, dg + (g.hsrc ? size_t(j.k) * 16 : 0), size_t(j.rows) * 16);
      }
    release_slot(ctx, g.slot);
    g.slot = nullptr;
  }
  return rc;
}

}  // namespace

extern "C" {

// nxec_encode_host + digests.  Calls whose chunks are all device-mapped (arena
// Chunks: RSCode::encode's own stripe) go through digest rounds: whichever
// waiting caller finds no round being launched takes every pending call,
// launches them as one k_gather_md5 pass per shape over pointer tables (zero
// copy: no H2D, no D2H) and hands leadership on right after the launch, so
// the next round starts while this one's MD5 chains (~10 ms per MiB on one
// lane, whatever the round's size) run -- up to NXEC_DIGEST_ROUNDS (4) rounds
// in flight.  (The agent service's rounds, below, finish before the next one
// starts: their host gathers of pageable buffers are the bottleneck there.)
// Other calls (pageable or misaligned buffers, k > 16, rows > 4) take the
// agent service's staged form as one request.
int nxec_encode_host_md5(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *data,
                         unsigned char *const *coding, unsigned char *md5_data, unsigned char *md5_code) {
  if (len < 0 || k < 1 || k > NXEC_MAX_K || rows < 1 || rows > NXEC_MAX_N || !coeffs || !data || !coding)
    return set_error(NXEC_ERR_INVALID, "nxec_encode_host_md5: invalid arguments");
  if (!md5_data && !md5_code) return nxec_encode_host(len, k, rows, coeffs, data, coding);
  if (len == 0) {  // RFC 1321 digest of the empty message
    static const unsigned char empty[16] = {0xd4, 0x1d, 0x8c, 0xd9, 0x8f, 0x00, 0xb2, 0x04,
                                            0xe9, 0x80, 0x09, 0x98, 0xec, 0xf8, 0x42, 0x7e};
    for (int j = 0; md5_data && j < k; j++) std::memcpy(md5_data + 16 * j, empty, 16);
    for (int r = 0; md5_code && r < rows; r++) std::memcpy(md5_code + 16 * r, empty, 16);
    return NXEC_OK;
  }
  // digests on the host pool or in the coding kernel (nxec_digest_place.cpp)
  if (digest_place_host(len, (md5_data ? k : 0) + (md5_code ? rows : 0)))
    return encode_host_md5_host_digests(len, k, rows, coeffs, data, coding, md5_data, md5_code);
  const double t_call = digest_clock_ns();
  int rc = NXEC_OK;
  struct Observe {  // the GPU-placed call's latency, whichever way it returns
    int64_t len;
    const int &rc;
    double t0;
    ~Observe() {
      if (rc == NXEC_OK) digest_gpu_observe(len, (digest_clock_ns() - t0) * 1e-6);
    }
  } observe{len, rc, t_call};
  nxec_ctx_t *ctx = nullptr;
  rc = default_ctx(&ctx);
  if (rc) return rc;
  if ((rc = ensure_device(ctx->device))) return rc;
  DigestJob job;
  job.len = len;
  job.k = k;
  job.rows = rows;
  job.coeffs = coeffs;
  job.md5_data = md5_data;
  job.md5_code = md5_code;
  static const bool rounds_env = [] {
    const char *e = std::getenv("NXEC_DIGEST_ROUNDS");
    return !(e && e[0] == '0');
  }();
  bool mapped = rounds_env && k <= kGatherMd5MaxK && rows <= kMaxRowsPerPass;
  for (int j = 0; j < k && mapped; j++) {
    void *dv = aligned16(data[j]) ? host_device_view_range(data[j], size_t(len)) : nullptr;
    mapped = dv != nullptr;
    job.in_dv.push_back(reinterpret_cast<uintptr_t>(dv));
  }
  for (int r = 0; r < rows && mapped; r++) {
    void *dv = aligned16(coding[r]) ? host_device_view_range(coding[r], size_t(len)) : nullptr;
    mapped = dv != nullptr;
    job.out_dv.push_back(reinterpret_cast<uintptr_t>(dv));
  }
  if (!mapped) {
    nxec_agent_req r;
    r.ninputs = k;
    r.noutputs = rows;
    r.matrix = coeffs;
    r.inputs = data;
    r.outputs = coding;
    r.md5 = md5_code;
    r.md5_inputs = md5_data;
    rc = nxec_agent_encode_batch(ctx, &r, 1, len, 0);
    return rc;
  }
  std::unique_lock<std::mutex> lk(ctx->dg_mu);
  ctx->dg_pending.push_back(&job);
  while (!job.done) {
    if (ctx->dg_leader || ctx->dg_pending.empty() || ctx->dg_inflight >= digest_rounds_max()) {
      ctx->dg_cv.wait(lk);
      continue;
    }
    ctx->dg_leader = true;
    ctx->dg_inflight++;
    std::vector<DigestJob *> jobs(ctx->dg_pending.begin(), ctx->dg_pending.end());
    ctx->dg_pending.clear();
    lk.unlock();
    DigestRound round;
    int rrc = NXEC_OK;
    std::string err;
    try {
      rrc = digest_round_launch(ctx, jobs, round);
    } catch (const std::exception &e) {
      rrc = set_error(NXEC_ERR_NOMEM, "nxec_encode_host_md5: %s", e.what());
    }
    lk.lock();
    ctx->dg_leader = false;  // the next round may launch while this one runs
    ctx->dg_cv.notify_all();
    lk.unlock();
    rrc = digest_round_wait(ctx, round, rrc);
    if (rrc) err = g_last_error;
    lk.lock();
    for (DigestJob *j : jobs) {
      j->rc = rrc;
      j->error = err;
      j->done = true;
    }
    ctx->dg_inflight--;
    ctx->dg_cv.notify_all();
  }
  lk.unlock();
  if (job.rc != NXEC_OK) g_last_error = job.error;
  rc = job.rc;
  return rc;
}

int nxec_ec_encode_data_status(int len, int k, int rows, const unsigned char *gftbls, const unsigned char *const *data,
                               unsigned char *const *coding) {
  if (!gftbls || k < 1 || rows < 1) return set_error(NXEC_ERR_INVALID, "nxec_ec_encode_data: invalid arguments");
  // byte [1] of each 32-byte ISA-L table is c*1 = c (gf_vect_mul_init, ec_base.c:169-274)
  std::vector<uint8_t> coeffs(static_cast<size_t>(rows) * k);
  for (size_t i = 0; i < coeffs.size(); i++) coeffs[i] = gftbls[32 * i + 1];
  return nxec_encode_host(len, k, rows, coeffs.data(), data, coding);
}

}  // extern "C"

namespace {

// The plainest path to the GPU, for the retry of the void drop-in: a new
// context (its own stream and staging), inputs copied into pinned staging, one
// H2D, the multiply, one D2H, synchronise, copy out.  No zero copy, no
// pipelining, nothing shared with the context whose call failed.
int encode_host_fresh_staged(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *data,
                             unsigned char *const *coding) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  (void)hipGetLastError();
  nxec_ctx_t *ctx = nullptr;
  int rc = nxec_ctx_create(dev, &ctx);
  if (rc) return rc;
  const int64_t stride = (static_cast<int64_t>(len) + 15) / 16 * 16;
  Slot *slot = nullptr;
  rc = acquire_slot(ctx, static_cast<size_t>(stride) * (k + rows), &slot);
  if (!rc) {
    for (int j = 0; j < k; j++) std::memcpy(slot->h + j * stride, data[j], static_cast<size_t>(len));
    rc = hip_check(hipMemcpyAsync(slot->d, slot->h, static_cast<size_t>(stride) * k, hipMemcpyHostToDevice, slot->stream),
                   "retry H2D");
    std::vector<int32_t> dst(rows);
    for (int r = 0; r < rows; r++) dst[r] = k + r;
    if (!rc)
      rc = nxec_stripes_mul(ctx, rows, k, coeffs, slot->d, nullptr, stride, 0, slot->d, dst.data(), stride, 0, nullptr,
                            len, 1, slot->stream);
    if (!rc)
      rc = hip_check(hipMemcpyAsync(slot->h + stride * k, slot->d + stride * k, static_cast<size_t>(stride) * rows,
                                    hipMemcpyDeviceToHost, slot->stream),
                     "retry D2H");
    const hipError_t e = hipStreamSynchronize(slot->stream);
    if (!rc) rc = hip_check(e, "retry sync");
    if (!rc)
      for (int r = 0; r < rows; r++) std::memcpy(coding[r], slot->h + (k + r) * stride, static_cast<size_t>(len));
    release_slot(ctx, slot);
  }
  nxec_ctx_destroy(ctx);
  return rc;
}

// testing hook: NXEC_TEST_FAIL_ENCODE=1 makes the first attempt of every
// nxec_ec_encode_data call fail as a device error would (no work done)
bool test_fail_first_attempt() {
  static const bool t = [] {
    const char *e = std::getenv("NXEC_TEST_FAIL_ENCODE");
    return e && e[0] == '1';
  }();
  return t;
}

}  // namespace

extern "C" {

// ISA-L's ec_encode_data has no error channel (erasure_code.h:98, rs.cc:89),
// so a failed device pass is retried once on a fresh context through the
// staged path (a transient error -- a busy queue, a lost stream -- does not
// take the proxy and its background repair thread down); only when that fails
// too does the process stop rather than return undefined parity.
void nxec_ec_encode_data(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                         unsigned char **coding) {
  int rc = test_fail_first_attempt() ? set_error(NXEC_ERR_HIP, "injected device error (NXEC_TEST_FAIL_ENCODE)")
                                     : nxec_ec_encode_data_status(len, k, rows, gftbls, data, coding);
  if (rc == NXEC_OK) return;
  if (rc != NXEC_ERR_INVALID) {
    std::fprintf(stderr, "nxec_ec_encode_data failed (%d): %s; retrying once on a fresh context (staged)\n", rc,
                 nxec_last_error());
    std::vector<uint8_t> coeffs(static_cast<size_t>(rows) * k);
    for (size_t i = 0; i < coeffs.size(); i++) coeffs[i] = gftbls[32 * i + 1];
    rc = encode_host_fresh_staged(len, k, rows, coeffs.data(), data, coding);
    if (rc == NXEC_OK) return;
  }
  std::fprintf(stderr, "nxec_ec_encode_data failed (%d): %s\n", rc, nxec_last_error());
  std::abort();
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
