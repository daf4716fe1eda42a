// In-process multi-GPU sharding ("one host thread + hipSetDevice +
// streams per GPU"): one context per member, the stripes of a batch split into
// contiguous ranges (sizes differ by at most one, as nexoedge_amd/dist.py
// shard_range).  Stripes are independent, so there is no collective and no
// peer traffic: each member codes its own range.
//
// Each member owns one long-lived host thread, started by nxec_group_create,
// bound once to the CPUs of its GPU's NUMA node (nxec_numa.cpp) with the
// member's device current, and fed through a FIFO of tasks.  A synchronous
// group call queues one task per member and waits for all of them; the _async
// forms queue the launches and return at once (a member's tasks run in
// submission order, each launching on the member context's stream), and
// nxec_group_wait queues a stream drain behind them -- so a step's encode and
// recover are two queued launches per member and one wait, as the ranks of
// bench.py issue them, not two host-synchronous fan-outs.  Members listed on
// the same device share kGroupStreams streams: with a stream each, 8 members'
// kernels interleaved their workgroups on one GPU (28-72 ms per step against
// 19.3 for the same work from 8 processes; profiles/r06_group_*.json).
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "nxec_runtime.h"

namespace nxec {
bool bind_thread_cpus(const std::vector<int> &cpus);
}  // namespace nxec

namespace {


struct MemberThread {
  int device = 0;
  nxec_ctx_t *ctx = nullptr;
  // the stream its launches go to: its context's, or -- a device listed more
  // than kGroupStreams times -- one of that device's first members' streams,
  // so one GPU's members do not interleave the workgroups of many kernels
  void *stream = nullptr;
  std::vector<int> cpus;  // its NUMA node's CPUs (empty: unknown)
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> tasks;
  bool stop = false;
  std::thread th;
  // first failure of an asynchronous task since the last nxec_group_wait
  int async_rc = NXEC_OK;
  std::string async_msg;

  void post(std::function<void()> t) {
    {
      std::lock_guard<std::mutex> lk(mu);
      tasks.push_back(std::move(t));
    }
    cv.notify_one();
  }
  void loop() {
    (void)nxec::bind_thread_cpus(cpus);
    (void)nxec::ensure_device(device);
    while (true) {
      std::function<void()> t;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [this] { return stop || !tasks.empty(); });
        if (tasks.empty()) return;  // stop, queue drained
        t = std::move(tasks.front());
        tasks.pop_front();
      }
      t();
    }
  }
};

// [lo, hi) of shard i of total over parts
void shard(int64_t total, int parts, int i, int64_t *lo, int64_t *hi) {
  const int64_t base = total / parts, extra = total % parts;
  *lo = i * base + (i < extra ? i : extra);
  *hi = *lo + base + (i < extra ? 1 : 0);
}

// a countdown the calling thread waits on
struct Latch {
  std::mutex mu;
  std::condition_variable cv;
  int left;
  explicit Latch(int n) : left(n) {}
  void done() {
    std::lock_guard<std::mutex> lk(mu);
    if (--left == 0) cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return left == 0; });
  }
};

}  // namespace

struct nxec_group {
  std::vector<MemberThread *> members;
  std::vector<nxec_ctx_t *> ctxs;
  std::vector<int> devices;
};

namespace {

// runs fn(i) on every member's thread and waits; the first failure's message
// becomes the caller's last error
template <class F>
int run_all(nxec_group *g, F fn) {
  const int nd = static_cast<int>(g->members.size());
  std::vector<int> rc(nd, NXEC_OK);
  std::vector<std::string> msg(nd);
  Latch latch(nd);
  for (int i = 0; i < nd; i++)
    g->members[i]->post([&, i] {
      rc[i] = fn(i);
      if (rc[i] != NXEC_OK) msg[i] = nxec_last_error();
      latch.done();
    });
  latch.wait();
  for (int i = 0; i < nd; i++)
    if (rc[i] != NXEC_OK) return nxec::set_error(rc[i], "device %d: %s", g->devices[i], msg[i].c_str());
  return NXEC_OK;
}

// queues fn(i) on every member's thread and returns; a failure is kept for nxec_group_wait
template <class F>
void post_all(nxec_group *g, F fn) {
  const int nd = static_cast<int>(g->members.size());
  for (int i = 0; i < nd; i++) {
    MemberThread *m = g->members[i];
    m->post([m, fn, i] {
      const int rc = fn(i);
      if (rc != NXEC_OK) {
        std::lock_guard<std::mutex> lk(m->mu);
        if (m->async_rc == NXEC_OK) {
          m->async_rc = rc;
          m->async_msg = nxec_last_error();
        }
      }
    });
  }
}

}  // namespace

extern "C" {

int nxec_group_create(const int *devices, int ndevices, nxec_group_t **out) {
  if (!out || ndevices < 1 || !devices) return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_create: invalid arguments");
  *out = nullptr;
  nxec_group *g = new nxec_group();
  for (int i = 0; i < ndevices; i++) {
    nxec_ctx_t *c = nullptr;
    const int rc = nxec_ctx_create(devices[i], &c);
    if (rc != NXEC_OK) {
      nxec_group_destroy(g);
      return rc;
    }
    MemberThread *m = new MemberThread();
    m->device = devices[i];
    m->ctx = c;
    // the device's first kGroupStreams members keep their own streams, later
    // ones take them in turn
    m->stream = nxec_ctx_stream(c);
    // (streams per device: two kernels in flight hide each other's ramp-up
    // and drain, many interleave their workgroups -- 8 members on one MI355X:
    // a stream each 28-72 ms per step, one shared 20.75, two 20.1-20.6,
    // against 19.3 for 8 processes; profiles/r06_group_hwq.log)
    const int kGroupStreams = nxec::tuning().group_streams;
    int same = 0;
    for (MemberThread *o : g->members) same += o->device == m->device;
    if (same >= kGroupStreams) {
      int seen = 0;
      for (MemberThread *o : g->members)
        if (o->device == m->device && seen++ == same % kGroupStreams) {
          m->stream = o->stream;
          break;
        }
    }
    char bus[64] = {0};
    int node = -1;
    if (nxec::device_bus_id(devices[i], bus, sizeof(bus)) == NXEC_OK) m->cpus = nxec::pci_node_cpus(bus, &node);
    try {
      m->th = std::thread([m] { m->loop(); });
    } catch (const std::system_error &e) {
      nxec_ctx_destroy(c);
      delete m;
      nxec_group_destroy(g);
      return nxec::set_error(NXEC_ERR_NOMEM, "nxec_group_create: member thread: %s", e.what());
    }
    g->members.push_back(m);
    g->ctxs.push_back(c);
    g->devices.push_back(devices[i]);
  }
  *out = g;
  return NXEC_OK;
}

void nxec_group_destroy(nxec_group_t *g) {
  if (!g) return;
  // every thread drains its queue and stops before any context goes (a
  // member may launch on the stream of the first member of its device)
  for (MemberThread *m : g->members) {
    {
      std::lock_guard<std::mutex> lk(m->mu);
      m->stop = true;
    }
    m->cv.notify_one();
  }
  for (MemberThread *m : g->members) m->th.join();
  for (MemberThread *m : g->members) {
    nxec_ctx_destroy(m->ctx);
    delete m;
  }
  delete g;
}

int nxec_group_size(const nxec_group_t *g) { return g ? static_cast<int>(g->ctxs.size()) : 0; }

nxec_ctx_t *nxec_group_ctx(nxec_group_t *g, int i) {
  return (g && i >= 0 && i < static_cast<int>(g->ctxs.size())) ? g->ctxs[i] : nullptr;
}

int nxec_group_shard(int64_t nstripes, int nparts, int part, int64_t *first, int64_t *count) {
  if (nstripes < 0 || nparts < 1 || part < 0 || part >= nparts || !first || !count)
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_shard: invalid arguments");
  int64_t lo = 0, hi = 0;
  shard(nstripes, nparts, part, &lo, &hi);
  *first = lo;
  *count = hi - lo;
  return NXEC_OK;
}

int nxec_group_rs_encode_host_batch(nxec_group_t *g, int n, int k, const unsigned char *h_data,
                                    unsigned char *h_parity, int64_t len, int64_t nstripes, int64_t batch_stripes) {
  if (!g || g->ctxs.empty()) return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_rs_encode_host_batch: null group");
  if (!nxec::valid_nk(n, k) || len < 0 || nstripes < 0)
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_rs_encode_host_batch: invalid arguments");
  const int nd = static_cast<int>(g->ctxs.size());
  const int p = n - k;
  return run_all(g, [&](int i) {
    int64_t lo = 0, hi = 0;
    shard(nstripes, nd, i, &lo, &hi);
    if (hi == lo) return static_cast<int>(NXEC_OK);
    return nxec_rs_encode_host_batch(g->ctxs[i], n, k, h_data + lo * k * len, h_parity + lo * p * len, len, hi - lo,
                                     batch_stripes);
  });
}

int nxec_group_rs_encode_stripes_async(nxec_group_t *g, int n, int k, unsigned char *const *d_stripes,
                                       int64_t chunk_stride, int64_t stripe_stride, int64_t len,
                                       const int64_t *nstripes) {
  if (!g || g->ctxs.empty() || !d_stripes || !nstripes)
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_rs_encode_stripes: invalid arguments");
  std::vector<unsigned char *> ptrs(d_stripes, d_stripes + g->ctxs.size());
  std::vector<int64_t> counts(nstripes, nstripes + g->ctxs.size());
  post_all(g, [g, n, k, ptrs, chunk_stride, stripe_stride, len, counts](int i) {
    return nxec_rs_encode_stripes(g->ctxs[i], n, k, ptrs[i], chunk_stride, stripe_stride, len, counts[i],
                                  g->members[i]->stream);
  });
  return NXEC_OK;
}

int nxec_group_rs_recover_stripes_async(nxec_group_t *g, int n, int k, const int32_t *failed, int nfailed,
                                        unsigned char *const *d_stripes, int64_t chunk_stride, int64_t stripe_stride,
                                        int64_t len, const int64_t *nstripes) {
  if (!g || g->ctxs.empty() || !d_stripes || !nstripes || nfailed < 0 || (nfailed > 0 && !failed))
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_rs_recover_stripes: invalid arguments");
  std::vector<unsigned char *> ptrs(d_stripes, d_stripes + g->ctxs.size());
  std::vector<int64_t> counts(nstripes, nstripes + g->ctxs.size());
  std::vector<int32_t> f(failed, failed + nfailed);
  post_all(g, [g, n, k, f, ptrs, chunk_stride, stripe_stride, len, counts](int i) {
    return nxec_rs_recover_stripes(g->ctxs[i], n, k, f.data(), static_cast<int>(f.size()), ptrs[i], chunk_stride,
                                   stripe_stride, len, counts[i], g->members[i]->stream);
  });
  return NXEC_OK;
}

int nxec_group_wait(nxec_group_t *g) {
  if (!g || g->ctxs.empty()) return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_wait: null group");
  // behind every queued task: drain the member's stream, then collect the
  // first failure of its asynchronous tasks since the last wait
  return run_all(g, [g](int i) {
    MemberThread *m = g->members[i];
    const int src = nxec_stream_sync(m->stream);
    std::lock_guard<std::mutex> lk(m->mu);
    const int rc = m->async_rc;
    const std::string msg = m->async_msg;
    m->async_rc = NXEC_OK;
    m->async_msg.clear();
    if (rc != NXEC_OK) return nxec::set_error(rc, "%s", msg.c_str());
    return src;
  });
}

int nxec_group_rs_encode_stripes(nxec_group_t *g, int n, int k, unsigned char *const *d_stripes, int64_t chunk_stride,
                                 int64_t stripe_stride, int64_t len, const int64_t *nstripes) {
  if (!g || g->ctxs.empty() || !d_stripes || !nstripes)
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_rs_encode_stripes: invalid arguments");
  return run_all(g, [&](int i) {
    int rc = nxec_rs_encode_stripes(g->ctxs[i], n, k, d_stripes[i], chunk_stride, stripe_stride, len, nstripes[i],
                                    g->members[i]->stream);
    return rc != NXEC_OK ? rc : nxec_stream_sync(g->members[i]->stream);
  });
}

int nxec_group_rs_recover_stripes(nxec_group_t *g, int n, int k, const int32_t *failed, int nfailed,
                                  unsigned char *const *d_stripes, int64_t chunk_stride, int64_t stripe_stride,
                                  int64_t len, const int64_t *nstripes) {
  if (!g || g->ctxs.empty() || !d_stripes || !nstripes)
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_rs_recover_stripes: invalid arguments");
  return run_all(g, [&](int i) {
    int rc = nxec_rs_recover_stripes(g->ctxs[i], n, k, failed, nfailed, d_stripes[i], chunk_stride, stripe_stride, len,
                                     nstripes[i], g->members[i]->stream);
    return rc != NXEC_OK ? rc : nxec_stream_sync(g->members[i]->stream);
  });
}

}  // extern "C"
