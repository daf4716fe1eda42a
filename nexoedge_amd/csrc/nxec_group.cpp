// In-process multi-GPU sharding: one context per device, the
// stripes of a batch split into contiguous ranges (sizes differ by at most
// one, as nexoedge_amd/dist.py shard_range), one host thread per device
// driving its own streams.  Stripes are independent, so there is no
// collective and no peer traffic: each device codes its own range.  Each
// device thread runs on the CPUs of its GPU's NUMA node (nxec_numa.cpp), so
// its staging copies and zero-copy PCIe traffic stay on that socket.
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "nxec_internal.h"

namespace nxec {
std::vector<int> pci_node_cpus(const char *bus_id, int *node);
bool bind_thread_cpus(const std::vector<int> &cpus);
int device_bus_id(int device, char *buf, int len);
}  // namespace nxec

struct nxec_group {
  std::vector<nxec_ctx_t *> ctxs;
  std::vector<int> devices;
  std::vector<std::vector<int>> cpus;  // per device: its NUMA node's CPUs (empty: unknown)
};

namespace {

// [lo, hi) of shard i of total over parts
void shard(int64_t total, int parts, int i, int64_t *lo, int64_t *hi) {
  const int64_t base = total / parts, extra = total % parts;
  *lo = i * base + (i < extra ? i : extra);
  *hi = *lo + base + (i < extra ? 1 : 0);
}

// runs fn(i) on one thread per device; the first failure's message becomes
// the caller's last error
template <class F>
int run_all(nxec_group *g, F fn) {
  const int nd = static_cast<int>(g->ctxs.size());
  std::vector<int> rc(nd, NXEC_OK);
  std::vector<std::string> msg(nd);
  std::vector<std::thread> th;
  th.reserve(static_cast<size_t>(nd));
  auto body = [&](int i) {
    rc[i] = fn(i);
    if (rc[i] != NXEC_OK) msg[i] = nxec_last_error();
  };
  for (int i = 0; i < nd; i++) {
    try {
      th.emplace_back([&, i] {
        (void)nxec::bind_thread_cpus(g->cpus[i]);
        body(i);
      });
    } catch (const std::system_error &) {
      body(i);  // no thread to be had: this device's share on the calling thread
    }
  }
  for (auto &t : th) t.join();
  for (int i = 0; i < nd; i++)
    if (rc[i] != NXEC_OK) return nxec::set_error(rc[i], "device %d: %s", g->devices[i], msg[i].c_str());
  return NXEC_OK;
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
    g->ctxs.push_back(c);
    g->devices.push_back(devices[i]);
    char bus[64] = {0};
    int node = -1;
    g->cpus.push_back(nxec::device_bus_id(devices[i], bus, sizeof(bus)) == NXEC_OK ? nxec::pci_node_cpus(bus, &node)
                                                                                   : std::vector<int>());
  }
  *out = g;
  return NXEC_OK;
}

void nxec_group_destroy(nxec_group_t *g) {
  if (!g) return;
  for (nxec_ctx_t *c : g->ctxs) nxec_ctx_destroy(c);
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

int nxec_group_rs_encode_stripes(nxec_group_t *g, int n, int k, unsigned char *const *d_stripes, int64_t chunk_stride,
                                 int64_t stripe_stride, int64_t len, const int64_t *nstripes) {
  if (!g || g->ctxs.empty() || !d_stripes || !nstripes)
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_rs_encode_stripes: invalid arguments");
  return run_all(g, [&](int i) {
    int rc = nxec_rs_encode_stripes(g->ctxs[i], n, k, d_stripes[i], chunk_stride, stripe_stride, len, nstripes[i],
                                    nullptr);
    return rc != NXEC_OK ? rc : nxec_stream_sync(nxec_ctx_stream(g->ctxs[i]));
  });
}

int nxec_group_rs_recover_stripes(nxec_group_t *g, int n, int k, const int32_t *failed, int nfailed,
                                  unsigned char *const *d_stripes, int64_t chunk_stride, int64_t stripe_stride,
                                  int64_t len, const int64_t *nstripes) {
  if (!g || g->ctxs.empty() || !d_stripes || !nstripes)
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_group_rs_recover_stripes: invalid arguments");
  return run_all(g, [&](int i) {
    int rc = nxec_rs_recover_stripes(g->ctxs[i], n, k, failed, nfailed, d_stripes[i], chunk_stride, stripe_stride, len,
                                     nstripes[i], nullptr);
    return rc != NXEC_OK ? rc : nxec_stream_sync(nxec_ctx_stream(g->ctxs[i]));
  });
}

}  // extern "C"
