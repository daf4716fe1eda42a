// Host runtime internals shared by libnxec's entry-point families:
//   nxec_context.cpp     errors, settings, contexts, staging slots, plumbing
//   nxec_stripes.cpp     device-resident stripe batches (encode / recover /
//                        decode / CAR / MD5 / fused encode + MD5, layouts)
//   nxec_objects.cpp     whole objects and batches of files (writeFileStripe /
//                        decodeFile over every stripe)
//   nxec_host_paths.cpp  host-resident batches, chunk frames, recover into frames
//   nxec_host_encode.cpp the per-stripe drop-in (ISA-L ec_encode_data,
//                        CodingUtils::encode, RSCode::encode's digests)
//   nxec_agent.cpp       the agent coding service
// Compute always goes to the gfx950 kernels; there is no CPU fallback.
#ifndef NXEC_RUNTIME_H
#define NXEC_RUNTIME_H

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "nxec.h"
#include "nxec_internal.h"
#include "nxec_tuning.h"

namespace nxec {

// ---- errors (the calling thread's last-error message) ----
int hip_err(hipError_t e, const char *what);
inline int hip_check(hipError_t e, const char *what) { return e == hipSuccess ? NXEC_OK : hip_err(e, what); }
const std::string &last_error();
void restore_error(const std::string &msg);

#define NXEC_HIP(call)                               \
  do {                                               \
    hipError_t e_ = (call);                          \
    if (e_ != hipSuccess) return hip_err(e_, #call); \
  } while (0)

// ---- deployment settings (INTEGRATION.md "Deployment settings") ----
// NXEC_HOST_DIRECT=0: never let kernels read or write pinned host memory in
// place (zero copy); every host path then stages through HBM by DMA.
bool host_direct_enabled();

// Fault injection for the tests: NXEC_TEST_FAULT names the faults to inject
// (comma-separated): "encode" fails the first attempt of every void ISA-L
// drop-in call as a device error would, "agent_round" makes every agent
// round's leader throw before it runs.
bool test_fault(const char *name);

// ---- host memory ----
// Copy into pinned staging (streaming stores with the NT-staging probe).
void stage_copy(void *dst, const void *src, size_t n);
// Copy out of pinned staging into a caller's buffer (streaming stores with the NT-staging probe).
void unstage_copy(void *dst, const void *src, size_t n);
// Device address of pinned / registered host memory (kernels read and write
// it over PCIe: zero copy), or nullptr for pageable memory or when the
// deployment turned zero copy off.
void *host_device_view(const void *h);
// The same for the whole range [h, h + bytes): both ends must lie in one
// mapping, else nullptr (a partly registered buffer is staged, not faulted).
void *host_device_view_range(const void *h, size_t bytes);
inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

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

// Device staging of the batched host entry points (nxec_encode_object_host,
// nxec_rs_encode_host_batch, staged nxec_rs_recover_frames), kept across calls
// (allocating ~4 GiB per call cost ~12 ms of a 150 ms call): kObjSlots
// batches in flight, one stream and one H2D-done event each.  The context's
// own stream serves as slot 0: HIP has 4 hardware queues per process
// (GPU_MAX_HW_QUEUES), and a fifth stream shares one, serialising two slots'
// copies (object write 44 -> 34 GiB/s).
constexpr int kObjSlots = 3;
struct ObjStage {
  uint8_t *d = nullptr;
  size_t cap = 0;  // bytes per slot
  hipStream_t streams[kObjSlots] = {};
  hipEvent_t h2d_done[kObjSlots] = {};
  bool borrowed0 = false;  // streams[0] is the context's stream
  // nxec_decode_frames' gather stream when streams[0] is borrowed (a gather
  // synchronises its stream per piece: on the context's stream that would
  // wait for other threads' work queued there too); made on first use
  hipStream_t aux = nullptr;
  void release();
};

// staging slots a context grows to before an asynchronous caller waits for
// one of its earlier calls (two in flight keep the GPU fed: the host plans
// call i + 1 while call i runs)
constexpr size_t kAsyncSlots = 4;

}  // namespace nxec

struct AgentJob;
struct DigestJob;

struct nxec_ctx {
  int device = 0;
  int num_cus = 0;
  int numa_node = -1;  // of the device's PCIe root (-1: unknown): its host copies run on that node's pool
  hipStream_t stream = nullptr;
  std::mutex slot_mu;
  std::vector<nxec::Slot *> free_slots;
  std::vector<nxec::Slot *> all_slots;
  std::mutex obj_mu;  // guards obj (one object host call at a time uses it)
  nxec::ObjStage obj;
  // agent-service aggregation (nxec_agent_encode_batch): concurrent callers'
  // requests join one round; one caller at a time leads and runs the round
  std::mutex agent_mu;
  std::condition_variable agent_cv;
  std::deque<AgentJob *> agent_pending;
  bool agent_leader = false;
  // nxec_encode_host_md5 rounds (zero copy): a leader launches every pending
  // call in one kernel and hands leadership on at once, so rounds overlap
  std::mutex dg_mu;
  std::condition_variable dg_cv;
  std::deque<DigestJob *> dg_pending;
  bool dg_leader = false;
  int dg_inflight = 0;
  // nxec_kernel_timing: event pairs around the coding launches, read by nxec_kernel_time
  std::mutex kt_mu;
  bool kt_on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> kt_pending;
  double kt_ms = 0;
  int64_t kt_launches = 0;
  // an all-zero device line of zero_bytes (chunks of a last stripe past its
  // data read from here: nxec_encode_objects_ex), grown on demand
  std::mutex zero_mu;
  uint8_t *zero = nullptr;
  size_t zero_bytes = 0;
  std::vector<uint8_t *> zero_retired;  // outgrown lines, freed by nxec_ctx_destroy
};

namespace nxec {

int ensure_device(int device);
// NUMA placement helpers (nxec_numa.cpp)
std::vector<int> pci_node_cpus(const char *bus_id, int *node);
int device_bus_id(int device, char *buf, int len);
int cpu_numa_node(int cpu);  // -1: unknown
std::vector<int> node_cpus(int node);  // empty: unknown
bool bind_thread_cpus(const std::vector<int> &cpus);
// A slot of at least `bytes` from the context's pool (best fit).  Slots an
// asynchronous call handed back busy go only to callers that may wait for
// them (may_wait: the asynchronous multi-file write, once the context holds
// kAsyncSlots); others get an idle slot or a new one.
int acquire_slot(nxec_ctx_t *ctx, size_t bytes, Slot **out, bool may_wait = false);
void release_slot(nxec_ctx_t *ctx, Slot *s);
// The context's persistent batch staging (kObjSlots slots of at least
// slot_bytes), or a private one in `priv` while another call holds the
// context's; the caller releases `priv` when it did not get the lock.
int batch_stage(nxec_ctx_t *ctx, size_t slot_bytes, std::unique_lock<std::mutex> &lk, ObjStage &priv, ObjStage **out);
// A default context leased for one call of an entry point that takes none
// (the drop-in): a member of the default pool (nxec_context.cpp), its device
// made current for the call; the destructor hands the member back and makes
// the caller's own device current again.
class DefaultLease {
 public:
  DefaultLease() = default;
  DefaultLease(const DefaultLease &) = delete;
  DefaultLease &operator=(const DefaultLease &) = delete;
  ~DefaultLease();
  nxec_ctx_t *ctx = nullptr;
  int device_inflight = 1;  // calls in flight on ctx's device, this one included
 private:
  friend int default_ctx(DefaultLease &lease, bool admit);
  friend int lease_admit(DefaultLease &lease);
  void *member_ = nullptr;
  void *gate_ = nullptr;  // the device's admission gate this call holds (pool_admit)
  int saved_device_ = -1;
};
// admit = false: skip the device's admission gate (a call that mostly waits
// for a shared digest round holds no staging of its own while it waits)
int default_ctx(DefaultLease &lease, bool admit = true);
// The device admission of a lease taken with admit = false (no-op when it
// already holds a place or the gate is off); returns the calls running.
int lease_admit(DefaultLease &lease);
inline hipStream_t pick_stream(nxec_ctx_t *ctx, void *stream) {
  return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}
// At least `bytes` of zeros on the context's device (never written after).
int zero_line(nxec_ctx_t *ctx, size_t bytes, const uint8_t **out);

// an event pair around a coding launch when nxec_kernel_timing is on (else nulls)
void kt_begin(nxec_ctx_t *ctx, hipStream_t st, hipEvent_t ev[2]);
void kt_end(nxec_ctx_t *ctx, const hipEvent_t ev[2], hipStream_t st);

// The strided (d_src_ptrs == nullptr) and gather forms of nxec_stripes_mul.
int stripes_mul_impl(nxec_ctx_t *ctx, int rows, int k, const unsigned char *coeffs, const unsigned char *d_src,
                     const unsigned char *const *d_src_ptrs, const int32_t *src_idx, int64_t src_cs, int64_t src_ss,
                     unsigned char *d_dst, unsigned char *const *d_dst_ptrs, const int32_t *dst_idx, int64_t dst_cs,
                     int64_t dst_ss, const int32_t *copy_idx, int64_t len, int64_t nstripes, void *stream);
// Fused write-path launch (encode + MD5 of all n chunks): data chunk j of
// stripe s at data + s*data_ss + j*data_cs, parity row r at parity + s*par_ss
// + r*par_cs, digests [s][n][16].  False when the fused kernel cannot take it.
bool encode_md5_args(int n, int k, const unsigned char *data, int64_t data_cs, int64_t data_ss, unsigned char *parity,
                     int64_t par_cs, int64_t par_ss, unsigned char *digests, int64_t len, int64_t nstripes,
                     MulMd5Args &a);

}  // namespace nxec

#endif  // NXEC_RUNTIME_H
