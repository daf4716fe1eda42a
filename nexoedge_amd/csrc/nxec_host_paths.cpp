// Host-resident batches and chunk frames (include/nxec.h §7): the write
// path's host batch (data in, parity out over PCIe), the wire-format adapter
// between received / sent chunk frames and strided device batches
// (io.cc:209-216, :334-336), its asynchronous forms, the recover straight
// into frames, and the host-inclusive object write.
#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <cstring>
#include <functional>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "nxec_runtime.h"

using namespace nxec;

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
void frame_copies(const FramePlan &fp, int64_t first, int64_t count, uint8_t *staging, HostLane lane, int node,
                  const std::function<void(int64_t item, int64_t off, int64_t n, uint8_t *stage)> &copy) {
  const int64_t job = int64_t(1) << 20;
  const int64_t jobs_per_item = (fp.seg + job - 1) / job;
  host_parallel_for(static_cast<int>(count * jobs_per_item), [&](int t) {
    const int64_t i = t / jobs_per_item, o = (t % jobs_per_item) * job;
    const int64_t b = fp.bytes(first + i);
    if (o < b) copy(first + i, o, std::min(job, b - o), staging + i * fp.seg + o);
  }, lane, node);
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
    frame_copies(fp, first, count, slots[s]->h, HostLane::kIn, ctx->numa_node, [&](int64_t item, int64_t o, int64_t nb, uint8_t *stage) {
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
    frame_copies(fp, first, count, slots[s]->h, HostLane::kOut, ctx->numa_node, [&](int64_t item, int64_t o, int64_t nb, uint8_t *stage) {
      unstage_copy(h_chunks[fp.chunk(item)] + fp.off(item) + o, stage, size_t(nb));
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
  try {
    r->frames.assign(f, f + nchunks);
    r->worker = std::thread([r, fn]() {
      r->rc = fn(r->frames.data());
      if (r->rc != NXEC_OK) r->error = last_error();
    });
  } catch (const std::bad_alloc &) {
    delete r;
    return set_error(NXEC_ERR_NOMEM, "nxec request: out of memory");
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
  if (rc != NXEC_OK) restore_error(req->error);
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

int nxec_decode_frames(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                       const unsigned char *const *in_frames, unsigned char *const *out_frames, int64_t len,
                       int64_t nstripes, int64_t batch_stripes) {
  if (!ctx || !valid_nk(n, k) || nfailed < 0 || (nfailed > 0 && !failed) || len < 0 || nstripes < 0 ||
      (nstripes > 0 && (!in_frames || !out_frames)))
    return set_error(NXEC_ERR_INVALID, "nxec_decode_frames: invalid arguments");
  if (len == 0 || nstripes == 0) return NXEC_OK;
  std::vector<int32_t> inputs(n);
  int ni = 0, mi = 0;
  int rc = nxec_rs_plan(n, k, failed, nfailed, 0, inputs.data(), &ni, &mi, nullptr);  // rs.cc:252-265
  if (rc) return rc;
  for (int64_t s = 0; s < nstripes; s++) {
    for (int j = 0; j < k; j++)
      if (!in_frames[s * n + inputs[j]] || !out_frames[s * k + j])
        return set_error(NXEC_ERR_INVALID, "nxec_decode_frames: stripe %lld: null frame", static_cast<long long>(s));
  }
  if ((rc = ensure_device(ctx->device))) return rc;
  // staging rows: the k chosen inputs [B][k][stride], then all k data chunks [B][k][stride]
  // (erased data chunks get inverse rows, rs.cc:196,228-230; surviving ones
  // are unit rows, i.e. copies of their input)
  std::vector<int32_t> targets, src(k), copy(k, -1);
  for (int i = 0; i < nfailed; i++)
    if (failed[i] < k) targets.push_back(failed[i]);
  for (int j = 0; j < k; j++) {
    src[j] = j;
    if (inputs[j] < k) copy[j] = inputs[j];
  }
  std::vector<uint8_t> dm(std::max<size_t>(1, targets.size() * size_t(k)));
  if (!targets.empty() &&
      (rc = nxec_rs_decode_matrix(n, k, inputs.data(), targets.data(), static_cast<int>(targets.size()), dm.data())))
    return rc;
  const int64_t stride = (len + 15) / 16 * 16;
  int64_t B = batch_stripes > 0 ? batch_stripes : std::max<int64_t>(1, (int64_t(128) << 20) / (int64_t(k) * stride));
  B = std::min(B, nstripes);
  const int64_t nb = (nstripes + B - 1) / B;
  std::unique_lock<std::mutex> lk;
  ObjStage priv, *pstg = nullptr;
  if ((rc = batch_stage(ctx, size_t(B) * 2 * k * stride, lk, priv, &pstg))) return rc;
  ObjStage &stg = *pstg;
  // batch b lives in staging slot b % kObjSlots; one stream per stage, none
  // of them the context's own (the gather's per-piece syncs on a
  // borrowed context stream waited for other callers' work)
  if (stg.borrowed0 && !stg.aux &&
      (rc = hip_check(hipStreamCreateWithFlags(&stg.aux, hipStreamNonBlocking), "decode_frames gather stream"))) {
    if (!lk.owns_lock()) priv.release();
    return rc;
  }
  hipStream_t s_gather = stg.borrowed0 ? stg.aux : stg.streams[0], s_decode = stg.streams[1],
              s_scatter = stg.streams[2];
  std::mutex mu;
  std::condition_variable cv;
  int64_t gathered = 0, decoded = 0, scattered = 0;  // batches done per stage
  int err = NXEC_OK;
  std::string err_msg;
  auto fail = [&](int code) {  // the first error wins; every stage stops
    std::lock_guard<std::mutex> g(mu);
    if (!err) {
      err = code;
      err_msg = last_error();
    }
    cv.notify_all();
  };
  auto wait_for = [&](const int64_t &counter, int64_t want) {
    std::unique_lock<std::mutex> g(mu);
    cv.wait(g, [&] { return err != NXEC_OK || counter >= want; });
    return err == NXEC_OK;
  };
  auto done = [&](int64_t &counter) {
    std::lock_guard<std::mutex> g(mu);
    counter++;
    cv.notify_all();
  };
  auto in_rows = [&](int64_t b) { return stg.d + (b % kObjSlots) * stg.cap; };
  auto out_rows = [&](int64_t b) { return in_rows(b) + size_t(B) * k * stride; };
  auto run_stage = [&](auto &&body) {
    return std::thread([&, body]() mutable {
      try {
        body();
      } catch (const std::exception &e) {
        fail(set_error(NXEC_ERR_NOMEM, "nxec_decode_frames: %s", e.what()));
      }
    });
  };
  // one gather / scatter call per batch: row (i, j) of a batch is chunk i * k + j at `stride`
  std::thread gatherer, scatterer;
  try {  // a stage that cannot start fails the call; the other one sees the error and stops
  gatherer = run_stage([&]() {
    std::vector<const unsigned char *> fr(static_cast<size_t>(B * k));
    for (int64_t b = 0; b < nb; b++) {
      if (b >= kObjSlots && !wait_for(scattered, b - kObjSlots + 1)) return;  // the slot's previous batch has left
      const int64_t s0 = b * B, m = std::min(B, nstripes - s0);
      for (int64_t i = 0; i < m; i++)
        for (int j = 0; j < k; j++) fr[size_t(i * k + j)] = in_frames[(s0 + i) * n + inputs[j]];
      if (int r = nxec_gather_chunks(ctx, fr.data(), m * k, len, in_rows(b), stride, s_gather)) return fail(r);
      done(gathered);
    }
  });
  scatterer = run_stage([&]() {
    for (int64_t b = 0; b < nb; b++) {
      if (!wait_for(decoded, b + 1)) return;
      const int64_t s0 = b * B, m = std::min(B, nstripes - s0);
      if (int r = nxec_scatter_chunks(ctx, out_rows(b), stride, m * k, len, out_frames + s0 * k, s_scatter))
        return fail(r);
      done(scattered);
    }
  });
  } catch (const std::exception &e) {
    fail(set_error(NXEC_ERR_NOMEM, "nxec_decode_frames: %s", e.what()));
  }
  for (int64_t b = 0; b < nb; b++) {  // decode on the calling thread
    if (!wait_for(gathered, b + 1)) break;
    const int64_t m = std::min(B, nstripes - b * B);
    int r = stripes_mul_impl(ctx, static_cast<int>(targets.size()), k, dm.data(), in_rows(b), nullptr, src.data(), stride,
                             int64_t(k) * stride, out_rows(b), nullptr, targets.data(), stride, int64_t(k) * stride,
                             copy.data(), len, m, s_decode);
    if (!r) r = hip_check(hipStreamSynchronize(s_decode), "decode_frames sync");
    if (r) {
      fail(r);
      break;
    }
    done(decoded);
  }
  if (gatherer.joinable()) gatherer.join();
  if (scatterer.joinable()) scatterer.join();
  (void)hipStreamSynchronize(s_gather);
  for (int i = 1; i < kObjSlots; i++) (void)hipStreamSynchronize(stg.streams[i]);
  if (!lk.owns_lock()) priv.release();
  if (err) restore_error(err_msg);
  return err;
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
