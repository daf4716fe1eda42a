// The per-stripe drop-in (include/nxec.h §1-§2): ISA-L's ec_encode_data
// with its exact signature (erasure_code.h:98) and the host-buffer encode
// behind CodingUtils::encode, RSCode::encode / decode and carRepairFinalize
// (coding_util.hh:12-31, rs.cc:57-236), with and without the digests the
// write path computes next (chunk_manager.cc:175).
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "nxec_runtime.h"

using namespace nxec;

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
    host_parallel_for(
        rows, [&](int r) {
          if (!out_mapped[r]) std::memcpy(coding[r], slot->h + chunk_off(k + r), size_t(len));
        },
        HostLane::kOut, ctx->numa_node);
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
  DefaultLease lease;
  int rc = default_ctx(lease);
  if (rc) return rc;
  nxec_ctx_t *ctx = lease.ctx;
  // calls in flight on this call's device (its PCIe link): few take the
  // pipelined zero-copy form, many the per-piece DMA form
  const int inflight = lease.device_inflight;
  // chunk buffers that are already pinned (the chunk arena, registered
  // receive pools): straight to the GPU, no staging memcpy
  if (ncopy == 0) {
    rc = encode_host_pinned(ctx, len, k, rows, coeffs, data, coding, inflight);
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
  const int64_t piece = (len >= 2 * kHostPiece && inflight <= 2) ? kHostPiece : stride;
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
  // Few callers: zero copy, the kernel works on the pinned staging itself over
  // PCIe (no copy-engine round trip: 1 caller 25.8 -> 33.6 GiB/s).  Many
  // callers: H2D -> kernel -> D2H per piece, whose copy engines share the link
  // better (4 callers 69.8 vs 52.0 GiB/s zero copy; profiles/r01_dropin*.jsonl).
  uint8_t *hv = inflight <= 2 ? static_cast<uint8_t *>(host_device_view(slot->h)) : nullptr;
  for (int pc = 0; pc < npieces && rc == NXEC_OK; pc++) {
    const int64_t off = pc * piece, pl = std::min<int64_t>(piece, len - off);
    host_parallel_for(
        k, [&](int j) { stage_copy(slot->h + j * stride + off, data[j] + off, static_cast<size_t>(pl)); }, HostLane::kIn,
        ctx->numa_node);
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
      host_parallel_for(nout, [&](int o) {
        unsigned char *to = nullptr;
        if (o < rows) {
          to = coding[o];
        } else {
          for (int j = 0; j < k; j++)
            if (copy_idx && copy_idx[j] == o - rows) to = copy_out[o - rows];
        }
        if (to) std::memcpy(to + off, slot->h + (k + o) * stride + off, static_cast<size_t>(pl));
      }, HostLane::kOut, ctx->numa_node);
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

// zero-copy digest rounds in flight (4; the rounds probe can change or disable them)
int digest_rounds_max() { return std::max(1, tuning().digest_rounds); }

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
// lane, whatever the round's size) run -- up to 4 rounds
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
  // admitted only for the staged form below: a zero-copy call waits for a
  // shared digest round (one launch for every pending call, ~10 ms per MiB of
  // chain) and holds no staging of its own, so gating it would only shrink
  // the rounds
  DefaultLease lease;
  if ((rc = default_ctx(lease, false))) return rc;
  nxec_ctx_t *ctx = lease.ctx;
  DigestJob job;
  job.len = len;
  job.k = k;
  job.rows = rows;
  job.coeffs = coeffs;
  job.md5_data = md5_data;
  job.md5_code = md5_code;
  bool mapped = tuning().digest_rounds != 0 && k <= kGatherMd5MaxK && rows <= kMaxRowsPerPass;
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
    lease_admit(lease);
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
    if (rrc) err = last_error();
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
  if (job.rc != NXEC_OK) restore_error(job.error);
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


}  // namespace

extern "C" {

// ISA-L's ec_encode_data has no error channel (erasure_code.h:98, rs.cc:89),
// so a failed device pass is retried once on a fresh context through the
// staged path (a transient error -- a busy queue, a lost stream -- does not
// take the proxy and its background repair thread down); only when that fails
// too does the process stop rather than return undefined parity.
void nxec_ec_encode_data(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                         unsigned char **coding) {
  // fault injection (NXEC_TEST_FAULT=encode): the first attempt fails as a device error would
  int rc = test_fault("encode") ? set_error(NXEC_ERR_HIP, "injected device error (NXEC_TEST_FAULT=encode)")
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

}  // extern "C"
