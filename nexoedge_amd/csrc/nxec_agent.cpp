// The agent coding service (include/nxec.h §6): the agent's ENC_CHUNK_REQ /
// RPR_CHUNK_REQ computations (CodingUtils::encode + Chunk::computeMD5 of the
// outputs, container_manager.cc:221-258, agent.cc:240-415) batched over many
// requests and concurrent callers, from and into host buffers.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "nxec_runtime.h"

using namespace nxec;

struct AgentJob {
  const nxec_agent_req *reqs;
  int nreqs;
  int64_t chunk_size, batch_bytes;
  int rc = NXEC_OK;
  bool done = false;
  std::string error;
};

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
  host_parallel_for(static_cast<int>(b.reqs.size()) * no, [&](int item) {  // scatter the outputs
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
  }, HostLane::kOut, ctx->numa_node);
  b.reqs.clear();
  return NXEC_OK;
}

}  // namespace

static bool agent_trace() { return tuning().agent_trace; }

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
  host_parallel_for(static_cast<int>(nid * (ni + no)), [&](int item) {
    const size_t q = static_cast<size_t>(item);
    if (q < nid * ni) {
      const unsigned char *p = reqs[ids[q / ni]].inputs[q % ni];
      in_dv[q] = aligned16(p) ? reinterpret_cast<uintptr_t>(host_device_view_range(p, cs)) : 0;
    } else {
      const size_t o = q - nid * ni;
      unsigned char *p = reqs[ids[o / no]].outputs[o % no];
      out_dv[o] = aligned16(p) ? reinterpret_cast<uintptr_t>(host_device_view_range(p, cs)) : 0;
    }
  }, HostLane::kIn, ctx->numa_node);
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
    host_parallel_for(static_cast<int>(nb * (ni + no)), [&](int item) {
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
    }, HostLane::kIn, ctx->numa_node);
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
  if (tuning().agent_batch_mb > 0) batch_bytes = int64_t(tuning().agent_batch_mb) << 20;
  // fused form (any chunk size): one k_gather_md5 launch per batch codes and hashes the
  // requests straight from and into pinned host memory (mapped caller
  // buffers, e.g. arena Chunks, are used in place; pageable ones go through
  // the slot); without zero copy (NXEC_HOST_DIRECT=0) H2D -> multiply -> MD5 -> D2H.
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
    if (tuning().agent_fused && host_direct_enabled() && ni <= kGatherMd5MaxK && no <= kMaxRowsPerPass) {
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
      host_parallel_for(static_cast<int>(nb) * ni, [&](int item) {  // gather into pinned staging
        const int64_t i = item / ni;
        const int j = item % ni;
        stage_copy(b.slot->h + (i * ni + j) * stride, reqs[ids[first + i]].inputs[j], chunk_size);
      }, HostLane::kIn, ctx->numa_node);
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
  if (!tuning().agent_aggregate) return agent_encode_impl(ctx, reqs, nreqs, chunk_size, batch_bytes);
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
      // fault injection (NXEC_TEST_FAULT=agent_round): the leader throws before
      // it runs; the round must still complete with an error, no waiter hangs
      if (test_fault("agent_round")) throw std::bad_alloc();
      rc = agent_encode_impl(ctx, merged.data(), static_cast<int>(merged.size()), cs0, bb);
      if (rc) err = last_error();
    } catch (const std::exception &e) {
      rc = set_error(NXEC_ERR_NOMEM, "nxec_agent_encode_batch: %s", e.what());
      err = last_error();
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
  if (job.rc != NXEC_OK) restore_error(job.error);
  return job.rc;
}
