// Whole objects and batches of files (include/nxec.h §5): writeFileStripe's
// coding + digests and decodeFile over every stripe of an object
// (chunk_manager.cc:66-452, 738-800, 1548-1556), the per-file loop of
// Proxy::writeFileStripes as one launch (proxy_file_ops.cc:557-666), and the
// object layouts they follow (rs.cc:52-55, chunk_manager.cc:390-399).
#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

#include "nxec_runtime.h"

using namespace nxec;

extern "C" {

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
  // the gather kernel reads and writes 16-byte vectors: chunk size, objects and parity slots aligned
  bool full_aligned = M % 16 == 0 && (reinterpret_cast<uintptr_t>(d_parity) & 15) == 0;
  // ragged stripes through the aligned work-queue kernel: parity slots must be
  // 16-byte aligned (else they join the byte-capable list kernel)
  const bool ragged_ok = p > 0 && M % 16 == 0 && (reinterpret_cast<uintptr_t>(d_parity) & 15) == 0 && k <= kMaxRaggedK;
  // one launch for every stripe's coding and every chunk's MD5 (k_files_md5):
  // full stripes and every last stripe as in-place requests (below); otherwise
  // the separate launches (pad copy, gather / ragged / list coding, MD5 list)
  const bool want_fused = tuning().fused_md5 && d_md5 && ragged_ok && p <= kMaxRowsPerPass && k <= kFilesMd5MaxK;
  std::vector<const uint8_t *> q_src;
  std::vector<uint8_t *> q_dst, q_dig;
  std::vector<int64_t> q_len;
  std::vector<uint64_t> q_slot, q_geom;  // per request: tail slot of chunk 0, cls | vm << 32
  std::vector<uint32_t> q_mask;          // per request: jm | j0 << 8 | mode << 16
  // full stripes are read in place: 16-byte aligned objects (any object whose
  // only stripe is its last one is read byte-wise, or padded, either way)
  for (int o = 0; o < nobjects && full_aligned; o++)
    full_aligned = (reinterpret_cast<uintptr_t>(d_objects[o]) & 15) == 0 || lengths[o] < int64_t(k) * M;
  // the fused launch plans only its own tables; the separate launches only theirs
  const bool fused = want_fused && full_aligned;
  const bool sep = !fused;
  // Without NXEC_OBJECTS_TAIL_INPLACE (whole tail arena) the kernel also
  // stores the data chunks of last stripes that it reads in place to their
  // tail-arena slots (tail_store)
  const bool tstore = fused && !(flags & NXEC_OBJECTS_TAIL_INPLACE);
  // chunks of a last stripe past the object's data read the context's zero line
  const uint8_t *zl = nullptr;
  if (fused && tail_total > 0 && (rc = zero_line(ctx, size_t(M) + 256, &zl))) return rc;
  // testing (NXEC_TEST_FAULT=zero_stall): hold the line between planning and
  // launch, while another caller grows the context's line
  if (zl && test_fault("zero_stall")) std::this_thread::sleep_for(std::chrono::milliseconds(400));
  bool any_mask = false;
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
          q_slot.push_back(0);
          q_geom.push_back(0);
          q_mask.push_back(uint32_t(k) | uint32_t(k) << 8);
        }
        if (sep && dig) {
          for (int j = 0; j < k; j++) items.push_back({obj + (s * k + j) * M, M, dig + j * 16});
          for (int i = 0; i < p; i++) items.push_back({par + i * M, M, dig + (k + i) * 16});
        }
      } else {  // last stripe (chunk_manager.cc:390-399)
        const int64_t cls = (cl + 15) / 16 * 16;
        uint8_t *td = d_tail + toff;
        if (sep) {
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
        if (fused) {
          // In place: the last stripe is an ordinary request.  Data chunk j
          // is the object's bytes [j*cl, (j+1)*cl) past its full stripes, zero
          // padded (chunk_manager.cc:390-399): the chunks wholly in the object
          // are read where they lie, the one holding its last vm < cl bytes is
          // the request's masked chunk (read in place up to vm, zero padded
          // by the kernel), the chunks past the data read the zero line.  A
          // whole chunk's last 16-byte vector may run up to 15 bytes past the
          // chunk (into the next one, or past the object's last byte but not
          // out of that byte's 4 KiB page: never into memory the object does
          // not touch).  Where it would leave the page (a chunk length that
          // is not a multiple of 16, the object ending within 16 bytes of a
          // page boundary) the chunks from that one on are first written zero
          // padded to their slots by one small copy launch and read from there.
          const uint8_t *tb = obj + nf * k * M;
          const int64_t rem = lengths[o] - nf * k * M;
          const int64_t jf = std::min<int64_t>(rem / cl, k), vm = jf < k ? rem - jf * cl : 0;
          const uintptr_t end = reinterpret_cast<uintptr_t>(tb) + uintptr_t(rem);
          const int64_t pend = static_cast<int64_t>(((end + 4095) & ~uintptr_t(4095)) - reinterpret_cast<uintptr_t>(tb));
          const int64_t jov = pend >= cls ? (pend - cls) / cl + 1 : 0;  // first chunk that would leave the page
          int64_t j0 = k, jm = k;
          if (jov < jf || !tuning().files_fold) {
            // (the fold probe off: round 4's in-place rule, the chunks from the partial one -- or
            // the first that would read past the object's last 16-byte line -- through the pad copy)
            const int64_t line = static_cast<int64_t>(((end + 15) & ~uintptr_t(15)) - reinterpret_cast<uintptr_t>(tb));
            j0 = tuning().files_fold ? jov : std::min(jf, line >= cls ? (line - cls) / cl + 1 : 0);
            for (int j = 0; j < k; j++) q_src.push_back(j < j0 ? tb + j * cl : td + j * cls);
            pads.push_back({tb + j0 * cl, td + j0 * cls, rem - j0 * cl, cl, cls, k - j0});
            pad_bstart.push_back(static_cast<uint32_t>(pad_blocks));
            pad_blocks += (cls / 16 * (k - j0) + 256 * kPadVecs - 1) / (256 * kPadVecs);
          } else {
            if (vm > 0) jm = jf;
            for (int j = 0; j < k; j++) q_src.push_back(j < jf || j == jm ? tb + j * cl : zl);
            any_mask |= jm < k;
          }
          for (int i = 0; i < p; i++) q_dst.push_back(par + i * M);
          q_len.push_back(cl);
          q_dig.push_back(dig);
          // the whole tail arena: the kernel stores chunks j < j0 to their
          // slots; NXEC_OBJECTS_TAIL_INPLACE: only the masked (partial) chunk
          const uint32_t mode = !tstore && jm < k ? 1u : 0u;
          q_slot.push_back(tstore || mode ? reinterpret_cast<uint64_t>(td) : 0);
          q_geom.push_back(uint64_t(cls) | uint64_t(vm) << 32);
          q_mask.push_back(uint32_t(jm) | uint32_t(j0) << 8 | mode << 16);
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
  std::vector<const uint8_t *> f_src;
  std::vector<uint8_t *> f_dst, f_dig;
  std::vector<int64_t> f_len;
  std::vector<uint64_t> f_slot, f_geom;
  std::vector<uint32_t> f_mask;
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
      f_slot.push_back(q_slot[o]);
      f_geom.push_back(q_geom[o]);
      f_mask.push_back(q_mask[o]);
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
                      {f_slot.data(), f_slot.size() * sizeof(uint64_t)},
                      {f_geom.data(), f_geom.size() * sizeof(uint64_t)},
                      {f_mask.data(), f_mask.size() * sizeof(uint32_t)},
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
  rc = acquire_slot(ctx, std::max<size_t>(off[kTabs], 16), &slot, async);
  if (rc) return rc;
  // the slot's staging may still be in use by an earlier call on its own stream
  rc = hip_check(hipStreamSynchronize(slot->stream), "slot sync");
  if (!rc && async && !slot->busy) rc = hip_check(hipEventCreateWithFlags(&slot->busy, hipEventDisableTiming), "slot event");
  for (int i = 0; i < kTabs && !rc; i++)
    if (tabs[i].bytes) std::memcpy(slot->h + off[i], tabs[i].h, tabs[i].bytes);
  if (!rc) rc = hip_check(hipMemcpyAsync(slot->d, slot->h, off[kTabs], hipMemcpyHostToDevice, st), "tables H2D");
  const int T0 = 11;  // the first eleven tables belong to the fused launch
  auto dptr = [&](int i) { return slot->d + off[i + T0]; };
  if (fused) {
    // the rare last stripes whose chunks could not all be read in place
    if (!rc && !pads.empty())
      rc = launch_pad_chunks(reinterpret_cast<const PadChunks *>(dptr(2)), reinterpret_cast<const uint32_t *>(dptr(3)),
                             int64_t(pads.size()), pad_blocks, st);
    // last-stripe tables only when some request stores to the tail arena or masks a chunk
    const bool any_store = std::any_of(f_slot.begin(), f_slot.end(), [](uint64_t t) { return t != 0; });
    fa.tail_store = tstore && any_store ? 1 : 0;
    fa.mask = any_mask ? 1 : 0;
    if (fa.tail_store || fa.mask) {
      fa.last_slot = reinterpret_cast<const uint64_t *>(slot->d + off[8]);
      fa.last_geom = reinterpret_cast<const uint64_t *>(slot->d + off[9]);
      fa.last_mask = reinterpret_cast<const uint32_t *>(slot->d + off[10]);
      fa.zero = zl;
    }
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
    std::memcpy(fa.coef, prow, size_t(p) * k);
    if (!rc) {
      hipEvent_t kt[2];
      kt_begin(ctx, st, kt);
      rc = launch_files_md5(fa, ctx->num_cus, st);
      kt_end(ctx, kt, st);
    }
    if (async) {  // the tables stay in the slot until the stream gets past the launches
      if (!rc) rc = hip_check(hipEventRecord(slot->busy, st), "slot event record");
      slot->busy_set = !rc;
      if (rc) (void)hipStreamSynchronize(st);
      release_slot(ctx, slot);
      return rc;
    }
    const int rc2 = hip_check(hipStreamSynchronize(st), "nxec_encode_objects sync");
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

}  // extern "C"
