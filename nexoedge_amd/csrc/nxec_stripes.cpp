// Device-resident stripe batches (include/nxec.h §3-§4): the GF(2^8)
// stripe multiply that every coding call reduces to, RSCode::encode /
// preDecode + decode / carRepairFinalize over a batch (rs.cc:57-322), the
// per-chunk MD5 launches, the fused encode + MD5 and recover + MD5 kernels,
// and the recommended batch layout.
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "nxec_runtime.h"

namespace nxec {

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

}  // namespace nxec

using namespace nxec;

extern "C" {

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

namespace nxec {

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

}  // namespace nxec

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
  // break the power-of-two chunk stride (profiles/r02_layout_sweep.log; the
  // pad per size class from r05_layout_big_pads.log, r05_config5_small_pads.log:
  // 4 MiB multiples 3 KiB, e.g. RS(16,4) 4 MiB 0.754 -> 0.772, RS(12,4)
  // 0.756 -> 0.781; 2 MiB 5 KiB; other sizes from 2 MiB 2 KiB)
  if (len >= 2 * kMiB) cs += len % (4 * kMiB) == 0 ? 3072 : len == 2 * kMiB ? 5120 : 2048;
  // smaller chunks: no rule carries across geometries, so only the shapes
  // measured (mean of encode and the contiguous / scattered recovers,
  // profiles/r05_config5_small_pads.log, r05_layout_small_chunk_pads.log)
  struct Measured {
    int n;
    int64_t len, pad;
  };
  static constexpr Measured kMeasured[] = {
      {20, 256 << 10, 4096},   // RS(16,4) 256 KiB: 0.755 -> 0.766
      {14, 128 << 10, 10240},  // RS(10,4) 128 KiB: 0.68 -> 0.78
      {14, 256 << 10, 12288},  // RS(10,4) 256 KiB: 0.71 -> 0.745
  };
  for (const Measured &m : kMeasured)
    if (n == m.n && len == m.len) cs += m.pad;
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

namespace {
std::mutex g_tuned_mu;
// (device, n, k, len, flags, budget_bytes): a later caller asking for a
// measurement at another budget gets its own (small scratch batches can rank
// the candidates differently from full-size ones)
std::map<std::tuple<int, int, int, int64_t, int, int64_t>, std::pair<int64_t, int64_t>> g_tuned;
}  // namespace

int nxec_layout_choose(int ncand, int rounds, const double *scores, double min_margin) {
  if (ncand < 1 || rounds < 1 || !scores || min_margin < 0)
    return set_error(NXEC_ERR_INVALID, "nxec_layout_choose: invalid arguments");
  auto at = [&](int r, int c) { return scores[static_cast<size_t>(r) * ncand + c]; };
  // relative spread of a candidate's scores across the rounds (-1: not measured in some round)
  auto spread = [&](int c, double *mean) {
    double lo = at(0, c), hi = lo, sum = 0;
    for (int r = 0; r < rounds; r++) {
      const double v = at(r, c);
      if (!(v > 0)) return -1.0;
      lo = std::min(lo, v);
      hi = std::max(hi, v);
      sum += v;
    }
    *mean = sum / rounds;
    return (hi - lo) / *mean;
  };
  double inc_mean = 0;
  const double inc_spread = spread(0, &inc_mean);
  if (inc_spread < 0) return 0;  // the incumbent unmeasured: keep it
  int best = 0;
  double best_mean = inc_mean;
  for (int c = 1; c < ncand; c++) {
    double mean = 0;
    const double sp = spread(c, &mean);
    if (sp < 0) continue;
    const double margin = std::max({min_margin, sp, inc_spread});
    bool wins = true;
    for (int r = 0; r < rounds && wins; r++) wins = at(r, c) > at(r, 0) * (1.0 + margin);
    if (wins && mean > best_mean) {
      best = c;
      best_mean = mean;
    }
  }
  return best;
}

int nxec_batch_layout_tuned(nxec_ctx_t *ctx, int n, int k, int64_t len, int flags, int64_t budget_bytes,
                            int64_t *chunk_stride, int64_t *stripe_stride) {
  if (!ctx || !valid_nk(n, k) || n == k || len <= 0 || !chunk_stride || !stripe_stride)
    return set_error(NXEC_ERR_INVALID, "nxec_batch_layout_tuned: invalid arguments");
  const auto key = std::make_tuple(ctx->device, n, k, len, flags, budget_bytes);
  {
    std::lock_guard<std::mutex> lk(g_tuned_mu);
    auto it = g_tuned.find(key);
    if (it != g_tuned.end()) {
      *chunk_stride = it->second.first;
      *stripe_stride = it->second.second;
      return NXEC_OK;
    }
  }
  int rc = ensure_device(ctx->device);
  if (rc) return rc;
  int64_t c0 = 0, s0 = 0;
  if ((rc = nxec_batch_layout(n, len, flags, &c0, &s0))) return rc;
  const int64_t packed = (len + 15) / 16 * 16;
  std::vector<std::pair<int64_t, int64_t>> cand = {{c0, s0}, {packed, n * packed}};
  // chunk pads: the 2-5 KiB class of the table, and the larger ones small
  // chunks want ((14,10) 128 KiB: 0.68 packed, 0.78 with 10 KiB;
  // profiles/r05_layout_small_chunk_pads.log)
  for (int64_t pad : {1536, 2048, 3072, 4096, 5120, 8192, 10240, 12288, 16384})
    cand.emplace_back(packed + pad, n * (packed + pad));
  cand.emplace_back(packed, (n + 1) * packed);  // an odd stripe stride in chunks
  std::sort(cand.begin() + 1, cand.end());
  cand.erase(std::unique(cand.begin() + 1, cand.end()), cand.end());
  cand.erase(std::remove(cand.begin() + 1, cand.end(), cand[0]), cand.end());
  size_t free_b = 0, total_b = 0;
  NXEC_HIP(hipMemGetInfo(&free_b, &total_b));
  int64_t budget = budget_bytes > 0 ? budget_bytes : int64_t(24) << 30;
  budget = std::min<int64_t>(budget, static_cast<int64_t>(free_b / 4));
  int64_t max_ss = 0;
  for (const auto &c : cand) max_ss = std::max(max_ss, c.second);
  if (budget < max_ss) budget = max_ss;
  uint8_t *d = nullptr;
  NXEC_HIP(hipMalloc(reinterpret_cast<void **>(&d), static_cast<size_t>(budget)));
  hipStream_t st = ctx->stream;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  rc = hip_check(hipEventCreate(&e0), "hipEventCreate");
  if (!rc) rc = hip_check(hipEventCreate(&e1), "hipEventCreate");
  if (!rc) rc = launch_fill(d, static_cast<size_t>(budget), 0x7A11ull, st);
  // the recovers scored beside the encode: the first min(n - k, 4) chunks,
  // and a scattered set (the slow patterns of DESIGN.md §3): the first
  // min(n - k, 4) of chunks 1, 4, n - 3, n - 1 (the bench's {1,4,11,13} for RS(10,4))
  std::vector<int32_t> first, scattered;
  for (int32_t c = 0; c < std::min(n - k, 4); c++) first.push_back(c);
  for (int32_t c : {1, 4, n - 3, n - 1})
    if (static_cast<int>(scattered.size()) < std::min(n - k, 4) && c >= 0 && c < n &&
        std::find(scattered.begin(), scattered.end(), c) == scattered.end())
      scattered.push_back(c);
  std::sort(scattered.begin(), scattered.end());
  // every candidate scored in kRounds interleaved rounds (the device's state
  // drifts less between candidates than between calls)
  constexpr int kRounds = 3;
  const int nc = static_cast<int>(cand.size());
  std::vector<double> score(static_cast<size_t>(kRounds) * nc, 0.0);
  for (int round = 0; round < kRounds && !rc; round++) {
    for (size_t ci = 0; ci < cand.size() && !rc; ci++) {
      const auto &c = cand[ci];
      const int64_t ns = budget / c.second;
      if (ns < 1) continue;
      // bytes per ms of one op (encode: (k + p) * len per stripe; recover: (k + e) * len)
      auto rate_of = [&](const std::vector<int32_t> *erased, double *out) {
        auto op = [&]() {
          return erased ? nxec_rs_recover_stripes(ctx, n, k, erased->data(), static_cast<int>(erased->size()), d,
                                                  c.first, c.second, len, ns, st)
                        : nxec_rs_encode_stripes(ctx, n, k, d, c.first, c.second, len, ns, st);
        };
        int r = op();  // warm
        if (!r) r = hip_check(hipEventRecord(e0, st), "hipEventRecord");
        for (int i = 0; i < 4 && !r; i++) r = op();
        if (!r) r = hip_check(hipEventRecord(e1, st), "hipEventRecord");
        float t = 0;
        if (!r) r = hip_check(hipEventSynchronize(e1), "hipEventSynchronize");
        if (!r) r = hip_check(hipEventElapsedTime(&t, e0, e1), "hipEventElapsedTime");
        *out = double(ns) * (k + (erased ? double(erased->size()) : double(n - k))) * len / (t / 4);
        return r;
      };
      // the score: encode, a contiguous and a scattered recover, equally weighted
      // (RECOVER_HEAVY: the scattered one twice)
      double r_enc = 0, r_first = 0, r_scat = 0;
      if ((rc = rate_of(nullptr, &r_enc)) || (rc = rate_of(&first, &r_first)) || (rc = rate_of(&scattered, &r_scat)))
        break;
      const double w = (flags & NXEC_LAYOUT_RECOVER_HEAVY) ? 2.0 : 1.0;
      score[static_cast<size_t>(round) * nc + ci] = (r_enc + r_first + w * r_scat) / (2.0 + w);
    }
  }
  // the table's layout (the incumbent, candidate 0) stays unless another
  // beats it in every round by more than the rounds' own spread (and 0.5 %)
  const std::pair<int64_t, int64_t> pick = rc ? cand[0] : cand[nxec_layout_choose(nc, kRounds, score.data(), 0.005)];
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipStreamSynchronize(st);
  (void)hipFree(d);
  if (rc) return rc;
  {
    std::lock_guard<std::mutex> lk(g_tuned_mu);
    g_tuned[key] = pick;
  }
  *chunk_stride = pick.first;
  *stripe_stride = pick.second;
  return NXEC_OK;
}

}  // extern "C"
