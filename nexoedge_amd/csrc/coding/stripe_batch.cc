// See stripe_batch.hh.  Reference behaviour per call site is cited inline.
#include "stripe_batch.hh"

#include <cstdio>
#include <cstring>

#include "rs.hh"

StripeBatch::StripeBatch(Coding *code, int device) : _code(code) {
  if (!dynamic_cast<RSCode *>(code) || nxec_ctx_create(device, &_ctx) != NXEC_OK) _ctx = nullptr;
}

StripeBatch::~StripeBatch() {
  if (_ctx) nxec_ctx_destroy(_ctx);
  for (unsigned char *p : {_parity, _md5, _tail})
    if (p) nxec_host_free_pinned(p);
  for (unsigned char *p : {_dChunks, _dObject, _dTail})
    if (p) nxec_dev_free(p);
}

bool StripeBatch::growHost(unsigned char **p, size_t *cap, size_t bytes) {
  if (*cap >= bytes && *p) return true;
  if (*p) nxec_host_free_pinned(*p);
  *p = nullptr;
  *cap = 0;
  void *q = nullptr;
  if (nxec_host_malloc_pinned(&q, bytes ? bytes : 1) != NXEC_OK) return false;
  *p = static_cast<unsigned char *>(q);
  *cap = bytes;
  return true;
}

bool StripeBatch::growDevice(unsigned char **p, size_t *cap, size_t bytes) {
  if (*cap >= bytes && *p) return true;
  if (*p) nxec_dev_free(*p);
  *p = nullptr;
  *cap = 0;
  void *q = nullptr;
  if (nxec_dev_malloc(&q, bytes ? bytes : 1) != NXEC_OK) return false;
  *p = static_cast<unsigned char *>(q);
  *cap = bytes;
  return true;
}

uint64_t StripeBatch::numStripes(uint64_t length, length_t maxChunkSize) const {
  int64_t ns = 0, nf = 0, cl = 0;
  if (nxec_object_layout(_code->getN(), _code->getK(), static_cast<int64_t>(length), maxChunkSize, &ns, &nf, &cl))
    return 0;
  return static_cast<uint64_t>(ns);
}

bool StripeBatch::encodeFile(const data_t *data, uint64_t length, length_t maxChunkSize, std::vector<Chunk> &chunks,
                             int chunkIdOffset, bool computeMD5) {
  chunks.clear();
  if (!_ctx || (length > 0 && !data)) return false;
  const int n = _code->getN(), k = _code->getK(), p = n - k;
  const int64_t M = maxChunkSize;
  int64_t ns = 0, nf = 0, cl = 0;
  if (nxec_object_layout(n, k, static_cast<int64_t>(length), M, &ns, &nf, &cl) != NXEC_OK) return false;
  if (ns == 0) return true;
  if (!growHost(&_parity, &_parityCap, static_cast<size_t>(ns) * (p > 0 ? p : 1) * M) ||
      (computeMD5 && !growHost(&_md5, &_md5Cap, static_cast<size_t>(ns) * n * 16)))
    return false;
  // writeFileStripe's encode + MD5 of every chunk (chunk_manager.cc:99,175), all stripes at once
  if (nxec_encode_object_host(_ctx, n, k, data, static_cast<int64_t>(length), M, _parity, computeMD5 ? _md5 : nullptr,
                              0) != NXEC_OK) {
    std::fprintf(stderr, "StripeBatch::encodeFile: %s\n", nxec_last_error());
    return false;
  }
  // the last stripe's data chunks, zero-padded (chunk_manager.cc:390-399)
  const bool tail = ns > nf;
  if (tail) {
    const size_t rem = static_cast<size_t>(length - static_cast<uint64_t>(nf) * k * M);
    if (!growHost(&_tail, &_tailCap, static_cast<size_t>(k) * cl)) return false;
    std::memcpy(_tail, data + static_cast<size_t>(nf) * k * M, rem);
    std::memset(_tail + rem, 0, static_cast<size_t>(k) * cl - rem);
  }
  chunks.resize(static_cast<size_t>(ns) * n);
  for (int64_t s = 0; s < ns; s++) {
    const bool last = s >= nf;
    const int64_t cs = last ? cl : M;
    for (int i = 0; i < n; i++) {
      Chunk &c = chunks[static_cast<size_t>(s) * n + i];
      // ids as encodeFile assigns them (chunk_manager.cc:442-446)
      c.setChunkId(chunkIdOffset + static_cast<int>(s) * n + i);
      unsigned char *d;
      if (i < k)
        d = last ? _tail + static_cast<size_t>(i) * cl : const_cast<unsigned char *>(data) + (s * k + i) * M;
      else
        d = _parity + (s * p + (i - k)) * M;
      c.data = d;
      c.size = static_cast<int>(cs);
      c.freeData = false;  // views into the file buffer / this batch
      if (computeMD5) {  // chunk_manager.cc:175's computeMD5 then returns the GPU digest
        std::memcpy(c.md5, _md5 + (s * n + i) * 16, 16);
        c.setDigestValid();
      }
    }
  }
  return true;
}

bool StripeBatch::decodeFile(std::vector<Chunk> &inputs, uint64_t length, length_t maxChunkSize,
                             const std::vector<chunk_id_t> &failed, data_t *out) {
  if (!_ctx || (length > 0 && !out)) return false;
  const int n = _code->getN(), k = _code->getK();
  const int64_t M = maxChunkSize;
  int64_t ns = 0, nf = 0, cl = 0;
  if (nxec_object_layout(n, k, static_cast<int64_t>(length), M, &ns, &nf, &cl) != NXEC_OK) return false;
  if (ns == 0) return true;
  if (inputs.size() != static_cast<size_t>(ns) * k) return false;
  // the plan every stripe shares: its input ids are the first k alive (rs.cc:252-265)
  std::vector<int32_t> f(failed.begin(), failed.end()), ids(n);
  int ni = 0, mi = 0;
  if (nxec_rs_plan(n, k, f.data(), static_cast<int>(f.size()), 0, ids.data(), &ni, &mi, nullptr) != NXEC_OK)
    return false;
  for (int64_t s = 0; s < ns; s++)
    for (int j = 0; j < k; j++) {
      const Chunk &c = inputs[static_cast<size_t>(s) * k + j];
      const int64_t want = s < nf ? M : cl;
      if (c.chunkId % n != ids[j] || c.size != want || !c.data) return false;  // decodeFile's id use, :775
    }
  // the staged stripes sit at the library's recover-heavy strides
  // (nxec_batch_layout): a degraded read's survivors are read with holes
  // ({1,4,11,13} lost), which the packed [s][n][M] layout serves at ~0.71 of
  // 8 TB/s and the padded stripe stride at ~0.78
  int64_t cst = M, sst = int64_t(n) * M;
  if (nxec_batch_layout(n, M, NXEC_LAYOUT_RECOVER_HEAVY, &cst, &sst) != NXEC_OK) return false;
  if (!growDevice(&_dChunks, &_dChunksCap, static_cast<size_t>(ns) * sst) ||
      !growDevice(&_dObject, &_dObjectCap, static_cast<size_t>(length)) ||
      !growDevice(&_dTail, &_dTailCap, static_cast<size_t>(k) * M))
    return false;
  void *st = nxec_ctx_stream(_ctx);
  // fetched chunks -> HBM, one gather per (chunk id, stripe kind)
  std::vector<const unsigned char *> frames;
  for (int j = 0; j < k; j++) {
    frames.clear();
    for (int64_t s = 0; s < nf; s++) frames.push_back(inputs[static_cast<size_t>(s) * k + j].data);
    if (nf > 0 && nxec_gather_chunks(_ctx, frames.data(), nf, M, _dChunks + ids[j] * cst, sst, st) != NXEC_OK)
      return false;
    if (ns > nf) {
      const unsigned char *fr = inputs[static_cast<size_t>(nf) * k + j].data;
      if (nxec_gather_chunks(_ctx, &fr, 1, cl, _dChunks + nf * sst + ids[j] * cst, M, st) != NXEC_OK) return false;
    }
  }
  // decodeFile for every stripe (chunk_manager.cc:738-800), straight into the object
  if (nxec_decode_object_ex(_ctx, n, k, f.data(), static_cast<int>(f.size()), _dChunks, cst, sst,
                            static_cast<int64_t>(length), M, _dObject, _dTail, st) != NXEC_OK)
    return false;
  if (nxec_memcpy_d2h(out, _dObject, static_cast<size_t>(length), st) != NXEC_OK) return false;
  return nxec_stream_sync(st) == NXEC_OK;
}
