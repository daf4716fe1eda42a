// Batched ChunkManager entry.
//
// The reference writes a file one stripe at a time: Proxy::writeFileStripes
// (proxy_file_ops.cc:557-666) calls ChunkManager::writeFileStripe
// (chunk_manager.cc:66-367) per stripe, which runs encodeFile (:369-452 ->
// RSCode::encode, rs.cc:57-92) and the MD5 of every chunk (:175,
// Chunk::computeMD5).  Reads mirror it: readFile (:639-736) -> decodeFile
// (:738-800 -> RSCode::decode) per stripe.  StripeBatch does a whole file --
// every stripe -- per call on the GPU:
//
//  * encodeFile: the stripe split of proxy_file_ops.cc (full stripes of
//    k * maxChunkSize bytes, a last stripe of ceil(rem / k)-byte chunks,
//    rs.cc:52-55, zero-padded, chunk_manager.cc:390-399), parity and the MD5
//    of all n chunks of every stripe, H2D -> encode -> MD5 -> D2H pipelined
//    (nxec_encode_object_host).  The result is one Chunk per chunk with the
//    reference's ids (chunkIdOffset + s * n + i, chunk_manager.cc:441-447),
//    sizes and digests.  Data chunks point into the caller's file buffer
//    (RSCode::encode's rs.cc:80 copy is gone; the last stripe's padded data
//    lives in the batch), parity chunks into the batch's pinned buffer: the
//    chunks do not own their data (freeData = false, as the reference's
//    event chunks often do) and stay valid until the next call on this batch
//    or its destruction.
//  * decodeFile: every stripe's k input chunks as fetched (sorted by id, the
//    first k alive, RSCode::preDecode's plan) -> the file bytes, through one
//    gather (frames -> HBM), one full-output decode launch
//    (nxec_decode_object) and one copy back.
//
// One StripeBatch per calling thread (it owns staging); the Coding instance
// may be shared.
#ifndef NXEC_CODING_STRIPE_BATCH_HH
#define NXEC_CODING_STRIPE_BATCH_HH

#include <cstdint>
#include <vector>

#include "coding.hh"
#include "nxec.h"

class StripeBatch {
 public:
  // code must be an RSCode; device: the GPU this batch runs on
  explicit StripeBatch(Coding *code, int device = 0);
  ~StripeBatch();
  StripeBatch(const StripeBatch &) = delete;
  StripeBatch &operator=(const StripeBatch &) = delete;

  bool ok() const { return _ctx != nullptr; }

  // number of stripes a file of `length` bytes takes (proxy_file_ops.cc:557-666)
  uint64_t numStripes(uint64_t length, length_t maxChunkSize) const;

  // write path of a whole file; chunks receives numStripes * n chunks, stripe-major
  bool encodeFile(const data_t *data, uint64_t length, length_t maxChunkSize, std::vector<Chunk> &chunks,
                  int chunkIdOffset = 0, bool computeMD5 = true);

  // read path of a whole file: inputs holds, stripe-major, the first k alive
  // chunks of every stripe (ids ascending, chunkId % n as in chunk_manager.cc:775),
  // `failed` the chunk ids absent in every stripe; out receives `length` bytes
  bool decodeFile(std::vector<Chunk> &inputs, uint64_t length, length_t maxChunkSize,
                  const std::vector<chunk_id_t> &failed, data_t *out);

 private:
  bool growHost(unsigned char **p, size_t *cap, size_t bytes);
  bool growDevice(unsigned char **p, size_t *cap, size_t bytes);

  Coding *_code;
  nxec_ctx_t *_ctx = nullptr;
  unsigned char *_parity = nullptr, *_md5 = nullptr, *_tail = nullptr;  // pinned host
  size_t _parityCap = 0, _md5Cap = 0, _tailCap = 0;
  unsigned char *_dChunks = nullptr, *_dObject = nullptr, *_dTail = nullptr;  // device
  size_t _dChunksCap = 0, _dObjectCap = 0, _dTailCap = 0;
};

#endif
