// Chunk: a chunk buffer plus its identity and checksum (reference:
// src/ds/chunk.hh:15-186) -- the same fields, methods and ownership rules, so
// proxy and agent code written against the reference compiles unchanged.
//
// Copy semantics are the reference's: Chunk declares no copy or move
// operators, so `a = b` and pass-by-value are the implicit memberwise
// (shallow) copy that aliases b's buffer.  The reference relies on it --
// `events[i].chunks[j] = file.chunks[idx]; events[i].chunks[j].freeData =
// false;` (chunk_manager.cc:176-178, :1275-1276, :1498-1499,
// proxy_file_ops.cc:585-586, agent.cc:366-367) hands a borrowed view of the
// same bytes to the send path -- and copy() / move() stay the explicit deep
// copy and ownership transfer.  As in the reference, a std::vector<Chunk>
// that owns buffers must not reallocate (resize first, then move() in place,
// chunk_manager.cc:765-775, :1129-1132).
//
// Two differences, the reasons this header exists:
//  * allocateData takes buffers of 64 KiB and more from libnxec's pinned host
//    arena (nxec_host_alloc, include/nxec.h §6) instead of
//    posix_memalign/malloc.  They are page aligned (>= the 32 bytes
//    chunk.hh:66 asks for) and device-mapped, so RSCode::encode /
//    CodingUtils::encode give them to the GPU without a staging copy.
//    release() returns arena buffers to the arena and free()s everything
//    else, so buffers the caller malloc()ed and attached (io.cc:213,
//    container_manager.cc:241) keep working.  Without a usable GPU, or past
//    the arena's bound, allocation falls back to ordinary memory.
//  * computeMD5 may return a digest the GPU computed in the coding pass that
//    produced the bytes (include/nxec.h §6b): RSCode::encode hashes all n
//    chunks of the stripe in its kernel and marks each chunk's digest valid
//    for exactly (data, size); RSCode::decode(isRepair) and, on request,
//    CodingUtils::encode leave their outputs' digests in a table keyed by
//    (pointer, length) and checked against a fingerprint of the bytes at
//    take time (nxec_digest.cpp).  A marked digest is used once and only
//    while the buffer is the one it was computed for: allocateData, copy,
//    move (of the destination), release and reset drop the mark, copyMeta
//    never carries it, and the mark also lapses when the calling thread's
//    digest epoch moves on (any Chunk::allocateData or freed Chunk buffer on
//    that thread, include/nxec.h §6b).  The reference's sequences between the
//    coding call and the hash write nothing to the chunks (chunk_manager.cc:99
//    -> :175, :1141 -> :1173, agent.cc:339 -> :342).
//    Rule for other callers: do not write new bytes into `data` between the
//    coding call and computeMD5 (the mark cannot see a store); call
//    allocateData, or dropDigest(), first.  NXEC_CHUNK_MD5=0 disables the
//    cached digests; verifyMD5 always hashes.
//
// File uuids are boost::uuids::uuid when boost is available (the Nexoedge
// build), else a 16-byte value type of the same layout.
#ifndef NXEC_CODING_CHUNK_HH
#define NXEC_CODING_CHUNK_HH

#include <openssl/evp.h>
#include <openssl/md5.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "define.hh"
#include "nxec.h"

#if __has_include(<boost/uuid/uuid.hpp>)
#include <boost/uuid/uuid.hpp>
#include <boost/uuid/uuid_generators.hpp>
#include <boost/uuid/uuid_io.hpp>
typedef boost::uuids::uuid chunk_uuid_t;
inline chunk_uuid_t chunk_nil_uuid() { return boost::uuids::nil_uuid(); }
inline std::string chunk_uuid_str(const chunk_uuid_t &u) { return boost::uuids::to_string(u); }
#else
struct chunk_uuid_t {
  uint8_t data[16];
  bool operator==(const chunk_uuid_t &o) const { return memcmp(data, o.data, 16) == 0; }
  bool operator!=(const chunk_uuid_t &o) const { return !(*this == o); }
};
inline chunk_uuid_t chunk_nil_uuid() { return chunk_uuid_t{}; }
inline std::string chunk_uuid_str(const chunk_uuid_t &u) {  // 8-4-4-4-12 hex, as boost prints it
  char s[37];
  int p = 0;
  for (int i = 0; i < 16; i++) {
    if (i == 4 || i == 6 || i == 8 || i == 10) s[p++] = '-';
    snprintf(s + p, 3, "%02x", u.data[i]);
    p += 2;
  }
  return std::string(s, 36);
}
#endif

// buffers at least this long come from the pinned arena (NXEC_CHUNK_ARENA_MIN
// overrides; 0 = never)
inline size_t chunk_arena_min_bytes() {
  static const size_t v = [] {
    const char *e = getenv("NXEC_CHUNK_ARENA_MIN");
    return e ? static_cast<size_t>(strtoull(e, nullptr, 10)) : static_cast<size_t>(64 * 1024);
  }();
  return v;
}

struct Chunk {
  unsigned char namespaceId;                 /**< namespace id */
  chunk_uuid_t fuuid;                        /**< file uuid */
  int chunkId;                               /**< chunk id */
  unsigned char *data;                       /**< chunk data */
  int size;                                  /**< chunk size */
  bool freeData;                             /**< whether to free data upon destruction */
  int fileVersion;                           /**< file version number */
  char chunkVersion[CHUNK_VERSION_MAX_LEN];  /**< chunk version number for revert */
  unsigned char md5[MD5_DIGEST_LENGTH];      /**< chunk md5 checksum */
  // md5 holds the digest the GPU computed for exactly these bytes: valid
  // while data == digestData, size == digestSize and the calling thread's
  // digest epoch is digestEpoch (not in the reference; see the top)
  const unsigned char *digestData;
  int digestSize;
  uint64_t digestEpoch;

  Chunk() { reset(); }
  ~Chunk() { release(); }

  void copyMeta(const Chunk &src, bool copySize = true) {
    setId(src.namespaceId, src.fuuid, src.chunkId);
    fileVersion = src.fileVersion;
    strncpy(chunkVersion, src.chunkVersion, CHUNK_VERSION_MAX_LEN);
    copyMD5(src);
    if (copySize) size = src.size;
  }

  void setId(unsigned char namespaceIdt, chunk_uuid_t uuidt, int chunkIdt) {
    namespaceId = namespaceIdt;
    fuuid = uuidt;
    chunkId = chunkIdt;
  }
  void setChunkId(int chunkIdt) { chunkId = chunkIdt; }

  // chunk.hh:55-85: no allocation for sizet <= 0; keep an owned buffer of the
  // same size unless alignment is requested
  bool allocateData(int sizet, bool aligned = false) {
    if (sizet <= 0) return false;
    dropDigest();  // the caller is about to (re)write the bytes
    nxec_digest_epoch_bump();  // ... and so may any other chunk of this thread
    if (data != NULL && size == sizet && freeData && !aligned) return true;
    unsigned char *datat = NULL;
    const size_t min = chunk_arena_min_bytes();
    if (min > 0 && static_cast<size_t>(sizet) >= min) {
      void *p = NULL;
      if (nxec_host_alloc(static_cast<size_t>(sizet), &p) == NXEC_OK) datat = static_cast<unsigned char *>(p);
    }
    if (datat == NULL) {
      if (aligned) {
        if (posix_memalign(reinterpret_cast<void **>(&datat), 32, sizet) != 0) datat = NULL;
      } else {
        datat = static_cast<unsigned char *>(malloc(sizet));
      }
    }
    if (datat == NULL) return false;
    if (freeData) freeBuffer(data);
    data = datat;
    size = sizet;
    freeData = true;
    return true;
  }

  // chunk.hh:87-95; a metadata-only source (no buffer) copies its metadata
  // and leaves this chunk without a buffer instead of reading NULL
  bool copy(const Chunk &src, bool aligned = false) {
    release();
    copyMeta(src);
    if (src.data == NULL && src.size > 0) return true;
    if (!allocateData(src.size, aligned)) return false;
    memcpy(data, src.data, size);
    return true;
  }

  // chunk.hh:97-106; a digest computed for the buffer travels with it
  bool move(Chunk &src) {
    release();
    copyMeta(src);
    data = src.data;
    size = src.size;
    freeData = src.freeData;
    digestData = src.digestData;
    digestSize = src.digestSize;
    digestEpoch = src.digestEpoch;
    src.data = 0;
    src.freeData = false;
    src.dropDigest();
    return true;
  }

  unsigned char getNamespaceId() const { return namespaceId; }
  int getChunkId() const { return chunkId; }
  chunk_uuid_t getFileUUID() const { return fuuid; }
  int getFileVersion() const { return fileVersion; }
  const char *getChunkVersion() const { return chunkVersion; }

  std::string getChunkName() const {
    return std::to_string(namespaceId) + "_" + chunk_uuid_str(fuuid) + "_" + std::to_string(fileVersion) + "_" +
           std::to_string(chunkId);
  }

  // chunk.hh:136-143 (OpenSSL MD5, as MD5Calculator does), or the digest the
  // coding pass that wrote these bytes computed on the GPU (see the top)
  bool computeMD5() {
    if (size <= 0) return false;
    if (data != NULL && nxec_chunk_md5_mode() > 0) {
      if (digestData == data && digestSize == size && digestEpoch == nxec_digest_epoch()) {
        dropDigest();  // used once
        return true;
      }
      if (nxec_digest_take(data, size, md5) == 1) return true;
    }
    dropDigest();
    unsigned int len = MD5_DIGEST_LENGTH;
    return EVP_Digest(data, static_cast<size_t>(size), md5, &len, EVP_md5(), NULL) == 1;
  }
  bool verifyMD5() {
    unsigned char cur[MD5_DIGEST_LENGTH];
    unsigned int len = MD5_DIGEST_LENGTH;
    EVP_Digest(data, static_cast<size_t>(size), cur, &len, EVP_md5(), NULL);
    return memcmp(md5, cur, MD5_DIGEST_LENGTH) == 0;
  }
  void copyMD5(const Chunk &src) { memcpy(md5, src.md5, MD5_DIGEST_LENGTH); }

  // marks md5 (already filled) as the digest of the current buffer
  void setDigestValid() {
    digestData = data;
    digestSize = size;
    digestEpoch = nxec_digest_epoch();
  }
  void dropDigest() {
    digestData = NULL;
    digestSize = 0;
    digestEpoch = 0;
  }

  // chunk.hh:158-164, kept as is (including its memcmp truthiness)
  bool matchMeta(const Chunk &in) {
    return chunkId == in.chunkId && memcmp(md5, in.md5, MD5_DIGEST_LENGTH) && size == in.size;
  }
  void resetMD5() { memset(md5, 0, MD5_DIGEST_LENGTH); }

  void reset() {
    namespaceId = INVALID_NAMESPACE_ID;
    fuuid = chunk_nil_uuid();
    chunkId = INVALID_CHUNK_ID;
    fileVersion = 0;
    chunkVersion[0] = 0;
    data = 0;
    size = 0;
    freeData = true;
    resetMD5();
    dropDigest();
  }

  void release() {
    if (freeData) freeBuffer(data);
    reset();
  }

  static void freeBuffer(unsigned char *p) {
    if (!p) return;
    nxec_digest_forget(p);
    if (nxec_host_arena_owns(p)) nxec_host_free(p);
    else free(p);
  }
};

#endif
