// Chunk buffer as the coding layer sees it (reference: src/ds/chunk.hh:15-130,
// reduced to the fields RSCode touches: id, data, size, ownership).  File
// identity, versions and MD5 belong to the proxy/agent and stay there.
#ifndef NXEC_CODING_CHUNK_HH
#define NXEC_CODING_CHUNK_HH

#include <stdlib.h>
#include <string.h>

struct Chunk {
  int chunkId = -1;
  unsigned char *data = nullptr;
  int size = 0;
  bool freeData = false;

  Chunk() = default;
  ~Chunk() { release(); }
  Chunk(const Chunk &o) { copy(o); }
  Chunk &operator=(const Chunk &o) {
    if (this != &o) copy(o);
    return *this;
  }
  Chunk(Chunk &&o) noexcept { move(o); }
  Chunk &operator=(Chunk &&o) noexcept {
    if (this != &o) move(o);
    return *this;
  }

  void setChunkId(int id) { chunkId = id; }
  int getChunkId() const { return chunkId; }

  // 32-byte aligned allocation when `aligned` (chunk.hh:55-89 semantics)
  bool allocateData(int n, bool aligned = false) {
    if (n <= 0) return false;
    if (data && size == n && freeData && !aligned) return true;
    unsigned char *p = nullptr;
    if (aligned) {
      if (posix_memalign(reinterpret_cast<void **>(&p), 32, n) != 0) p = nullptr;
    } else {
      p = static_cast<unsigned char *>(malloc(n));
    }
    if (!p) return false;
    if (freeData) free(data);
    data = p;
    size = n;
    freeData = true;
    return true;
  }

  bool copy(const Chunk &src, bool aligned = false) {
    release();
    chunkId = src.chunkId;
    if (src.size <= 0 || !src.data) return true;
    if (!allocateData(src.size, aligned)) return false;
    memcpy(data, src.data, size);
    return true;
  }

  bool move(Chunk &src) {
    release();
    chunkId = src.chunkId;
    data = src.data;
    size = src.size;
    freeData = src.freeData;
    src.data = nullptr;
    src.freeData = false;
    return true;
  }

  void release() {
    if (freeData) free(data);
    data = nullptr;
    size = 0;
    freeData = false;
  }
};

#endif
