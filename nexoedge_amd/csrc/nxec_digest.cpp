// Digests the GPU computed during a coding call, handed to Chunk::computeMD5
// (include/nxec.h §6b; reference chunk.hh:136-143).
//
// The reference hashes every chunk it has just coded, right after the coding
// call and on the same thread: chunk_manager.cc:99 (encodeFile) -> :175,
// :1141 (decode, isRepair) -> :1173, agent.cc:339 (CodingUtils::encode) ->
// :342.  The kernels behind those calls can hash the chunks in the same pass
// (k_gather_md5, nxec_encode_md5.hip); outputs that are plain memory regions
// (decode's repairedData + i*cs, the agent's malloc'd outputs) have no Chunk
// to carry the digest, so they are noted here, per thread, keyed by
// (pointer, length), and taken once by the computeMD5 on the same thread.
// Every noting call first clears the thread's table, so an entry lives only
// until the thread's next coding call; freeing a Chunk buffer forgets it.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nxec.h"

namespace {

struct Entry {
  const void *p;
  int64_t len;
  unsigned char md5[16];
};

constexpr size_t kMaxEntries = 512;

std::vector<Entry> &table() {
  thread_local std::vector<Entry> t;
  return t;
}

}  // namespace

extern "C" {

int nxec_chunk_md5_mode(void) {
  static const int mode = [] {
    const char *e = std::getenv("NXEC_CHUNK_MD5");
    if (!e || !e[0]) return 1;
    return std::atoi(e) < 0 ? 0 : std::atoi(e);
  }();
  return mode;
}

void nxec_digest_clear(void) { table().clear(); }

int nxec_digest_note(const void *p, int64_t len, const unsigned char *md5) {
  if (!p || len <= 0 || !md5) return NXEC_ERR_INVALID;
  std::vector<Entry> &t = table();
  for (Entry &e : t)
    if (e.p == p) {  // a newer digest for the same buffer replaces the old one
      e.len = len;
      std::memcpy(e.md5, md5, 16);
      return NXEC_OK;
    }
  if (t.size() >= kMaxEntries) t.erase(t.begin());
  Entry e;
  e.p = p;
  e.len = len;
  std::memcpy(e.md5, md5, 16);
  t.push_back(e);
  return NXEC_OK;
}

int nxec_digest_take(const void *p, int64_t len, unsigned char *md5) {
  std::vector<Entry> &t = table();
  for (size_t i = 0; i < t.size(); i++)
    if (t[i].p == p) {
      const bool hit = t[i].len == len;
      if (hit && md5) std::memcpy(md5, t[i].md5, 16);
      t.erase(t.begin() + static_cast<long>(i));
      return hit ? 1 : 0;
    }
  return 0;
}

void nxec_digest_forget(const void *p) {
  std::vector<Entry> &t = table();
  if (t.empty()) return;
  for (size_t i = 0; i < t.size(); i++)
    if (t[i].p == p) {
      t.erase(t.begin() + static_cast<long>(i));
      return;
    }
}

}  // extern "C"
