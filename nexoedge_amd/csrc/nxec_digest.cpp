// Digests the GPU computed during a coding call, handed to Chunk::computeMD5
// (include/nxec.h §6b; reference chunk.hh:136-143).
//
// The reference hashes every chunk it has just coded, right after the coding
// call and on the same thread: chunk_manager.cc:99 (encodeFile) -> :175,
// :1141 (decode, isRepair) -> :1173, agent.cc:339 (CodingUtils::encode) ->
// :342.  The kernels behind those calls can hash the chunks in the same pass
// (k_gather_md5, nxec_encode_md5.hip).
//
// Two carriers:
//  * RSCode::encode marks each Chunk itself (chunk.hh: digestData /
//    digestSize / digestEpoch).  The mark holds only while the calling
//    thread's digest epoch is unchanged: every Chunk::allocateData and every
//    freed Chunk buffer on the thread moves the epoch on.
//  * Outputs that are plain memory regions (decode's repairedData + i*cs, the
//    agent's malloc'd outputs) have no Chunk; they are noted here, keyed by
//    (pointer, length), for the computeMD5 on the noting thread.  The
//    reference frees such regions with plain free() (chunk_manager.cc:1137,
//    1143; container_manager.cc:241-252 leaves the agent's output to its
//    caller), which this library never sees, and malloc can hand the address
//    out again at the same length.  So each entry also records a 64-bit
//    fingerprint of the bytes it was computed over, and a take is a hit only
//    when the bytes at (pointer, length) still have that fingerprint: a
//    recycled or rewritten buffer is hashed afresh instead of inheriting a
//    stale digest.  The fingerprint reads the region once on the host (~10+
//    GB/s per thread against OpenSSL MD5's ~0.6 GB/s).  The table is global
//    under a mutex: nxec_digest_forget from any thread drops an entry, and a
//    noting call clears the calling thread's older entries first.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "nxec.h"
#include "nxec_internal.h"

namespace {

struct Entry {
  uint64_t owner;
  const void *p;
  int64_t len;
  uint64_t fp;
  unsigned char md5[16];
};

constexpr size_t kMaxEntries = 4096;

std::mutex g_mu;
std::vector<Entry> g_table;
std::atomic<uint64_t> g_next_owner{1};
std::atomic<size_t> g_count{0};  // entries in g_table (lets forget skip the lock when empty)

uint64_t self() {
  thread_local const uint64_t id = g_next_owner.fetch_add(1, std::memory_order_relaxed);
  return id;
}

uint64_t &epoch() {
  thread_local uint64_t e = 1;
  return e;
}

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t load64(const unsigned char *p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

}  // namespace

namespace nxec {

// 64-bit fingerprint of [p, p + len): four independent multiply-rotate lanes
// over 32-byte blocks, then the tail and the length.  Not cryptographic --
// it only has to tell a recycled or rewritten buffer from the bytes a digest
// was computed over.
uint64_t fingerprint64(const void *p, int64_t len) {
  constexpr uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull;
  const unsigned char *b = static_cast<const unsigned char *>(p);
  uint64_t a0 = P1 ^ static_cast<uint64_t>(len), a1 = P2, a2 = P3, a3 = P1 + P2;
  int64_t i = 0;
  for (; i + 32 <= len; i += 32) {
    a0 = rotl(a0 + load64(b + i) * P2, 31) * P1;
    a1 = rotl(a1 + load64(b + i + 8) * P2, 31) * P1;
    a2 = rotl(a2 + load64(b + i + 16) * P2, 31) * P1;
    a3 = rotl(a3 + load64(b + i + 24) * P2, 31) * P1;
  }
  uint64_t h = rotl(a0, 1) + rotl(a1, 7) + rotl(a2, 12) + rotl(a3, 18);
  for (; i + 8 <= len; i += 8) h = rotl(h ^ (load64(b + i) * P2), 27) * P1 + P3;
  for (; i < len; i++) h = rotl(h ^ (b[i] * P3), 11) * P1;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  return h ^ (h >> 32);
}

}  // namespace nxec

extern "C" {

int nxec_chunk_md5_mode(void) {
  static const int mode = [] {
    const char *e = std::getenv("NXEC_CHUNK_MD5");
    if (!e || !e[0]) return 1;
    return std::atoi(e) < 0 ? 0 : std::atoi(e);
  }();
  return mode;
}

uint64_t nxec_digest_epoch(void) { return epoch(); }
void nxec_digest_epoch_bump(void) { ++epoch(); }

void nxec_digest_clear(void) {
  const uint64_t me = self();
  std::lock_guard<std::mutex> g(g_mu);
  size_t w = 0;
  for (size_t i = 0; i < g_table.size(); i++)
    if (g_table[i].owner != me) g_table[w++] = g_table[i];
  g_table.resize(w);
  g_count.store(w, std::memory_order_relaxed);
}

int nxec_digest_note(const void *p, int64_t len, const unsigned char *md5) {
  if (!p || len <= 0 || !md5) return NXEC_ERR_INVALID;
  Entry e;
  e.owner = self();
  e.p = p;
  e.len = len;
  e.fp = nxec::fingerprint64(p, len);  // outside the lock
  std::memcpy(e.md5, md5, 16);
  std::lock_guard<std::mutex> g(g_mu);
  for (Entry &x : g_table)
    if (x.p == p) {  // a newer digest for the same buffer replaces the old one, whoever noted it
      x = e;
      return NXEC_OK;
    }
  if (g_table.size() >= kMaxEntries) g_table.erase(g_table.begin());
  g_table.push_back(e);
  g_count.store(g_table.size(), std::memory_order_relaxed);
  return NXEC_OK;
}

int nxec_digest_take(const void *p, int64_t len, unsigned char *md5) {
  const uint64_t me = self();
  Entry e;
  {
    std::lock_guard<std::mutex> g(g_mu);
    size_t i = 0;
    while (i < g_table.size() && !(g_table[i].p == p && g_table[i].owner == me)) i++;
    if (i == g_table.size()) return 0;
    e = g_table[i];
    g_table.erase(g_table.begin() + static_cast<long>(i));
    g_count.store(g_table.size(), std::memory_order_relaxed);
  }
  // the bytes must still be the ones the digest was computed over
  if (e.len != len || nxec::fingerprint64(p, len) != e.fp) return 0;
  if (md5) std::memcpy(md5, e.md5, 16);
  return 1;
}

void nxec_digest_forget(const void *p) {
  ++epoch();  // a Chunk buffer is going away: this thread's Chunk marks end here
  if (g_count.load(std::memory_order_relaxed) == 0) return;  // a racing note is for a live buffer, not p
  std::lock_guard<std::mutex> g(g_mu);
  for (size_t i = 0; i < g_table.size(); i++)
    if (g_table[i].p == p) {
      g_table.erase(g_table.begin() + static_cast<long>(i));
      g_count.store(g_table.size(), std::memory_order_relaxed);
      return;
    }
}

}  // extern "C"
