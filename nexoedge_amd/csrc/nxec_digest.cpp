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
//    under a mutex and keyed by address (note, take and forget are O(1)):
//    nxec_digest_forget from any thread drops an entry, nxec_digest_clear
//    drops the calling thread's, and a thread's entries go when it exits.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "nxec.h"
#include "nxec_internal.h"

namespace {

struct Entry {
  uint64_t owner;
  uint64_t serial;  // when it was noted (FIFO eviction)
  int64_t len;
  uint64_t fp;
  unsigned char md5[16];
};

constexpr size_t kMaxEntries = 4096;

// The table, keyed by buffer address: note / take / forget are O(1); `order`
// keeps (address, serial) in noting order for the FIFO bound (stale pairs of
// entries already taken or replaced are skipped when met).
std::mutex g_mu;
std::unordered_map<const void *, Entry> g_table;
std::deque<std::pair<const void *, uint64_t>> g_order;
uint64_t g_serial = 0;
std::atomic<uint64_t> g_next_owner{1};
std::atomic<size_t> g_count{0};  // entries in g_table (lets forget skip the lock when empty)
// Chunk digest epochs: drawn from one counter, so no two threads (and no
// two moments of one thread) ever hold the same value
std::atomic<uint64_t> g_epoch{1};

// drops the entries `owner` noted (the thread's own, listed in `mine`)
void drop_owner(uint64_t owner, std::vector<const void *> &mine) {
  std::lock_guard<std::mutex> g(g_mu);
  for (const void *p : mine) {
    auto it = g_table.find(p);
    if (it != g_table.end() && it->second.owner == owner) g_table.erase(it);
  }
  mine.clear();
  g_count.store(g_table.size(), std::memory_order_relaxed);
}

// The calling thread's identity and the buffers it noted; a thread that exits
// (the reference runs a thread per request) takes its entries with it.
struct Self {
  uint64_t id = g_next_owner.fetch_add(1, std::memory_order_relaxed);
  std::vector<const void *> noted;
  ~Self() {
    if (!noted.empty()) drop_owner(id, noted);
  }
};

Self &self() {
  thread_local Self s;
  return s;
}

uint64_t &epoch() {
  thread_local uint64_t e = g_epoch.fetch_add(1, std::memory_order_relaxed);
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

// A Chunk's mark (chunk.hh) is valid only on the thread that set it and only
// until that thread's epoch moves: a fresh epoch comes from the global counter.
uint64_t nxec_digest_epoch(void) { return epoch(); }
void nxec_digest_epoch_bump(void) { epoch() = g_epoch.fetch_add(1, std::memory_order_relaxed); }

void nxec_digest_clear(void) {
  Self &me = self();
  if (!me.noted.empty()) drop_owner(me.id, me.noted);
}

int nxec_digest_note(const void *p, int64_t len, const unsigned char *md5) {
  if (!p || len <= 0 || !md5) return NXEC_ERR_INVALID;
  Self &me = self();
  Entry e;
  e.owner = me.id;
  e.len = len;
  e.fp = nxec::fingerprint64(p, len);  // outside the lock
  std::memcpy(e.md5, md5, 16);
  std::lock_guard<std::mutex> g(g_mu);
  e.serial = ++g_serial;
  // a newer digest for the same buffer replaces the old one, whoever noted it
  g_table[p] = e;
  g_order.emplace_back(p, e.serial);
  me.noted.push_back(p);
  while (g_table.size() > kMaxEntries && !g_order.empty()) {  // FIFO bound: the oldest live entry goes
    const auto old = g_order.front();
    g_order.pop_front();
    auto it = g_table.find(old.first);
    if (it != g_table.end() && it->second.serial == old.second) g_table.erase(it);
  }
  if (g_order.size() > 4 * kMaxEntries) {  // stale pairs (taken / replaced entries) pile up: compact
    std::deque<std::pair<const void *, uint64_t>> live;
    for (const auto &o : g_order) {
      auto it = g_table.find(o.first);
      if (it != g_table.end() && it->second.serial == o.second) live.push_back(o);
    }
    g_order.swap(live);
  }
  g_count.store(g_table.size(), std::memory_order_relaxed);
  return NXEC_OK;
}

int nxec_digest_take(const void *p, int64_t len, unsigned char *md5) {
  const uint64_t me = self().id;
  Entry e;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_table.find(p);
    if (it == g_table.end() || it->second.owner != me) return 0;
    e = it->second;
    g_table.erase(it);
    g_count.store(g_table.size(), std::memory_order_relaxed);
  }
  // the bytes must still be the ones the digest was computed over
  if (e.len != len || nxec::fingerprint64(p, len) != e.fp) return 0;
  if (md5) std::memcpy(md5, e.md5, 16);
  return 1;
}

void nxec_digest_forget(const void *p) {
  nxec_digest_epoch_bump();  // a Chunk buffer is going away: this thread's Chunk marks end here
  if (g_count.load(std::memory_order_relaxed) == 0) return;  // a racing note is for a live buffer, not p
  std::lock_guard<std::mutex> g(g_mu);
  if (g_table.erase(p)) g_count.store(g_table.size(), std::memory_order_relaxed);
}

}  // extern "C"
