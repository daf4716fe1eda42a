// Pinned host arena for chunk buffers (Chunk::allocateData, chunk.hh:55-66 of
// the reference; nexoedge_amd/csrc/coding/chunk.hh here).
//
// The reference allocates every chunk with posix_memalign/malloc (pageable).
// A GPU can only reach pageable memory through a staging copy into pinned
// memory, which on the per-stripe RSCode path costs a second pass over every
// byte on the host.  Chunk buffers taken from this arena are pinned and
// device-mapped, so RSCode::encode / CodingUtils::encode hand them to the GPU
// directly: the kernel reads the data chunks and writes the parity chunks over
// PCIe (zero copy) or the copy engines DMA them with no host memcpy.
//
// Design: size classes (2^i and 1.5*2^i bytes, 4 KiB .. 1 GiB), one free list
// per class, blocks pinned once with hipHostMalloc and recycled (a chunk's
// lifetime is one request; pinning costs far more than reuse).  The arena is
// bounded: NXEC_HOST_ARENA_MAX bytes, by default an eighth of the host's
// physical memory and at most 16 GiB (pinned pages cannot be swapped or
// reclaimed).  Past the bound, or without a usable device, nxec_host_alloc
// fails and the caller falls back to ordinary memory; the first "no device"
// answer is remembered, so GPU-less hosts pay no runtime call per chunk.
// nxec_host_arena_trim hands free blocks back to the OS.  Ownership lookup is
// a map of block start -> class under one mutex (a few hundred ns, once per
// allocate/free).
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "nxec.h"
#include "nxec_internal.h"

namespace {

constexpr int kClasses = 2 * (30 - 12) + 1;  // 4 KiB .. 1 GiB

size_t class_bytes(int c) {
  const size_t base = size_t(4096) << (c / 2);
  return (c & 1) ? base + base / 2 : base;
}

int class_of(size_t bytes) {
  for (int c = 0; c < kClasses; c++)
    if (class_bytes(c) >= bytes) return c;
  return -1;
}

struct Arena {
  std::mutex mu;
  std::vector<void *> free_list[kClasses];
  std::unordered_map<void *, int> owner;  // every block ever pinned -> class
  size_t pinned = 0;                      // bytes pinned so far
  size_t in_use = 0;                      // bytes handed out
  size_t cap = size_t(16) << 30;
  bool disabled = false;
  // hipHostMalloc said there is no device at all: stop asking (read without
  // the lock, hence atomic; a bad current device on one thread is not that)
  std::atomic<bool> no_device{false};
  Arena() {
    const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
    if (pages > 0 && psz > 0) cap = std::min(cap, static_cast<size_t>(pages) * static_cast<size_t>(psz) / 8);
    if (const char *e = std::getenv("NXEC_HOST_ARENA_MAX")) cap = static_cast<size_t>(std::strtoull(e, nullptr, 10));
    if (cap == 0) disabled = true;
  }
};

Arena &arena() {
  static Arena *a = new Arena();  // never destroyed: chunks may be released during static teardown
  return *a;
}

}  // namespace

extern "C" {

int nxec_host_alloc(size_t bytes, void **p) {
  if (!p) return nxec::set_error(NXEC_ERR_INVALID, "nxec_host_alloc: null pointer");
  *p = nullptr;
  const int c = class_of(bytes == 0 ? 1 : bytes);
  Arena &a = arena();
  if (c < 0 || a.disabled) return nxec::set_error(NXEC_ERR_NOMEM, "nxec_host_alloc: %zu bytes not served", bytes);
  if (a.no_device.load(std::memory_order_relaxed)) return nxec::set_error(NXEC_ERR_NODEV, "nxec_host_alloc: no device");
  const size_t cb = class_bytes(c);
  {
    std::lock_guard<std::mutex> lk(a.mu);
    if (!a.free_list[c].empty()) {
      *p = a.free_list[c].back();
      a.free_list[c].pop_back();
      a.in_use += cb;
      return NXEC_OK;
    }
    if (a.pinned + cb > a.cap) return nxec::set_error(NXEC_ERR_NOMEM, "nxec_host_alloc: arena full");
    a.pinned += cb;  // reserve before pinning outside the lock
  }
  void *blk = nullptr;
  const hipError_t e = hipHostMalloc(&blk, cb, hipHostMallocDefault);
  std::lock_guard<std::mutex> lk(arena().mu);
  if (e != hipSuccess || !blk) {
    (void)hipGetLastError();
    a.pinned -= cb;
    if (e == hipErrorNoDevice) a.no_device.store(true, std::memory_order_relaxed);
    return nxec::set_error(e == hipErrorNoDevice ? NXEC_ERR_NODEV : NXEC_ERR_NOMEM, "nxec_host_alloc: %s",
                           hipGetErrorString(e));
  }
  a.owner.emplace(blk, c);
  a.in_use += cb;
  *p = blk;
  return NXEC_OK;
}

int nxec_host_arena_owns(const void *p) {
  if (!p) return 0;
  Arena &a = arena();
  std::lock_guard<std::mutex> lk(a.mu);
  return a.owner.count(const_cast<void *>(p)) ? 1 : 0;
}

int nxec_host_free(void *p) {
  if (!p) return NXEC_OK;
  Arena &a = arena();
  std::lock_guard<std::mutex> lk(a.mu);
  auto it = a.owner.find(p);
  if (it == a.owner.end()) return nxec::set_error(NXEC_ERR_INVALID, "nxec_host_free: %p is not an arena block", p);
  a.free_list[it->second].push_back(p);
  a.in_use -= class_bytes(it->second);
  return NXEC_OK;
}

int nxec_host_arena_stats(size_t *pinned_bytes, size_t *in_use_bytes) {
  Arena &a = arena();
  std::lock_guard<std::mutex> lk(a.mu);
  if (pinned_bytes) *pinned_bytes = a.pinned;
  if (in_use_bytes) *in_use_bytes = a.in_use;
  return NXEC_OK;
}

size_t nxec_host_arena_cap(void) { return arena().cap; }

int nxec_host_arena_trim(size_t keep_bytes) {
  Arena &a = arena();
  std::vector<void *> drop;
  {
    std::lock_guard<std::mutex> lk(a.mu);
    for (int c = kClasses - 1; c >= 0 && a.pinned > keep_bytes; c--)  // largest blocks first
      while (!a.free_list[c].empty() && a.pinned > keep_bytes) {
        void *p = a.free_list[c].back();
        a.free_list[c].pop_back();
        a.owner.erase(p);
        a.pinned -= class_bytes(c);
        drop.push_back(p);
      }
  }
  int rc = NXEC_OK;
  for (void *p : drop)  // unpinning takes a while: outside the lock
    if (hipHostFree(p) != hipSuccess) rc = nxec::set_error(NXEC_ERR_HIP, "nxec_host_arena_trim: hipHostFree failed");
  return rc;
}

}  // extern "C"
