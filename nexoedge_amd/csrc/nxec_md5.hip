// Per-chunk MD5 on gfx950.
//
// The reference computes an MD5 digest of every chunk on the write path
// (chunk_manager.cc:175 -> Chunk::computeMD5, chunk.hh:136, OpenSSL MD5 via
// checksum_calculator.hh:126), on repair (chunk_manager.cc:1173, agent.cc:342)
// and verifies it on reads (chunk_manager.cc:1555).  Once the coding itself
// runs at HBM speed, MD5 at ~0.6 GB/s per CPU core is the dominant cost of
// the write path.
//
// MD5 is a serial chain inside one message, so the parallelism is across
// chunks: one lane per chunk (a batch of 4096 RS(10,4) stripes is 57 344
// chunks = 896 waves, ~one per SIMD).  Each lane streams its chunk in 64-byte
// blocks (four 16-byte nontemporal loads, the next block's loads issued
// before the current block's 64 rounds) and runs the rounds in VGPRs.  The
// padding block(s) are formed in registers from the tail bytes.  Algorithm:
// RFC 1321; written from the specification.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "nxec_device.h"
#include "nxec_internal.h"

namespace nxec {

namespace {

using dev::md5_block;
using dev::u32x4;

template <bool NT>
__device__ __forceinline__ void load_block(const uint8_t *p, uint32_t (&m)[16]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p) + i;
    const u32x4 v = NT ? __builtin_nontemporal_load(q) : *q;
    m[4 * i] = v.x;
    m[4 * i + 1] = v.y;
    m[4 * i + 2] = v.z;
    m[4 * i + 3] = v.w;
  }
}

// Aligned streaming of the full 64-byte blocks.  A lane reads its chunk in
// groups of G blocks (G*64 contiguous bytes issued back to back, so the
// memory system sees G*64-byte runs per chunk instead of scattered 64-byte
// pieces from ~57k concurrent streams) through a ring of D group buffers:
// group g+D-1 is loaded while group g is hashed.  The ring is fully unrolled
// so every buffer is a fixed register set and the load->use distance is
// explicit to the waitcnt pass (a loop-carried copy of a prefetch buffer makes
// it wait on the loads it just issued).  Loads past the last group are
// clamped to it (re-reading it) so they stay unconditional; the < G leftover
// blocks are read one at a time.
template <int G, bool NT>
__device__ __forceinline__ void load_group(const uint8_t *p, uint32_t (&m)[G][16]) {
#pragma unroll
  for (int i = 0; i < G; i++) load_block<NT>(p + 64 * i, m[i]);
}

template <int D, int G, bool NT>
__device__ __forceinline__ void md5_stream(const uint8_t *p, int64_t nfull, uint32_t (&h)[4]) {
  constexpr int64_t kGroup = 64 * G;
  const int64_t ngroups = nfull / G;
  if (ngroups > 0) {
    uint32_t ring[D][G][16];
    const int64_t last = ngroups - 1;
#pragma unroll
    for (int j = 0; j < D - 1; j++) load_group<G, NT>(p + min(static_cast<int64_t>(j), last) * kGroup, ring[j]);
    int64_t g = 0;
    for (; g + D <= ngroups; g += D) {
#pragma unroll
      for (int j = 0; j < D; j++) {
        load_group<G, NT>(p + min(g + j + D - 1, last) * kGroup, ring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this group's rounds
#pragma unroll
        for (int i = 0; i < G; i++) md5_block(h, ring[j][i]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the last ngroups % D (< D) groups are already in ring[0 .. D-2]
#pragma unroll
    for (int j = 0; j < D - 1; j++)
      if (g + j < ngroups) {
#pragma unroll
        for (int i = 0; i < G; i++) md5_block(h, ring[j][i]);
      }
  }
  for (int64_t b = ngroups * G; b < nfull; b++) {
    uint32_t m[16];
    load_block<NT>(p + b * 64, m);
    md5_block(h, m);
  }
}

// Misaligned chunks (p % 16 != 0: ragged last-stripe chunks of arbitrary
// length packed back to back).  16-byte loads from the dword-aligned address
// at or below p (global_load_dwordx4 needs only dword alignment on gfx950),
// one extra dword per group, and every message word assembled with
// v_alignbit over the lane's own byte shift.  Streams blocks [0, nblk); the
// caller keeps nblk < the chunk's full-block count, so the extra dword after
// the last streamed block is still inside the chunk.
template <int D, int G>
__device__ __forceinline__ void md5_stream_u(const uint8_t *p, int64_t nblk, uint32_t (&h)[4]) {
  typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
  constexpr int W = 16 * G;  // dwords per group
  const uint32_t *pd = reinterpret_cast<const uint32_t *>(p - (reinterpret_cast<uintptr_t>(p) & 3));
  const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p) & 3) * 8;
  auto load = [&](int64_t g, uint32_t(&raw)[W + 1]) {
    const uint32_t *q = pd + g * W;
#pragma unroll
    for (int i = 0; i < W / 4; i++) {
      const u32x4 v = *reinterpret_cast<const u32x4_a4 *>(q + 4 * i);
      raw[4 * i] = v.x;
      raw[4 * i + 1] = v.y;
      raw[4 * i + 2] = v.z;
      raw[4 * i + 3] = v.w;
    }
    raw[W] = q[W];
  };
  auto hash = [&](const uint32_t(&raw)[W + 1], int nb) {
#pragma unroll
    for (int i = 0; i < G; i++) {
      if (i < nb) {
        uint32_t m[16];
#pragma unroll
        for (int t = 0; t < 16; t++) m[t] = __builtin_amdgcn_alignbit(raw[16 * i + t + 1], raw[16 * i + t], sb);
        md5_block(h, m);
      }
    }
  };
  const int64_t ngroups = nblk / G;
  if (ngroups > 0) {
    uint32_t ring[D][W + 1];
    const int64_t last = ngroups - 1;
#pragma unroll
    for (int j = 0; j < D - 1; j++) load(min(static_cast<int64_t>(j), last), ring[j]);
    int64_t g = 0;
    for (; g + D <= ngroups; g += D) {
#pragma unroll
      for (int j = 0; j < D; j++) {
        load(min(g + j + D - 1, last), ring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        hash(ring[j], G);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int j = 0; j < D - 1; j++)
      if (g + j < ngroups) hash(ring[j], G);
  }
  const int rest = static_cast<int>(nblk - ngroups * G);  // < G blocks, in one final group
  if (rest > 0) {
    uint32_t raw[W + 1];
    const uint32_t *q = pd + ngroups * W;
#pragma unroll
    for (int i = 0; i <= W; i++) raw[i] = i <= 16 * rest ? q[i] : 0u;
    hash(raw, rest);
  }
}

struct Md5Args {
  Md5Region r[kMaxMd5Regions];
  int64_t lane_end[kMaxMd5Regions];  // prefix sums of nchunks * nstripes
  int nregions;
  const Md5Item *items;  // list mode (items != nullptr): lane c hashes items[c]
  int64_t nitems;
  // verify mode (a region's ok != nullptr): its digests are the expected
  // ones; chunk (s, i) writes ok[s*ok_stripe_stride + i] = digest matches and
  // counts a mismatch into *nbad
  unsigned long long *nbad;
};

// one lane per chunk over the concatenated regions
template <int D, int G, bool NT>
__global__ __launch_bounds__(64) void k_md5(const Md5Args args) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
  const uint8_t *p;
  int64_t len;
  uint8_t *out;
  uint8_t *ok = nullptr;  // verify mode: this chunk's ok flag
  if (args.items) {
    if (c >= args.nitems) return;
    const Md5Item it = args.items[c];
    p = it.p;
    len = it.len;
    out = it.digest;
  } else {
    if (c >= args.lane_end[args.nregions - 1]) return;
    int ri = 0;
#pragma unroll
    for (int i = 0; i < kMaxMd5Regions - 1; i++)
      if (i < args.nregions - 1 && c >= args.lane_end[i]) ri = i + 1;
    const Md5Region &rg = args.r[ri];
    const int64_t cl = c - (ri ? args.lane_end[ri - 1] : 0);
    const int64_t s = cl / rg.nchunks, ci = cl - s * rg.nchunks;
    p = rg.base + s * rg.stripe_stride + ci * rg.chunk_stride;
    len = rg.len;
    out = rg.digests + s * rg.dig_stripe_stride + ci * 16;
    if (rg.ok) ok = rg.ok + s * rg.ok_stripe_stride + ci;
  }
  const bool aligned = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  const int64_t nfull = len / 64;
  uint32_t m[16];
  int64_t done = 0;  // full blocks hashed by a streaming path; the rest byte-wise
  if (aligned) {
    if (nfull > 0) md5_stream<D, G, NT>(p, nfull, h);
    done = nfull;
  } else if (nfull > 1) {
    md5_stream_u<2, 4>(p, nfull - 1, h);
    done = nfull - 1;
  }
  {
    for (int64_t b = done; b < nfull; b++) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const uint8_t *q = p + b * 64 + 4 * i;
        m[i] = q[0] | (q[1] << 8) | (q[2] << 16) | (static_cast<uint32_t>(q[3]) << 24);
      }
      md5_block(h, m);
    }
  }
  // tail + padding: 0x80, zeros, 64-bit little-endian bit length (RFC 1321 §3.1-3.2)
  const int rem = static_cast<int>(len - nfull * 64);
  const uint8_t *t = p + nfull * 64;
  const uint64_t bits = static_cast<uint64_t>(len) * 8;
  const int nblk = rem < 56 ? 1 : 2;
  for (int blk = 0; blk < nblk; blk++) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint32_t w = 0;
      for (int by = 0; by < 4; by++) {
        const int pos = blk * 64 + 4 * i + by;
        uint32_t v = 0;
        if (pos < rem) v = t[pos];
        else if (pos == rem) v = 0x80;
        w |= v << (8 * by);
      }
      m[i] = w;
    }
    if (blk == nblk - 1) {
      m[14] = static_cast<uint32_t>(bits);
      m[15] = static_cast<uint32_t>(bits >> 32);
    }
    md5_block(h, m);
  }
  if (ok) {  // Chunk::verifyMD5: recompute and compare (chunk_manager.cc:1555, container_manager.cc:187-207)
    bool same = true;
#pragma unroll
    for (int i = 0; i < 16; i++) same &= out[i] == static_cast<uint8_t>(h[i / 4] >> (8 * (i % 4)));
    *ok = same ? 1 : 0;
    if (!same && args.nbad) atomicAdd(args.nbad, 1ull);
    return;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = static_cast<uint8_t>(h[i / 4] >> (8 * (i % 4)));  // digest may be unaligned
}

// Kernel variant (prefetch ring depth D, group G blocks, nontemporal loads):
// default D=2 G=8 cached (512-byte runs per lane, 12.6 ms for 57 344 1-MiB chunks); NXEC_MD5_CFG="D,G,NT" overrides for tuning
// (tools/gpu_md5_tune.sh).  Cached loads: a lane reads each 64-byte block as
// four 16-byte loads and nontemporal loads refetch the line for each (3x
// slower, profiles/r01_md5_tune.log).
using Md5Kernel = void (*)(const Md5Args);

template <int D, int G>
Md5Kernel pick_nt(bool nt) {
  return nt ? k_md5<D, G, true> : k_md5<D, G, false>;
}

Md5Kernel md5_kernel() {
  static const Md5Kernel k = [] {
    const int d = tuning().md5_depth, g = tuning().md5_group;  // the ring-shape probe (nxec_tuning.h)
    const bool nt = tuning().md5_nt;
    if (d == 2 && g == 1) return pick_nt<2, 1>(nt);
    if (d == 4 && g == 1) return pick_nt<4, 1>(nt);
    if (d == 2 && g == 2) return pick_nt<2, 2>(nt);
    if (d == 3 && g == 2) return pick_nt<3, 2>(nt);
    if (d == 3 && g == 4) return pick_nt<3, 4>(nt);
    if (d == 2 && g == 4) return pick_nt<2, 4>(nt);
    return pick_nt<2, 8>(nt);
  }();
  return k;
}

}  // namespace

int launch_md5(const Md5Region *regions, int nregions, void *stream, unsigned long long *nbad) {
  Md5Args args{};
  args.nbad = nbad;
  int64_t total = 0;
  int nr = 0;
  for (int i = 0; i < nregions && i < kMaxMd5Regions; i++) {
    const int64_t lanes = static_cast<int64_t>(regions[i].nchunks) * regions[i].nstripes;
    if (lanes <= 0) continue;  // empty regions are dropped
    args.r[nr] = regions[i];
    total += lanes;
    args.lane_end[nr++] = total;
  }
  if (nr == 0) return NXEC_OK;
  args.nregions = nr;
  const int64_t blocks = (total + 63) / 64;
  const Md5Kernel kern = md5_kernel();
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(64), 0, static_cast<hipStream_t>(stream), args);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : set_error(NXEC_ERR_HIP, "launch k_md5: %s", hipGetErrorString(e));
}

int launch_md5_list(const Md5Item *d_items, int64_t nitems, void *stream) {
  if (nitems <= 0) return NXEC_OK;
  Md5Args args{};
  args.items = d_items;
  args.nitems = nitems;
  const int64_t blocks = (nitems + 63) / 64;
  hipLaunchKernelGGL(md5_kernel(), dim3(static_cast<unsigned>(blocks)), dim3(64), 0, static_cast<hipStream_t>(stream),
                     args);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : set_error(NXEC_ERR_HIP, "launch k_md5 (list): %s", hipGetErrorString(e));
}

}  // namespace nxec
