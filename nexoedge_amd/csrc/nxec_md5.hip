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

#include "nxec_internal.h"

namespace nxec {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

// Round r (0..63): function, message index and shift per RFC 1321 §3.4;
// K[r] = floor(|sin(r+1)| * 2^32).
constexpr uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

template <int R>
__device__ __forceinline__ void md5_round(uint32_t &a, uint32_t b, uint32_t c, uint32_t d, const uint32_t (&m)[16]) {
  constexpr int kShift[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
  constexpr int q = R / 16;
  // one v_bitop3_b32 per round function (truth table over (b, c, d), bit
  // index 4b+2c+d): F = b ? c : d (0xCA), G = d ? b : c (0xE4),
  // H = b ^ c ^ d (0x96), I = c ^ (b | ~d) (0x39)
  constexpr unsigned kTruth[4] = {0xCA, 0xE4, 0x96, 0x39};
  const uint32_t f = __builtin_amdgcn_bitop3_b32(b, c, d, kTruth[q]);
  constexpr int g = q == 0 ? R : q == 1 ? (5 * R + 1) & 15 : q == 2 ? (3 * R + 5) & 15 : (7 * R) & 15;
  constexpr uint32_t kr = kMd5K[R];  // compile-time constant: no load
  const uint32_t x = a + kr + m[g];    // off the critical path: a is 4 rounds old
  a = b + rotl(f + x, kShift[q][R & 3]);
}

template <int... Rs>
__device__ __forceinline__ void md5_rounds(uint32_t (&h)[4], const uint32_t (&m)[16], std::integer_sequence<int, Rs...>) {
  // the four state words rotate roles every round: (a,b,c,d) -> (d,a,b,c)
  uint32_t s[4] = {h[0], h[1], h[2], h[3]};
  (..., [&] {
    constexpr int ia = (64 - Rs) & 3, ib = (65 - Rs) & 3, ic = (66 - Rs) & 3, id = (67 - Rs) & 3;
    md5_round<Rs>(s[ia], s[ib], s[ic], s[id], m);
  }());
  h[0] += s[0];
  h[1] += s[1];
  h[2] += s[2];
  h[3] += s[3];
}

__device__ __forceinline__ void md5_block(uint32_t (&h)[4], const uint32_t (&m)[16]) {
  md5_rounds(h, m, std::make_integer_sequence<int, 64>{});
}

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
  // verify mode (ok != nullptr): the region's digests are the expected ones,
  // lane c writes ok[c] = digest matches, and counts mismatches into *nbad
  uint8_t *ok;
  unsigned long long *nbad;
};

// one lane per chunk over the concatenated regions
template <int D, int G, bool NT>
__global__ __launch_bounds__(64) void k_md5(const Md5Args args) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
  const uint8_t *p;
  int64_t len;
  uint8_t *out;
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
  if (args.ok) {  // Chunk::verifyMD5: recompute and compare (chunk_manager.cc:1555, container_manager.cc:187-207)
    bool same = true;
#pragma unroll
    for (int i = 0; i < 16; i++) same &= out[i] == static_cast<uint8_t>(h[i / 4] >> (8 * (i % 4)));
    args.ok[c] = same ? 1 : 0;
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
    int d = 2, g = 8, nt = 0;
    if (const char *e = getenv("NXEC_MD5_CFG")) sscanf(e, "%d,%d,%d", &d, &g, &nt);
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

int launch_md5(const Md5Region *regions, int nregions, void *stream, uint8_t *ok, unsigned long long *nbad) {
  Md5Args args{};
  args.ok = ok;
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
