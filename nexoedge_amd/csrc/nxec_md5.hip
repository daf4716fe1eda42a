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
  uint32_t f;
  int g;
  if (q == 0) {
    f = (b & c) | (~b & d);  // v_bfi
    g = R;
  } else if (q == 1) {
    f = (d & b) | (~d & c);
    g = (5 * R + 1) & 15;
  } else if (q == 2) {
    f = b ^ c ^ d;
    g = (3 * R + 5) & 15;
  } else {
    f = c ^ (b | ~d);
    g = (7 * R) & 15;
  }
  constexpr uint32_t kr = kMd5K[R];  // compile-time constant: an instruction literal, no load
  a = b + rotl(a + f + kr + m[g], kShift[q][R & 3]);
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

// Aligned streaming of the full 64-byte blocks with a ring of D block buffers:
// block b+D-1 is loaded while block b is hashed, so D-1 blocks (~0.75 us of
// rounds each) cover the HBM latency.  The ring is fully unrolled so every
// buffer is a fixed register set and the load->use distance is explicit to
// the waitcnt pass (a loop-carried copy of a prefetch buffer makes it wait on
// the loads it just issued).  Loads past the last block are clamped to it
// (re-reading one block) so they can stay unconditional.
template <int D, bool NT>
__device__ __forceinline__ void md5_stream(const uint8_t *p, int64_t nfull, uint32_t (&h)[4]) {
  uint32_t ring[D][16];
  const int64_t last = nfull - 1;
#pragma unroll
  for (int j = 0; j < D - 1; j++) load_block<NT>(p + min(static_cast<int64_t>(j), last) * 64, ring[j]);
  int64_t b = 0;
  for (; b + D <= nfull; b += D) {
#pragma unroll
    for (int j = 0; j < D; j++) {
      load_block<NT>(p + min(b + j + D - 1, last) * 64, ring[(j + D - 1) % D]);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this block's rounds
      md5_block(h, ring[j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // the last nfull % D (< D) blocks are already in ring[0 .. D-2]
#pragma unroll
  for (int j = 0; j < D - 1; j++)
    if (b + j < nfull) md5_block(h, ring[j]);
}

// one lane per chunk; chunk c of the batch = stripe c / nchunks, index c % nchunks
template <int D, bool NT>
__global__ __launch_bounds__(64) void k_md5(const uint8_t *base, int64_t chunk_stride, int64_t stripe_stride,
                                            int nchunks, int64_t len, int64_t total, uint8_t *digests,
                                            int aligned) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
  if (c >= total) return;
  const int64_t s = c / nchunks;
  const uint8_t *p = base + s * stripe_stride + (c - s * nchunks) * chunk_stride;
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  const int64_t nfull = len / 64;
  uint32_t m[16];
  if (aligned) {
    if (nfull > 0) md5_stream<D, NT>(p, nfull, h);
  } else {
    for (int64_t b = 0; b < nfull; b++) {
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
  uint32_t *o = reinterpret_cast<uint32_t *>(digests + c * 16);
  o[0] = h[0];
  o[1] = h[1];
  o[2] = h[2];
  o[3] = h[3];
}

int md5_depth() {
  static const int d = [] {
    const char *e = getenv("NXEC_MD5_DEPTH");  // tuning override: prefetch ring depth 2..4
    const int v = e ? atoi(e) : 3;
    return v >= 2 && v <= 4 ? v : 3;
  }();
  return d;
}

bool md5_nontemporal() {
  static const bool nt = [] {
    const char *e = getenv("NXEC_MD5_NT");  // tuning override: 0 = cached loads
    return !(e && e[0] == '0');
  }();
  return nt;
}

}  // namespace

int launch_md5(const uint8_t *base, int64_t chunk_stride, int64_t stripe_stride, int nchunks, int64_t len,
               int64_t nstripes, uint8_t *digests, void *stream) {
  const int64_t total = static_cast<int64_t>(nchunks) * nstripes;
  if (total <= 0) return NXEC_OK;
  const bool aligned = (reinterpret_cast<uintptr_t>(base) % 16 == 0) && (chunk_stride % 16 == 0) &&
                       (stripe_stride % 16 == 0);
  const int64_t blocks = (total + 63) / 64;
  const int d = md5_depth();
  const bool nt = md5_nontemporal();
  auto kern = nt ? (d == 2 ? k_md5<2, true> : d == 4 ? k_md5<4, true> : k_md5<3, true>)
                 : (d == 2 ? k_md5<2, false> : d == 4 ? k_md5<4, false> : k_md5<3, false>);
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(64), 0, static_cast<hipStream_t>(stream), base,
                     chunk_stride, stripe_stride, nchunks, len, total, digests, aligned ? 1 : 0);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : set_error(NXEC_ERR_HIP, "launch k_md5: %s", hipGetErrorString(e));
}

}  // namespace nxec
