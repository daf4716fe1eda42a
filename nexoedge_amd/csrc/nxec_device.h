// Device-side building blocks shared by the gfx950 kernels of libnxec:
// streaming 16-byte accesses, the packed-row GF(2^8) product tables and their
// lookup, the 4x4 byte transpose of packed accumulators, and the MD5 block
// function (RFC 1321, written from the specification).
#ifndef NXEC_DEVICE_H
#define NXEC_DEVICE_H

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

namespace nxec {
namespace dev {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Global-address-space access: pointers read from tables (per-request
// pointer tables, HBM or device-mapped host memory) are generic, and generic
// (flat) accesses count in lgkmcnt as well as vmcnt -- every wait for an LDS
// lookup then waited for the whole load ring too.  Global accesses reach the
// same memory (no LDS / scratch aperture involved).
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
__device__ __forceinline__ const g_u32x4 *gptr(const uint8_t *p) {
  return (const g_u32x4 *)(reinterpret_cast<uintptr_t>(p));
}
__device__ __forceinline__ g_u32x4 *gptr(uint8_t *p) { return (g_u32x4 *)(reinterpret_cast<uintptr_t>(p)); }
__device__ __forceinline__ u32x4 ld_global(const uint8_t *p) { return *gptr(p); }
__device__ __forceinline__ u32x4 ld_global_stream(const uint8_t *p) { return __builtin_nontemporal_load(gptr(p)); }
__device__ __forceinline__ void st_global_stream(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, gptr(p)); }

// Streaming (nontemporal) 16-byte accesses: every source byte is read once and
// every parity byte written once, so keep them from displacing the tables'
// neighbours in L2/MALL.  Measured +2-3 % at RS(10,4) 1 MiB (tools/microbench/tune_mul.hip).
// Always global: the gather forms' table pointers would otherwise be flat.
__device__ __forceinline__ u32x4 ld_stream(const uint8_t *p) { return ld_global_stream(p); }
__device__ __forceinline__ void st_stream(uint8_t *p, u32x4 v) { st_global_stream(p, v); }

// GF(2^8) product over the RS polynomial 0x11d (ISA-L gf_mul, ec_base.c:48-61)
__device__ __forceinline__ uint32_t gf_mul_dev(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    p ^= (b & 1u) ? a : 0u;
    a = (a << 1) ^ ((a & 0x80u) ? 0x11du : 0u);
    b >>= 1;
  }
  return p;
}

// Entry x of source j packs byte r = c(r, j) * x for every output row r <
// rows (<= 4); coef is row-major rows x k.  Copy c of the entry sits at
// tab[(j*256 + x)*R + c] so lane % R picks a copy in different LDS banks.
template <int R>
__device__ __forceinline__ void build_tables(const uint8_t *coef, int k, int rows, uint32_t *tab) {
  for (int i = threadIdx.x; i < k * 256; i += blockDim.x) {
    const int j = i >> 8;
    const uint32_t x = static_cast<uint32_t>(i & 255);
    uint32_t e = 0;
    for (int r = 0; r < rows; r++) e |= gf_mul_dev(coef[r * k + j], x) << (8 * r);
#pragma unroll
    for (int c = 0; c < R; c++) tab[i * R + c] = e;
  }
}

// acc[4q + b] ^= table entry of byte b of word q of the 16 source bytes d;
// tb = this lane's copy of one source's table.
template <int R>
__device__ __forceinline__ void lookup16(const char *tb, const u32x4 d, uint32_t acc[16]) {
  const uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
  for (int q = 0; q < 4; q++) {
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t x = (w[q] >> (8 * b)) & 0xffu;
      acc[4 * q + b] ^= *reinterpret_cast<const uint32_t *>(tb + x * (4 * R));
    }
  }
}

// acc[p] holds the 4 row products of column byte p; o[r] = row r's 16 bytes
// (byte r of acc[0..15]).  8 v_perm_b32 per 4 columns.
__device__ __forceinline__ void rows_of(const uint32_t acc[16], uint32_t (&o)[4][4]) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t a0 = acc[4 * q], a1 = acc[4 * q + 1], a2 = acc[4 * q + 2], a3 = acc[4 * q + 3];
    const uint32_t lo01 = __builtin_amdgcn_perm(a1, a0, 0x05010400u);
    const uint32_t hi01 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);
    const uint32_t lo23 = __builtin_amdgcn_perm(a3, a2, 0x05010400u);
    const uint32_t hi23 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
    o[0][q] = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
    o[1][q] = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
    o[2][q] = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
    o[3][q] = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
  }
}

// ---- MD5 (RFC 1321) ----

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
__device__ __forceinline__ void md5_round(uint32_t &a, uint32_t b, uint32_t c, uint32_t d, const uint32_t *m) {
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
__device__ __forceinline__ void md5_rounds(uint32_t (&h)[4], const uint32_t *m, std::integer_sequence<int, Rs...>) {
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

// one 64-byte block m[0..15] (little-endian message words) into state h
__device__ __forceinline__ void md5_block(uint32_t (&h)[4], const uint32_t *m) {
  md5_rounds(h, m, std::make_integer_sequence<int, 64>{});
}

__device__ __forceinline__ void md5_init(uint32_t (&h)[4]) {
  h[0] = 0x67452301u;
  h[1] = 0xefcdab89u;
  h[2] = 0x98badcfeu;
  h[3] = 0x10325476u;
}

// final block of a message whose length is a multiple of 64 bytes: 0x80,
// zeros, 64-bit little-endian bit length (RFC 1321 §3.1-3.2)
__device__ __forceinline__ void md5_pad_aligned(uint32_t (&h)[4], uint64_t len) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = 0;
  m[0] = 0x80u;
  m[14] = static_cast<uint32_t>(len * 8);
  m[15] = static_cast<uint32_t>((len * 8) >> 32);
  md5_block(h, m);
}

}  // namespace dev
}  // namespace nxec

#endif
