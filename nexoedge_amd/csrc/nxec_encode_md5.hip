// Fused GF(2^8) multiply + per-chunk MD5 of a stripe batch on gfx950
// (SURVEY §8f.1-f.2): the write path's encode + MD5 of all n chunks, and the
// repair path's recover + MD5 of the rebuilt chunks (chunk_manager.cc:1173).
// Described below for the write path (the harder case: every chunk hashed).
//
// The proxy's write path codes every stripe and then hashes every chunk it
// sends (chunk_manager.cc:66-452: RSCode::encode, then Chunk::computeMD5 at
// :175 for each of the n chunks).  Run as two kernels, the encode reads the
// data once (k*cs per stripe) and writes the parity, then the MD5 reads all n
// chunks again: 2x the HBM traffic of the encode alone, and the parity chains
// cannot start before the parity exists (encode 9.4 ms + MD5 ~12 ms for 4096
// RS(10,4) 1 MiB stripes).  Here both run in one kernel over one read:
//
//  * A workgroup owns S whole stripes (S*n <= 256 hashed chunks) and walks
//    them column by column, 256 bytes of every chunk per step.  MD5 is a
//    serial chain per chunk, so a chunk's bytes must reach its hash lane in
//    order; every chain of the batch runs at once (one lane each).
//  * Waves 0-3 ("code"): lane (stripe, 16-byte column vector) keeps the k
//    source vectors of the next three steps in flight (a 4-deep register
//    ring), computes this step's parity through single-copy packed-row LDS
//    tables (one SDWA address op per byte, one 3-way XOR per two lookups),
//    stores the parity to HBM, and drops the data and parity vectors into
//    this step's LDS buffer.
//  * Waves 4-7 ("hash"): lane h owns hashed chunk h; right after the step's
//    barrier it issues the 16 ds_read_b128 of its 256-byte row (rows 272
//    bytes apart, so a quarter-wave's rows hit distinct banks) and hashes the
//    PREVIOUS step's row from registers (4 MD5 blocks), so the reads have a
//    whole step to land.  Two LDS buffers, one LDS-only barrier per step;
//    global loads and stores stay in flight across it.
//  * Every SIMD holds one code and one hash wave.  A wave alone issues one
//    VALU op per 4 cycles and a SIMD can issue one per 2 (MI355X_MICROARCH.md
//    'Wave scheduling'), so the chains run near their single-wave rate while
//    the code wave uses the other issue slots and the LDS.  The chain (16 384
//    blocks x ~324 VALU x 4 cycles per 1 MiB chunk, ~10 ms at the loaded
//    clock) is the floor; measured 13.8 ms against the two kernels' 21.7 ms
//    (DESIGN.md §4).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <queue>
#include <utility>
#include <vector>

#include "nxec_device.h"
#include "nxec_internal.h"

// Design-probe kernels (role probes and the LDS-table A/B variants, selected
// by environment variables) are built only with `make PROBES=1`: they are
// measurement tools, not product paths, and double this file's build time.
#ifndef NXEC_DESIGN_PROBES
#define NXEC_DESIGN_PROBES 0
#endif

extern "C" int nxec_design_probes(void) { return NXEC_DESIGN_PROBES; }

namespace nxec {

namespace {

using dev::build_tables;
using dev::md5_block;
using dev::md5_init;
using dev::md5_pad_aligned;
using dev::rows_of;
using dev::u32x4;

constexpr int kEmBlock = 512;                  // 4 code waves + 4 hash waves
constexpr int kEmCodeLanes = 256;
constexpr int kEmVecs = kEncMd5Step / 16;      // 16-byte column vectors per chunk per step
constexpr int kEmRow = kEncMd5Step + 16;       // LDS row stride: bank rotation for the hash lanes' reads
constexpr int kEmMaxRows = 256;                // chunks per workgroup = hash lanes
constexpr int kEmMaxStripes = kEmCodeLanes / kEmVecs;
constexpr int kEmLds = 160 * 1024;

// Byte b of w times 4 (its table entry's byte offset) in one VALU op: an SDWA
// source select instead of v_bfe + v_lshl_add.  Not volatile: the compiler
// schedules these freely.
template <int B>
__device__ __forceinline__ uint32_t byte_x4(uint32_t w) {
  uint32_t r;
  if constexpr (B == 0)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(w));
  else if constexpr (B == 1)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(w));
  else if constexpr (B == 2)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(w));
  else
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(w));
  return r;
}

// acc[4q + b] ^= T_j0[byte b of word q of d0] ^ T_j1[... of d1] over the
// single-copy tables at LDS byte 0 (entry x of source j at j*1024 + 4x):
// one SDWA address op per byte, the source's table offset as the ds_read
// immediate, one v_bitop3 (3-way XOR) per two lookups.  The tables are the
// first bytes of the dynamic LDS and the kernel has no static LDS
// (prepare_encode_md5 checks), so an integer LDS address is the table offset.
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
__device__ __forceinline__ uint32_t ent(int table_off, uint32_t byte_off) {
  return *reinterpret_cast<lds_u32 *>(static_cast<uintptr_t>(byte_off + table_off));
}
__device__ __forceinline__ void lookup_pair(int j0, bool two, const u32x4 d0, const u32x4 d1, uint32_t acc[16]) {
  const uint32_t w0[4] = {d0.x, d0.y, d0.z, d0.w}, w1[4] = {d1.x, d1.y, d1.z, d1.w};
  const int t0 = j0 * 1024, t1 = t0 + 1024;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t a[4] = {byte_x4<0>(w0[q]), byte_x4<1>(w0[q]), byte_x4<2>(w0[q]), byte_x4<3>(w0[q])};
    if (two) {  // constant after unrolling
      const uint32_t b[4] = {byte_x4<0>(w1[q]), byte_x4<1>(w1[q]), byte_x4<2>(w1[q]), byte_x4<3>(w1[q])};
#pragma unroll
      for (int i = 0; i < 4; i++) acc[4 * q + i] = __builtin_amdgcn_bitop3_b32(acc[4 * q + i], ent(t0, a[i]), ent(t1, b[i]), 0x96);
    } else {
#pragma unroll
      for (int i = 0; i < 4; i++) acc[4 * q + i] ^= ent(t0, a[i]);
    }
  }
}

// Split-nibble tables without bank conflicts (the A/B of DESIGN.md §4's LDS
// floor; NXEC_EM_TABLES=nib, K = 10): source j's products of x and of x << 4
// (x = 0..15, 4 rows packed per entry) in 32 copies, copy c at bank c, so a
// 32-lane group's ds_read_b32 is served in one LDS cycle whatever the bytes.
// Entry (j, x, half, c) at byte j*4096 + x*256 + half*128 + 4c: the address
// of a nibble is one v_perm_b32 (nibble into byte 1, the lane's 4c | 128*half
// into byte 0).  Two lookups per byte (~3.75 VALU per byte against the
// single-copy table's 1.5, and 4x the table bytes: 40 KiB for k = 10).
__device__ __forceinline__ void build_nib_tables(const uint8_t *coef, int k, int rows, uint32_t *tab) {
  for (int i = threadIdx.x; i < k * 1024; i += blockDim.x) {
    const int half = (i >> 5) & 1, nib = (i >> 6) & 15, j = i >> 10;
    const uint32_t x = half ? static_cast<uint32_t>(nib) << 4 : static_cast<uint32_t>(nib);
    uint32_t e = 0;
    for (int r = 0; r < rows; r++) e |= dev::gf_mul_dev(coef[r * k + j], x) << (8 * r);
    tab[i] = e;
  }
}
__device__ __forceinline__ void lookup_nib(int j, const u32x4 d, uint32_t lane4, uint32_t acc[16]) {
  const uint32_t w[4] = {d.x, d.y, d.z, d.w};
  const int t = j * 4096;
  const uint32_t lane4h = lane4 | 128u;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t wl = w[q] & 0x0F0F0F0Fu, wh = (w[q] >> 4) & 0x0F0F0F0Fu;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t sel = 0x0C0C0000u | ((4u + b) << 8);
      const uint32_t al = __builtin_amdgcn_perm(wl, lane4, sel), ah = __builtin_amdgcn_perm(wh, lane4h, sel);
      acc[4 * q + b] = __builtin_amdgcn_bitop3_b32(acc[4 * q + b], ent(t, al), ent(t, ah), 0x96);
    }
  }
}

// prefetch ring depth: as many 4K-VGPR source buffers as fit in ~200 VGPRs
// (the rest of the code role needs ~20 with buffer-resource addressing)
template <int K>
constexpr int em_depth() {
#ifdef NXEC_EM_DEPTH  // design A/B of the ring depth (a separate build)
  if (K == 10) return NXEC_EM_DEPTH;
#endif
  return K * 4 * 4 <= 200 ? 4 : K * 4 * 3 <= 200 ? 3 : 2;
}

// Raw buffer resource over [base, base + 4 GiB) (gfx9 descriptor word 3) and
// nontemporal 16-byte accesses through it (cache policy 2 = nt on gfx950).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t em_rsrc(const void *base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, -1, 0x00020000);
}
__device__ __forceinline__ u32x4 em_load(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 2));
}
__device__ __forceinline__ u32x4 em_load_cached(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void em_store(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0)), v),
                                         r, voff, soff, 2);
}

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Hash waves of the fused kernels: lane h owns LDS row h (kEncMd5Step bytes
// of its chunk per step, two step buffers buf_bytes apart).  The row of step s
// is read right after barrier s, while the lane hashes step s - 1 from
// registers: the reads (queued behind the code waves' lookups in the LDS) get
// a whole step to land.  They are complete before barrier s + 1 (its fence
// waits for them), so the code waves may refill that buffer afterwards.
// Every hash wave takes part in every barrier; st is the state after the
// last data block (not yet padded).  PROBE bit 0: XOR instead of MD5 rounds.
// TAIL: the last step holds `tail` bytes (1..kEncMd5Step; the code lanes
// zeroed the rest of its row) of a `len`-byte chunk, and st comes back
// finished -- the step's full blocks, then the padding block(s) of RFC 1321
// §3.1-3.2 built in registers from the row.
template <int PROBE, bool TAIL = false>
__device__ __forceinline__ void hash_rows(const uint8_t *buf, uint32_t buf_bytes, int h, bool active, int nsteps,
                                          uint32_t (&st)[4], int tail = kEncMd5Step, uint64_t len = 0) {
  const u32x4 *row = reinterpret_cast<const u32x4 *>(buf + h * kEmRow);
  md5_init(st);
  auto fetch = [&](int step, uint32_t(&m)[kEncMd5Step / 4]) {
    const u32x4 *p = row + (step & 1) * (buf_bytes / 16);
#pragma unroll
    for (int i = 0; i < kEmVecs; i++) {
      const u32x4 x = p[i];
      m[4 * i] = x.x;
      m[4 * i + 1] = x.y;
      m[4 * i + 2] = x.z;
      m[4 * i + 3] = x.w;
    }
  };
  auto hash = [&](const uint32_t(&m)[kEncMd5Step / 4]) {
    if (PROBE & 1) {
#pragma unroll
      for (int i = 0; i < kEncMd5Step / 4; i++) st[i & 3] ^= m[i];
    } else {
#pragma unroll
      for (int b = 0; b < kEncMd5Step / 64; b++) md5_block(st, m + 16 * b);
    }
  };
  auto hash_last = [&](const uint32_t(&m)[kEncMd5Step / 4]) {
    if (!TAIL) {
      hash(m);
      return;
    }
    const int fb = tail / 64, r = tail % 64;  // uniform: one chunk size per launch
#pragma unroll
    for (int b = 0; b < kEncMd5Step / 64; b++)
      if (b < fb) md5_block(st, m + 16 * b);
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < kEncMd5Step / 64; b++)
        if (b == fb) x = m[16 * b + i];  // the partial block (none when fb == 4)
      w[i] = x | (i == r / 4 ? 0x80u << (8 * (r % 4)) : 0u);
    }
    const uint32_t lo = static_cast<uint32_t>(len * 8), hi = static_cast<uint32_t>((len * 8) >> 32);
    if (r < 56) {
      w[14] = lo;
      w[15] = hi;
      md5_block(st, w);
    } else {
      md5_block(st, w);
      uint32_t z[16];
#pragma unroll
      for (int i = 0; i < 16; i++) z[i] = 0;
      z[14] = lo;
      z[15] = hi;
      md5_block(st, z);
    }
  };
  uint32_t m0[kEncMd5Step / 4], m1[kEncMd5Step / 4];
  lds_barrier();
  if (active) fetch(0, m0);
  int step = 1;
  for (; step + 2 <= nsteps; step += 2) {
    lds_barrier();
    if (active) {
      fetch(step, m1);
      hash(m0);
    }
    lds_barrier();
    if (active) {
      fetch(step + 1, m0);
      hash(m1);
    }
  }
  if (step < nsteps) {  // nsteps even: one step left
    lds_barrier();
    if (active) {
      fetch(step, m1);
      hash(m0);
      hash_last(m1);
    }
  } else if (active) {
    hash_last(m0);
  }
}

// Hash lanes of the HG variant (NXEC_EM_HASHSRC=global):
// a lane whose chunk is a source (gsrc != nullptr) reads its 256 bytes of
// the step from global memory -- the code waves loaded them a few steps
// earlier with caching loads, so they come from L2 / the Infinity Cache --
// instead of an LDS row; output chunks keep their LDS rows.  Same
// double-buffered timing as hash_rows.
__device__ __forceinline__ void hash_rows_hg(const uint8_t *buf, uint32_t buf_bytes, int lds_row, const uint8_t *gsrc,
                                             bool active, int nsteps, uint32_t (&st)[4]) {
  const u32x4 *row = reinterpret_cast<const u32x4 *>(buf + lds_row * kEmRow);
  md5_init(st);
  auto fetch = [&](int step, uint32_t(&m)[kEncMd5Step / 4]) {
    if (gsrc) {
      const uint8_t *g = gsrc + static_cast<int64_t>(step) * kEncMd5Step;
#pragma unroll
      for (int i = 0; i < kEmVecs; i++) {
        const u32x4 x = dev::ld_global(g + 16 * i);
        m[4 * i] = x.x, m[4 * i + 1] = x.y, m[4 * i + 2] = x.z, m[4 * i + 3] = x.w;
      }
    } else {
      const u32x4 *p = row + (step & 1) * (buf_bytes / 16);
#pragma unroll
      for (int i = 0; i < kEmVecs; i++) {
        const u32x4 x = p[i];
        m[4 * i] = x.x, m[4 * i + 1] = x.y, m[4 * i + 2] = x.z, m[4 * i + 3] = x.w;
      }
    }
  };
  auto hash = [&](const uint32_t(&m)[kEncMd5Step / 4]) {
#pragma unroll
    for (int b = 0; b < kEncMd5Step / 64; b++) md5_block(st, m + 16 * b);
  };
  uint32_t m0[kEncMd5Step / 4], m1[kEncMd5Step / 4];
  lds_barrier();
  if (active) fetch(0, m0);
  int step = 1;
  for (; step + 2 <= nsteps; step += 2) {
    lds_barrier();
    if (active) {
      fetch(step, m1);
      hash(m0);
    }
    lds_barrier();
    if (active) {
      fetch(step + 1, m0);
      hash(m1);
    }
  }
  if (step < nsteps) {
    lds_barrier();
    if (active) {
      fetch(step, m1);
      hash(m0);
      hash(m1);
    }
  } else if (active) {
    hash(m0);
  }
}

// PROBE (design probes only, K = 10, NXEC_EM_PROBE; outputs are NOT valid):
// bit 0 skips the MD5 rounds (hash lanes only read their rows), bit 1 skips
// the table lookups (parity = first source), bit 2 skips every global load
// and store (sources made up in registers), to time each role alone.
// HSRC: the sources are hashed too (write and verified-read paths) -- a
// template parameter, not a runtime flag: a wave-uniform branch around the
// sources' LDS writes kept every ring buffer live longer and spilled from
// k = 8 (180 instead of 256+ VGPRs at k = 10).
template <int K, bool HSRC, int PROBE = 0, bool NIB = false, bool HG = false>
__global__ __launch_bounds__(kEmBlock) void k_mul_md5(const MulMd5Args a) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int nh = a.nhashed;  // hashed chunks per stripe
  // LDS rows per stripe: every hashed chunk, or (HG) only the outputs
  const int nrow = HG ? a.p : nh;
  constexpr int hsrc = HSRC && !HG ? K : 0;  // rows before the outputs' rows
  const int S = a.stripes_per_group;
  uint32_t *tab = reinterpret_cast<uint32_t *>(lds);
  uint8_t *buf = lds + K * (NIB ? 4096 : 1024);
  const uint32_t buf_bytes = static_cast<uint32_t>(S * nrow * kEmRow);
  if (NIB)
    build_nib_tables(a.coef, K, a.p, tab);
  else
    build_tables<1>(a.coef, K, a.p, tab);
  __syncthreads();
  const int64_t s0 = static_cast<int64_t>(blockIdx.x) * S;
  const int nS = static_cast<int>(min(static_cast<int64_t>(S), a.nstripes - s0));
  const int nsteps = static_cast<int>(a.len / kEncMd5Step);

  if (threadIdx.x < kEmCodeLanes) {
    // A code wave with no live stripe (S * 16 < 256 lanes: fewer stripes per
    // workgroup than it has code lanes) only keeps the step barriers; running
    // it as a shadow would repeat a live wave's loads and LDS lookups, and the
    // lookups are the code role's bound (bank conflicts).
    if ((threadIdx.x & ~63) >= nS * kEmVecs) {
      for (int s = 0; s < nsteps; s++) lds_barrier();
      return;
    }
    // ---- code waves: lane = (stripe ls, column vector v) ----
    // Lanes past the group's last stripe (a partial last group) shadow lane
    // (0, v): same loads, same values stored to the same places.  Everything
    // stays unconditional, so the compiler's vmcnt bookkeeping sees one path
    // and waits only for the ring slot it consumes.
    const int item = threadIdx.x;
    const int ls = item < nS * kEmVecs ? item / kEmVecs : 0, v = item % kEmVecs;
    // Global accesses go through buffer resources based at the group's first
    // stripe: the lane's part of the address is one 32-bit VGPR, the chunk
    // and step part an SGPR offset -- no 64-bit address pair per source,
    // output and copy (those pushed the copy-through variant into spills).
    // launch_mul_md5 checks that every offset of a group fits in 32 bits.
    const __amdgpu_buffer_rsrc_t rsrc_src = em_rsrc(a.src + s0 * a.src_stripe_stride);
    const __amdgpu_buffer_rsrc_t rsrc_dst = em_rsrc(a.dst + s0 * a.dst_stripe_stride);
    const uint32_t vsrc = static_cast<uint32_t>(ls * a.src_stripe_stride) + v * 16;
    const uint32_t vdst = static_cast<uint32_t>(ls * a.dst_stripe_stride) + v * 16;
    uint8_t *row = buf + ls * nrow * kEmRow + v * 16;
    auto load = [&](int step, u32x4(&d)[K]) {
      const uint32_t off = static_cast<uint32_t>(step) * kEncMd5Step;
#pragma unroll
      for (int j = 0; j < K; j++) {
        if (PROBE & 4)  // no HBM traffic: a value the compiler cannot fold
          d[j] = u32x4{vsrc ^ off, off + j, vsrc, static_cast<uint32_t>(j)};
        else if (HG)  // the hash lanes read these bytes again a few steps later
          d[j] = em_load_cached(rsrc_src, vsrc, a.src_off[j] + off);
        else
          d[j] = em_load(rsrc_src, vsrc, a.src_off[j] + off);
      }
    };
    auto run = [&](int step, const u32x4(&d)[K]) {
      uint8_t *rb = row + (step & 1) * buf_bytes;
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        if (hsrc) {  // wave-uniform
          *reinterpret_cast<u32x4 *>(rb + j * kEmRow) = d[j];
          if (j + 1 < K) *reinterpret_cast<u32x4 *>(rb + (j + 1) * kEmRow) = d[j + 1];
        }
        if (a.any_copy) {  // full-output decode: surviving data chunks pass through
          const uint32_t off = static_cast<uint32_t>(step) * kEncMd5Step;
          if (a.copy_off[j] != kNoCopy) em_store(rsrc_dst, vdst, a.copy_off[j] + off, d[j]);
          if (j + 1 < K && a.copy_off[j + 1] != kNoCopy) em_store(rsrc_dst, vdst, a.copy_off[j + 1] + off, d[j + 1]);
        }
        if (PROBE & 2) {
          if (j == 0) acc[0] = d[0].x, acc[5] = d[0].y, acc[10] = d[0].z, acc[15] = d[0].w;
        } else if (a.p > 0) {  // wave-uniform (p = 0: a verified copy, no rows to compute)
          if (NIB) {
            const uint32_t lane4 = (threadIdx.x & 31u) * 4u;
            lookup_nib(j, d[j], lane4, acc);
            if (j + 1 < K) lookup_nib(j + 1, d[j + 1], lane4, acc);
          } else {
            lookup_pair(j, j + 1 < K, d[j], d[j + 1 < K ? j + 1 : j], acc);
          }
        }
        // materialise the accumulators per source pair: left alone, LLVM
        // turns the XOR chains into trees over all k sources, which keeps 16
        // lookup results per source live at once (spills from k = 10)
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("" : "+v"(acc[i]));
      }
      uint32_t o[4][4];
      rows_of(acc, o);
      const uint32_t off = static_cast<uint32_t>(step) * kEncMd5Step;
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++) {
        if (r < a.p) {  // wave-uniform
          const u32x4 pv{o[r][0], o[r][1], o[r][2], o[r][3]};
          if (!(PROBE & 4)) em_store(rsrc_dst, vdst, a.dst_off[r] + off, pv);
          if (a.hash_dst) *reinterpret_cast<u32x4 *>(rb + (hsrc + r) * kEmRow) = pv;
        }
      }
      lds_barrier();  // this step's buffer is full
    };
    // ring of D register buffers: the loads of step s + D - 1 go out before
    // step s is computed, so ~(D-1) steps of sources are in flight per lane
    // (one step ahead left the chip at ~0.65 of 8 TB/s with no arithmetic at
    // all).  Loads past the last step re-read it, so they stay unconditional.
    constexpr int D = em_depth<K>();
    u32x4 ring[D][K];
    const int last = nsteps - 1;
#pragma unroll
    for (int j = 0; j < D - 1; j++) load(min(j, last), ring[j]);
    // whole rounds of D steps without exits (an exit inside the unrolled
    // round merges ring states at the loop head, and the compiler then drains
    // every load there), then the < D leftover steps
    int step = 0;
    for (; step + D <= nsteps; step += D) {
#pragma unroll
      for (int j = 0; j < D; j++) {
        load(min(step + j + D - 1, last), ring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run(step + j, ring[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < D - 1; j++) {
      if (step + j < nsteps) {
        load(min(step + j + D - 1, last), ring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run(step + j, ring[j]);
      }
    }
    return;
  }

  // ---- hash waves: lane h = hashed chunk (h / nh, h % nh) of the group = LDS row h ----
  if (a.hash_prio) __builtin_amdgcn_s_setprio(1);
  const int h = threadIdx.x - kEmCodeLanes;
  const bool active = h < nS * nh;
  uint32_t st[4];
  if (HG) {
    const int hls = active ? h / nh : 0, hc = active ? h - hls * nh : 0;
    const bool gsrc = active && hc < K;
    const uint8_t *gp = gsrc ? a.src + (s0 + hls) * a.src_stripe_stride + a.src_off[hc] : nullptr;
    hash_rows_hg(buf, buf_bytes, gsrc ? 0 : hls * nrow + (hc - K), gp, active, nsteps, st);
  } else {
    hash_rows<PROBE>(buf, buf_bytes, h, active, nsteps, st);
  }
  if (active) {
    md5_pad_aligned(st, static_cast<uint64_t>(a.len));
    const int ls = h / nh, c = h - ls * nh;
    uint8_t *out = a.digests + (s0 + ls) * a.digest_stripe_stride + a.digest_slot[c] * 16;
    if (a.ok) {  // Chunk::verifyMD5 (chunk_manager.cc:1553-1555): compare with the stored digest
      bool same = true;
#pragma unroll
      for (int i = 0; i < 16; i++) same &= out[i] == static_cast<uint8_t>(st[i / 4] >> (8 * (i % 4)));
      a.ok[(s0 + ls) * a.ok_stripe_stride + a.digest_slot[c]] = same ? 1 : 0;
      if (!same && a.nbad) atomicAdd(a.nbad, 1ull);
    } else {
#pragma unroll
      for (int i = 0; i < 16; i++) out[i] = static_cast<uint8_t>(st[i / 4] >> (8 * (i % 4)));  // digest may be unaligned
    }
  }
}

// ring depth of the pointer-table form: as many steps in flight as ~200
// VGPRs hold (its 64-bit source pointers take 2K of them), at most 8 -- its
// loads cross PCIe (microseconds each), so small k keeps more steps ahead
template <int K>
constexpr int gm_depth() {
  return (200 - 2 * K) / (4 * K) >= 8 ? 8 : (200 - 2 * K) / (4 * K) < 2 ? 2 : (200 - 2 * K) / (4 * K);
}
// k_files_md5 reads HBM (a step of ~2 us is many load latencies), and its
// last-stripe path needs registers of its own: at most 3 steps in flight,
// 2 from k = 13 (no spills through k = 16); without that path (TAIL = false)
// up to 4 as k_mul_md5, as the 64-bit source pointers leave room (4 through
// k = 11, 3 through 14, then 2)
template <int K, bool TAIL = true>
constexpr int fm_depth() {
  return !TAIL ? (gm_depth<K>() > 4 ? 4 : gm_depth<K>()) : K >= 13 ? 2 : gm_depth<K>() > 3 ? 3 : gm_depth<K>();
}

// The agent's requests (container_manager.cc:221-258 partial encodes and
// agent.cc:240-415 repairs, then the MD5 of every output, agent.cc:342): the
// same code/hash split as k_mul_md5 with every source and output behind a
// per-request pointer, so a batch is coded and hashed straight from and into
// pinned host buffers over PCIe -- no H2D, no D2H, one launch.  Requests are
// few (tens to ~a thousand) and each is one lane's chain, so a workgroup
// usually holds fewer requests than it has code lanes: the idle lanes read
// and write `scratch` in HBM (one address per lane) instead of shadowing a
// live request, which would multiply its PCIe reads.
// HSRC: the sources are hashed too (RSCode::encode's n digests per stripe,
// chunk_manager.cc:175): rows 0..K-1 of a request are its sources, then its
// outputs -- a template parameter for the reason k_mul_md5's is.
template <int K, bool HSRC>
__global__ __launch_bounds__(kEmBlock) void k_gather_md5(const GatherMd5Args a) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int hsrc = HSRC ? K : 0;  // rows before the outputs' rows
  const int nh = hsrc + a.p;
  const int S = a.stripes_per_group;
  uint32_t *tab = reinterpret_cast<uint32_t *>(lds);
  uint8_t *buf = lds + K * 1024;
  const uint32_t buf_bytes = static_cast<uint32_t>(S * nh * kEmRow);
  build_tables<1>(a.coef, K, a.p, tab);
  __syncthreads();
  const int64_t s0 = static_cast<int64_t>(blockIdx.x) * S;
  const int nS = static_cast<int>(min(static_cast<int64_t>(S), a.nstripes - s0));
  // any length: nfull whole steps, then a partial step of `tail` bytes
  const int nfull = static_cast<int>(a.len / kEncMd5Step);
  const int tail = static_cast<int>(a.len - static_cast<int64_t>(nfull) * kEncMd5Step);
  const int nsteps = nfull + (tail > 0);

  if (threadIdx.x < kEmCodeLanes) {
    if ((threadIdx.x & ~63) >= nS * kEmVecs) {  // no live request in this wave: barriers only
      for (int s = 0; s < nsteps; s++) lds_barrier();
      return;
    }
    const int item = threadIdx.x;
    const bool act = item < nS * kEmVecs;
    const int ls = act ? item / kEmVecs : 0, v = item % kEmVecs;
    const int64_t sx = s0 + ls;
    const uint8_t *sp[K];
#pragma unroll
    for (int j = 0; j < K; j++) sp[j] = act ? a.src_ptrs[sx * K + j] + v * 16 : a.scratch + v * 16;
    uint8_t *dp[kMaxRowsPerPass];
#pragma unroll
    for (int r = 0; r < kMaxRowsPerPass; r++)
      dp[r] = act && r < a.p ? a.dst_ptrs[sx * a.p + r] + v * 16 : a.scratch + 256 * (r + 1) + v * 16;
    const int64_t sstep = act ? kEncMd5Step : 0;  // idle lanes stay on their scratch line
    uint8_t *row = buf + ls * nh * kEmRow + v * 16;
    auto load = [&](int step, u32x4(&d)[K]) {
#pragma unroll
      for (int j = 0; j < K; j++) d[j] = dev::ld_global_stream(sp[j] + step * sstep);
    };
    auto run = [&](int step, const u32x4(&d)[K]) {
      uint8_t *rb = row + (step & 1) * buf_bytes;
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        if (HSRC && act) {
          *reinterpret_cast<u32x4 *>(rb + j * kEmRow) = d[j];
          if (j + 1 < K) *reinterpret_cast<u32x4 *>(rb + (j + 1) * kEmRow) = d[j + 1];
        }
        lookup_pair(j, j + 1 < K, d[j], d[j + 1 < K ? j + 1 : j], acc);
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("" : "+v"(acc[i]));
      }
      uint32_t o[4][4];
      rows_of(acc, o);
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++) {
        if (r < a.p) {  // wave-uniform
          const u32x4 pv{o[r][0], o[r][1], o[r][2], o[r][3]};
          dev::st_global_stream(dp[r] + step * sstep, pv);
          if (act) *reinterpret_cast<u32x4 *>(rb + (hsrc + r) * kEmRow) = pv;
        }
      }
      lds_barrier();
    };
    constexpr int D = gm_depth<K>();
    if (nfull > 0) {  // the whole steps through the ring (uniform branch)
      u32x4 ring[D][K];
      const int last = nfull - 1;
#pragma unroll
      for (int j = 0; j < D - 1; j++) load(min(j, last), ring[j]);
      int step = 0;
      for (; step + D <= nfull; step += D) {
#pragma unroll
        for (int j = 0; j < D; j++) {
          load(min(step + j + D - 1, last), ring[(j + D - 1) % D]);
          __builtin_amdgcn_sched_barrier(0);
          run(step + j, ring[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < D - 1; j++) {
        if (step + j < nfull) {
          load(min(step + j + D - 1, last), ring[(j + D - 1) % D]);
          __builtin_amdgcn_sched_barrier(0);
          run(step + j, ring[j]);
        }
      }
    }
    if (tail > 0) {
      // the partial last step: nothing past a chunk's end is read or written
      // (a caller's buffer may end at a page); a lane straddling the end moves
      // its bytes one at a time, lanes past it load zeros and store nothing,
      // so the step's LDS row is zero-padded for the hash lanes
      const int nb = act ? min(max(tail - v * 16, 0), 16) : 16;  // idle lanes: their scratch line
      const int64_t off = static_cast<int64_t>(nfull) * sstep;
      u32x4 d[K];
#pragma unroll
      for (int j = 0; j < K; j++) {
        if (nb == 16) {
          d[j] = dev::ld_global_stream(sp[j] + off);
        } else {
          uint32_t w[4] = {0, 0, 0, 0};
          for (int i = 0; i < nb; i++) w[i / 4] |= static_cast<uint32_t>(sp[j][off + i]) << (8 * (i % 4));
          d[j] = u32x4{w[0], w[1], w[2], w[3]};
        }
      }
      uint8_t *rb = row + (nfull & 1) * buf_bytes;
      if (HSRC && act) {  // zero past the end, as the hash lanes' padding expects
#pragma unroll
        for (int j = 0; j < K; j++) *reinterpret_cast<u32x4 *>(rb + j * kEmRow) = d[j];
      }
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j += 2) lookup_pair(j, j + 1 < K, d[j], d[j + 1 < K ? j + 1 : j], acc);
      uint32_t o[4][4];
      rows_of(acc, o);
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++) {
        if (r < a.p) {
          const u32x4 pv{o[r][0], o[r][1], o[r][2], o[r][3]};
          if (nb == 16) {
            dev::st_global_stream(dp[r] + off, pv);
          } else {
            const uint32_t w[4] = {pv.x, pv.y, pv.z, pv.w};
            for (int i = 0; i < nb; i++) dp[r][off + i] = static_cast<uint8_t>(w[i / 4] >> (8 * (i % 4)));
          }
          if (act) *reinterpret_cast<u32x4 *>(rb + (hsrc + r) * kEmRow) = pv;  // zero past the end: GF products of zeros
        }
      }
      lds_barrier();
    }
    return;
  }

  const int h = threadIdx.x - kEmCodeLanes;
  const bool active = h < nS * nh;
  uint32_t st[4];
  hash_rows<0, true>(buf, buf_bytes, h, active, nsteps, st, tail > 0 ? tail : kEncMd5Step,
                     static_cast<uint64_t>(a.len));
  if (active) {
    uint32_t *out = reinterpret_cast<uint32_t *>(a.digests + (s0 * nh + h) * 16);  // rows are (request, output) in order
#pragma unroll
    for (int i = 0; i < 4; i++) out[i] = st[i];
  }
}

// The multi-file write in one launch (nxec_encode_objects; the per-file
// loop of Proxy::writeFileStripes, proxy_file_ops.cc:557-666, with
// writeFileStripe's encode + Chunk::computeMD5 of all n chunks,
// chunk_manager.cc:66-452): k_mul_md5's code/hash split over pointer tables,
// every request (a full stripe read in place from its object, or a file's
// zero-padded last stripe in the tail arena) with its own chunk length.
//
// Requests are packed into slots (plan_files_slots): a slot is one stripe's
// worth of lanes -- 16 code lanes, k + p hash lanes -- that runs its requests
// back to back.  A batch of 6 000 requests on 256 CUs x 16 slots used to need
// a second wave of workgroups (18.8 ms for 4096 files of 1 B - 20 MiB); with
// the requests spread so that every slot's chains add up to about the
// longest one, it runs in one wave.  Per lane, a cursor (request of the
// slot's list, step inside it) replaces the fixed request: the load cursor
// runs D - 1 steps ahead of the compute cursor through the register ring,
// and at a request boundary a lane takes the next request's pointers from
// the workgroup's request table in LDS (no global load in the loop, so the
// ring's vmcnt bookkeeping is unchanged).  A hash lane finishes its chunk's
// digest at the request's last step (RFC 1321 padding built in registers,
// bytes past the chunk's end masked off) and starts the next chain at once.
// A lane past its request's end in that request's last step re-reads its
// last in-bounds vector, stores to scratch and leaves its LDS row alone.
// PROBE (design probes only, K = 10, NXEC_FM_PROBE; outputs are NOT valid),
// as k_mul_md5's: bit 0 no MD5 rounds, bit 1 no table lookups, bit 2 no
// global loads or stores, bit 3 (alone, 8) no tail-arena stores, bit 4
// (alone, 16) last stripes coded like whole stripes (no tail handling).
// TAIL = false: no request reads a last stripe from its object (a.tail_src is
// null: in place, last stripes are ordinary requests) -- every tail branch,
// its state and its registers compile out of the step loop.  TSTORE (with
// TAIL = false; a.tail_store): last stripes are in-place requests and the
// code lanes also store their whole data chunks to the tail arena.
template <int K, int PROBE = 0, bool TAIL = true, bool TSTORE = false>
__global__ __launch_bounds__(kEmBlock) void k_files_md5(const FilesMd5Args a) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int nh = K + a.p;
  const int S = a.slots_per_group;
  const int L = a.max_list;
  // request record: K sources, p outputs, digest base, length, tail source, tail bytes
  const int rec = K + a.p + 4;
  uint32_t *tab = reinterpret_cast<uint32_t *>(lds);
  uint8_t *buf = lds + K * 1024;
  const uint32_t buf_bytes = static_cast<uint32_t>(S * nh * kEmRow);
  uint64_t *rq = reinterpret_cast<uint64_t *>(buf + 2 * buf_bytes);  // [S][L][rec]
  build_tables<1>(a.coef, K, a.p, tab);
  const int64_t g0 = static_cast<int64_t>(blockIdx.x) * S;
  const int nS = static_cast<int>(min(static_cast<int64_t>(S), a.nslots - g0));
  for (int i = threadIdx.x; i < nS * L * rec; i += kEmBlock) {
    const int ls = i / (L * rec), li = (i / rec) % L, f = i % rec;
    const int first = a.slot_first[g0 + ls], cnt = a.slot_first[g0 + ls + 1] - first;
    uint64_t v = 0;
    if (li < cnt) {
      const int64_t r = a.slot_reqs[first + li];
      if (f < K)
        v = reinterpret_cast<uint64_t>(a.src_ptrs[r * K + f]);
      else if (f < K + a.p)
        v = reinterpret_cast<uint64_t>(a.dst_ptrs[r * a.p + (f - K)]);
      else if (f == K + a.p)
        v = reinterpret_cast<uint64_t>(a.dig_ptrs[r]);
      else if (f == K + a.p + 1)
        v = static_cast<uint64_t>(a.lens[r]);
      else if (f == K + a.p + 2)
        v = a.tail_src ? reinterpret_cast<uint64_t>(a.tail_src[r]) : 0;
      else
        v = a.tail_rem ? static_cast<uint64_t>(a.tail_rem[r]) : 0;
    }
    rq[i] = v;
  }
  __syncthreads();
  if (a.wg_clock && threadIdx.x == 0) a.wg_clock[blockIdx.x * 3] = __builtin_amdgcn_s_memrealtime();
  const int nsteps = a.wg_steps[blockIdx.x];
  auto steps_of = [](int64_t len) { return static_cast<int>((len + kEncMd5Step - 1) / kEncMd5Step); };

  if (threadIdx.x < kEmCodeLanes) {
    if ((threadIdx.x & ~63) >= nS * kEmVecs) {  // no live slot in this wave: barriers only
      for (int s = 0; s < nsteps; s++) lds_barrier();
      return;
    }
    const int item = threadIdx.x;
    const bool act = item < nS * kEmVecs;
    const int ls = act ? item / kEmVecs : 0, v = item % kEmVecs;
    const int cnt = act ? a.slot_first[g0 + ls + 1] - a.slot_first[g0 + ls] : 1;
    const uint64_t *q = rq + static_cast<int64_t>(ls) * L * rec;
    auto len_of = [&](int li) { return act ? static_cast<int64_t>(q[li * rec + K + a.p + 1]) : int64_t(16); };
    // last step with bytes of this lane's 16-byte column (-1: none)
    auto tmax_of = [&](int64_t len) {
      const int64_t vlen = (len + 15) / 16 * 16;
      return vlen > v * 16 ? static_cast<int>((vlen - 1 - v * 16) / kEncMd5Step) : -1;
    };
    // load cursor: request lr of the slot, step lt of it
    int lr = 0, lt = 0;
    int64_t len0 = len_of(0);
    int lT = steps_of(len0), ltcl = max(tmax_of(len0), 0);
    const uint8_t *sp[K];
    // a lane whose column holds no byte of the request (chunks under 256
    // bytes) reads the scratch line: nothing past a chunk's 16-byte padding is read
    // A last stripe read from its object (tail source != 0): data chunk j is
    // tail bytes [j*cl, (j+1)*cl), valid below min((j+1)*cl, rem): `tl` = cl
    // (0 for a full stripe), `jf` = chunks wholly valid, `last` = the valid
    // bytes of chunk jf (32-bit: cl <= 1 GiB), `end` = the end of the tail's
    // last 16-byte line (nothing at or past it is read), `zf` = the first
    // all-zero chunk (read from the zero scratch line, never masked), `jc` =
    // the first chunk whose 16-byte column vectors can run past `end` (only
    // chunks jc..zf-1 are clamped when loaded and, in place, shifted / masked
    // when computed: below jc a vector past the chunk's own end reads the next
    // chunk's bytes, which only reach parity bytes past cl -- outside the
    // parity chunk -- and row bytes the hash lanes mask off)
    auto tail_state = [&](int li, int64_t cl, uint32_t &tl, uint32_t &jf, uint32_t &last, const uint8_t *&end,
                          uint32_t &jc, uint32_t &zf) {
      const uint64_t tb = TAIL && act ? q[li * rec + K + a.p + 2] : uint64_t(0);
      const int64_t rem = TAIL && act ? static_cast<int64_t>(q[li * rec + K + a.p + 3]) : int64_t(0);
      const int64_t f = tb && cl > 0 ? min(rem / cl, static_cast<int64_t>(K)) : 0;
      tl = tb ? static_cast<uint32_t>(cl) : 0u;
      jf = static_cast<uint32_t>(f);
      last = f < K && tb ? static_cast<uint32_t>(rem - f * cl) : 0u;
      end = reinterpret_cast<const uint8_t *>((tb + static_cast<uint64_t>(rem) + 15) & ~uint64_t(15));
      const int64_t cls = (cl + 15) / 16 * 16;
      zf = tb ? static_cast<uint32_t>(f < K ? f + (last ? 1 : 0) : K) : static_cast<uint32_t>(K);
      jc = tb ? static_cast<uint32_t>(rem >= cls && cl > 0 ? min((rem - cls) / cl + 1, static_cast<int64_t>(K)) : 0)
              : static_cast<uint32_t>(K);
    };
    auto valid_of = [](int j, uint32_t tl, uint32_t jf, uint32_t last) {
      return static_cast<int32_t>(static_cast<uint32_t>(j) < jf ? tl : static_cast<uint32_t>(j) == jf ? last : 0u);
    };
    // source pointers of the lane's column: a full stripe's chunks, a tail's
    // object bytes (at any byte), or -- a lane whose column holds no byte of
    // the request (chunks under 256 bytes) -- the scratch line: nothing past a
    // chunk's 16-byte padding is read
    auto set_src = [&](int li, bool has) {
      const uint64_t tb = TAIL && act ? q[li * rec + K + a.p + 2] : uint64_t(0);
      const int64_t cl = len_of(li);
#pragma unroll
      for (int j = 0; j < K; j++)
        sp[j] = act && has ? (tb ? reinterpret_cast<const uint8_t *>(tb) + j * cl
                                 : reinterpret_cast<const uint8_t *>(q[li * rec + j])) + v * 16
                           : a.scratch + v * 16;
    };
    set_src(0, tmax_of(len0) >= 0);
    uint32_t ltl, ljf, llast, ljc, lzf;
    const uint8_t *lend;
    tail_state(0, len0, ltl, ljf, llast, lend, ljc, lzf);
    auto load = [&](u32x4(&d)[K]) {
      const int64_t off = static_cast<int64_t>(min(lt, ltcl)) * kEncMd5Step;
      const bool wtl = TAIL && !(PROBE & 16) && __builtin_amdgcn_ballot_w64(ltl != 0) != 0;  // wave-uniform: skip in full-stripe waves
#pragma unroll
      for (int j = 0; j < K; j++) {
        // a tail chunk's 16 bytes are read where they lie (global loads take
        // any byte address), except where they would run past the tail's
        // last 16-byte line: that lane reads the aligned line holding its
        // first byte (the compute step shifts it into place), or the scratch
        // line once nothing of the tail is left
        const uint8_t *pj = sp[j] + off;
        if (wtl && ltl && static_cast<uint32_t>(j) >= ljc) {  // the few chunks that reach the tail's end
          if (static_cast<uint32_t>(j) >= lzf)
            pj = a.scratch + v * 16;  // all zero
          else
            pj = pj + 16 <= lend ? pj
                 : pj < lend     ? reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(pj) & ~uintptr_t(15))
                                 : a.scratch + v * 16;
        }
        // plain (cached) loads: a chunk that is not 128-byte aligned (an
        // object at any 16-byte offset, a tail at any byte) shares its
        // boundary lines between consecutive steps; streaming loads fetched
        // them once per step
        if (PROBE & 4)  // no HBM traffic: a value the compiler cannot fold
          d[j] = u32x4{static_cast<uint32_t>(reinterpret_cast<uintptr_t>(pj)), static_cast<uint32_t>(lt),
                       static_cast<uint32_t>(j), static_cast<uint32_t>(v)};
        else if (a.cached_loads)
          d[j] = dev::ld_global(pj);
        else
          d[j] = dev::ld_global_stream(pj);
      }
      if (++lt == lT) {
        if (lr + 1 < cnt) {  // next request of the slot (pointers from the LDS table)
          lr++;
          lt = 0;
          const int64_t ln = len_of(lr);
          lT = steps_of(ln);
          ltcl = max(tmax_of(ln), 0);
          set_src(lr, tmax_of(ln) >= 0);
          tail_state(lr, ln, ltl, ljf, llast, lend, ljc, lzf);
        } else {
          lt = lT - 1;  // past the slot's end: re-read the last step
        }
      }
    };
    // compute cursor
    int cr = 0, ct = 0, cT = lT, ctmax = act ? tmax_of(len0) : -1;
    bool live = act;
    uint32_t ctl = ltl, cjf = ljf, clast = llast, cjc = ljc, czf = lzf;
    const uint8_t *cend = lend;
    // the tail source and the tail arena's chunk 0 (chunk j at + j*cls), kept
    // in registers: no per-step read of the request table
    const uint8_t *ctb = TAIL && act ? reinterpret_cast<const uint8_t *>(q[K + a.p + 2]) : nullptr;
    uint8_t *ctd = TAIL && act ? reinterpret_cast<uint8_t *>(q[0]) : nullptr;
    uint8_t *dp[kMaxRowsPerPass];
    auto set_dst = [&](int li) {
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++)
        dp[r] = act && r < a.p ? reinterpret_cast<uint8_t *>(q[li * rec + K + r]) + v * 16 : a.scratch;
    };
    set_dst(0);
    // a tail chunk's 16 bytes at column v of step ct, at the chunk's valid end
    // (the lane's bytes run past it): a lane whose load was the aligned line
    // holding its first byte shifts that line into place, then every byte
    // from the valid end on is zeroed (the reference's zero padding)
    auto tail_end = [&](int j, u32x4 x, int32_t nv) {
      const int32_t pos = ct * kEncMd5Step + v * 16;
      const uint8_t *addr = ctb + static_cast<int64_t>(j) * ctl + pos;
      if (addr + 16 > cend) {
        const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(addr)) & 15u, qd = sh >> 2, rb = sh & 3u;
        const uint32_t w[8] = {x.x, x.y, x.z, x.w, 0u, 0u, 0u, 0u};
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t lo = (qd & 2u) ? ((qd & 1u) ? w[i + 3] : w[i + 2]) : ((qd & 1u) ? w[i + 1] : w[i]);
          const uint32_t up = (qd & 2u) ? ((qd & 1u) ? w[i + 4] : w[i + 3]) : ((qd & 1u) ? w[i + 2] : w[i + 1]);
          o[i] = __builtin_amdgcn_alignbyte(up, lo, rb);
        }
        x = u32x4{o[0], o[1], o[2], o[3]};
      }
      const int32_t n = max(nv, 0);
      uint32_t m[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int keep = n - 4 * i;
        m[i] = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
      }
      return u32x4{x.x & m[0], x.y & m[1], x.z & m[2], x.w & m[3]};
    };
    uint8_t *row = buf + ls * nh * kEmRow + v * 16;
    // TSTORE: the compute request's tail slot 0 (nullptr: a full stripe), slot
    // stride, whole chunks stored (j < sj0) and its chunk length
    uint8_t *std_ = nullptr;
    int64_t scls = 0;
    int32_t sj0 = 0, scl = 0;
    auto set_store = [&](int li) {
      if (!TSTORE) return;
      std_ = act ? reinterpret_cast<uint8_t *>(q[li * rec + K + a.p + 2]) : nullptr;
      const uint64_t w = act ? q[li * rec + K + a.p + 3] : 0;
      scls = static_cast<int64_t>(w & ((uint64_t(1) << 40) - 1));
      sj0 = static_cast<int32_t>(w >> 40);
      scl = static_cast<int32_t>(len_of(li));
    };
    set_store(0);
    auto run = [&](int step, const u32x4(&d)[K]) {
      const bool ok = live && ct <= ctmax;
      // wave-uniform: only waves holding a last stripe store
      const bool wst = TSTORE && __builtin_amdgcn_ballot_w64(ok && std_ != nullptr) != 0;
      const bool tl = live && ctl != 0;
      const bool wtc = TAIL && !(PROBE & 16) && __builtin_amdgcn_ballot_w64(tl) != 0;  // wave-uniform: skip in full-stripe waves
      if (wtc) {
        // wait for this step's loads here, in uniform control flow: a first
        // use inside the per-lane tail branches below would be counted
        // conservatively (vmcnt(0)) and drain the loads of the steps ahead
#pragma unroll
        for (int j = 0; j < K; j++) asm volatile("" ::"v"(d[j].x), "v"(d[j].y), "v"(d[j].z), "v"(d[j].w));
      }
      uint8_t *rb = row + (step & 1) * buf_bytes;
      const int32_t pos = ct * kEncMd5Step + v * 16;
      const int64_t cls = (static_cast<int64_t>(ctl) + 15) / 16 * 16;
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        const int j1 = j + 1 < K ? j + 1 : j;
        u32x4 x0 = d[j], x1 = d[j1];
        if (wtc && tl) {
          const int32_t nv0 = valid_of(j, ctl, cjf, clast) - pos, nv1 = valid_of(j1, ctl, cjf, clast) - pos;
          // shift / mask only where it matters: chunks jc..zf-1 (zero chunks
          // were read as zeros); in copy mode also every chunk's last vector,
          // whose bytes past cl go to the tail arena and must be zero
          const bool m0 = static_cast<uint32_t>(j) < czf && (static_cast<uint32_t>(j) >= cjc || !a.tail_partial_only);
          const bool m1 = static_cast<uint32_t>(j1) < czf && (static_cast<uint32_t>(j1) >= cjc || !a.tail_partial_only);
          if (nv0 < 16 && m0) x0 = tail_end(j, x0, nv0);
          if (nv1 < 16 && m1) x1 = tail_end(j1, x1, nv1);
          if (ok) {  // the zero-padded data chunks into the tail arena (in place: only the partial one)
            const bool part0 = j == static_cast<int>(cjf) && clast != 0, part1 = j1 == static_cast<int>(cjf) && clast != 0;
            if (!(PROBE & 12) && (!a.tail_partial_only || part0)) dev::st_global_stream(ctd + j * cls + pos, x0);
            if (!(PROBE & 12) && j + 1 < K && (!a.tail_partial_only || part1))
              dev::st_global_stream(ctd + j1 * cls + pos, x1);
          }
        }
        if (ok) {  // past a request's end its row is left as is: the hash lanes mask it
          *reinterpret_cast<u32x4 *>(rb + j * kEmRow) = x0;
          if (j + 1 < K) *reinterpret_cast<u32x4 *>(rb + (j + 1) * kEmRow) = x1;
        }
        if (wst && ok && std_) {  // whole chunks to the tail arena, zero past the chunk's end
          const int32_t nv = scl - pos;
          uint32_t m[4];
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int keep = nv - 4 * i;
            m[i] = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
          }
          if (j < sj0)
            dev::st_global_stream(std_ + j * scls + pos, u32x4{x0.x & m[0], x0.y & m[1], x0.z & m[2], x0.w & m[3]});
          if (j + 1 < K && j + 1 < sj0)
            dev::st_global_stream(std_ + (j + 1) * scls + pos, u32x4{x1.x & m[0], x1.y & m[1], x1.z & m[2], x1.w & m[3]});
        }
        if (PROBE & 2) {
          if (j == 0) acc[0] = x0.x, acc[5] = x0.y, acc[10] = x0.z, acc[15] = x0.w;
        } else {
          lookup_pair(j, j + 1 < K, x0, x1, acc);
        }
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("" : "+v"(acc[i]));
      }
      uint32_t o[4][4];
      rows_of(acc, o);
      const int64_t off = static_cast<int64_t>(ct) * kEncMd5Step;
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++) {
        if (r < a.p) {  // wave-uniform
          const u32x4 pv{o[r][0], o[r][1], o[r][2], o[r][3]};
          if (!(PROBE & 4)) dev::st_global_stream(ok ? dp[r] + off : a.scratch + 256 * (r + 1) + v * 16, pv);
          if (ok) *reinterpret_cast<u32x4 *>(rb + (K + r) * kEmRow) = pv;
        }
      }
      lds_barrier();
      if (live && ++ct == cT) {
        if (cr + 1 < cnt) {
          cr++;
          ct = 0;
          const int64_t ln = len_of(cr);
          cT = steps_of(ln);
          ctmax = tmax_of(ln);
          set_dst(cr);
          tail_state(cr, ln, ctl, cjf, clast, cend, cjc, czf);
          if (TAIL) {
            ctb = reinterpret_cast<const uint8_t *>(q[cr * rec + K + a.p + 2]);
            ctd = reinterpret_cast<uint8_t *>(q[cr * rec]);
          }
          set_store(cr);
        } else {
          live = false;
        }
      }
    };
    constexpr int D = fm_depth<K, TAIL>();
    u32x4 ring[D][K];
#pragma unroll
    for (int j = 0; j < D - 1; j++) load(ring[j]);
    int step = 0;
    for (; step + D <= nsteps; step += D) {
#pragma unroll
      for (int j = 0; j < D; j++) {
        load(ring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run(step + j, ring[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < D - 1; j++) {
      if (step + j < nsteps) {
        load(ring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run(step + j, ring[j]);
      }
    }
    if (a.wg_clock && threadIdx.x == 0) a.wg_clock[blockIdx.x * 3 + 1] = __builtin_amdgcn_s_memrealtime();
    return;
  }

  // ---- hash lanes: lane h = chunk c of slot ls = LDS row h; one chain per request of the slot ----
  const int h = threadIdx.x - kEmCodeLanes;
  const bool active = h < nS * nh;
  const int ls = active ? h / nh : 0, c = active ? h - (h / nh) * nh : 0;
  const int cnt = active ? a.slot_first[g0 + ls + 1] - a.slot_first[g0 + ls] : 0;
  const uint64_t *q = rq + static_cast<int64_t>(ls) * L * rec;
  int hr = 0, ht = 0;
  int64_t hlen = active ? static_cast<int64_t>(q[K + a.p + 1]) : 1;
  int hT = steps_of(hlen);
  bool live = active;
  uint32_t st[4];
  md5_init(st);
  const u32x4 *rowp = reinterpret_cast<const u32x4 *>(buf + h * kEmRow);
  auto fetch = [&](int step, uint32_t(&m)[kEncMd5Step / 4]) {
    const u32x4 *p = rowp + (step & 1) * (buf_bytes / 16);
#pragma unroll
    for (int i = 0; i < kEmVecs; i++) {
      const u32x4 x = p[i];
      m[4 * i] = x.x;
      m[4 * i + 1] = x.y;
      m[4 * i + 2] = x.z;
      m[4 * i + 3] = x.w;
    }
  };
  auto proc = [&](const uint32_t(&m)[kEncMd5Step / 4]) {
    if (!live) return;
    if (ht < hT - 1) {
      if (PROBE & 1) {
#pragma unroll
        for (int i = 0; i < kEncMd5Step / 4; i++) st[i & 3] ^= m[i];
      } else {
#pragma unroll
        for (int b = 0; b < kEncMd5Step / 64; b++) md5_block(st, m + 16 * b);
      }
      ht++;
      return;
    }
    // the request's last step: its tail bytes, then RFC 1321 §3.1-3.2 padding
    const int my_tail = static_cast<int>(hlen - static_cast<int64_t>(hT - 1) * kEncMd5Step);
    const int fb = my_tail / 64, r = my_tail % 64;
#pragma unroll
    for (int b = 0; b < kEncMd5Step / 64; b++)
      if (b < fb) md5_block(st, m + 16 * b);
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < kEncMd5Step / 64; b++)
        if (b == fb) x = m[16 * b + i];
      // keep the word's bytes below r, then the 0x80 terminator
      const int keep = r - 4 * i;  // bytes of this word inside the chunk
      const uint32_t mask = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
      w[i] = (x & mask) | (i == r / 4 ? 0x80u << (8 * (r % 4)) : 0u);
    }
    const uint64_t bits = static_cast<uint64_t>(hlen) * 8;
    if (r >= 56) {
      md5_block(st, w);
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = 0;
    }
    w[14] = static_cast<uint32_t>(bits);
    w[15] = static_cast<uint32_t>(bits >> 32);
    md5_block(st, w);
    // a global (not flat) store: the digest may be unaligned
    typedef __attribute__((address_space(1))) uint8_t g_u8;
    g_u8 *out = reinterpret_cast<g_u8 *>(q[hr * rec + K + a.p] + static_cast<uint64_t>(c) * 16);
#pragma unroll
    for (int i = 0; i < 16; i++) out[i] = static_cast<uint8_t>(st[i / 4] >> (8 * (i % 4)));
    md5_init(st);
    if (hr + 1 < cnt) {
      hr++;
      ht = 0;
      hlen = static_cast<int64_t>(q[hr * rec + K + a.p + 1]);
      hT = steps_of(hlen);
    } else {
      live = false;
    }
  };
  uint32_t m0[kEncMd5Step / 4], m1[kEncMd5Step / 4];
  lds_barrier();
  if (active) fetch(0, m0);
  int step = 1;
  for (; step + 2 <= nsteps; step += 2) {
    lds_barrier();
    if (active) fetch(step, m1);
    proc(m0);
    lds_barrier();
    if (active) fetch(step + 1, m0);
    proc(m1);
  }
  if (step < nsteps) {
    lds_barrier();
    if (active) fetch(step, m1);
    proc(m0);
    proc(m1);
  } else {
    proc(m0);
  }
  if (a.wg_clock && threadIdx.x == kEmCodeLanes) a.wg_clock[blockIdx.x * 3 + 2] = __builtin_amdgcn_s_memrealtime();
}

using FmKernel = void (*)(const FilesMd5Args);
template <int... Ks>
constexpr std::array<FmKernel, sizeof...(Ks)> fm_table(std::integer_sequence<int, Ks...>) {
  return {{&k_files_md5<Ks + 1>...}};
}
const std::array<FmKernel, kFilesMd5MaxK> kFm = fm_table(std::make_integer_sequence<int, kFilesMd5MaxK>{});
template <int... Ks>
constexpr std::array<FmKernel, sizeof...(Ks)> fm_table_nt(std::integer_sequence<int, Ks...>) {
  return {{&k_files_md5<Ks + 1, 0, false>...}};
}
// no request with a tail source (in place): the tail-free step loop
const std::array<FmKernel, kFilesMd5MaxK> kFmNt = fm_table_nt(std::make_integer_sequence<int, kFilesMd5MaxK>{});
template <int... Ks>
constexpr std::array<FmKernel, sizeof...(Ks)> fm_table_st(std::integer_sequence<int, Ks...>) {
  return {{&k_files_md5<Ks + 1, 0, false, true>...}};
}
// in-place requests that also store last stripes' whole chunks to the tail arena
const std::array<FmKernel, kFilesMd5MaxK> kFmSt = fm_table_st(std::make_integer_sequence<int, kFilesMd5MaxK>{});
#if NXEC_DESIGN_PROBES
// bit 3 alone: no tail-arena stores (everything else as the product);
// bit 4 alone: last stripes read straight from the object like whole
// stripes, no clamps, masks or tail stores (timing only)
const FmKernel kFmProbe8 = &k_files_md5<10, 8>;
const FmKernel kFmProbe16 = &k_files_md5<10, 16>;
const FmKernel kFmProbe[8] = {&k_files_md5<10, 0>, &k_files_md5<10, 1>, &k_files_md5<10, 2>, &k_files_md5<10, 3>,
                              &k_files_md5<10, 4>, &k_files_md5<10, 5>, &k_files_md5<10, 6>, &k_files_md5<10, 7>};
#endif

using GmKernel = void (*)(const GatherMd5Args);
template <bool HSRC, int... Ks>
constexpr std::array<GmKernel, sizeof...(Ks)> gm_table(std::integer_sequence<int, Ks...>) {
  return {{&k_gather_md5<Ks + 1, HSRC>...}};
}
// [hash_src][k - 1]
const std::array<GmKernel, kGatherMd5MaxK> kGm[2] = {gm_table<false>(std::make_integer_sequence<int, kGatherMd5MaxK>{}),
                                                     gm_table<true>(std::make_integer_sequence<int, kGatherMd5MaxK>{})};

using EmKernel = void (*)(const MulMd5Args);
template <bool HSRC, int... Ks>
constexpr std::array<EmKernel, sizeof...(Ks)> em_table(std::integer_sequence<int, Ks...>) {
  return {{&k_mul_md5<Ks + 1, HSRC>...}};
}
// [hash_src][k - 1]
const std::array<EmKernel, kEncMd5MaxK> kEm[2] = {em_table<false>(std::make_integer_sequence<int, kEncMd5MaxK>{}),
                                                  em_table<true>(std::make_integer_sequence<int, kEncMd5MaxK>{})};

#if NXEC_DESIGN_PROBES
const EmKernel kEmNib = &k_mul_md5<10, true, 0, true>;
const EmKernel kEmHg = &k_mul_md5<10, true, 0, false, true>;
const EmKernel kEmProbe[8] = {&k_mul_md5<10, true, 0>, &k_mul_md5<10, true, 1>, &k_mul_md5<10, true, 2>,
                              &k_mul_md5<10, true, 3>, &k_mul_md5<10, true, 4>, &k_mul_md5<10, true, 5>,
                              &k_mul_md5<10, true, 6>, &k_mul_md5<10, true, 7>};
#endif

}  // namespace

bool mul_md5_eligible(int k, int rows, int64_t len, const void *src, int64_t src_stripe_stride, const uint32_t *src_off,
                      const void *dst, int64_t dst_stripe_stride, const uint32_t *dst_off, const uint32_t *copy_off) {
  if (k < 1 || k > kEncMd5MaxK || rows < 0 || rows > kMaxRowsPerPass) return false;
  if (len <= 0 || len % kEncMd5Step != 0 || len / kEncMd5Step >= (int64_t(1) << 31)) return false;
  if (const char *e = std::getenv("NXEC_FUSED_MD5"))
    if (e[0] == '0') return false;  // A/B: two kernels (coding, then MD5)
  uint64_t bits = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) |
                  static_cast<uint64_t>(src_stripe_stride) | static_cast<uint64_t>(dst_stripe_stride);
  for (int j = 0; j < k; j++) bits |= src_off[j];
  for (int r = 0; r < rows; r++) bits |= dst_off[r];
  if (copy_off)
    for (int j = 0; j < k; j++)
      if (copy_off[j] != kNoCopy) bits |= copy_off[j];
  return (bits & 15) == 0;
}

int prepare_encode_md5() {
  for (int i = 0; i < 2 * kEncMd5MaxK; i++) {
    const EmKernel fn = kEm[i / kEncMd5MaxK][i % kEncMd5MaxK];
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(fn)) != hipSuccess || fa.sharedSizeBytes != 0)
      return set_error(NXEC_ERR_HIP, "k_mul_md5: static LDS present (the tables must start at LDS byte 0)");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_mul_md5): %s", hipGetErrorString(e));
  }
  std::vector<FmKernel> fms(kFm.begin(), kFm.end());
  fms.insert(fms.end(), kFmNt.begin(), kFmNt.end());
  fms.insert(fms.end(), kFmSt.begin(), kFmSt.end());
  for (FmKernel fn : fms) {
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(fn)) != hipSuccess || fa.sharedSizeBytes != 0)
      return set_error(NXEC_ERR_HIP, "k_files_md5: static LDS present (the tables must start at LDS byte 0)");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_files_md5): %s", hipGetErrorString(e));
  }
  for (GmKernel fn : kGm[0]) {
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(fn)) != hipSuccess || fa.sharedSizeBytes != 0)
      return set_error(NXEC_ERR_HIP, "k_gather_md5: static LDS present (the tables must start at LDS byte 0)");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_gather_md5): %s", hipGetErrorString(e));
  }
  for (GmKernel fn : kGm[1]) {
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(fn)) != hipSuccess || fa.sharedSizeBytes != 0)
      return set_error(NXEC_ERR_HIP, "k_gather_md5: static LDS present (the tables must start at LDS byte 0)");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_gather_md5): %s", hipGetErrorString(e));
  }
#if NXEC_DESIGN_PROBES
  for (FmKernel fn : {kFmProbe[0], kFmProbe[1], kFmProbe[2], kFmProbe[3], kFmProbe[4], kFmProbe[5], kFmProbe[6],
                      kFmProbe[7], kFmProbe8, kFmProbe16}) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_files_md5 probe): %s", hipGetErrorString(e));
  }
  {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kEmNib), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_mul_md5 nib): %s", hipGetErrorString(e));
    e = hipFuncSetAttribute(reinterpret_cast<const void *>(kEmHg), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_mul_md5 hg): %s", hipGetErrorString(e));
  }
  for (EmKernel fn : kEmProbe) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_mul_md5 probe): %s", hipGetErrorString(e));
  }
#endif
  return NXEC_OK;
}

int launch_mul_md5(const MulMd5Args &in, int num_cus, void *stream) {
  if (in.nstripes <= 0) return NXEC_OK;
  MulMd5Args a = in;
  a.nhashed = (a.hash_src ? a.k : 0) + (a.hash_dst ? a.p : 0);
  if (a.nhashed < 1) return set_error(NXEC_ERR_INVALID, "mul+md5: nothing to hash");
  const int n = a.nhashed;
  // as many stripes per workgroup as its 256 hash lanes and code lanes hold,
  // but spread over every CU first (each chain is ~9 ms of one lane whatever
  // the batch: fewer stripes per CU means shorter code steps, not shorter chains)
  int64_t S = std::min(kEmMaxStripes, kEmMaxRows / n);  // n: hashed chunks per stripe
  const int64_t per_cu = (a.nstripes + std::max(num_cus, 1) - 1) / std::max(num_cus, 1);
  if (per_cu < S) S = per_cu;
  if (const char *e = std::getenv("NXEC_EM_S"))  // tuning only: stripes per workgroup
    S = std::max<int64_t>(1, std::min<int64_t>(std::atoi(e), std::min(kEmMaxStripes, kEmMaxRows / n)));
  a.stripes_per_group = static_cast<int32_t>(S);
  a.hash_prio = 0;
  if (const char *e = std::getenv("NXEC_EM_PRIO")) a.hash_prio = std::atoi(e);
  const int64_t grid = (a.nstripes + S - 1) / S;
  if (grid >= (int64_t(1) << 31)) return set_error(NXEC_ERR_INVALID, "encode+md5: batch too large for one launch");
  int lds = a.k * 1024 + static_cast<int>(2 * S * n * kEmRow);
  EmKernel fn = kEm[a.hash_src ? 1 : 0][a.k - 1];
#if NXEC_DESIGN_PROBES
  if (const char *e = std::getenv("NXEC_EM_PROBE"))
    if (a.k == 10 && a.hash_src) fn = kEmProbe[std::atoi(e) & 7];
  // A/B: conflict-free split-nibble tables (k = 10, sources hashed; 40 KiB of tables)
  if (const char *e = std::getenv("NXEC_EM_TABLES"))
    if (e[0] == 'n' && a.k == 10 && a.hash_src && 10 * 4096 + 2 * S * n * kEmRow <= kEmLds) {
      fn = kEmNib;
      lds = 10 * 4096 + static_cast<int>(2 * S * n * kEmRow);
    }
  // A/B: hash lanes read the source chunks from global memory (only the
  // outputs' rows in LDS; k = 10, sources hashed, full-output copies off)
  if (const char *e = std::getenv("NXEC_EM_HASHSRC"))
    if (e[0] == 'g' && a.k == 10 && a.hash_src && a.hash_dst && !a.any_copy && !a.ok) {
      fn = kEmHg;
      lds = 10 * 1024 + static_cast<int>(2 * S * a.p * kEmRow);
    }
#endif
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(kEmBlock), lds,
                     static_cast<hipStream_t>(stream), a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : set_error(NXEC_ERR_HIP, "launch k_mul_md5: %s", hipGetErrorString(e));
}

void plan_files_slots(const std::vector<int64_t> &lens, int k, int p, int num_cus, std::vector<int32_t> &slot_first,
                      std::vector<int32_t> &slot_reqs, std::vector<int32_t> &wg_steps, FilesMd5Args &a) {
  const int nh = k + p;
  const int64_t R = static_cast<int64_t>(lens.size());
  const int64_t Smax = std::min(kEmMaxStripes, kEmMaxRows / nh);
  const int64_t cus = std::max(num_cus, 1);
  const char *pe = std::getenv("NXEC_FILES_PACK");
  const bool pack = !(pe && pe[0] == '0');
  auto steps = [](int64_t len) { return (len + kEncMd5Step - 1) / kEncMd5Step; };
  // at most one workgroup per CU (its LDS), so 256 x Smax slots in one wave:
  // fewer requests than that get a slot each, spread over every CU first
  int64_t G, S;
  if (!pack || R <= cus * Smax) {
    G = R;
    S = std::min<int64_t>(Smax, (R + cus - 1) / cus);
  } else {
    G = cus * Smax;
    S = Smax;
  }
  S = std::max<int64_t>(S, 1);
  const int64_t lds_free = kEmLds - int64_t(k) * 1024 - 2 * S * nh * kEmRow;
  const int64_t Lmax = std::max<int64_t>(1, lds_free / (S * (k + p + 4) * 8));
  // slot of every request; loads and list lengths per slot
  std::vector<int32_t> slot_of(static_cast<size_t>(R));
  std::vector<int64_t> load(static_cast<size_t>(G), 0);
  std::vector<int32_t> cnt(static_cast<size_t>(G), 0);
  // longest request first into the least loaded slot (LPT; ties: lowest
  // slot).  The requests come longest first, so the first G of them land one
  // per empty slot in order; the rest go through a heap of (load, slot).  A
  // slot whose list fills the LDS request table takes no more; when every
  // slot is full a new one opens (a second wave of workgroups).
  const int64_t first = std::min(R, G);
  for (int64_t r = 0; r < first; r++) {
    slot_of[static_cast<size_t>(r)] = static_cast<int32_t>(r);
    load[static_cast<size_t>(r)] = steps(lens[static_cast<size_t>(r)]);
    cnt[static_cast<size_t>(r)] = 1;
  }
  if (R > G) {
    typedef std::pair<int64_t, int64_t> Item;  // (load, slot); a min-heap via std::greater
    std::vector<Item> heap;
    heap.reserve(static_cast<size_t>(G));
    for (int64_t g = 0; g < G; g++)
      if (cnt[static_cast<size_t>(g)] < Lmax) heap.push_back(Item(load[static_cast<size_t>(g)], g));
    std::make_heap(heap.begin(), heap.end(), std::greater<Item>());
    for (int64_t r = G; r < R; r++) {
      int64_t g = -1;
      if (!heap.empty()) {
        std::pop_heap(heap.begin(), heap.end(), std::greater<Item>());
        g = heap.back().second;
        heap.pop_back();
      } else {
        g = static_cast<int64_t>(load.size());
        load.push_back(0);
        cnt.push_back(0);
      }
      slot_of[static_cast<size_t>(r)] = static_cast<int32_t>(g);
      load[static_cast<size_t>(g)] += steps(lens[static_cast<size_t>(r)]);
      if (++cnt[static_cast<size_t>(g)] < Lmax) {  // full slots leave the heap for good
        heap.push_back(Item(load[static_cast<size_t>(g)], g));
        std::push_heap(heap.begin(), heap.end(), std::greater<Item>());
      }
    }
    G = static_cast<int64_t>(load.size());
  }
  // slot lists in request order (a counting sort by slot)
  slot_first.assign(static_cast<size_t>(G) + 1, 0);
  int64_t maxl = 1;
  for (int64_t g = 0; g < G; g++) {
    slot_first[static_cast<size_t>(g) + 1] = slot_first[static_cast<size_t>(g)] + cnt[static_cast<size_t>(g)];
    maxl = std::max<int64_t>(maxl, cnt[static_cast<size_t>(g)]);
  }
  slot_reqs.assign(static_cast<size_t>(R), 0);
  {
    std::vector<int32_t> fill(slot_first.begin(), slot_first.end() - 1);
    for (int64_t r = 0; r < R; r++) slot_reqs[static_cast<size_t>(fill[static_cast<size_t>(slot_of[static_cast<size_t>(r)])]++)] = static_cast<int32_t>(r);
  }
  const int64_t nwg = (G + S - 1) / S;
  wg_steps.assign(static_cast<size_t>(nwg), 0);
  for (int64_t g = 0; g < G; g++) {
    int32_t &w = wg_steps[static_cast<size_t>(g / S)];
    w = std::max<int32_t>(w, static_cast<int32_t>(load[static_cast<size_t>(g)]));
  }
  a.nslots = G;
  a.slots_per_group = static_cast<int32_t>(S);
  a.max_list = static_cast<int32_t>(maxl);
}

int launch_files_md5(const FilesMd5Args &in, int num_cus, void *stream) {
  if (in.nslots <= 0) return NXEC_OK;
  if (in.k < 1 || in.k > kFilesMd5MaxK || in.p < 1 || in.p > kMaxRowsPerPass || !in.src_ptrs || !in.dst_ptrs ||
      !in.lens || !in.dig_ptrs || !in.scratch || !in.slot_first || !in.slot_reqs || !in.wg_steps ||
      in.slots_per_group < 1 || in.max_list < 1)
    return set_error(NXEC_ERR_INVALID, "files+md5: unsupported arguments");
  FilesMd5Args a = in;
  a.cached_loads = 1;  // FETCH x2 60.0 -> 43.6 GB per 4096-file batch (= the data bytes), same time
  if (const char *e = std::getenv("NXEC_FILES_LOADS")) a.cached_loads = e[0] != '0';
  (void)num_cus;
  const int nh = a.k + a.p;
  const int64_t S = a.slots_per_group;
  if (S * nh > kEmMaxRows || S * kEmVecs > kEmCodeLanes)
    return set_error(NXEC_ERR_INVALID, "files+md5: %lld slots of %d chunks per workgroup", static_cast<long long>(S), nh);
  const int64_t grid = (a.nslots + S - 1) / S;
  if (grid >= (int64_t(1) << 31)) return set_error(NXEC_ERR_INVALID, "files+md5: batch too large for one launch");
  const int64_t lds = int64_t(a.k) * 1024 + 2 * S * nh * kEmRow + S * a.max_list * (a.k + a.p + 4) * 8;
  if (lds > kEmLds) return set_error(NXEC_ERR_INVALID, "files+md5: request table does not fit the LDS");
  FmKernel fn = a.tail_store ? kFmSt[a.k - 1] : a.tail_src ? kFm[a.k - 1] : kFmNt[a.k - 1];
  if (a.tail_store && (!a.tail_src || !a.tail_rem)) return set_error(NXEC_ERR_INVALID, "files+md5: tail-store tables");
#if NXEC_DESIGN_PROBES
  if (const char *e = std::getenv("NXEC_FM_PROBE"))
    if (a.k == 10)
      fn = std::atoi(e) == 8 ? kFmProbe8 : std::atoi(e) == 16 ? kFmProbe16 : kFmProbe[std::atoi(e) & 7];
#endif
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(kEmBlock), static_cast<unsigned>(lds),
                     static_cast<hipStream_t>(stream), a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : set_error(NXEC_ERR_HIP, "launch k_files_md5: %s", hipGetErrorString(e));
}

int launch_gather_md5(const GatherMd5Args &in, int num_cus, void *stream) {
  if (in.nstripes <= 0) return NXEC_OK;
  if (in.k < 1 || in.k > kGatherMd5MaxK || in.p < 1 || in.p > kMaxRowsPerPass || in.len <= 0 ||
      in.len / kEncMd5Step >= (int64_t(1) << 31) - 1 || !in.src_ptrs || !in.dst_ptrs || !in.digests || !in.scratch)
    return set_error(NXEC_ERR_INVALID, "gather+md5: unsupported arguments");
  GatherMd5Args a = in;
  const int nh = (a.hash_src ? a.k : 0) + a.p;  // hashed chunks per request
  // spread the requests over every CU first (each is one ~9 ms chain per
  // 1 MiB whatever the batch), then pack up to 16 per workgroup
  int64_t S = std::min(kEmMaxStripes, kEmMaxRows / nh);
  const int64_t per_cu = (a.nstripes + std::max(num_cus, 1) - 1) / std::max(num_cus, 1);
  if (per_cu < S) S = per_cu;
  a.stripes_per_group = static_cast<int32_t>(S);
  const int64_t grid = (a.nstripes + S - 1) / S;
  if (grid >= (int64_t(1) << 31)) return set_error(NXEC_ERR_INVALID, "gather+md5: batch too large for one launch");
  const int lds = a.k * 1024 + static_cast<int>(2 * S * nh * kEmRow);
  hipLaunchKernelGGL(kGm[a.hash_src ? 1 : 0][a.k - 1], dim3(static_cast<unsigned>(grid)), dim3(kEmBlock), lds,
                     static_cast<hipStream_t>(stream), a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : set_error(NXEC_ERR_HIP, "launch k_gather_md5: %s", hipGetErrorString(e));
}

}  // namespace nxec
