// Device helpers shared by the fused coding + MD5 kernels (k_mul_md5,
// k_gather_md5 in nxec_encode_md5.hip; k_files_md5 in nxec_files_md5.hip):
// the code role's LDS table lookups and buffer-resource memory ops, the hash
// role's step loop over LDS rows, the workgroup shape.  Internal linkage: each
// translation unit gets its own copy.
#pragma once

#include <hip/hip_runtime.h>

#include "nxec_device.h"
#include "nxec_internal.h"

// Design-probe kernels (role probes and the LDS-table A/B variants, selected
// by environment variables) are built only with `make PROBES=1`: they are
// measurement tools, not product paths, and double the build time.
#ifndef NXEC_DESIGN_PROBES
#define NXEC_DESIGN_PROBES 0
#endif

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


// ---- the decoupled form (k_mul_md5_ring) ----
// A ring of kRingSlots LDS buffers of kRingStep bytes per hashed chunk,
// handed between the roles by per-slot counters in LDS instead of a
// workgroup barrier per step: the code waves fill a slot once the hash waves
// have counted it free, the hash waves read it once the code waves have
// counted it ready.  Each role then waits only when the other is a whole
// ring behind or ahead, so a slow step of one role no longer stalls the other
// (a barrier per step cost every step the slower role's time).
constexpr int kRingStep = 128;               // bytes of a chunk per hash step (2 MD5 blocks)
constexpr int kRingRow = kRingStep + 16;     // row stride: a quarter-wave's 16-byte reads on distinct banks
constexpr int kRingSlots = 4;                // two code steps (256 bytes each) of slack

typedef __attribute__((address_space(3))) uint32_t lds_u32m;
__device__ __forceinline__ lds_u32m *lds_word(uint32_t byte_off) {
  return reinterpret_cast<lds_u32m *>(static_cast<uintptr_t>(byte_off));
}
// The wave waits (s_sleep between polls) until the LDS counter at byte
// cnt_off reaches `need`.  One asm block, not a C++ loop: a loop in the code
// waves' unrolled step would be a CFG loop inside the load ring, where the
// waitcnt pass drains every outstanding load at the loop head and register
// allocation splits the ring's live ranges (256 VGPRs + spills at k = 10).
// The poll's own s_waitcnt lgkmcnt(0) also orders the LDS reads that follow.
__device__ __forceinline__ void ring_wait(uint32_t cnt_off, uint32_t need) {
  uint32_t v, sv;
  asm volatile(
      "nxec_ring_poll_%=:\n"
      "  ds_read_b32 %0, %2\n"
      "  s_waitcnt lgkmcnt(0)\n"
      "  v_readfirstlane_b32 %1, %0\n"
      "  s_cmp_ge_u32 %1, %3\n"
      "  s_cbranch_scc1 nxec_ring_done_%=\n"
      "  s_sleep 1\n"
      "  s_branch nxec_ring_poll_%=\n"
      "nxec_ring_done_%=:"
      : "=&v"(v), "=&s"(sv)
      : "v"(cnt_off), "s"(need)
      : "scc", "memory");
}
// The counter at byte off, read now and waited for at its first use: issued a
// step early, its value is there when ring_wait_from looks at it, so a role
// that is not behind pays no LDS round trip per step.
__device__ __forceinline__ uint32_t ring_peek(uint32_t off) {
  return __hip_atomic_load(lds_word(off), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// ring_wait with an earlier read of the counter: returns at once when `seen`
// already reaches `need`, else polls (one asm block, as ring_wait).
// MEM: a compiler memory barrier too (the code waves: no LDS write of the
// slot may move above the wait); the hash waves order their reads with
// sched_barrier instead, so the waitcnt pass keeps their reads in flight.
template <bool MEM = true>
__device__ __forceinline__ void ring_wait_from(uint32_t seen, uint32_t cnt_off, uint32_t need) {
  uint32_t v, sv;
  if (MEM)
  asm volatile(
      "  v_readfirstlane_b32 %1, %4\n"
      "  s_cmp_ge_u32 %1, %3\n"
      "  s_cbranch_scc1 nxec_ringf_done_%=\n"
      "nxec_ringf_poll_%=:\n"
      "  s_sleep 1\n"
      "  ds_read_b32 %0, %2\n"
      "  s_waitcnt lgkmcnt(0)\n"
      "  v_readfirstlane_b32 %1, %0\n"
      "  s_cmp_ge_u32 %1, %3\n"
      "  s_cbranch_scc0 nxec_ringf_poll_%=\n"
      "nxec_ringf_done_%=:"
      : "=&v"(v), "=&s"(sv)
      : "v"(cnt_off), "s"(need), "v"(seen)
      : "scc", "memory");
  else
  asm volatile(
      "  v_readfirstlane_b32 %1, %4\n"
      "  s_cmp_ge_u32 %1, %3\n"
      "  s_cbranch_scc1 nxec_ringh_done_%=\n"
      "nxec_ringh_poll_%=:\n"
      "  s_sleep 1\n"
      "  ds_read_b32 %0, %2\n"
      "  s_waitcnt lgkmcnt(0)\n"
      "  v_readfirstlane_b32 %1, %0\n"
      "  s_cmp_ge_u32 %1, %3\n"
      "  s_cbranch_scc0 nxec_ringh_poll_%=\n"
      "nxec_ringh_done_%=:"
      : "=&v"(v), "=&s"(sv)
      : "v"(cnt_off), "s"(need), "v"(seen)
      : "scc");
}
// ring_signal once all but the wave's last 9 LDS operations are complete
// (LDS operations complete in order; scalar loads in lgkmcnt only make the
// wait longer).  The hash waves' form: no compiler memory barrier (their
// reads are ordered by sched_barrier), so the waitcnt pass keeps the reads
// issued before it in flight.
__device__ __forceinline__ void ring_signal_behind9(uint32_t cnt_off) {
  uint64_t save;
  const uint32_t one = 1;
  asm volatile(
      "s_waitcnt lgkmcnt(9)\n"
      "  s_mov_b64 %0, exec\n"
      "  s_mov_b64 exec, 1\n"
      "  ds_add_u32 %1, %2\n"
      "  s_mov_b64 exec, %0"
      : "=&s"(save)
      : "v"(cnt_off), "v"(one));
}
// Once the wave's LDS accesses so far are complete, lane 0 alone adds 1 to the
// counter at byte cnt_off (and at cnt_off2 when it differs).  Also one asm
// block: a lane-0 branch would be divergent control flow inside the code
// waves' unrolled step.
__device__ __forceinline__ void ring_signal(uint32_t cnt_off, uint32_t cnt_off2 = 0xffffffffu) {
  uint64_t save;
  const uint32_t one = 1;
  if (cnt_off2 == 0xffffffffu) {
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n"
        "  s_mov_b64 %0, exec\n"
        "  s_mov_b64 exec, 1\n"
        "  ds_add_u32 %1, %2\n"
        "  s_mov_b64 exec, %0"
        : "=&s"(save)
        : "v"(cnt_off), "v"(one)
        : "memory");
  } else {
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n"
        "  s_mov_b64 %0, exec\n"
        "  s_mov_b64 exec, 1\n"
        "  ds_add_u32 %1, %3\n"
        "  ds_add_u32 %2, %3\n"
        "  s_mov_b64 exec, %0"
        : "=&s"(save)
        : "v"(cnt_off), "v"(cnt_off2), "v"(one)
        : "memory");
  }
}

// ring depth of the pointer-table form: as many steps in flight as ~200
// VGPRs hold (its 64-bit source pointers take 2K of them), at most 8 -- its
// loads cross PCIe (microseconds each), so small k keeps more steps ahead
template <int K>
constexpr int gm_depth() {
  return (200 - 2 * K) / (4 * K) >= 8 ? 8 : (200 - 2 * K) / (4 * K) < 2 ? 2 : (200 - 2 * K) / (4 * K);
}

}  // namespace

// k_mul_md5_ring (nxec_encode_md5_ring.hip) for (hash_src, k), and its kernel attributes
void (*mul_md5_ring_kernel(bool hash_src, int k))(const MulMd5Args);
int prepare_encode_md5_ring();

}  // namespace nxec
