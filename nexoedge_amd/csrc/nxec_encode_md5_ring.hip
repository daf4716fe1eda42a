// k_mul_md5 with the code and hash roles decoupled: the
// write path's encode + MD5 of every chunk, the repair path's recover + MD5
// and the verified read, as k_mul_md5 (nxec_encode_md5.hip) computes them,
// but handed between the roles through a ring of LDS slots with counters
// instead of a workgroup barrier per step.  Its own translation unit, so it
// builds beside nxec_encode_md5.hip.  A design probe: measured against
// k_mul_md5 it lost, so only `make PROBES=1` builds it.
#include <hip/hip_runtime.h>

#include <array>
#include <utility>

#include "nxec_em_common.h"

#if NXEC_DESIGN_PROBES

namespace nxec {

namespace {

// k_mul_md5 with the roles decoupled (nxec_em_common.h
// "the decoupled form"): the same code lanes, loads, lookups and stores, the
// same one-lane-per-chunk MD5 chains, but no workgroup barrier in the loop.
// The LDS holds a ring of kRingSlots 128-byte steps of every hashed chunk; a
// 256-byte code step fills two consecutive slots (its lanes v < 8 the first,
// v >= 8 the second), after waiting until the hash waves have counted the
// slot pair free, and counts them ready; a hash wave waits for its slot to be
// counted ready, issues its row's eight 16-byte reads, hashes the previous
// slot's 128 bytes from registers while they land, and counts the slot free.
// The code role may run two code steps ahead of the hash role, and each role
// sleeps only when the other is that far off.
template <int K, bool HSRC>
__global__ __launch_bounds__(kEmBlock) void k_mul_md5_ring(const MulMd5Args a) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int nh = a.nhashed;
  constexpr int hsrc = HSRC ? K : 0;  // rows before the outputs' rows
  const int S = a.stripes_per_group;
  uint8_t *ring = lds + K * 1024;
  const uint32_t slot_bytes = static_cast<uint32_t>(S * nh * kRingRow);
  const uint32_t ready_off = static_cast<uint32_t>(K * 1024) + kRingSlots * slot_bytes, freed_off = ready_off + 16;
  build_tables<1>(a.coef, K, a.p, reinterpret_cast<uint32_t *>(lds));
  if (threadIdx.x < 2 * kRingSlots) *lds_word(ready_off + 4 * threadIdx.x) = 0;
  __syncthreads();
  const int64_t s0 = static_cast<int64_t>(blockIdx.x) * S;
  const int nS = static_cast<int>(min(static_cast<int64_t>(S), a.nstripes - s0));
  const int nsteps = static_cast<int>(a.len / kEncMd5Step);  // code steps; 2 * nsteps hash steps
  // waves taking part in the hand-off: those with a live lane
  const uint32_t ncw = static_cast<uint32_t>((nS * kEmVecs + 63) / 64), nhw = static_cast<uint32_t>((nS * nh + 63) / 64);

  if (threadIdx.x < kEmCodeLanes) {
    if ((threadIdx.x & ~63) >= nS * kEmVecs) return;  // no live stripe: not part of the hand-off
    const int item = threadIdx.x;
    const int ls = item < nS * kEmVecs ? item / kEmVecs : 0, v = item % kEmVecs;
    const __amdgpu_buffer_rsrc_t rsrc_src = em_rsrc(a.src + s0 * a.src_stripe_stride);
    const __amdgpu_buffer_rsrc_t rsrc_dst = em_rsrc(a.dst + s0 * a.dst_stripe_stride);
    const uint32_t vsrc = static_cast<uint32_t>(ls * a.src_stripe_stride) + v * 16;
    const uint32_t vdst = static_cast<uint32_t>(ls * a.dst_stripe_stride) + v * 16;
    const int half = v >> 3;  // which of the code step's two hash steps this lane's 16 bytes belong to
    uint8_t *row = ring + ls * nh * kRingRow + (v & 7) * 16;
    auto load = [&](int step, u32x4(&d)[K]) {
      const uint32_t off = static_cast<uint32_t>(step) * kEncMd5Step;
#pragma unroll
      for (int j = 0; j < K; j++) d[j] = em_load(rsrc_src, vsrc, a.src_off[j] + off);
    };
    // the freed counter of the next step's slot pair, read a step early (the
    // first two steps' slots start free)
    uint32_t seen = 0;
    auto run = [&](int step, const u32x4(&d)[K]) {
      const uint32_t off = static_cast<uint32_t>(step) * kEncMd5Step;
      // the slot pair of hash steps 2*step, 2*step + 1: free once the hash
      // waves have read steps 2*step - 4 and 2*step - 3 (in order: the
      // second).  Waited for first, so the sources go to the slot as the
      // lookups consume them (each dead after its pair, as in k_mul_md5).
      const uint32_t u1 = 2u * static_cast<uint32_t>(step) + 1u;
      ring_wait_from(seen, freed_off + 4 * (u1 % kRingSlots), nhw * (u1 / kRingSlots));
      uint8_t *rb = row + ((2 * step + half) % kRingSlots) * slot_bytes;
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        if (hsrc) {  // wave-uniform
          *reinterpret_cast<u32x4 *>(rb + j * kRingRow) = d[j];
          if (j + 1 < K) *reinterpret_cast<u32x4 *>(rb + (j + 1) * kRingRow) = d[j + 1];
        }
        if (a.any_copy) {  // full-output decode: surviving data chunks pass through
          if (a.copy_off[j] != kNoCopy) em_store(rsrc_dst, vdst, a.copy_off[j] + off, d[j]);
          if (j + 1 < K && a.copy_off[j + 1] != kNoCopy) em_store(rsrc_dst, vdst, a.copy_off[j + 1] + off, d[j + 1]);
        }
        if (a.p > 0) lookup_pair(j, j + 1 < K, d[j], d[j + 1 < K ? j + 1 : j], acc);
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("" : "+v"(acc[i]));
      }
      uint32_t o[4][4];
      rows_of(acc, o);
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++) {
        if (r < a.p) {  // wave-uniform
          const u32x4 pv{o[r][0], o[r][1], o[r][2], o[r][3]};
          em_store(rsrc_dst, vdst, a.dst_off[r] + off, pv);
          if (a.hash_dst) *reinterpret_cast<u32x4 *>(rb + (hsrc + r) * kRingRow) = pv;
        }
      }
      ring_signal(ready_off + 4 * ((u1 - 1) % kRingSlots), ready_off + 4 * (u1 % kRingSlots));
      seen = ring_peek(freed_off + 4 * ((u1 + 2) % kRingSlots));  // the next step's slot pair
    };
    constexpr int D = em_depth<K>();
    u32x4 ring_regs[D][K];
    const int last = nsteps - 1;
#pragma unroll
    for (int j = 0; j < D - 1; j++) load(min(j, last), ring_regs[j]);
    int step = 0;
    for (; step + D <= nsteps; step += D) {
#pragma unroll
      for (int j = 0; j < D; j++) {
        load(min(step + j + D - 1, last), ring_regs[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run(step + j, ring_regs[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < D - 1; j++) {
      if (step + j < nsteps) {
        load(min(step + j + D - 1, last), ring_regs[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run(step + j, ring_regs[j]);
      }
    }
    return;
  }

  // ---- hash waves: lane h = hashed chunk (h / nh, h % nh) of the group = row h of every slot ----
  const int h = threadIdx.x - kEmCodeLanes;
  if ((h & ~63) >= nS * nh) return;  // no live chunk: not part of the hand-off
  const bool active = h < nS * nh;
  const int nhs = 2 * nsteps;
  // lanes past the group's chunks read row 0 and hash it for nothing: no
  // branch in the loop (a path without the row reads would join the waitcnt
  // state and make every wait on the peek a full drain)
  const uint8_t *rowp = ring + (active ? h : 0) * kRingRow;
  uint32_t st[4];
  md5_init(st);
  // the ready counter of the next slot, read a step early (while the wave hashes)
  uint32_t seen = ring_peek(ready_off);
  // the peek goes out BEFORE the rows: waiting for its value then leaves the
  // rows in flight (LDS operations complete in order)
  auto fetch = [&](int u, uint32_t(&m)[kRingStep / 4]) {
    __builtin_amdgcn_sched_barrier(0);
    ring_wait_from<false>(seen, ready_off + 4 * (u % kRingSlots), ncw * static_cast<uint32_t>(u / kRingSlots + 1));
    __builtin_amdgcn_sched_barrier(0);
    seen = ring_peek(ready_off + 4 * ((u + 1) % kRingSlots));
    __builtin_amdgcn_sched_barrier(0);
    const u32x4 *p = reinterpret_cast<const u32x4 *>(rowp + (u % kRingSlots) * slot_bytes);
#pragma unroll
    for (int i = 0; i < kRingStep / 16; i++) {
      const u32x4 x = p[i];
      m[4 * i] = x.x, m[4 * i + 1] = x.y, m[4 * i + 2] = x.z, m[4 * i + 3] = x.w;
    }
    __builtin_amdgcn_sched_barrier(0);  // the peek and the row reads go out before the hashing
  };
  auto hash = [&](const uint32_t(&m)[kRingStep / 4]) {
#pragma unroll
    for (int b = 0; b < kRingStep / 64; b++) md5_block(st, m + 16 * b);
  };
  // Two register buffers: the rows of step u are read while step u - 1 is
  // hashed, and slot u is counted free once they are in.  (Reading two steps
  // ahead -- three buffers, slot u + 1 freed after hashing u -- narrows the
  // code role's lead to one code step and measured 16.6 ms against 14.3,
  // DESIGN.md §4 round 6.)
  uint32_t m0[kRingStep / 4], m1[kRingStep / 4];
  fetch(0, m0);
  ring_signal(freed_off + 0);
  auto step2 = [&](int u, const uint32_t(&cur)[kRingStep / 4], uint32_t(&next)[kRingStep / 4]) {
    fetch(u, next);
    hash(cur);
    __builtin_amdgcn_sched_barrier(0);
    ring_signal(freed_off + 4 * (u % kRingSlots));
    __builtin_amdgcn_sched_barrier(0);
  };
  int u = 1;
  for (; u + 2 <= nhs; u += 2) {
    step2(u, m0, m1);
    step2(u + 1, m1, m0);
  }
  if (u < nhs) {  // nhs is even: one step left
    step2(u, m0, m1);
    hash(m1);
  } else {
    hash(m0);
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
      for (int i = 0; i < 16; i++) out[i] = static_cast<uint8_t>(st[i / 4] >> (8 * (i % 4)));
    }
  }
}

using EmKernel = void (*)(const MulMd5Args);
template <bool HSRC, int... Ks>
constexpr std::array<EmKernel, sizeof...(Ks)> em_ring_table(std::integer_sequence<int, Ks...>) {
  return {{&k_mul_md5_ring<Ks + 1, HSRC>...}};
}
// [hash_src][k - 1]
const std::array<EmKernel, kEncMd5MaxK> kEmRing[2] = {
    em_ring_table<false>(std::make_integer_sequence<int, kEncMd5MaxK>{}),
    em_ring_table<true>(std::make_integer_sequence<int, kEncMd5MaxK>{})};

}  // namespace

void (*mul_md5_ring_kernel(bool hash_src, int k))(const MulMd5Args) { return kEmRing[hash_src ? 1 : 0][k - 1]; }

int prepare_encode_md5_ring() {
  for (int i = 0; i < 2 * kEncMd5MaxK; i++) {
    const EmKernel fn = kEmRing[i / kEncMd5MaxK][i % kEncMd5MaxK];
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(fn)) != hipSuccess || fa.sharedSizeBytes != 0)
      return set_error(NXEC_ERR_HIP, "k_mul_md5_ring: static LDS present (the tables must start at LDS byte 0)");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_mul_md5_ring): %s", hipGetErrorString(e));
  }
  return NXEC_OK;
}

}  // namespace nxec

#endif  // NXEC_DESIGN_PROBES
