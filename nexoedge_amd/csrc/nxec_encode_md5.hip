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
#include <utility>
#include <vector>

#include "nxec_em_common.h"

extern "C" int nxec_design_probes(void) { return NXEC_DESIGN_PROBES; }

namespace nxec {

namespace {

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
  if (!tuning().fused_md5) return false;  // probe: two kernels (coding, then MD5)
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
#if NXEC_DESIGN_PROBES
  if (int rc = prepare_encode_md5_ring()) return rc;
#endif
  for (int i = 0; i < 2 * kEncMd5MaxK; i++) {
    const EmKernel fn = kEm[i / kEncMd5MaxK][i % kEncMd5MaxK];
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(fn)) != hipSuccess || fa.sharedSizeBytes != 0)
      return set_error(NXEC_ERR_HIP, "k_mul_md5: static LDS present (the tables must start at LDS byte 0)");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_mul_md5): %s", hipGetErrorString(e));
  }
  if (int rc = prepare_files_md5()) return rc;
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
  if (tuning().em_stripes > 0)  // probe: stripes per workgroup
    S = std::max<int64_t>(1, std::min<int64_t>(tuning().em_stripes, std::min(kEmMaxStripes, kEmMaxRows / n)));
  a.stripes_per_group = static_cast<int32_t>(S);
  a.hash_prio = tuning().em_prio;
  const int64_t grid = (a.nstripes + S - 1) / S;
  if (grid >= (int64_t(1) << 31)) return set_error(NXEC_ERR_INVALID, "encode+md5: batch too large for one launch");
  int lds = a.k * 1024 + static_cast<int>(2 * S * n * kEmRow);
  EmKernel fn = kEm[a.hash_src ? 1 : 0][a.k - 1];
#if NXEC_DESIGN_PROBES
  // A/B: the decoupled form where its ring fits the LDS (k <= 20, S * n <=
  // 256 rows of 4 x 144 bytes: all but the widest hashed-source stripes)
  const int lds_ring = a.k * 1024 + static_cast<int>(kRingSlots * S * n * kRingRow) + 8 * 4;
  if (tuning().em_ring && lds_ring <= kEmLds) {
    fn = mul_md5_ring_kernel(a.hash_src != 0, a.k);
    lds = lds_ring;
  }
#endif
#if NXEC_DESIGN_PROBES
  if (tuning().em_probe >= 0 && a.k == 10 && a.hash_src) fn = kEmProbe[tuning().em_probe & 7];
  // A/B: conflict-free split-nibble tables (k = 10, sources hashed; 40 KiB of tables)
  if (tuning().em_nibble && a.k == 10 && a.hash_src && 10 * 4096 + 2 * S * n * kEmRow <= kEmLds) {
    fn = kEmNib;
    lds = 10 * 4096 + static_cast<int>(2 * S * n * kEmRow);
  }
  // A/B: hash lanes read the source chunks from global memory (only the
  // outputs' rows in LDS; k = 10, sources hashed, full-output copies off)
  if (tuning().em_hashsrc_global && a.k == 10 && a.hash_src && a.hash_dst && !a.any_copy && !a.ok) {
    fn = kEmHg;
    lds = 10 * 1024 + static_cast<int>(2 * S * a.p * kEmRow);
  }
#endif
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(kEmBlock), lds,
                     static_cast<hipStream_t>(stream), a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : set_error(NXEC_ERR_HIP, "launch k_mul_md5: %s", hipGetErrorString(e));
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
