// gfx950 (CDNA4) kernels of the Nexoedge RS coding path.
//
// One primitive: dst_r[i] = XOR_j c(r,j) (x) src_j[i] over GF(2^8)/0x11d, for
// r < rows <= 4 and every byte i of every stripe in a batch.  This is the work
// of ISA-L's ec_encode_data (ec_base.c:302-317; SIMD gf_4vect_dot_prod_*.asm)
// as called by rs.cc:89 (encode), rs.cc:230 (decode/repair), rs.cc:106 (CAR
// XOR) and coding_util.hh:21,28 (agent partial encode) -- re-designed for
// MI355X rather than translated:
//
//  * Table lookup in LDS.  For every source j the workgroup builds a
//    256-entry table whose 32-bit entry x packs the products c(r,j)*x of all
//    (<= 4) output rows.  One ds_read_b32 per source byte yields every row's
//    product at once, so each data byte is read from HBM once and looked up
//    once, whatever the number of rows (the reference's SIMD kernel and the
//    "one wavefront per row" alternative both re-touch the data per row).
//  * Bank-conflict-free-ish replication.  Random data bytes make LDS bank
//    conflicts data dependent; table copy c = lane % R sits in the bank bits
//    (address = ((j*256 + x)*R + c)*4), so with R = 16 a half-wave's 32 lanes
//    collide at most pairwise (4 LDS cycles per wave lookup instead of ~8 at
//    R = 1).  R = 16 for k <= 10 (k*16 KiB of LDS), R = 8 for k <= 20.
//  * HBM side: each lane owns one 16-byte column vector of the stripe; a wave
//    issues k global_load_dwordx4 (1 KiB contiguous per source, all k in
//    flight) and `rows` global_store_dwordx4 after an in-register 4x4 byte
//    transpose (v_perm_b32) of the packed accumulators.
//  * Persistent grid (one or two 1024-thread workgroups per CU) walks the
//    flattened (stripe, column-tile) space, so the tables are built once per
//    workgroup, not per tile.
//  * No MFMA: this is byte-wise lookup/XOR work bounded by HBM bandwidth.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "nxec_device.h"
#include "nxec_internal.h"

namespace nxec {

namespace {

constexpr int kBlock = 1024;       // threads per workgroup (16 waves)
constexpr int kMaxTemplK = 20;     // k with a fully unrolled kernel; larger k use the dynamic kernel
constexpr int kLdsBytes = 160 * 1024;
// next-tile prefetch doubles the source registers (4*K VGPRs); beyond these k
// the 128-VGPR budget of a 1024-thread workgroup would spill
constexpr int kPrefetchMaxK = 10;
constexpr int kPrefetchMaxKCopy = 8;  // k = 10 with copies fits (123 VGPRs) but measured 6-8% slower (full-output decode)
constexpr int kPermPrefetchMaxK = 4;
constexpr int kPermMaxK = 13;  // beyond this the single-row VALU kernel would spill (128-VGPR budget)

constexpr int kRingBytes = 16;  // work-queue broadcast ring, after the tables in dynamic LDS
constexpr bool queue_fits(int table_bytes) { return table_bytes + kRingBytes <= kLdsBytes; }

using dev::build_tables;
using dev::gf_mul_dev;
using dev::ld_stream;
using dev::lookup16;
using dev::rows_of;
using dev::st_stream;
using dev::u32x4;

template <int R>
__device__ __forceinline__ void build_tables(const MulArgs &a, int k, uint32_t *tab) {
  build_tables<R>(a.coef, a.k, a.rows, tab);
}

// Chunk addresses of stripe s.  GATHER is a template parameter so the
// per-source address math stays branch-free (uniform, SGPR-resident).
template <bool GATHER>
__device__ __forceinline__ uint8_t *dst_row(const MulArgs &a, uint32_t s, int r) {
  if (GATHER) return a.dst_ptrs[static_cast<size_t>(s) * a.dst_ptr_rows + a.dst_ptr_row0 + r];
  return a.dst + static_cast<int64_t>(s) * a.dst_stripe_stride + a.dst_off[r];
}

template <bool GATHER>
__device__ __forceinline__ const uint8_t *src_chunk(const MulArgs &a, uint32_t s, int j) {
  if (GATHER) return a.src_ptrs[static_cast<size_t>(s) * a.k + j];
  return a.src + static_cast<int64_t>(s) * a.src_stripe_stride + a.src_off[j];
}

// acc[p] holds the 4 row products of column byte p (p = 4q + b); write row r's
// 16 bytes = byte r of acc[0..15].  8 v_perm_b32 per 4 columns.
template <bool GATHER>
__device__ __forceinline__ void store_rows(const MulArgs &a, uint32_t s, uint32_t v, const uint32_t acc[16]) {
  uint32_t o[4][4];
  rows_of(acc, o);
#pragma unroll
  for (int r = 0; r < kMaxRowsPerPass; r++) {
    if (r < a.rows) st_stream(dst_row<GATHER>(a, s, r) + static_cast<size_t>(v) * 16, u32x4{o[r][0], o[r][1], o[r][2], o[r][3]});
  }
}

// the same transpose, row r (< rows) stored at row0 + r*row_stride + v*16
__device__ __forceinline__ void store_rows_ptr(uint8_t *row0, int64_t row_stride, int rows, uint32_t v,
                                               const uint32_t acc[16]) {
  uint32_t o[4][4];
  rows_of(acc, o);
#pragma unroll
  for (int r = 0; r < kMaxRowsPerPass; r++)
    if (r < rows) st_stream(row0 + r * row_stride + static_cast<size_t>(v) * 16, u32x4{o[r][0], o[r][1], o[r][2], o[r][3]});
}

// Column vector v (relative to the launch's vec_begin) of stripe s for tile t;
// tiles are kBlock consecutive vectors of one stripe.
struct TilePos {
  uint32_t s, v;
};
__device__ __forceinline__ TilePos tile_pos(uint32_t t, uint32_t tps) {
  const uint32_t s = t / tps;
  return {s, (t - s * tps) * kBlock + threadIdx.x};
}
// With stripe groups of sg > 1, tiles run column-major inside each group of
// sg consecutive stripes (the last group may be smaller).
__device__ __forceinline__ TilePos tile_pos(uint32_t t, uint32_t tps, uint32_t sg, uint32_t nstripes) {
  if (sg <= 1) return tile_pos(t, tps);
  const uint32_t per = sg * tps;
  const uint32_t g = t / per, w = t - g * per;
  const uint32_t gs = nstripes - g * sg < sg ? nstripes - g * sg : sg;
  const uint32_t c = w / gs;
  return {g * sg + (w - c * gs), c * kBlock + threadIdx.x};
}

// FULL: every tile is complete (vec_count % kBlock == 0), so no lane predicate
// and no exec-mask regions around the loads; the ragged remainder of a chunk
// gets its own predicated launch.
template <int K, bool GATHER, bool FULL>
__device__ __forceinline__ void load_tile(const MulArgs &a, TilePos p, uint32_t nvec, u32x4 (&d)[K]) {
  if (FULL || p.v < nvec) {
    const size_t off = (static_cast<size_t>(a.vec_begin) + p.v) * 16;
#pragma unroll
    for (int j = 0; j < K; j++) d[j] = ld_stream(src_chunk<GATHER>(a, p.s, j) + off);
  }
}

template <int K, bool COPY>
__device__ __forceinline__ void copy_through(const MulArgs &a, uint32_t s, uint32_t vg, const u32x4 (&d)[K]) {
  if (COPY) {
#pragma unroll
    for (int j = 0; j < K; j++) {
      const uint32_t c = a.copy_off[j];
      if (c != kNoCopy)
        st_stream(a.dst + static_cast<int64_t>(s) * a.dst_stripe_stride + c + static_cast<size_t>(vg) * 16, d[j]);
    }
  }
}

// --- algorithm 1: LDS product tables (any rows <= 4) ---
template <int K, int R, bool GATHER, bool COPY>
struct LdsBody {
  static constexpr int kLds = K * 1024 * R;
  static __device__ __forceinline__ void setup(const MulArgs &a, uint32_t *tab) { build_tables<R>(a, K, tab); }
  const char *tlane;
  __device__ explicit LdsBody(const uint32_t *tab)
      : tlane(reinterpret_cast<const char *>(tab) + (threadIdx.x % R) * 4) {}
  __device__ __forceinline__ void operator()(const MulArgs &a, uint32_t s, uint32_t vg, const u32x4 (&d)[K]) const {
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
    for (int j = 0; j < K; j++) lookup16<R>(tlane + j * 1024 * R, d[j], acc);
    store_rows<GATHER>(a, s, vg, acc);
    copy_through<K, COPY>(a, s, vg, d);
  }
};

// --- algorithm 2: VALU nibble tables via v_perm_b32 (rows == 1) ---
// c*x = c*(x & 15) ^ c*(x & 0xf0).  v_perm_b32 picks 4 bytes at once from an
// 8-byte pool; a 16-entry nibble table is two pools, chosen per byte by the
// nibble's bit 3.  That bit becomes a 0x00/0xFF byte mask through v_perm's
// sign-replication selectors (8..11 copy bit 7 of pool bytes 1,3,5,7), and
// v_bfi_b32 merges the two halves.  No LDS traffic per byte (only 2 uniform
// ds_read_b128 per source per tile for the 32-byte table), so a single-row
// pass (repair, agent partial encode, CAR XOR) is not bound by LDS banks.
// Measured k=12 rows=1: 0.678 of 8 TB/s vs 0.608 for the LDS tables
// (tools/microbench/shape_ceiling.hip).
__device__ __forceinline__ uint32_t perm_mul(const uint32_t *t, uint32_t nl, uint32_t nh, uint32_t ml, uint32_t mh) {
  const uint32_t l0 = __builtin_amdgcn_perm(t[1], t[0], nl), l1 = __builtin_amdgcn_perm(t[3], t[2], nl);
  const uint32_t h0 = __builtin_amdgcn_perm(t[5], t[4], nh), h1 = __builtin_amdgcn_perm(t[7], t[6], nh);
  return ((ml & l1) | (~ml & l0)) ^ ((mh & h1) | (~mh & h0));
}

template <int K, bool GATHER, bool COPY>
struct PermBody {
  static constexpr int kLds = K * 32;
  // table of source j: bytes [32j .. 32j+15] = c*n, [32j+16 .. 32j+31] = c*(n<<4)
  static __device__ __forceinline__ void setup(const MulArgs &a, uint32_t *tab) {
    uint8_t *tb = reinterpret_cast<uint8_t *>(tab);
    for (int i = threadIdx.x; i < K * 16; i += blockDim.x) {
      const int j = i >> 4, n = i & 15;
      const uint32_t c = a.coef[j];
      tb[32 * j + n] = static_cast<uint8_t>(gf_mul_dev(c, n));
      tb[32 * j + 16 + n] = static_cast<uint8_t>(gf_mul_dev(c, n << 4));
    }
  }
  const uint32_t *tab;
  __device__ explicit PermBody(const uint32_t *t) : tab(t) {}
  __device__ __forceinline__ void operator()(const MulArgs &a, uint32_t s, uint32_t vg, const u32x4 (&d)[K]) const {
    // opaque zero: keeps the (uniform) table reads next to their use instead of
    // hoisting K*8 registers out of the tile loop
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    const uint32_t *tt = tab + z;
    uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < K; j++) {
      const uint32_t w[4] = {d[j].x, d[j].y, d[j].z, d[j].w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t x = w[q], x4 = x << 4;
        const uint32_t nl = x & 0x07070707u, nh = (x >> 4) & 0x07070707u;
        const uint32_t ml = __builtin_amdgcn_perm(x4, x4 << 8, 0x0B090A08u);
        const uint32_t mh = __builtin_amdgcn_perm(x, x << 8, 0x0B090A08u);
        o[q] ^= perm_mul(tt + 8 * j, nl, nh, ml, mh);
      }
    }
    st_stream(dst_row<GATHER>(a, s, 0) + static_cast<size_t>(vg) * 16, u32x4{o[0], o[1], o[2], o[3]});
    copy_through<K, COPY>(a, s, vg, d);
  }
};

// Per-launch tile queues (one 128-byte slot per launch: [0] next tile, [1]
// workgroups finished).  The last workgroup to finish resets its slot, so a
// slot is clean for the next launch that draws it (host ring, kQueueSlots).
__device__ uint32_t g_tile_queue[kQueueSlots * 32];

// Work-queue grab: global_atomic_add with return, issued through inline asm
// so the compiler's wait-count bookkeeping never sees it.  Issued before a
// step's K loads, it is older than every op the compiler waits for, so the
// compiler's own waits stay correct (they can only wait longer), and the
// caller publishes g after an explicit vmcnt(K) -- instead of the vmcnt(0)
// (drain of every store) the compiler emits around a divergent atomic.
__device__ __forceinline__ uint32_t grab_async(uint32_t *q) {
  uint32_t g;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=&v"(g) : "v"(q), "v"(1u) : "memory");
  return g;
}
// ring[OFF/4] = g once at most N vector-memory ops are outstanding
template <int N, int OFF>
__device__ __forceinline__ void publish(uint32_t ring_base, uint32_t g) {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%2)\n\tds_write_b32 %0, %1 offset:%3" ::"v"(ring_base), "v"(g), "n"(N), "n"(OFF)
               : "memory");
}

// Persistent tile loop.
//
// Q (work queue, the default where 16 bytes of LDS are free): workgroups pull
// runs of T consecutive 16 KiB column tiles from a per-launch atomic counter
// (T = 1 for wide stripes; more for narrow ones so the counter is not
// hammered, tiles_per_grab()), the next run grabbed one run ahead and
// broadcast through a 4-entry LDS ring (one barrier per run).  In-flight tiles therefore always form one compact,
// ascending address window, and a workgroup slowed by a busy HBM channel
// simply takes fewer tiles: +12 % over static tile runs for the same bytes
// (tools/microbench/mem_pattern.hip, profiles/r01_mem_pattern.log).
//
// !Q (tables fill the whole 160 KiB), or queue_slot < 0 (NXEC_TILE_ORDER=static,
// for A/B only): workgroup b owns the contiguous tile run [b*ntiles/G, (b+1)*ntiles/G).
//
// PF: the next tile's loads go out before this tile's compute through two
// ping-pong register buffers (manual 2x unroll pinned by sched_barrier: no
// register copies, so the waitcnt pass keeps the prefetch in flight); a final
// prefetch past the end re-reads the current tile instead of branching, so
// every path has the same loads in flight.
//
// The geometry is the caller's: load(t, d) fetches tile t's K source vectors
// of this lane into d, run(t, d) computes and stores tile t.  ntiles tiles;
// slot >= 0 selects the queue (Q kernels), T = tiles per grab.
template <int K, bool PF, bool Q, bool QWAIT_K, class LoadF, class RunF>
__device__ __forceinline__ void tile_loop(const LoadF &load, const RunF &run, uint32_t ntiles, int32_t slot_arg,
                                          uint32_t T, uint32_t *ring) {
  if (Q && slot_arg >= 0) {
    uint32_t *q = g_tile_queue + static_cast<size_t>(slot_arg) * 32;
    if (threadIdx.x == 0) {
      ring[2] = atomicAdd(q, 1u);
      ring[3] = atomicAdd(q, 1u);
    }
    __syncthreads();
    // t: current tile; [t, rend) the rest of its run; nrun: first tile of the
    // run already grabbed for after it (all wave-uniform, SGPRs)
    auto run_start = [&](uint32_t r) -> uint32_t { return r * T; };
    uint32_t t = run_start(__builtin_amdgcn_readfirstlane(ring[2]));
    uint32_t nrun = run_start(__builtin_amdgcn_readfirstlane(ring[3]));
    uint32_t rend = t + T < ntiles ? t + T : ntiles;
    int slot = 0;
    // LDS byte address of ring[0], materialized once (a VGPR that no store
    // ever uses, so publishing never waits on the stores in flight)
    uint32_t ring_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(ring));
    asm volatile("" : "+v"(ring_base));
    // barrier that orders only the LDS ring (global loads stay in flight)
    auto ring_barrier = [] {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    };
    // one tile: at the last tile of a run, grab the run after next (thread 0,
    // early, so the atomic's latency hides behind this tile's work) and
    // broadcast it at the end; nxt (PF) receives the next tile's sources
    // (the grab is issued before this step's loads: the ring write then only
    // waits for the atomic, not for the loads and stores behind it)
    auto step = [&](u32x4(&cur)[K], u32x4(&nxt)[K], bool pf) {
      const bool edge = t + 1 >= rend;
      const uint32_t tn = edge ? nrun : t + 1;
      uint32_t g = 0;
      if (edge && threadIdx.x == 0) g = grab_async(q);
      if (pf) {
        load(tn < ntiles ? tn : t, nxt);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        load(t, cur);
        __builtin_amdgcn_sched_barrier(0);  // all K loads in flight before the lookups
      }
      run(t, cur);
      if (edge) {
        if (threadIdx.x == 0) {
          // >= K vector-memory ops (this step's loads) were issued after the
          // grab, so at most K outstanding means the grab has returned
          if (slot == 0) publish<QWAIT_K ? K : 0, 0>(ring_base, g);
          else publish<QWAIT_K ? K : 0, 4>(ring_base, g);
        }
        ring_barrier();
        const uint32_t nn = run_start(__builtin_amdgcn_readfirstlane(ring[slot]));
        slot ^= 1;
        rend = nrun + T < ntiles ? nrun + T : ntiles;
        nrun = nn;
      }
      t = tn;
      return t < ntiles;
    };
    if (t < ntiles) {
      if constexpr (PF) {
        u32x4 A[K], B[K];
        load(t, A);
        while (step(A, B, true) && step(B, A, true)) {
        }
      } else {
        bool more = true;
        while (more) {
          u32x4 d[K];
          more = step(d, d, false);
        }
      }
    }
    // every grab of this workgroup has returned (its values were consumed);
    // the last workgroup out resets the slot for the next launch
    if (threadIdx.x == 0) {
      __threadfence();
      if (atomicAdd(q + 1, 1u) == gridDim.x - 1) {
        atomicExch(q, 0u);
        atomicExch(q + 1, 0u);
      }
    }
    return;
  }
  // readfirstlane: the tile index is wave-uniform; keep its math on the SALU
  uint32_t t = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x) * ntiles) / gridDim.x));
  const uint32_t tend = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x + 1) * ntiles) / gridDim.x));
  if (t >= tend) return;
  if constexpr (PF) {
    u32x4 A[K], B[K];
    load(t, A);
    while (true) {
      const uint32_t tb = t + 1;
      load(tb < tend ? tb : t, B);
      __builtin_amdgcn_sched_barrier(0);
      run(t, A);
      if (tb >= tend) break;
      t = tb;
      const uint32_t ta = t + 1;
      load(ta < tend ? ta : t, A);
      __builtin_amdgcn_sched_barrier(0);
      run(t, B);
      if (ta >= tend) break;
      t = ta;
    }
  } else {
    for (; t < tend; t++) {
      u32x4 d[K];
      load(t, d);
      run(t, d);
    }
  }
}

// Fully unrolled vector kernels: all K source loads of a column vector in
// flight.  COPY: fused pass-through of sources (full-output decode); a
// separate instantiation so encode/recover kernels carry no copy registers.
// The queue ring lives in the dynamic LDS block after the tables (Q only
// where it fits: queue_fits()).
// Strided / gather geometry of a MulArgs launch: tile t = column tile
// t % tps of stripe t / tps.
template <int K, bool GATHER, bool FULL, bool PF, bool Q, class Body>
__device__ __forceinline__ void mul_tiles(const MulArgs &a, const Body &body, uint32_t *ring) {
  const uint32_t nvec = static_cast<uint32_t>(a.vec_count);
  const uint32_t tps = (nvec + kBlock - 1) / kBlock;
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const uint32_t sg = a.stripe_group, ns = static_cast<uint32_t>(a.nstripes);
  auto load = [&](uint32_t t, u32x4(&d)[K]) { load_tile<K, GATHER, FULL>(a, tile_pos(t, tps, sg, ns), nvec, d); };
  auto run = [&](uint32_t t, const u32x4(&d)[K]) {
    const TilePos p = tile_pos(t, tps, sg, ns);
    if (FULL || p.v < nvec) body(a, p.s, static_cast<uint32_t>(a.vec_begin) + p.v, d);
  };
  tile_loop<K, PF, Q, FULL>(load, run, ntiles, a.queue_slot, a.tiles_per_grab, ring);
}

template <int K, int R, bool GATHER, bool COPY, bool FULL>
__global__ __launch_bounds__(kBlock) void k_mul_vec(const MulArgs a) {
  constexpr bool PF = K <= ((COPY || !FULL) ? kPrefetchMaxKCopy : kPrefetchMaxK);
  constexpr bool Q = queue_fits(LdsBody<K, R, GATHER, COPY>::kLds);
  using Body = LdsBody<K, R, GATHER, COPY>;
  extern __shared__ uint32_t tab[];
  Body::setup(a, tab);
  __syncthreads();
  mul_tiles<K, GATHER, FULL, PF, Q>(a, Body(tab), tab + Body::kLds / 4);
}

template <int K, bool GATHER, bool COPY, bool FULL>
__global__ __launch_bounds__(kBlock) void k_mul_perm(const MulArgs a) {
  constexpr bool PF = K <= kPermPrefetchMaxK;
  using Body = PermBody<K, GATHER, COPY>;
  extern __shared__ uint32_t tab[];
  Body::setup(a, tab);
  __syncthreads();
  mul_tiles<K, GATHER, FULL, PF, true>(a, Body(tab), tab + Body::kLds / 4);
}

// --- ragged stripes (the last stripes of many objects) ---
// Stripes of different chunk lengths in one launch, through the same
// work-queue tile loop and LDS tables as k_mul_vec: tile t belongs to stripe
// tile_stripe[t] (a device map built per call), column tile
// t - stripe_tile0[s].  Every stripe is 16-byte aligned with 16-byte chunk
// strides and len rounded up to 16 (the zero-padded tail arena of
// nxec_encode_objects), so every lane moves whole 16-byte vectors.
struct RaggedArgs {
  const ListStripe *__restrict__ stripes;
  const uint32_t *__restrict__ tile_stripe;
  const uint32_t *__restrict__ stripe_tile0;
  uint32_t ntiles;
  int32_t k, rows, row0, queue_slot;
  uint32_t tiles_per_grab;
  uint8_t coef[kMaxRowsPerPass * (NXEC_MAX_K + 1)];
};

template <int K, int R>
__global__ __launch_bounds__(kBlock) void k_mul_ragged(const RaggedArgs a) {
  constexpr bool PF = K <= kPrefetchMaxKCopy;
  constexpr int kLds = K * 1024 * R;
  static_assert(queue_fits(kLds), "ragged kernels are queue-driven");
  extern __shared__ uint32_t tab[];
  build_tables<R>(a.coef, K, a.rows, tab);
  __syncthreads();
  const char *tl = reinterpret_cast<const char *>(tab) + (threadIdx.x % R) * 4;
  auto where = [&](uint32_t t, ListStripe &st, uint32_t &v) {
    const uint32_t s = a.tile_stripe[t];
    st = a.stripes[s];
    v = (t - a.stripe_tile0[s]) * kBlock + threadIdx.x;
  };
  auto load = [&](uint32_t t, u32x4(&d)[K]) {
    ListStripe st;
    uint32_t v;
    where(t, st, v);
    if (v * int64_t(16) < st.len) {
#pragma unroll
      for (int j = 0; j < K; j++) d[j] = ld_stream(st.src + j * st.src_cs + static_cast<size_t>(v) * 16);
    }
  };
  auto run = [&](uint32_t t, const u32x4(&d)[K]) {
    ListStripe st;
    uint32_t v;
    where(t, st, v);
    if (v * int64_t(16) < st.len) {
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j++) lookup16<R>(tl + j * 1024 * R, d[j], acc);
      store_rows_ptr(st.dst + a.row0 * st.dst_cs, st.dst_cs, a.rows, v, acc);
    }
  };
  // wave 0 (lane 0 = the tile's first vector) always issues its K loads
  tile_loop<K, PF, true, true>(load, run, a.ntiles, a.queue_slot, a.tiles_per_grab, tab + kLds / 4);
}

// Runtime-k vector kernel (k > kMaxTemplK), R = 1 tables, sources in groups of 4.
template <bool GATHER>
__global__ __launch_bounds__(kBlock) void k_mul_vec_dyn(const MulArgs a) {
  extern __shared__ uint32_t tab[];
  const int k = a.k;
  build_tables<1>(a, k, tab);
  __syncthreads();
  const uint32_t nvec = static_cast<uint32_t>(a.vec_count);
  const uint32_t tps = (nvec + kBlock - 1) / kBlock;
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const char *tl = reinterpret_cast<const char *>(tab);
  const uint32_t t0 = static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x) * ntiles) / gridDim.x);
  const uint32_t t1 = static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x + 1) * ntiles) / gridDim.x);
  for (uint32_t t = t0; t < t1; t++) {
    const uint32_t s = t / tps;
    const uint32_t vl = (t - s * tps) * kBlock + threadIdx.x;
    if (vl >= nvec) continue;
    const uint32_t v = static_cast<uint32_t>(a.vec_begin) + vl;
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0;
    for (int j0 = 0; j0 < k; j0 += 4) {
      u32x4 d[4];
#pragma unroll
      for (int jj = 0; jj < 4; jj++)
        if (j0 + jj < k) d[jj] = ld_stream(src_chunk<GATHER>(a, s, j0 + jj) + static_cast<size_t>(v) * 16);
#pragma unroll
      for (int jj = 0; jj < 4; jj++) {
        if (j0 + jj < k) {
          lookup16<1>(tl + (j0 + jj) * 1024, d[jj], acc);
          const uint32_t c = a.copy_off[j0 + jj];
          if (!GATHER && a.any_copy && c != kNoCopy)
            st_stream(a.dst + static_cast<int64_t>(s) * a.dst_stripe_stride + c + static_cast<size_t>(v) * 16, d[jj]);
        }
      }
    }
    store_rows<GATHER>(a, s, v, acc);
  }
}

// Byte-granular kernel: chunk tails past vec_count*16 and misaligned layouts.
template <bool GATHER>
__global__ __launch_bounds__(256) void k_mul_bytes(const MulArgs a) {
  extern __shared__ uint32_t tab[];
  const int k = a.k;
  build_tables<1>(a, k, tab);
  __syncthreads();
  const int64_t span = a.len - a.byte_begin;
  const int64_t total = span * a.nstripes;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t s = static_cast<uint32_t>(i / span);
    const int64_t pos = a.byte_begin + (i - static_cast<int64_t>(s) * span);
    uint32_t acc = 0;
    for (int j = 0; j < k; j++) {
      const uint8_t x = src_chunk<GATHER>(a, s, j)[pos];
      acc ^= tab[j * 256 + x];
      const uint32_t c = a.copy_off[j];
      if (!GATHER && a.any_copy && c != kNoCopy) a.dst[static_cast<int64_t>(s) * a.dst_stripe_stride + c + pos] = x;
    }
    for (int r = 0; r < a.rows; r++) dst_row<GATHER>(a, s, r)[pos] = static_cast<uint8_t>(acc >> (8 * r));
  }
}

// --- variable-length batches (many objects per call) ---
// One launch over stripes of different chunk lengths and layouts.  Work unit =
// one 16-byte column piece; workgroup b owns the contiguous unit run
// [b*T/G, (b+1)*T/G), finds its first stripe by binary search over the unit
// prefix once (thread 0, LDS broadcast), and every thread then advances its
// own stripe cursor monotonically.  R = 1 packed-row LDS tables; 16-byte
// vector loads where the piece is complete and aligned, bytes otherwise.
// Not the throughput path for big objects (their full stripes go through
// k_mul_vec in gather form); it covers the ragged last stripes.
struct ListArgs {
  const ListStripe *stripes;
  const int64_t *prefix;
  int64_t nstripes, total;
  int32_t k, rows, row0;
  uint8_t coef[kMaxRowsPerPass * (NXEC_MAX_K + 1)];
};

__global__ __launch_bounds__(256) void k_mul_list(const ListArgs a) {
  extern __shared__ uint32_t tab[];
  __shared__ int64_t s_first;
  const int k = a.k;
  for (int i = threadIdx.x; i < k * 256; i += blockDim.x) {
    const int j = i >> 8;
    uint32_t e = 0;
    for (int r = 0; r < a.rows; r++) e |= gf_mul_dev(a.coef[r * k + j], static_cast<uint32_t>(i & 255)) << (8 * r);
    tab[i] = e;
  }
  const int64_t u0 = static_cast<int64_t>(blockIdx.x) * a.total / gridDim.x;
  const int64_t u1 = static_cast<int64_t>(blockIdx.x + 1) * a.total / gridDim.x;
  if (threadIdx.x == 0) {
    int64_t lo = 0, hi = a.nstripes - 1;  // last s with prefix[s] <= u0
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (a.prefix[mid] <= u0) lo = mid;
      else hi = mid - 1;
    }
    s_first = lo;
  }
  __syncthreads();
  int64_t s = s_first;
  const char *tl = reinterpret_cast<const char *>(tab);
  for (int64_t u = u0 + threadIdx.x; u < u1; u += blockDim.x) {
    while (a.prefix[s + 1] <= u) s++;
    const ListStripe st = a.stripes[s];
    const int64_t off = (u - a.prefix[s]) * 16;
    const int64_t nb = st.len - off < 16 ? st.len - off : 16;
    const bool vec = nb == 16 && ((reinterpret_cast<uintptr_t>(st.src) | reinterpret_cast<uintptr_t>(st.dst) |
                                   static_cast<uint64_t>(st.src_cs) | static_cast<uint64_t>(st.dst_cs) |
                                   static_cast<uint64_t>(off)) & 15) == 0;
    uint8_t *drow0 = st.dst + static_cast<int64_t>(a.row0) * st.dst_cs + off;
    if (vec) {
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
      for (int j = 0; j < k; j++) lookup16<1>(tl + j * 1024, ld_stream(st.src + j * st.src_cs + off), acc);
      uint32_t o[4][4];
      rows_of(acc, o);
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++)
        if (r < a.rows) st_stream(drow0 + r * st.dst_cs, u32x4{o[r][0], o[r][1], o[r][2], o[r][3]});
    } else {
      for (int b = 0; b < nb; b++) {
        uint32_t acc = 0;
        for (int j = 0; j < k; j++) acc ^= tab[j * 256 + st.src[j * st.src_cs + off + b]];
        for (int r = 0; r < a.rows; r++) drow0[r * st.dst_cs + b] = static_cast<uint8_t>(acc >> (8 * r));
      }
    }
  }
}

// zero-padded copies (the last stripe of each object, chunk_manager.cc:390-399);
// blockIdx.y-less: item = blockIdx.x / kPadParts, each part a slice of it
constexpr int kPadParts = 8;
__global__ __launch_bounds__(256) void k_pad_copy(const PadCopy *items) {
  const PadCopy it = items[blockIdx.x / kPadParts];
  const int part = blockIdx.x % kPadParts;
  const int64_t per = ((it.dst_len + kPadParts - 1) / kPadParts + 15) / 16 * 16;
  const int64_t b0 = part * per, b1 = b0 + per < it.dst_len ? b0 + per : it.dst_len;
  for (int64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) it.dst[i] = i < it.src_len ? it.src[i] : 0;
}

// Last stripe of an object into the aligned tail arena: chunk j of the
// stripe = object bytes [j*cl, (j+1)*cl) (zero past the object's remaining
// rem bytes, chunk_manager.cc:390-399), written at dst + j*cls with
// cls = cl rounded up to 16 and zeros in [cl, cls).  One thread per 16-byte
// output vector; the 16 source bytes are assembled from dword-aligned loads
// with v_alignbit (the source offset j*cl has any alignment), bytes where
// the 20-byte window would leave the object.  Item i owns blocks
// [bstart[i], bstart[i+1]) of kPadVecs*256 vectors (thread 0 finds the item).
__global__ __launch_bounds__(256) void k_pad_chunks(const PadChunks *__restrict__ items,
                                                    const uint32_t *__restrict__ bstart, int64_t nitems) {
  __shared__ int64_t s_item;
  if (threadIdx.x == 0) {
    int64_t lo = 0, hi = nitems - 1;  // last item with bstart <= blockIdx.x
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (bstart[mid] <= blockIdx.x) lo = mid;
      else hi = mid - 1;
    }
    s_item = lo;
  }
  __syncthreads();
  const int64_t item = s_item;
  const PadChunks it = items[item];
  const int64_t vpc = it.cls / 16;  // vectors per chunk
  const int64_t u0 = static_cast<int64_t>(blockIdx.x - bstart[item]) * (256 * kPadVecs);
#pragma unroll
  for (int r = 0; r < kPadVecs; r++) {
    const int64_t u = u0 + r * 256 + threadIdx.x;  // output vector
    if (u >= vpc * it.k) break;
    const int64_t j = u / vpc, x = (u - j * vpc) * 16;  // chunk, byte offset in it
    const int64_t sidx = j * it.cl + x;                 // source byte of output byte x
    const int64_t nvalid = min(min(static_cast<int64_t>(16), it.cl - x), it.rem - sidx);  // may be <= 0
    uint32_t w[4] = {0, 0, 0, 0};
    if (nvalid > 0) {
      const uint8_t *sp = it.src + sidx;
      const uintptr_t base = reinterpret_cast<uintptr_t>(sp) & ~uintptr_t(3);
      if (nvalid == 16 && base + 20 <= reinterpret_cast<uintptr_t>(it.src + it.rem)) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(base);
        const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(sp) & 3) * 8;
        const uint32_t r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
        w[0] = __builtin_amdgcn_alignbit(r1, r0, sb);
        w[1] = __builtin_amdgcn_alignbit(r2, r1, sb);
        w[2] = __builtin_amdgcn_alignbit(r3, r2, sb);
        w[3] = __builtin_amdgcn_alignbit(r4, r3, sb);
      } else {
        for (int b = 0; b < nvalid; b++) w[b >> 2] |= static_cast<uint32_t>(sp[b]) << (8 * (b & 3));
      }
    }
    st_stream(it.dst + j * it.cls + x, u32x4{w[0], w[1], w[2], w[3]});
  }
}

// 16-byte vector copy; `dst` may be device-mapped pinned host memory, so a
// device -> host transfer runs as shader stores over PCIe on the compute
// queue instead of an SDMA copy (which would queue behind the H2D copies).
__global__ __launch_bounds__(256) void k_copy16(u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ void k_fill(uint8_t *p, int64_t bytes, uint64_t seed) {
  const int64_t words = (bytes + 7) / 8;
  const bool aligned = (reinterpret_cast<uintptr_t>(p) & 7) == 0;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < words;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    uint64_t z = seed + static_cast<uint64_t>(i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    if (aligned && (i + 1) * 8 <= bytes) {
      reinterpret_cast<uint64_t *>(p)[i] = z;
    } else {
      for (int b = 0; b < 8 && i * 8 + b < bytes; b++) p[i * 8 + b] = static_cast<uint8_t>(z >> (8 * b));
    }
  }
}

__global__ void k_checksum(const uint8_t *p, int64_t bytes, unsigned long long *out) {
  const int64_t words = (bytes + 7) / 8;
  const bool aligned = (reinterpret_cast<uintptr_t>(p) & 7) == 0;
  uint64_t acc = 0;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < words;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    uint64_t w = 0;
    if (aligned && (i + 1) * 8 <= bytes) {
      w = reinterpret_cast<const uint64_t *>(p)[i];
    } else {
      for (int b = 0; b < 8 && i * 8 + b < bytes; b++) w |= static_cast<uint64_t>(p[i * 8 + b]) << (8 * b);
    }
    acc += w * static_cast<uint64_t>(2 * i + 1);
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, static_cast<unsigned long long>(acc));
}

using KernelFn = void (*)(MulArgs);

template <int R, bool G, bool CP, bool FULL, int... Ks>
constexpr std::array<KernelFn, sizeof...(Ks)> vec_table(std::integer_sequence<int, Ks...>) {
  return {{&k_mul_vec<Ks + 1, R, G, CP, FULL>...}};
}

// One table per (form, R, full-tiles): indexed by k-1.  Strided full-tile
// kernels exist for every R (tuning knob NXEC_LDS_R); every other form only
// at the default R (16 for k <= 10, else 8).
using KTable = std::array<KernelFn, kMaxTemplK>;
template <int R, bool G, bool CP, bool FULL>
KTable make_table() {
  KTable t{};
  if constexpr (R == 16) {
    auto a = vec_table<16, G, CP, FULL>(std::make_integer_sequence<int, 10>{});
    for (int i = 0; i < 10; i++) t[i] = a[i];
  } else {
    auto a = vec_table<R, G, CP, FULL>(std::make_integer_sequence<int, kMaxTemplK>{});
    for (int i = 0; i < kMaxTemplK; i++) t[i] = a[i];
  }
  return t;
}
// [gather][copy][full]
const KTable kDefR16[2][2][2] = {
    {{make_table<16, false, false, false>(), make_table<16, false, false, true>()},
     {make_table<16, false, true, false>(), make_table<16, false, true, true>()}},
    {{make_table<16, true, false, false>(), make_table<16, true, false, true>()}, {KTable{}, KTable{}}}};
const KTable kDefR8[2][2][2] = {
    {{make_table<8, false, false, false>(), make_table<8, false, false, true>()},
     {make_table<8, false, true, false>(), make_table<8, false, true, true>()}},
    {{make_table<8, true, false, false>(), make_table<8, true, false, true>()}, {KTable{}, KTable{}}}};
const KTable kTuneR1 = make_table<1, false, false, true>();

template <bool G, int... Ks>
constexpr std::array<KernelFn, sizeof...(Ks)> perm_table(std::integer_sequence<int, Ks...>) {
  return {{&k_mul_perm<Ks + 1, G, false, true>...}};
}
// single-row kernels (complete tiles, no pass-through), [gather][k-1]
const std::array<KernelFn, kPermMaxK> kPerm[2] = {perm_table<false>(std::make_integer_sequence<int, kPermMaxK>{}),
                                                  perm_table<true>(std::make_integer_sequence<int, kPermMaxK>{})};

int hip_fail(hipError_t e, const char *what) {
  return set_error(NXEC_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

// LDS replication policy (the LDS-replication probe overrides it, nxec_tuning.h).
int choose_r(int k, bool tunable) {
  if (k > kMaxTemplK) return 1;
  const int want = tunable ? tuning().lds_r : 0;
  if (want == 1) return 1;
  if (want == 8) return 8;
  if (want == 16 && k <= 10) return 16;
  // the largest replication that leaves room for the tile-queue ring: the
  // queue's dynamic tile order is worth far more than R = 16's fewer LDS bank
  // conflicts (k = 10: 0.80 vs 0.64-0.73 of 8 TB/s, profiles/r01_mem_pattern.log)
  return k <= 9 ? 16 : 8;
}

KernelFn vec_kernel(int k, int r, bool gather, bool copy, bool full) {
  if (k > kMaxTemplK) return gather ? &k_mul_vec_dyn<true> : &k_mul_vec_dyn<false>;
  if (r == 1 && !gather && !copy && full) return kTuneR1[k - 1];
  if (r == 16 && k <= 10) return kDefR16[gather][copy][full][k - 1];
  return kDefR8[gather][copy][full][k - 1];
}


// dynamic LDS of a k_mul_vec instantiation: tables (+ the queue ring where it fits)
int table_lds(int k, int r) {
  const int t = k * 1024 * r;
  return queue_fits(t) ? t + kRingBytes : t;
}

}  // namespace

// single-row passes use the VALU nibble-table kernel (a probe forces LDS tables, nxec_tuning.h)
bool use_perm(int k, int rows, bool full, bool copy, bool gather) {
  if (rows != 1 || k > kPermMaxK || !full || copy) return false;
  if (k == 11 && !gather) return false;  // this instantiation alone spills (hipcc 7.2 schedule); LDS tables instead
  return !tuning().lds_single_row;
}

LaunchInfo plan_launch(int k, int rows, int64_t vec_count, int64_t nstripes, int num_cus, bool full, bool copy,
                       bool gather) {
  const bool tunable = !gather && !copy && full;
  LaunchInfo li{};
  li.block = kBlock;
  int per_cu = 1;
  if (use_perm(k, rows, full, copy, gather)) {
    li.perm = true;
    li.lds_copies = 0;
    li.lds_bytes = k * 32 + kRingBytes;
    li.variant = "vec_perm";
  } else {
    li.lds_copies = choose_r(k, tunable);
    li.lds_bytes = k * 1024 * li.lds_copies;
    const bool queued = k <= kMaxTemplK && queue_fits(li.lds_bytes);
    if (queued) li.lds_bytes += kRingBytes;
    per_cu = kLdsBytes / (li.lds_bytes > 0 ? li.lds_bytes : 1);
    if (per_cu > 2) per_cu = 2;  // 2 x 16 waves = the CU's 32-wave limit
    if (per_cu < 1) per_cu = 1;
    // queue-driven launches: one workgroup per CU keeps the in-flight window
    // tightest (two per CU measured 0.755 vs 0.798 of 8 TB/s, XOR probe)
    if (queued) per_cu = 1;
    li.variant = k > kMaxTemplK ? "vec_dyn" : "vec_lds";
  }
  const int64_t tps = (vec_count + kBlock - 1) / kBlock;
  int64_t ntiles = tps * nstripes;
  int64_t grid = static_cast<int64_t>(num_cus) * per_cu;
  if (grid > ntiles) grid = ntiles;
  li.grid = static_cast<int>(grid);
  return li;
}

int prepare_kernels() {
  auto raise = [](KernelFn fn, int lds) -> hipError_t {
    return hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  };
  for (int k = 1; k <= kMaxTemplK; k++) {
    for (int g = 0; g < 2; g++)
      for (int c = 0; c < 2; c++)
        for (int f = 0; f < 2; f++) {
          if (g && c) continue;
          for (int r : {16, 8}) {
            if (r == 16 && k > 10) continue;
            hipError_t e = raise(vec_kernel(k, r, g, c, f), table_lds(k, r));
            if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(k_mul_vec)");
          }
        }
    hipError_t e = raise(kTuneR1[k - 1], table_lds(k, 1));
    if (e == hipSuccess) e = raise(kDefR8[0][0][1][k - 1], table_lds(k, 8));
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(k_mul_vec tune)");
  }
  for (KernelFn fn : {&k_mul_vec_dyn<false>, &k_mul_vec_dyn<true>, &k_mul_bytes<false>, &k_mul_bytes<true>}) {
    hipError_t e = raise(fn, NXEC_MAX_K * 1024);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(dyn/bytes)");
  }
  return prepare_encode_md5();
}

// Work-queue run length: about 12 tiles' worth of chunk traffic per grab (a
// 16 KiB tile moves k + rows (+ copies) 16 KiB pieces), so wide stripes grab
// one tile at a time (the tightest in-flight window) and narrow ones (CAR XOR,
// small partial encodes) several, which keeps the single counter well under
// its atomic rate (~80 M/s) and the grab latency hidden.
uint32_t tiles_per_grab(const MulArgs &a) {
  int units = a.k + a.rows;
  if (a.any_copy)
    for (int j = 0; j < a.k; j++) units += a.copy_off[j] != kNoCopy;
  const int t = (12 + units - 1) / units;
  return static_cast<uint32_t>(t < 1 ? 1 : (t > 8 ? 8 : t));
}

// host side of the tile-queue ring: each vector launch draws the next slot
// (4096 launches would have to be in flight at once for two to share one)
std::atomic<uint32_t> g_next_slot{0};

// A slot is cleaned by the last workgroup of the launch that used it.  A
// launch that never completes (enqueue failure, aborted stream) would leave a
// non-zero counter behind, and the launch that draws the same slot 4096
// launches later would start past tile 0 and silently skip tiles.  Every
// failed launch therefore zeroes its slot from the host before returning.
int reset_queue_slots(int first, int count, hipStream_t st) {
  void *base = nullptr;
  hipError_t e = hipGetSymbolAddress(&base, HIP_SYMBOL(g_tile_queue));
  if (e == hipSuccess) {
    if (count <= 0) {
      first = 0;
      count = kQueueSlots;
    }
    e = hipMemsetAsync(static_cast<uint8_t *>(base) + static_cast<size_t>(first) * 128, 0,
                       static_cast<size_t>(count) * 128, st);
  }
  return e == hipSuccess ? NXEC_OK : hip_fail(e, "tile-queue reset");
}

int launch_failed(hipError_t e, const char *what, int slot, hipStream_t st) {
  const int rc = hip_fail(e, what);
  if (slot >= 0) (void)reset_queue_slots(slot, 1, st);
  return rc;
}


int launch_mul(const MulArgs &a, bool vec_ok, int num_cus, void *stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (a.nstripes <= 0 || a.len <= 0) return NXEC_OK;
  if (vec_ok && a.vec_count > 0) {
    const int64_t tps = (a.vec_count + kBlock - 1) / kBlock;
    if (tps * a.nstripes >= (int64_t(1) << 32) || a.vec_count >= (int64_t(1) << 32))
      return set_error(NXEC_ERR_INVALID, "batch too large for one launch (split nstripes)");
    const bool gather = a.src_ptrs != nullptr;
    const bool copy = a.any_copy != 0;
    // complete tiles first (no lane predicates), then the ragged remainder
    const int64_t full = a.vec_count / kBlock * kBlock;
    const int64_t parts[2][2] = {{0, full}, {full, a.vec_count - full}};
    for (int pi = 0; pi < 2; pi++) {
      if (parts[pi][1] <= 0) continue;
      MulArgs b = a;
      b.queue_slot = tuning().static_order ? -1 : static_cast<int32_t>(g_next_slot.fetch_add(1, std::memory_order_relaxed) % kQueueSlots);
      b.tiles_per_grab = tiles_per_grab(b);
      // chunks of >= 2 MiB at a power-of-two-aligned chunk stride: walk groups
      // of 8 stripes column-major, so the in-flight window spans 8 stripes
      // like it does at 1 MiB (4 MiB stride: 0.655 -> 0.711 of 8 TB/s,
      // profiles/r01_chunk_stride_group.log).  A padded stride (the
      // recommended layout, nxec_batch_layout) runs best stripe-major
      // (4 MiB + 2 KiB: 0.758 at sg 1, profiles/r02_layout_sweep.log).
      const bool aliased = a.src_ptrs != nullptr || a.src_chunk_stride % (int64_t(1) << 20) == 0;
      b.stripe_group = ((b.vec_count + kBlock - 1) / kBlock >= 128 && aliased) ? 8 : 1;
      if (tuning().stripe_group > 0) b.stripe_group = static_cast<uint32_t>(tuning().stripe_group);
      b.vec_begin = a.vec_begin + parts[pi][0];
      b.vec_count = parts[pi][1];
      const bool is_full = pi == 0;
      LaunchInfo li = plan_launch(b.k, b.rows, b.vec_count, b.nstripes, num_cus, is_full, copy, gather);
      KernelFn fn = li.perm ? kPerm[gather][b.k - 1] : vec_kernel(b.k, li.lds_copies, gather, copy, is_full);
      hipLaunchKernelGGL(fn, dim3(li.grid), dim3(li.block), li.lds_bytes, st, b);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return launch_failed(e, "launch k_mul_vec", b.queue_slot, st);
    }
  }
  if (a.byte_begin < a.len) {
    const int64_t total = (a.len - a.byte_begin) * a.nstripes;
    int64_t blocks = (total + 255) / 256;
    if (blocks > static_cast<int64_t>(num_cus) * 8) blocks = static_cast<int64_t>(num_cus) * 8;
    KernelFn fn = a.src_ptrs ? &k_mul_bytes<true> : &k_mul_bytes<false>;
    hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(blocks)), dim3(256), a.k * 1024, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "launch k_mul_bytes");
  }
  return NXEC_OK;
}

int reset_work_queues(void *stream) {
  const int rc = reset_queue_slots(0, 0, static_cast<hipStream_t>(stream));
  if (rc) return rc;
  const hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
  return e == hipSuccess ? NXEC_OK : hip_fail(e, "tile-queue reset sync");
}

int debug_poison_next_queue_slot(uint32_t next_tile) {
  void *base = nullptr;
  hipError_t e = hipGetSymbolAddress(&base, HIP_SYMBOL(g_tile_queue));
  const uint32_t slot = g_next_slot.load() % kQueueSlots;
  if (e == hipSuccess)
    e = hipMemcpy(static_cast<uint8_t *>(base) + static_cast<size_t>(slot) * 128, &next_tile, sizeof(next_tile),
                  hipMemcpyHostToDevice);
  return e == hipSuccess ? NXEC_OK : hip_fail(e, "tile-queue poison");
}

int launch_mul_list(int rows, int k, const uint8_t *coeffs, const ListStripe *d_stripes, const int64_t *d_prefix,
                    int64_t nstripes, int64_t total_units, int num_cus, void *stream) {
  if (nstripes <= 0 || total_units <= 0 || rows <= 0) return NXEC_OK;
  if (k < 1 || k > NXEC_MAX_K) return set_error(NXEC_ERR_INVALID, "k=%d out of range", k);
  int64_t blocks = (total_units + 255) / 256;
  if (blocks > static_cast<int64_t>(num_cus) * 8) blocks = static_cast<int64_t>(num_cus) * 8;
  for (int r0 = 0; r0 < rows; r0 += kMaxRowsPerPass) {
    ListArgs a;
    std::memset(&a, 0, sizeof(a));
    a.stripes = d_stripes;
    a.prefix = d_prefix;
    a.nstripes = nstripes;
    a.total = total_units;
    a.k = k;
    a.rows = rows - r0 < kMaxRowsPerPass ? rows - r0 : kMaxRowsPerPass;
    a.row0 = r0;
    for (int r = 0; r < a.rows; r++)
      for (int j = 0; j < k; j++) a.coef[r * k + j] = coeffs[static_cast<size_t>(r0 + r) * k + j];
    hipLaunchKernelGGL(k_mul_list, dim3(static_cast<unsigned>(blocks)), dim3(256), k * 1024,
                       static_cast<hipStream_t>(stream), a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "launch k_mul_list");
  }
  return NXEC_OK;
}

using RaggedFn = void (*)(RaggedArgs);
template <int... Ks>
constexpr std::array<RaggedFn, sizeof...(Ks)> ragged_table(std::integer_sequence<int, Ks...>) {
  return {{&k_mul_ragged<Ks + 1, (Ks + 1 <= 9 ? 16 : 8)>...}};
}
const std::array<RaggedFn, kMaxRaggedK> kRagged = ragged_table(std::make_integer_sequence<int, kMaxRaggedK>{});
int ragged_lds(int k) { return k * 1024 * (k <= 9 ? 16 : 8) + kRingBytes; }

int launch_mul_ragged(int rows, int k, const uint8_t *coeffs, const ListStripe *d_stripes, const uint32_t *d_tile_stripe,
                      const uint32_t *d_stripe_tile0, int64_t ntiles, int num_cus, void *stream) {
  if (ntiles <= 0 || rows <= 0) return NXEC_OK;
  if (k < 1 || k > kMaxRaggedK) return set_error(NXEC_ERR_INVALID, "ragged launch: k=%d unsupported", k);
  if (ntiles >= (int64_t(1) << 32)) return set_error(NXEC_ERR_INVALID, "ragged launch: too many tiles");
  static const bool raised = [] {
    for (int kk = 1; kk <= kMaxRaggedK; kk++)
      if (hipFuncSetAttribute(reinterpret_cast<const void *>(kRagged[kk - 1]),
                              hipFuncAttributeMaxDynamicSharedMemorySize, ragged_lds(kk)) != hipSuccess)
        return false;
    return true;
  }();
  if (!raised) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_mul_ragged) failed");
  const int64_t grid = std::min<int64_t>(num_cus, ntiles);
  for (int r0 = 0; r0 < rows; r0 += kMaxRowsPerPass) {
    RaggedArgs a;
    std::memset(&a, 0, sizeof(a));
    a.stripes = d_stripes;
    a.tile_stripe = d_tile_stripe;
    a.stripe_tile0 = d_stripe_tile0;
    a.ntiles = static_cast<uint32_t>(ntiles);
    a.k = k;
    a.rows = rows - r0 < kMaxRowsPerPass ? rows - r0 : kMaxRowsPerPass;
    a.row0 = r0;
    a.queue_slot = static_cast<int32_t>(g_next_slot.fetch_add(1, std::memory_order_relaxed) % kQueueSlots);
    a.tiles_per_grab = std::max(1, std::min(8, (12 + k + a.rows - 1) / (k + a.rows)));
    for (int r = 0; r < a.rows; r++)
      for (int j = 0; j < k; j++) a.coef[r * k + j] = coeffs[static_cast<size_t>(r0 + r) * k + j];
    hipLaunchKernelGGL(kRagged[k - 1], dim3(static_cast<unsigned>(grid)), dim3(kBlock), ragged_lds(k),
                       static_cast<hipStream_t>(stream), a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return launch_failed(e, "launch k_mul_ragged", a.queue_slot, static_cast<hipStream_t>(stream));
  }
  return NXEC_OK;
}

int launch_pad_chunks(const PadChunks *d_items, const uint32_t *d_bstart, int64_t nitems, int64_t nblocks,
                      void *stream) {
  if (nitems <= 0 || nblocks <= 0) return NXEC_OK;
  if (nblocks >= (int64_t(1) << 31)) return set_error(NXEC_ERR_INVALID, "pad-chunks launch too large");
  hipLaunchKernelGGL(k_pad_chunks, dim3(static_cast<unsigned>(nblocks)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     d_items, d_bstart, nitems);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : hip_fail(e, "launch k_pad_chunks");
}

int launch_pad_copy(const PadCopy *d_items, int64_t nitems, void *stream) {
  if (nitems <= 0) return NXEC_OK;
  if (nitems * kPadParts >= (int64_t(1) << 31)) return set_error(NXEC_ERR_INVALID, "too many pad-copy items");
  hipLaunchKernelGGL(k_pad_copy, dim3(static_cast<unsigned>(nitems * kPadParts)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), d_items);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : hip_fail(e, "launch k_pad_copy");
}

int launch_copy16(void *dst, const void *src, size_t bytes, int num_cus, void *stream) {
  if (bytes == 0) return NXEC_OK;
  if (bytes % 16 || (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15)
    return set_error(NXEC_ERR_INVALID, "copy16: unaligned");
  const int64_t n = static_cast<int64_t>(bytes / 16);
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, static_cast<int64_t>(num_cus) * 4);
  hipLaunchKernelGGL(k_copy16, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<u32x4 *>(dst), static_cast<const u32x4 *>(src), n);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : hip_fail(e, "launch k_copy16");
}

int launch_fill(void *d, size_t bytes, uint64_t seed, void *stream) {
  if (bytes == 0) return NXEC_OK;
  hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<uint8_t *>(d),
                     static_cast<int64_t>(bytes), seed);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : hip_fail(e, "launch k_fill");
}

int launch_checksum(const void *d, size_t bytes, uint64_t *d_out, void *stream) {
  hipLaunchKernelGGL(k_checksum, dim3(1024), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t *>(d), static_cast<int64_t>(bytes),
                     reinterpret_cast<unsigned long long *>(d_out));
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : hip_fail(e, "launch k_checksum");
}

}  // namespace nxec
