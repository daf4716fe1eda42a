// Design probe: which HBM access pattern moves the RS(10,4) encode bytes
// (10 source streams read, 4 parity streams written per stripe, 4096 stripes
// of 14 x 1 MiB) fastest on MI355X?  The GF arithmetic is replaced by XOR
// (the product runs within 1-4 % of an XOR kernel of the same pattern,
// profiles/r01_shape_ceiling*.log), so every row here is a memory ceiling.
//
// Knobs (template parameters of k_xor):
//   BLOCK  threads per workgroup            VPL  16-B vectors per lane per source per tile
//   LP/SP  load / store policy: 0 plain, 1 nontemporal builtin, 2 buffer op aux=sc0|sc1 (stream), 3 buffer op aux=nt|sc1
//   MAP    0 blocked tile runs per workgroup (product), 1 interleaved (t += grid), 2 one tile per workgroup
//   PF     ping-pong next-tile prefetch
//   WPC    workgroups per CU for persistent maps
// plus reference kernels: float4 copy (guide-style), read-only, write-only.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o mem_pattern mem_pattern.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "nxec.h"

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Args {
  uint8_t *buf;  // [stripe][K + ROWS][cs]
  int64_t cs, nstripes;
  uint32_t *queue;  // MAP 4 work counter (zeroed before each launch)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, 0x7fffffff, 0x00020000);
}

// base: wave-uniform; vo: per-lane byte offset
template <int LP>
__device__ __forceinline__ u32x4 ld(const uint8_t *base, uint32_t vo) {
  if constexpr (LP == 0) return *reinterpret_cast<const u32x4 *>(base + vo);
  else if constexpr (LP == 1) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base + vo));
  else {
    constexpr int aux = LP == 2 ? (1 | 16) : (2 | 16);
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), vo, 0, aux));
  }
}
template <int SP>
__device__ __forceinline__ void st(uint8_t *base, uint32_t vo, u32x4 v) {
  if constexpr (SP == 0) *reinterpret_cast<u32x4 *>(base + vo) = v;
  else if constexpr (SP == 1) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(base + vo));
  else {
    constexpr int aux = SP == 2 ? (1 | 16) : (2 | 16);
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base), vo, 0, aux);
  }
}

template <int K, int ROWS, int BLOCK, int VPL, int LP, int SP, int MAP, bool PF>
__global__ __launch_bounds__(BLOCK) void k_xor(const Args a) {
  constexpr uint32_t kTile = BLOCK * VPL * 16;
  const uint32_t tps = static_cast<uint32_t>(a.cs / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const int64_t sstride = (K + ROWS) * a.cs;
  uint32_t t, tend, step;
  if (MAP == 0) {
    t = static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x) * ntiles) / gridDim.x);
    tend = static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x + 1) * ntiles) / gridDim.x);
    step = 1;
  } else if (MAP == 1) {
    t = blockIdx.x;
    tend = ntiles;
    step = gridDim.x;
  } else if (MAP == 2) {
    t = blockIdx.x;
    tend = t + 1;
    step = 1;
  } else {
    // MAP 3: blocked runs, but each workgroup starts its sweep of every stripe
    // at its own column tile (rotation), so concurrent workgroups touch
    // different low address bits.  Handled in tile(): t is a run index.
    t = static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x) * ntiles) / gridDim.x);
    tend = static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x + 1) * ntiles) / gridDim.x);
    step = 1;
  }
  t = __builtin_amdgcn_readfirstlane(t);
  tend = __builtin_amdgcn_readfirstlane(tend);
  if (t >= tend) return;
  const uint32_t rot = MAP == 3 ? (blockIdx.x * 7u) % tps : 0u;
  auto colof = [&](uint32_t tt, uint32_t s) { uint32_t c = tt - s * tps + rot; return c >= tps ? c - tps : c; };
  auto load = [&](uint32_t tt, u32x4(&d)[VPL][K]) {
    const uint32_t s = tt / tps;
    const uint8_t *sp = a.buf + s * sstride + colof(tt, s) * kTile;
#pragma unroll
    for (int i = 0; i < VPL; i++)
#pragma unroll
      for (int j = 0; j < K; j++) d[i][j] = ld<LP>(sp + j * a.cs, threadIdx.x * 16 + i * BLOCK * 16);
  };
  auto body = [&](uint32_t tt, const u32x4(&d)[VPL][K]) {
    const uint32_t s = tt / tps;
    uint8_t *dp = a.buf + s * sstride + K * a.cs + colof(tt, s) * kTile;
#pragma unroll
    for (int i = 0; i < VPL; i++) {
      u32x4 x = d[i][0];
#pragma unroll
      for (int j = 1; j < K; j++) x ^= d[i][j];
#pragma unroll
      for (int r = 0; r < ROWS; r++) st<SP>(dp + r * a.cs, threadIdx.x * 16 + i * BLOCK * 16, x + static_cast<unsigned>(r));
    }
  };
  if constexpr (PF) {
    u32x4 A[VPL][K], B[VPL][K];
    load(t, A);
    while (true) {
      const uint32_t tb = t + step;
      load(tb < tend ? tb : t, B);
      __builtin_amdgcn_sched_barrier(0);
      body(t, A);
      if (tb >= tend) break;
      t = tb;
      const uint32_t ta = t + step;
      load(ta < tend ? ta : t, A);
      __builtin_amdgcn_sched_barrier(0);
      body(t, B);
      if (ta >= tend) break;
      t = ta;
    }
  } else {
    for (; t < tend; t += step) {
      u32x4 d[VPL][K];
      load(t, d);
      body(t, d);
    }
  }
}

// Burst / time-phased variant: each wave loads T tiles, then stores their
// T*ROWS outputs.  With PHASE, loads are issued only inside the read window
// and stores only inside the write window of a chip-wide period of P ticks of
// s_memrealtime (100 MHz), read window = RF/100 of it -- an attempt to keep
// the HBM channels from turning around between reads and writes.
__device__ __forceinline__ void wait_window(uint64_t P, uint64_t lo, uint64_t hi) {
  while (true) {
    const uint64_t ph = __builtin_amdgcn_s_memrealtime() % P;
    if (ph >= lo && ph < hi) return;
    __builtin_amdgcn_s_sleep(2);
  }
}
template <int K, int ROWS, int T, bool PHASE, int P, int RF>
__global__ __launch_bounds__(1024) void k_phase(const Args a) {
  constexpr uint32_t kTile = 1024 * 16;
  const uint32_t tps = static_cast<uint32_t>(a.cs / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const int64_t sstride = (K + ROWS) * a.cs;
  uint32_t t = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x) * ntiles) / gridDim.x));
  const uint32_t tend = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x + 1) * ntiles) / gridDim.x));
  constexpr uint64_t rlo = 0, rhi = (uint64_t)P * RF / 100;
  for (; t < tend; t += T) {
    u32x4 x[T];
    if (PHASE) wait_window(P, rlo, rhi);
#pragma unroll
    for (int u = 0; u < T; u++) {
      const uint32_t tt = t + u < tend ? t + u : t;
      const uint32_t s = tt / tps;
      const uint8_t *sp = a.buf + s * sstride + (tt - s * tps) * kTile;
      u32x4 d[K];
#pragma unroll
      for (int j = 0; j < K; j++) d[j] = ld<1>(sp + j * a.cs, threadIdx.x * 16);
      x[u] = d[0];
#pragma unroll
      for (int j = 1; j < K; j++) x[u] ^= d[j];
    }
    if (PHASE) wait_window(P, rhi, P);
#pragma unroll
    for (int u = 0; u < T; u++) {
      const uint32_t tt = t + u < tend ? t + u : t;
      const uint32_t s = tt / tps;
      uint8_t *dp = a.buf + s * sstride + K * a.cs + (tt - s * tps) * kTile;
#pragma unroll
      for (int r = 0; r < ROWS; r++) st<1>(dp + r * a.cs, threadIdx.x * 16, x[u] + static_cast<unsigned>(r));
    }
  }
}

// MAP 4: persistent workgroups pull tiles from a global counter (dynamic).
// G consecutive tiles per grab; the grab for the next run is made one run
// ahead (LDS broadcast, one barrier per run).  XCD: one counter per XCD
// (workgroup b runs on XCD b % 8 under round-robin placement), each owning a
// contiguous eighth of the tiles.  PF: next tile's loads issued before this
// tile's stores.
template <int K, int ROWS, int BLOCK, int G, bool XCD, bool PF, int LP = 1, int SP = 1>
__global__ __launch_bounds__(BLOCK) void k_queue(const Args a) {
  constexpr uint32_t kTile = BLOCK * 16;
  __shared__ uint32_t s_next[2];
  const uint32_t tps = static_cast<uint32_t>(a.cs / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const int64_t sstride = (K + ROWS) * a.cs;
  const uint32_t x = XCD ? blockIdx.x % 8 : 0;
  const uint32_t lo = XCD ? static_cast<uint32_t>((uint64_t)ntiles * x / 8) : 0;
  const uint32_t hi = XCD ? static_cast<uint32_t>((uint64_t)ntiles * (x + 1) / 8) : ntiles;
  uint32_t *q = a.queue + (XCD ? x * 32 : 0);
  if (threadIdx.x == 0) s_next[0] = lo + atomicAdd(q, 1u) * G;
  __syncthreads();
  uint32_t t = __builtin_amdgcn_readfirstlane(s_next[0]);
  int par = 0;
  auto load = [&](uint32_t tt, u32x4(&d)[K]) {
    const uint32_t s = tt / tps;
    const uint8_t *sp = a.buf + s * sstride + (tt - s * tps) * kTile;
#pragma unroll
    for (int j = 0; j < K; j++) d[j] = ld<LP>(sp + j * a.cs, threadIdx.x * 16);
  };
  auto body = [&](uint32_t tt, const u32x4(&d)[K]) {
    const uint32_t s = tt / tps;
    u32x4 xx = d[0];
#pragma unroll
    for (int j = 1; j < K; j++) xx ^= d[j];
    uint8_t *dp = a.buf + s * sstride + K * a.cs + (tt - s * tps) * kTile;
#pragma unroll
    for (int r = 0; r < ROWS; r++) st<SP>(dp + r * a.cs, threadIdx.x * 16, xx + static_cast<unsigned>(r));
  };
  while (t < hi) {
    if (threadIdx.x == 0) s_next[par ^ 1] = lo + atomicAdd(q, 1u) * G;
    const uint32_t te = t + G < hi ? t + G : hi;
    if constexpr (PF) {
      u32x4 A[K], B[K];
      load(t, A);
      for (uint32_t u = t; u < te; u += 2) {
        load(u + 1 < te ? u + 1 : u, B);
        __builtin_amdgcn_sched_barrier(0);
        body(u, A);
        if (u + 1 >= te) break;
        load(u + 2 < te ? u + 2 : u + 1, A);
        __builtin_amdgcn_sched_barrier(0);
        body(u + 1, B);
      }
    } else {
      for (uint32_t u = t; u < te; u++) {
        u32x4 d[K];
        load(u, d);
        body(u, d);
      }
    }
    __syncthreads();
    par ^= 1;
    t = __builtin_amdgcn_readfirstlane(s_next[par]);
  }
}

// read-only: K streams of every stripe, XOR-reduced, stored only if a
// (never-true) condition holds so the loads stay live
template <int K, int ROWS, int BLOCK, int LP>
__global__ __launch_bounds__(BLOCK) void k_read(const Args a, uint32_t *sink) {
  constexpr uint32_t kTile = BLOCK * 16;
  const uint32_t tps = static_cast<uint32_t>(a.cs / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const int64_t sstride = (K + ROWS) * a.cs;
  uint32_t t = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x) * ntiles) / gridDim.x));
  const uint32_t tend = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x + 1) * ntiles) / gridDim.x));
  u32x4 acc = {0, 0, 0, 0};
  for (; t < tend; t++) {
    const uint32_t s = t / tps;
    const uint8_t *sp = a.buf + s * sstride + (t - s * tps) * kTile;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; j++) d[j] = ld<LP>(sp + j * a.cs, threadIdx.x * 16);
#pragma unroll
    for (int j = 0; j < K; j++) acc ^= d[j];
  }
  if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[threadIdx.x] = acc.z;
}

// write-only: ROWS streams per stripe
template <int K, int ROWS, int BLOCK, int SP>
__global__ __launch_bounds__(BLOCK) void k_write(const Args a) {
  constexpr uint32_t kTile = BLOCK * 16;
  const uint32_t tps = static_cast<uint32_t>(a.cs / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const int64_t sstride = (K + ROWS) * a.cs;
  uint32_t t = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x) * ntiles) / gridDim.x));
  const uint32_t tend = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x + 1) * ntiles) / gridDim.x));
  for (; t < tend; t++) {
    const uint32_t s = t / tps;
    uint8_t *dp = a.buf + s * sstride + K * a.cs + (t - s * tps) * kTile;
#pragma unroll
    for (int r = 0; r < ROWS; r++) st<SP>(dp + r * a.cs, threadIdx.x * 16, u32x4{t, s, static_cast<unsigned>(r), 7u});
  }
}

// guide-style float4 copy: n16 vectors, grid-stride, 4 vectors in flight per thread
template <int LP, int SP>
__global__ __launch_bounds__(256) void k_copy(const uint8_t *src, uint8_t *dst, int64_t n16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  int64_t i = blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = ld<LP>(src + (i + u * stride) * 16, 0);
#pragma unroll
    for (int u = 0; u < 4; u++) st<SP>(dst + (i + u * stride) * 16, 0, v[u]);
  }
  for (; i < n16; i += stride) st<SP>(dst + i * 16, 0, ld<LP>(src + i * 16, 0));
}

__global__ void k_fill(uint64_t *p, long n, uint64_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

static hipEvent_t e0, e1;
static int g_reps = 5;
static const char *g_filter = nullptr;

template <class F>
static void timeit(const char *name, double bytes, F go) {
  if (g_filter && !strstr(name, g_filter)) return;
  go();
  CHECK(hipDeviceSynchronize());
  float best = 1e30f, tot = 0;
  for (int r = 0; r < g_reps; r++) {
    CHECK(hipEventRecord(e0, 0));
    go();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    tot += ms;
    if (ms < best) best = ms;
  }
  const float avg = tot / g_reps;
  printf("%-44s avg %7.3f ms  %7.1f GB/s (%.3f of 8T)  best %.3f\n", name, avg, bytes / (avg * 1e-3) / 1e9,
         bytes / (avg * 1e-3) / 8e12, bytes / (best * 1e-3) / 8e12);
  fflush(stdout);
}

#define XOR_VARIANT(BLOCK, VPL, LP, SP, MAP, PF, WPC)                                                           \
  do {                                                                                                          \
    constexpr uint32_t tile = BLOCK * VPL * 16;                                                                 \
    const long ntiles = (cs / tile) * S;                                                                        \
    const int grid = MAP == 2 ? (int)ntiles : ncu * WPC;                                                        \
    char nm[128];                                                                                               \
    snprintf(nm, sizeof nm, "xor B%d V%d L%d S%d M%d PF%d W%d", BLOCK, VPL, LP, SP, MAP, (int)PF, WPC);          \
    timeit(nm, bytes, [&] { hipLaunchKernelGGL((k_xor<10, 4, BLOCK, VPL, LP, SP, MAP, PF>), dim3(grid), dim3(BLOCK), 0, 0, a); }); \
  } while (0)

int main(int argc, char **argv) {
  g_reps = argc > 1 ? atoi(argv[1]) : 5;
  g_filter = argc > 2 ? argv[2] : nullptr;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const long S = 4096, cs = 1 << 20, stripe = 14 * cs;
  uint8_t *buf;
  CHECK(hipMalloc(&buf, S * stripe));
  k_fill<<<4096, 256>>>((uint64_t *)buf, S * stripe / 8, 99);
  uint32_t *sink;
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipDeviceSynchronize());
  uint32_t *queue;
  CHECK(hipMalloc(&queue, 1024));
  const Args a{buf, cs, S, queue};
  const double bytes = (double)S * stripe;
  printf("CUs %d, %ld stripes x 14 x 1 MiB = %.1f GiB per launch\n", ncu, S, bytes / (1 << 30));

  // references
  const int64_t half = 16l << 30;
  timeit("copy float4 16GiB plain", 2.0 * half, [&] { k_copy<0, 0><<<ncu * 32, 256>>>(buf, buf + half, half / 16); });
  timeit("copy float4 16GiB nt", 2.0 * half, [&] { k_copy<1, 1><<<ncu * 32, 256>>>(buf, buf + half, half / 16); });
  timeit("copy hipMemcpyDtoD 16GiB", 2.0 * half, [&] { CHECK(hipMemcpyAsync(buf + half, buf, half, hipMemcpyDeviceToDevice, 0)); });
  k_fill<<<4096, 256>>>((uint64_t *)buf, S * stripe / 8, 99);
  timeit("read-only 10 streams nt", bytes * 10 / 14, [&] { k_read<10, 4, 1024, 1><<<ncu, 1024>>>(a, sink); });
  timeit("read-only 10 streams plain", bytes * 10 / 14, [&] { k_read<10, 4, 1024, 0><<<ncu, 1024>>>(a, sink); });
  timeit("write-only 4 streams nt", bytes * 4 / 14, [&] { k_write<10, 4, 1024, 1><<<ncu, 1024>>>(a); });
  timeit("write-only 4 streams plain", bytes * 4 / 14, [&] { k_write<10, 4, 1024, 0><<<ncu, 1024>>>(a); });

  // the product's pattern and its neighbours
  XOR_VARIANT(1024, 1, 1, 1, 0, true, 1);   // product pattern
  {
    nxec_ctx_t *ctx;
    if (nxec_ctx_create(0, &ctx) == 0) {
      uint8_t coef[4][10];
      for (int r = 0; r < 4; r++)
        for (int j = 0; j < 10; j++) coef[r][j] = (uint8_t)(0x11 * (r + 1) + 3 * j + 1);
      int32_t dst[4] = {10, 11, 12, 13};
      hipStream_t st = (hipStream_t)nxec_ctx_stream(ctx);
      char desc[256];
      for (const char *r : {"16", "8"}) {
        setenv("NXEC_LDS_R", r, 1);
        nxec_describe_launch(ctx, 4, 10, cs, S, desc, sizeof desc);
        char nm[300];
        snprintf(nm, sizeof nm, "PRODUCT R=%s %s", r, desc);
        timeit(nm, bytes, [&] {
          nxec_stripes_mul(ctx, 4, 10, &coef[0][0], buf, nullptr, cs, stripe, buf, dst, cs, stripe, nullptr, cs, S, st);
          CHECK(hipStreamSynchronize(st));
        });
      }
      unsetenv("NXEC_LDS_R");
      nxec_ctx_destroy(ctx);
    }
  }
#define PHASE_VARIANT(T, PH, P, RF)                                                                        \
  timeit("phase T" #T " ph" #PH " P" #P " RF" #RF, bytes,                                                 \
         [&] { hipLaunchKernelGGL((k_phase<10, 4, T, PH, P, RF>), dim3(ncu), dim3(1024), 0, 0, a); })
  XOR_VARIANT(1024, 1, 1, 1, 3, true, 1);
  XOR_VARIANT(1024, 1, 1, 1, 3, false, 1);
  XOR_VARIANT(1024, 1, 1, 1, 1, true, 1);
  XOR_VARIANT(1024, 1, 1, 1, 1, true, 2);
  XOR_VARIANT(1024, 1, 1, 1, 2, false, 1);
  XOR_VARIANT(512, 1, 1, 1, 2, false, 1);
  XOR_VARIANT(256, 1, 1, 1, 2, false, 1);
  XOR_VARIANT(256, 2, 1, 1, 2, false, 1);
  XOR_VARIANT(512, 2, 1, 1, 0, false, 2);
  XOR_VARIANT(256, 4, 1, 1, 0, false, 4);
  XOR_VARIANT(256, 1, 1, 1, 3, true, 4);
  XOR_VARIANT(1024, 1, 0, 1, 2, false, 1);
  XOR_VARIANT(256, 1, 0, 1, 2, false, 1);
  XOR_VARIANT(256, 1, 1, 0, 2, false, 1);
#define QUEUE_VARIANT(BLOCK, G, XCDQ, PF, WPC)                                                                   \
  timeit("queue B" #BLOCK " G" #G " xcd" #XCDQ " PF" #PF " W" #WPC, bytes, [&] {                                \
    CHECK(hipMemsetAsync(queue, 0, 1024, 0));                                                                   \
    hipLaunchKernelGGL((k_queue<10, 4, BLOCK, G, XCDQ, PF>), dim3(ncu * WPC), dim3(BLOCK), 0, 0, a);           \
  })
  QUEUE_VARIANT(1024, 1, false, false, 1);
#define QPOL(LP, SP)                                                                                              \
  timeit("queue G1 LP" #LP " SP" #SP, bytes, [&] {                                                               \
    CHECK(hipMemsetAsync(queue, 0, 1024, 0));                                                                   \
    hipLaunchKernelGGL((k_queue<10, 4, 1024, 1, false, false, LP, SP>), dim3(ncu), dim3(1024), 0, 0, a);       \
  })
  QPOL(0, 0);
  QPOL(0, 1);
  QPOL(1, 0);
  QPOL(2, 1);
  QPOL(3, 1);
  QPOL(1, 2);
  QPOL(1, 3);
  QPOL(3, 3);
  QPOL(2, 2);
  QUEUE_VARIANT(1024, 1, false, false, 1);
  CHECK(hipFree(buf));
  return 0;
}
