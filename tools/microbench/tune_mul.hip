// Tuning probe for the product stripe-multiply kernel (nxec_kernels.hip):
// same LDS-table algorithm, with knobs for the memory side.  Design
// exploration only; the winning configuration is folded into the product.
//
//   NTL  : nontemporal (streaming) source loads
//   NTS  : nontemporal parity stores
//   PF   : software prefetch of the next tile's sources before computing this one
//   VPL  : 16-byte vectors per lane per tile (1 or 2, the 2nd one NT*16 bytes further)
//
// Build: hipcc --offload-arch=gfx950 -O3 -I../../include -o tune_mul tune_mul.hip \
//          -L../../nexoedge_amd/lib -lnxec -Wl,-rpath,'$ORIGIN/../../nexoedge_amd/lib'
// (also: make tune)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "nxec.h"
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                   \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                    \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

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

struct Args {
  const uint8_t *src;
  uint8_t *dst;
  int64_t cs;
  int64_t cstride;  // chunk stride (cs + pad)
  int64_t nstripes;
  int k, rows;
  uint8_t coef[4 * 32];
};

template <bool NTL>
__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
  if (NTL) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  return *reinterpret_cast<const u32x4 *>(p);
}
template <bool NTS>
__device__ __forceinline__ void st(uint8_t *p, u32x4 v) {
  if (NTS)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
  else
    *reinterpret_cast<u32x4 *>(p) = v;
}

template <int R>
__device__ __forceinline__ void lookup16(const char *tb, const u32x4 d, uint32_t acc[16]) {
  const uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t x = (w[q] >> (8 * b)) & 0xffu;
      acc[4 * q + b] ^= *reinterpret_cast<const uint32_t *>(tb + x * (4 * R));
    }
}

template <bool NTS>
__device__ __forceinline__ void store_rows(uint8_t *d0, int64_t cs, int rows, const uint32_t acc[16]) {
  uint32_t o[4][4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t a0 = acc[4 * q], a1 = acc[4 * q + 1], a2 = acc[4 * q + 2], a3 = acc[4 * q + 3];
    const uint32_t lo01 = __builtin_amdgcn_perm(a1, a0, 0x05010400u), hi01 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);
    const uint32_t lo23 = __builtin_amdgcn_perm(a3, a2, 0x05010400u), hi23 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
    o[0][q] = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
    o[1][q] = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
    o[2][q] = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
    o[3][q] = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
  }
#pragma unroll
  for (int r = 0; r < 4; r++)
    if (r < rows) st<NTS>(d0 + r * cs, u32x4{o[r][0], o[r][1], o[r][2], o[r][3]});
}

// PF: 0 none, 1 conditional next-tile prefetch, 2 unconditional (last tile re-reads itself)
template <int K, int R, int NT, int VPL, bool NTL, bool NTS, int PF>
__global__ __launch_bounds__(NT) void k_tune(const Args a) {
  extern __shared__ uint32_t tab[];
  for (int i = threadIdx.x; i < K * 256; i += NT) {
    const int j = i >> 8;
    const uint32_t x = i & 255;
    uint32_t e = 0;
    for (int r = 0; r < a.rows; r++) e |= gf_mul_dev(a.coef[r * K + j], x) << (8 * r);
#pragma unroll
    for (int c = 0; c < R; c++) tab[i * R + c] = e;
  }
  __syncthreads();
  const char *tl = reinterpret_cast<const char *>(tab) + (threadIdx.x % R) * 4;
  const uint32_t tile_bytes = NT * 16 * VPL;
  const uint32_t tps = static_cast<uint32_t>(a.cs / tile_bytes);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const int64_t sstride = static_cast<int64_t>(K + 4) * a.cstride;  // [stripe][k data][4 parity]
  uint32_t t = blockIdx.x;
  if (t >= ntiles) return;
  if constexpr (PF >= 3) {  // ping-pong buffers, manual 2x unroll: no register copies, no waits on the prefetch
    static_assert(VPL == 1, "PF3 is VPL 1");
    // PF 3: tiles interleaved over workgroups (t, t+grid, ...); PF 4: each
    // workgroup owns a contiguous run of tiles (stays inside a few stripes)
    uint32_t tend = ntiles, tstep = gridDim.x;
    if (PF == 4) {
      t = static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x) * ntiles) / gridDim.x);
      tend = static_cast<uint32_t>((static_cast<uint64_t>(blockIdx.x + 1) * ntiles) / gridDim.x);
      tstep = 1;
      if (t >= tend) return;
    }
    auto ld1 = [&](uint32_t tt, u32x4 (&dd)[K]) {
      const uint32_t s = tt / tps;
      const uint32_t off = (tt - s * tps) * tile_bytes + threadIdx.x * 16;
      const uint8_t *sp = a.src + s * sstride + off;
#pragma unroll
      for (int j = 0; j < K; j++) dd[j] = ld<NTL>(sp + j * a.cstride);
    };
    auto comp = [&](uint32_t tt, const u32x4 (&dd)[K]) {
      const uint32_t s = tt / tps;
      const uint32_t off = (tt - s * tps) * tile_bytes + threadIdx.x * 16;
      uint8_t *dp = a.dst + s * sstride + K * a.cstride + off;
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j++) lookup16<R>(tl + j * 1024 * R, dd[j], acc);
      store_rows<NTS>(dp, a.cstride, a.rows, acc);
    };
    u32x4 A[K], B[K];
    ld1(t, A);
    while (true) {
      uint32_t tb = t + tstep;
      ld1(tb < tend ? tb : t, B);
      __builtin_amdgcn_sched_barrier(0);
      comp(t, A);
      if (tb >= tend) break;
      t = tb;
      uint32_t ta = t + tstep;
      ld1(ta < tend ? ta : t, A);
      __builtin_amdgcn_sched_barrier(0);
      comp(t, B);
      if (ta >= tend) break;
      t = ta;
    }
    return;
  }
  u32x4 d[VPL][K];
  auto load = [&](uint32_t tt, u32x4 (&dd)[VPL][K]) {
    const uint32_t s = tt / tps;
    const uint32_t off = (tt - s * tps) * tile_bytes + threadIdx.x * 16;
    const uint8_t *sp = a.src + s * sstride + off;
#pragma unroll
    for (int v = 0; v < VPL; v++)
#pragma unroll
      for (int j = 0; j < K; j++) dd[v][j] = ld<NTL>(sp + j * a.cstride + v * NT * 16);
  };
  load(t, d);
  for (; t < ntiles; t += gridDim.x) {
    u32x4 nx[VPL][K];
    const bool more = PF && (t + gridDim.x < ntiles);
    if (PF == 1 && more) load(t + gridDim.x, nx);
    if (PF == 2) {
      load(more ? t + gridDim.x : t, nx);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch at the top of the iteration
    }
    const uint32_t s = t / tps;
    const uint32_t off = (t - s * tps) * tile_bytes + threadIdx.x * 16;
    uint8_t *dp = a.dst + s * sstride + K * a.cstride + off;
#pragma unroll
    for (int v = 0; v < VPL; v++) {
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j++) lookup16<R>(tl + j * 1024 * R, d[v][j], acc);
      store_rows<NTS>(dp + v * NT * 16, a.cstride, a.rows, acc);
    }
    if (PF == 2) {
#pragma unroll
      for (int v = 0; v < VPL; v++)
#pragma unroll
        for (int j = 0; j < K; j++) d[v][j] = nx[v][j];
    } else if (PF == 1) {
      if (more) {
#pragma unroll
        for (int v = 0; v < VPL; v++)
#pragma unroll
          for (int j = 0; j < K; j++) d[v][j] = nx[v][j];
      }
    } else if (t + gridDim.x < ntiles) {
      load(t + gridDim.x, d);
    }
  }
}

__global__ void k_fill(uint64_t *p, long n, uint64_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

__global__ void k_sum(const uint64_t *p, long n, unsigned long long *out) {
  uint64_t a = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    a += p[i] * (uint64_t)(2 * i + 1);
  atomicAdd(out, (unsigned long long)a);
}

__global__ void k_copy(const u32x4 *s, u32x4 *d, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) d[i] = s[i];
}
__global__ void k_read(const u32x4 *s, long n, unsigned *out) {
  u32x4 a = {0, 0, 0, 0};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) a ^= s[i];
  if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678u) *out = 1;
}

struct Variant {
  const char *name;
  void (*fn)(Args);
  int nt, lds, wgs_per_cu;
};

#define V(K, R, NT, VPL, NTL, NTS, PF, W) \
  Variant { #K "_R" #R "_NT" #NT "_VPL" #VPL "_ntl" #NTL "_nts" #NTS "_pf" #PF "_w" #W, k_tune<K, R, NT, VPL, NTL, NTS, PF>, NT, K * 1024 * R, W }

int main(int argc, char **argv) {
  constexpr int K = 10;
  const long cs = 1 << 20;
  const long S = argc > 1 ? atol(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const long pad = argc > 3 ? atol(argv[3]) : 0;
  const long cstride = cs + pad;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  uint8_t *buf;
  const long stripe = (K + 4) * cstride;
  CHECK(hipMalloc(&buf, S * stripe));
  k_fill<<<2048, 256>>>((uint64_t *)buf, S * stripe / 8, 777);
  unsigned long long *sum;
  CHECK(hipMalloc(&sum, 8));
  Args a{};
  a.src = buf;
  a.dst = buf;
  a.cs = cs;
  a.cstride = cstride;
  a.nstripes = S;
  a.k = K;
  a.rows = 4;
  // RS(14,10) parity rows (gf_gen_rs_matrix): row r coefficient j = (2^r)^j
  auto gm = [](uint32_t x, uint32_t y) {
    uint32_t p = 0;
    for (int i = 0; i < 8; i++) {
      if (y & 1) p ^= x;
      x = (x << 1) ^ ((x & 0x80) ? 0x11d : 0);
      y >>= 1;
    }
    return p;
  };
  for (int r = 0; r < 4; r++) {
    uint32_t g = 1;
    for (int i = 0; i < r; i++) g = gm(g, 2);
    uint32_t p = 1;
    for (int j = 0; j < K; j++) {
      a.coef[r * K + j] = p;
      p = gm(p, g);
    }
  }
  std::vector<Variant> vs = {
      V(10, 16, 1024, 1, false, false, 0, 1), V(10, 16, 1024, 1, true, true, 0, 1),
      V(10, 16, 1024, 1, true, true, 1, 1),    V(10, 16, 1024, 2, true, true, 0, 1),
      V(10, 8, 512, 1, true, true, 1, 2),      V(10, 8, 512, 1, true, true, 0, 2),
      V(10, 1, 1024, 1, true, true, 0, 2),    V(10, 1, 256, 1, true, true, 0, 8),
      V(10, 4, 256, 1, true, true, 1, 4),      V(10, 16, 1024, 1, true, true, 1, 1),
  };

  if (getenv("TUNE_FEW"))
    vs = {V(10, 16, 1024, 1, true, true, 3, 1), V(10, 16, 1024, 1, true, true, 4, 1), V(10, 8, 512, 1, true, true, 4, 2),
          V(10, 16, 1024, 1, true, true, 3, 1), V(10, 16, 1024, 1, true, true, 4, 1)};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = (double)S * (K + 4) * cs;
  printf("pad %ld (chunk stride %ld)\n", pad, cstride);
  unsigned long long ref = 0;
  // the product kernel (libnxec) on the same buffer, same process: A/B against the probes
  auto run_product = [&]() {
    nxec_ctx_t *ctx = nullptr;
    if (nxec_ctx_create(0, &ctx) != 0) {
      printf("nxec_ctx_create: %s\n", nxec_last_error());
      exit(1);
    }
    for (int pass = 0; pass < 2; pass++) {
      float tot = 0, best = 1e30f;
      nxec_rs_encode_stripes(ctx, K + 4, K, buf, cstride, stripe, cs, S, nullptr);
      CHECK(hipDeviceSynchronize());
      for (int r = 0; r < reps; r++) {
        CHECK(hipEventRecord(e0, (hipStream_t)nxec_ctx_stream(ctx)));
        nxec_rs_encode_stripes(ctx, K + 4, K, buf, cstride, stripe, cs, S, nullptr);
        CHECK(hipEventRecord(e1, (hipStream_t)nxec_ctx_stream(ctx)));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        tot += ms;
        best = ms < best ? ms : best;
      }
      CHECK(hipMemset(sum, 0, 8));
      k_sum<<<1024, 256>>>((const uint64_t *)buf, S * stripe / 8, sum);
      unsigned long long h;
      CHECK(hipMemcpy(&h, sum, 8, hipMemcpyDeviceToHost));
      printf("%-44s avg %7.3f ms best %7.3f ms  avg %7.1f GB/s (%.3f of 8T)  best %.3f  %s\n", "PRODUCT nxec_rs_encode_stripes",
             tot / reps, best, bytes / (tot / reps * 1e-3) / 1e9, bytes / (tot / reps * 1e-3) / 8e12,
             bytes / (best * 1e-3) / 8e12, h == ref ? "MATCH" : "MISMATCH");
    }
    nxec_ctx_destroy(ctx);
  };
  run_product();
  for (size_t i = 0; i < vs.size(); i++) {
    CHECK(hipFuncSetAttribute((const void *)vs[i].fn, hipFuncAttributeMaxDynamicSharedMemorySize, vs[i].lds));
    auto go = [&]() { hipLaunchKernelGGL(vs[i].fn, dim3(ncu * vs[i].wgs_per_cu), dim3(vs[i].nt), vs[i].lds, 0, a); };
    go();
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    float best = 1e30f, tot = 0;
    for (int r = 0; r < reps; r++) {
      CHECK(hipEventRecord(e0));
      go();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      tot += ms;
    }
    CHECK(hipMemset(sum, 0, 8));
    k_sum<<<1024, 256>>>((const uint64_t *)buf, S * stripe / 8, sum);
    unsigned long long h;
    CHECK(hipMemcpy(&h, sum, 8, hipMemcpyDeviceToHost));
    if (i == 0) ref = h;
    printf("%-44s avg %7.3f ms best %7.3f ms  avg %7.1f GB/s (%.3f of 8T)  best %.3f  %s\n", vs[i].name, tot / reps, best,
           bytes / (tot / reps * 1e-3) / 1e9, bytes / (tot / reps * 1e-3) / 8e12, bytes / (best * 1e-3) / 8e12,
           h == ref ? "MATCH" : "MISMATCH");
  }
  run_product();
  // bandwidth references on the same buffer
  if (!getenv("TUNE_FEW")) {
    const long n16 = S * stripe / 16 / 2;
    unsigned *o;
    CHECK(hipMalloc(&o, 4));
    for (int g : {2048, 4096, 8192}) {
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; r++) k_copy<<<g, 256>>>((const u32x4 *)buf, (u32x4 *)(buf + n16 * 16), n16);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("copy grid %d: %.1f GB/s (read+write)\n", g, 2.0 * n16 * 16 / (ms / reps * 1e-3) / 1e9);
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; r++) k_read<<<g, 256>>>((const u32x4 *)buf, 2 * n16, o);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("read grid %d: %.1f GB/s\n", g, 2.0 * n16 * 16 / (ms / reps * 1e-3) / 1e9);
    }
  }
  return 0;
}
