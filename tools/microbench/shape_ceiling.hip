// Design probe: for each stripe shape (k sources -> rows outputs), how close is
// the LDS-table kernel to the memory ceiling of the same access pattern, and
// would a VALU-only lookup (v_perm_b32 nibble tables, no LDS) do better?
//
//   mode 0  xor   : same loads/stores, outputs = XOR of sources (memory ceiling)
//   mode 1  lds   : the product's LDS-table algorithm (R copies)
//   mode 2  perm  : GF multiply by 16-entry nibble tables in VGPRs via v_perm_b32
//                   (4 bytes per instruction; per-byte select by the nibble's bit 3
//                   through v_perm sign-replication selectors + v_bfi)
//   PRODUCT       : libnxec nxec_stripes_mul on the same buffers
//
// Build: make tune
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

static uint32_t gm(uint32_t x, uint32_t y) {
  uint32_t p = 0;
  for (int i = 0; i < 8; i++) {
    if (y & 1) p ^= x;
    x = (x << 1) ^ ((x & 0x80) ? 0x11d : 0);
    y >>= 1;
  }
  return p;
}

struct Args {
  uint8_t *buf;            // [stripe][k + rows][cs]
  const uint32_t *ptab;    // lds mode: [k][256] packed rows;  perm mode: [rows][k][8] nibble tables
  int64_t cs, nstripes;
};

__device__ __forceinline__ u32x4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const u32x4 *)p); }
__device__ __forceinline__ void stnt(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (u32x4 *)p); }

// GF multiply of the 4 bytes of x by the coefficient whose nibble tables are
// t[0..3] (c*0..15) and t[4..7] (c*(0..15)<<4); masks precomputed per x.
__device__ __forceinline__ uint32_t perm_mul(const uint32_t *t, uint32_t nl, uint32_t nh, uint32_t ml, uint32_t mh) {
  const uint32_t l0 = __builtin_amdgcn_perm(t[1], t[0], nl), l1 = __builtin_amdgcn_perm(t[3], t[2], nl);
  const uint32_t h0 = __builtin_amdgcn_perm(t[5], t[4], nh), h1 = __builtin_amdgcn_perm(t[7], t[6], nh);
  return ((ml & l1) | (~ml & l0)) ^ ((mh & h1) | (~mh & h0));
}

template <int K, int ROWS, int MODE, int R>
__global__ __launch_bounds__(1024) void k_shape(const Args a) {
  extern __shared__ uint32_t tab[];
  if (MODE == 1) {
    for (int i = threadIdx.x; i < K * 256; i += 1024)
#pragma unroll
      for (int c = 0; c < R; c++) tab[i * R + c] = a.ptab[i];
  } else if (MODE == 2) {
    for (int i = threadIdx.x; i < ROWS * K * 8; i += 1024) tab[i] = a.ptab[i];
  }
  __syncthreads();
  const char *tl = reinterpret_cast<const char *>(tab) + (threadIdx.x % R) * 4;
  const uint32_t tps = static_cast<uint32_t>(a.cs / (1024 * 16));
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const int64_t sstride = (K + ROWS) * a.cs;
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint32_t s = t / tps;
    const uint32_t off = (t - s * tps) * 16384 + threadIdx.x * 16;
    const uint8_t *sp = a.buf + s * sstride + off;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; j++) d[j] = ldnt(sp + j * a.cs);
    uint32_t out[ROWS][4];
    if (MODE == 0) {
      u32x4 x = d[0];
#pragma unroll
      for (int j = 1; j < K; j++) x ^= d[j];
#pragma unroll
      for (int r = 0; r < ROWS; r++) {
        out[r][0] = x.x + r;
        out[r][1] = x.y;
        out[r][2] = x.z;
        out[r][3] = x.w;
      }
    } else if (MODE == 1) {
      uint32_t acc[16] = {};
#pragma unroll
      for (int j = 0; j < K; j++) {
        const uint32_t w[4] = {d[j].x, d[j].y, d[j].z, d[j].w};
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
          for (int b = 0; b < 4; b++)
            acc[4 * q + b] ^= *(const uint32_t *)(tl + j * 1024 * R + ((w[q] >> (8 * b)) & 0xff) * (4 * R));
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t a0 = acc[4 * q], a1 = acc[4 * q + 1], a2 = acc[4 * q + 2], a3 = acc[4 * q + 3];
        const uint32_t lo01 = __builtin_amdgcn_perm(a1, a0, 0x05010400u), hi01 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);
        const uint32_t lo23 = __builtin_amdgcn_perm(a3, a2, 0x05010400u), hi23 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
        const uint32_t o[4] = {__builtin_amdgcn_perm(lo23, lo01, 0x05040100u), __builtin_amdgcn_perm(lo23, lo01, 0x07060302u),
                               __builtin_amdgcn_perm(hi23, hi01, 0x05040100u), __builtin_amdgcn_perm(hi23, hi01, 0x07060302u)};
#pragma unroll
        for (int r = 0; r < ROWS; r++) out[r][q] = o[r];
      }
    } else {
#pragma unroll
      for (int r = 0; r < ROWS; r++)
#pragma unroll
        for (int q = 0; q < 4; q++) out[r][q] = 0;
      // opaque zero: keeps the table reads inside the loop (hoisting them would
      // need ROWS*K*8 registers)
      uint32_t z;
      asm volatile("s_mov_b32 %0, 0" : "=s"(z));
      const uint32_t *tt = tab + z;
#pragma unroll
      for (int j = 0; j < K; j++) {
        const uint32_t w[4] = {d[j].x, d[j].y, d[j].z, d[j].w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t x = w[q];
          const uint32_t nl = x & 0x07070707u, nh = (x >> 4) & 0x07070707u;
          const uint32_t x4 = x << 4;
          // sign-replication selectors 8..11 copy bit 7 of pool bytes 1,3,5,7
          const uint32_t ml = __builtin_amdgcn_perm(x4, x4 << 8, 0x0B090A08u);
          const uint32_t mh = __builtin_amdgcn_perm(x, x << 8, 0x0B090A08u);
#pragma unroll
          for (int r = 0; r < ROWS; r++) out[r][q] ^= perm_mul(tt + (r * K + j) * 8, nl, nh, ml, mh);
        }
      }
    }
    uint8_t *dp = a.buf + s * sstride + K * a.cs + off;
#pragma unroll
    for (int r = 0; r < ROWS; r++) stnt(dp + r * a.cs, u32x4{out[r][0], out[r][1], out[r][2], out[r][3]});
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

template <int K, int ROWS>
void run_shape(int ncu, long S, int reps, nxec_ctx_t *ctx) {
  const long cs = 1 << 20, stripe = (K + ROWS) * cs;
  uint8_t *buf;
  CHECK(hipMalloc(&buf, S * stripe));
  k_fill<<<2048, 256>>>((uint64_t *)buf, S * stripe / 8, 4242);
  unsigned long long *sum;
  CHECK(hipMalloc(&sum, 8));
  uint8_t coef[ROWS][K];
  for (int r = 0; r < ROWS; r++)
    for (int j = 0; j < K; j++) coef[r][j] = (uint8_t)gm(r + 1, gm(j + 1, 0x53) ^ (j * 7 + r));
  std::vector<uint32_t> packed(K * 256), nib(ROWS * K * 8);
  for (int j = 0; j < K; j++)
    for (int x = 0; x < 256; x++) {
      uint32_t e = 0;
      for (int r = 0; r < ROWS; r++) e |= gm(coef[r][j], x) << (8 * r);
      packed[j * 256 + x] = e;
    }
  for (int r = 0; r < ROWS; r++)
    for (int j = 0; j < K; j++)
      for (int i = 0; i < 16; i++) {
        uint32_t *t = &nib[(r * K + j) * 8];
        t[i / 4] |= gm(coef[r][j], i) << (8 * (i % 4));
        t[4 + i / 4] |= gm(coef[r][j], i << 4) << (8 * (i % 4));
      }
  uint32_t *dpk, *dnb;
  CHECK(hipMalloc(&dpk, packed.size() * 4));
  CHECK(hipMalloc(&dnb, nib.size() * 4));
  CHECK(hipMemcpy(dpk, packed.data(), packed.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dnb, nib.data(), nib.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = (double)S * (K + ROWS) * cs;
  constexpr int R = K <= 10 ? 16 : 8;
  struct M {
    const char *name;
    void (*fn)(Args);
    int lds;
    const uint32_t *tab;
  } ms[] = {{"xor(ceiling)", k_shape<K, ROWS, 0, 1>, 0, nullptr},
            {"lds", k_shape<K, ROWS, 1, R>, K * 1024 * R, dpk},
            {"perm", k_shape<K, ROWS, 2, 1>, ROWS * K * 32, dnb},
            {"PRODUCT", nullptr, 0, nullptr},
            {"PRODUCT-static", nullptr, 0, nullptr}};
  unsigned long long ref = 0;
  for (int mi = 0; mi < 5; mi++) {
    if (mi == 4) setenv("NXEC_TILE_ORDER", "static", 1);
    Args a{buf, ms[mi].tab, cs, S};
    auto go = [&]() {
      if (ms[mi].fn) {
        hipLaunchKernelGGL(ms[mi].fn, dim3(ncu), dim3(1024), ms[mi].lds, 0, a);
      } else {
        int32_t dst[ROWS];
        for (int r = 0; r < ROWS; r++) dst[r] = K + r;
        nxec_stripes_mul(ctx, ROWS, K, &coef[0][0], buf, nullptr, cs, stripe, buf, dst, cs, stripe, nullptr, cs, S,
                         nullptr);
      }
    };
    if (ms[mi].fn)
      CHECK(hipFuncSetAttribute((const void *)ms[mi].fn, hipFuncAttributeMaxDynamicSharedMemorySize, ms[mi].lds > 0 ? ms[mi].lds : 1024));
    go();
    CHECK(hipDeviceSynchronize());
    hipStream_t st = ms[mi].fn ? 0 : (hipStream_t)nxec_ctx_stream(ctx);
    float tot = 0;
    for (int r = 0; r < reps; r++) {
      CHECK(hipEventRecord(e0, st));
      go();
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms_;
      CHECK(hipEventElapsedTime(&ms_, e0, e1));
      tot += ms_;
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(sum, 0, 8));
    k_sum<<<1024, 256>>>((const uint64_t *)buf, S * stripe / 8, sum);
    unsigned long long h;
    CHECK(hipMemcpy(&h, sum, 8, hipMemcpyDeviceToHost));
    if (mi == 1) ref = h;
    printf("k=%2d rows=%d %-13s %7.3f ms  %7.1f GB/s  frac8T %.3f  %s\n", K, ROWS, ms[mi].name, tot / reps,
           bytes / (tot / reps * 1e-3) / 1e9, bytes / (tot / reps * 1e-3) / 8e12,
           mi == 0 ? "" : (h == ref ? "MATCH" : "MISMATCH"));
    unsetenv("NXEC_TILE_ORDER");
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(dpk));
  CHECK(hipFree(dnb));
  CHECK(hipFree(sum));
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  nxec_ctx_t *ctx;
  if (nxec_ctx_create(0, &ctx)) {
    printf("%s\n", nxec_last_error());
    return 1;
  }
  const int ncu = prop.multiProcessorCount;
  run_shape<10, 4>(ncu, 4096, reps, ctx);
  run_shape<12, 1>(ncu, 4096, reps, ctx);
  run_shape<16, 4>(ncu, 2048, reps, ctx);
  run_shape<4, 1>(ncu, 4096, reps, ctx);
  nxec_ctx_destroy(ctx);
  return 0;
}
