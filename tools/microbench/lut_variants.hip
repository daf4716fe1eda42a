// Microbenchmark: GF(2^8) table-lookup strategies for the k-source x 4-row
// stripe multiply on gfx950.  Standalone design probe (not product code):
// it decides which lookup strategy the product kernel in
// nexoedge_amd/csrc/nxec_kernels.hip uses.
//
//   V0  stream     : XOR of the k sources into 4 rows (no GF) -> bandwidth ceiling
//   V1  lds R=1    : one 256-dword table per source, entry = 4 packed row products
//   V2  lds R=8    : same, replicated 8x with copy = lane % 8 in the bank bits
//   V3  lds R=16   : replicated 16x (160 KiB at k=10, one 1024-thread WG per CU)
//   V4  bpermute   : 16-entry nibble tables held in VGPRs, ds_bpermute lookups
//
// Build: hipcc --offload-arch=gfx950 -O3 -o lut_variants lut_variants.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  while (b) { if (b & 1) p ^= a; a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1d : 0)); b >>= 1; }
  return p;
}

__device__ __forceinline__ void transpose_store(const uint32_t acc[16], uint8_t* d0, long cs) {
  uint32_t o[4][4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t a0 = acc[4 * q], a1 = acc[4 * q + 1], a2 = acc[4 * q + 2], a3 = acc[4 * q + 3];
    uint32_t lo01 = __builtin_amdgcn_perm(a1, a0, 0x05010400u);
    uint32_t hi01 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);
    uint32_t lo23 = __builtin_amdgcn_perm(a3, a2, 0x05010400u);
    uint32_t hi23 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
    o[0][q] = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
    o[1][q] = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
    o[2][q] = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
    o[3][q] = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
  }
#pragma unroll
  for (int r = 0; r < 4; r++)
    *(uint4*)(d0 + r * cs) = make_uint4(o[r][0], o[r][1], o[r][2], o[r][3]);
}

template <int K>
__global__ __launch_bounds__(256) void k_stream(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                long cs, long nstripes) {
  const long tile = (long)blockDim.x * 16, tps = cs / tile, nt = tps * nstripes;
  for (long t = blockIdx.x; t < nt; t += gridDim.x) {
    long s = t / tps, off = (t % tps) * tile + threadIdx.x * 16;
    const uint8_t* sp = src + s * K * cs + off;
    uint4 v[K];
#pragma unroll
    for (int j = 0; j < K; j++) v[j] = *(const uint4*)(sp + j * cs);
    uint4 a = v[0];
#pragma unroll
    for (int j = 1; j < K; j++) { a.x ^= v[j].x; a.y ^= v[j].y; a.z ^= v[j].z; a.w ^= v[j].w; }
    uint8_t* dp = dst + s * 4 * cs + off;
#pragma unroll
    for (int r = 0; r < 4; r++) *(uint4*)(dp + r * cs) = a;
  }
}

template <int K, int R, int NT>
__global__ __launch_bounds__(NT) void k_lds(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                            const uint32_t* __restrict__ ptab, long cs, long nstripes, int lds_only) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < K * 256 * R; i += NT) {
    int j = i / (256 * R), x = (i % (256 * R)) / R;
    lds[i] = ptab[j * 256 + x];
  }
  __syncthreads();
  const uint32_t cbase = (threadIdx.x % R) * 4;
  const long tile = (long)NT * 16, tps = cs / tile, nt = tps * nstripes;
  for (long t = blockIdx.x; t < nt; t += gridDim.x) {
    long s = t / tps, off = (t % tps) * tile + threadIdx.x * 16;
    const uint8_t* sp = src + s * K * cs + off;
    uint4 v[K];
#pragma unroll
    for (int j = 0; j < K; j++) v[j] = *(const uint4*)(sp + j * cs);
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0;
    int reps = lds_only ? 64 : 1;
    for (int rep = 0; rep < reps; rep++) {
#pragma unroll
      for (int j = 0; j < K; j++) {
        const char* tb = (const char*)lds + j * 256 * R * 4 + cbase;
        uint32_t w4[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
#pragma unroll
          for (int b = 0; b < 4; b++) {
            uint32_t x = (w4[q] >> (8 * b)) & 0xffu;
            acc[q * 4 + b] ^= *(const uint32_t*)(tb + x * (R * 4));
          }
        }
      }
      if (lds_only) {  // feed back so the loop is not collapsed / hoisted
#pragma unroll
        for (int j = 0; j < K; j++) { v[j].x ^= acc[j]; v[j].y ^= acc[(j + 5) & 15]; v[j].z ^= acc[(j + 10) & 15]; v[j].w ^= acc[(j + 15) & 15]; }
      }
    }
    transpose_store(acc, dst + s * 4 * cs + off, cs);
  }
}

// nibble tables in VGPRs: reg m holds sources 2m (lanes 0..31) and 2m+1 (lanes 32..63);
// within 32 lanes: 0..15 low-nibble table, 16..31 high-nibble table
template <int K>
__global__ __launch_bounds__(256) void k_bperm(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                               const uint32_t* __restrict__ ptab, long cs, long nstripes, int lds_only) {
  constexpr int NR = (K + 1) / 2;
  int treg[NR];
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int m = 0; m < NR; m++) {
    int j = 2 * m + (lane >> 5);
    int n = lane & 15;
    int x = (lane & 16) ? (n << 4) : n;
    treg[m] = (j < K) ? (int)ptab[j * 256 + x] : 0;
  }
  const long tile = (long)blockDim.x * 16, tps = cs / tile, nt = tps * nstripes;
  for (long t = blockIdx.x; t < nt; t += gridDim.x) {
    long s = t / tps, off = (t % tps) * tile + threadIdx.x * 16;
    const uint8_t* sp = src + s * K * cs + off;
    uint4 v[K];
#pragma unroll
    for (int j = 0; j < K; j++) v[j] = *(const uint4*)(sp + j * cs);
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0;
    int reps = lds_only ? 64 : 1;
    for (int rep = 0; rep < reps; rep++) {
#pragma unroll
      for (int j = 0; j < K; j++) {
        uint32_t w4[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
        const uint32_t hb = (j & 1) * 128;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          uint32_t nl = (w4[q] << 2) & 0x3c3c3c3cu;
          uint32_t nh = (w4[q] >> 2) & 0x3c3c3c3cu;
#pragma unroll
          for (int b = 0; b < 4; b++) {
            uint32_t al = ((nl >> (8 * b)) & 0xffu) + hb;
            uint32_t ah = ((nh >> (8 * b)) & 0xffu) + hb + 64;
            uint32_t pl = __builtin_amdgcn_ds_bpermute(al, treg[j >> 1]);
            uint32_t ph = __builtin_amdgcn_ds_bpermute(ah, treg[j >> 1]);
            acc[q * 4 + b] ^= pl ^ ph;
          }
        }
      }
      if (lds_only) {  // feed back so the loop is not collapsed / hoisted
#pragma unroll
        for (int j = 0; j < K; j++) { v[j].x ^= acc[j]; v[j].y ^= acc[(j + 5) & 15]; v[j].z ^= acc[(j + 10) & 15]; v[j].w ^= acc[(j + 15) & 15]; }
      }
    }
    transpose_store(acc, dst + s * 4 * cs + off, cs);
  }
}

__global__ void k_fill(uint64_t* p, long n, uint64_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

__global__ void k_sum(const uint64_t* p, long n, unsigned long long* out) {
  uint64_t a = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    a += p[i] * (uint64_t)(i | 1);
  atomicAdd(out, (unsigned long long)a);
}

int main(int argc, char** argv) {
  const int K = 10;
  long cs = 1 << 20;
  long S = argc > 1 ? atol(argv[1]) : 1024;
  int reps = argc > 2 ? atoi(argv[2]) : 5;
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  int ncu = prop.multiProcessorCount;
  printf("device %s CUs %d S=%ld cs=%ld\n", prop.gcnArchName, ncu, S, cs);
  uint8_t *src, *dst; uint32_t* ptab; unsigned long long* sum;
  CHECK(hipMalloc(&src, S * K * cs)); CHECK(hipMalloc(&dst, S * 4 * cs));
  CHECK(hipMalloc(&ptab, K * 256 * 4)); CHECK(hipMalloc(&sum, 8));
  k_fill<<<2048, 256>>>((uint64_t*)src, S * K * cs / 8, 12345);
  // RS(14,10) parity rows: row r coefficient for source j = (2^r)^j
  std::vector<uint32_t> h(K * 256);
  uint8_t coef[4][K];
  for (int r = 0; r < 4; r++) { uint8_t g = 1; for (int i = 0; i < r; i++) g = gmul(g, 2); uint8_t p = 1;
    for (int j = 0; j < K; j++) { coef[r][j] = p; p = gmul(p, g); } }
  for (int j = 0; j < K; j++) for (int x = 0; x < 256; x++) {
    uint32_t e = 0; for (int r = 0; r < 4; r++) e |= (uint32_t)gmul(coef[r][j], (uint8_t)x) << (8 * r);
    h[j * 256 + x] = e; }
  CHECK(hipMemcpy(ptab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipFuncSetAttribute((const void*)k_lds<K, 16, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize, K * 256 * 16 * 4));
  CHECK(hipFuncSetAttribute((const void*)k_lds<K, 8, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize, K * 256 * 8 * 4));
  CHECK(hipFuncSetAttribute((const void*)k_lds<K, 8, 512>, hipFuncAttributeMaxDynamicSharedMemorySize, K * 256 * 8 * 4));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  double bytes = (double)S * (K + 4) * cs;
  unsigned long long ref_sum = 0;
  for (int mode = 0; mode < 2; mode++) {
    for (int v = 0; v < 7; v++) {
      if (mode == 1 && v == 0) continue;
      long SS = mode ? 64 : S;
      auto launch = [&]() {
        switch (v) {
          case 0: k_stream<K><<<ncu * 8, 256>>>(src, dst, cs, SS); break;
          case 1: k_lds<K, 1, 256><<<ncu * 8, 256, K * 256 * 4>>>(src, dst, ptab, cs, SS, mode); break;
          case 2: k_lds<K, 8, 512><<<ncu * 2, 512, K * 256 * 8 * 4>>>(src, dst, ptab, cs, SS, mode); break;
          case 3: k_lds<K, 8, 1024><<<ncu, 1024, K * 256 * 8 * 4>>>(src, dst, ptab, cs, SS, mode); break;
          case 4: k_lds<K, 16, 1024><<<ncu, 1024, K * 256 * 16 * 4>>>(src, dst, ptab, cs, SS, mode); break;
          case 5: k_bperm<K><<<ncu * 8, 256>>>(src, dst, ptab, cs, SS, mode); break;
          case 6: k_lds<K, 1, 1024><<<ncu * 2, 1024, K * 256 * 4>>>(src, dst, ptab, cs, SS, mode); break;
        }
      };
      const char* names[] = {"stream", "lds_R1_256x8", "lds_R8_512x2", "lds_R8_1024x1", "lds_R16_1024x1", "bperm_256x8", "lds_R1_1024x2"};
      launch(); CHECK(hipGetLastError()); CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < reps; i++) launch();
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
      CHECK(hipMemset(sum, 0, 8));
      k_sum<<<1024, 256>>>((const uint64_t*)dst, SS * 4 * cs / 8, sum);
      unsigned long long hs; CHECK(hipMemcpy(&hs, sum, 8, hipMemcpyDeviceToHost));
      if (mode == 0 && v == 1) ref_sum = hs;
      if (mode == 0) {
        double gbs = (double)SS * (K + 4) * cs / (ms * 1e-3) / 1e9;
        printf("%-18s %8.3f ms  %8.1f GB/s  frac8T %.3f  sum %016llx %s\n", names[v], ms, gbs, gbs / 8000.0, hs,
               v == 0 ? "" : (hs == ref_sum ? "MATCH" : "MISMATCH"));
      } else {
        double lk = (double)SS * K * cs * 64 / (ms * 1e-3);
        printf("ldsonly %-18s %8.3f ms  %8.2f Glookups/s  %.2f lookups/clk/CU@2.1GHz\n", names[v], ms, lk / 1e9,
               lk / (ncu * 2.1e9));
      }
    }
  }
  // CPU spot check of a few bytes of V1 output: recompute
  {
    k_lds<K, 1, 256><<<ncu * 8, 256, K * 256 * 4>>>(src, dst, ptab, cs, S, 0); CHECK(hipDeviceSynchronize());
    int bad = 0;
    for (int t = 0; t < 64; t++) {
      long s = (t * 7919L) % S, off = (t * 104729L) % cs;
      uint8_t in[K]; for (int j = 0; j < K; j++) CHECK(hipMemcpy(&in[j], src + s * K * cs + j * cs + off, 1, hipMemcpyDeviceToHost));
      for (int r = 0; r < 4; r++) { uint8_t o; CHECK(hipMemcpy(&o, dst + s * 4 * cs + r * cs + off, 1, hipMemcpyDeviceToHost));
        uint8_t e = 0; for (int j = 0; j < K; j++) e ^= gmul(coef[r][j], in[j]); if (e != o) bad++; }
    }
    printf("cpu spot check: %s (%d bad)\n", bad ? "FAIL" : "OK", bad);
  }
  return 0;
}
