// Design probe (not product): read bandwidth of 16-byte global loads at a
// 16-byte-aligned, a 4-byte-aligned and a byte-misaligned offset, and of the
// two-load form (dwordx4 at the 4-byte-aligned address below + one dword
// after it, shifted with v_alignbyte).  Each lane walks a 256-byte window per
// step like k_files_md5's code lanes (16 lanes x 16 B), 4 GiB read per launch.
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench/unaligned_loads.hip -o build/unaligned_loads
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(1))) uint32_t g_u32;

__global__ void k_read(const uint8_t *base, int64_t nvec, int off, int mode, uint32_t *out) {
  const int64_t tid = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  const int64_t nthr = int64_t(gridDim.x) * blockDim.x;
  uint32_t acc = 0;
  for (int64_t i = tid; i < nvec; i += nthr) {
    const uint8_t *p = base + i * 16 + off;
    if (mode == 0) {
      const u32x4 v = *(const g_u32x4 *)(uintptr_t)p;
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    } else {  // dwordx4 at the 4-byte-aligned address below + the next dword, byte shift
      const uint8_t *a4 = (const uint8_t *)((uintptr_t)p & ~uintptr_t(3));
      const u32x4 v = *(const g_u32x4 *)(uintptr_t)a4;
      const uint32_t e = *(const g_u32 *)(uintptr_t)(a4 + 16);
      const uint32_t r = (uint32_t)((uintptr_t)p & 3);
      acc ^= __builtin_amdgcn_alignbyte(v.y, v.x, r) ^ __builtin_amdgcn_alignbyte(v.z, v.y, r) ^
             __builtin_amdgcn_alignbyte(v.w, v.z, r) ^ __builtin_amdgcn_alignbyte(e, v.w, r);
    }
  }
  out[tid] = acc;
}

int main() {
  const size_t bytes = size_t(4) << 30;
  uint8_t *d = nullptr;
  uint32_t *out = nullptr;
  if (hipMalloc(&d, bytes + 64) != hipSuccess || hipMalloc(&out, sizeof(uint32_t) << 22) != hipSuccess) return 1;
  hipMemset(d, 1, bytes + 64);
  const int64_t nvec = int64_t(bytes / 16);
  const int block = 256, grid = 256 * 16;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const struct {
    int off, mode;
    const char *name;
  } cases[] = {{0, 0, "aligned dwordx4"},      {4, 0, "4-byte-aligned dwordx4"}, {1, 0, "byte-misaligned dwordx4"},
               {7, 0, "byte-misaligned +7"},   {1, 1, "dwordx4 + dword, alignbyte (off 1)"},
               {0, 1, "dwordx4 + dword (off 0)"}};
  for (auto &c : cases) {
    hipLaunchKernelGGL(k_read, dim3(grid), dim3(block), 0, 0, d, nvec, c.off, c.mode, out);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_read, dim3(grid), dim3(block), 0, 0, d, nvec, c.off, c.mode, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    std::printf("%-38s %8.3f ms  %7.1f GB/s\n", c.name, ms, bytes / (ms * 1e-3) / 1e9);
  }
  hipFree(d);
  hipFree(out);
  return 0;
}
