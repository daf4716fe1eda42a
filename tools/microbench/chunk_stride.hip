// Design probe: product stripe-multiply rate vs chunk size and chunk stride
// (RS(16,4) encode, ~32 GiB per launch): does a power-of-two chunk stride of
// 4 MiB alias HBM channels where 1 MiB does not, and does padding help?
// Build: make tune
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "nxec.h"

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  nxec_ctx_t *ctx;
  if (nxec_ctx_create(0, &ctx)) return 1;
  hipStream_t st = (hipStream_t)nxec_ctx_stream(ctx);
  const int k = 16, rows = 4, n = 20;
  uint8_t coef[4 * 16];
  for (int i = 0; i < 4 * 16; i++) coef[i] = (uint8_t)(i * 37 + 11);
  const int64_t budget = 34ll << 30;
  uint8_t *buf;
  CHECK(hipMalloc(&buf, budget));
  nxec_fill_random(buf, budget, 7, st);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int64_t sizes[] = {65536, 262144, 1 << 20, 2 << 20, 4 << 20};
  const int64_t pads[] = {0, 256, 4096, 65536};
  for (int64_t cs : sizes)
    for (int64_t pad : pads) {
      const int64_t cstride = cs + pad, sstride = n * cstride;
      const int64_t ns = (32ll << 30) / (n * cs);
      if (ns * sstride > budget) continue;
      int32_t dst[4] = {16, 17, 18, 19};
      auto go = [&] {
        int rc = nxec_stripes_mul(ctx, rows, k, coef, buf, nullptr, cstride, sstride, buf, dst, cstride, sstride,
                                  nullptr, cs, ns, st);
        if (rc) { printf("err %s\n", nxec_last_error()); exit(1); }
      };
      go();
      CHECK(hipStreamSynchronize(st));
      float tot = 0;
      for (int r = 0; r < reps; r++) {
        CHECK(hipEventRecord(e0, st));
        go();
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        tot += ms;
      }
      const double bytes = (double)ns * n * cs, ms = tot / reps;
      const char *sgv = getenv("NXEC_STRIPE_GROUP");
      printf("sg %-2s cs %5ld KiB pad %6ld  stripes %6ld  %7.3f ms  %7.1f GB/s  frac8T %.3f\n", sgv ? sgv : "1", (long)(cs >> 10), (long)pad,
             (long)ns, ms, bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12);
      fflush(stdout);
    }
  CHECK(hipFree(buf));
  nxec_ctx_destroy(ctx);
  return 0;
}
