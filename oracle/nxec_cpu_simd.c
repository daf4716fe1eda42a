/* TEST INFRASTRUCTURE ONLY -- CPU baseline, never linked into libnxec.
 *
 * A production-class CPU stand-in for ISA-L 2.22's SIMD erasure-code kernels
 * (gf_{1..4}vect_dot_prod_{avx2,avx512}.asm behind ec_encode_data,
 * ISA-L ec_highlevel_func.c:95-173), which the reference links in production
 * but which cannot be assembled here (no nasm).  Written from the
 * published split-nibble method, not from ISA-L's sources:
 *
 *   c*x = T_lo[c][x & 15] ^ T_hi[c][x >> 4]       (GF(2^8), poly 0x11d)
 *
 * with the two 16-entry tables held in vector registers and looked up 32/64
 * bytes at a time by vpshufb.  Like ISA-L, up to 4 output rows are produced
 * per pass over the sources (each pass reads the k sources once), and the
 * byte tail uses scalar log/exp.  bench.py's cpu_baseline times it
 * (`kind: "port"`) beside the reference's own base-C build; tests check it
 * against the oracle.
 */
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include "nxec_oracle.h"

typedef struct {
  uint8_t lo[16];
  uint8_t hi[16];
} split_tbl;

static void make_tbl(uint8_t c, split_tbl *t) {
  for (int x = 0; x < 16; x++) {
    t->lo[x] = orc_gf_mul(c, (uint8_t)x);
    t->hi[x] = orc_gf_mul(c, (uint8_t)(x << 4));
  }
}

static void tail_bytes(size_t from, size_t len, int k, int rows, const uint8_t *coef, const uint8_t *const *src,
                       uint8_t *const *dst) {
  for (int r = 0; r < rows; r++)
    for (size_t i = from; i < len; i++) {
      uint8_t s = 0;
      for (int j = 0; j < k; j++) s ^= orc_gf_mul(coef[r * k + j], src[j][i]);
      dst[r][i] = s;
    }
}

/* ---- AVX-512BW: 64 bytes per vpshufb, rows <= 4 per pass ---- */
#define NXO_AVX512 __attribute__((target("avx512f,avx512bw")))
#define NXO_AVX2 __attribute__((target("avx2")))
#define NXO_INLINE static inline __attribute__((always_inline))

NXO_AVX512 NXO_INLINE size_t pass_avx512_r(size_t len, int k, const int rows, const split_tbl *t /* [rows][k] */,
                                          const uint8_t *const *src, uint8_t *const *dst) {
  const __m512i mask = _mm512_set1_epi8(0x0f);
  const size_t n64 = len & ~(size_t)63;
  for (size_t i = 0; i < n64; i += 64) {
    __m512i acc0 = _mm512_setzero_si512(), acc1 = acc0, acc2 = acc0, acc3 = acc0;
    for (int j = 0; j < k; j++) {
      const __m512i x = _mm512_loadu_si512((const void *)(src[j] + i));
      const __m512i lo = _mm512_and_si512(x, mask);
      const __m512i hi = _mm512_and_si512(_mm512_srli_epi64(x, 4), mask);
#define NXO_ROW(r, acc)                                                                                     \
  if (rows > r) {                                                                                           \
    const __m512i tl = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i *)t[r * k + j].lo));           \
    const __m512i th = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i *)t[r * k + j].hi));           \
    acc = _mm512_xor_si512(acc, _mm512_xor_si512(_mm512_shuffle_epi8(tl, lo), _mm512_shuffle_epi8(th, hi))); \
  }
      NXO_ROW(0, acc0)
      NXO_ROW(1, acc1)
      NXO_ROW(2, acc2)
      NXO_ROW(3, acc3)
#undef NXO_ROW
    }
    _mm512_storeu_si512((void *)(dst[0] + i), acc0);
    if (rows > 1) _mm512_storeu_si512((void *)(dst[1] + i), acc1);
    if (rows > 2) _mm512_storeu_si512((void *)(dst[2] + i), acc2);
    if (rows > 3) _mm512_storeu_si512((void *)(dst[3] + i), acc3);
  }
  return n64;
}

/* ---- AVX2: 32 bytes per vpshufb ---- */
NXO_AVX2 NXO_INLINE size_t pass_avx2_r(size_t len, int k, const int rows, const split_tbl *t,
                                      const uint8_t *const *src, uint8_t *const *dst) {
  const __m256i mask = _mm256_set1_epi8(0x0f);
  const size_t n32 = len & ~(size_t)31;
  for (size_t i = 0; i < n32; i += 32) {
    __m256i acc0 = _mm256_setzero_si256(), acc1 = acc0, acc2 = acc0, acc3 = acc0;
    for (int j = 0; j < k; j++) {
      const __m256i x = _mm256_loadu_si256((const __m256i *)(src[j] + i));
      const __m256i lo = _mm256_and_si256(x, mask);
      const __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
#define NXO_ROW(r, acc)                                                                                           \
  if (rows > r) {                                                                                                 \
    const __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[r * k + j].lo));            \
    const __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[r * k + j].hi));            \
    acc = _mm256_xor_si256(acc, _mm256_xor_si256(_mm256_shuffle_epi8(tl, lo), _mm256_shuffle_epi8(th, hi)));      \
  }
      NXO_ROW(0, acc0)
      NXO_ROW(1, acc1)
      NXO_ROW(2, acc2)
      NXO_ROW(3, acc3)
#undef NXO_ROW
    }
    _mm256_storeu_si256((__m256i *)(dst[0] + i), acc0);
    if (rows > 1) _mm256_storeu_si256((__m256i *)(dst[1] + i), acc1);
    if (rows > 2) _mm256_storeu_si256((__m256i *)(dst[2] + i), acc2);
    if (rows > 3) _mm256_storeu_si256((__m256i *)(dst[3] + i), acc3);
  }
  return n32;
}

/* rows as a compile-time constant in each instance (ISA-L keeps one asm
 * routine per row count, gf_{1,2,3,4}vect_dot_prod) */
NXO_AVX512 static size_t pass_avx512(size_t len, int k, int rows, const split_tbl *t, const uint8_t *const *src,
                                     uint8_t *const *dst) {
  switch (rows) {
    case 1: return pass_avx512_r(len, k, 1, t, src, dst);
    case 2: return pass_avx512_r(len, k, 2, t, src, dst);
    case 3: return pass_avx512_r(len, k, 3, t, src, dst);
    default: return pass_avx512_r(len, k, 4, t, src, dst);
  }
}

NXO_AVX2 static size_t pass_avx2(size_t len, int k, int rows, const split_tbl *t, const uint8_t *const *src,
                                 uint8_t *const *dst) {
  switch (rows) {
    case 1: return pass_avx2_r(len, k, 1, t, src, dst);
    case 2: return pass_avx2_r(len, k, 2, t, src, dst);
    case 3: return pass_avx2_r(len, k, 3, t, src, dst);
    default: return pass_avx2_r(len, k, 4, t, src, dst);
  }
}

int orc_simd_level(void) {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512bw")) return 512;
  if (__builtin_cpu_supports("avx2")) return 256;
  return 0;
}

/* dst[r] = sum_j coef[r*k+j] * src[j], r < rows (any rows, passes of 4).
 * level: 512 / 256 / 0 (scalar) or -1 for the best the CPU has.  Returns the
 * level used. */
int orc_simd_encode(int level, size_t len, int k, int rows, const uint8_t *coef, const uint8_t *const *src,
                    uint8_t *const *dst) {
  if (level < 0) level = orc_simd_level();
  split_tbl t[4 * 256];
  for (int r0 = 0; r0 < rows; r0 += 4) {
    const int rr = rows - r0 < 4 ? rows - r0 : 4;
    for (int r = 0; r < rr; r++)
      for (int j = 0; j < k; j++) make_tbl(coef[(r0 + r) * k + j], &t[r * k + j]);
    size_t done = 0;
    if (level >= 512)
      done = pass_avx512(len, k, rr, t, src, dst + r0);
    else if (level >= 256)
      done = pass_avx2(len, k, rr, t, src, dst + r0);
    tail_bytes(done, len, k, rr, coef + r0 * k, src, dst + r0);
  }
  return level;
}

/* ---- the reference's per-stripe coding calls, for bench.py's cpu_baseline ----
 * One call per host thread over a contiguous stripe range, so the timed loop
 * runs entirely in C (no interpreter between stripes).
 *
 * RSCode::encode (rs.cc:57-92): the k data chunks are copied out of the
 * caller's [k][cs] stripe buffer into the stripe's own chunk buffers (rs.cc:80)
 * and the parity is encoded from those copies (rs.cc:89).  Chunk buffers of
 * stripe s: chunks + s * n * cs, chunk i at + i * cs. */
void orc_simd_rscode_encode_range(int level, int n, int k, int64_t cs, int64_t lo, int64_t hi, const uint8_t *data,
                                  uint8_t *chunks, const uint8_t *parity_rows /* (n-k) x k */) {
  const uint8_t *src[256];
  uint8_t *dst[256];
  for (int64_t s = lo; s < hi; s++) {
    uint8_t *st = chunks + s * n * cs;
    memcpy(st, data + s * k * cs, (size_t)(k * cs)); /* rs.cc:80, one copy per chunk in the reference */
    for (int j = 0; j < k; j++) src[j] = st + j * cs;
    for (int r = 0; r < n - k; r++) dst[r] = st + (k + r) * cs;
    if (n > k) orc_simd_encode(level, (size_t)cs, k, n - k, parity_rows, src, dst);
  }
}

/* rows x k matrix applied to the chunks `ids` of every stripe in [lo, hi):
 * the repair rows of rs.cc:204-225 (rows = e, recover) or the k x k inverse of
 * rs.cc:196,228-230 (rows = k, the reference's full-output read decode).
 * Outputs of stripe s at out + s * rows * cs. */
void orc_simd_rscode_decode_range(int level, int n, int k, int64_t cs, int64_t lo, int64_t hi, const uint8_t *chunks,
                                  const int32_t *ids, int rows, const uint8_t *matrix, uint8_t *out) {
  const uint8_t *src[256];
  uint8_t *dst[256];
  for (int64_t s = lo; s < hi; s++) {
    const uint8_t *st = chunks + s * n * cs;
    for (int j = 0; j < k; j++) src[j] = st + (int64_t)ids[j] * cs;
    for (int r = 0; r < rows; r++) dst[r] = out + (s * rows + r) * cs;
    orc_simd_encode(level, (size_t)cs, k, rows, matrix, src, dst);
  }
}
