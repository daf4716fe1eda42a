// Probe: pageable -> staging copy rate on the host (glibc memcpy vs SSE2
// non-temporal stores), the agent gather / host-path staging copy pattern:
// 1 MiB pieces from 1 GiB of sources into a 256 MiB buffer.  Usage: host_copy THREADS NT
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
static void nt_copy(void *d, const void *s, size_t n) {
  char *dc = (char *)d; const char *sc = (const char *)s;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    __m128i a = _mm_loadu_si128((const __m128i *)(sc + i)), b = _mm_loadu_si128((const __m128i *)(sc + i + 16));
    __m128i c = _mm_loadu_si128((const __m128i *)(sc + i + 32)), e = _mm_loadu_si128((const __m128i *)(sc + i + 48));
    _mm_stream_si128((__m128i *)(dc + i), a); _mm_stream_si128((__m128i *)(dc + i + 16), b);
    _mm_stream_si128((__m128i *)(dc + i + 32), c); _mm_stream_si128((__m128i *)(dc + i + 48), e);
  }
  _mm_sfence();
  if (i < n) memcpy(dc + i, sc + i, n - i);
}
int main(int argc, char **argv) {
  const size_t cs = 1 << 20, nsrc = 1024, ndst = 256; int T = atoi(argv[1]); int nt = atoi(argv[2]);
  std::vector<char *> src(nsrc);
  for (auto &p : src) { p = (char *)aligned_alloc(64, cs); memset(p, 1, cs); }
  char *dst = (char *)aligned_alloc(64, ndst * cs); memset(dst, 0, ndst * cs);
  for (int rep = 0; rep < 3; rep++) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back([&, t] {
      for (size_t i = t; i < nsrc; i += T) { char *d = dst + (i % ndst) * cs; if (nt) nt_copy(d, src[i], cs); else memcpy(d, src[i], cs); }
    });
    for (auto &x : th) x.join();
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("threads %d %s: %.1f GB/s\n", T, nt ? "stream" : "memcpy", nsrc * cs / s / 1e9);
  }
}
