/* The ISA-L call sequence of rs.cc (constructor :26-27, encode :89, decode
 * :196,229-230) written against nxec_isal_compat.h exactly as the reference
 * writes it against <isa-l/erasure_code.h>: compiles as C, runs on the GPU.
 * Prints the SHA-256 of the parity and of the decoded data for
 * tests/test_cpp_surface.py.  Exit 0 iff decode restored the data. */
#include <openssl/sha.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nxec_isal_compat.h"

static void hex(const unsigned char *p, size_t n) {
  unsigned char d[32];
  SHA256(p, n, d);
  for (int i = 0; i < 32; i++) printf("%02x", d[i]);
}

int main(int argc, char **argv) {
  int n = argc > 1 ? atoi(argv[1]) : 14, k = argc > 2 ? atoi(argv[2]) : 10, cs = argc > 3 ? atoi(argv[3]) : 1000;
  unsigned char enc[128 * 128], gftbl[128 * 128 * 32], dm[128 * 128], inv[128 * 128];
  unsigned char *stripe = malloc((size_t)n * cs), *out = malloc((size_t)k * cs);
  unsigned char *datap[128], *codep[128], *inp[128], *outp[128];
  unsigned long long s = 1000003ull * n + 10007ull * k + cs; /* tests/helpers.py case_seed / fill_bytes */
  for (long i = 0; i < (long)k * cs; i += 8) {
    unsigned long long z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (int b = 0; b < 8 && i + b < (long)k * cs; b++) stripe[i + b] = (unsigned char)(z >> (8 * b));
  }
  gf_gen_rs_matrix(enc, n, k);               /* rs.cc:26 */
  ec_init_tables(k, n - k, &enc[k * k], gftbl); /* rs.cc:27 */
  for (int i = 0; i < k; i++) datap[i] = stripe + (long)i * cs;
  for (int i = k; i < n; i++) codep[i - k] = stripe + (long)i * cs;
  ec_encode_data(cs, k, n - k, gftbl, datap, codep); /* rs.cc:89 */
  printf("PARITY ");
  hex(stripe + (long)k * cs, (size_t)(n - k) * cs);
  printf("\n");
  /* decode from the last k chunks (first n-k erased), rs.cc:141-157,196,229-230 */
  for (int i = 0; i < k; i++) {
    memcpy(dm + i * k, enc + (n - k + i) * k, k);
    inp[i] = stripe + (long)(n - k + i) * cs;
    outp[i] = out + (long)i * cs;
  }
  if (gf_invert_matrix(dm, inv, k) < 0) return 2;
  ec_init_tables(k, k, inv, gftbl);
  ec_encode_data(cs, k, k, gftbl, inp, outp);
  printf("DECODED ");
  hex(out, (size_t)k * cs);
  printf("\n");
  int ok = memcmp(out, stripe, (size_t)k * cs) == 0;
  printf("%s\n", ok ? "OK" : "MISMATCH");
  return ok ? 0 : 1;
}
