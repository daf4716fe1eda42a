/*
 * gen_golden.c -- TEST INFRASTRUCTURE ONLY.  Runs in the build container,
 * never on the GPU box.
 *
 * Produces tests/golden/golden.json: known-answer vectors for the RS coding
 * path computed by the REFERENCE arithmetic (ISA-L 2.22 ec_base.c, built by
 * build_ref.sh into _ref/libisal_base.so).  The reference's own tests carry no
 * golden vectors, so these outputs of the reference itself are
 * what pins both the CPU oracle and the HIP path.
 *
 * The RSCode glue (which matrix rows, which inputs, output order) is restated
 * from src/common/coding/rs.cc with line citations; every arithmetic step is
 * an ISA-L call.  The cases follow src/tests/common/coding_test.cc:
 * encode (:192), decode with the first n-k chunks erased (:211-265), every
 * single-node repair (:269-427) incl. CAR partial encode per rack (:312-355),
 * every double failure (:432-533); plus the agent_test.cc:219-261 known answer.
 *
 * Usage: gen_golden > tests/golden/golden.json
 */
#include <openssl/sha.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ISA-L public API (include/erasure_code.h:74,98,870,905,931) */
void ec_init_tables(int k, int rows, unsigned char *a, unsigned char *gftbls);
void ec_encode_data(int len, int k, int rows, unsigned char *gftbls, unsigned char **data, unsigned char **coding);
void gf_gen_rs_matrix(unsigned char *a, int m, int k);
int gf_invert_matrix(unsigned char *in, unsigned char *out, const int n);
unsigned char gf_mul(unsigned char a, unsigned char b);
unsigned char gf_inv(unsigned char a);

static void fill_bytes(uint8_t *p, int64_t nbytes, uint64_t seed) { /* splitmix64, LE */
  uint64_t s = seed;
  for (int64_t i = 0; i < nbytes; i += 8) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (int b = 0; b < 8 && i + b < nbytes; b++) p[i + b] = (uint8_t)(z >> (8 * b));
  }
}

static uint64_t case_seed(int n, int k, int64_t cs) { return 1000003ull * n + 10007ull * k + (uint64_t)cs; }

static void hexs(const uint8_t *p, int64_t n) {
  putchar('"');
  for (int64_t i = 0; i < n; i++) printf("%02x", p[i]);
  putchar('"');
}
static void sha(const uint8_t *p, int64_t n) {
  uint8_t d[32];
  SHA256(p, (size_t)n, d);
  hexs(d, 32);
}
static void ids(const int *v, int n) {
  putchar('[');
  for (int i = 0; i < n; i++) printf("%s%d", i ? "," : "", v[i]);
  putchar(']');
}

/* ---- RSCode restated over ISA-L ---- */

/* rs.cc:57-92 */
static void ref_encode(int n, int k, const uint8_t *data, int64_t cs, uint8_t *stripe) {
  uint8_t enc[128 * 128], tbl[128 * 128 * 32];
  unsigned char *dp[128], *cp[128];
  gf_gen_rs_matrix(enc, n, k);                 /* rs.cc:26 */
  ec_init_tables(k, n - k, &enc[k * k], tbl);  /* rs.cc:27 */
  for (int i = 0; i < n; i++) {
    if (i < k) { memcpy(stripe + i * cs, data + i * cs, cs); dp[i] = stripe + i * cs; }  /* rs.cc:78-82 */
    else cp[i - k] = stripe + i * cs;
  }
  ec_encode_data((int)cs, k, n - k, tbl, dp, cp); /* rs.cc:89 */
}

/* rs.cc:238-322: returns ninputs (all alive ids) or -1, repair matrix when is_repair */
static int ref_pre_decode(int n, int k, const int *failed, int nf, int is_repair, int *inputs, uint8_t *rm) {
  if (nf > n - k) return -1;
  int er[128], e = 0, ni = 0;
  for (int i = 0; i < n; i++) {
    if (e < nf && failed[e] == i) { er[e++] = i; continue; }
    inputs[ni++] = i;
  }
  if (ni < k) return -1;
  if (!is_repair) return ni;
  uint8_t enc[128 * 128], dm[128 * 128], inv[128 * 128];
  gf_gen_rs_matrix(enc, n, k);
  for (int i = 0; i < ni; i++) memcpy(dm + i * k, enc + inputs[i] * k, k);  /* rs.cc:285-287 */
  if (gf_invert_matrix(dm, inv, k) < 0) return -1;                          /* rs.cc:290 */
  int i = 0;
  for (; i < e && er[i] < k; i++) memcpy(rm + k * i, inv + k * er[i], k);    /* rs.cc:308-310 */
  for (; i < e; i++)                                                         /* rs.cc:312-319 */
    for (int j = 0; j < k; j++) {
      uint8_t s = 0;
      for (int l = 0; l < k; l++) s ^= gf_mul(inv[l * k + j], enc[er[i] * k + l]);
      rm[i * k + j] = s;
    }
  return ni;
}

/* rs.cc:111-236 (non-CAR); inputs sorted ascending by id; returns #rows or -1 */
static int ref_decode(int n, int k, const int *in_ids, int nin, uint8_t **inp, int64_t cs, int is_repair,
                      const int *targets, int nt_in, int use_car, uint8_t *out) {
  if (nin < k && (!is_repair || !use_car)) return -1;
  uint8_t enc[128 * 128], dm[128 * 128], inv[128 * 128];
  int tg[128], nt = 0;
  gf_gen_rs_matrix(enc, n, k);
  for (int i = 0, idx = 0; i < n; i++) {                                     /* rs.cc:142-158 */
    if (idx < nin && in_ids[idx] == i) { memcpy(dm + idx * k, enc + i * k, k); idx++; }
    else if (is_repair && nt_in == 0) tg[nt++] = i;
  }
  if (is_repair && nt_in > 0) { memcpy(tg, targets, sizeof(int) * nt_in); nt = nt_in; }
  int nd = is_repair ? nt : k;
  unsigned char *dp[128];
  for (int i = 0; i < nd; i++) dp[i] = out + i * cs;
  if (is_repair && nd == 1 && use_car) {                                     /* rs.cc:184-192, 94-109 */
    if (nin == 1) { memcpy(dp[0], inp[0], cs); return 1; }
    uint8_t ones[128], g[128 * 32];
    memset(ones, 1, nin);
    ec_init_tables(nin, 1, ones, g);
    ec_encode_data((int)cs, nin, 1, g, inp, dp);
    return 1;
  }
  if (gf_invert_matrix(dm, inv, k) < 0) return -1;                           /* rs.cc:196 */
  uint8_t *fm = inv;
  if (is_repair) {                                                           /* rs.cc:207-225 */
    int i = 0;
    for (; i < nd && tg[i] < k; i++) memcpy(dm + k * i, inv + k * tg[i], k);
    for (; i < nd; i++)
      for (int j = 0; j < k; j++) {
        uint8_t s = 0;
        for (int l = 0; l < k; l++) s ^= gf_mul(inv[l * k + j], enc[tg[i] * k + l]);
        dm[i * k + j] = s;
      }
    fm = dm;
  }
  static uint8_t g[128 * 128 * 32];
  ec_init_tables(k, nd, fm, g);                                              /* rs.cc:229-230 */
  ec_encode_data((int)cs, k, nd, g, inp, dp);
  return nd;
}

static int first_case = 1;
static void sep(void) { if (!first_case) printf(",\n"); first_case = 0; }

static void case_encode(int n, int k, int64_t cs, int hex_limit) {
  uint64_t seed = case_seed(n, k, cs);
  uint8_t *data = malloc(k * cs), *st = malloc(n * cs);
  fill_bytes(data, k * cs, seed);
  ref_encode(n, k, data, cs, st);
  sep();
  printf("{\"n\":%d,\"k\":%d,\"cs\":%ld,\"seed\":%lu,\"parity_sha256\":", n, k, (long)cs, (unsigned long)seed);
  sha(st + k * cs, (n - k) * cs);
  if ((n - k) * cs <= hex_limit) { printf(",\"parity_hex\":"); hexs(st + k * cs, (n - k) * cs); }
  printf("}");
  free(data); free(st);
}

/* decode with erasures `failed` using the first k alive chunks (coding_test.cc:221-240) */
static void case_decode(int n, int k, int64_t cs, const int *failed, int nf, const char *tag) {
  uint64_t seed = case_seed(n, k, cs);
  uint8_t *data = malloc(k * cs), *st = malloc(n * cs), *out = malloc(k * cs);
  fill_bytes(data, k * cs, seed);
  ref_encode(n, k, data, cs, st);
  int in[128];
  int ni = ref_pre_decode(n, k, failed, nf, 0, in, NULL);
  uint8_t *inp[128];
  for (int i = 0; i < k; i++) inp[i] = st + in[i] * cs;
  int nd = ref_decode(n, k, in, k, inp, cs, 0, NULL, 0, 0, out);
  sep();
  printf("{\"n\":%d,\"k\":%d,\"cs\":%ld,\"seed\":%lu,\"pattern\":\"%s\",\"failed\":", n, k, (long)cs, (unsigned long)seed, tag);
  ids(failed, nf);
  printf(",\"ninputs\":%d,\"ok\":%d,\"data_sha256\":", ni, nd == k);
  sha(out, k * cs);
  printf(",\"matches_original\":%d}", memcmp(out, data, k * cs) == 0);
  free(data); free(st); free(out);
}

/* repair of `failed` (preDecode isRepair + decode isRepair with targets) -- coding_test.cc:269-533 */
static void case_repair(int n, int k, int64_t cs, const int *failed, int nf) {
  uint64_t seed = case_seed(n, k, cs);
  uint8_t *data = malloc(k * cs), *st = malloc(n * cs), *out = malloc(nf * cs);
  fill_bytes(data, k * cs, seed);
  ref_encode(n, k, data, cs, st);
  int in[128];
  uint8_t rm[128 * 128];
  int ni = ref_pre_decode(n, k, failed, nf, 1, in, rm);
  uint8_t *inp[128];
  for (int i = 0; i < k; i++) inp[i] = st + in[i] * cs;
  int nd = ref_decode(n, k, in, k, inp, cs, 1, failed, nf, 0, out);
  int good = 1;
  for (int i = 0; i < nf; i++) good &= memcmp(out + i * cs, st + failed[i] * cs, cs) == 0;
  sep();
  printf("{\"n\":%d,\"k\":%d,\"cs\":%ld,\"seed\":%lu,\"failed\":", n, k, (long)cs, (unsigned long)seed);
  ids(failed, nf);
  printf(",\"ninputs\":%d,\"repair_matrix_hex\":", ni);
  hexs(rm, nf * k);
  printf(",\"ok\":%d,\"repaired_sha256\":", nd == nf);
  sha(out, nf * cs);
  printf(",\"matches_original\":%d}", good);
  free(data); free(st); free(out);
}

/* CAR single-failure repair with racks of `g` chunks (chunk i on rack i/g),
 * partial encode per rack with the plan's repair row (coding_test.cc:312-355,
 * chunk_manager.cc:929-986, container_manager.cc:251), XOR finalize (rs.cc:94-109) */
static void case_car(int n, int k, int64_t cs, int failed, int g) {
  uint64_t seed = case_seed(n, k, cs);
  uint8_t *data = malloc(k * cs), *st = malloc(n * cs), *part = malloc(n * cs), *out = malloc(cs);
  fill_bytes(data, k * cs, seed);
  ref_encode(n, k, data, cs, st);
  int in[128];
  uint8_t rm[128 * 128];
  ref_pre_decode(n, k, &failed, 1, 1, in, rm);
  int np = 0, cidx = 0, gstart[128], gsize[128];
  while (cidx < k) {
    int rack = in[cidx] / g, start = cidx;
    unsigned char *pin[128], *pout[1];
    while (cidx < k && in[cidx] / g == rack) { pin[cidx - start] = st + in[cidx] * cs; cidx++; }
    pout[0] = part + np * cs;
    uint8_t tb[128 * 32];
    ec_init_tables(cidx - start, 1, rm + start, tb);                    /* CodingUtils::encode, coding_util.hh:25-31 */
    ec_encode_data((int)cs, cidx - start, 1, tb, pin, pout);
    gstart[np] = start; gsize[np] = cidx - start; np++;
  }
  uint8_t *pp[128];
  for (int i = 0; i < np; i++) pp[i] = part + i * cs;
  int dummy[128];
  for (int i = 0; i < np; i++) dummy[i] = i;
  ref_decode(n, k, dummy, np, pp, cs, 1, &failed, 1, 1, out);
  sep();
  printf("{\"n\":%d,\"k\":%d,\"cs\":%ld,\"seed\":%lu,\"failed\":%d,\"rack_size\":%d,\"repair_row_hex\":", n, k, (long)cs,
         (unsigned long)seed, failed, g);
  hexs(rm, k);
  printf(",\"groups\":[");
  for (int i = 0; i < np; i++) printf("%s[%d,%d]", i ? "," : "", gstart[i], gsize[i]);
  printf("],\"partials_sha256\":[");
  for (int i = 0; i < np; i++) { if (i) putchar(','); sha(part + i * cs, cs); }
  printf("],\"final_sha256\":");
  sha(out, cs);
  printf(",\"matches_original\":%d}", memcmp(out, st + failed * cs, cs) == 0);
  free(data); free(st); free(part); free(out);
}

static void mixed_pattern(int n, int k, int e, int *f) {
  int nd = e / 2, np = e - nd, c = 0;
  static const int dsel[] = {1, 4, 7, 10, 13};
  for (int i = 0; i < nd; i++) f[c++] = dsel[i] % k;
  int pids[2] = {n - 3, n - 1};
  for (int i = 2 - np; i < 2; i++) f[c++] = pids[i];
  (void)n;
}

int main(void) {
  int main_geo[][2] = {{4, 2}, {6, 4}, {14, 10}, {16, 12}, {20, 16}};
  int64_t main_cs[] = {1, 31, 64, 1000, 4096, 65537, 1 << 20};
  printf("{\n\"generator\":\"oracle/gen_golden.c over ISA-L 2.22.0 ec_base.c (reference, oracle/build_ref.sh)\",\n");
  printf("\"prng\":\"splitmix64 LE bytes, seed = 1000003*n + 10007*k + cs\",\n");

  /* field */
  static uint8_t mt[65536];
  for (int a = 0; a < 256; a++) for (int b = 0; b < 256; b++) mt[a * 256 + b] = gf_mul(a, b);
  uint8_t it[256];
  for (int a = 0; a < 256; a++) it[a] = gf_inv(a);
  printf("\"gf_mul_table_sha256\":"); sha(mt, 65536);
  printf(",\n\"gf_mul_row_3_hex\":"); hexs(mt + 3 * 256, 256);
  printf(",\n\"gf_inv_hex\":"); hexs(it, 256);

  /* encode matrices for every coding_test pair (coding_test.cc:597-615) + config geometries */
  printf(",\n\"matrices\":[\n");
  first_case = 1;
  for (int n = 4; n <= 12; n++)
    for (int m = 1; m <= n - 2; m++) {
      int k = n - m;
      uint8_t a[128 * 128];
      gf_gen_rs_matrix(a, n, k);
      sep(); printf("{\"n\":%d,\"k\":%d,\"hex\":", n, k); hexs(a, n * k); printf("}");
    }
  for (int gi = 2; gi < 5; gi++) {
    int n = main_geo[gi][0], k = main_geo[gi][1];
    uint8_t a[128 * 128];
    gf_gen_rs_matrix(a, n, k);
    sep(); printf("{\"n\":%d,\"k\":%d,\"hex\":", n, k); hexs(a, n * k); printf("}");
  }
  printf("\n]");

  /* ec_init_tables of the parity block */
  printf(",\n\"init_tables\":[\n");
  first_case = 1;
  for (int gi = 0; gi < 5; gi++) {
    int n = main_geo[gi][0], k = main_geo[gi][1];
    uint8_t a[128 * 128], t[128 * 128 * 32];
    gf_gen_rs_matrix(a, n, k);
    ec_init_tables(k, n - k, a + k * k, t);
    sep(); printf("{\"n\":%d,\"k\":%d,\"hex\":", n, k); hexs(t, (n - k) * k * 32); printf("}");
  }
  printf("\n]");

  /* matrix inverses of random-looking survivor sets */
  printf(",\n\"inverses\":[\n");
  first_case = 1;
  for (int gi = 0; gi < 5; gi++) {
    int n = main_geo[gi][0], k = main_geo[gi][1];
    uint8_t a[128 * 128], dm[128 * 128], inv[128 * 128];
    gf_gen_rs_matrix(a, n, k);
    int rows[128];
    for (int i = 0; i < k; i++) rows[i] = n - k + i; /* the last k chunks */
    for (int i = 0; i < k; i++) memcpy(dm + i * k, a + rows[i] * k, k);
    int r = gf_invert_matrix(dm, inv, k);
    sep(); printf("{\"n\":%d,\"k\":%d,\"rows\":", n, k); ids(rows, k);
    printf(",\"ret\":%d,\"inv_hex\":", r); hexs(inv, k * k); printf("}");
  }
  printf("\n]");

  /* encode */
  printf(",\n\"encode\":[\n");
  first_case = 1;
  for (int gi = 0; gi < 5; gi++)
    for (int ci = 0; ci < 7; ci++) case_encode(main_geo[gi][0], main_geo[gi][1], main_cs[ci], 4096);
  for (int n = 4; n <= 12; n++)
    for (int m = 1; m <= n - 2; m++) { case_encode(n, n - m, 1, 64); case_encode(n, n - m, 31, 4096); case_encode(n, n - m, 1000, 0); }
  /* config 1, literal sample reading (sample/storage_class.ini:6-9): (n,k)=(4,2), 4 MiB file -> 2 MiB chunks */
  case_encode(4, 2, 2 << 20, 4096);
  printf("\n]");

  /* decode */
  printf(",\n\"decode\":[\n");
  first_case = 1;
  int64_t dcs[] = {1, 1000, 65537, 1 << 20};
  for (int gi = 0; gi < 5; gi++) {
    int n = main_geo[gi][0], k = main_geo[gi][1], e = n - k, f[128];
    for (int ci = 0; ci < 4; ci++) {
      for (int i = 0; i < e; i++) f[i] = i;
      case_decode(n, k, dcs[ci], f, e, "first");
      for (int i = 0; i < e; i++) f[i] = n - e + i;
      case_decode(n, k, dcs[ci], f, e, "parity");
      mixed_pattern(n, k, e, f);
      case_decode(n, k, dcs[ci], f, e, "mixed");
      f[0] = 0;
      case_decode(n, k, dcs[ci], f, 1, "single0");
    }
  }
  for (int n = 4; n <= 12; n++)
    for (int m = 1; m <= n - 2; m++) {
      int f[128];
      for (int i = 0; i < m; i++) f[i] = i;
      case_decode(n, n - m, 1000, f, m, "first");
    }
  {
    int f[2] = {0, 1};
    case_decode(4, 2, 2 << 20, f, 2, "first");
    int g[2] = {2, 3};
    case_decode(4, 2, 2 << 20, g, 2, "parity");
    int h[2] = {1, 3};
    case_decode(4, 2, 2 << 20, h, 2, "mixed");
  }
  printf("\n]");

  /* repair: every single and double failure for the coding_test pairs; singles for the configs */
  printf(",\n\"repair\":[\n");
  first_case = 1;
  for (int n = 4; n <= 12; n++)
    for (int m = 1; m <= n - 2; m++) {
      int k = n - m;
      for (int a = 0; a < n; a++) {
        case_repair(n, k, 1000, &a, 1);
        if (m >= 2)
          for (int b = a + 1; b < n; b++) { int f[2] = {a, b}; case_repair(n, k, 1000, f, 2); }
      }
    }
  for (int gi = 2; gi < 5; gi++) {
    int n = main_geo[gi][0], k = main_geo[gi][1];
    for (int a = 0; a < n; a++) case_repair(n, k, 4096, &a, 1);
    int f4[4] = {1, 4, n - 3, n - 1};
    case_repair(n, k, 65537, f4, 4);
    int f0[1] = {0}, fl[1] = {n - 1};
    case_repair(n, k, 1 << 20, f0, 1);
    case_repair(n, k, 1 << 20, fl, 1);
  }
  for (int a = 0; a < 4; a++) case_repair(4, 2, 2 << 20, &a, 1); /* config 1, literal (4,2) 2 MiB */
  printf("\n]");

  /* CAR repair */
  printf(",\n\"car\":[\n");
  first_case = 1;
  int carf[] = {0, 5, 11, 12, 15};
  for (int i = 0; i < 5; i++) { case_car(16, 12, 1000, carf[i], 4); case_car(16, 12, 1 << 20, carf[i], 4); }
  for (int a = 0; a < 9; a++) case_car(9, 6, 1000, a, 3); /* docker/system_tests/repair_using_car.sh:7-16 */
  for (int a = 0; a < 14; a++) case_car(14, 10, 4096, a, 4);
  printf("\n]");

  /* agent_test.cc:219-261 known answer: ENC_CHUNK_REQ coefficients [1,1] over two 1024-B 'a' chunks -> zeros */
  {
    uint8_t c0[1024], c1[1024], o[1024], coef[2] = {1, 1}, tb[64];
    memset(c0, 'a', 1024); memset(c1, 'a', 1024);
    unsigned char *in[2] = {c0, c1}, *out[1] = {o};
    ec_init_tables(2, 1, coef, tb);
    ec_encode_data(1024, 2, 1, tb, in, out);
    int z = 0;
    for (int i = 0; i < 1024; i++) z += o[i] == 0;
    printf(",\n\"known_answer_agent_enc\":{\"coeffs\":[1,1],\"fill\":97,\"cs\":1024,\"zeros\":%d}", z);
  }
  printf("\n}\n");
  return 0;
}
