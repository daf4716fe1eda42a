/*
 * nxec_oracle.c -- TEST INFRASTRUCTURE ONLY (see nxec_oracle.h).
 *
 * Plain-C restatement of the reference RS coding path.  Each function names
 * the reference lines it follows.  Written from the math, not copied: the
 * GF(2^8) field is built here by repeated multiplication by the generator
 * instead of ISA-L's literal tables (ec_base.h:35,64); products are unique in
 * the field, so results are identical.
 */
#define _GNU_SOURCE
#include "nxec_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint8_t g_exp[512];
static uint8_t g_log[256];
static int g_ready = 0;

static void gf_setup(void) {
  if (g_ready) return;
  unsigned v = 1;
  for (int i = 0; i < 255; i++) {
    g_exp[i] = (uint8_t)v;
    g_log[v] = (uint8_t)i;
    v <<= 1;
    if (v & 0x100) v ^= 0x11d; /* ISA-L ec_base.c:171 reduction by 0x1d */
  }
  for (int i = 255; i < 512; i++) g_exp[i] = g_exp[i - 255];
  g_ready = 1;
}

/* ISA-L ec_base.c:48-60 (log/antilog multiply) */
uint8_t orc_gf_mul(uint8_t a, uint8_t b) {
  gf_setup();
  if (a == 0 || b == 0) return 0;
  return g_exp[g_log[a] + g_log[b]];
}

/* ISA-L ec_base.c:62-72; gf_inv(0) = 0 as in the reference */
uint8_t orc_gf_inv(uint8_t a) {
  gf_setup();
  if (a == 0) return 0;
  return g_exp[255 - g_log[a]];
}

/* ISA-L ec_base.c:74-91: identity on top, parity row i holds gen^j with
 * gen = 2^(i-k) (so the first parity row is all ones). */
void orc_gen_rs_matrix(uint8_t *a, int m, int k) {
  memset(a, 0, (size_t)k * m);
  for (int i = 0; i < k; i++) a[k * i + i] = 1;
  uint8_t gen = 1;
  for (int i = k; i < m; i++) {
    uint8_t p = 1;
    for (int j = 0; j < k; j++) {
      a[k * i + j] = p;
      p = orc_gf_mul(p, gen);
    }
    gen = orc_gf_mul(gen, 2);
  }
}

/* ISA-L ec_base.c:111-164 Gauss-Jordan with the same pivot rule (first
 * non-zero row below on a zero pivot).  Works on a copy of `in`. */
int orc_invert_matrix(const uint8_t *in, uint8_t *out, int n) {
  uint8_t *m = (uint8_t *)malloc((size_t)n * n);
  if (!m) return -1;
  memcpy(m, in, (size_t)n * n);
  memset(out, 0, (size_t)n * n);
  for (int i = 0; i < n; i++) out[i * n + i] = 1;
  for (int i = 0; i < n; i++) {
    if (m[i * n + i] == 0) {
      int j;
      for (j = i + 1; j < n; j++)
        if (m[j * n + i]) break;
      if (j == n) { free(m); return -1; }
      for (int c = 0; c < n; c++) {
        uint8_t t = m[i * n + c]; m[i * n + c] = m[j * n + c]; m[j * n + c] = t;
        t = out[i * n + c]; out[i * n + c] = out[j * n + c]; out[j * n + c] = t;
      }
    }
    uint8_t inv = orc_gf_inv(m[i * n + i]);
    for (int c = 0; c < n; c++) {
      m[i * n + c] = orc_gf_mul(m[i * n + c], inv);
      out[i * n + c] = orc_gf_mul(out[i * n + c], inv);
    }
    for (int r = 0; r < n; r++) {
      if (r == i) continue;
      uint8_t f = m[r * n + i];
      for (int c = 0; c < n; c++) {
        out[r * n + c] ^= orc_gf_mul(f, out[i * n + c]);
        m[r * n + c] ^= orc_gf_mul(f, m[i * n + c]);
      }
    }
  }
  free(m);
  return 0;
}

/* ISA-L ec_base.c:169-274 gf_vect_mul_init: 32-byte table per coefficient,
 * [0..15] = c*x, [16..31] = c*(x<<4); ec_init_tables (ec_base.c:36-46) lays
 * them out row-major rows x k. */
void orc_init_tables(int k, int rows, const uint8_t *a, uint8_t *g) {
  for (int i = 0; i < rows * k; i++) {
    uint8_t c = a[i];
    for (int x = 0; x < 16; x++) {
      g[32 * i + x] = orc_gf_mul(c, (uint8_t)x);
      g[32 * i + 16 + x] = orc_gf_mul(c, (uint8_t)(x << 4));
    }
  }
}

/* ISA-L ec_base.c:302-317: dest[l][i] = XOR_j src[j][i] * v[32*(l*k+j)+1] */
void orc_encode_data(int len, int k, int rows, const uint8_t *v, const uint8_t *const *src, uint8_t *const *dst) {
  uint8_t *a = (uint8_t *)malloc((size_t)rows * k + 1);
  for (int i = 0; i < rows * k; i++) a[i] = v[32 * i + 1];
  orc_matmul(len, k, rows, a, src, dst);
  free(a);
}

/* byte loop of ec_encode_data_base, with a 256-entry product row per
 * coefficient so the oracle finishes MiB-scale cases in seconds */
void orc_matmul(int len, int k, int rows, const uint8_t *a, const uint8_t *const *src, uint8_t *const *dst) {
  uint8_t *mt = (uint8_t *)malloc((size_t)256 * (rows * k > 0 ? rows * k : 1));
  for (int i = 0; i < rows * k; i++)
    for (int x = 0; x < 256; x++) mt[256 * i + x] = orc_gf_mul(a[i], (uint8_t)x);
  for (int l = 0; l < rows; l++) {
    uint8_t *d = dst[l];
    memset(d, 0, (size_t)len);
    for (int j = 0; j < k; j++) {
      const uint8_t *t = mt + 256 * (l * k + j);
      const uint8_t *s = src[j];
      for (int i = 0; i < len; i++) d[i] ^= t[s[i]];
    }
  }
  free(mt);
}

/* rs.cc:57-92: chunk i < k is a copy of data[i*cs..], parity via the
 * (n-k) x k lower block of the encode matrix (rs.cc:26-27,89). */
int orc_rs_encode(int n, int k, const uint8_t *data, int64_t cs, uint8_t *out) {
  if (n <= 0 || k <= 0 || n < k) return 0; /* rs.cc:16-18 */
  uint8_t *m = (uint8_t *)malloc((size_t)n * k);
  orc_gen_rs_matrix(m, n, k);
  const uint8_t **src = (const uint8_t **)malloc(sizeof(void *) * k);
  uint8_t **dst = (uint8_t **)malloc(sizeof(void *) * (n - k + 1));
  for (int i = 0; i < k; i++) {
    memcpy(out + i * cs, data + i * cs, (size_t)cs);
    src[i] = out + i * cs;
  }
  for (int i = k; i < n; i++) dst[i - k] = out + i * cs;
  orc_matmul((int)cs, k, n - k, m + k * k, src, dst);
  free(src); free(dst); free(m);
  return 1;
}

/* Rows of the repair matrix for targets given the first k inputs' inverse:
 * data target -> inverse row (rs.cc:207-211 / 305-310); parity target ->
 * encRow(target) x inverse (rs.cc:212-222 / 312-319). */
static void repair_rows(int k, const uint8_t *enc, const uint8_t *inv, const int32_t *targets, int nt, uint8_t *out) {
  int i = 0;
  for (; i < nt && targets[i] < k; i++) memcpy(out + k * i, inv + k * targets[i], (size_t)k);
  for (; i < nt; i++)
    for (int j = 0; j < k; j++) {
      uint8_t s = 0;
      for (int l = 0; l < k; l++) s ^= orc_gf_mul(inv[l * k + j], enc[targets[i] * k + l]);
      out[i * k + j] = s;
    }
}

/* rs.cc:238-322 */
int orc_rs_pre_decode(int n, int k, const int32_t *failed, int nfailed, int is_repair,
                      int32_t *input_ids, int *ninputs, int *min_inputs, uint8_t *repair_matrix) {
  *ninputs = 0;
  *min_inputs = 0;
  if (nfailed > n - k) return 0; /* rs.cc:244-247 */
  int32_t *erasures = (int32_t *)malloc(sizeof(int32_t) * (n + 1));
  int e = 0, ni = 0;
  for (int i = 0; i < n; i++) { /* rs.cc:255-265 */
    if (e < nfailed && failed[e] == i) { erasures[e++] = i; continue; }
    input_ids[ni++] = i;
  }
  *ninputs = ni;
  *min_inputs = k; /* rs.cc:269 */
  if (ni < k) { *ninputs = 0; *min_inputs = 0; free(erasures); return 0; }
  if (!is_repair) { free(erasures); return 1; }
  uint8_t *enc = (uint8_t *)malloc((size_t)n * k);
  uint8_t *dm = (uint8_t *)malloc((size_t)k * k);
  uint8_t *inv = (uint8_t *)malloc((size_t)k * k);
  orc_gen_rs_matrix(enc, n, k);
  for (int i = 0; i < k; i++) memcpy(dm + i * k, enc + input_ids[i] * k, (size_t)k); /* rs.cc:285-287, first k rows inverted */
  int ok = orc_invert_matrix(dm, inv, k) == 0;
  if (ok) repair_rows(k, enc, inv, erasures, e, repair_matrix);
  else { *ninputs = 0; *min_inputs = 0; }
  free(enc); free(dm); free(inv); free(erasures);
  return ok;
}

/* rs.cc:111-236 */
int orc_rs_decode(int n, int k, const int32_t *input_ids, int ninputs, const uint8_t *const *inputs,
                  int64_t cs, int is_repair, const int32_t *targets, int ntargets, int use_car,
                  uint8_t *out, int *ntargets_out) {
  if (ninputs < k && (!is_repair || !use_car)) return 0; /* rs.cc:134-137 */
  int32_t *tg = (int32_t *)malloc(sizeof(int32_t) * (n + 1));
  int nt = 0;
  int32_t *match_row = (int32_t *)malloc(sizeof(int32_t) * (n + 1));
  int matched = 0;
  /* rs.cc:142-158: inputs matched positionally against ascending ids */
  for (int i = 0, idx = 0; i < n; i++) {
    if (idx < ninputs && input_ids[idx] == i) { match_row[matched++] = i; idx++; }
    else if (is_repair && ntargets == 0) tg[nt++] = i;
  }
  if (is_repair && ntargets > 0) { memcpy(tg, targets, sizeof(int32_t) * ntargets); nt = ntargets; }
  int ndec = is_repair ? nt : k;
  if (ntargets_out) *ntargets_out = ndec;
  uint8_t **dst = (uint8_t **)malloc(sizeof(void *) * (ndec + 1));
  for (int i = 0; i < ndec; i++) dst[i] = out + i * cs;
  int ok = 1;
  if (is_repair && ndec == 1 && use_car) { /* rs.cc:184-192 -> carRepairFinalize rs.cc:94-109 */
    if (ninputs == 1) memcpy(dst[0], inputs[0], (size_t)cs);
    else {
      uint8_t *ones = (uint8_t *)malloc((size_t)ninputs);
      memset(ones, 1, (size_t)ninputs);
      orc_matmul((int)cs, ninputs, 1, ones, inputs, dst);
      free(ones);
    }
  } else {
    uint8_t *enc = (uint8_t *)malloc((size_t)n * k);
    uint8_t *dm = (uint8_t *)malloc((size_t)k * k);
    uint8_t *inv = (uint8_t *)malloc((size_t)k * k);
    orc_gen_rs_matrix(enc, n, k);
    /* rows of the first k matched inputs (rs.cc:150, inversion uses k x k) */
    for (int i = 0; i < k; i++) memcpy(dm + i * k, enc + match_row[i] * k, (size_t)k);
    if (matched < k || orc_invert_matrix(dm, inv, k) != 0) ok = 0; /* rs.cc:196-201 */
    if (ok) {
      uint8_t *fm = (uint8_t *)malloc((size_t)ndec * k + 1);
      if (is_repair) repair_rows(k, enc, inv, tg, nt, fm);
      else memcpy(fm, inv, (size_t)k * k);
      orc_matmul((int)cs, k, ndec, fm, inputs, dst); /* rs.cc:228-230 */
      free(fm);
    }
    free(enc); free(dm); free(inv);
  }
  free(dst); free(tg); free(match_row);
  return ok;
}

/* coding_util.hh:12-23 */
void orc_coding_utils_encode(const uint8_t *data, int ndata, uint8_t *code, int ncode, int cs, const uint8_t *matrix) {
  const uint8_t **src = (const uint8_t **)malloc(sizeof(void *) * (ndata + 1));
  uint8_t **dst = (uint8_t **)malloc(sizeof(void *) * (ncode + 1));
  for (int i = 0; i < ndata; i++) src[i] = data + (int64_t)i * cs;
  for (int i = 0; i < ncode; i++) dst[i] = code + (int64_t)i * cs;
  orc_matmul(cs, ndata, ncode, matrix, src, dst);
  free(src); free(dst);
}

void orc_fill_bytes(uint8_t *p, int64_t nbytes, uint64_t seed) {
  uint64_t s = seed;
  for (int64_t i = 0; i < nbytes; i += 8) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (int b = 0; b < 8 && i + b < nbytes; b++) p[i + b] = (uint8_t)(z >> (8 * b));
  }
}

/* bytes [word_off*8, word_off*8 + nbytes) of the same stream (the device
 * fill of a larger buffer, read back piecewise) */
void orc_fill_bytes_at(uint8_t *p, int64_t nbytes, uint64_t seed, int64_t word_off) {
  orc_fill_bytes(p, nbytes, seed + (uint64_t)word_off * 0x9E3779B97F4A7C15ull);
}

struct enc_job {
  int k, rows;
  const uint8_t *a, *src;
  uint8_t *dst;
  int64_t cs, s0, s1;
};

static void *enc_worker(void *arg) {
  struct enc_job *j = (struct enc_job *)arg;
  const uint8_t **src = (const uint8_t **)malloc(sizeof(void *) * j->k);
  uint8_t **dst = (uint8_t **)malloc(sizeof(void *) * j->rows);
  for (int64_t s = j->s0; s < j->s1; s++) {
    for (int i = 0; i < j->k; i++) src[i] = j->src + (s * j->k + i) * j->cs;
    for (int i = 0; i < j->rows; i++) dst[i] = j->dst + (s * j->rows + i) * j->cs;
    orc_matmul((int)j->cs, j->k, j->rows, j->a, src, dst);
  }
  free(src); free(dst);
  return NULL;
}

double orc_time_encode(int k, int rows, const uint8_t *a, const uint8_t *src, uint8_t *dst,
                       int64_t cs, int64_t nstripes, int threads) {
  if (threads < 1) threads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  struct enc_job *jobs = (struct enc_job *)malloc(sizeof(struct enc_job) * threads);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; t++) {
    jobs[t] = (struct enc_job){k, rows, a, src, dst, cs, nstripes * t / threads, nstripes * (t + 1) / threads};
    pthread_create(&th[t], NULL, enc_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th); free(jobs);
  return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
