// Host-side GF(2^8) arithmetic and RS planning for libnxec.
//
// Replaces the ISA-L calls of the reference coding layer (rs.cc, coding_util.hh)
// with the same semantics; the heavy byte work never runs here -- it is the
// HIP kernels' job (nxec_kernels.hip).  These are O(k^3) matrix routines on
// <= 128 x 128 matrices, microseconds per call.
#include <cstring>
#include <mutex>
#include <vector>

#include "nxec.h"
#include "nxec_internal.h"

namespace {

struct Field {
  uint8_t exp[512];
  uint8_t log[256];
  Field() {
    unsigned v = 1;
    for (int i = 0; i < 255; i++) {
      exp[i] = static_cast<uint8_t>(v);
      log[v] = static_cast<uint8_t>(i);
      v <<= 1;
      if (v & 0x100) v ^= 0x11d;  // x^8 = x^4 + x^3 + x^2 + 1
    }
    for (int i = 255; i < 512; i++) exp[i] = exp[i - 255];
    log[0] = 0;
  }
};

const Field &field() {
  static const Field f;
  return f;
}

}  // namespace

extern "C" unsigned char nxec_gf_mul(unsigned char a, unsigned char b) {
  if (a == 0 || b == 0) return 0;
  const Field &f = field();
  return f.exp[f.log[a] + f.log[b]];
}

extern "C" unsigned char nxec_gf_inv(unsigned char a) {
  if (a == 0) return 0;
  const Field &f = field();
  return f.exp[255 - f.log[a]];
}

// Vandermonde-style RS generator of ISA-L (ec_base.c:74-91): identity block,
// then row i >= k is (g^0, g^1, ..., g^(k-1)) with g = 2^(i-k).
extern "C" void nxec_gf_gen_rs_matrix(unsigned char *a, int m, int k) {
  if (!a || m <= 0 || k <= 0) return;
  std::memset(a, 0, static_cast<size_t>(m) * k);
  for (int i = 0; i < k && i < m; i++) a[k * i + i] = 1;
  unsigned char g = 1;
  for (int i = k; i < m; i++) {
    unsigned char p = 1;
    for (int j = 0; j < k; j++) {
      a[k * i + j] = p;
      p = nxec_gf_mul(p, g);
    }
    g = nxec_gf_mul(g, 2);
  }
}

// Gauss-Jordan elimination; pivot rule identical to ISA-L (ec_base.c:111-164):
// on a zero pivot swap in the first lower row with a non-zero entry.
extern "C" int nxec_gf_invert_matrix(unsigned char *in, unsigned char *out, const int n) {
  if (!in || !out || n <= 0) return -1;
  std::memset(out, 0, static_cast<size_t>(n) * n);
  for (int i = 0; i < n; i++) out[i * n + i] = 1;
  for (int c = 0; c < n; c++) {
    if (in[c * n + c] == 0) {
      int r = c + 1;
      while (r < n && in[r * n + c] == 0) r++;
      if (r == n) return -1;
      for (int x = 0; x < n; x++) {
        std::swap(in[c * n + x], in[r * n + x]);
        std::swap(out[c * n + x], out[r * n + x]);
      }
    }
    const unsigned char piv = nxec_gf_inv(in[c * n + c]);
    for (int x = 0; x < n; x++) {
      in[c * n + x] = nxec_gf_mul(in[c * n + x], piv);
      out[c * n + x] = nxec_gf_mul(out[c * n + x], piv);
    }
    for (int r = 0; r < n; r++) {
      if (r == c) continue;
      const unsigned char f = in[r * n + c];
      if (!f) continue;  // xor with 0*row is a no-op
      for (int x = 0; x < n; x++) {
        out[r * n + x] ^= nxec_gf_mul(f, out[c * n + x]);
        in[r * n + x] ^= nxec_gf_mul(f, in[c * n + x]);
      }
    }
  }
  return 0;
}

// 32-byte split-nibble tables of ISA-L (gf_vect_mul_init, ec_base.c:169-274),
// kept so callers holding ISA-L-layout tables can hand them to
// nxec_ec_encode_data unchanged.  The GPU kernels only read byte [1] (= c).
extern "C" void nxec_ec_init_tables(int k, int rows, unsigned char *a, unsigned char *g) {
  if (!a || !g) return;
  for (int i = 0; i < rows * k; i++) {
    const unsigned char c = a[i];
    for (int x = 0; x < 16; x++) {
      g[32 * i + x] = nxec_gf_mul(c, static_cast<unsigned char>(x));
      g[32 * i + 16 + x] = nxec_gf_mul(c, static_cast<unsigned char>(x << 4));
    }
  }
}

extern "C" void nxec_gen_rs_matrix(unsigned char *a, int n, int k) { nxec_gf_gen_rs_matrix(a, n, k); }

extern "C" int nxec_invert_matrix(const unsigned char *in, unsigned char *out, int k) {
  if (!in || !out || k <= 0) return -1;
  std::vector<unsigned char> tmp(in, in + static_cast<size_t>(k) * k);
  return nxec_gf_invert_matrix(tmp.data(), out, k);
}

extern "C" void nxec_init_tables(int k, int rows, const unsigned char *coeffs, unsigned char *tbls) {
  nxec_ec_init_tables(k, rows, const_cast<unsigned char *>(coeffs), tbls);  // reads coeffs only
}

namespace nxec {

// Rows that rebuild `targets` from the k inputs whose encode rows are `dm`
// (k x k, inverted here).  Data target t -> row t of the inverse; parity
// target t -> enc_row(t) x inverse.  rs.cc:196-225 and rs.cc:285-319.
int repair_rows(int n, int k, const std::vector<uint8_t> &enc, const int32_t *input_ids, const int32_t *targets,
                int ntargets, uint8_t *out) {
  std::vector<uint8_t> dm(static_cast<size_t>(k) * k), inv(static_cast<size_t>(k) * k);
  for (int i = 0; i < k; i++) {
    if (input_ids[i] < 0 || input_ids[i] >= n) return NXEC_ERR_INVALID;
    std::memcpy(&dm[static_cast<size_t>(i) * k], &enc[static_cast<size_t>(input_ids[i]) * k], k);
  }
  if (nxec_gf_invert_matrix(dm.data(), inv.data(), k) < 0) return NXEC_ERR_SINGULAR;
  for (int t = 0; t < ntargets; t++) {
    const int id = targets[t];
    if (id < 0 || id >= n) return NXEC_ERR_INVALID;
    uint8_t *row = out + static_cast<size_t>(t) * k;
    if (id < k) {
      std::memcpy(row, &inv[static_cast<size_t>(id) * k], k);
    } else {
      for (int j = 0; j < k; j++) {
        uint8_t s = 0;
        for (int l = 0; l < k; l++) s ^= nxec_gf_mul(inv[static_cast<size_t>(l) * k + j], enc[static_cast<size_t>(id) * k + l]);
        row[j] = s;
      }
    }
  }
  return NXEC_OK;
}

bool valid_nk(int n, int k) { return k > 0 && n >= k && n <= NXEC_MAX_N && k <= NXEC_MAX_K; }

}  // namespace nxec

extern "C" int nxec_rs_plan(int n, int k, const int32_t *failed, int nfailed, int is_repair, int32_t *input_ids,
                            int *ninputs, int *min_inputs, unsigned char *repair_matrix) {
  using namespace nxec;
  if (ninputs) *ninputs = 0;
  if (min_inputs) *min_inputs = 0;
  if (!valid_nk(n, k) || nfailed < 0 || (nfailed > 0 && !failed) || !input_ids)
    return set_error(NXEC_ERR_INVALID, "nxec_rs_plan: invalid arguments");
  if (nfailed > n - k) return set_error(NXEC_ERR_INVALID, "nxec_rs_plan: more failures than n-k");  // rs.cc:244
  std::vector<int32_t> erasures;
  int ni = 0, e = 0;
  for (int i = 0; i < n; i++) {  // rs.cc:255-265: failed list is ascending
    if (e < nfailed && failed[e] == i) {
      erasures.push_back(i);
      e++;
      continue;
    }
    input_ids[ni++] = i;
  }
  if (e != nfailed) return set_error(NXEC_ERR_INVALID, "nxec_rs_plan: failed ids must be ascending and < n");
  if (ninputs) *ninputs = ni;
  if (min_inputs) *min_inputs = k;
  if (!is_repair) return NXEC_OK;
  if (!repair_matrix && nfailed > 0) return set_error(NXEC_ERR_INVALID, "nxec_rs_plan: repair_matrix is NULL");
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
  nxec_gf_gen_rs_matrix(enc.data(), n, k);
  int rc = repair_rows(n, k, enc, input_ids, erasures.data(), nfailed, repair_matrix);
  if (rc != NXEC_OK) {
    if (ninputs) *ninputs = 0;
    if (min_inputs) *min_inputs = 0;
    return set_error(rc, "nxec_rs_plan: repair matrix not invertible");
  }
  return NXEC_OK;
}

extern "C" int nxec_rs_decode_matrix(int n, int k, const int32_t *input_ids, const int32_t *targets, int ntargets,
                                     unsigned char *out) {
  using namespace nxec;
  if (!valid_nk(n, k) || !input_ids || ntargets < 0 || (ntargets > 0 && (!targets || !out)))
    return set_error(NXEC_ERR_INVALID, "nxec_rs_decode_matrix: invalid arguments");
  std::vector<uint8_t> enc(static_cast<size_t>(n) * k);
  nxec_gf_gen_rs_matrix(enc.data(), n, k);
  int rc = repair_rows(n, k, enc, input_ids, targets, ntargets, out);
  if (rc != NXEC_OK) return set_error(rc, "nxec_rs_decode_matrix: inputs do not form an invertible matrix");
  return NXEC_OK;
}

extern "C" int nxec_car_plan(int n, int k, int failed, const int32_t *group_offsets, const int32_t *group_chunks,
                             int ngroups, int32_t *sub_offsets, int32_t *sub_chunks, unsigned char *sub_coeffs,
                             int *nsub) {
  using namespace nxec;
  if (nsub) *nsub = 0;
  if (!valid_nk(n, k) || n == k || failed < 0 || failed >= n || ngroups < 0 || (ngroups > 0 && (!group_offsets || !group_chunks)) ||
      !sub_offsets || !sub_chunks || !sub_coeffs || !nsub)
    return set_error(NXEC_ERR_INVALID, "nxec_car_plan: invalid arguments");
  std::vector<int32_t> inputs(n);
  std::vector<uint8_t> row(k);
  int ni = 0, mi = 0;
  const int32_t f = failed;
  int rc = nxec_rs_plan(n, k, &f, 1, 1, inputs.data(), &ni, &mi, row.data());
  if (rc) return rc;
  // chunk id -> position among the k selected inputs (chunk_manager.cc:932-936)
  std::vector<int> pos(n, -1);
  for (int i = 0; i < k; i++) pos[inputs[i]] = i;
  int filled = 0, ns = 0;
  sub_offsets[0] = 0;
  for (int g = 0; g < ngroups && filled < k; g++) {  // scan racks until every input is placed (:939)
    const int before = filled;
    for (int c = group_offsets[g]; c < group_offsets[g + 1]; c++) {
      const int cid = group_chunks[c];
      if (cid < 0 || cid >= n) return set_error(NXEC_ERR_INVALID, "nxec_car_plan: chunk id %d out of range", cid);
      if (pos[cid] < 0) continue;
      sub_chunks[filled] = cid;
      sub_coeffs[filled] = row[pos[cid]];
      pos[cid] = -1;  // a chunk listed twice is used once
      filled++;
    }
    if (filled > before) sub_offsets[++ns] = filled;
  }
  if (filled != k) return set_error(NXEC_ERR_INVALID, "nxec_car_plan: racks cover %d of the %d repair inputs", filled, k);
  *nsub = ns;
  return NXEC_OK;
}
