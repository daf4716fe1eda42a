/*
 * nxec_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Reed-Solomon coding path, used as the
 * parity checker for the MI355X (gfx950) HIP path in nexoedge_amd/.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * or call this library.  The product library (libnxec.so) never links it and
 * has no CPU fallback.
 *
 * Reference followed (paths under /root/reference; "ISA-L:" = inside the
 * vendored third-party/isa-l-2.22.0.tar.gz, pinned at
 * cmake/ExternalProjects.cmake:2-14):
 *   arithmetic  ISA-L:erasure_code/ec_base.c (v2.22.0)
 *   RS glue     src/common/coding/rs.cc, coding_util.hh
 *
 * Parity pinning: every function here is checked in tests/test_oracle_golden.py
 * against tests/golden/golden.json, which oracle/gen_golden.c produces by
 * calling the REFERENCE ISA-L code compiled from the tarball
 * (oracle/build_ref.sh -> oracle/_ref/libisal_base.so).
 */
#ifndef NXEC_ORACLE_H
#define NXEC_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* GF(2^8), polynomial x^8+x^4+x^3+x^2+1 (0x11d), generator 2 */
uint8_t orc_gf_mul(uint8_t a, uint8_t b);                 /* ISA-L ec_base.c:48-60 */
uint8_t orc_gf_inv(uint8_t a);                            /* ISA-L ec_base.c:62-72 */
void orc_gen_rs_matrix(uint8_t *a, int m, int k);         /* ISA-L ec_base.c:74-91 */
int orc_invert_matrix(const uint8_t *in, uint8_t *out, int n); /* ISA-L ec_base.c:111-164 (input not clobbered) */
void orc_init_tables(int k, int rows, const uint8_t *a, uint8_t *gftbls); /* ISA-L ec_base.c:36-46,169-274 */
void orc_encode_data(int len, int k, int rows, const uint8_t *gftbls,
                     const uint8_t *const *src, uint8_t *const *dst); /* ISA-L ec_base.c:302-317 */

/* matrix form of ec_init_tables + ec_encode_data: dst_r = XOR_j a[r*k+j] (x) src_j */
void orc_matmul(int len, int k, int rows, const uint8_t *a, const uint8_t *const *src, uint8_t *const *dst);

/* RSCode::encode (rs.cc:57-92): data is k*cs bytes (caller zero-padded), out is n*cs */
int orc_rs_encode(int n, int k, const uint8_t *data, int64_t cs, uint8_t *out);

/* RSCode::preDecode (rs.cc:238-322).  input_ids receives every alive chunk id
 * (ascending, n - nfailed of them); *min_inputs = k; when is_repair, the
 * nfailed x k repair matrix is written to repair_matrix.  Returns 1 on
 * success, 0 on failure (like the reference's bool). */
int orc_rs_pre_decode(int n, int k, const int32_t *failed, int nfailed, int is_repair,
                      int32_t *input_ids, int *ninputs, int *min_inputs, uint8_t *repair_matrix);

/* RSCode::decode (rs.cc:111-236).  inputs: ninputs chunks of cs bytes, ids
 * ascending in input_ids.  Non-repair: writes k*cs bytes (all data chunks).
 * Repair: targets (ntargets, may be 0 = every id absent from the inputs)
 * -> writes ntargets_out*cs bytes.  use_car selects the CAR finalize branch
 * (rs.cc:184-192).  Returns 1/0 like the reference. */
int orc_rs_decode(int n, int k, const int32_t *input_ids, int ninputs, const uint8_t *const *inputs,
                  int64_t cs, int is_repair, const int32_t *targets, int ntargets, int use_car,
                  uint8_t *out, int *ntargets_out);

/* CodingUtils::encode, contiguous form (coding_util.hh:12-23) */
void orc_coding_utils_encode(const uint8_t *data, int ndata, uint8_t *code, int ncode, int cs, const uint8_t *matrix);

/* deterministic test data: splitmix64 stream, little-endian bytes */
void orc_fill_bytes(uint8_t *p, int64_t nbytes, uint64_t seed);

/* multi-threaded timing helper for the CPU baseline: encodes nstripes
 * [stripe][k][cs] -> [stripe][rows][cs] with `threads` std threads over
 * stripes; returns seconds. */
double orc_time_encode(int k, int rows, const uint8_t *a, const uint8_t *src, uint8_t *dst,
                       int64_t cs, int64_t nstripes, int threads);

/* orc_fill_bytes' stream from 8-byte word `word_off` on */
void orc_fill_bytes_at(uint8_t *p, int64_t nbytes, uint64_t seed, int64_t word_off);

/* CPU baseline stand-in for ISA-L's SIMD kernels (nxec_cpu_simd.c):
 * split-nibble vpshufb, AVX-512BW (level 512) / AVX2 (256) / scalar (0);
 * level -1 = best available.  Returns the level used. */
int orc_simd_level(void);
int orc_simd_encode(int level, size_t len, int k, int rows, const uint8_t *coef, const uint8_t *const *src,
                    uint8_t *const *dst);
/* the reference's per-stripe calls over a stripe range (bench.py cpu_baseline):
 * RSCode::encode incl. the rs.cc:80 copy, and a rows x k decode/recover */
void orc_simd_rscode_encode_range(int level, int n, int k, int64_t cs, int64_t lo, int64_t hi, const uint8_t *data,
                                  uint8_t *chunks, const uint8_t *parity_rows);
void orc_simd_rscode_decode_range(int level, int n, int k, int64_t cs, int64_t lo, int64_t hi, const uint8_t *chunks,
                                  const int32_t *ids, int rows, const uint8_t *matrix, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
