/*
 * nxec.h -- C ABI of the MI355X-native Reed-Solomon coding path for Nexoedge.
 *
 * The reference calls its GF(2^8) arithmetic through five ISA-L entry points
 * (ISA-L 2.22 include/erasure_code.h:74,98,870,905,931), consumed by
 * /root/reference/src/common/coding/rs.cc:26,27,89,104,106,196,219,229,230,290,316
 * and coding_util.hh:20,21,27,28.  Section 1 below replaces those one-for-one
 * (same argument meaning, same layouts); section 2 is the drop-in for
 * ec_encode_data, executed on the GPU; sections 3-4 add the batched
 * device-resident stripe API the proxy ChunkManager / agent use through
 * RSCode (nexoedge_amd/csrc/coding/).  No torch types, no C++ types.
 *
 * Status codes: 0 ok, <0 error (nxec_last_error() says why).  There is no
 * CPU fallback: every compute entry point runs a gfx950 HIP kernel, and
 * fails with NXEC_ERR_NODEV when no device is usable.
 *
 * Thread safety: all entry points are re-entrant.  A context may be shared by
 * threads (the reference shares one RSCode across proxy/agent workers,
 * chunk_manager.cc:1779-1801); its host-staging slots are internally locked.
 */
#ifndef NXEC_H
#define NXEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NXEC_OK 0
#define NXEC_ERR_SINGULAR (-1) /* matrix not invertible (gf_invert_matrix's -1) */
#define NXEC_ERR_INVALID (-2)  /* bad argument */
#define NXEC_ERR_HIP (-3)      /* HIP runtime failure */
#define NXEC_ERR_NOMEM (-4)
#define NXEC_ERR_NODEV (-5)    /* no gfx950 device / HIP unavailable */

#define NXEC_MAX_N 128 /* CODING_MAX_N, coding.hh:13 */
#define NXEC_MAX_K 127

/* last error message of the calling thread ("" if none) */
const char *nxec_last_error(void);
/* library version string */
const char *nxec_version(void);
/* 1 when the library was built with the design-probe kernels (make PROBES=1:
 * the NXEC_EM_PROBE / NXEC_EM_TABLES / NXEC_EM_HASHSRC / NXEC_FM_PROBE A/B
 * variants of DESIGN.md section 4), 0 for the product build */
int nxec_design_probes(void);

/* ---------------------------------------------------------------------------
 * 1. Host GF(2^8) math (poly 0x11d) -- replaces the ISA-L calls in rs.cc.
 * ------------------------------------------------------------------------- */
/* ISA-L gf_mul (erasure_code.h:905); used at rs.cc:219,316 */
unsigned char nxec_gf_mul(unsigned char a, unsigned char b);
/* ISA-L gf_inv; gf_inv(0) == 0 */
unsigned char nxec_gf_inv(unsigned char a);
/* ISA-L gf_gen_rs_matrix (erasure_code.h:870); rs.cc:26.  a: m x k row-major */
void nxec_gf_gen_rs_matrix(unsigned char *a, int m, int k);
/* ISA-L gf_invert_matrix (erasure_code.h:931); rs.cc:196,290.  Like ISA-L it
 * clobbers `in`.  Returns 0, or -1 if singular. */
int nxec_gf_invert_matrix(unsigned char *in, unsigned char *out, const int n);
/* ISA-L ec_init_tables (erasure_code.h:74); rs.cc:27,104,229, coding_util.hh:20,27.
 * gftbls: 32 bytes per coefficient, rows x k, ISA-L layout
 * ([0..15] = c*x, [16..31] = c*(x<<4)); byte [1] of each is the coefficient. */
void nxec_ec_init_tables(int k, int rows, unsigned char *a, unsigned char *gftbls);

/* ---------------------------------------------------------------------------
 * 2. Drop-in synchronous host-buffer encode -- replaces ISA-L ec_encode_data
 *    (erasure_code.h:98) at rs.cc:89,106,230 and coding_util.hh:21,28.
 *    coding[r][i] = XOR_j c(r,j) * data[j][i], c from gftbls (byte [1]).
 *    Runs on a context of the default pool (below), staging through pinned
 *    memory.  The ISA-L signature has no
 *    error channel: on a device error the void form retries once on a fresh
 *    context through the plain staged path (H2D, multiply, D2H), and aborts
 *    with a message only when that fails too (or the arguments are invalid) --
 *    silent corruption is not an option.  The _status form returns the error.
 *    NXEC_TEST_FAIL_ENCODE=1 (testing) fails every first attempt.
 * ------------------------------------------------------------------------- */
void nxec_ec_encode_data(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
                         unsigned char **coding);
int nxec_ec_encode_data_status(int len, int k, int rows, const unsigned char *gftbls,
                               const unsigned char *const *data, unsigned char *const *coding);
/* same, taking the rows x k coefficient matrix directly (no 32-B tables) */
int nxec_encode_host(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *data,
                     unsigned char *const *coding);

/* The default pool: the contexts the entry points without a context argument
 * (this section: nxec_ec_encode_data, nxec_encode_host*, and RSCode /
 * CodingUtils through them) run on.  An unmodified proxy never selects a GPU
 * and shares one RSCode across its worker threads (chunk_manager.cc:
 * 1779-1801, zmq.cc:83), so each call leases the member nxec_default_pick
 * chooses and makes that member's device current for the call only (the
 * caller's current device is restored on return).
 *   devices = NULL, n = 0: one context per visible device (the default);
 *   n < 0: the calling thread's current device (the single-device rule of
 *          rounds 1-5);
 *   n > 0: the listed devices, one context per entry (a device listed twice
 *          gets two contexts).
 * Deployment setting NXEC_DEFAULT_DEVICES=all|current|<d,d,...> (read at the
 * first call; this function overrides it).  Contexts of earlier members stay
 * alive; calls in flight finish on the member they leased. */
int nxec_default_devices(const int *devices, int n);
/* The pool's members (up to max): device, NUMA node of its PCIe root (-1
 * unknown), calls served, calls in flight; *count = members.  With the
 * `current` rule: every device a call has used. */
int nxec_default_pool_stats(int *devices, int *nodes, unsigned long long *calls, int *inflight, int max, int *count);
/* The per-call choice among n members: the fewest calls in flight, where a
 * member on another NUMA node than the calling CPU's (caller_node; -1 or a
 * node of -1: unknown, no preference) counts half a call more -- a local
 * device wins ties, a remote one is taken only when it has fewer calls in
 * flight; on an exact tie `prev` (the member this thread used last; -1
 * none), else the lowest index.  Pure (no device); returns the index. */
int nxec_default_pick(int n, const int *inflight, const int *nodes, int caller_node, int prev);
/* Per-device admission of the calls above: at most *limit (8) run on one
 * device at once, later callers wait for a place (they were already counted
 * by the pick, so the next caller goes to a less busy member).  Reads the
 * device's gate: calls running now, the most that ran at once, calls that
 * found it full; reset != 0 restarts peak and waited.  (64 callers on one
 * GPU: 14-22 GiB/s unbounded, 62-66 with 8) */
int nxec_default_admission(int device, int *limit, int *running, int *peak, unsigned long long *waited, int reset);

/* nxec_encode_host plus fused pass-through: for j < k with copy_idx[j] >= 0,
 * data[j] is also delivered to copy_out[copy_idx[j]] by the same GPU pass
 * (the unit rows of a full-output decode, rs.cc:228-230).  rows may be 0. */
int nxec_encode_host_ex(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *data,
                        unsigned char *const *coding, const int32_t *copy_idx, unsigned char *const *copy_out);
/* nxec_encode_host plus the MD5 of the chunks in the same kernel pass
 * (RSCode::encode's stripe + chunk_manager.cc:175, RSCode::decode(isRepair) +
 * :1173, agent.cc:339 + :342): md5_data (k x 16, NULL = skip) receives the
 * digests of the k inputs, md5_code (rows x 16, NULL = skip) those of the
 * outputs (RFC 1321 byte order).  Pinned / registered buffers (the chunk
 * arena) are read and written in place over PCIe by one k_gather_md5 launch;
 * concurrent callers' calls of one chunk length are aggregated into one
 * launch (nxec_agent_encode_batch's rounds on the thread's default context).
 * Synchronous; thread-safe. */
int nxec_encode_host_md5(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *data,
                         unsigned char *const *coding, unsigned char *md5_data, unsigned char *md5_code);
/* Where nxec_encode_host_md5 hashes (the coding always runs on the GPU):
 * NXEC_DIGEST_GPU -- in the coding kernel (one ~10 ms/MiB MD5 chain per chunk,
 * thousands at once); NXEC_DIGEST_HOST -- OpenSSL on the library's digest
 * pool (NXEC_DIGEST_THREADS, default min(16, CPUs)) plus the calling thread,
 * the inputs' digests overlapping the GPU pass; NXEC_DIGEST_AUTO (default) --
 * per call, whichever the measured pool backlog and GPU latency say finishes
 * first (few callers: the pool; many: the surplus on the GPU).  Environment:
 * NXEC_DIGEST_PLACE=auto|gpu|host.  Returns the previous mode, or < 0. */
#define NXEC_DIGEST_AUTO 0
#define NXEC_DIGEST_GPU 1
#define NXEC_DIGEST_HOST 2
int nxec_set_digest_placement(int mode);
int nxec_digest_placement(void);
/* calls placed on the host pool / the GPU so far, and the pool's threads */
int nxec_digest_place_stats(unsigned long long *host_calls, unsigned long long *gpu_calls, int *host_threads);
/* the auto placement's inputs: the process's CPU budget (the smallest cgroup
 * quota from its own cgroup up, capped by the affinity mask; NXEC_DIGEST_CPUS
 * overrides) and the crossover H in calling threads (NXEC_DIGEST_HOST_CALLERS) */
int nxec_digest_place_params(double *cpu_budget, double *host_callers);

/* ---------------------------------------------------------------------------
 * 2b. The boundary under the names of SURVEY §8b (thin forms of the above,
 *     coefficient matrices instead of 32-B tables, non-clobbering inverse).
 * ------------------------------------------------------------------------- */
/* == nxec_gf_gen_rs_matrix (ISA-L gf_gen_rs_matrix, rs.cc:26) */
void nxec_gen_rs_matrix(unsigned char *a, int n, int k);
/* rs.cc:196,290 without ISA-L's clobbering of `in`: 0, or -1 if singular */
int nxec_invert_matrix(const unsigned char *in, unsigned char *out, int k);
/* == nxec_ec_init_tables with a const coefficient matrix (ISA-L 32-B layout) */
void nxec_init_tables(int k, int rows, const unsigned char *coeffs, unsigned char *tbls);
/* ec_init_tables + ec_encode_data from the rows x k matrix: == nxec_encode_host */
int nxec_encode_data(int len, int k, int rows, const unsigned char *coeffs, const unsigned char *const *src,
                     unsigned char *const *dst);

/* ---------------------------------------------------------------------------
 * 3. Contexts and batched device-resident stripe ops.
 *    Layout: stripe s, chunk c starts at base + s*stripe_stride + c*chunk_stride.
 *    `stream` is a hipStream_t (NULL = the context's stream).  Launches are
 *    asynchronous on that stream; buffers must stay valid until it drains.
 * ------------------------------------------------------------------------- */
typedef struct nxec_ctx nxec_ctx_t;

int nxec_ctx_create(int device, nxec_ctx_t **out);
void nxec_ctx_destroy(nxec_ctx_t *ctx);
void *nxec_ctx_stream(nxec_ctx_t *ctx);

/* The one primitive behind encode, recover, repair, agent partial encode and
 * CAR finalize: for every stripe s and byte i < len,
 *   dst(s, dst_idx[r])[i] = XOR_{j<k} coeffs[r*k + j] (x) src(s, src_idx[j])[i],  r < rows.
 * src_idx / dst_idx: chunk indices (NULL = 0..k-1 / 0..rows-1).
 * copy_idx (optional, NULL = none): for j < k with copy_idx[j] >= 0 the raw
 * source chunk is also written to dst chunk copy_idx[j] (fused survivor copy
 * of a full-output decode, rs.cc:175-181 semantics).
 * rows, k in 1..NXEC_MAX_K; len >= 0; nstripes >= 0. */
int nxec_stripes_mul(nxec_ctx_t *ctx, int rows, int k, const unsigned char *coeffs, const unsigned char *d_src,
                     const int32_t *src_idx, int64_t src_chunk_stride, int64_t src_stripe_stride,
                     unsigned char *d_dst, const int32_t *dst_idx, int64_t dst_chunk_stride,
                     int64_t dst_stripe_stride, const int32_t *copy_idx, int64_t len, int64_t nstripes,
                     void *stream);

/* SURVEY §8b's nxec_matmul_batch: nxec_stripes_mul with identity index maps
 * (src chunks 0..k-1, dst chunks 0..rows-1, no copies). */
int nxec_matmul_batch(nxec_ctx_t *ctx, int rows, int k, const unsigned char *coeffs, const unsigned char *d_src,
                      int64_t src_chunk_stride, int64_t src_stripe_stride, unsigned char *d_dst,
                      int64_t dst_chunk_stride, int64_t dst_stripe_stride, int64_t len, int64_t nstripes,
                      void *stream);

/* Gather form for non-contiguous chunks: d_src_ptrs is a DEVICE array of
 * nstripes*k device pointers ([s][j]), d_dst_ptrs of nstripes*rows. */
int nxec_stripes_mul_ptrs(nxec_ctx_t *ctx, int rows, int k, const unsigned char *coeffs,
                          const unsigned char *const *d_src_ptrs, unsigned char *const *d_dst_ptrs, int64_t len,
                          int64_t nstripes, void *stream);

/* ---------------------------------------------------------------------------
 * 4. RSCode-level batched ops over the [stripe][n][len] layout
 *    (RS with nexoedge's (n, k): n total chunks, k data chunks).
 * ------------------------------------------------------------------------- */
/* RSCode::encode (rs.cc:57-92) for a batch: chunks k..n-1 of every stripe are
 * computed from chunks 0..k-1. */
int nxec_rs_encode_stripes(nxec_ctx_t *ctx, int n, int k, unsigned char *d_stripes, int64_t chunk_stride,
                           int64_t stripe_stride, int64_t len, int64_t nstripes, void *stream);

/* Recover-only decode / repair in place: rebuilds the `nfailed` chunks listed
 * in `failed` (ascending) from the first k alive chunks, exactly the plan of
 * RSCode::preDecode(isRepair=true) (rs.cc:238-322).  Erased slots are only
 * written, never read. */
int nxec_rs_recover_stripes(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                            unsigned char *d_stripes, int64_t chunk_stride, int64_t stripe_stride, int64_t len,
                            int64_t nstripes, void *stream);

/* Full-output decode with RSCode::decode semantics (rs.cc:111-236, non-repair):
 * inputs = the first k alive chunks of d_stripes (ascending ids; `failed`
 * lists the erased ids), output = all k data chunks into d_out
 * ([s][j] at d_out + s*out_stripe_stride + j*out_chunk_stride).  Survivor data
 * chunks are copied from registers in the same pass (bit-identical to the
 * reference's unit rows of the inverse). */
int nxec_rs_decode_stripes(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                           const unsigned char *d_stripes, int64_t chunk_stride, int64_t stripe_stride,
                           unsigned char *d_out, int64_t out_chunk_stride, int64_t out_stripe_stride, int64_t len,
                           int64_t nstripes, void *stream);

/* The library's recommended HBM layout of a [stripe][chunk] batch with chunks
 * of `len` bytes (chunk c of stripe s at base + s*stripe_stride +
 * c*chunk_stride).  The batch layout is the caller's choice (every entry point
 * takes both strides); these strides avoid the DRAM channel/bank aliasing that
 * power-of-two chunk strides cause (profiles/r02_layout_*.log):
 *  - chunks >= 2 MiB: chunk_stride = len + a pad that breaks the
 *    power-of-two stride: 3 KiB for multiples of 4 MiB (RS(16,4) 4 MiB: 0.71
 *    packed, 0.754 with 2 KiB, 0.772 with 3 KiB of 8 TB/s, every erasure
 *    pattern >= 0.76; RS(12,4) 4 MiB 0.756 -> 0.781), 5 KiB at 2 MiB, 2 KiB
 *    otherwise;
 *  - measured smaller shapes: n = 20 with 256 KiB chunks +4 KiB (RS(16,4)
 *    0.755 -> 0.766), n = 14 with 128 KiB +10 KiB (0.68 -> 0.78) and 256
 *    KiB +12 KiB (0.71 -> 0.745); other small shapes: nxec_batch_layout_tuned;
 *  - stripes of 1 MiB-multiple chunks whose size is a power-of-two number of
 *    MiB: stripe_stride padded by one chunk to an odd multiple (RS(12,4) 1
 *    MiB: encode 0.80 -> 0.81, single-failure repair 0.74 -> 0.79);
 *  - NXEC_LAYOUT_RECOVER_HEAVY with any even number of such chunks: the same
 *    padding (RS(10,4) 1 MiB scattered 4-erasure recover 0.71 -> 0.78, encode
 *    0.80 -> 0.79);
 *  - otherwise the packed layout (chunk_stride = len rounded up to 16,
 *    stripe_stride = n * chunk_stride). */
#define NXEC_LAYOUT_RECOVER_HEAVY 1

/* The same choice measured on this device instead of read from the table
 * above: how DRAM channels and banks serve the k + rows streams of a column
 * depends on the chunk and stripe strides in ways no static rule captures
 * for every geometry (a 4 KiB chunk pad is worth +0.02 of 8
 * TB/s for RS(16,4) 256 KiB chunks and costs -0.11 at 1 MiB).  Scores
 * RS(n,k) encode, a contiguous and a scattered min(n-k,4)-erasure recover
 * (equal weights; NXEC_LAYOUT_RECOVER_HEAVY doubles the scattered one) over a
 * scratch batch of about budget_bytes (<= 0: 24 GiB, capped at a quarter of
 * the free device memory) for a few candidate layouts (the table's, packed,
 * chunk pads of 1.5-16 KiB, an odd stripe stride), each in three
 * interleaved rounds; the table's layout stays unless another beats it in
 * every round by more than the rounds' spread (nxec_layout_choose, at least
 * 0.5 %).  The result is cached per (device, n, k, len, flags, budget_bytes);
 * the first call for a shape takes ~2-4 s.  Uses ctx's
 * stream and device; the scratch batch is freed before it returns. */
int nxec_batch_layout_tuned(nxec_ctx_t *ctx, int n, int k, int64_t len, int flags, int64_t budget_bytes,
                            int64_t *chunk_stride, int64_t *stripe_stride);
/* The choice rule of nxec_batch_layout_tuned (pure; exported for tests):
 * scores[r * ncand + c] = candidate c's score in round r (c = 0 is the
 * incumbent, the table's layout; <= 0 = not measured).  A challenger replaces
 * the incumbent only when it beats it in EVERY round by more than
 * max(min_margin, the relative spread (max - min) / mean of its own and the
 * incumbent's scores across the rounds); among such challengers the highest
 * mean wins.  Otherwise (ties included) 0: the incumbent. */
int nxec_layout_choose(int ncand, int rounds, const double *scores, double min_margin);
int nxec_batch_layout(int n, int64_t len, int flags, int64_t *chunk_stride, int64_t *stripe_stride);

/* Host-resident batch encode (the proxy write path): h_data [s][k][len] in,
 * h_parity [s][n-k][len] out, both host memory.  When both are pinned or
 * registered (device-mapped) the kernel reads and writes them over PCIe
 * directly (zero copy; NXEC_HOST_DIRECT=0 disables); otherwise double-buffered
 * H2D -> kernel -> D2H over `batch_stripes` stripes per step.  Synchronous. */
int nxec_rs_encode_host_batch(nxec_ctx_t *ctx, int n, int k, const unsigned char *h_data,
                              unsigned char *h_parity, int64_t len, int64_t nstripes, int64_t batch_stripes);

/* Host planning of RSCode::preDecode (rs.cc:238-322): input_ids gets every
 * alive id ascending (n - nfailed of them, *ninputs), *min_inputs = k; with
 * is_repair the nfailed x k repair matrix goes to repair_matrix.  Returns 0,
 * NXEC_ERR_INVALID (too many failures) or NXEC_ERR_SINGULAR. */
int nxec_rs_plan(int n, int k, const int32_t *failed, int nfailed, int is_repair, int32_t *input_ids,
                 int *ninputs, int *min_inputs, unsigned char *repair_matrix);
/* Decode matrix rows (rs.cc:141-225): given the k ascending input ids, the
 * coefficient rows (ntargets x k) that rebuild each target id. */
int nxec_rs_decode_matrix(int n, int k, const int32_t *input_ids, const int32_t *targets, int ntargets,
                          unsigned char *out);

/* Cross-rack-aware (CAR) single-failure repair plan, chunk_manager.cc:929-986:
 * given the racks' chunk-id lists (as the coordinator's findChunkGroups
 * reports them: group g holds group_chunks[group_offsets[g] .. group_offsets[g+1])),
 * keep in each rack only the chunks chosen as repair inputs (the first k alive,
 * rs.cc:252-265) and attach to each its coefficient of the repair row.  Output:
 * *nsub sub-groups (sub_offsets[0..*nsub], sub_chunks, sub_coeffs in group
 * order; racks with no selected chunk are skipped).  Each sub-group is one
 * agent's partial encode (ENC_CHUNK_REQ, container_manager.cc:221-258); the
 * XOR of the partials is the lost chunk (rs.cc:94-109). */
int nxec_car_plan(int n, int k, int failed, const int32_t *group_offsets, const int32_t *group_chunks, int ngroups,
                  int32_t *sub_offsets, int32_t *sub_chunks, unsigned char *sub_coeffs, int *nsub);

/* Device-resident CAR repair over a batch: per stripe, one partial encode per
 * sub-group of the plan above into d_partials ([s][nsub][len], caller scratch,
 * partial_stripe_stride bytes per stripe), then the all-ones XOR of the
 * partials into chunk `failed` of d_stripes -- the agents' and proxy's work of
 * a CAR repair (agent.cc:240-415) on one GPU.  Partial g of stripe s is at
 * d_partials + s * partial_stripe_stride + g * partial_chunk_stride. */
int nxec_rs_car_repair_stripes(nxec_ctx_t *ctx, int n, int k, int failed, const int32_t *group_offsets,
                               const int32_t *group_chunks, int ngroups, unsigned char *d_stripes, int64_t chunk_stride,
                               int64_t stripe_stride, unsigned char *d_partials, int64_t partial_chunk_stride,
                               int64_t partial_stripe_stride, int64_t len, int64_t nstripes, void *stream);

/* MD5 digest of every chunk of a device-resident batch: the
 * checksum the reference computes per chunk on writes and repairs
 * (chunk_manager.cc:175,1173, agent.cc:342 -> Chunk::computeMD5, chunk.hh:136).
 * Chunk c of stripe s at d_base + s*stripe_stride + c*chunk_stride, len bytes;
 * digest (16 bytes, RFC 1321 byte order) at d_digests[(s*nchunks + c)*16]. */
int nxec_md5_chunks(nxec_ctx_t *ctx, const unsigned char *d_base, int64_t chunk_stride, int64_t stripe_stride,
                    int nchunks, int64_t len, int64_t nstripes, unsigned char *d_digests, void *stream);

/* Chunk::verifyMD5 over a batch: the read path's check of every fetched chunk
 * (chunk_manager.cc:1553-1555) and the agent's VRF_CHUNK_REQ scan
 * (ContainerManager::verifyChunks, container_manager.cc:187-207).  Hashes like
 * nxec_md5_chunks and compares with d_expected (same [s][c][16] layout):
 * d_ok[s*nchunks + c] = 1 if equal, 0 if not; *d_nbad (device, optional, not
 * reset) += the number of mismatches. */
int nxec_md5_verify_chunks(nxec_ctx_t *ctx, const unsigned char *d_base, int64_t chunk_stride, int64_t stripe_stride,
                           int nchunks, int64_t len, int64_t nstripes, const unsigned char *d_expected,
                           unsigned char *d_ok, unsigned long long *d_nbad, void *stream);

/* RSCode::encode plus Chunk::computeMD5 of all n chunks of every stripe of a
 * device-resident batch -- the write path's coding work (chunk_manager.cc:
 * 99-175) -- in one pass over the data: parity as nxec_rs_encode_stripes,
 * digests as nxec_md5_chunks (d_digests[(s*n + c)*16]).  One fused kernel
 * when n - k <= 4, k <= 20, len is a multiple of 256 and the layout is 16-byte
 * aligned; otherwise the encode, then the MD5 launch. */
int nxec_rs_encode_md5_stripes(nxec_ctx_t *ctx, int n, int k, unsigned char *d_stripes, int64_t chunk_stride,
                               int64_t stripe_stride, int64_t len, int64_t nstripes, unsigned char *d_digests,
                               void *stream);

/* Repair with checksums: nxec_rs_recover_stripes (rebuilds the `nfailed`
 * chunks in place from the first k alive ones, rs.cc:238-322) plus the MD5 of
 * every rebuilt chunk -- the proxy's repair step before it sends the chunks
 * out (chunk_manager.cc:1173, Chunk::computeMD5) -- in one pass.  Digest of
 * rebuilt chunk failed[r] of stripe s at d_digests[(s*nfailed + r)*16].  One
 * fused kernel when nfailed <= 4, k <= 20, len is a multiple of 256 and the
 * layout is 16-byte aligned; otherwise the recover, then the MD5 launch. */
int nxec_rs_recover_md5_stripes(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                                unsigned char *d_stripes, int64_t chunk_stride, int64_t stripe_stride, int64_t len,
                                int64_t nstripes, unsigned char *d_digests, void *stream);

/* ---- Object-level batched entry (ChunkManager write/read of a
 * whole object in one call instead of the per-stripe loop of
 * proxy_file_ops.cc:557-666 / chunk_manager.cc:99,787).
 *
 * Layout of an object of `length` bytes under (n,k) and max chunk size M
 * (storage class max_chunk_size): full stripes hold k*M data bytes with
 * chunk size M; a remainder r > 0 forms one last stripe with chunk size
 * ceil(r/k) (RSCode::getChunkSize, rs.cc:52-55), zero-padded to k chunks
 * (chunk_manager.cc:390-399).  Chunk (s, i) has id s*n + i
 * (chunk_manager.cc:441-447). */
int nxec_object_layout(int n, int k, int64_t length, int64_t max_chunk_size, int64_t *nstripes,
                       int64_t *full_stripes, int64_t *last_chunk_size);

/* Encode an object resident in HBM.  Data chunks are read in place (full
 * stripes: chunk (s, j) = d_object + s*k*M + j*M).  Parity chunk (s, i) is
 * written at d_parity + (s*(n-k) + i)*M ([nstripes][n-k][M]; the last stripe
 * uses the first last_chunk_size bytes of its slots).  d_tail (k*M bytes, may
 * be NULL when length is a multiple of k*M) receives the zero-padded data
 * chunks of the last stripe at j*last_chunk_size.  d_md5 (NULL = skip):
 * [nstripes][n][16] MD5 digests of every chunk (Chunk::computeMD5 of
 * writeFileStripe, chunk_manager.cc:175), one kernel launch. */
int nxec_encode_object(nxec_ctx_t *ctx, int n, int k, const unsigned char *d_object, int64_t length,
                       int64_t max_chunk_size, unsigned char *d_parity, unsigned char *d_tail, unsigned char *d_md5,
                       void *stream);

/* Read path (decodeFile, chunk_manager.cc:738-800, batched): chunks of the
 * object as fetched, chunk (s, i) at d_chunks + (s*n + i)*M (last stripe:
 * last_chunk_size bytes per slot), chunks `failed` (ascending, same for every
 * stripe) absent.  Writes the `length` object bytes to d_object; d_tail is
 * k*M bytes of scratch (may be NULL when length is a multiple of k*M). */
int nxec_decode_object(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                       const unsigned char *d_chunks, int64_t length, int64_t max_chunk_size, unsigned char *d_object,
                       unsigned char *d_tail, void *stream);
/* the same with chunk (s, i) at d_chunks + s*stripe_stride + i*chunk_stride
 * (e.g. the nxec_batch_layout(..., NXEC_LAYOUT_RECOVER_HEAVY) strides
 * StripeBatch::decodeFile stages fetched chunks at) */
int nxec_decode_object_ex(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                          const unsigned char *d_chunks, int64_t chunk_stride, int64_t stripe_stride, int64_t length,
                          int64_t max_chunk_size, unsigned char *d_object, unsigned char *d_tail, void *stream);

/* Read path with checksums: every chunk used as a decode input (the first k
 * alive ones of each stripe) has its MD5 checked against d_md5 ([ns][n][16],
 * as nxec_encode_object wrote it) -- Chunk::verifyMD5 on each fetched chunk,
 * chunk_manager.cc:1548-1556 with verifyChunkChecksum -- and the object is
 * decoded as nxec_decode_object does, in one pass over the chunks (fused
 * kernel for the full stripes when k <= 20, the lost data chunks <= 4 and
 * max_chunk_size is a multiple of 256).  d_ok [ns][n]: byte (s, c) = 1 if
 * chunk c of stripe s matched, 0 if not; entries of chunks that were not read
 * are left as they were.  *d_nbad (device, optional, not reset) += mismatches.
 * A stripe with a mismatch decodes to undefined bytes: re-plan it with the
 * bad chunks marked failed (the reference fails such a stripe's read). */
int nxec_decode_object_verify(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                              const unsigned char *d_chunks, int64_t length, int64_t max_chunk_size,
                              const unsigned char *d_md5, unsigned char *d_object, unsigned char *d_tail,
                              unsigned char *d_ok, unsigned long long *d_nbad, void *stream);

/* Many objects in one call (the proxy's per-file loop, proxy_file_ops.cc:557-666,
 * over a batch of files): object o (d_objects[o], a HOST array of device
 * pointers, lengths[o] bytes) is split as in nxec_object_layout; its stripes
 * follow the previous objects' in one global stripe order g.  Parity chunk
 * (g, i) at d_parity + (g*(n-k) + i)*M; digests (NULL = skip) at
 * d_md5 + g*n*16.  The data chunks of each object's last stripe (chunk size
 * cl) are written zero-padded to the d_tail arena (size from
 * nxec_objects_layout), objects in order, chunk j of an object at
 * tail_off + j*cls with cls = cl rounded up to 16 (bytes [cl, cls) zero;
 * the object's tail_off advances by k*cls).  Full stripes of all objects run
 * as one gather launch, last stripes as one work-queue launch over
 * variable-length stripes, every chunk's MD5 as one launch.  Synchronous
 * (returns when the work is done). */
int nxec_objects_layout(int n, int k, int nobjects, const int64_t *lengths, int64_t max_chunk_size,
                        int64_t *total_stripes, int64_t *tail_bytes);
int nxec_encode_objects(nxec_ctx_t *ctx, int n, int k, int nobjects, const unsigned char *const *d_objects,
                        const int64_t *lengths, int64_t max_chunk_size, unsigned char *d_parity,
                        unsigned char *d_tail, unsigned char *d_md5, void *stream);
/* The same with flags.  NXEC_OBJECTS_TAIL_INPLACE: a batching ChunkManager
 * that sends every chunk from where it lies (the full stripes' data chunks
 * are read in place already) needs only one data chunk of a last stripe
 * materialised: with cl = last_chunk_size and r = the object's bytes past its
 * full stripes, chunk j < r / cl is the object's bytes at
 * nf*k*M + j*cl (whole, in place), chunk j = r / cl < k -- when r % cl != 0 --
 * holds r % cl object bytes and is written zero-padded to its tail-arena
 * slot (same layout as above), and chunks past it are all zero bytes.
 * Parity and digests are those of the zero-padded stripe, as without the
 * flag; tail-arena slots of whole and all-zero chunks are left unspecified
 * (the one-launch path reads the last stripe in place and writes only the
 * partial chunk's slot -- one chunk of k -- except for an object that ends
 * within 16 bytes of a 4 KiB page boundary with a chunk length that is not
 * a multiple of 16, whose chunks from the one that would read past the
 * page are copied zero padded to their slots first). */
#define NXEC_OBJECTS_TAIL_INPLACE 1
/* NXEC_OBJECTS_ASYNC: return once the work is queued on `stream` (NULL: the
 * context's) instead of when it is done.  lengths[] and d_objects[] (host
 * arrays) may be reused at once; the objects, d_parity, d_tail and d_md5 are
 * in use until the stream gets past the call.  A batching ChunkManager plans
 * batch i + 1 on the host while batch i codes: its staging slot returns to
 * the context's pool with an event the next user of that slot waits on (up
 * to 4 calls in flight per context before one waits). */
#define NXEC_OBJECTS_ASYNC 2
int nxec_encode_objects_ex(nxec_ctx_t *ctx, int n, int k, int nobjects, const unsigned char *const *d_objects,
                           const int64_t *lengths, int64_t max_chunk_size, unsigned char *d_parity,
                           unsigned char *d_tail, unsigned char *d_md5, int flags, void *stream);

/* Device time of the coding launches of nxec_encode_objects(_ex) calls on ctx
 * (roofline measurement: HIP events on the launch stream around the call's
 * coding kernel -- k_files_md5 on the one-launch path; the pad copy, gather
 * launches and MD5 launch together on the separate path).  nxec_kernel_timing
 * turns it on (1) or off (0) and resets the totals; nxec_kernel_time waits for
 * the pending launches and returns the milliseconds and launches since. */
int nxec_kernel_timing(nxec_ctx_t *ctx, int enable);
int nxec_kernel_time(nxec_ctx_t *ctx, double *ms, int64_t *launches);

/* Host-inclusive form of nxec_encode_object: the object, parity
 * ([nstripes][n-k][M]) and digests ([nstripes][n][16], NULL = skip) are in
 * host memory (pin them -- nxec_host_malloc_pinned / nxec_host_register -- for
 * full PCIe rate).  Batches of batch_stripes stripes (<= 0: ~1 GiB of chunks)
 * stream H2D -> encode -> MD5 -> D2H on three concurrent streams.
 * Synchronous. */
int nxec_encode_object_host(nxec_ctx_t *ctx, int n, int k, const unsigned char *h_object, int64_t length,
                            int64_t max_chunk_size, unsigned char *h_parity, unsigned char *h_md5,
                            int64_t batch_stripes);

/* ---- Agent coding service: the agent's two compute steps,
 * batched over many requests.  Each request is CodingUtils::encode
 * (coding_util.hh:25-31) of `ninputs` host chunks by a noutputs x ninputs
 * matrix: the ENC_CHUNK_REQ partial encode (ContainerManager::
 * getEncodedChunks, container_manager.cc:221-258: 1 x g row) or the
 * RPR_CHUNK_REQ repair (agent.cc:240-415: all-ones 1 x G for CAR, the
 * proxy's e x k matrix otherwise), plus the MD5 of every output
 * (agent.cc:342) when md5 != NULL (and of every input when md5_inputs !=
 * NULL).  Requests with the same shape and matrix run as one kernel pass; staging is pinned and double-buffered so the host
 * gather of batch i+1 overlaps the GPU work of batch i.  batch_bytes bounds
 * the staging per batch (<= 0: 256 MiB).  Synchronous; thread-safe. */
typedef struct nxec_agent_req {
  int ninputs;
  int noutputs;
  const unsigned char *matrix;        /* noutputs x ninputs, row-major */
  const unsigned char *const *inputs; /* ninputs host chunks of chunk_size bytes */
  unsigned char *const *outputs;      /* noutputs host buffers of chunk_size bytes */
  unsigned char *md5;                 /* noutputs x 16 digest bytes, or NULL */
  unsigned char *md5_inputs;          /* ninputs x 16 digests of the inputs, or NULL
                                         (RSCode::encode hashes its data chunks too) */
} nxec_agent_req;

int nxec_agent_encode_batch(nxec_ctx_t *ctx, const nxec_agent_req *reqs, int nreqs, int64_t chunk_size,
                            int64_t batch_bytes);

/* ---- Chunk frames <-> device batch (the in-scope part of the
 * wire format).  IO::getChunkEventMessage mallocs and memcpys every received
 * chunk frame (common/io.cc:209-216) and sendChunkEventMessage sends one frame
 * per chunk (:334-336); these move such frames straight between their message
 * buffers and a strided device batch, so received chunks feed
 * nxec_rs_decode_stripes / nxec_decode_object and encoded chunks go out
 * without a per-chunk malloc.
 * nxec_gather_chunks:  h_chunks[i] (len bytes) -> d_dst + i*dst_stride
 * nxec_scatter_chunks: d_src + i*src_stride    -> h_chunks[i]
 * Any alignment; pinned / registered frames of >= 8 MiB are DMA'd directly, others
 * go through the context's pinned slots (host pool packs piece p while the copy
 * engine moves piece p-1).  Synchronous: the frames may be reused or read on
 * return.  `stream` orders the device side (NULL = context stream). */
int nxec_gather_chunks(nxec_ctx_t *ctx, const unsigned char *const *h_chunks, int64_t nchunks, int64_t len,
                       unsigned char *d_dst, int64_t dst_stride, void *stream);
int nxec_scatter_chunks(nxec_ctx_t *ctx, const unsigned char *d_src, int64_t src_stride, int64_t nchunks, int64_t len,
                        unsigned char *const *h_chunks, void *stream);

/* Asynchronous forms: the copy runs on a worker thread and the call returns
 * at once with a request handle (NULL when the arguments are rejected; the
 * error is then the return value).  The frame pointer array is copied, the
 * frames themselves and the device range must stay valid, and the frames
 * untouched, until nxec_request_wait.  One caller can so overlap receiving
 * request i+1 (gather, host->device) with sending request i (scatter,
 * device->host) -- IO::getChunkEventMessage / sendChunkEventMessage
 * (common/io.cc:104-364) in flight together.  Requests on one stream
 * serialise on the device: give the two directions different streams
 * (nxec_stream_create) to use both link directions at once. */
typedef struct nxec_request nxec_request_t;
int nxec_gather_chunks_async(nxec_ctx_t *ctx, const unsigned char *const *h_chunks, int64_t nchunks, int64_t len,
                             unsigned char *d_dst, int64_t dst_stride, void *stream, nxec_request_t **req);
int nxec_scatter_chunks_async(nxec_ctx_t *ctx, const unsigned char *d_src, int64_t src_stride, int64_t nchunks,
                              int64_t len, unsigned char *const *h_chunks, void *stream, nxec_request_t **req);
/* Waits for the request, frees it and returns its status (the request's error
 * message becomes the caller's nxec_last_error).  NULL is a no-op (0). */
int nxec_request_wait(nxec_request_t *req);

/* RSCode::decode's recover step (rs.cc:111-236 with the rs.cc:238-322 plan) on
 * chunk frames: frames[s*n + c] is chunk c of stripe s in host memory (len
 * bytes); the first k alive chunks are read, the `failed` ones written (other
 * entries may be NULL).  When every frame involved is pinned / registered
 * host memory (e.g. a receive-buffer pool passed to nxec_host_register) one
 * kernel reads the survivors and writes the recovered chunks over PCIe through
 * device pointer tables (zero copy); otherwise the frames are staged through
 * HBM in batches (nxec_gather_chunks, recover, nxec_scatter_chunks).
 * Synchronous. */
int nxec_rs_recover_frames(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                           unsigned char *const *frames, int64_t len, int64_t nstripes);

/* The proxy's read path on received frames, pipelined inside one call:
 * decodeFile (chunk_manager.cc:738-800, RSCode::decode's all-k output,
 * rs.cc:111-236) for a batch of stripes whose chunks arrived as frames
 * (io.cc:209-216).  in_frames[s*n + c] is chunk c of stripe s (len bytes, any
 * alignment, pageable or pinned); only the k chunks rs.cc:252-265 chooses are
 * read (entries of failed chunks may be NULL).  All k data chunks of stripe s
 * are written to out_frames[s*k + j].  The stripes go through HBM in batches
 * of batch_stripes (<= 0: about 128 MiB of chunks per batch) on three streams:
 * the gather of batch b + 1 (host -> device), the decode of batch b and the
 * scatter of batch b - 1 (device -> host) run at once, so both PCIe
 * directions and the host copy pool are busy together.  Synchronous. */
int nxec_decode_frames(nxec_ctx_t *ctx, int n, int k, const int32_t *failed, int nfailed,
                       const unsigned char *const *in_frames, unsigned char *const *out_frames, int64_t len,
                       int64_t nstripes, int64_t batch_stripes);

/* ---- Multi-GPU group in one process: one context per device,
 * a batch's stripes split into contiguous ranges (sizes differ by at most one),
 * one long-lived host thread per member (started by nxec_group_create, bound
 * once to its GPU's NUMA node); no collective, no peer traffic.  The plain
 * calls are synchronous; the _async forms below are not.  A device may appear
 * twice (two contexts on one GPU). */
typedef struct nxec_group nxec_group_t;
int nxec_group_create(const int *devices, int ndevices, nxec_group_t **out);
void nxec_group_destroy(nxec_group_t *g);
int nxec_group_size(const nxec_group_t *g);
nxec_ctx_t *nxec_group_ctx(nxec_group_t *g, int i);
/* stripes [first, first+count) of `nstripes` belong to part `part` of `nparts` */
int nxec_group_shard(int64_t nstripes, int nparts, int part, int64_t *first, int64_t *count);
/* nxec_rs_encode_host_batch over the group: device i encodes its shard of the
 * host [nstripes][k][len] data into host [nstripes][n-k][len] parity */
int nxec_group_rs_encode_host_batch(nxec_group_t *g, int n, int k, const unsigned char *h_data,
                                    unsigned char *h_parity, int64_t len, int64_t nstripes, int64_t batch_stripes);
/* device-resident shards: d_stripes[i] / nstripes[i] live on the group's device i */
int nxec_group_rs_encode_stripes(nxec_group_t *g, int n, int k, unsigned char *const *d_stripes, int64_t chunk_stride,
                                 int64_t stripe_stride, int64_t len, const int64_t *nstripes);
int nxec_group_rs_recover_stripes(nxec_group_t *g, int n, int k, const int32_t *failed, int nfailed,
                                  unsigned char *const *d_stripes, int64_t chunk_stride, int64_t stripe_stride,
                                  int64_t len, const int64_t *nstripes);
/* Asynchronous forms: each member's thread queues its shard's launches on its
 * context's stream and the call returns at once (the arrays are copied; a
 * member runs its calls in submission order).  Per-member failures (bad
 * arguments of one member's shard, a launch error) are kept and returned by
 * the next nxec_group_wait, which blocks until every call queued before it
 * has finished on every member's device. */
int nxec_group_rs_encode_stripes_async(nxec_group_t *g, int n, int k, unsigned char *const *d_stripes,
                                       int64_t chunk_stride, int64_t stripe_stride, int64_t len,
                                       const int64_t *nstripes);
int nxec_group_rs_recover_stripes_async(nxec_group_t *g, int n, int k, const int32_t *failed, int nfailed,
                                        unsigned char *const *d_stripes, int64_t chunk_stride, int64_t stripe_stride,
                                        int64_t len, const int64_t *nstripes);
int nxec_group_wait(nxec_group_t *g);

/* ---------------------------------------------------------------------------
 * 5. Device plumbing (memory, streams, events) so hosts without a GPU
 *    framework can drive section 3.  Thin wrappers over the HIP runtime.
 * ------------------------------------------------------------------------- */
int nxec_device_count(int *count);
int nxec_set_device(int device);
int nxec_device_info(int device, char *name, int name_len, int *num_cus, int64_t *total_mem);
int nxec_dev_malloc(void **p, size_t bytes);
int nxec_dev_free(void *p);
int nxec_host_malloc_pinned(void **p, size_t bytes);
int nxec_host_free_pinned(void *p);
int nxec_host_register(void *p, size_t bytes);
int nxec_host_unregister(void *p);
int nxec_memcpy_h2d(void *d_dst, const void *h_src, size_t bytes, void *stream);
int nxec_memcpy_d2h(void *h_dst, const void *d_src, size_t bytes, void *stream);
int nxec_memcpy_d2d(void *d_dst, const void *d_src, size_t bytes, void *stream);
int nxec_memset(void *d_dst, int value, size_t bytes, void *stream);
/* rows of `width` bytes, `height` of them, `pitch` apart (e.g. one chunk of every stripe) */
int nxec_memset2d(void *d_dst, size_t pitch, int value, size_t width, size_t height, void *stream);
int nxec_stream_create(void **stream);
int nxec_stream_destroy(void *stream);
int nxec_stream_sync(void *stream);
int nxec_device_sync(void);
int nxec_event_create(void **event);
int nxec_event_destroy(void *event);
int nxec_event_record(void *event, void *stream);
int nxec_event_elapsed_ms(void *start, void *stop, float *ms);
/* deterministic device fill: the splitmix64 byte stream (word i = mix(seed + (i+1)*0x9E3779B97F4A7C15), LE) */
int nxec_fill_random(void *d_dst, size_t bytes, uint64_t seed, void *stream);
/* order-sensitive 64-bit digest of a device buffer: sum_i word_i * (2i+1) (mod 2^64), tail bytes zero-padded */
int nxec_checksum(const void *d_src, size_t bytes, uint64_t *out, void *stream);

/* Describe the launch nxec_stripes_mul would use (kernel variant, LDS
 * replication, block/grid) -- for benchmarks and logs. */
int nxec_describe_launch(nxec_ctx_t *ctx, int rows, int k, int64_t len, int64_t nstripes, char *buf, int buf_len);

/* ---- NUMA placement (SURVEY §8e on a 2-socket host): the CPUs of the node a
 * GPU's PCIe root sits on, read from sysfs (<NXEC_SYSFS_ROOT>/sys/bus/pci/
 * devices/<bus id>/numa_node and /sys/devices/system/node/node<N>/cpulist).
 * Binding restricts the CALLING THREAD (and the threads it creates later, e.g.
 * the host worker pool) to that node's CPUs within its current affinity; the
 * node is -1 and nothing changes when sysfs does not know it.  Group device
 * threads bind themselves (nxec_group_*). */
int nxec_pci_numa_node(const char *bus_id, int *node);
int nxec_numa_node_cpus(int node, int *cpus, int max, int *count);
int nxec_bind_thread_to_pci(const char *bus_id, int *node);
int nxec_device_numa_node(int device, int *node);
int nxec_bind_thread_to_device(int device, int *node);

/* ---------------------------------------------------------------------------
 * 6. Pinned host arena for chunk buffers (Chunk::allocateData, reference
 *    chunk.hh:55-66).  Blocks are pinned and device-mapped and recycled by
 *    size class (nxec_host_arena_trim returns free ones to the OS); the arena
 *    is bounded by NXEC_HOST_ARENA_MAX bytes (default: an eighth of physical
 *    memory, at most 16 GiB; 0 disables).  nxec_encode_host
 *    (RSCode::encode, CodingUtils::encode) hands arena buffers to the GPU
 *    without a staging copy.  nxec_host_alloc fails (NXEC_ERR_NOMEM /
 *    NXEC_ERR_NODEV) when the arena is full or no device is usable: the
 *    caller then uses ordinary memory.  Page-aligned.  Thread-safe.
 * ------------------------------------------------------------------------- */
int nxec_host_alloc(size_t bytes, void **p);
/* returns the block to its free list; NXEC_ERR_INVALID if p is not an arena block */
int nxec_host_free(void *p);
/* 1 if p is the start of an arena block, else 0 */
int nxec_host_arena_owns(const void *p);
int nxec_host_arena_stats(size_t *pinned_bytes, size_t *in_use_bytes);
/* the arena's bound in bytes */
size_t nxec_host_arena_cap(void);
/* unpins free blocks (largest first) until at most keep_bytes stay pinned */
int nxec_host_arena_trim(size_t keep_bytes);
/* 1 if the whole host range [p, p + bytes) is pinned / registered memory of
 * one device mapping -- the test the host entry points apply before letting a
 * kernel read or write a buffer over PCIe (zero copy) -- else 0 */
int nxec_host_range_mapped(const void *p, size_t bytes);

/* ---------------------------------------------------------------------------
 * 6b. Digests computed by a coding pass, for Chunk::computeMD5 (reference
 *     chunk.hh:136-143).  The reference hashes the chunks it has just coded
 *     right after the coding call on the same thread (chunk_manager.cc:99 ->
 *     :175, :1141 -> :1173, agent.cc:339 -> :342); RSCode::encode (every
 *     chunk, marked on the Chunk itself) and RSCode::decode(isRepair) (the
 *     repaired regions) hash them in the same GPU kernel instead, and the
 *     regions' digests wait here, per calling thread, keyed by (pointer,
 *     length), together with a 64-bit fingerprint of the bytes: a take is a hit
 *     only on the noting thread, for the same length, and while the bytes
 *     still have that fingerprint (a buffer freed with plain free() and handed
 *     out again, or rewritten, is hashed afresh).  Each coding call clears the
 *     thread's entries first (nxec_digest_clear), a thread's entries go when
 *     it exits; an entry is taken once; nxec_digest_forget (any thread;
 *     Chunk::release calls it) drops the buffer's entry.  The marks
 *     RSCode::encode leaves on Chunks hold only on the marking thread and
 *     while its digest epoch is unchanged: Chunk::allocateData and every freed
 *     Chunk buffer move it on, to a value no thread has held before.
 *     nxec_chunk_md5_mode: NXEC_CHUNK_MD5 = 0 (never; computeMD5 hashes on the
 *     host), 1 (default: RSCode::encode, whose n digests per stripe the GPU
 *     finishes sooner than one host thread hashing them in turn), 2 (also the
 *     repaired chunks of RSCode::decode(isRepair) and the outputs of
 *     CodingUtils::encode -- the agent's RPR_CHUNK_REQ hashes them,
 *     agent.cc:342, its ENC_CHUNK_REQ does not, container_manager.cc:251;
 *     one to four chunks per call, so a GPU hash chain (~10 ms per MiB on one
 *     lane) only pays with many concurrent callers).
 * ------------------------------------------------------------------------- */
int nxec_chunk_md5_mode(void);
void nxec_digest_clear(void);
int nxec_digest_note(const void *p, int64_t len, const unsigned char *md5);
/* 1 and the digest in md5[16] if (p, len) was noted on this thread (the entry is removed), else 0 */
int nxec_digest_take(const void *p, int64_t len, unsigned char *md5);
void nxec_digest_forget(const void *p);
/* the calling thread's digest epoch, and moving it on */
uint64_t nxec_digest_epoch(void);
void nxec_digest_epoch_bump(void);

/* ---------------------------------------------------------------------------
 * 7. Recovery and testing hooks.
 * ------------------------------------------------------------------------- */
/* Zero every work-queue slot of the calling thread's current device
 * (synchronous).  Failed launches reset their own slot; this is for recovery
 * after a device error left launches unfinished. */
int nxec_reset_work_queues(void);
/* Testing only: store `next_tile` in the tile counter of the slot the next
 * coding launch will draw (simulates a launch that died mid-flight). */
int nxec_debug_poison_next_queue_slot(uint32_t next_tile);

/* ---------------------------------------------------------------------------
 * 8. Storage-class / proxy INI files, for hosts that drive the coding path
 *    without the reference's Config singleton (its sample/storage_class.ini
 *    and proxy.ini).  Same reading as Config (src/common/config.cc):
 *    classes in file order with exactly one `default = 1` (:267-282), coding
 *    "rs" case-insensitively (:664-670, :1286-1291), n / k / f -1 when absent
 *    and values <= 0 read as 0, max_chunk_size 0 when absent and clamped to
 *    [0, 2^30] (:672-705); misc.repair_using_car of proxy.ini (:320).
 * ------------------------------------------------------------------------- */
#define NXEC_CODING_RS 0      /* CodingScheme::RS (define.hh:47-50) */
#define NXEC_CODING_UNKNOWN 1 /* CodingScheme::UNKNOWN_CODE */
typedef struct nxec_storage_class {
  char name[64];
  int coding;
  int n, k, f;
  int64_t max_chunk_size;
  int is_default;
} nxec_storage_class;
/* Classes of the file in file order into out[0 .. min(*count, max)); *count =
 * number of classes (out may be NULL when max is 0: a sizing call).  NXEC_ERR_INVALID on an unreadable or malformed file,
 * a class without a boolean `default`, or two default classes. */
int nxec_storage_classes_load(const char *path, nxec_storage_class *out, int max, int *count);
/* misc.repair_using_car of a proxy.ini (0 / 1 / true / false) into *car. */
int nxec_proxy_repair_using_car(const char *path, int *car);

/* ---------------------------------------------------------------------------
 * 9. C++ surface ABI tripwire.  libnxec compiles RSCode, CodingOptions and
 *    the Chunk / DecodingPlan / ByteBuffer code it runs against
 *    the headers in nexoedge_amd/csrc/coding; a caller (the overlaid Nexoedge tree,
 *    tools/overlay_reference.sh) compiles the inline half of the same types
 *    against whatever headers its include graph reaches.  RSCode's public
 *    one-argument constructor is inline (rs.hh): it records the caller's
 *    sizes and offsets here and hands them to the exported constructor, which
 *    throws std::invalid_argument on any difference, so CodingGenerator::
 *    genCoding returns NULL instead of two layouts sharing one object
 *    (reference coding_generator.hh:19-22 catches it the same way).  A TU
 *    compiled against the reference's own rs.hh does not link at all: libnxec
 *    exports no RSCode::RSCode(CodingOptions).
 * ------------------------------------------------------------------------- */
#define NXEC_CXX_ABI_VERSION 1u
typedef struct nxec_cxx_abi {
  uint32_t version; /* NXEC_CXX_ABI_VERSION of the header the caller saw */
  uint32_t size_chunk, align_chunk;
  uint32_t off_chunk_uuid, off_chunk_id, off_chunk_data, off_chunk_size, off_chunk_free, off_chunk_md5,
      off_chunk_digest;
  uint32_t size_uuid;
  uint32_t size_coding_options;
  uint32_t size_byte_buffer;
  uint32_t size_decoding_plan;
  uint32_t size_rscode;
} nxec_cxx_abi;
/* NXEC_OK when *caller equals libnxec's own layout, else NXEC_ERR_INVALID with
 * the first differing field in nxec_last_error(). */
int nxec_cxx_abi_check(const nxec_cxx_abi *caller);
/* libnxec's own layout (what nxec_cxx_abi_check compares against) */
void nxec_cxx_abi_self(nxec_cxx_abi *out);

#ifdef __cplusplus
}
#endif
#endif /* NXEC_H */
