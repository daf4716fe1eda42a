// Internal declarations shared by the host runtime and the HIP kernels of libnxec.
#ifndef NXEC_INTERNAL_H
#define NXEC_INTERNAL_H

#include <cstdint>
#include <functional>
#include <vector>

#include "nxec.h"
#include "nxec_tuning.h"

namespace nxec {

// Runs fn(i) for i in [0, n) on the library's host worker pool (staging
// copies of the host entry points); returns when all are done.  `lane`: the
// copy's direction -- into pinned staging (kIn) or out of it (kOut); `node`:
// the NUMA node of the GPU the copies feed (its pool's threads run on that
// node's CPUs; -1: unknown, an unbound pool).
enum class HostLane { kIn, kOut };
void host_parallel_for(int n, const std::function<void(int)> &fn, HostLane lane = HostLane::kIn, int node = -1);

// Digest placement of nxec_encode_host_md5 (nxec_digest_place.cpp): true if
// the call's nhash digests of len bytes go to the host pool (their bytes are
// then reserved in its backlog), false for the GPU coding pass.
bool digest_place_host(int64_t len, int nhash);
// a GPU-placed call took `ms` end to end (feeds the placement's estimate)
void digest_gpu_observe(int64_t len, double ms);
// CLOCK_MONOTONIC in ns (the GPU-placed call's latency)
double digest_clock_ns();
// the host-placed call: GPU coding, digests on the pool and the calling thread
int encode_host_md5_host_digests(int len, int k, int rows, const unsigned char *coeffs,
                                 const unsigned char *const *data, unsigned char *const *coding,
                                 unsigned char *md5_data, unsigned char *md5_code);

// Sets the calling thread's last-error message and returns `code`.
int set_error(int code, const char *fmt, ...);
bool valid_nk(int n, int k);
int repair_rows(int n, int k, const std::vector<uint8_t> &enc, const int32_t *input_ids, const int32_t *targets,
                int ntargets, uint8_t *out);

constexpr int kMaxRowsPerPass = 4;  // one packed 32-bit LDS entry holds 4 row products
constexpr int kQueueSlots = 4096;   // per-launch tile-queue slots (device ring, see nxec_kernels.hip)
constexpr uint32_t kNoCopy = 0xFFFFFFFFu;
constexpr int64_t kHostPiece = 256 * 1024;  // column piece of the pipelined host entry points

// Kernel arguments of one GF(2^8) stripe-multiply pass (<= 4 output rows).
// Chunk (s, c) of the source lives at src + s*src_stripe_stride + c*src_chunk_stride
// (strided mode) or at src_ptrs[s*k + j] (gather mode, src_ptrs != nullptr).
struct MulArgs {
  const uint8_t *src;
  uint8_t *dst;
  const uint8_t *const *src_ptrs;
  uint8_t *const *dst_ptrs;
  int64_t src_chunk_stride, src_stripe_stride;
  int64_t dst_chunk_stride, dst_stripe_stride;
  int64_t len;         // bytes per chunk
  int64_t vec_begin;   // first 16-byte vector (per chunk) of this vector-kernel launch
  int64_t vec_count;   // 16-byte vectors per chunk handled by this vector-kernel launch
  int64_t byte_begin;  // first byte handled by the byte kernel
  int64_t nstripes;
  int32_t k, rows;
  int32_t any_copy;                 // copy_idx has entries >= 0
  int32_t dst_ptr_row0;             // gather mode: first row of this pass inside dst_ptrs[s*rows_total + r]
  int32_t dst_ptr_rows;             // gather mode: rows_total
  int32_t queue_slot;               // tile-queue slot of this launch (set by launch_mul)
  uint32_t tiles_per_grab;          // work-queue run length (set by launch_mul)
  uint32_t stripe_group;            // tiles column-major within groups of this many stripes (1 = stripe-major)
  // strided form: byte offsets of the chunks inside a stripe (idx * chunk_stride,
  // precomputed on the host; < 4 GiB so they stay single 32-bit SGPRs)
  uint32_t src_off[NXEC_MAX_K + 1];
  uint32_t dst_off[kMaxRowsPerPass];
  uint32_t copy_off[NXEC_MAX_K + 1];  // kNoCopy = none
  uint8_t coef[kMaxRowsPerPass * (NXEC_MAX_K + 1)];  // row-major rows x k
};

struct LaunchInfo {
  const char *variant;
  bool perm;        // VALU nibble-table kernel (single-row passes)
  int lds_copies;   // R: table replication factor
  int block;        // threads per workgroup
  int grid;         // workgroups
  int lds_bytes;
};

// Chooses and describes the vector-kernel launch for (k, len, nstripes).
LaunchInfo plan_launch(int k, int rows, int64_t vec_count, int64_t nstripes, int num_cus, bool full, bool copy,
                       bool gather);
// Enqueues one pass (vector kernel + byte kernel for tails / misaligned data).
int launch_mul(const MulArgs &a, bool vec_ok, int num_cus, void *stream);
// Zeroes every tile-queue slot of the current device (stream-ordered, then
// synchronised); for recovery after a device error.
int reset_work_queues(void *stream);
// Testing: stores `next_tile` in the counter of the slot the next launch draws.
int debug_poison_next_queue_slot(uint32_t next_tile);
// Raises the dynamic-LDS limit of every kernel instantiation (once per device).
int prepare_kernels();
int launch_fill(void *d, size_t bytes, uint64_t seed, void *stream);
// 16-byte-aligned copy by a kernel (dst may be device-mapped pinned host memory:
// a D2H that does not queue behind SDMA copies)
int launch_copy16(void *dst, const void *src, size_t bytes, int num_cus, void *stream);
// One MD5 launch hashes up to kMaxMd5Regions chunk sets: region r covers
// chunks (s, i), s < nstripes, i < nchunks, at base + s*stripe_stride +
// i*chunk_stride, each `len` bytes; digest at digests + s*dig_stripe_stride +
// i*16.  (A chain per chunk: one launch for everything, so its time is one
// chunk's hash, not a sum.)
constexpr int kMaxMd5Regions = 4;
struct Md5Region {
  const uint8_t *base;
  int64_t chunk_stride, stripe_stride, len, nstripes;
  uint8_t *digests;
  int64_t dig_stripe_stride;
  int nchunks;
  // verify mode (ok != nullptr): `digests` holds the expected digests; chunk
  // (s, i) writes ok[s*ok_stripe_stride + i] = match, *nbad += mismatches
  uint8_t *ok = nullptr;
  int64_t ok_stripe_stride = 0;
};
int launch_md5(const Md5Region *regions, int nregions, void *stream, unsigned long long *nbad = nullptr);
int launch_checksum(const void *d, size_t bytes, uint64_t *d_out, void *stream);

// Variable-length batch (many objects per call): stripe s has its own chunk
// length and layout.  Source chunk j at src + j*src_cs, output row r at
// dst + r*dst_cs.  prefix[s] = first 16-byte unit of stripe s (prefix[n] = total).
struct ListStripe {
  const uint8_t *src;
  uint8_t *dst;
  int64_t len, src_cs, dst_cs;
};
// rows x k coefficients (rows <= 4 per pass inside); d_stripes / d_prefix in device memory
int launch_mul_list(int rows, int k, const uint8_t *coeffs, const ListStripe *d_stripes, const int64_t *d_prefix,
                    int64_t nstripes, int64_t total_units, int num_cus, void *stream);
// Ragged stripes (aligned: src, dst, src_cs, dst_cs, len all multiples of 16)
// through the work-queue LDS-table kernel; tile t is column tile
// t - stripe_tile0[s] of stripe s = tile_stripe[t] (1024 16-byte vectors each).
constexpr int kMaxRaggedK = 19;
int launch_mul_ragged(int rows, int k, const uint8_t *coeffs, const ListStripe *d_stripes, const uint32_t *d_tile_stripe,
                      const uint32_t *d_stripe_tile0, int64_t ntiles, int num_cus, void *stream);
// Last stripe of an object into the aligned tail arena: dst + j*cls (j < k)
// receives object bytes [j*cl, (j+1)*cl) of src (zeros past rem) then zeros
// up to cls (a multiple of 16 >= cl).  Item i owns 256-thread blocks
// [bstart[i], bstart[i+1]) of kPadVecs*256 16-byte vectors (cls/16*k in all).
constexpr int kPadVecs = 8;
struct PadChunks {
  const uint8_t *src;
  uint8_t *dst;
  int64_t rem, cl, cls;
  int64_t k;
};
int launch_pad_chunks(const PadChunks *d_items, const uint32_t *d_bstart, int64_t nitems, int64_t nblocks,
                      void *stream);
// copy item i: dst[0 .. dst_len) = src[0 .. src_len) then zeros (src_len <= dst_len)
struct PadCopy {
  const uint8_t *src;
  uint8_t *dst;
  int64_t src_len, dst_len;
};
int launch_pad_copy(const PadCopy *d_items, int64_t nitems, void *stream);
// MD5 of a list of chunks: digest of p[0 .. len) to `digest`
struct Md5Item {
  const uint8_t *p;
  int64_t len;
  uint8_t *digest;
};
int launch_md5_list(const Md5Item *d_items, int64_t nitems, void *stream);

// Fused GF(2^8) multiply + MD5 (nxec_encode_md5.hip): per stripe s, output
// row r (< rows <= 4) = XOR_j coef[r][j] * source j, source j at src +
// s*src_stripe_stride + src_off[j], row r at dst + s*dst_stripe_stride +
// dst_off[r]; the MD5 of every source (hash_src) and/or every output
// (hash_dst) in the same pass, hashed chunk i (sources first) to digests +
// s*digest_stripe_stride + digest_slot[i]*16.  Chunks are walked in steps of
// kEncMd5Step bytes (len a multiple of it).  The write path (encode + MD5 of
// all n chunks) and the repair path (recover + MD5 of the rebuilt chunks).
constexpr int kEncMd5Step = 256;
constexpr int kEncMd5MaxK = 20;
struct MulMd5Args {
  const uint8_t *src;
  int64_t src_stripe_stride;
  uint8_t *dst;
  int64_t dst_stripe_stride;
  uint8_t *digests;
  int64_t digest_stripe_stride;
  int64_t len, nstripes;
  int32_t k, p;                  // sources, output rows
  int32_t hash_src, hash_dst;
  int32_t nhashed;               // set by launch_mul_md5
  int32_t stripes_per_group;     // set by launch_mul_md5
  int32_t hash_prio;             // hash waves at s_setprio 1 (set by launch_mul_md5)
  uint32_t src_off[NXEC_MAX_K + 1];
  uint32_t dst_off[kMaxRowsPerPass];
  // pass-through (full-output decode): source j also stored to dst +
  // s*dst_stripe_stride + copy_off[j] unless kNoCopy
  int32_t any_copy;
  uint32_t copy_off[NXEC_MAX_K + 1];
  uint8_t digest_slot[NXEC_MAX_K + 1 + kMaxRowsPerPass];
  uint8_t coef[kMaxRowsPerPass * (NXEC_MAX_K + 1)];  // p x k, row-major
  // verify mode (ok != nullptr): `digests` holds the expected digests; hashed
  // chunk i of stripe s writes ok[s*ok_stripe_stride + digest_slot[i]] = match
  // and counts a mismatch into *nbad (optional)
  uint8_t *ok;
  int64_t ok_stripe_stride;
  unsigned long long *nbad;
};
// k <= kEncMd5MaxK, 0 <= rows <= 4, len a positive multiple of kEncMd5Step,
// 16-byte aligned buffers, strides and offsets (NXEC_FUSED_MD5=0 disables, for A/B)
bool mul_md5_eligible(int k, int rows, int64_t len, const void *src, int64_t src_stripe_stride, const uint32_t *src_off,
                      const void *dst, int64_t dst_stripe_stride, const uint32_t *dst_off,
                      const uint32_t *copy_off = nullptr);
int prepare_encode_md5();
// k_files_md5's kernel attributes (nxec_files_md5.hip; called by prepare_encode_md5)
int prepare_files_md5();
int launch_mul_md5(const MulMd5Args &a, int num_cus, void *stream);

// The agent's form of the fused kernel (nxec_agent_encode_batch): request s
// reads source j at src_ptrs[s*k + j] and writes output r at dst_ptrs[s*p + r]
// (device addresses: HBM, or pinned host memory the kernel reads and writes
// over PCIe), the MD5 of every output to digests + (s*p + r)*16 -- with
// hash_src, of every source too: nh = k + p digests per request, chunk c
// (sources first) at digests + (s*nh + c)*16.  scratch: >=
// 2 KiB of device memory, the target of idle lanes' accesses.  Pointer tables
// and digests may be device-mapped host memory.  Any len > 0 (a partial last
// step never touches bytes past a chunk's end); every pointer 16-byte aligned.
constexpr int kGatherMd5MaxK = 16;
struct GatherMd5Args {
  const uint8_t *const *src_ptrs;
  uint8_t *const *dst_ptrs;
  uint8_t *digests;
  uint8_t *scratch;
  int64_t len, nstripes;
  int32_t k, p;
  int32_t hash_src;           // sources hashed too
  int32_t stripes_per_group;  // set by launch_gather_md5
  uint8_t coef[kMaxRowsPerPass * (NXEC_MAX_K + 1)];  // p x k, row-major
};
int launch_gather_md5(const GatherMd5Args &a, int num_cus, void *stream);

// The multi-file write in one launch (nxec_encode_objects): request s codes
// k sources src_ptrs[s*k + j] into p outputs dst_ptrs[s*p + r] and hashes
// all k + p chunks, lens[s] bytes each, digest of chunk c (sources first) at
// dig_ptrs[s] + c*16.  Bytes up to the next multiple of 16 past lens[s] are
// readable (except in a masked chunk, below); outputs are written up to that
// multiple.  Source pointers may be at any byte address (the objects' last
// stripes), outputs and tail slots 16-byte aligned, digests any; tables in
// device memory.
//
// Requests are packed into slots (one stripe's worth of code and hash lanes
// of a workgroup): slot g runs requests slot_reqs[slot_first[g] ..
// slot_first[g+1]) one after the other, each hash lane finishing one chunk's
// digest and starting the next chain at a request boundary, so a batch of
// more requests than the chip has slots (4096 = 256 CUs x 16) runs in one
// wave of workgroups with every slot's chains about equally long (longest
// request first into the least loaded slot; plan_files_slots).  Workgroup b
// owns slots [b*slots_per_group, ...) and runs wg_steps[b] steps of
// kEncMd5Step bytes (the longest of its slots' totals).
constexpr int kFilesMd5MaxK = 16;
struct FilesMd5Args {
  const uint8_t *const *src_ptrs;
  uint8_t *const *dst_ptrs;
  const int64_t *lens;
  uint8_t *const *dig_ptrs;
  uint8_t *scratch;  // >= 2 KiB of device memory: idle lanes' loads / stores
  const int32_t *slot_first;  // nslots + 1 entries
  const int32_t *slot_reqs;
  const int32_t *wg_steps;    // per workgroup
  int64_t nslots;
  int32_t k, p;
  int32_t slots_per_group;
  int32_t max_list;           // longest slot list (LDS request table rows per slot)
  int32_t cached_loads;       // plain loads (default); streaming with the loads probe
  uint8_t coef[kMaxRowsPerPass * (NXEC_MAX_K + 1)];  // p x k, row-major
  // Last stripes (null tables: none).  Per request s:
  //   last_slot[s]  the tail-arena slot of its data chunk 0 (0: nothing stored)
  //   last_geom[s]  cls | vm << 32: the slots' chunk stride, and the bytes of
  //                 the masked chunk that lie in the object
  //   last_mask[s]  jm | j0 << 8 | mode << 16: the masked data chunk (k:
  //                 none) -- read in place below vm, zero padded from vm, the
  //                 vector across vm rebuilt from aligned blocks --, the chunks a
  //                 whole-tail-arena call stores (j < j0), mode 1: store the
  //                 masked chunk zero padded to its slot
  const uint64_t *last_slot;
  const uint64_t *last_geom;
  const uint32_t *last_mask;
  const uint8_t *zero;  // >= max(lens) + 16 zero bytes: data chunks past a last stripe's data
  int32_t mask;         // some request has a masked chunk
  // Whole tail arena (no NXEC_OBJECTS_TAIL_INPLACE): the code lanes store a
  // last stripe's data chunks j < j0 to their slots, bytes past the chunk's
  // length zeroed
  int32_t tail_store;
};
// Slot plan for `lens` (descending): fills slot_first / slot_reqs / wg_steps
// and the args' nslots / slots_per_group / max_list.  NXEC_FILES_PACK=0 gives
// every request its own slot (one workgroup wave per 4096 requests; A/B).
void plan_files_slots(const std::vector<int64_t> &lens, int k, int p, int num_cus, std::vector<int32_t> &slot_first,
                      std::vector<int32_t> &slot_reqs, std::vector<int32_t> &wg_steps, FilesMd5Args &a);
int launch_files_md5(const FilesMd5Args &a, int num_cus, void *stream);

}  // namespace nxec

#endif
