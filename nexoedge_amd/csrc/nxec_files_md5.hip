// The multi-file write in one launch: k_files_md5 (nxec_encode_objects,
// the per-file loop of Proxy::writeFileStripes, proxy_file_ops.cc:557-666,
// with writeFileStripe's encode + Chunk::computeMD5 of all n chunks,
// chunk_manager.cc:66-452), its slot planner and launcher.  The code / hash
// wave split and the device helpers are k_mul_md5's (nxec_encode_md5.hip,
// nxec_em_common.h); this file is its own translation unit so the two build
// in parallel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <functional>
#include <utility>
#include <vector>

#include "nxec_em_common.h"

namespace nxec {

namespace {

// k_files_md5 reads HBM (a step of ~2 us is many load latencies): up to 4
// steps in flight as k_mul_md5, as the 64-bit source pointers leave room (4
// through k = 11, 3 through 14, then 2); the masked-chunk state costs one
// step from k = 11 and two from k = 13 (the deepest ring without spills;
// 3 and 4 steps measured the same at k = 10, profiles/r05_files_fold_ab.log)
#ifndef NXEC_FM_MASK_DEPTH
#define NXEC_FM_MASK_DEPTH 0  // design A/B: separate builds with -DNXEC_FM_MASK_DEPTH=D (0: by k)
#endif
template <int K, bool MASK>
constexpr int fm_depth() {
  constexpr int cap = !MASK ? 4 : NXEC_FM_MASK_DEPTH ? NXEC_FM_MASK_DEPTH : K <= 10 ? 4 : K <= 12 ? 3 : 2;
  return gm_depth<K>() > cap ? cap : gm_depth<K>();
}

// The multi-file write in one launch (nxec_encode_objects; the per-file
// loop of Proxy::writeFileStripes, proxy_file_ops.cc:557-666, with
// writeFileStripe's encode + Chunk::computeMD5 of all n chunks,
// chunk_manager.cc:66-452): k_mul_md5's code/hash split over pointer tables,
// every request (a full stripe, or a file's last stripe, read in place from
// its object) with its own chunk length.
//
// Requests are packed into slots (plan_files_slots): a slot is one stripe's
// worth of lanes -- 16 code lanes, k + p hash lanes -- that runs its requests
// back to back.  A batch of 6 000 requests on 256 CUs x 16 slots used to need
// a second wave of workgroups (18.8 ms for 4096 files of 1 B - 20 MiB); with
// the requests spread so that every slot's chains add up to about the
// longest one, it runs in one wave.  Per lane, a cursor (request of the
// slot's list, step inside it) replaces the fixed request: the load cursor
// runs D - 1 steps ahead of the compute cursor through the register ring,
// and at a request boundary a lane takes the next request's pointers from
// the workgroup's request table in LDS (no global load in the loop, so the
// ring's vmcnt bookkeeping is unchanged).  A hash lane finishes its chunk's
// digest at the request's last step (RFC 1321 padding built in registers,
// bytes past the chunk's end masked off) and starts the next chain at once.
// A lane past its request's end in that request's last step re-reads its
// last in-bounds vector, stores to scratch and leaves its LDS row alone.
//
// A last stripe (chunk_manager.cc:390-399) is an ordinary request whose data
// chunks are read where they lie in the object; the host points the chunks
// past the data at an all-zero line.  MASK: a request may name one data
// chunk jm that holds the object's last bytes (vm of them, fewer than the
// chunk length): the lane's vectors of that chunk are read in place while
// they lie inside the data, the one vector that straddles the end is rebuilt
// from the aligned 16-byte blocks holding its bytes (never a page past the
// object's last byte) and zero padded, and from there on the chunk reads the
// zero line -- no pad copy before the launch.  Both are rare per-lane events
// at steps computed once per request (one wave-uniform test per step), so the
// step loop keeps the tail-free form.  Chunks that start off a 4-byte
// boundary (a last stripe's chunk j at j * cl) are loaded as they lie: the
// shifted-load alternatives lost.  With store mode 1
// the code lanes also write that chunk, zero padded, to its tail-arena slot
// (NXEC_OBJECTS_TAIL_INPLACE: the one chunk of a last stripe the caller
// sends from the arena).  TSTORE (whole tail arena, no flag): the code lanes
// store every data chunk j < j0 of a last stripe to its slot, bytes past the
// chunk's length zeroed.
// PROBE (design probes only, K = 10; outputs are NOT valid), as k_mul_md5's:
// bit 0 no MD5 rounds, bit 1 no table lookups, bit 2 no global loads or stores.
template <int K, int PROBE = 0, bool MASK = false, bool TSTORE = false>
__global__ __launch_bounds__(kEmBlock) void k_files_md5(const FilesMd5Args a) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int nh = K + a.p;
  const int S = a.slots_per_group;
  const int L = a.max_list;
  // request record: K sources, p outputs, digest base, length, tail slot,
  // tail geometry (cls | vm << 32), mask (jm | j0 << 8 | mode << 16)
  const int rec = K + a.p + 5;
  uint32_t *tab = reinterpret_cast<uint32_t *>(lds);
  uint8_t *buf = lds + K * 1024;
  const uint32_t buf_bytes = static_cast<uint32_t>(S * nh * kEmRow);
  uint64_t *rq = reinterpret_cast<uint64_t *>(buf + 2 * buf_bytes);  // [S][L][rec]
  build_tables<1>(a.coef, K, a.p, tab);
  const int64_t g0 = static_cast<int64_t>(blockIdx.x) * S;
  const int nS = static_cast<int>(min(static_cast<int64_t>(S), a.nslots - g0));
  for (int i = threadIdx.x; i < nS * L * rec; i += kEmBlock) {
    const int ls = i / (L * rec), li = (i / rec) % L, f = i % rec;
    const int first = a.slot_first[g0 + ls], cnt = a.slot_first[g0 + ls + 1] - first;
    uint64_t v = 0;
    if (li < cnt) {
      const int64_t r = a.slot_reqs[first + li];
      if (f < K)
        v = reinterpret_cast<uint64_t>(a.src_ptrs[r * K + f]);
      else if (f < K + a.p)
        v = reinterpret_cast<uint64_t>(a.dst_ptrs[r * a.p + (f - K)]);
      else if (f == K + a.p)
        v = reinterpret_cast<uint64_t>(a.dig_ptrs[r]);
      else if (f == K + a.p + 1)
        v = static_cast<uint64_t>(a.lens[r]);
      else if (f == K + a.p + 2)
        v = a.last_slot ? a.last_slot[r] : 0;
      else if (f == K + a.p + 3)
        v = a.last_geom ? a.last_geom[r] : 0;
      else
        v = a.last_mask ? a.last_mask[r] : static_cast<uint64_t>(K | (K << 8));
    }
    rq[i] = v;
  }
  __syncthreads();
  const int nsteps = a.wg_steps[blockIdx.x];
  auto steps_of = [](int64_t len) { return static_cast<int>((len + kEncMd5Step - 1) / kEncMd5Step); };

  if (threadIdx.x < kEmCodeLanes) {
    if ((threadIdx.x & ~63) >= nS * kEmVecs) {  // no live slot in this wave: barriers only
      for (int s = 0; s < nsteps; s++) lds_barrier();
      return;
    }
    const int item = threadIdx.x;
    const bool act = item < nS * kEmVecs;
    const int ls = act ? item / kEmVecs : 0, v = item % kEmVecs;
    const int cnt = act ? a.slot_first[g0 + ls + 1] - a.slot_first[g0 + ls] : 1;
    const uint64_t *q = rq + static_cast<int64_t>(ls) * L * rec;
    auto len_of = [&](int li) { return act ? static_cast<int64_t>(q[li * rec + K + a.p + 1]) : int64_t(16); };
    // last step with bytes of this lane's 16-byte column (-1: none)
    auto tmax_of = [&](int64_t len) {
      const int64_t vlen = (len + 15) / 16 * 16;
      return vlen > v * 16 ? static_cast<int>((vlen - 1 - v * 16) / kEncMd5Step) : -1;
    };
    // load cursor: request lr of the slot, step lt of it
    int lr = 0, lt = 0;
    int64_t len0 = len_of(0);
    int lT = steps_of(len0), ltcl = max(tmax_of(len0), 0);
    const uint8_t *sp[K];
    // MASK: the load cursor's masked chunk (K: none) and the step at which
    // this lane's vector of it reaches the object's end (-1: none)
    int lj = K, lev = -1;
    // source pointers of the lane's column: a request's chunks, or -- a lane
    // whose column holds no byte of the request (chunks under 256 bytes) --
    // the scratch line: nothing past a chunk's 16-byte padding is read
    auto set_src = [&](int li, bool has) {
#pragma unroll
      for (int j = 0; j < K; j++)
        sp[j] = act && has ? reinterpret_cast<const uint8_t *>(q[li * rec + j]) + v * 16 : a.scratch + v * 16;
      if (MASK) {
        lj = act && has ? static_cast<int>(q[li * rec + K + a.p + 4] & 0xff) : K;
        lev = -1;
        if (lj < K) {  // the first step whose load would reach past the object's last byte
          const int32_t u = static_cast<int32_t>(q[li * rec + K + a.p + 3] >> 32) - v * 16 - 16;
          const int e = u < 0 ? 0 : u / kEncMd5Step + 1;
          lev = e <= ltcl ? e : -1;  // past ltcl the lane re-reads its last (in-object) vector
        }
      }
    };
    set_src(0, tmax_of(len0) >= 0);
    auto load = [&](u32x4(&d)[K]) {
      const int64_t off = static_cast<int64_t>(min(lt, ltcl)) * kEncMd5Step;
      if (MASK) {
        // this lane's vector of chunk lj reaches the object's end: from this
        // step on the chunk reads the zero line (the vector across the end
        // gets its bytes from the compute step).  A rare, wave-uniform branch:
        // the step's loads below stay the plain kernel's.
        const bool ev = lt == lev;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(ev) != 0, 0)) {
          if (ev) {
#pragma unroll
            for (int j = 0; j < K; j++)
              if (j == lj) sp[j] = a.zero + v * 16;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < K; j++) {
        const uint8_t *pj = sp[j] + off;
        // plain (cached) loads: a chunk that is not 128-byte aligned (an
        // object at any 16-byte offset, a last stripe at any byte) shares its
        // boundary lines between consecutive steps; streaming loads fetched
        // them once per step
        if (PROBE & 4)  // no HBM traffic: a value the compiler cannot fold
          d[j] = u32x4{static_cast<uint32_t>(reinterpret_cast<uintptr_t>(pj)), static_cast<uint32_t>(lt),
                       static_cast<uint32_t>(j), static_cast<uint32_t>(v)};
        else if (a.cached_loads)
          d[j] = dev::ld_global(pj);
        else
          d[j] = dev::ld_global_stream(pj);
      }
      if (++lt == lT) {
        if (lr + 1 < cnt) {  // next request of the slot (pointers from the LDS table)
          lr++;
          lt = 0;
          const int64_t ln = len_of(lr);
          lT = steps_of(ln);
          ltcl = max(tmax_of(ln), 0);
          set_src(lr, tmax_of(ln) >= 0);
        } else {  // past the slot's end: re-read the scratch line
          lt = lT - 1;
          ltcl = 0;
          set_src(lr, false);
        }
      }
    };
    // compute cursor
    int cr = 0, ct = 0, cT = lT, ctmax = act ? tmax_of(len0) : -1;
    bool live = act;
    uint8_t *dp[kMaxRowsPerPass];
    auto set_dst = [&](int li) {
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++)
        dp[r] = act && r < a.p ? reinterpret_cast<uint8_t *>(q[li * rec + K + r]) + v * 16 : a.scratch;
    };
    set_dst(0);
    uint8_t *row = buf + ls * nh * kEmRow + v * 16;
    // tail-arena stores of the compute request: slot of its chunk 0 (nullptr:
    // none), chunk stride, chunks stored whole (TSTORE: j < sj0), the chunk
    // stored zero padded (mode 1: sjm), chunk length
    uint8_t *std_ = nullptr;
    int64_t scls = 0;
    int32_t sj0 = 0, sjm = -1, scl = 0;
    // MASK: the compute request's masked chunk (K: none), its bytes in the
    // object and the step whose vector of this lane straddles its end (-1: none)
    int cj = K, chit = -1;
    int32_t cvm = 0;
    auto set_store = [&](int li) {
      if (!TSTORE && !MASK) return;
      std_ = act ? reinterpret_cast<uint8_t *>(q[li * rec + K + a.p + 2]) : nullptr;
      scls = static_cast<int64_t>(q[li * rec + K + a.p + 3] & 0xffffffffu);
      cvm = static_cast<int32_t>(q[li * rec + K + a.p + 3] >> 32);
      const uint64_t m = q[li * rec + K + a.p + 4];
      sj0 = static_cast<int32_t>((m >> 8) & 0xff);
      cj = act ? static_cast<int>(m & 0xff) : K;
      sjm = (m >> 16) & 1 ? static_cast<int32_t>(m & 0xff) : -1;
      scl = static_cast<int32_t>(len_of(li));
      if (MASK) {
        const int32_t u = cvm - v * 16, r = u % kEncMd5Step;
        chit = cj < K && u > 0 && r > 0 && r < 16 ? u / kEncMd5Step : -1;
      }
    };
    set_store(0);
    auto run = [&](int step, u32x4(&d)[K]) {
      const bool ok = live && ct <= ctmax;
      // wave-uniform: only waves holding a last stripe store, only steps with a straddling vector patch
      const bool wst = TSTORE && __builtin_amdgcn_ballot_w64(ok && std_ != nullptr) != 0;
      uint8_t *rb = row + (step & 1) * buf_bytes;
      const int32_t pos = ct * kEncMd5Step + v * 16;
      // MASK: this lane's vector of chunk cj straddles the object's end (it was
      // loaded as zeros): its valid bytes from the 16-byte aligned blocks that
      // hold them (an aligned block with a byte of the object never crosses a
      // page past it), shifted into place, the rest zero (the reference's
      // padding, chunk_manager.cc:390-399).  Two vector loads, not a load per
      // byte: the wave waits for them once.
      if (MASK) {
        const bool hit = ok && ct == chit;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(hit) != 0, 0)) {
          u32x4 sv = u32x4{0u, 0u, 0u, 0u};
          if (hit) {
            const uintptr_t at = static_cast<uintptr_t>(q[cr * rec + cj]) + pos;
            const int nv = cvm - pos, r = static_cast<int>(at & 15), qd = r >> 2, sh = r & 3;
            const uint8_t *blk = reinterpret_cast<const uint8_t *>(at - r);
            const u32x4 lo = dev::ld_global(blk);
            const u32x4 hi = r + nv > 16 ? dev::ld_global(blk + 16) : u32x4{0u, 0u, 0u, 0u};
            const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            uint32_t y[5], o[4];
#pragma unroll
            for (int m = 0; m < 5; m++) y[m] = qd == 0 ? w[m] : qd == 1 ? w[m + 1] : qd == 2 ? w[m + 2] : w[m + 3];
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const int keep = nv - 4 * i;  // bytes of this word inside the object
              const uint32_t mask = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
              o[i] = __builtin_amdgcn_alignbyte(y[i + 1], y[i], static_cast<uint32_t>(sh)) & mask;
            }
            sv = u32x4{o[0], o[1], o[2], o[3]};
          }
#pragma unroll
          for (int j = 0; j < K; j++)
            if (hit && j == cj) d[j] = sv;
        }
      }
      uint32_t acc[16];
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = 0;
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        const int j1 = j + 1 < K ? j + 1 : j;
        u32x4 x0 = d[j], x1 = d[j1];
        if (ok) {  // past a request's end its row is left as is: the hash lanes mask it
          *reinterpret_cast<u32x4 *>(rb + j * kEmRow) = x0;
          if (j + 1 < K) *reinterpret_cast<u32x4 *>(rb + (j + 1) * kEmRow) = x1;
        }
        if (wst && ok && std_) {  // data chunks to the tail arena, zero past the chunk's end
          const int32_t nv = scl - pos;
          uint32_t m[4];
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int keep = nv - 4 * i;
            m[i] = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
          }
          if (j < sj0)
            dev::st_global_stream(std_ + j * scls + pos, u32x4{x0.x & m[0], x0.y & m[1], x0.z & m[2], x0.w & m[3]});
          if (j + 1 < K && j + 1 < sj0)
            dev::st_global_stream(std_ + (j + 1) * scls + pos, u32x4{x1.x & m[0], x1.y & m[1], x1.z & m[2], x1.w & m[3]});
        }
        if (PROBE & 2) {
          if (j == 0) acc[0] = x0.x, acc[5] = x0.y, acc[10] = x0.z, acc[15] = x0.w;
        } else {
          lookup_pair(j, j + 1 < K, x0, x1, acc);
        }
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("" : "+v"(acc[i]));
      }
      // mode 1: the masked chunk, zero padded, to its slot (read back from this
      // lane's own LDS row: LDS accesses of one wave complete in order)
      if (MASK && __builtin_amdgcn_ballot_w64(ok && sjm >= 0) != 0 && ok && sjm >= 0)
        dev::st_global_stream(std_ + sjm * scls + pos, *reinterpret_cast<const u32x4 *>(rb + sjm * kEmRow));
      uint32_t o[4][4];
      rows_of(acc, o);
      const int64_t off = static_cast<int64_t>(ct) * kEncMd5Step;
#pragma unroll
      for (int r = 0; r < kMaxRowsPerPass; r++) {
        if (r < a.p) {  // wave-uniform
          const u32x4 pv{o[r][0], o[r][1], o[r][2], o[r][3]};
          if (!(PROBE & 4)) dev::st_global_stream(ok ? dp[r] + off : a.scratch + 256 * (r + 1) + v * 16, pv);
          if (ok) *reinterpret_cast<u32x4 *>(rb + (K + r) * kEmRow) = pv;
        }
      }
      lds_barrier();
      if (live && ++ct == cT) {
        if (cr + 1 < cnt) {
          cr++;
          ct = 0;
          const int64_t ln = len_of(cr);
          cT = steps_of(ln);
          ctmax = tmax_of(ln);
          set_dst(cr);
          set_store(cr);
        } else {
          live = false;
        }
      }
    };
    constexpr int D = fm_depth<K, MASK>();
    u32x4 ring[D][K];
#pragma unroll
    for (int j = 0; j < D - 1; j++) load(ring[j]);
    int step = 0;
    for (; step + D <= nsteps; step += D) {
#pragma unroll
      for (int j = 0; j < D; j++) {
        load(ring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run(step + j, ring[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < D - 1; j++) {
      if (step + j < nsteps) {
        load(ring[(j + D - 1) % D]);
        __builtin_amdgcn_sched_barrier(0);
        run(step + j, ring[j]);
      }
    }
    return;
  }

  // ---- hash lanes: lane h = chunk c of slot ls = LDS row h; one chain per request of the slot ----
  const int h = threadIdx.x - kEmCodeLanes;
  const bool active = h < nS * nh;
  const int ls = active ? h / nh : 0, c = active ? h - (h / nh) * nh : 0;
  const int cnt = active ? a.slot_first[g0 + ls + 1] - a.slot_first[g0 + ls] : 0;
  const uint64_t *q = rq + static_cast<int64_t>(ls) * L * rec;
  int hr = 0, ht = 0;
  int64_t hlen = active ? static_cast<int64_t>(q[K + a.p + 1]) : 1;
  int hT = steps_of(hlen);
  bool live = active;
  uint32_t st[4];
  md5_init(st);
  const u32x4 *rowp = reinterpret_cast<const u32x4 *>(buf + h * kEmRow);
  auto fetch = [&](int step, uint32_t(&m)[kEncMd5Step / 4]) {
    const u32x4 *p = rowp + (step & 1) * (buf_bytes / 16);
#pragma unroll
    for (int i = 0; i < kEmVecs; i++) {
      const u32x4 x = p[i];
      m[4 * i] = x.x;
      m[4 * i + 1] = x.y;
      m[4 * i + 2] = x.z;
      m[4 * i + 3] = x.w;
    }
  };
  auto proc = [&](const uint32_t(&m)[kEncMd5Step / 4]) {
    if (!live) return;
    if (ht < hT - 1) {
      if (PROBE & 1) {
#pragma unroll
        for (int i = 0; i < kEncMd5Step / 4; i++) st[i & 3] ^= m[i];
      } else {
#pragma unroll
        for (int b = 0; b < kEncMd5Step / 64; b++) md5_block(st, m + 16 * b);
      }
      ht++;
      return;
    }
    // the request's last step: its tail bytes, then RFC 1321 §3.1-3.2 padding
    const int my_tail = static_cast<int>(hlen - static_cast<int64_t>(hT - 1) * kEncMd5Step);
    const int fb = my_tail / 64, r = my_tail % 64;
#pragma unroll
    for (int b = 0; b < kEncMd5Step / 64; b++)
      if (b < fb) md5_block(st, m + 16 * b);
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < kEncMd5Step / 64; b++)
        if (b == fb) x = m[16 * b + i];
      // keep the word's bytes below r, then the 0x80 terminator
      const int keep = r - 4 * i;  // bytes of this word inside the chunk
      const uint32_t mask = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
      w[i] = (x & mask) | (i == r / 4 ? 0x80u << (8 * (r % 4)) : 0u);
    }
    const uint64_t bits = static_cast<uint64_t>(hlen) * 8;
    if (r >= 56) {
      md5_block(st, w);
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = 0;
    }
    w[14] = static_cast<uint32_t>(bits);
    w[15] = static_cast<uint32_t>(bits >> 32);
    md5_block(st, w);
    // a global (not flat) store: the digest may be unaligned
    typedef __attribute__((address_space(1))) uint8_t g_u8;
    g_u8 *out = reinterpret_cast<g_u8 *>(q[hr * rec + K + a.p] + static_cast<uint64_t>(c) * 16);
#pragma unroll
    for (int i = 0; i < 16; i++) out[i] = static_cast<uint8_t>(st[i / 4] >> (8 * (i % 4)));
    md5_init(st);
    if (hr + 1 < cnt) {
      hr++;
      ht = 0;
      hlen = static_cast<int64_t>(q[hr * rec + K + a.p + 1]);
      hT = steps_of(hlen);
    } else {
      live = false;
    }
  };
  uint32_t m0[kEncMd5Step / 4], m1[kEncMd5Step / 4];
  lds_barrier();
  if (active) fetch(0, m0);
  int step = 1;
  for (; step + 2 <= nsteps; step += 2) {
    lds_barrier();
    if (active) fetch(step, m1);
    proc(m0);
    lds_barrier();
    if (active) fetch(step + 1, m0);
    proc(m1);
  }
  if (step < nsteps) {
    lds_barrier();
    if (active) fetch(step, m1);
    proc(m0);
    proc(m1);
  } else {
    proc(m0);
  }
}

using FmKernel = void (*)(const FilesMd5Args);
template <bool MASK, bool TSTORE, int... Ks>
constexpr std::array<FmKernel, sizeof...(Ks)> fm_table(std::integer_sequence<int, Ks...>) {
  return {{&k_files_md5<Ks + 1, 0, MASK, TSTORE>...}};
}
// [plain / masked chunks / masked chunks + whole tail arena][k - 1]
const std::array<FmKernel, kFilesMd5MaxK> kFm[3] = {
    fm_table<false, false>(std::make_integer_sequence<int, kFilesMd5MaxK>{}),
    fm_table<true, false>(std::make_integer_sequence<int, kFilesMd5MaxK>{}),
    fm_table<true, true>(std::make_integer_sequence<int, kFilesMd5MaxK>{})};
#if NXEC_DESIGN_PROBES
const FmKernel kFmProbe[8] = {&k_files_md5<10, 0>, &k_files_md5<10, 1>, &k_files_md5<10, 2>, &k_files_md5<10, 3>,
                              &k_files_md5<10, 4>, &k_files_md5<10, 5>, &k_files_md5<10, 6>, &k_files_md5<10, 7>};
#endif

}  // namespace

int prepare_files_md5() {
  for (int t = 0; t < 3 * kFilesMd5MaxK; t++) {
    const FmKernel fn = kFm[t / kFilesMd5MaxK][t % kFilesMd5MaxK];
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(fn)) != hipSuccess || fa.sharedSizeBytes != 0)
      return set_error(NXEC_ERR_HIP, "k_files_md5: static LDS present (the tables must start at LDS byte 0)");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_files_md5): %s", hipGetErrorString(e));
  }
#if NXEC_DESIGN_PROBES
  for (FmKernel fn : kFmProbe) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, kEmLds);
    if (e != hipSuccess) return set_error(NXEC_ERR_HIP, "hipFuncSetAttribute(k_files_md5 probe): %s", hipGetErrorString(e));
  }
#endif
  return NXEC_OK;
}

void plan_files_slots(const std::vector<int64_t> &lens, int k, int p, int num_cus, std::vector<int32_t> &slot_first,
                      std::vector<int32_t> &slot_reqs, std::vector<int32_t> &wg_steps, FilesMd5Args &a) {
  const int nh = k + p;
  const int64_t R = static_cast<int64_t>(lens.size());
  const int64_t Smax = std::min(kEmMaxStripes, kEmMaxRows / nh);
  const int64_t cus = std::max(num_cus, 1);
  const bool pack = tuning().files_pack;
  auto steps = [](int64_t len) { return (len + kEncMd5Step - 1) / kEncMd5Step; };
  // at most one workgroup per CU (its LDS), so 256 x Smax slots in one wave:
  // fewer requests than that get a slot each, spread over every CU first
  int64_t G, S;
  if (!pack || R <= cus * Smax) {
    G = R;
    S = std::min<int64_t>(Smax, (R + cus - 1) / cus);
  } else {
    G = cus * Smax;
    S = Smax;
  }
  S = std::max<int64_t>(S, 1);
  const int64_t lds_free = kEmLds - int64_t(k) * 1024 - 2 * S * nh * kEmRow;
  const int64_t Lmax = std::max<int64_t>(1, lds_free / (S * (k + p + 5) * 8));
  // slot of every request; loads and list lengths per slot
  std::vector<int32_t> slot_of(static_cast<size_t>(R));
  std::vector<int64_t> load(static_cast<size_t>(G), 0);
  std::vector<int32_t> cnt(static_cast<size_t>(G), 0);
  // longest request first into the least loaded slot (LPT; ties: lowest
  // slot).  The requests come longest first, so the first G of them land one
  // per empty slot in order; the rest go through a heap of (load, slot).  A
  // slot whose list fills the LDS request table takes no more; when every
  // slot is full a new one opens (a second wave of workgroups).
  const int64_t first = std::min(R, G);
  for (int64_t r = 0; r < first; r++) {
    slot_of[static_cast<size_t>(r)] = static_cast<int32_t>(r);
    load[static_cast<size_t>(r)] = steps(lens[static_cast<size_t>(r)]);
    cnt[static_cast<size_t>(r)] = 1;
  }
  if (R > G) {
    typedef std::pair<int64_t, int64_t> Item;  // (load, slot); a min-heap via std::greater
    std::vector<Item> heap;
    heap.reserve(static_cast<size_t>(G));
    for (int64_t g = 0; g < G; g++)
      if (cnt[static_cast<size_t>(g)] < Lmax) heap.push_back(Item(load[static_cast<size_t>(g)], g));
    std::make_heap(heap.begin(), heap.end(), std::greater<Item>());
    for (int64_t r = G; r < R; r++) {
      int64_t g = -1;
      if (!heap.empty()) {
        std::pop_heap(heap.begin(), heap.end(), std::greater<Item>());
        g = heap.back().second;
        heap.pop_back();
      } else {
        g = static_cast<int64_t>(load.size());
        load.push_back(0);
        cnt.push_back(0);
      }
      slot_of[static_cast<size_t>(r)] = static_cast<int32_t>(g);
      load[static_cast<size_t>(g)] += steps(lens[static_cast<size_t>(r)]);
      if (++cnt[static_cast<size_t>(g)] < Lmax) {  // full slots leave the heap for good
        heap.push_back(Item(load[static_cast<size_t>(g)], g));
        std::push_heap(heap.begin(), heap.end(), std::greater<Item>());
      }
    }
    G = static_cast<int64_t>(load.size());
  }
  // slot lists in request order (a counting sort by slot)
  slot_first.assign(static_cast<size_t>(G) + 1, 0);
  int64_t maxl = 1;
  for (int64_t g = 0; g < G; g++) {
    slot_first[static_cast<size_t>(g) + 1] = slot_first[static_cast<size_t>(g)] + cnt[static_cast<size_t>(g)];
    maxl = std::max<int64_t>(maxl, cnt[static_cast<size_t>(g)]);
  }
  slot_reqs.assign(static_cast<size_t>(R), 0);
  {
    std::vector<int32_t> fill(slot_first.begin(), slot_first.end() - 1);
    for (int64_t r = 0; r < R; r++) slot_reqs[static_cast<size_t>(fill[static_cast<size_t>(slot_of[static_cast<size_t>(r)])]++)] = static_cast<int32_t>(r);
  }
  const int64_t nwg = (G + S - 1) / S;
  wg_steps.assign(static_cast<size_t>(nwg), 0);
  for (int64_t g = 0; g < G; g++) {
    int32_t &w = wg_steps[static_cast<size_t>(g / S)];
    w = std::max<int32_t>(w, static_cast<int32_t>(load[static_cast<size_t>(g)]));
  }
  a.nslots = G;
  a.slots_per_group = static_cast<int32_t>(S);
  a.max_list = static_cast<int32_t>(maxl);
}

int launch_files_md5(const FilesMd5Args &in, int num_cus, void *stream) {
  if (in.nslots <= 0) return NXEC_OK;
  if (in.k < 1 || in.k > kFilesMd5MaxK || in.p < 1 || in.p > kMaxRowsPerPass || !in.src_ptrs || !in.dst_ptrs ||
      !in.lens || !in.dig_ptrs || !in.scratch || !in.slot_first || !in.slot_reqs || !in.wg_steps ||
      in.slots_per_group < 1 || in.max_list < 1)
    return set_error(NXEC_ERR_INVALID, "files+md5: unsupported arguments");
  FilesMd5Args a = in;
  // cached loads: FETCH x2 60.0 -> 43.6 GB per 4096-file batch (= the data bytes), same time
  a.cached_loads = tuning().files_cached_loads ? 1 : 0;
  (void)num_cus;
  const int nh = a.k + a.p;
  const int64_t S = a.slots_per_group;
  if (S * nh > kEmMaxRows || S * kEmVecs > kEmCodeLanes)
    return set_error(NXEC_ERR_INVALID, "files+md5: %lld slots of %d chunks per workgroup", static_cast<long long>(S), nh);
  const int64_t grid = (a.nslots + S - 1) / S;
  if (grid >= (int64_t(1) << 31)) return set_error(NXEC_ERR_INVALID, "files+md5: batch too large for one launch");
  const int64_t lds = int64_t(a.k) * 1024 + 2 * S * nh * kEmRow + S * a.max_list * (a.k + a.p + 5) * 8;
  if (lds > kEmLds) return set_error(NXEC_ERR_INVALID, "files+md5: request table does not fit the LDS");
  if ((a.mask || a.tail_store) && (!a.last_slot || !a.last_geom || !a.last_mask || !a.zero))
    return set_error(NXEC_ERR_INVALID, "files+md5: last-stripe tables");
  FmKernel fn = kFm[a.tail_store ? 2 : a.mask ? 1 : 0][a.k - 1];
#if NXEC_DESIGN_PROBES
  if (tuning().fm_probe >= 0 && a.k == 10 && !a.mask && !a.tail_store) fn = kFmProbe[tuning().fm_probe & 7];
#endif
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(kEmBlock), static_cast<unsigned>(lds),
                     static_cast<hipStream_t>(stream), a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NXEC_OK : set_error(NXEC_ERR_HIP, "launch k_files_md5: %s", hipGetErrorString(e));
}

}  // namespace nxec
