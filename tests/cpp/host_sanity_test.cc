// Host-side sanity driver for the sanitizer builds (make asan / ubsan / tsan,
// SURVEY §5 "race detection / sanitizers"; the reference keeps ASan flags in
// CMakeLists.txt:37-39).  Runs without a GPU against a host-only build of
// libnxec (device code not compiled, --cuda-host-only): every path here is
// host code -- GF(2^8) planning (gf_host.cpp), argument validation of every
// entry point, the CodingOptions defaults source, Chunk ownership with the
// pinned arena falling back to malloc, RSCode's host copies through the
// worker pool, all under concurrency.  Compute entry points must fail with
// NXEC_ERR_NODEV (or INVALID) and never crash, leak or race.
//
// Exit 0 iff every check passed.
#include <algorithm>
#include <atomic>
#include <functional>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "coding/coding_generator.hh"
#include "coding/coding_options.hh"
#include "coding/coding_util.hh"
#include "nxec.h"
#include "nxec_internal.h"

static std::atomic<int> g_fail{0};
#define CHECK(cond, ...)            \
  do {                              \
    if (!(cond)) {                  \
      std::printf("FAIL ");         \
      std::printf(__VA_ARGS__);     \
      std::printf("\n");            \
      g_fail++;                     \
    }                               \
  } while (0)

static void gf_and_planning() {
  for (int a = 0; a < 256; a++) {
    CHECK(nxec_gf_mul(a, 1) == a, "mul by 1");
    if (a) CHECK(nxec_gf_mul(a, nxec_gf_inv(a)) == 1, "inverse %d", a);
  }
  std::mt19937 rng(7);
  std::vector<unsigned char> enc(NXEC_MAX_N * NXEC_MAX_K), rm(NXEC_MAX_N * NXEC_MAX_K);
  for (int n = 2; n <= NXEC_MAX_N; n += (n < 24 ? 1 : 13)) {
    for (int k = 1; k <= n && k <= NXEC_MAX_K; k += (k < 20 ? 1 : 17)) {
      nxec_gen_rs_matrix(enc.data(), n, k);
      std::vector<int32_t> ids(n);
      int ni = 0, mi = 0;
      const int maxf = std::min(n - k, 4);
      for (int nf = 0; nf <= maxf; nf++) {
        std::vector<int32_t> f;
        for (int c = 0; c < n && static_cast<int>(f.size()) < nf; c++)
          if (rng() % 3 == 0 || n - c <= nf - static_cast<int>(f.size())) f.push_back(c);
        int rc = nxec_rs_plan(n, k, f.data(), nf, 1, ids.data(), &ni, &mi, rm.data());
        // the Vandermonde-derived matrix is only guaranteed invertible in ISA-L's
        // documented range; elsewhere -1 (singular) is a valid answer
        CHECK(rc == NXEC_OK || rc == NXEC_ERR_SINGULAR, "plan (%d,%d) nf=%d rc=%d", n, k, nf, rc);
        if (rc == NXEC_OK) CHECK(ni == n - nf && mi == k, "plan sizes");
      }
      std::vector<int32_t> tooMany(n - k + 1);
      for (int i = 0; i <= n - k; i++) tooMany[i] = i;
      CHECK(nxec_rs_plan(n, k, tooMany.data(), n - k + 1, 1, ids.data(), &ni, &mi, rm.data()) == NXEC_ERR_INVALID,
            "too many failures rejected (%d,%d)", n, k);
    }
  }
  // CAR grouping (chunk_manager.cc:929-986) with racks of 4
  const int n = 16, k = 12;
  std::vector<int32_t> go, gc;
  for (int c = 0; c < n; c++) {
    if (c % 4 == 0) go.push_back(static_cast<int32_t>(gc.size()));
    gc.push_back(c);
  }
  go.push_back(static_cast<int32_t>(gc.size()));
  for (int f = 0; f < n; f++) {
    std::vector<int32_t> so(go.size() + 1), sc(k);
    std::vector<unsigned char> cf(k);
    int ns = 0;
    CHECK(nxec_car_plan(n, k, f, go.data(), gc.data(), static_cast<int>(go.size()) - 1, so.data(), sc.data(),
                        cf.data(), &ns) == NXEC_OK && ns >= 1,
          "car plan f=%d", f);
  }
  int64_t a = 0, b = 0, c = 0;
  CHECK(nxec_object_layout(14, 10, 0, 1 << 20, &a, &b, &c) == NXEC_OK && a == 0, "empty object");
  CHECK(nxec_object_layout(14, 10, (int64_t(1) << 40) + 7, 1 << 20, &a, &b, &c) == NXEC_OK && a == b + 1,
        "1 TiB object");
  CHECK(nxec_object_layout(14, 10, 5, 0, &a, &b, &c) == NXEC_ERR_INVALID, "zero chunk size rejected");
}

static void argument_validation() {
  unsigned char coef[4] = {1, 2, 3, 4}, buf[64] = {0};
  const unsigned char *src[2] = {buf, buf + 16};
  unsigned char *dst[2] = {buf + 32, buf + 48};
  CHECK(nxec_encode_host(16, 0, 1, coef, src, dst) == NXEC_ERR_INVALID, "k=0");
  CHECK(nxec_encode_host(-5, 2, 1, coef, src, dst) == NXEC_ERR_INVALID, "len<0");
  CHECK(nxec_encode_host(16, 2, 1, nullptr, src, dst) == NXEC_ERR_INVALID, "null coeffs");
  CHECK(nxec_ec_encode_data_status(16, 2, 1, nullptr, src, dst) == NXEC_ERR_INVALID, "null tables");
  const int rc = nxec_encode_host(16, 2, 1, coef, src, dst);
  CHECK(rc == NXEC_ERR_NODEV || rc == NXEC_ERR_HIP, "no device -> error, got %d", rc);
  nxec_ctx_t *ctx = nullptr;
  CHECK(nxec_ctx_create(0, &ctx) != NXEC_OK && ctx == nullptr, "no context without a device");
  CHECK(nxec_stripes_mul(nullptr, 1, 2, coef, buf, nullptr, 16, 32, buf, nullptr, 16, 32, nullptr, 16, 1, nullptr) ==
            NXEC_ERR_INVALID,
        "null ctx");
  CHECK(nxec_rs_encode_stripes(nullptr, 3, 4, buf, 16, 64, 16, 1, nullptr) == NXEC_ERR_INVALID, "n<k");
  CHECK(nxec_md5_chunks(nullptr, buf, 16, 64, 2, 16, 1, buf, nullptr) == NXEC_ERR_INVALID, "md5 null ctx");
  CHECK(nxec_rs_encode_md5_stripes(nullptr, 14, 10, buf, 256, 14 * 256, 256, 1, buf, nullptr) == NXEC_ERR_INVALID,
        "encode+md5 null ctx");
  {
    const int32_t lost[1] = {0};
    CHECK(nxec_rs_recover_md5_stripes(nullptr, 14, 10, lost, 1, buf, 256, 14 * 256, 256, 1, buf, nullptr) ==
              NXEC_ERR_INVALID,
          "recover+md5 null ctx");
  }
  CHECK(nxec_agent_encode_batch(nullptr, nullptr, 1, 16, 0) == NXEC_ERR_INVALID, "agent null");
  CHECK(nxec_gather_chunks(nullptr, nullptr, 1, 16, buf, 16, nullptr) == NXEC_ERR_INVALID, "gather null");
  nxec_request_t *req = nullptr;
  CHECK(nxec_gather_chunks_async(nullptr, nullptr, 1, 16, buf, 16, nullptr, &req) == NXEC_ERR_INVALID && !req,
        "async gather null");
  CHECK(nxec_request_wait(nullptr) == NXEC_OK, "wait(NULL)");
  CHECK(nxec_host_range_mapped(buf, sizeof(buf)) == 0, "stack memory is not mapped");
  void *p = nullptr;
  const int arc = nxec_host_alloc(1 << 20, &p);
  CHECK(arc != NXEC_OK && p == nullptr, "arena without device");
  CHECK(nxec_host_free(buf) == NXEC_ERR_INVALID, "free of a foreign pointer rejected");
  CHECK(nxec_host_arena_owns(buf) == 0, "foreign pointer not owned");
}

static void surface(int tid) {
  // CodingOptions defaults source (coding_options.hh) raced by setters
  CodingOptions::setDefaults(static_cast<coding_param_t>(14), static_cast<coding_param_t>(10), tid % 2 == 0);
  for (int i = 0; i < 200; i++) {
    CodingOptions o;
    const coding_param_t n = o.getN(), k = o.getK();
    CHECK((n == 14 && k == 10) || (n == 16 && k == 12), "torn defaults %d-%d", n, k);
    if (i % 50 == 0) CodingOptions::setDefaults(16, 12, true);
  }
  CodingOptions opt(14, 10, false);
  Coding *code = CodingGenerator::genCoding(CodingScheme::RS, opt);
  CHECK(code != nullptr, "genCoding");
  CodingOptions bad(4, 6, false);
  CHECK(CodingGenerator::genCoding(CodingScheme::RS, bad) == nullptr, "bad params rejected");
  if (!code) return;
  const int cs = 65536 + tid;
  std::vector<unsigned char> data(static_cast<size_t>(10) * cs, static_cast<unsigned char>(tid));
  std::vector<Chunk> stripe;
  // the host copy of rs.cc:80 runs on the worker pool, then the GPU call fails
  CHECK(!code->encode(data.data(), static_cast<length_t>(data.size()), stripe, nullptr), "encode without device");
  DecodingPlan plan;
  for (int f = 0; f < 14; f++) {
    plan.release();
    std::vector<chunk_id_t> failed{static_cast<chunk_id_t>(f)};
    CHECK(code->preDecode(failed, plan, nullptr, true), "preDecode %d", f);
    CHECK(plan.getRepairMatrixSize() == 10, "repair matrix size");
  }
  std::vector<chunk_id_t> five{0, 1, 2, 3, 4};
  CHECK(!code->preDecode(five, plan, nullptr, true), "5 failures rejected");
  // fewer than k inputs without CAR: refused (rs.cc:133-136), nothing leaks
  std::vector<Chunk> in(3);
  for (int i = 0; i < 3; i++) {
    CHECK(in[i].allocateData(cs, true), "allocateData");
    in[i].setChunkId(i);
    std::memset(in[i].data, i, cs);
  }
  unsigned char *out = nullptr;
  length_t osz = 0;
  CHECK(!code->decode(in, &out, osz, plan, nullptr), "insufficient inputs refused");
  CHECK(out == nullptr, "no buffer on refusal");
  // Chunk ownership as in the reference: copy() is deep, move() transfers,
  // `=` is the implicit shallow copy that borrowers disown (freeData = false)
  Chunk c1;
  CHECK(c1.copy(in[0]) && c1.data != in[0].data && std::memcmp(c1.data, in[0].data, cs) == 0, "deep copy");
  Chunk c2;
  c2.move(c1);
  CHECK(c1.data == nullptr && c2.size == cs, "move");
  {
    std::vector<Chunk> v(8);
    for (int i = 0; i < 8; i++) {
      v[i] = c2;  // chunk_manager.cc:176-178
      v[i].freeData = false;
      CHECK(v[i].data == c2.data && v[i].size == c2.size, "shallow alias");
    }
  }
  CHECK(c2.data != nullptr && c2.freeData, "owner intact after its borrowers died");
  CHECK(c2.computeMD5() && c2.verifyMD5(), "md5");
  Chunk meta;  // metadata-only source: copy() must not read a NULL buffer
  meta.setChunkId(3);
  meta.size = cs;
  Chunk c3;
  CHECK(c3.copy(meta) && c3.data == nullptr && c3.size == cs && c3.chunkId == 3, "metadata-only copy");
  // a digest noted for a buffer is taken once, by (pointer, length) only, on this thread
  unsigned char dg[16], got[16];
  for (int i = 0; i < 16; i++) dg[i] = static_cast<unsigned char>(tid * 16 + i);
  nxec_digest_clear();
  CHECK(nxec_digest_note(c2.data, cs, dg) == NXEC_OK, "note");
  CHECK(nxec_digest_take(c2.data, cs - 1, got) == 0, "length must match");
  CHECK(nxec_digest_note(c2.data, cs, dg) == NXEC_OK, "note again");
  CHECK(nxec_digest_take(c2.data, cs, got) == 1 && std::memcmp(got, dg, 16) == 0, "take");
  CHECK(nxec_digest_take(c2.data, cs, got) == 0, "taken once");
  CHECK(nxec_digest_note(c2.data, cs, dg) == NXEC_OK, "note for computeMD5");
  if (nxec_chunk_md5_mode() > 0) {
    CHECK(c2.computeMD5() && std::memcmp(c2.md5, dg, 16) == 0, "computeMD5 returns the noted digest");
    CHECK(c2.computeMD5() && c2.verifyMD5(), "then hashes again");
  }
  CHECK(nxec_digest_note(c2.data, cs, dg) == NXEC_OK, "note before release");
  unsigned char *gone = c2.data;
  c2.release();  // frees the buffer and forgets its digest
  CHECK(nxec_digest_take(gone, cs, got) == 0, "forgotten on release");
  delete code;
}

// the INI reader of include/nxec.h §8 (Config's reading of the sample files)
static std::string write_tmp(const char *text) {
  char path[] = "/tmp/nxec_ini_XXXXXX";
  const int fd = mkstemp(path);
  if (fd < 0) return std::string();
  const ssize_t w = write(fd, text, std::strlen(text));
  close(fd);
  return w == static_cast<ssize_t>(std::strlen(text)) ? std::string(path) : std::string();
}

static void ini_files() {
  const std::string sc = write_tmp(
      "[standard]\n; comment\ndefault = 1\ncoding = rs\nn = 4\nk = 2\nf = 1\nmax_chunk_size = 4194304\n\n"
      "[wide]\n# other comment\n  default=0\ncoding = RS\nn = 14\nk = 10\nf = 99999999999\nmax_chunk_size = 2000000000\n"
      "[odd]\ndefault = false\ncoding = lrc\nn = -3\n");
  nxec_storage_class c[4];
  int count = 0;
  CHECK(nxec_storage_classes_load(sc.c_str(), c, 4, &count) == NXEC_OK && count == 3, "three classes");
  CHECK(std::strcmp(c[0].name, "standard") == 0 && c[0].is_default && c[0].coding == NXEC_CODING_RS && c[0].n == 4 &&
            c[0].k == 2 && c[0].f == 1 && c[0].max_chunk_size == 4194304,
        "sample class");
  CHECK(!c[1].is_default && c[1].coding == NXEC_CODING_RS && c[1].n == 14 && c[1].f == -1 &&
            c[1].max_chunk_size == (int64_t(1) << 30),
        "clamped max_chunk_size, out-of-int f falls back to its default");
  CHECK(c[2].coding == NXEC_CODING_UNKNOWN && c[2].n == 0 && c[2].k == -1, "unknown coding, n <= 0 reads 0");
  CHECK(nxec_storage_classes_load(sc.c_str(), nullptr, 0, &count) == NXEC_OK && count == 3, "sizing call");
  const std::string two = write_tmp("[a]\ndefault = 1\n[b]\ndefault = 1\n");
  CHECK(nxec_storage_classes_load(two.c_str(), c, 4, &count) == NXEC_ERR_INVALID, "two defaults rejected");
  const std::string bad = write_tmp("[a]\ndefault = 1\njunk line\n");
  CHECK(nxec_storage_classes_load(bad.c_str(), c, 4, &count) == NXEC_ERR_INVALID, "malformed line rejected");
  const std::string dup = write_tmp("[a]\ndefault = 1\nn = 1\nn = 2\n");
  CHECK(nxec_storage_classes_load(dup.c_str(), c, 4, &count) == NXEC_ERR_INVALID, "duplicate key rejected");
  CHECK(nxec_storage_classes_load("/nonexistent/storage_class.ini", c, 4, &count) == NXEC_ERR_INVALID, "missing file");
  const std::string px = write_tmp("[proxy]\nnum_proxy = 1\n[misc]\nrepair_at_proxy = 1\nrepair_using_car = 1\n");
  int car = 0;
  CHECK(nxec_proxy_repair_using_car(px.c_str(), &car) == NXEC_OK && car == 1, "CAR flag");
  CHECK(CodingOptions::loadDefaults(sc.c_str(), px.c_str()) && CodingOptions::defaults().n == 4 &&
            CodingOptions::defaults().k == 2 && CodingOptions::defaults().repairUsingCAR,
        "defaults from the default class");
  CHECK(CodingOptions::loadDefaults(sc.c_str(), nullptr, "wide") && CodingOptions().getN() == 14 &&
            CodingOptions().getK() == 10 && !CodingOptions().repairUsingCAR(),
        "defaults from a named class");
  CHECK(!CodingOptions::loadDefaults(sc.c_str(), nullptr, "odd") && CodingOptions().getN() == 14, "invalid n kept old");
  CodingOptions::setDefaults(0, 0, false);
  for (const std::string &f : {sc, two, bad, dup, px}) unlink(f.c_str());
}

// the digest pool of nxec_encode_host_md5 (nxec_digest_place.cpp) from many
// threads: placed on the host, each call queues its inputs' digests, then the
// coding fails (no device here) and the call drains its own digests before it
// returns the error -- the queue, the helping callers and the pool threads
// under ASan / UBSan / TSan
static void digest_pool(int t) {
  const int cs = 70000 + t, k = 4;
  std::vector<std::vector<unsigned char>> d(k, std::vector<unsigned char>(cs, static_cast<unsigned char>(t)));
  std::vector<const unsigned char *> dp(k);
  for (int j = 0; j < k; j++) dp[j] = d[j].data();
  std::vector<unsigned char> out(cs), md_in(16 * k), md_out(16);
  unsigned char *op = out.data();
  const unsigned char coef[4] = {1, 1, 1, 1};
  for (int it = 0; it < 20; it++) {
    const int rc = nxec_encode_host_md5(cs, k, 1, coef, dp.data(), &op, md_in.data(), md_out.data());
    CHECK(rc == NXEC_OK || rc == NXEC_ERR_NODEV || rc == NXEC_ERR_HIP, "host-placed call returns");
  }
}

// The multi-file write's slot plan (nxec::plan_files_slots, host code of
// nxec_encode_objects): random batches, lengths descending as the runtime
// passes them.  Every request in exactly one slot, lists in request order,
// per-workgroup step counts = the longest slot of the group, the LDS request
// table fits, one request per slot while they fit one workgroup wave, and --
// greedy least-loaded placement -- the longest slot within the longest
// request of the average.
static void files_slot_plan() {
  std::mt19937_64 rng(20261017);
  int bound_checked = 0;
  for (int trial = 0; trial < 300; trial++) {
    const int k = 1 + static_cast<int>(rng() % nxec::kFilesMd5MaxK), p = 1 + static_cast<int>(rng() % 4);
    const int cus = trial % 3 == 0 ? 256 : 8 + static_cast<int>(rng() % 249);
    const int R = 1 + static_cast<int>(rng() % (trial % 4 == 0 ? 9000 : 600));
    const int64_t M = int64_t(1) << (12 + rng() % 9);  // 4 KiB .. 1 MiB chunks
    std::vector<int64_t> lens(static_cast<size_t>(R));
    for (auto &l : lens) l = rng() % 3 == 0 ? M : 1 + static_cast<int64_t>(rng() % static_cast<uint64_t>(M));
    std::sort(lens.begin(), lens.end(), std::greater<int64_t>());
    std::vector<int32_t> first, reqs, wg;
    nxec::FilesMd5Args a;
    std::memset(&a, 0, sizeof(a));
    nxec::plan_files_slots(lens, k, p, cus, first, reqs, wg, a);
    const int64_t G = a.nslots, S = a.slots_per_group, nh = k + p;
    CHECK(G >= 1 && S >= 1 && S <= 16 && S * nh <= 256, "plan %d: slots %lld, per group %lld", trial,
          static_cast<long long>(G), static_cast<long long>(S));
    CHECK(static_cast<int64_t>(first.size()) == G + 1 && first[0] == 0 && first.back() == R, "plan %d: slot_first",
          trial);
    std::vector<int> seen(static_cast<size_t>(R), 0);
    std::vector<int64_t> load(static_cast<size_t>(G), 0);
    int maxl = 0;
    int64_t total = 0, longest_req = 0;
    for (int64_t g = 0; g < G; g++) {
      CHECK(first[g + 1] >= first[g], "plan %d: slot %lld list", trial, static_cast<long long>(g));
      maxl = std::max(maxl, first[g + 1] - first[g]);
      for (int i = first[g]; i < first[g + 1]; i++) {
        const int r = reqs[static_cast<size_t>(i)];
        CHECK(r >= 0 && r < R, "plan %d: request %d", trial, r);
        if (r < 0 || r >= R) continue;
        seen[static_cast<size_t>(r)]++;
        if (i > first[g]) CHECK(reqs[static_cast<size_t>(i - 1)] < r, "plan %d: slot list order", trial);
        const int64_t st = (lens[static_cast<size_t>(r)] + nxec::kEncMd5Step - 1) / nxec::kEncMd5Step;
        load[static_cast<size_t>(g)] += st;
        total += st;
        longest_req = std::max(longest_req, st);
      }
    }
    for (int r = 0; r < R; r++) CHECK(seen[static_cast<size_t>(r)] == 1, "plan %d: request %d placed %d times", trial, r,
                                      seen[static_cast<size_t>(r)]);
    CHECK(a.max_list == maxl, "plan %d: max_list %d vs %d", trial, a.max_list, maxl);
    const int64_t lds = int64_t(k) * 1024 + 2 * S * nh * (nxec::kEncMd5Step + 16) + S * a.max_list * (k + p + 4) * 8;
    CHECK(lds <= 160 * 1024, "plan %d: LDS %lld", trial, static_cast<long long>(lds));
    const int64_t nwg = (G + S - 1) / S;
    CHECK(static_cast<int64_t>(wg.size()) == nwg, "plan %d: workgroups", trial);
    for (int64_t b = 0; b < nwg && static_cast<int64_t>(wg.size()) == nwg; b++) {
      int64_t w = 0;
      for (int64_t g = b * S; g < std::min(G, (b + 1) * S); g++) w = std::max(w, load[static_cast<size_t>(g)]);
      CHECK(wg[static_cast<size_t>(b)] == w, "plan %d: workgroup %lld steps", trial, static_cast<long long>(b));
    }
    const int64_t smax = std::min<int64_t>(16, 256 / nh);
    if (R <= int64_t(cus) * smax) CHECK(G == R, "plan %d: %d requests in %lld slots", trial, R, static_cast<long long>(G));
    if (G == int64_t(cus) * smax && R > G) {  // one wave, lists under the LDS cap: list scheduling bound
      const int64_t mx = *std::max_element(load.begin(), load.end());
      bound_checked++;
      CHECK(mx <= (total + G - 1) / G + longest_req, "plan %d: longest slot %lld, average %lld, longest request %lld",
            trial, static_cast<long long>(mx), static_cast<long long>(total / G), static_cast<long long>(longest_req));
    }
  }
  std::printf("files slot plans: 300 checked, %d against the list-scheduling bound\n", bound_checked);
}

// The default pool of the drop-in (nxec_context.cpp): reconfigured, queried
// and leased from many threads at once.  Without a device every lease fails
// with NXEC_ERR_NODEV (in list mode after picking a member); the sanitizers
// check the pool's locks, counters and the lease's release on that path.
static void default_pool(int t) {
  const unsigned char coef[2] = {1, 1};
  unsigned char a[64] = {0}, b[64] = {0}, out[64];
  const unsigned char *src[2] = {a, b};
  unsigned char *dst[1] = {out};
  const int lists[3][3] = {{0, 0, 0}, {0, 1, 0}, {2, 2, 2}};
  for (int it = 0; it < 200; it++) {
    if ((it + t) % 50 == 0) CHECK(nxec_default_devices(lists[(it + t) % 3], 1 + (it + t) % 3) == NXEC_OK, "configure");
    if ((it + t) % 97 == 0) CHECK(nxec_default_devices(nullptr, (it % 2) ? -1 : 0) == NXEC_OK, "configure all/current");
    const int rc = nxec_encode_host(64, 2, 1, coef, src, dst);
    CHECK(rc == NXEC_ERR_NODEV || rc == NXEC_ERR_HIP, "no device: the lease fails cleanly (%d)", rc);
    int dv[8], nd[8], inf[8], cnt = 0;
    unsigned long long calls[8];
    CHECK(nxec_default_pool_stats(dv, nd, calls, inf, 8, &cnt) == NXEC_OK, "stats");
    const int in[4] = {it % 3, 1, 0, 2}, nodes[4] = {0, 0, 1, 1};
    const int pick = nxec_default_pick(4, in, nodes, t % 2, it % 4);
    CHECK(pick >= 0 && pick < 4, "pick in range");
  }
}

int main() {
  gf_and_planning();
  files_slot_plan();
  argument_validation();
  ini_files();
  std::vector<std::thread> th;
  for (int t = 0; t < 8; t++) th.emplace_back(surface, t);
  for (auto &t : th) t.join();
  const int prev = nxec_set_digest_placement(NXEC_DIGEST_HOST);
  std::vector<std::thread> dt;
  for (int t = 0; t < 12; t++) dt.emplace_back(digest_pool, t);
  for (auto &t : dt) t.join();
  nxec_set_digest_placement(prev);
  std::vector<std::thread> pt;
  for (int t = 0; t < 8; t++) pt.emplace_back(default_pool, t);
  for (auto &t : pt) t.join();
  // every lease released: nothing left in flight
  {
    int dv[16], nd[16], inf[16], cnt = 0;
    unsigned long long calls[16];
    CHECK(nxec_default_pool_stats(dv, nd, calls, inf, 16, &cnt) == NXEC_OK, "final stats");
    for (int i = 0; i < cnt && i < 16; i++) CHECK(inf[i] == 0, "member %d still has %d calls in flight", i, inf[i]);
  }
  std::printf("%s %d failures\n", g_fail ? "FAILED" : "PASSED", g_fail.load());
  return g_fail ? 1 : 0;
}
