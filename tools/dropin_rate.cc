// Drop-in rate probe: an unmodified ChunkManager calls RSCode::encode /
// RSCode::decode once per stripe from its worker threads (proxy.ini:75 = 4
// ZMQ workers; chunk_manager.cc:99 encode, :787 decode) with pageable host
// buffers.  This times exactly that through the C++ surface
// (nexoedge_amd/csrc/coding), i.e. host -> pinned staging -> GPU -> host per
// call, for 1, 4 and 16 calling threads.  Bytes per stripe as in bench.py:
// encode (k+p)*cs, 4-erasure decode (k+e)*cs.  A third leg calls
// CodingUtils::encode (coding_util.hh:12-31, the agent's entry) on
// preallocated buffers: the transport alone, without RSCode::encode's own
// per-call chunk allocation + data copy (rs.cc:72-80).  A fourth leg,
// "writeFileStripe", is the whole coding side of the proxy's write of one
// stripe with the reference's own Chunk handling: ChunkManager::encodeFile
// (RSCode::encode, then file.chunks[i].move(stripe[i]), chunk_manager.cc:
// 427-447), Chunk::computeMD5 of every chunk and the shallow event copies
// (:172-179), the events and the file torn down; GiB/s of user data (k*cs per
// stripe), the unit of bench.py cpu_baseline.write_path_with_md5.  Run it with
// NXEC_CHUNK_MD5=0 for the host-hashed (OpenSSL) form.
//
// usage: dropin_rate [cs] [seconds] [all|agent|write|pool] [threads,...]
// Build: make tools   (build/dropin_rate)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "coding/coding_generator.hh"
#include "coding/coding_util.hh"
#include "nxec.h"

static void fill(uint8_t *p, size_t n, uint64_t s) {
  for (size_t i = 0; i < n; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    p[i] = static_cast<uint8_t>(s >> 56);
  }
}

int main(int argc, char **argv) {
  const int n = 14, k = 10, e = 4;
  const int cs = argc > 1 ? std::atoi(argv[1]) : (1 << 20);
  const double secs = argc > 2 ? std::atof(argv[2]) : 2.0;
  CodingOptions opt(n, k, false);
  Coding *code = CodingGenerator::genCoding(CodingScheme::RS, opt);
  if (!code) return 1;
  // argv[3] = "agent": only the agent-service leg; "write": only the writeFileStripe leg
  const bool agent_only = argc > 3 && std::strcmp(argv[3], "agent") == 0;
  const bool write_only = argc > 3 && std::strcmp(argv[3], "write") == 0;
  // "pool": only RSCode::decode and CodingUtils::encode, then the default
  // pool's members (device, NUMA node, calls served) -- the drop-in spread
  // over every visible GPU (bench.py host_inclusive.dropin_pool)
  const bool pool_only = argc > 3 && std::strcmp(argv[3], "pool") == 0;
  std::vector<int> tlist0{1, 4, 16};
  if (argc > 4) {
    tlist0.clear();
    for (const char *p = argv[4]; *p;) {
      tlist0.push_back(std::atoi(p));
      while (*p && *p != ',') p++;
      if (*p == ',') p++;
    }
  }
  // one timed leg of path `op` with `threads` callers; prints its line, returns GiB/s
  auto leg = [&](int threads, int op, double secs, bool quiet = false) -> double {
      std::atomic<long> stripes{0};
      std::atomic<bool> ok{true};
      unsigned long long h0 = 0, g0 = 0, h1 = 0, g1 = 0;
      int dthreads = 0;
      nxec_digest_place_stats(&h0, &g0, &dthreads);
      const auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> pool;
      for (int t = 0; t < threads; t++)
        pool.emplace_back([&, t] {
          std::vector<uint8_t> data(static_cast<size_t>(k) * cs);
          fill(data.data(), data.size(), 77 + t);
          std::vector<Chunk> stripe;
          if (!code->encode(data.data(), static_cast<length_t>(data.size()), stripe, nullptr)) ok = false;
          DecodingPlan plan;
          std::vector<chunk_id_t> failed = {0, 1, 2, 3};
          if (!code->preDecode(failed, plan, nullptr)) ok = false;
          std::vector<chunk_id_t> ids = plan.getInputChunkIds();
          std::vector<Chunk> in(k);
          for (int i = 0; i < k; i++) in[i].copy(stripe[ids[i]]);
          data_t *out = static_cast<data_t *>(std::malloc(static_cast<size_t>(k) * cs));
          std::vector<uint8_t> par(static_cast<size_t>(n - k) * cs);
          const uint8_t *enc = static_cast<RSCode *>(code)->getEncodeMatrix() + k * k;
          std::vector<uint8_t> m(enc, enc + (n - k) * k);
          bool first = true;  // verify the first decode of each thread only (memcmp is not the path)
          while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
            if (op == 0) {
              std::vector<Chunk> s2;
              if (!code->encode(data.data(), static_cast<length_t>(data.size()), s2, nullptr)) ok = false;
            } else if (op == 3) {
              // ChunkManager::encodeFile (chunk_manager.cc:427-447)
              std::vector<Chunk> s2;
              if (!code->encode(data.data(), static_cast<length_t>(data.size()), s2, nullptr)) ok = false;
              Chunk *fileChunks = new Chunk[s2.size()];
              for (size_t i = 0; i < s2.size(); i++) {
                fileChunks[i].move(s2.at(i));
                fileChunks[i].setChunkId(static_cast<int>(i));
              }
              // writeFileStripe (:149-179): MD5 of each chunk, then a borrowed view per event
              Chunk *events = new Chunk[s2.size()];
              for (size_t i = 0; i < s2.size(); i++) {
                if (!fileChunks[i].computeMD5()) ok = false;
                events[i] = fileChunks[i];
                events[i].freeData = false;
              }
              if (first) {  // verify the first stripe's digests (not the path)
                for (size_t i = 0; i < s2.size(); i++)
                  if (!events[i].verifyMD5()) ok = false;
                first = false;
              }
              delete[] events;
              delete[] fileChunks;
            } else if (op == 2) {
              if (!CodingUtils::encode(data.data(), k, par.data(), n - k, cs, m.data())) ok = false;
            } else {
              length_t osz = 0;
              if (!code->decode(in, &out, osz, plan, nullptr) ||
                  (first && std::memcmp(out, data.data(), data.size()) != 0))
                ok = false;
              first = false;
            }
            stripes++;
          }
          std::free(out);
        });
      for (auto &th : pool) th.join();
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      nxec_digest_place_stats(&h1, &g1, &dthreads);
      const double bytes = static_cast<double>(stripes) * (op == 3 ? k : k + (op != 1 ? n - k : e)) * cs;
      static const char *names[4] = {"RSCode::encode", "RSCode::decode", "CodingUtils::encode", "writeFileStripe"};
      static const char *place_names[4] = {"auto", "gpu", "host", "?"};
      if (!quiet)
        std::printf("{\"path\": \"%s per stripe\", \"threads\": %d, \"chunk\": %d, \"stripes\": %ld, "
                    "\"GiB_s%s\": %.2f, \"ms_per_call\": %.3f, \"chunk_md5\": %d, \"digest_place\": \"%s\", "
                    "\"digest_calls_host\": %llu, \"digest_calls_gpu\": %llu, \"digest_threads\": %d, \"ok\": %s}\n",
                    names[op], threads, cs, static_cast<long>(stripes), op == 3 ? "_user_data" : "",
                    bytes / dt / (1 << 30), 1e3 * dt * threads / static_cast<double>(stripes), nxec_chunk_md5_mode(),
                    place_names[nxec_digest_placement() & 3], h1 - h0, g1 - g0, dthreads, ok ? "true" : "false");
      std::fflush(stdout);
      return bytes / dt / (1 << 30);
  };
  // DROPIN_PLACES=host,gpu,auto (write leg only): every placement of
  // nxec_encode_host_md5's digests in one process, DROPIN_REPS rounds in
  // rotating order after a warm-up leg (arena pinning and first-touch page
  // faults land in the warm-up, not in whichever placement runs first), and
  // per caller count the median of each plus auto / best.
  const char *places_env = std::getenv("DROPIN_PLACES");
  if (write_only && places_env) {
    std::vector<int> places;
    for (const char *p = places_env; *p;) {
      places.push_back(std::strncmp(p, "gpu", 3) == 0 ? NXEC_DIGEST_GPU
                       : std::strncmp(p, "host", 4) == 0 ? NXEC_DIGEST_HOST : NXEC_DIGEST_AUTO);
      while (*p && *p != ',') p++;
      if (*p == ',') p++;
    }
    const int reps = std::getenv("DROPIN_REPS") ? std::atoi(std::getenv("DROPIN_REPS")) : 3;
    double cpus = 0, hcallers = 0;
    nxec_digest_place_params(&cpus, &hcallers);
    nxec_set_digest_placement(NXEC_DIGEST_HOST);
    leg(tlist0.empty() ? 1 : tlist0.back(), 3, 1.0);  // warm-up
    for (int threads : tlist0) {
      std::vector<std::vector<double>> got(places.size());
      for (int r = 0; r < reps; r++)
        for (size_t i = 0; i < places.size(); i++) {
          const size_t pi = (i + r) % places.size();
          nxec_set_digest_placement(places[pi]);
          got[pi].push_back(leg(threads, 3, secs));
        }
      std::printf("{\"summary\": \"writeFileStripe per stripe, median of %d\", \"threads\": %d, "
                  "\"cpu_budget\": %.1f, \"host_callers_H\": %.1f", reps, threads, cpus, hcallers);
      double best = 0, autov = -1;
      static const char *pn[3] = {"auto", "gpu", "host"};
      for (size_t i = 0; i < places.size(); i++) {
        std::vector<double> v = got[i];
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2];
        std::printf(", \"%s_GiB_s\": %.2f", pn[places[i] & 3], med);
        if (places[i] == NXEC_DIGEST_AUTO) autov = med;
        else best = std::max(best, med);
      }
      if (autov >= 0 && best > 0) std::printf(", \"auto_over_best\": %.3f", autov / best);
      std::printf("}\n");
      std::fflush(stdout);
    }
    delete code;
    return 0;
  }
  if (pool_only) {  // warm-up: every member's staging slots and the arena pinned before timing
    int tmax = 1;
    for (int t : tlist0) tmax = std::max(tmax, t);
    leg(tmax, 2, 0.5, true);
    leg(tmax, 1, 0.5, true);
  }
  for (int threads : tlist0) {
    if (agent_only) break;
    if (pool_only) {
      leg(threads, 2, secs);
      leg(threads, 1, secs);
      continue;
    }
    for (int op = write_only ? 3 : 0; op < 4; op++)  // 0 RSCode::encode, 1 RSCode::decode, 2 CodingUtils::encode,
      leg(threads, op, secs);                        // 3 writeFileStripe (encode + MD5 of every chunk + events)
  }
  if (pool_only) {
    int dv[64], nd[64], inf[64], cnt = 0;
    unsigned long long served[64];
    nxec_default_pool_stats(dv, nd, served, inf, 64, &cnt);
    std::printf("{\"pool_members\": [");
    for (int i = 0; i < cnt && i < 64; i++)
      std::printf("%s{\"device\": %d, \"node\": %d, \"calls\": %llu}", i ? ", " : "", dv[i], nd[i], served[i]);
    std::printf("]}\n");
    delete code;
    return 0;
  }
  if (write_only) {
    delete code;
    return 0;
  }
  // agent service: nxec_agent_encode_batch calls of 64
  // ENC_CHUNK_REQ partial encodes each (4 local chunks x 1 coefficient row ->
  // 1 chunk + MD5, container_manager.cc:251, agent.cc:342) from 1, 4 and 16
  // concurrent agent worker threads on one context; bytes = inputs + outputs
  {
    nxec_ctx_t *ctx = nullptr;
    if (nxec_ctx_create(0, &ctx) == NXEC_OK) {
      const int nreq = 64, ni = 4;
      const uint8_t row[4] = {0x1d, 0x3a, 0x74, 0xe8};
      std::vector<int> tlist{1, 4, 16};
      if (const char *e = std::getenv("DROPIN_AGENT_THREADS")) tlist = {std::atoi(e)};
      // DROPIN_AGENT_MD5=0: ENC_CHUNK_REQ-shaped requests (getEncodedChunks computes no digest)
      const char *me = std::getenv("DROPIN_AGENT_MD5");
      const bool with_md5 = !(me && me[0] == '0');
      // chunk buffers: pageable (the reference's containers malloc them,
      // fs.cc:180) or arena blocks (an agent whose container reads land in
      // Chunk::allocateData buffers): the fused kernel then reads and writes
      // them in place over PCIe
      for (int arena = 0; arena < 2; arena++)
      for (int threads : tlist) {
        std::atomic<long> calls{0};
        std::atomic<bool> ok{true};
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; t++)
          pool.emplace_back([&, t] {
            const size_t in_bytes = static_cast<size_t>(nreq) * ni * cs, out_bytes = static_cast<size_t>(nreq) * cs;
            std::vector<uint8_t> in_v, out_v, md5(static_cast<size_t>(nreq) * 16);
            uint8_t *in = nullptr, *out = nullptr;
            if (arena) {
              void *a = nullptr, *b = nullptr;
              if (nxec_host_alloc(in_bytes, &a) != NXEC_OK || nxec_host_alloc(out_bytes, &b) != NXEC_OK) {
                ok = false;
                return;
              }
              in = static_cast<uint8_t *>(a);
              out = static_cast<uint8_t *>(b);
            } else {
              in_v.resize(in_bytes);
              out_v.resize(out_bytes);
              in = in_v.data();
              out = out_v.data();
            }
            fill(in, in_bytes, 5 + t);
            std::vector<const unsigned char *> ip(static_cast<size_t>(nreq) * ni);
            std::vector<unsigned char *> op(nreq);
            std::vector<nxec_agent_req> reqs(nreq);
            for (int r = 0; r < nreq; r++) {
              for (int j = 0; j < ni; j++) ip[r * ni + j] = in + (static_cast<size_t>(r) * ni + j) * cs;
              op[r] = out + static_cast<size_t>(r) * cs;
              reqs[r] = {ni, 1, row, ip.data() + r * ni, op.data() + r, with_md5 ? md5.data() + r * 16 : nullptr};
            }
            while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
              if (nxec_agent_encode_batch(ctx, reqs.data(), nreq, cs, 0) != NXEC_OK) ok = false;
              calls++;
            }
            if (arena) {
              nxec_host_free(in);
              nxec_host_free(out);
            }
          });
        for (auto &th : pool) th.join();
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const double bytes = static_cast<double>(calls) * nreq * (ni + 1) * cs;
        std::printf("{\"path\": \"nxec_agent_encode_batch (64 x 4->1 partial encodes%s)\", \"buffers\": \"%s\", "
                    "\"threads\": %d, \"chunk\": %d, \"calls\": %ld, \"GiB_s\": %.2f, \"ms_per_call\": %.3f, "
                    "\"ok\": %s}\n",
                    with_md5 ? " + MD5" : "", arena ? "arena" : "pageable", threads, cs, static_cast<long>(calls), bytes / dt / (1 << 30),
                    1e3 * dt * threads / static_cast<double>(calls), ok ? "true" : "false");
        std::fflush(stdout);
      }
      nxec_ctx_destroy(ctx);
    }
  }
  delete code;
  return 0;
}
