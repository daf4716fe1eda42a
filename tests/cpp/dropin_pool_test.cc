// The default pool under an unmodified proxy's load: `threads` worker threads
// share one RSCode (chunk_manager.cc:1779-1801, zmq.cc:83) and call
// RSCode::encode, RSCode::decode (4 erasures, full output) and a repair
// decode per stripe, with the default pool forced to `members` contexts on
// device 0 (nxec_default_devices).  Every encode's parity is checked
// bit-exactly against the CPU oracle (oracle/liboracle.so, the checker only),
// every decode against the original data, every repair against the encoded
// chunk.  Passes iff every check holds, every member served calls, and no
// call changed the calling thread's current device (nxec_default_devices:
// the lease restores it).  Prints one JSON line.
//
// usage: dropin_pool_test [members=8] [threads=16] [iters=12] [cs=262144]
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../oracle/nxec_oracle.h"
#include "coding/coding_generator.hh"
#include "nxec.h"

static void fill(uint8_t *p, size_t n, uint64_t s) {
  for (size_t i = 0; i < n; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    p[i] = static_cast<uint8_t>(s >> 56);
  }
}

int main(int argc, char **argv) {
  const int members = argc > 1 ? std::atoi(argv[1]) : 8;
  const int threads = argc > 2 ? std::atoi(argv[2]) : 16;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 12;
  const int cs = argc > 4 ? std::atoi(argv[4]) : (256 << 10);
  const int n = 14, k = 10, p = n - k;
  std::vector<int> devs(members, 0);
  if (nxec_default_devices(devs.data(), members) != NXEC_OK) {
    std::printf("nxec_default_devices: %s\n", nxec_last_error());
    return 1;
  }
  CodingOptions opt(n, k, false);
  Coding *code = CodingGenerator::genCoding(CodingScheme::RS, opt);
  if (!code) return 1;
  std::atomic<long> bad_enc{0}, bad_dec{0}, bad_rep{0}, bad_dev{0}, calls{0};
  std::mutex mu;
  std::condition_variable cv;
  int ready = 0;
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; t++)
    pool.emplace_back([&, t] {
      {  // start together: the calls overlap, as a busy proxy's do
        std::unique_lock<std::mutex> lk(mu);
        if (++ready == threads) cv.notify_all();
        cv.wait(lk, [&] { return ready == threads; });
      }
      int dev0 = -1;
      (void)hipGetDevice(&dev0);
      std::vector<uint8_t> data(static_cast<size_t>(k) * cs), want(static_cast<size_t>(n) * cs);
      for (int it = 0; it < iters; it++) {
        fill(data.data(), data.size(), 1000003ull * t + it);
        orc_rs_encode(n, k, data.data(), cs, want.data());
        std::vector<Chunk> stripe;
        if (!code->encode(data.data(), static_cast<length_t>(data.size()), stripe, nullptr)) {
          bad_enc++;
          continue;
        }
        for (int i = 0; i < n; i++)
          if (stripe[i].size != cs ||
              std::memcmp(stripe[i].data, want.data() + static_cast<size_t>(i) * cs, cs) != 0)
            bad_enc++;
        // 4 erasures, rotating with the iteration (data and parity chunks)
        std::vector<chunk_id_t> failed;
        for (int e = 0; e < p; e++) failed.push_back(static_cast<chunk_id_t>((it + 3 * e) % n));
        std::sort(failed.begin(), failed.end());
        failed.erase(std::unique(failed.begin(), failed.end()), failed.end());
        DecodingPlan plan;
        if (!code->preDecode(failed, plan, nullptr)) {
          bad_dec++;
          continue;
        }
        std::vector<chunk_id_t> ids = plan.getInputChunkIds();
        std::vector<Chunk> in(k);
        for (int i = 0; i < k; i++) in[i].copy(stripe[ids[i]]);
        data_t *out = nullptr;
        length_t osz = 0;
        if (!code->decode(in, &out, osz, plan, nullptr) || osz != data.size() ||
            std::memcmp(out, data.data(), data.size()) != 0)
          bad_dec++;
        std::free(out);
        // repair of one lost chunk (the proxy's at-proxy repair, chunk_manager.cc:1141)
        std::vector<chunk_id_t> tg{static_cast<chunk_id_t>((it * 5 + t) % n)};
        DecodingPlan rplan;
        if (!code->preDecode(tg, rplan, nullptr, true)) {
          bad_rep++;
          continue;
        }
        ids = rplan.getInputChunkIds();
        const size_t sel = rplan.getMinNumInputChunks();
        std::vector<Chunk> rin(sel);
        for (size_t i = 0; i < sel; i++) rin[i].copy(stripe[ids[i]]);
        out = nullptr;
        if (!code->decode(rin, &out, osz, rplan, nullptr, true, tg) || osz != static_cast<length_t>(cs) ||
            std::memcmp(out, want.data() + static_cast<size_t>(tg[0]) * cs, cs) != 0)
          bad_rep++;
        std::free(out);
        calls += 3;
        int dev1 = -1;
        (void)hipGetDevice(&dev1);
        if (dev1 != dev0) bad_dev++;
      }
    });
  for (auto &th : pool) th.join();
  std::vector<int> d(members + 4), nd(members + 4), inf(members + 4);
  std::vector<unsigned long long> served(members + 4);
  int cnt = 0;
  const int src = nxec_default_pool_stats(d.data(), nd.data(), served.data(), inf.data(), members + 4, &cnt);
  int unused = 0;
  std::printf("{\"members\": %d, \"threads\": %d, \"iters\": %d, \"chunk\": %d, \"calls\": %ld, \"served\": [", cnt,
              threads, iters, cs, static_cast<long>(calls));
  for (int i = 0; i < cnt && i < members + 4; i++) {
    std::printf("%s%llu", i ? ", " : "", served[i]);
    unused += served[i] == 0;
  }
  const bool ok = src == NXEC_OK && cnt == members && unused == 0 && bad_enc == 0 && bad_dec == 0 && bad_rep == 0 &&
                  bad_dev == 0 && calls == 3L * threads * iters;
  std::printf("], \"bad_encode\": %ld, \"bad_decode\": %ld, \"bad_repair\": %ld, \"device_changed\": %ld, \"ok\": %s}\n",
              static_cast<long>(bad_enc), static_cast<long>(bad_dec), static_cast<long>(bad_rep),
              static_cast<long>(bad_dev), ok ? "true" : "false");
  delete code;
  return ok ? 0 : 1;
}
