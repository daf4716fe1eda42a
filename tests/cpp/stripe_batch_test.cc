// StripeBatch (nexoedge_amd/csrc/coding/stripe_batch.hh), the batched
// ChunkManager entry, against the per-stripe reference path on the GPU:
// every stripe's chunks from encodeFile equal RSCode::encode of that stripe
// (the call ChunkManager::encodeFile makes, chunk_manager.cc:427) with the
// same ids (:442-446) and MD5 (:175, OpenSSL here); decodeFile restores the
// file from the first k alive chunks of every stripe.
//
//   stripe_batch_test            -> correctness over geometries / lengths
//   stripe_batch_test rate MIB   -> write (encode + MD5) and read rates of a
//                                   MIB-MiB file, JSON lines
#include <openssl/evp.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "coding/coding_generator.hh"
#include "coding/stripe_batch.hh"

static int g_fail = 0;
#define EXPECT(cond, ...)       \
  do {                          \
    if (!(cond)) {              \
      std::printf("FAIL ");     \
      std::printf(__VA_ARGS__); \
      std::printf("\n");        \
      g_fail++;                 \
    }                           \
  } while (0)

static void fill(uint8_t *p, size_t n, uint64_t s) {
  for (size_t i = 0; i < n; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    p[i] = static_cast<uint8_t>(s >> 56);
  }
}

static void check_file(int n, int k, length_t M, uint64_t length) {
  CodingOptions opt(static_cast<coding_param_t>(n), static_cast<coding_param_t>(k));
  Coding *code = CodingGenerator::genCoding(CodingScheme::RS, opt);
  StripeBatch batch(code, 0);
  EXPECT(batch.ok(), "batch");
  std::vector<uint8_t> file(length + 1);
  fill(file.data(), length, 1000 + n * 7 + length);
  std::vector<Chunk> chunks;
  const int off = 3 * n;  // a file that starts at the 4th stripe of its object
  EXPECT(batch.encodeFile(file.data(), length, M, chunks, off), "encodeFile (%d,%d) %lu", n, k,
         static_cast<unsigned long>(length));
  const uint64_t ns = batch.numStripes(length, M);
  EXPECT(chunks.size() == ns * n, "chunk count");
  // per stripe: the reference's own path (proxy_file_ops.cc:557-666 stripe split,
  // zero-padded last stripe, RSCode::encode)
  for (uint64_t s = 0; s < ns && g_fail < 20; s++) {
    const uint64_t lo = s * static_cast<uint64_t>(k) * M;
    const uint64_t len = std::min<uint64_t>(static_cast<uint64_t>(k) * M, length - lo);
    const length_t cs = code->getChunkSize(static_cast<length_t>(len));
    std::vector<uint8_t> padded(static_cast<size_t>(k) * cs, 0);
    std::memcpy(padded.data(), file.data() + lo, len);
    std::vector<Chunk> ref;
    EXPECT(code->encode(padded.data(), static_cast<length_t>(padded.size()), ref, nullptr), "RSCode::encode");
    for (int i = 0; i < n && static_cast<int>(ref.size()) == n; i++) {
      const Chunk &c = chunks[s * n + i];
      EXPECT(c.chunkId == off + static_cast<int>(s) * n + i && c.size == static_cast<int>(cs), "chunk meta");
      EXPECT(c.size == ref[i].size && std::memcmp(c.data, ref[i].data, cs) == 0, "stripe %lu chunk %d bytes",
             static_cast<unsigned long>(s), i);
      unsigned char d[16];
      unsigned int dl = 16;
      EVP_Digest(c.data, static_cast<size_t>(c.size), d, &dl, EVP_md5(), nullptr);
      EXPECT(std::memcmp(d, c.md5, 16) == 0, "stripe %lu chunk %d md5", static_cast<unsigned long>(s), i);
    }
  }
  // read back with failures: the first k alive chunks of every stripe as inputs
  for (const std::vector<chunk_id_t> &failed :
       {std::vector<chunk_id_t>{}, std::vector<chunk_id_t>{0}, std::vector<chunk_id_t>{1, static_cast<chunk_id_t>(n - 1)}}) {
    if (static_cast<int>(failed.size()) > n - k) continue;
    std::vector<Chunk> inputs;
    inputs.reserve(ns * k);  // Chunk copies are shallow (as in the reference): never reallocate owners
    for (uint64_t s = 0; s < ns; s++) {
      int taken = 0;
      for (int i = 0; i < n && taken < k; i++) {
        bool lost = false;
        for (chunk_id_t f : failed) lost |= f == i;
        if (lost) continue;
        inputs.emplace_back();
        inputs.back().copy(chunks[s * n + i]);  // fetched copy
        taken++;
      }
    }
    std::vector<uint8_t> back(length + 1, 0xEE);
    EXPECT(batch.decodeFile(inputs, length, M, failed, back.data()), "decodeFile");
    EXPECT(std::memcmp(back.data(), file.data(), length) == 0, "decoded file (%d,%d) %lu lost %zu", n, k,
           static_cast<unsigned long>(length), failed.size());
    EXPECT(back[length] == 0xEE, "nothing written past the file");
  }
  delete code;
}

static void rate(uint64_t mib) {
  const int n = 14, k = 10;
  const length_t M = 1 << 20;
  CodingOptions opt(n, k);
  Coding *code = CodingGenerator::genCoding(CodingScheme::RS, opt);
  StripeBatch batch(code, 0);
  const uint64_t length = mib << 20;
  for (int pinned = 0; pinned < 2; pinned++) {
    unsigned char *file = nullptr;
    std::vector<uint8_t> pageable;
    if (pinned) {
      void *p = nullptr;
      if (nxec_host_malloc_pinned(&p, length) != NXEC_OK) return;
      file = static_cast<unsigned char *>(p);
    } else {
      pageable.resize(length);
      file = pageable.data();
    }
    fill(file, length, 5);
    std::vector<Chunk> chunks;
    batch.encodeFile(file, length, M, chunks);  // warm
    const int reps = 3;
    auto t0 = std::chrono::steady_clock::now();
    bool ok = true;
    for (int r = 0; r < reps; r++) ok &= batch.encodeFile(file, length, M, chunks);
    const double wt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
    std::vector<chunk_id_t> failed{0, 1, 2, 3};
    std::vector<Chunk> inputs;
    const uint64_t ns = batch.numStripes(length, M);
    inputs.reserve(ns * k);
    for (uint64_t s = 0; s < ns; s++)
      for (int i = 4; i < 4 + k; i++) {
        inputs.emplace_back();
        inputs.back().copy(chunks[s * n + i]);
      }
    std::vector<uint8_t> out(length);
    batch.decodeFile(inputs, length, M, failed, out.data());  // warm
    t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) ok &= batch.decodeFile(inputs, length, M, failed, out.data());
    const double rt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
    ok &= std::memcmp(out.data(), file, length) == 0;
    std::printf("{\"path\": \"StripeBatch\", \"file_MiB\": %lu, \"file_buffer\": \"%s\", "
                "\"write_encode_md5_GiB_s_user_data\": %.2f, \"read_decode_4lost_GiB_s_user_data\": %.2f, "
                "\"ok\": %s}\n",
                static_cast<unsigned long>(mib), pinned ? "pinned" : "pageable",
                length / wt / (1 << 30), length / rt / (1 << 30), ok ? "true" : "false");
    std::fflush(stdout);
    if (pinned) nxec_host_free_pinned(file);
  }
  delete code;
}

int main(int argc, char **argv) {
  if (argc > 2 && std::string(argv[1]) == "rate") {
    rate(std::strtoull(argv[2], nullptr, 10));
    return 0;
  }
  const length_t M = 65536;
  for (int g = 0; g < 3; g++) {
    const int n = g == 0 ? 14 : (g == 1 ? 6 : 9), k = g == 0 ? 10 : (g == 1 ? 4 : 6);
    for (uint64_t length : {uint64_t(1), uint64_t(k) * M - 3, uint64_t(k) * M, 3 * uint64_t(k) * M + 12345,
                            5 * uint64_t(k) * M + 7})
      check_file(n, k, M, length);
  }
  check_file(14, 10, 1 << 20, (uint64_t(10) << 20) * 4 + 999);
  std::printf("%s %d failures\n", g_fail ? "FAILED" : "PASSED", g_fail);
  return g_fail ? 1 : 0;
}
