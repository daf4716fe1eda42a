// C++ surface test: drives RSCode / CodingUtils / CodingGenerator /
// DecodingPlan (nexoedge_amd/csrc/coding) exactly the way the reference's
// src/tests/common/coding_test.cc does (encode :192, decode with the first
// n-k chunks erased :211-265, every single-node repair incl. the CAR partial
// encode per rack :269-427, every double failure :432-533), on MI355X.
//
// Self-checks every round trip like the reference (memcmp against the
// original data) and prints SHA-256 digests that tests/test_cpp_surface.py
// compares with tests/golden/golden.json.  Exit code 0 iff every check passed.
#include <openssl/sha.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "coding/coding_generator.hh"
#include "coding/coding_util.hh"

static int g_fail = 0;
#define EXPECT(cond, ...)                  \
  do {                                     \
    if (!(cond)) {                         \
      std::printf("FAIL ");                \
      std::printf(__VA_ARGS__);            \
      std::printf("\n");                   \
      g_fail++;                            \
    }                                      \
  } while (0)

static void fill_bytes(uint8_t *p, int64_t nbytes, uint64_t seed) {  // splitmix64, LE (tests/helpers.py)
  uint64_t s = seed;
  for (int64_t i = 0; i < nbytes; i += 8) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (int b = 0; b < 8 && i + b < nbytes; b++) p[i + b] = static_cast<uint8_t>(z >> (8 * b));
  }
}

static std::string sha(const uint8_t *p, size_t n) {
  uint8_t d[32];
  SHA256(p, n, d);
  char h[65];
  for (int i = 0; i < 32; i++) std::snprintf(h + 2 * i, 3, "%02x", d[i]);
  return std::string(h, 64);
}

static std::string hex(const uint8_t *p, size_t n) {
  std::string s;
  char b[3];
  for (size_t i = 0; i < n; i++) {
    std::snprintf(b, 3, "%02x", p[i]);
    s += b;
  }
  return s;
}

static bool run(int n, int k, int cs, bool car) {
  CodingOptions opt(static_cast<coding_param_t>(n), static_cast<coding_param_t>(k), car);
  Coding *code = CodingGenerator::genCoding(CodingScheme::RS, opt);
  EXPECT(code != nullptr, "genCoding(%d,%d)", n, k);
  if (!code) return false;
  const int before = g_fail;
  // geometry (coding_test.cc:116-144)
  const length_t fsize = static_cast<length_t>(k) * cs;
  EXPECT(code->getNumChunksPerNode() == 1, "chunks per node");
  EXPECT(code->getChunkSize(fsize) == static_cast<length_t>(cs), "chunk size");
  EXPECT(code->getChunkSize(fsize - 1) == static_cast<length_t>(cs), "chunk size ceil");
  EXPECT(code->getNumDataChunks() == static_cast<num_t>(k) && code->getNumCodeChunks() == static_cast<num_t>(n - k),
         "data/code chunks");
  EXPECT(code->getCodingStateSize() == 0, "state size");

  const uint64_t seed = 1000003ull * n + 10007ull * k + cs;
  std::vector<uint8_t> data(static_cast<size_t>(fsize));
  fill_bytes(data.data(), fsize, seed);
  std::vector<Chunk> stripe;
  EXPECT(code->encode(data.data(), fsize, stripe, nullptr), "encode");
  EXPECT(static_cast<int>(stripe.size()) == n, "stripe size");
  std::vector<uint8_t> parity;
  for (int i = k; i < n; i++) parity.insert(parity.end(), stripe[i].data, stripe[i].data + cs);
  for (int i = 0; i < n; i++) EXPECT(stripe[i].chunkId == i && stripe[i].size == cs, "chunk meta");
  std::printf("ENC %d %d %d %s\n", n, k, cs, sha(parity.data(), parity.size()).c_str());

  // decode with the first n-k chunks erased (coding_test.cc:211-265)
  DecodingPlan plan;
  std::vector<chunk_id_t> failed;
  for (int i = 0; i < n - k; i++) failed.push_back(static_cast<chunk_id_t>(i));
  EXPECT(code->preDecode(failed, plan, nullptr), "preDecode");
  EXPECT(plan.getMinNumInputChunks() == static_cast<size_t>(k), "min inputs");
  std::vector<chunk_id_t> ids = plan.getInputChunkIds();
  std::vector<Chunk> in(k);
  for (int i = 0; i < k; i++) in[i].copy(stripe[ids[i]]);
  data_t *out = nullptr;
  length_t outSize = 0;
  EXPECT(code->decode(in, &out, outSize, plan, nullptr), "decode");
  EXPECT(outSize == fsize && out && std::memcmp(out, data.data(), fsize) == 0, "decode content (%d,%d)", n, k);
  std::printf("DEC %d %d %d %s\n", n, k, cs, out ? sha(out, outSize).c_str() : "-");
  std::free(out);

  // full-output decode for more erasure sets: the last n-k (all parity: every
  // data chunk comes straight from the inputs) and every single chunk, into a
  // caller buffer (rs.cc:164-173)
  {
    std::vector<std::vector<chunk_id_t>> sets;
    std::vector<chunk_id_t> last;
    for (int i = k; i < n; i++) last.push_back(static_cast<chunk_id_t>(i));
    sets.push_back(last);
    for (int f = 0; f < n; f++) sets.push_back({static_cast<chunk_id_t>(f)});
    std::vector<unsigned char> buf(fsize);
    for (const auto &fs : sets) {
      plan.release();
      EXPECT(code->preDecode(fs, plan, nullptr), "preDecode set");
      std::vector<chunk_id_t> sid = plan.getInputChunkIds();
      std::vector<Chunk> sin(k);
      for (int i = 0; i < k; i++) sin[i].copy(stripe[sid[i]]);
      std::fill(buf.begin(), buf.end(), 0xEE);
      data_t *bp = buf.data();
      length_t bsz = 0;
      EXPECT(code->decode(sin, &bp, bsz, plan, nullptr) && bp == buf.data(), "decode set (%d,%d) first %d", n, k,
             static_cast<int>(fs[0]));
      EXPECT(bsz == fsize && std::memcmp(buf.data(), data.data(), fsize) == 0, "decode set content (%d,%d) first %d",
             n, k, static_cast<int>(fs[0]));
    }
  }

  // every single-node repair (coding_test.cc:269-427)
  for (int f = 0; f < n; f++) {
    plan.release();
    std::vector<chunk_id_t> tg{static_cast<chunk_id_t>(f)};
    EXPECT(code->preDecode(tg, plan, nullptr, true), "preDecode repair %d", f);
    ids = plan.getInputChunkIds();
    const num_t sel = static_cast<num_t>(plan.getMinNumInputChunks());
    std::vector<Chunk> rin;
    if (!car) {
      rin.resize(sel);
      for (num_t i = 0; i < sel; i++) rin[i].copy(stripe[ids[i]]);
    } else {
      // partial encode per rack (coding_test.cc:312-355), r = n-k racks
      const int r = n - k;
      data_t *rm = plan.getRepairMatrix();
      num_t cidx = 0;
      int inRack = 0;
      rin.reserve(r);  // owners must not be moved by a reallocation (shallow Chunk copies)
      for (int cr = 0, rn = 0; cr < r && cidx < sel; cr++, rn += inRack) {
        inRack = n / r + (cr < n % r);
        const int rackEnd = rn + inRack;
        const num_t start = cidx;
        if (ids[cidx] >= rackEnd) continue;
        std::vector<unsigned char *> pin;
        for (int i = rn; i < rackEnd && cidx < sel; i++) {
          if (i != ids[cidx]) continue;
          pin.push_back(stripe[ids[cidx]].data);
          cidx++;
        }
        Chunk part;
        part.allocateData(cs);
        unsigned char *pout[1] = {part.data};
        EXPECT(CodingUtils::encode(pin.data(), static_cast<int>(pin.size()), pout, 1, cs, rm + start),
               "partial encode");
        rin.emplace_back();
        rin.back().move(part);
      }
    }
    out = nullptr;
    EXPECT(code->decode(rin, &out, outSize, plan, nullptr, true, tg), "repair %d", f);
    EXPECT(out && outSize == static_cast<length_t>(cs) && std::memcmp(out, stripe[f].data, cs) == 0,
           "repair content (%d,%d) f=%d car=%d", n, k, f, car);
    std::printf("REP %d %d %d %d %s %s\n", n, k, cs, f, hex(plan.getRepairMatrix(), k).c_str(),
                out ? sha(out, cs).c_str() : "-");
    std::free(out);

    // every double failure (coding_test.cc:432-533)
    if (n - k < 2) continue;
    for (int g = f + 1; g < n; g++) {
      plan.release();
      std::vector<chunk_id_t> tg2{static_cast<chunk_id_t>(f), static_cast<chunk_id_t>(g)};
      EXPECT(code->preDecode(tg2, plan, nullptr, true), "preDecode double");
      ids = plan.getInputChunkIds();
      std::vector<Chunk> din(k);
      for (int i = 0; i < k; i++) din[i].copy(stripe[ids[i]]);
      out = nullptr;
      EXPECT(code->decode(din, &out, outSize, plan, nullptr, true, tg2), "double repair");
      EXPECT(out && std::memcmp(out, stripe[f].data, cs) == 0 && std::memcmp(out + cs, stripe[g].data, cs) == 0,
             "double repair content (%d,%d) %d,%d", n, k, f, g);
      std::printf("RP2 %d %d %d %d,%d %s %s\n", n, k, cs, f, g, hex(plan.getRepairMatrix(), 2 * k).c_str(),
                  out ? sha(out, 2 * cs).c_str() : "-");
      std::free(out);
    }
  }
  // generator rejects bad parameters (rs.cc:16-18, coding_generator.hh:19-22)
  CodingOptions bad(static_cast<coding_param_t>(k), static_cast<coding_param_t>(n));
  Coding *b = n > k ? CodingGenerator::genCoding(CodingScheme::RS, bad) : nullptr;
  EXPECT(b == nullptr, "bad params rejected");
  delete code;
  return g_fail == before;
}

int main(int argc, char **argv) {
  const int cs = argc > 1 ? std::atoi(argv[1]) : 1000;
  for (int car = 0; car <= 1; car++) {
    for (int n = 4; n <= 12; n++)
      for (int m = 1; m <= n - 2; m++) run(n, n - m, cs, car);
    run(14, 10, cs, car);
    run(16, 12, cs, car);
    run(20, 16, cs, car);
  }
  std::printf("%s %d failures\n", g_fail ? "FAILED" : "PASSED", g_fail);
  return g_fail ? 1 : 0;
}
