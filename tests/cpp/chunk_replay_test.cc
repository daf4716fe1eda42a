// Replays of the reference's Chunk ownership sequences against
// nexoedge_amd/csrc/coding/chunk.hh, which replaces src/ds/chunk.hh in an
// unmodified Nexoedge build.  The reference copies chunks with the implicit
// memberwise (shallow) copy and disowns the copy:
//   writeFileStripe       chunk_manager.cc:99,175-178  (encodeFile -> computeMD5
//                         -> events[i].chunks[j] = file.chunks[idx]; freeData = false)
//   verifyFileChecksums   chunk_manager.cc:1275-1276
//   accessChunks          chunk_manager.cc:1498-1499
//   writeFileStripes      proxy_file_ops.cc:584-586    (ownership handed down the array)
//   RPR_CHUNK_REQ         agent.cc:334-342, 365-367    (malloc'd outputs, encode, MD5, store events)
//   getEncodedChunks      container_manager.cc:221-258 (returned by value, freeData = false)
// and the explicit move of encodeFile (chunk_manager.cc:443-447) and of the
// read/repair inputs (:765-775, :1129-1132).  Every alias must point at the
// original buffer, every buffer must be freed exactly once (run under
// `make asan` with LeakSanitizer: no leak, no double free), and the MD5 every
// sequence computes must equal OpenSSL's of the bytes.
//
// With a GPU the stripe comes from RSCode::encode (and its digests from the
// fused kernel); without one (the sanitizer builds run on the CPU) the same
// chunks are built the way RSCode::encode allocates them (rs.cc:70-80) with
// the parity left as filled bytes -- the ownership sequences are what is
// tested there.
//
//   usage: chunk_replay_test [cs]       exit 0 iff every check passed
#include <openssl/evp.h>

#include <atomic>
#include <thread>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "coding/coding_generator.hh"
#include "coding/coding_util.hh"
#include "nxec.h"

static int g_fail = 0;
#define CHECK(cond, ...)        \
  do {                          \
    if (!(cond)) {              \
      std::printf("FAIL ");     \
      std::printf(__VA_ARGS__); \
      std::printf("\n");        \
      g_fail++;                 \
    }                           \
  } while (0)

// the parts of ChunkEvent (chunk_event.hh:10-75) and File (file.hh:91-94)
// these sequences touch: both delete [] their chunk arrays on release
struct Event {
  int numChunks = 0;
  Chunk *chunks = nullptr;
  ~Event() { delete[] chunks; }
};
struct FileRec {
  int numChunks = 0;
  Chunk *chunks = nullptr;
  unsigned char *data = nullptr;
  ~FileRec() {
    delete[] chunks;
    std::free(data);
  }
};

static void fill(unsigned char *p, size_t n, uint64_t s) {
  for (size_t i = 0; i < n; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    p[i] = static_cast<unsigned char>(s >> 56);
  }
}

static bool md5_ok(const Chunk &c) {
  unsigned char d[16];
  unsigned int dl = 16;
  EVP_Digest(c.data, static_cast<size_t>(c.size), d, &dl, EVP_md5(), nullptr);
  return std::memcmp(d, c.md5, 16) == 0;
}

static bool g_gpu = false;

// ChunkManager::encodeFile (chunk_manager.cc:369-452) for one stripe
static bool encodeFile(Coding *code, FileRec &file, int length, int chunkIdOffset) {
  std::vector<Chunk> stripe;
  if (g_gpu) {
    if (!code->encode(file.data, static_cast<length_t>(length), stripe, nullptr)) return false;
  } else {  // rs.cc:70-80's allocation and copy; parity bytes made up
    const int n = code->getN(), k = code->getK();
    const int cs = static_cast<int>(code->getChunkSize(static_cast<length_t>(length)));
    stripe.resize(n);
    for (int i = 0; i < n; i++) {
      stripe.at(i).setChunkId(i);
      if (!stripe.at(i).allocateData(cs, true)) return false;
      if (i < k) std::memcpy(stripe.at(i).data, file.data + static_cast<size_t>(i) * cs, cs);
      else fill(stripe.at(i).data, cs, 99 + i);
    }
  }
  file.numChunks = static_cast<int>(stripe.size());
  file.chunks = new Chunk[file.numChunks];
  for (int i = 0; i < file.numChunks; i++) {
    file.chunks[i].move(stripe.at(i));  // :444
    file.chunks[i].setId(0, chunk_nil_uuid(), i + chunkIdOffset);
    file.chunks[i].fileVersion = 1;
  }
  return true;
}

static void writeFileStripe(Coding *code, int cs) {
  const int n = code->getN(), k = code->getK();
  FileRec file;
  file.data = static_cast<unsigned char *>(std::malloc(static_cast<size_t>(k) * cs));
  fill(file.data, static_cast<size_t>(k) * cs, 5);
  CHECK(encodeFile(code, file, k * cs, 0), "encodeFile");
  if (file.numChunks != n) return;
  std::vector<unsigned char *> owned(n);
  for (int i = 0; i < n; i++) owned[i] = file.chunks[i].data;
  for (int i = 0; i < k; i++)
    CHECK(std::memcmp(file.chunks[i].data, file.data + static_cast<size_t>(i) * cs, cs) == 0, "data chunk %d", i);
  {
    const int numReqs = n;  // one chunk per node
    Event *events = new Event[numReqs * 2];
    for (int i = 0; i < numReqs; i++) {
      events[i].numChunks = 1;
      events[i].chunks = new Chunk[1];
      for (int j = 0; j < 1; j++) {
        const int chunkIdx = i + j;
        file.chunks[chunkIdx].computeMD5();                      // :175
        events[i].chunks[j] = file.chunks[chunkIdx];             // :176
        events[i].chunks[j].freeData = false;                    // :178
        CHECK(events[i].chunks[j].data == owned[chunkIdx], "event %d aliases the file's chunk", i);
        CHECK(md5_ok(file.chunks[chunkIdx]) && std::memcmp(events[i].chunks[j].md5, file.chunks[chunkIdx].md5, 16) == 0,
              "chunk %d md5 (%s)", chunkIdx, g_gpu ? "GPU digest" : "host");
      }
    }
    // the send path reads the events' chunks (ProxyIO::sendChunkRequestToAgent)
    for (int i = 0; i < numReqs; i++) CHECK(md5_ok(events[i].chunks[0]), "event %d md5 matches its bytes", i);
    delete[] events;  // :344-346: the borrowed views free nothing
  }
  for (int i = 0; i < n; i++) CHECK(file.chunks[i].data == owned[i] && file.chunks[i].freeData, "owner %d intact", i);

  // verifyFileChecksums (:1275-1276) and accessChunks (:1498-1499): views of the file's chunks
  {
    Event ev;
    ev.numChunks = n;
    ev.chunks = new Chunk[n];
    for (int i = 0; i < n; i++) {
      ev.chunks[i] = file.chunks[i];
      ev.chunks[i].freeData = false;
    }
    for (int i = 0; i < n; i++) CHECK(ev.chunks[i].data == owned[i] && ev.chunks[i].verifyMD5(), "verify view %d", i);
  }
  // a second computeMD5 of the same chunk hashes the bytes again (a GPU digest is used once)
  file.chunks[0].data[0] ^= 0x5a;
  CHECK(file.chunks[0].computeMD5() && md5_ok(file.chunks[0]), "computeMD5 after a write hashes again");
  file.chunks[0].data[0] ^= 0x5a;
}  // file teardown frees each chunk once

// Proxy::writeFileStripes' CLEAN_UP_PREVIOUS_STRIPES (proxy_file_ops.cc:581-595):
// chunks of stripes [startIdx, end) handed to the front of the array
static void handDown(Coding *code, int cs) {
  const int n = code->getN(), k = code->getK();
  const int stripes = 3, startIdx = 1;
  FileRec wf;
  wf.numChunks = n * stripes;
  wf.chunks = new Chunk[wf.numChunks];
  std::vector<unsigned char *> owned(wf.numChunks);
  for (int s = 0; s < stripes; s++) {
    FileRec swf;
    swf.data = static_cast<unsigned char *>(std::malloc(static_cast<size_t>(k) * cs));
    fill(swf.data, static_cast<size_t>(k) * cs, 40 + s);
    CHECK(encodeFile(code, swf, k * cs, s * n), "encodeFile stripe %d", s);
    if (swf.numChunks != n) return;
    for (int i = 0; i < n; i++) {  // proxy_file_ops.cc:651-653 takes the stripe's chunks over
      wf.chunks[s * n + i] = swf.chunks[i];
      swf.chunks[i].freeData = false;
      owned[s * n + i] = wf.chunks[s * n + i].data;
    }
  }
  // stripe 0 was written before startIdx: release it as the reference's later cleanup would
  for (int j = 0; j < startIdx * n; j++) wf.chunks[j].release();
  for (int j = startIdx * n; j < stripes * n; j++) {
    wf.chunks[j - startIdx * n] = wf.chunks[j];
    wf.chunks[j].freeData = false;
  }
  for (int j = 0; j < (stripes - startIdx) * n; j++)
    CHECK(wf.chunks[j].data == owned[j + startIdx * n] && wf.chunks[j].freeData, "handed-down chunk %d", j);
}

// ContainerManager::getEncodedChunks (container_manager.cc:221-258): a chunk
// returned by value, its buffer disowned; the caller frees it
static Chunk getEncodedChunks(std::vector<Chunk> &raw, unsigned char *matrix) {
  Chunk codedChunk;
  std::vector<unsigned char *> rawData(raw.size());
  for (size_t i = 0; i < raw.size(); i++) rawData[i] = raw[i].data;
  codedChunk.data = static_cast<unsigned char *>(std::malloc(raw[0].size));
  codedChunk.size = raw[0].size;
  if (g_gpu) CodingUtils::encode(rawData.data(), static_cast<int>(raw.size()), &codedChunk.data, 1, codedChunk.size, matrix);
  else std::memset(codedChunk.data, 0, codedChunk.size);
  codedChunk.freeData = false;
  return codedChunk;
}

// Agent RPR_CHUNK_REQ (agent.cc:315-367) with the ENC replies of the peers
static void agentRepair(int cs) {
  const int numReq = 3, numChunks = 3;  // 3 partials in, 1 local + 2 sent outputs
  std::vector<Chunk> local(4);
  for (int i = 0; i < 4; i++) {
    local[i].allocateData(cs);
    fill(local[i].data, cs, 70 + i);
  }
  unsigned char row[4] = {1, 2, 3, 4};
  Event replies;
  replies.numChunks = numReq;
  replies.chunks = new Chunk[numReq];
  for (int i = 0; i < numReq; i++) {
    replies.chunks[i] = getEncodedChunks(local, row);  // IO hands the reply over
    replies.chunks[i].freeData = true;                 // the message owns the bytes (io.cc:209-216)
  }
  unsigned char *input[numReq], *output[numChunks];
  Event event;
  event.numChunks = numChunks;
  event.chunks = new Chunk[numChunks];
  for (int i = 0; i < numReq; i++) input[i] = replies.chunks[i].data;
  for (int i = 0; i < numChunks; i++) {  // :333-337
    event.chunks[i].data = static_cast<unsigned char *>(std::malloc(cs));
    event.chunks[i].size = cs;
    output[i] = event.chunks[i].data;
  }
  unsigned char m[numChunks * numReq] = {1, 1, 1, 2, 3, 4, 5, 6, 7};
  if (g_gpu) CHECK(CodingUtils::encode(input, numReq, output, numChunks, cs, m), "CodingUtils::encode");
  else
    for (int i = 0; i < numChunks; i++) fill(output[i], cs, 80 + i);
  for (int i = 0; i < numChunks; i++) {  // :341-343
    CHECK(event.chunks[i].computeMD5() && md5_ok(event.chunks[i]), "RPR output %d md5", i);
  }
  const int numChunkReqsToSend = numChunks - 1;
  {
    Event *store = new Event[numChunkReqsToSend * 2];
    for (int i = 0; i < numChunkReqsToSend; i++) {  // :350-369
      store[i].numChunks = 1;
      store[i].chunks = new Chunk[1];
      store[i].chunks[0] = event.chunks[(i + 1) * 1 + 0];
      store[i].chunks[0].freeData = false;
      CHECK(store[i].chunks[0].data == output[i + 1] && md5_ok(store[i].chunks[0]), "store event %d", i);
    }
    delete[] store;
  }
  for (int i = 0; i < numChunks; i++) CHECK(event.chunks[i].data == output[i], "event output %d intact", i);
}

// decodeFile / repairFile inputs (chunk_manager.cc:765-775, :1129-1132): resize, then move from the replies
static void moveInputs(int cs) {
  const int num = 5;
  Event *replies = new Event[num];
  std::vector<unsigned char *> owned(num);
  for (int i = 0; i < num; i++) {
    replies[i].numChunks = 1;
    replies[i].chunks = new Chunk[1];
    replies[i].chunks[0].allocateData(cs);
    replies[i].chunks[0].setChunkId(20 + i);
    owned[i] = replies[i].chunks[0].data;
  }
  {
    std::vector<Chunk> inputChunks;
    inputChunks.resize(num);
    for (int i = 0; i < num; i++) {
      inputChunks.at(i).move(replies[i].chunks[0]);
      inputChunks.at(i).setChunkId(inputChunks.at(i).getChunkId() % 14);
      CHECK(inputChunks.at(i).data == owned[i] && replies[i].chunks[0].data == nullptr, "moved input %d", i);
    }
  }  // the inputs free the buffers
  delete[] replies;
}

// A one-slot allocator that hands a freed block straight back (what glibc's
// tcache does for a same-size malloc on one thread): it forces the recycled
// address the stale-digest cases below need, whichever thread frees.
struct RecyclingPool {
  unsigned char *slot = nullptr;
  unsigned char *alloc(size_t n) {
    unsigned char *p = slot ? slot : static_cast<unsigned char *>(std::malloc(n));
    slot = nullptr;
    return p;
  }
  void release(unsigned char *p) { slot = p; }
  ~RecyclingPool() { std::free(slot); }
};

static void md5_of(const unsigned char *p, int n, unsigned char *d) {
  unsigned int dl = 16;
  EVP_Digest(p, static_cast<size_t>(n), d, &dl, EVP_md5(), nullptr);
}

// Mode-2 digests of plain regions (include/nxec.h §6b) against a recycled
// buffer: a digest noted on thread A for (p, cs), the buffer freed with plain
// free() and handed out again at the same address and size on thread B with
// new bytes, then Chunk::computeMD5 on A must hash the new bytes (round-3
// advisor: container_manager.cc:241-252's ENC output is noted, never hashed,
// freed by the caller).  And nxec_digest_forget from another thread drops A's entry.
static void staleDigestAcrossThreads(int cs) {
  if (nxec_chunk_md5_mode() < 1) return;
  RecyclingPool pool;
  unsigned char *buf = pool.alloc(cs);
  fill(buf, cs, 901);
  unsigned char dOld[16], dNew[16];
  md5_of(buf, cs, dOld);
  nxec_digest_clear();
  CHECK(nxec_digest_note(buf, cs, dOld) == NXEC_OK, "note on A");
  unsigned char *again = nullptr;
  std::thread b([&] {
    pool.release(buf);      // free() on B ...
    again = pool.alloc(cs);  // ... and malloc of the same size hands it out again
    fill(again, cs, 902);    // new bytes
  });
  b.join();
  CHECK(again == buf, "recycled address");
  md5_of(again, cs, dNew);
  {
    Chunk c;
    c.data = again;
    c.size = cs;
    c.freeData = false;
    CHECK(c.computeMD5() && std::memcmp(c.md5, dNew, 16) == 0 && std::memcmp(c.md5, dOld, 16) != 0,
          "computeMD5 on A hashes the recycled buffer's new bytes, not the stale digest");
  }
  // the same bytes under a stale entry: the digest is right either way
  CHECK(nxec_digest_note(again, cs, dNew) == NXEC_OK, "note again");
  std::thread f([&] { nxec_digest_forget(again); });  // Chunk::freeBuffer on another thread
  f.join();
  unsigned char got[16];
  CHECK(nxec_digest_take(again, cs, got) == 0, "forget from another thread drops A's entry");
  pool.release(again);
}

// repairFile's tail (chunk_manager.cc:1137-1174) twice at one repairedData
// address: run 1's decode notes both repaired regions, the PUT loop hashes
// only the first (its bad_alloc exit at :1155-1158 leaves the loop), and
// repairedData is freed; run 2 gets the same address back with other bytes
// and a decode that notes nothing (NXEC_CHUNK_MD5 < 2, or the digest-less
// path), so computeMD5 of region 1 must hash run 2's bytes.
static void repairTailTwice(int cs) {
  if (nxec_chunk_md5_mode() < 1) return;
  RecyclingPool pool;
  const int nrep = 2;
  unsigned char *first = nullptr;
  for (int run = 0; run < 2; run++) {
    unsigned char *repairedData = pool.alloc(static_cast<size_t>(cs) * nrep);  // :1137
    if (run == 0) first = repairedData;
    else CHECK(repairedData == first, "run 2 reuses run 1's address");
    for (int t = 0; t < nrep; t++) fill(repairedData + static_cast<size_t>(t) * cs, cs, 1000 + 10 * run + t);
    if (run == 0) {  // what RSCode::decode(isRepair) leaves under NXEC_CHUNK_MD5=2 (rs.cc here)
      nxec_digest_clear();
      for (int t = 0; t < nrep; t++) {
        unsigned char d[16];
        md5_of(repairedData + static_cast<size_t>(t) * cs, cs, d);
        nxec_digest_note(repairedData + static_cast<size_t>(t) * cs, cs, d);
      }
    }
    const int hashed = run == 0 ? 1 : nrep;
    for (int t = 0; t < hashed; t++) {  // :1168-1174
      Chunk c;
      c.size = cs;
      c.data = repairedData + static_cast<size_t>(t) * cs;
      CHECK(c.computeMD5() && md5_ok(c), "run %d repaired chunk %d md5 matches its bytes", run, t);
      c.freeData = false;
    }
    pool.release(repairedData);  // free(repairedData) at the end of repairFile
  }
}

// RSCode::encode's marks on the Chunks themselves lapse when the thread
// allocates or frees chunk buffers before hashing (the rule in chunk.hh)
static void chunkMarkLapses(int cs) {
  if (nxec_chunk_md5_mode() < 1) return;
  Chunk c;
  c.allocateData(cs);
  fill(c.data, cs, 1200);
  std::memset(c.md5, 0xAB, 16);  // a digest that is not the bytes'
  c.setDigestValid();
  Chunk other;
  other.allocateData(cs);  // another chunk buffer on this thread: the epoch moves on
  CHECK(c.computeMD5() && md5_ok(c), "a mark from before an allocation is not trusted");
  std::memset(c.md5, 0xAB, 16);
  c.setDigestValid();
  { Chunk tmp; tmp.allocateData(cs); }  // allocated and freed
  CHECK(c.computeMD5() && md5_ok(c), "a mark from before a free is not trusted");
}

int main(int argc, char **argv) {
  const int cs = argc > 1 ? std::atoi(argv[1]) : (256 << 10);
  int dev = 0;
  g_gpu = nxec_device_count(&dev) == NXEC_OK && dev > 0;
  for (int nk : {0, 1}) {
    CodingOptions opt(nk ? 6 : 14, nk ? 4 : 10, false);
    Coding *code = CodingGenerator::genCoding(CodingScheme::RS, opt);
    CHECK(code != nullptr, "genCoding");
    if (!code) break;
    writeFileStripe(code, cs);
    writeFileStripe(code, 1000 + nk);  // small chunks: plain malloc, not the arena
    handDown(code, cs);
    delete code;
  }
  agentRepair(cs);
  moveInputs(cs);
  staleDigestAcrossThreads(cs);
  repairTailTwice(cs);
  chunkMarkLapses(cs);
  std::printf("%s %d failures (%s)\n", g_fail ? "FAILED" : "PASSED", g_fail, g_gpu ? "gpu" : "cpu");
  return g_fail ? 1 : 0;
}
