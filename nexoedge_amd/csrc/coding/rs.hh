// Reed-Solomon code over GF(2^8) on MI355X (reference: src/common/coding/rs.hh).
// Method semantics follow rs.cc line for line (see rs.cc here for citations);
// the byte work goes to libnxec's gfx950 kernels via include/nxec.h.
#ifndef NXEC_CODING_RS_HH
#define NXEC_CODING_RS_HH

#include <stddef.h>
#include <stdint.h>

#include "coding.hh"
#include "nxec.h"

class RSCode : public Coding {
 public:
  // rs.hh:12.  Inline on purpose: it records the layout of Chunk,
  // CodingOptions, ByteBuffer, DecodingPlan and RSCode as the *calling* TU
  // sees them and the exported constructor below compares that with
  // libnxec's own (include/nxec.h §9), throwing std::invalid_argument on a
  // difference -- the case of a Nexoedge TU whose include graph reached other
  // headers than the ones libnxec was built with.
  RSCode(CodingOptions options) : RSCode(options, callerAbi()) {}
  // rs.cc:11-30 plus the ABI check; throws std::invalid_argument
  RSCode(CodingOptions options, const nxec_cxx_abi &callerLayout);
  ~RSCode() {}

  num_t getNumDataChunks();
  num_t getNumCodeChunks();
  num_t getNumChunks();
  num_t getNumChunksPerNode();
  length_t getCodingStateSize();
  length_t getChunkSize(length_t dataSize);

  bool encode(data_t *data, length_t dataSize, std::vector<Chunk> &stripe, data_t **codingState);
  bool decode(std::vector<Chunk> &inputChunks, data_t **decodedData, length_t &decodedSize, DecodingPlan &plan,
              data_t *codingState, bool isRepair = false,
              std::vector<chunk_id_t> repairTargets = std::vector<chunk_id_t>());
  bool preDecode(const std::vector<chunk_id_t> &failedNodeIdx, DecodingPlan &plan, data_t *codingState,
                 bool isRepair = false);

  // ---- batched, device-resident entry points for a ChunkManager that keeps
  // ---- many stripes in HBM ([stripe][n][chunkSize] layout)
  bool encodeStripes(nxec_ctx_t *ctx, unsigned char *dStripes, int64_t chunkStride, int64_t stripeStride,
                     int64_t chunkSize, int64_t numStripes, void *stream = nullptr);
  bool recoverStripes(nxec_ctx_t *ctx, const std::vector<chunk_id_t> &failedChunkIdx, unsigned char *dStripes,
                      int64_t chunkStride, int64_t stripeStride, int64_t chunkSize, int64_t numStripes,
                      void *stream = nullptr);

  const uint8_t *getEncodeMatrix() const { return _encodeMatrix; }

  // the layout of the C++ surface as the TU that compiles this sees it
  static nxec_cxx_abi callerAbi() {
    nxec_cxx_abi a;
    a.version = NXEC_CXX_ABI_VERSION;
    a.size_chunk = sizeof(Chunk);
    a.align_chunk = alignof(Chunk);
    a.off_chunk_uuid = offsetof(Chunk, fuuid);
    a.off_chunk_id = offsetof(Chunk, chunkId);
    a.off_chunk_data = offsetof(Chunk, data);
    a.off_chunk_size = offsetof(Chunk, size);
    a.off_chunk_free = offsetof(Chunk, freeData);
    a.off_chunk_md5 = offsetof(Chunk, md5);
    a.off_chunk_digest = offsetof(Chunk, digestData);
    a.size_uuid = sizeof(Chunk::fuuid);
    a.size_coding_options = sizeof(CodingOptions);
    a.size_byte_buffer = sizeof(ByteBuffer);
    a.size_decoding_plan = sizeof(DecodingPlan);
    a.size_rscode = sizeof(RSCode);
    return a;
  }

 private:
  bool carRepairFinalize(unsigned char *inputp[], num_t numInputChunks, length_t chunkSize, unsigned char *decodep[]);

  uint8_t _encodeMatrix[CODING_MAX_N * CODING_MAX_N];
};

#endif
