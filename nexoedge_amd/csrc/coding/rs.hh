// Reed-Solomon code over GF(2^8) on MI355X (reference: src/common/coding/rs.hh).
// Method semantics follow rs.cc line for line (see rs.cc here for citations);
// the byte work goes to libnxec's gfx950 kernels via include/nxec.h.
#ifndef NXEC_CODING_RS_HH
#define NXEC_CODING_RS_HH

#include <stdint.h>

#include "coding.hh"
#include "nxec.h"

class RSCode : public Coding {
 public:
  explicit RSCode(CodingOptions options);
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

 private:
  bool carRepairFinalize(unsigned char *inputp[], num_t numInputChunks, length_t chunkSize, unsigned char *decodep[]);

  uint8_t _encodeMatrix[CODING_MAX_N * CODING_MAX_N];
};

#endif
