// Abstract coding scheme (reference: src/common/coding/coding.hh:15-194).
// Same virtual surface, so ChunkManager / Agent code written against the
// reference compiles unchanged against this header; the RS implementation
// behind it runs on MI355X through libnxec.
#ifndef NXEC_CODING_CODING_HH
#define NXEC_CODING_CODING_HH

#include <string>
#include <vector>

#include "chunk.hh"
#include "coding_options.hh"
#include "decoding_plan.hh"
#include "define.hh"

#define CODING_MAX_N (128)

class Coding {
 public:
  virtual ~Coding() {}

  std::string getName() const { return _name; }
  coding_param_t getN() { return _options.getN(); }
  coding_param_t getK() { return _options.getK(); }

  // geometry
  virtual num_t getNumDataChunks() = 0;
  virtual num_t getNumCodeChunks() = 0;
  virtual num_t getNumChunks() = 0;
  virtual num_t getNumChunksPerNode() = 0;
  virtual length_t getCodingStateSize() = 0;

  length_t getExtraDataSize() { return _extraDataSize; }
  bool modifyDataBuffer() { return _modifyDataBuffer; }
  bool storeCodeChunksOnly() { return _storeCodeChunksOnly; }

  // chunk size for a stripe holding dataSize bytes
  virtual length_t getChunkSize(length_t dataSize) = 0;

  // plan which chunks to fetch for a read (isRepair=false) or a repair
  virtual bool preDecode(const std::vector<chunk_id_t> &failedChunkIdx, DecodingPlan &plan, data_t *codingState,
                         bool isRepair = false) = 0;

  // data (k chunks, caller zero-padded) -> stripe of n chunks
  virtual bool encode(data_t *data, length_t dataSize, std::vector<Chunk> &stripe, data_t **codingState) = 0;

  // input chunks (sorted by id) -> all k data chunks (read) or the repair targets (repair)
  virtual bool decode(std::vector<Chunk> &inputChunks, data_t **decodedData, length_t &decodedSize,
                      DecodingPlan &plan, data_t *codingState, bool isRepair = false,
                      std::vector<chunk_id_t> repairTargets = std::vector<chunk_id_t>()) = 0;

 protected:
  Coding() : _storeCodeChunksOnly(false), _modifyDataBuffer(false), _extraDataSize(0) {}

  bool _storeCodeChunksOnly;
  bool _modifyDataBuffer;
  length_t _extraDataSize;

  CodingOptions _options;
  std::string _name;
};

#endif
