// Decoding / repair plan produced by Coding::preDecode (reference:
// src/common/coding/decoding_plan.hh:10-99): ids of the chunks to fetch, how
// many of them are needed, and for repairs the e x k repair matrix that the
// proxy hands to agents (chunk_manager.cc:929-1015).
#ifndef NXEC_CODING_DECODING_PLAN_HH
#define NXEC_CODING_DECODING_PLAN_HH

#include <vector>

#include "byte_buffer.hh"
#include "define.hh"

class DecodingPlan {
 public:
  DecodingPlan() = default;
  ~DecodingPlan() { release(); }

  void release() {
    releaseRepairMatrix();
    releaseInputChunks();
  }

  bool allocateRepairMatrix(length_t n) { return _repair.allocate(n); }
  data_t *getRepairMatrix() { return _repair.data(); }
  length_t getRepairMatrixSize() { return _repair.size(); }
  void releaseRepairMatrix() { _repair.release(); }

  void addInputChunkId(chunk_id_t id) { _inputs.push_back(id); }
  std::vector<chunk_id_t> getInputChunkIds() const { return _inputs; }
  size_t getNumInputChunks() const { return _inputs.size(); }
  size_t getMinNumInputChunks() const { return _minInputs; }
  void releaseInputChunks() {
    _inputs.clear();
    _minInputs = 0;
  }
  bool setMinNumInputChunks(num_t n) {
    if (n > getNumInputChunks()) return false;
    _minInputs = n;
    return true;
  }

 private:
  ByteBuffer _repair;
  std::vector<chunk_id_t> _inputs;
  num_t _minInputs = 0;
};

#endif
