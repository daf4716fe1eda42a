// Stateless GF(2^8) matrix x chunks helper used by the agent for partial
// encodes and repairs (reference: src/common/coding/coding_util.hh:10-32,
// called at container_manager.cc:251 and agent.cc:339).  Runs on MI355X.
#ifndef NXEC_CODING_UTIL_HH
#define NXEC_CODING_UTIL_HH

#include <vector>

#include "nxec.h"

class CodingUtils {
 public:
  // contiguous form: data = numDataChunks x chunkSize, code = numCodeChunks x chunkSize
  static bool encode(unsigned char *data, int numDataChunks, unsigned char *code, int numCodeChunks, int chunkSize,
                     unsigned char *matrix) {
    std::vector<const unsigned char *> in(numDataChunks > 0 ? numDataChunks : 1);
    std::vector<unsigned char *> out(numCodeChunks > 0 ? numCodeChunks : 1);
    for (int i = 0; i < numDataChunks; i++) in[i] = data + static_cast<long>(i) * chunkSize;
    for (int i = 0; i < numCodeChunks; i++) out[i] = code + static_cast<long>(i) * chunkSize;
    return nxec_encode_host(chunkSize, numDataChunks, numCodeChunks, matrix, in.data(), out.data()) == NXEC_OK;
  }
  // pointer-array form
  static bool encode(unsigned char **data, int numDataChunks, unsigned char **code, int numCodeChunks, int chunkSize,
                     unsigned char *matrix) {
    return nxec_encode_host(chunkSize, numDataChunks, numCodeChunks, matrix, data, code) == NXEC_OK;
  }
};

#endif
