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
  // pointer-array form.  NXEC_CHUNK_MD5=2: the outputs' digests come from the
  // same GPU pass and wait for Chunk::computeMD5 on this thread (the agent's
  // RPR_CHUNK_REQ hashes its outputs next, agent.cc:339-343; include/nxec.h §6b)
  static bool encode(unsigned char **data, int numDataChunks, unsigned char **code, int numCodeChunks, int chunkSize,
                     unsigned char *matrix) {
    if (nxec_chunk_md5_mode() < 2 || numCodeChunks < 1 || chunkSize <= 0)
      return nxec_encode_host(chunkSize, numDataChunks, numCodeChunks, matrix, data, code) == NXEC_OK;
    std::vector<unsigned char> md5(static_cast<size_t>(numCodeChunks) * 16);
    nxec_digest_clear();
    if (nxec_encode_host_md5(chunkSize, numDataChunks, numCodeChunks, matrix, data, code, nullptr, md5.data()) !=
        NXEC_OK)
      return false;
    for (int i = 0; i < numCodeChunks; i++) nxec_digest_note(code[i], chunkSize, md5.data() + 16 * i);
    return true;
  }
};

#endif
