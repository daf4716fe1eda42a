// Owned byte buffer used by DecodingPlan for the repair matrix (reference:
// src/ds/byte_buffer.hh; only allocate/data/size/release are used there).
#ifndef NXEC_CODING_BYTE_BUFFER_HH
#define NXEC_CODING_BYTE_BUFFER_HH

#include <stdlib.h>

#include "define.hh"

class ByteBuffer {
 public:
  ByteBuffer() = default;
  ~ByteBuffer() { release(); }
  ByteBuffer(const ByteBuffer &) = delete;
  ByteBuffer &operator=(const ByteBuffer &) = delete;

  bool allocate(length_t n) {
    release();
    if (n == 0) return true;
    _data = static_cast<data_t *>(calloc(n, 1));
    if (!_data) return false;
    _size = n;
    return true;
  }
  data_t *data() const { return _data; }
  length_t size() const { return _size; }
  void release() {
    free(_data);
    reset();
  }
  void reset() {
    _data = nullptr;
    _size = 0;
  }

 private:
  data_t *_data = nullptr;
  length_t _size = 0;
};

#endif
