// Owned (or borrowed) byte buffer; DecodingPlan keeps its repair matrix in one
// (reference: src/ds/byte_buffer.hh:10-177).  The whole public surface of the
// reference class, with its semantics, so the file can replace the
// reference's in a Nexoedge tree (tools/overlay_reference.sh):
//  * allocate(size, aligned): new[] or a 32-byte posix_memalign, one byte
//    even for size 0 (byte_buffer.hh:101-125); the old buffer is released
//    only after the new one exists;
//  * copy()/copyData() deep-copy, or borrow (deepCopy=false: the buffer is
//    not freed by this object, byte_buffer.hh:83-99,127-136); both refuse to
//    overwrite an allocated buffer;
//  * the copy constructor deep-copies, move assignment takes over.
#ifndef NXEC_CODING_BYTE_BUFFER_HH
#define NXEC_CODING_BYTE_BUFFER_HH

#include <stdlib.h>
#include <string.h>

#include <iostream>
#include <new>

#include "define.hh"

class ByteBuffer {
 public:
  ByteBuffer() { reset(); }
  explicit ByteBuffer(bool aligned) {
    reset();
    if (aligned) setAligned();
  }
  ByteBuffer(length_t size, bool aligned) : ByteBuffer(aligned) { allocate(size); }
  ~ByteBuffer() { release(); }

  ByteBuffer(const ByteBuffer &src) {
    reset();
    copy(src, /* deepCopy */ true);
  }
  ByteBuffer &operator=(ByteBuffer &&src) {
    if (this != &src) {
      release();
      _data = src._data;
      _size = src._size;
      _aligned = src._aligned;
      _copied = src._copied;
      src.reset();
    }
    return *this;
  }

  // alignment is a property of the next allocation; fixed once allocated
  bool setAligned() {
    if (_data != NULL) return false;
    _aligned = true;
    return true;
  }
  bool setUnaligned() {
    if (_data != NULL) return false;
    _aligned = false;
    return true;
  }

  bool copy(const ByteBuffer &src, bool deepCopy = true) { return copyData(src, deepCopy); }
  bool copySize(const ByteBuffer &src) {
    if (_data != NULL) return false;
    _size = src._size;
    return true;
  }
  bool copyData(const ByteBuffer &src, bool deepCopy = true) {
    if (_data != NULL) return false;
    if (!deepCopy) {
      _data = src._data;
      _size = src._size;
      _copied = true;  // borrowed: never freed here
      return true;
    }
    if (!allocate(src._size, src._aligned)) {
      reset();
      return false;
    }
    if (src._size > 0) memcpy(_data, src._data, src._size);
    return true;
  }
  bool setSize(length_t size) {
    if (_data != NULL) return false;
    _size = size;
    return true;
  }

  bool allocate(length_t size, bool aligned = false) {
    const size_t bytes = static_cast<size_t>(size) + (size == 0 ? 1 : 0);
    data_t *p = NULL;
    if (aligned) {
      if (posix_memalign(reinterpret_cast<void **>(&p), 32, bytes) != 0) p = NULL;
    } else {
      p = new (std::nothrow) data_t[bytes];
    }
    if (p == NULL) {
      std::cerr << "Failed to allocate aligned=" << aligned << " data of size " << size;
      return false;
    }
    release();
    _data = p;
    _size = size;
    _aligned = aligned;
    return true;
  }

  void release(bool /*freeData*/ = true) {
    if (!_copied && _data != NULL) {
      if (_aligned) free(_data);
      else delete[] _data;
    }
    reset();
  }

  data_t *data() { return _data; }
  const data_t *data() const { return _data; }
  length_t size() const { return _size; }
  bool empty() const { return _size == 0; }
  bool allocated() const { return _data != NULL; }
  bool aligned() const { return _aligned; }

  void reset() {
    _data = NULL;
    _size = 0;
    _aligned = false;
    _copied = false;
  }

 private:
  data_t *_data;
  length_t _size;
  bool _aligned;
  bool _copied;
};

#endif
