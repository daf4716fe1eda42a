// Scalar types of the Nexoedge coding layer (reference: src/common/define.hh:9-32,44-48).
#ifndef NXEC_CODING_DEFINE_HH
#define NXEC_CODING_DEFINE_HH

#include <stdint.h>

typedef uint32_t length_t;
typedef uint64_t offset_t;
typedef unsigned char data_t;
typedef uint16_t chunk_id_t;
typedef uint8_t coding_param_t;
typedef uint32_t num_t;

typedef unsigned char namespace_id_t;

#define INVALID_CHUNK_ID (int)(-1)
#define INVALID_NAMESPACE_ID (namespace_id_t)(-1)  // define.hh:28
#define CHUNK_VERSION_MAX_LEN (unsigned char)(128)  // define.hh:32

// coding schemes known to CodingGenerator (define.hh:44-48)
enum CodingScheme { RS, UNKNOWN_CODE };

#endif
