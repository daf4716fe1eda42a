// Scalar types of the Nexoedge coding layer (reference: src/common/define.hh:9-32,44-48).
//
// Inside a Nexoedge tree (tools/overlay_reference.sh) every overlaid header
// includes the reference's own src/common/define.hh first, so its guard
// __DEFINE_HH__ is set by the time this file is reached and the reference's
// definitions (enum CodingScheme at define.hh:47-50 among them) are the only
// ones: nothing here is declared twice.  Standalone (libnxec's own build, the
// tests) this file supplies the subset the coding layer uses, with the same
// types and values.
#ifndef NXEC_CODING_DEFINE_HH
#define NXEC_CODING_DEFINE_HH

#include <stdint.h>

#ifndef __DEFINE_HH__

typedef uint32_t length_t;
typedef uint64_t offset_t;
typedef unsigned char data_t;
typedef uint8_t namespace_id_t;
typedef uint16_t chunk_id_t;
typedef uint32_t version_id_t;
typedef uint8_t coding_param_t;
typedef uint32_t num_t;

#define INVALID_CHUNK_ID (int)(-1)
#define INVALID_NAMESPACE_ID (namespace_id_t)(-1)  // define.hh:28
#define CHUNK_VERSION_MAX_LEN (unsigned char)(128)  // define.hh:32

// coding schemes known to CodingGenerator (define.hh:47-50)
enum CodingScheme { RS, UNKNOWN_CODE };

#endif  // __DEFINE_HH__

#endif
