// Factory (reference: src/common/coding/coding_generator.hh:13-24): returns
// nullptr when the scheme is unknown or the parameters are rejected.
#ifndef NXEC_CODING_GENERATOR_HH
#define NXEC_CODING_GENERATOR_HH

#include <cstdio>
#include <exception>

#include "rs.hh"

class CodingGenerator {
 public:
  static Coding *genCoding(int codingScheme, CodingOptions options) {
    try {
      if (codingScheme == CodingScheme::RS) return new RSCode(options);
    } catch (std::exception &e) {
      std::fprintf(stderr, "Failed to init coding, %s\n", e.what());
      return nullptr;
    }
    return nullptr;
  }
};

#endif
