// Coding parameters (reference: src/common/coding/coding_options.{hh,cc}).
// The reference constructor pulls n, k and the CAR flag from the Config
// singleton (coding_options.cc:6-11); here they are constructor arguments,
// since the INI config lives in the proxy/agent, outside the coding path.
#ifndef NXEC_CODING_OPTIONS_HH
#define NXEC_CODING_OPTIONS_HH

#include <string>

#include "define.hh"

class CodingOptions {
 public:
  CodingOptions();
  CodingOptions(coding_param_t n, coding_param_t k, bool repairUsingCAR = false);
  ~CodingOptions();

  void setRepairUsingCAR();
  bool repairUsingCAR();
  bool setN(coding_param_t n);
  bool setK(coding_param_t k);
  coding_param_t getN();
  coding_param_t getK();
  std::string str(bool withRuntimeOptions = false);

 private:
  coding_param_t _n = 0;
  coding_param_t _k = 0;
  bool _car = false;
};

#endif
