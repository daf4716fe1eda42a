// See coding_options.hh (reference semantics: coding_options.cc:6-60).
#include "coding_options.hh"

CodingOptions::CodingOptions() = default;
CodingOptions::CodingOptions(coding_param_t n, coding_param_t k, bool car) : _n(n), _k(k), _car(car) {}
CodingOptions::~CodingOptions() = default;

void CodingOptions::setRepairUsingCAR() { _car = true; }
bool CodingOptions::repairUsingCAR() { return _car; }

// zero is rejected, anything else accepted (coding_options.cc:22-46)
bool CodingOptions::setK(coding_param_t k) {
  if (k == 0) return false;
  _k = k;
  return true;
}
bool CodingOptions::setN(coding_param_t n) {
  if (n == 0) return false;
  _n = n;
  return true;
}
coding_param_t CodingOptions::getN() { return _n; }
coding_param_t CodingOptions::getK() { return _k; }

// "n-k" plus the CAR flag digit on request (coding_options.cc:48-59)
std::string CodingOptions::str(bool withRuntimeOptions) {
  std::string s = std::to_string(_n) + "-" + std::to_string(_k);
  if (withRuntimeOptions) s += std::to_string(_car ? 1 : 0);
  return s;
}
