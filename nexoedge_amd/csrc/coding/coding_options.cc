// See coding_options.hh (reference semantics: coding_options.cc:6-60).
#include "coding_options.hh"

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <vector>

#include "nxec.h"

namespace {
// fixed defaults packed in one word (n | k << 8 | car << 16) so a reader never
// sees a half-updated triple; the provider, when set, takes precedence
std::atomic<uint32_t> g_fixed{0};
std::atomic<CodingOptions::DefaultsProvider> g_provider{nullptr};
}  // namespace

void CodingOptions::setDefaults(coding_param_t n, coding_param_t k, bool car) {
  g_fixed.store(static_cast<uint32_t>(n) | static_cast<uint32_t>(k) << 8 | (car ? 1u : 0u) << 16,
                std::memory_order_release);
}

void CodingOptions::setDefaultsProvider(DefaultsProvider provider) {
  g_provider.store(provider, std::memory_order_release);
}

CodingOptions::Defaults CodingOptions::defaults() {
  if (DefaultsProvider p = g_provider.load(std::memory_order_acquire)) return p();
  const uint32_t w = g_fixed.load(std::memory_order_acquire);
  return Defaults{static_cast<coding_param_t>(w & 0xff), static_cast<coding_param_t>((w >> 8) & 0xff),
                  ((w >> 16) & 1u) != 0};
}

bool CodingOptions::loadDefaults(const char *storageClassIni, const char *proxyIni, const char *storageClass) {
  int count = 0;
  if (nxec_storage_classes_load(storageClassIni, nullptr, 0, &count) != NXEC_OK) return false;
  std::vector<nxec_storage_class> classes(static_cast<size_t>(std::max(count, 1)));
  if (nxec_storage_classes_load(storageClassIni, classes.data(), static_cast<int>(classes.size()), &count) != NXEC_OK ||
      count > static_cast<int>(classes.size()))
    return false;
  const nxec_storage_class *sc = nullptr;
  for (int i = 0; i < count; i++)
    if (storageClass ? std::strcmp(classes[i].name, storageClass) == 0 : classes[i].is_default != 0) sc = &classes[i];
  if (!sc || sc->n < 1 || sc->k < 1 || sc->n > 255 || sc->k > 255) return false;
  int car = 0;
  if (proxyIni && nxec_proxy_repair_using_car(proxyIni, &car) != NXEC_OK) return false;
  setDefaults(static_cast<coding_param_t>(sc->n), static_cast<coding_param_t>(sc->k), car != 0);
  return true;
}

// coding_options.cc:6-11: the reference reads Config here
CodingOptions::CodingOptions() {
  const Defaults d = defaults();
  _n = d.n;
  _k = d.k;
  _car = d.repairUsingCAR;
}
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
