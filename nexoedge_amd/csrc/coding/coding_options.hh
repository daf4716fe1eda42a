// Coding parameters (reference: src/common/coding/coding_options.{hh,cc}).
//
// The reference's default constructor pulls n, k and the CAR flag out of the
// Config singleton (coding_options.cc:6-11), and ChunkManager relies on that:
// it builds its options with the default constructor plus setN/setK
// (chunk_manager.cc:25-27, :1789-1791), so the CAR flag reaches RSCode only
// through the constructor.  The coding library cannot link Config (boost INI
// reader, the whole proxy/agent configuration), so the default constructor
// reads a process-wide *defaults source* instead:
//
//   * a provider function, registered once (integration/config_bridge.cc
//     registers one that returns Config::getInstance().getN()/getK()/
//     isRepairUsingCAR(), evaluated at every construction exactly like the
//     reference), or
//   * fixed values from setDefaults(), or
//   * n = k = 0, CAR off when neither was set.
//
// Both setters are thread-safe; construction never blocks on them.
#ifndef NXEC_CODING_OPTIONS_HH
#define NXEC_CODING_OPTIONS_HH

#include <string>

#include "define.hh"

class CodingOptions {
 public:
  struct Defaults {
    coding_param_t n;
    coding_param_t k;
    bool repairUsingCAR;
  };
  typedef Defaults (*DefaultsProvider)();

  CodingOptions();  // n, k, CAR from the defaults source (coding_options.cc:6-11)
  CodingOptions(coding_param_t n, coding_param_t k, bool repairUsingCAR = false);
  ~CodingOptions();

  void setRepairUsingCAR();
  bool repairUsingCAR();
  bool setN(coding_param_t n);
  bool setK(coding_param_t k);
  coding_param_t getN();
  coding_param_t getK();
  std::string str(bool withRuntimeOptions = false);

  // ---- process-wide defaults source of the default constructor
  static void setDefaults(coding_param_t n, coding_param_t k, bool repairUsingCAR);
  static void setDefaultsProvider(DefaultsProvider provider);  // nullptr: back to setDefaults' values
  static Defaults defaults();                                  // what CodingOptions() would read now
  // setDefaults from the reference's INI files without its Config: n and k of
  // storage class `storageClass` (nullptr: the `default = 1` class) of a
  // storage_class.ini, the CAR flag from proxy.ini's misc.repair_using_car
  // (nullptr: off).  false (defaults unchanged) when a file is unreadable or
  // malformed, the class is missing, or its n / k do not fit coding_param_t.
  static bool loadDefaults(const char *storageClassIni, const char *proxyIni = nullptr,
                           const char *storageClass = nullptr);

 private:
  coding_param_t _n = 0;
  coding_param_t _k = 0;
  bool _car = false;
};

#endif
