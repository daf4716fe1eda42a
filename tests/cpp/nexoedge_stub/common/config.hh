// Test double of the one Config interface nexoedge_amd/integration/
// nxec_config_bridge.cc uses (the reference's src/common/config.hh:16-19,
// 91-92, 102: getInstance, getN, getK, isRepairUsingCAR).  It lives at
// common/config.hh so the bridge's "../config.hh" resolves from
// common/coding/ exactly as in the Nexoedge source tree.  The values are set
// by the test, standing in for storage_class.ini / general.ini.
#ifndef NXEC_TEST_STUB_CONFIG_HH
#define NXEC_TEST_STUB_CONFIG_HH

#include <string>

class Config {
 public:
  static Config &getInstance() {
    static Config instance;
    return instance;
  }
  int getN(std::string storageClass = "") const { return storageClass.empty() || storageClass == _class ? _n : 0; }
  int getK(std::string storageClass = "") const { return storageClass.empty() || storageClass == _class ? _k : 0; }
  bool isRepairUsingCAR() const { return _car; }
  bool isRepairAtProxy() const { return _atProxy; }

  // test-only setters
  void set(const std::string &storageClass, int n, int k, bool car, bool atProxy) {
    _class = storageClass;
    _n = n;
    _k = k;
    _car = car;
    _atProxy = atProxy;
  }

 private:
  Config() = default;
  std::string _class = "STANDARD";
  int _n = 0, _k = 0;
  bool _car = false, _atProxy = true;
};

#endif
