// Config bridge for the C++ surface drop-in (Option B).
//
// The reference's CodingOptions() reads n, k and the CAR flag from the Config
// singleton (src/common/coding/coding_options.cc:6-11).  ChunkManager depends
// on that: it constructs options with the default constructor and then only
// calls setN/setK (src/proxy/chunk_manager.cc:25-27, :1789-1791), so the
// `repair_using_car` setting reaches RSCode::decode (rs.cc:133,184) through
// the constructor alone.
//
// libnxec's CodingOptions() reads a registered provider instead of Config
// (the library does not link the proxy/agent configuration).  This file is
// compiled INTO the Nexoedge build, next to the other coding sources
// (src/common/coding/nxec_config_bridge.cc, added to ncloud_code's sources),
// where "../config.hh" is the reference's own Config.  Its static initializer
// registers a provider that asks Config on every construction, exactly as the
// reference constructor does, so no line of ChunkManager or Agent changes.
#include "../config.hh"
#include "coding_options.hh"

namespace {

CodingOptions::Defaults nxecConfigDefaults() {
  Config &config = Config::getInstance();
  return CodingOptions::Defaults{static_cast<coding_param_t>(config.getN()), static_cast<coding_param_t>(config.getK()),
                                 config.isRepairUsingCAR()};
}

// runs at load time of the proxy/agent binary; Config itself is only touched
// when the first CodingOptions is constructed (after Config::setConfigPath)
const bool nxecConfigBridgeRegistered = (CodingOptions::setDefaultsProvider(&nxecConfigDefaults), true);

}  // namespace
