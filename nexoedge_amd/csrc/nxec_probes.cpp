// Design-probe knobs read from the environment -- `make PROBES=1` only (see
// nxec_tuning.h; the product build compiles this file to nothing).
#include "nxec_tuning.h"

#if NXEC_DESIGN_PROBES
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace nxec {

namespace {
const char *knob(const char *name) { return std::getenv(name); }

Tuning read_tuning() {
  Tuning t;
  const char *e;
  if ((e = knob("NXEC_LDS_R"))) t.lds_r = std::atoi(e);
  if ((e = knob("NXEC_ALGO"))) t.lds_single_row = std::strcmp(e, "lds") == 0;
  if ((e = knob("NXEC_TILE_ORDER"))) t.static_order = std::strcmp(e, "static") == 0;
  if ((e = knob("NXEC_STRIPE_GROUP"))) t.stripe_group = std::atoi(e);
  if ((e = knob("NXEC_FUSED_MD5"))) t.fused_md5 = e[0] != '0';
  if ((e = knob("NXEC_EM_S"))) t.em_stripes = std::atoi(e);
  if ((e = knob("NXEC_EM_PRIO"))) t.em_prio = std::atoi(e);
  if ((e = knob("NXEC_EM_RING"))) t.em_ring = e[0] == '1';
  if ((e = knob("NXEC_EM_PROBE"))) t.em_probe = std::atoi(e);
  if ((e = knob("NXEC_EM_TABLES"))) t.em_nibble = e[0] == 'n';
  if ((e = knob("NXEC_EM_HASHSRC"))) t.em_hashsrc_global = e[0] == 'g';
  if ((e = knob("NXEC_FM_PROBE"))) t.fm_probe = std::atoi(e);
  if ((e = knob("NXEC_FILES_PACK"))) t.files_pack = e[0] != '0';
  if ((e = knob("NXEC_FILES_LOADS"))) t.files_cached_loads = e[0] != '0';
  if ((e = knob("NXEC_FILES_FOLD"))) t.files_fold = e[0] != '0';
  if ((e = knob("NXEC_MD5_CFG"))) {
    int d = 2, g = 8, nt = 0;
    if (std::sscanf(e, "%d,%d,%d", &d, &g, &nt) >= 2) t.md5_depth = d, t.md5_group = g, t.md5_nt = nt != 0;
  }
  if ((e = knob("NXEC_NT_STAGING"))) t.nt_staging = e[0] == '1';
  if ((e = knob("NXEC_HOST_LANES"))) t.host_lanes = e[0] == '1';
  if ((e = knob("NXEC_GROUP_STREAMS"))) t.group_streams = std::max(1, std::atoi(e));
  if ((e = knob("NXEC_POOL_ADMIT"))) t.pool_admit = std::max(0, std::atoi(e));
  if ((e = knob("NXEC_AGENT_FUSED"))) t.agent_fused = e[0] != '0';
  if ((e = knob("NXEC_AGENT_AGGREGATE"))) t.agent_aggregate = e[0] != '0';
  if ((e = knob("NXEC_AGENT_BATCH_MB"))) t.agent_batch_mb = std::atoi(e);
  if ((e = knob("NXEC_AGENT_TRACE"))) t.agent_trace = true;
  if ((e = knob("NXEC_DIGEST_ROUNDS"))) t.digest_rounds = std::atoi(e);
  if ((e = knob("NXEC_DIGEST_HOST_CALLERS"))) t.digest_host_callers = std::atof(e);
  return t;
}
}  // namespace

// re-read on every call: a probe run may change a knob between two calls
const Tuning &tuning() {
  thread_local Tuning t;
  t = read_tuning();
  return t;
}

}  // namespace nxec

#endif  // NXEC_DESIGN_PROBES
