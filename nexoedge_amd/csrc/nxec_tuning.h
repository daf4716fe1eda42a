// Design-probe knobs of libnxec (the A/Bs of DESIGN.md §4 and §10).
//
// The product build (make, NXEC_DESIGN_PROBES=0) compiles every knob to its
// default below: the A/B-only branches fold away and the library reads none
// of these environment variables.  `make PROBES=1` reads each knob once from
// the environment (nxec_probes.cpp) so the measured alternatives can be
// re-run.  Deployment settings -- the few variables a production host may
// set -- are not here; INTEGRATION.md lists them with their defaults.
#ifndef NXEC_TUNING_H
#define NXEC_TUNING_H

namespace nxec {

struct Tuning {
  // coding kernels (nxec_kernels.hip)
  int lds_r = 0;              // NXEC_LDS_R: force the LDS table replication (1, 8, 16; 0 = by k)
  bool lds_single_row = false;  // NXEC_ALGO=lds: single-row passes on LDS tables, not v_perm
  bool static_order = false;  // NXEC_TILE_ORDER=static: static tile runs instead of the work queue
  int stripe_group = 0;       // NXEC_STRIPE_GROUP: stripes per column-major tile group (0 = by stride)
  // fused coding + MD5 (nxec_encode_md5.hip, nxec_files_md5.hip)
  bool fused_md5 = true;      // NXEC_FUSED_MD5=0: coding and MD5 as separate launches
  int em_stripes = 0;         // NXEC_EM_S: stripes per k_mul_md5 workgroup (0 = by batch)
  int em_prio = 0;            // NXEC_EM_PRIO: s_setprio of the hash waves
  bool em_ring = false;       // NXEC_EM_RING=1: k_mul_md5_ring, the roles decoupled by LDS counters
  int em_probe = -1;          // NXEC_EM_PROBE: k_mul_md5 role probe (outputs invalid)
  bool em_nibble = false;     // NXEC_EM_TABLES=nib: split-nibble tables
  bool em_hashsrc_global = false;  // NXEC_EM_HASHSRC=global: hash lanes read sources from L2
  int fm_probe = -1;          // NXEC_FM_PROBE: k_files_md5 role probe (outputs invalid)
  bool files_pack = true;     // NXEC_FILES_PACK=0: one request per slot
  bool files_cached_loads = true;  // NXEC_FILES_LOADS=0: streaming loads in k_files_md5
  bool files_fold = true;     // NXEC_FILES_FOLD=0: last stripes' partial chunks through the pad copy (round 4)
  int md5_depth = 2, md5_group = 8;  // NXEC_MD5_CFG=D,G[,NT]: k_md5 ring depth / blocks per group
  bool md5_nt = false;
  // host paths (nxec_agent.cpp, nxec_host_encode.cpp)
  bool nt_staging = false;    // NXEC_NT_STAGING=1: streaming stores into pinned staging and out of it
  bool host_lanes = false;    // NXEC_HOST_LANES=1: a host-pool worker set per copy direction
  int group_streams = 2;      // NXEC_GROUP_STREAMS: streams per device of an nxec_group listing it repeatedly
  int pool_admit = 8;         // NXEC_POOL_ADMIT: drop-in calls running per device at most (0 = no gate)
  bool agent_fused = true;    // NXEC_AGENT_FUSED=0: H2D -> multiply -> MD5 -> D2H batches
  bool agent_aggregate = true;  // NXEC_AGENT_AGGREGATE=0: every agent call its own round
  int agent_batch_mb = 0;     // NXEC_AGENT_BATCH_MB: staging per agent batch (0 = the caller's)
  bool agent_trace = false;   // NXEC_AGENT_TRACE: per-batch timings on stderr
  int digest_rounds = 4;      // NXEC_DIGEST_ROUNDS: zero-copy digest rounds in flight (0 = off)
  double digest_host_callers = 0;  // NXEC_DIGEST_HOST_CALLERS: auto placement's caller bound (0 = CPUs)
};

#if NXEC_DESIGN_PROBES
const Tuning &tuning();
#else
inline constexpr Tuning kProductTuning{};
constexpr const Tuning &tuning() { return kProductTuning; }
#endif

}  // namespace nxec

#endif  // NXEC_TUNING_H
