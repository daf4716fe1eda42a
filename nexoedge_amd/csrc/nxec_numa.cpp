// NUMA placement of a GPU's host work (one host thread +
// hipSetDevice + streams per GPU).  The 8-GPU node is a 2-socket host
// (BENCH cpu_baseline.host: EPYC 9575F x 2); each GPU hangs off one socket's
// PCIe root, and the pinned staging, the arena chunks and the host worker
// pool of the rank (or group thread) driving that GPU should sit on that
// socket's memory and cores -- otherwise every staged byte and every
// zero-copy PCIe access of the GPU crosses the inter-socket link too.
//
// The mapping is read from sysfs the way the kernel exports it:
//   <root>/sys/bus/pci/devices/<domain:bus:dev.fn>/numa_node  ("-1" = unknown)
//   <root>/sys/devices/system/node/node<N>/cpulist            ("0-63,128-191")
// <root> is NXEC_SYSFS_ROOT (tests point it at a fake tree), default "".
// Binding intersects the node's CPUs with the thread's current affinity (a
// container's cpuset may hide some) and leaves the affinity alone when that
// is empty or the node is unknown.  No exec, no process re-launch.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "nxec_internal.h"

namespace {

std::string sysfs_root() {
  const char *e = std::getenv("NXEC_SYSFS_ROOT");
  return e ? std::string(e) : std::string();
}

bool read_line(const std::string &path, std::string *out) {
  std::ifstream f(path);
  if (!f) return false;
  std::getline(f, *out);
  return true;
}

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}; false on malformed text
bool parse_cpulist(const std::string &s, std::vector<int> *cpus) {
  cpus->clear();
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    while (!part.empty() && std::isspace(static_cast<unsigned char>(part.back()))) part.pop_back();
    while (!part.empty() && std::isspace(static_cast<unsigned char>(part.front()))) part.erase(part.begin());
    if (part.empty()) continue;
    char *end = nullptr;
    const long lo = std::strtol(part.c_str(), &end, 10);
    long hi = lo;
    if (*end == '-') hi = std::strtol(end + 1, &end, 10);
    if (*end != '\0' || lo < 0 || hi < lo || hi >= CPU_SETSIZE) return false;
    for (long c = lo; c <= hi; c++) cpus->push_back(static_cast<int>(c));
  }
  return true;
}

}  // namespace

namespace nxec {

// CPUs of the NUMA node the PCI device sits on (empty: unknown); *node = -1 when unknown
std::vector<int> pci_node_cpus(const char *bus_id, int *node) {
  *node = -1;
  std::vector<int> cpus;
  if (!bus_id) return cpus;
  std::string id(bus_id);
  for (char &c : id) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  std::string line;
  if (!read_line(sysfs_root() + "/sys/bus/pci/devices/" + id + "/numa_node", &line)) return cpus;
  const int nd = std::atoi(line.c_str());
  if (nd < 0) return cpus;
  *node = nd;
  if (!read_line(sysfs_root() + "/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist", &line) ||
      !parse_cpulist(line, &cpus))
    cpus.clear();
  return cpus;
}

// binds the calling thread to cpus ∩ its current affinity; false when that is empty
bool bind_thread_cpus(const std::vector<int> &cpus) {
  if (cpus.empty()) return false;
  cpu_set_t cur, want;
  CPU_ZERO(&want);
  if (pthread_getaffinity_np(pthread_self(), sizeof(cur), &cur) != 0) return false;
  int n = 0;
  for (int c : cpus)
    if (c < CPU_SETSIZE && CPU_ISSET(c, &cur)) {
      CPU_SET(c, &want);
      n++;
    }
  return n > 0 && pthread_setaffinity_np(pthread_self(), sizeof(want), &want) == 0;
}

// CPUs of NUMA node `node` (empty: unknown)
std::vector<int> node_cpus(int node) {
  std::vector<int> cpus;
  std::string line;
  if (node < 0 || !read_line(sysfs_root() + "/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", &line) ||
      !parse_cpulist(line, &cpus))
    cpus.clear();
  return cpus;
}

// NUMA node of a CPU (-1: unknown), from the nodes' cpulists, read once
int cpu_numa_node(int cpu) {
  static const std::vector<int> node_of = [] {
    std::vector<int> v;
    std::string line;
    std::vector<int> cpus;
    for (int nd = 0; nd < 64; nd++) {
      if (!read_line(sysfs_root() + "/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist", &line) ||
          !parse_cpulist(line, &cpus))
        continue;
      for (int c : cpus) {
        if (static_cast<size_t>(c) >= v.size()) v.resize(c + 1, -1);
        v[c] = nd;
      }
    }
    return v;
  }();
  return cpu >= 0 && static_cast<size_t>(cpu) < node_of.size() ? node_of[cpu] : -1;
}

int device_bus_id(int device, char *buf, int len) {
  const hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(e == hipErrorNoDevice ? NXEC_ERR_NODEV : NXEC_ERR_HIP, "hipDeviceGetPCIBusId(%d): %s", device,
                     hipGetErrorString(e));
  }
  return NXEC_OK;
}

}  // namespace nxec

extern "C" {

int nxec_pci_numa_node(const char *bus_id, int *node) {
  if (!bus_id || !node) return nxec::set_error(NXEC_ERR_INVALID, "nxec_pci_numa_node: null argument");
  (void)nxec::pci_node_cpus(bus_id, node);
  return NXEC_OK;
}

int nxec_numa_node_cpus(int node, int *cpus, int max, int *count) {
  if (node < 0 || !count || (max > 0 && !cpus)) return nxec::set_error(NXEC_ERR_INVALID, "nxec_numa_node_cpus: invalid arguments");
  std::string line;
  std::vector<int> v;
  if (!read_line(sysfs_root() + "/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", &line) ||
      !parse_cpulist(line, &v))
    return nxec::set_error(NXEC_ERR_INVALID, "nxec_numa_node_cpus: no cpulist for node %d", node);
  *count = static_cast<int>(v.size());
  for (int i = 0; i < max && i < *count; i++) cpus[i] = v[i];
  return NXEC_OK;
}

int nxec_bind_thread_to_pci(const char *bus_id, int *node) {
  if (!bus_id) return nxec::set_error(NXEC_ERR_INVALID, "nxec_bind_thread_to_pci: null bus id");
  int nd = -1;
  const std::vector<int> cpus = nxec::pci_node_cpus(bus_id, &nd);
  const bool bound = nxec::bind_thread_cpus(cpus);
  if (node) *node = bound ? nd : -1;
  return NXEC_OK;
}

int nxec_device_numa_node(int device, int *node) {
  if (!node) return nxec::set_error(NXEC_ERR_INVALID, "nxec_device_numa_node: null node");
  *node = -1;
  char bus[64] = {0};
  if (int rc = nxec::device_bus_id(device, bus, sizeof(bus))) return rc;
  return nxec_pci_numa_node(bus, node);
}

int nxec_bind_thread_to_device(int device, int *node) {
  if (node) *node = -1;
  char bus[64] = {0};
  if (int rc = nxec::device_bus_id(device, bus, sizeof(bus))) return rc;
  return nxec_bind_thread_to_pci(bus, node);
}

}  // extern "C"
