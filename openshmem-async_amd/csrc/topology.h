// Host CPU topology for placing the staging copy threads (staging.cpp):
// CPU lists, NUMA nodes and last-level-cache domains read from sysfs under a
// root directory ("/sys" in the library, a fake tree in
// tests/native/test_topology.cpp).  Host-only: no HIP.
#pragma once

#include <string>
#include <vector>

namespace shmx {
namespace topo {

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}
std::vector<int> parse_cpulist(const std::string &list);

// CPUs of NUMA node `node` that are also in `allowed` (in node order), or
// empty if the node is unknown.
std::vector<int> node_cpus(const std::string &sysroot, int node, const std::vector<int> &allowed);

// `cpus` grouped by the last-level (L3) cache they share, domains in order of
// their first CPU in `cpus`, each domain's CPUs in `cpus` order; empty if any
// CPU's L3 cannot be read (topology unknown).
std::vector<std::vector<int>> cache_domains(const std::string &sysroot, const std::vector<int> &cpus);

}  // namespace topo
}  // namespace shmx
