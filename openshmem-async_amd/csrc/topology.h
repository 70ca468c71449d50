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

// The CPUs the process's cgroup may use at once: ceil(quota / period) from
// cgroup v2 "<cgroot>/cpu.max" ("max 100000" = no limit) or cgroup v1
// "<cgroot>/cpu/cpu.cfs_quota_us" and "cpu.cfs_period_us" (-1 = no limit);
// 0 when there is no limit or it cannot be read.
int cgroup_cpu_quota(const std::string &cgroot);

// The staging copy threads of one PE on a node shared with other PEs
// (staging.cpp), as CPU sets per thread:
//   want       threads one PE would take alone (8);
//   budget     CPUs the whole job may keep busy (the cgroup quota, else the
//              allowed CPUs), shared by the pes_on_host PEs;
//   domains    the cache domains of the NUMA node of this PE's GPU;
//   rank       this PE's position among the PEs whose GPUs share that node.
// threads = min(want, budget / pes_on_host), at least 2 (one per gang); thread
// i runs in domains[(rank * threads + i) % domains.size()], so the PEs on one
// NUMA node take different domains while there are enough of them (every PE
// used to put its thread i on domain i).  Empty per-thread sets (unknown
// topology) leave the threads unpinned.
std::vector<std::vector<int>> plan_copy_threads(unsigned want, int budget, int pes_on_host, int rank,
                                                const std::vector<std::vector<int>> &domains);

}  // namespace topo
}  // namespace shmx
