// Host CPU topology from sysfs (topology.h).
#include "topology.h"

#include <algorithm>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <utility>

namespace shmx {
namespace topo {

std::vector<int> parse_cpulist(const std::string &list) {
    std::vector<int> cpus;
    std::stringstream ss(list);
    std::string item;
    while (std::getline(ss, item, ',')) {
        if (item.empty()) continue;
        const size_t dash = item.find('-');
        const int lo = std::atoi(item.c_str());
        const int hi = dash == std::string::npos ? lo : std::atoi(item.c_str() + dash + 1);
        for (int c = lo; c <= hi && c >= 0; ++c) cpus.push_back(c);
    }
    return cpus;
}

std::vector<int> node_cpus(const std::string &sysroot, int node, const std::vector<int> &allowed) {
    if (node < 0) return {};
    std::ifstream cf(sysroot + "/devices/system/node/node" + std::to_string(node) + "/cpulist");
    std::string list;
    if (!std::getline(cf, list)) return {};
    std::vector<int> out;
    for (int c : parse_cpulist(list))
        if (std::find(allowed.begin(), allowed.end(), c) != allowed.end()) out.push_back(c);
    return out;
}

std::vector<std::vector<int>> cache_domains(const std::string &sysroot, const std::vector<int> &cpus) {
    std::vector<std::pair<std::string, std::vector<int>>> doms;   // L3 shared_cpu_list -> CPUs
    for (int c : cpus) {
        const std::string base = sysroot + "/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index";
        std::string dom;
        for (int idx = 0; idx < 8 && dom.empty(); ++idx) {
            std::ifstream lv(base + std::to_string(idx) + "/level");
            int level = 0;
            if (!(lv >> level) || level != 3) continue;   // (index directories may have gaps)
            std::ifstream sh(base + std::to_string(idx) + "/shared_cpu_list");
            std::getline(sh, dom);
        }
        if (dom.empty()) return {};
        auto it = std::find_if(doms.begin(), doms.end(), [&](const auto &d) { return d.first == dom; });
        if (it == doms.end()) doms.push_back({dom, {c}});
        else it->second.push_back(c);
    }
    std::vector<std::vector<int>> out;
    for (auto &d : doms) out.push_back(std::move(d.second));
    return out;
}

int cgroup_cpu_quota(const std::string &cgroot) {
    long long quota = -1, period = 0;
    {
        std::ifstream v2(cgroot + "/cpu.max");
        std::string q;
        if (v2 >> q >> period) quota = q == "max" ? -1 : std::atoll(q.c_str());
    }
    if (period <= 0) {
        std::ifstream qf(cgroot + "/cpu/cpu.cfs_quota_us"), pf(cgroot + "/cpu/cpu.cfs_period_us");
        if (!(qf >> quota) || !(pf >> period)) return 0;
    }
    if (quota <= 0 || period <= 0) return 0;
    return (int)((quota + period - 1) / period);
}

std::vector<std::vector<int>> plan_copy_threads(unsigned want, int budget, int pes_on_host, int rank,
                                                const std::vector<std::vector<int>> &domains) {
    unsigned n = want < 2 ? 2 : want;
    if (budget > 0 && pes_on_host > 0) {
        const unsigned share = (unsigned)(budget / pes_on_host);
        n = std::max(2u, std::min(n, share));
    }
    std::vector<std::vector<int>> out(n);
    if (domains.empty()) return out;
    const size_t nd = domains.size(), base = (size_t)(rank < 0 ? 0 : rank) * n;
    for (unsigned i = 0; i < n; ++i) out[i] = domains[(base + i) % nd];
    return out;
}

}  // namespace topo
}  // namespace shmx
