// CPU test of the copy threads' placement logic (csrc/topology.cpp): a fake
// sysfs tree shaped like the MI355X hosts' (2 NUMA nodes, 8 L3 domains of 8
// cores x 2 hardware threads per node, CPU numbering 0-63,128-191 on node 0)
// and, if present, the real /sys of this machine.
//
//   test_topology FAKE_ROOT      prints "ok <checks>"
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <set>
#include <string>
#include <vector>

#include "topology.h"

using namespace shmx::topo;

static int checks = 0, fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        ++checks;                                                       \
        if (!(c)) {                                                     \
            ++fails;                                                    \
            std::printf("FAIL line %d: %s\n", __LINE__, #c);            \
        }                                                               \
    } while (0)

static void mkdirs(const std::string &p) {
    std::string cur;
    for (size_t i = 0; i < p.size(); ++i) {
        cur += p[i];
        if (p[i] == '/' || i + 1 == p.size()) mkdir(cur.c_str(), 0755);
    }
}

static void put(const std::string &path, const std::string &text) {
    mkdirs(path.substr(0, path.rfind('/')));
    std::ofstream(path) << text << "\n";
}

static std::string range(int lo, int hi) { return std::to_string(lo) + "-" + std::to_string(hi); }

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const std::string root = argv[1];

    // parse_cpulist
    CHECK(parse_cpulist("0-3,8,10-11") == (std::vector<int>{0, 1, 2, 3, 8, 10, 11}));
    CHECK(parse_cpulist("") .empty());
    CHECK(parse_cpulist("5") == std::vector<int>{5});
    CHECK(parse_cpulist("7,") == std::vector<int>{7});

    // the fake host: node n owns cores 64n..64n+63 and their siblings 128+64n..
    for (int n = 0; n < 2; ++n)
        put(root + "/devices/system/node/node" + std::to_string(n) + "/cpulist",
            range(64 * n, 64 * n + 63) + "," + range(128 + 64 * n, 128 + 64 * n + 63));
    for (int c = 0; c < 256; ++c) {
        const int core = c % 128, dom = core / 8;   // 16 domains of 8 cores
        const std::string base = root + "/devices/system/cpu/cpu" + std::to_string(c) + "/cache/";
        put(base + "index0/level", "1");
        put(base + "index0/shared_cpu_list", std::to_string(core) + "," + std::to_string(core + 128));
        put(base + "index2/level", "2");
        put(base + "index2/shared_cpu_list", std::to_string(core) + "," + std::to_string(core + 128));
        put(base + "index3/level", "3");
        put(base + "index3/shared_cpu_list",
            range(8 * dom, 8 * dom + 7) + "," + range(128 + 8 * dom, 128 + 8 * dom + 7));
    }
    std::vector<int> all;
    for (int c = 0; c < 256; ++c) all.push_back(c);

    // node_cpus: the node's CPUs, restricted to the allowed ones
    const std::vector<int> n1 = node_cpus(root, 1, all);
    CHECK(n1.size() == 128 && n1.front() == 64 && n1.back() == 255);
    CHECK(node_cpus(root, 1, {1, 2, 70, 200, 300}) == (std::vector<int>{70, 200}));
    CHECK(node_cpus(root, 2, all).empty());    // no such node
    CHECK(node_cpus(root, -1, all).empty());

    // cache_domains: node 1 -> 8 domains, in order, each its 8 cores + siblings
    const auto d = cache_domains(root, n1);
    CHECK(d.size() == 8);
    bool shape = d.size() == 8;
    for (size_t i = 0; shape && i < d.size(); ++i) {
        const int lo = 64 + 8 * (int)i;
        shape = d[i].size() == 16 && d[i].front() == lo && d[i][7] == lo + 7 && d[i][8] == lo + 128;
    }
    CHECK(shape);
    // a restricted allowed set keeps only its own domains' CPUs
    const auto d2 = cache_domains(root, node_cpus(root, 1, {64, 65, 80, 200}));
    CHECK(d2.size() == 3 && d2[0] == (std::vector<int>{64, 65}) && d2[1] == std::vector<int>{80} &&
          d2[2] == std::vector<int>{200});
    // a CPU whose L3 is unknown: topology unknown, empty
    CHECK(cache_domains(root, {64, 999}).empty());
    CHECK(cache_domains(root, {}).empty());

    // cgroup_cpu_quota: v2 cpu.max, v1 cfs files, no limit
    put(root + "/cg2/cpu.max", "1600000 100000");
    CHECK(cgroup_cpu_quota(root + "/cg2") == 16);
    put(root + "/cg2b/cpu.max", "150000 100000");       // 1.5 CPUs: 2 busy at most
    CHECK(cgroup_cpu_quota(root + "/cg2b") == 2);
    put(root + "/cg2c/cpu.max", "max 100000");
    CHECK(cgroup_cpu_quota(root + "/cg2c") == 0);
    put(root + "/cg1/cpu/cpu.cfs_quota_us", "800000");
    put(root + "/cg1/cpu/cpu.cfs_period_us", "100000");
    CHECK(cgroup_cpu_quota(root + "/cg1") == 8);
    put(root + "/cg1n/cpu/cpu.cfs_quota_us", "-1");
    put(root + "/cg1n/cpu/cpu.cfs_period_us", "100000");
    CHECK(cgroup_cpu_quota(root + "/cg1n") == 0);
    CHECK(cgroup_cpu_quota(root + "/nowhere") == 0);

    // plan_copy_threads: one PE alone keeps 8 threads, one per domain of its
    // GPU's node, in domain order
    {
        const auto p = plan_copy_threads(8, 16, 1, 0, d);
        CHECK(p.size() == 8);
        bool ok = p.size() == 8;
        for (size_t i = 0; ok && i < p.size(); ++i) ok = p[i] == d[i];
        CHECK(ok);
    }
    // 8 PEs on the host (4 per NUMA node, as an 8-GPU MI355X node), a 16-CPU
    // quota: 2 threads each, 16 in all; the 4 PEs of one node cover its 8
    // domains with no two threads on one domain
    {
        size_t total = 0;
        for (int node = 0; node < 2; ++node) {
            const auto dn = cache_domains(root, node_cpus(root, node, all));
            std::set<int> firsts;
            for (int rank = 0; rank < 4; ++rank) {
                const auto p = plan_copy_threads(8, 16, 8, rank, dn);
                CHECK(p.size() == 2);
                total += p.size();
                for (const auto &cpus : p) {
                    CHECK(!cpus.empty());
                    if (!cpus.empty()) CHECK(firsts.insert(cpus.front()).second);   // a fresh domain
                }
            }
            CHECK(firsts.size() == 8);
        }
        CHECK(total <= 16);
    }
    // 8 PEs on one node's GPU (the one-GPU rehearsal): 2 threads each over 8
    // domains, each domain twice at most (16 threads, 8 domains)
    {
        std::vector<int> uses(256, 0);
        for (int rank = 0; rank < 8; ++rank)
            for (const auto &cpus : plan_copy_threads(8, 16, 8, rank, d)) uses[cpus.front()]++;
        int most = 0;
        for (int u : uses) most = u > most ? u : most;
        CHECK(most == 2);
    }
    // a quota smaller than 2 per PE still leaves one thread per gang; no
    // quota information (budget 0) keeps the per-PE count; unknown topology:
    // unpinned threads
    CHECK(plan_copy_threads(8, 4, 8, 3, d).size() == 2);
    CHECK(plan_copy_threads(8, 0, 8, 3, d).size() == 8);
    {
        const auto p = plan_copy_threads(8, 64, 2, 1, {});
        CHECK(p.size() == 8 && p[0].empty() && p[7].empty());
    }
    // 2 PEs with 32 CPUs: 8 each, the second PE's 8 after the first's (wrapping)
    {
        const auto p0 = plan_copy_threads(8, 32, 2, 0, d), p1 = plan_copy_threads(8, 32, 2, 1, d);
        CHECK(p0.size() == 8 && p1.size() == 8 && p1[0] == d[0] && p0[0] == d[0]);
    }

    // this machine's /sys, when it has one: the domains partition the node's CPUs
    std::ifstream probe("/sys/devices/system/node/node0/cpulist");
    if (probe) {
        std::vector<int> real_all;
        for (int c = 0; c < 4096; ++c) real_all.push_back(c);
        const std::vector<int> cpus = node_cpus("/sys", 0, real_all);
        const auto rd = cache_domains("/sys", cpus);
        size_t total = 0;
        std::set<int> seen;
        for (const auto &x : rd) {
            total += x.size();
            seen.insert(x.begin(), x.end());
        }
        CHECK(rd.empty() || (total == cpus.size() && seen.size() == cpus.size()));
    }
    if (fails) return 1;
    std::printf("ok %d\n", checks);
    return 0;
}
