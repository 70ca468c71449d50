// Host test of the intra-node block (openshmem-async_amd/csrc/node.cpp) with
// real processes: N forked PEs attach one block and run the same random
// sequence of collectives on random active sets (PE_start, stride, size);
// non-members skip, as in OpenSHMEM.  Each collective checks
//   * the barrier property: every member arrived before any member leaves;
//   * descriptor exchange: after the entry barrier every member reads every
//     other member's descriptor of THIS call (then an exit barrier, as
//     shmemx_verify does);
//   * node::agree: every member gets the AND of the members' votes (the
//     collective failure path of DIRECT's peer mappings).
// No GPU: only the shared block, the pairwise counters and the descriptors.
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "shmem_reduce_mi355x.h"
#include "node.h"

// The two runtime hooks node.cpp calls (runtime.cpp in the library).
namespace shmx {
void trace(int, const char *, ...) {}
[[noreturn]] void fatal(const char *what, const char *detail) {
    std::fprintf(stderr, "FATAL %s: %s\n", what, detail);
    std::abort();
}
}  // namespace shmx

struct Set {
    int start, step, size;
};

int main(int argc, char **argv) {
    const int npes = argc > 1 ? std::atoi(argv[1]) : 6;
    const int ncalls = argc > 2 ? std::atoi(argv[2]) : 3000;
    // the same call sequence on every PE
    std::mt19937 rng(777);
    std::vector<Set> calls;
    for (int c = 0; c < ncalls; ++c) {
        const int step = 1 << (rng() % 3);
        const int start = (int)(rng() % npes);
        const int maxsize = (npes - 1 - start) / step + 1;
        calls.push_back(Set{start, step, 1 + (int)(rng() % maxsize)});
    }
    auto *arrived = static_cast<std::atomic<int> *>(mmap(nullptr, sizeof(std::atomic<int>) * ncalls,
                                                         PROT_READ | PROT_WRITE,
                                                         MAP_SHARED | MAP_ANONYMOUS, -1, 0));
    for (int c = 0; c < ncalls; ++c) new (&arrived[c]) std::atomic<int>(0);
    unsigned char key[16];
    for (int i = 0; i < 16; ++i) key[i] = (unsigned char)(getpid() >> (i % 4 * 8)) ^ (unsigned char)i;
    std::vector<pid_t> kids;
    for (int pe = 0; pe < npes; ++pe) {
        const pid_t k = fork();
        if (k == 0) {
            if (!shmx::node::attach(pe, npes, key, sizeof key)) _exit(10);
            shmx::node::barrier(0, 1, npes);
            int bad = 0;
            for (int c = 0; c < ncalls && !bad; ++c) {
                const Set &s = calls[c];
                const int idx = pe - s.start;
                if (idx < 0 || idx % s.step || idx / s.step >= s.size) continue;
                shmx::node::Desc d;
                d.aux = (uint64_t)c * 1000 + pe;
                shmx::node::put_desc(d);
                arrived[c].fetch_add(1);
                shmx::node::barrier(s.start, s.step, s.size);
                if (arrived[c].load() != s.size) bad = 1;
                for (int i = 0; i < s.size; ++i) {
                    const int q = s.start + i * s.step;
                    if (shmx::node::get_desc(q).aux != (uint64_t)c * 1000 + q) bad = 2;
                }
                shmx::node::barrier(s.start, s.step, s.size);
                if (c % 3 == 0) {
                    // collective AND: on some calls the last member votes no
                    const bool last = idx / s.step == s.size - 1;
                    const bool no = c % 2 == 0 && last;
                    const bool want = !(c % 2 == 0);
                    if (shmx::node::agree(s.start, s.step, s.size, !no) != want) bad = 3;
                }
            }
            shmx::node::barrier(0, 1, npes);
            shmx::node::detach(pe == 0);
            _exit(bad);
        }
        kids.push_back(k);
    }
    int fails = 0;
    for (pid_t k : kids) {
        int st = 0;
        waitpid(k, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) ++fails;
    }
    if (fails) {
        std::printf("FAIL %d PEs\n", fails);
        return 1;
    }
    std::printf("ok %d %d\n", npes, ncalls);
    return 0;
}
