// Intra-node shared block, host barrier and IPC peer mappings (node.h).
#include "node.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "state.h"

namespace shmx {
namespace node {

namespace {

struct RegionSlot {
    hipIpcMemHandle_t handle;
    uint64_t bytes;
    std::atomic<uint64_t> gen;   // 0 = never published
};

struct PeSlot {
    RegionSlot region[kNumRegions];
    Desc desc;
    std::atomic<int> vote;       // agree()
    std::atomic<int> gpu_numa;   // the GPU's NUMA node + 1 (0 = unknown)
    std::atomic<uint64_t> gpu_id;   // a hash of the GPU's PCI bus id (0 = unknown)
};

struct Shared {
    PeSlot pe[kMaxPes];
    // flag[to][from]: barriers `from` has entered together with `to`
    std::atomic<uint64_t> flag[kMaxPes][kMaxPes];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "lock-free 64-bit atomics needed");

struct Mapping {
    char *base = nullptr;
    uint64_t gen = 0;
    uint64_t bytes = 0;
};

struct Node {
    Shared *sh = nullptr;
    std::string name, xname;   // the block's and the exchange's /dev/shm names
    uint64_t hash = 0;
    char *xchg = nullptr;      // the exchange block: host mapping, device address
    char *xchg_dev = nullptr;
    // exchange calls so far with each PE, and the readers of this PE's
    // previous call with the pair counts of that call
    uint64_t xcount[kMaxPes] = {};
    int xlast_n = 0;
    int xlast_pe[kMaxPes] = {};
    uint64_t xlast_count[kMaxPes] = {};
    int pe = 0, npes = 0;
    uint64_t entered[kMaxPes] = {};     // barriers entered with each peer
    char *own[kNumRegions] = {};
    Mapping peer[kNumRegions][kMaxPes];
} g_node;

double barrier_timeout_s() {
    static const double t = [] {
        const char *e = std::getenv("SHMEMX_BARRIER_TIMEOUT");
        const double v = e ? std::atof(e) : 0.0;
        return v > 0 ? v : 600.0;
    }();
    return t;
}

char g_ipc_error[160] = "no IPC error";

// Waiting for a peer, by elapsed time: spin for the first 200 us (a barrier
// between busy PEs completes in microseconds, and a sleep — even a 5 us
// nanosleep, which the kernel's timer slack stretches to ~55 us — would add
// more than the whole barrier costs), then yield up to 10 ms, then sleep in
// 50 us steps, so PEs that wait long (more PE processes than free CPUs, a
// peer still copying) do not take the CPU from the ones doing the work.
struct Backoff {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    double waited_s = 0;
    void step() {
        if ((++spins & 63) == 0)
            waited_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (waited_s < 200e-6) {
            __builtin_ia32_pause();
        } else if (waited_s < 10e-3) {
            sched_yield();
        } else {
            struct timespec ts = {0, 50 * 1000};
            nanosleep(&ts, nullptr);
        }
    }
};

void close_peer(Region r, int q) {
    Mapping &mp = g_node.peer[r][q];
    if (mp.base) (void)hipIpcCloseMemHandle(mp.base);
    mp = Mapping{};
}

}  // namespace

bool up() { return g_node.sh != nullptr; }

bool attach(int pe, int npes, const void *key, size_t keylen) {
    if (g_node.sh) return true;
    if (npes < 1 || npes > kMaxPes || pe < 0 || pe >= npes) return false;
    // FNV-1a of the job id: a fresh name per job, so no stale block is reused
    uint64_t h = 1469598103934665603ull;
    const unsigned char *k = static_cast<const unsigned char *>(key);
    for (size_t i = 0; i < keylen; ++i) h = (h ^ k[i]) * 1099511628211ull;
    char name[64];
    snprintf(name, sizeof name, "/shmemx_node_%016llx", (unsigned long long)h);
    const int fd = shm_open(name, O_RDWR | O_CREAT, 0600);
    if (fd < 0) return false;
    // every PE sizes it; a fresh object reads as zeros
    if (ftruncate(fd, sizeof(Shared)) != 0) {
        close(fd);
        return false;
    }
    void *p = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return false;
    g_node.sh = static_cast<Shared *>(p);
    g_node.name = name;
    g_node.hash = h;
    g_node.pe = pe;
    g_node.npes = npes;
    std::memset(g_node.entered, 0, sizeof g_node.entered);
    trace(LOG_INIT, "node block %s attached (%zu bytes)", name, sizeof(Shared));
    return true;
}

void unlink_name() {
    if (g_node.sh && !g_node.name.empty()) shm_unlink(g_node.name.c_str());
    g_node.name.clear();
    if (!g_node.xname.empty()) shm_unlink(g_node.xname.c_str());
    g_node.xname.clear();
}

namespace {
// the slots, then done[reader][writer]
constexpr size_t kXchgDoneOff = kMaxPes * kXchgSlotBytes;
constexpr size_t kXchgBytes = kXchgDoneOff + kMaxPes * kMaxPes * sizeof(uint64_t);
std::atomic<uint64_t> &xchg_word(size_t off, int a, int b) {
    return reinterpret_cast<std::atomic<uint64_t> *>(g_node.xchg + off)[(size_t)a * kMaxPes + b];
}
void xchg_detach() {
    if (!g_node.xchg) return;
    if (g_node.xchg_dev) (void)hipHostUnregister(g_node.xchg);
    munmap(g_node.xchg, kXchgBytes);
    g_node.xchg = g_node.xchg_dev = nullptr;
}
}  // namespace

bool xchg_attach() {
    if (g_node.xchg_dev) return true;
    if (!g_node.sh) return false;
    char name[64];
    snprintf(name, sizeof name, "/shmemx_xchg_%016llx", (unsigned long long)g_node.hash);
    const int fd = shm_open(name, O_RDWR | O_CREAT, 0600);
    if (fd < 0) return false;
    g_node.xname = name;
    if (ftruncate(fd, kXchgBytes) != 0) {
        close(fd);
        return false;
    }
    void *p = mmap(nullptr, kXchgBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return false;
    g_node.xchg = static_cast<char *>(p);
    // page-locked and mapped into the GPU's address space: the service
    // workgroups of every member read and write it over PCIe
    void *d = nullptr;
    if (hipHostRegister(p, kXchgBytes, hipHostRegisterMapped) != hipSuccess ||
        hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
        (void)hipGetLastError();
        trace(LOG_INIT, "small-call exchange %s: page-locking failed", name);
        xchg_detach();
        return false;
    }
    g_node.xchg_dev = static_cast<char *>(d);
    trace(LOG_INIT, "small-call exchange %s (%zu bytes) at %p, device %p", name, kXchgBytes, p, d);
    return true;
}

char *xchg_host(int q) {
    return g_node.xchg_dev && q >= 0 && q < kMaxPes ? g_node.xchg + (size_t)q * kXchgSlotBytes : nullptr;
}

char *xchg_dev(int q) {
    return g_node.xchg_dev && q >= 0 && q < kMaxPes ? g_node.xchg_dev + (size_t)q * kXchgSlotBytes : nullptr;
}

void xchg_claim(int start, int step, int P, uint64_t *counts) {
    const int me = g_node.pe;
    Backoff bo;
    for (int i = 0; i < g_node.xlast_n; ++i) {
        const int r = g_node.xlast_pe[i];
        while (xchg_word(kXchgDoneOff, r, me).load(std::memory_order_acquire) < g_node.xlast_count[i]) {
            bo.step();
            if (bo.waited_s > barrier_timeout_s()) {
                char why[96];
                snprintf(why, sizeof why, "PE %d never finished reading this PE's exchange slot", r);
                fatal("node exchange", why);
            }
        }
    }
    int n = 0;
    for (int i = 0; i < P; ++i) {
        const int q = start + i * step;
        counts[i] = q == me ? 0 : ++g_node.xcount[q];
        if (q != me) {
            g_node.xlast_pe[n] = q;
            g_node.xlast_count[n++] = counts[i];
        }
    }
    g_node.xlast_n = n;
}

void xchg_finish(int start, int step, int P, const uint64_t *counts) {
    for (int i = 0; i < P; ++i) {
        const int q = start + i * step;
        if (q != g_node.pe) xchg_word(kXchgDoneOff, g_node.pe, q).store(counts[i], std::memory_order_release);
    }
}

void detach(bool unlink) {
    if (!g_node.sh) return;
    xchg_detach();
    for (int r = 0; r < kNumRegions; ++r)
        for (int q = 0; q < kMaxPes; ++q) close_peer(static_cast<Region>(r), q);
    if (unlink) unlink_name();
    munmap(g_node.sh, sizeof(Shared));
    g_node = Node{};
}

void barrier(int start, int step, int P) {
    Shared *sh = g_node.sh;
    if (!sh || P <= 1) return;
    const int me = g_node.pe;
    for (int i = 0; i < P; ++i) {
        const int q = start + i * step;
        if (q == me) continue;
        ++g_node.entered[q];
        sh->flag[q][me].fetch_add(1, std::memory_order_acq_rel);
    }
    Backoff bo;
    for (int i = 0; i < P; ++i) {
        const int q = start + i * step;
        if (q == me) continue;
        while (sh->flag[me][q].load(std::memory_order_acquire) < g_node.entered[q]) {
            bo.step();
            if (bo.waited_s > barrier_timeout_s()) {
                char why[96];
                snprintf(why, sizeof why, "PE %d never reached the barrier", q);
                fatal("node barrier", why);
            }
        }
    }
}

void publish(Region r, void *base, size_t bytes) {
    if (!g_node.sh) return;
    RegionSlot &s = g_node.sh->pe[g_node.pe].region[r];
    const hipError_t e = hipIpcGetMemHandle(&s.handle, base);
    if (e != hipSuccess) {
        // Not fatal: the region stays usable here, and a peer that tries to
        // map it sees bytes == 0 and fails its call collectively (DIRECT's
        // vote) or gets NULL (shmemx_heap_ptr).  The generation still moves,
        // so nobody keeps a mapping of what was published before.
        (void)hipGetLastError();
        trace(LOG_MEMORY, "hipIpcGetMemHandle(%s at %p): %s; peers cannot map it",
              r == kHeap ? "heap" : "scratch", base, hipGetErrorString(e));
        std::memset(&s.handle, 0, sizeof s.handle);
        bytes = 0;
    }
    s.bytes = bytes;
    s.gen.fetch_add(1, std::memory_order_release);
    g_node.own[r] = static_cast<char *>(base);
}

void unpublish(Region r) {
    if (!g_node.sh) return;
    g_node.own[r] = nullptr;
}

char *peer_base(Region r, int q) {
    if (!g_node.sh || q < 0 || q >= g_node.npes) return nullptr;
    if (q == g_node.pe) return g_node.own[r];
    RegionSlot &s = g_node.sh->pe[q].region[r];
    const uint64_t gen = s.gen.load(std::memory_order_acquire);
    if (gen == 0) {
        snprintf(g_ipc_error, sizeof g_ipc_error, "PE %d has not published its %s", q,
                 r == kHeap ? "heap" : "scratch");
        return nullptr;
    }
    Mapping &mp = g_node.peer[r][q];
    if (mp.base && mp.gen == gen) return mp.base;
    close_peer(r, q);
    if (s.bytes == 0) {
        snprintf(g_ipc_error, sizeof g_ipc_error, "PE %d could not export its %s", q,
                 r == kHeap ? "heap" : "scratch");
        return nullptr;
    }
    void *p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, s.handle, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        snprintf(g_ipc_error, sizeof g_ipc_error, "hipIpcOpenMemHandle(PE %d, %s, gen %llu): %s", q,
                 r == kHeap ? "heap" : "scratch", (unsigned long long)gen, hipGetErrorString(e));
        trace(LOG_MEMORY, "%s", g_ipc_error);
        return nullptr;
    }
    mp.base = static_cast<char *>(p);
    mp.gen = gen;
    mp.bytes = s.bytes;
    trace(LOG_MEMORY, "mapped PE %d's %s (%llu bytes) at %p", q, r == kHeap ? "heap" : "scratch",
          (unsigned long long)s.bytes, p);
    return mp.base;
}

const char *last_ipc_error() { return g_ipc_error; }

uint64_t region_gen(Region r, int q) {
    if (!g_node.sh || q < 0 || q >= g_node.npes) return 0;
    return g_node.sh->pe[q].region[r].gen.load(std::memory_order_acquire);
}

bool agree(int start, int step, int P, bool ok) {
    Shared *sh = g_node.sh;
    if (!sh || P <= 1) return ok;
    sh->pe[g_node.pe].vote.store(ok ? 1 : 0, std::memory_order_release);
    barrier(start, step, P);
    bool all = true;
    for (int i = 0; i < P; ++i)
        all &= sh->pe[start + i * step].vote.load(std::memory_order_acquire) != 0;
    barrier(start, step, P);   // every vote is read before any member votes again
    return all;
}

size_t peer_bytes(Region r, int q) {
    if (!g_node.sh || q < 0 || q >= g_node.npes) return 0;
    return g_node.sh->pe[q].region[r].bytes;
}

void put_desc(const Desc &d) {
    if (g_node.sh) g_node.sh->pe[g_node.pe].desc = d;   // published by the next barrier
}

Desc get_desc(int q) {
    return g_node.sh ? g_node.sh->pe[q].desc : Desc{};
}

void put_gpu_numa(int nd) {
    if (g_node.sh) g_node.sh->pe[g_node.pe].gpu_numa.store(nd < 0 ? 0 : nd + 1, std::memory_order_release);
}

void put_gpu_id(uint64_t id) {
    if (g_node.sh) g_node.sh->pe[g_node.pe].gpu_id.store(id, std::memory_order_release);
}

bool gpu_shared() {
    if (!g_node.sh) return false;
    const uint64_t mine = g_node.sh->pe[g_node.pe].gpu_id.load(std::memory_order_acquire);
    if (!mine) return false;
    for (int q = 0; q < g_node.npes; ++q)
        if (q != g_node.pe && g_node.sh->pe[q].gpu_id.load(std::memory_order_acquire) == mine) return true;
    return false;
}

int gpu_numa(int q) {
    if (!g_node.sh || q < 0 || q >= g_node.npes) return -1;
    return g_node.sh->pe[q].gpu_numa.load(std::memory_order_acquire) - 1;
}

int npes() { return g_node.sh ? g_node.npes : 0; }

}  // namespace node
}  // namespace shmx
