// Host view of the HBM symmetric heap: block states, page protection and the
// fault handler (mirror.h).  Host-only: the copies go through a Backend.
#include "mirror.h"

#include <linux/futex.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstring>

namespace shmx {
namespace mirror {

namespace {

struct View {
    char *base = nullptr;
    char *alias = nullptr;      // the same pages, always read-write
    size_t bytes = 0;
    size_t nblocks = 0;
    uint8_t *state = nullptr;   // one State per block (mmap'd: no allocator in the handler)
    // device writes in flight per block (begin_device_write .. end_device_write)
    uint16_t *pending = nullptr;
    Backend be{};
    // the last write fault's run, so a sequential writer unprotects growing
    // runs instead of faulting once per block
    size_t run_end = ~size_t(0);
    size_t run_len = 0;
    size_t fetch_end = ~size_t(0);   // the same for loads of DEVICE_NEWER blocks
    size_t fetch_len = 0;
    Stats st{};
} g_view;

std::atomic_flag g_lock = ATOMIC_FLAG_INIT;
struct sigaction g_prev_segv;
bool g_installed = false;

// The fault service: one request slot, because the handler holds the lock
// while it waits.  kIdle -> kAsked (handler) -> kDone (service) -> kIdle.
enum { kIdle = 0, kAsked = 1, kDone = 2, kStop = 3 };
std::atomic<int> g_req{kIdle};
size_t g_req_b0 = 0, g_req_nb = 0;
pthread_t g_service;
bool g_service_up = false;

void futex_wait(std::atomic<int> *a, int v) {
    syscall(SYS_futex, reinterpret_cast<int *>(a), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
void futex_wake(std::atomic<int> *a) {
    syscall(SYS_futex, reinterpret_cast<int *>(a), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
}

void *service_main(void *) {
    for (;;) {
        const int r = g_req.load(std::memory_order_acquire);
        if (r == kStop) return nullptr;
        if (r != kAsked) {
            futex_wait(&g_req, r);
            continue;
        }
        g_view.be.to_host((uint64_t)g_req_b0 * kBlock, g_req_nb * kBlock, g_view.be.ctx);
        g_req.store(kDone, std::memory_order_release);
        futex_wake(&g_req);
    }
}

struct Guard {
    Guard() {
        while (g_lock.test_and_set(std::memory_order_acquire)) {
        }
    }
    ~Guard() { g_lock.clear(std::memory_order_release); }
};

void protect(size_t b0, size_t nb, int prot) {
    if (nb) mprotect(g_view.base + b0 * kBlock, nb * kBlock, prot);
}

size_t block_of(uint64_t off) { return (size_t)(off / kBlock); }

// Blocks [b0, b0 + nb) of the device segment -> host view (through the
// alias: the view stays inaccessible until the bytes are there), then CLEAN.
// From the fault handler the copy runs on the service thread (the handler
// only stores, loads and sleeps on a futex); elsewhere in the caller's.
void fetch_run(size_t b0, size_t nb, bool in_handler) {
    if (in_handler && g_service_up && !pthread_equal(pthread_self(), g_service)) {
        g_req_b0 = b0;
        g_req_nb = nb;
        g_req.store(kAsked, std::memory_order_release);
        futex_wake(&g_req);
        for (int r; (r = g_req.load(std::memory_order_acquire)) != kDone;) futex_wait(&g_req, r);
        g_req.store(kIdle, std::memory_order_relaxed);
    } else {
        g_view.be.to_host((uint64_t)b0 * kBlock, nb * kBlock, g_view.be.ctx);
    }
    protect(b0, nb, PROT_READ);
    std::memset(g_view.state + b0, CLEAN, nb);
    g_view.st.blocks_fetched += nb;
}

void on_segv(int sig, siginfo_t *si, void *uc) {
    if (handle_fault(si->si_addr)) return;
    // not a fault of the host view: whatever was installed before
    if (g_prev_segv.sa_flags & SA_SIGINFO) {
        if (g_prev_segv.sa_sigaction) {
            g_prev_segv.sa_sigaction(sig, si, uc);
            return;
        }
    } else if (g_prev_segv.sa_handler != SIG_DFL && g_prev_segv.sa_handler != SIG_IGN) {
        g_prev_segv.sa_handler(sig);
        return;
    }
    // default action: the access faults again and the process dies on it
    signal(SIGSEGV, SIG_DFL);
}

}  // namespace

bool create(size_t bytes, const Backend &be) {
    if (g_view.base || !bytes) return false;
    const size_t nblocks = (bytes + kBlock - 1) / kBlock;
    const size_t vbytes = nblocks * kBlock;
    const int fd = memfd_create("shmemx_mirror", MFD_CLOEXEC);
    if (fd < 0) return false;
    if (ftruncate(fd, (off_t)vbytes) != 0) {
        close(fd);
        return false;
    }
    void *p = mmap(nullptr, vbytes, PROT_READ, MAP_SHARED, fd, 0);
    void *a = mmap(nullptr, vbytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);   // the mappings keep the pages
    void *s = mmap(nullptr, nblocks, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    void *w = mmap(nullptr, nblocks * sizeof(uint16_t), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS,
                   -1, 0);
    if (p == MAP_FAILED || a == MAP_FAILED || s == MAP_FAILED || w == MAP_FAILED) {
        if (p != MAP_FAILED) munmap(p, vbytes);
        if (a != MAP_FAILED) munmap(a, vbytes);
        if (s != MAP_FAILED) munmap(s, nblocks);
        if (w != MAP_FAILED) munmap(w, nblocks * sizeof(uint16_t));
        return false;
    }
    g_view.base = static_cast<char *>(p);
    g_view.alias = static_cast<char *>(a);
    g_view.bytes = vbytes;
    g_view.nblocks = nblocks;
    g_view.state = static_cast<uint8_t *>(s);   // zero: every block CLEAN
    g_view.pending = static_cast<uint16_t *>(w);
    g_view.be = be;
    g_view.run_end = g_view.fetch_end = ~size_t(0);
    g_view.run_len = g_view.fetch_len = 0;
    g_view.st = Stats{};
    g_req.store(kIdle);
    g_service_up = pthread_create(&g_service, nullptr, service_main, nullptr) == 0;
    // a forked child has no service thread: its faults copy in place (and
    // fail loudly if the GPU runtime is unusable there) instead of waiting
    // for a thread that does not exist
    static bool atfork_set = false;
    if (!atfork_set) atfork_set = pthread_atfork(nullptr, nullptr, [] { g_service_up = false; }) == 0;
    if (!g_installed) {
        struct sigaction sa;
        std::memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = on_segv;
        sa.sa_flags = SA_SIGINFO | SA_NODEFER;
        sigemptyset(&sa.sa_mask);
        sigaction(SIGSEGV, &sa, &g_prev_segv);
        g_installed = true;
    }
    return true;
}

void install_handler(const struct sigaction *prev) {
    if (!g_view.base) {
        if (prev) sigaction(SIGSEGV, prev, nullptr);
        return;
    }
    if (prev && (prev->sa_flags & SA_SIGINFO) && prev->sa_sigaction == on_segv) {
        sigaction(SIGSEGV, prev, nullptr);    // ours, with its own chain
    } else {
        struct sigaction sa;
        std::memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = on_segv;
        sa.sa_flags = SA_SIGINFO | SA_NODEFER;
        sigemptyset(&sa.sa_mask);
        sigaction(SIGSEGV, &sa, nullptr);
        if (prev) g_prev_segv = *prev;
        else std::memset(&g_prev_segv, 0, sizeof g_prev_segv);   // SIG_DFL
    }
    g_installed = true;
}

void destroy() {
    if (!g_view.base) return;
    if (g_service_up) {
        g_req.store(kStop, std::memory_order_release);
        futex_wake(&g_req);
        pthread_join(g_service, nullptr);
        g_service_up = false;
    }
    if (g_installed) {
        // put back what was there before, unless someone installed a handler
        // over ours since (it chains to ours, which then finds no view)
        struct sigaction cur;
        if (sigaction(SIGSEGV, nullptr, &cur) == 0 && (cur.sa_flags & SA_SIGINFO) &&
            cur.sa_sigaction == on_segv)
            sigaction(SIGSEGV, &g_prev_segv, nullptr);
        g_installed = false;
    }
    munmap(g_view.base, g_view.bytes);
    munmap(g_view.alias, g_view.bytes);
    munmap(g_view.state, g_view.nblocks);
    munmap(g_view.pending, g_view.nblocks * sizeof(uint16_t));
    g_view = View{};
}

bool active() { return g_view.base != nullptr; }
char *host_base() { return g_view.base; }
char *alias_base() { return g_view.alias; }
size_t view_bytes() { return g_view.bytes; }

bool contains(const void *p, size_t bytes) {
    const char *c = static_cast<const char *>(p);
    return g_view.base && c >= g_view.base && c < g_view.base + g_view.bytes &&
           bytes <= (size_t)(g_view.base + g_view.bytes - c);
}

uint64_t offset_of(const void *p) { return (uint64_t)(static_cast<const char *>(p) - g_view.base); }

namespace {

// flush() with the lock held
size_t flush_locked(uint64_t off, size_t bytes) {
    const size_t b0 = block_of(off), b1 = block_of(off + bytes - 1) + 1;
    size_t copied = 0;
    for (size_t b = b0; b < b1 && b < g_view.nblocks;) {
        if (g_view.state[b] != HOST_NEWER) {
            ++b;
            continue;
        }
        size_t e = b;
        while (e < b1 && e < g_view.nblocks && g_view.state[e] == HOST_NEWER) ++e;
        // read-only first, then CLEAN, then the copy: a store another thread
        // makes from here faults, waits for the lock, and finds the block
        // CLEAN (HOST_NEWER again, flushed by the next collective)
        protect(b, e - b, PROT_READ);
        std::memset(g_view.state + b, CLEAN, e - b);
        g_view.be.to_device((uint64_t)b * kBlock, (e - b) * kBlock, g_view.be.ctx);
        copied += e - b;
        b = e;
    }
    if (copied) g_view.be.drain(g_view.be.ctx);
    g_view.st.blocks_flushed += copied;
    if (copied) g_view.run_end = ~size_t(0);
    return copied;
}

// Blocks [b0, b1) become DEVICE_NEWER (no host access), lock held.
size_t mark_device_newer(size_t b0, size_t b1) {
    size_t n = 0;
    for (size_t b = b0; b < b1;) {
        if (g_view.state[b] == DEVICE_NEWER) {
            ++b;
            continue;
        }
        size_t e = b;
        while (e < b1 && g_view.state[e] != DEVICE_NEWER) ++e;
        protect(b, e - b, PROT_NONE);
        std::memset(g_view.state + b, DEVICE_NEWER, e - b);
        n += e - b;
        b = e;
    }
    g_view.st.blocks_device_newer += n;
    return n;
}

}  // namespace

size_t flush(uint64_t off, size_t bytes) {
    if (!g_view.base || !bytes) return 0;
    Guard g;
    return flush_locked(off, bytes);
}

size_t begin_device_write(uint64_t off, size_t bytes, bool *fresh) {
    if (!g_view.base || !bytes) return 0;
    Guard g;
    flush_locked(off, bytes);
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    const size_t n = mark_device_newer(b0, b1);
    for (size_t b = b0; b < b1; ++b) ++g_view.pending[b];
    if (fresh) *fresh = n == b1 - b0;
    return n;
}

void end_device_write(uint64_t off, size_t bytes) {
    if (!g_view.base || !bytes) return;
    Guard g;
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    for (size_t b = b0; b < b1; ++b)
        if (g_view.pending[b]) --g_view.pending[b];
}

size_t settle(uint64_t off, size_t bytes, bool fresh, bool copied) {
    if (!g_view.base || !bytes) return 0;
    Guard g;
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    for (size_t b = b0; b < b1; ++b)   // another write in flight, or a block already back
        if (g_view.pending[b] || g_view.state[b] != DEVICE_NEWER) return 0;
    if (!fresh) {
        fetch_run(b0, b1 - b0, false);
        return (b1 - b0) * kBlock;
    }
    // the rest of every block already equals HBM: only the written bytes
    // move, and their writer has completed (the caller's contract); with
    // `copied` the call's stream has put them into the alias already
    if (!copied)
        (g_view.be.to_host_done ? g_view.be.to_host_done : g_view.be.to_host)(off, bytes, g_view.be.ctx);
    protect(b0, b1 - b0, PROT_READ);
    std::memset(g_view.state + b0, CLEAN, b1 - b0);
    g_view.st.blocks_settled += b1 - b0;
    return copied ? 0 : bytes;
}

size_t flush_bytes(uint64_t off, size_t bytes) {
    if (!g_view.base || !bytes) return 0;
    Guard g;
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    const uint64_t end = off + bytes;
    size_t touched = 0;
    for (size_t b = b0; b < b1;) {
        if (g_view.state[b] != HOST_NEWER) {
            ++b;
            continue;
        }
        size_t e = b;
        while (e < b1 && g_view.state[e] == HOST_NEWER) ++e;
        // the operand's bytes inside blocks [b, e)
        const uint64_t lo = std::max<uint64_t>(off, (uint64_t)b * kBlock);
        const uint64_t hi = std::min<uint64_t>(end, (uint64_t)e * kBlock);
        g_view.be.to_device(lo, hi - lo, g_view.be.ctx);
        touched += e - b;
        b = e;
    }
    if (touched) g_view.be.drain(g_view.be.ctx);
    g_view.st.blocks_flushed += touched;
    return touched;
}

bool view_current(uint64_t off, size_t bytes) {
    if (!g_view.base || !bytes) return false;
    Guard g;
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    for (size_t b = b0; b < b1; ++b)
        if (g_view.state[b] == DEVICE_NEWER || g_view.pending[b]) return false;
    return true;
}

bool begin_light_write(uint64_t off, size_t bytes) {
    if (!g_view.base || !bytes) return false;
    Guard g;
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    for (size_t b = b0; b < b1; ++b)
        if (g_view.state[b] == DEVICE_NEWER || g_view.pending[b]) return false;
    for (size_t b = b0; b < b1; ++b) ++g_view.pending[b];
    return true;
}

size_t end_light_write(uint64_t off, size_t bytes, bool copied) {
    if (!g_view.base || !bytes) return 0;
    Guard g;
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    // the result's bytes into the alias first (if the call's stream did not),
    // then the write ends: a block another writer marked DEVICE_NEWER in the
    // meantime is fetched only after this (its fault waits for pending)
    if (!copied) g_view.be.to_host(off, bytes, g_view.be.ctx);
    for (size_t b = b0; b < b1; ++b)
        if (g_view.pending[b]) --g_view.pending[b];
    g_view.st.blocks_settled += b1 - b0;
    return copied ? 0 : bytes;
}

size_t device_wrote(uint64_t off, size_t bytes) {
    if (!g_view.base || !bytes) return 0;
    Guard g;
    // HOST_NEWER here would lose host stores: flush() runs first
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    return mark_device_newer(b0, b1);
}

size_t acquire(uint64_t off, size_t bytes, bool write) {
    if (!g_view.base || !bytes) return 0;
    Guard g;
    const size_t b0 = block_of(off), b1 = std::min(block_of(off + bytes - 1) + 1, g_view.nblocks);
    size_t fetched = 0;
    for (size_t b = b0; b < b1;) {
        size_t e = b;
        while (e < b1 && g_view.state[e] == g_view.state[b]) ++e;
        if (g_view.state[b] == DEVICE_NEWER) {
            fetch_run(b, e - b, false);
            fetched += e - b;
        }
        if (write && g_view.state[b] == CLEAN) {
            protect(b, e - b, PROT_READ | PROT_WRITE);
            std::memset(g_view.state + b, HOST_NEWER, e - b);
        }
        b = e;
    }
    return fetched;
}

void fetch_all() {
    if (!g_view.base) return;
    Guard g;
    for (size_t b = 0; b < g_view.nblocks;) {
        if (g_view.state[b] != DEVICE_NEWER) {
            ++b;
            continue;
        }
        size_t e = b;
        while (e < g_view.nblocks && g_view.state[e] == DEVICE_NEWER) ++e;
        fetch_run(b, e - b, false);
        b = e;
    }
}

bool handle_fault(void *addr) {
    if (!contains(addr, 1)) return false;
    bool waited = false;
    for (;; sched_yield()) {      // the lock is not held across the yield
        Guard g;
        const size_t b = block_of(offset_of(addr));
        switch (g_view.state[b]) {
        case DEVICE_NEWER: {
            if (g_view.pending[b]) {
                // a collective writing this block is being enqueued or run:
                // its result is not recorded yet, so fetching now would read
                // the old bytes; retry once that write has ended (writes to
                // other blocks do not hold this fault up)
                waited = true;
                continue;
            }
            // a load or a store of a block a collective wrote: bring it (and
            // the DEVICE_NEWER blocks right after it) back; a store faults
            // once more
            size_t want = 1;
            if (b == g_view.fetch_end) want = std::min(kMaxFetchRun, 2 * g_view.fetch_len);
            size_t e = b;
            // the run stops at a block with a write in flight: its bytes in
            // HBM are not the collective's yet
            while (e < g_view.nblocks && e - b < want && g_view.state[e] == DEVICE_NEWER && !g_view.pending[e])
                ++e;
            fetch_run(b, e - b, true);
            g_view.fetch_end = e;
            g_view.fetch_len = e - b;
            g_view.st.read_faults += 1;
            g_view.st.fault_waits += waited ? 1 : 0;
            return true;
        }
        case CLEAN: {
            // a store (CLEAN pages are readable): host newer from here; a
            // sequential writer gets runs that double up to kMaxWriteRun
            size_t want = 1;
            if (b == g_view.run_end) want = std::min(kMaxWriteRun, 2 * g_view.run_len);
            size_t e = b;
            while (e < g_view.nblocks && e - b < want && g_view.state[e] == CLEAN) ++e;
            protect(b, e - b, PROT_READ | PROT_WRITE);
            std::memset(g_view.state + b, HOST_NEWER, e - b);
            g_view.run_end = e;
            g_view.run_len = e - b;
            g_view.st.write_faults += 1;
            g_view.st.fault_waits += waited ? 1 : 0;
            return true;
        }
        default:
            // already HOST_NEWER (another thread resolved it first)
            protect(b, 1, PROT_READ | PROT_WRITE);
            return true;
        }
    }
}

Stats stats(bool reset) {
    Guard g;
    const Stats s = g_view.st;
    if (reset) g_view.st = Stats{};
    return s;
}

State state_of(uint64_t off) {
    if (!g_view.base || off >= g_view.bytes) return CLEAN;
    return static_cast<State>(g_view.state[block_of(off)]);
}

}  // namespace mirror
}  // namespace shmx
