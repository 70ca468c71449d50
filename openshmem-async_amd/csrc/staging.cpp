// Host-resident operands of the blocking entry points: the reference's
// symmetric heap is host memory (memory/symmem.c:168-227, dlmalloc), so
// target and source may live there.  They are staged over PCIe: small arrays
// bounce through page-locked buffers with one wait; large ones go in chunks,
// H2D on one copy stream, the reduction on the library stream, D2H on a
// second copy stream, so both PCIe directions and the device work overlap
// (DESIGN.md §6).  Pageable memory goes through a page-locked ring filled and
// emptied by a pool of CPU threads.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <fstream>
#include <sstream>
#include <string>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "heap.h"
#include "internal.h"
#include "shmem_reduce_mi355x.h"
#include "node.h"
#include "state.h"
#include "stage_plan.h"
#include "topology.h"

namespace shmx {

// Host-resident arrays move over PCIe in chunks of this size (pipelined);
// up to kSmallHostBytes they bounce through page-locked buffers instead.
constexpr size_t kStageChunkBytes = size_t(16) << 20;
constexpr size_t kSmallHostBytes = size_t(256) << 10;
constexpr size_t kRingSlots = 4;     // page-locked bounce slots per direction

// ------------------------------------------- page-locked ring, copy pool
// Pageable host arrays (dlmalloc'd heaps, numpy) cannot be DMA'd
// asynchronously; they go through kRingSlots page-locked slots per direction,
// filled and emptied by a small pool of CPU threads, so the CPU copies of
// one chunk overlap the PCIe transfers and device work of its neighbours.
// (A THP-backed ring registered with hipHostRegister measured the same:
// profiles/r05_e2e_nt.txt.)
void ring_free() {
    if (!g_state.ring) return;
    (void)hipHostFree(g_state.ring);
    g_state.ring = nullptr;
    g_state.ring_slot = 0;
}

static bool ring_reserve(size_t slot_bytes) {
    if (g_state.ring && g_state.ring_slot >= slot_bytes) return true;
    if (g_state.ring) {
        device_sync();
        ring_free();
    }
    const size_t bytes = 2 * kRingSlots * slot_bytes;
    if (hipHostMalloc(&g_state.ring, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        g_state.ring = nullptr;
        g_state.ring_slot = 0;
        return false;
    }
    g_state.ring_slot = slot_bytes;
    return true;
}
static char *ring_in(size_t slot) { return static_cast<char *>(g_state.ring) + slot * g_state.ring_slot; }
static char *ring_out(size_t slot) {
    return static_cast<char *>(g_state.ring) + (kRingSlots + slot) * g_state.ring_slot;
}

// A copy whose stores bypass the caches (32-byte non-temporal stores, then a
// store fence): a destination that is only read again by a DMA engine or,
// much later, by the program gains nothing from being cached, and the
// streaming stores skip the read-for-ownership of every destination line that
// a cached store pays (one memory read fewer per byte).  AVX2 when the CPU
// has it, memcpy otherwise.
__attribute__((target("avx2"))) static void nt_copy_avx2(char *dst, const char *src, size_t n) {
    size_t i = 0;
    const size_t head = std::min(n, (size_t)((32 - ((uintptr_t)dst & 31)) & 31));
    if (head) std::memcpy(dst, src, head);
    i = head;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 64));
        const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 96), d);
    }
    if (i < n) std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

static void copy_bytes(char *dst, const char *src, size_t n, bool nt) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (nt && avx2) nt_copy_avx2(dst, src, n);
    else std::memcpy(dst, src, n);
}

// Streaming stores for the ring's out-copy into the caller's target only: the
// out gang's 4 threads copy 94 against 81 GB/s with them in the copy lab, and
// the pipeline averages 36.0 against 34.9 GiB/s over interleaved runs, with
// the smaller dip (profiles/r05_e2e_nt.txt); into the ring they lose (30.3
// against 36.2: the H2D DMA reads the slot right after).
constexpr bool kNtIn = false, kNtOut = true;

static std::vector<int> allowed_cpus();
static const std::vector<std::vector<int>> &copy_threads();

namespace {
void pin_thread(std::thread &t, const std::vector<int> &cpus) {
    if (cpus.empty()) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus) CPU_SET(c, &set);
    (void)pthread_setaffinity_np(t.native_handle(), sizeof set, &set);
}

class CopyPool {
  public:
    // the staging budget (copy_threads): worker i on thread i's domain (the
    // caller does piece 0 where it runs)
    CopyPool() {
        const std::vector<std::vector<int>> &plan = copy_threads();
        nthreads_ = (unsigned)plan.size();
        for (unsigned i = 1; i < nthreads_; ++i) {
            workers_.emplace_back([this, i] { run(i); });
            pin_thread(workers_.back(), plan[i]);
        }
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : workers_) t.join();
    }
    // memcpy split over the pool; returns when every piece is done.  One
    // caller at a time: a second concurrent caller (the mirrored heap's fault
    // handler on another thread) copies on its own.
    void copy(void *dst, const void *src, size_t bytes, bool nt) {
        if (bytes < (size_t(4) << 20) || nthreads_ == 1 || busy_.exchange(true, std::memory_order_acquire)) {
            copy_bytes(static_cast<char *>(dst), static_cast<const char *>(src), bytes, nt);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            dst_ = static_cast<char *>(dst);
            src_ = static_cast<const char *>(src);
            bytes_ = bytes;
            nt_ = nt;
            pending_ = nthreads_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        piece(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
        busy_.store(false, std::memory_order_release);
    }

  private:
    void piece(unsigned i) {
        const size_t per = (bytes_ / nthreads_ + 63) & ~size_t(63);
        const size_t lo = std::min(bytes_, per * i), hi = std::min(bytes_, per * (i + 1));
        if (hi > lo) copy_bytes(dst_ + lo, src_ + lo, hi - lo, nt_);
    }
    void run(unsigned i) {
        unsigned long long seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            piece(i);
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    unsigned nthreads_ = 1;
    std::atomic<bool> busy_{false};
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    bool stop_ = false;
    unsigned long long gen_ = 0;
    unsigned pending_ = 0;
    char *dst_ = nullptr;
    const char *src_ = nullptr;
    size_t bytes_ = 0;
    bool nt_ = false;
};
}  // namespace

void parallel_copy(void *dst, const void *src, size_t bytes, bool nt) {
    static CopyPool pool;
    pool.copy(dst, src, bytes, nt);
}

// this process's allowed CPUs
static std::vector<int> allowed_cpus() {
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) != 0) return {};
    std::vector<int> out;
    for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &set)) out.push_back(c);
    return out;
}

// allowed CPUs of NUMA node `node` (empty if unknown)
static std::vector<int> node_cpus(int node) { return topo::node_cpus("/sys", node, allowed_cpus()); }

// NUMA node of a GPU (its PCI device's numa_node), or -1
int gpu_numa_node(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    std::string id(bus);
    for (auto &c : id) c = (char)std::tolower((unsigned char)c);
    std::ifstream nf("/sys/bus/pci/devices/" + id + "/numa_node");
    int node = -1;
    if (!(nf >> node) || node < 0) return -1;
    return node;
}

// The staging copy threads of this PE, as CPU sets (topo::plan_copy_threads),
// made once: the job's CPU budget (the cgroup quota, else this process's
// allowed CPUs) shared by the PEs on the node, at most 8 per PE
// ($SHMEMX_COPY_THREADS: that many, as given), each thread confined to its
// own last-level-cache domain (CCD) of the GPU's NUMA node, offset by the PE's
// rank among the PEs whose GPUs share that node.  One thread per domain runs
// 36.8-37.7 GiB/s where the scheduler's placement gave 27.2-37.7 (one PE,
// profiles/r05_e2e_spread.txt); with every PE putting its thread i on domain i
// (round 5), eight PEs stacked theirs on the same CCDs, and 8 x 15 threads
// against a 16-CPU quota ran pageable at 0.53 of pinned.
// Within a domain the scheduler picks an idle core; an unknown topology
// leaves the threads unpinned.
static const std::vector<std::vector<int>> &copy_threads() {
    static const std::vector<std::vector<int>> plan = [] {
        const char *e = std::getenv("SHMEMX_COPY_THREADS");
        const unsigned want = e && *e ? (unsigned)std::max(2, std::min(64, std::atoi(e))) : 8u;
        const std::vector<int> allowed = allowed_cpus();
        const int quota = topo::cgroup_cpu_quota("/sys/fs/cgroup");
        const int budget = e && *e ? 0 : quota > 0 ? std::min(quota, (int)allowed.size()) : (int)allowed.size();
        const int mine = gpu_numa_node(g_state.device);
        int pes = 1, rank = 0;
        if (node::up()) {
            pes = node::npes();
            for (int q = 0; q < g_state.pe; ++q) rank += node::gpu_numa(q) == mine ? 1 : 0;
        }
        const std::vector<std::vector<int>> domains =
            mine >= 0 ? topo::cache_domains("/sys", node_cpus(mine)) : std::vector<std::vector<int>>{};
        std::vector<std::vector<int>> p = topo::plan_copy_threads(want, budget, pes, rank, domains);
        if (log_enabled(LOG_INFO)) {
            std::string l;
            for (const auto &x : p) l += x.empty() ? "- " : std::to_string(x.front()) + "+" + std::to_string(x.size() - 1) + " ";
            trace(LOG_INFO, "staging copy threads: %zu (CPU budget %d over %d PEs, quota %d; rank %d on NUMA node "
                  "%d of %zu cache domains), first CPU+others of each: %s", p.size(), budget, pes, quota, rank,
                  mine, domains.size(), l.c_str());
        }
        return p;
    }();
    return plan;
}

namespace {
// A gang of CPU threads that runs one copy at a time in the background: the
// caller starts it and waits for it later, doing other work (enqueueing DMA,
// starting the other gang's copy) meanwhile.  The pageable staging pipeline
// has two: one fills the page-locked ring from the caller's source, the other
// empties it into the caller's target, at the same time (round 5: one pool
// doing both in turn left each copy waiting for the other).
class CopyGang {
  public:
    // worker i on the CPUs of per_thread[i] (empty: unpinned)
    explicit CopyGang(const std::vector<std::vector<int>> &per_thread)
        : n_(std::max<unsigned>(1u, (unsigned)per_thread.size())) {
        for (unsigned i = 0; i < n_; ++i) {
            workers_.emplace_back([this, i] { run(i); });
            if (i < per_thread.size()) pin_thread(workers_.back(), per_thread[i]);
        }
    }
    ~CopyGang() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : workers_) t.join();
    }
    void start(void *dst, const void *src, size_t bytes, bool nt) {
        wait();
        std::lock_guard<std::mutex> lk(mu_);
        dst_ = static_cast<char *>(dst);
        src_ = static_cast<const char *>(src);
        bytes_ = bytes;
        nt_ = nt;
        pending_ = n_;
        ++gen_;
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
    }

  private:
    void run(unsigned i) {
        unsigned long long seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            const size_t per = (bytes_ / n_ + 63) & ~size_t(63);
            const size_t lo = std::min(bytes_, per * i), hi = std::min(bytes_, per * (i + 1));
            if (hi > lo) copy_bytes(dst_ + lo, src_ + lo, hi - lo, nt_);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_all();
        }
    }
    unsigned n_;
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    bool stop_ = false;
    unsigned long long gen_ = 0;
    unsigned pending_ = 0;
    char *dst_ = nullptr;
    const char *src_ = nullptr;
    size_t bytes_ = 0;
    bool nt_ = false;
};

// The staging pipeline's two gangs, made on first use: this PE's copy
// threads (copy_threads) alternate between them, the in gang taking threads
// 0, 2, 4, ... and the out gang 1, 3, 5, ..., so no two share a domain
// while there are domains enough.
CopyGang &gang(int which) {
    static const std::array<std::vector<std::vector<int>>, 2> halves = [] {
        const std::vector<std::vector<int>> &all = copy_threads();
        std::array<std::vector<std::vector<int>>, 2> h;
        for (size_t i = 0; i < all.size(); ++i) h[i % 2].push_back(all[i]);
        return h;
    }();
    static CopyGang in(halves[0]), out(halves[1]);
    return which == 0 ? in : out;
}
}  // namespace

// The small-message bounce buffers: fine-grained (coherent) page-locked
// memory, so a kernel that reads or writes them in place sees the host's
// bytes and the host sees its stores after the stream wait, with no cached
// copy in any XCD's L2 across calls.
static bool small_bounce_reserve() {
    if (g_state.bounce) return true;
    if (hipHostMalloc(&g_state.bounce, 2 * kSmallHostBytes, hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        g_state.bounce = nullptr;
        g_state.bounce_bytes = 0;
        return false;
    }
    g_state.bounce_bytes = kSmallHostBytes;
    return true;
}

// Every member must issue the same sequence of collective calls, as every PE
// of the reference runs one call sequence (reduce-op.c:213-250).  Device
// arrays reduce in one call; host arrays above kSmallHostBytes in one call
// per staging chunk.  Before a collective call of that size the members
// compare their call counts (one 8-byte exchange); if any differs — one PE
// passed host arrays, another device arrays — every member returns
// SHMEMX_ENOTSUP instead of issuing mismatched collectives.
static bool calls_agree(int start, int logstride, int size, size_t ncalls) {
    std::vector<unsigned long long> all;
    if (exchange_u64(start, logstride, size, ncalls, all)) return false;
    for (unsigned long long v : all) {
        if (v != ncalls) {
            trace(LOG_REDUCTION, "members disagree on the call's chunking (%llu vs %zu calls: host "
                  "and device arrays mixed across PEs): ENOTSUP", v, ncalls);
            set_error(SHMEMX_ENOTSUP);
            return false;
        }
    }
    return true;
}

static void reduce_blocking_impl(int type, int op, void *target, const void *source, int nreduce,
                                 int start, int logstride, int size, bool trace_call);

// A blocking call's host-view target up to this many bytes (the bounce
// path's size) is copied back into the view before the call returns: its
// blocks come back CLEAN (ISx's round 42.8 -> 30.1 us, the host load 19.9 ->
// 0.26 us: profiles/r04_isx_mirror.txt).
static size_t mirror_settle_limit() { return kSmallHostBytes; }

// Whether a blocking call of `bytes` per PE over several PEs takes the
// exchange: every member decides alike (the same size and settings;
// g_state.xchg was agreed at init).
static bool xchg_eligible(size_t bytes) {
    return bytes <= node::kXchgSlotBytes && g_state.xchg && g_state.algo == SHMEMX_ALGO_AUTO &&
           !g_state.force_collective && service_available();
}

// The blocking entry point body: host- or device-resident arrays.  Operands
// in the mirrored heap's host view run on their HBM twins (heap.h).
void reduce_blocking(int type, int op, void *target, const void *source,
                     int nreduce, int start, int logstride, int size) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    const size_t sz = type_size(type);
    if (nreduce > 0 && sz && target && source && op_valid(type, op)) {
        const size_t bytes = sz * (size_t)nreduce;
        if (heap::twin(target) != target || heap::twin(source) != source) {
            // the host's stores to the operands' blocks go up on the library
            // stream, ahead of the call's own work there: no host wait for
            // them (the DIRECT / SIGNAL peers read this PE's HBM only after a
            // barrier that waits for the stream, or in stream order)
            heap::SameStreamFlush same_stream;
            // Small operands whose result one workgroup can also store into
            // the view's alias (the ISx nreduce = 1 use) take the light path:
            // only the source's own host-written bytes go up, and no block
            // changes state or protection (mirror.h begin_light_write), so
            // the host's next store into those blocks takes no fault either
            const size_t lim = mirror_settle_limit();
            void *adst = bytes <= lim ? heap::alias_device(target, bytes) : nullptr;
            const bool light = adst && heap::twin(target) != target && heap::twin(source) != source &&
                               copy_one_workgroup(type, adst, heap::twin(target), (size_t)nreduce);
            // PE_size 1 (a copy, reduce-op.c:213-216) on the light path, with
            // the source's view bytes current: they go through the coherent
            // bounce buffer (a CPU copy, as small host arrays do) and the copy
            // kernel reads them there, instead of a DMA to the source's HBM
            // twin first (its blocks keep their state: a HOST_NEWER block is
            // flushed whole by the next call that needs it in HBM).  ISx's
            // nreduce = 1 round: profiles/r05_isx_mirror.txt.
            // A small call over several PEs through the exchange (xchg_reduce)
            // on the same terms: the view's current bytes go into this PE's
            // exchange slot by a CPU copy, and the source's HBM twin, neither
            // flushed nor read, keeps its blocks' state.
            const bool xchg = size > 1 && xchg_eligible(bytes);
            const void *cur = light && (size == 1 || xchg) && !g_state.force_collective && bytes <= kSmallHostBytes
                                  ? heap::current_host_bytes(source, bytes) : nullptr;
            const void *s = nullptr;
            if (cur && size == 1 && small_bounce_reserve()) {
                std::memcpy(g_state.bounce, cur, bytes);
                s = g_state.bounce;
            } else if (cur && xchg) {
                g_state.xchg_src_host = cur;
                s = heap::twin(source);
            } else {
                s = light ? heap::device_operand_bytes(source, bytes) : heap::device_operand(source, bytes);
            }
            trace_reference_overlap(target, source, bytes);   // the caller's addresses
            // blocks of a host-view target: DEVICE_NEWER from before the call
            // (host accesses wait for it), or on the light path unchanged; the
            // blocking call completes on the library stream, its recorded writer
            heap::DeviceWrite t(target, bytes, g_state.stream, light);
            // a small result also goes straight into the view's page-locked
            // alias: the call's last kernel stores it there before the host
            // signal (one workgroup, so its own drained stores and
            // system-scope release precede the signal)
            void *dst = t.settle_dst(mirror_settle_limit());
            if (dst && !copy_one_workgroup(type, dst, t.ptr(), (size_t)nreduce)) dst = nullptr;
            g_state.settle_dst = dst;
            g_state.settled = false;
            reduce_blocking_impl(type, op, t.ptr(), s, nreduce, start, logstride, size, false);
            g_state.xchg_src_host = nullptr;
            const bool copied = g_state.settled;
            g_state.settle_dst = nullptr;
            g_state.settled = false;
            // the call's work is complete: a small result is back in the view
            // (copied above, or now), so the caller's system calls can read
            // it (larger targets are fetched on first access).
            // A call that failed wrote no target: on the light path the view
            // already holds the target's bytes, and HBM may not (a
            // host-written target block is not flushed there), so nothing is
            // copied back
            const bool failed = shmemx_reduce_last_error() != SHMEMX_OK;
            // A call that failed before its own work (a bad set, a call-count
            // mismatch) never waited for the library stream, where the flush
            // of the host's bytes (SameStreamFlush) may still be in flight:
            // settle()'s copy-back, and the next call on another stream, must
            // not read HBM before it has landed
            if (failed) SHMX_HIP(hipStreamSynchronize(g_state.stream));
            // every blocking call returns with its work complete: no writer
            // event on the library stream (it would keep the stream busy for
            // the next call's service check, service.hip)
            t.completed();
            t.settle(mirror_settle_limit(), copied || (failed && t.light()));
            return;
        }
    }
    reduce_blocking_impl(type, op, target, source, nreduce, start, logstride, size, true);
}

static void reduce_blocking_impl2(int type, int op, void *target, const void *source, int nreduce,
                                  int start, int logstride, int size, bool trace_call);

// A small blocking call over several PEs (<= 4 KiB per PE): the reference's
// barrier, gets and barrier (reduce-op.c:217-250) with the gets and the fold
// done by each member's resident service workgroup (service.hip), no kernel
// launch.  Each member leaves its source in its slot of the job's page-locked
// exchange (node.h; a device source by a service copy, a host one by the
// CPU), passes the entry barrier, has its workgroup fold every member's slot
// (its own order for the pairs where the order decides the answer, else
// PE_start's, as DIRECT and A2A do) into its target (a host target through
// the bounce buffer), and marks itself done with every member's slot; a
// member writes its slot again only once the readers of its previous call
// are done (node::xchg_claim), which takes the place of the reference's exit
// barrier.  Host memory is the meeting point, so no GPU reads
// another GPU's memory and no L2 write-back beyond each workgroup's own
// system-scope release is needed.
static void xchg_reduce(int type, int op, void *target, bool tdev, const void *source, bool sdev, size_t bytes,
                        int start, int logstride, int size) {
    const int step = 1 << logstride;
    if (log_enabled(LOG_REDUCTION))
        trace(LOG_REDUCTION, "type %d op %d nreduce %zu set (%d,%d,%d) algo service exchange%s", type, op,
              bytes / type_size(type), start, logstride, size, own_order_pair(type, op) ? " (own order)" : "");
    if (!tdev && !small_bounce_reserve())
        fatal("small multi-PE call", "no page-locked bounce buffer for a host target");
    uint64_t counts[node::kMaxPes];
    node::xchg_claim(start, step, size, counts);   // the slot is free again
    if (g_state.xchg_src_host) {   // a mirrored-heap source's current view bytes
        std::memcpy(node::xchg_host(g_state.pe), g_state.xchg_src_host, bytes);
    } else if (sdev) {
        if (!service_copy(node::xchg_dev(g_state.pe), nullptr, source, bytes))
            fatal("small multi-PE call", "the service workgroup did not take the source");
    } else {
        std::memcpy(node::xchg_host(g_state.pe), source, bytes);
    }
    node::barrier(start, step, size);
    char *bout = static_cast<char *>(g_state.bounce) + kSmallHostBytes;
    void *dst2 = tdev ? g_state.settle_dst : nullptr;
    service_fold(type, op, own_order_pair(type, op), start, logstride, size, tdev ? target : bout, dst2, bytes);
    node::xchg_finish(start, step, size, counts);   // (no exit barrier: xchg_claim)
    if (dst2) g_state.settled = true;
    if (!tdev) std::memcpy(target, bout, bytes);
}

// A blocking call returns as soon as its work's host signal arrives.
static void reduce_blocking_impl(int type, int op, void *target, const void *source, int nreduce,
                                 int start, int logstride, int size, bool trace_call) {
    struct Early {
        Early() { g_state.return_on_signal = true; }
        ~Early() { g_state.return_on_signal = false; }
    } early;
    reduce_blocking_impl2(type, op, target, source, nreduce, start, logstride, size, trace_call);
}

static void reduce_blocking_impl2(int type, int op, void *target, const void *source, int nreduce,
                                  int start, int logstride, int size, bool trace_call) {
    if (ensure_init()) {
        trace(LOG_FATAL, "reduction called before shmem_init with npes > 1");
        return;
    }
    if (!op_on_device(type, op)) {
        set_error(op_valid(type, op) ? SHMEMX_ENOTSUP : SHMEMX_EINVAL);
        return;
    }
    if (nreduce <= 0 || !target || !source) {
        if (nreduce < 0 || ((!target || !source) && nreduce > 0)) set_error(SHMEMX_EINVAL);
        else {  // n == 0: nothing moves, but validate membership like a call would
            shmemx_plan_t p;
            int rc = make_plan(type, op, 0, start, logstride, size, g_state.pe, g_state.npes,
                               g_state.algo, &p);
            if (rc) set_error(rc);
            else if (trace_call) trace_reference_overlap(target, source, 0);
        }
        return;
    }
    const size_t bytes = type_size(type) * (size_t)nreduce;
    // (the small-message bounce buffer is mapped into the GPU: a source
    // staged there by the mirrored heap's PE_size 1 light path is read in place)
    const bool tdev = device_accessible(target),
               sdev = (source == g_state.bounce && g_state.bounce) || device_accessible(source);
    hipStream_t s = g_state.stream;
    const bool collective = size > 1 || g_state.force_collective;
    shmemx_plan_t plan;
    {
        const int rc = make_plan(type, op, nreduce, start, logstride, size, g_state.pe,
                                 g_state.npes, g_state.algo, &plan);
        if (rc) {
            set_error(rc);
            return;
        }
    }
    if (trace_call) trace_reference_overlap(target, source, bytes);   // the caller's arrays
    // A small call over several PEs under auto: through the exchange and the
    // service workgroups (xchg_reduce).  Every member decides alike: the
    // same size, set and settings, and g_state.xchg was agreed at init.
    if (size > 1 && xchg_eligible(bytes)) {
        xchg_reduce(type, op, target, tdev, source, sdev, bytes, start, logstride, size);
        return;
    }
    if (tdev && sdev) {
        if (collective && bytes > kSmallHostBytes && !calls_agree(start, logstride, size, 1)) return;
        if (plan.nmembers == 1 && !collective && !overlap(target, source, bytes)) {
            // a one-member set is a copy (reduce-op.c:213-216): up to 4 KiB by
            // the resident service workgroup when the streams it is ordered
            // after are idle (no launch; service.hip), else the copy kernel,
            // which tells the host itself when it is done (one workgroup; a
            // marker kernel otherwise): no stream wait either way
            if (bytes <= kServiceMaxBytes && service_copy(target, g_state.settle_dst, source, bytes)) {
                if (g_state.settle_dst) g_state.settled = true;
                return;
            }
            const HostSignal sig = next_host_signal();
            const void *in[1] = {source};
            if (g_state.settle_dst) {
                // a small mirrored target: one copy kernel stores the result
                // into HBM and into the view's alias, and its workgroup signals
                SHMX_HIP(launch_copy2_signal(type, target, g_state.settle_dst, source, (size_t)nreduce, s, sig));
            } else {
                SHMX_HIP(launch_fold_signal(type, op, target, in, 1, (size_t)nreduce, s, sig));
            }
            wait_host_signal(sig, s);
            if (g_state.settle_dst) g_state.settled = true;
            return;
        }
        const int rc = reduce_device(type, op, target, source, nreduce, start, logstride, size,
                                     g_state.algo, s);
        // DIRECT and own-order GATHER over IPC return with their work done
        // (host barriers, or the fused launch's host signal): no stream wait
        // on top — a hipStreamSynchronize entered while a kernel is still
        // retiring costs ~9 us more than the kernel's remaining time
        // (profiles/r03_latency_ab.txt).  The stream-ordered algorithms end
        // with a marker the host spins on.
        const bool waits_itself = collective && (plan.algo == SHMEMX_ALGO_DIRECT ||
                                                 (plan.algo == SHMEMX_ALGO_GATHER && g_state.ipc_only));
        if (rc == SHMEMX_OK && (!waits_itself || g_state.settle_dst)) {
            const HostSignal sig = next_host_signal();
            if (g_state.settle_dst) {
                // a small mirrored target: the result into the view's alias,
                // by the one workgroup that then signals
                const void *res[1] = {target};
                SHMX_HIP(launch_fold_signal(type, op, g_state.settle_dst, res, 1, (size_t)nreduce, s, sig));
            } else {
                SHMX_HIP(launch_host_signal(sig, s));
            }
            wait_host_signal(sig, s);
            if (g_state.settle_dst) g_state.settled = true;
        } else if (rc != SHMEMX_OK) {
            SHMX_HIP(hipStreamSynchronize(s));
        }
        switch (signal_error()) {
        case 0: break;
        case 2: fatal("SIGNAL reduction", "a system fence before a device barrier missed an XCD");
        default: fatal("SIGNAL reduction", "a member never reached the device barrier");
        }
        return;
    }
    // Host-resident symmetric arrays (the reference's heap): stage over PCIe
    // in chunks, H2D on one copy stream, the reduction on the library stream,
    // D2H on a second copy stream, so the two PCIe directions and the device
    // work overlap.  Every PE cuts the same chunks, so the collective
    // sequence matches across PEs (calls_agree checks it).
    if (bytes <= kSmallHostBytes && !small_bounce_reserve()) {
        set_error(SHMEMX_ENOMEM);
        return;
    }
    if (bytes <= kSmallHostBytes && plan.nmembers == 1 && !g_state.force_collective) {
        // A one-member set is a copy (reduce-op.c:213-216).  The copy kernel
        // reads and writes the page-locked bounce buffers in place over PCIe
        // (zero-copy): one launch and one wait, no DMA commands.
        char *bin = static_cast<char *>(g_state.bounce);
        char *bout = bin + kSmallHostBytes;
        if (!sdev) std::memcpy(bin, source, bytes);
        void *t = tdev ? target : bout;
        const void *in[1] = {sdev ? source : bin};
        if (overlap(t, in[0], bytes)) {
            const int rc = reduce_device(type, op, t, in[0], nreduce, start, logstride, size, g_state.algo, s);
            SHMX_HIP(hipStreamSynchronize(s));
            if (!rc && !tdev) std::memcpy(target, bout, bytes);
            return;
        }
        // the service workgroup (service.hip), or the copy kernel, which
        // signals the host when its stores have landed
        if (!(bytes <= kServiceMaxBytes && service_copy(t, nullptr, in[0], bytes))) {
            const HostSignal sig = next_host_signal();
            SHMX_HIP(launch_fold_signal(type, op, t, in, 1, (size_t)nreduce, s, sig));
            wait_host_signal(sig, s);
        }
        if (!tdev) std::memcpy(target, bout, bytes);
        return;
    }
    if (bytes > g_state.stage_bytes) {
        device_sync();
        if (g_state.stage_src) SHMX_HIP(hipFree(g_state.stage_src));
        if (g_state.stage_tgt) SHMX_HIP(hipFree(g_state.stage_tgt));
        g_state.stage_src = g_state.stage_tgt = nullptr;
        g_state.stage_bytes = 0;
        if (hipMalloc(&g_state.stage_src, bytes) != hipSuccess ||
            hipMalloc(&g_state.stage_tgt, bytes) != hipSuccess) {
            (void)hipGetLastError();
            set_error(SHMEMX_ENOMEM);
            return;
        }
        g_state.stage_bytes = bytes;
    }
    if (bytes <= kSmallHostBytes) {
        // Small messages (the ISx nreduce = 1 case, isx.c:617): latency, not
        // bandwidth.  Bounce through the page-locked buffers; copy kernels on
        // the library stream move them to and from the device (no DMA
        // command: 25 vs 33 us per call at 32 KiB, profiles/archive/r01_host_latency.txt),
        // and the host waits once.
        char *bin = static_cast<char *>(g_state.bounce);
        char *bout = bin + kSmallHostBytes;
        // DIRECT and own-order GATHER over IPC take the bounce buffers
        // themselves (page-locked, device-accessible): the source goes
        // straight into the IPC scratch the peers read, the fold writes the
        // result into bout over PCIe, and the call returns with its work
        // done, so the copy kernels on either side and the extra wait go.
        // RCCL's algorithms need device memory: they keep the staging copies.
        const bool pulls = collective && (plan.algo == SHMEMX_ALGO_DIRECT ||
                                          (plan.algo == SHMEMX_ALGO_GATHER && g_state.ipc_only));
        const void *dsrc = source;
        if (!sdev) {
            std::memcpy(bin, source, bytes);
            if (pulls) {
                dsrc = bin;
            } else {
                const void *in[1] = {bin};
                fold_chain(type, op, g_state.stage_src, in, 1, (size_t)nreduce, s);
                dsrc = g_state.stage_src;
            }
        }
        void *dtgt = tdev ? target : pulls ? static_cast<void *>(bout) : g_state.stage_tgt;
        const int rc = reduce_device(type, op, dtgt, dsrc, nreduce, start, logstride, size,
                                     g_state.algo, s);
        if (!rc && pulls) {
            // the pulls returned with the result in place (host barriers, or
            // the fused launch's host signal)
        } else if (!rc) {
            // the last copy (or a marker) signals the host: no stream wait
            const HostSignal sig = next_host_signal();
            if (!tdev) {
                const void *in[1] = {dtgt};
                SHMX_HIP(launch_fold_signal(type, op, bout, in, 1, (size_t)nreduce, s, sig));
            } else {
                SHMX_HIP(launch_host_signal(sig, s));
            }
            wait_host_signal(sig, s);
        } else {
            SHMX_HIP(hipStreamSynchronize(s));
        }
        switch (signal_error()) {
        case 0: break;
        case 2: fatal("SIGNAL reduction", "a system fence before a device barrier missed an XCD");
        default: fatal("SIGNAL reduction", "a member never reached the device barrier");
        }
        if (!rc && !tdev) std::memcpy(target, bout, bytes);
        return;
    }
    if (!g_state.h2d) {
        SHMX_HIP(hipStreamCreateWithFlags(&g_state.h2d, hipStreamNonBlocking));
        SHMX_HIP(hipStreamCreateWithFlags(&g_state.d2h, hipStreamNonBlocking));
    }
    const size_t sz = type_size(type);
    const size_t g = sz >= 16 ? 1 : 16 / sz;
    static const size_t stage_chunk = [] {
        const char *e = std::getenv("SHMEMX_STAGE_CHUNK_MB");
        const int mb = e ? std::atoi(e) : 0;
        return mb > 0 ? size_t(mb) << 20 : kStageChunkBytes;
    }();
    size_t chunk = ((stage_chunk / sz) / g) * g;
    if (chunk == 0) chunk = g;
    // a host target that partially overlaps the host source would be
    // overwritten under a later chunk's H2D: no pipelining then
    const bool host_overlap = !tdev && !sdev && overlap(target, source, bytes);
    if (host_overlap) chunk = (size_t)nreduce;
    // The chunk schedule (elements, stage_plan.h: quarter and half chunks at
    // both ends, +1.1 %, profiles/r05_e2e_ramp.txt), the same on every PE
    // (calls_agree compares its length).
    std::vector<size_t> c_off, c_n;
    stage_plan((size_t)nreduce, chunk, g, !host_overlap, c_off, c_n);
    const size_t nchunks = c_n.size();
    if (collective && !calls_agree(start, logstride, size, nchunks)) return;
    // How each end reaches the device: directly (device memory), by DMA
    // (page-locked host memory), or through the page-locked bounce ring
    // (pageable memory: CPU copy by the worker pool, then DMA).
    const bool in_bounce = !sdev && !host_pinned(source) && !host_overlap;
    const bool out_bounce = !tdev && !host_pinned(target) && !host_overlap;
    const size_t chunk_bytes = chunk * sz;
    if ((in_bounce || out_bounce) && !ring_reserve(chunk_bytes)) {
        set_error(SHMEMX_ENOMEM);
        return;
    }
    while (g_state.events.size() < 2 * nchunks + 2 * kRingSlots) {
        hipEvent_t e;
        SHMX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        g_state.events.push_back(e);
    }
    hipEvent_t *ev_chunk = g_state.events.data();             // 2 per chunk
    hipEvent_t *ev_in_slot = ev_chunk + 2 * nchunks;          // ring slot free again
    hipEvent_t *ev_out_slot = ev_in_slot + kRingSlots;        // ring slot filled
    char *hsrc = static_cast<char *>(const_cast<void *>(source));
    char *htgt = static_cast<char *>(target);
    char *ssrc = static_cast<char *>(g_state.stage_src);
    char *stgt = static_cast<char *>(g_state.stage_tgt);
    // Pageable ends run through the ring with two CPU gangs working at once
    // (bounce in: source -> ring_in[k % kRingSlots], read by the H2D of chunk
    // k; bounce out: ring_out[k % kRingSlots], written by the D2H of chunk k,
    // -> target), so the CPU copies in and out overlap each other and the
    // DMA and the fold of the chunks between them.  Slot reuse: the in-copy
    // of chunk k waits for the H2D of chunk k - kRingSlots (event), the D2H of
    // chunk k for the out-copy of chunk k - kRingSlots (host side).
    auto count_of_chunk = [&](size_t k) { return c_n[k]; };
    auto start_in = [&](size_t k) {
        const size_t slot = k % kRingSlots;
        if (k >= kRingSlots) SHMX_HIP(hipEventSynchronize(ev_in_slot[slot]));
        gang(0).start(ring_in(slot), hsrc + c_off[k] * sz, count_of_chunk(k) * sz, kNtIn);
    };
    size_t out_started = 0;   // out-copies started; all but the last are complete
    auto start_out = [&]() {
        const size_t j = out_started++;
        SHMX_HIP(hipEventSynchronize(ev_out_slot[j % kRingSlots]));
        gang(1).start(htgt + c_off[j] * sz, ring_out(j % kRingSlots), count_of_chunk(j) * sz, kNtOut);
    };
    // the out-copy of chunk j has completed (starting the ones before it)
    auto out_done = [&](size_t j) {
        while (out_started <= j) start_out();
        gang(1).wait();
    };
    int rc = SHMEMX_OK;
    if (in_bounce && nchunks) start_in(0);
    for (size_t k = 0; k < nchunks && !rc; ++k) {
        const size_t off = c_off[k] * sz;
        const size_t b = count_of_chunk(k) * sz;
        const size_t slot = k % kRingSlots;
        const void *dsrc = hsrc + off;
        if (!sdev) {
            const char *from = hsrc + off;
            if (in_bounce) {
                gang(0).wait();              // chunk k is in its ring slot
                from = ring_in(slot);
            }
            SHMX_HIP(hipMemcpyAsync(ssrc + off, from, b, hipMemcpyHostToDevice, g_state.h2d));
            SHMX_HIP(hipEventRecord(ev_chunk[2 * k], g_state.h2d));
            if (in_bounce) SHMX_HIP(hipEventRecord(ev_in_slot[slot], g_state.h2d));
            SHMX_HIP(hipStreamWaitEvent(s, ev_chunk[2 * k], 0));
            dsrc = ssrc + off;
            if (in_bounce && k + 1 < nchunks) start_in(k + 1);   // runs while this chunk moves
        }
        void *dtgt = tdev ? static_cast<void *>(htgt + off) : static_cast<void *>(stgt + off);
        rc = reduce_device(type, op, dtgt, dsrc, (int)(b / sz), start, logstride, size, g_state.algo, s);
        if (!rc && !tdev) {
            SHMX_HIP(hipEventRecord(ev_chunk[2 * k + 1], s));
            SHMX_HIP(hipStreamWaitEvent(g_state.d2h, ev_chunk[2 * k + 1], 0));
            if (out_bounce) {
                if (k >= kRingSlots) out_done(k - kRingSlots);   // the slot's previous chunk is out
                SHMX_HIP(hipMemcpyAsync(ring_out(slot), dtgt, b, hipMemcpyDeviceToHost, g_state.d2h));
                SHMX_HIP(hipEventRecord(ev_out_slot[slot], g_state.d2h));
                // keep the out gang on the oldest chunk whose D2H is enqueued
                // one behind, so this thread is free to enqueue the next one
                if (k >= 1 && out_started < k) {
                    gang(1).wait();
                    start_out();
                }
            } else {
                SHMX_HIP(hipMemcpyAsync(htgt + off, dtgt, b, hipMemcpyDeviceToHost, g_state.d2h));
            }
        }
    }
    if (in_bounce) gang(0).wait();          // no copy still writes the ring
    if (out_bounce && !rc && nchunks) out_done(nchunks - 1);
    if (out_bounce) gang(1).wait();
    SHMX_HIP(hipStreamSynchronize(g_state.h2d));
    SHMX_HIP(hipStreamSynchronize(s));
    SHMX_HIP(hipStreamSynchronize(g_state.d2h));
}

}  // namespace shmx
