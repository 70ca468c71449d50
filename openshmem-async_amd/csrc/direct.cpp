// DIRECT algorithm: the reference's reduction (reduce-op.c:169-260) as the
// reference itself structures it — every PE reads its peers' symmetric
// source arrays — but with the reads done by a HIP kernel straight out of
// the peers' HBM over xGMI (IPC-mapped symmetric heap, node.h / heap.h)
// instead of 64-element shmem_getmem round trips into pWrk, and the fold
// fused into that same pass.
//
// Set order (SHMEMX_ALGO_DIRECT), two pull phases, no intermediate buffers:
//   1. reduce-scatter: member m folds slice m of the array from all P
//      sources in active-set order (PE_start first, as A2A does) into slice
//      m of its own target — one kernel reading all P sources at once;
//   2. all-gather: member m copies every other member's result slice from
//      that member's target into its own — one kernel for all P-1 slices.
// (P-1)/P of the array crosses xGMI in each phase, as reads only: a PE never
// stores into another GPU's HBM.  Peer data is read only after the owner's
// kernel has ended, a system-scope fence has run on every XCD of the owner
// (its L2 written back) and of the reader (stale peer lines dropped), and a
// barrier has passed (node_sync).  Every PE ends with the reference's
// PE_start result.
//
// Own order (SHMEMX_ALGO_GATHER on the IPC transport, and every call on the
// float / double / long double min and max pairs, own_order_pair): every PE
// folds the whole array in its own reference order, src_me first, then the
// other members ascending (reduce-op.c:219-248), reading (P-1) peer arrays:
// the reference's per-PE bits on every PE.  Small arrays take the fused one
// shot with the inputs in that order.
//
// Synchronisation is the reference's: a barrier before the peers' sources
// are read (reduce-op.c:217) and one after the targets are final (:250),
// plus one between the two phases; host barriers over the node block.  The
// one shot (small arrays, every member folds the whole array) runs as ONE
// fused launch when every member can take it (launch_signal_fold: the
// fence, both barriers as device handshakes and the fold in one kernel),
// after a fence-free host barrier that exchanges the descriptors; so does
// the two shot up to $SHMEMX_FUSED_TWOSHOT_KB (default 4 MiB) when every
// member's source and target are in its heap segment (three device
// handshakes and two grid barriers in the kernel, one host wait).
// Operands outside the symmetric heap (or a source that partially overlaps
// its target) are staged through a per-PE scratch region, also IPC-mapped,
// in chunks of half its size ($SHMEMX_DIRECT_SCRATCH_MB, default 512; every
// PE must use the same value).  A peer region that cannot be mapped fails
// the call with ENOTSUP on every member alike (map_members).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <unordered_set>
#include <vector>

#include "heap.h"
#include "internal.h"
#include "node.h"
#include "shmem_reduce_mi355x.h"
#include "state.h"

namespace shmx {

namespace {

constexpr size_t kDefaultScratchBytes = size_t(512) << 20;
constexpr size_t kDefaultOneShotBytes = size_t(256) << 10;
constexpr size_t kDefaultFusedTwoShotBytes = size_t(4) << 20;

// Arrays up to this size take the one-shot path ($SHMEMX_DIRECT_ONESHOT_KB).
size_t oneshot_bytes() {
    static const size_t b = [] {
        const char *e = std::getenv("SHMEMX_DIRECT_ONESHOT_KB");
        return e ? size_t(std::atol(e)) << 10 : kDefaultOneShotBytes;
    }();
    return b;
}

struct Scratch {
    char *base = nullptr;
    size_t bytes = 0;
} g_scratch;

bool ensure_scratch() {
    if (g_scratch.base) return true;
    size_t bytes = kDefaultScratchBytes;
    if (const char *e = std::getenv("SHMEMX_DIRECT_SCRATCH_MB")) {
        const long mb = std::atol(e);
        if (mb > 0) bytes = size_t(mb) << 20;
    }
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    g_scratch.base = static_cast<char *>(p);
    g_scratch.bytes = bytes;
    node::publish(node::kScratch, p, bytes);   // peers map it after the next barrier
    trace(LOG_MEMORY, "DIRECT scratch: %zu bytes of HBM at %p", bytes, p);
    return true;
}

std::unordered_set<uint64_t> g_voted;

// The region of each member that DIRECT reads: its source, and its target
// when the peers gather from it.
bool map_members(const std::vector<node::Desc> &desc, bool local_write, int start, int step,
                 int P) {
    std::vector<std::pair<node::Region, int>> regs;
    for (int i = 0; i < P; ++i) {
        regs.emplace_back(static_cast<node::Region>(desc[i].src.region), start + i * step);
        if (!local_write)
            regs.emplace_back(static_cast<node::Region>(desc[i].tgt.region), start + i * step);
    }
    return map_regions(regs, start, step, P);
}

}  // namespace

namespace {

// Host-side phase times of the DIRECT calls since the last reset
// (shmemx_direct_stats): microseconds, summed over calls.
enum Phase { kEntryWait, kEntryBarrier, kFold, kFoldBarrier, kGather, kExitBarrier, kNumPhases };
double g_phase_us[kNumPhases];
double g_calls;
double g_fused_calls;   // one-shot calls that ran as one fused launch (DIRECT and SIGNAL)
double g_fused2_calls;  // two-shot calls that ran as one fused launch

double now_us() {
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// Open (or reuse) the mappings of the given (region, PE) pairs.  The first
// time a set meets a given combination of region generations, the members
// vote (node::agree), so a mapping that fails on one PE fails the call on all
// of them alike; the combinations that passed are remembered, and every
// member decides identically whether to vote (same set, same regions, same
// generations from the shared block).
bool map_regions(const std::vector<std::pair<node::Region, int>> &regs, int start, int step, int P) {
    uint64_t key = 1469598103934665603ull;
    auto mix = [&key](uint64_t v) { key = (key ^ v) * 1099511628211ull; };
    mix((uint64_t)start);
    mix((uint64_t)step);
    mix((uint64_t)P);
    bool ok = true;
    for (const auto &rp : regs) {
        mix((uint64_t)rp.first);
        mix((uint64_t)rp.second);
        mix(node::region_gen(rp.first, rp.second));
        ok &= node::peer_base(rp.first, rp.second) != nullptr;
    }
    if (g_voted.count(key)) {   // every member mapped these before
        if (!ok) fatal("peer region mapped before is gone", node::last_ipc_error());
        return true;
    }
    if (!node::agree(start, step, P, ok)) return false;
    g_voted.insert(key);
    return true;
}

// ------------------------------------------------- fence coverage (XCDs)
// Every system fence records which XCD each of its blocks ran on
// (launch_sys_fence); a fence that did not reach every XCD of the device is
// run again (host-synchronous paths) or fails the SIGNAL call loudly.
namespace {

struct FenceState {
    unsigned int *host_seen = nullptr;         // host-coherent, kFenceBlocks words
    unsigned int *dev_seen = nullptr;          // device, kFenceBlocks words
    unsigned long long *dev_stats = nullptr;   // device: [checks, incomplete]
    unsigned int *gsync = nullptr;             // device: fused kernel's grid barrier
    int nxcc = 0;
    double host_checks = 0, host_refills = 0;
} g_fence;

void ensure_fence() {
    if (g_fence.host_seen) return;
    int dev = 0, nxcc = 0;
    SHMX_HIP(hipGetDevice(&dev));
    if (hipDeviceGetAttribute(&nxcc, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess || nxcc < 1) {
        (void)hipGetLastError();
        nxcc = 8;   // MI355X: 8 XCDs
    }
    g_fence.nxcc = nxcc > 16 ? 16 : nxcc;
    void *h = nullptr, *d = nullptr, *st = nullptr;
    SHMX_HIP(hipHostMalloc(&h, kFenceBlocks * sizeof(unsigned int), hipHostMallocCoherent));
    std::memset(h, 0, kFenceBlocks * sizeof(unsigned int));
    SHMX_HIP(hipMalloc(&d, kFenceBlocks * sizeof(unsigned int)));
    SHMX_HIP(hipMemset(d, 0, kFenceBlocks * sizeof(unsigned int)));
    SHMX_HIP(hipMalloc(&st, 2 * sizeof(unsigned long long)));
    SHMX_HIP(hipMemset(st, 0, 2 * sizeof(unsigned long long)));
    void *gs = nullptr;
    SHMX_HIP(hipMalloc(&gs, 2 * sizeof(unsigned int)));
    SHMX_HIP(hipMemset(gs, 0, 2 * sizeof(unsigned int)));
    g_fence.gsync = static_cast<unsigned int *>(gs);
    device_sync();
    g_fence.host_seen = static_cast<unsigned int *>(h);
    g_fence.dev_seen = static_cast<unsigned int *>(d);
    g_fence.dev_stats = static_cast<unsigned long long *>(st);
    trace(LOG_INIT, "system fences: %d blocks over %d XCDs", kFenceBlocks, g_fence.nxcc);
}

}  // namespace

void fence_and_wait(hipStream_t s) {
    ensure_fence();
    volatile unsigned int *seen = g_fence.host_seen;
    for (int attempt = 0;; ++attempt) {
        SHMX_HIP(launch_sys_fence(s, g_fence.host_seen));
        // Every block stores its record after its fence, and the fence kernel
        // starts only after all earlier work on s: once all kFenceBlocks
        // records are in, that work is complete and every XCD has fenced.
        // Polling the host-coherent records returns ~1.5 us sooner than
        // hipStreamSynchronize (profiles/archive/r02_sync_lab.txt); after a second
        // without them the stream wait takes over (and reports any error).
        {
            const auto t0 = std::chrono::steady_clock::now();
            int b = 0;
            for (unsigned spins = 0; b < kFenceBlocks;) {
                if (seen[b] & kFenceSeen) {
                    ++b;
                    continue;
                }
                if ((++spins & 1023) == 0 &&
                    std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1))
                    break;
            }
            if (b < kFenceBlocks) SHMX_HIP(hipStreamSynchronize(s));
        }
        unsigned int mask = 0;
        for (int b = 0; b < kFenceBlocks; ++b) {
            const unsigned int v = seen[b];
            if (v & kFenceSeen) mask |= 1u << (v & 15u);
            seen[b] = 0;
        }
        g_fence.host_checks += 1;
        if (__builtin_popcount(mask) >= g_fence.nxcc) return;
        g_fence.host_refills += 1;
        trace(LOG_INFO, "system fence reached XCD mask 0x%x (%d of %d XCDs): fencing again", mask,
              __builtin_popcount(mask), g_fence.nxcc);
        if (attempt >= 15) fatal("system fence", "an XCD never ran a fence block (16 attempts)");
    }
}

FenceRecords fence_records() {
    ensure_fence();
    return FenceRecords{g_fence.dev_seen, g_fence.nxcc, g_fence.dev_stats, g_fence.gsync};
}

void node_sync(int start, int step, int P, hipStream_t s, double *stream_us, double *barrier_us,
               double since_us) {
    const double t0 = since_us >= 0 ? since_us : now_us();
    if (P > 1) fence_and_wait(s);
    else SHMX_HIP(hipStreamSynchronize(s));
    const double t1 = now_us();
    node::barrier(start, step, P);
    if (stream_us) *stream_us += t1 - t0;
    if (barrier_us) *barrier_us += now_us() - t1;
}

void node_done(int start, int step, int P, hipStream_t s, double *stream_us, double *barrier_us,
               double since_us) {
    const double t0 = since_us >= 0 ? since_us : now_us();
    SHMX_HIP(hipStreamSynchronize(s));
    const double t1 = now_us();
    node::barrier(start, step, P);
    if (stream_us) *stream_us += t1 - t0;
    if (barrier_us) *barrier_us += now_us() - t1;
}

void count_fused_call() { g_fused_calls += 1; }
void count_fused_twoshot_call() { g_fused2_calls += 1; }

bool fused_oneshot_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SHMEMX_FUSED_ONESHOT");
        return !(e && e[0] == '0');
    }();
    return on;
}

namespace {
long twoshot_kb_from_env() {
    const char *e = std::getenv("SHMEMX_FUSED_TWOSHOT_KB");
    return e ? std::max(0L, std::atol(e)) : (long)(kDefaultFusedTwoShotBytes >> 10);
}
long g_fused_twoshot_kb = twoshot_kb_from_env();
}  // namespace

size_t fused_twoshot_bytes() { return size_t(g_fused_twoshot_kb) << 10; }

long set_fused_twoshot_kb(long kb) {
    const long prev = g_fused_twoshot_kb;
    g_fused_twoshot_kb = kb;
    return prev;
}

bool signal_args(int start, int step, int P, SignalArgs *sa) {
    unsigned long long *mine = heap::signal_area();
    if (!mine || P > kMaxFoldInputs) return false;
    *sa = SignalArgs{};
    sa->mine = mine;
    sa->P = P;
    sa->me = g_state.pe;
    sa->timeout_ticks = signal_timeout_ticks();
    sa->err = signal_error_word();
    const FenceRecords fr = fence_records();
    sa->seen = fr.seen;
    sa->nxcc = fr.nxcc;
    sa->fence_stats = fr.stats;
    const uint64_t sig = heap::signal_offset();
    for (int i = 0; i < P; ++i) {
        const int q = start + i * step;
        char *b = node::peer_base(node::kHeap, q);
        if (!b) return false;
        sa->pe[i] = q;
        sa->peer[i] = reinterpret_cast<const unsigned long long *>(b + sig);
    }
    return true;
}

int direct_stats(double *out, int nout, bool reset) {
    // [calls, 6 phase times, host fences, host refills, device fence
    // checks, device fences that missed an XCD, fused one-shot calls, fused
    // two-shot calls]
    double all[1 + kNumPhases + 6] = {g_calls};
    for (int i = 0; i < kNumPhases; ++i) all[1 + i] = g_phase_us[i];
    unsigned long long dev[2] = {0, 0};
    if (g_fence.dev_stats) {
        device_sync();
        SHMX_HIP(hipMemcpy(dev, g_fence.dev_stats, sizeof dev, hipMemcpyDeviceToHost));
    }
    all[1 + kNumPhases] = g_fence.host_checks;
    all[2 + kNumPhases] = g_fence.host_refills;
    all[3 + kNumPhases] = (double)dev[0];
    all[4 + kNumPhases] = (double)dev[1];
    all[5 + kNumPhases] = g_fused_calls;
    all[6 + kNumPhases] = g_fused2_calls;
    const int k = std::min(nout, (int)(sizeof all / sizeof all[0]));
    for (int i = 0; i < k; ++i) out[i] = all[i];
    if (reset) {
        g_calls = 0;
        for (double &v : g_phase_us) v = 0;
        g_fence.host_checks = g_fence.host_refills = 0;
        g_fused_calls = g_fused2_calls = 0;
        if (g_fence.dev_stats) SHMX_HIP(hipMemset(g_fence.dev_stats, 0, sizeof dev));
    }
    return k;
}

char *ipc_scratch(size_t *bytes) {
    if (!ensure_scratch()) return nullptr;
    *bytes = g_scratch.bytes;
    return g_scratch.base;
}

void direct_release() {
    if (g_fence.host_seen) {
        (void)hipHostFree(g_fence.host_seen);
        (void)hipFree(g_fence.dev_seen);
        (void)hipFree(g_fence.dev_stats);
        (void)hipFree(g_fence.gsync);
        g_fence = FenceState{};
    }
    if (!g_scratch.base) return;
    node::unpublish(node::kScratch);
    (void)hipFree(g_scratch.base);
    g_scratch = Scratch{};
}

namespace {

// DIRECT's one shot as one fused launch (launch_signal_fold): every member's
// source (heap or staged scratch, per the descriptors) and every member's
// heap segment (the signal counters) mapped, then the launch and one wait.
int direct_fused(int type, int op, char *tgt, size_t n, int start, int step, int P, int m,
                 bool own_order, const std::vector<node::Desc> &desc, bool stage_tgt, hipStream_t s) {
    std::vector<std::pair<node::Region, int>> regs;
    for (int i = 0; i < P; ++i) {
        regs.emplace_back(static_cast<node::Region>(desc[i].src.region), start + i * step);
        regs.emplace_back(node::kHeap, start + i * step);
    }
    if (!map_regions(regs, start, step, P)) {
        trace(LOG_REDUCTION, "DIRECT: a member could not map a peer region (%s)", node::last_ipc_error());
        return set_error(SHMEMX_ENOTSUP);
    }
    SignalFoldArgs fa{};
    if (!signal_args(start, step, P, &fa.sig)) fatal("DIRECT", "a mapped peer heap went missing");
    fa.gsync = fence_records().gsync;
    const size_t sz = type_size(type);
    char *const scratch_tgt = g_scratch.base + g_scratch.bytes / 2;
    fa.out = stage_tgt ? scratch_tgt : tgt;
    // set order, or mine (src_me first, then the others ascending)
    auto src_of = [&](int i) {
        return node::peer_base(static_cast<node::Region>(desc[i].src.region), start + i * step) + desc[i].src.off;
    };
    int k = 0;
    if (own_order) fa.ins[k++] = src_of(m);
    for (int i = 0; i < P; ++i)
        if (!own_order || i != m) fa.ins[k++] = src_of(i);
    fa.nins = P;
    fa.n = n;
    // The host spins on a page-locked word instead of waiting for the
    // stream: the kernel stores it itself when one workgroup did all the
    // work (an array of at most 4 elements per lane of one block: the ISx
    // nreduce = 1 call), a marker kernel after it otherwise.
    const HostSignal sig = next_host_signal();
    const bool self_signal = !stage_tgt && n <= kFusedTinyElems;
    if (self_signal) {
        fa.host_word = sig.word;
        fa.host_value = sig.value;
    }
    const double t0 = now_us();
    SHMX_HIP(launch_signal_fold(type, op, fa, s));   // reduce-op.c:217-250
    if (stage_tgt) SHMX_HIP(hipMemcpyAsync(tgt, scratch_tgt, n * sz, hipMemcpyDefault, s));
    if (!self_signal) SHMX_HIP(launch_host_signal(sig, s));
    wait_host_signal(sig, s);
    g_phase_us[kFold] += now_us() - t0;
    count_fused_call();
    switch (signal_error()) {
    case 0: break;
    case 2: fatal("DIRECT reduction", "a system fence before a device barrier missed an XCD");
    default: fatal("DIRECT reduction", "a member never reached the device barrier");
    }
    return SHMEMX_OK;
}

// DIRECT's two shot as one fused launch (launch_signal_fold, two_shot): every
// member's source and target in its heap segment, one chunk.  Slice fold,
// device handshake, gather of the peers' slices, device handshake, in the
// same kernel; then one wait.
int direct_fused2(int type, int op, char *tgt, size_t n, int start, int step, int P, int m,
                  const std::vector<node::Desc> &desc, hipStream_t s) {
    std::vector<std::pair<node::Region, int>> regs;
    for (int i = 0; i < P; ++i) regs.emplace_back(node::kHeap, start + i * step);
    if (!map_regions(regs, start, step, P)) {
        trace(LOG_REDUCTION, "DIRECT: a member could not map a peer heap (%s)", node::last_ipc_error());
        return set_error(SHMEMX_ENOTSUP);
    }
    SignalFoldArgs fa{};
    if (!signal_args(start, step, P, &fa.sig)) fatal("DIRECT", "a mapped peer heap went missing");
    fa.gsync = fence_records().gsync;
    const size_t sz = type_size(type);
    const size_t g = sz >= 16 ? 1 : 16 / sz;
    size_t slice = (n + P - 1) / P;
    slice = (slice + g - 1) / g * g;
    auto lo_of = [&](int i) { return std::min(n, (size_t)i * slice); };
    auto hi_of = [&](int i) { return std::min(n, (size_t)(i + 1) * slice); };
    fa.out = tgt;
    for (int i = 0; i < P; ++i) fa.ins[i] = node::peer_base(node::kHeap, start + i * step) + desc[i].src.off;
    fa.nins = P;
    fa.n = n;
    fa.two_shot = 1;
    fa.lo = lo_of(m);
    fa.hi = hi_of(m);
    for (int i = 0; i < P; ++i) {
        if (i == m || hi_of(i) <= lo_of(i)) continue;
        fa.gsrc[fa.nseg] = node::peer_base(node::kHeap, start + i * step) + desc[i].tgt.off + lo_of(i) * sz;
        fa.gdst[fa.nseg] = tgt + lo_of(i) * sz;
        fa.glen[fa.nseg++] = (hi_of(i) - lo_of(i)) * sz;
    }
    const double t0 = now_us();
    SHMX_HIP(launch_signal_fold(type, op, fa, s));   // reduce-op.c:217-250
    const HostSignal sig = next_host_signal();       // a marker: the host spins, no stream wait
    SHMX_HIP(launch_host_signal(sig, s));
    wait_host_signal(sig, s);
    g_phase_us[kFold] += now_us() - t0;
    count_fused_twoshot_call();
    switch (signal_error()) {
    case 0: break;
    case 2: fatal("DIRECT reduction", "a system fence before a device barrier missed an XCD");
    default: fatal("DIRECT reduction", "a member never reached the device barrier");
    }
    return SHMEMX_OK;
}

}  // namespace

int direct_reduce(int type, int op, char *tgt, const char *src, int nreduce, int start,
                  int logstride, const shmemx_plan_t &p, bool own_order, hipStream_t s) {
    const int P = p.nmembers, m = p.member, step = 1 << logstride;
    if (!node::up()) return set_error(SHMEMX_ENOTSUP);
    if (stream_capturing(s)) return set_error(SHMEMX_ENOTSUP);   // host barriers inside
    if (!own_order && P > kMaxFoldInputs) return set_error(SHMEMX_ENOTSUP);   // one gather launch
    if (!ensure_scratch()) return set_error(SHMEMX_ENOMEM);
    const size_t sz = (size_t)p.elem_size;
    const size_t n = (size_t)nreduce;
    const size_t bytes = n * sz;
    const size_t g = sz >= 16 ? 1 : 16 / sz;
    const size_t half = g_scratch.bytes / 2;
    const size_t cmax = std::max(g, (half / sz) / g * g);   // elements per staged chunk
    auto pe_of = [&](int i) { return start + i * step; };
    // Small arrays: one shot — every member folds the whole array itself (in
    // set order, so all agree, or each in its own) and writes only its own
    // target: one kernel and two barriers instead of two kernels and three.
    // Same decision on every member (n is collective).  Own order is the one
    // shot's schedule at every size.
    const bool one_shot = bytes <= oneshot_bytes();
    const bool local_write = own_order || one_shot;

    // Where my operands live for the peers.  A source that partially
    // overlaps the target (the reference's temporary, reduce-op.c:187-203)
    // or that is outside the heap is staged.  When each PE writes only its
    // own target, the target needs staging only if it aliases the source
    // (the peers still read the source); otherwise the peers read my result
    // slice from it, so it must be in the heap or staged.
    node::Desc d;
    uint64_t off = 0;
    const bool partial = tgt != src && tgt < src + bytes && src < tgt + bytes;
    const bool stage_src = partial || !heap::offset_of(src, bytes, &off);
    if (stage_src) d.src = node::Loc{node::kScratch, 0};
    else d.src = node::Loc{node::kHeap, off};
    bool stage_tgt;
    if (local_write) {
        stage_tgt = tgt < src + bytes && src < tgt + bytes;   // any aliasing
        d.tgt = node::Loc{};
    } else {
        stage_tgt = !heap::offset_of(tgt, bytes, &off);
        if (stage_tgt) d.tgt = node::Loc{node::kScratch, half};
        else d.tgt = node::Loc{node::kHeap, off};
    }
    // count: bit 0 "I stage through scratch", bit 1 "my target starts inside
    // my source" — then chunks must run last to first, as memmove would, or
    // a chunk's copy-out overwrites source elements of the next chunk
    // bit 2: "I can take the fused one-shot launch" (I have the signal
    // counters, at the top of my heap segment)
    // One chunk (n <= cmax, known alike everywhere): stage it right away.
    // bit 3: "I can take the fused two-shot launch" (source and target in my
    // heap segment, one chunk)
    const bool single = n <= cmax;
    const bool twoshot_size = !local_write && bytes <= fused_twoshot_bytes();
    d.count = (stage_src || stage_tgt ? 1 : 0) | (partial && tgt > src ? 2 : 0) |
              (one_shot && single && P <= kMaxFoldInputs && fused_oneshot_enabled() && heap::signal_area() ? 4 : 0) |
              (twoshot_size && single && !stage_src && !stage_tgt && heap::signal_area() ? 8 : 0);
    // aux: the size limits this PE decided with ($SHMEMX_DIRECT_ONESHOT_KB,
    // $SHMEMX_FUSED_TWOSHOT_KB / shmemx_set_fused_twoshot_kb), in KiB.  They
    // pick the schedule (one shot or two, fused or not) and with it the
    // number of barriers, so members that disagree on them must not start it.
    d.aux = (uint64_t)(oneshot_bytes() >> 10) << 32 | (uint64_t)(fused_twoshot_bytes() >> 10);
    node::put_desc(d);
    if (single && stage_src)
        SHMX_HIP(hipMemcpyAsync(g_scratch.base, src, bytes, hipMemcpyDefault, s));
    g_calls += 1;
    std::vector<node::Desc> desc(P);
    auto read_descs = [&] {
        for (int i = 0; i < P; ++i) desc[i] = i == m ? d : node::get_desc(pe_of(i));
    };
    {
        // The descriptors first, with no fence, on every call whatever its
        // size (so the barrier sequence never depends on a local setting).
        // Every member then sees the same descriptors and takes the same
        // path: a collective ENOTSUP if the members' size limits differ;
        // when every member can, the whole call is one fused launch (system
        // fence on every XCD, device barriers, fold (and gather), device
        // barrier — launch_signal_fold) and one wait, instead of fenced host
        // syncs around each kernel.
        const double t0 = now_us();
        node::barrier(start, step, P);
        g_phase_us[kEntryBarrier] += now_us() - t0;
        read_descs();
        for (int i = 1; i < P; ++i) {
            if (desc[i].aux != desc[0].aux) {
                trace(LOG_REDUCTION, "DIRECT: members disagree on SHMEMX_DIRECT_ONESHOT_KB / "
                      "SHMEMX_FUSED_TWOSHOT_KB (set member %d: %llu/%llu KiB, member 0: %llu/%llu KiB)",
                      i, (unsigned long long)(desc[i].aux >> 32), (unsigned long long)(desc[i].aux & 0xffffffffu),
                      (unsigned long long)(desc[0].aux >> 32), (unsigned long long)(desc[0].aux & 0xffffffffu));
                // nobody reads anyone's operands: the call ends here on every
                // member, after one more barrier, so that no member's next
                // call overwrites its descriptor before a slower member has
                // read this call's copy
                node::barrier(start, step, P);
                return set_error(SHMEMX_ENOTSUP);
            }
        }
        if (one_shot || twoshot_size) {
            const int bit = one_shot ? 4 : 8;
            bool fuse = true;
            for (int i = 0; i < P; ++i) fuse &= (desc[i].count & bit) != 0;
            if (fuse && one_shot)
                return direct_fused(type, op, tgt, n, start, step, P, m, own_order, desc, stage_tgt, s);
            if (fuse) return direct_fused2(type, op, tgt, n, start, step, P, m, desc, s);
        }
        // my source (and its staging) is complete; reduce-op.c:217
        node_sync(start, step, P, s, &g_phase_us[kEntryWait], &g_phase_us[kEntryBarrier]);
    }

    // Every member reads the same descriptors, so all cut the same chunks
    // and walk them in the same direction.
    bool chunked = false, backwards = false;
    for (int i = 0; i < P; ++i) {
        chunked |= (desc[i].count & 1) != 0;
        backwards |= (desc[i].count & 2) != 0;
    }
    if (!map_members(desc, local_write, start, step, P)) {
        trace(LOG_REDUCTION, "DIRECT: a member could not map a peer region (%s)", node::last_ipc_error());
        return set_error(SHMEMX_ENOTSUP);
    }
    std::vector<char *> sbase(P), tbase(P);
    for (int i = 0; i < P; ++i) {
        sbase[i] = node::peer_base(static_cast<node::Region>(desc[i].src.region), pe_of(i)) +
                   desc[i].src.off;
        if (!local_write)
            tbase[i] = node::peer_base(static_cast<node::Region>(desc[i].tgt.region), pe_of(i)) +
                       desc[i].tgt.off;
    }
    const size_t C = chunked ? cmax : std::max<size_t>(n, 1);
    const size_t nchunks = (n + C - 1) / C;
    char *const scratch_src = g_scratch.base;
    char *const scratch_tgt = g_scratch.base + half;
    std::vector<const void *> ins(P);
    for (size_t j = 0; j < nchunks; ++j) {
        const size_t k = backwards ? nchunks - 1 - j : j;
        const size_t c0 = k * C, cnt = std::min(C, n - c0);
        if (chunked && !single) {
            // the staged chunk in; the previous chunk's exit barrier has
            // already seen every member done reading my scratch
            if (stage_src)
                SHMX_HIP(hipMemcpyAsync(scratch_src, src + c0 * sz, cnt * sz, hipMemcpyDefault, s));
            node_sync(start, step, P, s, &g_phase_us[kEntryWait], &g_phase_us[kEntryBarrier]);
        }
        // a staged operand holds only the current chunk, at its region offset
        auto at = [&](char *base, const node::Loc &l, size_t elem) {
            return base + (l.region == node::kScratch ? elem - c0 : elem) * sz;
        };
        if (local_write) {
            // own order: src_me first, then the others ascending
            // (reduce-op.c:219-248); one shot: set order
            int k2 = 0;
            if (own_order) ins[k2++] = at(sbase[m], desc[m].src, c0);
            for (int i = 0; i < P; ++i)
                if (!own_order || i != m) ins[k2++] = at(sbase[i], desc[i].src, c0);
            char *out = stage_tgt ? scratch_tgt : tgt + c0 * sz;
            const double tf = now_us();
            fold_chain(type, op, out, ins.data(), P, cnt, s, true);
            // reduce-op.c:250: no member reads my source any more
            node_done(start, step, P, s, &g_phase_us[kFold], &g_phase_us[kExitBarrier], tf);
            if (stage_tgt)
                SHMX_HIP(hipMemcpyAsync(tgt + c0 * sz, scratch_tgt, cnt * sz, hipMemcpyDefault, s));
            continue;
        }
        // two shots: slice i of the chunk belongs to member i
        size_t slice = (cnt + P - 1) / P;
        slice = (slice + g - 1) / g * g;
        auto lo_of = [&](int i) { return std::min(cnt, (size_t)i * slice); };
        auto hi_of = [&](int i) { return std::min(cnt, (size_t)(i + 1) * slice); };
        const size_t lo = lo_of(m), hi = hi_of(m);
        // 1. my slice from every member's source, into my published target
        const double tf = now_us();
        if (hi > lo) {
            for (int i = 0; i < P; ++i) ins[i] = at(sbase[i], desc[i].src, c0 + lo);
            char *out = at(tbase[m], desc[m].tgt, c0 + lo);
            SHMX_HIP(launch_fold_peers(type, op, out, ins.data(), P, hi - lo, s));
        }
        // every member's slice is final
        node_sync(start, step, P, s, &g_phase_us[kFold], &g_phase_us[kFoldBarrier], tf);
        // 2. every other member's slice (and mine, if it was staged) into my target
        std::vector<const void *> from;
        std::vector<void *> to;
        std::vector<size_t> len;
        // from member m + 1 on, wrapping (m itself last, when staged): the
        // gather kernel gives its first blocks to its first segment, so the
        // members start on different peers' slices
        for (int r = 1; r <= P; ++r) {
            const int i = (m + r) % P;
            if (i == m && !stage_tgt) continue;
            if (hi_of(i) <= lo_of(i)) continue;
            from.push_back(at(tbase[i], desc[i].tgt, c0 + lo_of(i)));
            to.push_back(tgt + (c0 + lo_of(i)) * sz);
            len.push_back((hi_of(i) - lo_of(i)) * sz);
        }
        const double tg = now_us();
        SHMX_HIP(launch_gather(from.data(), to.data(), len.data(), (int)from.size(), s));
        // reduce-op.c:250: no member reads my slice any more
        node_done(start, step, P, s, &g_phase_us[kGather], &g_phase_us[kExitBarrier], tg);
    }
    if (local_write && stage_tgt) SHMX_HIP(hipStreamSynchronize(s));
    return SHMEMX_OK;
}

}  // namespace shmx
