// SIGNAL algorithm: DIRECT's pulls (direct.cpp) with the barriers moved onto
// the GPU, so a reduction is pure stream work — no host wait, no host
// barrier, capturable into a hipGraph.
//
// The reference synchronises its reduction with two linear barriers
// (reduce-op.c:217,250; barrier-linear.c:51-77: remote increments of pSync
// counters, then a wait until the local counter has heard from every peer).
// Here each barrier is two stream-ordered launches:
//   launch_sys_fence  every XCD writes back its L2 and drops stale peer lines
//                     (this GPU's results become visible over xGMI); each
//                     block records its XCD;
//   launch_signal     one wave checks that the fence reached every XCD (else
//                     the call fails loudly: error word 2), then bumps this PE's per-peer counters in its own
//                     signal area (system-scope stores) and polls the peers'
//                     counters for it over xGMI (system-scope loads);
// the counters live at the top of every PE's heap segment
// (heap::signal_area), at the same offset on every PE.
//
// Operands must be symmetric — both in the heap, which is what OpenSHMEM
// requires of source and target — so every member computes every peer's
// address from its own offsets, with no descriptor exchange.  A member whose
// operands are not in the heap returns ENOTSUP; its peers' device barriers
// then time out ($SHMEMX_SIGNAL_TIMEOUT seconds, default 20) and the next
// blocking call reports it.
//
// Two-shot (set order, PE_start bits on every member, as DIRECT):
//   barrier                 every source is final; nobody reads my target
//   fold                    slice m of all P sources -> my target's slice m
//   barrier                 every slice is final
//   gather                  the other P-1 slices from the peers' targets
//   barrier                 nobody reads my source or target any more
// — as ONE fused launch up to $SHMEMX_FUSED_TWOSHOT_KB (default 4 MiB):
// launch_signal_fold with two_shot, three handshakes and two grid barriers
// inside one 64-block kernel, instead of seven launches.
// One shot (arrays up to $SHMEMX_DIRECT_ONESHOT_KB, target != source):
//   barrier; fold all of every source -> my target; barrier — as ONE fused
//   launch (launch_signal_fold: the fence, both handshakes and the fold in
//   one kernel, with a self-resetting grid barrier).
// Own order (float / double / long double min and max, own_order_pair): the
//   one shot at every size, each member folding src_me first, then the other
//   members ascending (reduce-op.c:219-248); in place, into the private
//   temporary, copied over the target after the second barrier.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "heap.h"
#include "internal.h"
#include "node.h"
#include "shmem_reduce_mi355x.h"
#include "state.h"

namespace shmx {

namespace {

constexpr size_t kDefaultOneShotBytes = size_t(256) << 10;

size_t oneshot_bytes() {
    static const size_t b = [] {
        const char *e = std::getenv("SHMEMX_DIRECT_ONESHOT_KB");
        return e ? size_t(std::atol(e)) << 10 : kDefaultOneShotBytes;
    }();
    return b;
}

}  // namespace

unsigned long long signal_timeout_ticks() {   // s_memrealtime runs at 100 MHz
    static const unsigned long long t = [] {
        const char *e = std::getenv("SHMEMX_SIGNAL_TIMEOUT");
        const double s = e ? std::atof(e) : 0.0;
        return (unsigned long long)((s > 0 ? s : 20.0) * 1e8);
    }();
    return t;
}

// Host-mapped error word the signal kernels set on a timeout.
unsigned int *signal_error_word() {
    static unsigned int *w = [] {
        void *p = nullptr;
        SHMX_HIP(hipHostMalloc(&p, sizeof(unsigned int), hipHostMallocCoherent));
        *static_cast<volatile unsigned int *>(p) = 0;
        return static_cast<unsigned int *>(p);
    }();
    return w;
}

unsigned int signal_error() {
    volatile unsigned int *w = signal_error_word();
    const unsigned int e = *w;
    *w = 0;
    return e;
}

int signal_reduce(int type, int op, char *tgt, const char *src, int nreduce, int start,
                  int logstride, const shmemx_plan_t &p, bool own_order, hipStream_t s) {
    const int P = p.nmembers, m = p.member, step = 1 << logstride;
    if (!node::up() || P > kMaxFoldInputs) return set_error(SHMEMX_ENOTSUP);
    const size_t sz = (size_t)p.elem_size;
    const size_t n = (size_t)nreduce;
    const size_t bytes = n * sz;
    uint64_t soff = 0, toff = 0;
    const bool partial = tgt != src && tgt < src + bytes && src < tgt + bytes;
    if (partial || !heap::offset_of(src, bytes, &soff) || !heap::offset_of(tgt, bytes, &toff))
        return set_error(SHMEMX_ENOTSUP);
    if (!heap::signal_area()) return set_error(SHMEMX_ENOTSUP);
    // The peers' heap segments: mapped (and voted on) the first time this set
    // meets them, plain lookups afterwards.
    std::vector<std::pair<node::Region, int>> regs;
    for (int i = 0; i < P; ++i) regs.emplace_back(node::kHeap, start + i * step);
    if (!map_regions(regs, start, step, P)) {
        trace(LOG_REDUCTION, "SIGNAL: a member could not map a peer heap (%s)", node::last_ipc_error());
        return set_error(SHMEMX_ENOTSUP);
    }
    SignalArgs sa;
    if (!signal_args(start, step, P, &sa)) return set_error(SHMEMX_ENOTSUP);
    std::vector<char *> hb(P);
    for (int i = 0; i < P; ++i) hb[i] = node::peer_base(node::kHeap, start + i * step);
    // every whole source, in set order, or in my own (src_me first, then
    // the other members ascending: reduce-op.c:219-248)
    const void *ins[kMaxFoldInputs];
    {
        int k = 0;
        if (own_order) ins[k++] = hb[m] + soff;
        for (int i = 0; i < P; ++i)
            if (!own_order || i != m) ins[k++] = hb[i] + soff;
    }
    if (tgt != src && bytes <= oneshot_bytes() && fused_oneshot_enabled()) {
        // barrier, fold of every whole source, barrier: one fused launch
        SignalFoldArgs fa{};
        fa.sig = sa;
        fa.gsync = fence_records().gsync;
        fa.out = tgt;
        for (int i = 0; i < P; ++i) fa.ins[i] = ins[i];
        fa.nins = P;
        fa.n = n;
        SHMX_HIP(launch_signal_fold(type, op, fa, s));   // reduce-op.c:217-250
        count_fused_call();
        return SHMEMX_OK;
    }
    auto barrier = [&] {
        SHMX_HIP(launch_sys_fence(s, sa.seen));
        SHMX_HIP(launch_signal(sa, s));
    };
    if (tgt != src && (bytes <= oneshot_bytes() || own_order)) {   // the one shot, unfused
        barrier();   // reduce-op.c:217
        SHMX_HIP(launch_fold_peers(type, op, tgt, ins, P, n, s));
        barrier();   // reduce-op.c:250
        return SHMEMX_OK;
    }
    if (own_order) {
        // in place: the peers read my source (= my target) until the second
        // barrier, so the fold goes to the private temporary (the
        // reference's own temporary target, reduce-op.c:187-203, 251-259).
        // A captured call cannot allocate it: ENOTSUP before any barrier
        // (the peers' barriers then time out, as for any refused operand).
        if (stream_capturing(s) && g_state.tmp_bytes < bytes) return set_error(SHMEMX_ENOTSUP);
        void *t = grow(g_state.tmp, g_state.tmp_bytes, bytes);
        if (!t) return set_error(SHMEMX_ENOMEM);
        ws_acquire(s);
        barrier();   // reduce-op.c:217
        SHMX_HIP(launch_fold_peers(type, op, t, ins, P, n, s));
        barrier();   // reduce-op.c:250
        SHMX_HIP(hipMemcpyAsync(tgt, t, bytes, hipMemcpyDeviceToDevice, s));
        ws_release(s);
        return SHMEMX_OK;
    }
    const size_t g = sz >= 16 ? 1 : 16 / sz;
    size_t slice = (n + P - 1) / P;
    slice = (slice + g - 1) / g * g;
    auto lo_of = [&](int i) { return std::min(n, (size_t)i * slice); };
    auto hi_of = [&](int i) { return std::min(n, (size_t)(i + 1) * slice); };
    if (bytes <= fused_twoshot_bytes()) {
        // barrier, slice fold, barrier, gather, barrier: one fused launch
        SignalFoldArgs fa{};
        fa.sig = sa;
        fa.gsync = fence_records().gsync;
        fa.out = tgt;
        for (int i = 0; i < P; ++i) fa.ins[i] = hb[i] + soff;
        fa.nins = P;
        fa.n = n;
        fa.two_shot = 1;
        fa.lo = lo_of(m);
        fa.hi = hi_of(m);
        for (int i = 0; i < P; ++i) {
            if (i == m || hi_of(i) <= lo_of(i)) continue;
            fa.gsrc[fa.nseg] = hb[i] + toff + lo_of(i) * sz;
            fa.gdst[fa.nseg] = tgt + lo_of(i) * sz;
            fa.glen[fa.nseg++] = (hi_of(i) - lo_of(i)) * sz;
        }
        SHMX_HIP(launch_signal_fold(type, op, fa, s));   // reduce-op.c:217-250
        count_fused_twoshot_call();
        return SHMEMX_OK;
    }
    barrier();   // reduce-op.c:217
    if (hi_of(m) > lo_of(m)) {
        for (int i = 0; i < P; ++i) ins[i] = hb[i] + soff + lo_of(m) * sz;
        SHMX_HIP(launch_fold_peers(type, op, tgt + lo_of(m) * sz, ins, P, hi_of(m) - lo_of(m), s));
    }
    barrier();   // every member's slice is final
    const void *from[kMaxFoldInputs];
    void *to[kMaxFoldInputs];
    size_t len[kMaxFoldInputs];
    int k = 0;
    // the segments from member m + 1 on, wrapping: the gather kernel gives
    // its first blocks to its first segment, so member m starts on m + 1's
    // slice and no member's HBM and links take every reader at once
    for (int r = 1; r < P; ++r) {
        const int i = (m + r) % P;
        if (hi_of(i) <= lo_of(i)) continue;
        from[k] = hb[i] + toff + lo_of(i) * sz;
        to[k] = tgt + lo_of(i) * sz;
        len[k++] = (hi_of(i) - lo_of(i)) * sz;
    }
    SHMX_HIP(launch_gather(from, to, len, k, s));
    barrier();   // reduce-op.c:250
    return SHMEMX_OK;
}

}  // namespace shmx
