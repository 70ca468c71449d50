// gfx950 (MI355X, CDNA4) kernels for the OpenSHMEM reduction collectives.
//
// One kernel family does all the arithmetic of the path: the element-wise
// left fold of reduce-op.c:213-248,
//     write_to = source_me;  for each other PE p: write_to = op(write_to, src_p)
// here as ONE pass over all inputs instead of one pass per peer:
//     out[i] = op(...op(op(in0[i], in1[i]), in2[i])..., in_{k-1}[i])
// with the element ops of reduce-op.c:71-150 (sum a+b, prod a*b, and/or/xor,
// min a<b?a:b, max a>b?a:b).  nins == 2 with out == in0 is the reference's
// inner fold write_to[ti] = op(write_to[ti], pWrk[j]) (reduce-op.c:231-235);
// nins == 1 is the copy of reduce-op.c:213-216.
//
// Design for gfx950 (DESIGN.md "Kernels"):
//   * HBM-bound streaming: 16-byte loads/stores per lane (global_load_dwordx4),
//     a wave-instruction covers 1 KiB contiguous; UNROLL independent vectors
//     per input per lane are issued before any op, so a 256-lane workgroup
//     keeps UNROLL*nins*4 KiB in flight;
//   * whole-chunk fast path with no per-vector guards (a guarded unrolled load
//     makes hipcc wait vmcnt(0) per element), guarded path only for the last
//     partial chunk;
//   * scalar head/tail peeling so 8-byte-aligned (dlmalloc, dlmalloc.c:557)
//     or odd-length arrays still take the vector body;
//   * no LDS, no DPP: an element-wise fold has no intra-wave reduction and no
//     reuse, so an LDS round trip would be pure overhead;
//   * bit-exact with the reference's C: integers wrap in unsigned arithmetic,
//     short is computed in int and truncated, no FP contraction
//     (-ffp-contract=off), min/max are selects (not v_min_f64, whose NaN / -0
//     behaviour differs), complex products follow C99 Annex G / libgcc
//     __muldc3 including its NaN-recovery branch.
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "fold_ops.h"

namespace shmx {

// ------------------------------------------------------------ kernel clock
// shmemx_kernel_timing(1): the fold-family launches (2-input and P-input
// folds, the copy, the peers fold, the gather) go through
// hipExtLaunchKernelGGL with a start / stop event pair: the dispatch's own
// timestamps, i.e. the kernel alone, with no launch boundary and no
// event-marker latency (a marker pair around a 9 us fold reads 14.7 us,
// rocprofv3 8.6, profiles/r04_midsize.txt).  shmemx_kernel_times() hands
// the durations back in launch order.  Off (the default), the launches are
// plain hipLaunchKernelGGL.
enum KernelKind { kKindFold = 0, kKindCopy = 1, kKindPeers = 2, kKindGather = 3 };
namespace {
constexpr size_t kClockPairs = 4096;
struct KClock {
    std::mutex mu;
    std::atomic<bool> on{false};
    std::vector<hipEvent_t> ev;   // 2 per launch, created on first use
    std::vector<int> kind;
    size_t used = 0;              // pairs handed out since the last read
    size_t dropped = 0;           // launches past the ring, not timed
} g_kclock;

// a start / stop pair for the next launch, or false (timing off, ring full)
bool clock_pair(int kind, hipEvent_t *a, hipEvent_t *b) {
    if (!g_kclock.on.load(std::memory_order_relaxed)) return false;
    std::lock_guard<std::mutex> lk(g_kclock.mu);
    if (g_kclock.used >= kClockPairs) {
        ++g_kclock.dropped;
        return false;
    }
    if (g_kclock.ev.size() < 2 * (g_kclock.used + 1)) {
        // both events or neither: ev stays two per pair, kind one per pair
        hipEvent_t e0, e1;
        if (hipEventCreate(&e0) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (hipEventCreate(&e1) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipEventDestroy(e0);
            return false;
        }
        g_kclock.ev.push_back(e0);
        g_kclock.ev.push_back(e1);
        g_kclock.kind.push_back(0);
    }
    *a = g_kclock.ev[2 * g_kclock.used];
    *b = g_kclock.ev[2 * g_kclock.used + 1];
    g_kclock.kind[g_kclock.used++] = kind;
    return true;
}

// launches captured into a hipGraph are never timed (their events would
// belong to the capture, not to a run)
bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

template <typename K, typename... Args>
void launch_k(int kind, K kernel, dim3 grid, dim3 block, hipStream_t s, Args... args) {
    hipEvent_t a, b;
    if (g_kclock.on.load(std::memory_order_relaxed) && !capturing(s) && clock_pair(kind, &a, &b))
        hipExtLaunchKernelGGL(kernel, grid, block, 0, s, a, b, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
}
}  // namespace

int kernel_timing(int on) {
    std::lock_guard<std::mutex> lk(g_kclock.mu);
    g_kclock.on.store(on != 0);
    g_kclock.used = 0;
    g_kclock.dropped = 0;
    return 0;
}

int kernel_times(double *us, int *kind, int max, unsigned long long *dropped) {
    std::lock_guard<std::mutex> lk(g_kclock.mu);
    const int n = (int)std::min<size_t>(g_kclock.used, max > 0 ? (size_t)max : 0);
    for (int i = 0; i < n; ++i) {
        float ms = 0.f;
        if (hipEventSynchronize(g_kclock.ev[2 * i + 1]) != hipSuccess ||
            hipEventElapsedTime(&ms, g_kclock.ev[2 * i], g_kclock.ev[2 * i + 1]) != hipSuccess)
            return -1;
        us[i] = ms * 1e3;
        if (kind) kind[i] = g_kclock.kind[i];
    }
    if (dropped) *dropped = g_kclock.dropped;
    g_kclock.used = 0;
    g_kclock.dropped = 0;
    return n;
}

namespace {

struct FoldArgs {
    void *out;
    const void *ins[kMaxFoldInputs];
    int nins;
    size_t head;   // scalar elements before the first 16-B aligned vector
    size_t nvec;   // 16-B vectors in the aligned body
    size_t tail;   // scalar elements after it
    int peers;     // the inputs are other GPUs' HBM (launch_fold_peers)
    // one-workgroup launches of launch_fold_signal: store sig_value here when done
    unsigned long long *sig_word;
    unsigned long long sig_value;
    // a copy (nins == 1) may store to a second destination too
    // (launch_copy2_signal: a small blocking result into HBM and into the
    // mirrored heap's view in one launch); nullptr otherwise
    void *out2;
};

// The end of a one-workgroup fold that signals the host (launch_fold_signal):
// every wave drains its stores, the workgroup meets, and lane 0 stores the
// value with a system-scope release (the L2 written back first), so the host
// that sees it may use the result at once.
__device__ __forceinline__ void signal_host_done(const FoldArgs &args) {
    if (!args.sig_word) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(args.sig_word, args.sig_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}


// NIN > 0: number of inputs fixed at compile time (all loads hoisted);
// NIN == 0: runtime args.nins.
template <typename T, int OP, int NIN, int UNROLL, int NT>
__device__ __forceinline__ void fold_body(const FoldArgs &args) {
    constexpr int E = 16 / sizeof(T);
    const int nins = NIN > 0 ? NIN : args.nins;
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * kBlock;

    // Scalar head and tail (grid-stride: the whole array when the inputs
    // do not share one alignment).
    {
        T *out = static_cast<T *>(args.out);
        const size_t body_end = args.head + args.nvec * E;
        const size_t nscalar = args.head + args.tail;
        for (size_t s = tid; s < nscalar; s += nthr) {
            const size_t i = s < args.head ? s : body_end + (s - args.head);
            T acc = static_cast<const T *>(args.ins[0])[i];
            for (int k = 1; k < nins; ++k)
                acc = Op<T, OP>::ap(acc, static_cast<const T *>(args.ins[k])[i]);
            out[i] = acc;
            if constexpr (NIN == 1)
                if (args.out2) static_cast<T *>(args.out2)[i] = acc;
        }
    }
    if (args.nvec == 0) return;

    u32x4 *out = reinterpret_cast<u32x4 *>(static_cast<T *>(args.out) + args.head);
    u32x4 *out2 = NIN == 1 && args.out2 ? reinterpret_cast<u32x4 *>(static_cast<T *>(args.out2) + args.head)
                                        : nullptr;
    const size_t nvec = args.nvec;
    const size_t step = (size_t)gridDim.x * kBlock * UNROLL;
    for (size_t base = (size_t)blockIdx.x * kBlock * UNROLL; base < nvec;
         base += step) {
        const size_t v0 = base + threadIdx.x;
        if (base + (size_t)kBlock * UNROLL <= nvec) {
            // whole chunk in range: unguarded, every load issued up front
            u32x4 acc[UNROLL];
            const u32x4 *in0 = reinterpret_cast<const u32x4 *>(
                static_cast<const T *>(args.ins[0]) + args.head);
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) acc[u] = ld16<NT>(in0 + v0 + u * kBlock);
            if constexpr (NIN > 0) {
                u32x4 x[NIN > 1 ? NIN - 1 : 1][UNROLL];
#pragma unroll
                for (int k = 1; k < NIN; ++k) {
                    const u32x4 *ink = reinterpret_cast<const u32x4 *>(
                        static_cast<const T *>(args.ins[k]) + args.head);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u)
                        x[k - 1][u] = ld16<NT>(ink + v0 + u * kBlock);
                }
#pragma unroll
                for (int k = 1; k < NIN; ++k)
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u)
                        acc[u] = apply16<T, OP>(acc[u], x[k - 1][u]);
            } else if (std::is_same<T, ld80>::value && nins >= 3) {
                // soft-float ops are long: input k + 1's loads are issued
                // before input k is folded, so the arithmetic overlaps them
                // (P = 8 long double sum 115 -> 107 us)
                auto in_k = [&](int k) {
                    return reinterpret_cast<const u32x4 *>(static_cast<const T *>(args.ins[k]) + args.head);
                };
                u32x4 cur[UNROLL];
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) cur[u] = ld16<NT>(in_k(1) + v0 + u * kBlock);
                for (int k = 2; k < nins; ++k) {
                    u32x4 nxt[UNROLL];
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) nxt[u] = ld16<NT>(in_k(k) + v0 + u * kBlock);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) {
                        acc[u] = apply16<T, OP>(acc[u], cur[u]);
                        cur[u] = nxt[u];
                    }
                }
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) acc[u] = apply16<T, OP>(acc[u], cur[u]);
            } else {
                for (int k = 1; k < nins; ++k) {
                    const u32x4 *ink = reinterpret_cast<const u32x4 *>(
                        static_cast<const T *>(args.ins[k]) + args.head);
                    u32x4 x[UNROLL];
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) x[u] = ld16<NT>(ink + v0 + u * kBlock);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) acc[u] = apply16<T, OP>(acc[u], x[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) st16<NT>(out + v0 + u * kBlock, acc[u]);
            if constexpr (NIN == 1)
                if (out2)
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) st16<NT>(out2 + v0 + u * kBlock, acc[u]);
        } else {
            // last partial chunk: one vector at a time, guarded
            for (int u = 0; u < UNROLL; ++u) {
                const size_t v = v0 + (size_t)u * kBlock;
                if (v >= nvec) break;
                u32x4 acc = ld16<NT>(reinterpret_cast<const u32x4 *>(
                                         static_cast<const T *>(args.ins[0]) + args.head) + v);
                for (int k = 1; k < nins; ++k)
                    acc = apply16<T, OP>(acc, ld16<NT>(reinterpret_cast<const u32x4 *>(
                                                 static_cast<const T *>(args.ins[k]) + args.head) + v));
                st16<NT>(out + v, acc);
                if constexpr (NIN == 1)
                    if (out2) st16<NT>(out2 + v, acc);
            }
        }
    }
}

template <typename T, int OP, int NIN, int UNROLL, int NT>
__global__ __launch_bounds__(kBlock) void fold_kernel(FoldArgs args) {
    fold_body<T, OP, NIN, UNROLL, NT>(args);
    signal_host_done(args);
}

// 16-B vectors per lane per input for the runtime-nins kernel, and for the
// two-input fold (2 and 8 measured no faster at 32-64 Mi elements:
// DESIGN_history.md §4.2).
constexpr int kUnrollN = 4;
constexpr int kUnrollFold2 = 4;

// The P-input fold over inputs that live in the peers' HBM (DIRECT's and
// SIGNAL's fold phase).  The runtime-nins kernel above issues input k + 1's
// loads only after folding input k; with every input on another GPU, every
// resident wave would then wait on the same peer's link at the same time
// (all blocks start at input 0 together and stay in step behind that one
// link), so only one of the P - 1 links would carry traffic at a time.  Here
// every lane issues its U vectors of ALL inputs before folding any (uniform
// predicates, unrolled), so each wave has loads in flight on every link: 4
// vectors per input up to 8 inputs (32 in registers), 2 up to 16.  Round 2
// kept 16 vectors (2 per input at 8 inputs); at P = 8 x 16 Mi doubles on
// local HBM 4 per input runs 201.0 against 204.2 us, 1 per input 345 us
// (tools/peers_gather_lab.hip, profiles/r03_peers_gather_lab.txt).  The fold
// order is unchanged: input 0, then 1, ...
constexpr int peers_unroll(int maxin) { return maxin <= 8 ? 4 : 2; }

template <typename T, int OP, int MAXIN, int NT>
__global__ __launch_bounds__(kBlock) void fold_peers_kernel(FoldArgs args) {
    constexpr int E = 16 / sizeof(T);
    constexpr int U = peers_unroll(MAXIN);
    const int nins = args.nins;
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * kBlock;
    {
        T *out = static_cast<T *>(args.out);
        const size_t body_end = args.head + args.nvec * E;
        const size_t nscalar = args.head + args.tail;
        for (size_t s = tid; s < nscalar; s += nthr) {
            const size_t i = s < args.head ? s : body_end + (s - args.head);
            T acc = static_cast<const T *>(args.ins[0])[i];
            for (int k = 1; k < nins; ++k) acc = Op<T, OP>::ap(acc, static_cast<const T *>(args.ins[k])[i]);
            out[i] = acc;
        }
    }
    if (args.nvec == 0) return;
    auto in = [&](int k) {
        return reinterpret_cast<const u32x4 *>(static_cast<const T *>(args.ins[k]) + args.head);
    };
    u32x4 *out = reinterpret_cast<u32x4 *>(static_cast<T *>(args.out) + args.head);
    const size_t nvec = args.nvec;
    const size_t step = (size_t)gridDim.x * kBlock * U;
    for (size_t base = (size_t)blockIdx.x * kBlock * U; base < nvec; base += step) {
        const size_t v0 = base + threadIdx.x;
        if (base + (size_t)kBlock * U <= nvec) {
            u32x4 x[MAXIN][U];
#pragma unroll
            for (int k = 0; k < MAXIN; ++k)
                if (k < nins)
#pragma unroll
                    for (int u = 0; u < U; ++u) x[k][u] = ld16<NT>(in(k) + v0 + u * kBlock);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                u32x4 acc = x[0][u];
#pragma unroll
                for (int k = 1; k < MAXIN; ++k)
                    if (k < nins) acc = apply16<T, OP>(acc, x[k][u]);
                st16<NT>(out + v0 + u * kBlock, acc);
            }
        } else {
            for (int u = 0; u < U; ++u) {
                const size_t v = v0 + (size_t)u * kBlock;
                if (v >= nvec) break;
                u32x4 acc = ld16<NT>(in(0) + v);
                for (int k = 1; k < nins; ++k) acc = apply16<T, OP>(acc, ld16<NT>(in(k) + v));
                st16<NT>(out + v, acc);
            }
        }
    }
}


// One chunk of kBlock x unroll vectors per block (persistent grids, caps and
// XCD remaps measured no faster: DESIGN_history.md §4.2); the scalar-only
// case (inputs of different alignment) grid-strides over at most 2048 blocks.
static size_t grid_for(const FoldArgs &a, int unroll) {
    size_t work_blocks;
    if (a.nvec > 0)
        work_blocks = (a.nvec + (size_t)kBlock * unroll - 1) / ((size_t)kBlock * unroll);
    else
        work_blocks = (a.head + a.tail + kBlock - 1) / kBlock;
    const size_t cap = a.nvec == 0 ? 2048 : (size_t)1 << 30;
    size_t blocks = work_blocks < cap ? work_blocks : cap;
    if (blocks < 1) blocks = 1;
    if (blocks > (size_t)INT_MAX) blocks = INT_MAX;
    return blocks;
}

// The marker after the work: the stream's own value write (the command
// processor stores the word once everything before it on the stream has
// completed, its kernels' end-of-kernel releases included), 0.3-0.8 us
// faster per small call than a one-thread kernel storing it
// (profiles/r05_marker_ab.txt).  It publishes a multi-block result only
// through the preceding kernel's end-of-kernel release, which is system
// scope (HIP's default for a dispatch) and writes back every XCD's L2 (a
// marker kernel's own release would reach only the XCD it ran on, so it
// would not cover such a result either).  One-workgroup folds store the
// signal themselves after their own system-scope release.
hipError_t enqueue_marker(unsigned long long *word, unsigned long long value, hipStream_t stream) {
    return hipStreamWriteValue64(stream, word, value, 0);
}

template <typename T, int OP, int NT>
hipError_t launch_typed_grid(const FoldArgs &a, hipStream_t stream);

// A fold whose grid is not one workgroup cannot signal from inside (no
// arrival counter): it runs without, and the marker kernel follows it.
template <typename T, int OP, int NT>
hipError_t launch_typed(const FoldArgs &a0, hipStream_t stream) {
    if (!a0.sig_word) return launch_typed_grid<T, OP, NT>(a0, stream);
    // the grid launch_typed_grid will use (fold_kernel in every case but
    // the peers kernel, which never signals)
    const int u = a0.nins != 2 ? kUnrollN : kUnrollFold2;
    if (!a0.peers && grid_for(a0, u) == 1) return launch_typed_grid<T, OP, NT>(a0, stream);
    FoldArgs a = a0;
    a.sig_word = nullptr;
    const hipError_t e = launch_typed_grid<T, OP, NT>(a, stream);
    if (e != hipSuccess) return e;
    return enqueue_marker(a0.sig_word, a0.sig_value, stream);
}

template <typename T, int OP, int NT>
hipError_t launch_typed_grid(const FoldArgs &a, hipStream_t stream) {
    if (a.nins == 2) {
        // the two-input fold (reduce-op.c:231-235): the hot kernel
        launch_k(kKindFold, fold_kernel<T, OP, 2, kUnrollFold2, NT>, dim3((unsigned)grid_for(a, kUnrollFold2)),
                 dim3(kBlock), stream, a);
    } else if (a.peers && !kHeavyOp<T, OP>) {
        if (a.nins <= 4)
            launch_k(kKindPeers, fold_peers_kernel<T, OP, 4, NT>,
                     dim3((unsigned)grid_for(a, peers_unroll(4))), dim3(kBlock), stream, a);
        else if (a.nins <= 8)
            launch_k(kKindPeers, fold_peers_kernel<T, OP, 8, NT>,
                     dim3((unsigned)grid_for(a, peers_unroll(8))), dim3(kBlock), stream, a);
        else
            launch_k(kKindPeers, fold_peers_kernel<T, OP, 16, NT>,
                     dim3((unsigned)grid_for(a, peers_unroll(16))), dim3(kBlock), stream, a);
    } else {
        launch_k(kKindFold, fold_kernel<T, OP, 0, kUnrollN, NT>, dim3((unsigned)grid_for(a, kUnrollN)),
                 dim3(kBlock), stream, a);
    }
    return hipGetLastError();
}

// Cache policy: working sets of 32 MiB and more go non-temporal on both
// loads and stores.  Round 1 set the cut at the 256 MiB Infinity Cache from
// back-to-back (warm) runs; round 3 measured the 4-64 Mi-float fold cold
// (tools/cold_midsize_probe.py, profiles/r03_cold_midsize.txt): after a
// producer's writes leave dirty lines in the MALL, the default policy runs
// 3.1 / 4.1 TB/s at 48 / 192 MiB against 4.3 / 5.8 non-temporal (the
// default's stores evict those lines and pay their write-back); from a clean
// cache the default leads by 5-7 %, back to back the two tie.  So
// non-temporal, whose worst case is the better one, from 32 MiB up; below
// it a call is launch-bound and the default keeps L2/MALL hits.  (Loads or
// stores alone non-temporal, and the sc0/sc1 bits, measured no better:
// profiles/r03_policy_lab*.txt.)
constexpr size_t kNtThresholdBytes = size_t(32) << 20;

template <typename T, int OP>
hipError_t launch_nt(const FoldArgs &a, hipStream_t stream) {
    const size_t n = a.head + a.nvec * (16 / sizeof(T)) + a.tail;
    return (size_t)(a.nins + 1) * n * sizeof(T) >= kNtThresholdBytes ? launch_typed<T, OP, 3>(a, stream)
                                                                      : launch_typed<T, OP, 0>(a, stream);
}

// The copy (nins == 1: reduce-op.c:213-216, the whole PE_size = 1 call, and
// the private copy of an overlapping source): a compile-time one-input
// instance of the fold, non-temporal loads and stores from 32 MiB moved.  A
// copy moves bits, so it runs on one type per element size (short, int,
// long, and a 16-byte struct for complex double and long double) with no
// arithmetic.  Shape: ONE 16-B vector per lane, 4 KiB per workgroup, for
// large copies; up to 32 KiB, 8 vectors per lane, so the copy is one
// workgroup that can store the host signal itself (launch_fold_signal).
// Measured (tools/stream_lab.hip, profiles/r04_stream_lab_copy2_*.txt, in-stream
// cost after a flush, which also charges deferred write-backs; 256 / 512
// MiB): 1 vector per lane 6.44 / 6.55 TB/s, 8 vectors 6.38 / 6.18, 4 vectors
// 6.09 / 6.04, 64- or 128-lane blocks and wave-contiguous layouts 6.1-6.35;
// stores of 4 KiB per workgroup are the fast write shape
// (profiles/r04_stream_lab_write_*.txt: 6.7-6.9 against 6.0 at 16 KiB).
// Through the library (tools/copy_probe.py, profiles/r04_copy_probe.txt):
// 83.7 us at 256 MiB, 166.6 us at 512 MiB (6.41-6.44 TB/s).
// Default-policy stores look faster by kernel time alone (6.9-7.1) but leave
// up to 256 MiB dirty in the Infinity Cache for the next kernel to write back
// (4.9-5.2 TB/s charged), so the stores stay non-temporal.
constexpr int kUnrollCopy = 8;       // small copies: one workgroup up to 32 KiB
constexpr int kUnrollCopyLarge = 1;  // large copies: 4 KiB per workgroup

template <typename T, int NT>
hipError_t launch_copy_nt(const FoldArgs &a0, hipStream_t stream) {
    const bool small = a0.nvec <= (size_t)kBlock * kUnrollCopy;
    const size_t blocks = grid_for(a0, small ? kUnrollCopy : kUnrollCopyLarge);
    // a one-workgroup copy stores the host signal itself (launch_fold_signal);
    // a larger grid is followed by the marker kernel
    const bool self_signal = a0.sig_word && blocks == 1;
    FoldArgs a = a0;
    if (!self_signal) a.sig_word = nullptr;
    if (small)
        launch_k(kKindCopy, fold_kernel<T, SHMEMX_OP_SUM, 1, kUnrollCopy, NT>, dim3((unsigned)blocks), dim3(kBlock),
                 stream, a);
    else
        launch_k(kKindCopy, fold_kernel<T, SHMEMX_OP_SUM, 1, kUnrollCopyLarge, NT>, dim3((unsigned)blocks),
                 dim3(kBlock), stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || !a0.sig_word || self_signal) return e;
    return enqueue_marker(a0.sig_word, a0.sig_value, stream);
}

template <typename T>
hipError_t launch_copy(const FoldArgs &a, hipStream_t stream) {
    const size_t n = a.head + a.nvec * (16 / sizeof(T)) + a.tail;
    return 2 * n * sizeof(T) >= kNtThresholdBytes ? launch_copy_nt<T, 3>(a, stream)
                                                  : launch_copy_nt<T, 0>(a, stream);
}

template <typename T>
hipError_t launch_int_ops(int op, const FoldArgs &a, hipStream_t s) {
    switch (op) {
    case SHMEMX_OP_SUM: return launch_nt<T, SHMEMX_OP_SUM>(a, s);
    case SHMEMX_OP_PROD: return launch_nt<T, SHMEMX_OP_PROD>(a, s);
    case SHMEMX_OP_AND: return launch_nt<T, SHMEMX_OP_AND>(a, s);
    case SHMEMX_OP_OR: return launch_nt<T, SHMEMX_OP_OR>(a, s);
    case SHMEMX_OP_XOR: return launch_nt<T, SHMEMX_OP_XOR>(a, s);
    case SHMEMX_OP_MIN: return launch_nt<T, SHMEMX_OP_MIN>(a, s);
    case SHMEMX_OP_MAX: return launch_nt<T, SHMEMX_OP_MAX>(a, s);
    default: return hipErrorInvalidValue;
    }
}
template <typename T>
hipError_t launch_fp_ops(int op, const FoldArgs &a, hipStream_t s) {
    switch (op) {
    case SHMEMX_OP_SUM: return launch_nt<T, SHMEMX_OP_SUM>(a, s);
    case SHMEMX_OP_PROD: return launch_nt<T, SHMEMX_OP_PROD>(a, s);
    case SHMEMX_OP_MIN: return launch_nt<T, SHMEMX_OP_MIN>(a, s);
    case SHMEMX_OP_MAX: return launch_nt<T, SHMEMX_OP_MAX>(a, s);
    default: return hipErrorInvalidValue;
    }
}
template <typename T>
hipError_t launch_cplx_ops(int op, const FoldArgs &a, hipStream_t s) {
    switch (op) {
    case SHMEMX_OP_SUM: return launch_nt<T, SHMEMX_OP_SUM>(a, s);
    case SHMEMX_OP_PROD: return launch_nt<T, SHMEMX_OP_PROD>(a, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

size_t type_size(int type) {
    switch (type) {
    case SHMEMX_TYPE_SHORT: return sizeof(short);
    case SHMEMX_TYPE_INT: return sizeof(int);
    case SHMEMX_TYPE_LONG: return sizeof(long);
    case SHMEMX_TYPE_LONGLONG: return sizeof(long long);
    case SHMEMX_TYPE_FLOAT: return sizeof(float);
    case SHMEMX_TYPE_DOUBLE: return sizeof(double);
    case SHMEMX_TYPE_LONGDOUBLE: return sizeof(long double);
    case SHMEMX_TYPE_COMPLEXD: return 2 * sizeof(double);
    case SHMEMX_TYPE_COMPLEXF: return 2 * sizeof(float);
    default: return 0;
    }
}

bool op_valid(int type, int op) {
    if (type < 0 || type >= SHMEMX_NTYPES || op < 0 || op >= SHMEMX_NOPS) return false;
    switch (op) {
    case SHMEMX_OP_SUM:
    case SHMEMX_OP_PROD: return true;
    case SHMEMX_OP_AND:
    case SHMEMX_OP_OR:
    case SHMEMX_OP_XOR: return type <= SHMEMX_TYPE_LONGLONG;
    default: return type != SHMEMX_TYPE_COMPLEXD && type != SHMEMX_TYPE_COMPLEXF;
    }
}

bool op_on_device(int type, int op) { return op_valid(type, op); }

namespace {

// Split n elements into scalar head, 16-B vector body and scalar tail, given
// every array's address (the body only if all share one offset mod 16 that is
// a whole number of elements), then dispatch on type.
hipError_t dispatch(int type, int op, FoldArgs &a, const void *const *ptrs, int nptrs, size_t n,
                    hipStream_t stream) {
    const size_t sz = type_size(type);
    const uintptr_t off = reinterpret_cast<uintptr_t>(ptrs[0]) & 15u;
    bool same = (off % sz) == 0;
    for (int k = 1; k < nptrs && same; ++k)
        same = (reinterpret_cast<uintptr_t>(ptrs[k]) & 15u) == off;
    if (same) {
        size_t head = ((16 - off) & 15u) / sz;
        if (head > n) head = n;
        const size_t E = 16 / sz;
        a.head = head;
        a.nvec = (n - head) / E;
        a.tail = n - head - a.nvec * E;
    } else {
        a.head = n;
        a.nvec = 0;
        a.tail = 0;
    }
    if (a.nins == 1) {   // a copy: bits only, one kernel per element size
        switch (sz) {
        case 2: return launch_copy<short>(a, stream);
        case 4: return launch_copy<int>(a, stream);
        case 8: return launch_copy<long>(a, stream);
        case 16: return launch_copy<cplxd>(a, stream);
        default: return hipErrorInvalidValue;
        }
    }
    switch (type) {
    case SHMEMX_TYPE_SHORT: return launch_int_ops<short>(op, a, stream);
    case SHMEMX_TYPE_INT: return launch_int_ops<int>(op, a, stream);
    case SHMEMX_TYPE_LONG:
    case SHMEMX_TYPE_LONGLONG: return launch_int_ops<long>(op, a, stream);
    case SHMEMX_TYPE_FLOAT: return launch_fp_ops<float>(op, a, stream);
    case SHMEMX_TYPE_DOUBLE: return launch_fp_ops<double>(op, a, stream);
    case SHMEMX_TYPE_LONGDOUBLE: return launch_fp_ops<ld80>(op, a, stream);
    case SHMEMX_TYPE_COMPLEXD: return launch_cplx_ops<cplxd>(op, a, stream);
    case SHMEMX_TYPE_COMPLEXF: return launch_cplx_ops<cplxf>(op, a, stream);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_fold(int type, int op, void *out, const void *const *ins,
                       int nins, size_t n, hipStream_t stream) {
    if (!op_on_device(type, op) || nins < 1 || nins > kMaxFoldInputs || !out)
        return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    FoldArgs a{};
    a.out = out;
    a.nins = nins;
    const void *ptrs[kMaxFoldInputs + 1];
    ptrs[0] = out;
    for (int k = 0; k < nins; ++k) {
        if (!ins[k]) return hipErrorInvalidValue;
        a.ins[k] = ins[k];
        ptrs[k + 1] = ins[k];
    }
    return dispatch(type, op, a, ptrs, nins + 1, n, stream);
}

bool copy_one_workgroup(int type, const void *dst, const void *src, size_t n) {
    const size_t sz = type_size(type);
    if (!sz || !n) return false;
    const uintptr_t off = reinterpret_cast<uintptr_t>(dst) & 15u;
    if (off % sz != 0 || (reinterpret_cast<uintptr_t>(src) & 15u) != off)
        return n <= (size_t)kBlock;                    // all scalar: ceil(n / kBlock) blocks
    size_t head = ((16 - off) & 15u) / sz;
    if (head > n) head = n;
    const size_t E = 16 / sz, nvec = (n - head) / E, tail = n - head - nvec * E;
    if (nvec == 0) return head + tail <= (size_t)kBlock;
    return nvec <= (size_t)kBlock * kUnrollCopy;       // grid_for: one chunk per block
}

hipError_t launch_fold_signal(int type, int op, void *out, const void *const *ins, int nins, size_t n,
                              hipStream_t stream, const HostSignal &sig) {
    if (!op_on_device(type, op) || nins < 1 || nins > kMaxFoldInputs || !out || !sig.word)
        return hipErrorInvalidValue;
    if (n == 0) return launch_host_signal(sig, stream);
    FoldArgs a{};
    a.out = out;
    a.nins = nins;
    a.sig_word = sig.word;
    a.sig_value = sig.value;
    const void *ptrs[kMaxFoldInputs + 1];
    ptrs[0] = out;
    for (int k = 0; k < nins; ++k) {
        if (!ins[k]) return hipErrorInvalidValue;
        a.ins[k] = ins[k];
        ptrs[k + 1] = ins[k];
    }
    return dispatch(type, op, a, ptrs, nins + 1, n, stream);
}

hipError_t launch_copy2_signal(int type, void *out, void *out2, const void *in, size_t n, hipStream_t stream,
                               const HostSignal &sig) {
    if (!op_on_device(type, SHMEMX_OP_SUM) || !out || !out2 || !in || !sig.word) return hipErrorInvalidValue;
    if (n == 0) return launch_host_signal(sig, stream);
    FoldArgs a{};
    a.out = out;
    a.out2 = out2;
    a.nins = 1;
    a.ins[0] = in;
    a.sig_word = sig.word;
    a.sig_value = sig.value;
    const void *ptrs[3] = {out, out2, in};   // the vector body needs all three on one alignment
    return dispatch(type, SHMEMX_OP_SUM, a, ptrs, 3, n, stream);
}

hipError_t launch_host_signal(const HostSignal &sig, hipStream_t stream) {
    if (!sig.word) return hipErrorInvalidValue;
    return enqueue_marker(sig.word, sig.value, stream);
}

hipError_t launch_fold_peers(int type, int op, void *out, const void *const *ins, int nins, size_t n,
                             hipStream_t stream) {
    if (!op_on_device(type, op) || nins < 1 || nins > kMaxFoldInputs || !out)
        return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    FoldArgs a{};
    a.out = out;
    a.nins = nins;
    a.peers = 1;
    const void *ptrs[kMaxFoldInputs + 1];
    ptrs[0] = out;
    for (int k = 0; k < nins; ++k) {
        if (!ins[k]) return hipErrorInvalidValue;
        a.ins[k] = ins[k];
        ptrs[k + 1] = ins[k];
    }
    return dispatch(type, op, a, ptrs, nins + 1, n, stream);
}

// ------------------------------------------------------------ gather copy
// DIRECT's all-gather phase: up to kMaxFoldInputs byte ranges (each a slice
// of a peer's result, read over xGMI) copied into this PE's target by ONE
// launch, so the reads from all peers are in flight at once (one copy per
// peer would serialise the links).  Workgroups are dispatched in block
// order, so the block -> segment map decides which links are busy: with the
// segment as the slow index (blockIdx.y) the first ~2048 resident blocks
// would all read the same peer, one link at a time.  Consecutive RUNS of
// kGatherRun blocks take the segments in turn: a resident grid of ~2048
// blocks still spans every segment (kGatherRun x 7 = 1792), and each run
// streams 8 MiB contiguous per segment.  Measured on local HBM, 7 x 32 MiB
// (profiles/archive/r02c_pmc_kernels.json, profiles/r03_peers_gather_lab*.txt):
// blockIdx.y-major 77.4 us; single blocks in turn (round 2) 80.5, with 2
// vectors per lane 79.3; runs of 16-64 blocks 82-89; runs of 256 blocks
// with 8 vectors per lane 72.5 us warm, 74.9 cold (6.48 / 6.27 TB/s), the
// fastest shape of all, y-major included.
namespace {

struct CopySeg {
    const unsigned char *src;
    unsigned char *dst;
    size_t bytes;
};
struct GatherArgs {
    CopySeg seg[kMaxFoldInputs];
    int nseg;
    unsigned run;   // blocks per run (divides the blocks per segment)
};

constexpr int kGatherUnroll = 8;
constexpr unsigned kGatherRun = 256;

__global__ __launch_bounds__(kBlock) void gather_kernel(GatherArgs a) {
    const unsigned r = blockIdx.x / a.run;   // the run, and its segment
    const CopySeg sg = a.seg[r % a.nseg];
    const size_t bx = (size_t)(r / a.nseg) * a.run + blockIdx.x % a.run, nbx = gridDim.x / a.nseg;
    const size_t tid = bx * kBlock + threadIdx.x;
    const size_t nthr = nbx * kBlock;
    const uintptr_t d = reinterpret_cast<uintptr_t>(sg.dst);
    const uintptr_t s = reinterpret_cast<uintptr_t>(sg.src);
    size_t head = (16 - (d & 15)) & 15;
    if (head > sg.bytes) head = sg.bytes;
    if (((s + head) & 15) != 0) {   // source and target disagree mod 16: bytes
        for (size_t i = tid; i < sg.bytes; i += nthr) sg.dst[i] = sg.src[i];
        return;
    }
    const size_t nvec = (sg.bytes - head) / 16;
    const size_t tail0 = head + nvec * 16;
    if (tid < head) sg.dst[tid] = sg.src[tid];
    if (tid < sg.bytes - tail0) sg.dst[tail0 + tid] = sg.src[tail0 + tid];
    const u32x4 *in = reinterpret_cast<const u32x4 *>(sg.src + head);
    u32x4 *out = reinterpret_cast<u32x4 *>(sg.dst + head);
    const size_t step = nthr * kGatherUnroll;
    size_t v = bx * kBlock * kGatherUnroll + threadIdx.x;
    for (; v + (size_t)(kGatherUnroll - 1) * kBlock < nvec; v += step) {
        u32x4 x[kGatherUnroll];
#pragma unroll
        for (int u = 0; u < kGatherUnroll; ++u) x[u] = __builtin_nontemporal_load(in + v + u * kBlock);
#pragma unroll
        for (int u = 0; u < kGatherUnroll; ++u) __builtin_nontemporal_store(x[u], out + v + u * kBlock);
    }
    for (int u = 0; u < kGatherUnroll; ++u) {
        const size_t w = v + (size_t)u * kBlock;
        if (w < nvec) __builtin_nontemporal_store(__builtin_nontemporal_load(in + w), out + w);
    }
}

}  // namespace

hipError_t launch_gather(const void *const *srcs, void *const *dsts, const size_t *bytes, int nseg,
                         hipStream_t stream) {
    if (nseg < 0 || nseg > kMaxFoldInputs) return hipErrorInvalidValue;
    GatherArgs a{};
    size_t most = 0;
    int k = 0;
    for (int i = 0; i < nseg; ++i) {
        if (!bytes[i]) continue;
        if (!srcs[i] || !dsts[i]) return hipErrorInvalidValue;
        a.seg[k++] = CopySeg{static_cast<const unsigned char *>(srcs[i]),
                             static_cast<unsigned char *>(dsts[i]), bytes[i]};
        most = bytes[i] > most ? bytes[i] : most;
    }
    if (!k) return hipSuccess;
    // blocks per segment: one chunk of kBlock x kGatherUnroll vectors each
    // (a grid-stride loop beyond 65536), rounded up to whole runs
    size_t bx = (most / 16 + (size_t)kBlock * kGatherUnroll - 1) / ((size_t)kBlock * kGatherUnroll);
    if (bx < 1) bx = 1;
    if (bx > 65536) bx = 65536;
    const size_t run = bx < kGatherRun ? bx : kGatherRun;
    bx = (bx + run - 1) / run * run;
    a.nseg = k;
    a.run = (unsigned)run;
    launch_k(kKindGather, gather_kernel, dim3((unsigned)(bx * k)), dim3(kBlock), stream, a);
    return hipGetLastError();
}

}  // namespace shmx
