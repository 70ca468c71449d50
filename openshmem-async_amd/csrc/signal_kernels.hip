// gfx950 kernels of the device-side synchronisation of the IPC algorithms
// (DIRECT, SIGNAL): the system-scope fence on every XCD with
// its XCD records, the SIGNAL barrier wave, and the fused one-shot and
// two-shot launches (fence, grid barriers, peer handshakes, fold and gather
// in one kernel).  The element ops are fold_ops.h's, shared with the fold.
#include "fold_ops.h"

namespace shmx {

namespace {

// The per-XCD L2s are not coherent with each other or with the peers, so a
// system-scope fence must run on EVERY XCD.  Dispatch spreads workgroups
// round-robin over the XCDs in practice, so 64 one-wave blocks put 8 on each
// — but the block -> XCD map is not architecturally defined, so each block
// also records the XCD it ran on (HW_REG_XCC_ID) in seen[blockIdx.x]: the host
// (fence_and_wait) or the next signal_kernel checks that every XCD of the
// device reported, and refills or fails loudly if one did not.
// s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): id 20, offset 0, size 4
constexpr int kXccIdReg = 20 | (0 << 6) | ((4 - 1) << 11);

__global__ __launch_bounds__(64) void sys_fence_kernel(unsigned int *seen) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");   // system scope
        const unsigned int xcc = (unsigned int)__builtin_amdgcn_s_getreg(kXccIdReg) & 15u;
        __hip_atomic_store(seen + blockIdx.x, kFenceSeen | xcc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ void check_fence(const SignalArgs &a) {
    // lane b reads block b's record of the fence just before this kernel
    const int lane = threadIdx.x;
    unsigned int rec = 0;
    if (a.seen && lane < kFenceBlocks) {
        rec = __hip_atomic_load(a.seen + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.seen + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (!a.seen) return;
    int covered = 0;
#pragma unroll
    for (unsigned int x = 0; x < 16; ++x)
        covered += __ballot(rec == (kFenceSeen | x)) != 0 ? 1 : 0;
    if (lane == 0) {
        atomicAdd(a.fence_stats, 1ull);
        if (covered < a.nxcc) {
            atomicAdd(a.fence_stats + 1, 1ull);
            __hip_atomic_store(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ __launch_bounds__(64) void signal_kernel(SignalArgs a) {
    check_fence(a);
    const int i = threadIdx.x;
    if (i >= a.P || a.pe[i] == a.me) return;
    unsigned long long *mine = a.mine + a.pe[i];
    const unsigned long long want =
        __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
    __hip_atomic_store(mine, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long *theirs = a.peer[i] + a.me;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
            __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// ------------------------------------------------ fused one-shot (SIGNAL)
// Thread 0 of the last block to arrive: bump my counter for every peer
// (system-scope release: everything this GPU's blocks fenced before arriving
// is in memory first), then wait for every peer's counter for me.
__device__ void peer_handshake(const SignalArgs &a) {
    unsigned long long want[kMaxFoldInputs];
    for (int i = 0; i < a.P; ++i) {
        if (a.pe[i] == a.me) continue;
        unsigned long long *c = a.mine + a.pe[i];
        want[i] = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
        __hip_atomic_store(c, want[i], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < a.P; ++i) {
        if (a.pe[i] == a.me) continue;
        const unsigned long long *theirs = a.peer[i] + a.me;
        while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want[i]) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope
}

// One element of the one-shot fold: the peers' values are remote loads
// (µs each over xGMI), so all nins of them are issued before the first op
// instead of one load's latency per input; heavy ops keep the loop.
template <typename T, int OP>
__device__ __forceinline__ T fold_elem(const SignalFoldArgs &a, size_t i) {
    if constexpr (kHeavyOp<T, OP>) {
        T acc = static_cast<const T *>(a.ins[0])[i];
        for (int k = 1; k < a.nins; ++k) acc = Op<T, OP>::ap(acc, static_cast<const T *>(a.ins[k])[i]);
        return acc;
    } else {
        T x[kMaxFoldInputs];
#pragma unroll
        for (int k = 0; k < kMaxFoldInputs; ++k)
            if (k < a.nins) x[k] = static_cast<const T *>(a.ins[k])[i];
        T acc = x[0];
#pragma unroll
        for (int k = 1; k < kMaxFoldInputs; ++k)
            if (k < a.nins) acc = Op<T, OP>::ap(acc, x[k]);
        return acc;
    }
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void signal_fold_kernel(SignalFoldArgs a) {
    unsigned int *const count = a.gsync, *const gen = a.gsync + 1;
    // up to 4 elements per lane of one block: the last block to arrive folds
    // alone, and no block waits for a release or arrives at the exit
    const bool tiny = a.n <= kFusedTinyElems;
    static_assert(kFusedTinyElems == (size_t)4 * kBlock, "the tiny case is 4 elements per lane of one block");
    __shared__ int s_last;
    __shared__ unsigned int s_gen0;
    if (threadIdx.x == 0) {
        // entry: record this block's XCD, then write back the XCD's L2 and
        // drop stale peer lines (the fence also orders the record), arrive
        const unsigned int xcc = (unsigned int)__builtin_amdgcn_s_getreg(kXccIdReg) & 15u;
        __hip_atomic_store(a.sig.seen + blockIdx.x, kFenceSeen | xcc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");   // system scope
        const unsigned int gen0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == gridDim.x - 1;
        if (!s_last && !tiny) {
            // relaxed polls (an acquire load would invalidate the L2 on every
            // poll), one acquire once the generation moved
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.sig.timeout_ticks) {
                    // only if launches overlapped on this GPU (they must not)
                    __hip_atomic_store(a.sig.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        } else if (s_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        s_gen0 = gen0;   // for the checking wave
    }
    __syncthreads();
    // a tiny array is folded by the last block alone: the others have fenced
    // and arrived, and leave
    if (tiny && !s_last) return;
    if (s_last && threadIdx.x < 64) {
        // the last block's first wave: every block's XCD record at once (lane
        // b reads block b's), then lane 0 does the entry handshake
        const int lane = threadIdx.x;
        unsigned int rec = 0;
        if (lane < (int)gridDim.x) {
            rec = __hip_atomic_load(a.sig.seen + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sig.seen + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int covered = 0;
#pragma unroll
        for (unsigned int x = 0; x < 16; ++x) covered += __ballot(rec == (kFenceSeen | x)) != 0 ? 1 : 0;
        if (lane == 0) {
            atomicAdd(a.sig.fence_stats, 1ull);
            if (covered < a.sig.nxcc) {
                atomicAdd(a.sig.fence_stats + 1, 1ull);
                __hip_atomic_store(a.sig.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            peer_handshake(a.sig);   // reduce-op.c:217
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, s_gen0 + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    T *out = static_cast<T *>(a.out);
    if (tiny) {
        for (size_t i = threadIdx.x; i < a.n; i += kBlock) out[i] = fold_elem<T, OP>(a, i);
        if (a.host_word) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's stores landed
        __syncthreads();
        if (threadIdx.x == 0) {
            peer_handshake(a.sig);   // reduce-op.c:250
            // this workgroup did all the work: tell the host (system-scope
            // release: the L2 is written back first)
            if (a.host_word)
                __hip_atomic_store(a.host_word, a.host_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x, nthr = (size_t)gridDim.x * kBlock;
    for (size_t i = tid; i < a.n; i += nthr) out[i] = fold_elem<T, OP>(a, i);
    __syncthreads();
    // exit: the last block to finish reading tells the peers (reduce-op.c:250)
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        peer_handshake(a.sig);
    }
}

// ------------------------------------------------ fused two-shot (SIGNAL)
// The peers' operands are read over xGMI, where a load's latency (µs) rather
// than HBM bounds a 64-block grid: every lane issues its U 16-B loads from
// each of the nins inputs (uniform predicates, unrolled) before folding any,
// so a block keeps U x nins x 4 KiB in flight per step; U = 16 / MAXIN (4
// vectors per input up to 4 inputs, 2 up to 8, 1 up to 16: 16 vectors in
// registers either way).
template <typename T, int OP, int MAXIN>
__device__ __forceinline__ void fold_vecs(const SignalFoldArgs &a, u32x4 *out, size_t nvec, size_t tid,
                                          size_t nthr) {
    constexpr int U = kMaxFoldInputs / MAXIN;
    const size_t step = nthr * U;
    auto in = [&](int k) {
        return reinterpret_cast<const u32x4 *>(static_cast<const T *>(a.ins[k]) + a.lo);
    };
    size_t v = (tid / kBlock) * kBlock * U + tid % kBlock;   // U vectors of a block are kBlock apart
    for (; v + (size_t)(U - 1) * kBlock < nvec; v += step) {
        u32x4 x[MAXIN][U];
#pragma unroll
        for (int k = 0; k < MAXIN; ++k)
            if (k < a.nins)
#pragma unroll
                for (int u = 0; u < U; ++u) x[k][u] = __builtin_nontemporal_load(in(k) + v + u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 acc = x[0][u];
#pragma unroll
            for (int k = 1; k < MAXIN; ++k)
                if (k < a.nins) acc = apply16<T, OP>(acc, x[k][u]);
            out[v + u * kBlock] = acc;
        }
    }
    for (int u = 0; u < U; ++u) {   // the last partial step
        const size_t w = v + (size_t)u * kBlock;
        if (w >= nvec) break;
        u32x4 acc = __builtin_nontemporal_load(in(0) + w);
        for (int k = 1; k < a.nins; ++k) acc = apply16<T, OP>(acc, __builtin_nontemporal_load(in(k) + w));
        out[w] = acc;
    }
}

template <typename T, int OP>
__device__ __forceinline__ void fold_span(const SignalFoldArgs &a, size_t tid, size_t nthr) {
    constexpr int E = 16 / sizeof(T);
    const size_t lo = a.lo, n = a.hi - a.lo;
    T *const out = static_cast<T *>(a.out) + lo;
    bool vec = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    for (int k = 0; k < a.nins; ++k)
        vec &= (reinterpret_cast<uintptr_t>(static_cast<const T *>(a.ins[k]) + lo) & 15) == 0;
    const size_t nvec = vec ? n / E : 0;
    u32x4 *const vout = reinterpret_cast<u32x4 *>(out);
    // soft x87 and the complex products (Annex G recovery branch) unrolled
    // 16 vectors deep would spill: one vector of one input at a time
    if constexpr (kHeavyOp<T, OP>) {
        for (size_t v = tid; v < nvec; v += nthr) {
            u32x4 acc = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
                                                       static_cast<const T *>(a.ins[0]) + lo) + v);
            for (int k = 1; k < a.nins; ++k)
                acc = apply16<T, OP>(acc, __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
                                                  static_cast<const T *>(a.ins[k]) + lo) + v));
            vout[v] = acc;
        }
    } else if (a.nins <= 4) {
        fold_vecs<T, OP, 4>(a, vout, nvec, tid, nthr);
    } else if (a.nins <= 8) {
        fold_vecs<T, OP, 8>(a, vout, nvec, tid, nthr);
    } else {
        fold_vecs<T, OP, 16>(a, vout, nvec, tid, nthr);
    }
    for (size_t i = nvec * E + tid; i < n; i += nthr) {
        T acc = static_cast<const T *>(a.ins[0])[lo + i];
        for (int k = 1; k < a.nins; ++k) acc = Op<T, OP>::ap(acc, static_cast<const T *>(a.ins[k])[lo + i]);
        out[i] = acc;
    }
}

// The all-gather of the two-shot: every segment's loads of a step issued
// before any store, so all peers' links are busy at once (U vectors per
// segment per lane, as fold_vecs).
template <int MAXSEG>
__device__ __forceinline__ void gather_vecs(const SignalFoldArgs &a, size_t nvec, size_t tid, size_t nthr) {
    constexpr int U = kMaxFoldInputs / MAXSEG;
    for (size_t v = (tid / kBlock) * kBlock * U + tid % kBlock; v < nvec; v += nthr * U) {
        u32x4 x[MAXSEG][U];
#pragma unroll
        for (int k = 0; k < MAXSEG; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k < a.nseg && v + u * kBlock < a.glen[k] / 16)
                    x[k][u] = __builtin_nontemporal_load(static_cast<const u32x4 *>(a.gsrc[k]) + v + u * kBlock);
#pragma unroll
        for (int k = 0; k < MAXSEG; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k < a.nseg && v + u * kBlock < a.glen[k] / 16)
                    static_cast<u32x4 *>(a.gdst[k])[v + u * kBlock] = x[k][u];
    }
}

__device__ __forceinline__ void gather_span(const SignalFoldArgs &a, size_t tid, size_t nthr) {
    bool vec = true;
    size_t most = 0;
    for (int k = 0; k < a.nseg; ++k) {
        vec &= ((reinterpret_cast<uintptr_t>(a.gsrc[k]) | reinterpret_cast<uintptr_t>(a.gdst[k])) & 15) == 0;
        most = a.glen[k] > most ? a.glen[k] : most;
    }
    if (!vec) {
        for (int k = 0; k < a.nseg; ++k)
            for (size_t i = tid; i < a.glen[k]; i += nthr)
                static_cast<unsigned char *>(a.gdst[k])[i] = static_cast<const unsigned char *>(a.gsrc[k])[i];
        return;
    }
    if (a.nseg <= 4) gather_vecs<4>(a, most / 16, tid, nthr);
    else if (a.nseg <= 8) gather_vecs<8>(a, most / 16, tid, nthr);
    else gather_vecs<16>(a, most / 16, tid, nthr);
    for (int k = 0; k < a.nseg; ++k)
        for (size_t i = a.glen[k] / 16 * 16 + tid; i < a.glen[k]; i += nthr)
            static_cast<unsigned char *>(a.gdst[k])[i] = static_cast<const unsigned char *>(a.gsrc[k])[i];
}

// Grid barrier + peer handshake inside the kernel: every block writes back
// its XCD's L2 (its own stores become visible over xGMI) and arrives; the
// last one does the handshake and releases the generation gen_now + 1; every
// block then drops stale lines of the peers' memory (system acquire) before
// it reads what the peers wrote.
__device__ void grid_handshake(const SignalFoldArgs &a, unsigned int gen_now) {
    unsigned int *const count = a.gsync, *const gen = a.gsync + 1;
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope
        if (__hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            peer_handshake(a.sig);
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, gen_now + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen_now) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.sig.timeout_ticks) {
                    __hip_atomic_store(a.sig.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope
    }
    __syncthreads();
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void signal_fold2_kernel(SignalFoldArgs a) {
    unsigned int *const count = a.gsync, *const gen = a.gsync + 1;
    __shared__ int s_last;
    __shared__ unsigned int s_gen0;
    if (threadIdx.x == 0) {
        // entry, as the one shot: record the XCD, fence, arrive
        const unsigned int xcc = (unsigned int)__builtin_amdgcn_s_getreg(kXccIdReg) & 15u;
        __hip_atomic_store(a.sig.seen + blockIdx.x, kFenceSeen | xcc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");   // system scope
        const unsigned int gen0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == gridDim.x - 1;
        if (!s_last) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.sig.timeout_ticks) {
                    __hip_atomic_store(a.sig.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_gen0 = gen0;
    }
    __syncthreads();
    if (s_last && threadIdx.x < 64) {
        const int lane = threadIdx.x;
        unsigned int rec = 0;
        if (lane < (int)gridDim.x) {
            rec = __hip_atomic_load(a.sig.seen + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sig.seen + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int covered = 0;
#pragma unroll
        for (unsigned int x = 0; x < 16; ++x) covered += __ballot(rec == (kFenceSeen | x)) != 0 ? 1 : 0;
        if (lane == 0) {
            atomicAdd(a.sig.fence_stats, 1ull);
            if (covered < a.sig.nxcc) {
                atomicAdd(a.sig.fence_stats + 1, 1ull);
                __hip_atomic_store(a.sig.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            peer_handshake(a.sig);   // reduce-op.c:217: every source is final
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, s_gen0 + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x, nthr = (size_t)gridDim.x * kBlock;
    fold_span<T, OP>(a, tid, nthr);     // my slice from every member's source
    grid_handshake(a, s_gen0 + 1u);     // every member's slice is final
    gather_span(a, tid, nthr);          // the other slices from the peers' targets
    __syncthreads();
    // exit: the last block to finish reading tells the peers (reduce-op.c:250)
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        peer_handshake(a.sig);
    }
}

// Blocks of the fused launches: kFenceBlocks, so every XCD gets 8 (the entry
// check counts them); 8-32 blocks measured within 1 us of it
// (profiles/r05_fused_blocks.txt).
constexpr unsigned kFusedBlocks = kFenceBlocks;

template <typename T, int OP>
hipError_t sf_launch(const SignalFoldArgs &a, hipStream_t s) {
    if (a.two_shot)
        hipLaunchKernelGGL((signal_fold2_kernel<T, OP>), dim3(kFusedBlocks), dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL((signal_fold_kernel<T, OP>), dim3(kFusedBlocks), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename T>
hipError_t sf_ops(int op, const SignalFoldArgs &a, hipStream_t s) {
    constexpr bool integral = std::is_integral<T>::value;
    constexpr bool cplx = std::is_same<T, cplxd>::value || std::is_same<T, cplxf>::value;
    switch (op) {
    case SHMEMX_OP_SUM: return sf_launch<T, SHMEMX_OP_SUM>(a, s);
    case SHMEMX_OP_PROD: return sf_launch<T, SHMEMX_OP_PROD>(a, s);
    case SHMEMX_OP_AND:
        if constexpr (integral) return sf_launch<T, SHMEMX_OP_AND>(a, s);
        break;
    case SHMEMX_OP_OR:
        if constexpr (integral) return sf_launch<T, SHMEMX_OP_OR>(a, s);
        break;
    case SHMEMX_OP_XOR:
        if constexpr (integral) return sf_launch<T, SHMEMX_OP_XOR>(a, s);
        break;
    case SHMEMX_OP_MIN:
        if constexpr (!cplx) return sf_launch<T, SHMEMX_OP_MIN>(a, s);
        break;
    case SHMEMX_OP_MAX:
        if constexpr (!cplx) return sf_launch<T, SHMEMX_OP_MAX>(a, s);
        break;
    default: break;
    }
    return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_signal_fold(int type, int op, const SignalFoldArgs &a, hipStream_t stream) {
    if (!op_on_device(type, op) || a.nins < 1 || a.nins > kMaxFoldInputs || !a.out || !a.gsync ||
        !a.sig.seen || !a.sig.fence_stats || a.sig.P < 1 || a.sig.P > kMaxFoldInputs || !a.sig.mine ||
        !a.sig.err)
        return hipErrorInvalidValue;
    for (int k = 0; k < a.nins; ++k)
        if (!a.ins[k]) return hipErrorInvalidValue;
    for (int i = 0; i < a.sig.P; ++i)
        if (a.sig.pe[i] != a.sig.me && !a.sig.peer[i]) return hipErrorInvalidValue;
    if (a.two_shot) {
        if (a.lo > a.hi || a.hi > a.n || a.nseg < 0 || a.nseg > kMaxFoldInputs) return hipErrorInvalidValue;
        for (int k = 0; k < a.nseg; ++k)
            if (a.glen[k] && (!a.gsrc[k] || !a.gdst[k])) return hipErrorInvalidValue;
    }
    switch (type) {
    case SHMEMX_TYPE_SHORT: return sf_ops<short>(op, a, stream);
    case SHMEMX_TYPE_INT: return sf_ops<int>(op, a, stream);
    case SHMEMX_TYPE_LONG:
    case SHMEMX_TYPE_LONGLONG: return sf_ops<long>(op, a, stream);
    case SHMEMX_TYPE_FLOAT: return sf_ops<float>(op, a, stream);
    case SHMEMX_TYPE_DOUBLE: return sf_ops<double>(op, a, stream);
    case SHMEMX_TYPE_LONGDOUBLE: return sf_ops<ld80>(op, a, stream);
    case SHMEMX_TYPE_COMPLEXD: return sf_ops<cplxd>(op, a, stream);
    case SHMEMX_TYPE_COMPLEXF: return sf_ops<cplxf>(op, a, stream);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_signal(const SignalArgs &a, hipStream_t stream) {
    if (a.P < 1 || a.P > kMaxFoldInputs || !a.mine || !a.err) return hipErrorInvalidValue;
    for (int i = 0; i < a.P; ++i)
        if (a.pe[i] != a.me && !a.peer[i]) return hipErrorInvalidValue;
    hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_sys_fence(hipStream_t stream, unsigned int *seen) {
    if (!seen) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sys_fence_kernel, dim3(kFenceBlocks), dim3(64), 0, stream, seen);
    return hipGetLastError();
}

}  // namespace shmx
