// The resident service workgroup: small blocking calls without a kernel
// launch (VERDICT r05 "Next" #3).
//
// A one-member call (reduce-op.c:213-216: write_to = source, and nothing
// else) of at most kServiceMaxBytes is latency, not bandwidth: launching a
// one-workgroup copy and spinning on the word it stores costs 6.7 us on
// MI355X, almost all of it the launch (tools/service_lab.hip,
// profiles/r06_service_lab.txt), against 3.0-8.8 us for the reference's CPU
// algorithm.  Here one workgroup stays resident on its own
// non-blocking stream and polls a mailbox in page-locked, host-coherent
// memory: the host writes the call's descriptor and a sequence number into
// one 64-byte line, a polling wave reads that whole line with one scalar load
// (no second round trip over PCIe for the descriptor; a check word catches a
// torn read), drops stale lines (system-scope acquire) and hands the request
// to the copy waves, which copy, write back (system-scope release) and store
// the sequence number into a second host-coherent line the host spins on:
// 2.5-2.7 us per round trip for 16 bytes, 3.2 at 32 KiB (service_kernel).
//
// Ordering.  A blocking call is ordered after the legacy default stream and
// the library's stream (the buffers a plain HIP program, or PyTorch's
// default stream, just wrote).  When the runtime reports both idle
// (hipStreamQuery, 0.17 us for the two) the request is posted at once;
// otherwise the host first waits for them (hipStreamSynchronize: the same
// work the launched copy would wait for in stream order on the GPU), then
// posts.  Launching the copy on the (blocking) library stream instead would
// keep hipStreamQuery of that stream and of the null stream answering "not
// ready" for 12 and 31 us after the kernel is done (tools/queue_lab.hip
// "lag", profiles/r06_queue_lab.txt), so every next back-to-back call would
// take the launch path too, at 24 us from Python instead of 5.5.  The
// library stream is asked only when it may hold work nobody waited for
// (state.h lib_stream_dirty).
//
// Lifetime.  The workgroup leaves by itself after kIdleUs without a request
// (every wave reaches that exit: poller 0 decides, the LDS claim and request
// words release the others), at once when the host stores the quit word
// (service_quiesce: shmem_finalize, an atexit handler, and before the
// library's own device-wide synchronisations), and is launched again by the
// next call that finds its stream idle.  A request posted while it was
// leaving is noticed by the host (the stream has gone idle, the sequence
// number not served) and served by a fresh launch, which starts from the
// last sequence number completed.  A program's own hipDeviceSynchronize
// waits for it at most kIdleUs.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>

#include "fold_ops.h"
#include "internal.h"
#include "node.h"
#include "shmem_reduce_mi355x.h"
#include "state.h"

namespace shmx {

namespace {

constexpr unsigned long long kMix = 0x9E3779B97F4A7C15ull;
constexpr unsigned kIdleUs = 200;
// Waves 0-3 poll the mailbox, waves 4-15 copy.
constexpr int kSvcBlock = 1024;
constexpr int kPollWaves = 4;
constexpr int kCopyThreads = kSvcBlock - 64 * kPollWaves;
// Poller w reads the mailbox in the time slots w, w + 4, w + 8, ... of
// kSlot s_memrealtime ticks (10 ns each): a read of host memory takes ~1.2 us,
// so the four together read it every 0.33 us and stay that far apart.
constexpr unsigned long long kSlot = 33;
constexpr unsigned long long kExit = ~0ull;

// Written by the host: the first line (seq last, with release); by the
// device: the second.
struct alignas(64) Mailbox {
    unsigned long long seq;
    unsigned long long quit;
    const void *src;
    void *dst;
    void *dst2;   // a second destination (the mirrored heap's view), or null
    unsigned long long bytes;
    unsigned long long check;   // seq ^ src ^ dst ^ dst2 ^ bytes ^ cfg ^ kMix
    unsigned long long cfg;     // 0: a copy; else a fold of the exchange slots (fold_cfg)
    alignas(64) unsigned long long done;
};
static_assert(sizeof(Mailbox) == 128, "two lines");

// Global-memory views of the operands (their addresses arrive through LDS,
// which would leave generic flat accesses otherwise).
template <typename V>
using gptr = __attribute__((address_space(1))) V *;

// Copy thread t moves words t, t + 768, ... of the widest word the operands'
// alignment allows.  (A version that issued all of a lane's loads before its
// first store, unconditional and clamped, was slower: 2.72 against 2.35 us
// per 16-byte request, 3.70 against 3.56 at 32 KiB; tools/kernel_variants.hip.)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <typename V>
__device__ __forceinline__ void copy_as(int t, const unsigned char *src, unsigned char *dst, unsigned char *dst2,
                                        unsigned long long bytes) {
    const gptr<const V> s = (gptr<const V>)(src);
    const gptr<V> d = (gptr<V>)(dst);
    const gptr<V> d2 = (gptr<V>)(dst2);
    const unsigned long long n = bytes / sizeof(V);
    for (unsigned long long i = t; i < n; i += kCopyThreads) {
        const V x = s[i];
        d[i] = x;
        if (dst2) d2[i] = x;
    }
}

// A fold request: bit 0 set; type, op, the calling PE's own order or
// PE_start's, and the set (PE_start, logPE_stride, PE_size) with the caller.
struct FoldCfg {
    int type, op, own, start, logstride, size, me;
};
__host__ __device__ inline unsigned long long pack_cfg(const FoldCfg &f) {
    return 1ull | (unsigned long long)f.type << 1 | (unsigned long long)f.op << 5 |
           (unsigned long long)f.own << 8 | (unsigned long long)f.start << 9 |
           (unsigned long long)f.logstride << 16 | (unsigned long long)f.size << 24 |
           (unsigned long long)f.me << 32;
}
__device__ inline FoldCfg unpack_cfg(unsigned long long c) {
    return FoldCfg{(int)(c >> 1 & 15), (int)(c >> 5 & 7), (int)(c >> 8 & 1), (int)(c >> 9 & 127),
                   (int)(c >> 16 & 7), (int)(c >> 24 & 127), (int)(c >> 32 & 127)};
}

// The j-th input of PE me's fold: its own source first, then the other
// members in ascending order (reduce-op.c:219-248), or PE_start's order
// (every member the same bits: the DIRECT / A2A convention).
__device__ __forceinline__ int member_at(const FoldCfg &f, int j) {
    if (!f.own) return f.start + (j << f.logstride);
    const int r = (f.me - f.start) >> f.logstride;
    if (j == 0) return f.me;
    return f.start + ((j - 1 < r ? j - 1 : j) << f.logstride);
}

// The fold, for copy thread t: 16-byte word w of every member's slot (the
// slots are 4 KiB-aligned, in host memory), up to 8 members' words loaded
// before the first op, so a 4 KiB slot is one round trip over PCIe (768
// threads, 256 words); the word's elements folded in the member order, then
// stored element by element (the target's alignment is the caller's).
template <typename T, int OP>
__device__ void fold_slots(int t, const unsigned char *slots, unsigned char *dst, unsigned char *dst2,
                           unsigned long long bytes, const FoldCfg &f) {
    constexpr int E = 16 / sizeof(T);
    static_assert(E >= 1 && E * sizeof(T) == 16, "whole elements per 16-byte word");
    const unsigned long long n = bytes / sizeof(T), nw = (n + E - 1) / E;
    for (unsigned long long w = t; w < nw; w += kCopyThreads) {
        T acc[E];
        for (int j0 = 0; j0 < f.size; j0 += 8) {
            v4u v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (j0 + u < f.size)
                    v[u] = reinterpret_cast<const v4u *>(slots + (size_t)member_at(f, j0 + u) * node::kXchgSlotBytes)[w];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (j0 + u >= f.size) break;
                T x[E];
                __builtin_memcpy(x, &v[u], 16);
#pragma unroll
                for (int e = 0; e < E; ++e) acc[e] = j0 + u == 0 ? x[e] : Op<T, OP>::ap(acc[e], x[e]);
            }
        }
        const unsigned long long e0 = w * E;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (e0 + e < n) {
                reinterpret_cast<T *>(dst)[e0 + e] = acc[e];
                if (dst2) reinterpret_cast<T *>(dst2)[e0 + e] = acc[e];
            }
        }
    }
}

template <typename T>
__device__ void fold_int(int t, const unsigned char *sl, unsigned char *d, unsigned char *d2, unsigned long long b,
                         const FoldCfg &f) {
    switch (f.op) {
    case SHMEMX_OP_SUM: fold_slots<T, SHMEMX_OP_SUM>(t, sl, d, d2, b, f); break;
    case SHMEMX_OP_PROD: fold_slots<T, SHMEMX_OP_PROD>(t, sl, d, d2, b, f); break;
    case SHMEMX_OP_AND: fold_slots<T, SHMEMX_OP_AND>(t, sl, d, d2, b, f); break;
    case SHMEMX_OP_OR: fold_slots<T, SHMEMX_OP_OR>(t, sl, d, d2, b, f); break;
    case SHMEMX_OP_XOR: fold_slots<T, SHMEMX_OP_XOR>(t, sl, d, d2, b, f); break;
    case SHMEMX_OP_MIN: fold_slots<T, SHMEMX_OP_MIN>(t, sl, d, d2, b, f); break;
    default: fold_slots<T, SHMEMX_OP_MAX>(t, sl, d, d2, b, f); break;
    }
}
template <typename T>
__device__ void fold_fp(int t, const unsigned char *sl, unsigned char *d, unsigned char *d2, unsigned long long b,
                        const FoldCfg &f) {
    switch (f.op) {
    case SHMEMX_OP_SUM: fold_slots<T, SHMEMX_OP_SUM>(t, sl, d, d2, b, f); break;
    case SHMEMX_OP_PROD: fold_slots<T, SHMEMX_OP_PROD>(t, sl, d, d2, b, f); break;
    case SHMEMX_OP_MIN: fold_slots<T, SHMEMX_OP_MIN>(t, sl, d, d2, b, f); break;
    default: fold_slots<T, SHMEMX_OP_MAX>(t, sl, d, d2, b, f); break;
    }
}
template <typename T>
__device__ void fold_cplx(int t, const unsigned char *sl, unsigned char *d, unsigned char *d2,
                          unsigned long long b, const FoldCfg &f) {
    if (f.op == SHMEMX_OP_SUM) fold_slots<T, SHMEMX_OP_SUM>(t, sl, d, d2, b, f);
    else fold_slots<T, SHMEMX_OP_PROD>(t, sl, d, d2, b, f);
}
__device__ void fold_request(int t, const unsigned char *sl, unsigned char *d, unsigned char *d2,
                             unsigned long long b, unsigned long long cfg) {
    const FoldCfg f = unpack_cfg(cfg);
    switch (f.type) {
    case SHMEMX_TYPE_SHORT: fold_int<short>(t, sl, d, d2, b, f); break;
    case SHMEMX_TYPE_INT: fold_int<int>(t, sl, d, d2, b, f); break;
    case SHMEMX_TYPE_LONG:
    case SHMEMX_TYPE_LONGLONG: fold_int<long>(t, sl, d, d2, b, f); break;
    case SHMEMX_TYPE_FLOAT: fold_fp<float>(t, sl, d, d2, b, f); break;
    case SHMEMX_TYPE_DOUBLE: fold_fp<double>(t, sl, d, d2, b, f); break;
    case SHMEMX_TYPE_LONGDOUBLE: fold_fp<ld80>(t, sl, d, d2, b, f); break;
    case SHMEMX_TYPE_COMPLEXD: fold_cplx<cplxd>(t, sl, d, d2, b, f); break;
    default: fold_cplx<cplxf>(t, sl, d, d2, b, f); break;
    }
}

__device__ __forceinline__ unsigned long long lds_load(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool lds_cas(unsigned long long *p, unsigned long long expect, unsigned long long v) {
    return __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_WORKGROUP);
}

typedef unsigned int line_t __attribute__((ext_vector_type(16)));
__device__ __forceinline__ unsigned long long word(const line_t &v, int k) {
    return (unsigned long long)v[2 * k + 1] << 32 | v[2 * k];
}

// The mailbox is read with a scalar load (the whole 64-byte line, past the
// scalar cache: glc), not a vector one.  A vector read of host memory in
// flight holds up every later vector access of the CU (its vector memory path
// returns in order: six reads in flight made a 16-byte request take 7.3 us),
// so with vector reads one poller could have only one in flight and a
// request waited up to a whole read for the next one (2.3-3.4 us by the
// phase of the post, sawtooth).  Scalar reads do not stand in the copy's way:
// four polling waves, a read each, a quarter of a read apart, take 2.5-2.7 us
// whatever the phase (tools/kernel_variants.hip, profiles/r06_service_phase.txt).
// A poller that sees a new request claims it in LDS (compare-and-swap: the
// others see the same request), drops stale lines (system-scope acquire: it
// has no vector access in flight, so the wait is free) and hands it to the
// copy waves; the last copy wave to finish writes back (system-scope release)
// and stores the sequence number into the host's done line.  Leaving: poller
// 0 swaps the claim word to kExit once no copy is pending (a claim and the
// exit cannot both win), every poller then leaves, and the copy waves on
// s_req = kExit.  A request that lost to the exit is served by the host's
// relaunch (service_copy).
__global__ __launch_bounds__(kSvcBlock) void service_kernel(Mailbox *mb, unsigned long long served,
                                                         unsigned long long idle_ticks) {
    __shared__ unsigned long long s_claim, s_req, s_done, s_count, s_bytes, s_cfg;
    __shared__ const unsigned char *s_src;
    __shared__ unsigned char *s_dst, *s_dst2;
    if (threadIdx.x == 0) {
        s_claim = s_req = s_done = served;
        s_count = 0;
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    if (wave < kPollWaves) {
        unsigned long long last = served;
        unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            while (((__builtin_amdgcn_s_memrealtime() / kSlot) & (kPollWaves - 1)) != (unsigned)wave)
                __builtin_amdgcn_s_sleep(1);
            line_t v;
            asm volatile("s_load_dwordx16 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(mb) : "memory");
            const unsigned long long q = word(v, 0);
            const unsigned long long claim = lds_load(&s_claim);
            if (claim == kExit) break;
            if (q != last) {
                const unsigned long long a = word(v, 2), b = word(v, 3), b2 = word(v, 4), n = word(v, 5),
                                         c = word(v, 6), g = word(v, 7);
                if ((q ^ a ^ b ^ b2 ^ n ^ g ^ kMix) == c) {   // else a torn read: the next one
                    last = q;
                    t_last = __builtin_amdgcn_s_memrealtime();
                    if (claim != q && lds_cas(&s_claim, claim, q)) {
                        s_src = reinterpret_cast<const unsigned char *>(a);
                        s_dst = reinterpret_cast<unsigned char *>(b);
                        s_dst2 = reinterpret_cast<unsigned char *>(b2);
                        s_bytes = n;
                        s_cfg = g;
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // lines written since: dropped
                        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                        lds_store(&s_req, q);
                    }
                    continue;
                }
            }
            if (claim != last) {   // another poller's request
                last = claim;
                t_last = __builtin_amdgcn_s_memrealtime();
            }
            if (wave == 0 && (word(v, 1) || __builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) &&
                lds_load(&s_done) == claim && lds_cas(&s_claim, claim, kExit)) {
                lds_store(&s_req, kExit);
                break;
            }
        }
        return;
    }
    const int t = threadIdx.x - 64 * kPollWaves;
    unsigned long long seen = served;
    for (;;) {
        unsigned long long q;
        while ((q = lds_load(&s_req)) == seen) __builtin_amdgcn_s_sleep(1);
        if (q == kExit) return;
        seen = q;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned char *src = s_src;
        unsigned char *dst = s_dst, *dst2 = s_dst2;
        const unsigned long long n = s_bytes, cfg = s_cfg;
        const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) |
                             reinterpret_cast<uintptr_t>(dst2) | n;
        if (cfg) fold_request(t, src, dst, dst2, n, cfg);
        else if ((al & 15) == 0) copy_as<v4u>(t, src, dst, dst2, n);
        else if ((al & 7) == 0) copy_as<unsigned long long>(t, src, dst, dst2, n);
        else if ((al & 3) == 0) copy_as<unsigned>(t, src, dst, dst2, n);
        else if ((al & 1) == 0) copy_as<unsigned short>(t, src, dst, dst2, n);
        else copy_as<unsigned char>(t, src, dst, dst2, n);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores have landed
        if (threadIdx.x % 64 == 0 &&
            __hip_atomic_fetch_add(&s_count, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ==
                kCopyThreads / 64 - 1) {
            // the last copy wave: write back, then tell the host
            lds_store(&s_count, 0);
            __hip_atomic_store(&mb->done, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            lds_store(&s_done, q);
        }
    }
}

struct Service {
    Mailbox *mb = nullptr;
    hipStream_t stream = nullptr;
    int device = -1;
    unsigned long long seq = 0;
    bool launched = false;   // launched and not seen to have left
    std::chrono::steady_clock::time_point last_use{};
    bool exit_hook = false;
    // shmemx_service_stats: calls served, launches, calls that found the
    // legacy / the library stream busy (and waited for it first)
    unsigned long long served = 0, launches = 0, busy_null = 0, busy_lib = 0, folds = 0;
    // nanoseconds summed over the served calls: from entering service_copy
    // to the post, and from the post to seeing the result done
    unsigned long long ns_before_post = 0, ns_round_trip = 0;
} g_svc;

// $SHMEMX_SERVICE: 0 off, 1 on; unset: on unless another PE process of the
// job shares this GPU.  Several PE processes' resident workgroups on one GPU
// made every other kernel and copy of those processes several times slower
// (8 ranks on one MI355X: the host-resident call 91 -> 672 ms, the small-call
// timings minutes long; profiles/r06_bench_rehearsal_ipc_n8_b.json against
// SHMEMX_SERVICE=0), most likely because the GPU time-slices the processes'
// queues and a queue whose kernel never ends is switched out and back with
// its waves saved and restored.  One PE per GPU, the deployment this path is
// for, showed nothing of the kind.
bool enabled() {
    static const int env = [] {
        const char *e = std::getenv("SHMEMX_SERVICE");
        return e && *e == '0' ? 0 : e && *e == '1' ? 1 : -1;
    }();
    return env == 1 || (env < 0 && !g_state.gpu_shared);
}

void at_exit() { service_release(); }

bool ensure() {
    if (g_svc.mb && g_svc.device == g_state.device) return true;
    if (g_svc.mb) service_release();
    void *p = nullptr;
    if (hipHostMalloc(&p, sizeof(Mailbox), hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    std::memset(p, 0, sizeof(Mailbox));
    // a non-blocking stream of the greatest priority: a resident kernel on a
    // plain non-blocking stream holds up every later launch on the legacy
    // default stream until it leaves (HIP's null stream waits for it), one on
    // a high-priority stream does not (tools/queue_lab.hip,
    // profiles/r06_queue_lab.txt)
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) {
        (void)hipGetLastError();
        hi = 0;
    }
    if (hipStreamCreateWithPriority(&g_svc.stream, hipStreamNonBlocking, hi) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(p);
        return false;
    }
    g_svc.mb = static_cast<Mailbox *>(p);
    g_svc.device = g_state.device;
    g_svc.seq = 0;
    g_svc.launched = false;
    if (!g_svc.exit_hook) {   // after HIP's own initialisation: runs before its teardown
        std::atexit(at_exit);
        g_svc.exit_hook = true;
    }
    return true;
}

// (Re)launch, starting from the last request completed.
void launch() {
    const unsigned long long served = __atomic_load_n(&g_svc.mb->done, __ATOMIC_ACQUIRE);
    hipLaunchKernelGGL(service_kernel, dim3(1), dim3(kSvcBlock), 0, g_svc.stream, g_svc.mb, served,
                       (unsigned long long)kIdleUs * 100);   // s_memrealtime: 100 MHz
    SHMX_HIP(hipGetLastError());
    g_svc.launched = true;
    ++g_svc.launches;
}

bool stream_idle(hipStream_t s) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return true;
    if (e != hipErrorNotReady) SHMX_HIP(e);
    return false;
}

// Post one request and wait for it: a copy (cfg 0) or a fold (cfg = pack_cfg).
bool serve(void *dst, void *dst2, const void *src, size_t bytes, unsigned long long cfg) {
    // ordered after the legacy stream and the library stream: once both have
    // no work left (the resident workgroup's own stream, non-blocking, is
    // not part of the null stream's wait)
    if (!stream_idle(nullptr)) {
        ++g_svc.busy_null;
        SHMX_HIP(hipStreamSynchronize(nullptr));
    }
    if (g_state.lib_stream_dirty || g_state.lib_stream_exported) {
        if (!stream_idle(g_state.stream)) {
            ++g_svc.busy_lib;
            SHMX_HIP(hipStreamSynchronize(g_state.stream));
        }
        g_state.lib_stream_dirty = false;
    }
    if (!ensure()) return false;
    Mailbox *mb = g_svc.mb;
    const auto t_begin = std::chrono::steady_clock::now();
    // a workgroup that may have idled out: launch a fresh one first (one that
    // leaves between this check and the post is caught below)
    if (!g_svc.launched || t_begin - g_svc.last_use > std::chrono::microseconds(kIdleUs / 2)) {
        if (stream_idle(g_svc.stream)) launch();
    }
    const unsigned long long q = ++g_svc.seq;
    mb->src = src;
    mb->dst = dst;
    mb->dst2 = dst2;
    mb->bytes = bytes;
    mb->cfg = cfg;
    mb->check = q ^ reinterpret_cast<uintptr_t>(src) ^ reinterpret_cast<uintptr_t>(dst) ^
                reinterpret_cast<uintptr_t>(dst2) ^ (unsigned long long)bytes ^ cfg ^ kMix;
    __atomic_store_n(&mb->seq, q, __ATOMIC_RELEASE);
    const auto t_post = std::chrono::steady_clock::now();
    const volatile unsigned long long *done = &mb->done;
    for (unsigned k = 1; *done != q; ++k) {
        __builtin_ia32_pause();
        if ((k & 4095) == 0) {
            // left before it saw the request: serve it with a fresh launch
            if (stream_idle(g_svc.stream) && *done != q) launch();
            if (std::chrono::steady_clock::now() - t_begin > std::chrono::seconds(10))
                fatal("service workgroup", "a small call was not served within 10 s");
        }
    }
    g_svc.last_use = std::chrono::steady_clock::now();
    ++g_svc.served;
    if (cfg) ++g_svc.folds;
    g_svc.ns_before_post += (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(t_post - t_begin).count();
    g_svc.ns_round_trip +=
        (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(g_svc.last_use - t_post).count();
    return true;
}

}  // namespace

bool service_copy(void *dst, void *dst2, const void *src, size_t bytes) {
    if (!enabled() || bytes == 0 || bytes > kServiceMaxBytes || !dst || !src) return false;
    return serve(dst, dst2, src, bytes, 0);
}

bool service_available() { return enabled(); }

void service_fold(int type, int op, bool own_order, int start, int logstride, int size, void *dst, void *dst2,
                  size_t bytes) {
    const FoldCfg f{type, op, own_order ? 1 : 0, start, logstride, size, g_state.pe};
    if (!serve(dst, dst2, node::xchg_dev(0), bytes, pack_cfg(f)))
        fatal("service workgroup", "a small multi-PE call could not reach the service workgroup");
}

void service_quiesce() {
    if (!g_svc.mb || !g_svc.launched) return;
    __atomic_store_n(&g_svc.mb->quit, 1ull, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(g_svc.stream);
    __atomic_store_n(&g_svc.mb->quit, 0ull, __ATOMIC_RELEASE);
    g_svc.launched = false;
}

void service_release() {
    if (!g_svc.mb) return;
    service_quiesce();
    (void)hipStreamDestroy(g_svc.stream);
    (void)hipHostFree(g_svc.mb);
    g_svc.mb = nullptr;
    g_svc.stream = nullptr;
    g_svc.device = -1;
}

void device_sync() {
    service_quiesce();
    SHMX_HIP(hipDeviceSynchronize());
}

}  // namespace shmx

extern "C" int shmemx_service_stats(unsigned long long *out, int nout, int reset) {
    std::lock_guard<std::recursive_mutex> lk(shmx::g_mu);
    if (!out || nout < 0) return shmx::set_error(SHMEMX_EINVAL), -1;
    shmx::Service &v = shmx::g_svc;
    const unsigned long long all[7] = {v.served, v.launches, v.busy_null, v.busy_lib, v.ns_before_post,
                                       v.ns_round_trip, v.folds};
    const int k = nout < 7 ? nout : 7;
    for (int i = 0; i < k; ++i) out[i] = all[i];
    if (reset) v.served = v.launches = v.busy_null = v.busy_lib = v.ns_before_post = v.ns_round_trip = v.folds = 0;
    return k;
}
