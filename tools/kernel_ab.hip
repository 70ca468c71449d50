// Lab: the round trip of the library's service kernel (namespace L, the
// round-6 kernel of csrc/service.hip as of this lab) against the lab's
// line-read mailbox kernel (tools/service_lab.hip), with the same host code,
// and the library kernel's round trip against the gap the host leaves between
// seeing one request done and posting the next (the phase of the post against
// the kernel's one read of host memory in flight).  profiles/r06_service_phase.txt.
//
//   kernel_ab [bytes] [1: initialise the library first]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>
#include "shmem_reduce_mi355x.h"
namespace L {
constexpr unsigned long long kMix = 0x9E3779B97F4A7C15ull;
constexpr unsigned kIdleUs = 200;
constexpr int kSvcBlock = 256;

// Written by the host: the first line (seq last, with release); by the
// device: the second.
struct alignas(64) Mailbox {
    unsigned long long seq;
    unsigned long long quit;
    const void *src;
    void *dst;
    void *dst2;   // a second destination (the mirrored heap's view), or null
    unsigned long long bytes;
    unsigned long long check;   // seq ^ src ^ dst ^ dst2 ^ bytes ^ kMix
    unsigned long long pad;
    alignas(64) unsigned long long done;
};
static_assert(sizeof(Mailbox) == 128, "two lines");

// Global-memory views of the operands (their addresses arrive through LDS,
// which would leave generic flat accesses otherwise).
template <typename V>
using gptr = __attribute__((address_space(1))) V *;

// One pass: lane t moves words t, t + 256, ... (a 32 KiB copy of 16-byte
// words is 8 per lane).  Every lane issues all its loads before its first
// store: within a pass of 256 words that some lane needs, the loads are
// unconditional (an index past the end reads the last word again), only the
// stores are masked, so no load waits for another.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <typename V>
__device__ __forceinline__ void copy_as(const unsigned char *src, unsigned char *dst, unsigned char *dst2,
                                        unsigned long long bytes) {
    constexpr int U = 8;
    const gptr<const V> s = (gptr<const V>)(src);
    const gptr<V> d = (gptr<V>)(dst);
    const gptr<V> d2 = (gptr<V>)(dst2);
    const unsigned long long n = bytes / sizeof(V);
    for (unsigned long long base = 0; base < n; base += (unsigned long long)U * kSvcBlock) {
        V v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // (a uniform test: a pass no lane needs issues no load)
            if (base + (unsigned long long)u * kSvcBlock < n) {
                const unsigned long long i = base + threadIdx.x + (unsigned long long)u * kSvcBlock;
                v[u] = s[i < n ? i : n - 1];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long i = base + threadIdx.x + (unsigned long long)u * kSvcBlock;
            if (i < n) {
                d[i] = v[u];
                if (dst2) d2[i] = v[u];
            }
        }
    }
}

__global__ __launch_bounds__(kSvcBlock) void service_kernel(Mailbox *mb, unsigned long long served,
                                                         unsigned long long idle_ticks) {
    __shared__ unsigned long long s_seq, s_bytes;
    __shared__ const unsigned char *s_src;
    __shared__ unsigned char *s_dst, *s_dst2;
    unsigned long long last = served;
    unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (threadIdx.x < 64) {
            // wave 0: lanes 0-6 read the mailbox's first line in one load
            // instruction, every lane takes the words from them
            const unsigned long long *line = reinterpret_cast<const unsigned long long *>(mb);
            const int lane = threadIdx.x;
            unsigned long long q = 0;
            for (;;) {
                const unsigned long long v =
                    lane < 7 ? __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
                q = __shfl(v, 0);
                const unsigned long long quit = __shfl(v, 1);
                if (q != last) {
                    const unsigned long long a = __shfl(v, 2), b = __shfl(v, 3), b2 = __shfl(v, 4),
                                             n = __shfl(v, 5), c = __shfl(v, 6);
                    if ((q ^ a ^ b ^ b2 ^ n ^ kMix) == c) {
                        if (lane == 0) {
                            // lines of the source another kernel wrote since
                            // this one started are dropped (system scope)
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                            s_src = reinterpret_cast<const unsigned char *>(a);
                            s_dst = reinterpret_cast<unsigned char *>(b);
                            s_dst2 = reinterpret_cast<unsigned char *>(b2);
                            s_bytes = n;
                        }
                        break;
                    }
                    continue;   // torn read: the line again
                }
                if (quit || __builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) {
                    q = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0) s_seq = q;
        }
        __syncthreads();
        const unsigned long long q = s_seq;
        if (!q) return;   // idle or told to quit: every wave leaves here
        const unsigned char *src = s_src;
        unsigned char *dst = s_dst, *dst2 = s_dst2;
        const unsigned long long n = s_bytes;
        const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) |
                             reinterpret_cast<uintptr_t>(dst2) | n;
        if ((al & 15) == 0) copy_as<v4u>(src, dst, dst2, n);
        else if ((al & 7) == 0) copy_as<unsigned long long>(src, dst, dst2, n);
        else if ((al & 3) == 0) copy_as<unsigned>(src, dst, dst2, n);
        else if ((al & 1) == 0) copy_as<unsigned short>(src, dst, dst2, n);
        else copy_as<unsigned char>(src, dst, dst2, n);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's stores issued and done
        __syncthreads();
        if (threadIdx.x == 0)   // write back, then tell the host
            __hip_atomic_store(&mb->done, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last = q;
        t_last = __builtin_amdgcn_s_memrealtime();
        __syncthreads();   // the s_* words are read before wave 0 polls again
    }
}


}
struct alignas(64) LabMailbox {
    // one 64-byte line the device reads; the host writes the fields and
    // check first, seq last (release)
    unsigned long long seq;
    unsigned long long quit;
    const void *src;
    void *dst;
    unsigned long long bytes;
    unsigned long long check;   // seq ^ src ^ dst ^ bytes ^ kLabMix: a torn read shows
    unsigned long long pad[2];
    // the device's line
    alignas(64) unsigned long long done;   // (system-scope release)
    unsigned long long polls;   // heartbeat: polls so far (every 1024th)
};
constexpr unsigned long long kLabMix = 0x9E3779B97F4A7C15ull;

// LINE: wave 0's lanes 0-5 read the mailbox's first line with one load
// instruction (the descriptor arrives with the sequence number, no second
// round trip over PCIe); the check word catches a torn read
template <bool LINE>
__global__ __launch_bounds__(256) void service_kernel(LabMailbox *mb, unsigned long long served,
                                                      unsigned long long idle_ticks) {
    __shared__ unsigned long long s_seq;
    __shared__ const unsigned char *s_src;
    __shared__ unsigned char *s_dst;
    __shared__ unsigned long long s_bytes;
    unsigned long long last = served, npoll = 0;
    unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (LINE && threadIdx.x < 64) {
            const unsigned long long *line = reinterpret_cast<const unsigned long long *>(mb);
            const int lane = threadIdx.x;
            unsigned long long q = 0;
            for (;;) {
                const unsigned long long v =
                    lane < 6 ? __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
                q = __shfl(v, 0);
                const unsigned long long quit = __shfl(v, 1);
                if (q != last) {
                    const unsigned long long a = __shfl(v, 2), b = __shfl(v, 3), n = __shfl(v, 4),
                                             c = __shfl(v, 5);
                    if ((q ^ a ^ b ^ n ^ kLabMix) == c) {
                        if (lane == 0) {
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope: fresh lines
                            s_src = reinterpret_cast<const unsigned char *>(a);
                            s_dst = reinterpret_cast<unsigned char *>(b);
                            s_bytes = n;
                        }
                        break;
                    }
                    continue;   // torn: read the line again
                }
                if (quit || __builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) {
                    q = 0;
                    break;
                }
                if (lane == 0 && (++npoll & 1023) == 0)
                    __hip_atomic_store(&mb->polls, npoll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0) s_seq = q;
        } else if (!LINE && threadIdx.x == 0) {
            unsigned long long q = 0;
            for (;;) {
                q = __hip_atomic_load(&mb->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (q != last) break;
                if (__hip_atomic_load(&mb->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                    q = 0;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) {
                    q = 0;
                    break;
                }
                if ((++npoll & 1023) == 0)
                    __hip_atomic_store(&mb->polls, npoll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __builtin_amdgcn_s_sleep(1);
            }
            if (q) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope: fresh lines
                s_src = static_cast<const unsigned char *>(mb->src);
                s_dst = static_cast<unsigned char *>(mb->dst);
                s_bytes = mb->bytes;
            }
            s_seq = q;
        }
        __syncthreads();
        const unsigned long long q = s_seq;
        if (!q) return;   // every wave of the workgroup leaves together
        const unsigned char *src = s_src;
        unsigned char *dst = s_dst;
        const unsigned long long n = s_bytes;
        if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | n) & 15) == 0) {
            for (unsigned long long i = threadIdx.x; i < n / 16; i += 256)
                reinterpret_cast<uint4 *>(dst)[i] = reinterpret_cast<const uint4 *>(src)[i];
        } else {
            for (unsigned long long i = threadIdx.x; i < n; i += 256) dst[i] = src[i];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(&mb->done, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last = q;
        t_last = __builtin_amdgcn_s_memrealtime();
        __syncthreads();
    }
}



static double now_us() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
template <class F> static void run(const char *name, int reps, F f) {
    std::vector<double> v;
    for (int r = 0; r < reps + 100; ++r) { double t0 = now_us(); f(); if (r >= 100) v.push_back(now_us() - t0); }
    std::sort(v.begin(), v.end());
    std::printf("%-10s median %7.2f us p10 %7.2f p90 %7.2f\n", name, v[v.size()/2], v[v.size()/10], v[v.size()*9/10]);
}
int main(int argc, char **argv) {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    const int reps = 2000;
    const size_t bytes = argc > 1 ? std::atol(argv[1]) : 16;
    hipSetDevice(0);
    if (argc > 2 && argv[2][0] == '1') { shmemx_init_attr(0, 1, 0, nullptr); std::printf("library initialised\n"); }
    char *src, *tgt; hipMalloc(&src, 1 << 20); hipMalloc(&tgt, 1 << 20); hipMemset(src, 1, 1 << 20); hipDeviceSynchronize();
    int lo = 0, hi = 0; hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStream_t svc; hipStreamCreateWithPriority(&svc, hipStreamNonBlocking, hi);
    for (int round = 0; round < 2; ++round) {
      { // library kernel
        L::Mailbox *mb; hipHostMalloc((void **)&mb, sizeof *mb, hipHostMallocCoherent); std::memset(mb, 0, sizeof *mb);
        hipLaunchKernelGGL(L::service_kernel, dim3(1), dim3(L::kSvcBlock), 0, svc, mb, 0ull, 20000000ull);
        unsigned long long seq = 0;
        run("libkernel", reps, [&] {
            ++seq; mb->src = src; mb->dst = tgt; mb->dst2 = nullptr; mb->bytes = bytes;
            mb->check = seq ^ (uintptr_t)src ^ (uintptr_t)tgt ^ 0ull ^ bytes ^ L::kMix;
            __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
            const volatile unsigned long long *d = &mb->done; double t0 = now_us();
            while (*d != seq) if (now_us() - t0 > 2e6) { std::printf("hung\n"); std::exit(3); }
        });
        for (double gap : {0.2, 0.4, 0.6, 0.8, 1.0, 1.5, 2.0}) {
            std::vector<double> rt;
            for (int r = 0; r < reps; ++r) {
                { const double t0 = now_us(); while (now_us() - t0 < gap) {} }
                ++seq; mb->src = src; mb->dst = tgt; mb->dst2 = nullptr; mb->bytes = bytes;
                mb->check = seq ^ (uintptr_t)src ^ (uintptr_t)tgt ^ 0ull ^ bytes ^ L::kMix;
                __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
                const volatile unsigned long long *d = &mb->done; double t0 = now_us();
                while (*d != seq) if (now_us() - t0 > 2e6) { std::printf("hung\n"); std::exit(3); }
                rt.push_back(now_us() - t0);
            }
            std::sort(rt.begin(), rt.end());
            std::printf("libkernel gap %.1f us: post to done median %.2f p10 %.2f p90 %.2f\n", gap, rt[rt.size() / 2],
                        rt[rt.size() / 10], rt[rt.size() * 9 / 10]);
        }
        __atomic_store_n(&mb->quit, 1ull, __ATOMIC_RELEASE); hipStreamSynchronize(svc);
      }
      { // lab kernel
        LabMailbox *mb; hipHostMalloc((void **)&mb, sizeof *mb, hipHostMallocCoherent); std::memset(mb, 0, sizeof *mb);
        hipLaunchKernelGGL(service_kernel<true>, dim3(1), dim3(256), 0, svc, mb, 0ull, 20000000ull);
        unsigned long long seq = 0;
        run("labkernel", reps, [&] {
            ++seq; mb->src = src; mb->dst = tgt; mb->bytes = bytes;
            mb->check = seq ^ (uintptr_t)src ^ (uintptr_t)tgt ^ bytes ^ kLabMix;
            __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
            const volatile unsigned long long *d = &mb->done; double t0 = now_us();
            while (*d != seq) if (now_us() - t0 > 2e6) { std::printf("hung\n"); std::exit(3); }
        });
        hipStream_t lib; hipStreamCreate(&lib);
        for (int variant = 0; variant < 3; ++variant) {
        const char *names[3] = {"lab+query", "lab+attr", "lab+q+lib"};
        std::vector<double> rt;
        run(names[variant], reps, [&] {
            hipPointerAttribute_t pa;
            if (variant == 0) (void)hipStreamQuery(nullptr);
            if (variant == 1) { (void)hipPointerGetAttributes(&pa, src); (void)hipPointerGetAttributes(&pa, tgt); }
            if (variant == 2) { (void)hipStreamQuery(nullptr); (void)hipStreamQuery(lib); }
            ++seq; mb->src = src; mb->dst = tgt; mb->bytes = bytes;
            mb->check = seq ^ (uintptr_t)src ^ (uintptr_t)tgt ^ bytes ^ kLabMix;
            __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
            const volatile unsigned long long *d = &mb->done; double t0 = now_us();
            while (*d != seq) if (now_us() - t0 > 2e6) { std::printf("hung\n"); std::exit(3); }
            rt.push_back(now_us() - t0);
        });
        std::sort(rt.begin(), rt.end());
        std::printf("           post to done median %.2f us\n", rt[rt.size() / 2]);
        }
        __atomic_store_n(&mb->quit, 1ull, __ATOMIC_RELEASE); hipStreamSynchronize(svc);
      }
    }
    std::printf("ok\n");
}
