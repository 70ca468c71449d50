// Lab: where the microseconds of a small blocking one-member call go when it
// is served by the resident service workgroup (csrc/service.hip).  Links the
// library; medians (us) over `reps` calls of:
//   api        shmem_longlong_sum_to_all(tgt, src, n, 0, 0, 1, ...) on device arrays
//   attr2      two hipPointerGetAttributes (the entry point's operand checks)
//   query2     hipStreamQuery(null) + hipStreamQuery(the library stream)
//   devget     hipGetDevice (the entry point's device binding)
//
//   call_breakdown [reps] [n]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "shmem_reduce_mi355x.h"

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

// The lab's mailbox kernel (tools/service_lab.hip, line mode), in this
// process beside the library's, to tell the kernels apart from the process.
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


static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static void run(const char *name, int reps, const std::function<void()> &f) {
    std::vector<double> v;
    for (int r = 0; r < reps + 100; ++r) {
        const double t0 = now_us();
        f();
        if (r >= 100) v.push_back(now_us() - t0);
    }
    std::sort(v.begin(), v.end());
    std::printf("%-8s median %7.2f us  p10 %7.2f  p90 %7.2f\n", name, v[v.size() / 2], v[v.size() / 10],
                v[v.size() * 9 / 10]);
}

int main(int argc, char **argv) {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3000;
    const int n = argc > 2 ? std::atoi(argv[2]) : 1;
    CK(hipSetDevice(0));
    shmemx_init_attr(0, 1, 0, nullptr);
    long long *src = nullptr, *tgt = nullptr;
    CK(hipMalloc(&src, 1 << 20));
    CK(hipMalloc(&tgt, 1 << 20));
    CK(hipMemset(src, 1, 1 << 20));
    CK(hipDeviceSynchronize());
    static long psync[SHMEM_REDUCE_SYNC_SIZE];
    for (long &p : psync) p = SHMEM_SYNC_VALUE;
    run("api", reps, [&] { shmem_longlong_sum_to_all(tgt, src, n, 0, 0, 1, nullptr, psync); });
    // (handing the library stream out makes every later call ask about it)
    hipStream_t lib = static_cast<hipStream_t>(shmemx_get_stream());
    run("attr2", reps, [&] {
        hipPointerAttribute_t a;
        (void)hipPointerGetAttributes(&a, tgt);
        (void)hipPointerGetAttributes(&a, src);
    });
    run("query2", reps, [&] {
        (void)hipStreamQuery(nullptr);
        (void)hipStreamQuery(lib);
    });
    run("devget", reps, [&] {
        int d = 0;
        (void)hipGetDevice(&d);
    });
    run("api_x", reps, [&] { shmem_longlong_sum_to_all(tgt, src, n, 0, 0, 1, nullptr, psync); });
    unsigned long long st[6] = {0, 0, 0, 0, 0, 0};
    shmemx_service_stats(st, 6, 0);
    std::printf("service: served %llu launches %llu busy null %llu lib %llu; per call: %.2f us to the post, "
                "%.2f us post to done\n", st[0], st[1], st[2], st[3], st[0] ? st[4] * 1e-3 / st[0] : 0.0,
                st[0] ? st[5] * 1e-3 / st[0] : 0.0);
    // the lab kernel in this process: its own mailbox, stream, 16-byte copy
    {
        LabMailbox *mb = nullptr;
        CK(hipHostMalloc(reinterpret_cast<void **>(&mb), sizeof(LabMailbox), hipHostMallocCoherent));
        std::memset(mb, 0, sizeof *mb);
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        hipStream_t svc;
        CK(hipStreamCreateWithPriority(&svc, hipStreamNonBlocking, hi));
        unsigned long long seq = 0;
        for (int round = 0; round < 2; ++round) {
        // a fresh launch each round (the previous one told to leave); the
        // library's workgroup idles out between its rounds and is launched again
        hipLaunchKernelGGL(service_kernel<true>, dim3(1), dim3(256), 0, svc, mb, seq, 20000000ull);
        run("lab_line", reps, [&] {
            mb->src = src;
            mb->dst = tgt;
            mb->bytes = 16;
            ++seq;
            mb->check = seq ^ reinterpret_cast<uintptr_t>(src) ^ reinterpret_cast<uintptr_t>(tgt) ^ 16ull ^ kLabMix;
            __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
            const volatile unsigned long long *d = &mb->done;
            const double t0 = now_us();
            while (*d != seq)
                if (now_us() - t0 > 2e6) {
                    std::printf("lab kernel hung\n");
                    std::exit(3);
                }
        });
        // the same with the library's host spin (a pause per poll of the done word)
        run("lab_pause", reps, [&] {
            mb->src = src;
            mb->dst = tgt;
            mb->bytes = 16;
            ++seq;
            mb->check = seq ^ reinterpret_cast<uintptr_t>(src) ^ reinterpret_cast<uintptr_t>(tgt) ^ 16ull ^ kLabMix;
            __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
            const volatile unsigned long long *d = &mb->done;
            for (unsigned k = 1; *d != seq; ++k) {
                __builtin_ia32_pause();
                if ((k & 4095) == 0 && k > (1u << 26)) {
                    std::printf("lab kernel hung\n");
                    std::exit(3);
                }
            }
        });
        __atomic_store_n(&mb->quit, 1ull, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(svc));
        __atomic_store_n(&mb->quit, 0ull, __ATOMIC_RELEASE);
        run("api", reps, [&] { shmem_longlong_sum_to_all(tgt, src, n, 0, 0, 1, nullptr, psync); });
        { const double t0 = now_us(); while (now_us() - t0 < 2000) {} }
        }
    }
    shmem_finalize();
    std::printf("ok\n");
    return 0;
}
