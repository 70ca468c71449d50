// Lab: how fast can a blocking small call finish when its work is done by a
// workgroup that is already resident (polling a page-locked mailbox) instead
// of a fresh kernel launch?  (VERDICT r05 "Next" #3)
//
//   service_lab [reps] [bytes]
//
// Prints medians (us) of:
//   launch_self   hipLaunchKernelGGL of a one-workgroup copy that stores a
//                 host-coherent word itself (system-scope release), host spins
//                 (the library's PE_size 1 floor today);
//   mailbox       the host writes a descriptor (src, dst, bytes) and a
//                 sequence number into host-coherent memory; one resident
//                 workgroup polls it, acquires, copies, releases, and stores
//                 the sequence into a host-coherent done word; host spins;
//   mailbox_q     the same preceded by hipStreamQuery of the null stream and of
//                 a blocking stream (the ordering check the library needs);
//   query         hipStreamQuery(null) + hipStreamQuery(blocking stream) alone.
// The resident kernel leaves after an idle timeout (no request for
// idle_us), or at once when the host stores the quit word; the host waits for
// its stream before exiting.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

struct alignas(64) Mailbox {
    // one 64-byte line the device reads; the host writes the fields and
    // check first, seq last (release)
    unsigned long long seq;
    unsigned long long quit;
    const void *src;
    void *dst;
    unsigned long long bytes;
    unsigned long long check;   // seq ^ src ^ dst ^ bytes ^ kMix: a torn read shows
    unsigned long long pad[2];
    // the device's line
    alignas(64) unsigned long long done;   // (system-scope release)
    unsigned long long polls;   // heartbeat: polls so far (every 1024th)
};
constexpr unsigned long long kMix = 0x9E3779B97F4A7C15ull;

// LINE: wave 0's lanes 0-5 read the mailbox's first line with one load
// instruction (the descriptor arrives with the sequence number, no second
// round trip over PCIe); the check word catches a torn read
template <bool LINE>
__global__ __launch_bounds__(256) void service_kernel(Mailbox *mb, unsigned long long served,
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
                    if ((q ^ a ^ b ^ n ^ kMix) == c) {
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

__global__ __launch_bounds__(256) void copy_self(const unsigned char *src, unsigned char *dst,
                                                 unsigned long long n, unsigned long long *word,
                                                 unsigned long long v) {
    for (unsigned long long i = threadIdx.x; i < n / 16; i += 256)
        reinterpret_cast<uint4 *>(dst)[i] = reinterpret_cast<const uint4 *>(src)[i];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(word, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static const char *g_phase = "start";
static Mailbox *g_mb = nullptr;
static hipStream_t g_svc = nullptr;
// a host wait that has lasted more than 2 s: say where, stop the kernel, exit
static void watchdog(double t0, const char *what) {
    if (now_us() - t0 < 2e6) return;
    std::fprintf(stderr, "HUNG in %s (%s): seq %llu done %llu polls %llu svc query %d\n", g_phase, what,
                 g_mb ? g_mb->seq : 0ull, g_mb ? g_mb->done : 0ull, g_mb ? g_mb->polls : 0ull,
                 g_svc ? (int)hipStreamQuery(g_svc) : -1);
    if (g_mb) __atomic_store_n(&g_mb->quit, 1ull, __ATOMIC_RELEASE);
    std::exit(3);
}

static void report(const char *name, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    std::printf("%-12s median %8.2f us  p10 %7.2f  p90 %7.2f  max %8.2f\n", name, v[v.size() / 2],
                v[v.size() / 10], v[v.size() * 9 / 10], v.back());
}

int main(int argc, char **argv) {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3000;
    const size_t bytes = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 4096;
    CK(hipSetDevice(0));
    void *src = nullptr, *dst = nullptr;
    CK(hipMalloc(&src, 1 << 20));
    CK(hipMalloc(&dst, 1 << 20));
    CK(hipMemset(src, 7, 1 << 20));
    hipStream_t blocking, svc;
    CK(hipStreamCreate(&blocking));
    {
        // the library's choice: a non-blocking stream of the greatest priority
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        CK(hipStreamCreateWithPriority(&svc, hipStreamNonBlocking, hi));
    }
    Mailbox *mb = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&mb), sizeof(Mailbox), hipHostMallocCoherent));
    std::memset(mb, 0, sizeof *mb);
    g_mb = mb;
    g_svc = svc;
    unsigned long long *word = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&word), 64, hipHostMallocCoherent));
    *word = 0;
    CK(hipDeviceSynchronize());
    volatile unsigned long long *vw = word;

    std::vector<double> t;
    // 1. launch + self-signal
    g_phase = "launch_self";
    std::fprintf(stderr, "phase %s\n", g_phase);
    for (int i = 0; i < reps + 50; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(copy_self, dim3(1), dim3(256), 0, blocking, static_cast<const unsigned char *>(src),
                           static_cast<unsigned char *>(dst), (unsigned long long)bytes, word,
                           (unsigned long long)(i + 1));
        for (unsigned k = 1; *vw != (unsigned long long)(i + 1); ++k) {
            __builtin_ia32_pause();
            if ((k & 65535) == 0) watchdog(t0, "launch_self spin");
        }
        if (i >= 50) t.push_back(now_us() - t0);
    }
    CK(hipStreamSynchronize(blocking));
    report("launch_self", t);

    // 2. mailbox round trips (idle timeout 200 us)
    const unsigned long long idle_ticks = 200 * 100;   // s_memrealtime: 100 MHz
    unsigned long long seq = 0;
    bool line_mode = false;
    // (re)launch: the kernel starts from the last request the previous one
    // completed, so a request posted while it was leaving is served
    auto launch_service = [&] {
        const unsigned long long served = __atomic_load_n(&mb->done, __ATOMIC_ACQUIRE);
        if (line_mode)
            hipLaunchKernelGGL(service_kernel<true>, dim3(1), dim3(256), 0, svc, mb, served, idle_ticks);
        else
            hipLaunchKernelGGL(service_kernel<false>, dim3(1), dim3(256), 0, svc, mb, served, idle_ticks);
        CK(hipGetLastError());
    };
    auto post = [&](bool query) {
        if (query) {
            if (hipStreamQuery(nullptr) != hipSuccess || hipStreamQuery(blocking) != hipSuccess) {
                std::fprintf(stderr, "streams not idle\n");
            }
        }
        mb->src = src;
        mb->dst = dst;
        mb->bytes = bytes;
        ++seq;
        mb->check = seq ^ reinterpret_cast<uintptr_t>(src) ^ reinterpret_cast<uintptr_t>(dst) ^ bytes ^ kMix;
        __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
        const volatile unsigned long long *d = &mb->done;
        const double t0 = now_us();
        for (unsigned k = 1;; ++k) {
            if (*d == seq) return;
            __builtin_ia32_pause();
            if ((k & 65535) == 0) watchdog(t0, "mailbox spin");
            if ((k & 4095) == 0 && hipStreamQuery(svc) == hipSuccess && *d != seq) launch_service();
        }
    };
    g_phase = "mailbox";
    std::fprintf(stderr, "phase %s\n", g_phase);
    launch_service();
    t.clear();
    for (int i = 0; i < reps + 50; ++i) {
        const double t0 = now_us();
        post(false);
        if (i >= 50) t.push_back(now_us() - t0);
    }
    report("mailbox", t);
    g_phase = "mailbox_q";
    std::fprintf(stderr, "phase %s\n", g_phase);
    t.clear();
    for (int i = 0; i < reps + 50; ++i) {
        const double t0 = now_us();
        post(true);
        if (i >= 50) t.push_back(now_us() - t0);
    }
    report("mailbox_q", t);
    t.clear();
    for (int i = 0; i < reps; ++i) {
        const double t0 = now_us();
        (void)hipStreamQuery(nullptr);
        (void)hipStreamQuery(blocking);
        t.push_back(now_us() - t0);
    }
    report("query", t);
    // 3. after an idle gap longer than the timeout: relaunch on demand
    g_phase = "cold_relaunch";
    std::fprintf(stderr, "phase %s\n", g_phase);
    t.clear();
    for (int i = 0; i < 200; ++i) {
        const double ts = now_us();
        while (now_us() - ts < 400) {
        }
        const double t0 = now_us();
        if (hipStreamQuery(svc) == hipSuccess) launch_service();
        post(false);
        t.push_back(now_us() - t0);
    }
    report("cold_relaunch", t);
    // 4. the line-read variant, warm and after idle gaps
    g_phase = "line";
    std::fprintf(stderr, "phase %s\n", g_phase);
    __atomic_store_n(&mb->quit, 1ull, __ATOMIC_RELEASE);
    {
        const double t0 = now_us();
        while (hipStreamQuery(svc) == hipErrorNotReady) watchdog(t0, "service exit before line");
    }
    __atomic_store_n(&mb->quit, 0ull, __ATOMIC_RELEASE);
    line_mode = true;
    launch_service();
    t.clear();
    for (int i = 0; i < reps + 50; ++i) {
        const double t0 = now_us();
        post(false);
        if (i >= 50) t.push_back(now_us() - t0);
    }
    report("mailbox_line", t);
    t.clear();
    for (int i = 0; i < 200; ++i) {
        const double ts = now_us();
        while (now_us() - ts < 400) {
        }
        const double t0 = now_us();
        if (hipStreamQuery(svc) == hipSuccess) launch_service();
        post(false);
        t.push_back(now_us() - t0);
    }
    report("line_cold", t);
    // 5. gated posts: the host writes the descriptor and check word, and the
    // sequence number is stored by the null stream itself
    // (hipStreamWriteValue64), i.e. once everything enqueued on the legacy
    // stream before it, and on the blocking streams it waits for, has
    // completed; alone, and right after a kernel on a blocking stream (whose
    // retiring keeps hipStreamQuery(null) "not ready" for ~30 us)
    g_phase = "gated";
    std::fprintf(stderr, "phase %s\n", g_phase);
    auto post_gated = [&] {
        mb->src = src;
        mb->dst = dst;
        mb->bytes = bytes;
        ++seq;
        mb->check = seq ^ reinterpret_cast<uintptr_t>(src) ^ reinterpret_cast<uintptr_t>(dst) ^ bytes ^ kMix;
        CK(hipStreamWriteValue64(nullptr, &mb->seq, seq, 0));
        const volatile unsigned long long *d = &mb->done;
        const double t0 = now_us();
        for (unsigned k = 1;; ++k) {
            if (*d == seq) return;
            __builtin_ia32_pause();
            if ((k & 4095) == 0 && hipStreamQuery(svc) == hipSuccess && *d != seq) launch_service();
            if ((k & 65535) == 0) watchdog(t0, "gated spin");
        }
    };
    if (hipStreamQuery(svc) == hipSuccess) launch_service();
    t.clear();
    for (int i = 0; i < reps + 50; ++i) {
        const double t0 = now_us();
        post_gated();
        if (i >= 50) t.push_back(now_us() - t0);
    }
    report("gated", t);
    t.clear();
    for (int i = 0; i < 500; ++i) {
        const unsigned long long v = 7000000ull + i;
        hipLaunchKernelGGL(copy_self, dim3(1), dim3(256), 0, blocking, static_cast<const unsigned char *>(src),
                           static_cast<unsigned char *>(dst), (unsigned long long)bytes, word, v);
        while (*vw != v) __builtin_ia32_pause();
        const double t0 = now_us();
        post_gated();
        t.push_back(now_us() - t0);
    }
    report("gated_after", t);
    // correctness: dst holds src's bytes
    std::vector<unsigned char> h(bytes);
    g_phase = "check";
    CK(hipMemcpyAsync(h.data(), dst, bytes, hipMemcpyDeviceToHost, blocking));
    CK(hipStreamSynchronize(blocking));
    for (size_t i = 0; i < bytes; ++i)
        if (h[i] != 7) {
            std::printf("WRONG at %zu\n", i);
            return 1;
        }
    g_phase = "quit";
    std::fprintf(stderr, "phase %s\n", g_phase);
    __atomic_store_n(&mb->quit, 1ull, __ATOMIC_RELEASE);
    {
        const double t0 = now_us();
        while (hipStreamQuery(svc) == hipErrorNotReady) watchdog(t0, "service exit");
    }
    std::printf("ok bytes %zu reps %d\n", bytes, reps);
    return 0;
}
