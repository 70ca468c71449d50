// Lab: does a resident (persistent) workgroup on one stream hold up kernels
// on the process's other streams?  HIP multiplexes streams over a few
// hardware queues ($GPU_MAX_HW_QUEUES, 4 on the box), and a queue runs its
// packets in order: a stream that shares the resident kernel's queue would
// wait for it to leave.  (csrc/service.hip's design question.)
//
//   queue_lab [mode]     mode: plain | cumask_all | cumask_one | priority
//
// Creates the null stream's work, one blocking and six non-blocking streams
// (more streams than hardware queues), then the resident kernel's stream in
// the given way, parks a resident workgroup there (it polls a host word and
// leaves when told, or after 50 ms), and times a one-workgroup kernel that
// stores a host-coherent word on every other stream: a stream sharing the
// resident kernel's queue shows ~ the time until the resident one leaves.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void resident(unsigned long long *quit, unsigned long long *alive, unsigned long long ticks) {
    if (threadIdx.x != 0) return;
    __hip_atomic_store(alive, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (!__hip_atomic_load(quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) break;
        __builtin_amdgcn_s_sleep(2);
    }
    __hip_atomic_store(alive, 2ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void tiny(unsigned long long *word, unsigned long long v) {
    if (threadIdx.x == 0) __hip_atomic_store(word, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// mode "lag": after a one-workgroup kernel on a blocking stream has stored
// its host word, how long do hipStreamQuery(that stream) and
// hipStreamQuery(null) keep answering "not ready", and what does a
// hipStreamSynchronize cost at that point?  (median of 500)
static int lag_mode() {
    unsigned long long *h = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&h), 4096, hipHostMallocCoherent));
    std::memset(h, 0, 4096);
    volatile unsigned long long *word = h;
    hipStream_t b, nb;
    CK(hipStreamCreate(&b));
    CK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
    for (hipStream_t s : {b, nb}) {
        std::vector<double> q_own, q_null, t_sync;
        for (int i = 0; i < 600; ++i) {
            const unsigned long long v = (unsigned long long)i + 1 + (s == nb ? 100000 : 0);
            hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, h, v);
            while (*word != v) {
            }
            const double t0 = now_us();
            double own = -1, nul = -1;
            while (own < 0 || nul < 0) {
                const double t = now_us() - t0;
                if (own < 0 && hipStreamQuery(s) == hipSuccess) own = t;
                if (nul < 0 && hipStreamQuery(nullptr) == hipSuccess) nul = t;
                if (t > 1e5) break;
            }
            // and a launch whose completion is waited for with a synchronize
            hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, h, v + 1000000);
            while (*word != v + 1000000) {
            }
            const double t1 = now_us();
            CK(hipStreamSynchronize(s));
            if (i >= 100) {
                q_own.push_back(own);
                q_null.push_back(nul);
                t_sync.push_back(now_us() - t1);
            }
        }
        auto med = [](std::vector<double> v) {
            std::sort(v.begin(), v.end());
            return v[v.size() / 2];
        };
        std::printf("%s stream: after the host word, own query ready in %.2f us, null query in %.2f us; "
                    "a synchronize then takes %.2f us (medians)\n",
                    s == b ? "blocking" : "non-blocking", med(q_own), med(q_null), med(t_sync));
    }
    std::printf("ok\n");
    return 0;
}

int main(int argc, char **argv) {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    const std::string mode = argc > 1 ? argv[1] : "plain";
    if (mode == "lag") return lag_mode();
    CK(hipSetDevice(0));
    unsigned long long *h = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&h), 4096, hipHostMallocCoherent));
    std::memset(h, 0, 4096);
    volatile unsigned long long *word = h, *quit = h + 64, *alive = h + 128;
    std::vector<hipStream_t> others;
    std::vector<std::string> names;
    others.push_back(nullptr);
    names.push_back("null");
    hipStream_t b;
    CK(hipStreamCreate(&b));
    others.push_back(b);
    names.push_back("blocking");
    for (int i = 0; i < 6; ++i) {
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        others.push_back(s);
        names.push_back("nonblocking" + std::to_string(i));
    }
    hipStream_t svc;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    if (mode == "plain") {
        CK(hipStreamCreateWithFlags(&svc, hipStreamNonBlocking));
    } else if (mode == "priority") {
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        CK(hipStreamCreateWithPriority(&svc, hipStreamNonBlocking, hi));
    } else {
        std::vector<uint32_t> mask((ncu + 31) / 32, 0);
        if (mode == "cumask_all") {
            for (int c = 0; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
        } else {
            mask[0] = 1u;
        }
        CK(hipExtStreamCreateWithCUMask(&svc, (uint32_t)mask.size(), mask.data()));
    }
    // warm every stream (their queues get assigned) and time the tiny kernel alone
    unsigned long long v = 0;
    auto time_on = [&](hipStream_t s, double limit_us) {
        ++v;
        const double t0 = now_us();
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, h, v);
        while (*word != v) {
            if (now_us() - t0 > limit_us) return -1.0;
        }
        return now_us() - t0;
    };
    for (int rep = 0; rep < 3; ++rep)
        for (auto s : others) (void)time_on(s, 1e6);
    std::printf("mode %s (%d CUs)\n", mode.c_str(), ncu);
    for (size_t i = 0; i < others.size(); ++i) std::printf("  alone      %-14s %8.2f us\n", names[i].c_str(), time_on(others[i], 1e6));
    // the resident workgroup
    hipLaunchKernelGGL(resident, dim3(1), dim3(64), 0, svc, h + 64, h + 128, 5000000ull);   // 50 ms
    {
        const double t0 = now_us();
        while (*alive != 1) {
            if (now_us() - t0 > 2e6) {
                std::printf("resident kernel never started\n");
                return 3;
            }
        }
    }
    for (size_t i = 0; i < others.size(); ++i) {
        const double t = time_on(others[i], 20000);   // 20 ms
        if (t < 0) {
            std::printf("  resident   %-14s BLOCKED (> 20 ms)\n", names[i].c_str());
            // let it through, then continue
            const double t0 = now_us();
            while (*word != v && now_us() - t0 < 2e6) {
            }
        } else {
            std::printf("  resident   %-14s %8.2f us\n", names[i].c_str(), t);
        }
    }
    std::printf("  resident still up: %s\n", *alive == 1 ? "yes" : "no");
    __atomic_store_n(const_cast<unsigned long long *>(quit), 1ull, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(svc));
    CK(hipDeviceSynchronize());
    std::printf("ok\n");
    return 0;
}
