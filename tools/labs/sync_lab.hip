// Experiment harness (not part of the library): what a blocking call's
// "wait for my kernels" costs on one MI355X, per way of waiting.  Each line
// is the median over 2000 round trips of: launch a small copy kernel (one
// 8-byte element, like the ISx nreduce = 1 call), then wait for it.
//   sync          hipStreamSynchronize on the stream
//   event         hipEventRecord + hipEventSynchronize
//   marker_poll   a 1-thread kernel after it stores a sequence number into
//                 host-coherent memory; the host spins on that word
//   self_poll     the copy kernel's last block stores the sequence number
//                 itself (a block counter picks the last block)
//   fence64_sync  the library's 64-block system fence kernel, then sync
//   fence64_poll  the same kernel, host spinning on its 64 words
// With `spin` as argv[1], hipSetDeviceFlags(hipDeviceScheduleSpin) first.
//   Build: hipcc --offload-arch=gfx950 -O3 tools/labs/sync_lab.hip -o tools/labs/sync_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("%s: %s\n", #x, hipGetErrorString(e));                    \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

__global__ void copy1(long long *t, const long long *s, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) t[i] = s[i];
}

__global__ void copy1_self(long long *t, const long long *s, int n, unsigned int *count,
                           unsigned int *flag, unsigned int seq) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) t[i] = s[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        const unsigned int done = atomicAdd(count, 1u) + 1;
        if (done == gridDim.x) {
            *count = 0;
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ void marker(unsigned int *flag, unsigned int seq) {
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void fence64(unsigned int *seen, unsigned int seq) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
        __hip_atomic_store(seen + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "spin")) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    long long *s, *t;
    unsigned int *count, *flag, *seen;
    CK(hipMalloc(&s, 4096 * 8));
    CK(hipMalloc(&t, 4096 * 8));
    CK(hipMalloc(&count, 4));
    CK(hipMemset(count, 0, 4));
    CK(hipHostMalloc(&flag, 4, hipHostMallocCoherent));
    CK(hipHostMalloc(&seen, 64 * 4, hipHostMallocCoherent));
    *flag = 0;
    memset(seen, 0, 256);
    hipStream_t blocking, nonblocking;
    CK(hipStreamCreate(&blocking));
    CK(hipStreamCreateWithFlags(&nonblocking, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipDeviceSynchronize());
    unsigned int seq = 0;
    const int reps = 2000;
    for (hipStream_t st : {blocking, nonblocking}) {
        const char *sname = st == blocking ? "blocking" : "nonblocking";
        for (int mode = 0; mode < 6; ++mode) {
            static const char *names[] = {"sync", "event", "marker_poll", "self_poll", "fence64_sync",
                                          "fence64_poll"};
            std::vector<double> v;
            for (int r = 0; r < reps + 50; ++r) {
                const double t0 = now_us();
                ++seq;
                if (mode == 3) {
                    hipLaunchKernelGGL(copy1_self, dim3(1), dim3(64), 0, st, t, s, 1, count, flag, seq);
                } else {
                    hipLaunchKernelGGL(copy1, dim3(1), dim3(64), 0, st, t, s, 1);
                }
                switch (mode) {
                case 0: CK(hipStreamSynchronize(st)); break;
                case 1:
                    CK(hipEventRecord(ev, st));
                    CK(hipEventSynchronize(ev));
                    break;
                case 2:
                    hipLaunchKernelGGL(marker, dim3(1), dim3(1), 0, st, flag, seq);
                    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                    }
                    break;
                case 3:
                    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                    }
                    break;
                case 4:
                    hipLaunchKernelGGL(fence64, dim3(64), dim3(64), 0, st, seen, seq);
                    CK(hipStreamSynchronize(st));
                    break;
                case 5:
                    hipLaunchKernelGGL(fence64, dim3(64), dim3(64), 0, st, seen, seq);
                    for (int b = 0; b < 64; ++b)
                        while (__atomic_load_n(seen + b, __ATOMIC_ACQUIRE) != seq) {
                        }
                    break;
                }
                if (r >= 50) v.push_back(now_us() - t0);
            }
            CK(hipStreamSynchronize(st));
            std::sort(v.begin(), v.end());
            printf("%-11s %-13s median %6.2f us  p10 %6.2f  p90 %6.2f\n", sname, names[mode], v[v.size() / 2],
                   v[v.size() / 10], v[v.size() * 9 / 10]);
        }
    }
    // launch cost alone (no wait), 64 launches back to back
    {
        const double t0 = now_us();
        for (int r = 0; r < 64; ++r) hipLaunchKernelGGL(copy1, dim3(1), dim3(64), 0, nonblocking, t, s, 1);
        const double t1 = now_us();
        CK(hipStreamSynchronize(nonblocking));
        printf("launch alone: %.2f us per launch (host side)\n", (t1 - t0) / 64);
    }
    return 0;
}
