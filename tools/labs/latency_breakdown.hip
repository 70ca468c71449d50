// Experiment harness (not part of the library): where the ~14.6 us of a
// blocking small-message call at PE_size = 1 goes (the ISx use,
// shmem_longlong_sum_to_all with nreduce = 1, isx.c:617), on device arrays.
// Each line: median over 3000 calls, after 200 warm-up calls.
//   attr          one hipPointerGetAttributes (the call makes two)
//   api           shmem_longlong_sum_to_all(tgt, src, 1, 0, 0, 1, pWrk, pSync)
//   fold_sync     shmemx_fold_on_stream (the copy kernel) + hipStreamSynchronize
//   kernel_sync   a one-element copy kernel of this file + hipStreamSynchronize
//   kernel_marker the same + a 1-thread kernel storing a sequence number into
//                 host-coherent memory, the host spinning on it
//   kernel_self   the copy kernel storing the sequence number itself (one
//                 block: system-scope release store after its copy)
//   Build: hipcc --offload-arch=gfx950 -O3 -I include tools/labs/latency_breakdown.hip \
//            -L openshmem-async_amd -lshmem_reduce_mi355x -Wl,-rpath,$PWD/openshmem-async_amd \
//            -o tools/labs/latency_breakdown
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "shmem_reduce_mi355x.h"

#define CK(x)                                                                  \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("%s: %s\n", #x, hipGetErrorString(e));                    \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

__global__ void copy1(long long *t, const long long *s) { t[threadIdx.x] = s[threadIdx.x]; }

__global__ void copy1_self(long long *t, const long long *s, unsigned long long *flag,
                           unsigned long long seq) {
    t[threadIdx.x] = s[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void marker(unsigned long long *flag, unsigned long long seq) {
    __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static void run(const char *name, const std::function<void()> &f) {
    std::vector<double> v;
    for (int r = 0; r < 3200; ++r) {
        const double t0 = now_us();
        f();
        if (r >= 200) v.push_back(now_us() - t0);
    }
    std::sort(v.begin(), v.end());
    printf("%-14s median %7.2f us  p10 %7.2f  p90 %7.2f\n", name, v[v.size() / 2], v[v.size() / 10],
           v[v.size() * 9 / 10]);
}

int main() {
    shmem_init();
    long long *s, *t;
    CK(hipMalloc(&s, 64 * 8));
    CK(hipMalloc(&t, 64 * 8));
    CK(hipMemset(s, 1, 64 * 8));
    unsigned long long *flag;
    CK(hipHostMalloc(&flag, 8, hipHostMallocCoherent));
    *(volatile unsigned long long *)flag = 0;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    long pSync[SHMEM_REDUCE_SYNC_SIZE];
    for (long &x : pSync) x = SHMEM_SYNC_VALUE;
    long long pWrk[SHMEM_REDUCE_MIN_WRKDATA_SIZE];
    unsigned long long seq = 0;
    CK(hipDeviceSynchronize());
    run("attr", [&] {
        hipPointerAttribute_t a;
        (void)hipPointerGetAttributes(&a, t);
    });
    run("api", [&] { shmem_longlong_sum_to_all(t, s, 1, 0, 0, 1, pWrk, pSync); });
    run("fold_sync", [&] {
        shmemx_fold_on_stream(SHMEMX_TYPE_LONGLONG, SHMEMX_OP_SUM, t, s, 1, st);
        CK(hipStreamSynchronize(st));
    });
    run("kernel_sync", [&] {
        hipLaunchKernelGGL(copy1, dim3(1), dim3(1), 0, st, t, s);
        CK(hipStreamSynchronize(st));
    });
    run("kernel_marker", [&] {
        hipLaunchKernelGGL(copy1, dim3(1), dim3(1), 0, st, t, s);
        hipLaunchKernelGGL(marker, dim3(1), dim3(1), 0, st, flag, ++seq);
        while (*(volatile unsigned long long *)flag != seq) __builtin_ia32_pause();
    });
    run("kernel_self", [&] {
        hipLaunchKernelGGL(copy1_self, dim3(1), dim3(1), 0, st, t, s, flag, ++seq);
        while (*(volatile unsigned long long *)flag != seq) __builtin_ia32_pause();
    });
    // shmemx_checksum / shmemx_verify of 32 Mi doubles from C (VERDICT r02:
    // verify at 32 Mi doubles <= 50 us end to end)
    {
        const size_t n = size_t(32) << 20;
        double *big;
        CK(hipMalloc(&big, n * 8));
        CK(hipMemset(big, 0x3F, n * 8));
        CK(hipDeviceSynchronize());
        unsigned long long ck = 0;
        int eq = 0;
        std::vector<double> v;
        for (int pass = 0; pass < 2; ++pass) {
            v.clear();
            for (int r = 0; r < 230; ++r) {
                const double t0 = now_us();
                if (pass == 0) shmemx_checksum(SHMEMX_TYPE_DOUBLE, big, n, &ck);
                else shmemx_verify(SHMEMX_TYPE_DOUBLE, big, (int)n, 0, 0, 1, &eq);
                if (r >= 30) v.push_back(now_us() - t0);
            }
            std::sort(v.begin(), v.end());
            printf("%-14s median %7.2f us  p10 %7.2f  p90 %7.2f  (32 Mi doubles)\n",
                   pass == 0 ? "checksum_32Mi" : "verify_32Mi", v[v.size() / 2], v[v.size() / 10],
                   v[v.size() * 9 / 10]);
        }
        CK(hipFree(big));
    }
    CK(hipStreamSynchronize(st));
    shmem_finalize();
    return 0;
}
