// Experiment harness (not part of the library): loop shapes of the checksum
// kernel (openshmem-async_amd/csrc/checksum.hip) over 32 Mi doubles, timed
// with HIP events, every variant checked against the shipped one.
//   one      the shipped shape: one 16-B load per lane per iteration
//   pipe     the next iteration's load issued before this one is mixed
//   pipe2    two iterations ahead
//   unroll4  four independent loads per lane, then the mixing
//   Build: hipcc --offload-arch=gfx950 -O3 tools/labs/checksum_lab.hip -o tools/labs/checksum_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("%s: %s\n", #x, hipGetErrorString(e));                    \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t kPhi = 0x9E3779B97F4A7C15ull;
constexpr int B = 256;

__device__ __forceinline__ uint64_t fmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t pair(u32x4 x, uint64_t c) {
    return fmix((((uint64_t)x[1] << 32) | x[0]) + c) ^ fmix((((uint64_t)x[3] << 32) | x[2]) + c + kPhi);
}
__device__ __forceinline__ void finish(uint64_t h, unsigned long long *out) {
    // (lab: a plain atomic per wave is enough to keep the work alive)
    for (int o = 32; o > 0; o >>= 1) {
        h ^= (uint64_t)__shfl_xor((long long)h, o);
    }
    if ((threadIdx.x & 63) == 0) atomicXor(out, (unsigned long long)h);
}

template <int V>
__global__ __launch_bounds__(B) void ck(const u32x4 *v, size_t npairs, unsigned long long *out) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x, nthr = (size_t)gridDim.x * B;
    uint64_t h = 0, c = (2 * (uint64_t)tid + 1) * kPhi;
    const uint64_t dc = 2 * (uint64_t)nthr * kPhi;
    if constexpr (V == 0) {
        for (size_t i = tid; i < npairs; i += nthr, c += dc) h ^= pair(__builtin_nontemporal_load(v + i), c);
    } else if constexpr (V == 1 || V == 2) {
        // prefetch V iterations ahead (clamped index: no branch on the load)
        u32x4 q[V];
#pragma unroll
        for (int k = 0; k < V; ++k)
            q[k] = __builtin_nontemporal_load(v + std::min(tid + k * nthr, npairs - 1));
        for (size_t i = tid; i < npairs; i += nthr, c += dc) {
            const u32x4 cur = q[0];
#pragma unroll
            for (int k = 0; k + 1 < V; ++k) q[k] = q[k + 1];
            q[V - 1] = __builtin_nontemporal_load(v + std::min(i + V * nthr, npairs - 1));
            h ^= pair(cur, c);
        }
    } else {
        size_t i = tid;
        for (; i + 3 * nthr < npairs; i += 4 * nthr, c += 4 * dc) {
            u32x4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = __builtin_nontemporal_load(v + i + u * nthr);
#pragma unroll
            for (int u = 0; u < 4; ++u) h ^= pair(x[u], c + u * dc);
        }
        for (; i < npairs; i += nthr, c += dc) h ^= pair(__builtin_nontemporal_load(v + i), c);
    }
    finish(h, out);
}

int main() {
    const size_t n = size_t(32) << 20, npairs = n / 2;
    double *d = nullptr;
    unsigned long long *out = nullptr;
    CK(hipMalloc(&d, n * 8));
    CK(hipMalloc(&out, 8));
    std::vector<double> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (double)(i * 2654435761u % 1000003) / 7.0;
    CK(hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice));
    typedef void (*K)(const u32x4 *, size_t, unsigned long long *);
    struct Var { const char *name; K k; };
    const Var vars[] = {{"one", ck<0>}, {"pipe", ck<1>}, {"pipe2", ck<2>}, {"unroll4", ck<4>}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    unsigned long long want = 0;
    for (int grid : {2048, 4096, 8192, 16384}) {
        for (const Var &v : vars) {
            std::vector<float> t;
            unsigned long long got = 0;
            for (int r = 0; r < 12; ++r) {
                CK(hipMemset(out, 0, 8));
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(v.k, dim3(grid), dim3(B), 0, 0, reinterpret_cast<const u32x4 *>(d), npairs, out);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) t.push_back(ms);
                CK(hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost));
            }
            if (!want) want = got;
            std::sort(t.begin(), t.end());
            const double us = t[t.size() / 2] * 1e3;
            printf("grid %5d %-8s %7.1f us %6.2f TB/s %s\n", grid, v.name, us, n * 8 / us / 1e6,
                   got == want ? "" : "MISMATCH");
        }
    }
    return 0;
}
