// Experiment harness (not part of the library), round 3: is the checksum
// kernel's streaming loop bound by HBM or by its per-word mixing?  Same loop
// shape as csrc/checksum.hip (16-B nt loads, grid-stride, one partial per
// block stored to its own slot, no atomics), three mixes per 8-byte word:
//   fmix   splitmix64 finalise of (w + (j+1)*phi): the shipped checksum
//          (two 64-bit multiplies per word)
//   mum    one 32x32->64 multiply of the word's halves, each offset by
//          position constants (one v_mad_u64_u32 per word)
//   none   plain XOR of the words (the memory-only floor)
// 32 Mi doubles (256 MiB), grids 1024/2048/4096, median of 15 launches.
//   hipcc --offload-arch=gfx950 -O3 tools/labs/checksum_mix_lab.hip -o tools/labs/checksum_mix_lab
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

template <int M>
__device__ __forceinline__ uint64_t mix(uint64_t w, uint64_t c) {
    if constexpr (M == 0) return fmix(w + c);
    if constexpr (M == 1) {
        const uint64_t x = w + c;
        return (uint64_t)((uint32_t)x ^ 0x2545F491u) * (uint64_t)((uint32_t)(x >> 32) ^ 0x9E3779B9u) ^ x;
    }
    return w;
}

template <int M>
__global__ __launch_bounds__(B) void ck(const u32x4 *v, size_t npairs, unsigned long long *part) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x, nthr = (size_t)gridDim.x * B;
    uint64_t h = 0, c = (2 * (uint64_t)tid + 1) * kPhi;
    const uint64_t dc = 2 * (uint64_t)nthr * kPhi;
    for (size_t i = tid; i < npairs; i += nthr, c += dc) {
        const u32x4 x = __builtin_nontemporal_load(v + i);
        h ^= mix<M>(((uint64_t)x[1] << 32) | x[0], c) ^ mix<M>(((uint64_t)x[3] << 32) | x[2], c + kPhi);
    }
    __shared__ unsigned long long s[B / 64];
    for (int o = 32; o > 0; o >>= 1) h ^= (uint64_t)__shfl_xor((long long)h, o);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

int main() {
    const size_t n = size_t(32) << 20, npairs = n / 2;
    double *d = nullptr;
    unsigned long long *part = nullptr;
    CK(hipMalloc(&d, n * 8));
    CK(hipMalloc(&part, 8 * 4096));
    CK(hipMemset(d, 0x3c, n * 8));
    typedef void (*K)(const u32x4 *, size_t, unsigned long long *);
    struct Var {
        const char *name;
        K k;
    };
    const Var vars[] = {{"fmix", ck<0>}, {"mum", ck<1>}, {"none", ck<2>}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int grid : {1024, 2048, 4096}) {
        for (const Var &v : vars) {
            std::vector<float> t;
            for (int r = 0; r < 17; ++r) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(v.k, dim3(grid), dim3(B), 0, 0, reinterpret_cast<const u32x4 *>(d), npairs, part);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            const double us = t[t.size() / 2] * 1e3;
            printf("grid %5d %-5s %7.1f us %6.2f TB/s\n", grid, v.name, us, n * 8 / us / 1e6);
        }
    }
    return 0;
}
