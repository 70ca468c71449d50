// Experiment harness (not part of the library): variants of the 2-input
// double fold acc[i] += in[i] over 32 Mi elements on gfx950, timed with HIP
// events in interleaved rounds.  Build: hipcc --offload-arch=gfx950 -O3
// tools/labs/fold_lab.hip -o tools/labs/fold_lab ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                  \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("%s: %s\n", #x, hipGetErrorString(e));                    \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

template <int NT>
__device__ __forceinline__ f64x2 ld(const f64x2 *p) {
    if constexpr (NT & 1) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int NT>
__device__ __forceinline__ void st(f64x2 *p, f64x2 v) {
    if constexpr (NT & 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// V0: the library's shape (block B, U vectors per lane per input, strided by B)
template <int B, int U, int NT>
__global__ __launch_bounds__(B) void v_strided(f64x2 *acc, const f64x2 *in, size_t nvec) {
    const size_t base = (size_t)blockIdx.x * B * U;
    if (base + (size_t)B * U <= nvec) {
        f64x2 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld<NT>(acc + base + threadIdx.x + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld<NT>(in + base + threadIdx.x + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(acc + base + threadIdx.x + u * B, a[u] + b[u]);
    } else {
        for (int u = 0; u < U; ++u) {
            size_t v = base + threadIdx.x + u * B;
            if (v < nvec) st<NT>(acc + v, ld<NT>(acc + v) + ld<NT>(in + v));
        }
    }
}

// V6: per-array cache policy. P bit0: acc loads nt, bit1: stores nt,
// bit2: in loads nt (v_strided's NT = 1 is P = 5, NT = 3 is P = 7).
template <int B, int U, int P>
__global__ __launch_bounds__(B) void v_mixed(f64x2 *acc, const f64x2 *in, size_t nvec) {
    constexpr int LA = (P & 1) ? 1 : 0, LI = (P & 4) ? 1 : 0, S = (P & 2) ? 2 : 0;
    const size_t base = (size_t)blockIdx.x * B * U;
    if (base + (size_t)B * U <= nvec) {
        f64x2 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld<LA>(acc + base + threadIdx.x + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld<LI>(in + base + threadIdx.x + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) st<S>(acc + base + threadIdx.x + u * B, a[u] + b[u]);
    } else {
        for (int u = 0; u < U; ++u) {
            size_t v = base + threadIdx.x + u * B;
            if (v < nvec) st<S>(acc + v, ld<LA>(acc + v) + ld<LI>(in + v));
        }
    }
}
template <int B, int U, int P>
static void L_mixed(f64x2 *a, const f64x2 *b, size_t nv, hipStream_t s) {
    hipLaunchKernelGGL((v_mixed<B, U, P>), dim3((nv + B * U - 1) / (B * U)), dim3(B), 0, s, a, b, nv);
}

// V1: interleaved issue order (acc[u], in[u], acc[u+1], ...)
template <int B, int U, int NT>
__global__ __launch_bounds__(B) void v_interleave(f64x2 *acc, const f64x2 *in, size_t nvec) {
    const size_t base = (size_t)blockIdx.x * B * U;
    if (base + (size_t)B * U <= nvec) {
        f64x2 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = ld<NT>(acc + base + threadIdx.x + u * B);
            b[u] = ld<NT>(in + base + threadIdx.x + u * B);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(acc + base + threadIdx.x + u * B, a[u] + b[u]);
    } else {
        for (int u = 0; u < U; ++u) {
            size_t v = base + threadIdx.x + u * B;
            if (v < nvec) st<NT>(acc + v, ld<NT>(acc + v) + ld<NT>(in + v));
        }
    }
}

// V2: XCD-contiguous: block b runs on XCD b%8 (observed round-robin); give
// each XCD a contiguous eighth of the array.
template <int B, int U, int NT>
__global__ __launch_bounds__(B) void v_xcd(f64x2 *acc, const f64x2 *in, size_t nvec) {
    const unsigned nb = gridDim.x, b = blockIdx.x;
    const unsigned q = nb / 8, r = nb % 8, x = b % 8;
    const unsigned wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    const size_t base = (size_t)wg * B * U;
    if (base + (size_t)B * U <= nvec) {
        f64x2 a[U], bb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld<NT>(acc + base + threadIdx.x + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) bb[u] = ld<NT>(in + base + threadIdx.x + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(acc + base + threadIdx.x + u * B, a[u] + bb[u]);
    } else {
        for (int u = 0; u < U; ++u) {
            size_t v = base + threadIdx.x + u * B;
            if (v < nvec) st<NT>(acc + v, ld<NT>(acc + v) + ld<NT>(in + v));
        }
    }
}

// V3: persistent grid-stride, G blocks, loop over chunks
template <int B, int U, int NT>
__global__ __launch_bounds__(B) void v_persist(f64x2 *acc, const f64x2 *in, size_t nvec) {
    for (size_t base = (size_t)blockIdx.x * B * U; base < nvec; base += (size_t)gridDim.x * B * U) {
        if (base + (size_t)B * U <= nvec) {
            f64x2 a[U], b[U];
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = ld<NT>(acc + base + threadIdx.x + u * B);
#pragma unroll
            for (int u = 0; u < U; ++u) b[u] = ld<NT>(in + base + threadIdx.x + u * B);
#pragma unroll
            for (int u = 0; u < U; ++u) st<NT>(acc + base + threadIdx.x + u * B, a[u] + b[u]);
        } else {
            for (int u = 0; u < U; ++u) {
                size_t v = base + threadIdx.x + u * B;
                if (v < nvec) st<NT>(acc + v, ld<NT>(acc + v) + ld<NT>(in + v));
            }
        }
    }
}

// V4: persistent and software-pipelined: chunk k+1's loads are issued before
// chunk k's stores, so every wave writes one chunk while reading the next
// (the in-place fold otherwise reads and writes the same lines back to back).
// The lab arrays are a whole number of chunks per block (32 Mi doubles).
template <int B, int U, int NT>
__global__ __launch_bounds__(B) void v_pipe(f64x2 *acc, const f64x2 *in, size_t nvec) {
    const size_t step = (size_t)gridDim.x * B * U;
    size_t base = (size_t)blockIdx.x * B * U;
    if (base + (size_t)B * U > nvec) return;
    f64x2 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld<NT>(acc + base + threadIdx.x + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = ld<NT>(in + base + threadIdx.x + u * B);
    for (;;) {
        const bool more = base + step + (size_t)B * U <= nvec;
        const size_t nb = more ? base + step : base;     // unconditional loads: counted waits
        f64x2 a2[U], b2[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a2[u] = ld<NT>(acc + nb + threadIdx.x + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) b2[u] = ld<NT>(in + nb + threadIdx.x + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(acc + base + threadIdx.x + u * B, a[u] + b[u]);
        if (!more) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = a2[u];
            b[u] = b2[u];
        }
        base = nb;
    }
}

struct Variant {
    const char *name;
    void (*launch)(f64x2 *, const f64x2 *, size_t, hipStream_t);
};

template <int B, int U, int NT>
void L_strided(f64x2 *a, const f64x2 *b, size_t nv, hipStream_t s) {
    hipLaunchKernelGGL((v_strided<B, U, NT>), dim3((nv + B * U - 1) / (B * U)), dim3(B), 0, s, a, b, nv);
}
template <int B, int U, int NT>
void L_inter(f64x2 *a, const f64x2 *b, size_t nv, hipStream_t s) {
    hipLaunchKernelGGL((v_interleave<B, U, NT>), dim3((nv + B * U - 1) / (B * U)), dim3(B), 0, s, a, b, nv);
}
template <int B, int U, int NT>
void L_xcd(f64x2 *a, const f64x2 *b, size_t nv, hipStream_t s) {
    hipLaunchKernelGGL((v_xcd<B, U, NT>), dim3((nv + B * U - 1) / (B * U)), dim3(B), 0, s, a, b, nv);
}
template <int B, int U, int NT, int G>
void L_persist(f64x2 *a, const f64x2 *b, size_t nv, hipStream_t s) {
    hipLaunchKernelGGL((v_persist<B, U, NT>), dim3(G), dim3(B), 0, s, a, b, nv);
}

template <int B, int U, int NT, int G>
void L_pipe(f64x2 *a, const f64x2 *b, size_t nv, hipStream_t s) {
    hipLaunchKernelGGL((v_pipe<B, U, NT>), dim3(G), dim3(B), 0, s, a, b, nv);
}

// Mode "offsets": does the distance between acc and in matter (channel /
// bank camping)?  One 1 GiB arena; acc at 0, in at 256 MiB + delta.
static int offsets_mode(size_t n) {
    const size_t nvec = n / 2;
    char *arena;
    CK(hipMalloc(&arena, size_t(1) << 30));
    CK(hipMemset(arena, 0, size_t(1) << 30));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t deltas[] = {0, 256, 4096, 65536, 1 << 20, 2 << 20, 4 << 20, 8 << 20,
                             16 << 20, 32 << 20, 64 << 20, (size_t)3 << 20, 12345 * 16};
    for (size_t d : deltas) {
        f64x2 *acc = reinterpret_cast<f64x2 *>(arena);
        const f64x2 *in = reinterpret_cast<const f64x2 *>(arena + (size_t(256) << 20) + d);
        std::vector<float> ts;
        for (int r = 0; r < 7; ++r) {
            for (int w = 0; w < 2; ++w) L_strided<256, 4, 3>(acc, in, nvec, s);
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < 20; ++i) L_strided<256, 4, 3>(acc, in, nvec, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms / 20);
        }
        std::sort(ts.begin(), ts.end());
        printf("delta %10zu  %8.2f us  %7.1f GB/s\n", d, ts[3] * 1e3, 24.0 * n / (ts[3] * 1e-3) / 1e9);
    }
    return 0;
}

// Mode "pairs": separately allocated (acc, in) pairs in one process, and
// pairs carved from one arena: is the rate a property of the allocation?
static int pairs_mode(size_t n) {
    const size_t nvec = n / 2, bytes = n * 8;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_pair = [&](f64x2 *acc, const f64x2 *in) {
        std::vector<float> ts;
        for (int r = 0; r < 5; ++r) {
            for (int w = 0; w < 2; ++w) L_strided<256, 4, 3>(acc, in, nvec, s);
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < 20; ++i) L_strided<256, 4, 3>(acc, in, nvec, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms / 20);
        }
        std::sort(ts.begin(), ts.end());
        return ts[2] * 1e3f;
    };
    std::vector<void *> ptrs;
    for (int p = 0; p < 6; ++p) {
        void *a, *b;
        CK(hipMalloc(&a, bytes));
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(a, 0, bytes));
        CK(hipMemset(b, 0, bytes));
        ptrs.push_back(a);
        ptrs.push_back(b);
        printf("separate pair %d  acc %p in %p  %8.2f us\n", p, a, b,
               time_pair((f64x2 *)a, (const f64x2 *)b));
    }
    // cross pairs: acc of pair i with in of pair j
    for (int p = 0; p < 6; ++p)
        printf("cross acc%d in%d  %8.2f us\n", p, (p + 1) % 6,
               time_pair((f64x2 *)ptrs[2 * p], (const f64x2 *)ptrs[2 * ((p + 1) % 6) + 1]));
    for (void *q : ptrs) CK(hipFree(q));
    // pairs carved from one 4 GiB arena at assorted offsets
    char *arena;
    CK(hipMalloc(&arena, size_t(4) << 30));
    CK(hipMemset(arena, 0, size_t(4) << 30));
    const size_t offs[][2] = {{0, 256ull << 20}, {512ull << 20, 1024ull << 20},
                              {(3ull << 30), (1ull << 30) + (6ull << 20)},
                              {(2ull << 30) + 4096, (600ull << 20)},
                              {(1536ull << 20), (3ull << 30) + (512ull << 20)},
                              {(2560ull << 20) + 65536, (100ull << 20)}};
    for (auto &o : offs)
        printf("arena acc+%zu MiB in+%zu MiB  %8.2f us\n", o[0] >> 20, o[1] >> 20,
               time_pair((f64x2 *)(arena + o[0]), (const f64x2 *)(arena + o[1])));
    return 0;
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : (32ull << 20);
    int cold = argc > 2 ? atoi(argv[2]) : 0;
    if (cold == 2) return offsets_mode(n);
    if (cold == 3) return pairs_mode(n);
    const size_t nvec = n / 2;
    f64x2 *acc, *in;
    double *scratch;
    CK(hipMalloc(&acc, n * 8));
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&scratch, size_t(1) << 30));
    CK(hipMemset(acc, 0, n * 8));
    CK(hipMemset(in, 0, n * 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<Variant> mixed = {
        {"mixed_p7_ldA_ldI_st_nt", L_mixed<256, 4, 7>},
        {"mixed_p6_ldI_st_nt", L_mixed<256, 4, 6>},
        {"mixed_p3_ldA_st_nt", L_mixed<256, 4, 3>},
        {"mixed_p5_ldA_ldI_nt", L_mixed<256, 4, 5>},
        {"mixed_p4_ldI_nt", L_mixed<256, 4, 4>},
        {"mixed_p1_ldA_nt", L_mixed<256, 4, 1>},
        {"mixed_p2_st_nt", L_mixed<256, 4, 2>},
        {"mixed_p7_again", L_mixed<256, 4, 7>},
    };
    std::vector<Variant> vs = {
        {"strided_b256_u4_nt3", L_strided<256, 4, 3>},
        {"strided_b256_u2_nt3", L_strided<256, 2, 3>},
        {"strided_b512_u4_nt3", L_strided<512, 4, 3>},
        {"strided_b512_u2_nt3", L_strided<512, 2, 3>},
        {"strided_b1024_u2_nt3", L_strided<1024, 2, 3>},
        {"strided_b1024_u1_nt3", L_strided<1024, 1, 3>},
        {"strided_b128_u8_nt3", L_strided<128, 8, 3>},
        {"inter_b256_u4_nt3", L_inter<256, 4, 3>},
        {"inter_b512_u2_nt3", L_inter<512, 2, 3>},
        {"xcd_b256_u4_nt3", L_xcd<256, 4, 3>},
        {"xcd_b512_u4_nt3", L_xcd<512, 4, 3>},
        {"persist_b256_u4_nt3_g2048", L_persist<256, 4, 3, 2048>},
        {"persist_b512_u4_nt3_g1024", L_persist<512, 4, 3, 1024>},
        {"persist_b1024_u2_nt3_g512", L_persist<1024, 2, 3, 512>},
        {"strided_b256_u4_nt1", L_strided<256, 4, 1>},
        {"strided_b256_u4_nt2", L_strided<256, 4, 2>},
        {"pipe_b256_u4_nt3_g1024", L_pipe<256, 4, 3, 1024>},
        {"pipe_b256_u4_nt3_g2048", L_pipe<256, 4, 3, 2048>},
        {"pipe_b256_u4_nt3_g4096", L_pipe<256, 4, 3, 4096>},
        {"pipe_b256_u2_nt3_g2048", L_pipe<256, 2, 3, 2048>},
        {"pipe_b256_u2_nt3_g4096", L_pipe<256, 2, 3, 4096>},
        {"pipe_b512_u2_nt3_g2048", L_pipe<512, 2, 3, 2048>},
        {"pipe_b256_u4_nt1_g2048", L_pipe<256, 4, 1, 2048>},
        {"pipe_b256_u2_nt3_g8192", L_pipe<256, 2, 3, 8192>},
        {"strided_b256_u4_nt3_again", L_strided<256, 4, 3>},
    };
    if (cold >= 4) {  // modes 4 (warm) and 5 (cold): the per-array policies
        vs = mixed;
        cold -= 4;
    }
    const int K = cold ? 1 : 20, R = 7;
    std::vector<std::vector<float>> t(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < R; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int w = 0; w < 2; ++w) vs[v].launch(acc, in, nvec, s);
            float tot = 0;
            for (int k = 0; k < (cold ? 5 : 1); ++k) {
                if (cold) CK(hipMemsetAsync(scratch, r + k, size_t(1) << 30, s));
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < K; ++i) vs[v].launch(acc, in, nvec, s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                tot += ms / K;
            }
            t[v].push_back(tot / (cold ? 5 : 1));
        }
    }
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        const float med = t[v][R / 2];
        printf("%-28s %8.2f us  %7.1f GB/s  (best %7.1f)\n", vs[v].name, med * 1e3,
               24.0 * n / (med * 1e-3) / 1e9, 24.0 * n / (t[v][0] * 1e-3) / 1e9);
    }
    return 0;
}
