// Experiment harness (not part of the library): cache-policy bits of the
// 2-input double fold acc[i] += in[i] over 32 Mi elements on gfx950.
// The shipped kernel uses __builtin_nontemporal_load/store (the `nt` bit) on
// every access.  gfx950 loads and stores also take `sc0` and `sc1`
// (MI355X_MICROARCH.md: sc1 stores are write-through and drop the line from
// the XCD's L2, plain/sc0/nt stores keep it).  Buffer loads/stores with an
// explicit cache-policy operand (aux: sc0 = 1, nt = 2, sc1 = 16) set each
// combination per array.  Timed with HIP events in interleaved rounds, warm
// (back to back) and cold (a 1 GiB read-only sweep before every step, so no
// dirty line is left in the Infinity Cache).
//   hipcc --offload-arch=gfx950 -O3 tools/labs/policy_lab.hip -o tools/labs/policy_lab
//   tools/labs/policy_lab [n_elems] [cold 0|1] [list 0|1]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("%s: %s\n", #x, hipGetErrorString(e));                    \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

// the shipped shape: 256 lanes, 4 vectors per lane per input, nt everywhere
template <int B, int U>
__global__ __launch_bounds__(B) void v_global_nt(f64x2 *acc, const f64x2 *in, size_t nvec) {
    const size_t base = (size_t)blockIdx.x * B * U;
    if (base + (size_t)B * U > nvec) return;
    f64x2 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(acc + base + threadIdx.x + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in + base + threadIdx.x + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u] + b[u], acc + base + threadIdx.x + u * B);
}

// buffer loads/stores, cache-policy operand per array
template <int B, int U, int LA, int LI, int S>
__global__ __launch_bounds__(B) void v_buffer(f64x2 *acc, const f64x2 *in, size_t nvec) {
    const size_t base = (size_t)blockIdx.x * B * U;
    if (base + (size_t)B * U > nvec) return;
    const int bytes = (int)(nvec * 16 > 0x7fffffff ? 0x7fffffff : nvec * 16);
    __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(acc, (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ri =
        __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, bytes, 0x00020000);
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, (int)((base + threadIdx.x + u * B) * 16), 0, LA);
#pragma unroll
    for (int u = 0; u < U; ++u)
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)((base + threadIdx.x + u * B) * 16), 0, LI);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        f64x2 x = __builtin_bit_cast(f64x2, a[u]) + __builtin_bit_cast(f64x2, b[u]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), ra,
                                               (int)((base + threadIdx.x + u * B) * 16), 0, S);
    }
}

// read-only sweep of the scratch (evicts the fold's arrays, leaves nothing dirty)
__global__ __launch_bounds__(256) void sweep(const u32x4 *p, size_t nvec, unsigned *sink) {
    unsigned x = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
        u32x4 v = __builtin_nontemporal_load(p + i);
        x ^= v.x ^ v.w;
    }
    if (x == 0x12345678u) sink[0] = x;
}

typedef void (*Launch)(f64x2 *, const f64x2 *, size_t, hipStream_t);
struct Variant {
    const char *name;
    Launch launch;
};

template <int B, int U>
void L_global(f64x2 *a, const f64x2 *b, size_t nvec, hipStream_t s) {
    v_global_nt<B, U><<<dim3((unsigned)(nvec / (B * U))), dim3(B), 0, s>>>(a, b, nvec);
}
template <int B, int U, int LA, int LI, int S>
void L_buffer(f64x2 *a, const f64x2 *b, size_t nvec, hipStream_t s) {
    v_buffer<B, U, LA, LI, S><<<dim3((unsigned)(nvec / (B * U))), dim3(B), 0, s>>>(a, b, nvec);
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : (32ull << 20);
    const int cold = argc > 2 ? atoi(argv[2]) : 0;
    const size_t nvec = n / 2;
    if (nvec % 1024) {
        printf("n must be a multiple of 2048\n");
        return 1;
    }
    f64x2 *acc, *in;
    u32x4 *scratch;
    unsigned *sink;
    CK(hipMalloc(&acc, n * 8));
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&scratch, size_t(1) << 30));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(acc, 0, n * 8));
    CK(hipMemset(in, 0, n * 8));
    CK(hipMemset(scratch, 1, size_t(1) << 30));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // aux: sc0 = 1, nt = 2, sc1 = 16
    std::vector<Variant> vs = {
        {"global_nt (shipped)", L_global<256, 4>},
        {"buf ld nt/nt st nt", L_buffer<256, 4, 2, 2, 2>},
        {"buf ld nt/nt st sc1", L_buffer<256, 4, 2, 2, 16>},
        {"buf ld nt/nt st sc0sc1", L_buffer<256, 4, 2, 2, 17>},
        {"buf ld nt/nt st sc1nt", L_buffer<256, 4, 2, 2, 18>},
        {"buf ld nt/nt st sc0nt", L_buffer<256, 4, 2, 2, 3>},
        {"buf ld sc1/sc1 st nt", L_buffer<256, 4, 16, 16, 2>},
        {"buf ld sc1nt st sc1nt", L_buffer<256, 4, 18, 18, 18>},
        {"buf ld sc0sc1nt all", L_buffer<256, 4, 19, 19, 19>},
        {"buf ld plain st sc1", L_buffer<256, 4, 0, 0, 16>},
        {"buf ld nt/nt st plain", L_buffer<256, 4, 2, 2, 0>},
        {"buf u8 nt all", L_buffer<256, 8, 2, 2, 2>},
        {"buf u8 ld nt st sc1nt", L_buffer<256, 8, 2, 2, 18>},
        {"global_nt (again)", L_global<256, 4>},
    };
    // list 1: the store's sc0 bit (round-3 follow-up), more rounds
    std::vector<Variant> focus = {
        {"global_nt (shipped)", L_global<256, 4>},
        {"buf ld nt/nt st sc0nt", L_buffer<256, 4, 2, 2, 3>},
        {"buf ld sc0nt/sc0nt st nt", L_buffer<256, 4, 3, 3, 2>},
        {"buf ld sc0nt all", L_buffer<256, 4, 3, 3, 3>},
        {"buf ld nt/nt st nt", L_buffer<256, 4, 2, 2, 2>},
        {"buf u2 ld nt st sc0nt", L_buffer<256, 2, 2, 2, 3>},
        {"global_nt (again)", L_global<256, 4>},
        {"buf ld nt/nt st sc0nt (again)", L_buffer<256, 4, 2, 2, 3>},
    };
    const int list = argc > 3 ? atoi(argv[3]) : 0;
    if (list == 1) vs = focus;
    const int K = cold ? 1 : 20, R = list == 1 ? 15 : 7;
    std::vector<std::vector<float>> t(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < R; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int w = 0; w < 2; ++w) vs[v].launch(acc, in, nvec, s);
            float tot = 0;
            const int reps = cold ? 5 : 1;
            for (int k = 0; k < reps; ++k) {
                if (cold) sweep<<<4096, 256, 0, s>>>(scratch, (size_t(1) << 30) / 16, sink);
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < K; ++i) vs[v].launch(acc, in, nvec, s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                tot += ms / K;
            }
            t[v].push_back(tot / reps);
        }
    }
    printf("n = %zu doubles, %s\n", n, cold ? "cold (1 GiB read-only sweep before each step)"
                                            : "warm (20 back to back)");
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        const float med = t[v][R / 2];
        printf("%-26s %8.2f us  %7.1f GB/s  (best %7.1f)\n", vs[v].name, med * 1e3,
               24.0 * n / (med * 1e-3) / 1e9, 24.0 * n / (t[v][0] * 1e-3) / 1e9);
    }
    return 0;
}
