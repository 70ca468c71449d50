// Experiment harness (not part of the library), round 3: the P = 8 input fold
// over separate arrays (fold_peers_kernel's job, 8 x 16 Mi doubles, 1.13 GiB
// per launch) with buffer loads instead of global loads.  Each block builds
// one buffer descriptor per input at its own chunk (scalar registers) and all
// inputs share one 32-bit lane offset, so the per-input 64-bit address
// arithmetic and its VGPRs go away; the cache-policy operand (sc0 = 1, nt = 2,
// sc1 = 16) is set per variant.  Timed warm (back to back) and cold (a 1 GiB
// read-only sweep before every launch), interleaved rounds.
//   hipcc --offload-arch=gfx950 -O3 tools/labs/peers_buf_lab.hip -o tools/labs/peers_buf_lab
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

constexpr int P = 8;
struct Ins {
    const f64x2 *p[P];
};

// the shipped shape (round 3): every lane issues U vectors of all 8 inputs
template <int U, int NB>
__global__ __launch_bounds__(NB, 1) void peers(f64x2 *out, Ins in) {
    const size_t v0 = (size_t)blockIdx.x * NB * U + threadIdx.x;
    f64x2 x[P][U];
#pragma unroll
    for (int k = 0; k < P; ++k)
#pragma unroll
        for (int u = 0; u < U; ++u) x[k][u] = __builtin_nontemporal_load(in.p[k] + v0 + u * NB);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        f64x2 acc = x[0][u];
#pragma unroll
        for (int k = 1; k < P; ++k) acc += x[k][u];
        __builtin_nontemporal_store(acc, out + v0 + u * NB);
    }
}

// buffer loads: descriptor per input at this block's chunk, shared offset
template <int U, int NB, int LP, int SP>
__global__ __launch_bounds__(NB, 1) void peers_buf(f64x2 *out, Ins in) {
    const size_t chunk = (size_t)blockIdx.x * NB * U;
    constexpr int bytes = NB * U * 16;
    __amdgpu_buffer_rsrc_t r[P];
#pragma unroll
    for (int k = 0; k < P; ++k)
        r[k] = __builtin_amdgcn_make_buffer_rsrc((void *)(in.p[k] + chunk), (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out + chunk, (short)0, bytes, 0x00020000);
    const int off = threadIdx.x * 16;
    u32x4 x[P][U];
#pragma unroll
    for (int k = 0; k < P; ++k)
#pragma unroll
        for (int u = 0; u < U; ++u) x[k][u] = __builtin_amdgcn_raw_buffer_load_b128(r[k], off + u * NB * 16, 0, LP);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        f64x2 acc = __builtin_bit_cast(f64x2, x[0][u]);
#pragma unroll
        for (int k = 1; k < P; ++k) acc += __builtin_bit_cast(f64x2, x[k][u]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), ro, off + u * NB * 16, 0, SP);
    }
}

// the runtime-nins loop (input k + 1's loads after input k is folded)
template <int U>
__global__ __launch_bounds__(256) void rt(f64x2 *out, Ins in) {
    const size_t v0 = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f64x2 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * 256);
    for (int k = 1; k < P; ++k) {
        f64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(in.p[k] + v0 + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += x[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(acc[u], out + v0 + u * 256);
}

__global__ void sweep(const f64x2 *p, size_t n, double *sink) {
    f64x2 a = {0, 0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a += __builtin_nontemporal_load(p + i);
    if (a[0] == 12345.678) *sink = a[1];
}

static f64x2 *g_out, *g_ins[P], *g_scratch;
static double *g_sink;
static size_t g_n;

static Ins ins() {
    Ins in;
    for (int k = 0; k < P; ++k) in.p[k] = g_ins[k];
    return in;
}
template <int U, int NB>
void L_peers(hipStream_t s) {
    hipLaunchKernelGGL((peers<U, NB>), dim3(g_n / (NB * U)), dim3(NB), 0, s, g_out, ins());
}
template <int U, int NB, int LP, int SP>
void L_buf(hipStream_t s) {
    hipLaunchKernelGGL((peers_buf<U, NB, LP, SP>), dim3(g_n / (NB * U)), dim3(NB), 0, s, g_out, ins());
}
template <int U>
void L_rt(hipStream_t s) {
    hipLaunchKernelGGL((rt<U>), dim3(g_n / (256 * U)), dim3(256), 0, s, g_out, ins());
}

struct Variant {
    const char *name;
    void (*launch)(hipStream_t);
};

int main(int argc, char **argv) {
    const size_t elems = argc > 1 ? strtoull(argv[1], 0, 10) : (size_t(16) << 20);
    g_n = elems / 2;
    if (g_n % 4096) {
        printf("elements must be a multiple of 8192\n");
        return 1;
    }
    const size_t scratch_vec = (size_t(1) << 30) / 16;
    CK(hipMalloc(&g_out, g_n * 16));
    for (int k = 0; k < P; ++k) {
        CK(hipMalloc(&g_ins[k], g_n * 16));
        CK(hipMemset(g_ins[k], 0, g_n * 16));
    }
    CK(hipMalloc(&g_scratch, scratch_vec * 16));
    CK(hipMemset(g_scratch, 0, scratch_vec * 16));
    CK(hipMalloc(&g_sink, 8));
    const double bytes = 9.0 * g_n * 16;
    std::vector<Variant> vs = {
        {"peers_u4_b256 global (shipped)", L_peers<4, 256>},
        {"buf_u4_b256 nt", L_buf<4, 256, 2, 2>},
        {"buf_u2_b256 nt", L_buf<2, 256, 2, 2>},
        {"buf_u2_b512 nt", L_buf<2, 512, 2, 2>},
        {"buf_u4_b256 ld sc0nt", L_buf<4, 256, 3, 2>},
        {"buf_u4_b256 ld plain", L_buf<4, 256, 0, 2>},
        {"buf_u1_b1024 nt", L_buf<1, 1024, 2, 2>},
        {"rt_u4 global (runtime loop)", L_rt<4>},
        {"peers_u4_b256 global (again)", L_peers<4, 256>},
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = 7, reps = 10;
    std::vector<std::vector<float>> warm(vs.size()), cold(vs.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            vs[i].launch(s);
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k) vs[i].launch(s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            warm[i].push_back(ms / reps);
            for (int k = 0; k < 3; ++k) {
                hipLaunchKernelGGL(sweep, dim3(4096), dim3(256), 0, s, g_scratch, scratch_vec, g_sink);
                CK(hipEventRecord(e0, s));
                vs[i].launch(s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                cold[i].push_back(ms);
            }
        }
    }
    CK(hipGetLastError());
    printf("# P = 8 fold over separate arrays, %zu doubles per input (%.2f GiB per launch); median us, TB/s\n",
           elems, bytes / (1 << 30));
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(warm[i].begin(), warm[i].end());
        std::sort(cold[i].begin(), cold[i].end());
        const double w = warm[i][warm[i].size() / 2] * 1e-3, c = cold[i][cold[i].size() / 2] * 1e-3;
        printf("%-34s warm %8.1f us %6.2f TB/s   cold %8.1f us %6.2f TB/s\n", vs[i].name, w * 1e6,
               bytes / w / 1e12, c * 1e6, bytes / c / 1e12);
    }
    return 0;
}
