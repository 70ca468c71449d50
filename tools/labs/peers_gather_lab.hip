// Experiment harness (not part of the library), VERDICT r02 next-step 5:
// the two kernels below 80 % of HBM peak on local HBM.
//
//   peers<U, NB>   fold_peers_kernel's shape at MAXIN = 8: every lane issues
//                  U 16-B vectors of ALL 8 inputs before folding any (the
//                  shipped kernel: U = 2, 256-lane blocks); U = 4 keeps 32
//                  vectors in registers (launch bounds let the compiler use
//                  up to 256 VGPRs); U = 1 keeps 8.
//   rt<U>          the runtime-nins loop (input k + 1's loads after input k
//                  is folded), the local-HBM reference.
//   gather<U, IL>  gather_kernel's shape: 7 segments, IL = 1 interleaves the
//                  segments across consecutive blocks (shipped, every
//                  peer's link busy at once), IL = 0 takes the segment from
//                  blockIdx.y; U vectors per lane per step.
//   copy<U>        one contiguous copy of the same bytes (the ceiling).
// All loads and stores non-temporal, 16-B vectors; n a multiple of every
// chunk size.  Timed with HIP events, interleaved rounds, warm (back to back)
// and cold (a 1 GiB read-only sweep before every launch: evicts, leaves
// nothing dirty).
//   Build: hipcc --offload-arch=gfx950 -O3 tools/labs/peers_gather_lab.hip -o tools/labs/peers_gather_lab
//   Run:   tools/labs/peers_gather_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));

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

__device__ __forceinline__ f64x2 ld(const f64x2 *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(f64x2 *p, f64x2 v) { __builtin_nontemporal_store(v, p); }

template <int U, int NB>
__global__ __launch_bounds__(NB, 1) void peers(f64x2 *out, Ins in, int nins) {
    const size_t v0 = (size_t)blockIdx.x * NB * U + threadIdx.x;
    f64x2 x[P][U];
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (k < nins)
#pragma unroll
            for (int u = 0; u < U; ++u) x[k][u] = ld(in.p[k] + v0 + u * NB);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        f64x2 acc = x[0][u];
#pragma unroll
        for (int k = 1; k < P; ++k)
            if (k < nins) acc += x[k][u];
        st(out + v0 + u * NB, acc);
    }
}

template <int U>
__global__ __launch_bounds__(256) void rt(f64x2 *out, Ins in, int nins) {
    const size_t v0 = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f64x2 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = ld(in.p[0] + v0 + u * 256);
    for (int k = 1; k < nins; ++k) {
        f64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld(in.p[k] + v0 + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += x[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + v0 + u * 256, acc[u]);
}

struct Segs {
    const f64x2 *src[P];
    f64x2 *dst[P];
};

// nvec vectors per segment, one chunk of 256 * U vectors per block.  IL = 0:
// segment from blockIdx.y; IL = 1: consecutive blocks take the segments in
// turn; IL = R > 1: runs of R consecutive blocks per segment, in turn (every
// segment still has blocks resident at once while R * nseg stays under the
// resident grid, ~2048 blocks).
template <int U, int IL>
__global__ __launch_bounds__(256) void gather(Segs s, int nseg, size_t nvec) {
    int seg;
    size_t bx;
    if (IL == 0) {
        seg = blockIdx.y;
        bx = blockIdx.x;
    } else {
        const size_t run = blockIdx.x / IL, in_run = blockIdx.x % IL;
        seg = run % nseg;
        bx = (run / nseg) * IL + in_run;
    }
    const size_t v0 = bx * 256 * U + threadIdx.x;
    if (v0 >= nvec) return;
    f64x2 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld(s.src[seg] + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) st(s.dst[seg] + v0 + u * 256, x[u]);
}

template <int U>
__global__ __launch_bounds__(256) void copy(f64x2 *dst, const f64x2 *src) {
    const size_t v0 = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f64x2 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld(src + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) st(dst + v0 + u * 256, x[u]);
}

__global__ void sweep(const f64x2 *p, size_t n, double *sink) {
    f64x2 a = {0, 0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a += ld(p + i);
    if (a[0] == 12345.678) *sink = a[1];   // never true: keeps the loads
}

struct Variant {
    const char *name;
    double bytes;
    void (*launch)(hipStream_t);
};

static f64x2 *g_out, *g_ins[P], *g_gsrc, *g_gdst, *g_scratch;
static double *g_sink;
static size_t g_n;   // vectors per fold input
static size_t g_seg; // vectors per gather segment

template <int U, int NB>
void L_peers(hipStream_t s) {
    Ins in;
    for (int k = 0; k < P; ++k) in.p[k] = g_ins[k];
    hipLaunchKernelGGL((peers<U, NB>), dim3(g_n / (NB * U)), dim3(NB), 0, s, g_out, in, P);
}
template <int U>
void L_rt(hipStream_t s) {
    Ins in;
    for (int k = 0; k < P; ++k) in.p[k] = g_ins[k];
    hipLaunchKernelGGL((rt<U>), dim3(g_n / (256 * U)), dim3(256), 0, s, g_out, in, P);
}
template <int U, int IL>
void L_gather(hipStream_t s) {
    Segs sg;
    for (int k = 0; k < 7; ++k) {
        sg.src[k] = g_gsrc + (k + 1) * g_seg;
        sg.dst[k] = g_gdst + (k + 1) * g_seg;
    }
    const unsigned bx = (unsigned)(g_seg / (256 * U));
    if (IL)
        hipLaunchKernelGGL((gather<U, IL>), dim3(bx * 7), dim3(256), 0, s, sg, 7, g_seg);
    else
        hipLaunchKernelGGL((gather<U, 0>), dim3(bx, 7), dim3(256), 0, s, sg, 7, g_seg);
}
template <int U>
void L_copy(hipStream_t s) {
    hipLaunchKernelGGL((copy<U>), dim3(7 * g_seg / (256 * U)), dim3(256), 0, s, g_gdst + g_seg,
                       g_gsrc + g_seg);
}

int main() {
    g_n = (size_t(16) << 20) / 2;     // 16 Mi doubles per fold input
    g_seg = (size_t(4) << 20) / 2;    // 4 Mi doubles per gather segment (P = 8 at 32 Mi)
    const size_t scratch_vec = (size_t(1) << 30) / 16;
    CK(hipMalloc(&g_out, g_n * 16));
    for (int k = 0; k < P; ++k) {
        CK(hipMalloc(&g_ins[k], g_n * 16));
        CK(hipMemset(g_ins[k], 0, g_n * 16));
    }
    CK(hipMalloc(&g_gsrc, 8 * g_seg * 16));
    CK(hipMalloc(&g_gdst, 8 * g_seg * 16));
    CK(hipMemset(g_gsrc, 0, 8 * g_seg * 16));
    CK(hipMalloc(&g_scratch, scratch_vec * 16));
    CK(hipMemset(g_scratch, 0, scratch_vec * 16));
    CK(hipMalloc(&g_sink, 8));
    const double fold_bytes = 9.0 * g_n * 16, gather_bytes = 14.0 * g_seg * 16;
    std::vector<Variant> vs = {
        {"peers_u2_b256 (shipped)", fold_bytes, L_peers<2, 256>},
        {"peers_u4_b256", fold_bytes, L_peers<4, 256>},
        {"peers_u1_b256", fold_bytes, L_peers<1, 256>},
        {"peers_u2_b512", fold_bytes, L_peers<2, 512>},
        {"peers_u1_b512", fold_bytes, L_peers<1, 512>},
        {"rt_u4 (runtime loop)", fold_bytes, L_rt<4>},
        {"gather_u4_il (round 2)", gather_bytes, L_gather<4, 1>},
        {"gather_u8_il", gather_bytes, L_gather<8, 1>},
        {"gather_u2_il (round 3)", gather_bytes, L_gather<2, 1>},
        {"gather_u4_y", gather_bytes, L_gather<4, 0>},
        {"gather_u8_y", gather_bytes, L_gather<8, 0>},
        {"gather_u8_run32", gather_bytes, L_gather<8, 32>},
        {"gather_u8_run64", gather_bytes, L_gather<8, 64>},
        {"gather_u8_run128", gather_bytes, L_gather<8, 128>},
        {"gather_u8_run256", gather_bytes, L_gather<8, 256>},
        {"gather_u4_run128", gather_bytes, L_gather<4, 128>},
        {"gather_u4_run256", gather_bytes, L_gather<4, 256>},
        {"gather_u2_run256", gather_bytes, L_gather<2, 256>},
        {"copy_u4 (same bytes, contiguous)", gather_bytes, L_copy<4>},
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = 5, reps = 10;
    std::vector<std::vector<float>> warm(vs.size()), cold(vs.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            vs[i].launch(s);   // warm-up
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
    printf("# peers / gather lab: fold P = 8 x 16 Mi doubles (1.13 GiB per launch), gather 7 x 32 MiB "
           "(448 MiB); median us, TB/s\n");
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(warm[i].begin(), warm[i].end());
        std::sort(cold[i].begin(), cold[i].end());
        const double w = warm[i][warm[i].size() / 2] * 1e-3, c = cold[i][cold[i].size() / 2] * 1e-3;
        printf("%-36s warm %8.1f us %6.2f TB/s   cold %8.1f us %6.2f TB/s\n", vs[i].name, w * 1e6,
               vs[i].bytes / w / 1e12, c * 1e6, vs[i].bytes / c / 1e12);
    }
    return 0;
}
