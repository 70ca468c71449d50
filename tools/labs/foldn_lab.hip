// Experiment harness (not part of the library): shapes of the P-input fold
//     out[i] = in0[i] + in1[i] + ... + in_{P-1}[i]      (double, left fold)
// the fold step of A2A / DIRECT / SIGNAL (reduce-op.c:219-248 as one pass).
// Variants, all 256-lane blocks, 16-B vectors, nt loads + nt stores:
//   rt<U>       the library's round-1 runtime-nins loop: input k+1's loads
//               issue only after input k is folded
//   pipe<U>     runtime nins, double-buffered: input k+1's loads issue before
//               input k is folded
//   st<P,U>     nins fixed at compile time: every input's loads issued first
//   pred<U>     up to 8 inputs, loads under uniform (scalar) predicates, so
//               they all issue up front for any nins <= 8 (round 2: 3.2-5.6
//               TB/s, dropped from the list)
//   rdonly<U>   rt's loads only (reads ceiling for P streams; rdonly's
//               GB/s counts the P input streams plus the never-written output)
// Timed with HIP events, interleaved rounds, warm (back to back) and cold
// (a 1 GiB scratch rewritten before every launch).
//   Build: hipcc --offload-arch=gfx950 -O3 tools/labs/foldn_lab.hip -o tools/labs/foldn_lab
//   Run:   tools/labs/foldn_lab <n per input> <cold 0|1> [skew bytes, -1 = separate]
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

constexpr int B = 256;
constexpr int MAXP = 8;
struct Ins {
    const f64x2 *p[MAXP];
};

__device__ __forceinline__ f64x2 ld(const f64x2 *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(f64x2 *p, f64x2 v) { __builtin_nontemporal_store(v, p); }

// Every variant handles whole chunks only (n is a multiple of B*U*2 here).
template <int U>
__global__ __launch_bounds__(B) void rt(f64x2 *out, Ins in, int P) {
    const size_t v0 = (size_t)blockIdx.x * B * U + threadIdx.x;
    f64x2 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = ld(in.p[0] + v0 + u * B);
    for (int k = 1; k < P; ++k) {
        f64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld(in.p[k] + v0 + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += x[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + v0 + u * B, acc[u]);
}

template <int U>
__global__ __launch_bounds__(B) void pipe(f64x2 *out, Ins in, int P) {
    const size_t v0 = (size_t)blockIdx.x * B * U + threadIdx.x;
    f64x2 acc[U], cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = ld(in.p[0] + v0 + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = ld(in.p[1] + v0 + u * B);
    for (int k = 2; k < P; ++k) {
        f64x2 nxt[U];
#pragma unroll
        for (int u = 0; u < U; ++u) nxt[u] = ld(in.p[k] + v0 + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc[u] += cur[u];
            cur[u] = nxt[u];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + v0 + u * B, acc[u] + cur[u]);
}

template <int P, int U>
__global__ __launch_bounds__(B) void stat(f64x2 *out, Ins in, int) {
    const size_t v0 = (size_t)blockIdx.x * B * U + threadIdx.x;
    f64x2 x[P][U];
#pragma unroll
    for (int k = 0; k < P; ++k)
#pragma unroll
        for (int u = 0; u < U; ++u) x[k][u] = ld(in.p[k] + v0 + u * B);
#pragma unroll
    for (int k = 1; k < P; ++k)
#pragma unroll
        for (int u = 0; u < U; ++u) x[0][u] += x[k][u];
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + v0 + u * B, x[0][u]);
}

template <int U>
__global__ __launch_bounds__(B) void pred(f64x2 *out, Ins in, int P) {
    const size_t v0 = (size_t)blockIdx.x * B * U + threadIdx.x;
    f64x2 x[MAXP][U];
#pragma unroll
    for (int k = 0; k < MAXP; ++k)
        if (k < P)
#pragma unroll
            for (int u = 0; u < U; ++u) x[k][u] = ld(in.p[k] + v0 + u * B);
#pragma unroll
    for (int k = 1; k < MAXP; ++k)
        if (k < P)
#pragma unroll
            for (int u = 0; u < U; ++u) x[0][u] += x[k][u];
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + v0 + u * B, x[0][u]);
}

// read-only ceiling: the P inputs are loaded and folded, the result stored
// only where it can never be true (keeps the loads alive)
template <int U>
__global__ __launch_bounds__(B) void rdonly(f64x2 *out, Ins in, int P) {
    const size_t v0 = (size_t)blockIdx.x * B * U + threadIdx.x;
    f64x2 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = ld(in.p[0] + v0 + u * B);
    for (int k = 1; k < P; ++k) {
        f64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld(in.p[k] + v0 + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += x[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (acc[u].x == -1.0) st(out + v0 + u * B, acc[u]);
}

// round-2b variants for the P = 8, 16 Mi case (77 % of peak):
//   pol<U,L,S>  rt's loop, load / store cache policy chosen (1 = nt)
//   seq<U,R>    rt's loop, but each block walks R consecutive chunks, so it
//               streams R*B*U*16 contiguous bytes per input (DRAM row reuse)
template <int U, int L, int S>
__global__ __launch_bounds__(B) void pol(f64x2 *out, Ins in, int P) {
    const size_t v0 = (size_t)blockIdx.x * B * U + threadIdx.x;
    auto l = [](const f64x2 *q) { if constexpr (L) return __builtin_nontemporal_load(q); else return *q; };
    f64x2 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = l(in.p[0] + v0 + u * B);
    for (int k = 1; k < P; ++k) {
        f64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = l(in.p[k] + v0 + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += x[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if constexpr (S) __builtin_nontemporal_store(acc[u], out + v0 + u * B);
        else out[v0 + u * B] = acc[u];
    }
}

template <int U, int R>
__global__ __launch_bounds__(B) void seq(f64x2 *out, Ins in, int P) {
    for (int r = 0; r < R; ++r) {
        const size_t v0 = ((size_t)blockIdx.x * R + r) * B * U + threadIdx.x;
        f64x2 acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = ld(in.p[0] + v0 + u * B);
        for (int k = 1; k < P; ++k) {
            f64x2 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = ld(in.p[k] + v0 + u * B);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += x[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st(out + v0 + u * B, acc[u]);
    }
}

// round-2c variants for the same case: block size, and a persistent
// grid-stride grid of G blocks (G from the grid the host passes)
template <int U, int BS>
__global__ __launch_bounds__(BS) void rtb(f64x2 *out, Ins in, int P) {
    const size_t v0 = (size_t)blockIdx.x * BS * U + threadIdx.x;
    f64x2 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = ld(in.p[0] + v0 + u * BS);
    for (int k = 1; k < P; ++k) {
        f64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld(in.p[k] + v0 + u * BS);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += x[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + v0 + u * BS, acc[u]);
}

__device__ size_t g_nchunks;   // set by the host before the rtg launches
template <int U>
__global__ __launch_bounds__(B) void rtg(f64x2 *out, Ins in, int P) {
    for (size_t c = blockIdx.x; c < g_nchunks; c += gridDim.x) {
        const size_t v0 = c * B * U + threadIdx.x;
        f64x2 acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = ld(in.p[0] + v0 + u * B);
        for (int k = 1; k < P; ++k) {
            f64x2 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = ld(in.p[k] + v0 + u * B);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += x[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st(out + v0 + u * B, acc[u]);
    }
}

__global__ void flush(f64x2 *p, size_t n, double v) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = f64x2{v, v};
}

typedef void (*Kern)(f64x2 *, Ins, int);
struct Var {
    const char *name;
    Kern k;
    int U;
    int P;        // 0 = any
    int bs = 256;  // block size
    int grid = 0;  // 0: one chunk per block; else a persistent grid of this many
};

template <int P>
void add_static(std::vector<Var> &v) {
    v.push_back({"st_u1", stat<P, 1>, 1, P});
    v.push_back({"st_u2", stat<P, 2>, 2, P});
    v.push_back({"st_u4", stat<P, 4>, 4, P});
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (size_t(4) << 20);
    const int cold = argc > 2 ? atoi(argv[2]) : 0;
    // skew < 0: every input its own hipMalloc; else all inputs in one block at
    // k * (n * 8 + skew) bytes (the A2A workspace layout when skew = 0)
    const long skew = argc > 3 ? atol(argv[3]) : -1;
    const size_t nvec = n / 2;
    std::vector<f64x2 *> bufs(MAXP + 1);
    if (skew < 0) {
        for (auto &b : bufs) CK(hipMalloc(&b, n * 8));
    } else {
        char *blk = nullptr;
        CK(hipMalloc(&blk, (MAXP + 1) * (n * 8 + (size_t)skew)));
        for (int k = 0; k <= MAXP; ++k) bufs[k] = reinterpret_cast<f64x2 *>(blk + k * (n * 8 + (size_t)skew));
    }
    for (auto &b : bufs) hipLaunchKernelGGL(flush, dim3(4096), dim3(256), 0, 0, b, nvec, 1.0);
    f64x2 *scratch = nullptr;
    const size_t sn = (size_t(1) << 30) / 16;
    CK(hipMalloc(&scratch, sn * 16));
    CK(hipDeviceSynchronize());
    const bool round2b = getenv("FOLDN_2B") != nullptr;
    const bool round2c = getenv("FOLDN_2C") != nullptr;
    std::vector<Var> vars = {{"rt_u4", rt<4>, 4, 0}, {"rt_u2", rt<2>, 2, 0},
                             {"pipe_u4", pipe<4>, 4, 0}, {"pipe_u2", pipe<2>, 2, 0},
                             {"rdonly_u4", rdonly<4>, 4, 0}};
    if (round2c) {
        vars = {{"rt_u4", rt<4>, 4, 0},
                {"b256_u2", rtb<2, 256>, 2, 0, 256},   {"b512_u1", rtb<1, 512>, 1, 0, 512},
                {"b512_u2", rtb<2, 512>, 2, 0, 512},   {"b512_u4", rtb<4, 512>, 4, 0, 512},
                {"b1024_u1", rtb<1, 1024>, 1, 0, 1024}, {"b1024_u2", rtb<2, 1024>, 2, 0, 1024},
                {"g512_u4", rtg<4>, 4, 0, 256, 512},   {"rdonly_u4", rdonly<4>, 4, 0}};
    } else if (round2b) {
        // U is the block's footprint divisor below (grid = nvec / (B*U)); seq
        // counts its R chunks in it
        vars = {{"rt_u4", rt<4>, 4, 0},          {"rt_u8", rt<8>, 8, 0},
                {"pol_u4_L0S1", pol<4, 0, 1>, 4, 0}, {"pol_u4_L1S0", pol<4, 1, 0>, 4, 0},
                {"pol_u4_L0S0", pol<4, 0, 0>, 4, 0}, {"seq_u4_r2", seq<4, 2>, 8, 0},
                {"seq_u4_r4", seq<4, 4>, 16, 0},     {"seq_u4_r16", seq<4, 16>, 64, 0},
                {"rdonly_u4", rdonly<4>, 4, 0}};
    } else {
        add_static<3>(vars);
        add_static<4>(vars);
        add_static<6>(vars);
        add_static<8>(vars);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("# skew %ld (%s)\n", skew, skew < 0 ? "separate allocations" : "one block, inputs k*(n*8+skew) apart");
    printf("# n=%zu per input, %s; GB/s = (P+1)*n*8 / launch time (median of rounds)\n", n,
           cold ? "cold (1 GiB scratch rewritten before each launch)" : "warm (back to back)");
    for (int P : {2, 3, 4, 6, 8}) {
        if (P == 2 && !round2c) continue;
        if ((round2b || round2c) && P != 2 && P != 4 && P != 8) continue;
        Ins in{};
        for (int k = 0; k < P; ++k) in.p[k] = bufs[k];
        std::vector<std::vector<float>> t(vars.size());
        for (int round = 0; round < 7; ++round) {
            for (size_t vi = 0; vi < vars.size(); ++vi) {
                const Var &v = vars[vi];
                if (v.P && v.P != P) continue;
                const size_t nch = nvec / ((size_t)v.bs * v.U);
                CK(hipMemcpyToSymbol(HIP_SYMBOL(g_nchunks), &nch, sizeof nch));
                const dim3 grid((unsigned)(v.grid ? v.grid : nch));
                float total = 0;
                const int reps = cold ? 5 : 10;
                for (int r = 0; r < reps + 1; ++r) {
                    if (cold) hipLaunchKernelGGL(flush, dim3(8192), dim3(256), 0, 0, scratch, sn, (double)r);
                    CK(hipEventRecord(e0, 0));
                    hipLaunchKernelGGL(v.k, grid, dim3(v.bs), 0, 0, bufs[MAXP], in, P);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (r) total += ms;
                }
                t[vi].push_back(total / reps);
            }
        }
        // correctness of every variant (sum of P ones)
        for (size_t vi = 0; vi < vars.size(); ++vi) {
            const Var &v = vars[vi];
            if (v.P && v.P != P) continue;
            CK(hipMemset(bufs[MAXP], 0, n * 8));
            const size_t nch = nvec / ((size_t)v.bs * v.U);
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_nchunks), &nch, sizeof nch));
            hipLaunchKernelGGL(v.k, dim3((unsigned)(v.grid ? v.grid : nch)), dim3(v.bs), 0, 0,
                               bufs[MAXP], in, P);
            double h[4];
            CK(hipMemcpy(h, reinterpret_cast<double *>(bufs[MAXP]) + n - 4, sizeof h, hipMemcpyDeviceToHost));
            const bool ok = h[3] == (double)P || v.k == rdonly<4>;
            std::sort(t[vi].begin(), t[vi].end());
            const double ms = t[vi][t[vi].size() / 2];
            printf("P=%d %-8s %8.1f us %7.1f GB/s %s\n", P, v.name, ms * 1e3,
                   (P + 1) * n * 8 / (ms * 1e-3) / 1e9, ok ? "" : "WRONG");
        }
        fflush(stdout);
    }
    return 0;
}
