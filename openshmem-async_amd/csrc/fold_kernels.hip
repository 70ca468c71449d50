// gfx950 (MI355X, CDNA4) kernels for the OpenSHMEM reduction collectives.
//
// One kernel family does all the arithmetic of the path: the element-wise
// left fold of reduce-op.c:213-248,
//     write_to = source_me;  for each other PE p: write_to = op(write_to, src_p)
// here as ONE pass over all inputs instead of one pass per peer:
//     out[i] = op(...op(op(in0[i], in1[i]), in2[i])..., in_{k-1}[i])
// with the element ops of reduce-op.c:71-150 (sum a+b, prod a*b, and/or/xor,
// min a<b?a:b, max a>b?a:b).  nins == 2 with out == in0 is the reference's
// inner fold write_to[ti] = op(write_to[ti], pWrk[j]) (reduce-op.c:231-235);
// nins == 1 is the copy of reduce-op.c:213-216.
//
// Design for gfx950 (DESIGN.md "Kernels"):
//   * HBM-bound streaming: 16-byte loads/stores per lane (global_load_dwordx4),
//     a wave-instruction covers 1 KiB contiguous; UNROLL independent vectors
//     per input per lane are issued before any op, so a 256-lane workgroup
//     keeps UNROLL*nins*4 KiB in flight;
//   * whole-chunk fast path with no per-vector guards (a guarded unrolled load
//     makes hipcc wait vmcnt(0) per element), guarded path only for the last
//     partial chunk;
//   * scalar head/tail peeling so 8-byte-aligned (dlmalloc, dlmalloc.c:557)
//     or odd-length arrays still take the vector body;
//   * no LDS, no DPP: an element-wise fold has no intra-wave reduction and no
//     reuse, so an LDS round trip would be pure overhead;
//   * bit-exact with the reference's C: integers wrap in unsigned arithmetic,
//     short is computed in int and truncated, no FP contraction
//     (-ffp-contract=off), min/max are selects (not v_min_f64, whose NaN / -0
//     behaviour differs), complex products follow C99 Annex G / libgcc
//     __muldc3 including its NaN-recovery branch.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>
#include <type_traits>

#include "internal.h"
#include "ld80.h"
#include "shmem_reduce_mi355x.h"

namespace shmx {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct cplxd { double re, im; };
struct cplxf { float re, im; };

// ------------------------------------------------------------- element ops
template <typename T> struct Wide { using U = std::make_unsigned_t<T>; };
template <> struct Wide<short> { using U = unsigned int; };  // int promotion

template <typename T>
__device__ __forceinline__ T add_wrap(T a, T b) {
    using U = typename Wide<T>::U;
    return (T)((U)a + (U)b);
}
template <typename T>
__device__ __forceinline__ T mul_wrap(T a, T b) {
    using U = typename Wide<T>::U;
    return (T)((U)a * (U)b);
}

// C99 Annex G complex multiply as libgcc's __muldc3 / __mulsc3 compute it.
template <typename S>
__device__ __forceinline__ void cmul(S a, S b, S c, S d, S &xr, S &yr) {
    S ac = a * c, bd = b * d, ad = a * d, bc = b * c;
    S x = ac - bd, y = ad + bc;
    if (__builtin_isnan(x) && __builtin_isnan(y)) {
        bool recalc = false;
        const S inf = __builtin_inf();
        if (__builtin_isinf(a) || __builtin_isinf(b)) {
            a = __builtin_copysign(__builtin_isinf(a) ? S(1) : S(0), a);
            b = __builtin_copysign(__builtin_isinf(b) ? S(1) : S(0), b);
            if (__builtin_isnan(c)) c = __builtin_copysign(S(0), c);
            if (__builtin_isnan(d)) d = __builtin_copysign(S(0), d);
            recalc = true;
        }
        if (__builtin_isinf(c) || __builtin_isinf(d)) {
            c = __builtin_copysign(__builtin_isinf(c) ? S(1) : S(0), c);
            d = __builtin_copysign(__builtin_isinf(d) ? S(1) : S(0), d);
            if (__builtin_isnan(a)) a = __builtin_copysign(S(0), a);
            if (__builtin_isnan(b)) b = __builtin_copysign(S(0), b);
            recalc = true;
        }
        if (!recalc && (__builtin_isinf(ac) || __builtin_isinf(bd) ||
                        __builtin_isinf(ad) || __builtin_isinf(bc))) {
            if (__builtin_isnan(a)) a = __builtin_copysign(S(0), a);
            if (__builtin_isnan(b)) b = __builtin_copysign(S(0), b);
            if (__builtin_isnan(c)) c = __builtin_copysign(S(0), c);
            if (__builtin_isnan(d)) d = __builtin_copysign(S(0), d);
            recalc = true;
        }
        if (recalc) {
            x = inf * (a * c - b * d);
            y = inf * (a * d + b * c);
        }
    }
    xr = x;
    yr = y;
}

template <typename T, int OP> struct Op;

// Integer types: all seven ops (reduce-op.c:85-90,120-123,144-147).
#define SHMX_INT_OPS(T)                                                        \
    template <> struct Op<T, SHMEMX_OP_SUM> {                                \
        __device__ static T ap(T a, T b) { return add_wrap(a, b); } };       \
    template <> struct Op<T, SHMEMX_OP_PROD> {                               \
        __device__ static T ap(T a, T b) { return mul_wrap(a, b); } };       \
    template <> struct Op<T, SHMEMX_OP_AND> {                                \
        __device__ static T ap(T a, T b) { return (T)(a & b); } };           \
    template <> struct Op<T, SHMEMX_OP_OR> {                                 \
        __device__ static T ap(T a, T b) { return (T)(a | b); } };           \
    template <> struct Op<T, SHMEMX_OP_XOR> {                                \
        __device__ static T ap(T a, T b) { return (T)(a ^ b); } };           \
    template <> struct Op<T, SHMEMX_OP_MIN> {                                \
        __device__ static T ap(T a, T b) { return a < b ? a : b; } };        \
    template <> struct Op<T, SHMEMX_OP_MAX> {                                \
        __device__ static T ap(T a, T b) { return a > b ? a : b; } };
SHMX_INT_OPS(short)
SHMX_INT_OPS(int)
SHMX_INT_OPS(long)
#undef SHMX_INT_OPS

// Real floating types: sum, prod, min, max (reduce-op.c:88-89,148-149).
#define SHMX_FP_OPS(T)                                                         \
    template <> struct Op<T, SHMEMX_OP_SUM> {                                \
        __device__ static T ap(T a, T b) { return a + b; } };                \
    template <> struct Op<T, SHMEMX_OP_PROD> {                               \
        __device__ static T ap(T a, T b) { return a * b; } };               \
    template <> struct Op<T, SHMEMX_OP_MIN> {                                \
        __device__ static T ap(T a, T b) { return a < b ? a : b; } };        \
    template <> struct Op<T, SHMEMX_OP_MAX> {                                \
        __device__ static T ap(T a, T b) { return a > b ? a : b; } };
SHMX_FP_OPS(float)
SHMX_FP_OPS(double)
#undef SHMX_FP_OPS

// Complex: sum and prod (reduce-op.c:92-93).
#define SHMX_CPLX_OPS(C, S)                                                    \
    template <> struct Op<C, SHMEMX_OP_SUM> {                                \
        __device__ static C ap(C a, C b) {                                   \
            return C{a.re + b.re, a.im + b.im}; } };                         \
    template <> struct Op<C, SHMEMX_OP_PROD> {                               \
        __device__ static C ap(C a, C b) {                                   \
            C r; cmul<S>(a.re, a.im, b.re, b.im, r.re, r.im); return r; } };
SHMX_CPLX_OPS(cplxd, double)
SHMX_CPLX_OPS(cplxf, float)
#undef SHMX_CPLX_OPS

// long double: x87 80-bit in software (ld80.h), sum/prod/min/max
// (reduce-op.c:91,150).
using x87::ld80;
template <> struct Op<ld80, SHMEMX_OP_SUM> {
    __device__ static ld80 ap(ld80 a, ld80 b) { return x87::add(a, b); } };
template <> struct Op<ld80, SHMEMX_OP_PROD> {
    __device__ static ld80 ap(ld80 a, ld80 b) { return x87::mul(a, b); } };
template <> struct Op<ld80, SHMEMX_OP_MIN> {
    __device__ static ld80 ap(ld80 a, ld80 b) { return x87::less(a, b) ? a : b; } };
template <> struct Op<ld80, SHMEMX_OP_MAX> {
    __device__ static ld80 ap(ld80 a, ld80 b) { return x87::greater(a, b) ? a : b; } };

// ------------------------------------------------------- vector plumbing
// NT: bit 0 = non-temporal loads, bit 1 = non-temporal stores.
template <int NT>
__device__ __forceinline__ u32x4 ld16(const u32x4 *p) {
    if constexpr ((NT & 1) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int NT>
__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
    if constexpr ((NT & 2) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <typename T, int OP>
__device__ __forceinline__ u32x4 apply16(u32x4 a, u32x4 b) {
    constexpr int E = 16 / sizeof(T);
    union U { u32x4 v; T e[E]; };
    U x, y;
    x.v = a;
    y.v = b;
#pragma unroll
    for (int e = 0; e < E; ++e) x.e[e] = Op<T, OP>::ap(x.e[e], y.e[e]);
    return x.v;
}

struct FoldArgs {
    void *out;
    const void *ins[kMaxFoldInputs];
    int nins;
    size_t head;   // scalar elements before the first 16-B aligned vector
    size_t nvec;   // 16-B vectors in the aligned body
    size_t tail;   // scalar elements after it
    int peers;     // the inputs are other GPUs' HBM (launch_fold_peers)
};

constexpr int kBlock = 256;  // 4 waves of 64

// NIN > 0: number of inputs fixed at compile time (all loads hoisted);
// NIN == 0: runtime args.nins.
template <typename T, int OP, int NIN, int UNROLL, int NT>
__global__ __launch_bounds__(kBlock) void fold_kernel(FoldArgs args) {
    constexpr int E = 16 / sizeof(T);
    const int nins = NIN > 0 ? NIN : args.nins;
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * kBlock;

    // Scalar head and tail (grid-stride: the whole array when the inputs
    // do not share one alignment).
    {
        T *out = static_cast<T *>(args.out);
        const size_t body_end = args.head + args.nvec * E;
        const size_t nscalar = args.head + args.tail;
        for (size_t s = tid; s < nscalar; s += nthr) {
            const size_t i = s < args.head ? s : body_end + (s - args.head);
            T acc = static_cast<const T *>(args.ins[0])[i];
            for (int k = 1; k < nins; ++k)
                acc = Op<T, OP>::ap(acc, static_cast<const T *>(args.ins[k])[i]);
            out[i] = acc;
        }
    }
    if (args.nvec == 0) return;

    u32x4 *out = reinterpret_cast<u32x4 *>(static_cast<T *>(args.out) + args.head);
    const size_t nvec = args.nvec;
    const size_t step = (size_t)gridDim.x * kBlock * UNROLL;
    for (size_t base = (size_t)blockIdx.x * kBlock * UNROLL; base < nvec;
         base += step) {
        const size_t v0 = base + threadIdx.x;
        if (base + (size_t)kBlock * UNROLL <= nvec) {
            // whole chunk in range: unguarded, every load issued up front
            u32x4 acc[UNROLL];
            const u32x4 *in0 = reinterpret_cast<const u32x4 *>(
                static_cast<const T *>(args.ins[0]) + args.head);
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) acc[u] = ld16<NT>(in0 + v0 + u * kBlock);
            if constexpr (NIN > 0) {
                u32x4 x[NIN > 1 ? NIN - 1 : 1][UNROLL];
#pragma unroll
                for (int k = 1; k < NIN; ++k) {
                    const u32x4 *ink = reinterpret_cast<const u32x4 *>(
                        static_cast<const T *>(args.ins[k]) + args.head);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u)
                        x[k - 1][u] = ld16<NT>(ink + v0 + u * kBlock);
                }
#pragma unroll
                for (int k = 1; k < NIN; ++k)
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u)
                        acc[u] = apply16<T, OP>(acc[u], x[k - 1][u]);
            } else if (std::is_same<T, ld80>::value && nins >= 3) {
                // soft-float ops are long: input k + 1's loads are issued
                // before input k is folded, so the arithmetic overlaps them
                // (P = 8 long double sum 115 -> 107 us)
                auto in_k = [&](int k) {
                    return reinterpret_cast<const u32x4 *>(static_cast<const T *>(args.ins[k]) + args.head);
                };
                u32x4 cur[UNROLL];
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) cur[u] = ld16<NT>(in_k(1) + v0 + u * kBlock);
                for (int k = 2; k < nins; ++k) {
                    u32x4 nxt[UNROLL];
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) nxt[u] = ld16<NT>(in_k(k) + v0 + u * kBlock);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) {
                        acc[u] = apply16<T, OP>(acc[u], cur[u]);
                        cur[u] = nxt[u];
                    }
                }
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) acc[u] = apply16<T, OP>(acc[u], cur[u]);
            } else {
                for (int k = 1; k < nins; ++k) {
                    const u32x4 *ink = reinterpret_cast<const u32x4 *>(
                        static_cast<const T *>(args.ins[k]) + args.head);
                    u32x4 x[UNROLL];
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) x[u] = ld16<NT>(ink + v0 + u * kBlock);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) acc[u] = apply16<T, OP>(acc[u], x[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) st16<NT>(out + v0 + u * kBlock, acc[u]);
        } else {
            // last partial chunk: one vector at a time, guarded
            for (int u = 0; u < UNROLL; ++u) {
                const size_t v = v0 + (size_t)u * kBlock;
                if (v >= nvec) break;
                u32x4 acc = ld16<NT>(reinterpret_cast<const u32x4 *>(
                                         static_cast<const T *>(args.ins[0]) + args.head) + v);
                for (int k = 1; k < nins; ++k)
                    acc = apply16<T, OP>(acc, ld16<NT>(reinterpret_cast<const u32x4 *>(
                                                 static_cast<const T *>(args.ins[k]) + args.head) + v));
                st16<NT>(out + v, acc);
            }
        }
    }
}

// 16-B vectors per lane per input for the runtime-nins kernel.
constexpr int kUnrollN = 4;

// The P-input fold over inputs that live in the peers' HBM (DIRECT's and
// SIGNAL's fold phase).  The runtime-nins kernel above issues input k + 1's
// loads only after folding input k; with every input on another GPU, every
// resident wave would then wait on the same peer's link at the same time
// (all blocks start at input 0 together and stay in step behind that one
// link), so only one of the P - 1 links would carry traffic at a time.  Here
// every lane issues its U vectors of ALL inputs before folding any (uniform
// predicates, unrolled), so each wave has loads in flight on every link; U =
// 16 / MAXIN keeps 16 vectors in registers (4 per input up to 4 inputs, 2 up
// to 8, 1 up to 16).  The fold order is unchanged: input 0, then 1, ...
template <typename T, int OP, int MAXIN, int NT>
__global__ __launch_bounds__(kBlock) void fold_peers_kernel(FoldArgs args) {
    constexpr int E = 16 / sizeof(T);
    constexpr int U = kMaxFoldInputs / MAXIN;
    const int nins = args.nins;
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * kBlock;
    {
        T *out = static_cast<T *>(args.out);
        const size_t body_end = args.head + args.nvec * E;
        const size_t nscalar = args.head + args.tail;
        for (size_t s = tid; s < nscalar; s += nthr) {
            const size_t i = s < args.head ? s : body_end + (s - args.head);
            T acc = static_cast<const T *>(args.ins[0])[i];
            for (int k = 1; k < nins; ++k) acc = Op<T, OP>::ap(acc, static_cast<const T *>(args.ins[k])[i]);
            out[i] = acc;
        }
    }
    if (args.nvec == 0) return;
    auto in = [&](int k) {
        return reinterpret_cast<const u32x4 *>(static_cast<const T *>(args.ins[k]) + args.head);
    };
    u32x4 *out = reinterpret_cast<u32x4 *>(static_cast<T *>(args.out) + args.head);
    const size_t nvec = args.nvec;
    const size_t step = (size_t)gridDim.x * kBlock * U;
    for (size_t base = (size_t)blockIdx.x * kBlock * U; base < nvec; base += step) {
        const size_t v0 = base + threadIdx.x;
        if (base + (size_t)kBlock * U <= nvec) {
            u32x4 x[MAXIN][U];
#pragma unroll
            for (int k = 0; k < MAXIN; ++k)
                if (k < nins)
#pragma unroll
                    for (int u = 0; u < U; ++u) x[k][u] = ld16<NT>(in(k) + v0 + u * kBlock);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                u32x4 acc = x[0][u];
#pragma unroll
                for (int k = 1; k < MAXIN; ++k)
                    if (k < nins) acc = apply16<T, OP>(acc, x[k][u]);
                st16<NT>(out + v0 + u * kBlock, acc);
            }
        } else {
            for (int u = 0; u < U; ++u) {
                const size_t v = v0 + (size_t)u * kBlock;
                if (v >= nvec) break;
                u32x4 acc = ld16<NT>(in(0) + v);
                for (int k = 1; k < nins; ++k) acc = apply16<T, OP>(acc, ld16<NT>(in(k) + v));
                st16<NT>(out + v, acc);
            }
        }
    }
}

// long double and the complex products: soft-float / Annex G code unrolled
// 16 vectors deep would spill; they keep the runtime-nins kernel.
template <typename T, int OP>
constexpr bool kHeavyOp = std::is_same<T, ld80>::value ||
                          ((std::is_same<T, cplxd>::value || std::is_same<T, cplxf>::value) &&
                           OP == SHMEMX_OP_PROD);

static size_t grid_for(const FoldArgs &a, int unroll) {
    const FoldTuning &tune = fold_tuning();
    size_t work_blocks;
    if (a.nvec > 0)
        work_blocks = (a.nvec + (size_t)kBlock * unroll - 1) / ((size_t)kBlock * unroll);
    else
        work_blocks = (a.head + a.tail + kBlock - 1) / kBlock;
    // The scalar-only case (inputs of different alignment) is capped hard; the
    // vector body runs one chunk per block unless a cap is set.
    size_t cap = tune.max_blocks > 0 ? (size_t)tune.max_blocks : (size_t)1 << 30;
    if (a.nvec == 0 && cap > 2048) cap = 2048;
    size_t blocks = work_blocks < cap ? work_blocks : cap;
    if (blocks < 1) blocks = 1;
    if (blocks > (size_t)INT_MAX) blocks = INT_MAX;
    return blocks;
}

template <typename T, int OP, int NT>
hipError_t launch_typed(const FoldArgs &a, hipStream_t stream) {
    if (a.nins == 2) {
        // the two-input fold (reduce-op.c:231-235): the hot kernel.  The
        // soft-float long double kernels exist at unroll 4 only.
        if constexpr (std::is_same<T, ld80>::value) {
            hipLaunchKernelGGL((fold_kernel<T, OP, 2, 4, NT>), dim3((unsigned)grid_for(a, 4)),
                               dim3(kBlock), 0, stream, a);
        } else {
            const int u = fold_tuning().unroll;
            const dim3 grid((unsigned)grid_for(a, u));
            if (u == 2)
                hipLaunchKernelGGL((fold_kernel<T, OP, 2, 2, NT>), grid, dim3(kBlock), 0, stream, a);
            else if (u == 8)
                hipLaunchKernelGGL((fold_kernel<T, OP, 2, 8, NT>), grid, dim3(kBlock), 0, stream, a);
            else
                hipLaunchKernelGGL((fold_kernel<T, OP, 2, 4, NT>), grid, dim3(kBlock), 0, stream, a);
        }
    } else if (a.peers && !kHeavyOp<T, OP> && (NT == 0 || NT == 3)) {
        if (a.nins <= 4)
            hipLaunchKernelGGL((fold_peers_kernel<T, OP, 4, NT>), dim3((unsigned)grid_for(a, 4)),
                               dim3(kBlock), 0, stream, a);
        else if (a.nins <= 8)
            hipLaunchKernelGGL((fold_peers_kernel<T, OP, 8, NT>), dim3((unsigned)grid_for(a, 2)),
                               dim3(kBlock), 0, stream, a);
        else
            hipLaunchKernelGGL((fold_peers_kernel<T, OP, 16, NT>), dim3((unsigned)grid_for(a, 1)),
                               dim3(kBlock), 0, stream, a);
    } else {
        hipLaunchKernelGGL((fold_kernel<T, OP, 0, kUnrollN, NT>), dim3((unsigned)grid_for(a, kUnrollN)),
                           dim3(kBlock), 0, stream, a);
    }
    return hipGetLastError();
}

// Cache policy: streams larger than the 256 MiB Infinity Cache go
// non-temporal on both loads and stores (measured +15-20 % at 768 MiB,
// profiles/ and DESIGN.md); smaller working sets keep the default policy so
// back-to-back calls can hit in the MALL.
constexpr size_t kNtThresholdBytes = size_t(256) << 20;

template <typename T, int OP>
hipError_t launch_nt(const FoldArgs &a, hipStream_t stream) {
    int mode = fold_tuning().nontemporal;
    if (mode < 0) {
        const size_t n = a.head + a.nvec * (16 / sizeof(T)) + a.tail;
        mode = (size_t)(a.nins + 1) * n * sizeof(T) >= kNtThresholdBytes ? 3 : 0;
    }
    if constexpr (std::is_same<T, ld80>::value) {  // fewer soft-float variants
        return mode ? launch_typed<T, OP, 3>(a, stream) : launch_typed<T, OP, 0>(a, stream);
    } else {
        if (a.peers) return mode ? launch_typed<T, OP, 3>(a, stream) : launch_typed<T, OP, 0>(a, stream);
        switch (mode & 3) {
        case 0: return launch_typed<T, OP, 0>(a, stream);
        case 1: return launch_typed<T, OP, 1>(a, stream);
        case 2: return launch_typed<T, OP, 2>(a, stream);
        default: return launch_typed<T, OP, 3>(a, stream);
        }
    }
}

template <typename T>
hipError_t launch_int_ops(int op, const FoldArgs &a, hipStream_t s) {
    switch (op) {
    case SHMEMX_OP_SUM: return launch_nt<T, SHMEMX_OP_SUM>(a, s);
    case SHMEMX_OP_PROD: return launch_nt<T, SHMEMX_OP_PROD>(a, s);
    case SHMEMX_OP_AND: return launch_nt<T, SHMEMX_OP_AND>(a, s);
    case SHMEMX_OP_OR: return launch_nt<T, SHMEMX_OP_OR>(a, s);
    case SHMEMX_OP_XOR: return launch_nt<T, SHMEMX_OP_XOR>(a, s);
    case SHMEMX_OP_MIN: return launch_nt<T, SHMEMX_OP_MIN>(a, s);
    case SHMEMX_OP_MAX: return launch_nt<T, SHMEMX_OP_MAX>(a, s);
    default: return hipErrorInvalidValue;
    }
}
template <typename T>
hipError_t launch_fp_ops(int op, const FoldArgs &a, hipStream_t s) {
    switch (op) {
    case SHMEMX_OP_SUM: return launch_nt<T, SHMEMX_OP_SUM>(a, s);
    case SHMEMX_OP_PROD: return launch_nt<T, SHMEMX_OP_PROD>(a, s);
    case SHMEMX_OP_MIN: return launch_nt<T, SHMEMX_OP_MIN>(a, s);
    case SHMEMX_OP_MAX: return launch_nt<T, SHMEMX_OP_MAX>(a, s);
    default: return hipErrorInvalidValue;
    }
}
template <typename T>
hipError_t launch_cplx_ops(int op, const FoldArgs &a, hipStream_t s) {
    switch (op) {
    case SHMEMX_OP_SUM: return launch_nt<T, SHMEMX_OP_SUM>(a, s);
    case SHMEMX_OP_PROD: return launch_nt<T, SHMEMX_OP_PROD>(a, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

FoldTuning &fold_tuning() {
    static FoldTuning t = [] {
        FoldTuning r{0, -1, 4};
        if (const char *e = std::getenv("SHMEMX_FOLD_MAX_BLOCKS")) r.max_blocks = std::atoi(e);
        if (const char *e = std::getenv("SHMEMX_FOLD_NT")) r.nontemporal = std::atoi(e);
        if (const char *e = std::getenv("SHMEMX_FOLD_UNROLL")) r.unroll = std::atoi(e);
        return r;
    }();
    return t;
}

size_t type_size(int type) {
    switch (type) {
    case SHMEMX_TYPE_SHORT: return sizeof(short);
    case SHMEMX_TYPE_INT: return sizeof(int);
    case SHMEMX_TYPE_LONG: return sizeof(long);
    case SHMEMX_TYPE_LONGLONG: return sizeof(long long);
    case SHMEMX_TYPE_FLOAT: return sizeof(float);
    case SHMEMX_TYPE_DOUBLE: return sizeof(double);
    case SHMEMX_TYPE_LONGDOUBLE: return sizeof(long double);
    case SHMEMX_TYPE_COMPLEXD: return 2 * sizeof(double);
    case SHMEMX_TYPE_COMPLEXF: return 2 * sizeof(float);
    default: return 0;
    }
}

bool op_valid(int type, int op) {
    if (type < 0 || type >= SHMEMX_NTYPES || op < 0 || op >= SHMEMX_NOPS) return false;
    switch (op) {
    case SHMEMX_OP_SUM:
    case SHMEMX_OP_PROD: return true;
    case SHMEMX_OP_AND:
    case SHMEMX_OP_OR:
    case SHMEMX_OP_XOR: return type <= SHMEMX_TYPE_LONGLONG;
    default: return type != SHMEMX_TYPE_COMPLEXD && type != SHMEMX_TYPE_COMPLEXF;
    }
}

bool op_on_device(int type, int op) { return op_valid(type, op); }

namespace {

// Split n elements into scalar head, 16-B vector body and scalar tail, given
// every array's address (the body only if all share one offset mod 16 that is
// a whole number of elements), then dispatch on type.
hipError_t dispatch(int type, int op, FoldArgs &a, const void *const *ptrs, int nptrs, size_t n,
                    hipStream_t stream) {
    const size_t sz = type_size(type);
    const uintptr_t off = reinterpret_cast<uintptr_t>(ptrs[0]) & 15u;
    bool same = (off % sz) == 0;
    for (int k = 1; k < nptrs && same; ++k)
        same = (reinterpret_cast<uintptr_t>(ptrs[k]) & 15u) == off;
    if (same) {
        size_t head = ((16 - off) & 15u) / sz;
        if (head > n) head = n;
        const size_t E = 16 / sz;
        a.head = head;
        a.nvec = (n - head) / E;
        a.tail = n - head - a.nvec * E;
    } else {
        a.head = n;
        a.nvec = 0;
        a.tail = 0;
    }
    switch (type) {
    case SHMEMX_TYPE_SHORT: return launch_int_ops<short>(op, a, stream);
    case SHMEMX_TYPE_INT: return launch_int_ops<int>(op, a, stream);
    case SHMEMX_TYPE_LONG:
    case SHMEMX_TYPE_LONGLONG: return launch_int_ops<long>(op, a, stream);
    case SHMEMX_TYPE_FLOAT: return launch_fp_ops<float>(op, a, stream);
    case SHMEMX_TYPE_DOUBLE: return launch_fp_ops<double>(op, a, stream);
    case SHMEMX_TYPE_LONGDOUBLE: return launch_fp_ops<ld80>(op, a, stream);
    case SHMEMX_TYPE_COMPLEXD: return launch_cplx_ops<cplxd>(op, a, stream);
    case SHMEMX_TYPE_COMPLEXF: return launch_cplx_ops<cplxf>(op, a, stream);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_fold(int type, int op, void *out, const void *const *ins,
                       int nins, size_t n, hipStream_t stream) {
    if (!op_on_device(type, op) || nins < 1 || nins > kMaxFoldInputs || !out)
        return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    FoldArgs a{};
    a.out = out;
    a.nins = nins;
    const void *ptrs[kMaxFoldInputs + 1];
    ptrs[0] = out;
    for (int k = 0; k < nins; ++k) {
        if (!ins[k]) return hipErrorInvalidValue;
        a.ins[k] = ins[k];
        ptrs[k + 1] = ins[k];
    }
    return dispatch(type, op, a, ptrs, nins + 1, n, stream);
}

hipError_t launch_fold_peers(int type, int op, void *out, const void *const *ins, int nins, size_t n,
                             hipStream_t stream) {
    if (!op_on_device(type, op) || nins < 1 || nins > kMaxFoldInputs || !out)
        return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    FoldArgs a{};
    a.out = out;
    a.nins = nins;
    a.peers = 1;
    const void *ptrs[kMaxFoldInputs + 1];
    ptrs[0] = out;
    for (int k = 0; k < nins; ++k) {
        if (!ins[k]) return hipErrorInvalidValue;
        a.ins[k] = ins[k];
        ptrs[k + 1] = ins[k];
    }
    return dispatch(type, op, a, ptrs, nins + 1, n, stream);
}

// ------------------------------------------------------------ gather copy
// DIRECT's all-gather phase: up to kMaxFoldInputs byte ranges (each a slice
// of a peer's result, read over xGMI) copied into this PE's target by ONE
// launch, so the reads from all peers are in flight at once (one copy per
// peer would serialise the links).  Consecutive blocks take the segments in
// turn: workgroups are dispatched in block order, and with the segment as
// the slow index (blockIdx.y) the first ~2048 resident blocks would all read
// the same peer, one link at a time.  On local HBM (one GPU) this costs 4 %
// against the y-major order (80.5 vs 77.4 us, 7 x 32 MiB), and runs of 16
// blocks per segment cost 15 % (89.3 us): profiles/r02c_pmc_kernels.json.
namespace {

struct CopySeg {
    const unsigned char *src;
    unsigned char *dst;
    size_t bytes;
};
struct GatherArgs {
    CopySeg seg[kMaxFoldInputs];
    int nseg;
};

constexpr int kGatherUnroll = 4;
constexpr unsigned kGatherRun = 1;   // consecutive blocks on one segment

__global__ __launch_bounds__(kBlock) void gather_kernel(GatherArgs a) {
    // runs of kGatherRun consecutive blocks per segment, the runs dealt out
    // to the segments in turn
    const unsigned run = blockIdx.x / kGatherRun;
    const CopySeg sg = a.seg[run % a.nseg];
    const size_t bx = (size_t)(run / a.nseg) * kGatherRun + blockIdx.x % kGatherRun;
    const size_t nbx = gridDim.x / a.nseg;
    const size_t tid = bx * kBlock + threadIdx.x;
    const size_t nthr = nbx * kBlock;
    const uintptr_t d = reinterpret_cast<uintptr_t>(sg.dst);
    const uintptr_t s = reinterpret_cast<uintptr_t>(sg.src);
    size_t head = (16 - (d & 15)) & 15;
    if (head > sg.bytes) head = sg.bytes;
    if (((s + head) & 15) != 0) {   // source and target disagree mod 16: bytes
        for (size_t i = tid; i < sg.bytes; i += nthr) sg.dst[i] = sg.src[i];
        return;
    }
    const size_t nvec = (sg.bytes - head) / 16;
    const size_t tail0 = head + nvec * 16;
    if (tid < head) sg.dst[tid] = sg.src[tid];
    if (tid < sg.bytes - tail0) sg.dst[tail0 + tid] = sg.src[tail0 + tid];
    const u32x4 *in = reinterpret_cast<const u32x4 *>(sg.src + head);
    u32x4 *out = reinterpret_cast<u32x4 *>(sg.dst + head);
    const size_t step = nthr * kGatherUnroll;
    size_t v = bx * kBlock * kGatherUnroll + threadIdx.x;
    for (; v + (size_t)(kGatherUnroll - 1) * kBlock < nvec; v += step) {
        u32x4 x[kGatherUnroll];
#pragma unroll
        for (int u = 0; u < kGatherUnroll; ++u) x[u] = __builtin_nontemporal_load(in + v + u * kBlock);
#pragma unroll
        for (int u = 0; u < kGatherUnroll; ++u) __builtin_nontemporal_store(x[u], out + v + u * kBlock);
    }
    for (int u = 0; u < kGatherUnroll; ++u) {
        const size_t w = v + (size_t)u * kBlock;
        if (w < nvec) __builtin_nontemporal_store(__builtin_nontemporal_load(in + w), out + w);
    }
}

// The per-XCD L2s are not coherent with each other or with the peers, so a
// system-scope fence must run on EVERY XCD.  Dispatch spreads workgroups
// round-robin over the XCDs in practice, so 64 one-wave blocks put 8 on each
// — but the block -> XCD map is not architecturally defined, so each block
// also records the XCD it ran on (HW_REG_XCC_ID) in seen[blockIdx.x]: the host
// (fence_and_wait) or the next signal_kernel checks that every XCD of the
// device reported, and refills or fails loudly if one did not.
// s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): id 20, offset 0, size 4
constexpr int kXccIdReg = 20 | (0 << 6) | ((4 - 1) << 11);

__global__ __launch_bounds__(64) void sys_fence_kernel(unsigned int *seen) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");   // system scope
        const unsigned int xcc = (unsigned int)__builtin_amdgcn_s_getreg(kXccIdReg) & 15u;
        __hip_atomic_store(seen + blockIdx.x, kFenceSeen | xcc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ void check_fence(const SignalArgs &a) {
    // lane b reads block b's record of the fence just before this kernel
    const int lane = threadIdx.x;
    unsigned int rec = 0;
    if (a.seen && lane < kFenceBlocks) {
        rec = __hip_atomic_load(a.seen + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.seen + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (!a.seen) return;
    int covered = 0;
#pragma unroll
    for (unsigned int x = 0; x < 16; ++x)
        covered += __ballot(rec == (kFenceSeen | x)) != 0 ? 1 : 0;
    if (lane == 0) {
        atomicAdd(a.fence_stats, 1ull);
        if (covered < a.nxcc) {
            atomicAdd(a.fence_stats + 1, 1ull);
            __hip_atomic_store(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ __launch_bounds__(64) void signal_kernel(SignalArgs a) {
    check_fence(a);
    const int i = threadIdx.x;
    if (i >= a.P || a.pe[i] == a.me) return;
    unsigned long long *mine = a.mine + a.pe[i];
    const unsigned long long want =
        __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
    __hip_atomic_store(mine, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long *theirs = a.peer[i] + a.me;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
            __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// ------------------------------------------------ fused one-shot (SIGNAL)
// Thread 0 of the last block to arrive: bump my counter for every peer
// (system-scope release: everything this GPU's blocks fenced before arriving
// is in memory first), then wait for every peer's counter for me.
__device__ void peer_handshake(const SignalArgs &a) {
    unsigned long long want[kMaxFoldInputs];
    for (int i = 0; i < a.P; ++i) {
        if (a.pe[i] == a.me) continue;
        unsigned long long *c = a.mine + a.pe[i];
        want[i] = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
        __hip_atomic_store(c, want[i], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < a.P; ++i) {
        if (a.pe[i] == a.me) continue;
        const unsigned long long *theirs = a.peer[i] + a.me;
        while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want[i]) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope
}

// One element of the one-shot fold: the peers' values are remote loads
// (µs each over xGMI), so all nins of them are issued before the first op
// instead of one load's latency per input; heavy ops keep the loop.
template <typename T, int OP>
__device__ __forceinline__ T fold_elem(const SignalFoldArgs &a, size_t i) {
    if constexpr (kHeavyOp<T, OP>) {
        T acc = static_cast<const T *>(a.ins[0])[i];
        for (int k = 1; k < a.nins; ++k) acc = Op<T, OP>::ap(acc, static_cast<const T *>(a.ins[k])[i]);
        return acc;
    } else {
        T x[kMaxFoldInputs];
#pragma unroll
        for (int k = 0; k < kMaxFoldInputs; ++k)
            if (k < a.nins) x[k] = static_cast<const T *>(a.ins[k])[i];
        T acc = x[0];
#pragma unroll
        for (int k = 1; k < kMaxFoldInputs; ++k)
            if (k < a.nins) acc = Op<T, OP>::ap(acc, x[k]);
        return acc;
    }
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void signal_fold_kernel(SignalFoldArgs a) {
    unsigned int *const count = a.gsync, *const gen = a.gsync + 1;
    // up to 4 elements per lane of one block: the last block to arrive folds
    // alone, and no block waits for a release or arrives at the exit
    const bool tiny = a.n <= (size_t)4 * kBlock;
    __shared__ int s_last;
    __shared__ unsigned int s_gen0;
    if (threadIdx.x == 0) {
        // entry: record this block's XCD, then write back the XCD's L2 and
        // drop stale peer lines (the fence also orders the record), arrive
        const unsigned int xcc = (unsigned int)__builtin_amdgcn_s_getreg(kXccIdReg) & 15u;
        __hip_atomic_store(a.sig.seen + blockIdx.x, kFenceSeen | xcc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");   // system scope
        const unsigned int gen0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == gridDim.x - 1;
        if (!s_last && !tiny) {
            // relaxed polls (an acquire load would invalidate the L2 on every
            // poll), one acquire once the generation moved
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.sig.timeout_ticks) {
                    // only if launches overlapped on this GPU (they must not)
                    __hip_atomic_store(a.sig.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        } else if (s_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        s_gen0 = gen0;   // for the checking wave
    }
    __syncthreads();
    // a tiny array is folded by the last block alone: the others have fenced
    // and arrived, and leave
    if (tiny && !s_last) return;
    if (s_last && threadIdx.x < 64) {
        // the last block's first wave: every block's XCD record at once (lane
        // b reads block b's), then lane 0 does the entry handshake
        const int lane = threadIdx.x;
        unsigned int rec = 0;
        if (lane < (int)gridDim.x) {
            rec = __hip_atomic_load(a.sig.seen + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sig.seen + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int covered = 0;
#pragma unroll
        for (unsigned int x = 0; x < 16; ++x) covered += __ballot(rec == (kFenceSeen | x)) != 0 ? 1 : 0;
        if (lane == 0) {
            atomicAdd(a.sig.fence_stats, 1ull);
            if (covered < a.sig.nxcc) {
                atomicAdd(a.sig.fence_stats + 1, 1ull);
                __hip_atomic_store(a.sig.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            peer_handshake(a.sig);   // reduce-op.c:217
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, s_gen0 + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    T *out = static_cast<T *>(a.out);
    if (tiny) {
        for (size_t i = threadIdx.x; i < a.n; i += kBlock) out[i] = fold_elem<T, OP>(a, i);
        __syncthreads();
        if (threadIdx.x == 0) peer_handshake(a.sig);   // reduce-op.c:250
        return;
    }
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x, nthr = (size_t)gridDim.x * kBlock;
    for (size_t i = tid; i < a.n; i += nthr) out[i] = fold_elem<T, OP>(a, i);
    __syncthreads();
    // exit: the last block to finish reading tells the peers (reduce-op.c:250)
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        peer_handshake(a.sig);
    }
}

// ------------------------------------------------ fused two-shot (SIGNAL)
// The peers' operands are read over xGMI, where a load's latency (µs) rather
// than HBM bounds a 64-block grid: every lane issues its U 16-B loads from
// each of the nins inputs (uniform predicates, unrolled) before folding any,
// so a block keeps U x nins x 4 KiB in flight per step; U = 16 / MAXIN (4
// vectors per input up to 4 inputs, 2 up to 8, 1 up to 16: 16 vectors in
// registers either way).
template <typename T, int OP, int MAXIN>
__device__ __forceinline__ void fold_vecs(const SignalFoldArgs &a, u32x4 *out, size_t nvec, size_t tid,
                                          size_t nthr) {
    constexpr int U = kMaxFoldInputs / MAXIN;
    const size_t step = nthr * U;
    auto in = [&](int k) {
        return reinterpret_cast<const u32x4 *>(static_cast<const T *>(a.ins[k]) + a.lo);
    };
    size_t v = (tid / kBlock) * kBlock * U + tid % kBlock;   // U vectors of a block are kBlock apart
    for (; v + (size_t)(U - 1) * kBlock < nvec; v += step) {
        u32x4 x[MAXIN][U];
#pragma unroll
        for (int k = 0; k < MAXIN; ++k)
            if (k < a.nins)
#pragma unroll
                for (int u = 0; u < U; ++u) x[k][u] = __builtin_nontemporal_load(in(k) + v + u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 acc = x[0][u];
#pragma unroll
            for (int k = 1; k < MAXIN; ++k)
                if (k < a.nins) acc = apply16<T, OP>(acc, x[k][u]);
            out[v + u * kBlock] = acc;
        }
    }
    for (int u = 0; u < U; ++u) {   // the last partial step
        const size_t w = v + (size_t)u * kBlock;
        if (w >= nvec) break;
        u32x4 acc = __builtin_nontemporal_load(in(0) + w);
        for (int k = 1; k < a.nins; ++k) acc = apply16<T, OP>(acc, __builtin_nontemporal_load(in(k) + w));
        out[w] = acc;
    }
}

template <typename T, int OP>
__device__ __forceinline__ void fold_span(const SignalFoldArgs &a, size_t tid, size_t nthr) {
    constexpr int E = 16 / sizeof(T);
    const size_t lo = a.lo, n = a.hi - a.lo;
    T *const out = static_cast<T *>(a.out) + lo;
    bool vec = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    for (int k = 0; k < a.nins; ++k)
        vec &= (reinterpret_cast<uintptr_t>(static_cast<const T *>(a.ins[k]) + lo) & 15) == 0;
    const size_t nvec = vec ? n / E : 0;
    u32x4 *const vout = reinterpret_cast<u32x4 *>(out);
    // soft x87 and the complex products (Annex G recovery branch) unrolled
    // 16 vectors deep would spill: one vector of one input at a time
    if constexpr (kHeavyOp<T, OP>) {
        for (size_t v = tid; v < nvec; v += nthr) {
            u32x4 acc = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
                                                       static_cast<const T *>(a.ins[0]) + lo) + v);
            for (int k = 1; k < a.nins; ++k)
                acc = apply16<T, OP>(acc, __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
                                                  static_cast<const T *>(a.ins[k]) + lo) + v));
            vout[v] = acc;
        }
    } else if (a.nins <= 4) {
        fold_vecs<T, OP, 4>(a, vout, nvec, tid, nthr);
    } else if (a.nins <= 8) {
        fold_vecs<T, OP, 8>(a, vout, nvec, tid, nthr);
    } else {
        fold_vecs<T, OP, 16>(a, vout, nvec, tid, nthr);
    }
    for (size_t i = nvec * E + tid; i < n; i += nthr) {
        T acc = static_cast<const T *>(a.ins[0])[lo + i];
        for (int k = 1; k < a.nins; ++k) acc = Op<T, OP>::ap(acc, static_cast<const T *>(a.ins[k])[lo + i]);
        out[i] = acc;
    }
}

// The all-gather of the two-shot: every segment's loads of a step issued
// before any store, so all peers' links are busy at once (U vectors per
// segment per lane, as fold_vecs).
template <int MAXSEG>
__device__ __forceinline__ void gather_vecs(const SignalFoldArgs &a, size_t nvec, size_t tid, size_t nthr) {
    constexpr int U = kMaxFoldInputs / MAXSEG;
    for (size_t v = (tid / kBlock) * kBlock * U + tid % kBlock; v < nvec; v += nthr * U) {
        u32x4 x[MAXSEG][U];
#pragma unroll
        for (int k = 0; k < MAXSEG; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k < a.nseg && v + u * kBlock < a.glen[k] / 16)
                    x[k][u] = __builtin_nontemporal_load(static_cast<const u32x4 *>(a.gsrc[k]) + v + u * kBlock);
#pragma unroll
        for (int k = 0; k < MAXSEG; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k < a.nseg && v + u * kBlock < a.glen[k] / 16)
                    static_cast<u32x4 *>(a.gdst[k])[v + u * kBlock] = x[k][u];
    }
}

__device__ __forceinline__ void gather_span(const SignalFoldArgs &a, size_t tid, size_t nthr) {
    bool vec = true;
    size_t most = 0;
    for (int k = 0; k < a.nseg; ++k) {
        vec &= ((reinterpret_cast<uintptr_t>(a.gsrc[k]) | reinterpret_cast<uintptr_t>(a.gdst[k])) & 15) == 0;
        most = a.glen[k] > most ? a.glen[k] : most;
    }
    if (!vec) {
        for (int k = 0; k < a.nseg; ++k)
            for (size_t i = tid; i < a.glen[k]; i += nthr)
                static_cast<unsigned char *>(a.gdst[k])[i] = static_cast<const unsigned char *>(a.gsrc[k])[i];
        return;
    }
    if (a.nseg <= 4) gather_vecs<4>(a, most / 16, tid, nthr);
    else if (a.nseg <= 8) gather_vecs<8>(a, most / 16, tid, nthr);
    else gather_vecs<16>(a, most / 16, tid, nthr);
    for (int k = 0; k < a.nseg; ++k)
        for (size_t i = a.glen[k] / 16 * 16 + tid; i < a.glen[k]; i += nthr)
            static_cast<unsigned char *>(a.gdst[k])[i] = static_cast<const unsigned char *>(a.gsrc[k])[i];
}

// Grid barrier + peer handshake inside the kernel: every block writes back
// its XCD's L2 (its own stores become visible over xGMI) and arrives; the
// last one does the handshake and releases the generation gen_now + 1; every
// block then drops stale lines of the peers' memory (system acquire) before
// it reads what the peers wrote.
__device__ void grid_handshake(const SignalFoldArgs &a, unsigned int gen_now) {
    unsigned int *const count = a.gsync, *const gen = a.gsync + 1;
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope
        if (__hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            peer_handshake(a.sig);
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, gen_now + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen_now) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.sig.timeout_ticks) {
                    __hip_atomic_store(a.sig.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope
    }
    __syncthreads();
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void signal_fold2_kernel(SignalFoldArgs a) {
    unsigned int *const count = a.gsync, *const gen = a.gsync + 1;
    __shared__ int s_last;
    __shared__ unsigned int s_gen0;
    if (threadIdx.x == 0) {
        // entry, as the one shot: record the XCD, fence, arrive
        const unsigned int xcc = (unsigned int)__builtin_amdgcn_s_getreg(kXccIdReg) & 15u;
        __hip_atomic_store(a.sig.seen + blockIdx.x, kFenceSeen | xcc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");   // system scope
        const unsigned int gen0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == gridDim.x - 1;
        if (!s_last) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.sig.timeout_ticks) {
                    __hip_atomic_store(a.sig.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_gen0 = gen0;
    }
    __syncthreads();
    if (s_last && threadIdx.x < 64) {
        const int lane = threadIdx.x;
        unsigned int rec = 0;
        if (lane < (int)gridDim.x) {
            rec = __hip_atomic_load(a.sig.seen + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sig.seen + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int covered = 0;
#pragma unroll
        for (unsigned int x = 0; x < 16; ++x) covered += __ballot(rec == (kFenceSeen | x)) != 0 ? 1 : 0;
        if (lane == 0) {
            atomicAdd(a.sig.fence_stats, 1ull);
            if (covered < a.sig.nxcc) {
                atomicAdd(a.sig.fence_stats + 1, 1ull);
                __hip_atomic_store(a.sig.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            peer_handshake(a.sig);   // reduce-op.c:217: every source is final
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, s_gen0 + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x, nthr = (size_t)gridDim.x * kBlock;
    fold_span<T, OP>(a, tid, nthr);     // my slice from every member's source
    grid_handshake(a, s_gen0 + 1u);     // every member's slice is final
    gather_span(a, tid, nthr);          // the other slices from the peers' targets
    __syncthreads();
    // exit: the last block to finish reading tells the peers (reduce-op.c:250)
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        peer_handshake(a.sig);
    }
}

template <typename T, int OP>
hipError_t sf_launch(const SignalFoldArgs &a, hipStream_t s) {
    if (a.two_shot)
        hipLaunchKernelGGL((signal_fold2_kernel<T, OP>), dim3(kFenceBlocks), dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL((signal_fold_kernel<T, OP>), dim3(kFenceBlocks), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename T>
hipError_t sf_ops(int op, const SignalFoldArgs &a, hipStream_t s) {
    constexpr bool integral = std::is_integral<T>::value;
    constexpr bool cplx = std::is_same<T, cplxd>::value || std::is_same<T, cplxf>::value;
    switch (op) {
    case SHMEMX_OP_SUM: return sf_launch<T, SHMEMX_OP_SUM>(a, s);
    case SHMEMX_OP_PROD: return sf_launch<T, SHMEMX_OP_PROD>(a, s);
    case SHMEMX_OP_AND:
        if constexpr (integral) return sf_launch<T, SHMEMX_OP_AND>(a, s);
        break;
    case SHMEMX_OP_OR:
        if constexpr (integral) return sf_launch<T, SHMEMX_OP_OR>(a, s);
        break;
    case SHMEMX_OP_XOR:
        if constexpr (integral) return sf_launch<T, SHMEMX_OP_XOR>(a, s);
        break;
    case SHMEMX_OP_MIN:
        if constexpr (!cplx) return sf_launch<T, SHMEMX_OP_MIN>(a, s);
        break;
    case SHMEMX_OP_MAX:
        if constexpr (!cplx) return sf_launch<T, SHMEMX_OP_MAX>(a, s);
        break;
    default: break;
    }
    return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_signal_fold(int type, int op, const SignalFoldArgs &a, hipStream_t stream) {
    if (!op_on_device(type, op) || a.nins < 1 || a.nins > kMaxFoldInputs || !a.out || !a.gsync ||
        !a.sig.seen || !a.sig.fence_stats || a.sig.P < 1 || a.sig.P > kMaxFoldInputs || !a.sig.mine ||
        !a.sig.err)
        return hipErrorInvalidValue;
    for (int k = 0; k < a.nins; ++k)
        if (!a.ins[k]) return hipErrorInvalidValue;
    for (int i = 0; i < a.sig.P; ++i)
        if (a.sig.pe[i] != a.sig.me && !a.sig.peer[i]) return hipErrorInvalidValue;
    if (a.two_shot) {
        if (a.lo > a.hi || a.hi > a.n || a.nseg < 0 || a.nseg > kMaxFoldInputs) return hipErrorInvalidValue;
        for (int k = 0; k < a.nseg; ++k)
            if (a.glen[k] && (!a.gsrc[k] || !a.gdst[k])) return hipErrorInvalidValue;
    }
    switch (type) {
    case SHMEMX_TYPE_SHORT: return sf_ops<short>(op, a, stream);
    case SHMEMX_TYPE_INT: return sf_ops<int>(op, a, stream);
    case SHMEMX_TYPE_LONG:
    case SHMEMX_TYPE_LONGLONG: return sf_ops<long>(op, a, stream);
    case SHMEMX_TYPE_FLOAT: return sf_ops<float>(op, a, stream);
    case SHMEMX_TYPE_DOUBLE: return sf_ops<double>(op, a, stream);
    case SHMEMX_TYPE_LONGDOUBLE: return sf_ops<ld80>(op, a, stream);
    case SHMEMX_TYPE_COMPLEXD: return sf_ops<cplxd>(op, a, stream);
    case SHMEMX_TYPE_COMPLEXF: return sf_ops<cplxf>(op, a, stream);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_signal(const SignalArgs &a, hipStream_t stream) {
    if (a.P < 1 || a.P > kMaxFoldInputs || !a.mine || !a.err) return hipErrorInvalidValue;
    for (int i = 0; i < a.P; ++i)
        if (a.pe[i] != a.me && !a.peer[i]) return hipErrorInvalidValue;
    hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_sys_fence(hipStream_t stream, unsigned int *seen) {
    if (!seen) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sys_fence_kernel, dim3(kFenceBlocks), dim3(64), 0, stream, seen);
    return hipGetLastError();
}

hipError_t launch_gather(const void *const *srcs, void *const *dsts, const size_t *bytes, int nseg,
                         hipStream_t stream) {
    if (nseg < 0 || nseg > kMaxFoldInputs) return hipErrorInvalidValue;
    GatherArgs a{};
    size_t most = 0;
    int k = 0;
    for (int i = 0; i < nseg; ++i) {
        if (!bytes[i]) continue;
        if (!srcs[i] || !dsts[i]) return hipErrorInvalidValue;
        a.seg[k++] = CopySeg{static_cast<const unsigned char *>(srcs[i]),
                             static_cast<unsigned char *>(dsts[i]), bytes[i]};
        most = bytes[i] > most ? bytes[i] : most;
    }
    if (!k) return hipSuccess;
    size_t bx = (most / 16 + (size_t)kBlock * kGatherUnroll - 1) / ((size_t)kBlock * kGatherUnroll);
    if (bx < 1) bx = 1;
    if (bx > 65535) bx = 65535;
    bx = (bx + kGatherRun - 1) / kGatherRun * kGatherRun;   // whole runs per segment
    a.nseg = k;
    hipLaunchKernelGGL(gather_kernel, dim3((unsigned)(bx * k)), dim3(kBlock), 0, stream, a);
    return hipGetLastError();
}

}  // namespace shmx
