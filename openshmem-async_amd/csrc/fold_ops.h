// Element ops and 16-byte vector plumbing shared by the gfx950 kernels of
// the path (fold_kernels.hip: the fold and gather kernels; signal_kernels.hip:
// the system fences, device barriers and fused one-/two-shot launches).
// Internal to libshmem_reduce_mi355x.so; everything here has internal linkage
// in each kernel file.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
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

constexpr int kBlock = 256;  // 4 waves of 64

// long double and the complex products: soft-float / Annex G code unrolled
// 16 vectors deep would spill; they keep the runtime-nins kernel.
template <typename T, int OP>
constexpr bool kHeavyOp = std::is_same<T, ld80>::value ||
                          ((std::is_same<T, cplxd>::value || std::is_same<T, cplxf>::value) &&
                           OP == SHMEMX_OP_PROD);

}  // namespace

}  // namespace shmx
