#line 1 "oracle/ref_ops_harness.c"
/*
 * TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the
 * product (openshmem-async_amd/).
 *
 * This file is not compiled on its own.  oracle/build_ref.sh feeds gcc, as one
 * translation unit read from a pipe:
 *   1. #include <complex.h>;
 *   2. the reference's OWN element-operation text, read where it lies:
 *      /root/reference/src/reduce/reduce-op.c:71-150 (SHMEM_MATH_FUNC,
 *      SHMEM_LOGIC_FUNC, SHMEM_MINIMAX_FUNC and their instantiations), which
 *      needs nothing but <complex.h>;
 *   3. this file, which exports those static functions through one C entry
 *      point.
 * The output is oracle/_ref/libref_ops.so (git-ignored).  Nothing of the
 * reference is written to disk or committed.  The rest of reduce-op.c (the
 * fold loop, :169-260) needs GASNet through comms/comms.h and stays
 * unbuildable here.
 *
 * ref_op_apply(type, op, a, b, out, n): out[i] = the_op(a[i], b[i]) with
 * the_op the reference's own <op>_<type>_func, called through a function
 * pointer as reduce-op.c:233 does.  Type and op numbering are the oracle's
 * (reduce_oracle.h).  Returns 0, or -1 when the reference defines no such
 * function (e.g. xor on double, min on complex).
 */
#include <stddef.h>

enum {
    REF_SHORT = 0, REF_INT, REF_LONG, REF_LONGLONG, REF_FLOAT, REF_DOUBLE,
    REF_LONGDOUBLE, REF_COMPLEXD, REF_COMPLEXF
};
enum { REF_SUM = 0, REF_PROD, REF_AND, REF_OR, REF_XOR, REF_MIN, REF_MAX };

#define REF_APPLY(T, FN)                                                       \
    do {                                                                       \
        T (*volatile the_op)(T, T) = FN;                                       \
        const T *x = (const T *)a, *y = (const T *)b;                         \
        T *z = (T *)out;                                                       \
        for (long i = 0; i < n; ++i) z[i] = (*the_op)(x[i], y[i]);            \
        return 0;                                                              \
    } while (0)

#define REF_CASES_MATH(TC, N, T)                                               \
    case TC * 8 + REF_SUM: REF_APPLY(T, sum_##N##_func);                       \
    case TC * 8 + REF_PROD: REF_APPLY(T, prod_##N##_func);
#define REF_CASES_LOGIC(TC, N, T)                                              \
    case TC * 8 + REF_AND: REF_APPLY(T, and_##N##_func);                       \
    case TC * 8 + REF_OR: REF_APPLY(T, or_##N##_func);                         \
    case TC * 8 + REF_XOR: REF_APPLY(T, xor_##N##_func);
#define REF_CASES_MINIMAX(TC, N, T)                                            \
    case TC * 8 + REF_MIN: REF_APPLY(T, min_##N##_func);                       \
    case TC * 8 + REF_MAX: REF_APPLY(T, max_##N##_func);

int ref_op_apply(int type, int op, const void *a, const void *b, void *out, long n)
{
    if (type < 0 || op < 0 || op > 7 || n < 0) return -1;
    switch (type * 8 + op) {
    REF_CASES_MATH(REF_SHORT, short, short)
    REF_CASES_MATH(REF_INT, int, int)
    REF_CASES_MATH(REF_LONG, long, long)
    REF_CASES_MATH(REF_LONGLONG, longlong, long long)
    REF_CASES_MATH(REF_FLOAT, float, float)
    REF_CASES_MATH(REF_DOUBLE, double, double)
    REF_CASES_MATH(REF_LONGDOUBLE, longdouble, long double)
    REF_CASES_MATH(REF_COMPLEXD, complexd, double complex)
    REF_CASES_MATH(REF_COMPLEXF, complexf, float complex)
    REF_CASES_LOGIC(REF_SHORT, short, short)
    REF_CASES_LOGIC(REF_INT, int, int)
    REF_CASES_LOGIC(REF_LONG, long, long)
    REF_CASES_LOGIC(REF_LONGLONG, longlong, long long)
    REF_CASES_MINIMAX(REF_SHORT, short, short)
    REF_CASES_MINIMAX(REF_INT, int, int)
    REF_CASES_MINIMAX(REF_LONG, long, long)
    REF_CASES_MINIMAX(REF_LONGLONG, longlong, long long)
    REF_CASES_MINIMAX(REF_FLOAT, float, float)
    REF_CASES_MINIMAX(REF_DOUBLE, double, double)
    REF_CASES_MINIMAX(REF_LONGDOUBLE, longdouble, long double)
    default:
        return -1;
    }
}
