/*
 * TEST INFRASTRUCTURE ONLY (see reduce_oracle.h).  Not part of the product.
 *
 * A CPU restatement, written from scratch, of the reference reduction
 * algorithm in /root/reference/src/reduce/reduce-op.c:
 *
 *   - element ops .................. reduce-op.c:71-150
 *       sum a+b, prod a*b            (SHMEM_MATH_FUNC,   :71-93)
 *       and a&b, or a|b, xor a^b     (SHMEM_LOGIC_FUNC,  :100-123)
 *       min a<b?a:b, max a>b?a:b     (SHMEM_MINIMAX_FUNC,:130-150)
 *   - linear fold .................. reduce-op.c:169-260 (SHMEM_UDR_TYPE_OP)
 *       write_to = source; barrier; for every other PE of the active set in
 *       ascending order: pull 64 elements into pWrk (shmem_getmem, :230),
 *       fold them element by element through a function pointer (:231-235);
 *       the nreduce % 64 remainder likewise (:238-245); barrier.
 *   - which type x op pairs exist .. reduce-op.c:388-431
 *
 * Integer arithmetic is done on the unsigned type of the same width and
 * converted back: gcc emits plain wrapping add/imul for the reference's signed
 * ops, so the bits are identical and this file has no signed-overflow UB.
 * `short` follows C's promotion: computed in int, truncated on return (:85).
 * Floating point is IEEE binary32/64 via SSE, x87 80-bit for long double, and
 * C99 complex (double complex * uses libgcc __muldc3, as the reference does).
 *
 * The reference's fold cannot be built in this container (its reduce-op.c
 * pulls in comms/gasnet/comms-shared.h:46 -> <gasnet.h>, an external library
 * that is not installed).  Its element ops (:71-150) need only <complex.h>:
 * oracle/build_ref.sh compiles them from the reference's text into
 * oracle/_ref/libref_ops.so, and tests/test_ref_ops.py holds the ops below to
 * that build bit for bit (fixture: tests/golden/ref_element_ops.json).  See
 * DESIGN.md §3 for the rest of the pinning.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include "reduce_oracle.h"

#include <complex.h>
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

typedef long double ldouble;
typedef double complex cdouble;
typedef float complex cfloat;

/* ---------------------------------------------------------------- ops ---- */
/* One static function per (op, type), called through a pointer per element,
 * exactly like the reference's (*the_op)(write_to[ti], pWrk[j]).            */

#define ORC_INT_OPS(N, T, U)                                                   \
    static T orc_sum_##N(T a, T b) { return (T)((U)a + (U)b); }              \
    static T orc_prod_##N(T a, T b) { return (T)((U)a * (U)b); }             \
    static T orc_and_##N(T a, T b) { return (T)(a & b); }                    \
    static T orc_or_##N(T a, T b) { return (T)(a | b); }                     \
    static T orc_xor_##N(T a, T b) { return (T)(a ^ b); }                    \
    static T orc_min_##N(T a, T b) { return a < b ? a : b; }                 \
    static T orc_max_##N(T a, T b) { return a > b ? a : b; }

#define ORC_FP_OPS(N, T)                                                       \
    static T orc_sum_##N(T a, T b) { return a + b; }                         \
    static T orc_prod_##N(T a, T b) { return a * b; }                        \
    static T orc_min_##N(T a, T b) { return a < b ? a : b; }                 \
    static T orc_max_##N(T a, T b) { return a > b ? a : b; }

#define ORC_CPLX_OPS(N, T)                                                     \
    static T orc_sum_##N(T a, T b) { return a + b; }                         \
    static T orc_prod_##N(T a, T b) { return a * b; }

/* short is promoted to int by the reference's `(a) + (b)` and truncated on
 * return; doing it in unsigned int gives the same low 16 bits.            */
ORC_INT_OPS(short, short, unsigned int)
ORC_INT_OPS(int, int, unsigned int)
ORC_INT_OPS(long, long, unsigned long)
ORC_INT_OPS(longlong, long long, unsigned long long)
ORC_FP_OPS(float, float)
ORC_FP_OPS(double, double)
ORC_FP_OPS(longdouble, ldouble)
ORC_CPLX_OPS(complexd, cdouble)
/* complex float sum, component by component.  `a + b` on float complex lets
 * gcc -O2 commute the adds (b.im + a.im), and which operand an SSE add puts
 * first decides only which NaN payload survives a NaN + NaN.  The reference
 * built with its configure defaults (-std=c99, no -O) keeps a's in both
 * components: SSE returns its first operand, quieted, when that is a NaN,
 * else the second, quieted, when that is one.  That choice is made here
 * explicitly, and tests/test_ref_ops.py holds this file to that build
 * (oracle/_ref, reduce-op.c:71-93 compiled from the reference's text).    */
static float orc_addf_first(float a, float b)
{
    uint32_t u;
    if (a != a) { memcpy(&u, &a, 4); u |= 0x00400000u; memcpy(&a, &u, 4); return a; }
    if (b != b) { memcpy(&u, &b, 4); u |= 0x00400000u; memcpy(&b, &u, 4); return b; }
    return a + b;
}
static cfloat orc_sum_complexf(cfloat a, cfloat b)
{
    float c[2] = {orc_addf_first(crealf(a), crealf(b)), orc_addf_first(cimagf(a), cimagf(b))};
    cfloat r;
    memcpy(&r, c, sizeof r);
    return r;
}
static cfloat orc_prod_complexf(cfloat a, cfloat b) { return a * b; }

/* ----------------------------------------------------- linear fold ------ */
/* fold_<T>: the body of the per-peer loop, reduce-op.c:224-245.  `peer` is the
 * peer's source as reached through shmem_getmem; pWrk staging is reproduced
 * with a memcpy of 64 elements at a time (a 0-byte get for nrem == 0 too).  */
#define ORC_FOLD(N, T)                                                         \
    static void orc_fold_##N(T (*fn)(T, T), T *write_to, const T *peer,      \
                             int nreduce)                                    \
    {                                                                        \
        T wrk[ORC_WRKDATA];                                                  \
        const int nloops = nreduce / ORC_WRKDATA;                            \
        const int nrem = nreduce % ORC_WRKDATA;                              \
        int ti = 0, si = 0;                                                  \
        for (int k = 0; k < nloops; ++k) {                                   \
            memcpy(wrk, peer + si, ORC_WRKDATA * sizeof(T));                 \
            for (int j = 0; j < ORC_WRKDATA; ++j, ++ti)                      \
                write_to[ti] = (*fn)(write_to[ti], wrk[j]);                  \
            si += ORC_WRKDATA;                                               \
        }                                                                    \
        memcpy(wrk, peer + si, (size_t)nrem * sizeof(T));                    \
        for (int j = 0; j < nrem; ++j, ++ti)                                 \
            write_to[ti] = (*fn)(write_to[ti], wrk[j]);                      \
    }                                                                        \
    static void orc_copy_##N(T *write_to, const T *src, int nreduce)         \
    {                                                                        \
        for (int j = 0; j < nreduce; ++j) write_to[j] = src[j];              \
    }

ORC_FOLD(short, short)
ORC_FOLD(int, int)
ORC_FOLD(long, long)
ORC_FOLD(longlong, long long)
ORC_FOLD(float, float)
ORC_FOLD(double, double)
ORC_FOLD(longdouble, ldouble)
ORC_FOLD(complexd, cdouble)
ORC_FOLD(complexf, cfloat)

size_t oracle_type_size(int type)
{
    static const size_t sz[ORC_NTYPES] = {
        sizeof(short), sizeof(int), sizeof(long), sizeof(long long),
        sizeof(float), sizeof(double), sizeof(ldouble), sizeof(cdouble),
        sizeof(cfloat)};
    return (type >= 0 && type < ORC_NTYPES) ? sz[type] : 0;
}

int oracle_op_valid(int type, int op)
{
    if (type < 0 || type >= ORC_NTYPES || op < 0 || op >= ORC_NOPS) return 0;
    switch (op) {
    case ORC_SUM: case ORC_PROD: return 1;                       /* :388-405 */
    case ORC_AND: case ORC_OR: case ORC_XOR:                     /* :406-417 */
        return type <= ORC_LONGLONG;
    default:                                                     /* :418-431 */
        return type != ORC_COMPLEXD && type != ORC_COMPLEXF;
    }
}

/* Type-erased dispatch: copy + fold for one (type, op). */
typedef struct {
    void (*copy)(void *w, const void *s, int n);
    void (*fold)(const void *fn, void *w, const void *peer, int n);
    const void *fn;
} orc_kernel_t;

#define ORC_ADAPT(N, T)                                                        \
    static void orc_copy_v_##N(void *w, const void *s, int n)                \
    { orc_copy_##N((T *)w, (const T *)s, n); }                               \
    static void orc_fold_v_##N(const void *fn, void *w, const void *p, int n)\
    { orc_fold_##N((T (*)(T, T))fn, (T *)w, (const T *)p, n); }

ORC_ADAPT(short, short)
ORC_ADAPT(int, int)
ORC_ADAPT(long, long)
ORC_ADAPT(longlong, long long)
ORC_ADAPT(float, float)
ORC_ADAPT(double, double)
ORC_ADAPT(longdouble, ldouble)
ORC_ADAPT(complexd, cdouble)
ORC_ADAPT(complexf, cfloat)

#define ORC_ROW_INT(N)                                                         \
    { (const void *)orc_sum_##N, (const void *)orc_prod_##N,                 \
      (const void *)orc_and_##N, (const void *)orc_or_##N,                   \
      (const void *)orc_xor_##N, (const void *)orc_min_##N,                  \
      (const void *)orc_max_##N }
#define ORC_ROW_FP(N)                                                          \
    { (const void *)orc_sum_##N, (const void *)orc_prod_##N, 0, 0, 0,        \
      (const void *)orc_min_##N, (const void *)orc_max_##N }
#define ORC_ROW_CPLX(N)                                                        \
    { (const void *)orc_sum_##N, (const void *)orc_prod_##N, 0, 0, 0, 0, 0 }

static int orc_kernel(int type, int op, orc_kernel_t *k)
{
    static const void *fns[ORC_NTYPES][ORC_NOPS] = {
        ORC_ROW_INT(short), ORC_ROW_INT(int), ORC_ROW_INT(long),
        ORC_ROW_INT(longlong), ORC_ROW_FP(float), ORC_ROW_FP(double),
        ORC_ROW_FP(longdouble), ORC_ROW_CPLX(complexd), ORC_ROW_CPLX(complexf)};
    static void (*const copies[ORC_NTYPES])(void *, const void *, int) = {
        orc_copy_v_short, orc_copy_v_int, orc_copy_v_long, orc_copy_v_longlong,
        orc_copy_v_float, orc_copy_v_double, orc_copy_v_longdouble,
        orc_copy_v_complexd, orc_copy_v_complexf};
    static void (*const folds[ORC_NTYPES])(const void *, void *, const void *,
                                           int) = {
        orc_fold_v_short, orc_fold_v_int, orc_fold_v_long, orc_fold_v_longlong,
        orc_fold_v_float, orc_fold_v_double, orc_fold_v_longdouble,
        orc_fold_v_complexd, orc_fold_v_complexf};
    if (!oracle_op_valid(type, op)) return -1;
    k->copy = copies[type];
    k->fold = folds[type];
    k->fn = fns[type][op];
    return 0;
}

/* PE `i`-th member of the active set: PE_start + i * 2^logPE_stride (:219-247) */
static int orc_member(int PE_start, int logPE_stride, int i)
{
    return PE_start + i * (1 << logPE_stride);
}

static int orc_check_set(int npes, int PE_start, int logPE_stride, int PE_size,
                         int nreduce)
{
    if (npes < 1 || PE_start < 0 || logPE_stride < 0 || logPE_stride > 30 ||
        PE_size < 1 || nreduce < 0)
        return -1;
    if ((long)PE_start + (long)(PE_size - 1) * (1L << logPE_stride) >= npes)
        return -1;
    return 0;
}

int oracle_reduce_sim(int type, int op, int npes, int PE_start,
                      int logPE_stride, int PE_size, int nreduce,
                      const void *sources, void *targets)
{
    orc_kernel_t k;
    if (orc_kernel(type, op, &k) ||
        orc_check_set(npes, PE_start, logPE_stride, PE_size, nreduce))
        return -1;
    const size_t sz = oracle_type_size(type);
    const size_t stride = sz * (size_t)nreduce;
    const char *src = (const char *)sources;
    char *tgt = (char *)targets;
    /* Every PE reads its peers' sources between the two barriers and writes
     * only its own target (or a temporary, copied back after the second
     * barrier, :187-203,251-259), so each PE's result is a function of the
     * original sources only; simulate the PEs one after another.           */
    void *write_to = malloc(stride ? stride : 1);
    if (!write_to) return -1;
    for (int m = 0; m < PE_size; ++m) {
        const int me = orc_member(PE_start, logPE_stride, m);
        k.copy(write_to, src + (size_t)me * stride, nreduce);     /* :213-216 */
        for (int i = 0; i < PE_size; ++i) {                       /* :219-248 */
            const int pe = orc_member(PE_start, logPE_stride, i);
            if (pe == me) continue;
            k.fold(k.fn, write_to, src + (size_t)pe * stride, nreduce);
        }
        memcpy(tgt + (size_t)me * stride, write_to, stride);
    }
    free(write_to);
    return 0;
}

/* One PE's target only (PE `pe`, a member of the set): the same loop as
 * oracle_reduce_sim for that PE alone (reduce-op.c:213-248), so a test can
 * check a full-size array without simulating every member.               */
int oracle_reduce_one(int type, int op, int npes, int PE_start, int logPE_stride,
                      int PE_size, int nreduce, const void *sources, int pe, void *target)
{
    orc_kernel_t k;
    if (orc_kernel(type, op, &k) ||
        orc_check_set(npes, PE_start, logPE_stride, PE_size, nreduce))
        return -1;
    int member = 0;
    for (int m = 0; m < PE_size; ++m) member |= orc_member(PE_start, logPE_stride, m) == pe;
    if (!member) return -1;
    const size_t stride = oracle_type_size(type) * (size_t)nreduce;
    const char *src = (const char *)sources;
    k.copy(target, src + (size_t)pe * stride, nreduce);                /* :213-216 */
    for (int i = 0; i < PE_size; ++i) {                                /* :219-248 */
        const int q = orc_member(PE_start, logPE_stride, i);
        if (q == pe) continue;
        k.fold(k.fn, target, src + (size_t)q * stride, nreduce);
    }
    return 0;
}

/* ------------------------------------------- neighbouring collectives ---- */

int oracle_broadcast_sim(size_t esize, int npes, int PE_root, int PE_start,
                         int logPE_stride, int PE_size, size_t nelems,
                         const void *sources, size_t src_stride,
                         void *targets, size_t tgt_stride)
{
    if (orc_check_set(npes, PE_start, logPE_stride, PE_size, 0) || PE_root < 0 ||
        PE_root >= PE_size)
        return -1;
    /* root = PE_root * step + PE_start (broadcast-linear.c:61); every other
     * member gets the root's source with one getmem (:64-67)               */
    const int root = orc_member(PE_start, logPE_stride, PE_root);
    const char *src = (const char *)sources + (size_t)root * src_stride;
    for (int m = 0; m < PE_size; ++m) {
        const int pe = orc_member(PE_start, logPE_stride, m);
        if (pe != root)
            memcpy((char *)targets + (size_t)pe * tgt_stride, src, nelems * esize);
    }
    return 0;
}

int oracle_collect_sim(size_t esize, int npes, int PE_start, int logPE_stride,
                       int PE_size, const size_t *nelems, const void *sources,
                       size_t src_stride, void *targets, size_t tgt_stride)
{
    if (orc_check_set(npes, PE_start, logPE_stride, PE_size, 0)) return -1;
    /* acc_off runs left to right through the set (collect-linear.c:83-110);
     * each member puts its slice at that offset on every member (:112-124) */
    size_t acc_off = 0;
    for (int i = 0; i < PE_size; ++i) {
        const int from = orc_member(PE_start, logPE_stride, i);
        const size_t nb = nelems[from] * esize;
        for (int m = 0; m < PE_size; ++m) {
            const int to = orc_member(PE_start, logPE_stride, m);
            memcpy((char *)targets + (size_t)to * tgt_stride + acc_off,
                   (const char *)sources + (size_t)from * src_stride, nb);
        }
        acc_off += nb;
    }
    return 0;
}

/* ------------------------------------------------------------ inputs ---- */

uint64_t oracle_splitmix64(uint64_t seed, uint64_t i)
{
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static double orc_unit53(uint64_t r) { return (double)(r >> 11) * 0x1p-53; }
static float orc_unit24(uint64_t r) { return (float)(r >> 40) * 0x1p-24f; }

void oracle_fill(int type, int kind, uint64_t seed, void *dst, size_t n)
{
    for (size_t i = 0; i < n; ++i) {
        const uint64_t r = oracle_splitmix64(seed, i);
        switch (type) {
        case ORC_SHORT:
            ((short *)dst)[i] = kind ? (short)(uint16_t)r
                                     : (short)((int)(r >> 53) - 1024);
            break;
        case ORC_INT:
            ((int *)dst)[i] = kind ? (int)(uint32_t)r
                                   : (int)((int64_t)(r >> 43) - (1 << 20));
            break;
        case ORC_LONG:
            ((long *)dst)[i] = kind ? (long)r : (long)((int64_t)(r >> 43) - (1 << 20));
            break;
        case ORC_LONGLONG:
            ((long long *)dst)[i] =
                kind ? (long long)r : (long long)((int64_t)(r >> 43) - (1 << 20));
            break;
        case ORC_FLOAT:
            ((float *)dst)[i] = kind ? orc_unit24(r) * 2.0f - 1.0f
                                     : 1.0f + orc_unit24(r);
            break;
        case ORC_DOUBLE:
            ((double *)dst)[i] = kind ? orc_unit53(r) * 2.0 - 1.0
                                      : 1.0 + orc_unit53(r);
            break;
        case ORC_LONGDOUBLE: {
            ldouble v = kind ? (ldouble)orc_unit53(r) * 2.0L - 1.0L
                             : 1.0L + (ldouble)orc_unit53(r);
            memset((ldouble *)dst + i, 0, sizeof(ldouble));
            ((ldouble *)dst)[i] = v;
            break;
        }
        case ORC_COMPLEXD: {
            const uint64_t r2 = oracle_splitmix64(seed ^ 0xC0FFEEULL, i);
            double re = kind ? orc_unit53(r) * 2.0 - 1.0 : 1.0 + orc_unit53(r);
            double im = kind ? orc_unit53(r2) * 2.0 - 1.0 : 1.0 + orc_unit53(r2);
            ((double *)dst)[2 * i] = re;
            ((double *)dst)[2 * i + 1] = im;
            break;
        }
        case ORC_COMPLEXF: {
            const uint64_t r2 = oracle_splitmix64(seed ^ 0xC0FFEEULL, i);
            float re = kind ? orc_unit24(r) * 2.0f - 1.0f : 1.0f + orc_unit24(r);
            float im = kind ? orc_unit24(r2) * 2.0f - 1.0f : 1.0f + orc_unit24(r2);
            ((float *)dst)[2 * i] = re;
            ((float *)dst)[2 * i + 1] = im;
            break;
        }
        default:
            break;
        }
    }
}

uint64_t oracle_fnv1a(const void *p, size_t nbytes)
{
    const unsigned char *b = (const unsigned char *)p;
    uint64_t h = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < nbytes; ++i) {
        h ^= b[i];
        h *= 0x100000001b3ULL;
    }
    return h;
}

/* Hash only the value bytes (long double: the 10 x87 bytes, not padding). */
static uint64_t orc_hash_elems(int type, const void *p, size_t n)
{
    if (type != ORC_LONGDOUBLE) return oracle_fnv1a(p, n * oracle_type_size(type));
    uint64_t h = 0xcbf29ce484222325ULL;
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < n; ++i)
        for (size_t j = 0; j < 10; ++j) {
            h ^= b[i * sizeof(ldouble) + j];
            h *= 0x100000001b3ULL;
        }
    return h;
}

static double orc_now(void);

/* ------------------------------------------------ the local fold alone -- */
/* The per-peer step of the reference's loop (reduce-op.c:224-245) on its
 * own, write_to = op(write_to, peer) over nreduce elements through the
 * 64-element pWrk staging and the per-element indirect call: the CPU twin of
 * the 1-GPU bench step.  One process, optionally pinned to core `pin`; one
 * warm-up fold, then `reps` timed folds; per-fold seconds to times_out.   */
int oracle_fold_time(int type, int op, int nreduce, int reps, int pin, double *times_out)
{
    orc_kernel_t k;
    if (orc_kernel(type, op, &k) || nreduce < 0 || reps < 1 || reps > 64) return -1;
    cpu_set_t old;
    CPU_ZERO(&old);
    const int have_old = sched_getaffinity(0, sizeof(old), &old) == 0;
    if (pin >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(pin, &set);
        sched_setaffinity(0, sizeof(set), &set);
    }
    const size_t bytes = oracle_type_size(type) * (size_t)nreduce;
    char *acc = malloc(bytes ? bytes : 1), *in = malloc(bytes ? bytes : 1);
    int rc = -1;
    if (acc && in) {
        oracle_fill(type, 0, 0x5EED0000ULL, acc, (size_t)nreduce);
        oracle_fill(type, 0, 0x5EED0001ULL, in, (size_t)nreduce);
        k.fold(k.fn, acc, in, nreduce);                   /* warm-up, first touch */
        for (int r = 0; r < reps; ++r) {
            const double t0 = orc_now();
            k.fold(k.fn, acc, in, nreduce);
            times_out[r] = orc_now() - t0;
        }
        rc = 0;
    }
    free(acc);
    free(in);
    if (pin >= 0 && have_old) sched_setaffinity(0, sizeof(old), &old);
    return rc;
}

/* ------------------------------------------------ fork-per-PE harness ---- */
/* One process per PE, every PE's source/target in one MAP_SHARED mapping, the
 * barrier a process-shared pthread barrier over the active set: the model of
 * the GASNet smp conduit (reference oshrun.in:97-98), where shmem_getmem on a
 * peer is a copy out of that peer's segment.                                */

typedef struct {
    pthread_barrier_t bar;
    double times[64];
    int failed;
} orc_shared_t;

static double orc_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void orc_pe_main(const orc_kernel_t *k, int type, int kind, int me,
                        int is_root, int PE_start, int logPE_stride,
                        int PE_size, int nreduce, char *src_all, char *tgt_all,
                        size_t stride, uint64_t seed, int reps, int pin,
                        orc_shared_t *sh)
{
    if (pin >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(pin, &set);
        sched_setaffinity(0, sizeof(set), &set);
    }
    char *mysrc = src_all + (size_t)me * stride;
    char *mytgt = tgt_all + (size_t)me * stride;
    oracle_fill(type, kind, seed, mysrc, (size_t)nreduce);     /* first touch */
    memset(mytgt, 0, stride);
    pthread_barrier_wait(&sh->bar);
    for (int r = 0; r <= reps; ++r) {
        pthread_barrier_wait(&sh->bar);       /* everyone enters the call */
        const double t0 = orc_now();
        k->copy(mytgt, mysrc, nreduce);                           /* :213-216 */
        pthread_barrier_wait(&sh->bar);                           /* :217     */
        for (int i = 0; i < PE_size; ++i) {                       /* :219-248 */
            const int pe = orc_member(PE_start, logPE_stride, i);
            if (pe == me) continue;
            k->fold(k->fn, mytgt, src_all + (size_t)pe * stride, nreduce);
        }
        pthread_barrier_wait(&sh->bar);                           /* :250     */
        const double t1 = orc_now();
        if (is_root && r > 0 && r - 1 < 64) sh->times[r - 1] = t1 - t0;
    }
}

int oracle_reduce_fork(int type, int op, int npes, int PE_start,
                       int logPE_stride, int PE_size, int nreduce,
                       int fill_kind, uint64_t base_seed, int reps,
                       int pin_base, double *times_out, uint64_t *hashes_out)
{
    orc_kernel_t k;
    if (orc_kernel(type, op, &k) ||
        orc_check_set(npes, PE_start, logPE_stride, PE_size, nreduce) ||
        reps < 1 || reps > 64)
        return -1;
    const size_t stride = oracle_type_size(type) * (size_t)nreduce;
    const size_t seg = stride ? stride : 1;
    char *src = mmap(NULL, seg * (size_t)npes, PROT_READ | PROT_WRITE,
                     MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    char *tgt = mmap(NULL, seg * (size_t)npes, PROT_READ | PROT_WRITE,
                     MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    orc_shared_t *sh = mmap(NULL, sizeof(*sh), PROT_READ | PROT_WRITE,
                            MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (src == MAP_FAILED || tgt == MAP_FAILED || sh == MAP_FAILED) return -1;
    memset(sh, 0, sizeof(*sh));
    pthread_barrierattr_t ba;
    pthread_barrierattr_init(&ba);
    pthread_barrierattr_setpshared(&ba, PTHREAD_PROCESS_SHARED);
    pthread_barrier_init(&sh->bar, &ba, (unsigned)PE_size);
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    if (ncpu < 1) ncpu = 1;

    pid_t pids[1024];
    int nchild = 0, rc = 0;
    for (int m = 0; m < PE_size && m < 1024; ++m) {
        const int me = orc_member(PE_start, logPE_stride, m);
        pid_t pid = fork();
        if (pid < 0) { rc = -1; break; }
        if (pid == 0) {
            const int pin = pin_base >= 0 ? (int)((pin_base + m) % ncpu) : -1;
            orc_pe_main(&k, type, fill_kind, me, m == 0, PE_start,
                        logPE_stride, PE_size, nreduce, src, tgt, stride,
                        base_seed + (uint64_t)me, reps, pin, sh);
            _exit(0);
        }
        pids[nchild++] = pid;
    }
    for (int c = 0; c < nchild; ++c) {
        int st = 0;
        while (waitpid(pids[c], &st, 0) < 0 && errno == EINTR) {}
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = -1;
    }
    if (rc == 0) {
        for (int r = 0; r < reps; ++r) times_out[r] = sh->times[r];
        for (int p = 0; p < npes; ++p) {
            int active = 0;
            for (int m = 0; m < PE_size; ++m)
                active |= orc_member(PE_start, logPE_stride, m) == p;
            hashes_out[p] = active ? orc_hash_elems(type, tgt + (size_t)p * stride,
                                                    (size_t)nreduce)
                                   : 0;
        }
    }
    pthread_barrier_destroy(&sh->bar);
    munmap(src, seg * (size_t)npes);
    munmap(tgt, seg * (size_t)npes);
    munmap(sh, sizeof(*sh));
    return rc;
}
