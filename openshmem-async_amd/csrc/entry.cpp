// The 44 drop-in entry points.  Each replaces one
// SHMEM_REDUCE_TYPE_OP(op, name, type) instantiation of the reference
// (/root/reference/src/reduce/reduce-op.c:372-431): same name, same
// signature (src/shmem.h:1412-1648), pshmem_* strong with a weak shmem_*
// alias as with --enable-pshmem (reduce-op.c:275-364).  pWrk and pSync are
// accepted for ABI compatibility and not used: the exchange runs over RCCL,
// not through pWrk, and completion is stream order + a host wait, not the
// pSync barrier, so pSync keeps its SHMEM_SYNC_VALUE contents.
#include <complex>

#include "internal.h"
#include "shmem_reduce_mi355x.h"

namespace shmx {
void reduce_blocking(int type, int op, void *target, const void *source,
                     int nreduce, int start, int logstride, int size);
int reduce_on_stream(int type, int op, void *target, const void *source,
                     int nreduce, int start, int logstride, int size, int algo,
                     void *stream);
void debug_checks(const char *name, const void *target, const void *source);
}  // namespace shmx

#define SHMX_ENTRY(Name, Op, T, TYPE, OPC)                                     \
    void pshmem_##Name##_##Op##_to_all(T *target, T *source, int nreduce,    \
                                       int PE_start, int logPE_stride,       \
                                       int PE_size, T *pWrk, long *pSync)    \
    {                                                                        \
        (void)pWrk;                                                          \
        (void)pSync;                                                         \
        shmx::debug_checks("shmem_" #Name "_" #Op "_to_all", target, source); \
        shmx::reduce_blocking(TYPE, OPC, target, source, nreduce, PE_start,  \
                              logPE_stride, PE_size);                        \
    }                                                                        \
    void shmem_##Name##_##Op##_to_all(T *, T *, int, int, int, int, T *,     \
                                      long *)                                \
        __attribute__((weak, alias("pshmem_" #Name "_" #Op "_to_all")));

#define SHMX_ARITH(Name, T, TYPE)                                              \
    SHMX_ENTRY(Name, sum, T, TYPE, SHMEMX_OP_SUM)                            \
    SHMX_ENTRY(Name, prod, T, TYPE, SHMEMX_OP_PROD)
#define SHMX_LOGIC(Name, T, TYPE)                                              \
    SHMX_ENTRY(Name, and, T, TYPE, SHMEMX_OP_AND)                            \
    SHMX_ENTRY(Name, or, T, TYPE, SHMEMX_OP_OR)                              \
    SHMX_ENTRY(Name, xor, T, TYPE, SHMEMX_OP_XOR)
#define SHMX_MINMAX(Name, T, TYPE)                                             \
    SHMX_ENTRY(Name, min, T, TYPE, SHMEMX_OP_MIN)                            \
    SHMX_ENTRY(Name, max, T, TYPE, SHMEMX_OP_MAX)

extern "C" {

// sum / prod (reduce-op.c:388-405)
SHMX_ARITH(short, short, SHMEMX_TYPE_SHORT)
SHMX_ARITH(int, int, SHMEMX_TYPE_INT)
SHMX_ARITH(long, long, SHMEMX_TYPE_LONG)
SHMX_ARITH(longlong, long long, SHMEMX_TYPE_LONGLONG)
SHMX_ARITH(double, double, SHMEMX_TYPE_DOUBLE)
SHMX_ARITH(float, float, SHMEMX_TYPE_FLOAT)
SHMX_ARITH(longdouble, long double, SHMEMX_TYPE_LONGDOUBLE)
SHMX_ARITH(complexd, std::complex<double>, SHMEMX_TYPE_COMPLEXD)
SHMX_ARITH(complexf, std::complex<float>, SHMEMX_TYPE_COMPLEXF)
// and / or / xor (reduce-op.c:406-417)
SHMX_LOGIC(short, short, SHMEMX_TYPE_SHORT)
SHMX_LOGIC(int, int, SHMEMX_TYPE_INT)
SHMX_LOGIC(long, long, SHMEMX_TYPE_LONG)
SHMX_LOGIC(longlong, long long, SHMEMX_TYPE_LONGLONG)
// max / min (reduce-op.c:418-431)
SHMX_MINMAX(short, short, SHMEMX_TYPE_SHORT)
SHMX_MINMAX(int, int, SHMEMX_TYPE_INT)
SHMX_MINMAX(long, long, SHMEMX_TYPE_LONG)
SHMX_MINMAX(longlong, long long, SHMEMX_TYPE_LONGLONG)
SHMX_MINMAX(double, double, SHMEMX_TYPE_DOUBLE)
SHMX_MINMAX(float, float, SHMEMX_TYPE_FLOAT)
SHMX_MINMAX(longdouble, long double, SHMEMX_TYPE_LONGDOUBLE)

// Fortran forwarders (reference src/fortran/fortran.c:1003-1054): every
// argument by reference, pSync an INTEGER array, the C routine does the work.
#define SHMX_FORTRAN(Op, Fname, Cname, T)                                      \
    void pshmem_##Fname##_##Op##_to_all_(T *target, T *source, int *nreduce, \
                                         int *PE_start, int *logPE_stride,   \
                                         int *PE_size, T *pWrk, int *pSync)  \
    {                                                                        \
        pshmem_##Cname##_##Op##_to_all(target, source, *nreduce, *PE_start,  \
                                       *logPE_stride, *PE_size, pWrk,        \
                                       reinterpret_cast<long *>(pSync));     \
    }                                                                        \
    void shmem_##Fname##_##Op##_to_all_(T *, T *, int *, int *, int *, int *,\
                                        T *, int *)                          \
        __attribute__((weak, alias("pshmem_" #Fname "_" #Op "_to_all_")));

#define SHMX_FORTRAN_REAL(Op)                                                  \
    SHMX_FORTRAN(Op, int2, short, short)                                     \
    SHMX_FORTRAN(Op, int4, int, int)                                         \
    SHMX_FORTRAN(Op, int8, long, long)                                       \
    SHMX_FORTRAN(Op, real4, float, float)                                    \
    SHMX_FORTRAN(Op, real8, double, double)                                  \
    SHMX_FORTRAN(Op, real16, longdouble, long double)
#define SHMX_FORTRAN_INT(Op)                                                   \
    SHMX_FORTRAN(Op, int2, short, short)                                     \
    SHMX_FORTRAN(Op, int4, int, int)                                         \
    SHMX_FORTRAN(Op, int8, long, long)

SHMX_FORTRAN_REAL(sum)
SHMX_FORTRAN_REAL(prod)
SHMX_FORTRAN_REAL(max)
SHMX_FORTRAN_REAL(min)
SHMX_FORTRAN_INT(and)
SHMX_FORTRAN_INT(or)
SHMX_FORTRAN_INT(xor)
SHMX_FORTRAN(sum, comp4, complexf, std::complex<float>)
SHMX_FORTRAN(sum, comp8, complexd, std::complex<double>)
SHMX_FORTRAN(prod, comp4, complexf, std::complex<float>)
SHMX_FORTRAN(prod, comp8, complexd, std::complex<double>)

// Stream-ordered typed forms of all 44 (header Part 3): the error code is
// returned (and left in shmemx_reduce_last_error()).
#define SHMX_STREAM(Name, Op, T, TYPE, OPC)                                    \
    int shmemx_##Name##_##Op##_to_all_on_stream(                             \
        T *target, const T *source, int nreduce, int PE_start,               \
        int logPE_stride, int PE_size, void *stream)                         \
    {                                                                        \
        return shmx::reduce_on_stream(TYPE, OPC, target, source, nreduce,    \
                                      PE_start, logPE_stride, PE_size,       \
                                      SHMEMX_ALGO_AUTO, stream);             \
    }
#define SHMX_STREAM_ARITH(Name, T, TYPE)                                       \
    SHMX_STREAM(Name, sum, T, TYPE, SHMEMX_OP_SUM)                           \
    SHMX_STREAM(Name, prod, T, TYPE, SHMEMX_OP_PROD)
#define SHMX_STREAM_LOGIC(Name, T, TYPE)                                       \
    SHMX_STREAM(Name, and, T, TYPE, SHMEMX_OP_AND)                           \
    SHMX_STREAM(Name, or, T, TYPE, SHMEMX_OP_OR)                             \
    SHMX_STREAM(Name, xor, T, TYPE, SHMEMX_OP_XOR)
#define SHMX_STREAM_MINMAX(Name, T, TYPE)                                      \
    SHMX_STREAM(Name, min, T, TYPE, SHMEMX_OP_MIN)                           \
    SHMX_STREAM(Name, max, T, TYPE, SHMEMX_OP_MAX)
SHMX_STREAM_ARITH(short, short, SHMEMX_TYPE_SHORT)
SHMX_STREAM_ARITH(int, int, SHMEMX_TYPE_INT)
SHMX_STREAM_ARITH(long, long, SHMEMX_TYPE_LONG)
SHMX_STREAM_ARITH(longlong, long long, SHMEMX_TYPE_LONGLONG)
SHMX_STREAM_ARITH(float, float, SHMEMX_TYPE_FLOAT)
SHMX_STREAM_ARITH(double, double, SHMEMX_TYPE_DOUBLE)
SHMX_STREAM_ARITH(longdouble, long double, SHMEMX_TYPE_LONGDOUBLE)
SHMX_STREAM_ARITH(complexd, std::complex<double>, SHMEMX_TYPE_COMPLEXD)
SHMX_STREAM_ARITH(complexf, std::complex<float>, SHMEMX_TYPE_COMPLEXF)
SHMX_STREAM_LOGIC(short, short, SHMEMX_TYPE_SHORT)
SHMX_STREAM_LOGIC(int, int, SHMEMX_TYPE_INT)
SHMX_STREAM_LOGIC(long, long, SHMEMX_TYPE_LONG)
SHMX_STREAM_LOGIC(longlong, long long, SHMEMX_TYPE_LONGLONG)
SHMX_STREAM_MINMAX(short, short, SHMEMX_TYPE_SHORT)
SHMX_STREAM_MINMAX(int, int, SHMEMX_TYPE_INT)
SHMX_STREAM_MINMAX(long, long, SHMEMX_TYPE_LONG)
SHMX_STREAM_MINMAX(longlong, long long, SHMEMX_TYPE_LONGLONG)
SHMX_STREAM_MINMAX(float, float, SHMEMX_TYPE_FLOAT)
SHMX_STREAM_MINMAX(double, double, SHMEMX_TYPE_DOUBLE)
SHMX_STREAM_MINMAX(longdouble, long double, SHMEMX_TYPE_LONGDOUBLE)

}  // extern "C"
