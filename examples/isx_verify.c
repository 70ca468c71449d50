/*
 * The reference's only known-answer use of the reduction path, rewritten as
 * a stand-alone C99 program against this library: ISx's final verification
 * (reference examples/ISx/SHMEM/isx.c:615-624) sums every PE's bucket size
 * with shmem_longlong_sum_to_all(&total, &my_bucket_size, 1, 0, 0, NUM_PES,
 * llWrk, pSync) and requires total == NUM_KEYS_PER_PE * NUM_PES.
 *
 * Like ISx, the arrays are static (host) variables and pSync is initialised
 * to SHMEM_SYNC_VALUE; the library stages them through the GPU.  With
 * ISX_SHMEM_MALLOC=1 in the environment the arrays are shmem_malloc'd
 * instead and written by host code — under the default (mirrored) heap that
 * is a host view of the HBM heap, and the reductions run device-resident on
 * its HBM twin (the program then prints the mirror's counters).  Exits 0 on
 * success.  Also checks pSync is left at SHMEM_SYNC_VALUE and that a few
 * other entry points (int/double/long xor) agree with the C definition.
 *
 *   cc -std=c99 -Iinclude examples/isx_verify.c -Lopenshmem-async_amd \
 *      -lshmem_reduce_mi355x -Wl,-rpath,$PWD/openshmem-async_amd -o isx_verify
 */
#include <stdio.h>
#include <stdlib.h>

#include "shmem_reduce_mi355x.h"

#define NUM_KEYS_PER_PE 1048576ULL

static long pSync[SHMEM_REDUCE_SYNC_SIZE];
static long long llWrk[SHMEM_REDUCE_MIN_WRKDATA_SIZE];
static long long s_total_num_keys;
static long long s_my_bucket_size;
static double s_dsrc[1000], s_dtgt[1000];
static long s_lsrc[257], s_ltgt[257];

int main(void)
{
    int i, fail = 0;
    for (i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i) pSync[i] = SHMEM_SYNC_VALUE;
    shmem_init();
    const int me = shmem_my_pe(), npes = shmem_n_pes();
    long long *ptotal = &s_total_num_keys, *pmine = &s_my_bucket_size;
    double *dsrc = s_dsrc, *dtgt = s_dtgt;
    long *lsrc = s_lsrc, *ltgt = s_ltgt;
    const char *heap = getenv("ISX_SHMEM_MALLOC");
    if (heap && heap[0] == '1') {   /* symmetric objects from shmem_malloc */
        ptotal = shmem_malloc(sizeof *ptotal);
        pmine = shmem_malloc(sizeof *pmine);
        dsrc = shmem_malloc(1000 * sizeof *dsrc);
        dtgt = shmem_malloc(1000 * sizeof *dtgt);
        lsrc = shmem_malloc(257 * sizeof *lsrc);
        ltgt = shmem_malloc(257 * sizeof *ltgt);
        if (!ptotal || !pmine || !dsrc || !dtgt || !lsrc || !ltgt) {
            printf("PE %d: shmem_malloc failed\n", me);
            return 1;
        }
        *ptotal = 0;
    }
#define total_num_keys (*ptotal)
#define my_bucket_size (*pmine)

    /* every PE holds NUM_KEYS_PER_PE keys, spread unevenly over the buckets */
    my_bucket_size = (long long)NUM_KEYS_PER_PE + (me % 2 ? -(me * 37) : (me + 1) * 37);
    long long expect_extra = 0;
    for (i = 0; i < npes; ++i) expect_extra += (i % 2 ? -(i * 37) : (i + 1) * 37);

    shmem_longlong_sum_to_all(ptotal, pmine, 1, 0, 0, npes, llWrk, pSync);
    if (total_num_keys != (long long)(NUM_KEYS_PER_PE * npes) + expect_extra) {
        printf("PE %d: Verification Failed: total %lld\n", me, total_num_keys);
        fail = 1;
    }

    for (i = 0; i < 1000; ++i) dsrc[i] = 0.25 * i + me;
    shmem_double_sum_to_all(dtgt, dsrc, 1000, 0, 0, npes, NULL, pSync);
    for (i = 0; i < 1000 && !fail; ++i) {
        double want = 0;
        for (int p = 0; p < npes; ++p) want += 0.25 * i + p;  /* exact in binary */
        if (dtgt[i] != want) { printf("PE %d: double sum [%d] %g != %g\n", me, i, dtgt[i], want); fail = 1; }
    }

    for (i = 0; i < 257; ++i) lsrc[i] = (long)(0x9E3779B97F4A7C15ULL * (unsigned long long)(i + 1 + 1000 * me));
    shmem_long_xor_to_all(ltgt, lsrc, 257, 0, 0, npes, NULL, pSync);
    for (i = 0; i < 257 && !fail; ++i) {
        long want = 0;
        for (int p = 0; p < npes; ++p)
            want ^= (long)(0x9E3779B97F4A7C15ULL * (unsigned long long)(i + 1 + 1000 * p));
        if (ltgt[i] != want) { printf("PE %d: long xor [%d]\n", me, i); fail = 1; }
    }

    for (i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i)
        if (pSync[i] != SHMEM_SYNC_VALUE) { printf("PE %d: pSync[%d] changed\n", me, i); fail = 1; }
    if (shmemx_reduce_last_error()) { printf("PE %d: last error %d\n", me, shmemx_reduce_last_error()); fail = 1; }
    if (heap && heap[0] == '1') {
        unsigned long long st[7] = {0, 0, 0, 0, 0, 0, 0};
        shmemx_mirror_stats(st, 7, 0);
        printf("PE %d: mirror write faults %llu read faults %llu flushed %llu fetched %llu settled %llu blocks\n",
               me, st[0], st[1], st[2], st[3], st[6]);
    }
    const long long total = total_num_keys;
    shmem_finalize();
    if (!fail) printf("PE %d of %d: ISx verification passed (total %lld)\n", me, npes, total);
    return fail;
}
