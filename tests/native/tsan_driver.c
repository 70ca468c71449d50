/*
 * Test infrastructure (tests/test_gpu_tsan.py): the library's host code under
 * ThreadSanitizer on one MI355X, driven by several threads of one PE at once.
 * The library is rebuilt with -Xarch_host -fsanitize=thread (tests/native/
 * Makefile, target tsan: host code only; the GPU kernels are the shipped
 * objects).  Worker threads make PE_size 1 calls (reduce-op.c:213-216: a copy,
 * no peer) on their own pageable host arrays (the small-message bounce and
 * the staging ring with its two copy gangs), on their own device arrays
 * through the stream-ordered form on their own streams, and on their own
 * blocks of the mirrored heap (host stores, the call, host loads that fault
 * and fetch through the service thread), while the main thread makes
 * world-set calls.  Every thread checks its results; a TSan report fails the
 * run (halt_on_error).
 *
 *   tsan_driver [threads] [iterations]      prints "ok <cases>"
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "shmem_reduce_mi355x.h"

static long pSync[SHMEM_REDUCE_SYNC_SIZE];
static int me, npes, iters = 6;
static int nfails;
static long ncases;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
/* $TSAN_DRIVER_NEGATIVE: the workers write this word unsynchronised, a race
 * TSan must report (the negative control of tests/test_gpu_tsan.py) */
static volatile long racy;
static int negative;

static void fail(int w, int line, const char *what) {
    pthread_mutex_lock(&mu);
    ++nfails;
    printf("PE %d thread %d FAIL line %d: %s\n", me, w, line, what);
    fflush(stdout);
    pthread_mutex_unlock(&mu);
}

static void count(long k) {
    pthread_mutex_lock(&mu);
    ncases += k;
    pthread_mutex_unlock(&mu);
}

#define CHECK(cond, what)                      \
    do {                                       \
        if (!(cond)) fail(w, __LINE__, what);  \
    } while (0)

#define HEAP_N 65543   /* > 256 KiB of longs: the block-marking path */

struct Work {
    int w;
    long *heap_src, *heap_tgt;   /* this thread's own mirrored-heap blocks */
};

static void *worker(void *arg) {
    struct Work *wk = arg;
    const int w = wk->w;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        fail(w, __LINE__, "stream");
        return NULL;
    }
    const size_t big = ((size_t)20 << 20) / 8 + 5;   /* two staging chunks */
    double *hs = malloc(big * sizeof *hs), *ht = malloc(big * sizeof *ht);
    long *ds = NULL, *dt = NULL;
    const int dn = 50000 + w;
    if (!hs || !ht || hipMalloc((void **)&ds, dn * sizeof *ds) != hipSuccess ||
        hipMalloc((void **)&dt, dn * sizeof *dt) != hipSuccess) {
        fail(w, __LINE__, "allocation");
        return NULL;
    }
    long *dh = malloc(dn * sizeof *dh);
    for (int it = 0; it < iters; ++it) {
        /* pageable host arrays: one bounce-buffer call, one staged call */
        const size_t ns[2] = {1000, it % 3 == 0 ? big : 30001};
        for (int k = 0; k < 2; ++k) {
            const size_t n = ns[k];
            for (size_t i = 0; i < n; ++i) hs[i] = (double)(i * 3 + (size_t)w + (size_t)it);
            memset(ht, 0xff, n * sizeof *ht);
            shmem_double_sum_to_all(ht, hs, (int)n, me, 0, 1, NULL, pSync);
            int ok = 1;
            for (size_t i = 0; i < n && ok; ++i) ok = ht[i] == hs[i];
            CHECK(ok, "host arrays");
        }
        /* device arrays on this thread's own stream */
        for (int i = 0; i < dn; ++i) dh[i] = (long)i * 5 - w - it;
        if (hipMemcpyAsync(ds, dh, dn * sizeof *dh, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemsetAsync(dt, 0, dn * sizeof *dt, s) != hipSuccess) {
            fail(w, __LINE__, "copy");
            break;
        }
        CHECK(shmemx_long_sum_to_all_on_stream(dt, ds, dn, me, 0, 1, s) == 0, "stream form");
        memset(dh, 0, dn * sizeof *dh);
        if (hipMemcpyAsync(dh, dt, dn * sizeof *dh, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            fail(w, __LINE__, "copy back");
            break;
        }
        int ok = 1;
        for (int i = 0; i < dn && ok; ++i) ok = dh[i] == (long)i * 5 - w - it;
        CHECK(ok, "stream form result");
        /* this thread's mirrored-heap blocks: host stores, the call, host loads */
        if (wk->heap_src) {
            for (int i = 0; i < HEAP_N; ++i) wk->heap_src[i] = (long)i * 11 + w * 7 + it;
            shmem_longlong_sum_to_all((long long *)wk->heap_tgt, (long long *)wk->heap_src, HEAP_N, me, 0,
                                      1, NULL, pSync);
            ok = 1;
            for (int i = 0; i < HEAP_N && ok; ++i) ok = wk->heap_tgt[i] == (long)i * 11 + w * 7 + it;
            CHECK(ok, "heap view");
        }
        if (negative) racy = racy + w + 1;
        count(3);
    }
    free(dh);
    (void)hipFree(ds);
    (void)hipFree(dt);
    (void)hipStreamDestroy(s);
    free(hs);
    free(ht);
    return NULL;
}

int main(int argc, char **argv) {
    const int nthreads = argc > 1 ? atoi(argv[1]) : 3;
    if (argc > 2) iters = atoi(argv[2]);
    negative = getenv("TSAN_DRIVER_NEGATIVE") != NULL;
    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i) pSync[i] = SHMEM_SYNC_VALUE;
    shmem_init();
    me = shmem_my_pe();
    npes = shmem_n_pes();
    struct Work wk[16];
    pthread_t th[16];
    const int mirrored = getenv("SHMEMX_HEAP_MEMORY") && !strcmp(getenv("SHMEMX_HEAP_MEMORY"), "mirrored");
    for (int w = 0; w < nthreads && w < 16; ++w) {   /* shmem_malloc is collective: main thread */
        wk[w].w = w;
        wk[w].heap_src = mirrored ? shmem_align(65536, HEAP_N * sizeof(long)) : NULL;
        wk[w].heap_tgt = mirrored ? shmem_align(65536, HEAP_N * sizeof(long)) : NULL;
    }
    int *wsrc = shmem_malloc(1024 * sizeof(int)), *wtgt = shmem_malloc(1024 * sizeof(int));
    for (int w = 0; w < nthreads && w < 16; ++w) pthread_create(&th[w], NULL, worker, &wk[w]);
    const int w = -1;
    for (int c = 0; c < 40; ++c) {   /* world calls while the workers run */
        for (int i = 0; i < 1024; ++i) wsrc[i] = i + me * 1000 + c;
        shmem_int_sum_to_all(wtgt, wsrc, 1024, 0, 0, npes, NULL, pSync);
        int ok = 1;
        for (int i = 0; i < 1024 && ok; ++i) {
            int want = 0;
            for (int p = 0; p < npes; ++p) want += i + p * 1000 + c;
            ok = wtgt[i] == want;
        }
        CHECK(ok, "world call");
        count(1);
    }
    for (int k = 0; k < nthreads && k < 16; ++k) pthread_join(th[k], NULL);
    unsigned long long ms[7] = {0};
    if (mirrored && shmemx_mirror_stats(ms, 7, 0) == 7)   /* the workers' reads faulted and fetched */
        printf("mirror read_faults %llu blocks_fetched %llu\n", ms[1], ms[3]);
    shmem_barrier_all();
    for (int k = 0; k < nthreads && k < 16; ++k) {
        if (wk[k].heap_src) shmem_free(wk[k].heap_src);
        if (wk[k].heap_tgt) shmem_free(wk[k].heap_tgt);
    }
    shmem_free(wsrc);
    shmem_free(wtgt);
    shmem_finalize();
    if (negative) printf("negative control: no report\n");
    if (nfails) return 1;
    printf("ok %ld\n", ncases);
    return 0;
}
