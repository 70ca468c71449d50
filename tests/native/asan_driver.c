/*
 * Test infrastructure (tests/test_gpu_asan.py): the whole library's host code
 * under AddressSanitizer on one MI355X.  The library is rebuilt with
 * -Xarch_host -fsanitize=address (tests/native/Makefile, target asan: host
 * code only; the GPU kernels are the shipped objects), and this C program
 * drives its host paths from C as a reference program would: pageable host
 * arrays through the staging pipeline (copy gangs, page-locked ring) and the
 * small-message bounce, device arrays, the mirrored symmetric heap (host view,
 * fault handler, flush / settle), stream-ordered calls with every algorithm,
 * the collectives beside the reductions, checksum / verify, error paths, and
 * finalize.  One process per PE, bootstrapped by shmem_init from the
 * environment (SHMEM_PE / SHMEM_NPES / SHMEM_BOOTSTRAP_FILE).
 *
 * Values are small integers, so every sum is exact in any order and the
 * expected result is computed here without the oracle.  Prints
 * "ok <cases>" on success; a failed check prints a line and exits 1; an ASan
 * report aborts the process.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "shmem_reduce_mi355x.h"

static long pSync[SHMEM_REDUCE_SYNC_SIZE];
static long pSyncB[SHMEM_BCAST_SYNC_SIZE];
static double pWrk[SHMEM_REDUCE_MIN_WRKDATA_SIZE];
static int me, npes, ncases, nfails;

#define CHECK(cond, ...)                                                       \
    do {                                                                       \
        ++ncases;                                                              \
        if (!(cond)) {                                                         \
            ++nfails;                                                          \
            printf("PE %d FAIL line %d: ", me, __LINE__);                      \
            printf(__VA_ARGS__);                                               \
            printf("\n");                                                      \
            fflush(stdout);                                                    \
        }                                                                      \
    } while (0)

#define HIPCK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("PE %d: %s: %s\n", me, #x, hipGetErrorString(e_));          \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

static int member_index(int pe, int start, int logstride, int size) {
    const int step = 1 << logstride;
    if (pe < start || (pe - start) % step) return -1;
    const int m = (pe - start) / step;
    return m < size ? m : -1;
}

/* element i of PE p's source: small non-negative integers */
static long val(int p, size_t i) { return (long)((i * 7 + (size_t)p * 13) % 1000); }

static void fill_double(double *a, int p, size_t n) {
    for (size_t i = 0; i < n; ++i) a[i] = (double)val(p, i);
}

/* the sum over the set's members of val(p, i), as a double */
static int check_double_sum(const double *got, size_t n, int start, int logstride, int size,
                            const char *what) {
    for (size_t i = 0; i < n; ++i) {
        long want = 0;
        for (int m = 0; m < size; ++m) want += val(start + m * (1 << logstride), i);
        if (got[i] != (double)want) {
            printf("PE %d %s: element %zu = %.17g, want %ld\n", me, what, i, got[i], want);
            return 0;
        }
    }
    return 1;
}

/* pageable host arrays: small (bounce buffers), mid and > one 16 MiB staging
 * chunk (the pipelined ring with both copy gangs); out of place, in place,
 * and partially overlapping */
static void host_arrays(int start, int logstride, int size) {
    const size_t sizes[] = {1, 1023, 70001, ((size_t)40 << 20) / 8 + 3};
    for (int k = 0; k < 4; ++k) {
        const size_t n = sizes[k];
        double *src = malloc((n + 8) * sizeof *src), *tgt = malloc(n * sizeof *tgt);
        fill_double(src, me, n);
        memset(tgt, 0xff, n * sizeof *tgt);
        shmem_double_sum_to_all(tgt, src, (int)n, start, logstride, size, pWrk, pSync);
        CHECK(shmemx_reduce_last_error() == 0, "host double sum n=%zu: error %d", n,
              shmemx_reduce_last_error());
        CHECK(check_double_sum(tgt, n, start, logstride, size, "host"), "host double sum n=%zu", n);
        shmem_double_sum_to_all(src, src, (int)n, start, logstride, size, pWrk, pSync);
        CHECK(check_double_sum(src, n, start, logstride, size, "in place"), "in place n=%zu", n);
        fill_double(src, me, n);
        shmem_double_sum_to_all(src + 3, src, (int)n, start, logstride, size, pWrk, pSync);
        CHECK(check_double_sum(src + 3, n, start, logstride, size, "overlap"), "overlap n=%zu", n);
        free(src);
        free(tgt);
    }
    /* 16-byte elements through the staging copies: long double and complex */
    {
        const size_t n = 4099;
        long double *ls = malloc(n * sizeof *ls), *lt = malloc(n * sizeof *lt);
        for (size_t i = 0; i < n; ++i) ls[i] = (long double)val(me, i);
        shmem_longdouble_max_to_all(lt, ls, (int)n, start, logstride, size, (long double *)pWrk, pSync);
        int ok = 1;
        for (size_t i = 0; i < n && ok; ++i) {
            long best = -1;
            for (int m = 0; m < size; ++m) {
                const long v = val(start + m * (1 << logstride), i);
                if (v > best) best = v;
            }
            ok = lt[i] == (long double)best;
        }
        CHECK(ok, "host long double max");
        free(ls);
        free(lt);
    }
}

/* device arrays through the blocking entry point and every algorithm of the
 * stream-ordered one (ENOTSUP accepted where the transport lacks it) */
static void device_arrays(int start, int logstride, int size) {
    const size_t n = 70001;
    long *h = malloc(n * sizeof *h), *back = malloc(n * sizeof *back);
    long *ds, *dt;
    HIPCK(hipMalloc((void **)&ds, n * sizeof *ds));
    HIPCK(hipMalloc((void **)&dt, n * sizeof *dt));
    for (size_t i = 0; i < n; ++i) h[i] = val(me, i) * 1000003L + me;
    HIPCK(hipMemcpy(ds, h, n * sizeof *h, hipMemcpyHostToDevice));
    shmem_long_xor_to_all(dt, ds, (int)n, start, logstride, size, (long *)pWrk, pSync);
    HIPCK(hipMemcpy(back, dt, n * sizeof *back, hipMemcpyDeviceToHost));
    int ok = shmemx_reduce_last_error() == 0;
    for (size_t i = 0; i < n && ok; ++i) {
        long want = 0;
        for (int m = 0; m < size; ++m) {
            const int p = start + m * (1 << logstride);
            want ^= val(p, i) * 1000003L + p;
        }
        ok = back[i] == want;
    }
    CHECK(ok, "device long xor");
    for (int algo = SHMEMX_ALGO_AUTO; algo < SHMEMX_NALGOS; ++algo) {
        if (algo == SHMEMX_ALGO_SIGNAL) continue;   /* heap operands only: below */
        HIPCK(hipMemset(dt, 0, n * sizeof *dt));
        const int rc = shmemx_reduce_on_stream(SHMEMX_TYPE_LONG, SHMEMX_OP_XOR, dt, ds, (int)n, start,
                                               logstride, size, algo, NULL);
        HIPCK(hipDeviceSynchronize());
        if (rc == SHMEMX_ENOTSUP) continue;
        CHECK(rc == 0, "on_stream algo %d: error %d", algo, rc);
        HIPCK(hipMemcpy(back, dt, n * sizeof *back, hipMemcpyDeviceToHost));
        int same = 1;
        for (size_t i = 0; i < n && same; ++i) {
            long want = 0;
            for (int m = 0; m < size; ++m) {
                const int p = start + m * (1 << logstride);
                want ^= val(p, i) * 1000003L + p;
            }
            same = back[i] == want;
        }
        CHECK(same, "on_stream algo %d: wrong result", algo);
    }
    unsigned long long sum1 = 0, sum2 = 0;
    CHECK(shmemx_checksum(SHMEMX_TYPE_LONG, dt, n, &sum1) == 0, "checksum");
    CHECK(shmemx_checksum(SHMEMX_TYPE_LONG, dt, n, &sum2) == 0 && sum1 == sum2, "checksum repeat");
    HIPCK(hipFree(ds));
    HIPCK(hipFree(dt));
    free(h);
    free(back);
}

/* the symmetric heap (mirrored by default: a host view of HBM): host stores,
 * reductions on the HBM twin, host reads; SIGNAL on heap operands; the
 * collectives beside the reductions; realloc / align; a failed call on a
 * host-written target leaves the host's bytes */
static void heap(int start, int logstride, int size) {
    const size_t n = 16411;
    int *s = shmem_malloc(n * sizeof *s), *t = shmem_malloc(n * sizeof *t);
    CHECK(s && t, "shmem_malloc");
    for (size_t i = 0; i < n; ++i) s[i] = (int)val(me, i) - 500;
    if (member_index(me, start, logstride, size) >= 0) {
        shmem_int_max_to_all(t, s, (int)n, start, logstride, size, (int *)pWrk, pSync);
        int ok = shmemx_reduce_last_error() == 0;
        for (size_t i = 0; i < n && ok; ++i) {
            int best = -1000;
            for (int m = 0; m < size; ++m) {
                const int v = (int)val(start + m * (1 << logstride), i) - 500;
                if (v > best) best = v;
            }
            ok = t[i] == best;
        }
        CHECK(ok, "heap int max");
        /* SIGNAL, stream-ordered: on a mirrored heap on the HBM twins (the
         * host's stores go up first, the view re-reads the result), on a
         * device heap on the objects themselves */
        void *dsrc = shmemx_mirror_device_ptr(s), *dtgt = shmemx_mirror_device_ptr(t);
        const int mirrored = dsrc != NULL && dtgt != NULL;
        if (!mirrored) {
            dsrc = s;
            dtgt = t;
        }
        memset(t, 0, n * sizeof *t);
        if (mirrored)
            CHECK(shmemx_mirror_sync(s, n * sizeof *s) == 0 && shmemx_mirror_sync(t, n * sizeof *t) == 0,
                  "mirror_sync");
        const int rc = shmemx_reduce_on_stream(SHMEMX_TYPE_INT, SHMEMX_OP_SUM, dtgt, dsrc, (int)n, start,
                                               logstride, size, SHMEMX_ALGO_SIGNAL, NULL);
        HIPCK(hipDeviceSynchronize());
        const char *hm = getenv("SHMEMX_HEAP_MEMORY");
        if (hm && !strcmp(hm, "host")) {
            /* page-locked host objects: the stream-ordered form takes device
             * memory only (EINVAL) */
            CHECK(rc == SHMEMX_EINVAL || rc == SHMEMX_ENOTSUP, "signal on a host heap: error %d", rc);
        } else if (rc != SHMEMX_ENOTSUP) {
            CHECK(rc == 0, "signal on heap: error %d", rc);
            if (mirrored) CHECK(shmemx_mirror_invalidate(t, n * sizeof *t) == 0, "mirror_invalidate");
            int sok = 1;
            for (size_t i = 0; i < n && sok; ++i) {
                int want = 0;
                for (int m = 0; m < size; ++m) want += (int)val(start + m * (1 << logstride), i) - 500;
                sok = t[i] == want;
            }
            CHECK(sok, "signal on heap: wrong result");
        }
    }
    shmem_barrier_all();

    /* a failed call (PE_size past the job) on a host-written 64 KiB target */
    const size_t nf = 65536 / sizeof(long);
    long *ft = shmem_malloc(nf * sizeof *ft), *fs = shmem_malloc(nf * sizeof *fs);
    for (size_t i = 0; i < nf; ++i) {
        ft[i] = (long)i ^ 0x5a5a;
        fs[i] = (long)i;
    }
    shmem_long_sum_to_all(ft, fs, (int)nf, 0, 0, npes + 1, (long *)pWrk, pSync);
    CHECK(shmemx_reduce_last_error() == SHMEMX_EINVAL, "bad set: error %d", shmemx_reduce_last_error());
    int kept = 1;
    for (size_t i = 0; i < nf && kept; ++i) kept = ft[i] == ((long)i ^ 0x5a5a);
    CHECK(kept, "failed call changed the host's target bytes");
    shmem_barrier_all();

    /* broadcast / fcollect over the whole job */
    long *b = shmem_malloc(1025 * sizeof *b), *c = shmem_malloc((size_t)npes * 257 * sizeof *c);
    for (int i = 0; i < 1025; ++i) b[i] = me == 0 ? i * 3 : -1;
    for (int i = 0; i < 257; ++i) c[(size_t)me * 257 + i] = 0;
    long *bt = shmem_malloc(1025 * sizeof *bt), *cs = shmem_malloc(257 * sizeof *cs);
    for (int i = 0; i < 257; ++i) cs[i] = me * 1000 + i;
    shmem_broadcast64(bt, b, 1025, 0, 0, 0, npes, pSyncB);
    int bok = 1;
    if (me != 0)
        for (int i = 0; i < 1025 && bok; ++i) bok = bt[i] == i * 3;
    CHECK(bok, "broadcast64");
    shmem_barrier_all();
    shmem_fcollect64(c, cs, 257, 0, 0, npes, pSyncB);
    int cok = 1;
    for (int p = 0; p < npes && cok; ++p)
        for (int i = 0; i < 257 && cok; ++i) cok = c[(size_t)p * 257 + i] == p * 1000 + i;
    CHECK(cok, "fcollect64");
    shmem_barrier_all();

    /* realloc keeps the contents; align honours the alignment */
    int *r = shmem_realloc(s, 2 * n * sizeof *r);
    int rok = r != NULL;
    for (size_t i = 0; i < n && rok; ++i) rok = r[i] == (int)val(me, i) - 500;
    CHECK(rok, "shmem_realloc");
    void *al = shmem_align(4096, 1000);
    CHECK(al && ((size_t)al & 4095) == 0, "shmem_align");
    shmem_barrier_all();
    shmem_free(al);
    shmem_free(r);
    shmem_free(t);
    shmem_free(ft);
    shmem_free(fs);
    shmem_free(b);
    shmem_free(c);
    shmem_free(bt);
    shmem_free(cs);
}

int main(void) {
    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i) pSync[i] = SHMEM_SYNC_VALUE;
    for (int i = 0; i < SHMEM_BCAST_SYNC_SIZE; ++i) pSyncB[i] = SHMEM_SYNC_VALUE;
    shmem_init();
    me = shmem_my_pe();
    npes = shmem_n_pes();

    /* $ASAN_DRIVER_NEGATIVE=1: the negative control — a host source array
     * shorter than nreduce, so the library's own staging copy reads past
     * it; ASan must report a heap-buffer-overflow from inside the library */
    if (getenv("ASAN_DRIVER_NEGATIVE")) {
        double *shortsrc = malloc(100 * sizeof *shortsrc), *tgt = malloc(1000 * sizeof *tgt);
        fill_double(shortsrc, me, 100);
        shmem_double_sum_to_all(tgt, shortsrc, 1000, 0, 0, npes, pWrk, pSync);
        printf("negative control: no report\n");
        free(shortsrc);
        free(tgt);
        return 2;
    }

    /* the whole job, then (3 PEs and up) a strided partial set whose
     * non-members skip the call, as in the reference's active-set walk */
    host_arrays(0, 0, npes);
    device_arrays(0, 0, npes);
    if (npes >= 3) {
        const int size = (npes + 1) / 2;
        if (member_index(me, 0, 1, size) >= 0) {
            host_arrays(0, 1, size);
            device_arrays(0, 1, size);
        }
        shmem_barrier_all();
    }
    heap(0, 0, npes);
    if (npes >= 3) heap(0, 1, (npes + 1) / 2);

    for (int i = 0; i < SHMEM_REDUCE_SYNC_SIZE; ++i)
        CHECK(pSync[i] == SHMEM_SYNC_VALUE, "pSync[%d] = %ld after the calls", i, pSync[i]);
    shmem_barrier_all();
    shmem_finalize();
    if (nfails) {
        printf("PE %d: %d of %d checks failed\n", me, nfails, ncases);
        return 1;
    }
    printf("ok %d\n", ncases);
    return 0;
}
