/* Per-call wall time of a blocking reduction entry point, called from C
 * (measurement infrastructure for bench.py's small-message extras): the
 * caller passes the address of shmem_<T>_<op>_to_all (the library's own
 * export, resolved by the caller), and this loop calls it `reps` times with
 * the same arguments, timing each call with CLOCK_MONOTONIC.  It removes the
 * Python caller's ~3 us per call from the library's latency figures; it calls
 * nothing but the entry point it is given.  Built by tools/Makefile as
 * libcalltimer.so (gcc, no HIP). */
#define _POSIX_C_SOURCE 199309L
#include <time.h>

typedef void (*to_all_fn)(void *target, const void *source, int nreduce, int PE_start,
                          int logPE_stride, int PE_size, void *pWrk, long *pSync);

static double now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e6 + (double)ts.tv_nsec * 1e-3;
}

/* out_us[i] = microseconds of call i, i < reps; `warm` untimed calls first. */
int call_timer_to_all(void *fn, void *target, const void *source, int nreduce, int PE_start,
                      int logPE_stride, int PE_size, void *pWrk, long *pSync, int warm, int reps,
                      double *out_us) {
    to_all_fn f = (to_all_fn)fn;
    if (!f || reps < 0 || warm < 0 || (reps > 0 && !out_us)) return -1;
    for (int i = 0; i < warm; ++i) f(target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync);
    for (int i = 0; i < reps; ++i) {
        const double t0 = now_us();
        f(target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync);
        out_us[i] = now_us() - t0;
    }
    return 0;
}
