/*
 * TEST INFRASTRUCTURE ONLY — never linked into, loaded by, or called from the
 * product (openshmem-async_amd/).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / the timed
 * CPU baseline.
 *
 * CPU restatement of the reference's reduction algorithm
 * (/root/reference/src/reduce/reduce-op.c).  See reduce_oracle.c for the
 * per-function citations and DESIGN.md "Oracle" for how it is pinned.
 */
#ifndef REDUCE_ORACLE_H
#define REDUCE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Numbering is shared by convention with include/shmem_reduce_mi355x.h
 * (SHMEMX_TYPE_* / SHMEMX_OP_*); tests assert the two agree. */
enum {
    ORC_SHORT = 0, ORC_INT, ORC_LONG, ORC_LONGLONG, ORC_FLOAT, ORC_DOUBLE,
    ORC_LONGDOUBLE, ORC_COMPLEXD, ORC_COMPLEXF, ORC_NTYPES
};
enum { ORC_SUM = 0, ORC_PROD, ORC_AND, ORC_OR, ORC_XOR, ORC_MIN, ORC_MAX, ORC_NOPS };

/* _SHMEM_REDUCE_MIN_WRKDATA_SIZE on LP64 (shmem.h:1400-1405,2046). */
#define ORC_WRKDATA 64

size_t oracle_type_size(int type);
/* 1 if the reference defines shmem_<type>_<op>_to_all (reduce-op.c:388-431). */
int oracle_op_valid(int type, int op);

/*
 * Simulate every PE of the active set (PE_start, logPE_stride, PE_size) on a
 * machine of npes PEs calling shmem_<type>_<op>_to_all at once.
 *   sources : npes * nreduce elements, PE p's source at p * nreduce
 *   targets : npes * nreduce elements, PE p's target at p * nreduce;
 *             written only for PEs in the active set (like the reference)
 * Returns 0, or -1 on invalid arguments.
 */
int oracle_reduce_sim(int type, int op, int npes, int PE_start,
                      int logPE_stride, int PE_size, int nreduce,
                      const void *sources, void *targets);
/* PE `pe`'s target alone (a member of the set), as oracle_reduce_sim
 * computes it. */
int oracle_reduce_one(int type, int op, int npes, int PE_start, int logPE_stride,
                      int PE_size, int nreduce, const void *sources, int pe, void *target);

/*
 * The same algorithm run as one forked process per PE over MAP_SHARED
 * segments (the GASNet smp/PSHM model, reference oshrun.in:97-98): this is the
 * timed CPU baseline.  Each PE's source is filled from splitmix64 (see
 * oracle_fill) with seed base_seed + pe.  Runs `reps` timed calls after one
 * warm-up call; writes PE PE_start's per-call wall times (seconds) to
 * times_out[0..reps-1] and a 64-bit FNV-1a hash of every active PE's final
 * target into hashes_out[0..npes-1] (0 for inactive PEs).
 * pin_base >= 0 pins PE p to core (pin_base + p) % ncpu.
 * Returns 0 on success.
 */
/*
 * The reference's per-peer fold step alone (reduce-op.c:224-245): acc =
 * op(acc, in) over nreduce elements with the 64-element pWrk staging and an
 * indirect call per element, in this process (pinned to core `pin` if >= 0).
 * One warm-up fold, then `reps` timed folds (seconds each) to times_out.
 */
int oracle_fold_time(int type, int op, int nreduce, int reps, int pin, double *times_out);

int oracle_reduce_fork(int type, int op, int npes, int PE_start,
                       int logPE_stride, int PE_size, int nreduce,
                       int fill_kind, uint64_t base_seed, int reps,
                       int pin_base, double *times_out, uint64_t *hashes_out);

/* The neighbouring collectives, byte-level restatements.
 * PE p's source at sources + p * src_stride, PE p's target at
 * targets + p * tgt_stride (bytes).  Only members' targets are written.     */
/* broadcast-linear.c:54-74: every member but the root receives the root's
 * nelems * esize bytes; the root's target is left alone. */
int oracle_broadcast_sim(size_t esize, int npes, int PE_root, int PE_start,
                         int logPE_stride, int PE_size, size_t nelems,
                         const void *sources, size_t src_stride,
                         void *targets, size_t tgt_stride);
/* fcollect-linear.c:69-91 (nelems equal on all PEs) and collect-linear.c:
 * 57-130 (per-PE nelems[p]): member i's source lands at the running byte
 * offset sum_{j<i} nelems[member j] * esize of every member's target. */
int oracle_collect_sim(size_t esize, int npes, int PE_start, int logPE_stride,
                       int PE_size, const size_t *nelems, const void *sources,
                       size_t src_stride, void *targets, size_t tgt_stride);

/* splitmix64 stream: word i of seed s = splitmix64 output number i+1. */
uint64_t oracle_splitmix64(uint64_t seed, uint64_t i);
/* Fill `n` elements of `type` from splitmix64(seed, i).  fill_kind:
 *   0 = "positive"  (floats uniform [1,2); ints small: [-2^20, 2^20) for
 *                    int/long/longlong, [-2^10,2^10) for short)
 *   1 = "mixed"     (floats uniform [-1,1); ints full-width bit patterns) */
void oracle_fill(int type, int fill_kind, uint64_t seed, void *dst, size_t n);

uint64_t oracle_fnv1a(const void *p, size_t nbytes);

#ifdef __cplusplus
}
#endif
#endif
