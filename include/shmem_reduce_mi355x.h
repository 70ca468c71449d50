/*
 * shmem_reduce_mi355x.h — C ABI of the MI355X-native OpenSHMEM reduction
 * collectives (libshmem_reduce_mi355x.so).
 *
 * Part 1 declares, with the reference's exact prototypes, the 44
 * shmem_<TYPE>_<OP>_to_all entry points that replace
 * /root/reference/src/reduce/reduce-op.c:372-431 (declared in the reference at
 * src/shmem.h:1412-1648, profiling names src/pshmem.h:328-526).  As with the
 * reference built --enable-pshmem (reduce-op.c:275-364), every pshmem_* name is
 * the strong symbol and every shmem_* name a weak alias of it, so profilers
 * (TAU and friends) can still interpose.
 *
 * Part 2 is the minimum runtime the path needs: the PE identity that
 * GET_STATE(mype)/shmem_my_pe() give the reference (utils/state.h,
 * updown/updown.c:131-184), here one PE = one process = one MI355X.
 *
 * Part 3 holds extensions (shmemx_*): stream-ordered (graph-capturable)
 * forms of the reduction, the local fold kernel on its own, the algorithm
 * selector, the exchange plan query and error reporting.
 *
 * Semantics kept from the reference (see DESIGN.md "Boundary"):
 *   - blocking collective over the active set PE_start + i*2^logPE_stride,
 *     i < PE_size; every member calls with the same arguments;
 *   - target/source may be host memory (as the reference's symmetric heap,
 *     memory/symmem.c:168-227) or device memory; they may be the same array;
 *   - pWrk is accepted and never touched; pSync is never written (so it stays
 *     all SHMEM_SYNC_VALUE, the state barrier-linear.c:75 restores);
 *   - no return value.  Bad arguments (nreduce < 0, caller not in the active
 *     set, ...) leave target untouched and set shmemx_reduce_last_error();
 *     HIP/RCCL failures print a FATAL line and abort, like the reference's
 *     shmemi_trace(SHMEM_LOG_FATAL) (utils/trace.c:424-427).
 */
#ifndef SHMEM_REDUCE_MI355X_H
#define SHMEM_REDUCE_MI355X_H

#include <stddef.h>

#ifdef __cplusplus
#include <complex>
#define SHMEMX_COMPLEX(T) std::complex<T>
extern "C" {
#else
#include <complex.h>
#define SHMEMX_COMPLEX(T) T complex
#endif

/* Constants as the reference defines them on LP64 (shmem.h:1400-1410). */
#ifndef SHMEM_REDUCE_SYNC_SIZE
#define SHMEM_REDUCE_SYNC_SIZE        128L
#define SHMEM_REDUCE_MIN_WRKDATA_SIZE 64L
#define SHMEM_SYNC_VALUE              (-1L)
#endif

/* ------------------------------------------------------------------------ */
/* Part 1: the 44 reduction entry points (shmem.h:1412-1648).               */

#define SHMEMX_DECL_REDUCE(Name, Op, T)                                        \
    void shmem_##Name##_##Op##_to_all(T *target, T *source, int nreduce,     \
                                      int PE_start, int logPE_stride,        \
                                      int PE_size, T *pWrk, long *pSync);    \
    void pshmem_##Name##_##Op##_to_all(T *target, T *source, int nreduce,    \
                                       int PE_start, int logPE_stride,       \
                                       int PE_size, T *pWrk, long *pSync);

#define SHMEMX_DECL_ARITH(Name, T) \
    SHMEMX_DECL_REDUCE(Name, sum, T) SHMEMX_DECL_REDUCE(Name, prod, T)
#define SHMEMX_DECL_LOGIC(Name, T)                                             \
    SHMEMX_DECL_REDUCE(Name, and, T) SHMEMX_DECL_REDUCE(Name, or, T)         \
    SHMEMX_DECL_REDUCE(Name, xor, T)
#define SHMEMX_DECL_MINMAX(Name, T) \
    SHMEMX_DECL_REDUCE(Name, min, T) SHMEMX_DECL_REDUCE(Name, max, T)

/* sum/prod: 9 types (reduce-op.c:388-405) */
SHMEMX_DECL_ARITH(short, short)
SHMEMX_DECL_ARITH(int, int)
SHMEMX_DECL_ARITH(long, long)
SHMEMX_DECL_ARITH(longlong, long long)
SHMEMX_DECL_ARITH(float, float)
SHMEMX_DECL_ARITH(double, double)
SHMEMX_DECL_ARITH(longdouble, long double)
SHMEMX_DECL_ARITH(complexd, SHMEMX_COMPLEX(double))
SHMEMX_DECL_ARITH(complexf, SHMEMX_COMPLEX(float))
/* and/or/xor: 4 integer types (reduce-op.c:406-417) */
SHMEMX_DECL_LOGIC(short, short)
SHMEMX_DECL_LOGIC(int, int)
SHMEMX_DECL_LOGIC(long, long)
SHMEMX_DECL_LOGIC(longlong, long long)
/* min/max: 7 real types (reduce-op.c:418-431) */
SHMEMX_DECL_MINMAX(short, short)
SHMEMX_DECL_MINMAX(int, int)
SHMEMX_DECL_MINMAX(long, long)
SHMEMX_DECL_MINMAX(longlong, long long)
SHMEMX_DECL_MINMAX(float, float)
SHMEMX_DECL_MINMAX(double, double)
SHMEMX_DECL_MINMAX(longdouble, long double)

/* Fortran bindings (reference src/fortran/fortran.c:1003-1054, gfortran
 * name mangling FORTRANIFY(sym) = sym##_): arguments by reference, pSync an
 * INTEGER array; each forwards to the C routine above. */
#define SHMEMX_DECL_FORTRAN(Fname, Op, T)                                      \
    void shmem_##Fname##_##Op##_to_all_(T *target, T *source, int *nreduce,  \
                                        int *PE_start, int *logPE_stride,    \
                                        int *PE_size, T *pWrk, int *pSync);  \
    void pshmem_##Fname##_##Op##_to_all_(T *target, T *source, int *nreduce, \
                                         int *PE_start, int *logPE_stride,   \
                                         int *PE_size, T *pWrk, int *pSync);
#define SHMEMX_DECL_FORTRAN_REAL(Op)                                           \
    SHMEMX_DECL_FORTRAN(int2, Op, short) SHMEMX_DECL_FORTRAN(int4, Op, int)  \
    SHMEMX_DECL_FORTRAN(int8, Op, long) SHMEMX_DECL_FORTRAN(real4, Op, float)\
    SHMEMX_DECL_FORTRAN(real8, Op, double)                                   \
    SHMEMX_DECL_FORTRAN(real16, Op, long double)
#define SHMEMX_DECL_FORTRAN_INT(Op)                                            \
    SHMEMX_DECL_FORTRAN(int2, Op, short) SHMEMX_DECL_FORTRAN(int4, Op, int)  \
    SHMEMX_DECL_FORTRAN(int8, Op, long)
SHMEMX_DECL_FORTRAN_REAL(sum)
SHMEMX_DECL_FORTRAN_REAL(prod)
SHMEMX_DECL_FORTRAN_REAL(max)
SHMEMX_DECL_FORTRAN_REAL(min)
SHMEMX_DECL_FORTRAN_INT(and)
SHMEMX_DECL_FORTRAN_INT(or)
SHMEMX_DECL_FORTRAN_INT(xor)
SHMEMX_DECL_FORTRAN(comp4, sum, SHMEMX_COMPLEX(float))
SHMEMX_DECL_FORTRAN(comp8, sum, SHMEMX_COMPLEX(double))
SHMEMX_DECL_FORTRAN(comp4, prod, SHMEMX_COMPLEX(float))
SHMEMX_DECL_FORTRAN(comp8, prod, SHMEMX_COMPLEX(double))

/* ------------------------------------------------------------------------ */
/* Part 2: runtime (replaces shmem_init updown.c:160, shmem_my_pe/n_pes).   */

/* Bootstrap from the environment: PE = $SHMEM_PE or $RANK, npes =
 * $SHMEM_NPES or $WORLD_SIZE (default 1), device = $LOCAL_RANK or PE mod the
 * visible device count.  With npes > 1 the RCCL unique id is exchanged through
 * the file $SHMEM_BOOTSTRAP_FILE (PE 0 writes it, the others wait for it);
 * launchers that have their own channel should call shmemx_init_attr(). */
void shmem_init(void);
void shmem_finalize(void);
int shmem_my_pe(void);
int shmem_n_pes(void);
void pshmem_init(void);
void pshmem_finalize(void);
int pshmem_my_pe(void);
int pshmem_n_pes(void);

/* ------------------------------------------------------------------------ */
/* Part 2b: the collectives next to the reductions and the symmetric heap   */
/* (SURVEY.md §8f).  Reference prototypes: shmem.h:595-651 (barrier),       */
/* :1654-1684 (broadcast, [f]collect), :821-941 (symmetric heap).  The heap */
/* is one HBM segment per PE; by default shmem_malloc returns addresses in  */
/* a host view of it (the mirrored heap, below), so host code dereferences  */
/* symmetric objects as with the reference's host heap while collectives    */
/* run on HBM.  $SHMEMX_HEAP_MEMORY=device returns the HBM addresses        */
/* themselves (for programs whose own kernels use them); =host makes the    */
/* heap page-locked host memory.                                            */

#ifndef SHMEM_BCAST_SYNC_SIZE
#define SHMEM_BCAST_SYNC_SIZE   64L
#define SHMEM_BARRIER_SYNC_SIZE 64L
#define SHMEM_COLLECT_SYNC_SIZE 64L
#endif

#define SHMEMX_DECL_BOTH(ret, name, args) ret name args; ret p##name args;
SHMEMX_DECL_BOTH(void, shmem_barrier, (int PE_start, int logPE_stride, int PE_size, long *pSync))
SHMEMX_DECL_BOTH(void, shmem_barrier_all, (void))
SHMEMX_DECL_BOTH(void, shmem_broadcast32, (void *target, const void *source, size_t nelems,
                 int PE_root, int PE_start, int logPE_stride, int PE_size, long *pSync))
SHMEMX_DECL_BOTH(void, shmem_broadcast64, (void *target, const void *source, size_t nelems,
                 int PE_root, int PE_start, int logPE_stride, int PE_size, long *pSync))
SHMEMX_DECL_BOTH(void, shmem_fcollect32, (void *target, const void *source, size_t nelems,
                 int PE_start, int logPE_stride, int PE_size, long *pSync))
SHMEMX_DECL_BOTH(void, shmem_fcollect64, (void *target, const void *source, size_t nelems,
                 int PE_start, int logPE_stride, int PE_size, long *pSync))
SHMEMX_DECL_BOTH(void, shmem_collect32, (void *target, const void *source, size_t nelems,
                 int PE_start, int logPE_stride, int PE_size, long *pSync))
SHMEMX_DECL_BOTH(void, shmem_collect64, (void *target, const void *source, size_t nelems,
                 int PE_start, int logPE_stride, int PE_size, long *pSync))
SHMEMX_DECL_BOTH(void *, shmem_malloc, (size_t size))
SHMEMX_DECL_BOTH(void *, shmem_align, (size_t alignment, size_t size))
SHMEMX_DECL_BOTH(void, shmem_free, (void *ptr))
SHMEMX_DECL_BOTH(void *, shmem_realloc, (void *ptr, size_t size))
SHMEMX_DECL_BOTH(void *, shmalloc, (size_t size))
SHMEMX_DECL_BOTH(void, shfree, (void *ptr))
SHMEMX_DECL_BOTH(void *, shrealloc, (void *ptr, size_t size))
SHMEMX_DECL_BOTH(void *, shmemalign, (size_t alignment, size_t size))

/* ------------------------------------------------------------------------ */
/* Part 3: extensions.                                                      */

/* Type and op codes. */
enum {
    SHMEMX_TYPE_SHORT = 0, SHMEMX_TYPE_INT, SHMEMX_TYPE_LONG,
    SHMEMX_TYPE_LONGLONG, SHMEMX_TYPE_FLOAT, SHMEMX_TYPE_DOUBLE,
    SHMEMX_TYPE_LONGDOUBLE, SHMEMX_TYPE_COMPLEXD, SHMEMX_TYPE_COMPLEXF,
    SHMEMX_NTYPES
};
enum {
    SHMEMX_OP_SUM = 0, SHMEMX_OP_PROD, SHMEMX_OP_AND, SHMEMX_OP_OR,
    SHMEMX_OP_XOR, SHMEMX_OP_MIN, SHMEMX_OP_MAX, SHMEMX_NOPS
};

/* Exchange algorithms (DESIGN.md "Multi-GPU").
 *   AUTO    on the whole job RCCL (ALLREDUCE up to 4 MiB) for what RCCL
 *           reduces exactly as specified, A2A otherwise; a partial set takes
 *           A2A ($SHMEMX_AUTO_PARTIAL may name rccl / allreduce: the set's own
 *           communicator, so far run against the RCCL test double only);
 *           float / double / long double min and max take GATHER (below)
 *   RCCL    ncclReduceScatter + ncclAllGather (+ ncclAllReduce on the
 *           <P*16-byte tail); RCCL-native type/op only; the whole job on the
 *           world communicator, a partial set on its own members-only
 *           communicator (made at the set's first RCCL call, cached)
 *   A2A     shard exchange (grouped ncclSend/ncclRecv) -> HIP fold of the P
 *           shards in active-set order -> shard all-gather; any set, any op;
 *           every PE gets the reference's PE_start result bit for bit
 *   GATHER  every PE receives every source and folds in its own reference
 *           order: bit-exact with the reference on EVERY PE, (P-1)x traffic
 *   ALLREDUCE  one ncclAllReduce (RCCL-native pairs, any set, as RCCL)
 *   DIRECT  one HIP kernel per PE reads slice m of every member's source
 *           straight from the peers' HBM (IPC-mapped symmetric heap, over
 *           xGMI) and folds it in active-set order into its own target; a
 *           second kernel pulls the other members' result slices.  Host
 *           barriers around and between (the reference's two plus one).
 *           Any set of <= 16 PEs, any op, PE_start bits on every PE.
 *           Operands outside the symmetric heap are staged through an IPC
 *           scratch region.  Host-synchronous.  Arrays up to 256 KiB
 *           ($SHMEMX_DIRECT_ONESHOT_KB) take one shot: every PE folds the
 *           whole array, as one fused launch (fence, device barriers and
 *           fold in one kernel) when every member has a heap segment.
 *   SIGNAL  DIRECT's pulls with device-side barriers (per-peer counters in
 *           each PE's heap segment, polled over xGMI): no host wait,
 *           stream-ordered, capturable.  Source and target must both be in
 *           the symmetric heap on every member (ENOTSUP otherwise); calls on
 *           one PE must not overlap in time.  The one shot is one fused
 *           launch.  A peer that never arrives
 *           times out after $SHMEMX_SIGNAL_TIMEOUT s (default 20); the next
 *           blocking call then aborts with a FATAL line.
 * With $SHMEMX_TRANSPORT=ipc there is no RCCL communicator: AUTO means
 * DIRECT, GATHER runs as a DIRECT-style kernel in each PE's own order, and
 * RCCL / A2A / ALLREDUCE are ENOTSUP; SIGNAL runs on both transports.
 * Float, double and long double min / max: a<b?a:b under NaN and +-0 gives
 * each PE its own reference answer (reduce-op.c:130-142, 219-248), so on
 * these six pairs every algorithm folds in the calling PE's own order: A2A
 * runs as GATHER, DIRECT and SIGNAL read every member's whole source. */
enum {
    SHMEMX_ALGO_AUTO = 0, SHMEMX_ALGO_RCCL, SHMEMX_ALGO_A2A,
    SHMEMX_ALGO_GATHER, SHMEMX_ALGO_ALLREDUCE, SHMEMX_ALGO_DIRECT, SHMEMX_ALGO_SIGNAL,
    SHMEMX_NALGOS
};

/* Error codes returned by shmemx_* and stored for shmemx_reduce_last_error. */
enum {
    SHMEMX_OK = 0,
    SHMEMX_EINVAL = 1,     /* bad argument (nreduce < 0, bad set, ...)     */
    SHMEMX_ENOTMEMBER = 2, /* calling PE is not in the active set          */
    SHMEMX_ENOTSUP = 3,    /* type/op/algorithm combination not supported  */
    SHMEMX_ENOINIT = 4,    /* runtime not initialised and npes > 1         */
    SHMEMX_ENOMEM = 5,     /* device workspace allocation failed           */
    SHMEMX_EDEVICE = 6     /* HIP or RCCL reported an error                */
};

/* Bootstrap with a caller-distributed RCCL unique id (128 bytes): PE `pe` of
 * `npes` on HIP device `device` (-1: pe mod device count).  PE 0 creates the
 * id with shmemx_get_uniqueid() and the launcher broadcasts it.  The id also
 * names the job's intra-node block (/dev/shm) that carries the symmetric-heap
 * IPC handles and the host barrier; all PEs run on one node.
 * $SHMEMX_TRANSPORT=ipc (set alike on every PE) skips RCCL entirely. */
int shmemx_uniqueid_size(void);
int shmemx_get_uniqueid(void *uid_out);
int shmemx_init_attr(int pe, int npes, int device, const void *uid);
int shmemx_initialized(void);

/* The HIP stream (hipStream_t) the blocking entry points run on. */
void *shmemx_get_stream(void);

/* Algorithm used by the entry points (default AUTO, or $SHMEM_REDUCE_ALGO =
 * auto|rccl|a2a|gather|allreduce|direct).  Returns the previous value. */
int shmemx_set_algo(int algo);

/* Stream-ordered reduction: enqueue on `stream` (hipStream_t; NULL = the
 * runtime's stream) and return without waiting.  Buffers must be device
 * memory.  Capturable into a hipGraph once a call of the same shape has run
 * (workspaces are allocated on first use). */
int shmemx_reduce_on_stream(int type, int op, void *target, const void *source,
                            int nreduce, int PE_start, int logPE_stride,
                            int PE_size, int algo, void *stream);

/* The local element-wise fold, reduce-op.c:231-235 as one HIP kernel:
 *   acc[i] = op(acc[i], in[i])                              (fold2)
 *   out[i] = op(...op(op(ins[0][i], ins[1][i]), ins[2][i])..., ins[nins-1][i])
 * out may alias ins[0].  Device pointers, stream-ordered.  These local folds
 * (and shmemx_gather_on_stream) need no shmem_init and leave the calling
 * thread's current HIP device as it was; with a NULL stream after shmem_init
 * they launch on the PE's device.  Every other entry point makes the PE's
 * device current on the calling thread (hipSetDevice) and leaves it so. */
int shmemx_fold_on_stream(int type, int op, void *acc, const void *in,
                          size_t nelems, void *stream);
int shmemx_fold_n_on_stream(int type, int op, void *out,
                            const void *const *ins, int nins, size_t nelems,
                            void *stream);
/* The same fold for inputs that live in other GPUs' HBM (IPC-mapped peer
 * memory, as DIRECT and SIGNAL read it): every lane issues its loads of all
 * inputs before folding any, so every peer's xGMI link carries traffic at
 * once (the kernel above folds input k before loading input k + 1, which
 * keeps all waves behind one link at a time).  Same results, bit for bit. */
int shmemx_fold_n_peers_on_stream(int type, int op, void *out,
                                  const void *const *ins, int nins, size_t nelems,
                                  void *stream);

/* DIRECT's all-gather step as one launch: nseg (<= 16) byte ranges
 * srcs[i] -> dsts[i] copied concurrently (blockIdx.y = segment), so reads
 * from every peer's HBM are in flight at once.  Device (or IPC-mapped peer)
 * pointers, stream-ordered; ranges must not overlap. */
int shmemx_gather_on_stream(const void *const *srcs, void *const *dsts,
                            const size_t *bytes, int nseg, void *stream);

/* Register (on != 0) or deregister the symmetric heap's HBM segment with
 * the library's RCCL communicator (ncclCommRegister), so RCCL may use
 * collectives' heap operands in place instead of staging them through its
 * own buffers.  Off by default: the N > 1 bench times the RCCL algorithms
 * both ways (extras.rccl_registered) before it is adopted.  A collective over
 * the whole job (the PEs agree with an ncclAllReduce that every one of them
 * registered): every PE must call it, in the same order as the other world
 * collectives, or the callers hang.  ENOTSUP without an RCCL communicator or
 * an HBM segment. */
int shmemx_rccl_register_heap(int on);

/* The kernel clock: with on != 0, every launch of the fold family (the
 * 2-input and P-input folds, the copy of a one-member call, the peers fold,
 * the gather) carries start / stop events of its own dispatch
 * (hipExtLaunchKernelGGL), i.e. the kernel's execution time alone, with no
 * launch boundary and no event-marker latency; up to 4096 launches are
 * timed between reads.  shmemx_kernel_times waits for them and writes up to
 * max durations in microseconds to us[] and their kinds (0 fold, 1 copy,
 * 2 peers fold, 3 gather) to kind[] (may be NULL), in launch order, and the
 * launches past the 4096 that went untimed to *dropped (may be NULL); it
 * returns how many were written and starts over.  Off by default; timing
 * does not change what runs. */
/* The resident service workgroup (DESIGN.md §6 "Small messages"): a
 * blocking one-member call (PE_size 1, a copy) of at most 32 KiB is done by
 * one workgroup that stays on the GPU polling a host-coherent mailbox, with
 * no kernel launch, after the legacy default stream's and the library
 * stream's earlier work (the host waits for them first when they still have
 * some); it leaves after 200 us without a request (so a
 * program's hipDeviceSynchronize waits that long at most) and at
 * shmem_finalize.  A blocking call over several PEs of at most 4 KiB per PE
 * under SHMEMX_ALGO_AUTO is served the same way: each member leaves its
 * source in a page-locked exchange shared by the job's PEs, and after the
 * entry barrier its workgroup folds every member's source into its target
 * (no kernel launch, no GPU reading another GPU's memory); a member writes
 * its part of the exchange again only once the readers of its previous call
 * are done with it.  $SHMEMX_SERVICE=0 turns both off (every PE alike); they are also
 * off when several PE processes of the job share one GPU, unless
 * $SHMEMX_SERVICE=1.  Stats:
 * out[0] requests served, out[1] launches of the workgroup, out[2] / out[3]
 * requests that found the legacy default stream / the library's stream busy
 * and waited for it, out[4] / out[5] nanoseconds summed over the served
 * requests from the check's start to the post / from the post to the result,
 * out[6] folds of the exchange (multi-PE calls); returns how many were
 * written. */
int shmemx_service_stats(unsigned long long *out, int nout, int reset);

int shmemx_kernel_timing(int on);
int shmemx_kernel_times(double *us, int *kind, int max, unsigned long long *dropped);

/* Members-only RCCL communicators this PE holds for partial active sets
 * (PE_start, logPE_stride, PE_size other than the whole job): the RCCL
 * algorithms run on a set's own communicator, made by its members alone at
 * the set's first RCCL call and cached until shmem_finalize.  Returns how
 * many exist; $SHMEMX_SET_COMMS=0 (every PE alike) keeps partial sets on the
 * world communicator's grouped send/recv schedules instead. */
int shmemx_set_comms(void);

/* Largest DIRECT / SIGNAL two-shot call, in KiB, that runs as one fused
 * launch (default $SHMEMX_FUSED_TWOSHOT_KB, else 4096; 0 = never).  Every
 * member of a set must hold the same value when it calls (the members choose
 * their schedules independently).  Returns the previous value, or -1 (and
 * EINVAL) for kb < 0. */
long shmemx_set_fused_twoshot_kb(long kb);

/* How a call would be executed (pure host logic, no device needed). */
typedef struct {
    int algo;          /* resolved SHMEMX_ALGO_* (never AUTO)               */
    int member;        /* index of `pe` in the active set, -1 if none       */
    int nmembers;      /* PE_size                                           */
    int elem_size;     /* bytes per element                                 */
    long long chunk;   /* elements per shard (A2A) / per RCCL shard (RCCL)  */
    long long main;    /* RCCL: elements done by reduce-scatter+all-gather  */
    long long tail;    /* RCCL: elements done by the all-reduce tail        */
    long long ws_bytes;/* device workspace this call needs                  */
} shmemx_plan_t;
int shmemx_reduce_plan(int type, int op, int nreduce, int PE_start,
                       int logPE_stride, int PE_size, int pe, int npes,
                       int algo, shmemx_plan_t *plan);

/* Address of the symmetric object `addr` (in this PE's symmetric heap) as
 * mapped on this PE for PE `pe`'s copy — a device pointer a HIP kernel here
 * can load from / store to over xGMI (the shmem_ptr idea, querying/ptr.c).
 * NULL if `addr` is not in the heap segment or the peer is not mapped.  For a
 * mirrored heap's host-view address: `addr` itself for this PE, NULL for the
 * others (a store into a peer's HBM would go behind that peer's host view);
 * device-side puts take the twin (shmemx_mirror_device_ptr), whose peer
 * addresses this returns, and the receiver calls shmemx_mirror_invalidate on
 * the range after the barrier that orders the puts. */
void *shmemx_heap_ptr(const void *addr, int pe);

/* Mirrored heap (the default; $SHMEMX_HEAP_MEMORY=mirrored): the symmetric
 * heap is HBM and shmem_malloc returns addresses in a host view of it, so
 * host code reads and
 * writes symmetric objects as with the reference's host heap
 * (memory/symmem.c:168-227).  The collectives run on the HBM copy; the view
 * is kept coherent in 64 KiB blocks (page protection: a block the host stored
 * to is copied up when a collective next uses it, a block a collective wrote
 * is copied back when the host next touches it), so only touched blocks
 * cross PCIe.  Host-view addresses must not be handed to HIP calls directly.
 *   shmemx_mirror_device_ptr  the HBM twin of a host-view address (for the
 *                             caller's own kernels), NULL if not in the view;
 *   shmemx_mirror_sync        copy the host's stores in [addr, addr + bytes)
 *                             to HBM now;
 *   shmemx_mirror_invalidate  after the caller's own kernels wrote the HBM
 *                             twin: the host view re-reads it on next access;
 *   shmemx_mirror_acquire     make [addr, addr + bytes) current in the view
 *                             (and, with for_write, writable) now, for code
 *                             that cannot take the page fault: a system call
 *                             given a view address (write(2) of a result,
 *                             read(2) into a source) fails with EFAULT on a
 *                             block the library has not opened;
 *   shmemx_mirror_stats       out[0..6] = write faults, read faults, blocks
 *                             copied to HBM (whole, or a small operand's own
 *                             bytes of them), blocks copied back, blocks
 *                             marked device-newer, faults that waited for a
 *                             collective writing their block, blocks whose
 *                             result a blocking call put into the view
 *                             before returning (up to
 *                             $SHMEMX_MIRROR_SETTLE_KB, default 256 KiB);
 *                             returns how many were filled.
 * A host access to a block a collective is writing waits for it (from any
 * thread), then reads the result; a fetch waits only for the streams that
 * wrote the view (the caller's stream of a stream-ordered call, not the whole
 * device), and its HIP work runs on a service thread, never in the SIGSEGV
 * handler ("Mirrored heap"). */
void *shmemx_mirror_device_ptr(const void *addr);
int shmemx_mirror_sync(const void *addr, size_t bytes);
int shmemx_mirror_invalidate(const void *addr, size_t bytes);
int shmemx_mirror_acquire(const void *addr, size_t bytes, int for_write);
int shmemx_mirror_stats(unsigned long long *out, int nout, int reset);

/* Host-side phase times of the DIRECT algorithm since the last reset, for
 * tuning: out[0] = calls, then microseconds summed over them: [1] waiting for
 * this PE's source (entry fence + stream), [2] entry barrier, [3] fold kernel
 * (reduce-scatter from the peers' HBM), [4] barrier after it, [5] gather
 * kernel (all-gather from the peers' HBM), [6] exit barrier(s); then the
 * system-fence coverage counters (every XCD must run the fence that hands
 * data to the peers): [7] fences checked on the host, [8] of them run again
 * because a block did not reach some XCD, [9] fences checked by the SIGNAL
 * device barrier, [10] of them incomplete (the call fails); [11] one-shot
 * calls (DIRECT or SIGNAL) that ran as one fused launch, [12] two-shot calls
 * that did ($SHMEMX_FUSED_TWOSHOT_KB, default 4096).  Fills at most
 * nout values and returns how many; reset != 0 zeroes the counters. */
int shmemx_direct_stats(double *out, int nout, int reset);

/* Page-lock a host range that will be handed to the entry points — the
 * reference's symmetric heap segment, posix_memalign'd once at start-up
 * (comms-inline.h:752-769) and handed to shmemi_mem_init (:794).  Host
 * targets/sources inside it then take the pinned H2D/reduce/D2H pipeline
 * instead of the pageable bounce ring.  SHMEMX_OK, or SHMEMX_EDEVICE when HIP
 * refuses (the range stays pageable and still works).  Unregister before the
 * range is freed. */
int shmemx_host_register(void *base, size_t bytes);
int shmemx_host_unregister(void *base);

/* Element size in bytes of a SHMEMX_TYPE_* (0 if unknown); 1 if the
 * reference defines shmem_<type>_<op>_to_all (reduce-op.c:388-431);
 * 1 if this build runs that pair on the GPU. */
size_t shmemx_type_size(int type);
int shmemx_op_valid(int type, int op);
int shmemx_op_on_device(int type, int op);

/* Position-aware 64-bit checksum of nelems elements (host or device memory;
 * long double: value bytes only) — XOR over 8-byte words w_j of
 * splitmix64-finalise(w_j + (j+1) * 0x9E3779B97F4A7C15); computed by a gfx950
 * kernel (wave shuffle + LDS partials).  shmemx_verify: collective over the
 * active set, *all_equal = 1 iff every member's target has the same checksum
 * (what the A2A and RCCL algorithms guarantee after a reduction). */
int shmemx_checksum(int type, const void *ptr, size_t nelems, unsigned long long *out);
int shmemx_verify(int type, const void *target, int nreduce, int PE_start,
                  int logPE_stride, int PE_size, int *all_equal);

/* Last error of this thread and its text. */
int shmemx_reduce_last_error(void);
const char *shmemx_reduce_error_string(int err);

/* Last words.  FATAL conditions abort the process, as the reference's
 * SHMEM_LOG_FATAL exits it (trace.c:424-427); so do GPU memory faults (HSA)
 * and a launcher's SIGTERM when another PE died.  A caller holding a result
 * it must not lose registers it here: on SIGABRT, SIGSEGV, SIGBUS, SIGFPE,
 * SIGILL or SIGTERM the text is written to stdout and the process leaves
 * with _exit: exit_code for SIGTERM, 128 + the signal number for the others
 * (a crash stays visible in the exit status).  Calling again replaces the
 * text; NULL uninstalls and restores the previous handlers.  SHMEMX_OK or
 * SHMEMX_ENOMEM. */
int shmemx_set_fatal_note(const char *text, int exit_code);

/* Typed stream-ordered forms of all 44 entry points: shmemx_reduce_on_stream
 * with the type and op in the name, SHMEMX_ALGO_AUTO (or the algorithm set
 * with shmemx_set_algo / $SHMEM_REDUCE_ALGO).  Return SHMEMX_OK or the error
 * code (also left in shmemx_reduce_last_error()). */
#define SHMEMX_DECL_REDUCE_STREAM(Name, Op, T)                                 \
    int shmemx_##Name##_##Op##_to_all_on_stream(                             \
        T *target, const T *source, int nreduce, int PE_start,               \
        int logPE_stride, int PE_size, void *stream);
#define SHMEMX_DECL_STREAM_ARITH(Name, T)                                      \
    SHMEMX_DECL_REDUCE_STREAM(Name, sum, T) SHMEMX_DECL_REDUCE_STREAM(Name, prod, T)
#define SHMEMX_DECL_STREAM_LOGIC(Name, T)                                      \
    SHMEMX_DECL_REDUCE_STREAM(Name, and, T) SHMEMX_DECL_REDUCE_STREAM(Name, or, T) \
    SHMEMX_DECL_REDUCE_STREAM(Name, xor, T)
#define SHMEMX_DECL_STREAM_MINMAX(Name, T)                                     \
    SHMEMX_DECL_REDUCE_STREAM(Name, min, T) SHMEMX_DECL_REDUCE_STREAM(Name, max, T)
SHMEMX_DECL_STREAM_ARITH(short, short)
SHMEMX_DECL_STREAM_ARITH(int, int)
SHMEMX_DECL_STREAM_ARITH(long, long)
SHMEMX_DECL_STREAM_ARITH(longlong, long long)
SHMEMX_DECL_STREAM_ARITH(float, float)
SHMEMX_DECL_STREAM_ARITH(double, double)
SHMEMX_DECL_STREAM_ARITH(longdouble, long double)
SHMEMX_DECL_STREAM_ARITH(complexd, SHMEMX_COMPLEX(double))
SHMEMX_DECL_STREAM_ARITH(complexf, SHMEMX_COMPLEX(float))
SHMEMX_DECL_STREAM_LOGIC(short, short)
SHMEMX_DECL_STREAM_LOGIC(int, int)
SHMEMX_DECL_STREAM_LOGIC(long, long)
SHMEMX_DECL_STREAM_LOGIC(longlong, long long)
SHMEMX_DECL_STREAM_MINMAX(short, short)
SHMEMX_DECL_STREAM_MINMAX(int, int)
SHMEMX_DECL_STREAM_MINMAX(long, long)
SHMEMX_DECL_STREAM_MINMAX(longlong, long long)
SHMEMX_DECL_STREAM_MINMAX(float, float)
SHMEMX_DECL_STREAM_MINMAX(double, double)
SHMEMX_DECL_STREAM_MINMAX(longdouble, long double)

#ifdef __cplusplus
}
#endif
#endif /* SHMEM_REDUCE_MI355X_H */
