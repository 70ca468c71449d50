// Runtime state shared by runtime.cpp (init, planner, reductions) and
// collectives.cpp (barrier, broadcast, [f]collect, symmetric heap).
// Internal to libshmem_reduce_mi355x.so.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "node.h"
#include "shmem_reduce_mi355x.h"

#include <chrono>
#include <mutex>
#include <utility>
#include <vector>

namespace shmx {

struct State {
    bool inited = false;
    int pe = 0;
    int npes = 1;
    int device = 0;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    int algo = SHMEMX_ALGO_AUTO;
    // $SHMEMX_TRANSPORT=ipc: no RCCL communicator; every collective runs over
    // the node block and IPC-mapped HBM (node.h, direct.cpp)
    bool ipc_only = false;
    // every PE of the job has the intra-node block: agreed once at init (an
    // RCCL all-reduce of each PE's attach result on the RCCL transport; on the
    // IPC transport a PE without it is fatal).  AUTO's plan reads this, never
    // per-process state, so every PE plans alike.
    bool node_shared = false;
    bool xchg = false;   // every PE mapped the small-call exchange (node.h), agreed at init
    // another PE process of the job uses this GPU (node::gpu_shared): the
    // service workgroup stays off unless $SHMEMX_SERVICE=1 (service.hip)
    bool gpu_shared = false;
    // a mirrored-heap source's current host-view bytes, for the exchange
    // (staging.cpp reduce_blocking; its HBM twin is not flushed)
    const void *xchg_src_host = nullptr;
    // the heap segment registered with the RCCL communicator
    // (shmemx_rccl_register_heap), or nullptr
    void *rccl_reg = nullptr;
    // a registration was refused (on any PE; agreed): not tried again
    bool rccl_reg_refused = false;
    // test hook ($SHMEMX_FORCE_COLLECTIVE=1): a 1-PE job still builds an RCCL
    // communicator and runs the collective schedules, so a one-GPU box can
    // execute every RCCL call of the path
    bool force_collective = false;
    // inside a blocking entry point: wait_host_signal returns as soon as the
    // work's host signal arrives, without seeing the stream idle
    bool return_on_signal = false;
    // the library stream may hold work nobody has waited for: a
    // stream-ordered call enqueued on it (cleared when a blocking call's own
    // work on it, enqueued behind, has been seen complete), or the stream was
    // handed out (shmemx_get_stream: anything may be on it).  Otherwise every
    // piece of work on it has completed, and the service workgroup
    // (service.hip) need not ask the runtime, whose answer lags a kernel's
    // completion by microseconds.
    bool lib_stream_dirty = false;
    bool lib_stream_exported = false;
    // inside a blocking call on a small host-view target (staging.cpp): the
    // device address where the call's last kernel also stores the result (the
    // view's page-locked alias, heap.h DeviceWrite::settle_dst), and whether
    // it did, before the host signal
    void *settle_dst = nullptr;
    bool settled = false;
    // grow-only device workspaces
    void *ws = nullptr;        // A2A shard receive area / GATHER sources
    size_t ws_bytes = 0;
    void *tmp = nullptr;       // overlap temporary (reduce-op.c:187-203)
    size_t tmp_bytes = 0;
    void *stage_src = nullptr; // host-resident endpoints
    void *stage_tgt = nullptr;
    size_t stage_bytes = 0;
    hipEvent_t ws_event = nullptr;  // last use of ws/tmp, on stream ws_stream
    hipStream_t ws_stream = nullptr;
    void *token = nullptr;     // barrier tokens / collect counts
    size_t token_bytes = 0;
    void *cws_src = nullptr;   // staging for host buffers of the other collectives
    size_t cws_src_bytes = 0;
    void *cws_tgt = nullptr;
    size_t cws_tgt_bytes = 0;
    void *ring = nullptr;      // page-locked bounce ring (large pageable arrays)
    size_t ring_slot = 0;
    void *bounce = nullptr;    // page-locked host bounce buffers (small messages)
    size_t bounce_bytes = 0;
    hipStream_t h2d = nullptr;  // staging copy streams and their chunk events
    hipStream_t d2h = nullptr;
    std::vector<hipEvent_t> events;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
};

extern State g_state;
extern std::recursive_mutex g_mu;   // the reference's state is not thread-safe either

int set_error(int e);               // thread-local last error (shmemx_reduce_last_error)
void clear_error();
// Trace facilities ($SHMEM_LOG_LEVELS, $SHMEM_LOG_FILE; utils/trace.c) and
// the "%-8.8f PE %d: LEVEL: msg" line of utils/trace.c:400-431.
enum { LOG_FATAL = 0, LOG_INIT, LOG_BARRIER, LOG_BROADCAST, LOG_REDUCTION, LOG_COLLECT,
       LOG_MEMORY, LOG_INFO, LOG_N };
bool log_enabled(int level);
void trace(int level, const char *fmt, ...);
[[noreturn]] void fatal(const char *what, const char *detail);

#define SHMX_HIP(call)                                                         \
    do {                                                                     \
        hipError_t e_ = (call);                                              \
        if (e_ != hipSuccess) ::shmx::fatal(#call, hipGetErrorString(e_));   \
    } while (0)
#define SHMX_NCCL(call)                                                        \
    do {                                                                     \
        ncclResult_t r_ = (call);                                            \
        if (r_ != ncclSuccess) ::shmx::fatal(#call, ncclGetErrorString(r_)); \
    } while (0)

int ensure_init();                  // single-PE auto-init; ENOINIT if npes > 1
// HIP's current device is per host thread, and the library makes streams,
// events and workspaces lazily on whatever thread calls it: every entry point
// (through ensure_init) and the mirrored heap's service thread make the PE's
// device current first, so a thread other than shmem_init's does not make
// them on device 0 (one PE per GPU: LOCAL_RANK > 0 is never device 0).
void bind_device();
// Members-only RCCL communicators of partial active sets (set_comm.cpp):
// set_comm returns the set's cached communicator, creating it first (a
// collective over the set's members alone: `member` is this PE's index in it)
// if this is the set's first RCCL call.  $SHMEMX_SET_COMMS=0 turns them off.
bool set_comms_enabled();
bool set_comm_cached(int start, int logstride, int size);
int set_comms_cached();
ncclComm_t set_comm(int start, int logstride, int size, int member, hipStream_t s);
// Before a set's first RCCL call: the members agree (every member has room
// under $SHMEMX_SET_COMMS_MAX) and make the communicator; false = refused,
// alike on every member, and remembered (set_comm_refused).
bool set_comm_prepare(int start, int logstride, int size, int member, hipStream_t s);
bool set_comm_refused(int start, int logstride, int size);
void set_comms_release();
// memcpy split over the staging pool's CPU threads (staging.cpp); a caller
// that finds the pool busy copies alone (the mirrored heap's fault handler
// uses it too)
// nt: streaming (non-temporal) stores, for a destination nothing reads soon
void parallel_copy(void *dst, const void *src, size_t bytes, bool nt = false);
void ring_free();   // the staging ring (staging.cpp), at finalize
int gpu_numa_node(int device);   // NUMA node of a HIP device's PCI function, or -1
// The resident service workgroup (service.hip): a small one-member blocking
// call's copy (reduce-op.c:213-216) done by a workgroup that is already on
// the GPU, polling a host-coherent mailbox, instead of a launch.  dst2: a
// second destination or null.  Ordered after the legacy and the library
// stream (waits for them on the host when they still have work).  false =
// not taken ($SHMEMX_SERVICE=0, or no mailbox): the caller launches.
constexpr size_t kServiceMaxBytes = size_t(32) << 10;
bool service_copy(void *dst, void *dst2, const void *src, size_t bytes);
// Small multi-PE blocking calls (staging.cpp): every member has left its
// source in its exchange slot (node.h) and passed the entry barrier; the
// service workgroup folds the members' slots, in the calling PE's own order
// or PE_start's, into dst (and dst2 if not null).  Aborts if the workgroup
// cannot be reached (the members decided on this path together).
bool service_available();   // $SHMEMX_SERVICE is not 0
void service_fold(int type, int op, bool own_order, int start, int logstride, int size, void *dst, void *dst2,
                  size_t bytes);
void service_quiesce();   // the workgroup leaves now, if it is up
void service_release();   // shmem_finalize (and at exit)
void device_sync();       // service_quiesce, then hipDeviceSynchronize
// The plan of one call (shmemx_reduce_plan) and the device-resident engine
// (runtime.cpp); the host staging of the blocking entry points (staging.cpp)
// runs the engine chunk by chunk.
int make_plan(int type, int op, int nreduce, int start, int logstride, int size, int pe, int npes,
              int algo, shmemx_plan_t *p);
int reduce_device(int type, int op, void *target, const void *source, int nreduce, int start,
                  int logstride, int size, int algo, hipStream_t s);
bool overlap(const void *a, const void *b, size_t bytes);   // distinct, overlapping ranges
// reduce-op.c:199-210's REDUCTION trace line for the caller's arrays
void trace_reference_overlap(const void *target, const void *source, size_t bytes);
bool is_member(int pe, int start, int logstride, int size, int *index);
bool device_accessible(const void *ptr);
bool host_pinned(const void *ptr);
void *grow(void *&buf, size_t &have, size_t need);   // grow-only device buffer
bool stream_capturing(hipStream_t s);
// The workspaces (ws, tmp) serve every stream: a use on stream s first waits
// for the last use when that was on another stream, and records itself.
void ws_acquire(hipStream_t s);
void ws_release(hipStream_t s);
// min / max of float, double, long double: the reference's answer depends on
// the calling PE's own fold order (runtime.cpp), so every multi-PE algorithm
// folds these in that order
bool own_order_pair(int type, int op);
// out = left fold of ins[0..nins) in groups of kMaxFoldInputs (any nins);
// peers: the inputs are in other GPUs' HBM (launch_fold_peers)
void fold_chain(int type, int op, void *out, const void **ins, int nins, size_t n, hipStream_t s,
                bool peers = false);
// DIRECT algorithm (direct.cpp); own_order: every PE folds in its own
// reference order (GATHER semantics on the IPC transport)
int direct_reduce(int type, int op, char *tgt, const char *src, int nreduce, int start,
                  int logstride, const shmemx_plan_t &p, bool own_order, hipStream_t s);
void direct_release();
// This PE's IPC scratch region (allocated and published on first use).
char *ipc_scratch(size_t *bytes);
// System-scope fence on every XCD (launch_sys_fence), then wait for stream s;
// a fence whose blocks did not reach every XCD of the device is run again
// (logged under SHMEM_LOG_LEVELS=info; counted in shmemx_direct_stats).
void fence_and_wait(hipStream_t s);
// The device-side fence records and counters the SIGNAL barrier checks.
struct SignalArgs;   // internal.h
struct FenceRecords {
    unsigned int *seen;
    int nxcc;
    unsigned long long *stats;
    unsigned int *gsync;   // the fused one-shot kernel's grid barrier (2 words)
};
FenceRecords fence_records();
// SignalArgs for the members of a set over their mapped heap segments (the
// signal counters at heap::signal_offset()); false if this PE has no heap
// segment or a member's segment is not mapped.
bool signal_args(int start, int step, int P, SignalArgs *sa);
// A one-shot reduction as one fused launch (launch_signal_fold): count it in
// shmemx_direct_stats.
void count_fused_call();
// A two-shot reduction as one fused launch (launch_signal_fold, two_shot):
// counted apart in shmemx_direct_stats.
void count_fused_twoshot_call();
// $SHMEMX_FUSED_ONESHOT=0 turns the fused one-shot launch off (DIRECT's and
// SIGNAL's one shot then take their multi-launch schedules); default on.
bool fused_oneshot_enabled();
// Two-shot calls up to this many bytes run as one fused launch
// ($SHMEMX_FUSED_TWOSHOT_KB, default 4 MiB; 0 turns it off).
size_t fused_twoshot_bytes();
long set_fused_twoshot_kb(long kb);   // shmemx_set_fused_twoshot_kb; returns the previous value
// Hand data between the members' GPUs: fence_and_wait, then the host barrier
// over the set.
// Optionally adds the time spent waiting for the stream (from since_us, a
// steady-clock stamp in microseconds, if >= 0) and in the barrier.
void node_sync(int start, int step, int P, hipStream_t s, double *stream_us = nullptr,
               double *barrier_us = nullptr, double since_us = -1);
// The end of a pull phase: this PE's kernels have finished reading the
// peers' arrays (hipStreamSynchronize, no fence: nothing is handed over —
// the next phase that publishes data runs node_sync, whose fence also drops
// any peer lines this PE's L2 still holds), then the host barrier.
void node_done(int start, int step, int P, hipStream_t s, double *stream_us = nullptr,
               double *barrier_us = nullptr, double since_us = -1);
// Map the peers' regions a collective reads (node::peer_base), voting across
// the set the first time a combination is met; false on every member alike
// if any member failed (direct.cpp).
bool map_regions(const std::vector<std::pair<node::Region, int>> &regs, int start, int step, int P);
// SIGNAL algorithm (signal.cpp): DIRECT's pulls with device-side barriers,
// stream-ordered and graph-capturable; symmetric-heap operands only.
// own_order: every member folds the whole array in its own reference order.
int signal_reduce(int type, int op, char *tgt, const char *src, int nreduce, int start,
                  int logstride, const shmemx_plan_t &p, bool own_order, hipStream_t s);
// After the stream has drained: 0, or 1 if a SIGNAL barrier timed out, 2 if
// a fence before one missed an XCD.  (Clears it.)
unsigned int signal_error();
// The host-mapped error word the device barriers set, and their timeout in
// s_memrealtime ticks ($SHMEMX_SIGNAL_TIMEOUT).
unsigned int *signal_error_word();
unsigned long long signal_timeout_ticks();
// Every member's 8-byte value in set order: a collective over the active set
// (collectives.cpp; RCCL all-gather / grouped p2p, or the node block's
// descriptors on the IPC transport).  Validates the set like a call would.
int exchange_u64(int start, int logstride, int size, unsigned long long mine,
                 std::vector<unsigned long long> &all);
// DIRECT phase times since the last reset (shmemx_direct_stats).
int direct_stats(double *out, int nout, bool reset);
// Broadcast and [f]collect on the IPC transport (ipc_coll.cpp): members pull
// from the root's / each other's heap or scratch over IPC mappings.  target
// and source are device pointers (the caller stages host buffers).
int ipc_broadcast(char *target, const char *source, size_t bytes, int root_idx, int start,
                  int step, int P, int m, hipStream_t s);
int ipc_collect(char *target, const char *source, size_t esize, size_t nelems, int start,
                int step, int P, int m, size_t *total_out, hipStream_t s);

}  // namespace shmx
