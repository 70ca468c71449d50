// Internal interfaces between the C-ABI/runtime (runtime.cpp, entry.cpp) and
// the gfx950 kernels (fold_kernels.hip).  Not installed; not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace shmx {

// Upper bound on inputs one fold launch reads; longer folds are chained
// (out = fold(ins[0..15]); out = fold(out, ins[16..30]); ...) which keeps the
// reference's left-to-right order.
constexpr int kMaxFoldInputs = 16;

// Element sizes per SHMEMX_TYPE_* (long double is the host's 16-byte x87
// slot; long and long long are both 8 bytes on LP64).
size_t type_size(int type);
bool op_valid(int type, int op);       // reference defines the pair
bool op_on_device(int type, int op);   // this build has a HIP kernel for it

// out[i] = op(...op(ins[0][i], ins[1][i])..., ins[nins-1][i]) for i < n.
// nins in [1, kMaxFoldInputs]; nins == 1 is a copy.  out may be the very
// same array as any input (each element is read by the lane that writes it,
// before it writes it) but must not partially overlap one.  Returns
// hipSuccess or the launch error.
hipError_t launch_fold(int type, int op, void *out, const void *const *ins,
                       int nins, size_t n, hipStream_t stream);

// A host-visible completion signal: a page-locked, host-coherent word and
// the value a launch stores there (system-scope release) once its work is
// done.  A blocking call spins on the word instead of waiting for the stream:
// 6.8 against 11.9 us for a one-element copy when the kernel stores it
// itself, 9.6 with a one-thread marker kernel after it
// (tools/latency_breakdown.hip, profiles/r03_latency_breakdown.txt).
struct HostSignal {
    unsigned long long *word;
    unsigned long long value;
};
// The next signal value (the word is shared: blocking calls hold the
// library lock), and the wait for it: spin until the word holds the value or
// the stream has drained; after ~2 ms of spinning (long work) or an error
// the stream wait takes over (and reports the error).
HostSignal next_host_signal();
void wait_host_signal(const HostSignal &sig, hipStream_t s);
// launch_fold whose completion stores sig: the fold kernel itself when the
// launch is one workgroup (every wave drains its stores, then lane 0 of the
// workgroup stores the value with a system-scope release), otherwise a
// one-thread marker kernel right after it.
hipError_t launch_fold_signal(int type, int op, void *out, const void *const *ins, int nins, size_t n,
                              hipStream_t stream, const HostSignal &sig);
// Does a copy (launch_fold with nins == 1) of n elements of `type` from
// src to dst run as ONE workgroup (so launch_fold_signal's workgroup stores
// the signal itself, after its own stores drained and a system-scope
// release)?
bool copy_one_workgroup(int type, const void *dst, const void *src, size_t n);
// A copy (launch_fold with nins == 1) of n elements of `type` from `in` to
// both `out` and `out2` in one launch, then sig as launch_fold_signal stores
// it (a small blocking result into HBM and into the mirrored heap's view).
hipError_t launch_copy2_signal(int type, void *out, void *out2, const void *in, size_t n, hipStream_t stream,
                               const HostSignal &sig);
// The one-thread marker kernel alone: stores sig once everything enqueued
// before it on the stream has completed.
hipError_t launch_host_signal(const HostSignal &sig, hipStream_t stream);

// launch_fold for inputs in other GPUs' HBM (DIRECT and SIGNAL): every lane
// issues its loads of all inputs before folding any, so every peer's link is
// busy at once; same results as launch_fold.
hipError_t launch_fold_peers(int type, int op, void *out, const void *const *ins, int nins, size_t n,
                             hipStream_t stream);

// Copy nseg (<= kMaxFoldInputs) byte ranges srcs[i] -> dsts[i] in one launch
// (DIRECT all-gather: the peers' result slices, read concurrently).
hipError_t launch_gather(const void *const *srcs, void *const *dsts, const size_t *bytes, int nseg,
                         hipStream_t stream);

// System-scope release + acquire on every XCD's L2 (buffer_wbl2 sc0 sc1 +
// buffer_inv sc0 sc1 from blocks spread over all 8 XCDs), stream-ordered:
// this GPU's writes become visible to peers reading its HBM over xGMI, and
// no line of a peer's memory cached here survives into the next kernel.
// Enqueued before every host barrier that hands data between GPUs.
// Each of the kFenceBlocks blocks stores kFenceSeen | (its XCC id) into
// seen[block] (system scope), so the reader can prove every XCD fenced:
// fence_and_wait (host, seen host-coherent) or the next signal_kernel (seen
// in device memory; it also clears the records).
constexpr int kFenceBlocks = 64;
constexpr unsigned int kFenceSeen = 0x100u;
hipError_t launch_sys_fence(hipStream_t stream, unsigned int *seen);

// Device-side barrier of the SIGNAL algorithm (signal.cpp): the reference's
// linear barrier (barrier-linear.c:51-77: every member bumps a counter of
// every other member, then waits for its own to reach PE_size - 1) as one
// 64-lane wave, with the counters kept where only their owner writes them.
// cnt[q] in a PE's signal area = barriers that PE has entered together with
// PE q.  Lane i (member i != me) bumps mine[pe[i]] with a system-scope store,
// then polls peer[i][me] (member i's counter for me, read over xGMI) until it
// has caught up.  Counter state lives on the device, so a captured graph
// replays correctly.  A wait longer than timeout_ticks (s_memrealtime, 100
// MHz) sets *err and gives up, so a missing peer never hangs the GPU.
// Enqueue launch_sys_fence first: it publishes this GPU's writes and drops
// stale peer lines on every XCD, which a single wave cannot do.
struct SignalArgs {
    unsigned long long *mine;
    const unsigned long long *peer[kMaxFoldInputs];
    int pe[kMaxFoldInputs];
    int P, me;
    unsigned long long timeout_ticks;
    unsigned int *err;   // host-mapped: 1 = a peer timed out, 2 = a fence missed an XCD
    // the preceding launch_sys_fence's records (device memory, kFenceBlocks
    // words): fewer than nxcc distinct XCDs sets *err = 2.  fence_stats[0] +=
    // 1 per check, fence_stats[1] += 1 per incomplete fence (device memory).
    unsigned int *seen;
    int nxcc;
    unsigned long long *fence_stats;
};
hipError_t launch_signal(const SignalArgs &a, hipStream_t stream);

// The one-shot reduction of a small array as ONE launch (SIGNAL's one shot,
// and DIRECT's when every member can take it): kFenceBlocks blocks each run
// the system fence and record their XCD; the last block to arrive checks
// the XCD coverage and does the entry handshake with the peers (the signal
// counters of SignalArgs); every block then folds its share of
// out[i] = op(...op(ins[0][i], ins[1][i])..., ins[nins-1][i]); the last block
// to finish does the exit handshake.  gsync: 2 words of device memory, zero
// at the first launch and left zero (an arrival counter, a generation).
// sig.seen must hold kFenceBlocks words.  Launches on one GPU must not
// overlap (stream order, or one stream).
//
// Two-shot (two_shot != 0: SIGNAL's and DIRECT's two-shot schedule for
// mid-size arrays, as ONE launch): after the entry handshake every block
// folds its share of elements [lo, hi) only (out, ins indexed alike), then
// every block writes back its XCD's L2 and arrives; the last block does the
// mid handshake with the peers (every member's slice is final) and releases
// the grid; every block drops stale peer lines (system acquire) and copies
// the nseg byte ranges gsrc[k] -> gdst[k] (the peers' result slices); the
// last block to finish does the exit handshake.
// The fused one shot folds an array of at most this many elements (4 per
// lane of one 256-lane workgroup) in the last workgroup to arrive alone.
constexpr size_t kFusedTinyElems = 4 * 256;
struct SignalFoldArgs {
    SignalArgs sig;
    // the one shot's tiny case (one workgroup does all the work): stores
    // host_value into host_word after its exit handshake (nullptr: no store)
    unsigned long long *host_word;
    unsigned long long host_value;
    unsigned int *gsync;
    void *out;
    const void *ins[kMaxFoldInputs];
    int nins;
    size_t n;
    int two_shot;
    size_t lo, hi;
    int nseg;
    const void *gsrc[kMaxFoldInputs];
    void *gdst[kMaxFoldInputs];
    size_t glen[kMaxFoldInputs];   // bytes
};
hipError_t launch_signal_fold(int type, int op, const SignalFoldArgs &a, hipStream_t stream);

// Position-aware 64-bit checksum of n elements of `type` at device address
// ptr (16-byte aligned) into out[0], then `epoch` into out[1] (device memory
// or host-mapped page-locked memory: system-scope stores, in that order),
// stream-ordered, one launch.  Calls must not overlap in time (one arrival
// counter per process).
constexpr int kChecksumMaxBlocks = 4096;
hipError_t launch_checksum(int type, const void *ptr, size_t n, unsigned long long *out,
                           unsigned long long epoch, hipStream_t stream);

// The kernel clock (fold_kernels.hip; shmemx_kernel_timing /
// shmemx_kernel_times): while on, every fold-family launch carries a
// start / stop event pair of its own dispatch (hipExtLaunchKernelGGL), up to
// 4096 launches between reads.  kernel_times waits for them and returns
// their durations (us) and kinds (0 fold, 1 copy, 2 peers fold, 3 gather)
// in launch order, then starts over.
int kernel_timing(int on);
int kernel_times(double *us, int *kind, int max, unsigned long long *dropped);


}  // namespace shmx
