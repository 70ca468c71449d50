// Intra-node layer: what the reference gets from GASNet's segment table and
// active messages (comms/gasnet/comms-inline.h:722-801, barrier-linear.c),
// rebuilt for "one PE per GPU, all GPUs in one node":
//
//   * a small POSIX shared-memory block per job (/dev/shm), named from the
//     job's unique id, holding per-PE IPC handles of two device regions (the
//     symmetric heap segment and a DIRECT-algorithm scratch region), per-call
//     descriptors, and pairwise barrier counters;
//   * a host barrier over any active set (PE_start, logPE_stride, PE_size);
//   * peer mappings of those regions (hipIpcOpenMemHandle), so a HIP kernel
//     on this GPU loads from and stores to another PE's HBM over xGMI, the
//     way the reference's shmem_getmem reads a peer's symmetric segment.
//
// Internal to libshmem_reduce_mi355x.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace shmx {
namespace node {

constexpr int kMaxPes = 64;
enum Region { kHeap = 0, kScratch = 1, kNumRegions = 2 };

// Where a PE's operand of the current call lives: in one of its regions at
// an offset (peer-addressable), or nowhere (count only).
struct Loc {
    int32_t region = -1;   // kHeap, kScratch, or -1
    uint64_t off = 0;
};

// Per-call descriptor a PE publishes before the entry barrier of a
// collective; members read each other's after it.
struct Desc {
    Loc src, tgt;
    int64_t count = 0;     // elements or bytes this PE contributes (collect)
    uint64_t aux = 0;      // checksum (verify)
};

// Attach the job's shared block; `key` is the job's unique id (every PE
// passes the same bytes).  Returns false (and leaves the layer down) on any
// OS error.
bool attach(int pe, int npes, const void *key, size_t keylen);
void detach(bool unlink);
void unlink_name();   // the block stays mapped; the /dev/shm name goes
bool up();

// Host barrier among the members start + i*step, i < P (the caller is one of
// them).  Aborts after $SHMEMX_BARRIER_TIMEOUT seconds (default 600).
void barrier(int start, int step, int P);

// Publish one of this PE's device regions (base, bytes); bumps its generation.
void publish(Region r, void *base, size_t bytes);
void unpublish(Region r);
// Base of PE `pe`'s region as mapped here (own base for pe == me); nullptr
// if the peer has not published it.  Opens / re-opens the IPC mapping when
// the peer's generation changed.
char *peer_base(Region r, int pe);
size_t peer_bytes(Region r, int pe);
const char *last_ipc_error();   // why the last peer_base() returned nullptr

// Generation of PE `pe`'s region (0 = never published); a mapping opened at
// one generation stays valid until the owner publishes again.
uint64_t region_gen(Region r, int pe);

// Collective AND of `ok` over the set (two barriers): every member returns
// the same answer, so a failure on one PE (say, an IPC mapping it could not
// open) turns into the same error return on all of them instead of a hang.
bool agree(int start, int step, int P, bool ok);

// The small-call exchange (staging.cpp, service.hip): a second shared-memory
// block of the job, page-locked and mapped into this GPU (hipHostRegister),
// with one slot of kXchgSlotBytes per PE (its source for the others' service
// workgroups) and, per pair of PEs, how many of their calls together the
// reader has finished reading the writer's slot for.  A PE writes its slot
// again only once every reader of its previous call is done with it (host
// side, at the start of its next call; normally at once), so a call needs no
// exit barrier.  xchg_attach maps and registers the block (false on any
// error; every PE calls it at init and the job agrees); the name goes with
// unlink_name().
constexpr size_t kXchgSlotBytes = 4096;
bool xchg_attach();
char *xchg_host(int pe);   // a slot's host address (nullptr if not attached)
char *xchg_dev(int pe);    // the same slot's device address
// Start this PE's part of a call over the members start + i * step, i < P:
// wait until the readers of its previous call are done with its slot, and
// count the call with every other member (counts[i] for member i).
void xchg_claim(int start, int step, int P, uint64_t *counts);
// After this PE's fold: it is done reading every member's slot of this call.
void xchg_finish(int start, int step, int P, const uint64_t *counts);

void put_desc(const Desc &d);
Desc get_desc(int pe);

// The NUMA node of each PE's GPU (-1 unknown), published by every PE before
// shmem_init's first barrier: the staging copy threads of the PEs that share
// a NUMA node take different cache domains (staging.cpp).
void put_gpu_numa(int node);
int gpu_numa(int pe);
// A hash of this PE's GPU's PCI bus id, published with the NUMA node; after
// init's barrier gpu_shared() says whether another PE process of the job
// uses the same GPU (tests and rehearsals put several on one).
void put_gpu_id(uint64_t id);
bool gpu_shared();
int npes();   // PEs attached to the block (0 if it is down)

}  // namespace node
}  // namespace shmx
