// Host view of the HBM symmetric heap (the default heap mode;
// $SHMEMX_HEAP_MEMORY=mirrored).
//
// The reference's symmetric heap is host memory (memory/symmem.c:168-227,
// comms-inline.h:722-801): programs write symmetric objects with plain host
// stores and hand them to the collectives.  Here the heap lives in HBM (so
// reductions run device-resident and peers read it over xGMI), and in this
// mode shmem_malloc returns an address in a HOST VIEW of the same segment —
// same size, same offsets.  The library keeps the two coherent at block
// granularity (kBlock bytes), using page protection to learn what the host
// touched:
//
//   CLEAN        host view == HBM; host pages read-only.  A host store
//                faults: the block (and, for a sequential run, its
//                neighbours) becomes HOST_NEWER, read-write.
//   HOST_NEWER   the host wrote it; HBM is stale.  A collective that reads or
//                writes the block copies it host -> HBM first (flush), then it
//                is CLEAN again.
//   DEVICE_NEWER a collective wrote the block in HBM; host pages have no
//                access.  A host load or store faults: the block (and the
//                DEVICE_NEWER blocks after it, a doubling run on sequential
//                faults up to kMaxFetchRun) is copied
//                HBM -> host and becomes CLEAN.
//
// So data crosses PCIe only for blocks the host actually touched, and a
// reduction on symmetric objects is the device-resident call: its kernels,
// DIRECT's peer reads and RCCL all work on the HBM segment.
//
// The core (block states, protection, fault handling) is host-only code over
// a copy backend, testable without a GPU (tests/native/test_mirror.cpp); the
// library's backend moves blocks with HIP.
#pragma once

#include <csignal>
#include <cstddef>
#include <cstdint>

namespace shmx {
namespace mirror {

constexpr size_t kBlock = size_t(64) << 10;
// Sequential access gets doubling runs per fault: stores unprotect up to
// kMaxWriteRun blocks at once (a run past the written range costs only its
// flush), loads fetch up to kMaxFetchRun DEVICE_NEWER blocks.
constexpr size_t kMaxWriteRun = 32;    // 2 MiB
constexpr size_t kMaxFetchRun = 128;   // 8 MiB

enum State : uint8_t { CLEAN = 0, HOST_NEWER = 1, DEVICE_NEWER = 2 };

// How blocks move between the host view and the device segment.  The view
// is one memfd mapped twice: the protected view the program uses, and an
// ALIAS of the same pages that is always read-write.  The backend reads and
// writes the alias, so the copies never need the view unprotected, and a
// DMA engine may work on the alias (page-locked once) while the view's
// protection changes — its pages' virtual range is a different one.
struct Backend {
    // alias [off, off + bytes) -> device segment at offset off
    void (*to_device)(uint64_t off, size_t bytes, void *ctx);
    // device segment at offset off -> alias (it first waits for the device
    // work that may have written it: every write ended by end_device_write
    // or marked by device_wrote).  Called from an ordinary thread context
    // (the caller's, or the fault service thread's), never a signal handler.
    void (*to_host)(uint64_t off, size_t bytes, void *ctx);
    // every to_device issued so far has landed
    void (*drain)(void *ctx);
    void *ctx;
    // settle()'s copy: as to_host, for bytes whose writer is known to have
    // completed (a blocking call that has returned), so it waits for no
    // writer; nullptr = to_host
    void (*to_host_done)(uint64_t off, size_t bytes, void *ctx) = nullptr;
};

// Reserve a host view of `bytes` (rounded up to kBlock) and its alias, every
// block CLEAN (the device segment must hold the same bytes: zero), install
// the SIGSEGV handler and start the fault service thread.  false on failure.
//
// The fault handler itself makes no backend (HIP) call: those are not
// async-signal-safe, and the faulting thread may be anywhere.  A fault that
// needs bytes from the device hands the run to the service thread (one
// request slot, futex wake-ups) and waits for it with plain atomics; the
// service thread runs Backend::to_host in an ordinary thread context.
bool create(size_t bytes, const Backend &be);
void destroy();
bool active();
char *host_base();
char *alias_base();
size_t view_bytes();
// (Re)install the view's SIGSEGV handler, chaining to `prev` for faults
// outside the view (shmemx_set_fatal_note(NULL) restores its own saved
// disposition, which may predate the view).
void install_handler(const struct sigaction *prev);

// Is [p, p + bytes) inside the host view?  Offset of p.
bool contains(const void *p, size_t bytes);
uint64_t offset_of(const void *p);

// Before a collective reads or writes [off, off + bytes) of the device
// segment: copy every HOST_NEWER block that overlaps it to the device (whole
// blocks), mark them CLEAN, and drain.  Each run is made read-only BEFORE its
// copy, so a store another thread makes meanwhile faults, waits for the lock
// and marks the block HOST_NEWER again (it is not lost).  Returns the blocks
// copied.
size_t flush(uint64_t off, size_t bytes);
// Before a collective WRITES [off, off + bytes): flush the overlapped
// HOST_NEWER blocks, then mark every overlapped block DEVICE_NEWER (no host
// access) and count one device write in flight on each of them, all under
// the lock.  A host access to any of those blocks — the target itself, or a
// neighbouring object in the same block, from any thread — waits until the
// writes in flight on THAT block have ended (end_device_write), then fetches
// it, whose bytes are then the collective's; faults on other blocks do not
// wait.  *fresh (if given): no overlapped block was DEVICE_NEWER before, so
// all their other bytes equal HBM (settle()).  Returns the blocks marked.
size_t begin_device_write(uint64_t off, size_t bytes, bool *fresh = nullptr);
// The write begun on [off, off + bytes) is enqueued and its completion is
// recorded where Backend::to_host waits for it.
void end_device_write(uint64_t off, size_t bytes);
// After a blocking collective that wrote [off, off + bytes) has completed and
// ended its write: make its blocks CLEAN (readable by host code and system
// calls alike) instead of leaving them to a fault.  With `fresh` (from
// begin_device_write) only [off, off + bytes) is copied back; otherwise the
// blocks whole.  Nothing happens if another write is in flight on them.
// `copied` (with `fresh`): the call's own stream already wrote the result
// into the alias (a copy kernel before its host signal), so only the block
// states and protections change.  Returns the bytes copied here.
size_t settle(uint64_t off, size_t bytes, bool fresh, bool copied = false);
// The light path of a BLOCKING call on small operands (heap.h DeviceWrite,
// staging.cpp), which changes no block state and no page protection:
// flush_bytes() sends the part of a small source [off, off + bytes) that lies
// in HOST_NEWER blocks to HBM and leaves those blocks HOST_NEWER (writable:
// the host's next store takes no fault; the next call that needs the whole
// block flushes it whole).  Returns the blocks touched (counted as flushed).
// The copy's drain follows Backend::drain (a blocking call's work follows it
// on the same stream).
size_t flush_bytes(uint64_t off, size_t bytes);
// begin_light_write(): a small target whose blocks are CLEAN or HOST_NEWER
// with no write in flight counts one write in flight on each and keeps its
// state: the call's own stream stores the result into HBM AND into the alias
// (the view's bytes), so the blocks stay what they were — CLEAN blocks equal
// HBM again, HOST_NEWER ones are flushed whole later, the result included.
// False (nothing changed) if a block is DEVICE_NEWER or has a write in flight:
// the caller takes begin_device_write instead.
bool begin_light_write(uint64_t off, size_t bytes);
// Are the view's bytes [off, off + bytes) current (no overlapped block
// DEVICE_NEWER, no device write in flight on one), so host code may read
// them without a fault and they are the operand's value?
bool view_current(uint64_t off, size_t bytes);
// The light write has ended and its work completed: `copied` = the call's
// stream stored the result into the alias; otherwise it is copied back here
// (Backend::to_host).  Counts the blocks as settled; returns bytes copied.
size_t end_light_write(uint64_t off, size_t bytes, bool copied);
// After a collective wrote [off, off + bytes) in HBM without
// begin_device_write (a collect target, whose length is known only after
// the exchange): the overlapped blocks become DEVICE_NEWER (call flush on the
// range first).  Returns the blocks.
size_t device_wrote(uint64_t off, size_t bytes);
// Make [off, off + bytes) accessible to host code that cannot take the page
// fault — system calls (write(2) of a result, read(2) into a source), other
// libraries' DMA: DEVICE_NEWER blocks are copied back (readable, CLEAN), and
// with `write` every block becomes HOST_NEWER (read-write).  Returns the
// blocks copied back.
size_t acquire(uint64_t off, size_t bytes, bool write);
// Make the whole view current on the host (every DEVICE_NEWER block copied
// back), e.g. before the view is released.
void fetch_all();

// The fault hook: true if `addr` is in the host view and the fault was
// resolved (the faulting access can be retried).  The library's own
// handlers (and the fatal-note handler) call it before anything else.
bool handle_fault(void *addr);

struct Stats {
    uint64_t write_faults, read_faults, blocks_flushed, blocks_fetched, blocks_device_newer;
    uint64_t fault_waits;   // faults that waited for a device write in flight
    uint64_t blocks_settled;   // made CLEAN by settle() (the written bytes copied back)
};
Stats stats(bool reset);
State state_of(uint64_t off);   // tests

}  // namespace mirror
}  // namespace shmx
