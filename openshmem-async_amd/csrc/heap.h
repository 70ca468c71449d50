// The symmetric heap on HBM (memory/symmem.c:168-227, memalloc.c:64-146).
//
// One device segment per PE, sized by $SHMEM_SYMMETRIC_HEAP_SIZE (the
// reference's variable and unit syntax, utils/unitparse.c:102-135), carved by
// a deterministic first-fit allocator: identical collective call sequences
// give identical offsets on every PE, so an address in this PE's heap names
// the same object at the same offset in every other PE's heap — the
// reference's symmetric-address rule (comms-inline.h:514-545).  The segment
// is exported over IPC (node.h), so kernels reach a peer's copy over xGMI.
// Requests the segment cannot hold fall back to private hipMalloc blocks
// (still HBM, still usable by every algorithm, but not peer-addressable).
//
// Internal to libshmem_reduce_mi355x.so.
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>

namespace shmx {
namespace heap {

// The segment allocator alone (arena.cpp), host-only and testable without a
// GPU (tests/native/test_heap.cpp): offsets within [0, capacity).
class Arena {
  public:
    static constexpr uint64_t kGranule = 256;   // every block starts 256-B aligned
    static constexpr uint64_t kNone = ~uint64_t(0);
    explicit Arena(uint64_t capacity = 0) { reset(capacity); }
    void reset(uint64_t capacity);
    // offset of a new block of `bytes` aligned to `alignment` (a power of
    // two), or kNone if it does not fit
    uint64_t alloc(uint64_t bytes, uint64_t alignment);
    uint64_t size_of(uint64_t off) const;   // requested size of the live block at off, or 0
    bool free(uint64_t off);
    uint64_t capacity() const { return capacity_; }
    uint64_t free_bytes() const;
    size_t live_blocks() const { return used_.size(); }

  private:
    struct Used {
        uint64_t start, len, bytes;   // extent [start, start + len) holds the block
    };
    uint64_t capacity_ = 0;
    std::map<uint64_t, uint64_t> free_;   // start -> length, coalesced
    std::map<uint64_t, Used> used_;       // user offset -> extent
};

// $SHMEM_SYMMETRIC_HEAP_SIZE syntax: digits with an optional k/m/g/t/p/e
// (powers of 1024); false if malformed.
bool parse_size(const char *s, uint64_t *bytes);

void *alloc(size_t alignment, size_t bytes);   // local part of shmem_malloc/align
bool free(void *p);
size_t size_of(const void *p);                  // 0 if not a heap block
// Offset of [p, p + bytes) inside this PE's segment; false if not inside it.
bool offset_of(const void *p, size_t bytes, uint64_t *off);
// The reference's symmetric-address test (shmemi_symmetric_addr_lookup,
// comms-inline.h:519-545): p lies in the heap segment or a private heap
// block, or in the executable's writable data/bss — the global and static
// variables the reference makes symmetric (globalvar/globalvar.c:99-369).
bool is_symmetric(const void *p);
// The library's signal area at the top of the segment (outside the arena):
// 64 KiB, zero at creation, at signal_offset() from the segment base on every
// PE.  nullptr if there is no segment.
unsigned long long *signal_area();
uint64_t signal_offset();
// Mirrored heap (the default, mirror.h).  A collective
// about to read or write [p, p + bytes): if that range lies in the host view,
// the host's stores in it go to HBM and the HBM twin's address is returned;
// any other p is returned as it is.
void *device_operand(const void *p, size_t bytes);
// The same for an operand whose length is not known yet (a collect target):
// every host store from p to the end of the view goes to HBM.
void *device_operand_open(const void *p);
// After a collective wrote [p, p + bytes) (a host-view address) in HBM: the
// host view of it is stale until the next host access fetches it, which
// first waits for `stream` (the stream the collective ran on) — or, for
// nullptr (shmemx_mirror_invalidate: writes on streams the library never
// saw), for the whole device.
void device_wrote(const void *p, size_t bytes, void *stream);
// A collective that writes [p, p + bytes): construct it before the
// collective is enqueued and let it go after.  For a host-view target the
// constructor flushes the host's stores, marks the blocks DEVICE_NEWER and
// opens a write in flight (host accesses to them wait, mirror.h); the
// destructor records `stream` as their writer (a fetch waits for what was
// enqueued on it) and closes the write.  ptr() is the address to write: the
// HBM twin of a host-view address, p itself otherwise.
class DeviceWrite {
  public:
    // light: a BLOCKING call's small target whose result the call's stream
    // also stores into the view's alias (settle_dst): no block state or
    // protection changes (mirror::begin_light_write); taken only if the
    // blocks allow it, else the ordinary DEVICE_NEWER marking
    DeviceWrite(void *p, size_t bytes, void *stream, bool light = false);
    ~DeviceWrite() { close(); }
    DeviceWrite(const DeviceWrite &) = delete;
    DeviceWrite &operator=(const DeviceWrite &) = delete;
    void *ptr() const { return dev_; }
    bool light() const { return light_; }
    // the write has completed (a blocking call waited for its work): close()
    // records no writer event to wait for
    void completed() { stream_ = nullptr; done_ = true; }
    // record the writer and end the write in flight (the destructor's work);
    // a light write's result goes into the view here unless `copied`
    void close(bool copied = false);
    // After a BLOCKING call's work has completed: if the target is at most
    // `limit` bytes, close the write and copy the result back into the view
    // (mirror::settle), so its blocks are CLEAN — readable by system calls
    // as well as by plain loads — when the call returns.  Larger targets
    // keep the lazy fetch.  Returns the bytes copied back.
    size_t settle(size_t limit, bool copied = false);
    // Where the call's own stream may store the result for settle(limit,
    // true): the device address of the view's page-locked alias at the
    // target's offset, when the target is at most `limit` bytes, its blocks
    // were current before the call (only the result's bytes differ), and the
    // alias region is page-locked; else nullptr.
    void *settle_dst(size_t limit) const;

  private:
    void *dev_;
    void *stream_;
    uint64_t off_ = 0;
    size_t bytes_ = 0;
    bool open_;
    bool fresh_ = false;
    bool light_ = false;
    bool done_ = false;
};
// While one lives (a blocking call, whose every kernel and copy runs on the
// library stream): flushes of host-view blocks to HBM are enqueued on that
// stream without the host waiting for them; the call's own work follows
// them in stream order, and the call waits for its work anyway.  A host
// store racing with the call on its source is the program's race, as in the
// reference (the source must not change during the collective).
class SameStreamFlush {
  public:
    SameStreamFlush();
    ~SameStreamFlush();
    SameStreamFlush(const SameStreamFlush &) = delete;
    SameStreamFlush &operator=(const SameStreamFlush &) = delete;

  private:
    bool prev_;
};
// A blocking call's small source: only its own bytes that the host wrote go
// to HBM (mirror::flush_bytes), no state change; returns the HBM twin.
const void *device_operand_bytes(const void *p, size_t bytes);
// A host-view operand [p, p + bytes) whose view bytes are current
// (mirror::view_current): the same bytes through the view's alias (readable
// by host code without a fault), else nullptr.
const void *current_host_bytes(const void *p, size_t bytes);
// The device address of the view's page-locked alias at host-view address
// p (bytes inside one alias region), or nullptr.
void *alias_device(const void *p, size_t bytes);
// The HBM twin of a host-view address (p itself otherwise), with no change
// of block state.
void *twin(const void *p);
// shmemx_mirror_acquire: [p, p + bytes) of the view made current (and, with
// `write`, writable) for host code that cannot take a page fault; false if
// the range is not in the view.
bool host_acquire(const void *p, size_t bytes, bool write);
// Every host store in the view to HBM (barriers: peers may read it next).
void flush_view();
// Offset of a host-view address in the segment; false if not in the view.
bool view_offset(const void *p, uint64_t *off);
void release_all();                             // shmem_finalize
// The HBM segment (base and bytes, the signal area excluded), or false if
// there is none yet (no shmem_malloc) or it is host memory.
bool segment(void **base, size_t *bytes);

}  // namespace heap
}  // namespace shmx
