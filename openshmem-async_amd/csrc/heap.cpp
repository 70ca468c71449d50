// The symmetric heap on HBM (heap.h): one segment per PE, exported over IPC.
#include <hip/hip_runtime.h>
#include <link.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "heap.h"
#include "mirror.h"
#include "node.h"
#include "shmem_reduce_mi355x.h"
#include "state.h"

namespace shmx {
namespace heap {

namespace {

// The reference's default is 32 MiB (comms-shared.h:74) for a host heap; an
// MI355X PE has 288 GB of HBM, and the heap holds whole reduction operands.
constexpr uint64_t kDefaultHeapBytes = uint64_t(4) << 30;
// The top of the segment is the library's own: the SIGNAL algorithm's
// counters (signal_area()), zeroed at creation, at the same offset on every
// PE and mapped by the peers together with the heap.
constexpr uint64_t kSignalBytes = uint64_t(64) << 10;

struct Private {
    void *base;     // what hipMalloc returned
    size_t bytes;   // what the caller asked for
};

// $SHMEMX_HEAP_MEMORY picks what shmem_malloc hands out:
//   mirrored (default)  the segment is HBM and shmem_malloc returns addresses
//                       in a host view of it (mirror.h): host code reads and
//                       writes symmetric objects as in the reference (whose
//                       heap is host memory, memory/symmem.c:168-227), the
//                       collectives run on the HBM twin, and only the blocks
//                       the host touched cross PCIe;
//   device (or hbm)     the HBM segment itself: device addresses, for
//                       programs whose own kernels use symmetric objects;
//   host                page-locked host memory instead of HBM
//                       (comms-inline.h:752-769): reductions on it take the
//                       pinned host pipeline; peers cannot map host segments,
//                       so shmemx_heap_ptr returns NULL for them (as the
//                       reference's shmem_ptr always does) and DIRECT/SIGNAL
//                       are not used on them.
enum HeapMode { kMirrored, kDevice, kHost };

HeapMode heap_mode() {
    static const HeapMode m = [] {
        const char *e = std::getenv("SHMEMX_HEAP_MEMORY");
        const std::string v = e ? e : "";
        if (v.empty() || v == "mirrored") return kMirrored;
        if (v == "device" || v == "hbm") return kDevice;
        if (v == "host") return kHost;
        fatal("shmem_malloc", "SHMEMX_HEAP_MEMORY must be mirrored, device (hbm) or host");
    }();
    return m;
}

bool host_kind() { return heap_mode() == kHost; }
bool mirrored() { return heap_mode() == kMirrored; }

hipError_t seg_alloc(void **p, size_t bytes) {
    return host_kind() ? hipHostMalloc(p, bytes, hipHostMallocDefault) : hipMalloc(p, bytes);
}

hipError_t seg_free(void *p) { return host_kind() ? hipHostFree(p) : hipFree(p); }

// Private blocks (outside the segment) of a mirrored heap are page-locked
// host memory, staged per call like any host operand.
hipError_t priv_alloc(void **p, size_t bytes) {
    return mirrored() ? hipHostMalloc(p, bytes, hipHostMallocDefault) : seg_alloc(p, bytes);
}
hipError_t priv_free(void *p) { return mirrored() ? hipHostFree(p) : seg_free(p); }

struct Heap {
    char *base = nullptr;     // the segment (nullptr until the first allocation)
    char *view = nullptr;     // its host view (mirrored mode), else nullptr
    bool failed = false;      // the segment could not be allocated
    bool checked = false;     // every PE's segment state compared (first allocation)
    Arena arena;
    std::map<void *, Private> priv;   // blocks outside the segment
} g_heap;

// The mirrored heap's copies (mirror::Backend) work on the view's alias
// (mirror.h), never on the view's own pages: a pageable hipMemcpy pins the
// pages it touches, and every later protection change of pinned view pages
// costs a driver invalidation (28 ms per repeated 32 MiB call, profiles/
// r02_mirror_probe_pageable.txt).  The alias is page-locked in 256 MiB
// regions the first time a copy touches them, and the DMA engines then move
// blocks straight between HBM and its pages; a region HIP refuses to lock
// goes through a page-locked bounce buffer instead (CPU copy of one half
// overlapping the DMA of the other).  A fetch first waits for the streams
// that wrote the view's blocks (the writers below), then copies on a stream
// of its own, so it never queues behind unrelated work on the library's or
// the caller's streams.
constexpr size_t kMirRegion = size_t(256) << 20;
constexpr size_t kMirStage = size_t(8) << 20;
struct MirStage {
    char *buf = nullptr;
    hipEvent_t done[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    int next = 0;
    hipStream_t fetch = nullptr;   // the fetches' own stream (non-blocking)
    std::vector<uint8_t> region;   // 0 untried, 1 page-locked, 2 refused
    std::vector<char *> region_dev;   // device address of a page-locked region
} g_mst;

// The streams collectives on view operands ran on, each with an event
// recorded after its last such collective.  A fetch waits for the armed
// ones (and for the whole device after shmemx_mirror_invalidate, whose
// writers the library never saw).  Guarded by g_wmu: the fault service
// thread fetches while the caller's thread may be recording.
struct Writer {
    hipStream_t stream;
    hipEvent_t done;
    bool armed;
};
std::mutex g_wmu;
std::vector<Writer> g_writers;
bool g_sync_device = false;

void record_writer(void *stream) {
    std::lock_guard<std::mutex> lk(g_wmu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (!s || (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)) {
        // unknown writers, or work captured into a graph that runs later:
        // the next fetch waits for the device (a replayed graph's writes to
        // the view need shmemx_mirror_invalidate afterwards)
        g_sync_device = true;
        return;
    }
    for (Writer &w : g_writers) {
        if (w.stream == s) {
            SHMX_HIP(hipEventRecord(w.done, s));
            w.armed = true;
            return;
        }
    }
    Writer w{s, nullptr, true};
    SHMX_HIP(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    SHMX_HIP(hipEventRecord(w.done, s));
    g_writers.push_back(w);
}

void wait_writers() {
    std::lock_guard<std::mutex> lk(g_wmu);
    if (g_sync_device) {
        device_sync();
        g_sync_device = false;
        for (Writer &w : g_writers) w.armed = false;
        return;
    }
    for (Writer &w : g_writers) {
        if (!w.armed) continue;
        SHMX_HIP(hipEventSynchronize(w.done));
        w.armed = false;
    }
}

hipStream_t mir_fetch_stream() {
    if (!g_mst.fetch) SHMX_HIP(hipStreamCreateWithFlags(&g_mst.fetch, hipStreamNonBlocking));
    return g_mst.fetch;
}

void mir_stage_ready() {
    if (g_mst.buf) return;
    void *p = nullptr;
    SHMX_HIP(hipHostMalloc(&p, kMirStage, hipHostMallocDefault));
    g_mst.buf = static_cast<char *>(p);
    for (hipEvent_t &e : g_mst.done) SHMX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

// Is the alias region holding offset `off` page-locked (locking it now)?
bool mir_locked(uint64_t off) {
    const size_t r = (size_t)(off / kMirRegion);
    if (g_mst.region.size() <= r) g_mst.region.resize(r + 1, 0);
    if (g_mst.region[r] == 0) {
        const size_t len = std::min<size_t>(kMirRegion, mirror::view_bytes() - r * kMirRegion);
        const bool ok = hipHostRegister(mirror::alias_base() + r * kMirRegion, len,
                                        hipHostRegisterDefault) == hipSuccess;
        if (!ok) (void)hipGetLastError();
        g_mst.region[r] = ok ? 1 : 2;
        trace(LOG_MEMORY, "mirrored heap: alias region %zu (%zu bytes) %s", r, len,
              ok ? "page-locked" : "not page-locked (bounce buffer)");
    }
    return g_mst.region[r] == 1;
}

// Device address of alias bytes [off, off + bytes) (inside one page-locked
// region), or nullptr: kernels may store a small result there directly.
char *mir_alias_device(uint64_t off, size_t bytes) {
    const size_t r = (size_t)(off / kMirRegion);
    if (!bytes || (off + bytes - 1) / kMirRegion != r || !mir_locked(off)) return nullptr;
    if (g_mst.region_dev.size() <= r) g_mst.region_dev.resize(r + 1, nullptr);
    if (!g_mst.region_dev[r]) {
        void *d = nullptr;
        if (hipHostGetDevicePointer(&d, mirror::alias_base() + r * kMirRegion, 0) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        g_mst.region_dev[r] = static_cast<char *>(d);
    }
    return g_mst.region_dev[r] + (off - r * kMirRegion);
}

// [off, off + bytes) cut at region boundaries
template <typename F>
void mir_by_region(uint64_t off, size_t bytes, F f) {
    while (bytes) {
        const size_t n = std::min<size_t>(bytes, kMirRegion - off % kMirRegion);
        f(off, n, mir_locked(off));
        off += n;
        bytes -= n;
    }
}

void mir_to_device(uint64_t off, size_t bytes, void *) {
    bind_device();
    mir_by_region(off, bytes, [](uint64_t o, size_t len, bool locked) {
        const char *src = mirror::alias_base() + o;
        if (locked) {
            SHMX_HIP(hipMemcpyAsync(g_heap.base + o, src, len, hipMemcpyHostToDevice, g_state.stream));
            return;
        }
        mir_stage_ready();
        const size_t half = kMirStage / 2;
        for (size_t done = 0; done < len; done += half) {
            const size_t n = std::min(half, len - done);
            const int h = g_mst.next;
            g_mst.next ^= 1;
            if (g_mst.used[h]) SHMX_HIP(hipEventSynchronize(g_mst.done[h]));
            parallel_copy(g_mst.buf + h * half, src + done, n);
            SHMX_HIP(hipMemcpyAsync(g_heap.base + o + done, g_mst.buf + h * half, n,
                                    hipMemcpyHostToDevice, g_state.stream));
            SHMX_HIP(hipEventRecord(g_mst.done[h], g_state.stream));
            g_mst.used[h] = true;
        }
    });
}

void mir_copy_to_host(uint64_t off, size_t bytes);

void mir_to_host(uint64_t off, size_t bytes, void *) {
    bind_device();
    wait_writers();
    mir_copy_to_host(off, bytes);
}

// settle(): a blocking call's result, whose work has completed (its host
// signal arrived), so no writer event is waited for (~half of the copy-back's
// cost, profiles/r04_isx_mirror.txt)
void mir_to_host_done(uint64_t off, size_t bytes, void *) { mir_copy_to_host(off, bytes); }

void mir_copy_to_host(uint64_t off, size_t bytes) {
    bind_device();   // also runs on the fault service thread
    const hipStream_t fs = mir_fetch_stream();
    mir_by_region(off, bytes, [fs](uint64_t o, size_t len, bool locked) {
        char *dst = mirror::alias_base() + o;
        if (locked) {
            SHMX_HIP(hipMemcpyAsync(dst, g_heap.base + o, len, hipMemcpyDeviceToHost, fs));
            SHMX_HIP(hipStreamSynchronize(fs));
            return;
        }
        mir_stage_ready();
        // halves in turn: the DMA of chunk k + 1 overlaps the CPU copy of chunk k
        const size_t half = kMirStage / 2;
        const size_t nchunks = (len + half - 1) / half;
        // the to_device half of the ring may still be in flight
        for (int h = 0; h < 2; ++h)
            if (g_mst.used[h]) SHMX_HIP(hipEventSynchronize(g_mst.done[h]));
        auto dma = [&](size_t k) {
            const size_t n = std::min(half, len - k * half);
            SHMX_HIP(hipMemcpyAsync(g_mst.buf + (k & 1) * half, g_heap.base + o + k * half, n,
                                    hipMemcpyDeviceToHost, fs));
            SHMX_HIP(hipEventRecord(g_mst.done[k & 1], fs));
        };
        dma(0);
        for (size_t k = 0; k < nchunks; ++k) {
            if (k + 1 < nchunks) dma(k + 1);
            SHMX_HIP(hipEventSynchronize(g_mst.done[k & 1]));
            parallel_copy(dst + k * half, g_mst.buf + (k & 1) * half, std::min(half, len - k * half));
        }
        g_mst.used[0] = g_mst.used[1] = false;   // every DMA has landed
    });
}
// Set by SameStreamFlush: the flushed blocks' consumer is the library stream
// itself, which the copies are enqueued on, so nothing needs to wait here.
thread_local bool t_same_stream_flush = false;

void mir_drain(void *) {
    if (!t_same_stream_flush) SHMX_HIP(hipStreamSynchronize(g_state.stream));
}

bool ensure_segment() {
    if (g_heap.base) return true;
    if (g_heap.failed) return false;
    uint64_t bytes = kDefaultHeapBytes;
    if (const char *e = std::getenv("SHMEM_SYMMETRIC_HEAP_SIZE")) {
        if (!parse_size(e, &bytes) || bytes == 0)
            fatal("shmem_malloc", "unusable SHMEM_SYMMETRIC_HEAP_SIZE");
    }
    bytes += kSignalBytes;
    bytes = (bytes + (uint64_t(1) << 21) - 1) & ~((uint64_t(1) << 21) - 1);   // 2 MiB pages
    void *p = nullptr;
    if (seg_alloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        g_heap.failed = true;
        trace(LOG_MEMORY, "symmetric heap segment of %llu bytes not available",
              (unsigned long long)bytes);
        return false;
    }
    g_heap.base = static_cast<char *>(p);
    g_heap.arena.reset(bytes - kSignalBytes);
    if (host_kind()) {
        std::memset(g_heap.base + (bytes - kSignalBytes), 0, kSignalBytes);
    } else {
        // a mirrored heap starts with HBM and host view equal (zero), so
        // every block starts CLEAN; otherwise only the signal area is zeroed
        const uint64_t zero_from = mirrored() ? 0 : bytes - kSignalBytes;
        SHMX_HIP(hipMemset(g_heap.base + zero_from, 0, bytes - zero_from));
        device_sync();
        node::publish(node::kHeap, p, bytes);   // peers map it after the allocation's barrier
        if (mirrored()) {
            if (!mirror::create(g_heap.arena.capacity(), mirror::Backend{mir_to_device, mir_to_host,
                                                                        mir_drain, nullptr,
                                                                        mir_to_host_done}))
                fatal("shmem_malloc", "cannot reserve the host view of the mirrored heap");
            g_heap.view = mirror::host_base();
        }
    }
    trace(LOG_MEMORY, "symmetric heap segment: %llu bytes of %s at %p%s%p", (unsigned long long)bytes,
          host_kind() ? "page-locked host memory" : "HBM", p,
          g_heap.view ? ", host view at " : "", static_cast<void *>(g_heap.view));
    return true;
}

bool in_segment(const void *p) {
    const char *c = static_cast<const char *>(p);
    return g_heap.base && c >= g_heap.base && c < g_heap.base + g_heap.arena.capacity();
}

bool in_view(const void *p) {
    const char *c = static_cast<const char *>(p);
    return g_heap.view && c >= g_heap.view && c < g_heap.view + g_heap.arena.capacity();
}

}  // namespace

void *alloc(size_t alignment, size_t bytes) {
    if (!bytes) return nullptr;
    // The first allocation (a collective call on every PE, shmem_malloc's
    // rule, symmem.c:209) checks that the segment exists on every PE or on
    // none: a PE without it would carve its objects elsewhere and the heap
    // would no longer be symmetric, which the IPC algorithms and heap_ptr
    // rely on (the reference's heap-attach failure is fatal too).
    if (!g_heap.checked && g_state.npes > 1 && node::up()) {
        g_heap.checked = true;
        const bool mine = ensure_segment();
        const bool all_have = node::agree(0, 1, g_state.npes, mine);
        const bool none_has = node::agree(0, 1, g_state.npes, !mine);   // then all use private blocks
        if (!all_have && !none_has)
            fatal("shmem_malloc", "the symmetric heap segment could not be allocated on every PE "
                                  "(SHMEM_SYMMETRIC_HEAP_SIZE)");
        // and one size everywhere (published before the votes' barriers), or
        // the arenas would run out at different allocations
        if (all_have && !node::agree(0, 1, g_state.npes,
                                     node::peer_bytes(node::kHeap, 0) == node::peer_bytes(node::kHeap, g_state.pe)))
            fatal("shmem_malloc", "SHMEM_SYMMETRIC_HEAP_SIZE differs across PEs");
    }
    if (ensure_segment()) {
        const uint64_t off = g_heap.arena.alloc(bytes, alignment ? alignment : 1);
        if (off != Arena::kNone) return (g_heap.view ? g_heap.view : g_heap.base) + off;
    }
    // Outside the segment: a private block.  Every PE makes the same choice,
    // since the segment's state is the same on every PE.
    const size_t pad = alignment > 256 ? alignment : 0;
    void *base = nullptr;
    if (priv_alloc(&base, bytes + pad) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    uintptr_t u = reinterpret_cast<uintptr_t>(base);
    if (pad) u = (u + alignment - 1) & ~(uintptr_t)(alignment - 1);
    void *p = reinterpret_cast<void *>(u);
    g_heap.priv[p] = Private{base, bytes};
    return p;
}

bool free(void *p) {
    if (in_segment(p)) return g_heap.arena.free((uint64_t)(static_cast<char *>(p) - g_heap.base));
    if (in_view(p)) return g_heap.arena.free((uint64_t)(static_cast<char *>(p) - g_heap.view));
    auto it = g_heap.priv.find(p);
    if (it == g_heap.priv.end()) return false;
    device_sync();
    SHMX_HIP(priv_free(it->second.base));
    g_heap.priv.erase(it);
    return true;
}

size_t size_of(const void *p) {
    if (in_segment(p)) return g_heap.arena.size_of((uint64_t)(static_cast<const char *>(p) - g_heap.base));
    if (in_view(p)) return g_heap.arena.size_of((uint64_t)(static_cast<const char *>(p) - g_heap.view));
    auto it = g_heap.priv.find(const_cast<void *>(p));
    return it == g_heap.priv.end() ? 0 : it->second.bytes;
}

bool offset_of(const void *p, size_t bytes, uint64_t *off) {
    if (!in_segment(p)) return false;
    const uint64_t o = (uint64_t)(static_cast<const char *>(p) - g_heap.base);
    if (bytes > g_heap.arena.capacity() - o) return false;
    *off = o;
    return true;
}

namespace {

struct Range {
    uintptr_t lo, hi;
};

// Writable PT_LOAD segments of the main program (.data and .bss): the first
// object dl_iterate_phdr reports.
int collect_main_data(struct dl_phdr_info *info, size_t, void *arg) {
    auto *out = static_cast<std::vector<Range> *>(arg);
    for (int i = 0; i < info->dlpi_phnum; ++i) {
        const ElfW(Phdr) &ph = info->dlpi_phdr[i];
        if (ph.p_type == PT_LOAD && (ph.p_flags & PF_W))
            out->push_back({info->dlpi_addr + ph.p_vaddr, info->dlpi_addr + ph.p_vaddr + ph.p_memsz});
    }
    return 1;   // the main program only
}

const std::vector<Range> &main_data() {
    static const std::vector<Range> r = [] {
        std::vector<Range> v;
        dl_iterate_phdr(collect_main_data, &v);
        return v;
    }();
    return r;
}

}  // namespace

bool is_symmetric(const void *p) {
    if (in_segment(p) || in_view(p)) return true;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (const auto &kv : g_heap.priv) {
        const uintptr_t b = reinterpret_cast<uintptr_t>(kv.first);
        if (a >= b && a < b + kv.second.bytes) return true;
    }
    for (const Range &r : main_data())
        if (a >= r.lo && a < r.hi) return true;
    return false;
}

unsigned long long *signal_area() {
    if (host_kind() || !ensure_segment()) return nullptr;
    return reinterpret_cast<unsigned long long *>(g_heap.base + g_heap.arena.capacity());
}

uint64_t signal_offset() { return g_heap.arena.capacity(); }

void *device_operand(const void *p, size_t bytes) {
    if (!in_view(p) || bytes > g_heap.arena.capacity() - (uint64_t)(static_cast<const char *>(p) - g_heap.view))
        return const_cast<void *>(p);
    const uint64_t off = (uint64_t)(static_cast<const char *>(p) - g_heap.view);
    mirror::flush(off, bytes);
    return g_heap.base + off;
}

const void *current_host_bytes(const void *p, size_t bytes) {
    if (!bytes || !in_view(p) ||
        bytes > g_heap.arena.capacity() - (uint64_t)(static_cast<const char *>(p) - g_heap.view))
        return nullptr;
    const uint64_t off = (uint64_t)(static_cast<const char *>(p) - g_heap.view);
    return mirror::view_current(off, bytes) ? mirror::alias_base() + off : nullptr;
}

const void *device_operand_bytes(const void *p, size_t bytes) {
    if (!in_view(p) || bytes > g_heap.arena.capacity() - (uint64_t)(static_cast<const char *>(p) - g_heap.view))
        return p;
    const uint64_t off = (uint64_t)(static_cast<const char *>(p) - g_heap.view);
    mirror::flush_bytes(off, bytes);
    return g_heap.base + off;
}

void *alias_device(const void *p, size_t bytes) {
    if (!bytes || !in_view(p) ||
        bytes > g_heap.arena.capacity() - (uint64_t)(static_cast<const char *>(p) - g_heap.view))
        return nullptr;
    return mir_alias_device((uint64_t)(static_cast<const char *>(p) - g_heap.view), bytes);
}

void *device_operand_open(const void *p) {
    if (!in_view(p)) return const_cast<void *>(p);
    const uint64_t off = (uint64_t)(static_cast<const char *>(p) - g_heap.view);
    mirror::flush(off, g_heap.arena.capacity() - off);
    return g_heap.base + off;
}

void device_wrote(const void *p, size_t bytes, void *stream) {
    if (!bytes || !in_view(p)) return;
    record_writer(stream);
    mirror::device_wrote((uint64_t)(static_cast<const char *>(p) - g_heap.view), bytes);
}

void *twin(const void *p) {
    return in_view(p) ? g_heap.base + (static_cast<const char *>(p) - g_heap.view) : const_cast<void *>(p);
}

DeviceWrite::DeviceWrite(void *p, size_t bytes, void *stream, bool light)
    : dev_(p), stream_(stream), open_(false) {
    if (!bytes || !in_view(p) ||
        bytes > g_heap.arena.capacity() - (uint64_t)(static_cast<const char *>(p) - g_heap.view))
        return;
    const uint64_t off = (uint64_t)(static_cast<const char *>(p) - g_heap.view);
    light_ = light && mirror::begin_light_write(off, bytes);
    if (light_) fresh_ = true;
    else mirror::begin_device_write(off, bytes, &fresh_);
    dev_ = g_heap.base + off;
    off_ = off;
    bytes_ = bytes;
    open_ = true;
}

void DeviceWrite::close(bool copied) {
    if (!open_) return;
    open_ = false;
    if (!done_) record_writer(stream_);
    if (light_) mirror::end_light_write(off_, bytes_, copied);
    else mirror::end_device_write(off_, bytes_);
}

size_t DeviceWrite::settle(size_t limit, bool copied) {
    if (!open_) return 0;
    if (light_) {
        close(copied);
        return copied ? 0 : bytes_;
    }
    if (bytes_ > limit) return 0;
    close();
    return mirror::settle(off_, bytes_, fresh_, copied && fresh_);
}

void *DeviceWrite::settle_dst(size_t limit) const {
    if (!open_ || !fresh_ || (bytes_ > limit && !light_)) return nullptr;
    return mir_alias_device(off_, bytes_);
}

bool host_acquire(const void *p, size_t bytes, bool write) {
    if (!in_view(p) || bytes > g_heap.arena.capacity() - (uint64_t)(static_cast<const char *>(p) - g_heap.view))
        return false;
    mirror::acquire((uint64_t)(static_cast<const char *>(p) - g_heap.view), bytes, write);
    return true;
}

void flush_view() {
    if (g_heap.view) mirror::flush(0, g_heap.arena.capacity());
}

bool view_offset(const void *p, uint64_t *off) {
    if (!in_view(p)) return false;
    *off = (uint64_t)(static_cast<const char *>(p) - g_heap.view);
    return true;
}

SameStreamFlush::SameStreamFlush() : prev_(t_same_stream_flush) { t_same_stream_flush = true; }
SameStreamFlush::~SameStreamFlush() { t_same_stream_flush = prev_; }

bool segment(void **base, size_t *bytes) {
    if (!g_heap.base || host_kind()) return false;
    *base = g_heap.base;
    *bytes = g_heap.arena.capacity();
    return true;
}

void release_all() {
    if (g_heap.view) {
        for (size_t r = 0; r < g_mst.region.size(); ++r)
            if (g_mst.region[r] == 1) (void)hipHostUnregister(mirror::alias_base() + r * kMirRegion);
        mirror::destroy();
        g_heap.view = nullptr;
    }
    if (g_mst.buf) {
        (void)hipHostFree(g_mst.buf);
        for (hipEvent_t e : g_mst.done) (void)hipEventDestroy(e);
    }
    if (g_mst.fetch) (void)hipStreamDestroy(g_mst.fetch);
    g_mst = MirStage{};
    {
        std::lock_guard<std::mutex> lk(g_wmu);
        for (Writer &w : g_writers) (void)hipEventDestroy(w.done);
        g_writers.clear();
        g_sync_device = false;
    }
    for (auto &kv : g_heap.priv) (void)priv_free(kv.second.base);
    if (g_heap.base) {
        node::unpublish(node::kHeap);
        (void)seg_free(g_heap.base);
    }
    g_heap.priv.clear();
    g_heap.base = nullptr;
    g_heap.failed = false;
    g_heap.checked = false;
    g_heap.arena.reset(0);
}

}  // namespace heap
}  // namespace shmx
