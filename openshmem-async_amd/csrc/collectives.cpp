// The collectives next to the reduction path, built
// on the same runtime (one PE per GPU, one RCCL communicator, the library's
// blocking stream):
//
//   shmem_barrier / shmem_barrier_all   barrier/barrier.c:74-127,
//                                       barrier-linear.c:51-77
//   shmem_broadcast32/64                broadcast/broadcast-linear.c:54-74
//   shmem_fcollect32/64                 fcollect/fcollect-linear.c:69-91
//   shmem_collect32/64                  collect/collect-linear.c:57-130
//   shmem_malloc/free/realloc/align     memory/symmem.c:168-227 (+ the
//   (and shmalloc/shfree/shrealloc/     deprecated names, shmem.h:821-941)
//   shmemalign)
//
// Full active set: RCCL collectives (ncclBroadcast, ncclAllGather,
// ncclAllReduce for the barrier token).  Any other set: grouped
// ncclSend/ncclRecv between its members only (the members alone call, as in
// OpenSHMEM, so no sub-communicator is needed).  Host buffers are staged
// through device workspaces; pSync is never written.
//
// The symmetric heap is HBM (heap.h): shmem_malloc returns device memory
// from this PE's IPC-exported segment, collectively (a barrier_all follows,
// symmem.c:209), so a program keeps its symmetric arrays resident on the GPU,
// the reductions take the device-resident path, and the DIRECT algorithm
// reads peers' copies in place.
//
// On the IPC transport ($SHMEMX_TRANSPORT=ipc, no RCCL communicator) the
// barrier is the node block's host barrier (node.h).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "heap.h"
#include "internal.h"
#include "node.h"
#include "shmem_reduce_mi355x.h"
#include "state.h"

namespace shmx {

namespace {

struct SetInfo {
    int P = 0, m = -1, step = 1, start = 0;
    bool world = false;
    int peer(int i) const { return start + i * step; }
};

// Validate (PE_start, logPE_stride, PE_size) and the caller's membership.
int set_info(int start, int logstride, int size, SetInfo &si) {
    if (int rc = ensure_init()) return rc;
    if (start < 0 || logstride < 0 || logstride > 30 || size < 1) return set_error(SHMEMX_EINVAL);
    if ((long long)start + (long long)(size - 1) * (1LL << logstride) >= g_state.npes)
        return set_error(SHMEMX_EINVAL);
    si.P = size;
    si.start = start;
    si.step = 1 << logstride;
    si.world = start == 0 && (logstride == 0 || size == 1) && size == g_state.npes;
    if (!is_member(g_state.pe, start, logstride, size, &si.m)) return set_error(SHMEMX_ENOTMEMBER);
    if ((size > 1 || g_state.force_collective) && !g_state.comm && !node::up())
        return set_error(SHMEMX_ENOINIT);
    return SHMEMX_OK;
}

bool collective(const SetInfo &si) { return si.P > 1 || g_state.force_collective; }


// A device view of a possibly host-resident buffer.
struct DevBuf {
    char *dev = nullptr;
    char *host = nullptr;   // non-null: staged, copy back to here
    size_t bytes = 0;
};

DevBuf device_in(const void *p, size_t bytes, void *&ws, size_t &ws_bytes, hipStream_t s) {
    DevBuf b;
    b.bytes = bytes;
    if (!bytes || device_accessible(p)) {
        b.dev = static_cast<char *>(const_cast<void *>(p));
        return b;
    }
    b.dev = static_cast<char *>(grow(ws, ws_bytes, bytes));
    if (!b.dev) return b;
    SHMX_HIP(hipMemcpyAsync(b.dev, p, bytes, hipMemcpyHostToDevice, s));
    return b;
}

DevBuf device_out(void *p, size_t bytes, void *&ws, size_t &ws_bytes) {
    DevBuf b;
    b.bytes = bytes;
    if (!bytes || device_accessible(p)) {
        b.dev = static_cast<char *>(p);
        return b;
    }
    b.dev = static_cast<char *>(grow(ws, ws_bytes, bytes));
    b.host = static_cast<char *>(p);
    return b;
}

void finish(const DevBuf &out, hipStream_t s) {
    if (out.host && out.dev)
        SHMX_HIP(hipMemcpyAsync(out.host, out.dev, out.bytes, hipMemcpyDeviceToHost, s));
    SHMX_HIP(hipStreamSynchronize(s));
}

// Device token area for barriers (one byte per member, grown as needed).
char *token_area(int P) {
    return static_cast<char *>(grow(g_state.token, g_state.token_bytes,
                                    (size_t)(P < 64 ? 64 : P) + 64));
}

int barrier_impl(int start, int logstride, int size) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    SetInfo si;
    if (int rc = set_info(start, logstride, size, si)) return rc;
    hipStream_t s = g_state.stream;
    g_state.lib_stream_dirty = true;   // until someone sees it drained (service.hip)
    // mirrored heap: the host's stores to symmetric objects reach HBM, where
    // the peers' kernels read them after the barrier
    heap::flush_view();
    // quiet: everything this PE enqueued before the barrier is complete, and
    // (system-scope fence on every XCD) visible to the peers, whose stores
    // through shmemx_heap_ptr this GPU will then not see through stale lines
    const bool coll = collective(si);
    if (coll && si.P > 1) fence_and_wait(s);
    else SHMX_HIP(hipStreamSynchronize(s));
    trace(LOG_BARRIER, "set (%d,%d,%d) member %d", start, logstride, size, si.m);
    if (!coll) return SHMEMX_OK;
    if (!g_state.comm) {   // IPC transport
        node::barrier(si.start, si.step, si.P);
        return SHMEMX_OK;
    }
    char *tok = token_area(si.P);
    if (!tok) return set_error(SHMEMX_ENOMEM);
    if (si.world) {
        SHMX_NCCL(ncclAllReduce(tok, tok, 1, ncclUint8, ncclMax, g_state.comm, s));
    } else {
        // every member hears from every other member (one byte each way)
        SHMX_NCCL(ncclGroupStart());
        for (int i = 0; i < si.P; ++i) {
            if (i == si.m) continue;
            SHMX_NCCL(ncclSend(tok, 1, ncclUint8, si.peer(i), g_state.comm, s));
            SHMX_NCCL(ncclRecv(tok + 64 + i, 1, ncclUint8, si.peer(i), g_state.comm, s));
        }
        SHMX_NCCL(ncclGroupEnd());
    }
    SHMX_HIP(hipStreamSynchronize(s));
    return SHMEMX_OK;
}

int broadcast_impl(size_t esize, void *target, const void *source, size_t nelems, int root_idx,
                   int start, int logstride, int size) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    SetInfo si;
    if (int rc = set_info(start, logstride, size, si)) return rc;
    if (root_idx < 0 || root_idx >= size) return set_error(SHMEMX_EINVAL);
    const size_t bytes = nelems * esize;
    trace(LOG_BROADCAST, "%zu bytes from set member %d, set (%d,%d,%d) member %d", bytes, root_idx,
          start, logstride, size, si.m);
    if (!bytes || !collective(si)) return SHMEMX_OK;  // the root's target is never written
    if ((si.m == root_idx && !source) || (si.m != root_idx && !target)) return set_error(SHMEMX_EINVAL);
    hipStream_t s = g_state.stream;
    g_state.lib_stream_dirty = true;   // until someone sees it drained (service.hip)
    // mirrored heap: operands in the host view run on their HBM twins (a
    // non-root's target is DEVICE_NEWER from here, heap.h DeviceWrite)
    if (si.m == root_idx) source = heap::device_operand(source, bytes);
    heap::DeviceWrite tw(si.m == root_idx ? nullptr : target, bytes, s);
    if (si.m != root_idx) target = tw.ptr();
    if (!g_state.comm) {   // IPC transport
        return ipc_broadcast(static_cast<char *>(target), static_cast<const char *>(source),
                             bytes, root_idx, si.start, si.step, si.P, si.m, s);
    }
    const int root = si.peer(root_idx);
    const bool is_root = si.m == root_idx;
    DevBuf in, out;
    if (is_root) {
        in = device_in(source, bytes, g_state.cws_src, g_state.cws_src_bytes, s);
        if (!in.dev) return set_error(SHMEMX_ENOMEM);
    } else {
        out = device_out(target, bytes, g_state.cws_tgt, g_state.cws_tgt_bytes);
        if (!out.dev) return set_error(SHMEMX_ENOMEM);
    }
    if (si.world) {
        // in place on the root (sendbuff == recvbuff): its target is untouched
        char *buf = is_root ? in.dev : out.dev;
        SHMX_NCCL(ncclBroadcast(buf, buf, bytes, ncclUint8, root, g_state.comm, s));
    } else {
        SHMX_NCCL(ncclGroupStart());
        if (is_root) {
            for (int i = 0; i < si.P; ++i)
                if (i != si.m) SHMX_NCCL(ncclSend(in.dev, bytes, ncclUint8, si.peer(i), g_state.comm, s));
        } else {
            SHMX_NCCL(ncclRecv(out.dev, bytes, ncclUint8, root, g_state.comm, s));
        }
        SHMX_NCCL(ncclGroupEnd());
    }
    finish(out, s);
    return SHMEMX_OK;
}

// fcollect (equal counts) and collect (per-PE counts): member i's source
// lands at element offset off[i] of every member's target, in set order.
int collect_impl(size_t esize, void *target, const void *source, size_t nelems, int start,
                 int logstride, int size, bool fixed) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    SetInfo si;
    if (int rc = set_info(start, logstride, size, si)) return rc;
    hipStream_t s = g_state.stream;
    g_state.lib_stream_dirty = true;   // until someone sees it drained (service.hip)
    // mirrored heap: operands in the host view run on their HBM twins (the
    // target's length is known only after the counts are exchanged)
    void *const user_target = target;
    if (nelems && source) source = heap::device_operand(source, nelems * esize);
    if (target) target = heap::device_operand_open(target);
    if (collective(si) && !g_state.comm) {   // IPC transport
        if (nelems && !source) return set_error(SHMEMX_EINVAL);
        size_t total = 0;
        const int rc = ipc_collect(static_cast<char *>(target), static_cast<const char *>(source), esize,
                                   nelems, si.start, si.step, si.P, si.m, &total, s);
        if (rc == SHMEMX_OK && target) heap::device_wrote(user_target, total, s);
        trace(LOG_COLLECT, "%s over IPC: %zu bytes mine, %zu in all, set (%d,%d,%d)",
              fixed ? "fcollect" : "collect", nelems * esize, total, start, logstride, size);
        return rc;
    }
    std::vector<long long> counts(si.P, (long long)nelems);
    if (!fixed && collective(si)) {
        // every member's count (the reference passes it down a chain of
        // shmem_long_p, collect-linear.c:83-110)
        long long *cnt = static_cast<long long *>(grow(g_state.token, g_state.token_bytes,
                                                       sizeof(long long) * (si.P + 8)));
        if (!cnt) return set_error(SHMEMX_ENOMEM);
        const long long mine = (long long)nelems;
        SHMX_HIP(hipMemcpyAsync(cnt + si.m, &mine, sizeof mine, hipMemcpyHostToDevice, s));
        if (si.world) {
            SHMX_NCCL(ncclAllGather(cnt + si.m, cnt, 1, ncclInt64, g_state.comm, s));
        } else {
            SHMX_NCCL(ncclGroupStart());
            for (int i = 0; i < si.P; ++i) {
                if (i == si.m) continue;
                SHMX_NCCL(ncclSend(cnt + si.m, 1, ncclInt64, si.peer(i), g_state.comm, s));
                SHMX_NCCL(ncclRecv(cnt + i, 1, ncclInt64, si.peer(i), g_state.comm, s));
            }
            SHMX_NCCL(ncclGroupEnd());
        }
        SHMX_HIP(hipMemcpyAsync(counts.data(), cnt, sizeof(long long) * si.P,
                                hipMemcpyDeviceToHost, s));
        SHMX_HIP(hipStreamSynchronize(s));
    }
    std::vector<size_t> off(si.P + 1, 0);
    for (int i = 0; i < si.P; ++i) off[i + 1] = off[i] + (size_t)counts[i] * esize;
    const size_t mine = (size_t)counts[si.m] * esize, total = off[si.P];
    trace(LOG_COLLECT, "%s: %zu of %zu bytes at offset %zu, set (%d,%d,%d)",
          fixed ? "fcollect" : "collect", mine, total, off[si.m], start, logstride, size);
    if (!total) return SHMEMX_OK;
    if (!target || (mine && !source)) return set_error(SHMEMX_EINVAL);
    DevBuf in = device_in(source, mine, g_state.cws_src, g_state.cws_src_bytes, s);
    DevBuf out = device_out(target, total, g_state.cws_tgt, g_state.cws_tgt_bytes);
    if ((mine && !in.dev) || !out.dev) return set_error(SHMEMX_ENOMEM);
    if (mine && in.dev != out.dev + off[si.m])
        SHMX_HIP(hipMemcpyAsync(out.dev + off[si.m], in.dev, mine, hipMemcpyDeviceToDevice, s));
    if (collective(si)) {
        if (si.world && fixed && !g_state.force_collective) {
            SHMX_NCCL(ncclAllGather(out.dev + off[si.m], out.dev, mine, ncclUint8, g_state.comm, s));
        } else {
            SHMX_NCCL(ncclGroupStart());
            for (int i = 0; i < si.P; ++i) {
                if (i == si.m) continue;
                const size_t bi = off[i + 1] - off[i];
                if (mine) SHMX_NCCL(ncclSend(out.dev + off[si.m], mine, ncclUint8, si.peer(i), g_state.comm, s));
                if (bi) SHMX_NCCL(ncclRecv(out.dev + off[i], bi, ncclUint8, si.peer(i), g_state.comm, s));
            }
            SHMX_NCCL(ncclGroupEnd());
        }
    }
    finish(out, s);
    heap::device_wrote(user_target, total, s);
    return SHMEMX_OK;
}

// ------------------------------------------------------- checksum, verify
int checksum_impl(int type, const void *ptr, size_t nelems, unsigned long long *out) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    if (int rc = ensure_init()) return rc;
    if (!out || type_size(type) == 0) return set_error(SHMEMX_EINVAL);
    hipStream_t s = g_state.stream;
    g_state.lib_stream_dirty = true;   // until someone sees it drained (service.hip)
    const size_t bytes = nelems * type_size(type);
    if (bytes) ptr = heap::device_operand(ptr, bytes);   // mirrored heap: the HBM twin
    DevBuf in = device_in(ptr, bytes, g_state.cws_src, g_state.cws_src_bytes, s);
    if (bytes && !in.dev) return set_error(SHMEMX_ENOMEM);
    // The kernel stores the result straight into page-locked host memory,
    // then this call's epoch behind it: the host polls the epoch instead of
    // waiting for the stream (no copy command, no completion signal to wake
    // on; ~10 us per call).  A kernel that never gets there (an error) is
    // caught by the stream query every few microseconds, and then by the
    // stream wait, which reports it.
    static volatile unsigned long long *host_word = [] {
        void *p = nullptr;
        SHMX_HIP(hipHostMalloc(&p, 2 * sizeof(unsigned long long), hipHostMallocCoherent));
        return static_cast<volatile unsigned long long *>(p);
    }();
    static unsigned long long epoch = 0;
    ++epoch;
    if (launch_checksum(type, in.dev, nelems, const_cast<unsigned long long *>(host_word), epoch, s) !=
        hipSuccess)
        return set_error(SHMEMX_EINVAL);
    for (unsigned spins = 1; host_word[1] != epoch; ++spins) {
        if ((spins & 1023) == 0 && hipStreamQuery(s) != hipErrorNotReady) {
            SHMX_HIP(hipStreamSynchronize(s));   // done (or failed: FATAL)
            if (host_word[1] != epoch) fatal("shmemx_checksum", "the checksum kernel finished without a result");
            break;
        }
        __builtin_ia32_pause();
    }
    *out = host_word[0];
    return SHMEMX_OK;
}

}  // namespace

// Every member's 8-byte value, in set order (a collective over the set).
int exchange_u64(int start, int logstride, int size, unsigned long long mine,
                 std::vector<unsigned long long> &all) {
    SetInfo si;
    if (int rc = set_info(start, logstride, size, si)) return rc;
    all.assign(si.P, mine);
    if (collective(si) && (!g_state.comm || node::up())) {
        // the values travel in the node block's descriptors (host only: two
        // host barriers, where an RCCL all-gather costs a stream round trip);
        // RCCL only when the PEs share no node block
        node::Desc d;
        d.aux = mine;
        node::put_desc(d);
        node::barrier(si.start, si.step, si.P);
        for (int i = 0; i < si.P; ++i) all[i] = node::get_desc(si.peer(i)).aux;
        node::barrier(si.start, si.step, si.P);   // all read before any descriptor changes
    } else if (collective(si)) {
        hipStream_t s = g_state.stream;
        g_state.lib_stream_dirty = true;
    g_state.lib_stream_dirty = true;   // until someone sees it drained (service.hip)
        unsigned long long *d = static_cast<unsigned long long *>(
            grow(g_state.token, g_state.token_bytes, sizeof(unsigned long long) * (si.P + 8)));
        if (!d) return set_error(SHMEMX_ENOMEM);
        SHMX_HIP(hipMemcpyAsync(d + si.m, &mine, sizeof mine, hipMemcpyHostToDevice, s));
        if (si.world) {
            SHMX_NCCL(ncclAllGather(d + si.m, d, 1, ncclUint64, g_state.comm, s));
        } else {
            SHMX_NCCL(ncclGroupStart());
            for (int i = 0; i < si.P; ++i) {
                if (i == si.m) continue;
                SHMX_NCCL(ncclSend(d + si.m, 1, ncclUint64, si.peer(i), g_state.comm, s));
                SHMX_NCCL(ncclRecv(d + i, 1, ncclUint64, si.peer(i), g_state.comm, s));
            }
            SHMX_NCCL(ncclGroupEnd());
        }
        SHMX_HIP(hipMemcpyAsync(all.data(), d, sizeof(unsigned long long) * si.P,
                                hipMemcpyDeviceToHost, s));
        SHMX_HIP(hipStreamSynchronize(s));
    }
    return SHMEMX_OK;
}

namespace {

int verify_impl(int type, const void *target, int nreduce, int start, int logstride, int size,
                int *all_equal) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    SetInfo si;
    if (int rc = set_info(start, logstride, size, si)) return rc;
    if (!all_equal || nreduce < 0) return set_error(SHMEMX_EINVAL);
    unsigned long long mine = 0;
    if (int rc = checksum_impl(type, target, (size_t)nreduce, &mine)) return rc;
    std::vector<unsigned long long> all;
    if (int rc = exchange_u64(start, logstride, size, mine, all)) return rc;
    int eq = 1;
    for (unsigned long long v : all) eq &= v == mine;
    *all_equal = eq;
    trace(LOG_INFO, "verify: checksum %016llx, set (%d,%d,%d) %s", mine, start, logstride, size,
          eq ? "consistent" : "INCONSISTENT");
    return SHMEMX_OK;
}

// ---------------------------------------------------------- symmetric heap
void *heap_alloc(size_t alignment, size_t bytes) {
    if (ensure_init()) return nullptr;
    if (!bytes) return nullptr;
    void *p = heap::alloc(alignment, bytes);
    if (!p) set_error(SHMEMX_ENOMEM);
    trace(LOG_MEMORY, "shmem_malloc(%zu bytes, align %zu) = %p (HBM)", bytes, alignment, p);
    // $SHMEMX_RCCL_REGISTER=1: the segment is registered with RCCL as soon as
    // it exists (shmemx_rccl_register_heap; adopted from the N > 1 bench's
    // extras.rccl_registered); every PE allocates alike, so every PE registers
    static const bool reg = [] {
        const char *e = std::getenv("SHMEMX_RCCL_REGISTER");
        return e && *e == '1';
    }();
    if (p && reg && g_state.comm && !g_state.rccl_reg) {
        const int err = shmemx_reduce_last_error();
        (void)shmemx_rccl_register_heap(1);
        set_error(err);   // a refused registration is not the allocation's error
    }
    return p;
}

void heap_free(void *p) {
    if (!heap::free(p)) set_error(SHMEMX_EINVAL);
}

}  // namespace
}  // namespace shmx

using namespace shmx;

extern "C" {

void pshmem_barrier(int PE_start, int logPE_stride, int PE_size, long *pSync) {
    (void)pSync;
    barrier_impl(PE_start, logPE_stride, PE_size);
}

void pshmem_barrier_all(void) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (ensure_init()) return;
    barrier_impl(0, 0, g_state.npes);
}

void pshmem_broadcast32(void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync) {
    (void)pSync;
    broadcast_impl(4, target, source, nelems, PE_root, PE_start, logPE_stride, PE_size);
}

void pshmem_broadcast64(void *target, const void *source, size_t nelems, int PE_root, int PE_start,
                        int logPE_stride, int PE_size, long *pSync) {
    (void)pSync;
    broadcast_impl(8, target, source, nelems, PE_root, PE_start, logPE_stride, PE_size);
}

void pshmem_fcollect32(void *target, const void *source, size_t nelems, int PE_start,
                       int logPE_stride, int PE_size, long *pSync) {
    (void)pSync;
    collect_impl(4, target, source, nelems, PE_start, logPE_stride, PE_size, true);
}

void pshmem_fcollect64(void *target, const void *source, size_t nelems, int PE_start,
                       int logPE_stride, int PE_size, long *pSync) {
    (void)pSync;
    collect_impl(8, target, source, nelems, PE_start, logPE_stride, PE_size, true);
}

void pshmem_collect32(void *target, const void *source, size_t nelems, int PE_start,
                      int logPE_stride, int PE_size, long *pSync) {
    (void)pSync;
    collect_impl(4, target, source, nelems, PE_start, logPE_stride, PE_size, false);
}

void pshmem_collect64(void *target, const void *source, size_t nelems, int PE_start,
                      int logPE_stride, int PE_size, long *pSync) {
    (void)pSync;
    collect_impl(8, target, source, nelems, PE_start, logPE_stride, PE_size, false);
}

void *pshmem_malloc(size_t size) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    void *p = heap_alloc(0, size);
    pshmem_barrier_all();   // symmetric allocation is collective (symmem.c:209)
    return p;
}

void *pshmem_align(size_t alignment, size_t size) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    if (alignment == 0 || (alignment & (alignment - 1))) {
        set_error(SHMEMX_EINVAL);
        return nullptr;
    }
    void *p = heap_alloc(alignment, size);
    pshmem_barrier_all();
    return p;
}

void pshmem_free(void *ptr) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    pshmem_barrier_all();
    if (ptr) heap_free(ptr);
}

void *pshmem_realloc(void *ptr, size_t size) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    if (!ptr) return pshmem_malloc(size);
    if (!size) {
        pshmem_free(ptr);
        return nullptr;
    }
    const size_t old_bytes = heap::size_of(ptr);
    if (!old_bytes) {
        set_error(SHMEMX_EINVAL);
        return nullptr;
    }
    void *p = heap_alloc(0, size);
    if (p) {
        // the old contents move on the device (a mirrored heap's host stores
        // go up first, and the new block's host view is refreshed from HBM)
        const size_t keep = old_bytes < size ? old_bytes : size;
        const void *src = heap::device_operand(ptr, keep);
        {
            heap::DeviceWrite dst(p, keep, g_state.stream);
            // complete before the old block is freed (a device-to-device
            // hipMemcpy would return before the copy ran); the library stream
            // is ordered after the legacy default stream, so earlier writes
            // land first
            SHMX_HIP(hipMemcpyAsync(dst.ptr(), src, keep, hipMemcpyDefault, g_state.stream));
            SHMX_HIP(hipStreamSynchronize(g_state.stream));
        }
        heap_free(ptr);
    }
    pshmem_barrier_all();
    return p;
}

int shmemx_checksum(int type, const void *ptr, size_t nelems, unsigned long long *out) {
    return checksum_impl(type, ptr, nelems, out);
}

int shmemx_verify(int type, const void *target, int nreduce, int PE_start, int logPE_stride,
                  int PE_size, int *all_equal) {
    return verify_impl(type, target, nreduce, PE_start, logPE_stride, PE_size, all_equal);
}

void *pshmalloc(size_t size) { return pshmem_malloc(size); }
void pshfree(void *ptr) { pshmem_free(ptr); }
void *pshrealloc(void *ptr, size_t size) { return pshmem_realloc(ptr, size); }
void *pshmemalign(size_t alignment, size_t size) { return pshmem_align(alignment, size); }

#define SHMX_WEAK(ret, name, args) ret name args __attribute__((weak, alias("p" #name)));
SHMX_WEAK(void, shmem_barrier, (int, int, int, long *))
SHMX_WEAK(void, shmem_barrier_all, (void))
SHMX_WEAK(void, shmem_broadcast32, (void *, const void *, size_t, int, int, int, int, long *))
SHMX_WEAK(void, shmem_broadcast64, (void *, const void *, size_t, int, int, int, int, long *))
SHMX_WEAK(void, shmem_fcollect32, (void *, const void *, size_t, int, int, int, long *))
SHMX_WEAK(void, shmem_fcollect64, (void *, const void *, size_t, int, int, int, long *))
SHMX_WEAK(void, shmem_collect32, (void *, const void *, size_t, int, int, int, long *))
SHMX_WEAK(void, shmem_collect64, (void *, const void *, size_t, int, int, int, long *))
SHMX_WEAK(void *, shmem_malloc, (size_t))
SHMX_WEAK(void *, shmem_align, (size_t, size_t))
SHMX_WEAK(void, shmem_free, (void *))
SHMX_WEAK(void *, shmem_realloc, (void *, size_t))
SHMX_WEAK(void *, shmalloc, (size_t))
SHMX_WEAK(void, shfree, (void *))
SHMX_WEAK(void *, shrealloc, (void *, size_t))
SHMX_WEAK(void *, shmemalign, (size_t, size_t))

}  // extern "C"
