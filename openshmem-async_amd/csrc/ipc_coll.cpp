// Broadcast and [f]collect on the IPC transport ($SHMEMX_TRANSPORT=ipc):
// the collectives next to the reduction without RCCL.
//
// As in the reference's linear algorithms (broadcast-linear.c:54-74 — every
// non-root gets the root's source; fcollect-linear.c:69-91 /
// collect-linear.c:57-130 — every member gets every member's source at its
// running offset), each PE pulls what it needs with a HIP kernel straight out
// of the other PEs' HBM: from the symmetric heap when the operand lives there,
// otherwise from the owner's IPC scratch region, in rounds of half the
// scratch.  Loads only, after the owner's copy has completed and a barrier
// (the discipline of direct.cpp).  Host targets land in a device staging
// buffer first.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "heap.h"
#include "internal.h"
#include "node.h"
#include "shmem_reduce_mi355x.h"
#include "state.h"

namespace shmx {

namespace {

// Where `p` (bytes long) can be read by the peers: the heap, or nowhere.
bool in_heap(const void *p, size_t bytes, uint64_t *off) {
    return bytes && device_accessible(p) && heap::offset_of(p, bytes, off);
}

char *device_target(void *target, size_t bytes, bool *staged) {
    *staged = false;
    if (!bytes || device_accessible(target)) return static_cast<char *>(target);
    *staged = true;
    return static_cast<char *>(grow(g_state.cws_tgt, g_state.cws_tgt_bytes, bytes));
}

char *mapped(const node::Loc &l, int pe) {
    char *b = node::peer_base(static_cast<node::Region>(l.region), pe);
    if (!b) fatal("IPC collective: a member's region is not mapped", node::last_ipc_error());
    return b + l.off;
}

// Copy segments (any number) with one gather launch per 16.
void pull(std::vector<const void *> &from, std::vector<void *> &to, std::vector<size_t> &len,
          hipStream_t s) {
    for (size_t i = 0; i < from.size(); i += kMaxFoldInputs) {
        const int k = (int)std::min<size_t>(kMaxFoldInputs, from.size() - i);
        SHMX_HIP(launch_gather(from.data() + i, to.data() + i, len.data() + i, k, s));
    }
}

}  // namespace

int ipc_broadcast(char *target, const char *source, size_t bytes, int root_idx, int start,
                  int step, int P, int m, hipStream_t s) {
    size_t sbytes = 0;
    char *scr = ipc_scratch(&sbytes);
    if (!scr) return set_error(SHMEMX_ENOMEM);
    const size_t half = sbytes / 2;
    const bool root = m == root_idx;
    node::Desc d;
    uint64_t off = 0;
    bool staged = false;
    if (root) {
        staged = !in_heap(source, bytes, &off);
        d.src = staged ? node::Loc{node::kScratch, 0} : node::Loc{node::kHeap, off};
        d.count = staged ? 1 : 0;
    }
    node::put_desc(d);
    const bool single = bytes <= half;
    if (root && staged && single) SHMX_HIP(hipMemcpyAsync(scr, source, bytes, hipMemcpyDefault, s));
    node_sync(start, step, P, s);
    const int root_pe = start + root_idx * step;
    const node::Desc rd = root ? d : node::get_desc(root_pe);
    const bool chunked = rd.count != 0;
    char *rbase = root ? nullptr : mapped(rd.src, root_pe);
    bool tstaged = false;
    char *dst = root ? nullptr : device_target(target, bytes, &tstaged);
    if (!root && !dst) fatal("IPC broadcast", "no device staging buffer");
    const size_t C = chunked ? half : bytes;
    for (size_t c0 = 0; c0 < bytes; c0 += C) {
        const size_t cnt = std::min(C, bytes - c0);
        if (chunked && !single) {
            if (root) SHMX_HIP(hipMemcpyAsync(scr, source + c0, cnt, hipMemcpyDefault, s));
            node_sync(start, step, P, s);
        }
        if (!root) {
            std::vector<const void *> from{rbase + (chunked ? 0 : c0)};
            std::vector<void *> to{dst + c0};
            std::vector<size_t> len{cnt};
            pull(from, to, len, s);
        }
        node_done(start, step, P, s);   // the root's copy is no longer read
    }
    if (tstaged) {
        SHMX_HIP(hipMemcpyAsync(target, dst, bytes, hipMemcpyDeviceToHost, s));
        SHMX_HIP(hipStreamSynchronize(s));
    }
    return SHMEMX_OK;
}

int ipc_collect(char *target, const char *source, size_t esize, size_t nelems, int start,
                int step, int P, int m, size_t *total_out, hipStream_t s) {
    size_t sbytes = 0;
    char *scr = ipc_scratch(&sbytes);
    if (!scr) return set_error(SHMEMX_ENOMEM);
    const size_t half = sbytes / 2;
    const size_t mine = nelems * esize;
    node::Desc d;
    uint64_t off = 0;
    const bool staged = mine && !in_heap(source, mine, &off);
    d.src = staged ? node::Loc{node::kScratch, 0} : node::Loc{node::kHeap, off};
    d.count = (int64_t)nelems;   // collect-linear.c:83-110 passes these down a chain
    d.aux = staged ? 1 : 0;
    node::put_desc(d);
    // a staged source that fits is staged now (it is its own round 0)
    const bool prestaged = staged && mine <= half;
    if (prestaged) SHMX_HIP(hipMemcpyAsync(scr, source, mine, hipMemcpyDefault, s));
    node_sync(start, step, P, s);

    std::vector<node::Desc> desc(P);
    std::vector<size_t> len(P), offs(P + 1, 0);
    bool any_staged = false, late_stage = false;
    size_t most = 0;
    for (int i = 0; i < P; ++i) {
        desc[i] = i == m ? d : node::get_desc(start + i * step);
        len[i] = (size_t)desc[i].count * esize;
        offs[i + 1] = offs[i] + len[i];
        if (desc[i].aux) {
            any_staged = true;
            late_stage |= len[i] > half;
        }
        most = std::max(most, len[i]);
    }
    const size_t total = offs[P];
    *total_out = total;
    std::vector<char *> base(P, nullptr);
    for (int i = 0; i < P; ++i)
        if (len[i]) base[i] = mapped(desc[i].src, start + i * step);
    bool tstaged = false;
    char *dst = device_target(target, total, &tstaged);
    if (total && !dst) fatal("IPC collect", "no device staging buffer");
    const size_t H = any_staged ? half : std::max<size_t>(most, 1);
    const size_t rounds = total ? (most + H - 1) / H : 0;
    // every descriptor is read before any member may write its next one
    if (!rounds) node::barrier(start, step, P);
    for (size_t r = 0; r < rounds; ++r) {
        if (r > 0 || late_stage) {
            if (staged && !prestaged && mine > r * H)
                SHMX_HIP(hipMemcpyAsync(scr, source + r * H, std::min(H, mine - r * H), hipMemcpyDefault, s));
            node_sync(start, step, P, s);
        }
        std::vector<const void *> from;
        std::vector<void *> to;
        std::vector<size_t> n;
        for (int i = 0; i < P; ++i) {
            if (len[i] <= r * H) continue;
            from.push_back(base[i] + (desc[i].aux ? 0 : r * H));
            to.push_back(dst + offs[i] + r * H);
            n.push_back(std::min(H, len[i] - r * H));
        }
        pull(from, to, n, s);
        node_done(start, step, P, s);   // nobody reads this round's copies any more
    }
    if (tstaged) {
        SHMX_HIP(hipMemcpyAsync(target, dst, total, hipMemcpyDeviceToHost, s));
        SHMX_HIP(hipStreamSynchronize(s));
    }
    return SHMEMX_OK;
}

}  // namespace shmx
