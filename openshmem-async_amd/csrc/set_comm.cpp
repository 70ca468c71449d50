// Members-only RCCL communicators for partial active sets (SURVEY.md §8(e):
// "a (PE_start, logPE_stride, PE_size) sub-communicator ... cached").
//
// The reference walks the active set member by member and only members call
// (reduce-op.c:219-247); a PE outside the set never enters the collective.
// ncclCommSplit is collective over the whole parent communicator, so every
// non-member would have to join it: instead the set's first member makes a
// fresh unique id and hands it to the other members over the world
// communicator with grouped ncclSend/ncclRecv (point to point, members only),
// and the members run ncclCommInitRank among themselves, rank = index in the
// set.  The communicator is cached per (PE_start, logPE_stride, PE_size) for
// the life of the job, so a set pays the setup once and then gets RCCL's own
// reduce-scatter / all-gather / all-reduce kernels, as the whole job does.
//
// Every member of a set meets it at the same call (OpenSHMEM's rule that all
// members issue the same collective sequence), so every member finds the set
// cached, or not, alike: the planner's choices stay identical across them.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <tuple>
#include <vector>

#include "state.h"

namespace shmx {

namespace {

using SetKey = std::tuple<int, int, int>;

std::map<SetKey, ncclComm_t> &cache() {
    static std::map<SetKey, ncclComm_t> c;
    return c;
}

// sets whose members agreed not to make a communicator (some member's cache
// was full): they keep the world communicator's schedules
std::set<SetKey> &refused() {
    static std::set<SetKey> r;
    return r;
}

// $SHMEMX_SET_COMMS_MAX: communicators one PE keeps (default 16; RCCL's
// buffers cost device memory per communicator)
size_t cache_cap() {
    static const size_t cap = [] {
        const char *e = std::getenv("SHMEMX_SET_COMMS_MAX");
        const long v = e && *e ? std::atol(e) : 16;
        return (size_t)(v < 0 ? 0 : v);
    }();
    return cap;
}

// one key per set of PEs: a one-member or a stride-free set has one spelling
SetKey key_of(int start, int logstride, int size) {
    return SetKey(start, size == 1 ? 0 : logstride, size);
}

}  // namespace

bool set_comms_enabled() {
    // $SHMEMX_SET_COMMS=0: partial sets keep the grouped send/recv schedules
    // on the world communicator (A2A / GATHER); every PE must agree
    static const bool on = [] {
        const char *e = std::getenv("SHMEMX_SET_COMMS");
        return !(e && *e == '0');
    }();
    return on;
}

bool set_comm_cached(int start, int logstride, int size) {
    return cache().count(key_of(start, logstride, size)) != 0;
}

int set_comms_cached() { return (int)cache().size(); }

bool set_comm_refused(int start, int logstride, int size) {
    return refused().count(key_of(start, logstride, size)) != 0;
}

bool set_comm_prepare(int start, int logstride, int size, int member, hipStream_t s) {
    const SetKey k = key_of(start, logstride, size);
    if (cache().count(k)) return true;
    if (refused().count(k)) return false;
    // the members agree first (one 8-byte exchange among them): every member
    // must have room, or none makes the communicator and all plan without it
    std::vector<unsigned long long> all;
    const unsigned long long mine = cache().size() < cache_cap() ? 1 : 0;
    if (exchange_u64(start, logstride, size, mine, all)) {
        refused().insert(k);   // (a bad set fails alike on every member)
        return false;
    }
    for (unsigned long long v : all) {
        if (!v) {
            refused().insert(k);
            trace(LOG_INFO, "set (%d,%d,%d): a member holds %zu set communicators already "
                  "($SHMEMX_SET_COMMS_MAX); the set keeps the world communicator", start, logstride, size,
                  cache_cap());
            return false;
        }
    }
    return set_comm(start, logstride, size, member, s) != nullptr;
}

ncclComm_t set_comm(int start, int logstride, int size, int member, hipStream_t s) {
    const SetKey k = key_of(start, logstride, size);
    auto it = cache().find(k);
    if (it != cache().end()) return it->second;
    if (!g_state.comm) fatal("set communicator", "no world RCCL communicator");
    const int step = 1 << logstride;
    ncclUniqueId id;
    std::memset(&id, 0, sizeof id);
    if (member == 0 && ncclGetUniqueId(&id) != ncclSuccess) fatal("set communicator", "ncclGetUniqueId failed");
    // the id travels device to device on the world communicator, from the
    // first member to each of the others (members only)
    void *buf = nullptr;
    SHMX_HIP(hipMalloc(&buf, sizeof id));
    if (member == 0) SHMX_HIP(hipMemcpyAsync(buf, &id, sizeof id, hipMemcpyHostToDevice, s));
    SHMX_NCCL(ncclGroupStart());
    if (member == 0) {
        for (int i = 1; i < size; ++i)
            SHMX_NCCL(ncclSend(buf, sizeof id, ncclUint8, start + i * step, g_state.comm, s));
    } else {
        SHMX_NCCL(ncclRecv(buf, sizeof id, ncclUint8, start, g_state.comm, s));
    }
    SHMX_NCCL(ncclGroupEnd());
    if (member != 0) SHMX_HIP(hipMemcpyAsync(&id, buf, sizeof id, hipMemcpyDeviceToHost, s));
    SHMX_HIP(hipStreamSynchronize(s));
    SHMX_HIP(hipFree(buf));
    ncclComm_t c = nullptr;
    SHMX_NCCL(ncclCommInitRank(&c, size, id, member));
    cache()[k] = c;
    trace(LOG_INIT, "RCCL communicator of set (%d,%d,%d) up: rank %d of %d", start, logstride, size, member,
          size);
    return c;
}

void set_comms_release() {
    for (auto &kv : cache())
        if (kv.second) (void)ncclCommDestroy(kv.second);
    cache().clear();
    refused().clear();
}

}  // namespace shmx
