// Test double of RCCL (tests only, never shipped): the subset of the RCCL C
// API libshmem_reduce_mi355x.so calls, with RCCL's semantics, for several
// processes that share ONE GPU — which the real RCCL refuses.  It lets the
// library's own RCCL-transport code (reduce-scatter + all-gather with a tail,
// all-reduce, A2A and GATHER over grouped send/recv, broadcast, [f]collect,
// barrier, verify) run across real processes with real device pointers on a
// one-GPU box, against the oracle.
//
// Loaded by the test with RTLD_GLOBAL after torch and before the library,
// so the library's nccl* references bind here; its libamdhip64 dependency
// then resolves to the HIP runtime torch already loaded.
//
// Mechanism: every call first waits for its stream (RCCL orders after the
// stream's earlier work), copies device data to the host, moves it between
// processes through per-(sender, receiver) mailboxes in one /dev/shm segment
// per communicator, and copies results back.  Collectives are built from the
// same point-to-point engine; reductions combine the ranks' data in rank
// order NOT the reference's: a reduce-scatter folds chunk c in ring order,
// starting at rank (c + 1) mod n and ending at c, as RCCL's ring reduce-
// scatter does; an all-reduce splits the array into n chunks and folds chunk
// j in descending rotation j, j - 1, ..., j + 1 (mod n), yet another order.
// So a floating sum or product through the RCCL transport differs from the
// reference's PE_start-order fold in its last bits, as real RCCL's does, and
// the tests must hold it to the stated bound, not to bit equality.  Group
// calls run at ncclGroupEnd.  Nothing here is fast; it is exact arithmetic in
// a fixed order, and it deadlocks only where RCCL would.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sched.h>
#include <time.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

struct ncclComm {
    int rank = 0, n = 1;
    char *base = nullptr;
    size_t cap = 0, stride = 0, bytes = 0;
};

namespace {

constexpr uint64_t kMagic = 0x4641'4b45'5243'434cULL;   // "FAKERCCL"

struct Header {
    std::atomic<int> attached;
};
constexpr size_t kHeader = 4096;

struct Box {
    std::atomic<uint64_t> len;   // bytes waiting in data, 0 = empty
};
constexpr size_t kBoxHead = 64;

[[noreturn]] void die(const char *what) {
    std::fprintf(stderr, "fake_rccl: %s\n", what);
    std::abort();
}

void check(hipError_t e, const char *what) {
    if (e != hipSuccess) {
        std::fprintf(stderr, "fake_rccl: %s: %s\n", what, hipGetErrorString(e));
        std::abort();
    }
}

Box *box(const ncclComm *c, int from, int to) {
    return reinterpret_cast<Box *>(c->base + kHeader + ((size_t)from * c->n + to) * c->stride);
}
char *box_data(Box *b) { return reinterpret_cast<char *>(b) + kBoxHead; }

size_t dt_size(ncclDataType_t t) {
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: die("unsupported data type");
    }
}

std::string shm_name(const ncclUniqueId &id) {
    char hex[33];
    for (int i = 0; i < 16; ++i) std::snprintf(hex + 2 * i, 3, "%02x", (unsigned char)id.internal[8 + i]);
    return std::string("/fake_rccl_") + hex;
}

// ------------------------------------------------------ point-to-point engine
struct P2p {
    bool send;
    int peer;
    char *host;
    size_t bytes, done;
};

// Progress every pending send/recv until all are complete; messages between
// one pair in one direction go in call order, in mailbox-sized pieces.
// Waiting: spin, then yield, then sleep in growing steps, so 8 ranks waiting
// on each other do not starve the ones copying (the box gives a job a CPU
// share, not a CPU per rank).
void backoff(unsigned spins) {
    if (spins < 256) return;
    if (spins < 1024) {
        sched_yield();
        return;
    }
    struct timespec ts = {0, (long)(spins < 1024 + 64 ? 5 : 50) * 1000};
    nanosleep(&ts, nullptr);
}

void run(const ncclComm *c, std::vector<P2p> &ops) {
    const auto t0 = std::chrono::steady_clock::now();
    unsigned idle = 0;
    for (;;) {
        bool left = false, progressed = false;
        for (size_t i = 0; i < ops.size(); ++i) {
            P2p &o = ops[i];
            if (o.done == o.bytes) continue;
            bool blocked = false;   // an earlier message on the same lane first
            for (size_t j = 0; j < i && !blocked; ++j)
                blocked = ops[j].send == o.send && ops[j].peer == o.peer && ops[j].done < ops[j].bytes;
            left = true;
            if (blocked) continue;
            if (o.send) {
                Box *b = box(c, c->rank, o.peer);
                if (b->len.load(std::memory_order_acquire) != 0) continue;
                const size_t k = std::min(c->cap, o.bytes - o.done);
                std::memcpy(box_data(b), o.host + o.done, k);
                b->len.store(k, std::memory_order_release);
                o.done += k;
            } else {
                Box *b = box(c, o.peer, c->rank);
                const uint64_t k = b->len.load(std::memory_order_acquire);
                if (k == 0) continue;
                if (k > o.bytes - o.done) die("message longer than the posted receive");
                std::memcpy(o.host + o.done, box_data(b), k);
                b->len.store(0, std::memory_order_release);
                o.done += k;
            }
            progressed = true;
        }
        if (!left) return;
        if (progressed) {
            idle = 0;
        } else {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
                die("no progress for 120 s (unmatched send/recv)");
            backoff(++idle);
        }
    }
}

std::vector<char> to_host(const void *dev, size_t bytes) {
    std::vector<char> h(bytes);
    if (bytes) check(hipMemcpy(h.data(), dev, bytes, hipMemcpyDefault), "hipMemcpy D2H");
    return h;
}
void to_dev(void *dev, const char *host, size_t bytes) {
    if (bytes) check(hipMemcpy(dev, host, bytes, hipMemcpyDefault), "hipMemcpy H2D");
}
void wait_stream(hipStream_t s) { check(hipStreamSynchronize(s), "hipStreamSynchronize"); }

// ------------------------------------------------------------- reductions
template <typename T>
void combine_t(T *acc, const T *x, size_t n, ncclRedOp_t op) {
    for (size_t i = 0; i < n; ++i) {
        switch (op) {
        case ncclSum: acc[i] = acc[i] + x[i]; break;
        case ncclProd: acc[i] = acc[i] * x[i]; break;
        case ncclMin: acc[i] = x[i] < acc[i] ? x[i] : acc[i]; break;
        case ncclMax: acc[i] = x[i] > acc[i] ? x[i] : acc[i]; break;
        default: die("unsupported reduction op");
        }
    }
}
// wrapping integer arithmetic, as RCCL's
template <typename T, typename U>
void combine_int(T *acc, const T *x, size_t n, ncclRedOp_t op) {
    if (op == ncclSum || op == ncclProd) {
        for (size_t i = 0; i < n; ++i)
            acc[i] = (T)(op == ncclSum ? (U)acc[i] + (U)x[i] : (U)acc[i] * (U)x[i]);
        return;
    }
    combine_t(acc, x, n, op);
}

void combine(char *acc, const char *x, size_t count, ncclDataType_t t, ncclRedOp_t op) {
    switch (t) {
    case ncclInt32: combine_int<int32_t, uint32_t>((int32_t *)acc, (const int32_t *)x, count, op); break;
    case ncclUint32: combine_int<uint32_t, uint32_t>((uint32_t *)acc, (const uint32_t *)x, count, op); break;
    case ncclInt64: combine_int<int64_t, uint64_t>((int64_t *)acc, (const int64_t *)x, count, op); break;
    case ncclUint64: combine_int<uint64_t, uint64_t>((uint64_t *)acc, (const uint64_t *)x, count, op); break;
    case ncclUint8: combine_int<uint8_t, uint32_t>((uint8_t *)acc, (const uint8_t *)x, count, op); break;
    case ncclInt8: combine_int<int8_t, uint32_t>((int8_t *)acc, (const int8_t *)x, count, op); break;
    case ncclFloat32: combine_t((float *)acc, (const float *)x, count, op); break;
    case ncclFloat64: combine_t((double *)acc, (const double *)x, count, op); break;
    default: die("unsupported reduction type");
    }
}

// Every rank's `bytes` of `mine`, in rank order (the exchange of all-reduce,
// all-gather and, chunk by chunk, reduce-scatter).
std::vector<std::vector<char>> exchange(const ncclComm *c, const std::vector<std::vector<char>> &out,
                                        size_t in_bytes) {
    std::vector<std::vector<char>> in(c->n);
    std::vector<P2p> ops;
    for (int p = 0; p < c->n; ++p) {
        if (p == c->rank) continue;
        in[p].resize(in_bytes);
        ops.push_back({true, p, const_cast<char *>(out[p].data()), out[p].size(), 0});
        ops.push_back({false, p, in[p].data(), in_bytes, 0});
    }
    run(c, ops);
    return in;
}

// pending group
struct Pending {
    bool send;
    void *buf;
    size_t bytes;
    int peer;
    ncclComm *comm;
    hipStream_t stream;
};
int g_depth = 0;
std::vector<Pending> g_group;

bool ranges_overlap(const void *a, size_t na, const void *b, size_t nb) {
    const char *x = static_cast<const char *>(a), *y = static_cast<const char *>(b);
    return na && nb && x < y + nb && y < x + na;
}

// Buffer rules real RCCL does not check but relies on (anything else is a
// race there, even where this double would happen to get it right): a
// collective is in place only in RCCL's exact layout, and a group's receive
// buffers overlap neither each other nor any of its send buffers.
void check_layout(const char *what, const void *send, size_t send_bytes, const void *recv,
                  size_t recv_bytes, const void *inplace_send) {
    if (send == inplace_send) return;
    if (ranges_overlap(send, send_bytes, recv, recv_bytes)) {
        std::fprintf(stderr, "fake_rccl: %s: send and receive buffers overlap outside RCCL's in-place layout\n",
                     what);
        std::abort();
    }
}

void flush_group() {
    if (g_group.empty()) return;
    for (size_t i = 0; i < g_group.size(); ++i) {
        if (g_group[i].send) continue;
        for (size_t j = 0; j < g_group.size(); ++j)
            if (j != i && ranges_overlap(g_group[i].buf, g_group[i].bytes, g_group[j].buf, g_group[j].bytes))
                die(g_group[j].send ? "a group receives into one of its send buffers"
                                    : "two receives of a group overlap");
    }
    for (const Pending &p : g_group) wait_stream(p.stream);
    ncclComm *c = g_group.front().comm;
    std::vector<std::vector<char>> host(g_group.size());
    std::vector<P2p> ops;
    for (size_t i = 0; i < g_group.size(); ++i) {
        const Pending &p = g_group[i];
        if (p.comm != c) die("one group over two communicators");
        host[i] = p.send ? to_host(p.buf, p.bytes) : std::vector<char>(p.bytes);
        ops.push_back({p.send, p.peer, host[i].data(), p.bytes, 0});
    }
    run(c, ops);
    for (size_t i = 0; i < g_group.size(); ++i)
        if (!g_group[i].send) to_dev(g_group[i].buf, host[i].data(), g_group[i].bytes);
    g_group.clear();
}

}  // namespace

extern "C" {

const char *ncclGetErrorString(ncclResult_t r) {
    return r == ncclSuccess ? "no error (fake_rccl)" : "error (fake_rccl)";
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    std::memset(id, 0, sizeof *id);
    std::memcpy(id->internal, &kMagic, 8);
    const int fd = open("/dev/urandom", O_RDONLY);
    if (fd < 0 || read(fd, id->internal + 8, 16) != 16) die("cannot read /dev/urandom");
    close(fd);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *out, int nranks, ncclUniqueId id, int rank) {
    uint64_t magic;
    std::memcpy(&magic, id.internal, 8);
    if (magic != kMagic) die("unique id not made by fake_rccl");
    if (nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    auto *c = new ncclComm;
    c->rank = rank;
    c->n = nranks;
    const char *kb = std::getenv("FAKE_RCCL_BOX_KB");
    c->cap = (size_t)(kb ? std::atoi(kb) : 1024) << 10;
    c->stride = kBoxHead + c->cap;
    c->bytes = kHeader + (size_t)nranks * nranks * c->stride;
    const std::string name = shm_name(id);
    const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)c->bytes) != 0) die("cannot create the shared segment");
    c->base = static_cast<char *>(mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
    close(fd);
    if (c->base == MAP_FAILED) die("mmap");
    auto *h = reinterpret_cast<Header *>(c->base);
    h->attached.fetch_add(1);
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    while (h->attached.load() < nranks) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) die("ranks missing at init");
        backoff(++spins);
    }
    if (rank == 0) shm_unlink(name.c_str());   // every rank has it mapped
    *out = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (c) {
        munmap(c->base, c->bytes);
        delete c;
    }
    return ncclSuccess;
}

// buffer registration: the double moves data through its own mailboxes
// whatever is registered; it records nothing
ncclResult_t ncclCommRegister(const ncclComm_t, void *, size_t, void **handle) {
    static int token;
    *handle = &token;
    return ncclSuccess;
}

ncclResult_t ncclCommDeregister(const ncclComm_t, void *) { return ncclSuccess; }

ncclResult_t ncclGroupStart() {
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth == 0) flush_group();
    return ncclSuccess;
}

static ncclResult_t p2p(bool send, void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c,
                        hipStream_t s) {
    if (peer < 0 || peer >= c->n || peer == c->rank) return ncclInvalidArgument;
    g_group.push_back({send, buf, count * dt_size(t), peer, c, s});
    if (g_depth == 0) flush_group();
    return ncclSuccess;
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c,
                      hipStream_t s) {
    return p2p(true, const_cast<void *>(buf), count, t, peer, c, s);
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
    return p2p(false, buf, count, t, peer, c, s);
}

ncclResult_t ncclAllReduce(const void *send, void *recv, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t c, hipStream_t s) {
    if (g_depth) die("collective inside a group (not used by the library)");
    const size_t b = count * dt_size(t);
    check_layout("ncclAllReduce", send, b, recv, b, recv);
    wait_stream(s);
    std::vector<std::vector<char>> out(c->n, to_host(send, b));
    auto in = exchange(c, out, b);
    in[c->rank] = out[c->rank];
    // chunk j of n (contiguous elements) in descending rotation from j
    const size_t es = dt_size(t), per = (count + c->n - 1) / c->n;
    std::vector<char> acc(b);
    for (int j = 0; j < c->n; ++j) {
        const size_t lo = std::min(count, j * per), hi = std::min(count, (j + 1) * per);
        if (hi == lo) continue;
        std::memcpy(acc.data() + lo * es, in[j].data() + lo * es, (hi - lo) * es);
        for (int k = 1; k < c->n; ++k) {
            const int p = ((j - k) % c->n + c->n) % c->n;
            combine(acc.data() + lo * es, in[p].data() + lo * es, hi - lo, t, op);
        }
    }
    to_dev(recv, acc.data(), b);
    return ncclSuccess;
}

ncclResult_t ncclReduceScatter(const void *send, void *recv, size_t count, ncclDataType_t t,
                               ncclRedOp_t op, ncclComm_t c, hipStream_t s) {
    if (g_depth) die("collective inside a group (not used by the library)");
    const size_t b = count * dt_size(t);
    // in place: recvbuff == sendbuff + rank * recvcount
    check_layout("ncclReduceScatter", send, b * c->n, recv, b,
                 static_cast<const char *>(recv) - (size_t)c->rank * b);
    wait_stream(s);
    const std::vector<char> all = to_host(send, b * c->n);
    std::vector<std::vector<char>> out(c->n);
    for (int p = 0; p < c->n; ++p) out[p].assign(all.begin() + p * b, all.begin() + (p + 1) * b);
    auto in = exchange(c, out, b);
    in[c->rank] = out[c->rank];
    // ring order: my chunk starts at rank + 1 and ends with my own
    std::vector<char> acc = in[(c->rank + 1) % c->n];
    for (int k = 2; k <= c->n; ++k) combine(acc.data(), in[(c->rank + k) % c->n].data(), count, t, op);
    to_dev(recv, acc.data(), b);
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t t, ncclComm_t c,
                           hipStream_t s) {
    if (g_depth) die("collective inside a group (not used by the library)");
    const size_t b = count * dt_size(t);
    // in place: sendbuff == recvbuff + rank * sendcount
    check_layout("ncclAllGather", send, b, recv, b * c->n,
                 static_cast<const char *>(recv) + (size_t)c->rank * b);
    wait_stream(s);
    std::vector<std::vector<char>> out(c->n, to_host(send, b));
    auto in = exchange(c, out, b);
    in[c->rank] = out[c->rank];
    std::vector<char> all(b * c->n);
    for (int p = 0; p < c->n; ++p)
        if (b) std::memcpy(all.data() + p * b, in[p].data(), b);
    to_dev(recv, all.data(), all.size());
    return ncclSuccess;
}

ncclResult_t ncclBroadcast(const void *send, void *recv, size_t count, ncclDataType_t t, int root,
                           ncclComm_t c, hipStream_t s) {
    if (g_depth) die("collective inside a group (not used by the library)");
    if (root < 0 || root >= c->n) return ncclInvalidArgument;
    const size_t b = count * dt_size(t);
    if (c->rank == root) check_layout("ncclBroadcast", send, b, recv, b, recv);
    wait_stream(s);
    std::vector<P2p> ops;
    std::vector<char> data;
    if (c->rank == root) {
        data = to_host(send, b);
        for (int p = 0; p < c->n; ++p)
            if (p != root) ops.push_back({true, p, data.data(), b, 0});
    } else {
        data.resize(b);
        ops.push_back({false, root, data.data(), b, 0});
    }
    run(c, ops);
    if (c->rank != root || recv != send) to_dev(recv, data.data(), b);
    return ncclSuccess;
}

}  // extern "C"
