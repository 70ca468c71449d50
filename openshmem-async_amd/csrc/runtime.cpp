// Host runtime of libshmem_reduce_mi355x.so: PE identity, HIP stream, RCCL
// communicator, device workspaces, and the reduction engine that every
// shmem_<T>_<op>_to_all entry point (entry.cpp) lands in.
//
// Reference mapping (all paths under /root/reference/src):
//   shmemi_udr_<T>_to_all  reduce/reduce-op.c:169-260  -> reduce_device()
//     copy write_to=source (:213-216)     -> fold kernel, 1 input (P == 1)
//     barrier (:217,:250)                  -> stream order of RCCL + kernels
//     per-peer shmem_getmem into pWrk      -> RCCL shard exchange over xGMI
//       (:219-248, ptp/putget.c:234-240)
//     (*the_op)(write_to, pWrk) (:231-235) -> one fold kernel over P shards
//     overlap temp (:166-167,187-203)      -> stage source to a workspace
//   GET_STATE(mype) utils/state.h:100-101  -> g_state.pe
//   shmem_init      updown/updown.c:160    -> shmem_init / shmemx_init_attr
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>

#include "heap.h"
#include "internal.h"
#include "mirror.h"
#include "node.h"
#include "shmem_reduce_mi355x.h"
#include "state.h"

namespace shmx {

State g_state;

std::recursive_mutex g_mu;
static thread_local int t_last_error = SHMEMX_OK;

int set_error(int e) {
    t_last_error = e;
    return e;
}

void clear_error() { t_last_error = SHMEMX_OK; }

// Trace facility with the reference's interface (utils/trace.c:55-140,
// 240-431): $SHMEM_LOG_LEVELS lists facilities (delimiters ",:;",
// case-insensitive, "all"), $SHMEM_LOG_FILE redirects the output, FATAL is
// always on; lines are "%-8.8f PE %d: LEVEL: msg" with seconds since start.
static const char *const kLogNames[LOG_N] = {"FATAL", "INIT", "BARRIER", "BROADCAST",
                                             "REDUCTION", "COLLECT", "MEMORY", "INFO"};

struct LogState {
    bool on[LOG_N] = {true};
    FILE *out = stderr;
    LogState() {
        if (const char *levels = std::getenv("SHMEM_LOG_LEVELS")) {
            std::string all(levels);
            size_t pos = 0;
            while (pos <= all.size()) {
                const size_t end = all.find_first_of(",:;", pos);
                std::string tok = all.substr(pos, end == std::string::npos ? std::string::npos : end - pos);
                for (auto &c : tok) c = (char)std::toupper((unsigned char)c);
                for (int i = 0; i < LOG_N; ++i)
                    if (tok == "ALL" || tok == kLogNames[i]) on[i] = true;
                if (end == std::string::npos) break;
                pos = end + 1;
            }
        }
        if (const char *f = std::getenv("SHMEM_LOG_FILE")) {
            if (FILE *fp = std::fopen(f, "a")) out = fp;
        }
    }
};

static LogState &log_state() {
    static LogState st;
    return st;
}

bool log_enabled(int level) { return level >= 0 && level < LOG_N && log_state().on[level]; }

void trace(int level, const char *fmt, ...) {
    if (!log_enabled(level)) return;
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                   g_state.t0).count();
    char msg[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    FILE *out = log_state().out;
    fprintf(out, "%-8.8f PE %d: %s: %s\n", t, g_state.pe, kLogNames[level], msg);
    fflush(out);
}

[[noreturn]] void fatal(const char *what, const char *detail) {
    trace(LOG_FATAL, "%s: %s", what, detail);
    std::abort();
}

static int env_int(const char *a, const char *b, int dflt);

HostSignal next_host_signal() {
    static unsigned long long *word = [] {
        void *p = nullptr;
        SHMX_HIP(hipHostMalloc(&p, sizeof(unsigned long long), hipHostMallocCoherent));
        *static_cast<volatile unsigned long long *>(p) = 0;
        return static_cast<unsigned long long *>(p);
    }();
    static unsigned long long value = 0;
    return HostSignal{word, ++value};
}

void wait_host_signal(const HostSignal &sig, hipStream_t s) {
    // Only a blocking entry point spins on the word and returns the moment it
    // arrives.  Anywhere else (DIRECT under the stream-ordered API) the caller
    // may wait for the stream right after, and a hipStreamSynchronize entered
    // while a kernel is still retiring costs ~9 us more than the retiring
    // itself; polling hipStreamQuery until the stream is idle is worse still
    // (profiles/r03_latency_ab.txt): there the stream wait is the wait.
    if (!g_state.return_on_signal) {
        SHMX_HIP(hipStreamSynchronize(s));
        if (s == g_state.stream) g_state.lib_stream_dirty = false;
        return;
    }
    const volatile unsigned long long *w = sig.word;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned k = 1;; ++k) {
        if (*w == sig.value) {
            // everything enqueued on s before the signal has completed
            if (s == g_state.stream) g_state.lib_stream_dirty = false;
            return;
        }
        __builtin_ia32_pause();
        if ((k & 1023) == 0) {
            // a drained stream (its work is complete whatever the word says)
            // or an error: the stream wait settles it; long work: stop spinning
            const hipError_t e = hipStreamQuery(s);
            if (e != hipErrorNotReady) break;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
        }
    }
    SHMX_HIP(hipStreamSynchronize(s));
    if (s == g_state.stream) g_state.lib_stream_dirty = false;
}

static int env_int(const char *a, const char *b, int dflt) {
    for (const char *k : {a, b}) {
        if (!k) continue;
        if (const char *v = std::getenv(k)) {
            if (*v) return std::atoi(v);
        }
    }
    return dflt;
}

static int parse_algo(const char *s) {
    if (!s) return SHMEMX_ALGO_AUTO;
    std::string v(s);
    if (v == "rccl") return SHMEMX_ALGO_RCCL;
    if (v == "a2a") return SHMEMX_ALGO_A2A;
    if (v == "gather") return SHMEMX_ALGO_GATHER;
    if (v == "allreduce") return SHMEMX_ALGO_ALLREDUCE;
    if (v == "direct") return SHMEMX_ALGO_DIRECT;
    if (v == "signal") return SHMEMX_ALGO_SIGNAL;
    return SHMEMX_ALGO_AUTO;
}

static bool ipc_transport_env() {
    const char *t = std::getenv("SHMEMX_TRANSPORT");
    return t && std::string(t) == "ipc";
}

// A job id: RCCL's unique id, or 128 random bytes on the IPC transport
// (which never starts RCCL).
static bool make_uid(ncclUniqueId *id) {
    if (!ipc_transport_env()) return ncclGetUniqueId(id) == ncclSuccess;
    const int fd = open("/dev/urandom", O_RDONLY);
    if (fd < 0) return false;
    const bool ok = read(fd, id, sizeof *id) == (ssize_t)sizeof *id;
    close(fd);
    return ok;
}

// Settings every PE must share: they choose each call's algorithm and
// schedule, and every member of a set must run the same one (reduce-op.c:
// 213-250: one call sequence on every PE).  A launcher that exports one on
// some ranks only would make the plans diverge and the collectives mismatch,
// so init compares a hash of them across the PEs once.
// (SHMEM_SYMMETRIC_HEAP_SIZE is compared as the sizes themselves, at the
// first allocation: heap.cpp.)
static const char *const kPlanSettings[] = {
    "SHMEM_REDUCE_ALGO",        "SHMEMX_AUTO_FULL",         "SHMEMX_AUTO_PARTIAL",
    "SHMEMX_ALLREDUCE_MAX_KB",  "SHMEMX_DIRECT_ONESHOT_KB", "SHMEMX_FUSED_TWOSHOT_KB",
    "SHMEMX_FUSED_ONESHOT",     "SHMEMX_SET_COMMS",         "SHMEMX_SET_COMMS_MAX",
    "SHMEMX_STAGE_CHUNK_MB",    "SHMEMX_DIRECT_SCRATCH_MB", "SHMEMX_TRANSPORT"};

static std::string plan_settings() {
    std::string t;
    for (const char *k : kPlanSettings) {
        const char *v = std::getenv(k);
        if (v) t += std::string(k) + "=" + v + " ";
    }
    return t;
}

static void check_plan_settings() {
    const std::string mine = plan_settings();
    unsigned long long h = 1469598103934665603ull;   // FNV-1a
    for (unsigned char c : mine) h = (h ^ c) * 1099511628211ull;
    std::vector<unsigned long long> all;
    if (exchange_u64(0, 0, g_state.npes, h, all)) fatal("shmem_init", "cannot compare the PEs' settings");
    for (size_t q = 0; q < all.size(); ++q) {
        if (all[q] == h) continue;
        const std::string why = "the algorithm settings differ across PEs (PE " + std::to_string(q) +
                                " has others); this PE's: " + (mine.empty() ? "(none set)" : mine);
        fatal("shmem_init", why.c_str());
    }
}

static int init_locked(int pe, int npes, int device, const void *uid) {
    if (g_state.inited) return SHMEMX_OK;
    if (npes < 1 || pe < 0 || pe >= npes) return set_error(SHMEMX_EINVAL);
    int ndev = 0;
    SHMX_HIP(hipGetDeviceCount(&ndev));
    if (ndev < 1) fatal("shmem_init", "no HIP device visible");
    if (device < 0 && !(npes == 1 && hipGetDevice(&device) == hipSuccess)) device = pe % ndev;
    if (device < 0 || device >= ndev) return set_error(SHMEMX_EINVAL);
    SHMX_HIP(hipSetDevice(device));
    // A BLOCKING stream: ordered after the legacy default stream, where a
    // plain HIP program (and PyTorch's default stream) writes the buffers it
    // then hands to the blocking entry points.  Work on other non-blocking
    // streams must be synchronised by the caller, as for any HIP library.
    SHMX_HIP(hipStreamCreate(&g_state.stream));
    g_state.force_collective = env_int("SHMEMX_FORCE_COLLECTIVE", nullptr, 0) != 0;
    g_state.ipc_only = ipc_transport_env();
    g_state.node_shared = false;
    g_state.xchg = false;
    g_state.gpu_shared = false;
    if (npes > 1 || g_state.force_collective) {
        ncclUniqueId id;
        if (npes > 1) {
            if (!uid) return set_error(SHMEMX_EINVAL);
            std::memcpy(&id, uid, sizeof id);
        } else if (!make_uid(&id)) {
            fatal("shmem_init", "cannot make a job id");
        }
        if (!g_state.ipc_only) SHMX_NCCL(ncclCommInitRank(&g_state.comm, npes, id, pe));
        // the intra-node block (symmetric-heap IPC handles, host barrier):
        // required on the IPC transport, an extra (DIRECT) otherwise
        bool attached = node::attach(pe, npes, &id, sizeof id);
        if (!attached && g_state.ipc_only) fatal("shmem_init", "cannot attach the intra-node block (/dev/shm)");
        if (g_state.comm && npes > 1) {
            // every PE must have the block, or none uses it
            int *flag = nullptr;
            SHMX_HIP(hipMalloc(&flag, sizeof(int)));
            const int mine = attached ? 1 : 0;
            SHMX_HIP(hipMemcpyAsync(flag, &mine, sizeof mine, hipMemcpyHostToDevice, g_state.stream));
            SHMX_NCCL(ncclAllReduce(flag, flag, 1, ncclInt32, ncclMin, g_state.comm, g_state.stream));
            int all = 0;
            SHMX_HIP(hipMemcpyAsync(&all, flag, sizeof all, hipMemcpyDeviceToHost, g_state.stream));
            SHMX_HIP(hipStreamSynchronize(g_state.stream));
            SHMX_HIP(hipFree(flag));
            if (attached && !all) node::detach(false);
            attached = all != 0;
        }
        g_state.node_shared = attached;
        if (!attached) trace(LOG_INIT, "no intra-node block: the DIRECT algorithm is unavailable");
        // Every PE is attached after a first barrier (it also makes the IPC
        // transport's init collective, like ncclCommInitRank, so a bootstrap
        // file is removed only once every PE has read it); the name can go
        // then, so a job that dies leaves nothing in /dev/shm.
        if (attached) {
            node::put_gpu_numa(gpu_numa_node(device));   // (staging.cpp's copy threads)
            {
                char bus[64] = {0};
                uint64_t id = 0;
                if (hipDeviceGetPCIBusId(bus, sizeof bus, device) == hipSuccess) {
                    id = 1469598103934665603ull;   // FNV-1a, never 0 for a real id
                    for (const char *c = bus; *c; ++c) id = (id ^ (unsigned char)*c) * 1099511628211ull;
                } else {
                    (void)hipGetLastError();
                }
                node::put_gpu_id(id);
            }
            const bool xchg = npes > 1 && node::xchg_attach();   // (opened before the names go)
            node::barrier(0, 1, npes);
            if (pe == 0) node::unlink_name();
            g_state.xchg = npes > 1 && node::agree(0, 1, npes, xchg);
            g_state.gpu_shared = node::gpu_shared();
        }
    }
    g_state.pe = pe;
    g_state.npes = npes;
    g_state.device = device;
    g_state.algo = parse_algo(std::getenv("SHMEM_REDUCE_ALGO"));
    g_state.inited = true;
    if (npes > 1) check_plan_settings();
    trace(LOG_INIT, "PE %d of %d on HIP device %d%s%s", pe, npes, device,
          g_state.comm ? ", RCCL communicator up" : "", node::up() ? ", node block up" : "");
    return SHMEMX_OK;
}

// Exchange the RCCL id through a file: PE 0 writes it (atomically, via
// rename), the others wait for a file no older than this process (minus a
// margin), so a stale id from an earlier job is never used.
static int file_bootstrap(int pe, int npes, int device) {
    std::string path;
    if (const char *p = std::getenv("SHMEM_BOOTSTRAP_FILE")) path = p;
    else {
        const char *port = std::getenv("MASTER_PORT");
        path = std::string("/tmp/shmem_mi355x_uid.") + (port ? port : "0");
    }
    ncclUniqueId id;
    const time_t started = time(nullptr);
    if (pe == 0) {
        if (!make_uid(&id)) fatal("shmem_init", "cannot make a job id");
        const std::string tmp = path + ".tmp." + std::to_string(getpid());
        FILE *f = fopen(tmp.c_str(), "wb");
        if (!f || fwrite(&id, sizeof id, 1, f) != 1) fatal("shmem_init", "cannot write bootstrap file");
        fclose(f);
        if (rename(tmp.c_str(), path.c_str()) != 0) fatal("shmem_init", "cannot publish bootstrap file");
    } else {
        for (int waited_ms = 0;; waited_ms += 20) {
            struct stat st;
            if (stat(path.c_str(), &st) == 0 && st.st_size == (off_t)sizeof id &&
                st.st_mtime + 30 >= started) {
                FILE *f = fopen(path.c_str(), "rb");
                if (f) {
                    const bool ok = fread(&id, sizeof id, 1, f) == 1;
                    fclose(f);
                    if (ok) break;
                }
            }
            if (waited_ms > 300000) fatal("shmem_init", "timed out waiting for the bootstrap file");
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
        }
    }
    const int rc = init_locked(pe, npes, device, &id);
    if (pe == 0) unlink(path.c_str());  // every PE has read it: the init is collective
    return rc;
}

void bind_device() {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != g_state.device) SHMX_HIP(hipSetDevice(g_state.device));
}

int ensure_init() {
    if (g_state.inited) {
        bind_device();
        return SHMEMX_OK;
    }
    const int npes = env_int("SHMEM_NPES", "WORLD_SIZE", 1);
    if (npes != 1) return set_error(SHMEMX_ENOINIT);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return init_locked(0, 1, dev, nullptr);
}

// ----------------------------------------------------------------- plans

bool is_member(int pe, int start, int logstride, int size, int *index) {
    const int step = 1 << logstride;
    if (pe < start || (pe - start) % step) return false;
    const int i = (pe - start) / step;
    if (i >= size) return false;
    if (index) *index = i;
    return true;
}

static bool rccl_dtype(int type, ncclDataType_t *dt) {
    switch (type) {
    case SHMEMX_TYPE_INT: *dt = ncclInt32; return true;
    case SHMEMX_TYPE_LONG:
    case SHMEMX_TYPE_LONGLONG: *dt = ncclInt64; return true;
    case SHMEMX_TYPE_FLOAT: *dt = ncclFloat32; return true;
    case SHMEMX_TYPE_DOUBLE: *dt = ncclFloat64; return true;
    default: return false;
    }
}

// Pairs RCCL reduces exactly as reduce-op.c specifies: every integer op it
// has (wrapping sum/prod, min, max), and float/double sum/prod (rounding
// order differs from the reference's linear fold: ULP tolerance).
// Float min/max are excluded: a<b?a:b is not RCCL's NaN/-0 behaviour.
static bool rccl_native(int type, int op) {
    ncclDataType_t dt;
    if (!rccl_dtype(type, &dt)) return false;
    const bool fp = type == SHMEMX_TYPE_FLOAT || type == SHMEMX_TYPE_DOUBLE;
    switch (op) {
    case SHMEMX_OP_SUM:
    case SHMEMX_OP_PROD: return true;
    case SHMEMX_OP_MIN:
    case SHMEMX_OP_MAX: return !fp;
    default: return false;
    }
}

// The six pairs whose reference answer depends on the calling PE beyond
// rounding: min and max of float, double and long double.  a<b?a:b
// (reduce-op.c:130-142) returns its second operand when either one is a NaN
// or both are zeros (+0 and -0 compare equal), and PE k folds src_k first,
// then the other members ascending (:219-248); so wherever an element's
// inputs hold a NaN or both signed zeros, PE k's answer can differ from
// PE_start's by a whole value (2 PEs, sources 1.0 and NaN: PE 0 gets
// min(1.0, NaN) = NaN, PE 1 gets min(NaN, 1.0) = 1.0).  No schedule that
// hands every member one shared result can give that, so for these pairs
// every algorithm folds in the calling PE's own order: every member reads
// every member's whole source ((P-1)·S per PE, against 2(P-1)/P·S for a
// shared result).
bool own_order_pair(int type, int op) {
    return (op == SHMEMX_OP_MIN || op == SHMEMX_OP_MAX) &&
           (type == SHMEMX_TYPE_FLOAT || type == SHMEMX_TYPE_DOUBLE || type == SHMEMX_TYPE_LONGDOUBLE);
}

static ncclRedOp_t rccl_op(int op) {
    switch (op) {
    case SHMEMX_OP_SUM: return ncclSum;
    case SHMEMX_OP_PROD: return ncclProd;
    case SHMEMX_OP_MIN: return ncclMin;
    default: return ncclMax;
    }
}

// Up to this many bytes, AUTO takes one RCCL all-reduce for the RCCL-native
// pairs on the full set ($SHMEMX_ALLREDUCE_MAX_KB, default 4 MiB); above it,
// the reduce-scatter + all-gather form.
static long long allreduce_max_bytes() {
    static const long long b = (long long)env_int("SHMEMX_ALLREDUCE_MAX_KB", nullptr, 4096) << 10;
    return b;
}

// AUTO's per-size table, from the driver's multi-GPU bench
// (extras.auto_recommendation.env): $SHMEMX_AUTO_FULL for the whole job,
// $SHMEMX_AUTO_PARTIAL for partial and strided sets, each a list of
// "bytes:algo" cut points in ascending order ("0:allreduce,3145728:rccl":
// arrays of fewer than 3 MiB per PE take one all-reduce, larger ones
// reduce-scatter + all-gather).  Names: allreduce, rccl, a2a, direct, gather.
// A cut whose algorithm cannot serve a call (an RCCL algorithm for a pair
// RCCL does not reduce as the reference does, DIRECT without the node block)
// falls back to the built-in rule, so every PE still plans alike.  Unset or
// unparsable: the built-in rule alone (the bad value is reported once).
struct AutoCut {
    long long bytes;
    int algo;
};

static std::vector<AutoCut> parse_auto_table(const char *var) {
    std::vector<AutoCut> cuts;
    const char *e = std::getenv(var);
    if (!e || !*e) return cuts;
    std::string s(e);
    size_t pos = 0;
    long long last = -1;
    while (pos <= s.size()) {
        const size_t end = std::min(s.find(',', pos), s.size());
        const std::string item = s.substr(pos, end - pos);
        const size_t colon = item.find(':');
        char *stop = nullptr;
        const long long b = colon == std::string::npos ? -1 : std::strtoll(item.c_str(), &stop, 10);
        const std::string name = colon == std::string::npos ? "" : item.substr(colon + 1);
        const int a = parse_algo(name.c_str());
        const bool named = name == "allreduce" || name == "rccl" || name == "a2a" || name == "direct" ||
                           name == "gather";
        if (b < 0 || stop != item.c_str() + colon || !named || b <= last) {
            trace(LOG_INFO, "%s=\"%s\": unusable cut \"%s\"; the built-in rule applies", var, e,
                  item.c_str());
            return {};
        }
        cuts.push_back({b, a});
        last = b;
        pos = end + 1;
    }
    return cuts;
}

// Set while reduce_device plans a call being captured into a hipGraph:
// the table's DIRECT (host barriers, refused under capture) then falls back
// to the built-in rule, so captured calls still plan.  Every PE of a set
// must capture its calls alike (as for every stream-ordered collective).
static thread_local bool t_planning_capture = false;
// Set while reduce_device plans a call on a partial set that is being
// captured: a set whose RCCL communicator does not exist yet cannot take an
// RCCL algorithm (creating one is not a stream operation).
static thread_local bool t_capturing = false;

// The table's algorithm for an array of `bytes` per PE, or AUTO.
static int auto_table_algo(bool world, long long bytes) {
    static const std::vector<AutoCut> full = parse_auto_table("SHMEMX_AUTO_FULL");
    static const std::vector<AutoCut> partial = parse_auto_table("SHMEMX_AUTO_PARTIAL");
    const std::vector<AutoCut> &t = world ? full : partial;
    int algo = SHMEMX_ALGO_AUTO;
    for (const AutoCut &c : t)
        if (bytes >= c.bytes) algo = c.algo;
    return algo;
}

int make_plan(int type, int op, int nreduce, int start, int logstride,
                     int size, int pe, int npes, int algo, shmemx_plan_t *p) {
    std::memset(p, 0, sizeof *p);
    p->member = -1;
    if (!op_valid(type, op)) return SHMEMX_EINVAL;
    if (nreduce < 0 || start < 0 || logstride < 0 || logstride > 30 || size < 1 ||
        npes < 1 || algo < 0 || algo >= SHMEMX_NALGOS)
        return SHMEMX_EINVAL;
    if ((long long)start + (long long)(size - 1) * (1LL << logstride) >= npes)
        return SHMEMX_EINVAL;
    int m = -1;
    if (!is_member(pe, start, logstride, size, &m)) return SHMEMX_ENOTMEMBER;
    if (!op_on_device(type, op)) return SHMEMX_ENOTSUP;
    const long long n = nreduce;
    const int P = size;
    const int sz = (int)type_size(type);
    const long long g = sz >= 16 ? 1 : 16 / sz;  // elements per 16-byte granule
    const bool world = start == 0 && (logstride == 0 || size == 1) && size == npes;
    // RCCL's own collectives serve the whole job on the world communicator
    // and a partial set on the set's members-only communicator (set_comm.cpp)
    const bool set_rccl = world || (set_comms_enabled() && !set_comm_refused(start, logstride, size) &&
                                    (!t_capturing || set_comm_cached(start, logstride, size)));
    const bool rccl_ok = set_rccl && rccl_native(type, op) && !g_state.ipc_only;
    // each member's own fold order (own_order_pair): GATHER's exchange, or
    // DIRECT / SIGNAL reading every member's whole source
    const bool own = P > 1 && own_order_pair(type, op);
    if (algo == SHMEMX_ALGO_AUTO && P > 1) {
        const int t = auto_table_algo(world, n * sz);
        const bool pull_ok = g_state.node_shared && P <= kMaxFoldInputs && !t_planning_capture;
        if (((t == SHMEMX_ALGO_RCCL || t == SHMEMX_ALGO_ALLREDUCE) && rccl_ok) ||
            (t == SHMEMX_ALGO_A2A && !g_state.ipc_only && !own) || (t == SHMEMX_ALGO_DIRECT && pull_ok) ||
            t == SHMEMX_ALGO_GATHER)
            algo = t;
    }
    if (algo == SHMEMX_ALGO_AUTO && own) algo = SHMEMX_ALGO_GATHER;
    // A2A's owner hands one result to every member: for these pairs its
    // exchange is GATHER's
    if (algo == SHMEMX_ALGO_A2A && own) algo = SHMEMX_ALGO_GATHER;
    if (algo == SHMEMX_ALGO_AUTO) {
        if (g_state.ipc_only) algo = SHMEMX_ALGO_DIRECT;
        // A partial set keeps A2A under the built-in rule: the reference's
        // PE_start bits for float sums too, and no blocking communicator
        // set-up at a set's first call.  Its members-only RCCL communicator
        // (set_comm.cpp, so far run against the RCCL test double only) is
        // taken when asked for: an explicit rccl / allreduce, or
        // $SHMEMX_AUTO_PARTIAL naming one.
        else if (!rccl_ok || !world) algo = SHMEMX_ALGO_A2A;
        // Small arrays are latency-bound: one RCCL all-reduce (one launch,
        // and RCCL's own small-message all-reduce algorithms) instead of
        // reduce-scatter + all-gather (+ a tail all-reduce).
        else algo = n * sz <= allreduce_max_bytes() ? SHMEMX_ALGO_ALLREDUCE : SHMEMX_ALGO_RCCL;
    }
    if ((algo == SHMEMX_ALGO_RCCL || algo == SHMEMX_ALGO_ALLREDUCE) && !(set_rccl && rccl_native(type, op)))
        return SHMEMX_ENOTSUP;
    if (g_state.ipc_only && algo != SHMEMX_ALGO_DIRECT && algo != SHMEMX_ALGO_GATHER &&
        algo != SHMEMX_ALGO_SIGNAL)
        return SHMEMX_ENOTSUP;   // no RCCL communicator on the IPC transport
    if ((algo == SHMEMX_ALGO_DIRECT || algo == SHMEMX_ALGO_SIGNAL) && size > kMaxFoldInputs)
        return SHMEMX_ENOTSUP;
    p->algo = algo;
    p->member = m;
    p->nmembers = P;
    p->elem_size = sz;
    if (P == 1 && !g_state.force_collective) {
        p->chunk = n;
        return SHMEMX_OK;
    }
    switch (algo) {
    case SHMEMX_ALGO_RCCL:
        p->chunk = (n / (P * g)) * g;
        p->main = p->chunk * P;
        p->tail = n - p->main;
        break;
    case SHMEMX_ALGO_ALLREDUCE:
        p->chunk = n;
        p->main = n;
        break;
    case SHMEMX_ALGO_A2A: {
        long long c = (n + P - 1) / P;
        c = (c + g - 1) / g * g;
        p->chunk = c;
        p->ws_bytes = c * P * sz;
        break;
    }
    case SHMEMX_ALGO_DIRECT:
    case SHMEMX_ALGO_SIGNAL: {   // slice per member (own order: all of it); no workspace
        const long long c = (n + P - 1) / P;
        p->chunk = own ? n : (c + g - 1) / g * g;
        break;
    }
    default:  // GATHER (IPC transport: read in place, no workspace)
        p->chunk = n;
        p->ws_bytes = g_state.ipc_only ? 0 : n * P * sz;
        break;
    }
    return SHMEMX_OK;
}

// ------------------------------------------------------------- workspaces

void *grow(void *&buf, size_t &have, size_t need) {
    if (need <= have) return buf;
    if (buf) {
        // the old buffer may still be in use on any caller stream
        device_sync();
        SHMX_HIP(hipFree(buf));
        buf = nullptr;
        have = 0;
    }
    if (hipMalloc(&buf, need) != hipSuccess) {
        (void)hipGetLastError();
        buf = nullptr;
        return nullptr;
    }
    have = need;
    return buf;
}

// The device workspaces (ws, tmp) are shared by every stream-ordered call:
// a use on stream s waits for the previous use when that was on another
// stream.  Skipped while s is being captured into a graph (a captured graph
// lives on one stream; events recorded in a capture do not fire until replay).
bool stream_capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

void ws_acquire(hipStream_t s) {
    if (g_state.ws_stream && g_state.ws_stream != s && !stream_capturing(s))
        SHMX_HIP(hipStreamWaitEvent(s, g_state.ws_event, 0));
}

void ws_release(hipStream_t s) {
    if (stream_capturing(s)) return;
    if (!g_state.ws_event) SHMX_HIP(hipEventCreateWithFlags(&g_state.ws_event, hipEventDisableTiming));
    SHMX_HIP(hipEventRecord(g_state.ws_event, s));
    g_state.ws_stream = s;
}

bool overlap(const void *a, const void *b, size_t bytes) {
    const char *x = static_cast<const char *>(a), *y = static_cast<const char *>(b);
    return x != y && x < y + bytes && y < x + bytes;
}

// The reference's own trace messages (reduce-op.c:199-210), from the caller's
// target and source, before any staging.  Like OVERLAP_CHECK (:166-167) an
// in-place call counts as overlapping; unlike it, the range is the array's
// bytes, not its byte count taken as an element count (which only widens the
// check).
void trace_reference_overlap(const void *target, const void *source, size_t bytes) {
    if (!log_enabled(LOG_REDUCTION)) return;
    const char *t = static_cast<const char *>(target), *s = static_cast<const char *>(source);
    const bool ov = t < s + bytes && s < t + bytes;
    trace(LOG_REDUCTION, ov ? "target (%p) and source (%p, size %ld) overlap, using temporary target"
                            : "target (%p) and source (%p, size %ld) do not overlap",
          target, source, (long)bytes);
}

static long long count_of(long long n, long long chunk, int i) {
    const long long lo = chunk * i;
    return std::max(0LL, std::min(chunk, n - lo));
}

void fold_chain(int type, int op, void *out, const void **ins, int nins, size_t n,
                hipStream_t s, bool peers) {
    // Left fold in groups of kMaxFoldInputs: out = fold(ins[0..15]);
    // out = fold(out, ins[16..30]); ... (same order as one long fold).
    auto fold = peers ? launch_fold_peers : launch_fold;
    int done = std::min(nins, kMaxFoldInputs);
    SHMX_HIP(fold(type, op, out, ins, done, n, s));
    while (done < nins) {
        const void *grp[kMaxFoldInputs];
        grp[0] = out;
        int k = 1;
        while (k < kMaxFoldInputs && done < nins) grp[k++] = ins[done++];
        SHMX_HIP(fold(type, op, out, grp, k, n, s));
    }
}

static int reduce_exchange(int type, int op, char *tgt, const char *src, int nreduce,
                           int start, int logstride, const shmemx_plan_t &p, hipStream_t s,
                           bool &uses_ws);

// The engine: device-resident target/source, stream-ordered.
int reduce_device(int type, int op, void *target, const void *source,
                         int nreduce, int start, int logstride, int size,
                         int algo, hipStream_t s) {
    shmemx_plan_t p;
    const bool partial = !(start == 0 && (logstride == 0 || size == 1) && size == g_state.npes);
    const bool capturing = (algo == SHMEMX_ALGO_AUTO || partial) && stream_capturing(s);
    t_planning_capture = algo == SHMEMX_ALGO_AUTO && capturing;
    t_capturing = capturing;
    int rc = make_plan(type, op, nreduce, start, logstride, size, g_state.pe,
                       g_state.npes, algo, &p);
    // a partial set's first RCCL call: its members agree on and make its
    // communicator; if they refuse (a member's cache is full), all of them
    // plan again without it (A2A under auto, ENOTSUP for an explicit rccl)
    if (!rc && partial && size > 1 && (p.algo == SHMEMX_ALGO_RCCL || p.algo == SHMEMX_ALGO_ALLREDUCE) &&
        !set_comm_cached(start, logstride, size) && !set_comm_prepare(start, logstride, size, p.member, s))
        rc = make_plan(type, op, nreduce, start, logstride, size, g_state.pe, g_state.npes, algo, &p);
    t_planning_capture = false;
    t_capturing = false;
    if (rc) return set_error(rc);
    if (nreduce == 0) return SHMEMX_OK;
    const bool collective = size > 1 || g_state.force_collective;
    const bool own = size > 1 && own_order_pair(type, op);
    if (collective && p.algo == SHMEMX_ALGO_SIGNAL) {
        if (log_enabled(LOG_REDUCTION))
            trace(LOG_REDUCTION, "type %d op %d nreduce %d set (%d,%d,%d) member %d algo signal%s",
                  type, op, nreduce, start, logstride, size, p.member, own ? " (own order)" : "");
        return signal_reduce(type, op, static_cast<char *>(target), static_cast<const char *>(source),
                             nreduce, start, logstride, p, own, s);
    }
    const bool over_ipc = p.algo == SHMEMX_ALGO_DIRECT ||
                          (p.algo == SHMEMX_ALGO_GATHER && g_state.ipc_only);
    if (collective && over_ipc) {
        const bool own_order = p.algo == SHMEMX_ALGO_GATHER || own;
        if (log_enabled(LOG_REDUCTION))
            trace(LOG_REDUCTION, "type %d op %d nreduce %d set (%d,%d,%d) member %d algo %s%s",
                  type, op, nreduce, start, logstride, size, p.member,
                  p.algo == SHMEMX_ALGO_DIRECT ? "direct" : "gather (ipc)", own_order ? " (own order)" : "");
        return direct_reduce(type, op, static_cast<char *>(target), static_cast<const char *>(source),
                             nreduce, start, logstride, p, own_order, s);
    }
    if (collective && !g_state.comm) return set_error(SHMEMX_ENOINIT);
    const size_t sz = (size_t)p.elem_size;
    const size_t bytes = sz * (size_t)nreduce;
    char *tgt = static_cast<char *>(target);
    const char *src = static_cast<const char *>(source);

    if (log_enabled(LOG_REDUCTION)) {
        static const char *const algos[SHMEMX_NALGOS] = {"auto", "rccl", "a2a", "gather",
                                                         "allreduce", "direct", "signal"};
        trace(LOG_REDUCTION, "type %d op %d nreduce %d set (%d,%d,%d) member %d algo %s chunk %lld",
              type, op, nreduce, start, logstride, size, p.member, algos[p.algo], p.chunk);
    }
    // Partially overlapping target/source: reduce from a private copy of the
    // source (the reference's temporary target, reduce-op.c:187-203).
    bool uses_ws = false;
    if (overlap(tgt, src, bytes)) {
        void *t = grow(g_state.tmp, g_state.tmp_bytes, bytes);
        if (!t) return set_error(SHMEMX_ENOMEM);
        ws_acquire(s);
        uses_ws = true;
        const void *in[1] = {src};
        fold_chain(type, op, t, in, 1, (size_t)nreduce, s);
        src = static_cast<const char *>(t);
    }
    const int xrc = reduce_exchange(type, op, tgt, src, nreduce, start, logstride, p, s, uses_ws);
    if (uses_ws) ws_release(s);
    return xrc;
}

// The exchange + fold of reduce_device once the source is safe to read.
static int reduce_exchange(int type, int op, char *tgt, const char *src, int nreduce,
                           int start, int logstride, const shmemx_plan_t &p, hipStream_t s,
                           bool &uses_ws) {
    const int size = p.nmembers;
    const size_t sz = (size_t)p.elem_size;
    const size_t bytes = sz * (size_t)nreduce;

    const int P = size, m = p.member, step = 1 << logstride;
    if (P == 1 && !g_state.force_collective) {  // reduce-op.c:213-216, no peers: a copy
        if (tgt != src) {
            const void *in[1] = {src};
            fold_chain(type, op, tgt, in, 1, (size_t)nreduce, s);
        }
        return SHMEMX_OK;
    }
    auto peer = [&](int i) { return start + i * step; };

    if (p.algo == SHMEMX_ALGO_ALLREDUCE || p.algo == SHMEMX_ALGO_RCCL) {
        // the whole job: the world communicator; a partial set: its own
        // members-only communicator, rank = index in the set
        const bool world = start == 0 && (step == 1 || P == 1) && P == g_state.npes;
        ncclComm_t comm = world ? g_state.comm : set_comm(start, logstride, P, m, s);
        ncclDataType_t dt;
        rccl_dtype(type, &dt);
        const ncclRedOp_t rop = rccl_op(op);
        if (p.algo == SHMEMX_ALGO_ALLREDUCE) {  // one RCCL all-reduce, in place allowed
            SHMX_NCCL(ncclAllReduce(src, tgt, (size_t)nreduce, dt, rop, comm, s));
            return SHMEMX_OK;
        }
        if (p.chunk > 0) {
            char *mine = tgt + (size_t)m * (size_t)p.chunk * sz;
            SHMX_NCCL(ncclReduceScatter(src, mine, (size_t)p.chunk, dt, rop, comm, s));
            SHMX_NCCL(ncclAllGather(mine, tgt, (size_t)p.chunk, dt, comm, s));
        }
        if (p.tail > 0) {
            const size_t off = (size_t)p.main * sz;
            SHMX_NCCL(ncclAllReduce(src + off, tgt + off, (size_t)p.tail, dt, rop, comm, s));
        }
        return SHMEMX_OK;
    }

    char *ws = static_cast<char *>(grow(g_state.ws, g_state.ws_bytes, (size_t)p.ws_bytes));
    if (!ws) return set_error(SHMEMX_ENOMEM);
    if (!uses_ws) ws_acquire(s);
    uses_ws = true;
    const long long n = nreduce;

    if (p.algo == SHMEMX_ALGO_A2A) {
        const size_t cb = (size_t)p.chunk * sz;
        const long long my_cnt = count_of(n, p.chunk, m);
        // 1. shard exchange: member i gets chunk i of every source
        SHMX_NCCL(ncclGroupStart());
        for (int i = 0; i < P; ++i) {
            if (i == m) continue;
            const long long ci = count_of(n, p.chunk, i);
            if (ci > 0) SHMX_NCCL(ncclSend(src + i * cb, (size_t)ci * sz, ncclUint8, peer(i), g_state.comm, s));
            if (my_cnt > 0) SHMX_NCCL(ncclRecv(ws + i * cb, (size_t)my_cnt * sz, ncclUint8, peer(i), g_state.comm, s));
        }
        SHMX_NCCL(ncclGroupEnd());
        // 2. fold the P copies of my chunk in active-set order (PE_start first)
        if (my_cnt > 0) {
            std::vector<const void *> ins(P);
            for (int i = 0; i < P; ++i) ins[i] = (i == m) ? src + m * cb : ws + i * cb;
            fold_chain(type, op, tgt + m * cb, ins.data(), P, (size_t)my_cnt, s);
        }
        // 3. shard all-gather: RCCL's own all-gather (in place) when the set
        // is the whole job and every shard is full, grouped p2p otherwise
        const bool world = start == 0 && step == 1 && P == g_state.npes;
        if (world && n == (long long)P * p.chunk) {
            SHMX_NCCL(ncclAllGather(tgt + m * cb, tgt, cb, ncclUint8, g_state.comm, s));
            return SHMEMX_OK;
        }
        SHMX_NCCL(ncclGroupStart());
        for (int i = 0; i < P; ++i) {
            if (i == m) continue;
            const long long ci = count_of(n, p.chunk, i);
            if (my_cnt > 0) SHMX_NCCL(ncclSend(tgt + m * cb, (size_t)my_cnt * sz, ncclUint8, peer(i), g_state.comm, s));
            if (ci > 0) SHMX_NCCL(ncclRecv(tgt + i * cb, (size_t)ci * sz, ncclUint8, peer(i), g_state.comm, s));
        }
        SHMX_NCCL(ncclGroupEnd());
        return SHMEMX_OK;
    }

    // GATHER: every source to every member (RCCL's all-gather on the whole
    // job, grouped p2p on a partial set), then the reference's own order on
    // each PE: r = src_me; r = op(r, src_p) for p ascending, p != me.
    if (start == 0 && step == 1 && P == g_state.npes) {
        SHMX_NCCL(ncclAllGather(src, ws, bytes, ncclUint8, g_state.comm, s));
    } else {
        SHMX_NCCL(ncclGroupStart());
        for (int i = 0; i < P; ++i) {
            if (i == m) continue;
            SHMX_NCCL(ncclSend(src, bytes, ncclUint8, peer(i), g_state.comm, s));
            SHMX_NCCL(ncclRecv(ws + (size_t)i * bytes, bytes, ncclUint8, peer(i), g_state.comm, s));
        }
        SHMX_NCCL(ncclGroupEnd());
    }
    {
        std::vector<const void *> ins;
        ins.reserve(P);
        ins.push_back(src);
        for (int i = 0; i < P; ++i)
            if (i != m) ins.push_back(ws + (size_t)i * bytes);
        fold_chain(type, op, tgt, ins.data(), P, (size_t)nreduce, s);
    }
    return SHMEMX_OK;
}

bool device_accessible(const void *ptr) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// Page-locked host memory (hipHostMalloc / hipHostRegister): DMA-able, so
// chunked copies overlap; pageable memory is copied through HIP's own
// staging, where chunking only adds overhead (measured).
bool host_pinned(const void *ptr) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

}  // namespace shmx

// ------------------------------------------------------------- internal API
// (used by entry.cpp; C++ linkage, not exported in the header)
namespace shmx {

// $SHMEMX_DEBUG=1: the checks the reference's wrappers make when configured
// with --enable-debug (reduce-op.c:379-381, utils.h:64-116): target and
// source must be symmetric (heap, or the program's globals), else FATAL.
void debug_checks(const char *name, const void *target, const void *source) {
    static const bool on = env_int("SHMEMX_DEBUG", nullptr, 0) != 0;
    if (!on) return;
    std::lock_guard<std::recursive_mutex> lk(g_mu);   // the heap's block table
    const void *args[2] = {target, source};
    for (int i = 0; i < 2; ++i) {
        if (heap::is_symmetric(args[i])) continue;
        trace(LOG_FATAL, "%s(), argument #%d @ %p is not symmetric", name, i + 1, args[i]);
        std::abort();
    }
}

int reduce_on_stream(int type, int op, void *target, const void *source,
                     int nreduce, int start, int logstride, int size, int algo,
                     void *stream) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    t_last_error = SHMEMX_OK;
    if (int rc = ensure_init()) return rc;
    if (nreduce > 0 && (!target || !source)) return set_error(SHMEMX_EINVAL);
    // Operands in the mirrored heap's host view: the host's stores go to HBM
    // now (host-synchronous), and the call runs on the HBM twins.
    const size_t bytes = op_valid(type, op) && nreduce > 0 ? type_size(type) * (size_t)nreduce : 0;
    const void *src = bytes ? heap::device_operand(source, bytes) : source;
    // the stream-ordered form takes device memory only (RCCL and the kernels
    // dereference it); host arrays go through the blocking entry points
    if (nreduce > 0 && (!device_accessible(heap::twin(target)) || !device_accessible(src)))
        return set_error(SHMEMX_EINVAL);
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g_state.stream;
    if (s == g_state.stream) g_state.lib_stream_dirty = true;   // (service.hip)
    if (nreduce >= 0 && op_valid(type, op))
        trace_reference_overlap(target, source, type_size(type) * (size_t)nreduce);
    // the host view of the target is stale from here: a host access to its
    // blocks waits until the call is enqueued, then for `s` (the writer), and
    // reads the result
    heap::DeviceWrite t(target, bytes, s);
    // a host-view target whose range runs past the heap: DeviceWrite opened
    // nothing and ptr() is still the view address, which no kernel may write
    // 
    uint64_t voff = 0;
    if (bytes && t.ptr() == target && heap::view_offset(target, &voff)) return set_error(SHMEMX_EINVAL);
    return reduce_device(type, op, t.ptr(), src, nreduce, start, logstride, size,
                         algo == SHMEMX_ALGO_AUTO ? g_state.algo : algo, s);
}

}  // namespace shmx

// ------------------------------------------------------------------ C ABI

using namespace shmx;

extern "C" {

void pshmem_init(void) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (g_state.inited) return;
    const int npes = env_int("SHMEM_NPES", "WORLD_SIZE", 1);
    const int pe = npes > 1 ? env_int("SHMEM_PE", "RANK", 0) : 0;
    const int dev = npes > 1 ? env_int("LOCAL_RANK", nullptr, -1) : -1;
    if (npes < 1 || pe < 0 || pe >= npes) {
        char why[128];
        snprintf(why, sizeof why, "bad PE identity from the environment: pe %d of %d", pe, npes);
        fatal("shmem_init", why);
    }
    const int rc = npes > 1 ? file_bootstrap(pe, npes, dev) : init_locked(0, 1, dev, nullptr);
    if (rc) fatal("shmem_init", shmemx_reduce_error_string(rc));
}

void pshmem_finalize(void) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (!g_state.inited) return;
    (void)hipStreamSynchronize(g_state.stream);
    service_release();
    // collective: no PE frees memory its peers may still be reading
    if (node::up()) node::barrier(0, 1, g_state.npes);
    if (g_state.comm && g_state.rccl_reg) (void)ncclCommDeregister(g_state.comm, g_state.rccl_reg);
    g_state.rccl_reg = nullptr;
    g_state.rccl_reg_refused = false;
    set_comms_release();
    heap::release_all();
    direct_release();
    node::detach(g_state.pe == 0);
    if (g_state.comm) {
        ncclCommDestroy(g_state.comm);
        g_state.comm = nullptr;
    }
    for (void **b : {&g_state.ws, &g_state.tmp, &g_state.stage_src, &g_state.stage_tgt,
                     &g_state.token, &g_state.cws_src, &g_state.cws_tgt}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    g_state.ws_bytes = g_state.tmp_bytes = g_state.stage_bytes = 0;
    g_state.token_bytes = g_state.cws_src_bytes = g_state.cws_tgt_bytes = 0;
    ring_free();
    if (g_state.bounce) (void)hipHostFree(g_state.bounce);
    g_state.bounce = nullptr;
    g_state.bounce_bytes = 0;
    for (hipEvent_t e : g_state.events) (void)hipEventDestroy(e);
    g_state.events.clear();
    for (hipStream_t *st : {&g_state.h2d, &g_state.d2h}) {
        if (*st) (void)hipStreamDestroy(*st);
        *st = nullptr;
    }
    (void)hipStreamDestroy(g_state.stream);
    g_state.stream = nullptr;
    g_state.node_shared = false;
    g_state.xchg = false;
    g_state.gpu_shared = false;
    g_state.inited = false;
}

int pshmem_my_pe(void) { return g_state.pe; }
int pshmem_n_pes(void) { return g_state.npes; }

void shmem_init(void) __attribute__((weak, alias("pshmem_init")));
void shmem_finalize(void) __attribute__((weak, alias("pshmem_finalize")));
int shmem_my_pe(void) __attribute__((weak, alias("pshmem_my_pe")));
int shmem_n_pes(void) __attribute__((weak, alias("pshmem_n_pes")));

int shmemx_uniqueid_size(void) { return (int)sizeof(ncclUniqueId); }

int shmemx_get_uniqueid(void *uid_out) {
    if (!uid_out) return set_error(SHMEMX_EINVAL);
    ncclUniqueId id;
    if (!make_uid(&id)) return set_error(SHMEMX_EDEVICE);
    std::memcpy(uid_out, &id, sizeof id);
    return SHMEMX_OK;
}

int shmemx_init_attr(int pe, int npes, int device, const void *uid) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    return init_locked(pe, npes, device, uid);
}

int shmemx_initialized(void) { return g_state.inited ? 1 : 0; }

void *shmemx_heap_ptr(const void *addr, int pe) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (!g_state.inited || pe < 0 || pe >= g_state.npes) return nullptr;
    uint64_t off = 0;
    // A host-view address of the mirrored heap: itself for this PE, NULL for
    // a peer (as the reference's shmem_ptr).  A store through a peer's HBM
    // address would change HBM behind that peer's view, which would go on
    // serving (and later flush over it) its stale copy.  Device-side puts take
    // the twin (shmemx_mirror_device_ptr), whose peers' addresses this
    // returns, and the receiving PE calls shmemx_mirror_invalidate after the
    // barrier.
    if (heap::view_offset(addr, &off)) return pe == g_state.pe ? const_cast<void *>(addr) : nullptr;
    if (!heap::offset_of(addr, 1, &off)) return nullptr;
    if (pe == g_state.pe) return const_cast<void *>(addr);
    char *b = node::peer_base(node::kHeap, pe);
    return b ? b + off : nullptr;
}

int shmemx_mirror_stats(unsigned long long *out, int nout, int reset) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (!out || nout < 0) return set_error(SHMEMX_EINVAL);
    const mirror::Stats st = mirror::stats(reset != 0);
    const unsigned long long all[7] = {st.write_faults, st.read_faults, st.blocks_flushed,
                                       st.blocks_fetched, st.blocks_device_newer, st.fault_waits,
                                       st.blocks_settled};
    const int k = nout < 7 ? nout : 7;
    for (int i = 0; i < k; ++i) out[i] = all[i];
    return k;
}

void *shmemx_mirror_device_ptr(const void *addr) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    uint64_t off = 0;
    if (!heap::view_offset(addr, &off)) return nullptr;
    return heap::device_operand(addr, 0);
}

int shmemx_mirror_sync(const void *addr, size_t bytes) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    uint64_t off = 0;
    if (!heap::view_offset(addr, &off)) return set_error(SHMEMX_EINVAL);
    (void)heap::device_operand(addr, bytes);
    return SHMEMX_OK;
}

int shmemx_mirror_invalidate(const void *addr, size_t bytes) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    uint64_t off = 0;
    if (!heap::view_offset(addr, &off)) return set_error(SHMEMX_EINVAL);
    (void)heap::device_operand(addr, bytes);   // host stores first: they are not lost
    heap::device_wrote(addr, bytes, nullptr);  // writers unknown: the next fetch waits for the device
    return SHMEMX_OK;
}

int shmemx_mirror_acquire(const void *addr, size_t bytes, int for_write) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (!heap::host_acquire(addr, bytes, for_write != 0)) return set_error(SHMEMX_EINVAL);
    return SHMEMX_OK;
}

int shmemx_direct_stats(double *out, int nout, int reset) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (!out || nout < 0) {
        set_error(SHMEMX_EINVAL);
        return 0;
    }
    return direct_stats(out, nout, reset != 0);
}

int shmemx_host_register(void *base, size_t bytes) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    if (!base || !bytes) return set_error(SHMEMX_EINVAL);
    if (int rc = ensure_init()) return set_error(rc);
    if (hipHostRegister(base, bytes, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();
        return set_error(SHMEMX_EDEVICE);
    }
    trace(LOG_MEMORY, "host range %p (%zu bytes) page-locked", base, bytes);
    return SHMEMX_OK;
}

int shmemx_host_unregister(void *base) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    clear_error();
    if (!base) return set_error(SHMEMX_EINVAL);
    if (hipHostUnregister(base) != hipSuccess) {
        (void)hipGetLastError();
        return set_error(SHMEMX_EINVAL);
    }
    return SHMEMX_OK;
}

void *shmemx_get_stream(void) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (ensure_init()) return nullptr;
    g_state.lib_stream_exported = true;   // the caller may put anything on it (service.hip)
    return g_state.stream;
}

int shmemx_set_algo(int algo) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    const int prev = g_state.algo;
    if (algo >= 0 && algo < SHMEMX_NALGOS) g_state.algo = algo;
    return prev;
}

int shmemx_reduce_on_stream(int type, int op, void *target, const void *source,
                            int nreduce, int PE_start, int logPE_stride,
                            int PE_size, int algo, void *stream) {
    return reduce_on_stream(type, op, target, source, nreduce, PE_start,
                            logPE_stride, PE_size, algo, stream);
}

// The local folds need no shmem_init (they run on the caller's stream) and
// leave the calling thread's current device as they found it: a
// caller's stream carries its own device; after shmem_init a NULL stream
// means the PE's device, made current for the launch and then restored.
class LocalDevice {
  public:
    explicit LocalDevice(void *stream) {
        if (stream || !g_state.inited) return;
        if (hipGetDevice(&prev_) != hipSuccess || prev_ == g_state.device) {
            prev_ = -1;
            return;
        }
        SHMX_HIP(hipSetDevice(g_state.device));
    }
    ~LocalDevice() {
        if (prev_ >= 0) (void)hipSetDevice(prev_);
    }

  private:
    int prev_ = -1;
};

int shmemx_fold_on_stream(int type, int op, void *acc, const void *in,
                          size_t nelems, void *stream) {
    t_last_error = SHMEMX_OK;
    const LocalDevice dev(stream);
    if (!op_on_device(type, op)) return set_error(op_valid(type, op) ? SHMEMX_ENOTSUP : SHMEMX_EINVAL);
    if (nelems == 0) return SHMEMX_OK;
    if (!acc || !in) return set_error(SHMEMX_EINVAL);
    const void *ins[2] = {acc, in};
    if (launch_fold(type, op, acc, ins, 2, nelems, static_cast<hipStream_t>(stream)) != hipSuccess)
        return set_error(SHMEMX_EDEVICE);
    return SHMEMX_OK;
}

static int fold_n(int type, int op, void *out, const void *const *ins, int nins, size_t nelems,
                  void *stream, bool peers) {
    auto launch = peers ? launch_fold_peers : launch_fold;
    t_last_error = SHMEMX_OK;
    const LocalDevice dev(stream);
    if (!op_on_device(type, op)) return set_error(op_valid(type, op) ? SHMEMX_ENOTSUP : SHMEMX_EINVAL);
    if (nins < 1 || !ins) return set_error(SHMEMX_EINVAL);
    if (nelems == 0) return SHMEMX_OK;
    if (!out) return set_error(SHMEMX_EINVAL);
    for (int k = 0; k < nins; ++k)
        if (!ins[k]) return set_error(SHMEMX_EINVAL);
    int done = std::min(nins, kMaxFoldInputs);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (launch(type, op, out, ins, done, nelems, s) != hipSuccess) return set_error(SHMEMX_EDEVICE);
    while (done < nins) {
        const void *grp[kMaxFoldInputs];
        grp[0] = out;
        int k = 1;
        while (k < kMaxFoldInputs && done < nins) grp[k++] = ins[done++];
        if (launch(type, op, out, grp, k, nelems, s) != hipSuccess) return set_error(SHMEMX_EDEVICE);
    }
    return SHMEMX_OK;
}

int shmemx_fold_n_on_stream(int type, int op, void *out, const void *const *ins,
                            int nins, size_t nelems, void *stream) {
    return fold_n(type, op, out, ins, nins, nelems, stream, false);
}

int shmemx_fold_n_peers_on_stream(int type, int op, void *out, const void *const *ins,
                                  int nins, size_t nelems, void *stream) {
    return fold_n(type, op, out, ins, nins, nelems, stream, true);
}

int shmemx_gather_on_stream(const void *const *srcs, void *const *dsts, const size_t *bytes,
                            int nseg, void *stream) {
    t_last_error = SHMEMX_OK;
    const LocalDevice dev(stream);
    if (nseg < 0 || nseg > kMaxFoldInputs || (nseg > 0 && (!srcs || !dsts || !bytes)))
        return set_error(SHMEMX_EINVAL);
    for (int i = 0; i < nseg; ++i)
        if (bytes[i] && overlap(srcs[i], dsts[i], bytes[i])) return set_error(SHMEMX_EINVAL);
    if (launch_gather(srcs, dsts, bytes, nseg, static_cast<hipStream_t>(stream)) != hipSuccess)
        return set_error(SHMEMX_EINVAL);
    return SHMEMX_OK;
}

int shmemx_reduce_plan(int type, int op, int nreduce, int PE_start,
                       int logPE_stride, int PE_size, int pe, int npes,
                       int algo, shmemx_plan_t *plan) {
    if (!plan) return SHMEMX_EINVAL;
    // make_plan reads this process's set-communicator cache (set_comm.cpp),
    // which another thread's first RCCL call on a set may be filling: under
    // the library lock, as every entry point
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    return make_plan(type, op, nreduce, PE_start, logPE_stride, PE_size, pe, npes, algo, plan);
}

long shmemx_set_fused_twoshot_kb(long kb) {
    if (kb < 0) {
        set_error(SHMEMX_EINVAL);
        return -1;
    }
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    return set_fused_twoshot_kb(kb);
}

int shmemx_rccl_register_heap(int on) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    if (int rc = ensure_init()) return rc;
    if (!g_state.comm) return set_error(SHMEMX_ENOTSUP);
    if (on && !g_state.rccl_reg) {
        // once per segment: a refusal is remembered (the next shmem_malloc
        // does not try again), and the PEs agree, so all register or none
        if (g_state.rccl_reg_refused) return set_error(SHMEMX_ENOTSUP);
        void *base = nullptr;
        size_t bytes = 0;
        const bool have = heap::segment(&base, &bytes);
        SHMX_HIP(hipStreamSynchronize(g_state.stream));
        if (have && ncclCommRegister(g_state.comm, base, bytes, &g_state.rccl_reg) != ncclSuccess) {
            g_state.rccl_reg = nullptr;
            trace(LOG_INFO, "ncclCommRegister of the heap segment (%zu bytes) failed", bytes);
        }
        bool all = g_state.rccl_reg != nullptr;
        if (g_state.npes > 1) {
            int *flag = static_cast<int *>(grow(g_state.token, g_state.token_bytes, 64));
            if (!flag) fatal("shmemx_rccl_register_heap", "no device memory for the agreement");
            const int mine = all ? 1 : 0;
            int every = 0;
            SHMX_HIP(hipMemcpyAsync(flag, &mine, sizeof mine, hipMemcpyHostToDevice, g_state.stream));
            SHMX_NCCL(ncclAllReduce(flag, flag, 1, ncclInt32, ncclMin, g_state.comm, g_state.stream));
            SHMX_HIP(hipMemcpyAsync(&every, flag, sizeof every, hipMemcpyDeviceToHost, g_state.stream));
            SHMX_HIP(hipStreamSynchronize(g_state.stream));
            all = every != 0;
        }
        if (!all) {
            if (g_state.rccl_reg) (void)ncclCommDeregister(g_state.comm, g_state.rccl_reg);
            g_state.rccl_reg = nullptr;
            g_state.rccl_reg_refused = true;
            trace(LOG_INFO, "heap segment not registered with RCCL (refused on some PE)");
            return set_error(SHMEMX_ENOTSUP);
        }
        trace(LOG_INFO, "heap segment %p (%zu bytes) registered with the RCCL communicator", base, bytes);
    } else if (!on && g_state.rccl_reg) {
        SHMX_HIP(hipStreamSynchronize(g_state.stream));
        (void)ncclCommDeregister(g_state.comm, g_state.rccl_reg);
        g_state.rccl_reg = nullptr;
    }
    return SHMEMX_OK;
}

int shmemx_set_comms(void) {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    return set_comms_cached();
}

int shmemx_kernel_timing(int on) { return kernel_timing(on); }

int shmemx_kernel_times(double *us, int *kind, int max, unsigned long long *dropped) {
    if (!us || max < 0) return set_error(SHMEMX_EINVAL);
    const int n = kernel_times(us, kind, max, dropped);
    if (n < 0) fatal("shmemx_kernel_times", "a timed kernel failed");
    return n;
}

size_t shmemx_type_size(int type) { return type_size(type); }
int shmemx_op_valid(int type, int op) { return op_valid(type, op) ? 1 : 0; }
int shmemx_op_on_device(int type, int op) { return op_on_device(type, op) ? 1 : 0; }
int shmemx_reduce_last_error(void) { return t_last_error; }

const char *shmemx_reduce_error_string(int err) {
    switch (err) {
    case SHMEMX_OK: return "success";
    case SHMEMX_EINVAL: return "invalid argument";
    case SHMEMX_ENOTMEMBER: return "calling PE is not in the active set";
    case SHMEMX_ENOTSUP: return "type/op/algorithm not supported";
    case SHMEMX_ENOINIT: return "runtime not initialised (npes > 1 needs shmem_init)";
    case SHMEMX_ENOMEM: return "device workspace allocation failed";
    case SHMEMX_EDEVICE: return "HIP or RCCL error";
    default: return "unknown error";
    }
}

}  // extern "C"
