"""One PE of test_gpu_ipc.py: P of these processes share the box's one GPU on
the IPC transport ($SHMEMX_TRANSPORT=ipc: no RCCL, the node block's host
barrier, symmetric heap segments mapped into each other over IPC), so the
multi-PE reduction path runs for real across processes — every member's
kernel reads the other members' HBM.

    SHMEM_PE=p SHMEM_NPES=P SHMEM_BOOTSTRAP_FILE=f python gpu_ipc_child.py OUT.json SCENARIO

Checks every result against the oracle restatement of reduce-op.c on the
same seeded inputs (all PEs' sources are reproducible from the seeds), and
writes {"pe", "fails", "ncases"} to OUT.json.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402
import shmem_mi355x as shm  # noqa: E402
from gpu_util import order_bound, same_bits, to_dev  # noqa: E402

out_path, scenario = sys.argv[1], sys.argv[2]
# a PE that stops making progress leaves its Python stack in its log every
# 90 s (the library's own barriers abort after $SHMEMX_BARRIER_TIMEOUT)
import faulthandler  # noqa: E402
faulthandler.dump_traceback_later(90, repeat=True)
pe, npes = int(os.environ["SHMEM_PE"]), int(os.environ["SHMEM_NPES"])
if os.environ.get("FAKE_RCCL"):
    # the RCCL test double (tests/native/fake_rccl.cpp), global before the
    # library loads, so its nccl* calls bind there and PEs may share the GPU
    import ctypes
    ctypes.CDLL(os.environ["FAKE_RCCL"], mode=ctypes.RTLD_GLOBAL)
torch.cuda.set_device(0)
shm.init()
assert shm.my_pe() == pe and shm.n_pes() == npes
fails = []
ncases = 0
extra = {}    # scenario-specific report fields


def member(start, log, size):
    step = 1 << log
    return pe >= start and (pe - start) % step == 0 and (pe - start) // step < size


def active_sets():
    s = [(0, 0, npes), (npes - 1, 0, 1)]
    if npes >= 3:
        s += [(1, 0, npes - 1), (0, 1, (npes + 1) // 2)]
    if npes >= 4:
        s += [(1, 1, npes // 2)]
    if npes >= 8:
        s += [(0, 2, npes // 4), (2, 0, npes - 3)]   # stride 4; an offset run
    return s


# min / max of float, double, long double: a<b?a:b under NaN and +-0 makes
# each PE's reference answer depend on its own fold order (reduce-op.c:130-142,
# 219-248), and every algorithm gives each PE that answer (runtime.cpp
# own_order_pair)
OWN_ORDER = {(t, o) for t in ("float", "double", "longdouble") for o in ("min", "max")}


def elements_differing(t, a, b):
    """How many elements of a and b differ in their value bytes (long double:
    the 10 bytes of the x87 value)."""
    if not len(a):
        return 0
    w = 10 if t == "longdouble" else a.itemsize
    return int((a.view(np.uint8).reshape(len(a), -1)[:, :w] != b.view(np.uint8).reshape(len(b), -1)[:, :w])
               .any(axis=1).sum())


def expected(t, op, srcs, st, algo):
    start, log, size = st
    ref = oracle.reduce_sim(t, op, srcs, start, log, size)
    # DIRECT / SIGNAL / A2A: PE_start's fold order on every member; GATHER, and
    # every algorithm on the OWN_ORDER pairs: each PE's own.  RCCL / ALLREDUCE:
    # RCCL's order (the test double's ring and rotated orders), held against
    # PE_start's fold within the stated bound.
    if size > 1 and (t, op) in OWN_ORDER:
        extra["own_order_differs"] = extra.get("own_order_differs", 0) + elements_differing(t, ref[pe], ref[start])
        return ref[pe]
    return ref[start] if algo != "gather" else ref[pe]


# $RCCL_TOL_SCALE: the bound's multiplier for RCCL-ordered float sums and
# products (0 = the negative control: only bit-identical results pass)
TOL_SCALE = float(os.environ.get("RCCL_TOL_SCALE", "1"))
extra["rccl_inexact_elements"] = 0


def resolved(t, op, n, st, algo):
    """The algorithm a call on set st runs (auto resolved by the library's
    own planner, as every member plans alike)."""
    if algo != "auto":
        return algo
    try:
        return shm.plan(t, op, n, *st, pe, npes, "auto").algo
    except shm.ShmemError:
        return algo


def matches(got, want, t, op, srcs, st, algo):
    """got against the reference's result `want`: bit for bit, except the
    RCCL-ordered (rccl / allreduce) float sums and products, which must lie
    within the stated ULP bound of it (gpu_util.order_bound)."""
    if algo in ("rccl", "allreduce") and st[2] > 1:
        members = [st[0] + i * (1 << st[1]) for i in range(st[2])]
        ok, inexact = order_bound(got, want, srcs[members], op, TOL_SCALE)
        extra["rccl_inexact_elements"] += inexact
        return ok
    return same_bits(got, want)


def twin(p):
    """The address the test's own HIP copies use for heap pointer p: on a
    mirrored heap the host-view address's HBM twin (view addresses never go
    to HIP, mirror.h), p itself otherwise.  The collectives still get p."""
    return shm.mirror_device_ptr(p) if MIRRORED else p


def heap_write(p, src, nbytes):
    """Fill heap bytes [p, p + nbytes) with a HIP copy.  Mirrored heap: the
    host's stores around them go up first (shmemx_mirror_sync), then the copy
    into the twin, then the view learns its blocks changed on the device
    (shmemx_mirror_invalidate), as INTEGRATION.md prescribes for the caller's
    own device writes."""
    if MIRRORED:
        shm.mirror_sync(p, nbytes)
    shm.memcpy(twin(p), src, nbytes)
    if MIRRORED:
        shm.mirror_invalidate(p, nbytes)


def read(ptr, t, n):
    a = np.empty(n, oracle.NP_DTYPE[t])
    if n:
        shm.memcpy(a, twin(ptr), a.nbytes)
    return a


def run_case(t, op, n, st, algo, mode, seed, expect_algo=None, special=False):
    """One collective call; every PE runs the same sequence, non-members skip.
    expect_algo: the algorithm `auto` resolved to, for the fold order.
    special: NaN / +-0 sources (oracle.special_sources)."""
    global ncases
    srcs = oracle.special_sources(t, npes, n, seed) if special else \
        oracle.sources(t, 1, npes, n, base_seed=seed)
    if not member(*st):
        return
    ncases += 1
    mine = np.ascontiguousarray(srcs[pe])
    ran = expect_algo or resolved(t, op, n, st, algo)
    want = expected(t, op, srcs, st, ran)
    sz = mine.itemsize
    tag = f"{t} {op} n={n} set={st} algo={algo} mode={mode}"
    print(tag, flush=True)   # progress, in the PE's log
    if mode == "host":
        tgt = np.zeros_like(mine)
        src = mine.copy()
        shm.set_algo(algo)
        shm.to_all(t, op, tgt, src, n, *st)
        shm.set_algo("auto")
        got = tgt
    elif mode == "hostinplace":     # one pageable array, target == source
        buf = mine.copy()
        shm.set_algo(algo)
        shm.to_all(t, op, buf, buf, n, *st)
        shm.set_algo("auto")
        got = buf
    elif mode == "hostheap":
        # $SHMEMX_HEAP_MEMORY=host: symmetric objects the host writes directly
        src = host_view(HEAP_SRC, mine.dtype, n)
        tgt = host_view(HEAP_TGT, mine.dtype, n)
        src[:] = mine
        tgt[:] = np.zeros_like(mine)
        shm.set_algo(algo)
        shm.to_all(t, op, HEAP_TGT, HEAP_SRC, n, *st)
        shm.set_algo("auto")
        got = tgt.copy()
    elif mode == "device":
        s, d = to_dev(torch, mine), to_dev(torch, np.zeros_like(mine))
        torch.cuda.synchronize()
        shm.reduce_on_stream(t, op, d, s, n, *st, algo)
        torch.cuda.synchronize()
        got = d.cpu().numpy().view(mine.dtype) if t == "longdouble" else d.cpu().numpy()
    else:
        # symmetric heap: SRC/TGT are heap blocks, identical offsets on all PEs
        src_p = HEAP_SRC
        if mode == "heap":
            tgt_p = HEAP_TGT
        elif mode == "heapoff":   # heap operands off 16-B alignment, differently
            src_p, tgt_p = HEAP_SRC + sz, HEAP_TGT + 3 * sz
        elif mode == "inplace":
            tgt_p = src_p
        else:  # "overlap": target = source + 3 elements (partial overlap)
            tgt_p = src_p + 3 * sz
        if n:
            heap_write(src_p, mine, mine.nbytes)
        if mode in ("heap", "heapoff") and n:
            heap_write(tgt_p, np.full(mine.nbytes, 0xAB, np.uint8), mine.nbytes)
        shm.reduce_on_stream(t, op, tgt_p, src_p, n, *st, algo)
        torch.cuda.synchronize()
        got = read(tgt_p, t, n)
    if not matches(got, want, t, op, srcs, st, ran):
        w = 10 if t == "longdouble" else sz
        a = got.view(np.uint8).reshape(n, -1)[:, :w]
        b = want.view(np.uint8).reshape(n, -1)[:, :w]
        bad = np.flatnonzero((a != b).any(axis=1))
        fails.append(f"{tag}: {len(bad)} elements differ, first at {bad[:4].tolist()}")
    if shm.last_error():
        fails.append(f"{tag}: last_error {shm.last_error()}")


def host_view(ptr, dtype, n):
    """A numpy array over host memory at `ptr` (the host-kind heap)."""
    import ctypes
    nbytes = max(1, n) * np.dtype(dtype).itemsize
    buf = (ctypes.c_char * nbytes).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=n)


def place(arr, mode, heap_ptr):
    """arr in `mode` memory: (handle passed to the library, reader)."""
    if mode == "view":   # the mirrored heap's host view: plain host stores
        v = host_view(heap_ptr, arr.dtype, arr.size)
        v[:] = arr
        return heap_ptr, lambda: v.copy()
    if mode == "host":
        a = arr.copy()
        return a, lambda: a
    if mode == "device":
        t = torch.from_numpy(arr.copy()).cuda()
        torch.cuda.synchronize()
        return t, lambda: t.cpu().numpy()
    if arr.nbytes:
        heap_write(heap_ptr, arr, arr.nbytes)
    return heap_ptr, lambda: read_raw(heap_ptr, arr.dtype, arr.size)


def read_raw(ptr, dtype, n):
    a = np.empty(n, dtype)
    if n:
        shm.memcpy(a, twin(ptr), a.nbytes)
    return a


def run_bcast(bits, n, root, st, mode, seed):
    """shmem_broadcast{32,64}; every non-root member gets the root's source,
    the root's target is untouched (broadcast-linear.c:54-74)."""
    global ncases
    dt = np.int32 if bits == 32 else np.int64
    rng = np.random.default_rng(seed)
    srcs = rng.integers(-2**31, 2**31 - 1, size=(npes, n)).astype(dt)
    tgts = np.full((npes, n), -7, dt)
    if not member(*st):
        return
    ncases += 1
    want = oracle.broadcast_sim(srcs, tgts, root, *st)[pe]
    src, _ = place(srcs[pe], mode, HEAP_SRC)
    tgt, get = place(tgts[pe], mode, HEAP_TGT)
    print(f"broadcast{bits} n={n} root={root} set={st} mode={mode}", flush=True)
    shm.broadcast(bits, tgt, src, n, root, *st)
    torch.cuda.synchronize()
    if not np.array_equal(get(), want) or shm.last_error():
        fails.append(f"broadcast{bits} n={n} root={root} set={st} mode={mode} err={shm.last_error()}")


def run_collect(bits, counts, st, mode, seed):
    """shmem_fcollect (equal counts) / shmem_collect: member i's source lands
    at the running offset (fcollect-linear.c:69-91, collect-linear.c:57-130)."""
    global ncases
    dt = np.int32 if bits == 32 else np.int64
    fixed = len(set(counts)) == 1
    rng = np.random.default_rng(seed)
    maxn = max(counts)
    srcs = rng.integers(-2**31, 2**31 - 1, size=(npes, maxn)).astype(dt)
    cap = sum(counts) + 5
    tgts = np.full((npes, cap), -7, dt)
    if not member(*st):
        return
    ncases += 1
    want = oracle.collect_sim(srcs, counts, tgts, *st)[pe]
    src, _ = place(np.ascontiguousarray(srcs[pe, :counts[pe]]), mode, HEAP_SRC)
    tgt, get = place(tgts[pe], mode, HEAP_TGT)
    kind = "fcollect" if fixed else "collect"
    print(f"{kind}{bits} counts={counts} set={st} mode={mode}", flush=True)
    getattr(shm, kind)(bits, tgt, src, counts[pe], *st)
    torch.cuda.synchronize()
    if not np.array_equal(get(), want) or shm.last_error():
        fails.append(f"{kind}{bits} counts={counts} set={st} mode={mode} err={shm.last_error()}")


MIRRORED = os.environ.get("SHMEMX_HEAP_MEMORY", "mirrored") == "mirrored"   # the default
CAP = 1 << 23 if not (MIRRORED or os.environ.get("SHMEMX_HEAP_MEMORY") == "host") else 48 << 20
HEAP_SRC = shm.malloc(CAP + 64)
HEAP_TGT = shm.malloc(CAP)
assert HEAP_SRC and HEAP_TGT, "shmem_malloc failed"
HOST_HEAP = os.environ.get("SHMEMX_HEAP_MEMORY") == "host"
for q in range(npes if scenario != "heapcheck" else 0):   # (heapcheck may run on private blocks)
    # a host-kind heap is not peer-addressable: NULL, as the reference's
    # shmem_ptr; nor is a mirrored heap's host view (a peer's store would go
    # behind that peer's view), whose HBM twin is
    want_null = (HOST_HEAP or MIRRORED) and q != pe
    if bool(shm.heap_ptr(HEAP_SRC, q)) == want_null:
        fails.append(f"heap_ptr(SRC, {q}) = {shm.heap_ptr(HEAP_SRC, q)}")
    if MIRRORED and not shm.heap_ptr(twin(HEAP_SRC), q):
        fails.append(f"heap_ptr(twin(SRC), {q}) is NULL")

seed = 0x1000
if scenario == "full":
    # every reference pair, every active set, both IPC algorithms, heap operands
    for (t, op) in shm.REFERENCE_PAIRS:
        for st in active_sets():
            for algo in ("direct", "gather"):
                seed += 1
                run_case(t, op, 1013, st, algo, "heap", seed)
    # operand placement: heap, in place, partial overlap, torch device, host
    for t, op in (("double", "sum"), ("long", "xor"), ("longdouble", "max"), ("complexf", "prod"),
                  ("short", "min")):
        for mode in ("inplace", "overlap", "device", "host"):
            for algo in ("direct", "gather"):
                seed += 1
                run_case(t, op, 4103, (0, 0, npes), algo, mode, seed)
    # 100003 doubles: the fused two-shot launch; 1 Mi: the multi-launch two shot
    for n in (0, 1, 2, 63, 65, 100003, 1 << 20):
        seed += 1
        run_case("double", "sum", n, (0, 0, npes), "auto", "heap", seed)
    # pageable host arrays over several 16 MiB staging chunks (the copy gangs
    # filling and draining the page-locked ring), separate and in place
    for t, op, mode in (("double", "sum", "host"), ("long", "xor", "hostinplace"), ("int", "max", "host")):
        seed += 1
        run_case(t, op, (40 << 20) // oracle.NP_DTYPE[t]().itemsize + 3, (0, 0, npes), "auto", mode, seed)
    # heap operands off 16-B alignment through the fused one- and two-shot
    for t, op in (("double", "sum"), ("short", "max"), ("int", "prod")):
        for n in (1013, 100003):
            seed += 1
            run_case(t, op, n, (0, 0, npes), "direct", "heapoff", seed)
    # put through heap_ptr, then a barrier: PE q's slot p holds p + 1.  On a
    # mirrored heap the puts go to the peers' twins, and each PE invalidates
    # its view of the slots after the barrier, then reads them with host loads
    slots = np.zeros(npes, np.int64)
    heap_write(HEAP_TGT, slots, slots.nbytes)
    shm.barrier_all()
    for q in range(npes):
        shm.memcpy(shm.heap_ptr(twin(HEAP_TGT), q) + 8 * pe, np.array([pe + 1], np.int64), 8)
    shm.barrier_all()
    if MIRRORED:
        shm.mirror_invalidate(HEAP_TGT, 8 * npes)
        got = host_view(HEAP_TGT, np.int64, npes).copy()
    else:
        got = read(HEAP_TGT, "long", npes)
    if list(got) != list(range(1, npes + 1)):
        fails.append(f"heap_ptr puts + barrier_all: {list(got)}")
    # the neighbouring collectives over IPC, against their oracles
    for st in active_sets():
        size = st[2]
        for mode in ("heap", "device", "host"):
            for bits in (32, 64):
                seed += 1
                run_bcast(bits, 1031, seed % size, st, mode, seed)
                seed += 1
                run_collect(bits, [517] * npes, st, mode, seed)
                seed += 1
                run_collect(bits, [(37 * (q + 1)) % 101 for q in range(npes)], st, mode, seed)
    seed += 1
    run_collect(64, [0] * npes, (0, 0, npes), "device", seed)
    # subset barriers interleaved with world ones (pairwise counters)
    for st in active_sets():
        if member(*st):
            shm.barrier(*st)
        shm.barrier_all()
elif scenario == "chunk":
    # $SHMEMX_DIRECT_SCRATCH_MB=1: staged operands go through the scratch in
    # 512 KiB chunks, so these take several chunks per call
    for t, op in (("double", "sum"), ("long", "xor"), ("longdouble", "max"), ("int", "prod")):
        for mode in ("device", "inplace", "overlap"):
            for algo in ("direct", "gather"):
                seed += 1
                run_case(t, op, 200003 if t != "longdouble" else 70001, (0, 0, npes), algo, mode, seed)
        for st in active_sets():
            seed += 1
            run_case(t, op, 150001, st, "direct", "device", seed)
    # broadcast / collect through several scratch rounds (1 MiB scratch)
    for mode in ("device", "host", "heap"):
        seed += 1
        run_bcast(64, 300001, 1, (0, 0, npes), mode, seed)
        seed += 1
        run_collect(64, [100003, 30001, 0][:npes] + [7] * max(0, npes - 3), (0, 0, npes), mode, seed)
        seed += 1
        run_collect(32, [150001] * npes, (0, 0, npes), mode, seed)
elif scenario == "signal":
    # SIGNAL: device-side barriers, stream-ordered, heap operands only.  Every
    # reference pair on every active set (one-shot and two-shot sizes), in
    # place, interleaved sets, and a captured graph replayed with new inputs.
    for (t, op) in shm.REFERENCE_PAIRS:
        for st in active_sets():
            for n in (1013, 70001 if t != "longdouble" else 20001):
                seed += 1
                run_case(t, op, n, st, "signal", "heap", seed)
    for t, op in (("double", "sum"), ("long", "xor"), ("float", "min")):
        for n in (4103, 300007):
            seed += 1
            run_case(t, op, n, (0, 0, npes), "signal", "inplace", seed)
    # heap operands off 16-B alignment (source +1, target +3 elements): the
    # fused launches' scalar fold and byte gather
    for t, op in (("double", "sum"), ("short", "max"), ("float", "prod"), ("complexd", "prod"),
                  ("longdouble", "sum")):
        for n in (1013, 70001):
            seed += 1
            run_case(t, op, n, (0, 0, npes), "signal", "heapoff", seed)
    for n in (0, 1, 2, 63, 65, 1 << 20):
        seed += 1
        run_case("double", "sum", n, (0, 0, npes), "signal", "heap", seed)
    # a torch (non-heap) operand is refused up front, before any barrier
    if member(0, 0, npes):
        d = torch.zeros(64, dtype=torch.float64, device="cuda")
        try:
            shm.reduce_on_stream("double", "sum", d, HEAP_SRC, 64, 0, 0, npes, "signal")
            fails.append("signal with a torch target: no error")
        except shm.ShmemError as e:
            if e.code != 3:
                fails.append(f"signal with a torch target: error {e.code}, want ENOTSUP")
    # graph capture: the barriers' counters live on the device, so replays
    # stay in step across PEs; each replay reduces fresh inputs.  50000
    # doubles take the two-shot schedule, 20000 the fused one-shot launch
    # (its grid barrier resets itself, so replays need no host step).
    stream = torch.cuda.Stream()
    for n in (50000, 20000):
        torch.cuda.synchronize()
        shm.reduce_on_stream("double", "sum", HEAP_TGT, HEAP_SRC, n, 0, 0, npes, "signal",
                             stream.cuda_stream)          # warm: maps and votes
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            shm.reduce_on_stream("double", "sum", HEAP_TGT, HEAP_SRC, n, 0, 0, npes, "signal",
                                 stream.cuda_stream)
        for rep_i in range(5):
            seed += 1
            srcs = oracle.sources("double", 1, npes, n, base_seed=seed)
            heap_write(HEAP_SRC, np.ascontiguousarray(srcs[pe]), n * 8)
            torch.cuda.synchronize()
            graph.replay()
            torch.cuda.synchronize()
            ncases += 1
            want = oracle.reduce_sim("double", "sum", srcs, 0, 0, npes)[0]
            if not same_bits(read(HEAP_TGT, "double", n), want):
                fails.append(f"graph replay {rep_i} n={n}: wrong result")
        del graph
elif scenario == "hostheap":
    # $SHMEMX_HEAP_MEMORY=host: shmem_malloc returns page-locked host memory,
    # as the reference's heap is; the host writes the symmetric objects and
    # the blocking calls stage them through the pinned pipeline
    assert HOST_HEAP
    for (t, op) in shm.REFERENCE_PAIRS:
        for st in active_sets():
            seed += 1
            run_case(t, op, 1013, st, "auto", "hostheap", seed)
    for n in (1, 65, (40 << 20) // 8 + 3):
        seed += 1
        run_case("double", "sum", n, (0, 0, npes), "auto", "hostheap", seed)
    for st in active_sets():
        seed += 1
        run_bcast(64, 1031, 0, st, "heap", seed)
        seed += 1
        run_collect(32, [(37 * (q + 1)) % 101 for q in range(npes)], st, "heap", seed)
elif scenario == "rccl":
    # The default RCCL transport, with the RCCL test double standing in for
    # librccl ($FAKE_RCCL): the library's own RCCL call sequences — reduce-
    # scatter + all-gather with the all-reduce tail, one all-reduce, A2A and
    # GATHER over grouped send/recv, broadcast / [f]collect / barrier /
    # verify over RCCL — across real processes and device pointers.
    def usable(t, op, n, st, algo):
        try:
            shm.plan(t, op, n, *st, st[0], npes, algo)
            return True
        except shm.ShmemError:
            return False

    for (t, op) in shm.REFERENCE_PAIRS:
        for st in active_sets():
            for algo in ("auto", "rccl", "allreduce", "a2a", "gather"):
                if not usable(t, op, 1013, st, algo):
                    continue
                seed += 1
                run_case(t, op, 1013, st, algo, "device", seed)
    for t, op in (("double", "sum"), ("int", "max"), ("long", "xor"), ("float", "prod")):
        for algo in ("auto", "rccl", "allreduce", "a2a", "gather"):
            if not usable(t, op, 4103, (0, 0, npes), algo):
                continue
            for mode in ("heap", "inplace", "overlap", "host"):
                seed += 1
                run_case(t, op, 4103, (0, 0, npes), algo, mode, seed)
    for n in (0, 1, 2, 63, 65, 1 << 20, (4 << 20) // 8 + 13, (6 << 20) + 5):
        seed += 1
        run_case("double", "sum", n, (0, 0, npes), "auto", "device", seed)   # all-reduce, then RS+AG+tail
    seed += 1
    run_case("long", "sum", (6 << 20) + 5, (0, 0, npes), "rccl", "device", seed)
    # pageable host arrays across staging chunks, separate and in place
    for t, op, mode in (("double", "sum", "host"), ("long", "xor", "hostinplace")):
        seed += 1
        run_case(t, op, (5 << 20) + 3, (0, 0, npes), "auto", mode, seed)
    # A2A with every shard full on the whole job: its all-gather is RCCL's
    # own (in place), not grouped p2p
    for t, op in (("long", "xor"), ("float", "min"), ("short", "and"), ("double", "sum")):
        for mode in ("device", "inplace"):
            seed += 1
            run_case(t, op, 24576, (0, 0, npes), "a2a", mode, seed)
    for st in active_sets():
        size = st[2]
        for mode in ("heap", "device", "host"):
            for bits in (32, 64):
                seed += 1
                run_bcast(bits, 1031, seed % size, st, mode, seed)
                seed += 1
                run_collect(bits, [517] * npes, st, mode, seed)
                seed += 1
                run_collect(bits, [(37 * (q + 1)) % 101 for q in range(npes)], st, mode, seed)
    extra["set_comms"] = shm.set_comms()
    for st in active_sets():
        if member(*st):
            shm.barrier(*st)
            ncases += 1
            n = 4099
            v = torch.arange(n, dtype=torch.float64, device="cuda")
            if not shm.verify("double", v, n, *st):
                fails.append(f"verify of identical arrays on {st}")
            w = v.clone()
            w[pe % n] += 1
            if st[2] > 1 and shm.verify("double", w, n, *st):
                fails.append(f"verify of differing arrays on {st} said equal")
        shm.barrier_all()
elif scenario == "rccl_order":
    # RCCL-ordered float sums and products on the RCCL transport (the test
    # double folds in ring / rotated order, as RCCL does, not in PE_start's):
    # the whole job on the world communicator and every partial set on its
    # members-only communicator, reduce-scatter + all-gather (+ tail) and one
    # all-reduce, mixed-sign sources, each held against the reference's
    # PE_start fold within the stated bound ($RCCL_TOL_SCALE scales it).
    sets = [st for st in active_sets() if st[2] > 1]
    for t, op in (("double", "sum"), ("float", "sum"), ("double", "prod"), ("float", "prod")):
        for st in sets:
            for algo in ("rccl", "allreduce"):
                for n in (4103, 300007):
                    seed += 1
                    run_case(t, op, n, st, algo, "device", seed)
    # two different partial sets back to back, alternating (each member meets
    # each set at the same call, so no member waits for a communicator the
    # others are not building)
    if npes >= 3:
        for rep in range(3):
            for st in ((0, 0, npes - 1), (1, 0, npes - 1)):
                seed += 1
                run_case("int", "sum", 1000 + rep, st, "auto", "device", seed)
    extra["set_comms"] = shm.set_comms()
elif scenario == "setcap":
    # $SHMEMX_SET_COMMS_MAX: a PE keeps at most that many set communicators;
    # a set whose members do not all have room keeps the world communicator
    # (auto: A2A), decided alike on every member.  Every partial set, twice,
    # auto on an RCCL-native pair and a bitwise one, against the oracle.
    for rep in range(2):
        for st in active_sets():
            if st[2] < 2 or st == (0, 0, npes):
                continue
            for t, op in (("double", "sum"), ("long", "xor")):
                seed += 1
                run_case(t, op, 2053, st, "auto", "device", seed)
    extra["set_comms"] = shm.set_comms()
elif scenario == "soak":
    # Random calls, the same sequence on every PE (one seeded generator):
    # type/op pair, size (edges favoured), active set, algorithm and operand
    # placement, on whichever transport the environment selects.
    import random
    rng = random.Random(int(os.environ.get("SOAK_SEED", "7")))
    iters = int(os.environ.get("SOAK_ITERS", "60"))
    rccl = os.environ.get("SHMEMX_TRANSPORT") != "ipc"
    algos = ("auto", "rccl", "allreduce", "a2a", "gather", "direct", "signal") if rccl else \
        ("auto", "direct", "gather", "signal")
    sets = active_sets()
    edges = (0, 1, 2, 3, 7, 15, 16, 17, 63, 64, 65, 127, 1023, 4096, 4097, 32768 + 1)
    for it in range(iters):
        if rng.random() < 0.2:
            # a neighbouring collective instead: broadcast, fcollect or collect
            st = rng.choice(sets)
            mode = rng.choice(("heap", "device", "host"))
            bits = rng.choice((32, 64))
            kind = rng.choice(("bcast", "fcollect", "collect"))
            seed += 1
            if kind == "bcast":
                run_bcast(bits, rng.choice((0, 1, 5, 1031, 70001)), rng.randrange(st[2]), st, mode, seed)
            elif kind == "fcollect":
                run_collect(bits, [rng.choice((0, 1, 17, 517, 20000))] * npes, st, mode, seed)
            else:
                run_collect(bits, [rng.randrange(0, 20000) for _ in range(npes)], st, mode, seed)
            continue
        t, op = rng.choice(shm.REFERENCE_PAIRS)
        n = rng.choice(edges) if rng.random() < 0.5 else rng.randrange(1, 300000)
        if t == "longdouble":
            n = min(n, 40000)
        st = rng.choice(sets)
        algo = rng.choice(algos)
        # on the mirrored heap also "hostheap": host stores into the view, the
        # blocking call on the view addresses, host loads of the result
        # (the small-result copy-back, the same-stream flush, lazy fetches)
        extra_modes = ("hostheap",) if MIRRORED else ()
        mode = rng.choice(("heap", "device", "inplace", "overlap", "host", "heapoff") + extra_modes)
        if algo == "signal":
            mode = rng.choice(("heap", "inplace", "heapoff") + extra_modes)     # symmetric operands only
        if (n + 3) * 16 > CAP:
            n = CAP // 16 - 3
        try:
            shm.plan(t, op, n, *st, st[0], npes, algo)
        except shm.ShmemError:
            continue                               # not a valid (set, algo) pair here
        seed += 1
        run_case(t, op, n, st, algo, mode, seed)
elif scenario == "autotable":
    # $SHMEMX_AUTO_FULL / $SHMEMX_AUTO_PARTIAL (runtime.cpp make_plan): the
    # plan `auto` resolves to for each case of $AUTO_EXPECT ([type, op, n,
    # PE_start, logPE_stride, PE_size, expected algorithm] rows), then the
    # call itself through `auto`, against the oracle
    for t, op, n, st0, st1, st2, want_algo in json.loads(os.environ["AUTO_EXPECT"]):
        st = (st0, st1, st2)
        seed += 1
        if not member(*st):
            continue
        got_algo = shm.plan(t, op, n, *st, pe, npes, "auto").algo
        extra.setdefault("plans", []).append([t, op, n, list(st), got_algo])
        if got_algo != want_algo:
            fails.append(f"auto plan {t} {op} n={n} set={st}: {got_algo}, want {want_algo}")
        run_case(t, op, n, st, "auto", "device", seed, expect_algo=got_algo)
elif scenario == "refops":
    # The multi-PE kernels' element ops against the REFERENCE'S OWN
    # (tests/golden/ref_element_ops.json: reduce-op.c:71-150 compiled from its
    # text).  2 PEs: PE 0's source is the fixture's a, PE 1's is b, for all 44
    # pairs on special values and random bits.  DIRECT and SIGNAL give every PE
    # PE_start's order, op(a, b); own-order GATHER, and every algorithm on the
    # float / double / long double min and max, give PE 1 op(b, a).  The
    # one-shot/two-shot and fused/unfused schedules come from the test's env.
    import base64
    with open(os.path.join(HERE, "golden", "ref_element_ops.json")) as f:
        cases = json.load(f)["cases"]
    for t, c in cases.items():
        dt = np.dtype(oracle.NP_DTYPE[t])
        ab = [np.frombuffer(base64.b64decode(c[k]), dtype=dt).copy() for k in ("a", "b")]
        mine = ab[pe]
        n = mine.size
        for op, o in c["ops"].items():
            for algo in ("direct", "signal", "gather"):
                ncases += 1
                own = algo == "gather" or (t, op) in OWN_ORDER
                key = "ba" if (own and pe == 1) else "ab"
                want = np.frombuffer(base64.b64decode(o[key]), dtype=dt)
                heap_write(HEAP_SRC, mine, mine.nbytes)
                heap_write(HEAP_TGT, np.full(mine.nbytes, 0xAB, np.uint8), mine.nbytes)
                shm.reduce_on_stream(t, op, HEAP_TGT, HEAP_SRC, n, 0, 0, npes, algo)
                torch.cuda.synchronize()
                got = read(HEAP_TGT, t, n)
                if op in ("sum", "prod") and t in ("float", "double", "complexd", "complexf"):
                    ft = np.float32 if t in ("float", "complexf") else np.float64
                    g, w = got.view(ft), want.view(ft)
                    ok = (np.array_equal(np.isnan(g), np.isnan(w))
                          and g[~np.isnan(w)].tobytes() == w[~np.isnan(w)].tobytes())
                else:
                    ok = same_bits(got, want)
                if not ok or shm.last_error():
                    fails.append(f"refops {t} {op} algo={algo}: differs from the reference "
                                 f"(last_error {shm.last_error()})")
elif scenario == "ownorder":
    # min / max of float, double and long double on NaN / +-0 sources, where
    # each PE's reference answer depends on its own fold order: every
    # algorithm the transport has (auto first), every active set, one-shot
    # (fused) and larger sizes, heap / in-place / device operands; every PE
    # against its own oracle result.  extra["own_order_differs"] counts the
    # elements where that differs from PE_start's (the test requires > 0).
    rccl = os.environ.get("SHMEMX_TRANSPORT") != "ipc"
    algos = ("auto", "a2a", "gather", "direct", "signal") if rccl else ("auto", "gather", "direct", "signal")
    for t in ("float", "double", "longdouble"):
        for op in ("min", "max"):
            for st in active_sets():
                for algo in algos:
                    for n, mode in ((1013, "heap"), (70001, "inplace"), (40007, "device")):
                        if algo == "signal" and mode == "device":
                            mode = "heap"
                        try:
                            shm.plan(t, op, n, *st, st[0], npes, algo)
                        except shm.ShmemError:
                            continue
                        seed += 1
                        run_case(t, op, n, st, algo, mode, seed, special=True)
        if not rccl:
            extra["auto_algo"] = shm.plan(t, "min", 1013, 0, 0, npes, pe, npes, "auto").algo
    # the blocking drop-in entry point on host arrays, auto
    for t in ("float", "double"):
        seed += 1
        run_case(t, "max", 4103, (0, 0, npes), "auto", "host", seed, special=True)
elif scenario == "xchg":
    # Small blocking calls over several PEs under auto (<= 4 KiB per PE):
    # each member's resident service workgroup folds the members' exchange
    # slots (staging.cpp xchg_reduce), no kernel launch.  Every reference
    # pair at 1 element, at the 4 KiB limit and one element past it (DIRECT /
    # RCCL again), every active set, heap operands; host and in-place host
    # operands for a few pairs; the own-order pairs on NaN / +-0 sources.
    shm.service_stats(reset=True)
    for (t, op) in shm.REFERENCE_PAIRS:
        sz = oracle.NP_DTYPE[t]().itemsize
        for n in (1, 4096 // sz, 4096 // sz + 1):
            for st in active_sets():
                seed += 1
                run_case(t, op, n, st, "auto", "heap", seed, special=(t, op) in OWN_ORDER)
    for (t, op) in (("int", "sum"), ("double", "max"), ("longdouble", "sum"), ("complexf", "prod")):
        for mode in ("host", "hostinplace"):
            for st in active_sets():
                seed += 1
                run_case(t, op, 4096 // oracle.NP_DTYPE[t]().itemsize, st, "auto", mode, seed,
                         special=(t, op) in OWN_ORDER)
    extra["folds"] = shm.service_stats(reset=True)["folds"]
    if npes > 1 and not extra["folds"]:
        fails.append("no small multi-PE call was folded by the service workgroup")
    # configs[0]'s call (int sum, n = 1024, PEs 0-1) timed from C on this
    # heap (on the mirrored heap: host-written view addresses), for the log
    if npes >= 2 and pe < 2:
        sys.path.insert(0, os.path.dirname(HERE))
        import bench  # noqa: E402  (call_times_us: the C call timer)
        vals = (np.arange(1024, dtype=np.int32) * 3 + pe).astype(np.int32)
        if MIRRORED:
            host_view(HEAP_SRC, np.int32, 1024)[:] = vals
        else:
            heap_write(HEAP_SRC, vals, vals.nbytes)
        ts = bench.call_times_us("int", "sum", HEAP_TGT, HEAP_SRC, 1024, 0, 0, 2, np.full(128, -1, np.int64), 20, 300)
        if ts:
            extra["config0_c_us"] = round(float(np.median(ts)), 2)
elif scenario == "config0":
    # BASELINE.json configs[0]: shmem_int_sum_to_all, nreduce = 1024, on 2 PEs
    # (the reference's "oshrun loopback"), through the C entry point itself
    # with the reference's pWrk and pSync arguments, on the HIP path.  Sources
    # are the oracle's (SURVEY §8d seeds, kind 0), so the test runner can hold
    # every PE's target against oracle_reduce_fork, the fork-per-PE run of the
    # restated reduce-op.c (the GASNet smp model); here each target is also
    # compared element for element with the oracle's simulation.
    n = 1024
    srcs = oracle.sources("int", 0, npes, n)
    want = oracle.reduce_sim("int", "sum", srcs, 0, 0, npes)[pe]
    modes = ("view", "host") if MIRRORED else ("heap", "device", "host")
    extra["target_hash"] = {}
    for mode in modes:
        ncases += 1
        pwrk = np.zeros(64, np.int32)                   # SHMEM_REDUCE_MIN_WRKDATA_SIZE
        psync = np.full(128, -1, np.int64)              # SHMEM_REDUCE_SYNC_SIZE x SHMEM_SYNC_VALUE
        src, _ = place(np.ascontiguousarray(srcs[pe]), mode, HEAP_SRC)
        tgt, get = place(np.full(n, -7, np.int32), mode, HEAP_TGT)
        shm.barrier_all()
        print(f"config0 int sum n={n} mode={mode}", flush=True)
        shm.to_all("int", "sum", tgt, src, n, 0, 0, npes, pwrk, psync)
        torch.cuda.synchronize()
        got = np.ascontiguousarray(get())
        extra["target_hash"][mode] = oracle.value_hash("int", got)
        if shm.last_error() or not same_bits(got, want):
            fails.append(f"config0 mode={mode}: error {shm.last_error()} / wrong result")
        if not np.all(psync == -1):
            fails.append(f"config0 mode={mode}: pSync not left at SHMEM_SYNC_VALUE")
        algo = shm.plan("int", "sum", n, 0, 0, npes, pe, npes, "auto").algo
        extra.setdefault("algo", {})[mode] = algo
elif scenario == "configs":
    # BASELINE.json configs at full size through the blocking drop-in entry
    # points, every PE a process: long and/or/xor over 64 Mi elements
    # (configs[3]) and double sum over 32 Mi (configs[2]).  Every PE
    # regenerates all P sources on the GPU and folds them with torch in the
    # reference's PE_start order; the result must match bit for bit, and the
    # checksums of all PEs' targets must agree (shmemx_verify).
    big = 64 * 1024 * 1024 * 8
    BIG_SRC, BIG_TGT = shm.malloc(big), shm.malloc(big)
    assert BIG_SRC and BIG_TGT, "shmem_malloc of the config operands failed"

    def gen(t, q, n, salt):
        g = torch.Generator(device="cuda")
        g.manual_seed(0xC0F1C + 97 * q + salt)
        if t == "long":
            return torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
        return torch.rand(n, dtype=torch.float64, device="cuda", generator=g) + 1.0

    cases = [("long", op, 64 * 1024 * 1024) for op in ("and", "or", "xor")]
    cases += [("double", "sum", 32 * 1024 * 1024)]
    for salt, (t, op, n) in enumerate(cases):
        ncases += 1
        print(f"config {t} {op} n={n}", flush=True)
        heap_write(BIG_SRC, gen(t, pe, n, salt), n * 8)
        heap_write(BIG_TGT, torch.zeros(n, dtype=torch.int64, device="cuda"), n * 8)
        torch.cuda.synchronize()
        shm.to_all(t, op, BIG_TGT, BIG_SRC, n, 0, 0, npes)
        if shm.last_error():
            fails.append(f"config {t} {op}: last_error {shm.last_error()}")
            continue
        got = torch.empty(n, dtype=torch.int64 if t == "long" else torch.float64, device="cuda")
        shm.memcpy(got, twin(BIG_TGT), n * 8)
        f = {"and": torch.bitwise_and, "or": torch.bitwise_or, "xor": torch.bitwise_xor,
             "sum": torch.add}[op]
        want = gen(t, 0, n, salt)
        for q in range(1, npes):
            want = f(want, gen(t, q, n, salt))
        torch.cuda.synchronize()
        if not torch.equal(got.view(torch.int64), want.view(torch.int64)):
            bad = int((got.view(torch.int64) != want.view(torch.int64)).sum())
            fails.append(f"config {t} {op} n={n}: {bad} elements differ")
        # and against the oracle itself on every element (the restated
        # reduce-op.c fold in PE_start's order, this PE's target alone:
        # oracle_reduce_one), not only torch's fold
        srcs = np.stack([gen(t, q, n, salt).cpu().numpy() for q in range(npes)])
        ref = oracle.reduce_one(t, op, srcs, 0, 0, npes, 0)
        del srcs
        if not same_bits(got.cpu().numpy(), ref):
            fails.append(f"config {t} {op} n={n}: elements differ from the oracle (full size)")
        extra["oracle_full_elements"] = extra.get("oracle_full_elements", 0) + n
        if not shm.verify(t, BIG_TGT, n, 0, 0, npes):
            fails.append(f"config {t} {op} n={n}: targets differ across PEs")
        del got, want
    shm.free(BIG_TGT)
    shm.free(BIG_SRC)
elif scenario == "configs8":
    # BASELINE.json's 8-PE workloads as 8 PE processes on the one GPU, through
    # the blocking drop-in entry points (the reference's peer loop at PE_size
    # 8, reduce-op.c:219-248): configs[2], double sum over 32 Mi elements, on
    # DIRECT (auto on this transport), SIGNAL and own-order GATHER; configs[4],
    # the float sum sweep 4 Ki .. 256 Mi (x4 steps; $CONFIGS8_MAX caps it).
    # Every PE regenerates all P sources on the GPU and folds them with torch
    # in the reference's order (PE_start first; GATHER: its own source
    # first), one IEEE add at a time, so the result must match bit for bit;
    # shmemx_verify checks the targets agree across the set.
    maxn = int(os.environ.get("CONFIGS8_MAX", str(256 * 1024 * 1024)))
    big = max(32 * 1024 * 1024 * 8, maxn * 4)
    BIG_SRC, BIG_TGT = shm.malloc(big), shm.malloc(big)
    assert BIG_SRC and BIG_TGT, "shmem_malloc of the config operands failed"

    def gen(t, q, n, salt):
        g = torch.Generator(device="cuda")
        g.manual_seed(0x8E8 + 131 * q + salt)
        dt = torch.float64 if t == "double" else torch.float32
        return torch.rand(n, dtype=dt, device="cuda", generator=g) + 1.0

    cases = [("double", 32 * 1024 * 1024, algo) for algo in ("auto", "signal", "gather")]
    n = 4096
    while n <= maxn:
        cases.append(("float", n, "auto"))
        n *= 4
    cases += [("float", 16 * 1024 * 1024 + 5, "signal"), ("float", 4096 + 3, "gather")]
    for salt, (t, n, algo) in enumerate(cases):
        ncases += 1
        print(f"configs8 {t} sum n={n} algo={algo}", flush=True)
        dt = torch.float64 if t == "double" else torch.float32
        sz = 8 if t == "double" else 4
        heap_write(BIG_SRC, gen(t, pe, n, salt), n * sz)
        heap_write(BIG_TGT, torch.zeros(n, dtype=dt, device="cuda"), n * sz)
        torch.cuda.synchronize()
        shm.set_algo(algo)
        shm.to_all(t, "sum", BIG_TGT, BIG_SRC, n, 0, 0, npes)
        shm.set_algo("auto")
        if shm.last_error():
            fails.append(f"configs8 {t} n={n} {algo}: last_error {shm.last_error()}")
            continue
        got = torch.empty(n, dtype=dt, device="cuda")
        shm.memcpy(got, twin(BIG_TGT), n * sz)
        order = list(range(npes))
        if algo == "gather":
            order = [pe] + [q for q in order if q != pe]
        want = gen(t, order[0], n, salt)
        for q in order[1:]:
            want = want + gen(t, q, n, salt)
        torch.cuda.synchronize()
        iv = torch.int64 if t == "double" else torch.int32
        if not torch.equal(got.view(iv), want.view(iv)):
            bad = int((got.view(iv) != want.view(iv)).sum())
            fails.append(f"configs8 {t} n={n} {algo}: {bad} elements differ")
        # against the oracle itself (each PE's own order for GATHER,
        # PE_start's otherwise): every element up to 256 MiB per PE
        # (configs[2] whole: 32 Mi doubles; oracle_reduce_one folds this PE's
        # target alone, ~2 GiB of host memory per PE), 64 Ki sampled
        # elements above that
        if n * sz <= 256 << 20:
            srcs = np.stack([gen(t, q, n, salt).cpu().numpy() for q in range(npes)])
            ref = oracle.reduce_one(t, "sum", srcs, 0, 0, npes, pe if algo == "gather" else 0)
            if not same_bits(got.cpu().numpy(), ref):
                fails.append(f"configs8 {t} n={n} {algo}: elements differ from the oracle (full size)")
            extra.setdefault("oracle_full_elements", 0)
            extra["oracle_full_elements"] += n
        else:
            smp = torch.arange(0, n, max(1, n // 65536), device="cuda")
            srcs = np.stack([gen(t, q, n, salt)[smp].cpu().numpy() for q in range(npes)])
            ref = oracle.reduce_sim(t, "sum", srcs, 0, 0, npes)[pe if algo == "gather" else 0]
            if not same_bits(got[smp].cpu().numpy(), ref):
                fails.append(f"configs8 {t} n={n} {algo}: sampled elements differ from the oracle")
        del srcs
        if algo != "gather" and not shm.verify(t, BIG_TGT, n, 0, 0, npes):
            fails.append(f"configs8 {t} n={n} {algo}: targets differ across PEs")
        del got, want
    shm.free(BIG_TGT)
    shm.free(BIG_SRC)
elif scenario == "mirrored":
    # $SHMEMX_HEAP_MEMORY=mirrored: shmem_malloc returns host-view addresses
    # of the HBM heap.  Host code writes the sources with plain stores (numpy
    # over the view), the blocking drop-in calls run on the HBM twins
    # (DIRECT reads the peers' HBM on the IPC transport), and host code reads
    # the targets back — against the oracle, bit for bit; only the blocks the
    # host touched cross PCIe.
    assert MIRRORED
    import time
    shm.direct_stats(reset=True)
    for (t, op) in shm.REFERENCE_PAIRS:
        for st in active_sets():
            seed += 1
            run_case(t, op, 1013, st, "auto", "hostheap", seed)
    for n in (1, 65, (40 << 20) // 8 + 3):
        seed += 1
        run_case("double", "sum", n, (0, 0, npes), "auto", "hostheap", seed)
    # in place on the view
    n = 200003
    srcs = oracle.sources("long", 1, npes, n, base_seed=0x515)
    v = host_view(HEAP_SRC, np.int64, n)
    v[:] = srcs[pe]
    shm.to_all("long", "xor", HEAP_SRC, HEAP_SRC, n, 0, 0, npes)
    ncases += 1
    if shm.last_error() or not same_bits(v.copy(), oracle.reduce_sim("long", "xor", srcs, 0, 0, npes)[0]):
        fails.append(f"mirrored in place long xor n={n}: error {shm.last_error()} / wrong result")
    # untouched sources do not move again: the second identical call copies
    # nothing host -> HBM, and reading the target back fetches only its blocks
    n = (32 << 20) // 8
    srcs = oracle.sources("double", 1, npes, n, base_seed=0x616)
    src, tgt = host_view(HEAP_SRC, np.float64, n), host_view(HEAP_TGT, np.float64, n)
    src[:] = srcs[pe]
    want = oracle.reduce_sim("double", "sum", srcs, 0, 0, npes)[0]
    world = (0, 0, npes)
    ran32 = resolved("double", "sum", n, world, "auto")
    shm.to_all("double", "sum", HEAP_TGT, HEAP_SRC, n, 0, 0, npes)
    ncases += 1
    if not matches(tgt.copy(), want, "double", "sum", srcs, world, ran32):
        fails.append("mirrored 32 MiB double sum: wrong result")
    shm.mirror_stats(reset=True)
    t0 = time.time()
    shm.to_all("double", "sum", HEAP_TGT, HEAP_SRC, n, 0, 0, npes)
    dt = time.time() - t0
    st = shm.mirror_stats(reset=True)
    nblk = (n * 8) // (64 << 10)          # the target spans nblk or nblk + 1 blocks
    if st["blocks_flushed"] != 0 or st["blocks_device_newer"] not in (nblk, nblk + 1):
        fails.append(f"mirrored repeat call moved blocks: {st}")
    got = tgt.copy()
    st = shm.mirror_stats(reset=True)
    if not matches(got, want, "double", "sum", srcs, world, ran32) or st["blocks_fetched"] not in (nblk, nblk + 1):
        fails.append(f"mirrored read-back: {st}")
    print(f"repeat 32 MiB call on untouched mirrored operands: {dt * 1e3:.2f} ms", flush=True)
    # a system call given a view address does not take the page fault: on the
    # target a collective just wrote it fails with EFAULT, and
    # shmemx_mirror_acquire opens the range first (write(2) of a result)
    import ctypes
    import errno
    import tempfile
    shm.to_all("double", "sum", HEAP_TGT, HEAP_SRC, n, 0, 0, npes)
    nb = 1 << 20
    with tempfile.TemporaryFile() as f:
        raw = (ctypes.c_char * nb).from_address(HEAP_TGT)
        try:
            os.write(f.fileno(), raw)
            fails.append("mirrored: write(2) of a device-newer target did not fail")
        except OSError as e:
            if e.errno != errno.EFAULT:
                fails.append(f"mirrored: write(2) failed with {e}, want EFAULT")
        shm.mirror_acquire(HEAP_TGT, nb)
        if os.write(f.fileno(), raw) != nb:
            fails.append("mirrored: short write(2) after shmemx_mirror_acquire")
        f.seek(0)
        if not matches(np.frombuffer(f.read(), dtype=np.float64), want[:nb // 8], "double", "sum",
                       srcs[:, :nb // 8], world, ran32):
            fails.append("mirrored: write(2) after shmemx_mirror_acquire wrote wrong bytes")
    ncases += 1
    # a SMALL result (<= 256 KiB) comes back into the
    # view before the blocking call returns: write(2) of it works with no
    # shmemx_mirror_acquire, the blocks are CLEAN, and the
    # copy-back moved only the result's bytes
    for m, t in ((512, "double"), (1, "longlong"), ((256 << 10) // 8, "long")):
        srcs = oracle.sources(t, 1, npes, m, base_seed=0x727 + m)
        host_view(HEAP_SRC, oracle.NP_DTYPE[t], m)[:] = srcs[pe]
        shm.mirror_stats(reset=True)
        shm.to_all(t, "sum", HEAP_TGT, HEAP_SRC, m, 0, 0, npes)
        st = shm.mirror_stats(reset=True)
        ncases += 1
        with tempfile.TemporaryFile() as f:
            raw = (ctypes.c_char * (m * 8)).from_address(HEAP_TGT)
            try:
                wrote = os.write(f.fileno(), raw)
            except OSError as e:
                wrote = f"{e}"
            f.seek(0)
            back = np.frombuffer(f.read(), dtype=oracle.NP_DTYPE[t])
        if wrote != m * 8 or not matches(back, oracle.reduce_sim(t, "sum", srcs, 0, 0, npes)[0], t, "sum",
                                         srcs, (0, 0, npes), resolved(t, "sum", m, (0, 0, npes), "auto")):
            fails.append(f"mirrored: write(2) of a fresh {m * 8}-byte {t} result without acquire: {wrote}")
        if st["blocks_settled"] < 1 or st["blocks_fetched"] != 0:
            fails.append(f"mirrored: {m * 8}-byte result not settled by the call: {st}")
    # the light path (ISx's round: host store, blocking call, host load, with
    # nreduce = 1): past the first round no page fault, no block marked
    # device-newer, only the source's own bytes flushed, the result settled
    # into the view by the call, on every PE
    s8, t8 = shm.malloc(8), shm.malloc(8)
    sv, tv = host_view(s8, np.int64, 1), host_view(t8, np.int64, 1)
    shm.service_stats(reset=True)
    for r in range(21):
        if r == 1:
            shm.mirror_stats(reset=True)
        sv[0] = 1000 * (pe + 1) + r
        shm.to_all("longlong", "sum", t8, s8, 1, 0, 0, npes)
        want = sum(1000 * (q + 1) + r for q in range(npes))
        if int(tv[0]) != want:
            fails.append(f"mirrored light path round {r}: {int(tv[0])}, want {want}")
            break
    st = shm.mirror_stats(reset=True)
    ncases += 1
    # (one PE: PE_size 1, a copy: the source goes through the coherent bounce
    # buffer; several PEs: through the exchange, by a CPU copy from the view
    # into the PE's slot; either way nothing is flushed and the source's block
    # stays HOST_NEWER.  Without the service workgroup — off by default when,
    # as here, several PE processes share the GPU — the source's bytes are
    # flushed to its HBM twin every round.)
    no_flush = npes == 1 or shm.service_stats(reset=True)["folds"] > 0
    flushed_ok = st["blocks_flushed"] == 0 if no_flush else st["blocks_flushed"] >= 20
    if (st["write_faults"] or st["read_faults"] or st["blocks_device_newer"] or st["blocks_fetched"]
            or st["blocks_settled"] < 20 or not flushed_ok):
        fails.append(f"mirrored light path: 20 ISx rounds changed block states: {st}")
    if npes == 1:
        # the source's host-written bytes never went to HBM: a stream-ordered
        # call on it (device side) flushes its block first and sees them
        sv[0] = 424242
        shm.reduce_on_stream("longlong", "sum", t8, s8, 1, 0, 0, 1, "auto", 0)
        torch.cuda.synchronize()
        ncases += 1
        if int(tv[0]) != 424242:
            fails.append(f"mirrored light path: a stream-ordered call after the bounce rounds read {int(tv[0])}")
    # a light call that fails (this PE outside the set, or a set past npes)
    # writes nothing: the host's own bytes of the target stay, though its
    # block was never flushed to HBM
    sv[0] = 5
    tv[0] = 1234567 + pe
    if npes > 1:
        shm.to_all("longlong", "sum", t8, s8, 1, (pe + 1) % npes, 0, 1)
    else:
        shm.to_all("longlong", "sum", t8, s8, 1, 0, 0, 2)
    ncases += 1
    if shm.last_error() == 0 or int(tv[0]) != 1234567 + pe:
        fails.append(f"mirrored light path: a failed call (error {shm.last_error()}) left {int(tv[0])}")
    shm.free(t8)
    shm.free(s8)
    # the same for a target past the light path (64 KiB: its blocks are
    # flushed to HBM on the library stream and copied back by the failed
    # call's settle), ADVICE r04: the settle waits for the flush, so the view
    # keeps the host's own bytes
    m = 8192
    s64, t64 = shm.malloc(m * 8), shm.malloc(m * 8)
    sv, tv = host_view(s64, np.int64, m), host_view(t64, np.int64, m)
    for rep in range(3):
        sv[:] = np.arange(m) + rep
        pattern = np.arange(m, dtype=np.int64) * 7 + 1000 * pe + rep
        tv[:] = pattern
        if npes > 1:
            shm.to_all("longlong", "sum", t64, s64, m, (pe + 1) % npes, 0, 1)
        else:
            shm.to_all("longlong", "sum", t64, s64, m, 0, 0, 2)
        ncases += 1
        if shm.last_error() == 0 or not np.array_equal(tv.copy(), pattern):
            fails.append(f"mirrored 64 KiB target: a failed call (error {shm.last_error()}) changed the view")
            break
    shm.free(t64)
    shm.free(s64)
    # and read(2) straight into a source: acquired for writing first, then
    # the reduction sees the bytes the system call stored
    m = 50000
    srcs = oracle.sources("long", 1, npes, m, base_seed=0x717)
    with tempfile.TemporaryFile() as f:
        f.write(np.ascontiguousarray(srcs[pe]).tobytes())
        f.seek(0)
        shm.mirror_acquire(HEAP_SRC, m * 8, for_write=True)
        got_n = os.readv(f.fileno(), [(ctypes.c_char * (m * 8)).from_address(HEAP_SRC)])
    shm.to_all("long", "xor", HEAP_TGT, HEAP_SRC, m, 0, 0, npes)
    ncases += 1
    if got_n != m * 8 or not same_bits(host_view(HEAP_TGT, np.int64, m).copy(),
                                       oracle.reduce_sim("long", "xor", srcs, 0, 0, npes)[0]):
        fails.append(f"mirrored: read(2) into an acquired source ({got_n} bytes) then xor: wrong result")
    # SIGNAL (device barriers) on the view addresses: the twins are symmetric
    seed += 1
    srcs = oracle.sources("float", 1, npes, 70001, base_seed=seed)
    host_view(HEAP_SRC, np.float32, 70001)[:] = srcs[pe]
    shm.reduce_on_stream("float", "sum", HEAP_TGT, HEAP_SRC, 70001, 0, 0, npes, "signal")
    ncases += 1
    if not same_bits(host_view(HEAP_TGT, np.float32, 70001).copy(),
                     oracle.reduce_sim("float", "sum", srcs, 0, 0, npes)[0]):
        fails.append("mirrored SIGNAL float sum: wrong result")
    # broadcast and collect on view addresses
    for st in active_sets():
        seed += 1
        run_bcast(64, 1031, 0, st, "view", seed)
        seed += 1
        run_collect(32, [(37 * (q + 1)) % 101 for q in range(npes)], st, "view", seed)
    # shmem_realloc keeps the contents the host wrote through the view
    ncases += 1
    p1 = shm.malloc(1000 * 8)
    v1 = host_view(p1, np.int64, 1000)
    v1[:] = np.arange(1000) * 3 + pe
    p2 = shm.realloc(p1, 3000 * 8)
    if not p2 or not np.array_equal(host_view(p2, np.int64, 1000).copy(), np.arange(1000) * 3 + pe):
        fails.append("mirrored shmem_realloc lost the host-written contents")
    shm.free(p2)
    if npes > 1 and not shm.direct_stats(reset=False)["calls"] and os.environ.get("SHMEMX_TRANSPORT") == "ipc":
        fails.append("mirrored calls did not run DIRECT on the HBM twins")
elif scenario == "mirror_stream":
    # The mirrored view's fetch is ordered after the stream that wrote it, a
    # non-blocking torch stream included (reduce-op.c:250-259 returns only
    # once the target holds the result; here the stream-ordered form returns
    # at once, and a host read of the target must still see the result).  On
    # one non-blocking stream: a long run of 256 MiB folds on other buffers,
    # then a fold that rewrites the source's HBM twin (source + 1), then
    # shmemx_double_sum_to_all_on_stream on the view addresses (PE_size 1: a
    # copy, reduce-op.c:213-216).  The host reads the target right away, with
    # no synchronisation: it must be source + 1 everywhere, and still be after
    # the stream completes.
    assert MIRRORED and npes == 1
    n = (32 << 20) // 8                      # 32 MiB target: 512 blocks (CAP is 48 MiB)
    big = (256 << 20) // 8
    srcs = oracle.sources("double", 1, 1, n, base_seed=0xA11)
    src, tgt = host_view(HEAP_SRC, np.float64, n), host_view(HEAP_TGT, np.float64, n)
    src[:] = srcs[0]                         # host stores (HOST_NEWER)
    tgt[:] = -1.0
    want = srcs[0] + 1.0
    stream = torch.cuda.Stream()
    x = torch.rand(big, dtype=torch.float64, device="cuda")
    y = torch.rand(big, dtype=torch.float64, device="cuda")
    ones = torch.ones(n, dtype=torch.float64, device="cuda")
    shm.mirror_sync(HEAP_SRC, n * 8)         # the host's source bytes in HBM
    torch.cuda.synchronize()
    shm.mirror_stats(reset=True)
    for rep in range(2):
        for _ in range(40):                  # ~5 ms of folds ahead of the call
            shm.fold("double", "sum", y, x, big, stream.cuda_stream)
        shm.fold("double", "sum", twin(HEAP_SRC), ones, n, stream.cuda_stream)   # source += 1 in HBM
        shm.reduce_on_stream("double", "sum", HEAP_TGT, HEAP_SRC, n, 0, 0, 1, "auto", stream.cuda_stream)
        ncases += 1
        early = tgt.copy()                   # faults: waits for the stream, fetches
        busy = not stream.query()            # (a sample only: the fetch has waited by now)
        stream.synchronize()
        late = tgt.copy()
        if not same_bits(early, want):
            fails.append(f"rep {rep}: host read right after the stream-ordered call: "
                         f"{int((early != want).sum())} elements differ")
        if not same_bits(late, want):
            fails.append(f"rep {rep}: host read after stream.synchronize(): "
                         f"{int((late != want).sum())} elements differ")
        extra.setdefault("stream_busy_after_read", []).append(busy)
        # next round: the source's twin was rewritten behind the view
        shm.mirror_invalidate(HEAP_SRC, n * 8)
        if not same_bits(src.copy(), want):   # (this fetch waits for the whole device)
            fails.append(f"rep {rep}: invalidated source view reads stale bytes")
        want = want + 1.0
    st = shm.mirror_stats(reset=True)
    extra["mirror_stats"] = st
    if not st["blocks_fetched"]:
        fails.append(f"no block was fetched: {st}")
elif scenario == "mixed":
    # Members passing different memory kinds: host arrays above 256 KiB go in
    # 16 MiB staging chunks (one collective call each), device arrays in one
    # call.  The members compare call counts first and all return ENOTSUP
    # (reduce-op.c:213-250: every PE runs one call sequence), and the job
    # goes on: matching calls right after are correct.  Small arrays (one
    # call either way) mix freely.
    import time
    for n in (4 * 1024 * 1024 + 3, 30000):
        srcs = oracle.sources("double", 1, npes, n, base_seed=0x31 + n)
        want = expected("double", "sum", srcs, (0, 0, npes), "auto")
        host = pe % 2 == 0
        src = srcs[pe].copy() if host else torch.from_numpy(srcs[pe].copy()).cuda()
        tgt = np.zeros(n) if host else torch.zeros(n, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        t0 = time.time()
        shm.to_all("double", "sum", tgt, src, n, 0, 0, npes)
        err = shm.last_error()
        ncases += 1
        big = n * 8 > 256 * 1024
        if big and (err != 3 or time.time() - t0 > 30):
            fails.append(f"mixed kinds n={n}: error {err} after {time.time() - t0:.1f} s, want ENOTSUP")
        got = tgt if host else tgt.cpu().numpy()
        if big and np.any(got != 0):
            fails.append(f"mixed kinds n={n}: target written despite ENOTSUP")
        if not big and (err or not matches(got, want, "double", "sum", srcs, (0, 0, npes),
                                           resolved("double", "sum", n, (0, 0, npes), "auto"))):
            fails.append(f"mixed kinds n={n} (one call either way): error {err} / wrong result")
        # the same call with matching kinds right after
        run_case("double", "sum", n, (0, 0, npes), "auto", "device", 0x77 + n)
elif scenario == "limits":
    # DIRECT members whose size limits differ: every member returns ENOTSUP
    # with its target untouched, the member that differed aligns at once, and
    # the next call is correct everywhere.  20 rounds back to back: the ENOTSUP
    # path ends with a barrier, so a member that retries at once
    # cannot overwrite its descriptor before a slower member has read it.
    import time
    default_kb = shm.set_fused_twoshot_kb(4096)
    shm.set_fused_twoshot_kb(default_kb)
    for rep in range(20):
        n = (100003, 7, 300001)[rep % 3]
        if pe == rep % npes:
            shm.set_fused_twoshot_kb(default_kb + 1024)
        srcs = oracle.sources("double", 1, npes, n, base_seed=0x11B0 + rep)
        s = to_dev(torch, np.ascontiguousarray(srcs[pe]))
        d = to_dev(torch, np.zeros(n))
        torch.cuda.synchronize()
        t0 = time.time()
        try:
            shm.reduce_on_stream("double", "sum", d, s, n, 0, 0, npes, "direct")
            err = 0
        except shm.ShmemError as e:
            err = e.code
        torch.cuda.synchronize()
        ncases += 1
        if err != 3 or time.time() - t0 > 30 or bool(d.abs().sum().item()):
            fails.append(f"limits rep {rep}: error {err} after {time.time() - t0:.1f} s, want ENOTSUP, "
                         "target untouched")
        if pe == rep % npes:
            shm.set_fused_twoshot_kb(default_kb)
        run_case("double", "sum", n, (0, 0, npes), "direct", "device", 0x11C0 + rep)
elif scenario == "big":
    # Arrays past 2 GiB per PE through the multi-PE paths.  The reference
    # computes its byte count as an int (reduce-op.c:180) and stops at 2 GiB;
    # every offset, shard, slice and count here is 64-bit.  long xor and long
    # sum (wrapping) over 2.5 GiB + 40 B per PE (an odd length: scalar tails
    # at the far end), on the heap, through each algorithm in $BIG_ALGOS;
    # against torch's fold of every PE's regenerated source (integer results:
    # any order is exact) on every element, 64 Ki sampled elements against
    # the oracle, and identical on every PE.
    n = (1 << 28) + (1 << 26) + 5
    nbytes = n * 8
    BIG_SRC, BIG_TGT = shm.malloc(nbytes), shm.malloc(nbytes)
    assert BIG_SRC and BIG_TGT, "shmem_malloc of the 2.5 GiB operands failed"

    def gen(q, salt):
        g = torch.Generator(device="cuda")
        g.manual_seed(0xB16 + 131 * q + salt)
        return torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)

    smp = torch.arange(0, n, n // 65536, device="cuda")
    smp = torch.cat([smp, torch.arange(n - 7, n, device="cuda")])   # the tail too
    salt = 0
    for op in ("xor", "sum"):
        for algo in os.environ.get("BIG_ALGOS", "auto").split(","):
            salt += 1
            ncases += 1
            print(f"big long {op} n={n} algo={algo}", flush=True)
            heap_write(BIG_SRC, gen(pe, salt), nbytes)
            heap_write(BIG_TGT, torch.zeros(n, dtype=torch.int64, device="cuda"), nbytes)
            torch.cuda.synchronize()
            shm.set_algo(algo)
            shm.to_all("long", op, BIG_TGT, BIG_SRC, n, 0, 0, npes)
            shm.set_algo("auto")
            if shm.last_error():
                fails.append(f"big {op} {algo}: last_error {shm.last_error()}")
                continue
            got = torch.empty(n, dtype=torch.int64, device="cuda")
            shm.memcpy(got, twin(BIG_TGT), nbytes)
            f = torch.bitwise_xor if op == "xor" else torch.add
            want = gen(0, salt)
            for q in range(1, npes):
                want = f(want, gen(q, salt))
            torch.cuda.synchronize()
            if not torch.equal(got, want):
                bad = int((got != want).sum())
                first = int((got != want).nonzero()[0])
                fails.append(f"big {op} {algo}: {bad} elements differ, the first at {first}")
            del want
            srcs = np.stack([gen(q, salt)[smp].cpu().numpy() for q in range(npes)])
            ref = oracle.reduce_sim("long", op, srcs, 0, 0, npes)[0]
            if not same_bits(got[smp].cpu().numpy(), ref):
                fails.append(f"big {op} {algo}: sampled elements differ from the oracle")
            del got
            if not shm.verify("long", BIG_TGT, n, 0, 0, npes):
                fails.append(f"big {op} {algo}: targets differ across PEs")
    extra["big_bytes_per_pe"] = nbytes
    shm.free(BIG_TGT)
    shm.free(BIG_SRC)
elif scenario == "ramp":
    # Run with $SHMEMX_STAGE_CHUNK_MB=1: host arrays of a few MiB take the
    # staging pipeline with its quarter / half chunks at both ends
    # (stage_plan.h), pageable and in place, odd lengths included, every
    # type width, on the world and a partial set; and pinned (page-locked)
    # arrays through the same schedule
    for t, op, n in (("double", "sum", (5 << 20) // 8 + 3), ("int", "xor", (6 << 20) // 4 + 1),
                     ("short", "max", (4 << 20) // 2 + 5), ("complexd", "sum", (3 << 20) // 16 + 1)):
        for mode in ("host", "hostinplace"):
            for st in ((0, 0, npes), (npes - 1, 0, 1)):
                seed += 1
                run_case(t, op, n, st, "auto", mode, seed)
    n = (5 << 20) // 8 + 7
    srcs = oracle.sources("long", 1, npes, n, base_seed=0x7A3)
    want = oracle.reduce_sim("long", "sum", srcs, 0, 0, npes)[pe]
    src = torch.from_numpy(srcs[pe].copy()).pin_memory()
    tgt = torch.zeros(n, dtype=torch.int64).pin_memory()
    shm.to_all("long", "sum", tgt, src, n, 0, 0, npes)
    ncases += 1
    if not np.array_equal(tgt.numpy(), want) or shm.last_error():
        fails.append("pinned long sum through the ramped staging pipeline wrong")
elif scenario == "heapcheck":
    # one world call on heap objects (segment or, when no PE has a segment,
    # private blocks alike on every PE), checked against the oracle
    n = 1000
    srcs = oracle.sources("long", 0, npes, n, base_seed=0x4EA9)
    want = oracle.reduce_sim("long", "sum", srcs, 0, 0, npes)[pe]
    private_host = MIRRORED and not shm.mirror_device_ptr(HEAP_SRC)   # page-locked private blocks
    if private_host:
        host_view(HEAP_SRC, np.int64, n)[:] = srcs[pe]
    else:
        heap_write(HEAP_SRC, srcs[pe], n * 8)
    shm.to_all("long", "sum", HEAP_TGT, HEAP_SRC, n, 0, 0, npes)
    got = host_view(HEAP_TGT, np.int64, n).copy() if private_host else read(HEAP_TGT, "long", n)
    extra["private_blocks"] = bool(private_host or not shm.heap_ptr(HEAP_SRC, pe))
    ncases += 1
    if not np.array_equal(got, want):
        fails.append("world long sum on heap objects wrong")
elif scenario == "threads":
    # Several host threads of one PE call the library at once (the reference
    # program's threads, each on its own arrays).  Workers make PE_size 1
    # calls on their own PE (reduce-op.c:213-216: a copy; no peer takes part,
    # so the PEs' call orders stay aligned) on host arrays (staging, small and
    # chunked), on torch tensors through the stream form on their own
    # non-blocking stream, and on their own 64 KiB-aligned mirrored heap
    # blocks (host stores, blocking call, host reads that fault and fetch on
    # the service thread); meanwhile the main thread runs world-set
    # collectives against the oracle.  Each worker first makes no device
    # current itself: the library binds the PE's device on the calling thread.
    import threading
    nthreads, iters = 4, int(os.environ.get("THREAD_ITERS", "25"))
    heap_n = (4096, 65536 + 7)               # a light-path call and a block-marking one
    blocks = []
    for _ in range(nthreads):                # shmem_malloc is collective: main thread, same order
        pair = []
        for n in heap_n:
            nb = (n * 8 + 65535) & ~65535
            pair.append((shm.align(65536, nb), shm.align(65536, nb)))
        blocks.append(pair)
    lock = threading.Lock()
    counts = [0] * nthreads

    def worker(w):
        rng = np.random.default_rng(0x7E + 31 * pe + w)
        stream = None
        try:
            for it in range(iters):
                # host arrays: one bounce-buffer call, and a chunked pageable one
                for n in (1000, 300001 if it % 5 == 0 else 20000):
                    src = rng.standard_normal(n)
                    tgt = np.full(n, np.nan)
                    shm.to_all("double", "sum", tgt, src, n, pe, 0, 1)
                    if not same_bits(tgt, src) or shm.last_error():
                        with lock:
                            fails.append(f"thread {w} it {it}: host n={n} wrong")
                # torch tensors on this thread's own stream
                if stream is None:
                    stream = torch.cuda.Stream(device=0)
                n = 50000 + w
                with torch.cuda.stream(stream):
                    s = torch.randint(-1000, 1000, (n,), dtype=torch.int64, device="cuda")
                    d = torch.zeros_like(s)
                shm.reduce_on_stream("long", "sum", d, s, n, pe, 0, 1, "auto", stream.cuda_stream)
                stream.synchronize()
                if not torch.equal(d, s):
                    with lock:
                        fails.append(f"thread {w} it {it}: stream form wrong")
                # mirrored heap view: host stores, the call, host loads
                if MIRRORED:
                    for (hs, ht), n in zip(blocks[w], heap_n):
                        want = rng.integers(-2**40, 2**40, n).astype(np.int64)
                        host_view(hs, np.int64, n)[:] = want
                        shm.to_all("longlong", "sum", ht, hs, n, pe, 0, 1)
                        got = host_view(ht, np.int64, n).copy()
                        if not np.array_equal(got, want) or shm.last_error():
                            with lock:
                                fails.append(f"thread {w} it {it}: heap n={n}: "
                                             f"{int((got != want).sum())} elements differ")
                counts[w] += 1
        except Exception as e:                # noqa: BLE001 — reported, not raised in a thread
            with lock:
                fails.append(f"thread {w}: {type(e).__name__}: {e}")

    threads = [threading.Thread(target=worker, args=(w,)) for w in range(nthreads)]
    for t in threads:
        t.start()
    srcs = oracle.sources("int", 0, npes, 1024, base_seed=0x7B00)
    want = oracle.reduce_sim("int", "sum", srcs, 0, 0, npes)[pe]
    src, tgt = host_view(HEAP_SRC, np.int32, 1024), host_view(HEAP_TGT, np.int32, 1024)
    main_calls = 0
    # a fixed count (every PE makes the same world calls), most of them while
    # the workers run
    for _ in range(int(os.environ.get("THREAD_MAIN_CALLS", "200"))):
        if MIRRORED:
            src[:] = srcs[pe]
            tgt[:] = 0
            shm.to_all("int", "sum", HEAP_TGT, HEAP_SRC, 1024, 0, 0, npes)
            got = tgt.copy()
        else:
            got = np.zeros(1024, np.int32)
            shm.to_all("int", "sum", got, srcs[pe].copy(), 1024, 0, 0, npes)
        if not np.array_equal(got, want):
            fails.append(f"main call {main_calls}: world int sum wrong")
        main_calls += 1
    extra["workers_alive_after_main"] = sum(t.is_alive() for t in threads)
    for t in threads:
        t.join()
    ncases = sum(counts) + main_calls
    extra["worker_iterations"] = counts
    extra["main_calls"] = main_calls
    if MIRRORED:
        extra["mirror_stats"] = shm.mirror_stats()
    for pair in blocks:
        for hs, ht in pair:
            shm.free(ht)
            shm.free(hs)
elif scenario == "signal_timeout":
    # one SIGNAL call together (maps and votes), then PE 0 calls again alone:
    # its device barrier must give up after $SHMEMX_SIGNAL_TIMEOUT seconds and
    # the blocking call abort with a FATAL line, not hang the GPU
    import time
    shm.set_algo("signal")
    shm.to_all("double", "sum", HEAP_TGT, HEAP_SRC, 64, 0, 0, npes)
    torch.cuda.synchronize()
    if pe == 0:
        t0 = time.time()
        print("calling alone", flush=True)
        shm.to_all("double", "sum", HEAP_TGT, HEAP_SRC, 64, 0, 0, npes)
        fails.append(f"returned after {time.time() - t0:.1f} s")
    else:
        time.sleep(8)            # keep the heap mapped while PE 0 waits
    with open(out_path, "w") as f:
        json.dump({"pe": pe, "fails": fails, "ncases": 1}, f)
    os._exit(0)
else:
    raise SystemExit(f"unknown scenario {scenario}")

# every system fence that handed data between PEs reached every XCD: none
# had to be run again (host paths) or failed its check (SIGNAL barrier)
stats = shm.direct_stats(reset=False)
fences = {k: stats[k] for k in shm.FENCE_STATS}
if fences["fence_refills_host"] or fences["fences_device_incomplete"]:
    fails.append(f"system fences missed an XCD: {fences}")
# small heap calls ran as one fused launch (DIRECT's and SIGNAL's one shot)
fences["fused_calls"] = stats["fused_calls"]
if (scenario in ("full", "signal") and npes > 1 and os.environ.get("SHMEMX_DIRECT_ONESHOT_KB") != "0"
        and os.environ.get("SHMEMX_FUSED_ONESHOT") != "0" and not stats["fused_calls"]):
    fails.append("no one-shot call ran as a fused launch")
if scenario == "ownorder" and npes > 1 and not stats["fused_calls"]:
    fails.append("no own-order one-shot call ran as a fused launch")
# and mid-size heap calls (100003 doubles; SIGNAL's 70001-element cases) as one
# fused two-shot launch
fences["fused_twoshot_calls"] = stats["fused_twoshot_calls"]
if (scenario in ("full", "signal") and npes > 1 and os.environ.get("SHMEMX_FUSED_TWOSHOT_KB") != "0"
        and not stats["fused_twoshot_calls"]):
    fails.append("no two-shot call ran as a fused launch")
shm.free(HEAP_TGT)
shm.free(HEAP_SRC)
shm.finalize()
with open(out_path, "w") as f:
    json.dump(dict(extra, pe=pe, fails=fails, ncases=ncases, fences=fences), f)
