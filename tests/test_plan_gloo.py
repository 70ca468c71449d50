"""Multi-PE path on CPU: world_size 2 and 4 over torch.distributed gloo.

Each rank asks the C library for its plan (shmemx_reduce_plan: algorithm,
member index, shard size, RCCL main/tail split) and then runs exactly the
exchange schedule runtime.cpp enqueues on RCCL, with gloo point-to-point
messages standing in for ncclSend/ncclRecv and the oracle folding the
received shards in the order the HIP kernel uses:

  A2A    shard i of every source -> member i; fold in active-set order;
         shard all-gather              -> must equal the reference PE_start
                                          result on every member, bit for bit
         (DIRECT and SIGNAL pull exactly these slices over xGMI instead)
  GATHER every source -> every member; fold me first, then ascending
                                       -> must equal the reference PE me
                                          result, bit for bit
         (float / double / long double min and max plan every algorithm
         this way: a2a turns into gather, DIRECT and SIGNAL read every
         member's whole source; kind 2 = NaN / +-0 sources on which PE k's
         reference answer differs from PE_start's)
  RCCL   main = P * chunk elements reduce-scattered (each shard folded in
         ring order, from member m + 1 round to m, as RCCL's ring does) +
         all-gathered, the tail all-reduced (descending member order)
                                  -> within the stated ULP bound of the
                                     reference (bit-exact for integers); on a
                                     partial set the same schedule runs on
                                     the set's members-only communicator

This proves the decomposition (plan + schedule) on CPU; the GPU tests prove
the fold kernel, and RCCL moves the bytes.
"""
import multiprocessing as mp
import os
import socket
import sys
import traceback

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    # (type, op, kind, n, set, algo)
    ("double", "sum", 0, 1000, None, "a2a"),
    ("double", "sum", 0, 4103, None, "gather"),
    ("double", "sum", 0, 4103, None, "rccl"),
    ("int", "sum", 1, 4103, None, "rccl"),
    ("double", "sum", 0, 4103, None, "auto"),    # small: one all-reduce
    ("long", "max", 1, 1001, None, "allreduce"),
    ("float", "prod", 0, 0, None, "allreduce"),
    ("double", "prod", 0, 4103, None, "rccl"),
    ("float", "prod", 0, 1001, None, "allreduce"),
    ("float", "sum", 1, 4099, None, "rccl"),     # mixed signs, ragged tail
    ("long", "xor", 1, 777, None, "auto"),
    ("long", "and", 1, 65, None, "a2a"),
    ("short", "max", 1, 130, None, "auto"),
    ("float", "min", 1, 1001, None, "auto"),
    ("complexd", "prod", 0, 99, None, "a2a"),
    ("complexf", "sum", 1, 5, None, "gather"),
    ("double", "prod", 0, 3, None, "a2a"),     # fewer elements than PEs
    ("double", "sum", 0, 0, None, "a2a"),      # nreduce = 0
    ("int", "min", 1, 300, "strided", "auto"),   # partial sets: A2A under auto
    ("int", "min", 1, 300, "strided", "allreduce"),   # ... RCCL on their own communicator when named
    ("double", "sum", 0, 300, "offset", "auto"),
    ("double", "sum", 1, 4103, "strided", "rccl"),
    ("float", "sum", 1, 4099, "offset", "rccl"),
    ("float", "prod", 1, 1001, "offset", "allreduce"),
    ("long", "max", 1, 999, "offset", "rccl"),
    ("long", "xor", 1, 999, "offset", "auto"),      # no RCCL op: A2A still
    # DIRECT / SIGNAL pull the same slices A2A exchanges (slice m of every
    # source -> member m, fold in set order, slices gathered back)
    ("double", "sum", 0, 4103, None, "direct"),
    ("long", "xor", 1, 1001, "strided", "signal"),
    ("float", "max", 1, 3, None, "signal"),      # fewer elements than PEs
    ("int", "prod", 1, 0, None, "direct"),
    ("longdouble", "sum", 0, 257, "offset", "signal"),
    # min / max of float, double, long double on NaN / +-0 inputs (kind 2):
    # each member's own reference answer under every algorithm
    ("float", "min", 2, 1001, None, "auto"),
    ("double", "max", 2, 777, "offset", "a2a"),
    ("longdouble", "min", 2, 129, "strided", "direct"),
    ("float", "max", 2, 300, None, "signal"),
    ("double", "min", 2, 65, None, "gather"),
    ("longdouble", "max", 2, 1000, None, "auto"),
]
OWN_ORDER = {(t, o) for t in ("float", "double", "longdouble") for o in ("min", "max")}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _set_for(kind, world):
    if kind is None:
        return (0, 0, world)
    if kind == "strided":
        return (0, 1, world // 2) if world >= 4 else (1, 0, 1)
    return (1, 0, world - 1)  # offset


def _send(dist, arr, dst):
    import torch
    dist.send(torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy()), dst)


def _recv(dist, nbytes, src):
    import torch
    t = torch.empty(nbytes, dtype=torch.uint8)
    dist.recv(t, src)
    return t.numpy()


def _exchange(dist, me, sends, recvs):
    """sends: {peer: array}, recvs: {peer: nbytes}; lower rank sends first."""
    got = {}
    for peer in sorted(set(sends) | set(recvs)):
        if me < peer:
            if peer in sends:
                _send(dist, sends[peer], peer)
            if peer in recvs:
                got[peer] = _recv(dist, recvs[peer], peer)
        else:
            if peer in recvs:
                got[peer] = _recv(dist, recvs[peer], peer)
            if peer in sends:
                _send(dist, sends[peer], peer)
    return got


def _bits(a, t):
    """Value bytes (long double: the 10 bytes of the x87 value, not the
    slot's padding, which the oracle leaves unspecified as C does)."""
    if t == "longdouble":
        return a.view(np.uint8).reshape(len(a), -1)[:, :10].tobytes()
    return a.tobytes()


def _run_case(dist, shm, oracle, rank, world, case):
    t, op, kind, n, setkind, algo = case
    s = _set_for(setkind, world)
    members = [s[0] + i * (1 << s[1]) for i in range(s[2])]
    if kind == 2:
        srcs = oracle.special_sources(t, world, n, 0x5EED0000 + n)
    else:
        srcs = oracle.sources(t, kind, world, n, base_seed=0x5EED0000 + n)
    want = oracle.reduce_sim(t, op, srcs, *s)
    own = (t, op) in OWN_ORDER and len(members) > 1
    if kind == 2 and len(members) > 1:
        # the inputs discriminate: some member's reference answer differs
        # from PE_start's, so a shared result would fail this case
        assert any(_bits(want[q], t) != _bits(want[members[0]], t) for q in members), case
    if rank not in members:
        with pytest.raises(shm.ShmemError):
            shm.plan(t, op, n, *s, rank, world, algo)
        return
    p = shm.plan(t, op, n, *s, rank, world, algo)
    P, m, dt = p.nmembers, p.member, srcs.dtype
    src = srcs[rank]
    out = np.zeros(n, dtype=dt)
    if P == 1:
        out[:] = src
    elif p.algo in ("a2a", "direct", "signal") and not own:
        c = p.chunk
        cnt = [max(0, min(c, n - i * c)) for i in range(P)]
        lo = m * c
        sends = {members[i]: src[i * c:i * c + cnt[i]] for i in range(P) if i != m and cnt[i]}
        recvs = {members[i]: cnt[m] * dt.itemsize for i in range(P) if i != m and cnt[m]}
        got = _exchange(dist, rank, sends, recvs)
        if cnt[m]:
            shards = np.stack([src[lo:lo + cnt[m]] if i == m else
                               got[members[i]].view(dt) for i in range(P)])
            out[lo:lo + cnt[m]] = oracle.reduce_sim(t, op, shards, 0, 0, P)[0]
        sends = {members[i]: out[lo:lo + cnt[m]] for i in range(P) if i != m and cnt[m]}
        recvs = {members[i]: cnt[i] * dt.itemsize for i in range(P) if i != m and cnt[i]}
        got = _exchange(dist, rank, sends, recvs)
        for i in range(P):
            if i != m and cnt[i]:
                out[i * c:i * c + cnt[i]] = got[members[i]].view(dt)
        assert _bits(out, t) == _bits(want[members[0]], t), case
    elif p.algo == "gather" or own:
        assert p.algo != "a2a", case
        sends = {members[i]: src for i in range(P) if i != m}
        recvs = {members[i]: n * dt.itemsize for i in range(P) if i != m}
        got = _exchange(dist, rank, sends, recvs) if n else {}
        full = np.stack([src if i == m else got[members[i]].view(dt) for i in range(P)]) \
            if n else np.zeros((P, 0), dt)
        out = oracle.reduce_sim(t, op, full, 0, 0, P)[m]
        assert _bits(out, t) == _bits(want[rank], t), case
    elif p.algo == "allreduce":
        # one all-reduce: every member gets the whole reduction, in RCCL's
        # order (here: descending member order, unlike the reference's)
        assert p.chunk == n and p.main == n and p.tail == 0
        sends = {members[i]: src for i in range(P) if i != m}
        recvs = {members[i]: n * dt.itemsize for i in range(P) if i != m}
        got = _exchange(dist, rank, sends, recvs) if n else {}
        full = np.stack([src if i == m else got[members[i]].view(dt) for i in range(P)][::-1]) \
            if n else np.zeros((P, 0), dt)
        out = oracle.reduce_sim(t, op, full, 0, 0, P)[0]
        _check_rccl(out, want[rank], srcs[members], dt, case, op)
    else:  # rccl: reduce-scatter main part, all-gather, all-reduce tail
        c, main = p.chunk, p.main
        assert main + p.tail == n
        if c:
            sends = {members[i]: src[i * c:(i + 1) * c] for i in range(P) if i != m}
            recvs = {members[i]: c * dt.itemsize for i in range(P) if i != m}
            got = _exchange(dist, rank, sends, recvs)
            shards = [src[m * c:(m + 1) * c] if i == m else got[members[i]].view(dt) for i in range(P)]
            ring = [(m + 1 + k) % P for k in range(P)]       # RCCL's ring order, not PE_start's
            out[m * c:(m + 1) * c] = oracle.reduce_sim(t, op, np.stack([shards[i] for i in ring]),
                                                       0, 0, P)[0]
            sends = {members[i]: out[m * c:(m + 1) * c] for i in range(P) if i != m}
            got = _exchange(dist, rank, sends, recvs)
            for i in range(P):
                if i != m:
                    out[i * c:(i + 1) * c] = got[members[i]].view(dt)
        if p.tail:
            sends = {members[i]: src[main:] for i in range(P) if i != m}
            recvs = {members[i]: p.tail * dt.itemsize for i in range(P) if i != m}
            got = _exchange(dist, rank, sends, recvs)
            tails = np.stack([src[main:] if i == m else got[members[i]].view(dt)
                              for i in range(P)][::-1])
            out[main:] = oracle.reduce_sim(t, op, tails, 0, 0, P)[0]
        _check_rccl(out, want[rank], srcs[members], dt, case, op)


def _check_rccl(out, want, member_srcs, dt, case, op):
    """RCCL's reduction order is not the reference's: integers (and min /
    max) bit-exact; floating sum within 2 gamma(P-1) sum_p |x_p| and floating
    prod within 2 gamma(P-1) |prod_p x_p| (BASELINE north_star; the same
    check the GPU tests make, tests/gpu_util.py order_bound)."""
    from gpu_util import order_bound
    ok, _ = order_bound(out.astype(dt), want, member_srcs, op)
    assert ok, case


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import torch.distributed as dist
        import oracle
        import shmem_mi355x as shm
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}",
                                rank=rank, world_size=world)
        for case in CASES:
            _run_case(dist, shm, oracle, rank, world, case)
            dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 4])
def test_multi_pe_schedule_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, msg = q.get(timeout=600)
        results[r] = msg
    for p in procs:
        p.join(timeout=60)
    bad = {r: m for r, m in results.items() if m != "ok"}
    assert not bad, "\n".join(f"rank {r}:\n{m}" for r, m in bad.items())
