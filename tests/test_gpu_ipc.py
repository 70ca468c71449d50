"""Multi-process reductions on one GPU over the IPC transport (DIRECT and
own-order GATHER), checked against the oracle restatement of reduce-op.c.

P processes (one PE each) share the box's GPU; with $SHMEMX_TRANSPORT=ipc the
library starts no RCCL communicator (RCCL refuses two ranks on one device),
so everything that crosses PEs — the symmetric heap's IPC mappings, the
DIRECT kernels that read and write the other PEs' HBM, the host barrier over
the node block, staging through the IPC scratch — runs for real across
processes.  See tests/gpu_ipc_child.py for the cases.
"""
import json
import os
import signal
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def start_pes(tmp_path, npes, scenario, extra_env=None):
    boot = str(tmp_path / "uid")
    # $GPU_TEST_LOGDIR: keep the PEs' logs (one line per case) where the GPU
    # box hands files back, under a directory per test
    logdir = os.environ.get("GPU_TEST_LOGDIR")
    if logdir:
        test = os.environ.get("PYTEST_CURRENT_TEST", scenario).split(" ")[0]
        logdir = os.path.join(logdir, "".join(c if c.isalnum() or c in "-_." else "_" for c in test))
        os.makedirs(logdir, exist_ok=True)
    procs = []
    for pe in range(npes):
        env = dict(os.environ, SHMEM_PE=str(pe), SHMEM_NPES=str(npes), LOCAL_RANK="0",
                   SHMEM_BOOTSTRAP_FILE=boot, SHMEMX_TRANSPORT="ipc",
                   SHMEMX_BARRIER_TIMEOUT="120")
        # All PEs share one GPU here, each process with its own hardware
        # queues: 8 PEs x 4 queues (the box's GPU_MAX_HW_QUEUES) plus the test
        # runner's own oversubscribe the GPU's queue slots, and every copy and
        # sync then waits its queue's turn (8-PE tests crawled, minutes per
        # case, in the full suite only).  Two queues per PE keep the total
        # well inside.
        if npes > 4:
            env["GPU_MAX_HW_QUEUES"] = "2"
        env.pop("RANK", None)
        env.pop("WORLD_SIZE", None)
        for k, v in (extra_env or {}).items():   # None: unset; "PE<p>:VAR" for PE p only
            if ":" in k:
                who, k = k.split(":", 1)
                if who != f"PE{pe}":
                    continue
            if v is None:
                env.pop(k, None)
            else:
                env[k] = v
        out = str(tmp_path / f"pe{pe}.json")
        log = open(os.path.join(logdir, f"pe{pe}.log") if logdir else tmp_path / f"pe{pe}.log", "w")
        procs.append((subprocess.Popen([sys.executable, os.path.join(HERE, "gpu_ipc_child.py"), out,
                                        scenario], env=env, stdout=log, stderr=subprocess.STDOUT,
                                       start_new_session=True), out, log))
    return procs


def wait_pes(procs, timeout):
    """Exit codes and log texts of every PE (killing stragglers)."""
    try:
        rcs = [p.wait(timeout=timeout) for p, _, _ in procs]
    finally:
        for p, _, _ in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    logs = []
    for _, _, log in procs:
        log.close()
        logs.append(open(log.name).read())
    return rcs, logs


def run_pes(tmp_path, npes, scenario, extra_env=None, timeout=900):
    procs = start_pes(tmp_path, npes, scenario, extra_env)
    rcs, logs = wait_pes(procs, timeout)
    if any(rcs):
        raise AssertionError("\n".join(f"--- PE {pe} exit {rc}:\n" + log[-1500:]
                                       for pe, (rc, log) in enumerate(zip(rcs, logs))))
    reports = []
    for _, out, _ in procs:
        with open(out) as f:
            reports.append(json.load(f))
    return reports


def fences_checked(reports, device=False):
    """Every PE ran system fences and each reached every XCD the first time
    (the child fails a PE whose fence needed a refill or failed its check)."""
    key = "fences_device" if device else "fences_host"
    for r in reports:
        assert r["fences"][key] > 0, f"PE {r['pe']}: no {key}: {r['fences']}"
        assert r["fences"]["fence_refills_host"] == 0 and r["fences"]["fences_device_incomplete"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2, 4, 8])
@pytest.mark.parametrize("shots", ["auto", "two"])
def test_ipc_transport_all_pairs_sets_placements(tmp_path, npes, shots):
    # "auto": arrays up to 256 KiB take DIRECT's one-shot path; "two": every
    # size takes reduce-scatter + all-gather
    env = {"SHMEMX_DIRECT_ONESHOT_KB": "0"} if shots == "two" else {}
    reports = run_pes(tmp_path, npes, "full", env)
    assert sorted(r["pe"] for r in reports) == list(range(npes))
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
    fences_checked(reports)


@pytest.mark.gpu
@pytest.mark.parametrize("schedule", ["fused-one", "fused-two", "unfused-two"])
def test_ipc_reference_element_ops_two_pes(tmp_path, schedule):
    """DIRECT, SIGNAL and own-order GATHER across 2 PE processes against the
    reference's own compiled element ops (tests/golden/ref_element_ops.json,
    reduce-op.c:71-150): all 44 pairs on special values and random bits, PE 0
    holding a and PE 1 b, through the fused one-shot launch, the fused
    two-shot launch, and the multi-launch two shot (peers fold + gather)."""
    env = {"fused-one": {},
           "fused-two": {"SHMEMX_DIRECT_ONESHOT_KB": "0"},
           "unfused-two": {"SHMEMX_DIRECT_ONESHOT_KB": "0", "SHMEMX_FUSED_TWOSHOT_KB": "0",
                           "SHMEMX_FUSED_ONESHOT": "0"}}[schedule]
    reports = run_pes(tmp_path, 2, "refops", env, timeout=600)
    for r in reports:
        assert r["ncases"] == 44 * 3
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
    fences_checked(reports)
    if schedule == "fused-one":
        assert all(r["fences"]["fused_calls"] > 0 for r in reports)
    elif schedule == "fused-two":
        assert all(r["fences"]["fused_twoshot_calls"] > 0 for r in reports)
    else:
        assert all(r["fences"]["fused_calls"] == 0 and r["fences"]["fused_twoshot_calls"] == 0
                   for r in reports)


@pytest.mark.gpu
@pytest.mark.parametrize("transport,npes", [("ipc", 2), ("ipc", 3), ("ipc", 8), ("rccl", 2), ("rccl", 3),
                                            ("rccl", 8)])
def test_own_order_min_max_on_nan_and_signed_zeros(tmp_path, transport, npes):
    """min / max of float, double and long double on NaN / +-0 sources
    (oracle.special_sources), where a<b?a:b gives PE k a different answer
    from PE_start's (reduce-op.c:130-142, 219-248): every PE gets its OWN
    reference result under auto and every explicit algorithm of the
    transport, every active set, fused one-shot and larger sizes, heap,
    in-place and device operands (the RCCL transport on the RCCL test
    double).  The inputs discriminate: the PEs' reference answers differ
    from PE_start's on many elements, so a schedule that hands every member
    PE_start's result fails here."""
    env = {"SHMEMX_TRANSPORT": transport, "SHMEMX_HEAP_MEMORY": "device"}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    reports = run_pes(tmp_path, npes, "ownorder", env)
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
    assert sum(r["own_order_differs"] for r in reports) > 1000
    # PE_start itself folds in set order; every other PE differs somewhere
    assert all(r["own_order_differs"] > 0 for r in reports if r["pe"] > 0)


@pytest.mark.gpu
@pytest.mark.parametrize("transport,npes,heap", [("ipc", 2, "device"), ("ipc", 3, "mirrored"), ("ipc", 8, "device"),
                                                 ("rccl", 3, "device")])
def test_small_multi_pe_calls_through_the_service_exchange(tmp_path, transport, npes, heap):
    """Blocking calls of at most 4 KiB per PE over several PEs under auto:
    each member leaves its source in the job's page-locked exchange, passes
    the entry barrier, its resident service workgroup folds every member's
    slot into its target, then the exit barrier (reduce-op.c:217-250's
    barrier, gets, barrier, with no kernel launch).  Every reference pair at
    1 element, at the limit and one past it, every active set, heap / host /
    in-place operands, own-order pairs on NaN / +-0 sources; every PE against
    the oracle (its own order where that decides the answer, else
    PE_start's), and the folds are counted, so the path is the one that ran."""
    # (SHMEMX_SERVICE=1: the PE processes share the one GPU here, where the
    # service workgroup is otherwise off)
    env = {"SHMEMX_TRANSPORT": transport, "SHMEMX_HEAP_MEMORY": heap, "SHMEMX_SERVICE": "1"}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    reports = run_pes(tmp_path, npes, "xchg", env, timeout=300)
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
        assert r["folds"] > 0
    print("configs[0] call from C, us per PE:", [r.get("config0_c_us") for r in reports if r["pe"] < 2])


@pytest.mark.gpu
@pytest.mark.parametrize("transport,heap", [("ipc", "device"), ("ipc", "mirrored"), ("rccl", "device")])
def test_baseline_config0_int_sum_1024_two_pes(tmp_path, transport, heap):
    """BASELINE.json configs[0]: shmem_int_sum_to_all, nreduce = 1024, 2 PEs,
    as 2 PE processes through the C entry point on the HIP path (DIRECT's
    fused one shot on the IPC transport; RCCL's all-reduce on the RCCL
    transport, with the RCCL test double), from heap, device and host arrays
    and, on the mirrored heap, host-written view addresses.  Every PE's
    target is held bit for bit against oracle_reduce_fork: the restated
    reduce-op.c run as one forked process per PE over shared segments (the
    GASNet smp loopback the reference's oshrun uses), on the same sources."""
    import oracle
    env = {"SHMEMX_TRANSPORT": transport, "SHMEMX_HEAP_MEMORY": heap}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    npes, n = 2, 1024
    _, want = oracle.reduce_fork("int", "sum", npes, 0, 0, npes, n, kind=0, reps=1)
    reports = run_pes(tmp_path, npes, "config0", env, timeout=300)
    for r in reports:
        assert not r["fails"], f"PE {r['pe']}: {r['fails']}"
        modes = ("view", "host") if heap == "mirrored" else ("heap", "device", "host")
        assert r["ncases"] == len(modes)
        assert r["target_hash"] == {m: want[r["pe"]] for m in modes}, (r["target_hash"], want)
        # the GPU path ran: DIRECT's pulls on the IPC transport, RCCL's all-reduce on RCCL
        assert set(r["algo"].values()) == {"direct" if transport == "ipc" else "allreduce"}, r["algo"]


@pytest.mark.gpu
@pytest.mark.parametrize("table", ["set", "bad"])
def test_auto_table_from_environment(tmp_path, table):
    """`auto`'s per-size choice read from $SHMEMX_AUTO_FULL /
    $SHMEMX_AUTO_PARTIAL (the values the N > 1 bench prints as
    extras.auto_recommendation.env), on 4 PE processes over the RCCL
    transport with the RCCL test double: the plan each size resolves to, a
    cut RCCL cannot serve (long xor) falling back to the built-in rule, and
    every call bit-exact against the oracle.  "bad": an unparsable value
    leaves the built-in rule alone."""
    fake = os.path.join(HERE, "native", "libfake_rccl.so")
    KiB = 1024
    if table == "set":
        env = {"SHMEMX_AUTO_FULL": f"0:gather,{4 * KiB}:a2a,{64 * KiB}:rccl",
               "SHMEMX_AUTO_PARTIAL": "0:direct"}
        expect = [["double", "sum", 16, 0, 0, 4, "gather"],          # 128 B
                  ["double", "sum", 1024, 0, 0, 4, "a2a"],           # 8 KiB
                  ["double", "sum", 65536, 0, 0, 4, "rccl"],         # 512 KiB
                  ["long", "xor", 65536, 0, 0, 4, "a2a"],            # no RCCL op: built-in rule
                  ["int", "max", 3000, 0, 0, 4, "a2a"],
                  ["double", "sum", 4099, 0, 1, 2, "direct"],        # every other PE
                  ["float", "min", 777, 1, 0, 3, "direct"]]
    else:
        env = {"SHMEMX_AUTO_FULL": "fast please", "SHMEMX_AUTO_PARTIAL": "0:signal"}
        expect = [["double", "sum", 16, 0, 0, 4, "allreduce"],
                  ["double", "sum", 1 << 20, 0, 0, 4, "rccl"],
                  ["long", "xor", 4096, 0, 0, 4, "a2a"],
                  ["float", "max", 4099, 0, 0, 4, "gather"],       # each PE's own order
                  # a partial set: A2A (its own RCCL communicator only when named)
                  ["double", "sum", 4099, 0, 1, 2, "a2a"],
                  ["double", "sum", 1 << 20, 1, 0, 3, "a2a"],
                  ["long", "xor", 4099, 1, 0, 3, "a2a"]]
    env.update({"SHMEMX_TRANSPORT": "rccl", "FAKE_RCCL": fake, "AUTO_EXPECT": json.dumps(expect)})
    reports = run_pes(tmp_path, 4, "autotable", env, timeout=300)
    for r in reports:
        assert not r["fails"], f"PE {r['pe']}: {r['fails']}"
        assert r["ncases"] > 0


@pytest.mark.gpu
def test_ipc_eight_pe_baseline_configs(tmp_path):
    """BASELINE.json configs[2] (double sum, 32 Mi, 8 PEs) on DIRECT, SIGNAL
    and own-order GATHER, and configs[4] (float sum sweep 4 Ki .. 256 Mi, 8
    PEs), as 8 PE processes sharing the GPU through the blocking drop-in entry
    points: bit-exact against torch's fold of the regenerated sources in the
    reference's order, identical across PEs, every fence on every XCD; and
    against the oracle restatement itself on every element of every case up
    to 256 MiB per PE (configs[2] whole), 64 Ki samples of the 1 GiB one."""
    reports = run_pes(tmp_path, 8, "configs8", timeout=900)
    for r in reports:
        assert r["ncases"] == 14
        assert not r["fails"], f"PE {r['pe']}: {r['fails']}"
        assert r["oracle_full_elements"] == 3 * (32 << 20) + sum(4096 * 4 ** k for k in range(8)) + (16 << 20) + 5 \
            + 4096 + 3, r.get("oracle_full_elements")
    fences_checked(reports)
    fences_checked(reports, device=True)


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2, 3, 4, 8])
def test_rccl_transport_with_rccl_double(tmp_path, npes):
    """The default RCCL transport across PE processes on the one GPU, with
    the RCCL test double (tests/native/fake_rccl.cpp) in place of librccl:
    every reference pair on every active set through AUTO, RCCL (reduce-
    scatter + all-gather + all-reduce tail), ALLREDUCE, A2A and GATHER, heap /
    device / host / in-place / overlapping operands, sizes across the
    all-reduce threshold, and broadcast, [f]collect, barrier and verify over
    RCCL — all against the oracle: bit for bit, except float sum / prod
    through RCCL's collectives, which the double folds in ring order (not
    PE_start's) and which must lie within the stated ULP bound.  Partial sets
    take A2A under auto and RCCL's collectives on their members-only
    communicators when named."""
    fake = os.path.join(HERE, "native", "libfake_rccl.so")
    assert os.path.exists(fake), "tests/native/libfake_rccl.so not built (make -C tests/native)"
    # at 3 PEs with the heap segment registered with RCCL at its first
    # allocation (SHMEMX_RCCL_REGISTER=1): the same results
    reports = run_pes(tmp_path, npes, "rccl", {"SHMEMX_TRANSPORT": "rccl", "FAKE_RCCL": fake,
                                               "SHMEMX_RCCL_REGISTER": "1" if npes == 3 else "0"},
                      timeout=600)
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
    if npes >= 3:
        # the double's order is not PE_start's: some float results differ in bits
        assert sum(r["rccl_inexact_elements"] for r in reports) > 0


@pytest.mark.gpu
def test_rccl_transport_without_set_comms(tmp_path):
    """$SHMEMX_SET_COMMS=0: partial sets keep the grouped send/recv schedules
    on the world communicator (no set communicator is made, auto takes A2A
    there, an explicit rccl on a partial set is refused), every case still
    against the oracle (4 PE processes, RCCL test double)."""
    fake = os.path.join(HERE, "native", "libfake_rccl.so")
    reports = run_pes(tmp_path, 4, "rccl", {"SHMEMX_TRANSPORT": "rccl", "FAKE_RCCL": fake,
                                           "SHMEMX_SET_COMMS": "0"}, timeout=600)
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
        assert r["set_comms"] == 0, r["set_comms"]


@pytest.mark.gpu
@pytest.mark.parametrize("cap", ["1", "0"])
def test_set_comms_cap(tmp_path, cap):
    """$SHMEMX_SET_COMMS_MAX: no PE holds more set communicators than the cap;
    a set whose members do not all have room keeps the world communicator
    (auto plans A2A there), agreed among its members so none waits for a
    communicator the others are not building; every call against the oracle
    (4 PE processes, RCCL test double)."""
    fake = os.path.join(HERE, "native", "libfake_rccl.so")
    # auto takes a partial set's communicator only when the table asks for it
    reports = run_pes(tmp_path, 4, "setcap", {"SHMEMX_TRANSPORT": "rccl", "FAKE_RCCL": fake,
                                             "SHMEMX_SET_COMMS_MAX": cap,
                                             "SHMEMX_AUTO_PARTIAL": "0:allreduce,4194304:rccl"}, timeout=300)
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
        assert r["set_comms"] <= int(cap), r["set_comms"]
    if cap == "1":
        assert any(r["set_comms"] == 1 for r in reports)


@pytest.mark.gpu
@pytest.mark.parametrize("npes,scale", [(4, "1"), (8, "1"), (4, "0")])
def test_rccl_order_within_bound(tmp_path, npes, scale):
    """Float sum and prod through RCCL's reduce-scatter + all-gather and
    all-reduce, on the whole job and on every partial set's members-only
    communicator, with the RCCL test double folding in ring / rotated order
    (as RCCL does): within |d| <= 2 gamma(P-1) sum|x| (sum) / 2 gamma(P-1)
    |prod x| (prod) of the reference's PE_start fold (reduce-op.c:219-248),
    with results that really differ in bits.  scale "0": the negative control
    (bound 0) must fail on float sums, which proves the bound is what passes
    them."""
    fake = os.path.join(HERE, "native", "libfake_rccl.so")
    env = {"SHMEMX_TRANSPORT": "rccl", "FAKE_RCCL": fake, "RCCL_TOL_SCALE": scale}
    reports = run_pes(tmp_path, npes, "rccl_order", env, timeout=600)
    partial = 6 if npes == 8 else 3          # active_sets() with more than one member, minus the world
    for r in reports:
        assert r["ncases"] > 0
        # every partial set this PE belongs to has its own communicator
        assert r["set_comms"] >= 1 and r["set_comms"] <= partial + 2, r["set_comms"]
    inexact = sum(r["rccl_inexact_elements"] for r in reports)
    assert inexact > 0
    if scale == "0":
        bad = [f for r in reports for f in r["fails"]]
        assert any(" sum " in f and ("double" in f or "float" in f) for f in bad), bad[:5]
    else:
        for r in reports:
            assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"


@pytest.mark.gpu
@pytest.mark.parametrize("transport,npes,heap", [("ipc", 3, "device"), ("rccl", 4, "device"), ("ipc", 8, "device"),
                                                ("rccl", 8, "device"), ("ipc", 3, "mirrored"),
                                                ("rccl", 4, "mirrored"), ("ipc", 8, "mirrored")])
def test_soak_random_calls(tmp_path, transport, npes, heap):
    """Random collective calls, the same seeded sequence on every PE: any
    reference pair, size (edges favoured), active set, algorithm the transport
    offers and operand placement, each against the oracle.  The RCCL
    transport runs on the RCCL test double.  On the mirrored heap the draw
    also includes blocking calls on host-view operands the host writes and
    reads.  $SOAK_ITERS / $SOAK_SEED make longer or different runs."""
    env = {"SHMEMX_TRANSPORT": transport, "SOAK_ITERS": os.environ.get("SOAK_ITERS", "60"),
           "SOAK_SEED": os.environ.get("SOAK_SEED", "7"), "SHMEMX_HEAP_MEMORY": heap}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    reports = run_pes(tmp_path, npes, "soak", env, timeout=900)
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"


@pytest.mark.gpu
def test_ipc_baseline_configs_full_size(tmp_path):
    """BASELINE.json configs[3] (long and/or/xor, 64 Mi, 4 PEs) and configs[2]'s
    double sum over 32 Mi, as 4 PE processes through the blocking drop-in
    entry points: bit-exact against torch's fold of all regenerated sources in
    PE_start order and against the oracle restatement on every element, and
    identical on every PE."""
    reports = run_pes(tmp_path, 4, "configs", timeout=600)
    for r in reports:
        assert r["ncases"] == 4
        assert not r["fails"], f"PE {r['pe']}: {r['fails']}"
        assert r["oracle_full_elements"] == 3 * (64 << 20) + (32 << 20), r.get("oracle_full_elements")


@pytest.mark.gpu
@pytest.mark.parametrize("transport,algos", [("ipc", "auto,signal,gather"), ("rccl", "auto,gather")])
def test_beyond_2gib_per_pe_multi_pe(tmp_path, transport, algos):
    """2.5 GiB per PE (past the reference's int byte count, reduce-op.c:180)
    through the multi-PE paths, 2 PE processes: DIRECT (auto on IPC), SIGNAL
    and GATHER over IPC; A2A (auto for xor) and RCCL reduce-scatter +
    all-gather (auto for sum) and GATHER over the RCCL test double.  Every
    element checked, identical on both PEs."""
    env = {"SHMEMX_TRANSPORT": transport, "SHMEM_SYMMETRIC_HEAP_SIZE": "8G", "BIG_ALGOS": algos,
           "SHMEMX_HEAP_MEMORY": "device"}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    reports = run_pes(tmp_path, 2, "big", env, timeout=600)
    for r in reports:
        assert r["ncases"] == 2 * len(algos.split(","))
        assert not r["fails"], f"PE {r['pe']}: {r['fails']}"
        assert r["big_bytes_per_pe"] > 2 << 30


@pytest.mark.gpu
def test_ipc_direct_staged_in_chunks(tmp_path):
    # a 1 MiB scratch: every staged operand crosses several chunks per call
    reports = run_pes(tmp_path, 3, "chunk", {"SHMEMX_DIRECT_SCRATCH_MB": "1"})
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"


@pytest.mark.gpu
@pytest.mark.parametrize("heap", ["static", "mirrored"])
def test_isx_c_program_four_pes(tmp_path, heap):
    """The C99 ISx verification program (examples/isx_verify.c: the
    reference's known-answer check, isx.c:615-624) as four PE processes,
    shmem_init bootstrapping through a file.  "static": static host arrays,
    as ISx has them.  "mirrored": the arrays are shmem_malloc'd and written
    by host code on a $SHMEMX_HEAP_MEMORY=mirrored heap; the reduction trace
    shows every call running on HBM (DIRECT, or the service exchange for the
    small ones; device pointers, no staging) and
    the mirror moved the touched blocks both ways."""
    repo = os.path.dirname(HERE)
    libdir = os.path.join(repo, "openshmem-async_amd")
    exe = tmp_path / "isx_verify"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(repo, "include"),
                    os.path.join(repo, "examples", "isx_verify.c"), "-L", libdir,
                    "-lshmem_reduce_mi355x", f"-Wl,-rpath,{libdir}", "-o", str(exe)], check=True)
    npes, procs = 4, []
    for pe in range(npes):
        env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE")}
        env.update(SHMEM_PE=str(pe), SHMEM_NPES=str(npes), LOCAL_RANK="0",
                   SHMEM_BOOTSTRAP_FILE=str(tmp_path / "uid"), SHMEMX_TRANSPORT="ipc",
                   SHMEMX_BARRIER_TIMEOUT="120")
        if heap == "mirrored":
            env.update(ISX_SHMEM_MALLOC="1", SHMEMX_HEAP_MEMORY="mirrored",
                       SHMEM_LOG_LEVELS="reduction", SHMEM_LOG_FILE=str(tmp_path / f"trace{pe}.log"))
        procs.append(subprocess.Popen([str(exe)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True, start_new_session=True))
    try:
        outs = [p.communicate(timeout=300)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    for pe, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"PE {pe}: {out[-2000:]}"
        assert f"PE {pe} of {npes}: ISx verification passed" in out
        if heap == "mirrored":
            import re
            # host stores went up (flushed); the small results came back into
            # the view with the blocking calls (settled, <= 256 KiB), so the
            # host's reads of them took no fault
            m = re.search(r"flushed (\d+) fetched (\d+) settled (\d+) blocks", out)
            assert m and int(m.group(1)) > 0 and int(m.group(3)) > 0, out
            trace = open(tmp_path / f"trace{pe}.log").read()
            calls = [ln for ln in trace.splitlines() if " algo " in ln]
            # (a call of at most 4 KiB per PE: the service exchange)
            assert len(calls) == 3 and all("algo direct" in ln or "algo service exchange" in ln
                                           for ln in calls), trace


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2, 3, 4, 8])
def test_ipc_signal_device_barriers(tmp_path, npes):
    """SIGNAL: DIRECT's pulls with device-side barriers (counters in the
    heap segments, polled across processes), stream-ordered: every reference
    pair on every active set, one-shot and two-shot, in place, and a
    captured hipGraph replayed with fresh inputs."""
    reports = run_pes(tmp_path, npes, "signal")
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
    fences_checked(reports, device=True)


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", ["full", "signal"])
def test_ipc_one_shot_unfused(tmp_path, scenario):
    """$SHMEMX_FUSED_ONESHOT=0 and $SHMEMX_FUSED_TWOSHOT_KB=0: DIRECT's and
    SIGNAL's one shot and two shot on their multi-launch schedules (fence +
    barrier launches around a plain fold and gather), the paths the fused
    launches replaced, still bit-exact on every pair."""
    reports = run_pes(tmp_path, 3, scenario, {"SHMEMX_FUSED_ONESHOT": "0", "SHMEMX_FUSED_TWOSHOT_KB": "0"})
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
        assert r["fences"]["fused_calls"] == 0 and r["fences"]["fused_twoshot_calls"] == 0
    fences_checked(reports, device=scenario == "signal")


@pytest.mark.gpu
def test_ipc_signal_missing_peer_times_out(tmp_path):
    """A peer that never reaches a SIGNAL barrier: the waiting PE's device
    barrier gives up after $SHMEMX_SIGNAL_TIMEOUT and the blocking call aborts
    with a FATAL line; the GPU is not left spinning."""
    procs = start_pes(tmp_path, 2, "signal_timeout", {"SHMEMX_SIGNAL_TIMEOUT": "2"})
    rcs, logs = wait_pes(procs, 120)
    assert rcs[1] == 0, logs[1][-1500:]
    assert rcs[0] != 0, logs[0][-1500:]
    assert "never reached the device barrier" in logs[0], logs[0][-1500:]


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [1, 3])
def test_ipc_host_kind_heap(tmp_path, npes):
    """$SHMEMX_HEAP_MEMORY=host: shmem_malloc returns page-locked host memory,
    as the reference's symmetric heap is (comms-inline.h:752-769), so host code
    writes symmetric objects directly; every reference pair on every active
    set, 40 MiB arrays across staging chunks, broadcast and collect, against
    the oracle; peers' heap_ptr is NULL."""
    reports = run_pes(tmp_path, npes, "hostheap", {"SHMEMX_HEAP_MEMORY": "host"})
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"


@pytest.mark.gpu
def test_direct_limit_mismatch_then_immediate_retry(tmp_path):
    """DIRECT members whose size limits differ (one PE per round raises its
    fused two-shot limit) all return ENOTSUP with the target untouched; that
    PE aligns at once and the very next call is correct on every PE, 20
    rounds back to back over 3 PE processes (the ENOTSUP path's closing
    barrier)."""
    reports = run_pes(tmp_path, 3, "limits", {"SHMEMX_TRANSPORT": "ipc"}, timeout=300)
    for r in reports:
        assert r["ncases"] == 40
        assert not r["fails"], f"PE {r['pe']}: {r['fails']}"


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["ipc", "rccl"])
def test_mixed_memory_kinds_fail_collectively(tmp_path, transport):
    """Even PEs pass host arrays, odd PEs device arrays: above 256 KiB the
    host PEs would issue one collective per 16 MiB staging chunk and the
    device PEs one, so the members compare call counts and all return
    ENOTSUP within seconds (no hang); matching calls afterwards work, and
    small arrays (one call either way) still mix."""
    env = {"SHMEMX_TRANSPORT": transport}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    reports = run_pes(tmp_path, 2, "mixed", env, timeout=300)
    for r in reports:
        assert r["ncases"] == 4
        assert not r["fails"], f"PE {r['pe']}: {r['fails']}"


@pytest.mark.gpu
def test_mirrored_view_fetch_waits_for_non_blocking_stream(tmp_path):
    """A host read of a mirrored target right after a stream-ordered call on
    a non-blocking torch stream, behind ~5 ms of other work on that stream and
    a kernel that rewrote the source's HBM twin: the fault waits for the
    stream (the writer recorded at the call) and reads the result, not the
    stale bytes; the view stays right after the stream completes."""
    reports = run_pes(tmp_path, 1, "mirror_stream", {"SHMEMX_HEAP_MEMORY": "mirrored"}, timeout=300)
    r = reports[0]
    assert not r["fails"], r["fails"]
    assert r["ncases"] == 2 and r["mirror_stats"]["blocks_fetched"] > 0, r


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["ipc", "rccl"])
def test_staging_chunk_ramp(tmp_path, transport):
    """Host arrays through the staging pipeline with 1 MiB chunks, so calls
    of a few MiB get the ramped schedule (quarter and half chunks at both
    ends, stage_plan.h): pageable out of place and in place, pinned, odd
    lengths, 2- to 16-byte elements, world and one-member sets, against the
    oracle on 2 PEs."""
    env = {"SHMEMX_TRANSPORT": transport, "SHMEMX_STAGE_CHUNK_MB": "1"}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    for r in run_pes(tmp_path, 2, "ramp", env, timeout=300):
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["ipc", "rccl"])
def test_algorithm_settings_differing_across_pes_is_fatal(tmp_path, transport):
    """An algorithm setting exported on one PE only ($SHMEM_REDUCE_ALGO here)
    would make the PEs plan different schedules for the same call: shmem_init
    compares the settings and fails on every PE with a FATAL line naming this
    PE's, instead of mismatched collectives later."""
    env = {"SHMEMX_TRANSPORT": transport, "PE1:SHMEM_REDUCE_ALGO": "gather"}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    procs = start_pes(tmp_path, 2, "heapcheck", env)
    rcs, logs = wait_pes(procs, 120)
    for pe, (rc, log) in enumerate(zip(rcs, logs)):
        assert rc != 0 and "algorithm settings differ across PEs" in log, f"PE {pe} exit {rc}:\n{log[-2000:]}"
    assert "SHMEM_REDUCE_ALGO=gather" in logs[1] and "SHMEM_REDUCE_ALGO" not in logs[0], logs


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["mirrored", "device"])
def test_heap_segment_on_some_pes_only_is_fatal(tmp_path, mode):
    """A PE whose symmetric heap segment cannot be allocated (a heap size no
    GPU holds) while its peer's can: the first shmem_malloc fails on both PEs
    with a FATAL line, instead of one PE carving its objects outside the
    segment (an asymmetric heap); with the size on every PE, both use private
    blocks alike and the calls are right.  Segments of different sizes
    (SHMEM_SYMMETRIC_HEAP_SIZE set differently) are FATAL as well."""
    env = {"SHMEMX_HEAP_MEMORY": mode, "PE1:SHMEM_SYMMETRIC_HEAP_SIZE": "4000000G"}
    procs = start_pes(tmp_path, 2, "heapcheck", env)
    rcs, logs = wait_pes(procs, 120)
    for pe, (rc, log) in enumerate(zip(rcs, logs)):
        assert rc != 0 and "could not be allocated on every PE" in log, f"PE {pe} exit {rc}:\n{log[-2000:]}"
    # segments on both PEs, of different sizes: FATAL on both too
    procs = start_pes(tmp_path, 2, "heapcheck", {"SHMEMX_HEAP_MEMORY": mode, "PE1:SHMEM_SYMMETRIC_HEAP_SIZE": "2G"})
    rcs, logs = wait_pes(procs, 120)
    for pe, (rc, log) in enumerate(zip(rcs, logs)):
        assert rc != 0 and "SHMEM_SYMMETRIC_HEAP_SIZE differs across PEs" in log, f"PE {pe} exit {rc}:\n{log[-2000:]}"
    env = {"SHMEMX_HEAP_MEMORY": mode, "SHMEM_SYMMETRIC_HEAP_SIZE": "4000000G"}
    for r in run_pes(tmp_path, 2, "heapcheck", env, timeout=120):
        assert not r["fails"] and r["ncases"] == 1 and r["private_blocks"], r


@pytest.mark.gpu
@pytest.mark.parametrize("transport,npes,mode", [("ipc", 2, "mirrored"), ("rccl", 2, "device")])
def test_threads_of_one_pe(tmp_path, transport, npes, mode):
    """Four host threads per PE call the library at once (PE_size 1 calls on
    host arrays, torch tensors on their own streams, and their own mirrored
    heap blocks read back through the view) while each PE's main thread runs
    world-set collectives: every result right, nothing deadlocks."""
    env = {"SHMEMX_TRANSPORT": transport, "SHMEMX_HEAP_MEMORY": mode}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    reports = run_pes(tmp_path, npes, "threads", env, timeout=300)
    for r in reports:
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
        assert r["worker_iterations"] == [25] * 4, r
        if mode == "mirrored":
            assert r["mirror_stats"]["blocks_fetched"] > 0, r


@pytest.mark.gpu
def test_ipc_full_scenario_on_mirrored_heap(tmp_path):
    """The 2-PE "full" scenario (every reference pair and active set on heap
    operands, in place, overlap, torch and host arrays, heap_ptr puts,
    broadcast and [f]collect) with the library's default heap mode: the
    collectives get host-view addresses, the test's own HIP copies the twins
    (shmemx_mirror_device_ptr) with sync/invalidate around them, and peers'
    heap_ptr of a view address is NULL while the twin's is not."""
    reports = run_pes(tmp_path, 2, "full", {"SHMEMX_HEAP_MEMORY": None})
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
    fences_checked(reports)


@pytest.mark.gpu
@pytest.mark.parametrize("transport,npes,mode", [("ipc", 1, "mirrored"), ("ipc", 4, "mirrored"),
                                                ("rccl", 3, "mirrored"), ("ipc", 2, None)])
def test_mirrored_heap(tmp_path, transport, npes, mode):
    """$SHMEMX_HEAP_MEMORY=mirrored: shmem_malloc returns a host view of the
    HBM heap; host code writes and reads symmetric objects with plain stores
    and loads, the collectives run device-resident on the HBM twins (DIRECT
    over the peers' HBM on the IPC transport), only touched blocks cross
    PCIe (a repeated call on untouched sources copies nothing up), against
    the oracle for every reference pair and active set, SIGNAL, in place,
    broadcast and collect.  mode None: the variable unset — the mirrored
    heap is the library's default."""
    env = {"SHMEMX_TRANSPORT": transport, "SHMEMX_HEAP_MEMORY": mode}
    if transport == "rccl":
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    reports = run_pes(tmp_path, npes, "mirrored", env, timeout=600)
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"
