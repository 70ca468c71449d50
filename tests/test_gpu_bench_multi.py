"""bench.py's N > 1 path, run the way the driver runs it
(`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`),
with every rank on the box's one GPU: on the default RCCL transport through
the RCCL test double (tests/native/fake_rccl.cpp), and on the IPC transport.

This is the code the driver's 8-GPU scaling run executes: gloo bootstrap,
the timed region with its barriers and max over ranks, the correctness guard
on the whole target (tolerance check + shmemx_verify), every extra (other
algorithms, config curves, latencies, DIRECT/SIGNAL over the peers' HBM, the
coherence check, the crossover and partial-set tables, auto_recommendation).
The numbers are a shared GPU's and are never reported; what is asserted is
that the line comes out, says correct, and carries no error where the
transport supports the algorithm.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

# algorithms that need an RCCL communicator: refused (ENOTSUP) on the IPC transport
RCCL_ONLY = ("rccl", "allreduce", "a2a")


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def strings(x, path=""):
    """(path, text) of every string leaf of a JSON value."""
    if isinstance(x, dict):
        for k, v in x.items():
            yield from strings(v, f"{path}.{k}")
    elif isinstance(x, list):
        for i, v in enumerate(x):
            yield from strings(v, f"{path}[{i}]")
    elif isinstance(x, str):
        yield path, x


@pytest.mark.gpu
@pytest.mark.parametrize("transport,npes", [("rccl", 2), ("ipc", 2), ("rccl", 4), ("ipc", 4), ("rccl", 8), ("ipc", 8)])
def test_bench_multi_rank_line(tmp_path, transport, npes):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(SHMEMX_SHARE_GPU="1", SHMEMX_BARRIER_TIMEOUT="120", PYTHONUNBUFFERED="1")
    if transport == "ipc":
        env["SHMEMX_TRANSPORT"] = "ipc"
    else:
        env.pop("SHMEMX_TRANSPORT", None)
        env["FAKE_RCCL"] = os.path.join(HERE, "native", "libfake_rccl.so")
    if npes > 4:
        env["GPU_MAX_HW_QUEUES"] = "2"     # 8 processes' queues on one GPU (test_gpu_ipc.py)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={npes}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", str(npes), "--steps", "3", "--warmup", "1",
           "--nreduce", str(1 << 20), "--extras-max-nreduce", str(1 << 20), "--extras-timeout", "240"]
    logdir = os.environ.get("GPU_TEST_LOGDIR")
    err_path = (os.path.join(logdir, f"bench_multi_{transport}_{npes}.err") if logdir
                else str(tmp_path / "bench.err"))
    if logdir:
        os.makedirs(logdir, exist_ok=True)
    with open(err_path, "w") as err:
        p = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=err, text=True,
                           timeout=420, start_new_session=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    tail = open(err_path).read()[-3000:]
    assert p.returncode == 0, f"exit {p.returncode}\n{p.stdout[-2000:]}\n{tail}"
    assert len(lines) == 1, f"want one JSON line, got {len(lines)}\n{p.stdout[-2000:]}"
    line = json.loads(lines[0])
    assert line["correct"] is True
    assert line["n_gpus"] == npes and line["steps"] == 3 and line["value"] > 0
    # value = algbw; the whole job's rate beside it
    # (both rounded to 0.01 in the line)
    assert abs(line["aggregate_GiBps"] - npes * line["value"]) <= 0.005 * (npes + 1) + 1e-9, line
    assert "algbw" in line["value_definition"]
    # the guard checked every element of the timed target against the
    # regenerated sources' PE_start fold, within the bound
    g = line["guard"]
    assert g["elements_checked"] == 1 << 20 and g["elements_out_of_bound"] == 0, g
    assert g["same_on_every_pe"] is True and g["max_err_over_bound"] <= 1.0, g
    roof = line["roofline"]
    assert roof["bound"] == "xgmi" and "153 GB/s per link in EACH direction" in roof["peak_basis"], roof
    assert roof["peak"] == (npes - 1) * 153.0
    # the reference's CPU src/reduce on this host in the same run (north_star):
    # the line's own config on N PE processes, one core each
    cpu = line["cpu_baseline"]
    assert isinstance(cpu, dict) and cpu["cores"] == npes and cpu["value"] > 0, cpu
    assert cpu["unit"] == "GiB/s" and cpu["kind"] == "port" and f"on {npes} PEs" in cpu["sample"], cpu
    sp = cpu["spread"]
    assert sp["min_ms"] <= sp["median_ms"] <= sp["max_ms"] and sp["calls"] >= 3, sp
    extras = line["extras"]
    assert "note" not in extras, extras.get("note")     # no watchdog, no fatal signal
    for algo in ("direct", "signal"):
        c = extras["coherence"][algo]
        assert isinstance(c, dict) and c["calls"] == 60 and c["mismatched_elements"] == 0, c
    for k in ("direct_heap", "signal_heap"):
        assert isinstance(extras[k], dict) and extras[k]["correct"] is True, extras[k]
    x = extras["xgmi_links"]     # raw pull / push rates over the IPC-mapped heap
    assert isinstance(x, dict) and x["push_visible_after_barrier"] is True, x
    assert set(x["GBps_per_gpu"]) == {"pull_one", "pull_all", "push_one", "push_all"}
    assert all(v > 0 for v in x["GBps_per_gpu"].values()), x
    assert roof["measured_link_ceiling_GBps"] == x["GBps_per_gpu"]["pull_all"], roof
    assert roof["frac_of_measured_links"] > 0, roof
    if transport == "rccl":           # the RCCL algorithms with the heap registered with RCCL
        rr = extras["rccl_registered"]
        assert isinstance(rr, dict) and rr["algo_rccl_correct"] is True and rr["algo_allreduce_correct"] is True, rr
        assert rr["algo_rccl_GiBps"] > 0 and rr["algo_allreduce_GiBps"] > 0, rr
    else:
        assert "rccl_registered" not in extras
    cfg = extras["configs"]            # config 5's curve: algbw and busbw per size
    assert set(cfg["float_sum_busbw_GBps_vs_nreduce"]) == set(cfg["float_sum_GiBps_vs_nreduce"]), cfg
    for k, a in cfg["float_sum_algbw_GBps_vs_nreduce"].items():
        assert a > 0 and abs(cfg["float_sum_busbw_GBps_vs_nreduce"][k] - a * 2 * (npes - 1) / npes) < 0.02, (k, a)
    he = extras["host_resident_e2e"]   # host-resident operands on every PE, exact sums
    assert isinstance(he, dict) and he["correct"] is True and he["last_error"] == 0 and he["GiBps"] > 0, he
    assert he["nreduce"] == 1 << 20, he
    assert he["pageable"]["correct"] is True and he["pageable"]["GiBps"] > 0, he
    c0 = extras["config0"]             # BASELINE configs[0] through the product, 2 PEs
    for k in ("n1_heap", "n1_host", "n1024_heap", "n1024_host", "n4096_heap", "n4096_host"):
        assert c0[k]["correct"] is True and c0[k]["median_us"] > 0, (k, c0)
    pa = extras["push_allreduce"]      # the store-based exchange, exact integer sums
    assert isinstance(pa, dict) and pa["correct"] is True and pa["GiBps"] > 0, pa
    bad = []
    for path, text in strings(extras):
        if path.endswith("_note") or path.startswith(".auto_recommendation") or ".recommend_env." in path:
            continue     # labels and algorithm names, not outcomes
        if path == ".partial_sets" and npes < 4 and text == "needs N >= 4":
            continue
        refused = "ENOTSUP" in text and transport == "ipc" and any(
            f".{a}" in path or f"algo_{a}_" in path for a in RCCL_ONLY)
        if not refused:
            bad.append(f"{path}: {text[:160]}")
    assert not bad, "\n".join(bad[:20])
    # every timed crossover / partial-set call left exact targets
    for algo, row in extras["algo_crossover"]["correct"].items():
        for n, ok in row.items():
            assert ok is True or (transport == "ipc" and algo in RCCL_ONLY), (algo, n, ok)
    rec = extras["auto_recommendation"]
    assert "full" in rec and rec["env"].get("SHMEMX_AUTO_FULL", "").startswith("0:"), rec
    if npes >= 4:
        p2 = extras["partial_sets"]
        for shape in ("first_half_correct", "every_other_correct"):
            for algo, row in p2[shape].items():
                for n, ok in row.items():
                    assert ok is True or (transport == "ipc" and algo in RCCL_ONLY), (shape, algo, n, ok)
        assert rec["env"].get("SHMEMX_AUTO_PARTIAL", "").startswith("0:"), rec


@pytest.mark.gpu
def test_bench_multi_watchdog_cut_keeps_line(tmp_path):
    """The extras' watchdog fires in the middle of the crossover table (2
    ranks, RCCL test double, only that extra, a 1.5 s budget): rank 0 still
    prints the one line, correct, with the watchdog's note, the crossover
    cells measured so far, and an auto_recommendation built from them."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(SHMEMX_SHARE_GPU="1", SHMEMX_BARRIER_TIMEOUT="120", PYTHONUNBUFFERED="1",
               FAKE_RCCL=os.path.join(HERE, "native", "libfake_rccl.so"))
    env.pop("SHMEMX_TRANSPORT", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--nreduce", str(1 << 20), "--extras-max-nreduce", str(1 << 20),
           "--extras-only", "algo_crossover", "--extras-timeout", "1.5"]
    err_path = str(tmp_path / "bench.err")
    with open(err_path, "w") as err:
        p = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=err, text=True,
                           timeout=300, start_new_session=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    tail = open(err_path).read()[-3000:]
    assert p.returncode == 0, f"exit {p.returncode}\n{p.stdout[-2000:]}\n{tail}"
    assert len(lines) == 1, f"want one JSON line, got {len(lines)}\n{p.stdout[-2000:]}"
    line = json.loads(lines[0])
    assert line["correct"] is True and line["value"] > 0
    extras = line["extras"]
    assert "timeout" in extras.get("note", ""), extras.get("note")
    assert set(extras) <= {"note", "algo_crossover", "auto_recommendation"}, sorted(extras)
    assert isinstance(extras["algo_crossover"], dict)
    rec = extras["auto_recommendation"]
    assert isinstance(rec, dict) and "cut short" in rec.get("note", ""), rec
    assert isinstance(rec.get("env"), dict)


@pytest.mark.gpu
def test_bench_multi_guard_catches_a_corrupt_element(tmp_path):
    """The N > 1 guard's negative control: one element of rank 0's timed
    target moved by far more than the bound (--corrupt-guard-test) turns the
    line's correct false and the exit status 1 (2 ranks, IPC transport)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(SHMEMX_SHARE_GPU="1", SHMEMX_BARRIER_TIMEOUT="120", PYTHONUNBUFFERED="1", SHMEMX_TRANSPORT="ipc")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--nreduce", str(1 << 20), "--extras", "0", "--no-cpu-baseline", "--corrupt-guard-test"]
    err_path = str(tmp_path / "bench.err")
    with open(err_path, "w") as err:
        p = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=err, text=True,
                           timeout=300, start_new_session=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, f"want one JSON line\n{p.stdout[-2000:]}\n{open(err_path).read()[-2000:]}"
    line = json.loads(lines[0])
    assert line["correct"] is False and p.returncode != 0
    assert line["guard"]["elements_out_of_bound"] >= 1, line["guard"]
