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


def run_pes(tmp_path, npes, scenario, extra_env=None, timeout=900):
    boot = str(tmp_path / "uid")
    procs = []
    for pe in range(npes):
        env = dict(os.environ, SHMEM_PE=str(pe), SHMEM_NPES=str(npes), LOCAL_RANK="0",
                   SHMEM_BOOTSTRAP_FILE=boot, SHMEMX_TRANSPORT="ipc",
                   SHMEMX_BARRIER_TIMEOUT="120")
        env.pop("RANK", None)
        env.pop("WORLD_SIZE", None)
        env.update(extra_env or {})
        out = str(tmp_path / f"pe{pe}.json")
        log = open(tmp_path / f"pe{pe}.log", "w")
        procs.append((subprocess.Popen([sys.executable, os.path.join(HERE, "gpu_ipc_child.py"), out,
                                        scenario], env=env, stdout=log, stderr=subprocess.STDOUT,
                                       start_new_session=True), out, log))
    reports = []
    try:
        rcs = [p.wait(timeout=timeout) for p, _, _ in procs]
        if any(rcs):
            tails = []
            for (p, _, log), rc in zip(procs, rcs):
                log.close()
                tails.append(f"--- PE {procs.index((p, _, log))} exit {rc}:\n" + open(log.name).read()[-1500:])
            raise AssertionError("\n".join(tails))
        for p, out, log in procs:
            log.close()
            with open(out) as f:
                reports.append(json.load(f))
    finally:
        for p, _, _ in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    return reports


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2, 4])
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


@pytest.mark.gpu
def test_ipc_direct_staged_in_chunks(tmp_path):
    # a 1 MiB scratch: every staged operand crosses several chunks per call
    reports = run_pes(tmp_path, 3, "chunk", {"SHMEMX_DIRECT_SCRATCH_MB": "1"})
    for r in reports:
        assert r["ncases"] > 0
        assert not r["fails"], f"PE {r['pe']}: {r['fails'][:10]}"


@pytest.mark.gpu
def test_isx_c_program_four_pes(tmp_path):
    """The C99 ISx verification program (examples/isx_verify.c: the
    reference's known-answer check, isx.c:615-624, on static host arrays) as
    four PE processes, shmem_init bootstrapping through a file."""
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
