"""The library's host code under AddressSanitizer + UBSan on the GPU: the C driver
tests/native/asan_driver.c linked with an ASan build of the library
(tests/native/Makefile, target asan; host side only, the shipped GPU kernel
objects) runs every host path of the product that a reference program
reaches — pageable host arrays through the staging pipeline and its copy
gangs, the small-message bounce, device arrays, the mirrored heap's fault
handler and coherence, stream-ordered calls with every algorithm, the
collectives beside the reductions, checksum, error paths, finalize — on one
PE (plain and with the collective schedules forced onto a one-rank RCCL
communicator) and on three PE processes sharing the GPU (IPC transport, and
the RCCL transport over the RCCL test double, where a strided partial set
makes its own communicator).  The first ASan or UBSan report fails the run.

The CPU suite's test_sanitize_host.py covers the parts that run without a
GPU (arena, node barrier, soft x87) under ASan + UBSan."""
import os
import signal
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ASAN = os.path.join(HERE, "native", "asan")

# handle_segv=0: the mirrored heap's own SIGSEGV handler serves host-view
# faults (ASan's would report them); leaks are not checked (the HIP runtime
# keeps its allocations to exit)
ASAN_OPTIONS = "handle_segv=0:allow_user_segv_handler=1:detect_leaks=0:halt_on_error=1"
UBSAN_OPTIONS = "print_stacktrace=1:halt_on_error=1"

MODES = {   # heap: mirrored is the product default; the suite's conftest sets device
    "one_pe": ("asan_driver", 1, {"SHMEMX_HEAP_MEMORY": "mirrored"}),
    "one_pe_collective": ("asan_driver", 1, {"SHMEMX_HEAP_MEMORY": "mirrored", "SHMEMX_FORCE_COLLECTIVE": "1"}),
    "three_pes_ipc": ("asan_driver", 3, {"SHMEMX_HEAP_MEMORY": "mirrored", "SHMEMX_TRANSPORT": "ipc"}),
    "three_pes_ipc_host_heap": ("asan_driver", 3, {"SHMEMX_HEAP_MEMORY": "host", "SHMEMX_TRANSPORT": "ipc"}),
    "three_pes_rccl_double": ("asan_driver_fake", 3, {"SHMEMX_HEAP_MEMORY": "mirrored"}),
}


def run_driver(tmp_path, exe, npes, extra):
    """Start the driver as npes PE processes; (exit code, output) per PE."""
    path = os.path.join(ASAN, exe)
    assert os.path.exists(path), f"{path} not built (make -C tests/native asan)"
    procs = []
    for pe in range(npes):
        env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "SHMEM_PE", "SHMEM_NPES")}
        env.update(ASAN_OPTIONS=ASAN_OPTIONS, UBSAN_OPTIONS=UBSAN_OPTIONS, SHMEMX_BARRIER_TIMEOUT="120",
                   LOCAL_RANK="0", **extra)
        if npes > 1:
            env.update(SHMEM_PE=str(pe), SHMEM_NPES=str(npes), SHMEM_BOOTSTRAP_FILE=str(tmp_path / "uid"))
        with open(tmp_path / f"pe{pe}.log", "w") as log:
            procs.append(subprocess.Popen([path], env=env, stdout=log, stderr=subprocess.STDOUT,
                                          start_new_session=True))
    try:
        for p in procs:
            p.wait(timeout=240)
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    return [(p.returncode, open(tmp_path / f"pe{pe}.log").read()) for pe, p in enumerate(procs)]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", sorted(MODES))
def test_host_code_under_asan_on_gpu(tmp_path, mode):
    exe, npes, extra = MODES[mode]
    for pe, (rc, out) in enumerate(run_driver(tmp_path, exe, npes, extra)):
        assert "AddressSanitizer" not in out and "runtime error" not in out, f"PE {pe}:\n{out[-6000:]}"
        assert rc == 0, f"PE {pe} exit {rc}:\n{out[-4000:]}"
        assert out.strip().splitlines()[-1].startswith("ok "), out[-2000:]


@pytest.mark.gpu
def test_asan_negative_control(tmp_path):
    """The same build reports an overflow made inside the library: a host
    source shorter than nreduce, read by the staging copy."""
    [(rc, out)] = run_driver(tmp_path, "asan_driver", 1, {"SHMEMX_HEAP_MEMORY": "mirrored",
                                                          "ASAN_DRIVER_NEGATIVE": "1"})
    assert rc != 0 and "AddressSanitizer: heap-buffer-overflow" in out, out[-4000:]
    assert "negative control: no report" not in out
