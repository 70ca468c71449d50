"""The library's host code under ThreadSanitizer on the GPU, with several
threads of one PE calling it at once: tests/native/tsan_driver.c linked with a
TSan build of the library (tests/native/Makefile, target tsan; host side only,
the shipped GPU kernel objects).  Worker threads make PE_size 1 calls on their
own pageable host arrays (bounce buffers, the staging ring and its two copy
gangs), device arrays on their own streams, and mirrored-heap blocks read back
through the host view (the fault handler and its service thread), while the
main thread makes world-set calls.  The first TSan report fails the run."""
import os
import signal
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TSAN = os.path.join(HERE, "native", "tsan")

# halt on the first report; the mirrored heap's SIGSEGV handler serves its own
# faults (TSan passes synchronous signals straight to it)
# (the ROCm runtime's own reports are suppressed: tests/native/tsan.supp)
TSAN_OPTIONS = ("halt_on_error=1:second_deadlock_stack=1:report_signal_unsafe=0:suppressions="
                + os.path.join(HERE, "native", "tsan.supp"))

MODES = {
    "one_pe_mirrored": (1, {"SHMEMX_HEAP_MEMORY": "mirrored"}),
    "two_pes_ipc_mirrored": (2, {"SHMEMX_HEAP_MEMORY": "mirrored", "SHMEMX_TRANSPORT": "ipc"}),
}


def run_driver(tmp_path, npes, extra, args=("3", "6")):
    """Start the driver as npes PE processes; (exit code, output) per PE."""
    path = os.path.join(TSAN, "tsan_driver")
    assert os.path.exists(path), f"{path} not built (make -C tests/native tsan)"
    procs = []
    for pe in range(npes):
        env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "SHMEM_PE", "SHMEM_NPES")}
        env.update(TSAN_OPTIONS=TSAN_OPTIONS, SHMEMX_BARRIER_TIMEOUT="120", LOCAL_RANK="0", **extra)
        if npes > 1:
            env.update(SHMEM_PE=str(pe), SHMEM_NPES=str(npes), SHMEM_BOOTSTRAP_FILE=str(tmp_path / "uid"))
        with open(tmp_path / f"pe{pe}.log", "w") as log:
            procs.append(subprocess.Popen([path, *args], env=env, stdout=log, stderr=subprocess.STDOUT,
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
def test_host_code_under_tsan_with_threads(tmp_path, mode):
    npes, extra = MODES[mode]
    for pe, (rc, out) in enumerate(run_driver(tmp_path, npes, extra)):
        assert "ThreadSanitizer" not in out, f"PE {pe}:\n{out[-8000:]}"
        assert rc == 0, f"PE {pe} exit {rc}:\n{out[-4000:]}"
        assert out.strip().splitlines()[-1].startswith("ok "), out[-2000:]
        fetched = [ln for ln in out.splitlines() if ln.startswith("mirror ")]
        assert fetched and int(fetched[0].split()[-1]) > 0, out[-2000:]   # the fault path ran


@pytest.mark.gpu
def test_tsan_negative_control(tmp_path):
    """The same build and options report a race: two driver threads write one
    word unsynchronised ($TSAN_DRIVER_NEGATIVE), so the suppressions do not
    silence the driver's or the library's own code."""
    [(rc, out)] = run_driver(tmp_path, 1, {"SHMEMX_HEAP_MEMORY": "mirrored", "TSAN_DRIVER_NEGATIVE": "1"},
                             args=("2", "1"))
    assert rc != 0 and "ThreadSanitizer: data race" in out, out[-4000:]
    assert "tsan_driver.c" in out, out[-4000:]
