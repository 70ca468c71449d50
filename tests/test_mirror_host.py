"""CPU check of the mirrored heap's core (openshmem-async_amd/csrc/mirror.cpp):
the block states, page protection and SIGSEGV path that keep the host view
of the HBM symmetric heap coherent ($SHMEMX_HEAP_MEMORY=mirrored), driven by
random host stores / loads and collective-style flushes and device writes
against a model, with a memcpy backend in place of HIP
(tests/native/test_mirror.cpp).  Plain, and under ASan + UBSan (ASan's own
SIGSEGV handler off, so the view's handler sees the faults)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "openshmem-async_amd", "csrc")
SRCS = [os.path.join(REPO, "tests", "native", "test_mirror.cpp"), os.path.join(CSRC, "mirror.cpp"),
        os.path.join(CSRC, "fatal_note.cpp")]
INCLUDE = os.path.join(REPO, "include")


@pytest.mark.parametrize("flags", [["-O2"], ["-O1", "-g", "-fsanitize=address,undefined",
                                              "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]],
                         ids=["plain", "asan_ubsan"])
def test_mirror_core_against_model(tmp_path, flags):
    exe = tmp_path / "test_mirror"
    subprocess.run(["g++", *flags, "-std=c++17", "-pthread", "-Wall", "-Wextra", "-I", CSRC, "-I", INCLUDE, *SRCS,
                    "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="handle_segv=0:allow_user_segv_handler=1:detect_leaks=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([str(exe), "4000"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert "ok 4000" in out.stdout, out.stdout[-2000:]
    assert "runtime error" not in out.stderr, out.stderr[-3000:]
