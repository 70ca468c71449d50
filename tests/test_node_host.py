"""CPU check of the intra-node block (openshmem-async_amd/csrc/node.cpp): the
host barrier over arbitrary active sets and the per-call descriptors, with
real forked processes and a random sequence of collectives on random sets
(tests/native/test_node_barrier.cpp).  The GPU half of the layer (IPC
mappings) is covered by tests/test_gpu_ipc.py."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("npes", [2, 5, 8])
def test_node_barrier_and_descriptors_random_sets(tmp_path, npes):
    exe = tmp_path / "test_node_barrier"
    csrc = os.path.join(REPO, "openshmem-async_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I", csrc,
                    "-I", os.path.join(REPO, "include"), "-I", "/opt/rocm/include",
                    os.path.join(REPO, "tests", "native", "test_node_barrier.cpp"),
                    os.path.join(csrc, "node.cpp"), "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)], check=True)
    env = dict(os.environ, SHMEMX_BARRIER_TIMEOUT="60")
    out = subprocess.run([str(exe), str(npes), "3000"], capture_output=True, text=True, timeout=300,
                         env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith(f"ok {npes}")
