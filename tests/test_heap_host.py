"""CPU check of the symmetric-heap arena (openshmem-async_amd/csrc/arena.cpp):
the allocator that carves each PE's HBM segment, compiled for the host and
driven by random alloc/free sequences (tests/native/test_heap.cpp)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_arena_random_sequences_and_size_syntax(tmp_path):
    exe = tmp_path / "test_heap"
    csrc = os.path.join(REPO, "openshmem-async_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-I", csrc,
                    os.path.join(REPO, "tests", "native", "test_heap.cpp"),
                    os.path.join(csrc, "arena.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "200000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout
    assert out.stdout.startswith("ok 200000")
