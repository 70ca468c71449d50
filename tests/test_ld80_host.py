"""CPU check of the GPU's software x87 (openshmem-async_amd/csrc/ld80.h): the
same source compiled for the host and compared with the host's x87 unit on
random and special 80-bit encodings (add, mul, <, >), value bytes exact.
The GPU build of the same code is checked on the device in
test_gpu_fold.py::test_longdouble_x87_encodings."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_soft_x87_matches_host_x87(tmp_path):
    exe = tmp_path / "test_ld80"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "openshmem-async_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "test_ld80.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "3000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert out.stdout.startswith("ok 3000000")
