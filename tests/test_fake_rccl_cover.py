"""The RCCL test double (tests/native/fake_rccl.cpp, used by the GPU tests to
run the RCCL transport with several PEs on one GPU) must define every RCCL
function the product library imports; otherwise some RCCL-transport path
would silently bind to the real librccl in those tests."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _syms(path, flag):
    out = subprocess.run(["nm", "-D", flag, path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1].split("@")[0] for ln in out.splitlines() if ln.strip()}


def test_double_defines_every_imported_rccl_function():
    lib = os.path.join(REPO, "openshmem-async_amd", "libshmem_reduce_mi355x.so")
    fake = os.path.join(REPO, "tests", "native", "libfake_rccl.so")
    imported = {s for s in _syms(lib, "--undefined-only") if s.startswith("nccl")}
    assert imported, "the library imports no nccl* symbols?"
    missing = imported - _syms(fake, "--defined-only")
    assert not missing, f"fake_rccl lacks {sorted(missing)}"
