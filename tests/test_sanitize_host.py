"""The host-compilable parts of the library under AddressSanitizer and
UndefinedBehaviorSanitizer (gcc, -fno-sanitize-recover: the first report
fails the run): the symmetric-heap arena (arena.cpp), the intra-node block's
host barrier and descriptors over forked PEs (node.cpp), the soft x87
arithmetic the GPU runs for long double (ld80.h), and the copy threads'
placement over a fake sysfs tree (topology.cpp) and the staging chunk
schedule (stage_plan.h).  The same harnesses run
unsanitized, at larger sizes, in test_heap_host.py, test_node_host.py and
test_ld80_host.py.  GPU-side sanitizers are not available on the MI355X pool."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "openshmem-async_amd", "csrc")
NATIVE = os.path.join(REPO, "tests", "native")
SAN = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
       "-fno-omit-frame-pointer"]
HIP_LINK = ["-D__HIP_PLATFORM_AMD__", "-I", os.path.join(REPO, "include"), "-I", "/opt/rocm/include",
            "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]

CASES = {
    "arena": ([os.path.join(NATIVE, "test_heap.cpp"), os.path.join(CSRC, "arena.cpp")], [], ["50000"], "ok 50000"),
    "node": ([os.path.join(NATIVE, "test_node_barrier.cpp"), os.path.join(CSRC, "node.cpp")], HIP_LINK,
             ["4", "1000"], "ok 4"),
    "ld80": ([os.path.join(NATIVE, "test_ld80.cpp")], [], ["300000"], "ok 300000"),
    # the host staging pipeline's chunk schedule (stage_plan.h)
    "stage_plan": ([os.path.join(NATIVE, "test_stage_plan.cpp")], [], [], "ok "),
    # the copy threads' placement (staging.cpp: cache domains of the GPU's node)
    "topology": ([os.path.join(NATIVE, "test_topology.cpp"), os.path.join(CSRC, "topology.cpp")], [],
                 ["{tmp}/sys"], "ok "),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_host_code_under_asan_ubsan(tmp_path, name):
    srcs, extra, args, want = CASES[name]
    exe = tmp_path / f"{name}_san"
    subprocess.run(["g++", *SAN, "-I", CSRC, *srcs, *extra, "-o", str(exe)], check=True)
    env = dict(os.environ, SHMEMX_BARRIER_TIMEOUT="60",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    args = [a.replace("{tmp}", str(tmp_path)) for a in args]
    out = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert out.stdout.startswith(want), out.stdout[-2000:]
    assert "runtime error" not in out.stderr, out.stderr[-4000:]


def test_gpu_asan_build_is_instrumented():
    """tests/test_gpu_asan.py's library build is really instrumented: its host
    objects call the ASan runtime, which the drivers carry, and the driver
    that runs over the RCCL test double binds it before the library."""
    asan = os.path.join(REPO, "tests", "native", "asan")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "native"), "asan"], check=True)
    lib = subprocess.run(["nm", "-D", os.path.join(asan, "libshmem_reduce_mi355x.so")],
                         capture_output=True, text=True, check=True).stdout
    assert "__asan_report_load8" in lib and "__asan_init" in lib
    for exe in ("asan_driver", "asan_driver_fake"):
        syms = subprocess.run(["nm", os.path.join(asan, exe)], capture_output=True, text=True,
                              check=True).stdout
        assert "__asan_init" in syms
    needed = subprocess.run(["readelf", "-d", os.path.join(asan, "asan_driver_fake")], capture_output=True,
                            text=True).stdout
    libs = [ln.split("[")[1].rstrip("]") for ln in needed.splitlines() if "(NEEDED)" in ln]
    assert libs.index("libfake_rccl.so") < libs.index("libshmem_reduce_mi355x.so")
