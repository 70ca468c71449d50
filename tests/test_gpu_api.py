"""GPU tests of the drop-in entry points (shmem_<T>_<op>_to_all) at one PE.

On one PE the reference's call is `write_to = source` plus two barriers
(reduce-op.c:213-217,250): target must equal source, for device- and
host-resident arrays (the reference's symmetric heap is host memory,
memory/symmem.c:168-227), in place or not, and pWrk/pSync are left alone.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_runtime_single_pe(cuda, shm):
    shm.init()
    assert shm.my_pe() == 0 and shm.n_pes() == 1
    assert shm.get_stream() != 0


@pytest.mark.parametrize("t", ["short", "int", "long", "longlong", "float", "double",
                               "complexd", "complexf"])
def test_api_pe1_device_copy(cuda, shm, oracle, t):
    import torch
    n = 4103
    src = oracle.fill(t, 1, 77, n)
    want = oracle.reduce_sim(t, "sum", src[None, :], 0, 0, 1)[0]
    s = torch.from_numpy(src).cuda()
    d = torch.zeros_like(s)
    psync = np.full(128, -1, dtype=np.int64)
    pwrk = np.zeros(64, dtype=src.dtype)
    shm.to_all(t, "sum", d, s, n, 0, 0, 1, pwrk, psync)
    assert shm.last_error() == 0
    assert d.cpu().numpy().tobytes() == want.tobytes()
    assert (psync == -1).all()


@pytest.mark.parametrize("t,op", [("double", "sum"), ("int", "and"), ("float", "max"),
                                  ("long", "xor")])
def test_api_pe1_host_arrays(cuda, shm, oracle, t, op):
    """Host-resident symmetric arrays go H2D -> device path -> D2H."""
    n = 100003
    src = oracle.fill(t, 1, 99, n)
    tgt = np.zeros_like(src)
    psync = np.full(128, -1, dtype=np.int64)
    shm.to_all(t, op, tgt, src, n, 0, 0, 1, None, psync)
    assert shm.last_error() == 0
    assert tgt.tobytes() == src.tobytes()
    # in place on host memory
    src2 = src.copy()
    shm.to_all(t, op, src2, src2, n, 0, 0, 1, None, psync)
    assert src2.tobytes() == src.tobytes()
    assert (psync == -1).all()


def test_api_pe1_in_place_and_overlap_device(cuda, shm, oracle):
    import torch
    n = 70001
    src = oracle.fill("double", 1, 5, n + 10)
    buf = torch.from_numpy(src).cuda()
    shm.to_all("double", "sum", buf, buf, n, 0, 0, 1)   # in place
    assert buf.cpu().numpy().tobytes() == src.tobytes()
    # partial overlap: target = source + 3 elements (reference's temp path)
    shm.to_all("double", "sum", buf[3:], buf, n, 0, 0, 1)
    got = buf.cpu().numpy()
    assert got[3:3 + n].tobytes() == src[:n].tobytes()
    assert got[:3].tobytes() == src[:3].tobytes()


def test_api_zero_and_invalid(cuda, shm):
    import torch
    d = torch.full((16,), 7.0, dtype=torch.float64, device="cuda")
    s = torch.ones(16, dtype=torch.float64, device="cuda")
    shm.to_all("double", "sum", d, s, 0, 0, 0, 1)            # n == 0: no effect
    assert shm.last_error() == 0 and (d == 7.0).all()
    shm.to_all("double", "sum", d, s, -1, 0, 0, 1)           # n < 0 (reference: UB)
    assert shm.last_error() == 1 and (d == 7.0).all()
    shm.to_all("double", "sum", d, s, 16, 1, 0, 1)           # set {1} beyond npes
    assert shm.last_error() == 1 and (d == 7.0).all()
    shm.to_all("double", "sum", d, s, 16, 0, 0, 2)           # set beyond npes
    assert shm.last_error() == 1 and (d == 7.0).all()


def test_typed_stream_forms_return_error_codes(cuda, shm, oracle):
    """shmemx_<T>_<op>_to_all_on_stream for all 44 pairs: a valid call returns
    SHMEMX_OK with the result, a bad one the error code (not void)."""
    import torch
    L = shm.lib()
    n = 1000
    for t, op in shm.REFERENCE_PAIRS:
        f = getattr(L, f"shmemx_{t}_{op}_to_all_on_stream")
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 4 + [ctypes.c_void_p]
        src = oracle.fill(t, 1, 11, n)
        s = torch.from_numpy(src.view(np.uint8)).cuda()
        d = torch.zeros_like(s)
        assert f(d.data_ptr(), s.data_ptr(), n, 0, 0, 1, None) == 0, (t, op)
        torch.cuda.synchronize()
        assert d.cpu().numpy().tobytes() == src.tobytes(), (t, op)
        assert f(d.data_ptr(), s.data_ptr(), -1, 0, 0, 1, None) == 1, (t, op)      # EINVAL
        assert shm.last_error() == 1
        assert f(d.data_ptr(), s.data_ptr(), n, 0, 0, 2, None) == 1, (t, op)       # set beyond npes


def test_longdouble_entry_point(cuda, shm, oracle):
    """shmem_longdouble_*_to_all run on the GPU (soft x87, ld80.h): host
    arrays at PE_size = 1 copy the value bytes."""
    src = oracle.fill("longdouble", 1, 5, 1000)
    tgt = np.zeros_like(src)
    for op in ("sum", "prod", "min", "max"):
        tgt[:] = 0
        shm.to_all("longdouble", op, tgt, src, len(src), 0, 0, 1)
        assert shm.last_error() == 0
        assert np.array_equal(tgt, src)


def test_reduce_on_stream_torch_stream(cuda, shm, oracle):
    import torch
    n = 1 << 20
    src = oracle.fill("float", 1, 3, n)
    s = torch.from_numpy(src).cuda()
    d = torch.zeros_like(s)
    st = torch.cuda.Stream()
    shm.reduce_on_stream("float", "sum", d, s, n, 0, 0, 1, "auto", st.cuda_stream)
    st.synchronize()
    assert d.cpu().numpy().tobytes() == src.tobytes()


def test_hip_graph_capture_and_replay(cuda, shm):
    """The stream-ordered entry points are capturable (no allocation or host
    sync inside once a call of the same shape has run): capture a 3-input fold
    and a PE_size=1 reduction into one graph, change the inputs, replay."""
    import torch
    n = (1 << 20) + 5
    a = torch.rand(n, dtype=torch.float64, device="cuda")
    b = torch.rand(n, dtype=torch.float64, device="cuda")
    c = torch.rand(n, dtype=torch.float64, device="cuda")
    out = torch.empty_like(a)
    out2 = torch.empty_like(a)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        shm.fold_n("double", "sum", out, [a, b, c], n, s.cuda_stream)
        shm.reduce_on_stream("double", "sum", out2, out, n, 0, 0, 1, "auto", s.cuda_stream)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream().cuda_stream
        shm.fold_n("double", "sum", out, [a, b, c], n, st)
        shm.reduce_on_stream("double", "sum", out2, out, n, 0, 0, 1, "auto", st)
    for _ in range(2):
        a.uniform_(); b.uniform_(); c.uniform_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, (a + b) + c)
        assert torch.equal(out2, out)


def test_fortran_forwarder(cuda, shm, oracle):
    """shmem_real8_sum_to_all_ (fortran.c:1003-1016): args by reference."""
    import torch
    n = 1001
    src = oracle.fill("double", 1, 11, n)
    s = torch.from_numpy(src).cuda()
    d = torch.zeros_like(s)
    c_int = ctypes.c_int
    psync = np.full(128, -1, dtype=np.int32)
    f = shm.lib().shmem_real8_sum_to_all_
    f.restype = None
    f(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(s.data_ptr()), ctypes.byref(c_int(n)),
      ctypes.byref(c_int(0)), ctypes.byref(c_int(0)), ctypes.byref(c_int(1)), None,
      ctypes.c_void_p(psync.ctypes.data))
    assert shm.last_error() == 0
    assert d.cpu().numpy().tobytes() == src.tobytes()
    assert (psync == -1).all()


def test_rccl_schedules_one_rank(cuda):
    """Every RCCL call of the multi-PE path (reduce-scatter, all-gather,
    all-reduce, grouped send/recv schedules) on a one-rank communicator,
    called directly and captured into HIP graphs that are replayed."""
    import subprocess
    import sys
    env = dict(os.environ, SHMEMX_FORCE_COLLECTIVE="1")
    here = os.path.dirname(os.path.abspath(__file__))
    out = subprocess.run([sys.executable, os.path.join(here, "gpu_collective_p1.py")],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout + out.stderr


@pytest.mark.parametrize("t", ["double", "short", "complexd", "longdouble"])
def test_host_staging_pipeline_many_chunks(cuda, shm, oracle, t):
    """Host-resident arrays larger than one 16 MiB staging chunk, every
    combination of host/device endpoints, in place, and a partial overlap."""
    import torch
    from gpu_util import from_dev, to_dev
    isz = np.dtype(oracle.NP_DTYPE[t]).itemsize
    n = (48 << 20) // isz + 5
    src = oracle.fill(t, 1, 21, n)
    for tgt_host, src_host in ((True, True), (True, False), (False, True)):
        s = src if src_host else to_dev(torch, src)
        if tgt_host:
            d = np.zeros_like(src)
        else:
            d = to_dev(torch, np.zeros_like(src))
        shm.to_all(t, "sum", d, s, n, 0, 0, 1)
        assert shm.last_error() == 0
        got = d if tgt_host else from_dev(d, src.dtype)
        assert got.tobytes() == src.tobytes(), (tgt_host, src_host)
    buf = src.copy()
    shm.to_all(t, "prod", buf, buf, n, 0, 0, 1)                     # in place, host
    assert buf.tobytes() == src.tobytes()
    big = np.concatenate([src, src[:7]])
    shm.to_all(t, "sum", big[3:].ctypes.data, big.ctypes.data, n, 0, 0, 1)   # overlap
    assert big[3:3 + n].tobytes() == src.tobytes()


def test_host_register_heap_segment(cuda, shm, oracle):
    """shmemx_host_register on one page-aligned host block carved into source
    and target (the reference's posix_memalign'd heap segment,
    comms-inline.h:752-769): the arrays inside take the pinned pipeline, across
    several 16 MiB chunks, and the results stay exact; unregistering an
    unknown range is EINVAL."""
    import mmap
    n = (40 << 20) // 8 + 3
    seg = mmap.mmap(-1, 2 * n * 8 + 4096)                   # page-aligned, pageable
    base = np.frombuffer(seg, dtype=np.uint8)
    src = base[:n * 8].view(np.float64)
    tgt = base[n * 8 + 8:n * 8 + 8 + n * 8].view(np.float64)   # 8-byte aligned, as dlmalloc
    src[:] = oracle.fill("double", 1, 5, n)
    shm.host_register(base, base.nbytes)
    try:
        for op in ("sum", "max"):
            tgt[:] = 0
            shm.to_all("double", op, tgt, src, n, 0, 0, 1)
            assert shm.last_error() == 0
            assert tgt.tobytes() == src.tobytes()
    finally:
        shm.host_unregister(base)
    with pytest.raises(shm.ShmemError):
        shm.host_unregister(base)
    del src, tgt, base
    seg.close()


def test_c_program_isx_verification(cuda, tmp_path):
    """A plain C99 program (examples/isx_verify.c) linked against the library:
    the reference's ISx verification (isx.c:615-624) with static host arrays,
    plus double sum / long xor checks, run as its own process."""
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libdir = os.path.join(repo, "openshmem-async_amd")
    exe = tmp_path / "isx_verify"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(repo, "include"),
                    os.path.join(repo, "examples", "isx_verify.c"), "-L", libdir,
                    "-lshmem_reduce_mi355x", f"-Wl,-rpath,{libdir}", "-o", str(exe)], check=True)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ISx verification passed" in out.stdout


def test_debug_symmetry_check(cuda, tmp_path):
    """$SHMEMX_DEBUG=1 makes the wrappers' --enable-debug checks live
    (reduce-op.c:379-381, utils.h:98-116): the C program's static arrays (the
    reference's symmetric globals) and shmem_malloc blocks pass; a torch
    tensor as target or source is FATAL with the reference's message."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libdir = os.path.join(repo, "openshmem-async_amd")
    exe = tmp_path / "isx_verify"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(repo, "include"),
                    os.path.join(repo, "examples", "isx_verify.c"), "-L", libdir,
                    "-lshmem_reduce_mi355x", f"-Wl,-rpath,{libdir}", "-o", str(exe)], check=True)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["SHMEMX_DEBUG"] = "1"
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ISx verification passed" in out.stdout
    for args, pos in (("t, a", 1), ("b + 8, t", 2)):
        code = (f"import sys, torch; sys.path.insert(0, {libdir!r}); import shmem_mi355x as s; "
                "s.init(); a = s.malloc(8 * 64); b = s.malloc(8 * 64); "
                "s.to_all('double', 'sum', b, a, 64, 0, 0, 1); print('heap ok', flush=True); "
                "t = torch.zeros(64, dtype=torch.float64, device='cuda'); "
                f"s.to_all('double', 'sum', {args}, 63, 0, 0, 1)")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                           timeout=120)
        assert "heap ok" in r.stdout, r.stderr[-2000:]
        assert r.returncode != 0
        assert f"FATAL: shmem_double_sum_to_all(), argument #{pos} @ " in r.stderr, r.stderr[-2000:]
        assert "is not symmetric" in r.stderr


@pytest.mark.parametrize("n", [1, 7, 4096, 32768])
def test_host_small_messages_bounce_path(cuda, shm, oracle, n):
    """Host arrays up to 256 KiB take the page-locked bounce path; mixed
    host/device endpoints included."""
    import torch
    src = oracle.fill("int", 1, n, n)
    tgt = np.zeros_like(src)
    shm.to_all("int", "xor", tgt, src, n, 0, 0, 1)
    assert shm.last_error() == 0 and tgt.tobytes() == src.tobytes()
    d = torch.zeros(n, dtype=torch.int32, device="cuda")
    shm.to_all("int", "max", d, src, n, 0, 0, 1)                 # host -> device
    assert d.cpu().numpy().tobytes() == src.tobytes()
    tgt[:] = 0
    shm.to_all("int", "min", tgt, d, n, 0, 0, 1)                 # device -> host
    assert tgt.tobytes() == src.tobytes()
    # in place and partially overlapping host arrays (the one-member set is a
    # copy of the source as it was on entry, reduce-op.c:187-216)
    buf = np.concatenate([src, np.zeros(5, src.dtype)])
    shm.to_all("int", "sum", buf, buf, n, 0, 0, 1)
    assert shm.last_error() == 0 and buf[:n].tobytes() == src.tobytes()
    shm.to_all("int", "sum", buf[3:], buf, n, 0, 0, 1)
    assert shm.last_error() == 0 and buf[3:n + 3].tobytes() == src.tobytes()
    # fresh data through the same bounce buffers on every call
    for k in range(3):
        fresh = oracle.fill("int", 10 + k, n, n)
        shm.to_all("int", "or", tgt, fresh, n, 0, 0, 1)
        assert tgt.tobytes() == fresh.tobytes()


def test_trace_facility(cuda, tmp_path):
    """$SHMEM_LOG_LEVELS / $SHMEM_LOG_FILE as the reference's utils/trace.c:
    facility names with ",:;" delimiters, the "%-8.8f PE %d: LEVEL: msg"
    line, and the reference's own reduction messages (reduce-op.c:199-210)."""
    import re
    import subprocess
    import sys
    log = tmp_path / "shmem.log"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, numpy as np, torch; sys.path.insert(0, %r); import shmem_mi355x as s; "
            "s.init(); a = np.arange(10.0); b = np.zeros(10); "
            "s.to_all('double', 'sum', b, a, 10, 0, 0, 1); s.to_all('double', 'sum', a, a, 10, 0, 0, 1); "
            "print(hex(b.ctypes.data), hex(a.ctypes.data)); "
            "p = s.malloc(1 << 20); s.free(p); s.finalize()") % os.path.join(repo, "openshmem-async_amd")
    env = dict(os.environ, SHMEM_LOG_LEVELS="reduction;Init,memory", SHMEM_LOG_FILE=str(log))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    text = log.read_text()
    lines = text.strip().splitlines()
    assert all(re.match(r"^\d+\.\d{8} PE 0: [A-Z]+: ", ln) for ln in lines), text
    assert any(": INIT: PE 0 of 1" in ln for ln in lines)
    # the reference's messages name the caller's host arrays (not staging
    # buffers), and an in-place call counts as overlapping (OVERLAP_CHECK)
    b_addr, a_addr = out.stdout.split()[-2:]
    assert any(f"target ({b_addr}) and source ({a_addr}, size 80) do not overlap" in ln
               for ln in lines), text
    assert any(f"target ({a_addr}) and source ({a_addr}, size 80) overlap, using temporary target"
               in ln for ln in lines), text
    assert any(": MEMORY: shmem_malloc(1048576" in ln for ln in lines)
    assert not any(": BARRIER: " in ln for ln in lines)          # not requested
