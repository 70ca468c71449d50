"""The resident service workgroup (openshmem-async_amd/csrc/service.hip): a
blocking one-member call (reduce-op.c:213-216, write_to = source) of at most
32 KiB is done by a workgroup that stays on the GPU polling a host-coherent
mailbox, with no kernel launch.  These tests hold it to the same bytes as the
launched copy, check that it only runs when the streams it is ordered after
are idle, that it comes back after idling out, that it never keeps the
device busy for long, and that a process may end with it up."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

KIB32 = 32 * 1024


def _bytes_of(t, a):
    return a.tobytes()


@pytest.mark.parametrize("t", ["short", "int", "long", "float", "double", "complexd", "complexf"])
def test_service_copies_every_size_and_alignment(cuda, shm, oracle, t):
    """Sizes from one element to 32 KiB and one element past it, source and
    target at every offset class the copy distinguishes (16, 8, 4, 2 bytes):
    bit-exact; up to 32 KiB the service served the call, past it the launched
    copy did."""
    import torch
    esz = np.dtype(oracle.NP_DTYPE[t]).itemsize
    big = torch.zeros(KIB32 // 4 + 64, dtype=torch.int32, device="cuda")   # raw bytes, 16-B aligned
    out = torch.zeros_like(big)
    base_s, base_d = big.data_ptr(), out.data_ptr()
    shm.init()
    shm.service_stats(reset=True)
    served = 0
    for n in (1, 2, 3, 7, 63, 255, 256, 1000, KIB32 // esz - 1, KIB32 // esz, KIB32 // esz + 1):
        for off_s, off_d in ((0, 0), (esz, esz), (0, esz), (3 * esz, esz)):
            src = oracle.fill(t, 1, 1000 + n + off_s, n)
            raw = np.frombuffer(src.tobytes(), np.uint8)
            big.view(torch.uint8)[off_s:off_s + raw.size].copy_(torch.from_numpy(raw.copy()))
            out.view(torch.uint8).fill_(0xAB)
            torch.cuda.synchronize()
            shm.to_all(t, "sum", base_d + off_d, base_s + off_s, n, 0, 0, 1)
            assert shm.last_error() == 0
            got = out.view(torch.uint8)[off_d:off_d + raw.size].cpu().numpy()
            assert got.tobytes() == raw.tobytes(), (t, n, off_s, off_d)
            # nothing past the target was touched
            after = out.view(torch.uint8)[off_d + raw.size:off_d + raw.size + 16].cpu().numpy()
            assert (after == 0xAB).all(), (t, n, off_s, off_d)
            if n * esz <= KIB32:
                served += 1
    st = shm.service_stats(reset=True)
    assert st["served"] == served, st
    assert st["launches"] >= 1


def test_service_ordered_after_the_default_stream(cuda, shm):
    """A kernel on the legacy default stream still writing the source when
    the blocking call starts: the call sees its bytes (the service notices
    the stream busy and the host waits for it before posting, as the launched
    copy would wait for it in stream order), and the calls after it go
    straight to the mailbox again: nothing the library did leaves a stream
    looking busy (a launch on the blocking library stream would, for 12-31
    us, and every next back-to-back call would then launch too)."""
    import torch
    shm.init()
    n = 512
    big = torch.zeros(1 << 27, dtype=torch.float64, device="cuda")   # 1 GiB
    dst = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    shm.service_stats(reset=True)
    for rep in range(5):
        big.fill_(float(rep + 1))          # ~0.2 ms on the default stream
        shm.to_all("double", "sum", dst, big, n, 0, 0, 1)
        assert shm.last_error() == 0
        assert (dst.cpu().numpy() == rep + 1).all(), rep
    st = shm.service_stats(reset=True)
    assert st["null_stream_busy"] >= 1 and st["served"] == 5, st
    big.fill_(7.0)
    t0 = time.perf_counter()
    for _ in range(200):
        shm.to_all("double", "sum", dst, big, n, 0, 0, 1)
    dt = time.perf_counter() - t0
    st = shm.service_stats(reset=True)
    assert st["served"] == 200 and st["null_stream_busy"] <= 2 and st["library_stream_busy"] == 0, st
    assert (dst.cpu().numpy() == 7.0).all()
    assert dt < 0.02, dt   # 200 calls at mailbox speed (with the fill's wait)


def test_service_comes_back_after_idling_out(cuda, shm, oracle):
    """Calls 1 ms apart (the workgroup leaves after 200 us idle): every call
    correct, served by a fresh launch each time."""
    import torch
    shm.init()
    n = 1024
    src = torch.from_numpy(oracle.fill("long", 1, 5, n)).cuda()
    dst = torch.zeros_like(src)
    torch.cuda.synchronize()
    shm.service_stats(reset=True)
    for k in range(20):
        time.sleep(0.001)
        src.add_(1)
        torch.cuda.synchronize()
        shm.to_all("long", "sum", dst, src, n, 0, 0, 1)
        assert torch.equal(dst, src), k
    st = shm.service_stats(reset=True)
    assert st["served"] == 20 and st["launches"] >= 10, st


def test_service_back_to_back_calls_one_launch(cuda, shm):
    """Back-to-back small calls are served by one resident workgroup, and a
    device-wide synchronisation right after them waits for it only briefly
    (it leaves 200 us after its last request)."""
    import torch
    shm.init()
    src = torch.arange(8, dtype=torch.int64, device="cuda")
    dst = torch.zeros_like(src)
    torch.cuda.synchronize()
    shm.service_stats(reset=True)
    for _ in range(2000):
        shm.to_all("long", "sum", dst, src, 8, 0, 0, 1)
    st = shm.service_stats(reset=True)
    assert st["served"] == 2000 and st["launches"] <= 20, st
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 0.05
    assert torch.equal(dst, src)


def test_service_host_arrays(cuda, shm, oracle):
    """Host arrays at one PE take the page-locked bounce buffers; the service
    copies between them on the GPU."""
    shm.init()
    shm.service_stats(reset=True)
    for t, n in (("double", 1), ("int", 1024), ("long", 4096), ("short", 333)):
        src = oracle.fill(t, 1, 71, n)
        tgt = np.zeros_like(src)
        shm.to_all(t, "sum", tgt, src, n, 0, 0, 1)
        assert shm.last_error() == 0 and tgt.tobytes() == src.tobytes(), (t, n)
    assert shm.service_stats(reset=True)["served"] == 4


def test_service_off_switch(tmp_path):
    """$SHMEMX_SERVICE=0: the same calls, none served."""
    code = ("import sys; sys.path.insert(0, %r); import numpy as np, torch, shmem_mi355x as shm\n"
            "torch.cuda.set_device(0); shm.init()\n"
            "s = torch.arange(64, dtype=torch.float64, device='cuda'); d = torch.zeros_like(s)\n"
            "torch.cuda.synchronize()\n"
            "for _ in range(10): shm.to_all('double', 'sum', d, s, 64, 0, 0, 1)\n"
            "assert torch.equal(d, s)\n"
            "st = shm.service_stats(); assert st['served'] == 0 and st['launches'] == 0, st\n"
            "print('ok')\n") % os.path.join(REPO, "openshmem-async_amd")
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SHMEMX_SERVICE="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_service_process_exits_with_it_up(tmp_path):
    """A program that ends right after a small call (no shmem_finalize, the
    workgroup still resident) exits cleanly and promptly: the library's exit
    handler tells it to leave and waits for it."""
    code = ("import sys; sys.path.insert(0, %r); import numpy as np, torch, shmem_mi355x as shm\n"
            "torch.cuda.set_device(0); shm.init()\n"
            "s = torch.arange(64, dtype=torch.float64, device='cuda'); d = torch.zeros_like(s)\n"
            "torch.cuda.synchronize()\n"
            "shm.to_all('double', 'sum', d, s, 64, 0, 0, 1)\n"
            "assert shm.service_stats()['served'] == 1\n"
            "print('ok', flush=True)\n") % os.path.join(REPO, "openshmem-async_amd")
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
    assert time.time() - t0 < 100


def test_service_does_not_hold_up_the_default_stream(cuda, shm):
    """While the workgroup is resident (between small calls, before its idle
    exit), work on the legacy default stream (PyTorch's) runs at once: the
    service's stream is a high-priority non-blocking one, which HIP's null
    stream does not wait for (tools/queue_lab.hip).  Blocked, every op below
    would wait ~200 us for the idle exit."""
    import torch
    shm.init()
    src = torch.arange(16, dtype=torch.int64, device="cuda")
    dst = torch.zeros_like(src)
    x = torch.zeros(16, device="cuda")
    torch.cuda.synchronize()
    shm.service_stats(reset=True)
    ts = []
    for _ in range(50):
        shm.to_all("long", "sum", dst, src, 16, 0, 0, 1)
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()   # (device-wide: also waits for the resident workgroup)
        ts.append(time.perf_counter() - t0)
    ts2 = []
    for _ in range(50):
        shm.to_all("long", "sum", dst, src, 16, 0, 0, 1)
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.current_stream().synchronize()   # the default stream alone
        ts2.append(time.perf_counter() - t0)
    st = shm.service_stats(reset=True)
    assert st["served"] == 100, st
    assert float(x[0]) == 100.0
    ts2.sort()
    assert ts2[len(ts2) // 2] < 100e-6, ts2[len(ts2) // 2]
