"""GPU tests of the neighbouring collectives and the HBM symmetric heap
 through the C ABI, against the oracle restatements.

In process (one PE): the single-member semantics — broadcast leaves the root's
target alone, [f]collect copies, barrier returns — for host and device
buffers, error codes, and shmem_malloc/align/realloc/free feeding a
device-resident reduction.  In a child process with SHMEMX_FORCE_COLLECTIVE=1
the RCCL paths (ncclBroadcast, ncclAllGather, the count exchange, the barrier
all-reduce) run on a one-rank communicator."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bits", [32, 64])
def test_single_pe_semantics(cuda, shm, oracle, bits):
    import torch
    dt = np.int32 if bits == 32 else np.int64
    n = 1001
    src = np.arange(n, dtype=dt) * 3 - 7
    for dev in (False, True):
        s = torch.from_numpy(src).cuda() if dev else src
        t = torch.full((n,), -1, dtype=torch.from_numpy(src).dtype, device="cuda") if dev \
            else np.full(n, -1, dtype=dt)
        shm.broadcast(bits, t, s, n, 0, 0, 0, 1)
        assert shm.last_error() == 0
        got = t.cpu().numpy() if dev else t
        want = oracle.broadcast_sim(src[None, :], np.full((1, n), -1, dt), 0, 0, 0, 1)[0]
        assert (got == want).all() and (got == -1).all()          # root untouched
        for fn in (shm.fcollect, shm.collect):
            t2 = torch.zeros(n, dtype=t.dtype if dev else torch.int64, device="cuda") if dev \
                else np.zeros(n, dtype=dt)
            fn(bits, t2, s, n, 0, 0, 1)
            assert shm.last_error() == 0
            got = t2.cpu().numpy() if dev else t2
            want = oracle.collect_sim(src[None, :], [n], np.zeros((1, n), dt), 0, 0, 1)[0]
            assert (got == want).all()
    shm.barrier(0, 0, 1)
    assert shm.last_error() == 0
    shm.barrier_all()
    assert shm.last_error() == 0


def test_collective_errors(cuda, shm):
    t = np.zeros(4, np.int64)
    shm.broadcast(64, t, t, 4, 1, 0, 0, 1)        # root index outside the set
    assert shm.last_error() == 1
    shm.fcollect(64, t, t, 4, 0, 0, 2)            # set beyond npes
    assert shm.last_error() == 1
    shm.barrier(1, 0, 1)
    assert shm.last_error() == 1


def test_symmetric_heap_on_hbm(cuda, shm, oracle):
    import torch
    n = 1 << 20
    a = shm.malloc(n * 8)
    b = shm.align(4096, n * 8)
    assert a and b and b % 4096 == 0
    src = oracle.fill("double", 1, 9, n)
    # the heap is device memory: fill it, reduce device-resident, read back
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(a, src.ctypes.data, n * 8, 1) == 0          # H2D
    shm.to_all("double", "sum", b, a, n, 0, 0, 1)
    out = np.zeros(n)
    assert hip.hipMemcpy(out.ctypes.data, b, n * 8, 2) == 0          # D2H
    assert out.tobytes() == src.tobytes()
    c = shm.realloc(a, 2 * n * 8)                                    # grow keeps the data
    assert c
    out2 = np.zeros(n)
    assert hip.hipMemcpy(out2.ctypes.data, c, n * 8, 2) == 0
    assert out2.tobytes() == src.tobytes()
    shm.free(c)
    shm.free(b)
    assert shm.last_error() == 0
    assert shm.malloc(0) == 0


def test_collectives_rccl_paths_one_rank(cuda):
    env = dict(os.environ, SHMEMX_FORCE_COLLECTIVE="1")
    here = os.path.dirname(os.path.abspath(__file__))
    out = subprocess.run([sys.executable, os.path.join(here, "gpu_collectives_p1.py")],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout + out.stderr
