"""Host-resident end-to-end rate (32 Mi doubles, PE_size = 1) for one setting
of SHMEMX_COPY_THREADS / SHMEMX_STAGE_CHUNK_MB (set by the caller)."""
import os, statistics, sys, time
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm
torch.cuda.set_device(0); shm.init_attr(0, 1, 0, None)
n = 32 * 1024 * 1024
src = np.random.default_rng(1).random(n) + 1; tgt = np.zeros(n)
shm.to_all("double", "sum", tgt, src, n, 0, 0, 1)
ts = []
for _ in range(int(os.environ.get("E2E_REPS", "7"))):
    t0 = time.perf_counter(); shm.to_all("double", "sum", tgt, src, n, 0, 0, 1); ts.append(time.perf_counter() - t0)
t = statistics.median(ts)
import ctypes  # noqa: E402


def node_of(a):
    """NUMA node of the array's first page (move_pages query, x86-64 syscall 279)."""
    libc = ctypes.CDLL(None, use_errno=True)
    page = ctypes.c_void_p(a.ctypes.data & ~4095)
    status = ctypes.c_int(-1)
    libc.syscall(279, 0, ctypes.c_ulong(1), ctypes.byref(page), None, ctypes.byref(status), 0)
    return status.value
print(f"threads={os.environ.get('SHMEMX_COPY_THREADS','dflt')} chunkMB={os.environ.get('SHMEMX_STAGE_CHUNK_MB','dflt')} "
      f"nodes src {node_of(src)} tgt {node_of(tgt)} cpu {os.sched_getaffinity(0).__len__()} "
      f"{t*1e3:.2f} ms {n*8/t/2**30:.1f} GiB/s (min {n*8/max(ts)/2**30:.1f} max {n*8/min(ts)/2**30:.1f}) "
      f"ok={bool((tgt==src).all())}", flush=True)
