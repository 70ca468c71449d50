"""The library's copy (the PE_size = 1 call's kernel, reduce-op.c:213-216) at
256 and 512 MiB: HIP events over 20 back-to-back launches, on torch arrays
and on symmetric-heap blocks; run under rocprofv3 --kernel-trace for each
launch's kernel name and duration (tools/trace_by_grid.py)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
os.environ.setdefault("SHMEMX_HEAP_MEMORY", "device")
import shmem_mi355x as shm  # noqa: E402

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
s = torch.cuda.Stream()
for mib in (256, 512):
    n = mib << 17                           # doubles
    src_t = torch.rand(n, dtype=torch.float64, device="cuda")
    dst_t = torch.empty_like(src_t)
    hs, ht = shm.malloc(n * 8), shm.malloc(n * 8)
    shm.memcpy(hs, src_t, n * 8)
    for where, (dst, src) in (("torch", (dst_t, src_t)), ("heap", (ht, hs))):
        for _ in range(3):
            shm.fold_n("double", "sum", dst, [src], n, s.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            shm.fold_n("double", "sum", dst, [src], n, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 20 * 1e-3
        print(f"copy {mib} MiB {where}: {t * 1e6:.1f} us/launch, {2 * n * 8 / t / 1e12:.3f} TB/s", flush=True)
    shm.free(ht)
    shm.free(hs)
    del src_t, dst_t
shm.finalize()
