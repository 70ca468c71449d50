"""Does writing the fold's result over its own input (acc = acc + in, the
reference's in-place inner fold) cost against writing a third array?  32 Mi
doubles, HIP events, 3 * n * 8 bytes per launch."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
os.environ.setdefault("SHMEMX_HEAP_MEMORY", "device")   # device addresses from shmem_malloc
import shmem_mi355x as shm  # noqa: E402

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
s = torch.cuda.Stream()
for n in (16 << 20, 32 << 20, 64 << 20):
    blk = [shm.malloc(n * 8) for _ in range(3)]
    a, b, c = blk

    def timeit(fn, reps=30):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    for r in range(2):
        t_in = timeit(lambda: shm.fold("double", "sum", a, b, n, s.cuda_stream))
        t_out = timeit(lambda: shm.fold_n("double", "sum", c, [a, b], n, s.cuda_stream))
        print(f"n={n >> 20}Mi round {r}: in place {t_in * 1e6:7.1f} us {3 * n * 8 / t_in / 1e9:7.1f} GB/s"
              f" | out of place {t_out * 1e6:7.1f} us {3 * n * 8 / t_out / 1e9:7.1f} GB/s", flush=True)
    for p in blk:
        shm.free(p)
