"""Host-resident end-to-end rate with page-locked arrays (32 Mi doubles,
PE_size = 1) for one $SHMEMX_STAGE_CHUNK_MB (set by the caller), plus the
raw PCIe rates of one direction alone and both at once for comparison."""
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
n = 32 * 1024 * 1024
src = (torch.rand(n, dtype=torch.float64) + 1).pin_memory()
tgt = torch.zeros(n, dtype=torch.float64).pin_memory()
shm.to_all("double", "sum", tgt, src, n, 0, 0, 1)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    shm.to_all("double", "sum", tgt, src, n, 0, 0, 1)
    ts.append(time.perf_counter() - t0)
t = statistics.median(ts)
ok = bool(torch.equal(tgt, src))
line = (f"chunkMB={os.environ.get('SHMEMX_STAGE_CHUNK_MB', 'dflt')} {t * 1e3:.2f} ms "
        f"{n * 8 / t / 2**30:.1f} GiB/s ok={ok}")
if os.environ.get("RAW") == "1":
    d = torch.empty(n, dtype=torch.float64, device="cuda")
    d2 = torch.empty(n, dtype=torch.float64, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 3

    def both():
        with torch.cuda.stream(s1):
            d.copy_(src, non_blocking=True)
        with torch.cuda.stream(s2):
            tgt.copy_(d2, non_blocking=True)
    h2d = timed(lambda: d.copy_(src, non_blocking=True))
    d2h = timed(lambda: tgt.copy_(d2, non_blocking=True))
    bi = timed(both)
    line += (f" | raw H2D {n * 8 / h2d / 1e9:.1f} GB/s, D2H {n * 8 / d2h / 1e9:.1f} GB/s, "
             f"both at once {2 * n * 8 / bi / 1e9:.1f} GB/s total ({bi * 1e3:.2f} ms)")
print(line, flush=True)
