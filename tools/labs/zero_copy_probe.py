"""Can the fold kernel stream page-locked host arrays over PCIe directly
(zero-copy), instead of staging them through HBM in chunks?  Times the
1-input fold (the PE_size = 1 copy) and the 2-input fold with both operands in
pinned host memory, against the staged blocking call, 32 Mi doubles."""
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
stream = shm.get_stream()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


for unroll in (4, 2, 8):
    shm.set_fold_tuning(0, -1, unroll)
    t1 = timed(lambda: shm.fold_n("double", "sum", tgt, [src], n, stream))
    ok1 = bool(torch.equal(tgt, src))
    print(f"unroll {unroll}: zero-copy copy (1-input fold) {t1 * 1e3:.2f} ms "
          f"{n * 8 / t1 / 2**30:.1f} GiB/s, PCIe {2 * n * 8 / t1 / 1e9:.1f} GB/s ok={ok1}", flush=True)
shm.set_fold_tuning(0, -1, 4)
for nt in (0, 1, 2, 3):
    shm.set_fold_tuning(0, nt, 4)
    t1 = timed(lambda: shm.fold_n("double", "sum", tgt, [src], n, stream))
    print(f"nt {nt}: zero-copy copy {t1 * 1e3:.2f} ms", flush=True)
shm.set_fold_tuning(0, -1, 4)
acc = src.clone().pin_memory()
t2 = timed(lambda: shm.fold("double", "sum", acc, src, n, stream), reps=3)
print(f"zero-copy 2-input fold acc += in {t2 * 1e3:.2f} ms, PCIe {3 * n * 8 / t2 / 1e9:.1f} GB/s",
      flush=True)
t3 = timed(lambda: shm.to_all("double", "sum", tgt, src, n, 0, 0, 1))
print(f"staged blocking call {t3 * 1e3:.2f} ms {n * 8 / t3 / 2**30:.1f} GiB/s", flush=True)
