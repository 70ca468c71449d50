"""Config-4 shape (long and/or/xor, 64 Mi elements, the 2-input fold at
N = 1): torch-allocated operands (as bench.py's config extras had them) vs
operands in the symmetric heap (shmem_malloc, as the headline has them),
and the double sum at 32 Mi and 64 Mi on the heap for scale.  HIP events,
median of 5 x 20 launches; TB/s = 3 * n * 8 B / launch."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
os.environ.setdefault("SHMEMX_HEAP_MEMORY", "device")   # device addresses from shmem_malloc
import shmem_mi355x as shm  # noqa: E402


def rate(t, op, acc, inp, n, s):
    for _ in range(3):
        shm.fold(t, op, acc, inp, n, s.cuda_stream)
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            shm.fold(t, op, acc, inp, n, s.cuda_stream)
        e1.record(s)
        e1.synchronize()
        res.append(e0.elapsed_time(e1) / 20 * 1e-3)
    dt = statistics.median(res)
    return 3 * n * 8 / dt / 1e12, dt * 1e6


def main():
    torch.cuda.set_device(0)
    shm.init_attr(0, 1, 0, None)
    s = torch.cuda.Stream()
    n = 64 * 1024 * 1024
    x = torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda")
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    for op in ("and", "xor"):
        tb, us = rate("long", op, y, x, n, s)
        print(f"torch arrays long {op} 64Mi: {tb:.2f} TB/s {us:.1f} us", flush=True)
    a, b = shm.malloc(n * 8), shm.malloc(n * 8)
    assert a and b
    shm.memcpy(a, x.data_ptr(), n * 8)
    shm.memcpy(b, x.data_ptr(), n * 8)
    torch.cuda.synchronize()
    for op in ("and", "xor"):
        tb, us = rate("long", op, b, a, n, s)
        print(f"heap arrays  long {op} 64Mi: {tb:.2f} TB/s {us:.1f} us", flush=True)
    for m in (32, 64):
        tb, us = rate("double", "sum", b, a, m * 1024 * 1024, s)
        print(f"heap arrays  double sum {m}Mi: {tb:.2f} TB/s {us:.1f} us", flush=True)


if __name__ == "__main__":
    main()
