"""Experiment (not part of the library): does the bench kernel's time depend on
where its two 256 MiB operands sit?  The 2-input double fold over 32 Mi
elements (the bench step) is timed with HIP events on its own stream for
  * torch: pairs of separately allocated torch tensors (what bench.py used);
  * heap:  pairs carved from the symmetric HBM heap (shmem_malloc), the
           layout the reference itself gives source/target (one heap segment,
           memory/symmem.c:168-227).
Each pair: 3 rounds x 30 launches, interleaved across pairs; avg us per launch.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
os.environ.setdefault("SHMEMX_HEAP_MEMORY", "device")   # device addresses from shmem_malloc
import shmem_mi355x as shm  # noqa: E402

N = 32 * 1024 * 1024
NB = N * 8


def main():
    torch.cuda.set_device(0)
    shm.init_attr(0, 1, 0, None)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    pairs = []
    for k in range(6):
        a = torch.rand(N, dtype=torch.float64, device="cuda") + 1
        b = torch.rand(N, dtype=torch.float64, device="cuda") + 1
        pairs.append((f"torch{k}", a, b, a.data_ptr(), b.data_ptr()))
    blocks = [shm.malloc(NB) for _ in range(12)]      # 3 GiB of the heap segment
    if not all(blocks):
        sys.exit("heap alloc failed")
    for blk in blocks:
        shm.memcpy(blk, pairs[0][1], NB)
    for k, (i, j) in enumerate([(0, 1), (2, 3), (4, 6), (5, 9), (7, 11), (10, 8)]):
        pairs.append((f"heap{k}", None, None, blocks[i], blocks[j]))
    torch.cuda.synchronize()
    res = {p[0]: [] for p in pairs}
    for rnd in range(3):
        for name, _, _, pa, pb in pairs:
            for _ in range(3):
                shm.fold("double", "sum", pa, pb, N, sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(30):
                shm.fold("double", "sum", pa, pb, N, sp)
            e1.record(stream)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / 30)
    for name, _, _, pa, pb in pairs:
        print(f"{name:7s} acc {pa:#x} in {pb:#x} delta {pb - pa:+#x}  "
              + "  ".join(f"{t:7.2f}" for t in res[name]) + " us", flush=True)


if __name__ == "__main__":
    main()
