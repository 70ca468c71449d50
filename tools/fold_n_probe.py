"""HBM rate of the P-input fold (the fold step of A2A / DIRECT / GATHER, and
the 1-input copy of PE_size = 1) on one GPU: (P + 1) * n * 8 bytes per launch
over the launch time, double sum, n = 16 Mi elements per input."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
n = 16 * 1024 * 1024
ins = [torch.rand(n, dtype=torch.float64, device="cuda") for _ in range(16)]
out = torch.empty(n, dtype=torch.float64, device="cuda")
s = torch.cuda.Stream()
for P in (1, 2, 3, 4, 6, 8, 12, 16):
    for _ in range(3):
        shm.fold_n("double", "sum", out, ins[:P], n, s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    reps = 20
    for _ in range(reps):
        shm.fold_n("double", "sum", out, ins[:P], n, s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    print(f"P={P:2d}: {t * 1e6:8.1f} us  {(P + 1) * n * 8 / t / 1e9:7.1f} GB/s", flush=True)
