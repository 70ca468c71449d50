"""HBM rate of the P-input fold (the fold step of A2A / DIRECT / GATHER, and
the 1-input copy of PE_size = 1) on one GPU: (P + 1) * n * 8 bytes per launch
over the launch time, double sum, n = 16 Mi (and 4 Mi) elements per input;
"runtime" = shmemx_fold_n_on_stream (input k + 1 loaded after folding input
k), "peers" = shmemx_fold_n_peers_on_stream (every input's loads in flight
first: DIRECT's and SIGNAL's fold, built for inputs across xGMI links), here
on local HBM."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
N = 16 * 1024 * 1024
ins = [torch.rand(N, dtype=torch.float64, device="cuda") for _ in range(16)]
outbuf = torch.empty(N, dtype=torch.float64, device="cuda")
s = torch.cuda.Stream()
for n in (N, N // 4):
    out = outbuf[:n]
    for P in (1, 2, 3, 4, 6, 8, 12, 16):
        row = []
        for peers in (False, True):
            args = ("double", "sum", out, [x[:n] for x in ins[:P]], n, s.cuda_stream, peers)
            for _ in range(3):
                shm.fold_n(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            reps = 20
            for _ in range(reps):
                shm.fold_n(*args)
            e1.record(s)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / reps * 1e-3
            row.append(f"{'peers' if peers else 'runtime'} {t * 1e6:8.1f} us {(P + 1) * n * 8 / t / 1e9:7.1f} GB/s")
        print(f"n={n:9d} P={P:2d}: " + "   ".join(row), flush=True)
