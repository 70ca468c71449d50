"""Child process for test_gpu_collectives.py: RCCL paths of broadcast,
fcollect, collect and barrier on a one-rank communicator
(SHMEMX_FORCE_COLLECTIVE=1).  Prints "ok" or raises."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

assert os.environ.get("SHMEMX_FORCE_COLLECTIVE") == "1"
torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
for bits, dt in ((32, torch.int32), (64, torch.int64)):
    for n in (1, 1000, 1 << 20):
        s = torch.arange(n, dtype=dt, device="cuda") * 5 + 1
        t = torch.full((n,), -1, dtype=dt, device="cuda")
        shm.broadcast(bits, t, s, n, 0, 0, 0, 1)
        assert shm.last_error() == 0 and bool((t == -1).all()), "root target must stay"
        for fn in (shm.fcollect, shm.collect):
            t = torch.zeros(n, dtype=dt, device="cuda")
            fn(bits, t, s, n, 0, 0, 1)
            torch.cuda.synchronize()
            assert shm.last_error() == 0 and torch.equal(t, s), fn.__name__
            h = np.zeros(n, dtype=np.int32 if bits == 32 else np.int64)
            fn(bits, h, s.cpu().numpy(), n, 0, 0, 1)                   # host buffers
            assert (h == s.cpu().numpy()).all(), fn.__name__ + " host"
shm.barrier(0, 0, 1)
shm.barrier_all()
assert shm.last_error() == 0
print("ok")
# verify over a one-rank communicator (RCCL all-gather of the checksums)
x = torch.arange(4097, dtype=torch.float64, device="cuda")
assert shm.verify("double", x, 4097, 0, 0, 1)
print("ok")
