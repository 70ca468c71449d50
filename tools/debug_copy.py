import os, sys
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd")); sys.path.insert(0, os.path.join(REPO, "oracle"))
import shmem_mi355x as shm, oracle
torch.cuda.set_device(0)
for t in ("double", "complexf", "complexd", "int", "float"):
    for n in (2048, 2049, 4096, 4097, 4103, 8199):
        src = oracle.fill(t, 1, 77, n)
        s = torch.from_numpy(src).cuda()
        for mode in ("fold1", "to_all", "fold3"):
            d = torch.zeros_like(s)
            if mode == "fold1":
                shm.fold_n(t, "sum", d, [s], n)
            elif mode == "to_all":
                shm.to_all(t, "sum", d, s, n, 0, 0, 1)
            else:
                z = torch.zeros_like(s)
                shm.fold_n(t, "sum", d, [s, z, z], n)
            torch.cuda.synchronize()
            got = d.cpu().numpy()
            bad = np.nonzero(got != src)[0]
            print(t, n, mode, "bad", len(bad), bad[:3], bad[-1:] if len(bad) else "", flush=True)
