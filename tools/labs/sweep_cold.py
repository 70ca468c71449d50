"""Cold-cache check of the fold's cache policy at several sizes: before every
timed launch a 1 GiB scratch buffer is rewritten (evicts L2 and the 256 MiB
Infinity Cache), so each launch streams from HBM.  Compared with the
back-to-back (warm) rate of the same config."""
import json, os, statistics, sys
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm
torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
st = torch.cuda.Stream(); sp = st.cuda_stream
scratch = torch.empty(1 << 27, dtype=torch.float64, device="cuda")  # 1 GiB
out = {}
for n in (1 << 24, 1 << 25, 1 << 26):
    acc = torch.rand(n, dtype=torch.float64, device="cuda") + 1
    inp = torch.rand(n, dtype=torch.float64, device="cuda") + 1
    row = {}
    for (nt, u) in ((0, 4), (1, 2), (1, 4), (3, 2), (3, 4)):
        shm.set_fold_tuning(0, nt, u)
        cold, warm = [], []
        for rep in range(7):
            with torch.cuda.stream(st):
                scratch.fill_(rep)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(st); shm.fold("double", "sum", acc, inp, n, sp); e.record(st)
            torch.cuda.synchronize(); cold.append(s.elapsed_time(e) * 1e-3)
            s.record(st)
            for _ in range(10): shm.fold("double", "sum", acc, inp, n, sp)
            e.record(st); torch.cuda.synchronize(); warm.append(s.elapsed_time(e) * 1e-4)
        row[f"nt{nt}_u{u}"] = {"cold_GBps": round(24 * n / statistics.median(cold) / 1e9, 1),
                               "warm_GBps": round(24 * n / statistics.median(warm) / 1e9, 1)}
    out[f"n={n}"] = row
    del acc, inp
print(json.dumps(out, indent=1))
