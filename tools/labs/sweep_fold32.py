"""Variance-aware sweep at the bench size (32 Mi doubles, acc = acc + in):
every (nt mode, unroll) config, 7 interleaved rounds of 20 launches each,
median / min / max of the per-launch time.  One JSON object on stdout."""
import json, os, statistics, sys
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
st = torch.cuda.Stream(); sp = st.cuda_stream
n = 32 * 1024 * 1024
acc = torch.rand(n, dtype=torch.float64, device="cuda") + 1
inp = torch.rand(n, dtype=torch.float64, device="cuda") + 1
torch.cuda.synchronize()
K = 20
def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record(st)
    for _ in range(K): fn()
    e.record(st); torch.cuda.synchronize()
    return s.elapsed_time(e) / K * 1e-3
configs = [(0, nt, u) for nt in (0, 1, 2, 3) for u in (2, 4, 8)]
res = {c: [] for c in configs}
for rnd in range(7):
    for c in configs:
        shm.set_fold_tuning(*c)
        for _ in range(3): shm.fold("double", "sum", acc, inp, n, sp)
        res[c].append(timed(lambda: shm.fold("double", "sum", acc, inp, n, sp)))
out = {}
for c, ts in res.items():
    out[f"nt{c[1]}_u{c[2]}"] = {"med_GBps": round(24 * n / statistics.median(ts) / 1e9, 1),
                                "min_GBps": round(24 * n / max(ts) / 1e9, 1),
                                "max_GBps": round(24 * n / min(ts) / 1e9, 1)}
print(json.dumps(out, indent=1))
