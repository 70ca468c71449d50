"""Sweep the fold kernel's launch shape (grid cap, non-temporal mode, unroll)
at several sizes, acc = acc + in on doubles, against PyTorch's add_/copy_ as
device references.  Interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24); prints one JSON object."""
import json, os, statistics, sys
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
st = torch.cuda.Stream(); sp = st.cuda_stream
out = {}
for n in (1 << 20, 1 << 23, 1 << 25, 1 << 26):
    acc = torch.rand(n, dtype=torch.float64, device="cuda") + 1
    inp = torch.rand(n, dtype=torch.float64, device="cuda") + 1
    dst = torch.empty_like(acc)
    torch.cuda.synchronize()
    K = 20 if n >= 1 << 25 else 100

    def timed(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record(st)
        for _ in range(K):
            fn()
        e.record(st)
        torch.cuda.synchronize()
        return s.elapsed_time(e) / K * 1e-3

    configs = [(mb, nt, u) for mb in (0, 2048) for nt in (0, 1, 2, 3) for u in (2, 4)]
    res = {c: [] for c in configs}
    base = {"torch_add_": [], "torch_copy_": []}
    for rnd in range(3):
        for c in configs:
            shm.set_fold_tuning(*c)
            for _ in range(3):
                shm.fold("double", "sum", acc, inp, n, sp)
            res[c].append(timed(lambda: shm.fold("double", "sum", acc, inp, n, sp)))
        with torch.cuda.stream(st):
            base["torch_add_"].append(timed(lambda: acc.add_(inp)))
            base["torch_copy_"].append(timed(lambda: dst.copy_(inp)))
    row = {}
    for c, ts in res.items():
        t = statistics.median(ts)
        row[f"mb{c[0]}_nt{c[1]}_u{c[2]}"] = round(24 * n / t / 1e9, 1)
    for k, ts in base.items():
        t = statistics.median(ts)
        row[k] = round((24 if k == "torch_add_" else 16) * n / t / 1e9, 1)
    row["best"] = max((v, k) for k, v in row.items() if k.startswith("mb"))
    out[f"n={n}"] = row
    del acc, inp, dst
shm.set_fold_tuning(0, -1, 4)
print(json.dumps(out, indent=1))
