"""The cold mid-size fold (VERDICT r02 "what's weak" #2): why does the float
sum 2-input fold run at 36-47 % of HBM peak at 4-16 Mi elements when every
step is preceded by a cache flush, and 79 % at 64 Mi?

Two candidate causes:
  * the flush itself: bench.py's cold curve rewrites a 1 GiB scratch before
    every step, which leaves up to 256 MiB of dirty lines in the Infinity
    Cache (MALL); the timed fold then pays for writing them back to HBM;
  * the fold's cache policy: non-temporal loads + stores only when the
    working set is >= 256 MiB (fold_kernels.hip kNtThresholdBytes).

For each flush kind, size and policy the fold is launched `reps` times, each
launch after its own flush, timed alone with HIP events on the stream:
  fill   scratch.fill_(k): 1 GiB of writes (the bench's flush until r03)
  read   a read-only sweep of the 1 GiB scratch (evicts, leaves nothing dirty)
  fill+read  fill, then the read sweep (the dirty lines are written back
         before the timed launch starts)
  warm   no flush, back to back
usage: cold_midsize_probe.py [reps] [flush,...] [n,...] [nt,...] (nt -1 = the
shipped choice).  Prints one {"config": ...} line per (flush, n, nt) in launch order, so
tools/summarize_pmc.py can attach rocprofv3 FETCH_SIZE / WRITE_SIZE passes
(run under rocprofv3 with one counter per pass).
"""
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
flushes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fill", "read", "fill+read", "warm"]
sizes = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1 << 22, 1 << 24, 1 << 26]
nts = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 3]   # -1 = shipped auto
torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
st = torch.cuda.Stream()
sp = st.cuda_stream
scratch = torch.empty(1 << 27, dtype=torch.float64, device="cuda")   # 1 GiB
sink = torch.empty(1, dtype=torch.float64, device="cuda")


def flush(kind, k):
    with torch.cuda.stream(st):
        if "fill" in kind:
            scratch.fill_(k)
        if "read" in kind:
            torch.sum(scratch, dim=0, out=sink)


for kind in flushes:
    for n in sizes:
        acc = torch.rand(n, dtype=torch.float32, device="cuda") + 1
        inp = torch.rand(n, dtype=torch.float32, device="cuda") + 1
        for nt in nts:
            shm.set_fold_tuning(0, nt, 4)
            torch.cuda.synchronize()
            times = []
            for k in range(reps):
                if kind != "warm":
                    flush(kind, k)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                shm.fold("float", "sum", acc, inp, n, sp)
                e1.record(st)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) * 1e-3)
            t = statistics.median(times)
            print(json.dumps({"config": f"{kind} n={n} nt={nt}", "flush": kind, "n": n, "nt": nt,
                              "alg_bytes": 12 * n, "median_us": round(t * 1e6, 2),
                              "TBps": round(12 * n / t / 1e12, 3),
                              "frac_of_8TBps": round(12 * n / t / 8e12, 3)}), flush=True)
        del acc, inp
shm.set_fold_tuning(0, -1, 4)
shm.finalize()
