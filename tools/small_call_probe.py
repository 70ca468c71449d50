"""Where a small blocking reduction's time goes on one MI355X (VERDICT r04
#5): BASELINE configs[0]'s call, shmem_int_sum_to_all, at nreduce 1, 1024 and
4096, each call timed alone from C (tools/libcalltimer.so), from symmetric-heap
operands (HBM) and from host arrays.  One PE; with $SHMEMX_FORCE_COLLECTIVE=1
the call runs the collective schedule with no peer to wait for: on the IPC
transport ($SHMEMX_TRANSPORT=ipc) DIRECT's fused one-shot launch, on the RCCL
transport a one-rank RCCL all-reduce.  Run it plain for the wall times and
under `rocprofv3 --kernel-trace --stats` for the kernels' own durations
(tools/gpu_steps.sh small_calls): the difference is launch, completion
signalling and host work.

    python tools/small_call_probe.py [calls]
Prints one JSON line: per (n, operands), the median / min / p90 microseconds.
"""
import json
import os
import statistics
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
sys.path.insert(0, REPO)
os.environ.setdefault("SHMEMX_HEAP_MEMORY", "device")
import shmem_mi355x as shm  # noqa: E402
import torch  # noqa: E402,F401
from bench import call_times_us  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
psync = np.full(128, -1, np.int64)
hs, ht = shm.malloc(4096 * 4), shm.malloc(4096 * 4)
out = {"transport": os.environ.get("SHMEMX_TRANSPORT", "rccl"),
       "force_collective": os.environ.get("SHMEMX_FORCE_COLLECTIVE", "0"), "calls": calls}
for n in (1, 1024, 4096):
    src = (np.arange(n, dtype=np.int32) % 977) + 5
    for where in ("heap", "host"):
        if where == "heap":
            shm.memcpy(hs, src, n * 4)
            s, t = hs, ht
        else:
            s, t = src.copy(), np.zeros(n, np.int32)
        ts = call_times_us("int", "sum", t, s, n, 0, 0, 1, psync, 20, calls)
        got = np.empty(n, np.int32)
        if where == "heap":
            shm.memcpy(got, ht, n * 4)
        else:
            got = t
        ts.sort()
        out[f"n{n}_{where}"] = {"median_us": round(statistics.median(ts), 2), "min_us": round(ts[0], 2),
                                "p90_us": round(ts[int(0.9 * len(ts))], 2),
                                "algo": shm.plan("int", "sum", n, 0, 0, 1, 0, 1, "auto").algo,
                                "correct": bool(np.array_equal(got, src)) and shm.last_error() == 0}
print(json.dumps(out), flush=True)
shm.free(ht)
shm.free(hs)
