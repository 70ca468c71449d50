"""The small one-member blocking call from Python and from C, with the
resident service workgroup (csrc/service.hip) or without it
($SHMEMX_SERVICE=0 in the environment), device and host operands: medians in
microseconds, plus the service counters.  Prints one JSON line.

    python tools/service_probe.py [reps]
"""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
sys.path.insert(0, REPO)
heap_mode = os.environ.get("SHMEMX_HEAP_MEMORY")
import shmem_mi355x as shm  # noqa: E402
import bench  # noqa: E402  (call_times_us: the C call timer)
if heap_mode is None:
    os.environ.pop("SHMEMX_HEAP_MEMORY", None)   # (bench sets "device"): the library's default

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
torch.cuda.set_device(0)
shm.init()
psync = np.full(128, -1, np.int64)
out = {"service_env": os.environ.get("SHMEMX_SERVICE", "1"), "heap": os.environ.get("SHMEMX_HEAP_MEMORY")}
if "--gangs" in sys.argv:
    # a large pageable host call first: the staging ring and its copy gangs exist
    big = np.arange(8 << 20, dtype=np.float64)
    tb = np.zeros_like(big)
    shm.to_all("double", "sum", tb, big, big.size, 0, 0, 1, None, psync)
    assert np.array_equal(tb, big)
    out["gangs"] = True
for n in (1, 1024):
    for where in ("device", "host"):
        if where == "device":
            src = torch.arange(n, dtype=torch.int64, device="cuda")
            tgt = torch.zeros_like(src)
            torch.cuda.synchronize()
        else:
            src = np.arange(n, dtype=np.int64)
            tgt = np.zeros_like(src)
        shm.service_stats(reset=True)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            shm.to_all("longlong", "sum", tgt, src, n, 0, 0, 1, None, psync)
            ts.append(time.perf_counter() - t0)
        st = shm.service_stats(reset=True)
        ct = bench.call_times_us("longlong", "sum", tgt, src, n, 0, 0, 1, psync, 5, reps)
        st_c = shm.service_stats(reset=True)
        out[f"n{n}_{where}"] = {"python_us": round(statistics.median(ts) * 1e6, 2),
                                "python_p90_us": round(sorted(ts)[len(ts) * 9 // 10] * 1e6, 2),
                                "c_us": round(statistics.median(ct), 2) if ct else None,
                                "service_python": st, "service_c": st_c}
# ISx's round on the mirrored heap (tools/isx_mirror_latency.py's loop):
# view operands, the light path (source through the bounce buffer, result
# into HBM and the view's alias by the same copy)
import ctypes  # noqa: E402
s_p, t_p = shm.malloc(8), shm.malloc(8)
if os.environ.get("SHMEMX_HEAP_MEMORY", "mirrored") == "mirrored":
    sv = np.frombuffer((ctypes.c_char * 8).from_address(s_p), dtype=np.int64)
    tv = np.frombuffer((ctypes.c_char * 8).from_address(t_p), dtype=np.int64)
    shm.service_stats(reset=True)
    ts = []
    for r in range(reps):
        sv[0] = 1000 + r
        t0 = time.perf_counter()
        shm.to_all("longlong", "sum", t_p, s_p, 1, 0, 0, 1, None, psync)
        ts.append(time.perf_counter() - t0)
        assert int(tv[0]) == 1000 + r
    out["isx_mirrored_call_us"] = round(statistics.median(ts) * 1e6, 2)
    out["isx_service"] = shm.service_stats(reset=True)
    out["isx_mirror_stats"] = shm.mirror_stats(reset=True)
# the device call again with a second Python thread alive (bench.py keeps a
# threading.Timer watchdog)
import threading  # noqa: E402
timer = threading.Timer(3600, lambda: None)
timer.start()
src = torch.arange(1, dtype=torch.int64, device="cuda")
tgt = torch.zeros_like(src)
torch.cuda.synchronize()
shm.service_stats(reset=True)
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    shm.to_all("longlong", "sum", tgt, src, 1, 0, 0, 1, None, psync)
    ts.append(time.perf_counter() - t0)
timer.cancel()
out["with_timer_thread_us"] = round(statistics.median(ts) * 1e6, 2)
out["with_timer_service"] = shm.service_stats(reset=True)
print(json.dumps(out))
