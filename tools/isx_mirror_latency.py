"""The ISx use on the mirrored heap (the default heap mode): every PE stores
its bucket size into a shmem_malloc'd long long with a plain host store, calls
shmem_longlong_sum_to_all(nreduce = 1) (examples/ISx/SHMEM/isx.c:615-624),
then reads the total with a plain host load.  One PE here (the copy path of
reduce-op.c:213-216); $SHMEMX_FORCE_COLLECTIVE=1 runs the collective schedule
instead.  The light path: only the source's 8 written bytes go up, no block
changes state or protection, and the call's last kernel stores the result
into the view as well (profiles/r04_isx_mirror.txt has the cost of the
result left DEVICE_NEWER instead: the host load faults and fetches its 64 KiB
block).

    python tools/isx_mirror_latency.py [rounds]
Prints one JSON line: medians in microseconds of the call alone, the host
load after it, and the whole store + call + load round; the mirror counters.
"""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
os.environ.setdefault("SHMEMX_HEAP_MEMORY", "mirrored")
import shmem_mi355x as shm  # noqa: E402
import torch  # noqa: E402,F401

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
shm.init_attr(0, 1, 0, None)
s_p, t_p = shm.malloc(8), shm.malloc(8)
src = np.frombuffer((ctypes.c_char * 8).from_address(s_p), dtype=np.int64)
tgt = np.frombuffer((ctypes.c_char * 8).from_address(t_p), dtype=np.int64)
psync = np.full(128, -1, np.int64)
call, load, total = [], [], []
for r in range(rounds + 50):
    t0 = time.perf_counter()
    src[0] = 1000 + r                       # the bucket size (a host store)
    t1 = time.perf_counter()
    shm.to_all("longlong", "sum", t_p, s_p, 1, 0, 0, 1, None, psync)
    t2 = time.perf_counter()
    got = int(tgt[0])                       # the total (a host load)
    t3 = time.perf_counter()
    assert got == 1000 + r, (got, r)
    if r >= 50:
        call.append(t2 - t1)
        load.append(t3 - t2)
        total.append(t3 - t0)
    if r == 49:
        shm.mirror_stats(reset=True)
st = shm.mirror_stats(reset=True)
print(json.dumps({
    "force_collective": os.environ.get("SHMEMX_FORCE_COLLECTIVE", "0"),
    "rounds": rounds, "call_us": round(statistics.median(call) * 1e6, 2),
    "host_load_us": round(statistics.median(load) * 1e6, 2),
    "round_us": round(statistics.median(total) * 1e6, 2),
    "mirror_stats_per_round": {k: round(v / rounds, 3) for k, v in st.items()}}), flush=True)
shm.finalize()
