"""shmemx_checksum / shmemx_verify per call at 32 Mi doubles: host clock
(launch + stream wait + the Python call), for the grid cap in
$SHMEMX_CHECKSUM_BLOCKS (run under rocprofv3 --kernel-trace for the kernel's
own time)."""
import json
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
n = 32 * 1024 * 1024
src = torch.rand(n, dtype=torch.float64, device="cuda")
torch.cuda.synchronize()
ref = shm.checksum("double", src, n)
out = {"blocks_cap": os.environ.get("SHMEMX_CHECKSUM_BLOCKS", "4096")}
for name, fn in (("checksum", lambda: shm.checksum("double", src, n)),
                 ("verify", lambda: shm.verify("double", src, n, 0, 0, 1))):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    out[f"{name}_us_median"] = round(statistics.median(ts) * 1e6, 2)
    out[f"{name}_us_min"] = round(min(ts) * 1e6, 2)
assert shm.checksum("double", src, n) == ref
print(json.dumps(out), flush=True)
shm.finalize()
