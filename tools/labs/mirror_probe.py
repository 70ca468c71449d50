"""Where the time goes in the mirrored heap ($SHMEMX_HEAP_MEMORY=mirrored),
one PE: host stores into a shmem_malloc'd source (write faults), the blocking
shmem_double_sum_to_all on the HBM twins (flush of the touched blocks, the
kernel, marking the target device-newer), the host reading the target back
(read faults, fetches), and the same call again on untouched operands.

    SHMEMX_HEAP_MEMORY=mirrored python tools/labs/mirror_probe.py [nreduce ...]
"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

assert os.environ.get("SHMEMX_HEAP_MEMORY") == "mirrored"
import torch  # noqa: E402,F401

shm.init_attr(0, 1, 0, None)


def view(ptr, n):
    return np.frombuffer((ctypes.c_char * (n * 8)).from_address(ptr), dtype=np.float64, count=n)


def ms(t0):
    return round((time.perf_counter() - t0) * 1e3, 3)


for n in [int(a) for a in sys.argv[1:]] or [4 << 20, 32 << 20]:
    s_p, t_p = shm.malloc(n * 8), shm.malloc(n * 8)
    src, tgt = view(s_p, n), view(t_p, n)
    vals = np.random.default_rng(n).random(n)
    row = {"nreduce": n, "MiB": n * 8 >> 20}
    shm.mirror_stats(reset=True)
    t0 = time.perf_counter()
    src[:] = vals
    row["host_write_ms"] = ms(t0)
    row["write"] = shm.mirror_stats(reset=True)
    t0 = time.perf_counter()
    shm.to_all("double", "sum", t_p, s_p, n, 0, 0, 1)
    row["call1_ms"] = ms(t0)
    row["call1"] = shm.mirror_stats(reset=True)
    t0 = time.perf_counter()
    got = tgt.copy()
    row["host_read_ms"] = ms(t0)
    row["read"] = shm.mirror_stats(reset=True)
    assert np.array_equal(got, vals)
    for k in range(3):
        t0 = time.perf_counter()
        shm.to_all("double", "sum", t_p, s_p, n, 0, 0, 1)
        row[f"repeat{k}_ms"] = ms(t0)
    row["repeat"] = shm.mirror_stats(reset=True)
    t0 = time.perf_counter()
    got = tgt.copy()
    row["host_read2_ms"] = ms(t0)
    assert np.array_equal(got, vals)
    # steady state, as a reference program iterates: the host rewrites the
    # source, calls, reads the target back; per-phase medians of 5 rounds
    phases = {"host_write": [], "call": [], "host_read": []}
    for k in range(5):
        vals2 = vals + k
        t0 = time.perf_counter()
        src[:] = vals2
        phases["host_write"].append(ms(t0))
        t0 = time.perf_counter()
        shm.to_all("double", "sum", t_p, s_p, n, 0, 0, 1)
        phases["call"].append(ms(t0))
        t0 = time.perf_counter()
        got = tgt.copy()
        phases["host_read"].append(ms(t0))
        assert np.array_equal(got, vals2)
    row["steady_ms"] = {k: sorted(v)[2] for k, v in phases.items()}
    row["steady_call_GiBps"] = round(n * 8 / (row["steady_ms"]["call"] * 1e-3) / 2**30, 1)
    # the same round trip on plain numpy arrays (the host-array path)
    h_s, h_t = vals.copy(), np.empty_like(vals)
    shm.to_all("double", "sum", h_t, h_s, n, 0, 0, 1)
    t0 = time.perf_counter()
    shm.to_all("double", "sum", h_t, h_s, n, 0, 0, 1)
    row["numpy_arrays_call_ms"] = ms(t0)
    # the same call on plain device arrays, for the floor
    d_s = torch.from_numpy(vals).cuda()
    d_t = torch.empty_like(d_s)
    torch.cuda.synchronize()
    shm.to_all("double", "sum", d_t, d_s, n, 0, 0, 1)
    t0 = time.perf_counter()
    shm.to_all("double", "sum", d_t, d_s, n, 0, 0, 1)
    row["device_arrays_call_ms"] = ms(t0)
    print(row, flush=True)
    shm.free(t_p)
    shm.free(s_p)
    del d_s, d_t
