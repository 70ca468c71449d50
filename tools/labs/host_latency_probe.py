"""Small blocking calls on HOST arrays (the ISx shape, nreduce = 1 .. 32 Ki
longlong): microseconds per call for the one-member copy path and for the
collective path (SHMEMX_FORCE_COLLECTIVE=1: a one-rank RCCL communicator).
Every case re-checks the result with fresh data.  (The committed profile
also has the collective path with DMA bounce copies, the earlier design.)
"""
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child():
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime in the process)
    sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
    import shmem_mi355x as shm
    shm.init_attr(0, 1, 0, None)
    out = []
    for n in (1, 64, 4096, 32768):
        src = np.arange(n, dtype=np.int64)
        tgt = np.zeros(n, dtype=np.int64)
        for _ in range(50):
            shm.to_all("longlong", "sum", tgt, src, n, 0, 0, 1)
        reps = 2000
        t0 = time.perf_counter()
        for _ in range(reps):
            shm.to_all("longlong", "sum", tgt, src, n, 0, 0, 1)
        us = (time.perf_counter() - t0) / reps * 1e6
        ok = True
        for k in range(20):
            src[:] = np.arange(n, dtype=np.int64) * (k + 3) + k
            shm.to_all("longlong", "sum", tgt, src, n, 0, 0, 1)
            ok &= shm.last_error() == 0 and tgt.tobytes() == src.tobytes()
        out.append(f"n={n}: {us:7.2f} us/call correct={ok}")
    print("; ".join(out))


def main():
    if len(sys.argv) > 1:
        child()
        return
    cases = [("one-member copy (zero-copy bounce)", {}),
             ("collective, kernel bounce copies", {"SHMEMX_FORCE_COLLECTIVE": "1"})]
    for name, extra in cases:
        env = dict(os.environ, **extra)
        r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True,
                           text=True, timeout=120)
        print(f"{name:40s} {r.stdout.strip()} {('rc=%d ' % r.returncode + r.stderr[-500:]) if r.returncode else ''}",
              flush=True)


if __name__ == "__main__":
    main()
