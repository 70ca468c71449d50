"""Experiment (not part of the library): the fixed cost of DIRECT's and
SIGNAL's synchronisation on one GPU.  With $SHMEMX_FORCE_COLLECTIVE=1 a 1-PE
job runs the collective schedules, so every fence kernel, signal kernel and
host barrier of the two algorithms executes, with no peer to wait for: what
is left is the floor each algorithm adds per call.  Heap operands, double
sum; per-call times from back-to-back calls (SIGNAL: stream-ordered, one
sync at the end; DIRECT: host-synchronous by design)."""
import os
import sys
import time

os.environ.setdefault("SHMEMX_FORCE_COLLECTIVE", "1")
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
os.environ.setdefault("SHMEMX_HEAP_MEMORY", "device")   # device addresses from shmem_malloc
import shmem_mi355x as shm  # noqa: E402


def main():
    torch.cuda.set_device(0)
    shm.init_attr(0, 1, 0, None)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    nmax = 32 * 1024 * 1024
    hs, ht = shm.malloc(nmax * 8), shm.malloc(nmax * 8)
    shm.memcpy(hs, torch.rand(nmax, dtype=torch.float64), nmax * 8)
    for n in (1, 4096, 32768, 1 << 20, nmax):
        row = []
        for algo in ("direct", "signal"):
            for _ in range(3):
                shm.reduce_on_stream("double", "sum", ht, hs, n, 0, 0, 1, algo, sp)
            torch.cuda.synchronize()
            reps = 200 if n <= 1 << 20 else 20
            t0 = time.perf_counter()
            for _ in range(reps):
                shm.reduce_on_stream("double", "sum", ht, hs, n, 0, 0, 1, algo, sp)
            torch.cuda.synchronize()
            row.append((time.perf_counter() - t0) / reps * 1e6)
        print(f"n={n:>9}  direct {row[0]:9.1f} us   signal {row[1]:9.1f} us", flush=True)
    st = shm.direct_stats(reset=True)
    print("direct phase totals (us):", {k: round(v, 1) for k, v in st.items()}, flush=True)


if __name__ == "__main__":
    main()
