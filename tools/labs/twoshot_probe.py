"""Experiment (not part of the library): microseconds per mid-size call of
DIRECT and SIGNAL (double sum, full set, heap operands), N PE processes
launched by torch.distributed.run; on the one-GPU box with
SHMEMX_SHARE_GPU=1 SHMEMX_TRANSPORT=ipc, all on device 0.  Run it once with
the fused two-shot launch (default) and once with SHMEMX_FUSED_TWOSHOT_KB=0
(the multi-launch schedules) to compare.  Each call is checked against a
torch fold of the regenerated sources in set order.
"""
import os
import sys
import time

os.environ.setdefault("SHMEMX_HEAP_MEMORY", "device")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402


def main():
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local = 0 if os.environ.get("SHMEMX_SHARE_GPU") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    shm.init_from_torch_distributed(device=local)

    def maxr(x):
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def per_call(fn, reps):
        for _ in range(10):
            fn()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return round(maxr((time.perf_counter() - t0) / reps * 1e6), 1)

    big = 16 << 20
    hs, ht = shm.malloc(big), shm.malloc(big)
    res = {"fused_twoshot_kb": os.environ.get("SHMEMX_FUSED_TWOSHOT_KB", "default"), "npes": world}
    sizes = [float(x) for x in os.environ.get("PROBE_KIB", "512,1024,2048,4096,8192,16384").split(",")]
    for kib in sizes:
        n = max(1, int(kib * 1024) // 8)
        g = torch.Generator(device="cuda")
        srcs = []
        for p in range(world):
            g.manual_seed(1000 + p)
            srcs.append(torch.rand(n, dtype=torch.float64, device="cuda", generator=g) + 1.0)
        want = srcs[0].clone()
        for p in range(1, world):
            want += srcs[p]
        shm.memcpy(hs, srcs[rank], n * 8)
        torch.cuda.synchronize()
        row = {}
        for algo in ("direct", "signal"):
            def call():
                shm.reduce_on_stream("double", "sum", ht, hs, n, 0, 0, world, algo)
                torch.cuda.synchronize()
            shm.direct_stats(reset=True)
            row[algo] = per_call(call, 200 if kib <= 256 else 100 if kib <= 4096 else 30)
            st = shm.direct_stats(reset=True)
            row[algo + "_fused2"] = int(st.get("fused_twoshot_calls", 0))
            got = torch.empty(n, dtype=torch.float64, device="cuda")
            shm.memcpy(got, ht, n * 8)
            torch.cuda.synchronize()
            row[algo + "_exact"] = bool(torch.equal(got.view(torch.int64), want.view(torch.int64)))
        res[f"{kib:g}KiB"] = row
    if rank == 0:
        print(res, flush=True)
    shm.free(ht)
    shm.free(hs)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()
    if any(k.startswith("ROCPROF") for k in os.environ):
        shm.finalize()   # leave normally: the profiler writes at exit
        return
    os._exit(0)


if __name__ == "__main__":
    main()
