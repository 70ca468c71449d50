"""Experiment (not part of the library): where a small multi-PE call's time
goes, N PE processes (launched by torch.distributed.run; on the one-GPU box
with SHMEMX_SHARE_GPU=1 SHMEMX_TRANSPORT=ipc, all on device 0; a 1-PE job
with SHMEMX_FORCE_COLLECTIVE=1 runs the same schedules with no peer).

Per call, microseconds, max over ranks, 300 calls each:
  barrier_all            shmem_barrier_all (system fence on every XCD + the
                         node barrier)
  direct n=1             the blocking DIRECT call on heap operands, with the
                         per-phase split from shmemx_direct_stats
  signal n=1             SIGNAL (device barriers) + stream synchronize
  blocking n=1 device    the drop-in call on torch device arrays

$PROBE_STEPS: what runs before each measurement, in order (comma list; the
probe measures after every step): none, copy (three 256 MiB torch copies),
fold (three 32 Mi shmemx_fold calls), gather (three 32 Mi own-order GATHER
reductions of torch arrays), direct (three 32 Mi DIRECT reductions on heap
arrays), events (a torch timing-event pair recorded on a side stream), sleep
(3 s idle).
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

    def per_call(fn, reps=300):
        for _ in range(20):
            fn()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return round(maxr((time.perf_counter() - t0) / reps * 1e6), 1)

    hs, ht = shm.malloc(4096 * 8), shm.malloc(4096 * 8)
    shm.memcpy(hs, torch.zeros(4096 * 8, dtype=torch.uint8), 4096 * 8)
    src1 = torch.arange(1, dtype=torch.int64, device="cuda")
    tgt1 = torch.zeros(1, dtype=torch.int64, device="cuda")

    def measure():
        out = {"barrier_all": per_call(shm.barrier_all)}

        def signal():
            shm.reduce_on_stream("longlong", "sum", ht, hs, 1, 0, 0, world, "signal")
            torch.cuda.synchronize()
        if os.environ.get("PROBE_SIGNAL_FIRST") == "1":   # order check (shared-GPU artefacts)
            out["signal_n1_first"] = per_call(signal)

        def direct():
            shm.reduce_on_stream("longlong", "sum", ht, hs, 1, 0, 0, world, "direct")
            torch.cuda.synchronize()
        shm.direct_stats(reset=True)
        out["direct_n1"] = per_call(direct)
        st = shm.direct_stats(reset=True)
        calls = st.pop("calls")
        out["direct_n1_phases"] = {k.replace("_us", ""): round(maxr(st[k] / calls), 1)
                                   for k in shm.DIRECT_PHASES if st[k]}

        out["signal_n1"] = per_call(signal)
        out["blocking_n1_device"] = per_call(lambda: shm.to_all("longlong", "sum", tgt1, src1, 1, 0, 0, world))
        return out

    n = 32 * 1024 * 1024
    big = None
    steps = [p for p in os.environ.get("PROBE_STEPS", "none").split(",") if p]
    for what in steps:
        if what in ("copy", "fold", "gather", "direct") and big is None:
            big = {"src": torch.rand(n, dtype=torch.float64, device="cuda") + 1.0}
            big["tgt"] = torch.empty_like(big["src"])
            big["hs"], big["ht"] = shm.malloc(n * 8), shm.malloc(n * 8)
            shm.memcpy(big["hs"], big["src"], n * 8)
            torch.cuda.synchronize()
        for _ in range(3):
            if what == "copy":
                big["tgt"].copy_(big["src"])
            elif what == "fold":
                shm.fold("double", "sum", big["ht"], big["hs"], n)
            elif what == "gather":
                shm.reduce_on_stream("double", "sum", big["tgt"], big["src"], n, 0, 0, world, "gather")
            elif what == "direct":
                shm.reduce_on_stream("double", "sum", big["ht"], big["hs"], n, 0, 0, world, "direct")
            elif what == "events":
                s = torch.cuda.Stream()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                b.record(s)
                b.synchronize()
                break
            elif what == "sleep":
                time.sleep(3)
                break
        torch.cuda.synchronize()
        dist.barrier()
        res = measure()
        if rank == 0:
            print(f"after {what}: {res}", flush=True)
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
