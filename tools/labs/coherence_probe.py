"""Experiment: bench.py's coherence extra, per size and algorithm, with the
first mismatching elements printed (N PE processes via torch.distributed.run;
on the one-GPU box with SHMEMX_SHARE_GPU=1 SHMEMX_TRANSPORT=ipc)."""
import os
import sys

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
    sizes = [int(x) for x in os.environ.get("PROBE_N", "128,131072,2097152").split(",")]
    iters = int(os.environ.get("PROBE_ITERS", "6"))
    stream = torch.cuda.Stream() if os.environ.get("PROBE_SIDE_STREAM", "1") == "1" else None
    sp = stream.cuda_stream if stream is not None else 0
    hs, ht = shm.malloc(max(sizes) * 8), shm.malloc(max(sizes) * 8)
    for algo in os.environ.get("PROBE_ALGOS", "direct,signal").split(","):
        for it in range(iters):
            for n in sizes:
                base = torch.arange(n, device="cuda", dtype=torch.float64).remainder_(1024)
                shm.memcpy(hs, base + (7 * rank + 3 * it), n * 8)
                shm.reduce_on_stream("double", "sum", ht, hs, n, 0, 0, world, algo, sp)
                torch.cuda.synchronize()
                got = torch.empty(n, device="cuda", dtype=torch.float64)
                shm.memcpy(got, ht, n * 8)
                want = base * world + (7 * world * (world - 1) // 2 + 3 * it * world)
                bad = (got != want).nonzero().flatten()
                if rank == 0 or bad.numel():
                    line = f"rank {rank} {algo} it={it} n={n}: {bad.numel()} bad"
                    if bad.numel():
                        i = bad[:4].tolist()
                        line += f" first {i} got {got[i].tolist()} want {want[i].tolist()}" \
                                f" last {bad[-1].item()}"
                    print(line, flush=True)
    shm.free(ht)
    shm.free(hs)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    main()
