"""Every shipped kernel of the path, launched through the C ABI at the sizes
VERDICT r01 asks counters for, for rocprofv3 passes (kernel trace, then
FETCH_SIZE and WRITE_SIZE in separate --pmc runs; tools/gpu_steps.sh pmc_kernels):

  fold2_double_sum   fold_kernel, 2 inputs, acc += in, 32 Mi doubles (headline)
  fold2_long_{and,or,xor}   2 inputs, 64 Mi longs (configs[3]'s fold)
  foldP4_double_sum  P-input fold, P = 4, 16 Mi doubles per input
  foldP8_double_sum  P = 8, 16 Mi - 2048 doubles per input (distinct grid)
  foldP{4,8}_peers_double_sum  the same folds through fold_peers_kernel
                     (shmemx_fold_n_peers_on_stream: DIRECT's and SIGNAL's fold)
  foldP8_shard       P = 8 over one 4 Mi-double A2A shard per input, inputs
                     contiguous in one block (the A2A workspace layout)
  gather7            gather_kernel, 7 segments of 4 Mi doubles (DIRECT's
                     all-gather at P = 8, 32 Mi doubles)
  copy64Mi           the PE_size = 1 call (shmemx_reduce_on_stream, a copy:
                     reduce-op.c:213-216) over 64 Mi doubles, 512 MiB: the copy
                     kernel fold_kernel<long,SUM,1 input,1 vector,nt>
  checksum           checksum_kernel over 32 Mi doubles
  verify             shmemx_verify at one PE (the same checksum kernel: its
                     launches join checksum's run in the trace)

Prints one JSON line per config: launches, HIP-event average launch time on
the launch stream, algorithmic bytes per launch and the rate.
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
REPS = int(os.environ.get("PMC_REPS", "10"))
s = torch.cuda.Stream()
Mi = 1024 * 1024


def timed(name, fn, alg_bytes, grid_hint, blocking=False, shares_run=False):
    """blocking: the call synchronises itself (shmemx_checksum), so it is timed
    on the host clock, launch + wait included.  shares_run: this config
    launches the same kernel at the same grid as the one before it, so
    tools/summarize_pmc.py finds its launches in that config's run."""
    fn()
    torch.cuda.synchronize()
    if blocking:
        import time
        t0 = time.perf_counter()
        for _ in range(REPS):
            fn()
        us = (time.perf_counter() - t0) / REPS * 1e6
    else:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(REPS):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / REPS * 1e3
    print(json.dumps({"config": name, "launches": REPS + 1, "avg_us": round(us, 2),
                      "alg_bytes": alg_bytes, "GBps": round(alg_bytes / us / 1e3, 1),
                      "grid_hint": grid_hint, "shares_run": shares_run}), flush=True)


def blocks(nvec, unroll=4):
    return (nvec + 256 * unroll - 1) // (256 * unroll)


n = 32 * Mi
acc = torch.rand(n, dtype=torch.float64, device="cuda")
inp = torch.rand(n, dtype=torch.float64, device="cuda")
timed("fold2_double_sum", lambda: shm.fold("double", "sum", acc, inp, n, s.cuda_stream),
      3 * 8 * n, blocks(n // 2))
del acc, inp

n = 64 * Mi
a = torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda")
b = torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda")
for op in ("and", "or", "xor"):
    timed(f"fold2_long_{op}", lambda: shm.fold("long", op, a, b, n, s.cuda_stream),
          3 * 8 * n, blocks(n // 2))
del a, b

n = 16 * Mi
ins = [torch.rand(n, dtype=torch.float64, device="cuda") for _ in range(8)]
out = torch.empty(n, dtype=torch.float64, device="cuda")
timed("foldP4_double_sum", lambda: shm.fold_n("double", "sum", out, ins[:4], n, s.cuda_stream),
      5 * 8 * n, blocks(n // 2))
m = n - 2048
timed("foldP8_double_sum", lambda: shm.fold_n("double", "sum", out, ins, m, s.cuda_stream),
      9 * 8 * m, blocks(m // 2))
# the peers kernel (DIRECT's and SIGNAL's fold: every input's loads in flight)
timed("foldP4_peers_double_sum", lambda: shm.fold_n("double", "sum", out, ins[:4], n, s.cuda_stream,
                                                    peers=True),
      5 * 8 * n, blocks(n // 2))
timed("foldP8_peers_double_sum", lambda: shm.fold_n("double", "sum", out, ins, m, s.cuda_stream,
                                                    peers=True),
      9 * 8 * m, blocks(m // 2, 2))
del ins, out

# configs[2]'s own shape for DIRECT's fold: 32 Mi doubles on 8 PEs, each PE
# folds one 4 Mi-double slice from 8 separate arrays (the peers' sources)
n = 4 * Mi
ins = [torch.rand(n, dtype=torch.float64, device="cuda") for _ in range(8)]
out = torch.empty(n, dtype=torch.float64, device="cuda")
timed("foldP8_peers_slice4Mi", lambda: shm.fold_n("double", "sum", out, ins, n, s.cuda_stream, peers=True),
      9 * 8 * n, blocks(n // 2, 4))
del ins, out

n = 4 * Mi
ws = torch.rand(8 * n, dtype=torch.float64, device="cuda")
shard = [ws[i * n:(i + 1) * n] for i in range(8)]
out = torch.empty(n, dtype=torch.float64, device="cuda")
timed("foldP8_shard", lambda: shm.fold_n("double", "sum", out, shard, n, s.cuda_stream),
      9 * 8 * n, blocks(n // 2))
del ws, shard, out

n = 32 * Mi
src = torch.rand(n, dtype=torch.float64, device="cuda")
dst = torch.empty(n, dtype=torch.float64, device="cuda")
sl = n // 8
segs = [(src[i * sl:(i + 1) * sl], dst[i * sl:(i + 1) * sl]) for i in range(1, 8)]
timed("gather7", lambda: shm.gather([x for x, _ in segs], [y for _, y in segs], [sl * 8] * 7,
                                    s.cuda_stream),
      2 * 7 * sl * 8, None)
assert torch.equal(dst[sl:], src[sl:]), "gather copied wrong bytes"
del dst

# configs[1]'s literal drop-in call at PE_size = 1: a copy (reduce-op.c:213-216)
n2 = 64 * Mi
csrc = torch.rand(n2, dtype=torch.float64, device="cuda")
cdst = torch.empty(n2, dtype=torch.float64, device="cuda")
timed("copy64Mi", lambda: shm.reduce_on_stream("double", "sum", cdst, csrc, n2, 0, 0, 1, "auto",
                                               s.cuda_stream),
      2 * 8 * n2, n2 // 2)
torch.cuda.synchronize()
assert torch.equal(cdst, csrc), "the PE_size = 1 call copied wrong bytes"
del csrc, cdst

timed("checksum", lambda: shm.checksum("double", src, n), 8 * n, None, blocking=True)
# shmemx_verify at one PE: the checksum launch, the stream wait and the
# (here empty) exchange — the whole call on the host clock
timed("verify", lambda: shm.verify("double", src, n, 0, 0, 1), 8 * n, None, blocking=True,
      shares_run=True)
