"""Child process for test_gpu_api.py::test_rccl_schedules_one_rank: with
SHMEMX_FORCE_COLLECTIVE=1 a one-PE job runs the full RCCL / ALLREDUCE / A2A /
GATHER schedules (RCCL communicator of one rank), so every RCCL call of the
path executes on a one-GPU box; host arrays take the collective path's
bounce and staging copies; the stream-ordered schedules are also captured
into HIP graphs and replayed.  Prints "ok" or raises."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402
import shmem_mi355x as shm  # noqa: E402

assert os.environ.get("SHMEMX_FORCE_COLLECTIVE") == "1"
torch.cuda.set_device(0)
shm.init_attr(0, 1, 0, None)
for t, op, algos in [("double", "sum", ("rccl", "allreduce", "a2a", "gather", "direct")),
                     ("int", "max", ("rccl", "allreduce", "a2a", "gather", "direct")),
                     ("long", "xor", ("a2a", "gather", "direct")),
                     ("complexf", "prod", ("a2a", "gather", "direct")),
                     ("longdouble", "min", ("a2a", "gather", "direct"))]:
    for n in (1, 7, 4103, 1 << 20):
        src = oracle.fill(t, 1, 3, n)
        for algo in algos:
            raw = src.view(np.uint8) if t == "longdouble" else src
            s = torch.from_numpy(raw.copy()).cuda()
            d = torch.zeros_like(s)
            shm.reduce_on_stream(t, op, d, s, n, 0, 0, 1, algo)
            torch.cuda.synchronize()
            assert d.cpu().numpy().tobytes() == raw.tobytes(), (t, op, n, algo)
            shm.reduce_on_stream(t, op, s, s, n, 0, 0, 1, algo)       # in place
            torch.cuda.synchronize()
            assert s.cpu().numpy().tobytes() == raw.tobytes(), (t, op, n, algo, "in place")

# Host arrays through the collective path's small-message bounce (copy
# kernels bounce -> staging -> bounce around the one-rank RCCL call): host ->
# device, device -> host, host -> host in place and partially overlapping,
# and fresh data on every call through the same bounce buffers; bytewise
# against the oracle (a one-member set is a copy, reduce-op.c:213-216).
for t in ("long", "double", "short"):
    for n in (1, 7, 32768):
        for k in range(3):                       # fresh data each call
            src = oracle.fill(t, 1, 40 + k + n, n)
            want = oracle.reduce_sim(t, "sum", src[None, :], 0, 0, 1)[0]
            d = torch.zeros(n, dtype=getattr(torch, {"long": "int64", "double": "float64",
                                                    "short": "int16"}[t]), device="cuda")
            shm.to_all(t, "sum", d, src, n, 0, 0, 1)                 # host -> device
            assert shm.last_error() == 0 and d.cpu().numpy().tobytes() == want.tobytes(), (t, n, k, "h2d")
            h = np.zeros_like(src)
            shm.to_all(t, "sum", h, d, n, 0, 0, 1)                   # device -> host
            assert h.tobytes() == want.tobytes(), (t, n, k, "d2h")
            buf = np.concatenate([src, np.zeros(5, src.dtype)])
            shm.to_all(t, "sum", buf, buf, n, 0, 0, 1)               # host, in place
            assert buf[:n].tobytes() == want.tobytes(), (t, n, k, "in place")
            shm.to_all(t, "sum", buf[3:], buf, n, 0, 0, 1)           # host, partial overlap
            assert buf[3:n + 3].tobytes() == want.tobytes(), (t, n, k, "overlap")

# HIP graph capture of the stream-ordered collective schedules on the real
# RCCL (one rank): RS + AG (+ the ragged tail's all-reduce), the single
# all-reduce, A2A's grouped send/recv + fold + all-gather and GATHER, and
# AUTO, each warmed once (workspaces sized outside the capture), captured,
# then replayed on fresh inputs.  DIRECT is refused under capture (host
# barriers), so it is not here.
st = torch.cuda.Stream()
for t, op, algo, n in [("double", "sum", "rccl", (1 << 20) + 3), ("double", "sum", "allreduce", 4103),
                       ("int", "max", "rccl", 65536), ("long", "xor", "a2a", 70001),
                       ("float", "min", "gather", 4103), ("double", "sum", "auto", (1 << 20) + 3)]:
    s = torch.from_numpy(oracle.fill(t, 1, 5, n)).cuda()
    d = torch.zeros_like(s)
    st.wait_stream(torch.cuda.current_stream())
    shm.reduce_on_stream(t, op, d, s, n, 0, 0, 1, algo, st.cuda_stream)       # warm
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        shm.reduce_on_stream(t, op, d, s, n, 0, 0, 1, algo, st.cuda_stream)
    for k in range(3):
        src = oracle.fill(t, 1, 60 + k, n)
        s.copy_(torch.from_numpy(src))
        d.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert d.cpu().numpy().tobytes() == src.tobytes(), (t, op, algo, n, "graph replay", k)
    del g
print("ok")
