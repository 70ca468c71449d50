"""Experiment (not part of the library): the 2-input fold (acc = op(acc, in),
reduce-op.c:231-235) for every reference (type, op) pair through the C ABI
(shmemx_fold_on_stream), 256 MiB per array, HIP events on the stream, median
of 10 launches after 3 warm ones.  GB/s counts the algorithmic 3 x 256 MiB
(read acc, read in, write acc); a pair far below the HBM rate of the others
is compute-bound (the soft-float long double, the complex products).

    python tools/labs/type_fold_probe.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402

BYTES = 256 << 20
SIZES = {"short": 2, "int": 4, "long": 8, "longlong": 8, "float": 4, "double": 8,
         "longdouble": 16, "complexd": 16, "complexf": 8}


def main():
    torch.cuda.set_device(0)
    shm.init_attr(0, 1, 0, None)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    # random bytes, then made benign for the float types: small positive
    # values keep every op on its normal (non-NaN, non-overflow) path
    acc = torch.empty(BYTES, dtype=torch.uint8, device="cuda")
    inp = torch.empty(BYTES, dtype=torch.uint8, device="cuda")
    rows = []
    for (t, op) in shm.REFERENCE_PAIRS:
        sz = SIZES[t]
        n = BYTES // sz
        if t in ("float", "complexf"):
            acc.view(torch.float32).uniform_(1.0, 1.0001, generator=g)
            inp.view(torch.float32).uniform_(1.0, 1.0001, generator=g)
        elif t in ("double", "complexd"):
            acc.view(torch.float64).uniform_(1.0, 1.0001, generator=g)
            inp.view(torch.float64).uniform_(1.0, 1.0001, generator=g)
        elif t == "longdouble":
            # x87 1.0: mantissa 0x8000000000000000, exponent 0x3FFF, padding 0
            v = torch.zeros(n, 2, dtype=torch.int64, device="cuda")
            v[:, 0] = -0x8000000000000000
            v[:, 1] = 0x3FFF
            acc.view(torch.int64).copy_(v.view(-1))
            inp.view(torch.int64).copy_(v.view(-1))
        else:
            acc.random_(0, 256, generator=g)
            inp.random_(0, 256, generator=g)
        torch.cuda.synchronize()
        for _ in range(3):
            shm.fold(t, op, acc, inp, n, sp)
        times = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            shm.fold(t, op, acc, inp, n, sp)
            e1.record(stream)
            e1.synchronize()
            times.append(e0.elapsed_time(e1) * 1e-3)
        times.sort()
        t_med = times[len(times) // 2]
        gbs = 3 * BYTES / t_med / 1e9
        rows.append((t, op, t_med * 1e6, gbs))
        print(f"{t:>10} {op:>4}  {t_med * 1e6:8.1f} us  {gbs:7.1f} GB/s  {gbs / 8000:5.1%} of 8 TB/s", flush=True)
    # the P-input fold (A2A / DIRECT / GATHER's fold step) at P = 8, 64 MiB
    # per input, for the types whose op is the most arithmetic per byte
    P, IB = 8, 64 << 20
    ins = [torch.empty(IB, dtype=torch.uint8, device="cuda") for _ in range(P)]
    out = torch.empty(IB, dtype=torch.uint8, device="cuda")
    for (t, op) in (("double", "sum"), ("longdouble", "sum"), ("longdouble", "prod"),
                    ("longdouble", "max"), ("complexd", "prod"), ("complexf", "prod"), ("short", "sum")):
        sz = SIZES[t]
        n = IB // sz
        for x in ins:
            if t == "longdouble":
                v = torch.zeros(n, 2, dtype=torch.int64, device="cuda")
                v[:, 0] = -0x8000000000000000
                v[:, 1] = 0x3FFF
                x.view(torch.int64).copy_(v.view(-1))
            elif t in ("double", "complexd"):
                x.view(torch.float64).uniform_(1.0, 1.0001, generator=g)
            elif t == "complexf":
                x.view(torch.float32).uniform_(1.0, 1.0001, generator=g)
            else:
                x.random_(0, 256, generator=g)
        torch.cuda.synchronize()
        for _ in range(3):
            shm.fold_n(t, op, out, ins, n, sp)
        times = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            shm.fold_n(t, op, out, ins, n, sp)
            e1.record(stream)
            e1.synchronize()
            times.append(e0.elapsed_time(e1) * 1e-3)
        times.sort()
        t_med = times[len(times) // 2]
        gbs = (P + 1) * IB / t_med / 1e9
        print(f"P={P} {t:>10} {op:>4}  {t_med * 1e6:8.1f} us  {gbs:7.1f} GB/s  {gbs / 8000:5.1%} of 8 TB/s",
              flush=True)
    shm.finalize()


if __name__ == "__main__":
    main()
