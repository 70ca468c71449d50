"""GPU results against the committed golden vectors (tests/golden).

For every golden case whose type/op has a device kernel, every member PE's
expected hash is reproduced on the GPU by folding the sources in that PE's
reference order (reduce-op.c:213-248: itself first, then the other members
ascending) — the GATHER algorithm's per-PE computation — and the PE_start
hash also by the A2A order (set order), which is what every PE receives from
the A2A path.  Inputs are regenerated from the committed seeds.
"""
import json
import os

import numpy as np
import pytest
from gpu_util import from_dev, to_dev

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_gpu_reproduces_golden_hashes(cuda, shm, oracle):
    import torch
    with open(os.path.join(GOLDEN, "reduce_hashes.json")) as f:
        g = json.load(f)
    npes = g["npes"]
    groups = {}
    for key, want in g["cases"].items():
        t, op, k, n, sset = key.split("|")
        groups.setdefault((t, int(k[1:]), int(n[1:])), []).append((op, sset, want))
    checked = 0
    for (t, kind, n), cases in groups.items():
        if n == 0 or not shm.op_on_device(t, "sum"):
            continue
        seed = 0x5EED0000 + 1009 * list(oracle.TYPES).index(t) + n
        srcs = oracle.sources(t, kind, npes, n, base_seed=seed)
        dev = [to_dev(torch, srcs[p]) for p in range(npes)]
        out = torch.empty_like(dev[0])
        for op, sset, want in cases:
            if not shm.op_on_device(t, op):
                continue
            s = tuple(int(x) for x in sset[3:].split(","))
            mem = [s[0] + i * (1 << s[1]) for i in range(s[2])]
            for me in mem:
                order = [me] + [p for p in mem if p != me]
                shm.fold_n(t, op, out, [dev[p] for p in order], n)
                got = from_dev(out, srcs.dtype)
                assert f"{oracle.value_hash(t, got):016x}" == want[me], (t, op, kind, n, s, me)
                checked += 1
            shm.fold_n(t, op, out, [dev[p] for p in mem], n)
            got = from_dev(out, srcs.dtype)
            assert f"{oracle.value_hash(t, got):016x}" == want[mem[0]], (t, op, kind, n, s, "a2a")
    assert checked > 10000


def test_gpu_reproduces_golden_special_values(cuda, shm):
    import torch
    with open(os.path.join(GOLDEN, "special_values.json")) as f:
        g = json.load(f)
    np_t = {"short": np.int16, "int": np.int32, "long": np.int64, "float": np.float32,
            "double": np.float64}
    for key, c in g.items():
        t, op = key.split("|")
        dt = np.dtype(np_t[t])
        ut = f"u{dt.itemsize}"
        a = torch.from_numpy(np.array(c["a"], dtype=ut).view(dt)).cuda()
        b = torch.from_numpy(np.array(c["b"], dtype=ut).view(dt)).cuda()
        for order, pe in (((a, b), "pe0"), ((b, a), "pe1")):
            out = torch.empty_like(a)
            shm.fold_n(t, op, out, list(order), a.numel())
            got = out.cpu().numpy()
            want = np.array(c[pe], dtype=ut).view(dt)
            if t in ("float", "double") and op in ("sum", "prod"):
                assert np.array_equal(np.isnan(got), np.isnan(want)), key
                m = ~np.isnan(want)
                assert got[m].tobytes() == want[m].tobytes(), key
            else:
                assert got.view(ut).tolist() == c[pe], (key, pe)
