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


def _nan_rule_equal(got, want, ft):
    """IEEE sum/prod: NaN where the reference has NaN (the payload is the
    hardware's choice), every other value bit for bit."""
    g, w = got.view(ft), want.view(ft)
    if not np.array_equal(np.isnan(g), np.isnan(w)):
        return False
    m = ~np.isnan(w)
    return g[m].tobytes() == w[m].tobytes()


@pytest.mark.parametrize("peers", [False, True])
def test_gpu_matches_reference_element_ops(cuda, shm, oracle, peers):
    """The GPU's element ops against the REFERENCE'S OWN: tests/golden/
    ref_element_ops.json holds what reduce-op.c:71-150, compiled from its text
    (oracle/build_ref.sh), computes on special values and random bits for all
    44 pairs, both operand orders (PE 0 and PE 1 of a 2-PE reduction).  Through
    the runtime-nins fold and, with peers=True, the every-input-in-flight fold
    DIRECT and SIGNAL use.  Bit for bit, except the NaN payload of an IEEE
    float/double (or complex component) sum or product; long double (soft x87)
    is bit for bit, NaN payloads included."""
    import base64

    import torch
    from gpu_util import empty_like_dev, value_bytes
    with open(os.path.join(GOLDEN, "ref_element_ops.json")) as f:
        g = json.load(f)["cases"]
    checked = 0
    for t, c in g.items():
        dt = np.dtype(oracle.NP_DTYPE[t])
        a = np.frombuffer(base64.b64decode(c["a"]), dtype=dt).copy()
        b = np.frombuffer(base64.b64decode(c["b"]), dtype=dt).copy()
        da, db = to_dev(torch, a), to_dev(torch, b)
        for op, o in c["ops"].items():
            assert shm.op_on_device(t, op), (t, op)
            for ins, key in (([da, db], "ab"), ([db, da], "ba")):
                out = empty_like_dev(torch, a)
                shm.fold_n(t, op, out, ins, a.size, peers=peers)
                torch.cuda.synchronize()
                got = from_dev(out, dt)
                want = np.frombuffer(base64.b64decode(o[key]), dtype=dt)
                if op in ("sum", "prod") and t in ("float", "double", "complexd", "complexf"):
                    ft = np.float32 if t in ("float", "complexf") else np.float64
                    assert _nan_rule_equal(got, want, ft), (t, op, key)
                else:
                    assert value_bytes(got) == value_bytes(want), (t, op, key)
                checked += a.size
    assert checked > 40000
