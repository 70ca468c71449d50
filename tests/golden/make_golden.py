#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.json).

Source of truth: the oracle (oracle/reduce_oracle.c, a restatement of the
reference's src/reduce/reduce-op.c).  The reference itself cannot be built
here (it needs GASNet, see DESIGN.md "Oracle"), so these vectors are the
oracle's outputs, frozen: they pin the oracle against regressions and let the
GPU box compare against committed values.  Inputs are not stored; they are
regenerated from (type, kind, seed) by oracle.fill (splitmix64).

Files:
  reduce_hashes.json  per case, the FNV-1a hash of every PE's target
                      (0 for PEs outside the active set), 8 PEs, the case
                      grid of SURVEY.md §8c
  special_values.json raw outputs for NaN / +-0 / inf / subnormal / integer
                      extreme inputs, 2 PEs, both PE orders
  isx_known_answer.json  the reference's own known-answer check
                      (examples/ISx/SHMEM/isx.c:615-624): the longlong sum of
                      every PE's bucket size equals NUM_KEYS_PER_PE * NUM_PES

usage: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

NPES = 8
SIZES = [0, 1, 63, 64, 65, 127, 128, 1000, 4103, 65536 + 13]   # SURVEY.md §8c grid
SETS = [(0, 0, 1), (0, 0, 2), (0, 0, 3), (0, 0, 4), (0, 0, 8), (1, 0, 3), (0, 1, 4), (1, 1, 3),
        (2, 0, 5), (0, 2, 2)]
ALL_OPS = ["sum", "prod", "and", "or", "xor", "min", "max"]


def case_key(t, op, kind, n, s):
    return f"{t}|{op}|k{kind}|n{n}|set{s[0]},{s[1]},{s[2]}"


def seed_for(t, n):
    return 0x5EED0000 + 1009 * list(O.TYPES).index(t) + n


def hashes():
    out = {}
    for t in O.TYPES:
        for op in ALL_OPS:
            if not O.op_valid(t, op):
                continue
            for kind in (0, 1):
                for n in SIZES:
                    srcs = O.sources(t, kind, NPES, n, base_seed=seed_for(t, n))
                    for s in SETS:
                        tg = O.reduce_sim(t, op, srcs, *s)
                        members = {s[0] + i * (1 << s[1]) for i in range(s[2])}
                        out[case_key(t, op, kind, n, s)] = [
                            f"{O.value_hash(t, tg[p]):016x}" if p in members else "0"
                            for p in range(NPES)]
    return out


def special_inputs(t):
    if t in ("float", "double"):
        ft = np.float32 if t == "float" else np.float64
        tiny = np.finfo(ft).tiny
        v = [np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf, 1.0, -1.0, tiny, -tiny, tiny / 4,
             np.finfo(ft).max, -np.finfo(ft).max, 2.5]
        return np.array(v, dtype=ft)
    info = np.iinfo(O.NP_DTYPE[t])
    return np.array([info.min, info.max, 0, -1, 1, info.min + 1, info.max - 1, 12345],
                    dtype=info.dtype)


def specials():
    out = {}
    for t in ("short", "int", "long", "float", "double"):
        v = special_inputs(t)
        a, b = np.repeat(v, len(v)), np.tile(v, len(v))
        srcs = np.stack([a, b])
        for op in ALL_OPS:
            if not O.op_valid(t, op):
                continue
            tg = O.reduce_sim(t, op, srcs, 0, 0, 2)
            out[f"{t}|{op}"] = {"a": a.view(f"u{a.itemsize}").tolist(),
                                "b": b.view(f"u{b.itemsize}").tolist(),
                                "pe0": tg[0].view(f"u{a.itemsize}").tolist(),
                                "pe1": tg[1].view(f"u{a.itemsize}").tolist()}
    return out


def isx():
    """ISx verification (isx.c:615-624): sum_to_all(&total, &my_bucket_size,
    1, 0, 0, NUM_PES) == NUM_KEYS_PER_PE * NUM_PES on every PE."""
    rng = np.random.default_rng(2015)
    cases = []
    for npes in (1, 2, 3, 4, 8):
        keys_per_pe = int(rng.integers(1 << 10, 1 << 24))
        total = keys_per_pe * npes
        # a random partition of the keys into per-PE buckets
        cuts = np.sort(rng.integers(0, total + 1, size=npes - 1))
        buckets = np.diff(np.concatenate([[0], cuts, [total]])).astype(np.int64)
        got = O.reduce_sim("longlong", "sum", buckets.reshape(npes, 1), 0, 0, npes)[:, 0]
        assert (got == total).all()
        cases.append({"npes": npes, "NUM_KEYS_PER_PE": keys_per_pe,
                      "my_bucket_size": buckets.tolist(), "total_num_keys": total})
    return cases


def main():
    with open(os.path.join(HERE, "reduce_hashes.json"), "w") as f:
        json.dump({"npes": NPES, "sizes": SIZES, "sets": SETS, "cases": hashes()}, f,
                  separators=(",", ":"))
    with open(os.path.join(HERE, "special_values.json"), "w") as f:
        json.dump(specials(), f, separators=(",", ":"))
    with open(os.path.join(HERE, "isx_known_answer.json"), "w") as f:
        json.dump(isx(), f, indent=1)


if __name__ == "__main__":
    main()
