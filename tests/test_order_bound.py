"""The ULP bound the RCCL-ordered float sums and products are held to
(tests/gpu_util.py order_bound; BASELINE.json north_star: "within a stated
ULP tolerance for float/double sum and prod"), checked on CPU against folds in
other orders: it accepts every order of the same sources, rejects a result off
by a few bounds, and with scale 0 (the GPU tests' negative control) rejects a
reordered fold that differs in bits."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import oracle  # noqa: E402
from gpu_util import order_bound  # noqa: E402


def fold(srcs, order, op):
    acc = srcs[order[0]].copy()
    for p in order[1:]:
        acc = acc + srcs[p] if op == "sum" else acc * srcs[p]
    return acc


@pytest.mark.parametrize("t", ["float", "double"])
@pytest.mark.parametrize("op", ["sum", "prod"])
@pytest.mark.parametrize("P", [3, 8])
def test_every_order_within_bound(t, op, P):
    srcs = oracle.sources(t, 1, P, 20000, base_seed=0xB0B + P)
    want = oracle.reduce_sim(t, op, srcs, 0, 0, P)[0]
    rng = np.random.default_rng(P)
    differ = 0
    for _ in range(6):
        got = fold(srcs, list(rng.permutation(P)), op)
        ok, inexact = order_bound(got, want, srcs, op)
        assert ok
        differ += inexact
        if inexact:
            # the negative control: bound 0 rejects what differs in bits
            assert not order_bound(got, want, srcs, op, scale=0.0)[0]
    if op == "prod" or P > 3:
        # reordering changes last bits (not a 3-term sum of these sources:
        # every 2-term partial sum of values in [-1, 1) on their 2^-23 /
        # 2^-52 grid is exact, so any order rounds the exact sum once)
        assert differ > 0


@pytest.mark.parametrize("t", ["float", "double"])
def test_rejects_results_off_by_more_than_the_bound(t):
    P = 4
    srcs = oracle.sources(t, 1, P, 5000, base_seed=0xC0C)
    want = oracle.reduce_sim(t, "sum", srcs, 0, 0, P)[0]
    u = np.finfo(want.dtype).eps / 2
    k = P - 1
    bound = 2 * k * u / (1 - k * u) * np.abs(srcs.astype(np.float64)).sum(axis=0)
    bad = want.copy()
    bad[1234] = want[1234] + want.dtype.type(3 * bound[1234]) + np.sign(want[1234]) * np.finfo(want.dtype).tiny
    assert not order_bound(bad, want, srcs, "sum")[0]
    nan = want.copy()
    nan[7] = np.nan
    assert not order_bound(nan, want, srcs, "sum")[0]


def test_integers_and_min_max_stay_bit_exact():
    srcs = oracle.sources("long", 1, 4, 100)
    want = oracle.reduce_sim("long", "sum", srcs, 0, 0, 4)[0]
    assert order_bound(want, want, srcs, "sum") == (True, 0)
    off = want.copy()
    off[3] += 1
    assert not order_bound(off, want, srcs, "sum")[0]
    f = oracle.sources("double", 1, 4, 100)
    w = oracle.reduce_sim("double", "max", f, 0, 0, 4)[0]
    w2 = w.copy()
    w2[0] = np.nextafter(w2[0], 2.0)
    assert not order_bound(w2, w, f, "max")[0]
