"""CPU tests of the oracle restatements of the neighbouring collectives
(SURVEY.md §8f): broadcast (broadcast-linear.c:54-74) and [f]collect
(fcollect-linear.c:69-91, collect-linear.c:57-130), against the definitions
written directly in numpy."""
import numpy as np
import pytest

SETS = [(0, 0, 1), (0, 0, 2), (0, 0, 8), (1, 0, 3), (0, 1, 4), (1, 1, 3), (2, 0, 5)]


def members(s):
    return [s[0] + i * (1 << s[1]) for i in range(s[2])]


@pytest.mark.parametrize("dt", [np.int32, np.int64])
@pytest.mark.parametrize("s", SETS)
def test_broadcast(oracle, dt, s):
    rng = np.random.default_rng(1)
    srcs = rng.integers(-2**30, 2**30, size=(8, 77)).astype(dt)
    tg0 = np.full_like(srcs, -7)
    for root in range(s[2]):
        out = oracle.broadcast_sim(srcs, tg0, root, *s)
        rpe = members(s)[root]
        for p in range(8):
            if p in members(s) and p != rpe:
                assert (out[p] == srcs[rpe]).all()
            else:
                assert (out[p] == -7).all()          # root and non-members untouched
    with pytest.raises(ValueError):
        oracle.broadcast_sim(srcs, tg0, s[2], *s)


@pytest.mark.parametrize("dt", [np.int32, np.int64])
@pytest.mark.parametrize("s", SETS)
def test_fcollect_and_collect(oracle, dt, s):
    rng = np.random.default_rng(2)
    maxn = 50
    srcs = rng.integers(-2**30, 2**30, size=(8, maxn)).astype(dt)
    mem = members(s)
    for fixed in (True, False):
        nel = [maxn] * 8 if fixed else [int(x) for x in rng.integers(0, maxn + 1, size=8)]
        tg0 = np.full((8, maxn * 8), -3, dtype=dt)
        out = oracle.collect_sim(srcs, nel, tg0, *s)
        want = np.concatenate([srcs[p][:nel[p]] for p in mem])
        for p in range(8):
            if p in mem:
                assert (out[p][:len(want)] == want).all()
                assert (out[p][len(want):] == -3).all()
            else:
                assert (out[p] == -3).all()
