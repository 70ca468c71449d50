"""CPU tests of the oracle (the restatement of reduce-op.c used as checker).

Pinning, in order of strength (DESIGN.md "Oracle"):
  1. the reference's own known-answer check, ISx (isx.c:615-624);
  2. an independent numpy formulation of reduce-op.c's semantics (per-PE
     left fold in the reference's order, C operators), bit-exact;
  3. the committed golden vectors (regression);
  4. the fork-per-PE harness (the GASNet smp model) agreeing with the
     single-process simulation.
"""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def members(s):
    return [s[0] + i * (1 << s[1]) for i in range(s[2])]


def test_splitmix_and_fill_match_c(oracle):
    L = oracle.lib()
    for i in (0, 1, 7, 1000):
        assert int(L.oracle_splitmix64(12345, i)) == int(oracle.splitmix64(12345, 1, start=i)[0])
    for t in oracle.TYPES:
        for kind in (0, 1):
            n = 333
            a = np.zeros(n, oracle.NP_DTYPE[t])
            L.oracle_fill(oracle.TYPES[t], kind, 42, a.ctypes.data, n)
            b = oracle.fill(t, kind, 42, n)
            if t == "longdouble":
                assert np.array_equal(a, b)
            else:
                assert a.tobytes() == b.tobytes(), (t, kind)


def test_isx_known_answer(oracle):
    """The only known-answer use of the path in the reference."""
    with open(os.path.join(GOLDEN, "isx_known_answer.json")) as f:
        cases = json.load(f)
    for c in cases:
        b = np.array(c["my_bucket_size"], dtype=np.int64).reshape(c["npes"], 1)
        got = oracle.reduce_sim("longlong", "sum", b, 0, 0, c["npes"])[:, 0]
        assert (got == c["NUM_KEYS_PER_PE"] * c["npes"]).all()
        assert (got == c["total_num_keys"]).all()


def _np_op(op, a, b):
    if op == "sum":
        return a + b
    if op == "prod":
        return a * b
    if op == "and":
        return a & b
    if op == "or":
        return a | b
    if op == "xor":
        return a ^ b
    if op == "min":
        return np.where(a < b, a, b)
    return np.where(a > b, a, b)


def _numpy_reference(t, op, srcs, s):
    """reduce-op.c:213-248 in numpy: PE me computes src[me] then folds every
    other member in ascending order, C semantics (wrapping ints, short via
    int, IEEE ops, selects for min/max)."""
    out = np.zeros_like(srcs)
    mem = members(s)
    for me in mem:
        r = srcs[me].copy()
        for p in mem:
            if p == me:
                continue
            if t == "short":
                r = _np_op(op, r.astype(np.int32), srcs[p].astype(np.int32)).astype(np.int16)
            else:
                with np.errstate(over="ignore", invalid="ignore"):
                    r = _np_op(op, r, srcs[p]).astype(srcs.dtype)
        out[me] = r
    return out


@pytest.mark.parametrize("t", ["short", "int", "long", "longlong", "float", "double",
                               "longdouble", "complexd", "complexf"])
def test_oracle_matches_independent_numpy(oracle, t):
    ops = [o for o in ("sum", "prod", "and", "or", "xor", "min", "max") if oracle.op_valid(t, o)]
    for op in ops:
        if t in ("complexd", "complexf") and op == "prod":
            continue  # numpy's complex multiply is not libgcc's __muldc3; see below
        for kind in (0, 1):
            for s in [(0, 0, 1), (0, 0, 2), (0, 0, 4), (1, 0, 3), (0, 1, 4), (1, 1, 3)]:
                srcs = oracle.sources(t, kind, 8, 130, base_seed=0xABC + kind)
                want = _numpy_reference(t, op, srcs, s)
                got = oracle.reduce_sim(t, op, srcs, *s)
                for me in members(s):
                    if t == "longdouble":
                        assert np.array_equal(got[me], want[me]), (op, kind, s, me)
                    else:
                        assert got[me].tobytes() == want[me].tobytes(), (op, kind, s, me)


@pytest.mark.parametrize("t", ["complexd", "complexf"])
def test_oracle_complex_prod_finite_close_to_numpy(oracle, t):
    srcs = oracle.sources(t, 1, 4, 500)
    got = oracle.reduce_sim(t, "prod", srcs, 0, 0, 4)
    want = srcs[0] * srcs[1] * srcs[2] * srcs[3]
    eps = np.finfo(np.float64 if t == "complexd" else np.float32).eps
    assert np.allclose(got[0], want, rtol=16 * eps, atol=0)


def test_fold_order_is_pe_dependent(oracle):
    """PE 0 and PE 1 agree (a+b == b+a), PEs >= 2 differ in the
    last bits for floating sums; integers agree everywhere."""
    # kind 0: [1, 2) values whose 4-term sums need rounding (the kind-1
    # [-1, 1) values are multiples of 2^-52 and mostly sum exactly)
    srcs = oracle.sources("double", 0, 4, 4096)
    out = oracle.reduce_sim("double", "sum", srcs, 0, 0, 4)
    assert out[0].tobytes() == out[1].tobytes()
    assert out[2].tobytes() != out[0].tobytes()
    assert out[3].tobytes() != out[0].tobytes()
    isrcs = oracle.sources("long", 1, 4, 4096)
    iout = oracle.reduce_sim("long", "sum", isrcs, 0, 0, 4)
    assert all(iout[p].tobytes() == iout[0].tobytes() for p in range(4))


def test_inactive_pes_untouched_and_zero_length(oracle):
    srcs = oracle.sources("int", 1, 8, 100)
    tg = np.full_like(srcs, 0x5A5A5A5A)
    out = oracle.reduce_sim("int", "xor", srcs, 1, 1, 3, targets=tg)
    for p in range(8):
        if p in (1, 3, 5):
            assert not (out[p] == 0x5A5A5A5A).all()
        else:
            assert (out[p] == 0x5A5A5A5A).all()
    empty = np.zeros((8, 0), np.int32)
    assert oracle.reduce_sim("int", "sum", empty, 0, 0, 8).shape == (8, 0)


def test_invalid_arguments_rejected(oracle):
    srcs = oracle.sources("int", 1, 4, 10)
    with pytest.raises(ValueError):
        oracle.reduce_sim("int", "sum", srcs, 0, 0, 5)     # beyond npes
    with pytest.raises(ValueError):
        oracle.reduce_sim("float", "xor", oracle.sources("float", 1, 4, 10), 0, 0, 4)
    with pytest.raises(ValueError):
        oracle.reduce_sim("complexd", "min", oracle.sources("complexd", 1, 2, 10), 0, 0, 2)


def test_golden_hashes(oracle):
    """Every committed case reproduces (regression pin of the oracle)."""
    with open(os.path.join(GOLDEN, "reduce_hashes.json")) as f:
        g = json.load(f)
    npes = g["npes"]
    cache = {}
    for key, want in g["cases"].items():
        t, op, k, n, sset = key.split("|")
        kind, n = int(k[1:]), int(n[1:])
        s = tuple(int(x) for x in sset[3:].split(","))
        ck = (t, kind, n)
        if ck not in cache:
            seed = 0x5EED0000 + 1009 * list(oracle.TYPES).index(t) + n
            cache[ck] = oracle.sources(t, kind, npes, n, base_seed=seed)
        tg = oracle.reduce_sim(t, op, cache[ck], *s)
        mem = set(members(s))
        got = [f"{oracle.value_hash(t, tg[p]):016x}" if p in mem else "0" for p in range(npes)]
        assert got == want, key


def test_golden_special_values(oracle):
    with open(os.path.join(GOLDEN, "special_values.json")) as f:
        g = json.load(f)
    for key, c in g.items():
        t, op = key.split("|")
        dt = np.dtype(oracle.NP_DTYPE[t])
        ut = f"u{dt.itemsize}"
        a = np.array(c["a"], dtype=ut).view(dt)
        b = np.array(c["b"], dtype=ut).view(dt)
        tg = oracle.reduce_sim(t, op, np.stack([a, b]), 0, 0, 2)
        assert tg[0].view(ut).tolist() == c["pe0"], key
        assert tg[1].view(ut).tolist() == c["pe1"], key


def test_min_max_nan_semantics(oracle):
    """a<b?a:b is not fmin: NaN on either side returns b (reduce-op.c:135)."""
    nan = np.nan
    srcs = np.array([[nan, 1.0, -0.0, 0.0], [1.0, nan, 0.0, -0.0]])
    out = oracle.reduce_sim("double", "min", srcs, 0, 0, 2)
    assert out[0][0] == 1.0 and np.isnan(out[1][0])       # PE-dependent
    assert np.isnan(out[0][1]) and out[1][1] == 1.0
    assert np.signbit(out[0][2]) == False and np.signbit(out[1][2]) == True  # noqa: E712


@pytest.mark.parametrize("s", [(0, 0, 2), (0, 0, 4), (1, 1, 3), (2, 0, 3)])
def test_fork_harness_agrees_with_sim(oracle, s):
    npes = 8
    n = 1000
    times, hashes = oracle.reduce_fork("double", "sum", npes, *s, n, kind=1,
                                       base_seed=0x5EED0000, reps=2, pin_base=-1)
    srcs = oracle.sources("double", 1, npes, n, base_seed=0x5EED0000)
    tg = oracle.reduce_sim("double", "sum", srcs, *s)
    mem = set(members(s))
    for p in range(npes):
        want = oracle.value_hash("double", tg[p]) if p in mem else 0
        assert hashes[p] == want, p
    assert all(t > 0 for t in times)


def test_config1_int_sum_1024_two_pes_fork(oracle):
    """BASELINE.json configs[0]: shmem_int_sum_to_all, nreduce = 1024, 2 PEs
    as 2 processes over shared memory (the reference's oshrun smp loopback
    model, oshrun.in:97-98): both PEs hold the exact sum."""
    times, hashes = oracle.reduce_fork("int", "sum", 2, 0, 0, 2, 1024, kind=1, reps=3)
    srcs = oracle.sources("int", 1, 2, 1024)
    want = (srcs[0].astype(np.int64) + srcs[1]).astype(np.int32)     # wraps like C
    assert hashes[0] == hashes[1] == oracle.value_hash("int", want)


def test_fold_time_is_the_local_reduce(oracle):
    """oracle_fold_time (bench.py's cpu_baseline: the N = 1 GPU step's
    workload on one core) runs the reference's per-peer fold and reports one
    positive time per repetition; bad arguments are refused."""
    t = oracle.fold_time("double", "sum", 100000, reps=3, pin=-1)
    assert len(t) == 3 and all(x > 0 for x in t)
    with pytest.raises(RuntimeError):
        oracle.fold_time("double", "xor", 10, reps=1)


def test_reduce_one_matches_reduce_sim():
    """oracle_reduce_one (one PE's target, for full-size GPU checks) is the
    same loop as oracle_reduce_sim: every pair, several active sets, every
    member, value bytes equal (long double padding is unspecified)."""
    import oracle as O
    cases = 0
    for t in O.TYPES:
        for op in O.OPS:
            if not O.op_valid(t, op):
                continue
            srcs = O.sources(t, 1, 5, 1001)
            for st in ((0, 0, 5), (1, 1, 2), (2, 0, 3), (4, 0, 1)):
                ref = O.reduce_sim(t, op, srcs, *st)
                for m in range(st[2]):
                    pe = st[0] + m * (1 << st[1])
                    assert O.value_hash(t, ref[pe]) == O.value_hash(t, O.reduce_one(t, op, srcs, *st, pe))
                    cases += 1
    assert cases == 484
