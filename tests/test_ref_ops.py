"""The oracle's element operations against the REFERENCE'S OWN, compiled.

reduce-op.c:71-150 (every <op>_<type>_func the reference defines) builds on
its own: oracle/build_ref.sh compiles that text, where it lies, into
oracle/_ref/libref_ops.so.  tests/golden/ref_element_ops.json holds what it
computes on special values (NaN payloads, signalling NaNs, +-0, +-inf,
subnormals, integer extremes, x87 pseudo-encodings, Annex G complex inf/NaN
mixes) and seeded random bit patterns, in both operand orders
(tests/golden/make_ref_ops.py).

  * the fixture pins the oracle on every host, the GPU box included;
  * where the reference is present, the fixture is re-derived from it and the
    oracle is held against it on a million random bit patterns per pair.
Test infrastructure only.
"""
import base64
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def fixture():
    with open(os.path.join(GOLDEN, "ref_element_ops.json")) as f:
        return json.load(f)


def _dec(oracle, s, t):
    return np.frombuffer(base64.b64decode(s), dtype=oracle.NP_DTYPE[t]).copy()


def _value_bytes(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.longdouble:
        return np.ascontiguousarray(a.view(np.uint8).reshape(-1, a.itemsize)[:, :10]).tobytes()
    return a.tobytes()


def _ref_lib(oracle):
    import ctypes
    path = os.path.join(os.path.dirname(oracle.LIB_PATH), "_ref", "libref_ops.so")
    if not os.path.exists(path):
        pytest.skip("oracle/_ref not built (no /root/reference on this host)")
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.ref_op_apply.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, ctypes.c_long]
    L.ref_op_apply.restype = ctypes.c_int
    return L


def _ref_apply(L, oracle, t, op, a, b):
    out = np.zeros_like(a)
    rc = L.ref_op_apply(oracle.TYPES[t], oracle.OPS[op], a.ctypes.data, b.ctypes.data,
                        out.ctypes.data, a.size)
    return out if rc == 0 else None


def test_fixture_covers_every_reference_pair(oracle, fixture):
    """The reference defines <op>_<type>_func exactly for the pairs the oracle
    (and the API, reduce-op.c:388-431) accepts."""
    n = 0
    for t in oracle.TYPES:
        have = set(fixture["cases"][t]["ops"])
        want = {op for op in oracle.OPS if oracle.op_valid(t, op)}
        assert have == want, t
        n += len(have)
    assert n == 44


def test_oracle_element_ops_reproduce_reference_fixture(oracle, fixture):
    """PE 0 of a 2-PE reduction computes op(a, b), PE 1 op(b, a)
    (reduce-op.c:213-248); the oracle must give the reference's bytes in both
    orders, NaN payloads included (both are x86 code)."""
    checked = 0
    for t, c in fixture["cases"].items():
        a, b = _dec(oracle, c["a"], t), _dec(oracle, c["b"], t)
        for op, o in c["ops"].items():
            tg = oracle.reduce_sim(t, op, np.stack([a, b]), 0, 0, 2)
            assert _value_bytes(tg[0]) == _value_bytes(_dec(oracle, o["ab"], t)), (t, op)
            assert _value_bytes(tg[1]) == _value_bytes(_dec(oracle, o["ba"], t)), (t, op)
            checked += 2 * a.size
    assert checked > 40000


def test_fixture_is_what_the_reference_computes(oracle, fixture):
    L = _ref_lib(oracle)
    for t, c in fixture["cases"].items():
        a, b = _dec(oracle, c["a"], t), _dec(oracle, c["b"], t)
        for op in oracle.OPS:
            got = _ref_apply(L, oracle, t, op, a, b)
            if op not in c["ops"]:
                assert got is None, (t, op)
                continue
            assert got.tobytes() == _dec(oracle, c["ops"][op]["ab"], t).tobytes(), (t, op)
            got = _ref_apply(L, oracle, t, op, b, a)
            assert got.tobytes() == _dec(oracle, c["ops"][op]["ba"], t).tobytes(), (t, op)


def _random_bits(oracle, t, n, seed):
    dt = np.dtype(oracle.NP_DTYPE[t])
    w = oracle.splitmix64(seed, n * max(1, dt.itemsize // 8))
    if dt.itemsize < 8:
        return w.astype(f"u{dt.itemsize}").view(dt)
    raw = w.view(np.uint8).reshape(n, dt.itemsize).copy()
    if t == "longdouble":
        raw[:, 10:] = 0
    return raw.view(dt).reshape(n)


@pytest.mark.parametrize("t", ["short", "int", "long", "longlong", "float", "double",
                               "longdouble", "complexd", "complexf"])
def test_oracle_matches_reference_on_random_bits(oracle, t):
    """Random bit patterns (every exponent, NaN and subnormal the type has),
    2^20 pairs per (type, op), both orders, against the compiled reference."""
    L = _ref_lib(oracle)
    n = 1 << 20 if t != "longdouble" else 1 << 18
    a = _random_bits(oracle, t, n, 0xA11CE + oracle.TYPES[t])
    b = _random_bits(oracle, t, n, 0xB0B0 + oracle.TYPES[t])
    for op in oracle.OPS:
        if not oracle.op_valid(t, op):
            continue
        tg = oracle.reduce_sim(t, op, np.stack([a, b]), 0, 0, 2)
        assert _value_bytes(tg[0]) == _value_bytes(_ref_apply(L, oracle, t, op, a, b)), (t, op)
        assert _value_bytes(tg[1]) == _value_bytes(_ref_apply(L, oracle, t, op, b, a)), (t, op)


def test_reference_build_stays_in_this_container():
    """oracle/_ref (an object compiled from the reference's text) never travels
    to the GPU box: .gpurunignore lists it (SURVEY.md "neither source nor
    objects ship"), and no GPU test loads it (they read the golden fixture)."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(repo, ".gpurunignore")) as f:
        pats = [ln.strip() for ln in f if ln.strip() and not ln.startswith("#")]
    assert "./oracle/_ref" in pats, pats
    for name in os.listdir(os.path.join(repo, "tests")):
        if name.startswith("test_gpu") and name.endswith(".py"):
            with open(os.path.join(repo, "tests", name)) as f:
                assert "libref_ops" not in f.read(), name
