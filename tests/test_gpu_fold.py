"""GPU parity of the fold kernels against the oracle (through the C ABI).

The fold kernel is the arithmetic of the whole path: every PE's result in the
reference is a left fold of the active set's sources (reduce-op.c:213-248).
On the GPU the multi-PE exchange only moves bytes (RCCL), so a fold of P
sources in a given order on one GPU must equal the oracle's output of the PE
whose order that is:
  * order 0..P-1            -> the reference's PE_start (A2A path, all PEs)
  * order me, others asc.   -> the reference's PE `me`  (GATHER path)
Bit-exact for every type/op (floats included: same op order, same IEEE ops).
"""
import numpy as np
import pytest
from gpu_util import from_dev, same_bits, to_dev

pytestmark = pytest.mark.gpu

DEVICE_PAIRS = [
    ("short", o) for o in ("sum", "prod", "and", "or", "xor", "min", "max")] + [
    ("int", o) for o in ("sum", "prod", "and", "or", "xor", "min", "max")] + [
    ("long", o) for o in ("sum", "prod", "and", "or", "xor", "min", "max")] + [
    ("longlong", o) for o in ("sum", "prod", "and", "or", "xor", "min", "max")] + [
    ("float", o) for o in ("sum", "prod", "min", "max")] + [
    ("double", o) for o in ("sum", "prod", "min", "max")] + [
    ("longdouble", o) for o in ("sum", "prod", "min", "max")] + [
    ("complexd", "sum"), ("complexd", "prod"), ("complexf", "sum"), ("complexf", "prod")]

SIZES = [1, 2, 63, 64, 65, 127, 1000, 4103, 65536 + 13]


@pytest.mark.parametrize("t,op", DEVICE_PAIRS)
def test_fold_pe_start_order_matches_oracle(cuda, shm, oracle, t, op):
    import torch
    for kind in (0, 1):
        for P in (1, 2, 3, 5, 8):
            for n in (SIZES if P in (2, 5) else SIZES[:7]):
                srcs = oracle.sources(t, kind, P, n, base_seed=0x5EED0000 + 97 * P + n)
                want = oracle.reduce_sim(t, op, srcs, 0, 0, P)[0]
                ins = [to_dev(torch, srcs[p]) for p in range(P)]
                out = torch.empty_like(ins[0])
                shm.fold_n(t, op, out, ins, n)
                torch.cuda.synchronize()
                got = from_dev(out, srcs.dtype)
                assert same_bits(got, want), f"{t} {op} kind={kind} P={P} n={n}"


@pytest.mark.parametrize("t,op", [("double", "sum"), ("double", "prod"), ("float", "sum"),
                                  ("float", "prod"), ("double", "min"), ("complexd", "prod"),
                                  ("complexf", "sum")])
def test_fold_gather_order_every_pe(cuda, shm, oracle, t, op):
    """GATHER algorithm order (me first, then ascending) == reference PE me."""
    import torch
    P, n = 5, 4103
    srcs = oracle.sources(t, 1, P, n)
    want = oracle.reduce_sim(t, op, srcs, 0, 0, P)
    dev = [to_dev(torch, srcs[p]) for p in range(P)]
    for me in range(P):
        order = [me] + [p for p in range(P) if p != me]
        out = torch.empty_like(dev[0])
        shm.fold_n(t, op, out, [dev[p] for p in order], n)
        torch.cuda.synchronize()
        assert same_bits(from_dev(out, srcs.dtype), want[me]), f"PE {me}"


@pytest.mark.parametrize("t,op", [("double", "sum"), ("int", "xor"), ("short", "max"),
                                  ("float", "min"), ("complexf", "prod")])
def test_fold_in_place_acc(cuda, shm, oracle, t, op):
    """shmemx_fold: acc = op(acc, in), the inner loop reduce-op.c:231-235."""
    import torch
    n = 10007
    srcs = oracle.sources(t, 1, 2, n)
    want = oracle.reduce_sim(t, op, srcs, 0, 0, 2)[0]
    acc, inp = to_dev(torch, srcs[0]), to_dev(torch, srcs[1])
    shm.fold(t, op, acc, inp, n)
    torch.cuda.synchronize()
    assert same_bits(acc.cpu().numpy(), want)


@pytest.mark.parametrize("t", ["double", "int", "short", "complexf"])
def test_fold_misaligned_and_mixed_alignment(cuda, shm, oracle, t):
    """Head/tail peeling (same offset mod 16) and the all-scalar path
    (inputs at different offsets mod 16), as 8-byte dlmalloc pointers give."""
    import torch
    P, n = 3, 5003
    srcs = oracle.sources(t, 1, P, n + 8)
    isz = srcs.itemsize
    for offs in ([1, 1, 1, 1], [0, 1, 2, 3], [3, 0, 1, 1], [1, 0, 0, 0]):
        if 16 // isz <= 1 and any(offs):
            continue
        want = oracle.reduce_sim(t, "sum", np.stack([srcs[p][offs[p + 1]:offs[p + 1] + n]
                                                     for p in range(P)]), 0, 0, P)[0]
        dev = [to_dev(torch, srcs[p]) for p in range(P)]
        outbuf = torch.zeros(n + 8, dtype=dev[0].dtype, device="cuda")
        out = outbuf[offs[0]:offs[0] + n]
        ins = [dev[p][offs[p + 1]:offs[p + 1] + n] for p in range(P)]
        shm.fold_n(t, "sum", out, ins, n)
        torch.cuda.synchronize()
        got = outbuf.cpu().numpy()
        assert same_bits(got[offs[0]:offs[0] + n], want), f"offs={offs}"
        assert not got[:offs[0]].any() and not got[offs[0] + n:].any(), "wrote outside"


def test_fold_long_chain_beyond_16_inputs(cuda, shm, oracle):
    """More inputs than one launch takes: chained launches keep the order."""
    import torch
    P, n = 37, 999
    srcs = oracle.sources("double", 1, P, n)
    want = oracle.reduce_sim("double", "sum", srcs, 0, 0, P)[0]
    dev = [to_dev(torch, srcs[p]) for p in range(P)]
    out = torch.empty_like(dev[0])
    shm.fold_n("double", "sum", out, dev, n)
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), want)


def _special(t):
    if t in ("float", "double"):
        ft = np.float32 if t == "float" else np.float64
        tiny = np.finfo(ft).tiny
        vals = [np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf, 1.0, -1.0,
                tiny, -tiny, tiny / 4, np.finfo(ft).max, -np.finfo(ft).max, 2.5]
        return np.array(vals, dtype=ft)
    info = np.iinfo({"short": np.int16, "int": np.int32, "long": np.int64}[t])
    return np.array([info.min, info.max, 0, -1, 1, info.min + 1, info.max - 1, 12345],
                    dtype=info.dtype)


@pytest.mark.parametrize("t", ["float", "double", "short", "int", "long"])
def test_fold_special_values_all_pairs(cuda, shm, oracle, t):
    """NaN / +-0 / inf / subnormals / integer wrap, every ordered pair, every op.
    min/max are selects: bit-exact even for NaN payloads and signed zeros.
    sum/prod: bit-exact except NaN results, which must be NaN on both sides
    (the NaN payload an add produces is not specified by IEEE 754)."""
    import torch
    v = _special(t)
    a = np.repeat(v, len(v))
    b = np.tile(v, len(v))
    srcs = np.stack([a, b])
    ops = ["sum", "prod", "min", "max"] + ([] if t in ("float", "double") else ["and", "or", "xor"])
    for op in ops:
        for order in ((0, 1), (1, 0)):
            want = oracle.reduce_sim(t, op, srcs[list(order)], 0, 0, 2)[0]
            out = torch.empty(len(a), dtype=to_dev(torch, a).dtype, device="cuda")
            shm.fold_n(t, op, out, [to_dev(torch, srcs[order[0]]), to_dev(torch, srcs[order[1]])],
                       len(a))
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            if t in ("float", "double") and op in ("sum", "prod"):
                nan_w, nan_g = np.isnan(want), np.isnan(got)
                assert np.array_equal(nan_w, nan_g), op
                assert same_bits(got[~nan_g], want[~nan_w]), op
            else:
                assert same_bits(got, want), (op, order)


@pytest.mark.parametrize("t", ["complexd", "complexf"])
def test_complex_prod_annex_g(cuda, shm, oracle, t):
    """Complex multiply with inf/NaN parts: the __muldc3 recovery branch."""
    import torch
    ft = np.float64 if t == "complexd" else np.float32
    parts = np.array([0.0, -0.0, 1.0, -2.0, np.inf, -np.inf, np.nan, 3.5], dtype=ft)
    zs = np.array([complex(x, y) for x in parts for y in parts],
                  dtype=np.complex128 if t == "complexd" else np.complex64)
    a, b = np.repeat(zs, len(zs)), np.tile(zs, len(zs))
    want = oracle.reduce_sim(t, "prod", np.stack([a, b]), 0, 0, 2)[0]
    out = torch.empty(len(a), dtype=to_dev(torch, a).dtype, device="cuda")
    shm.fold_n(t, "prod", out, [to_dev(torch, a), to_dev(torch, b)], len(a))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for comp in ("real", "imag"):
        g, w = getattr(got, comp), getattr(want, comp)
        assert np.array_equal(np.isnan(g), np.isnan(w)), comp
        m = ~np.isnan(w)
        assert g[m].tobytes() == w[m].tobytes(), comp


def test_fold_full_size_double_sum(cuda, shm, oracle):
    """BASELINE configs[1] size (32 Mi doubles): acc += in must equal the
    oracle's 2-PE PE_start result; checked exactly against numpy's a+b (one
    IEEE add per element, the identical operation) and on a sampled window
    against the oracle itself."""
    import torch
    n = 32 * 1024 * 1024
    a = oracle.fill("double", 0, 0x5EED0000, n)
    b = oracle.fill("double", 0, 0x5EED0001, n)
    acc, inp = to_dev(torch, a), to_dev(torch, b)
    shm.fold("double", "sum", acc, inp, n)
    torch.cuda.synchronize()
    got = acc.cpu().numpy()
    assert same_bits(got, a + b)
    lo = n // 2 - 4099
    win = oracle.reduce_sim("double", "sum", np.stack([a[lo:lo + 8192], b[lo:lo + 8192]]), 0, 0, 2)[0]
    assert same_bits(got[lo:lo + 8192], win)


def _random_x87(rng, n):
    """n random 80-bit encodings in 16-byte slots: normals over the whole
    exponent range and near 1, denormals, pseudo-denormals, zeros, infs,
    quiet/signalling NaNs, pseudo-NaNs and unnormals, and raw patterns."""
    sig = rng.integers(0, 2**64, size=n, dtype=np.uint64)
    exp = rng.integers(0, 0x8000, size=n, dtype=np.uint64)
    cls = rng.integers(0, 8, size=n)
    top = np.uint64(1 << 63)
    sig = np.where(cls == 0, sig | top, sig)                                   # normal
    exp = np.where(cls == 0, 1 + exp % 0x7FFE, exp)
    sig = np.where(cls == 1, sig | top, sig)                                   # near 1.0
    exp = np.where(cls == 1, 16380 + exp % 7, exp)
    exp = np.where(cls == 2, 0, exp)                                           # denormal / pseudo
    sig = np.where(cls == 3, top, sig)                                         # inf
    exp = np.where(cls == 3, 0x7FFF, exp)
    sig = np.where(cls == 4, sig | top, sig)                                   # NaN
    exp = np.where(cls == 4, 0x7FFF, exp)
    sig = np.where(cls == 5, 0, sig)                                           # zero
    exp = np.where(cls == 5, 0, exp)
    sign = rng.integers(0, 2, size=n, dtype=np.uint64) << np.uint64(15)
    slots = np.zeros((n, 2), dtype=np.uint64)
    slots[:, 0] = sig
    slots[:, 1] = exp | sign
    return slots.view(np.longdouble).reshape(n)


def test_longdouble_x87_encodings(cuda, shm, oracle):
    """The soft x87 on the GPU against the host x87 (through the oracle) over
    random 80-bit encodings, every op, both PE orders, value bytes exact."""
    import torch
    rng = np.random.default_rng(87)
    n = 1 << 16
    a, b = _random_x87(rng, n), _random_x87(rng, n)
    b[: n // 4] = a[: n // 4]                       # equal operands
    b[n // 4: n // 2] = -a[n // 4: n // 2]          # exact cancellation
    srcs = np.stack([a, b])
    for op in ("sum", "prod", "min", "max"):
        for order in ((0, 1), (1, 0)):
            want = oracle.reduce_sim("longdouble", op, srcs[list(order)], 0, 0, 2)[0]
            out = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
            shm.fold_n("longdouble", op, out, [to_dev(torch, srcs[order[0]]),
                                               to_dev(torch, srcs[order[1]])], n)
            torch.cuda.synchronize()
            got = from_dev(out, np.longdouble)
            assert same_bits(got, want), (op, order)


@pytest.mark.parametrize("peers", [False, True])
def test_fold_fuzz_against_oracle(cuda, shm, oracle, peers):
    """400 random cases: type, op, 1..20 inputs, 0..70 000 elements, random
    element offsets per array (same or different alignment mod 16), kind.
    peers: the same through shmemx_fold_n_peers_on_stream (DIRECT's and
    SIGNAL's fold, all inputs' loads in flight), which must agree bit for bit."""
    import torch
    rng = np.random.default_rng(20251015 + peers)
    pairs = DEVICE_PAIRS
    for case in range(400):
        t, op = pairs[rng.integers(len(pairs))]
        P = int(rng.integers(1, 21))
        n = int(rng.integers(0, 70000)) if case % 4 else int(rng.integers(0, 300))
        kind = int(rng.integers(0, 2))
        srcs = oracle.sources(t, kind, P, n + 8, base_seed=int(rng.integers(1 << 40)))
        offs = rng.integers(0, 4, size=P + 1) if case % 3 else np.full(P + 1, int(rng.integers(0, 4)))
        dt = srcs.dtype
        if dt.itemsize >= 16:
            offs[:] = 0
        view = np.stack([srcs[p][offs[p + 1]:offs[p + 1] + n] for p in range(P)])
        want = oracle.reduce_sim(t, op, view, 0, 0, P)[0]
        dev = [to_dev(torch, srcs[p]) for p in range(P)]
        isz = dt.itemsize
        ins = [d[offs[p + 1] * isz:(offs[p + 1] + n) * isz] if dt == np.longdouble
               else d[offs[p + 1]:offs[p + 1] + n] for p, d in enumerate(dev)]
        outbuf = to_dev(torch, np.zeros(n + 8, dtype=dt))
        out = outbuf[offs[0] * isz:(offs[0] + n) * isz] if dt == np.longdouble \
            else outbuf[offs[0]:offs[0] + n]
        shm.fold_n(t, op, out, ins, n, peers=peers)
        torch.cuda.synchronize()
        got = from_dev(outbuf, dt)
        assert same_bits(got[offs[0]:offs[0] + n], want), (case, t, op, P, n, list(offs))
        assert not np.any(got[:offs[0]] != 0) and not np.any(got[offs[0] + n:] != 0), case


@pytest.mark.parametrize("t", ["short", "int", "long", "float", "double", "longdouble", "complexd", "complexf"])
def test_copy_moves_bits_every_size_offset_and_nt_path(cuda, shm, t):
    """The copy (one input: the PE_size = 1 call, reduce-op.c:213-216) runs one
    bit-moving kernel per element size (fold_kernels.hip launch_copy): random
    bytes, NaN payloads and long double padding included, come out identical,
    at every element offset mod 16 (the scalar head and tail), for lengths
    around one workgroup's chunk, and above the 32 MiB non-temporal cut; the
    bytes around the target are untouched."""
    import torch
    sz = shm.type_size(t)
    rng = np.random.default_rng(hash(t) & 0xFFFF)
    chunk = 256 * 8 * 16 // sz              # one workgroup: 256 lanes x 8 vectors
    lens = [1, 3, chunk - 1, chunk, chunk + 1, 3 * chunk + 7, (17 << 20) // sz + 5]
    for n in lens:
        for off in range(0, 16, sz) if n < 1 << 20 else (0, 16 - sz if sz < 16 else 0):
            src = torch.from_numpy(rng.integers(0, 256, n * sz + 64, dtype=np.uint8)).cuda()
            dst = torch.full((n * sz + 64,), 0xA5, dtype=torch.uint8, device="cuda")
            s_off = off if n % 2 else (off + sz) % 16   # same / different alignment mod 16
            shm.fold_n(t, "sum", dst[off:off + n * sz], [src[s_off:s_off + n * sz]], n)
            torch.cuda.synchronize()
            assert torch.equal(dst[off:off + n * sz], src[s_off:s_off + n * sz]), (t, n, off, s_off)
            assert bool((dst[:off] == 0xA5).all()) and bool((dst[off + n * sz:] == 0xA5).all()), (t, n, off)


def test_kernel_clock_times_fold_and_copy(cuda, shm):
    """shmemx_kernel_timing / shmemx_kernel_times: every fold-family launch
    while on is timed by its own dispatch events, in launch order, with its
    kind; off, nothing is recorded; results are unchanged."""
    import torch
    n = 8 << 20
    a = torch.rand(n, dtype=torch.float64, device="cuda")
    b = torch.rand(n, dtype=torch.float64, device="cuda")
    want = a + b
    shm.kernel_timing(True)
    shm.fold("double", "sum", a, b, n)                       # a += b: the 2-input fold
    shm.fold_n("double", "sum", b, [a], n)                   # b = a: the copy
    shm.fold_n("double", "max", a, [a, b, a], n)             # the P-input fold
    torch.cuda.synchronize()
    kt, dropped = shm.kernel_times()
    shm.kernel_timing(False)
    assert [k for k, _ in kt] == ["fold", "copy", "fold"] and dropped == 0, kt
    # 192 / 128 / 256 MiB: tens of microseconds each at HBM speed
    assert all(5.0 < us < 5000.0 for _, us in kt), kt
    assert torch.equal(a, want) and torch.equal(b, want)
    shm.fold("double", "sum", a, b, n)
    torch.cuda.synchronize()
    assert shm.kernel_times() == ([], 0)
