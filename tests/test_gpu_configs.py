"""BASELINE.json configs as GPU parity cases at their full sizes, through
size-independent properties (the oracle restatement is far too slow there):

* configs[1]/[2]: double sum, nreduce = 32 Mi — see test_gpu_fold.py
  (test_fold_full_size_double_sum, bit-exact vs numpy a+b).
* configs[3]: long and/or/xor, nreduce = 64 Mi, 4 PEs — the A2A fold of 4
  sources must equal an independent reduction (torch bitwise ops on the GPU,
  order-free for bitwise ops) bit for bit, and the fold must be idempotent /
  have the algebraic identities of each op (x & x = x, x ^ x = 0).
* configs[4]: float sum, nreduce 4 Ki .. 256 Mi (x4 steps) — the 2-input fold
  equals torch's a + b (one IEEE add, the same operation) bit for bit at
  every size of the sweep, 8-PE fold in set order equals the left fold.
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("op", ["and", "or", "xor"])
def test_config4_long_bitwise_64mi_4pes(cuda, shm, op):
    import torch
    n, P = 64 * 1024 * 1024, 4
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    srcs = [torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
            for _ in range(P)]
    out = torch.empty_like(srcs[0])
    shm.fold_n("long", op, out, srcs, n)
    f = {"and": torch.bitwise_and, "or": torch.bitwise_or, "xor": torch.bitwise_xor}[op]
    want = srcs[0].clone()
    for s in srcs[1:]:
        want = f(want, s)
    torch.cuda.synchronize()
    assert torch.equal(out, want)
    # identities on the same 64 Mi elements: x op x
    same = torch.empty_like(out)
    shm.fold_n("long", op, same, [srcs[0], srcs[0]], n)
    torch.cuda.synchronize()
    assert torch.equal(same, torch.zeros_like(same) if op == "xor" else srcs[0])


def test_config5_float_sum_size_sweep(cuda, shm):
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    n = 4 * 1024
    while n <= 256 * 1024 * 1024:
        a = torch.rand(n, dtype=torch.float32, device="cuda", generator=g) + 1
        b = torch.rand(n, dtype=torch.float32, device="cuda", generator=g) - 0.5
        acc = a.clone()
        shm.fold("float", "sum", acc, b, n)
        torch.cuda.synchronize()
        assert torch.equal(acc, a + b), n
        del a, b, acc
        n *= 4
    # 8 sources (8 PEs) in set order == the left fold
    n = 1 << 22
    srcs = [torch.rand(n, dtype=torch.float32, device="cuda", generator=g) for _ in range(8)]
    out = torch.empty_like(srcs[0])
    shm.fold_n("float", "sum", out, srcs, n)
    want = srcs[0].clone()
    for s in srcs[1:]:
        want = want + s
    torch.cuda.synchronize()
    assert torch.equal(out, want)


def test_beyond_2gib_and_max_nreduce(cuda, shm):
    """The reference computes the byte count as an int (reduce-op.c:180), so
    it breaks above 2 GiB; here offsets are 64-bit everywhere.  nreduce =
    INT_MAX shorts (4 GiB per array, odd length: scalar tail at the far end)
    through the blocking drop-in call at PE_size = 1 (a copy), and a
    2.5 GiB long xor fold checked by the involution (a ^ b) ^ b == a."""
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(31)
    n = 2**31 - 1
    src = torch.randint(-2**15, 2**15, (n,), dtype=torch.int16, device="cuda", generator=g)
    tgt = torch.zeros_like(src)
    shm.to_all("short", "max", tgt, src, n, 0, 0, 1)
    assert shm.last_error() == 0
    torch.cuda.synchronize()
    assert torch.equal(tgt, src)
    assert torch.equal(tgt[-3:], src[-3:])
    del src, tgt
    torch.cuda.empty_cache()
    n = 320 * 1024 * 1024 + 3
    a = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
    b = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
    acc = a.clone()
    shm.fold("long", "xor", acc, b, n)
    torch.cuda.synchronize()
    assert torch.equal(acc, torch.bitwise_xor(a, b))
    shm.fold("long", "xor", acc, b, n)
    torch.cuda.synchronize()
    assert torch.equal(acc, a)
