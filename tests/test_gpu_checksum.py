"""shmemx_checksum / shmemx_verify on the GPU against the host twin
(tests/gpu_util.py::checksum64), and the checksum-of-checksums property at the
bench size."""
import numpy as np
import pytest
from gpu_util import checksum64, to_dev

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("t", ["short", "int", "long", "float", "double", "longdouble",
                               "complexd", "complexf"])
def test_checksum_matches_host_twin(cuda, shm, oracle, t):
    import torch
    for n in (0, 1, 3, 5, 64, 1001, 65537, 1 << 20):
        a = oracle.fill(t, 1, 1000 + n, n)
        if t == "longdouble" and n:
            raw = a.view(np.uint8).reshape(-1, 16)
            raw[:, 10:] = np.arange(6, dtype=np.uint8) + 1       # junk padding is ignored
        want = checksum64(a)
        assert shm.checksum(t, to_dev(torch, a), n) == want, (t, n)
        assert shm.checksum(t, a, n) == want, (t, n, "host")         # staged
    # position-aware: swapping two elements changes it
    a = oracle.fill(t, 1, 7, 100)
    b = a.copy()
    b[[3, 70]] = b[[70, 3]]
    if a[3] != a[70]:
        assert shm.checksum(t, a, 100) != shm.checksum(t, b, 100)


def test_checksum_of_checksums_full_size(cuda, shm, oracle):
    """The fold at the bench size (32 Mi doubles) checked whole by checksum:
    GPU checksum of the GPU result == host checksum of numpy's a + b."""
    import torch
    n = 32 * 1024 * 1024
    a = oracle.fill("double", 0, 11, n)
    b = oracle.fill("double", 0, 12, n)
    acc, inp = to_dev(torch, a), to_dev(torch, b)
    shm.fold("double", "sum", acc, inp, n)
    torch.cuda.synchronize()
    assert shm.checksum("double", acc, n) == checksum64(a + b)


def test_verify_single_pe(cuda, shm):
    import torch
    x = torch.arange(1000, dtype=torch.float64, device="cuda")
    assert shm.verify("double", x, 1000, 0, 0, 1)
