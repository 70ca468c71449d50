"""Helpers for the GPU tests: numpy <-> device buffers for every reduction
type (long double travels as raw 16-byte slots; torch has no such dtype) and
value-level bit comparison (long double: the 10 x87 bytes of each slot)."""
import numpy as np


def to_dev(torch, a: np.ndarray):
    a = np.ascontiguousarray(a)
    if a.dtype == np.longdouble:
        return torch.from_numpy(a.view(np.uint8).copy()).cuda()
    return torch.from_numpy(a).cuda()


def empty_like_dev(torch, a: np.ndarray):
    a = np.ascontiguousarray(a)
    if a.dtype == np.longdouble:
        return torch.zeros(a.nbytes, dtype=torch.uint8, device="cuda")
    return torch.zeros(a.shape, dtype=to_dev(torch, a[:0]).dtype, device="cuda")


def from_dev(t, dtype) -> np.ndarray:
    host = t.cpu().numpy()
    if np.dtype(dtype) == np.longdouble:
        return host.view(np.longdouble)
    return host


def value_bytes(a: np.ndarray) -> bytes:
    a = np.ascontiguousarray(a)
    if a.dtype == np.longdouble:
        return np.ascontiguousarray(a.view(np.uint8).reshape(-1, a.itemsize)[:, :10]).tobytes()
    return a.tobytes()


def same_bits(a: np.ndarray, b: np.ndarray) -> bool:
    return a.dtype == b.dtype and a.shape == b.shape and value_bytes(a) == value_bytes(b)


def order_bound(got: np.ndarray, want: np.ndarray, member_srcs: np.ndarray, op: str,
                scale: float = 1.0):
    """A floating sum / product whose fold order is not the reference's (RCCL's
    ring or tree) against `want`, the reference's PE_start-order fold
    (reduce-op.c:219-248), within the bound BASELINE.json's north_star states:

        |got - want| <= 2 gamma(P-1) sum_p |x_p|     (sum)
        |got - want| <= 2 gamma(P-1) |prod_p x_p|    (prod, + 2(P-1) x the
                                                      smallest subnormal for
                                                      gradual underflow)

    gamma(k) = k u / (1 - k u), u = 2^-24 (float) / 2^-53 (double): each order
    is within gamma(P-1) of the exact value.  NaN must match NaN and an
    infinity the same infinity.  `scale` multiplies the bound (0: the negative
    control, only bit-identical elements pass).  Integers, and any other op,
    are compared bit for bit.  Returns (ok, elements that differ in bits)."""
    got, want = np.ascontiguousarray(got), np.ascontiguousarray(want)
    if got.dtype.kind != "f" or op not in ("sum", "prod") or got.dtype == np.longdouble:
        return same_bits(got, want), 0
    iv = np.int32 if got.dtype.itemsize == 4 else np.int64
    inexact = int(np.count_nonzero(got.view(iv) != want.view(iv)))
    fi = np.finfo(got.dtype)
    k = len(member_srcs) - 1
    u = float(fi.eps) / 2
    gamma = k * u / (1 - k * u)
    wide = np.float64 if got.dtype == np.float32 else np.longdouble
    x = np.asarray(member_srcs).astype(wide)
    if op == "sum":
        bound = 2 * gamma * np.abs(x).sum(axis=0)
    else:
        bound = 2 * gamma * np.abs(np.prod(x, axis=0)) + 2 * k * float(fi.smallest_subnormal)
    bound = bound * scale
    g, w = got.astype(wide), want.astype(wide)
    gn, wn = np.isnan(g), np.isnan(w)
    fin = np.isfinite(g) & np.isfinite(w)
    inf = ~fin & ~gn & ~wn
    ok = (np.array_equal(gn, wn) and bool(np.all(g[inf] == w[inf]))
          and bool(np.all(np.abs(g[fin] - w[fin]) <= bound[fin])))
    return ok, inexact


def checksum64(a: np.ndarray) -> int:
    """Host twin of shmemx_checksum (openshmem-async_amd/csrc/checksum.hip):
    XOR over the little-endian 8-byte words w_j of the element bytes (long
    double: 10 value bytes per 16-byte slot, the rest zero) of
    splitmix64-finalise(w_j + (j + 1) * 0x9E3779B97F4A7C15)."""
    a = np.ascontiguousarray(a)
    b = a.view(np.uint8).reshape(-1)
    if a.dtype == np.longdouble:
        b = b.reshape(-1, 16).copy()
        b[:, 10:] = 0
        b = b.reshape(-1)
    pad = (-len(b)) % 8
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    w = b.view("<u8")
    if len(w) == 0:
        return 0
    j = np.arange(1, len(w) + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = w + j * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return int(np.bitwise_xor.reduce(z))
