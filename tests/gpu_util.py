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
