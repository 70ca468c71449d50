"""TEST INFRASTRUCTURE ONLY — ctypes view of oracle/liboracle_reduce.so plus the
numpy input generator shared by the tests, the golden-fixture script and
bench.py's cpu_baseline leg.  Never imported by the product
(openshmem-async_amd/).

The oracle is a CPU restatement of /root/reference/src/reduce/reduce-op.c
(see reduce_oracle.c for the line-by-line citations).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle_reduce.so")

TYPES = {"short": 0, "int": 1, "long": 2, "longlong": 3, "float": 4,
         "double": 5, "longdouble": 6, "complexd": 7, "complexf": 8}
OPS = {"sum": 0, "prod": 1, "and": 2, "or": 3, "xor": 4, "min": 5, "max": 6}
NP_DTYPE = {"short": np.int16, "int": np.int32, "long": np.int64,
            "longlong": np.int64, "float": np.float32, "double": np.float64,
            "longdouble": np.longdouble, "complexd": np.complex128,
            "complexf": np.complex64}
WRKDATA = 64  # _SHMEM_REDUCE_MIN_WRKDATA_SIZE (shmem.h:1400-1405)

_lib = None


def build() -> None:
    """Compile the restatement (gcc, oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.oracle_reduce_sim.argtypes = [i, i, i, i, i, i, i, vp, vp]
        L.oracle_reduce_sim.restype = i
        L.oracle_reduce_one.argtypes = [i, i, i, i, i, i, i, vp, i, vp]
        L.oracle_reduce_one.restype = i
        L.oracle_reduce_fork.argtypes = [i, i, i, i, i, i, i, i, ctypes.c_uint64, i, i,
                                         ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_reduce_fork.restype = i
        L.oracle_fold_time.argtypes = [i, i, i, i, i, ctypes.POINTER(ctypes.c_double)]
        L.oracle_fold_time.restype = i
        L.oracle_fill.argtypes = [i, i, ctypes.c_uint64, vp, ctypes.c_size_t]
        L.oracle_fill.restype = None
        L.oracle_splitmix64.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_type_size.argtypes = [i]
        L.oracle_type_size.restype = ctypes.c_size_t
        L.oracle_op_valid.argtypes = [i, i]
        L.oracle_op_valid.restype = i
        sz_t = ctypes.c_size_t
        L.oracle_broadcast_sim.argtypes = [sz_t, i, i, i, i, i, sz_t, vp, sz_t, vp, sz_t]
        L.oracle_broadcast_sim.restype = i
        L.oracle_collect_sim.argtypes = [sz_t, i, i, i, i, ctypes.POINTER(sz_t), vp, sz_t, vp, sz_t]
        L.oracle_collect_sim.restype = i
        L.oracle_fnv1a.argtypes = [vp, ctypes.c_size_t]
        L.oracle_fnv1a.restype = ctypes.c_uint64
        _lib = L
    return _lib


def op_valid(type_name: str, op: str) -> bool:
    return bool(lib().oracle_op_valid(TYPES[type_name], OPS[op]))


# ------------------------------------------------------------------ inputs
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """Words start..start+n-1 of the stream `seed` (same as oracle_splitmix64)."""
    i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _unit53(r):
    return (r >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def _unit24(r):
    return (r >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)


def fill(type_name: str, kind: int, seed: int, n: int) -> np.ndarray:
    """numpy twin of oracle_fill (kind 0 = positive/small, 1 = mixed/full)."""
    r = splitmix64(seed, n)
    t = type_name
    if t == "short":
        return (r & np.uint64(0xFFFF)).astype(np.uint16).view(np.int16) if kind else \
            ((r >> np.uint64(53)).astype(np.int64) - 1024).astype(np.int16)
    if t == "int":
        return (r & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32) if kind else \
            ((r >> np.uint64(43)).astype(np.int64) - (1 << 20)).astype(np.int32)
    if t in ("long", "longlong"):
        return r.view(np.int64).copy() if kind else \
            ((r >> np.uint64(43)).astype(np.int64) - (1 << 20))
    if t == "float":
        u = _unit24(r)
        return (u * np.float32(2.0) - np.float32(1.0)) if kind else (np.float32(1.0) + u)
    if t == "double":
        u = _unit53(r)
        return (u * 2.0 - 1.0) if kind else (1.0 + u)
    if t == "longdouble":
        u = _unit53(r).astype(np.longdouble)
        return (u * np.longdouble(2) - np.longdouble(1)) if kind else (np.longdouble(1) + u)
    if t in ("complexd", "complexf"):
        r2 = splitmix64(seed ^ 0xC0FFEE, n)
        if t == "complexd":
            re, im = _unit53(r), _unit53(r2)
            if kind:
                re, im = re * 2.0 - 1.0, im * 2.0 - 1.0
            else:
                re, im = 1.0 + re, 1.0 + im
            out = np.empty(n, np.complex128)
        else:
            re, im = _unit24(r), _unit24(r2)
            if kind:
                re, im = re * np.float32(2) - np.float32(1), im * np.float32(2) - np.float32(1)
            else:
                re, im = np.float32(1) + re, np.float32(1) + im
            out = np.empty(n, np.complex64)
        out.real, out.imag = re, im
        return out
    raise KeyError(t)


def sources(type_name: str, kind: int, npes: int, n: int, base_seed: int = 0x5EED0000) -> np.ndarray:
    """[npes, n] array: PE p's source from seed base_seed + p."""
    out = np.empty((npes, n), NP_DTYPE[type_name])
    for p in range(npes):
        out[p] = fill(type_name, kind, base_seed + p, n)
    return out


def special_sources(type_name: str, npes: int, n: int, seed: int) -> np.ndarray:
    """[npes, n] sources of float / double / long double drawn from NaNs of
    both signs, both zeros, +-1, 2, +-inf and the smallest normal: the inputs
    on which a<b?a:b / a>b?a:b (reduce-op.c:130-142) make each PE's answer
    depend on its own fold order (reduce-op.c:219-248)."""
    dt = NP_DTYPE[type_name]
    if type_name == "longdouble":
        nan = np.longdouble("nan")
        pool = np.array([nan, -nan, 0.0, -0.0, 1.0, -1.0, 2.0, np.inf, -np.inf,
                         np.finfo(np.longdouble).tiny], dtype=dt)
    else:
        pool = np.array([np.nan, -np.nan, 0.0, -0.0, 1.0, -1.0, 2.0, np.inf, -np.inf,
                         np.finfo(dt).tiny], dtype=dt)
    idx = (splitmix64(seed, npes * n) % np.uint64(len(pool))).astype(np.int64)
    return np.ascontiguousarray(pool[idx].reshape(npes, n))


# --------------------------------------------------------------- the oracle
def reduce_sim(type_name: str, op: str, srcs: np.ndarray, PE_start: int, logPE_stride: int,
               PE_size: int, targets: np.ndarray | None = None) -> np.ndarray:
    """Every PE's target after shmem_<type>_<op>_to_all on the active set.

    srcs: [npes, n].  targets: prefilled [npes, n] (PEs outside the set keep
    their contents); default a copy of srcs' zeros."""
    srcs = np.ascontiguousarray(srcs, dtype=NP_DTYPE[type_name])
    npes, n = srcs.shape
    if targets is None:
        targets = np.zeros_like(srcs)
    else:
        targets = np.ascontiguousarray(targets.copy(), dtype=NP_DTYPE[type_name])
    rc = lib().oracle_reduce_sim(TYPES[type_name], OPS[op], npes, PE_start, logPE_stride,
                                 PE_size, n, srcs.ctypes.data, targets.ctypes.data)
    if rc != 0:
        raise ValueError(f"oracle_reduce_sim rejected {type_name} {op} set "
                         f"({PE_start},{logPE_stride},{PE_size}) npes={npes} n={n}")
    return targets


def reduce_one(type_name: str, op: str, srcs: np.ndarray, PE_start: int, logPE_stride: int,
               PE_size: int, pe: int) -> np.ndarray:
    """PE `pe`'s target after shmem_<type>_<op>_to_all (srcs: [npes, n]),
    without simulating the other members: full-size checks."""
    srcs = np.ascontiguousarray(srcs, dtype=NP_DTYPE[type_name])
    npes, n = srcs.shape
    out = np.empty(n, dtype=NP_DTYPE[type_name])
    rc = lib().oracle_reduce_one(TYPES[type_name], OPS[op], npes, PE_start, logPE_stride, PE_size,
                                 n, srcs.ctypes.data, pe, out.ctypes.data)
    if rc != 0:
        raise ValueError(f"oracle_reduce_one rejected {type_name} {op} set "
                         f"({PE_start},{logPE_stride},{PE_size}) pe={pe}")
    return out


def reduce_fork(type_name: str, op: str, npes: int, PE_start: int, logPE_stride: int,
                PE_size: int, nreduce: int, kind: int = 0, base_seed: int = 0x5EED0000,
                reps: int = 3, pin_base: int = 0):
    """Fork-per-PE run (GASNet smp model).  Returns (times[s], hashes[npes])."""
    times = (ctypes.c_double * reps)()
    hashes = (ctypes.c_uint64 * npes)()
    rc = lib().oracle_reduce_fork(TYPES[type_name], OPS[op], npes, PE_start, logPE_stride,
                                  PE_size, nreduce, kind, base_seed, reps, pin_base,
                                  times, hashes)
    if rc != 0:
        raise RuntimeError("oracle_reduce_fork failed")
    return list(times), list(hashes)


def fold_time(type_name: str, op: str, nreduce: int, reps: int = 5, pin: int = -1) -> list:
    """The reference's per-peer fold step alone (acc = op(acc, in), pWrk
    staging, indirect call per element): per-fold seconds."""
    times = (ctypes.c_double * reps)()
    rc = lib().oracle_fold_time(TYPES[type_name], OPS[op], nreduce, reps, pin, times)
    if rc != 0:
        raise RuntimeError("oracle_fold_time failed")
    return list(times)


def value_hash(type_name: str, arr: np.ndarray) -> int:
    """FNV-1a of the value bytes (long double: the 10 x87 bytes of each slot)."""
    a = np.ascontiguousarray(arr, dtype=NP_DTYPE[type_name])
    if type_name == "longdouble":
        a = np.ascontiguousarray(a.view(np.uint8).reshape(-1, a.itemsize)[:, :10])
    return int(lib().oracle_fnv1a(a.ctypes.data, a.nbytes))


def broadcast_sim(srcs: np.ndarray, targets: np.ndarray, PE_root: int, PE_start: int,
                  logPE_stride: int, PE_size: int) -> np.ndarray:
    """shmem_broadcast{32,64} on every PE (srcs/targets: [npes, nelems])."""
    srcs = np.ascontiguousarray(srcs)
    out = np.ascontiguousarray(targets.copy())
    npes, n = srcs.shape
    rc = lib().oracle_broadcast_sim(srcs.itemsize, npes, PE_root, PE_start, logPE_stride, PE_size,
                                    n, srcs.ctypes.data, srcs.strides[0], out.ctypes.data,
                                    out.strides[0])
    if rc:
        raise ValueError("oracle_broadcast_sim rejected the arguments")
    return out


def collect_sim(srcs: np.ndarray, nelems, targets: np.ndarray, PE_start: int,
                logPE_stride: int, PE_size: int) -> np.ndarray:
    """shmem_[f]collect{32,64} on every PE.  srcs: [npes, maxn] (PE p uses
    nelems[p] leading elements), targets: [npes, capacity]."""
    srcs = np.ascontiguousarray(srcs)
    out = np.ascontiguousarray(targets.copy())
    npes = srcs.shape[0]
    ne = (ctypes.c_size_t * npes)(*nelems)
    rc = lib().oracle_collect_sim(srcs.itemsize, npes, PE_start, logPE_stride, PE_size, ne,
                                  srcs.ctypes.data, srcs.strides[0], out.ctypes.data,
                                  out.strides[0])
    if rc:
        raise ValueError("oracle_collect_sim rejected the arguments")
    return out
