"""Python view of libshmem_reduce_mi355x.so (ctypes, no torch types in the ABI).

The product is the C ABI in ``include/shmem_reduce_mi355x.h``; this module is
the thin host-side mirror used by the tests and ``bench.py``.  It keeps the
reference's names and argument meaning: ``to_all("double", "sum", target,
source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync)`` calls the C
entry point ``shmem_double_sum_to_all`` (reference src/reduce/reduce-op.c:
372-431, prototype src/shmem.h:1412-1648) with raw pointers.

Array arguments may be torch tensors (device or host), numpy arrays, or plain
integer addresses.  Loading fails loudly when the shared library has not been
built: there is no Python or CPU fallback for any reduction.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libshmem_reduce_mi355x.so")

# SHMEMX_TYPE_* / SHMEMX_OP_* / SHMEMX_ALGO_* of the header.
TYPES = {"short": 0, "int": 1, "long": 2, "longlong": 3, "float": 4,
         "double": 5, "longdouble": 6, "complexd": 7, "complexf": 8}
OPS = {"sum": 0, "prod": 1, "and": 2, "or": 3, "xor": 4, "min": 5, "max": 6}
ALGOS = {"auto": 0, "rccl": 1, "a2a": 2, "gather": 3, "allreduce": 4, "direct": 5,
         "signal": 6}
ERRORS = {0: "OK", 1: "EINVAL", 2: "ENOTMEMBER", 3: "ENOTSUP", 4: "ENOINIT",
          5: "ENOMEM", 6: "EDEVICE"}

# Which (type, op) pairs the reference exports (reduce-op.c:388-431).
REFERENCE_PAIRS = [(t, o) for t in TYPES for o in ("sum", "prod")] + \
    [(t, o) for t in ("short", "int", "long", "longlong") for o in ("and", "or", "xor")] + \
    [(t, o) for t in ("short", "int", "long", "longlong", "float", "double", "longdouble")
     for o in ("max", "min")]


class ShmemError(RuntimeError):
    """A shmemx_* call returned an error code."""

    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {ERRORS.get(code, code)}")
        self.code = code


class Plan(ctypes.Structure):
    _fields_ = [("algo", ctypes.c_int), ("member", ctypes.c_int),
                ("nmembers", ctypes.c_int), ("elem_size", ctypes.c_int),
                ("chunk", ctypes.c_longlong), ("main", ctypes.c_longlong),
                ("tail", ctypes.c_longlong), ("ws_bytes", ctypes.c_longlong)]


_lib = None


def device_code_sha256(path: str = LIB_PATH) -> str | None:
    """sha256 of the library's gfx950 device code (its ELF .hip_fatbin
    section): what a rocprofv3 counter pass over the kernels measured.  Host
    code changes leave it alone; any kernel change moves it.  None if the
    file or the section is missing."""
    import hashlib
    import struct
    try:
        with open(path, "rb") as f:
            elf = f.read()
    except OSError:
        return None
    if elf[:4] != b"\x7fELF" or elf[4] != 2:          # ELF64 only
        return None
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)

    def sect(i):
        name, _, _, _, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        return name, off, size
    _, stroff, _ = sect(shstrndx)
    for i in range(shnum):
        name, off, size = sect(i)
        end = elf.index(b"\0", stroff + name)
        if elf[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(elf[off:off + size]).hexdigest()
    return None


def lib() -> ctypes.CDLL:
    """Load the shared library (once).  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is not built; run `make -C openshmem-async_amd` "
            "(or __graft_entry__.build()) — there is no fallback path")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7
    # and loads it by path.  Import torch first (when present) so that the
    # library's DT_NEEDED libamdhip64.so.7 / librccl.so.1 bind to the copies
    # already loaded; loading ours first would put two HIP runtimes in the
    # process and the second sees no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.shmemx_reduce_on_stream.argtypes = [i, i, vp, vp, i, i, i, i, i, vp]
    L.shmemx_reduce_on_stream.restype = i
    L.shmemx_fold_on_stream.argtypes = [i, i, vp, vp, sz, vp]
    L.shmemx_fold_on_stream.restype = i
    L.shmemx_fold_n_on_stream.argtypes = [i, i, vp, ctypes.POINTER(vp), i, sz, vp]
    L.shmemx_fold_n_on_stream.restype = i
    L.shmemx_fold_n_peers_on_stream.argtypes = [i, i, vp, ctypes.POINTER(vp), i, sz, vp]
    L.shmemx_fold_n_peers_on_stream.restype = i
    L.shmemx_gather_on_stream.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp),
                                          ctypes.POINTER(sz), i, vp]
    L.shmemx_gather_on_stream.restype = i
    L.shmemx_reduce_plan.argtypes = [i, i, i, i, i, i, i, i, i, ctypes.POINTER(Plan)]
    L.shmemx_reduce_plan.restype = i
    L.shmemx_get_uniqueid.argtypes = [vp]
    L.shmemx_get_uniqueid.restype = i
    L.shmemx_uniqueid_size.restype = i
    L.shmemx_init_attr.argtypes = [i, i, i, vp]
    L.shmemx_init_attr.restype = i
    L.shmemx_get_stream.restype = vp
    L.shmemx_set_algo.argtypes = [i]
    L.shmemx_set_algo.restype = i
    L.shmemx_rccl_register_heap.argtypes = [i]
    L.shmemx_rccl_register_heap.restype = i
    L.shmemx_set_comms.restype = i
    L.shmemx_kernel_timing.argtypes = [i]
    L.shmemx_kernel_timing.restype = i
    L.shmemx_kernel_times.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int), i,
                                      ctypes.POINTER(ctypes.c_ulonglong)]
    L.shmemx_kernel_times.restype = i
    L.shmemx_set_fused_twoshot_kb.argtypes = [ctypes.c_long]
    L.shmemx_set_fused_twoshot_kb.restype = ctypes.c_long
    L.shmemx_type_size.argtypes = [i]
    L.shmemx_type_size.restype = sz
    L.shmemx_op_valid.argtypes = [i, i]
    L.shmemx_op_on_device.argtypes = [i, i]
    L.shmemx_reduce_last_error.restype = i
    L.shmemx_reduce_error_string.argtypes = [i]
    L.shmemx_reduce_error_string.restype = ctypes.c_char_p
    for bits in (32, 64):
        for name in (f"shmem_broadcast{bits}", f"pshmem_broadcast{bits}"):
            getattr(L, name).argtypes = [vp, vp, sz, i, i, i, i, vp]
            getattr(L, name).restype = None
        for kind in ("fcollect", "collect"):
            for name in (f"shmem_{kind}{bits}", f"pshmem_{kind}{bits}"):
                getattr(L, name).argtypes = [vp, vp, sz, i, i, i, vp]
                getattr(L, name).restype = None
    L.shmemx_checksum.argtypes = [i, vp, sz, ctypes.POINTER(ctypes.c_ulonglong)]
    L.shmemx_checksum.restype = i
    L.shmemx_verify.argtypes = [i, vp, i, i, i, i, ctypes.POINTER(i)]
    L.shmemx_verify.restype = i
    L.shmem_barrier.argtypes = [i, i, i, vp]
    L.shmem_barrier.restype = None
    L.shmem_barrier_all.restype = None
    L.shmem_malloc.argtypes = [sz]
    L.shmem_malloc.restype = vp
    L.shmemx_heap_ptr.argtypes = [vp, i]
    L.shmemx_heap_ptr.restype = vp
    L.shmem_align.argtypes = [sz, sz]
    L.shmem_align.restype = vp
    L.shmem_realloc.argtypes = [vp, sz]
    L.shmem_realloc.restype = vp
    L.shmem_free.argtypes = [vp]
    L.shmem_free.restype = None
    L.shmemx_mirror_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), i, i]
    L.shmemx_mirror_stats.restype = i
    L.shmemx_mirror_device_ptr.argtypes = [vp]
    L.shmemx_mirror_device_ptr.restype = vp
    L.shmemx_mirror_sync.argtypes = [vp, sz]
    L.shmemx_mirror_sync.restype = i
    L.shmemx_mirror_invalidate.argtypes = [vp, sz]
    L.shmemx_mirror_invalidate.restype = i
    L.shmemx_mirror_acquire.argtypes = [vp, sz, i]
    L.shmemx_mirror_acquire.restype = i
    L.shmemx_direct_stats.argtypes = [ctypes.POINTER(ctypes.c_double), i, i]
    L.shmemx_direct_stats.restype = i
    L.shmemx_service_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), i, i]
    L.shmemx_service_stats.restype = i
    L.shmemx_host_register.argtypes = [vp, sz]
    L.shmemx_host_register.restype = i
    L.shmemx_host_unregister.argtypes = [vp]
    L.shmemx_host_unregister.restype = i
    L.shmemx_set_fatal_note.argtypes = [ctypes.c_char_p, i]
    L.shmemx_set_fatal_note.restype = i
    for t, o in REFERENCE_PAIRS:
        for prefix in ("shmem", "pshmem"):
            f = getattr(L, f"{prefix}_{t}_{o}_to_all")
            f.argtypes = [vp, vp, i, i, i, i, vp, vp]
            f.restype = None
    _lib = L
    return L


def addr(x) -> int | None:
    """Raw address of a torch tensor, numpy array, ctypes object or int."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    return ctypes.addressof(x)


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise ShmemError(rc, what)


# ------------------------------------------------------------------ runtime
def init_attr(pe: int, npes: int, device: int = -1, uid: bytes | None = None) -> None:
    buf = None
    if uid is not None:
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
    _check(lib().shmemx_init_attr(pe, npes, device, buf), "shmemx_init_attr")


def get_uniqueid() -> bytes:
    n = lib().shmemx_uniqueid_size()
    buf = ctypes.create_string_buffer(n)
    _check(lib().shmemx_get_uniqueid(buf), "shmemx_get_uniqueid")
    return buf.raw


def init_from_torch_distributed(device: int = -1) -> None:
    """Bootstrap every rank of an initialised torch.distributed group (gloo is
    enough: it only carries the 128-byte RCCL id)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    if world == 1:
        init_attr(0, 1, device, None)
        return
    n = lib().shmemx_uniqueid_size()
    t = torch.zeros(n, dtype=torch.uint8)
    if rank == 0:
        t.copy_(torch.frombuffer(bytearray(get_uniqueid()), dtype=torch.uint8))
    dist.broadcast(t, src=0)
    init_attr(rank, world, device, bytes(t.numpy().tobytes()))


def init() -> None:
    lib().shmem_init()


def finalize() -> None:
    lib().shmem_finalize()


def my_pe() -> int:
    return lib().shmem_my_pe()


def n_pes() -> int:
    return lib().shmem_n_pes()


def get_stream() -> int:
    return lib().shmemx_get_stream() or 0


def set_fused_twoshot_kb(kb: int) -> int:
    """shmemx_set_fused_twoshot_kb: the largest DIRECT/SIGNAL two-shot call
    (KiB) run as one fused launch; returns the previous limit.  Collective in
    effect: every member must set the same value."""
    prev = lib().shmemx_set_fused_twoshot_kb(kb)
    if prev < 0:
        raise ShmemError(1, "shmemx_set_fused_twoshot_kb")
    return prev


def set_algo(name: str) -> str:
    prev = lib().shmemx_set_algo(ALGOS[name])
    return {v: k for k, v in ALGOS.items()}[prev]


def last_error() -> int:
    return lib().shmemx_reduce_last_error()


# --------------------------------------------------------------- reductions
def to_all(type_name: str, op: str, target, source, nreduce: int, PE_start: int,
           logPE_stride: int, PE_size: int, pWrk=None, pSync=None) -> None:
    """shmem_<type>_<op>_to_all, blocking (reference reduce-op.c:372-386)."""
    f = getattr(lib(), f"shmem_{type_name}_{op}_to_all")
    f(addr(target), addr(source), nreduce, PE_start, logPE_stride, PE_size,
      addr(pWrk), addr(pSync))


def reduce_on_stream(type_name: str, op: str, target, source, nreduce: int,
                     PE_start: int = 0, logPE_stride: int = 0, PE_size: int = 1,
                     algo: str = "auto", stream: int = 0) -> None:
    rc = lib().shmemx_reduce_on_stream(TYPES[type_name], OPS[op], addr(target), addr(source),
                                       nreduce, PE_start, logPE_stride, PE_size,
                                       ALGOS[algo], stream or None)
    _check(rc, f"shmemx_reduce_on_stream({type_name},{op})")


def fold(type_name: str, op: str, acc, inp, nelems: int, stream: int = 0) -> None:
    """acc[i] = op(acc[i], inp[i]) on the GPU (reduce-op.c:231-235)."""
    rc = lib().shmemx_fold_on_stream(TYPES[type_name], OPS[op], addr(acc), addr(inp),
                                     nelems, stream or None)
    _check(rc, f"shmemx_fold_on_stream({type_name},{op})")


def fold_n(type_name: str, op: str, out, ins, nelems: int, stream: int = 0, peers: bool = False) -> None:
    """shmemx_fold_n_on_stream, or with peers=True shmemx_fold_n_peers_on_stream
    (every input's loads in flight before any op: the peers' HBM over xGMI)."""
    arr = (ctypes.c_void_p * len(ins))(*[addr(x) for x in ins])
    fn = lib().shmemx_fold_n_peers_on_stream if peers else lib().shmemx_fold_n_on_stream
    rc = fn(TYPES[type_name], OPS[op], addr(out), arr, len(ins), nelems, stream or None)
    _check(rc, f"shmemx_fold_n{'_peers' if peers else ''}_on_stream({type_name},{op})")


def gather(srcs, dsts, nbytes, stream: int = 0) -> None:
    """shmemx_gather_on_stream: copy byte ranges srcs[i] -> dsts[i] in one
    launch (DIRECT's all-gather kernel)."""
    k = len(srcs)
    a = (ctypes.c_void_p * k)(*[addr(x) for x in srcs])
    b = (ctypes.c_void_p * k)(*[addr(x) for x in dsts])
    c = (ctypes.c_size_t * k)(*nbytes)
    _check(lib().shmemx_gather_on_stream(a, b, c, k, stream or None), "shmemx_gather_on_stream")


@dataclass
class PlanInfo:
    algo: str
    member: int
    nmembers: int
    elem_size: int
    chunk: int
    main: int
    tail: int
    ws_bytes: int


def plan(type_name: str, op: str, nreduce: int, PE_start: int, logPE_stride: int,
         PE_size: int, pe: int, npes: int, algo: str = "auto") -> PlanInfo:
    p = Plan()
    rc = lib().shmemx_reduce_plan(TYPES[type_name], OPS[op], nreduce, PE_start, logPE_stride,
                                  PE_size, pe, npes, ALGOS[algo], ctypes.byref(p))
    _check(rc, "shmemx_reduce_plan")
    inv = {v: k for k, v in ALGOS.items()}
    return PlanInfo(inv[p.algo], p.member, p.nmembers, p.elem_size, p.chunk, p.main,
                    p.tail, p.ws_bytes)


def rccl_register_heap(on: bool) -> None:
    """shmemx_rccl_register_heap: the heap segment (de)registered with RCCL."""
    _check(lib().shmemx_rccl_register_heap(1 if on else 0), "shmemx_rccl_register_heap")


def set_comms() -> int:
    """shmemx_set_comms: members-only RCCL communicators held for partial sets."""
    return lib().shmemx_set_comms()


KERNEL_KINDS = ("fold", "copy", "peers_fold", "gather")


def kernel_timing(on: bool) -> None:
    """shmemx_kernel_timing: time every fold-family launch from here on
    (start/stop events of the dispatch itself, kernel time only)."""
    lib().shmemx_kernel_timing(1 if on else 0)


def kernel_times(max_launches: int = 4096):
    """shmemx_kernel_times: [(kind, microseconds)] of the launches timed since
    the last read, in launch order (waits for them), and the untimed count."""
    us = (ctypes.c_double * max_launches)()
    kind = (ctypes.c_int * max_launches)()
    dropped = ctypes.c_ulonglong(0)
    n = lib().shmemx_kernel_times(us, kind, max_launches, ctypes.byref(dropped))
    return [(KERNEL_KINDS[kind[i]], us[i]) for i in range(n)], dropped.value


def type_size(type_name: str) -> int:
    return lib().shmemx_type_size(TYPES[type_name])


def op_on_device(type_name: str, op: str) -> bool:
    return bool(lib().shmemx_op_on_device(TYPES[type_name], OPS[op]))


# ------------------------------------------- neighbouring collectives, heap
def barrier(PE_start: int, logPE_stride: int, PE_size: int, pSync=None) -> None:
    lib().shmem_barrier(PE_start, logPE_stride, PE_size, addr(pSync))


def barrier_all() -> None:
    lib().shmem_barrier_all()


def broadcast(bits: int, target, source, nelems: int, PE_root: int, PE_start: int,
              logPE_stride: int, PE_size: int, pSync=None) -> None:
    """shmem_broadcast{32,64} (reference broadcast/broadcast.c)."""
    getattr(lib(), f"shmem_broadcast{bits}")(addr(target), addr(source), nelems, PE_root,
                                             PE_start, logPE_stride, PE_size, addr(pSync))


def fcollect(bits: int, target, source, nelems: int, PE_start: int, logPE_stride: int,
             PE_size: int, pSync=None) -> None:
    getattr(lib(), f"shmem_fcollect{bits}")(addr(target), addr(source), nelems, PE_start,
                                            logPE_stride, PE_size, addr(pSync))


def collect(bits: int, target, source, nelems: int, PE_start: int, logPE_stride: int,
            PE_size: int, pSync=None) -> None:
    getattr(lib(), f"shmem_collect{bits}")(addr(target), addr(source), nelems, PE_start,
                                           logPE_stride, PE_size, addr(pSync))


def heap_ptr(address: int, pe: int) -> int:
    """shmemx_heap_ptr: PE `pe`'s copy of a symmetric-heap address, as mapped
    on this PE (0 if not mapped)."""
    return lib().shmemx_heap_ptr(address, pe) or 0


DIRECT_PHASES = ("entry_wait_us", "entry_barrier_us", "fold_us", "fold_barrier_us",
                 "gather_us", "exit_barrier_us")


FENCE_STATS = ("fences_host", "fence_refills_host", "fences_device", "fences_device_incomplete")
DIRECT_COUNTS = ("fused_calls", "fused_twoshot_calls")


def direct_stats(reset: bool = True) -> dict:
    """shmemx_direct_stats: DIRECT calls since the last reset, the host-side
    microseconds summed over them per phase, and the system-fence coverage
    counters (fences checked on the host / refilled because a fence missed an
    XCD; fences checked by the SIGNAL barrier / found incomplete), and the
    one-shot calls that ran as one fused launch."""
    names = DIRECT_PHASES + FENCE_STATS + DIRECT_COUNTS
    buf = (ctypes.c_double * (1 + len(names)))()
    k = lib().shmemx_direct_stats(buf, len(buf), 1 if reset else 0)
    out = {"calls": buf[0]}
    out.update({name: buf[i + 1] for i, name in enumerate(names[:max(0, k - 1)])})
    return out


SERVICE_STATS = ("served", "launches", "null_stream_busy", "library_stream_busy", "ns_before_post",
                 "ns_round_trip", "folds")


def service_stats(reset: bool = False) -> dict:
    """shmemx_service_stats: small one-member blocking calls the resident
    service workgroup served, its launches, and the calls that found the
    legacy default stream / the library's stream busy and waited for it
    first."""
    buf = (ctypes.c_ulonglong * len(SERVICE_STATS))()
    k = lib().shmemx_service_stats(buf, len(buf), 1 if reset else 0)
    return {name: buf[i] for i, name in enumerate(SERVICE_STATS[:max(0, k)])}


MIRROR_STATS = ("write_faults", "read_faults", "blocks_flushed", "blocks_fetched",
                "blocks_device_newer", "fault_waits", "blocks_settled")


def mirror_stats(reset: bool = False) -> dict:
    """shmemx_mirror_stats: the mirrored heap's fault and block counters."""
    buf = (ctypes.c_ulonglong * len(MIRROR_STATS))()
    k = lib().shmemx_mirror_stats(buf, len(buf), 1 if reset else 0)
    return {name: buf[i] for i, name in enumerate(MIRROR_STATS[:k])}


def mirror_device_ptr(address: int) -> int:
    return lib().shmemx_mirror_device_ptr(address) or 0


def mirror_sync(address: int, nbytes: int) -> None:
    _check(lib().shmemx_mirror_sync(address, nbytes), "shmemx_mirror_sync")


def mirror_invalidate(address: int, nbytes: int) -> None:
    _check(lib().shmemx_mirror_invalidate(address, nbytes), "shmemx_mirror_invalidate")


def mirror_acquire(address: int, nbytes: int, for_write: bool = False) -> None:
    """shmemx_mirror_acquire: open [address, address + nbytes) of the view to
    code that cannot take the page fault (system calls)."""
    _check(lib().shmemx_mirror_acquire(address, nbytes, 1 if for_write else 0),
           "shmemx_mirror_acquire")


def host_register(buf, nbytes: int) -> None:
    """shmemx_host_register: page-lock a host range (the reference's heap
    segment) so host operands inside it take the pinned pipeline."""
    _check(lib().shmemx_host_register(addr(buf), nbytes), "shmemx_host_register")


def host_unregister(buf) -> None:
    _check(lib().shmemx_host_unregister(addr(buf)), "shmemx_host_unregister")


def set_fatal_note(text: str | None, exit_code: int = 1) -> None:
    """shmemx_set_fatal_note: text written to stdout if the process dies on
    SIGABRT/SIGSEGV/SIGBUS/SIGFPE/SIGILL/SIGTERM, then _exit(exit_code) for
    SIGTERM and _exit(128 + signal) for the others; None uninstalls."""
    raw = None if text is None else text.encode()
    _check(lib().shmemx_set_fatal_note(raw, exit_code), "shmemx_set_fatal_note")


_hip = None


def memcpy(dst, src, nbytes: int) -> None:
    """hipMemcpy(kind = default) between any host/device addresses (heap
    pointers are plain device addresses, not tensors), complete on return.
    A device-to-device hipMemcpy returns before the copy has run (it is only
    ordered on the legacy default stream), so a reduction enqueued right
    after it on a non-blocking stream (torch.cuda.Stream, the stream-ordered
    API) could read the old bytes: the device is synchronised here."""
    global _hip
    if _hip is None:
        lib()   # torch's HIP runtime first
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipMemcpy.restype = ctypes.c_int
        _hip.hipDeviceSynchronize.restype = ctypes.c_int
    rc = _hip.hipMemcpy(addr(dst), addr(src), nbytes, 4)   # hipMemcpyDefault
    if rc == 0:
        rc = _hip.hipDeviceSynchronize()
    if rc != 0:
        raise ShmemError(6, f"hipMemcpy failed ({rc})")


def malloc(nbytes: int) -> int:
    """shmem_malloc: symmetric HBM allocation (device address, 0 on failure)."""
    return lib().shmem_malloc(nbytes) or 0


def align(alignment: int, nbytes: int) -> int:
    return lib().shmem_align(alignment, nbytes) or 0


def realloc(ptr: int, nbytes: int) -> int:
    return lib().shmem_realloc(ptr or None, nbytes) or 0


def free(ptr: int) -> None:
    lib().shmem_free(ptr or None)


def checksum(type_name: str, ptr, nelems: int) -> int:
    """shmemx_checksum: position-aware 64-bit checksum (gfx950 kernel)."""
    out = ctypes.c_ulonglong(0)
    _check(lib().shmemx_checksum(TYPES[type_name], addr(ptr), nelems, ctypes.byref(out)),
           "shmemx_checksum")
    return out.value


def verify(type_name: str, target, nreduce: int, PE_start: int, logPE_stride: int,
           PE_size: int) -> bool:
    """shmemx_verify: do all members of the set hold the same target?"""
    eq = ctypes.c_int(0)
    _check(lib().shmemx_verify(TYPES[type_name], addr(target), nreduce, PE_start, logPE_stride,
                               PE_size, ctypes.byref(eq)), "shmemx_verify")
    return bool(eq.value)
