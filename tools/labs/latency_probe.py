"""Where the small blocking call's time goes (PE_size = 1, device arrays).

Prints microseconds per iteration for: a torch kernel + synchronize (the HIP
launch + completion floor), the fold kernel on the library stream + that
stream's synchronize, the library's pointer classification, and the whole
blocking shmem_longlong_sum_to_all at nreduce = 1.
"""
import ctypes
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "openshmem-async_amd"))
import shmem_mi355x as shm  # noqa: E402


def per_call(fn, reps=2000):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    torch.cuda.set_device(0)
    shm.init_attr(0, 1, 0, None)
    L = shm.lib()
    hip = ctypes.CDLL("libamdhip64.so.7")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    d = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib_stream = shm.get_stream()
    res = {}
    res["torch_add_sync"] = per_call(lambda: (d.add_(1), torch.cuda.synchronize()))
    res["hip_stream_sync_idle"] = per_call(lambda: hip.hipStreamSynchronize(ctypes.c_void_p(lib_stream)))
    res["fold_libstream_sync"] = per_call(
        lambda: (shm.fold("longlong", "sum", d, s, 1, lib_stream),
                 hip.hipStreamSynchronize(ctypes.c_void_p(lib_stream))))
    res["fold_enqueue_only"] = per_call(lambda: shm.fold("longlong", "sum", d, s, 1, lib_stream))
    torch.cuda.synchronize()
    attr = ctypes.create_string_buffer(256)
    res["hipPointerGetAttributes"] = per_call(
        lambda: hip.hipPointerGetAttributes(attr, ctypes.c_void_p(d.data_ptr())))
    f = L.shmem_longlong_sum_to_all
    args = (ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(s.data_ptr()), 1, 0, 0, 1, None, None)
    res["to_all_n1_device"] = per_call(lambda: f(*args))
    for k, v in res.items():
        print(f"{k:28s} {v:8.2f} us")


if __name__ == "__main__":
    main()
