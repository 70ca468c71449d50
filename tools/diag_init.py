import ctypes, os, sys, faulthandler
faulthandler.enable()
mode = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if mode == "torch_first":
    import torch
    print("torch", torch.__version__, torch.cuda.is_available(), flush=True)
    torch.cuda.set_device(0)
    x = torch.ones(4, device="cuda"); torch.cuda.synchronize()
    print("torch ok", flush=True)
L = ctypes.CDLL(os.path.join(REPO, "openshmem-async_amd", "libshmem_reduce_mi355x.so"))
print("loaded", flush=True)
L.shmemx_init_attr.argtypes = [ctypes.c_int]*3 + [ctypes.c_void_p]
rc = L.shmemx_init_attr(0, 1, 0, None)
print("init rc", rc, flush=True)
L.shmemx_get_stream.restype = ctypes.c_void_p
print("stream", L.shmemx_get_stream(), flush=True)
