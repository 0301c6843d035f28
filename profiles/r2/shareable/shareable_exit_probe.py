"""Exit-time behaviour of the shareable MemPool (which teardown step crashes): variant via argv[1]."""
import ctypes
import faulthandler
import sys

faulthandler.enable()
import torch  # noqa: E402

sys.path.insert(0, ".")
import pccl_amd as pccl  # noqa: E402

v = sys.argv[1]
with pccl.shareable_memory("cuda:0"):
    a = torch.ones(1 << 20, device="cuda:0")
print("alloc ok", pccl.memory.is_shareable(a), pccl.memory.live_bytes(), flush=True)
if v == "del_tensor":
    del a
    torch.cuda.synchronize()
    print("del ok", flush=True)
elif v == "del_pool":
    del a
    pccl.memory._pools.clear()
    import gc
    gc.collect()
    print("pool deleted", pccl.memory.live_bytes(), flush=True)
elif v == "leak":
    for p in pccl.memory._pools.values():
        ctypes.pythonapi.Py_IncRef(ctypes.py_object(p))
    ctypes.pythonapi.Py_IncRef(ctypes.py_object(pccl.memory._allocator))
print("exiting", flush=True)
