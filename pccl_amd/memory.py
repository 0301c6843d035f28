"""Shareable device memory for the fault-safe zero-copy xGMI path.

Same-host peers all-reduce device tensors over xGMI (``csrc/client/ipc.cpp``). In the default fault-safe mode
(``PCCL_IPC_MODE=safe``) a peer process may only touch another process's memory through a VMM allocation shared as
a file descriptor: the importer holds its own reference to the physical pages, so a peer that is SIGKILLed while the
others' kernels read its input or write its output leaves valid memory behind. Ordinary PyTorch tensors are
therefore staged — copied into such a buffer before the op and out of one after it, three times the HBM traffic of
the all-reduce kernel alone. Tensors allocated here are fd-shareable from the start and are reduced in place::

    import pccl_amd as pccl
    with pccl.shareable_memory():                 # torch.cuda.MemPool backed by libpccl's VMM allocator
        grads = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    comm.all_reduce(grads, out, ...)              # out-of-place ops read / write both buffers directly

``DataParallel`` and ``DiLoCo`` (``pccl_amd.parallel``) allocate their communication buffers here automatically.
The reference has no counterpart (its CUDA path is a TCP ring); this is the MI355X-native design that makes the
xGMI fast path both zero-copy and safe under peer death.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading

from . import _native

_lock = threading.RLock()
_allocator = None
_pools: dict = {}


def _immortal(obj) -> None:
    """Keeps `obj` alive until the process exits. Measured on MI355X (profiles/r2/shareable/shareable_exit_probe.py): when
    the interpreter's final garbage collection destroys a MemPool backed by a pluggable allocator, the process dies
    with SIGSEGV; deleting it earlier or never is fine. The OS reclaims the memory at exit."""
    ctypes.pythonapi.Py_IncRef(ctypes.py_object(obj))


def _torch():
    import torch
    return torch


def available() -> bool:
    """True when shareable allocations can be made here (HIP device present and torch's MemPool API available)."""
    torch = _torch()
    return bool(torch.cuda.is_available() and hasattr(torch.cuda, "MemPool") and _native.C.pcclxHipDeviceCount() > 0)


def _get_allocator():
    global _allocator
    with _lock:
        if _allocator is None:
            from torch.cuda.memory import CUDAPluggableAllocator
            # the same file the ctypes bindings loaded: dlopen returns that handle, so the allocation registry that
            # the all-reduce consults is the one these entry points fill
            _allocator = CUDAPluggableAllocator(_native.LIB_PATH, "pcclxShareableMalloc", "pcclxShareableFree")
            _immortal(_allocator)
        return _allocator


def shareable_pool(device=None):
    """The process-wide ``torch.cuda.MemPool`` of shareable memory for ``device`` (default: the current device)."""
    torch = _torch()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _lock:  # one pool per device even when several peer threads ask at once
        pool = _pools.get(idx)
        if pool is None:
            alloc = _get_allocator()
            with torch.cuda.device(idx):
                pool = torch.cuda.MemPool(alloc.allocator())
            _immortal(pool)
            _pools[idx] = pool
    return pool


_ctx_locks: dict = {}
_tls = threading.local()


@contextlib.contextmanager
def shareable_memory(device=None):
    """Context manager: CUDA tensors allocated inside come from the shareable pool of ``device``.

    PyTorch lets only one thread at a time route allocations to a given MemPool ("already recording to mempool_id"),
    so threads entering this context for the same device take turns (keep the body to allocations); nested use in
    one thread is a no-op."""
    torch = _torch()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    pool = shareable_pool(dev)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    active = getattr(_tls, "active", None)
    if active is None:
        active = _tls.active = set()
    if idx in active:
        yield pool
        return
    with _lock:
        lk = _ctx_locks.setdefault(idx, threading.Lock())
    with lk:
        active.add(idx)
        try:
            with torch.cuda.use_mem_pool(pool, dev):
                yield pool
        finally:
            active.discard(idx)


def empty(*size, dtype=None, device=None):
    """``torch.empty`` in shareable memory (``device`` must be a HIP device)."""
    torch = _torch()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    with shareable_memory(dev):
        return torch.empty(*size, dtype=dtype, device=dev)


def zeros(*size, dtype=None, device=None):
    t = empty(*size, dtype=dtype, device=device)
    t.zero_()
    return t


def empty_like(t):
    return empty(t.shape, dtype=t.dtype, device=t.device)


def is_shareable(t) -> bool:
    """True if all of ``t``'s bytes lie in one live shareable allocation."""
    if getattr(t, "device", None) is None or t.device.type != "cuda":
        return False
    off = ctypes.c_uint64()
    size = ctypes.c_size_t()
    return bool(_native.C.pcclxShareableQuery(ctypes.c_void_p(t.data_ptr()), t.numel() * t.element_size(),
                                              ctypes.byref(off), ctypes.byref(size)))


def live_bytes() -> int:
    """Bytes currently held in shareable allocations by this process (PyTorch's cache included)."""
    return int(_native.C.pcclxShareableLiveBytes())


def ipc_buffer_stats() -> dict:
    """How this process's xGMI/IPC ops handed their buffers to the peers since start: direct (zero-copy) vs staged
    (copy-in / copy-out through VMM comm buffers), per input and output; plus ``quarantined`` (staged comm buffers of
    aborted ops, never reissued) and ``zombie_drains`` (abort drains that waited for a dead peer's threads to finish
    tearing down its address space, i.e. its GPU queues), ``preflight_failed`` / ``preflight_passed`` (cross-GPU write
    probes on the first op of an arena whose peers span several GPUs), ``reclaimed`` (quarantined buffers handed out
    again once no peer could still touch them for the aborted op) and ``quarantine_freed`` (quarantined VMM buffers
    freed beyond the 8 GiB quarantine cap)."""
    out = (ctypes.c_uint64 * 10)()
    n = int(_native.C.pcclxIpcStatsEx(out, 10))
    keys = ("direct_in", "direct_out", "staged_in", "staged_out", "quarantined", "zombie_drains", "preflight_failed",
            "preflight_passed", "reclaimed", "quarantine_freed")
    return {k: int(out[i]) for i, k in enumerate(keys[:n])}


def staging_pool_stats(reset_peak: bool = False) -> dict:
    """Bytes of the library's staging pools in this process: per pool (``pinned`` host, ``device`` HBM, plain
    ``host``) the bytes leased out now (``in_use``), the most leased out at once (``peak``, since the last
    ``reset_peak=True`` call), the free bytes kept cached for reuse (``cached``) and the fresh runtime allocations so far
    (``allocs``, pool misses) with the microseconds they took (``alloc_us``). The device rings size their staging
    by the op's segment chunk (PCCL_SEGMENT_CHUNK_MIB), not by the tensor."""
    out = (ctypes.c_uint64 * 15)()
    n = int(_native.C.pcclxPoolStats(out, 15, 1 if reset_peak else 0))
    res = {pool: {"in_use": int(out[3 * k]), "peak": int(out[3 * k + 1]), "cached": int(out[3 * k + 2])}
           for k, pool in enumerate(("pinned", "device", "host"))}
    if n >= 15:  # fresh runtime allocations (pool misses) and the microseconds they took
        for k, pool in enumerate(("pinned", "device", "host")):
            res[pool]["allocs"] = int(out[9 + k])
            res[pool]["alloc_us"] = int(out[12 + k])
    return res


def reserve_staging(*, pinned_bytes: int = 0, pinned_count: int = 0, device_bytes: int = 0, device_count: int = 0,
                    device=None) -> None:
    """Fills the library's staging pools ahead of the first ops: ``pinned_count`` pinned host buffers of
    ``pinned_bytes`` and ``device_count`` HBM buffers of ``device_bytes`` on ``device`` (default: the current GPU) are
    allocated and kept cached for the ops' leases (``pcclxPoolReserve``). The call releases the GIL, so a thread can
    run it next to ``Communicator.connect()``, whose wait for admission it then overlaps (otherwise a fresh process
    allocates this staging inside its first op)."""
    dev = -1
    if device_count and device_bytes:
        torch = _torch()
        d = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        dev = d.index if d.index is not None else torch.cuda.current_device()
    rc = int(_native.C.pcclxPoolReserve(int(pinned_bytes), int(pinned_count), int(device_bytes), int(device_count), dev))
    if rc != 0:
        raise MemoryError(f"pcclxPoolReserve failed ({rc})")


def reserve_device_ring_staging(nbytes: int, world: int, *, device=None, in_place: bool = False,
                                segment_chunk: int = 128 << 20, peers: int = 1) -> None:
    """reserve_staging with what one device-ring all-reduce of ``nbytes`` per peer at ``world`` peers leases: 3 pinned
    send + 3 pinned receive + 3 HBM buffers of one ring chunk (at most the segment chunk, PCCL_SEGMENT_CHUNK_MIB), and
    for an in-place op an HBM backup of the input (csrc/client/ring_device.cpp); ``peers``: how many peers of this
    process (threads) run such an op at the same time."""
    stage = min(-(-int(nbytes) // max(1, int(world))), int(segment_chunk)) + 4096
    k = max(1, int(peers))
    reserve_staging(pinned_bytes=stage, pinned_count=6 * k, device_bytes=stage, device_count=3 * k, device=device)
    if in_place:
        reserve_staging(device_bytes=int(nbytes), device_count=k, device=device)


def pcie_stats() -> dict:
    """Bytes this process's device rings moved between pinned host staging and HBM so far (counted where the copies and
    the kernels that read / write pinned memory are queued): ``h2d`` and ``d2h``. With one process per GPU this is
    what that GPU's PCIe link carried for the library."""
    out = (ctypes.c_uint64 * 2)()
    _native.C.pcclxPcieStats(out, 2)
    return {"h2d": int(out[0]), "d2h": int(out[1])}


def maybe_shareable(device) -> contextlib.AbstractContextManager:
    """``shareable_memory(device)`` for HIP devices when available, a no-op context otherwise (CPU tensors, no GPU,
    or PCCL_SHAREABLE_BUFFERS=0)."""
    import os
    torch = _torch()
    dev = torch.device(device)
    if dev.type != "cuda" or os.environ.get("PCCL_SHAREABLE_BUFFERS", "1") == "0" or not available():
        return contextlib.nullcontext()
    return shareable_memory(dev)
