// Shareable device memory: VMM allocations (hipMemCreate) that pccl-amd publishes as POSIX fds (vmm_share.hpp) the
// moment they are created, so that an xGMI all-reduce can hand them to peer processes as they are.
//
// Why: in the fault-safe IPC mode (PCCL_IPC_MODE=safe, the default) a peer process may only ever touch another
// process's memory through a VMM fd import — an importer holds its own reference to the physical pages, so a peer
// SIGKILLed mid-kernel leaves valid memory behind (profiles/r2/ipc/vmm_exporter_death_probe.log). Ordinary
// (hipMalloc / PyTorch caching allocator) buffers therefore cost a copy-in and a copy-out through staged comm
// buffers: 3x the HBM traffic of the one-shot push kernel alone. Buffers allocated from this allocator are already
// fd-shareable: the all-reduce reads and writes them in place, fault-safe and zero-copy.
//
// The allocator entry points have the signature of PyTorch's pluggable allocator (torch.cuda.MemPool +
// CUDAPluggableAllocator, see pccl_amd/memory.py), so `with pccl_amd.shareable_memory(): t = torch.empty(...)`
// places tensors here; the caching allocator sub-allocates inside our allocations and lookup() resolves any pointer
// into (allocation, offset).
#pragma once

#include <cstddef>
#include <cstdint>

#include "vmm_share.hpp"

namespace pccl::client::shareable {

// allocates `bytes` of shareable device memory on `device` (rounded up to the VMM granularity); nullptr on failure
void *alloc(size_t bytes, int device);
// releases an allocation returned by alloc() (must be the allocation base); unknown pointers are ignored
void free(void *p);

struct Share {
    VmmHandle handle;   // what a peer process needs to import the allocation
    uint64_t offset = 0; // of the looked-up pointer inside the allocation
    size_t size = 0;     // allocation size
    int device = -1;
};
// resolves a pointer anywhere inside a live shareable allocation that holds [p, p + bytes)
bool lookup(const void *p, size_t bytes, Share &out);
// live allocations / bytes (tests, diagnostics)
size_t live_allocations();
size_t live_bytes();

} // namespace pccl::client::shareable
