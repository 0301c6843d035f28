// Device backend interface. The HIP implementation lives in a separately built plugin (libpccl_hip.so, sources in
// csrc/hip/) that libpccl.so loads with dlopen at pcclInit, so that CPU-only hosts never initialize a GPU runtime and
// so that an application which already loaded PyTorch's HIP runtime shares it (same SONAME) instead of loading a
// second copy. All kernel entry points are asynchronous on the given stream.
#pragma once

#include <cstddef>
#include <cstdint>

#include "../kernels/optim_common.hpp"
#include "../kernels/quant_common.hpp"
#include "types.hpp"

namespace pccl {

using DevStream = void *; // hipStream_t
using DevEvent = void *;  // hipEvent_t

constexpr size_t kIpcHandleBytes = 64;

struct DevPtrInfo {
    bool is_device = false; // device (or managed) memory addressable by kernels
    int device = -1;
};

class DeviceBackend {
public:
    virtual ~DeviceBackend() = default;

    virtual int device_count() = 0;
    virtual bool pointer_info(const void *p, DevPtrInfo &out) = 0;
    virtual bool set_device(int dev) = 0;
    virtual int current_device() = 0;
    // process-independent identity of a device (hash of its PCI bus id): peers compare it to find GPU sharing
    virtual uint64_t device_uid(int dev) = 0;
    // visible device with this uid (-1: not visible to this process); whether `dev` can map `peer`'s memory
    virtual int device_of_uid(uint64_t uid) = 0;
    virtual bool can_access_peer(int dev, int peer) = 0;
    // kernels on `dev` may dereference plain (hipMalloc) pointers of `peer` from now on (idempotent)
    virtual bool enable_peer_access(int dev, int peer) = 0;

    // memory
    virtual void *alloc_device(size_t n) = 0;
    virtual void free_device(void *p) = 0;
    virtual void *alloc_pinned(size_t n) = 0; // host memory, device-mapped (kernels may read/write it)
    virtual void free_pinned(void *p) = 0;
    virtual bool ipc_export(void *dev_ptr, uint8_t handle[kIpcHandleBytes]) = 0;
    virtual void *ipc_open(const uint8_t handle[kIpcHandleBytes]) = 0;
    virtual void ipc_close(void *mapped) = 0;
    // Fault-safe inter-process sharing (virtual memory management): device memory created with hipMemCreate and
    // exported as a POSIX fd. An importer maps the fd into its own address space and holds its own reference to the
    // physical memory, so the memory stays valid when the exporter dies mid-kernel (profiles/r2/ipc/). `size` is
    // rounded up to the allocation granularity (returned in *alloc_size / expected by the others).
    virtual void *vmm_alloc(size_t n, int device, int *fd_out, size_t *alloc_size) = 0;
    virtual void vmm_free(void *p) = 0;                                // exporter side: unmap + release
    virtual void *vmm_import(int fd, size_t size, int device) = 0;    // importer side (does not take the fd)
    virtual void vmm_unmap(void *p) = 0;                               // importer side
    // allocation containing `p` (IPC handles always map the allocation base; offsets travel separately)
    virtual bool address_range(const void *p, void **base, size_t *size) = 0;

    // streams / events
    virtual DevStream create_stream() = 0; // non-blocking stream on the current device
    virtual void destroy_stream(DevStream s) = 0;
    virtual bool stream_sync(DevStream s) = 0;
    virtual DevEvent create_event() = 0;
    virtual void destroy_event(DevEvent e) = 0;
    virtual bool event_record(DevEvent e, DevStream s) = 0;
    virtual int event_query(DevEvent e) = 0; // 1 complete, 0 pending, -1 error
    virtual bool event_sync(DevEvent e) = 0;
    // work submitted to `s` after this call waits for `e` (recorded on any stream of the same device)
    virtual bool stream_wait_event(DevStream s, DevEvent e) = 0;
    virtual bool memcpy_async(void *dst, const void *src, size_t n, DevStream s) = 0; // any direction
    virtual bool memcpy_sync(void *dst, const void *src, size_t n) = 0;
    // copy as a kernel of at most max_grid workgroups (0 = one per tile); any memory the device can address
    virtual bool copy_kernel(void *dst, const void *src, size_t n, int max_grid, DevStream s) = 0;
    virtual bool device_sync() = 0;

    // kernels
    virtual bool reduce(void *dst, const void *src, size_t count, DType t, ReduceOp op, DevStream s) = 0;
    // dst = op(dst, src) and out = the result (out: pinned host memory, the next ring step's payload)
    virtual bool reduce_copy(void *dst, const void *src, void *out, size_t count, DType t, ReduceOp op,
                             DevStream s) = 0;
    virtual bool dequant_reduce(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                                const kernels::QuantParams &p, DevStream s) = 0;
    // dequant_reduce that also writes each workgroup's (min, max) of the stored results as two doubles to
    // mm_partials[2 * k ...] (device memory), k < *blocks <= max_blocks: the min / max of a chunk produced by several
    // such launches is minmax_fold over all their partials (no second pass over the chunk)
    virtual bool dequant_reduce_minmax(void *dst, const void *src_q, size_t count, DType vtype, DType qtype,
                                       ReduceOp op, const kernels::QuantParams &p, double *mm_partials, int max_blocks,
                                       int *blocks, DevStream s) = 0;
    virtual bool quantize(void *dst_q, const void *src, size_t count, DType vtype, DType qtype,
                          const kernels::QuantParams &p, DevStream s) = 0;
    // quantize, and overwrite `src` with D(Q(src)) in the same pass (bit-identical to quantize followed by
    // dequant_reduce(..., ReduceOp::Set, ...) of the quantized bytes)
    virtual bool quantize_setback(void *dst_q, void *src, size_t count, DType vtype, DType qtype,
                                  const kernels::QuantParams &p, DevStream s) = 0;
    // writes {min, max} as two doubles to `out2` (pinned host or device memory)
    virtual bool minmax(const void *src, size_t count, DType vtype, double *out2, DevStream s) = 0;
    // folds n_partials (min, max) pairs (device memory) of `count` elements into `out2` (asynchronous)
    virtual bool minmax_fold(const double *partials, int n_partials, size_t count, double *out2, DevStream s) = 0;
    virtual bool finalize_avg(void *dst, size_t count, DType t, size_t world_size, DevStream s) = 0;

    // Intra-node xGMI kernels. srcs[k] points to shard `count` elements in peer k's buffer (IPC-mapped);
    // every dsts[0..ndst) receives op(srcs[0..n)) reduced in order 0..n-1 (the own output and, in the one-shot push
    // all-reduce, the IPC-mapped outputs of the peers). Avg divides by n at the end.
    // max_grid: workgroup budget of this launch (0 = default); peers sharing one GPU split the chip between them.
    // release_system: a destination is another GPU's memory (system-scope release at kernel end)
    virtual bool multi_reduce(void *const *dsts, int ndst, const void *const *srcs, int n, size_t count, DType t,
                              ReduceOp op, DevStream s, int max_grid = 0, bool release_system = false) = 0;
    // dst regions gathered from n sources: dst[k*stride ...] = srcs[k] for k != skip (count elements each,
    // segment k has counts[k] elements at element offset offsets[k]).
    virtual bool multi_gather(void *dst, const void *const *srcs, const size_t *offsets, const size_t *counts, int n,
                              int skip, DType t, DevStream s, bool release_system = false) = 0;

    // Simple hash of device memory (bit-identical to kernels::simplehash_host). Synchronous (syncs `s` only).
    virtual uint32_t simplehash(const void *dev_ptr, size_t n_bytes, DevStream s) = 0;
    // Asynchronous variant: the final kernel writes the hash to `out_pinned` (pinned host memory) when `s` reaches
    // it; several hashes can be queued on one stream and collected with a single stream_sync. 16-byte aligned input.
    virtual bool simplehash_async(const void *dev_ptr, size_t n_bytes, uint32_t *out_pinned, DevStream s) = 0;
    // CRC-32C kernel pass over n_tiles 16 KiB tiles at a 16-byte aligned device pointer. Returns one raw CRC partial
    // per workgroup (each covers tiles_per_wg tiles, the last one the remainder). `tables` = 12 x 256 words (8 slicing
    // tables + the 16 KiB tile-shift table), `levels` = the 8 tree multipliers. Synchronous. Use device_crc32c().
    virtual bool crc32c_tiles(const void *dev_ptr, size_t n_tiles, const uint32_t *tables, const uint32_t *levels,
                              uint32_t *partials, size_t max_partials, size_t &n_partials, size_t &tiles_per_wg,
                              DevStream s) = 0;
    // Fills device memory with the reference test pattern (random_init_kernel of the reference tests).
    virtual bool fill_test_pattern(void *dev_ptr, size_t n_u64, DevStream s) = 0;

    // fused DiLoCo outer step (csrc/kernels/optim_common.hpp); outer/mom/pg fp32, local F32/BF16/F16
    virtual bool pseudo_grad(float *pg, const float *outer, const void *local, size_t count, DType local_t,
                             DevStream s) = 0;
    virtual bool outer_sgd(float *outer, float *mom, const float *pg, void *local, size_t count, DType local_t,
                           const kernels::OuterSgdParams &p, DevStream s) = 0;
};

// Waits for `e` by polling with short sleeps (2 us doubling to 100 us) instead of the runtime's synchronize, which
// busy-waits: the device ring's sender / op threads wait on staging copies for milliseconds at a time, and the
// loopback-TCP ring is CPU-bound (kernel socket copies on the box's CPU share, bench extra cpu_cores_busy_rank0), so
// every spinning waiter takes a core from the socket copies.
bool event_wait_polling(DeviceBackend *be, DevEvent e);

// Returns the process-wide backend (nullptr if HIP is unavailable). Loaded lazily and thread-safely.
DeviceBackend *device_backend();
bool device_backend_available();

// Standard CRC-32C of device memory: HIP kernel over the 16-byte aligned 16 KiB tiles, host-side fold of the
// workgroup partials plus the unaligned head and the tail (bit-identical to kernels::crc32c). `ok` reports failure.
uint32_t device_crc32c(DeviceBackend *be, const void *dev_ptr, size_t n_bytes, DevStream s, bool *ok = nullptr);

} // namespace pccl

// Plugin entry point (exported by libpccl_hip.so).
extern "C" pccl::DeviceBackend *pccl_create_hip_backend();
