// HIP implementation of pccl::DeviceBackend (built as libpccl_hip.so for gfx950, loaded by libpccl.so via dlopen).
// Kernel families live in hip_reduce.hip / hip_quant.hip / hip_ipc.hip / hip_hash.hip (see kernels.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <vector>
#include <memory>
#include <mutex>

#include "../common/device_backend.hpp"
#include "launchers.hpp"

namespace pccl {
namespace {

#define HIP_OK(expr) (hipSuccess == (expr))

class HipBackend final : public DeviceBackend {
public:
    HipBackend() { (void)hipGetDeviceCount(&n_devices_); }

    int device_count() override { return n_devices_; }

    bool pointer_info(const void *p, DevPtrInfo &out) override {
        out = DevPtrInfo{};
        if (p == nullptr || n_devices_ == 0) return true;
        hipPointerAttribute_t attr{};
        if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
            (void)hipGetLastError(); // unregistered host memory: clear the sticky error
            return true;
        }
        if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) {
            out.is_device = true;
            out.device = attr.device;
        }
        return true;
    }

    bool set_device(int dev) override { return HIP_OK(hipSetDevice(dev)); }
    uint64_t device_uid(int dev) override {
        char bus[64] = {};
        if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) {
            (void)hipGetLastError();
            return static_cast<uint64_t>(dev) + 1;
        }
        uint64_t h = 1469598103934665603ull; // FNV-1a
        for (const char *c = bus; *c; ++c) h = (h ^ static_cast<uint8_t>(*c)) * 1099511628211ull;
        return h;
    }
    int device_of_uid(uint64_t uid) override {
        const int n = device_count();
        for (int d = 0; d < n; ++d)
            if (device_uid(d) == uid) return d;
        return -1;
    }
    bool can_access_peer(int dev, int peer) override {
        if (dev == peer) return true;
        int ok = 0;
        if (hipDeviceCanAccessPeer(&ok, dev, peer) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return ok != 0;
    }
    bool enable_peer_access(int dev, int peer) override {
        if (dev == peer) return true;
        std::lock_guard l(peer_mtx_);
        if (peer_enabled_.count({dev, peer})) return true;
        int cur = -1;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(dev);
        const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
        (void)hipGetLastError();
        if (cur >= 0) (void)hipSetDevice(cur);
        const bool ok = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
        if (ok) peer_enabled_.insert({dev, peer});
        return ok;
    }
    int current_device() override {
        int d = -1;
        (void)hipGetDevice(&d);
        return d;
    }

    void *alloc_device(size_t n) override {
        void *p = nullptr;
        if (!HIP_OK(hipMalloc(&p, n ? n : 1))) return nullptr;
        return p;
    }
    void free_device(void *p) override {
        if (p) (void)hipFree(p);
    }
    void *alloc_pinned(size_t n) override {
        void *p = nullptr;
        if (!HIP_OK(hipHostMalloc(&p, n ? n : 1, hipHostMallocPortable | hipHostMallocMapped))) return nullptr;
        return p;
    }
    void free_pinned(void *p) override {
        if (p) (void)hipHostFree(p);
    }
    bool ipc_export(void *dev_ptr, uint8_t handle[kIpcHandleBytes]) override {
        hipIpcMemHandle_t h;
        if (!HIP_OK(hipIpcGetMemHandle(&h, dev_ptr))) return false;
        static_assert(sizeof(h) <= kIpcHandleBytes, "ipc handle size");
        std::memset(handle, 0, kIpcHandleBytes);
        std::memcpy(handle, &h, sizeof(h));
        return true;
    }
    void *ipc_open(const uint8_t handle[kIpcHandleBytes]) override {
        hipIpcMemHandle_t h;
        std::memcpy(&h, handle, sizeof(h));
        void *p = nullptr;
        if (!HIP_OK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess))) {
            (void)hipGetLastError();
            return nullptr;
        }
        return p;
    }
    void ipc_close(void *mapped) override {
        if (mapped) (void)hipIpcCloseMemHandle(mapped);
    }

    void *vmm_alloc(size_t n, int device, int *fd_out, size_t *alloc_size) override {
        hipMemAllocationProp prop = vmm_prop(device);
        size_t gran = 0;
        if (!HIP_OK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum)) || gran == 0)
            return nullptr;
        const size_t size = (std::max<size_t>(n, 1) + gran - 1) / gran * gran;
        void *p = nullptr;
        VmmMap m{size, {}, true, device};
        {
            // a retained allocation of this device that fits (at most 2x): still mapped, re-exported below
            std::lock_guard l(vmm_mtx_);
            auto best = retained_.end();
            for (auto it = retained_.begin(); it != retained_.end(); ++it)
                if (it->second.device == device && it->second.size >= size && it->second.size <= 2 * size &&
                    (best == retained_.end() || it->second.size < best->second.size))
                    best = it;
            if (best != retained_.end()) {
                p = best->first;
                m = best->second;
                retained_bytes_ -= m.size;
                retained_.erase(best);
            }
        }
        if (!p) {
            if (!HIP_OK(hipMemCreate(&m.handle, size, &prop, 0))) return nullptr;
            p = vmm_map(m.handle, size, device, gran);
            if (!p) {
                (void)hipMemRelease(m.handle);
                return nullptr;
            }
        }
        int fd = -1;
        if (!HIP_OK(hipMemExportToShareableHandle(&fd, m.handle, hipMemHandleTypePosixFileDescriptor, 0)) || fd < 0) {
            vmm_unmap_raw(p, m.size);
            (void)hipMemRelease(m.handle);
            return nullptr;
        }
        {
            std::lock_guard l(vmm_mtx_);
            vmm_[p] = m;
        }
        *fd_out = fd;
        *alloc_size = m.size;
        return p;
    }
    void vmm_free(void *p) override {
        VmmMap m;
        {
            std::lock_guard l(vmm_mtx_);
            auto it = vmm_.find(p);
            if (it == vmm_.end()) return;
            m = it->second;
            vmm_.erase(it);
            // exported comm buffers outlive their communicator in this cache (mapped, VA kept): unmapping is what
            // costs address space (see vmm_unmap_raw)
            if (m.owns_handle && retained_bytes_ + m.size <= vmm_retain_cap()) {
                retained_bytes_ += m.size;
                retained_[p] = m;
                return;
            }
        }
        vmm_unmap_raw(p, m.size);
        if (m.owns_handle) (void)hipMemRelease(m.handle);
    }
    void *vmm_import(int fd, size_t size, int device) override {
        hipMemGenericAllocationHandle_t h{};
        int fd_copy = fd; // the runtime takes a pointer to the fd
        if (!HIP_OK(hipMemImportFromShareableHandle(&h, &fd_copy, hipMemHandleTypePosixFileDescriptor))) return nullptr;
        hipMemAllocationProp prop = vmm_prop(device);
        size_t gran = 0;
        if (!HIP_OK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum)) || gran == 0) {
            (void)hipMemRelease(h);
            return nullptr;
        }
        void *p = vmm_map(h, size, device, gran);
        (void)hipMemRelease(h); // the mapping keeps the physical memory alive (even after the exporter's death)
        if (!p) return nullptr;
        std::lock_guard l(vmm_mtx_);
        vmm_[p] = VmmMap{size, h, false, device};
        return p;
    }
    void vmm_unmap(void *p) override { vmm_free(p); }
    bool address_range(const void *p, void **base, size_t *size) override {
        hipDeviceptr_t b = nullptr;
        size_t n = 0;
        if (hipMemGetAddressRange(&b, &n, const_cast<void *>(p)) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        *base = reinterpret_cast<void *>(b);
        *size = n;
        return true;
    }

    DevStream create_stream() override {
        hipStream_t s = nullptr;
        if (!HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking))) return nullptr;
        return s;
    }
    void destroy_stream(DevStream s) override {
        if (!s) return;
        {
            std::lock_guard l(scratch_mtx_);
            auto it = scratch_.find(s);
            if (it != scratch_.end()) {
                (void)hipFree(it->second.dev);
                (void)hipHostFree(it->second.host);
                scratch_.erase(it);
            }
        }
        (void)hipStreamDestroy(static_cast<hipStream_t>(s));
    }
    bool stream_sync(DevStream s) override { return HIP_OK(hipStreamSynchronize(static_cast<hipStream_t>(s))); }
    DevEvent create_event() override {
        hipEvent_t e = nullptr;
        if (!HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming))) return nullptr;
        return e;
    }
    void destroy_event(DevEvent e) override {
        if (e) (void)hipEventDestroy(static_cast<hipEvent_t>(e));
    }
    bool event_record(DevEvent e, DevStream s) override {
        return HIP_OK(hipEventRecord(static_cast<hipEvent_t>(e), static_cast<hipStream_t>(s)));
    }
    int event_query(DevEvent e) override {
        const hipError_t r = hipEventQuery(static_cast<hipEvent_t>(e));
        if (r == hipSuccess) return 1;
        if (r == hipErrorNotReady) return 0;
        return -1;
    }
    bool event_sync(DevEvent e) override { return HIP_OK(hipEventSynchronize(static_cast<hipEvent_t>(e))); }
    bool stream_wait_event(DevStream s, DevEvent e) override {
        return HIP_OK(hipStreamWaitEvent(static_cast<hipStream_t>(s), static_cast<hipEvent_t>(e), 0));
    }
    bool memcpy_async(void *dst, const void *src, size_t n, DevStream s) override {
        if (n == 0) return true;
        return HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDefault, static_cast<hipStream_t>(s)));
    }
    bool memcpy_sync(void *dst, const void *src, size_t n) override {
        if (n == 0) return true;
        return HIP_OK(hipMemcpy(dst, src, n, hipMemcpyDefault));
    }
    bool device_sync() override { return HIP_OK(hipDeviceSynchronize()); }
    bool copy_kernel(void *dst, const void *src, size_t n, int max_grid, DevStream s) override {
        return hipk::launch_copy_bytes(dst, src, n, max_grid, static_cast<hipStream_t>(s));
    }

    bool reduce(void *dst, const void *src, size_t count, DType t, ReduceOp op, DevStream s) override {
        return hipk::launch_reduce(dst, src, count, t, op, static_cast<hipStream_t>(s));
    }
    bool reduce_copy(void *dst, const void *src, void *out, size_t count, DType t, ReduceOp op, DevStream s) override {
        return hipk::launch_reduce_copy(dst, src, out, count, t, op, static_cast<hipStream_t>(s));
    }
    bool dequant_reduce(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                        const kernels::QuantParams &p, DevStream s) override {
        return hipk::launch_dequant_reduce(dst, src_q, count, vtype, qtype, op, p, static_cast<hipStream_t>(s));
    }
    bool dequant_reduce_minmax(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                               const kernels::QuantParams &p, double *mm, int max_blocks, int *blocks,
                               DevStream s) override {
        if (!mm || max_blocks < 1) return false;
        return hipk::launch_dequant_reduce(dst, src_q, count, vtype, qtype, op, p, static_cast<hipStream_t>(s), mm,
                                           max_blocks, blocks);
    }
    bool quantize(void *dst_q, const void *src, size_t count, DType vtype, DType qtype, const kernels::QuantParams &p,
                  DevStream s) override {
        return hipk::launch_quantize(dst_q, src, count, vtype, qtype, p, static_cast<hipStream_t>(s));
    }
    bool quantize_setback(void *dst_q, void *src, size_t count, DType vtype, DType qtype,
                          const kernels::QuantParams &p, DevStream s) override {
        return hipk::launch_quantize(dst_q, src, count, vtype, qtype, p, static_cast<hipStream_t>(s), true);
    }
    bool minmax(const void *src, size_t count, DType vtype, double *out2, DevStream s) override {
        // the partials scratch is per stream; threads sharing a stream (e.g. the null stream) take turns until the
        // result has landed, so interleaved launches can never mix their partials
        Scratch &sc = scratch_for(s);
        std::lock_guard l(*sc.mtx);
        return hipk::launch_minmax(src, count, vtype, sc.dev, out2, static_cast<hipStream_t>(s)) &&
               hipStreamSynchronize(static_cast<hipStream_t>(s)) == hipSuccess;
    }
    bool minmax_fold(const double *partials, int n, size_t count, double *out2, DevStream s) override {
        return hipk::launch_minmax_fold(partials, n, count, out2, static_cast<hipStream_t>(s));
    }
    bool finalize_avg(void *dst, size_t count, DType t, size_t ws, DevStream s) override {
        return hipk::launch_finalize_avg(dst, count, t, ws, static_cast<hipStream_t>(s));
    }
    bool multi_reduce(void *const *dsts, int ndst, const void *const *srcs, int n, size_t count, DType t, ReduceOp op,
                      DevStream s, int max_grid, bool release_system) override {
        return hipk::launch_multi_reduce(dsts, ndst, srcs, n, count, t, op, static_cast<hipStream_t>(s), max_grid,
                                         release_system);
    }
    bool multi_gather(void *dst, const void *const *srcs, const size_t *offsets, const size_t *counts, int n, int skip,
                      DType t, DevStream s, bool release_system) override {
        return hipk::launch_multi_gather(dst, srcs, offsets, counts, n, skip, t, static_cast<hipStream_t>(s),
                                         release_system);
    }
    uint32_t simplehash(const void *dev_ptr, size_t n_bytes, DevStream s) override {
        if (n_bytes == 0) return 0;
        Scratch &sc = scratch_for(s);
        std::lock_guard l(*sc.mtx);
        auto *out = reinterpret_cast<uint32_t *>(sc.host);
        if (!hipk::launch_simplehash(dev_ptr, n_bytes, reinterpret_cast<uint32_t *>(sc.dev), out,
                                     static_cast<hipStream_t>(s)) ||
            hipStreamSynchronize(static_cast<hipStream_t>(s)) != hipSuccess) {
            std::fprintf(stderr, "[pccl_hip] simplehash failed\n");
            return 0;
        }
        return out[0];
    }
    bool simplehash_async(const void *dev_ptr, size_t n_bytes, uint32_t *out_pinned, DevStream s) override {
        if (n_bytes == 0) {
            *out_pinned = 0;
            return true;
        }
        // the per-stream partials are reused by the next hash on the same stream only after this one's final kernel
        // (stream order), so only the launch itself is serialised
        Scratch &sc = scratch_for(s);
        std::lock_guard l(*sc.mtx);
        return hipk::launch_simplehash(dev_ptr, n_bytes, reinterpret_cast<uint32_t *>(sc.dev), out_pinned,
                                       static_cast<hipStream_t>(s));
    }
    bool crc32c_tiles(const void *dev_ptr, size_t n_tiles, const uint32_t *tables, const uint32_t *levels,
                      uint32_t *partials, size_t max_partials, size_t &n_partials, size_t &tiles_per_wg,
                      DevStream s) override {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return false;
        void *tab = nullptr;
        {
            std::lock_guard l(scratch_mtx_);
            auto it = crc_tables_.find(dev);
            if (it == crc_tables_.end()) {
                if (!HIP_OK(hipMalloc(&tab, 12 * 256 * sizeof(uint32_t))) ||
                    !HIP_OK(hipMemcpy(tab, tables, 12 * 256 * sizeof(uint32_t), hipMemcpyHostToDevice)))
                    return false;
                crc_tables_[dev] = tab;
            } else {
                tab = it->second;
            }
        }
        Scratch &sc = scratch_for(s);
        std::lock_guard l(*sc.mtx);
        auto *part = reinterpret_cast<uint32_t *>(sc.dev); // 16 KiB of scratch: up to 4096 partials
        size_t grid = 0;
        const auto st = static_cast<hipStream_t>(s);
        if (!hipk::launch_crc32c(dev_ptr, n_tiles, tab, levels, part, std::min<size_t>(max_partials, 4096), grid,
                                 tiles_per_wg, st) ||
            !HIP_OK(hipMemcpyAsync(partials, part, grid * sizeof(uint32_t), hipMemcpyDeviceToHost, st)) ||
            !HIP_OK(hipStreamSynchronize(st)))
            return false;
        n_partials = grid;
        return true;
    }
    bool fill_test_pattern(void *dev_ptr, size_t n_u64, DevStream s) override {
        return hipk::launch_test_pattern(dev_ptr, n_u64, static_cast<hipStream_t>(s));
    }
    bool pseudo_grad(float *pg, const float *outer, const void *local, size_t count, DType lt, DevStream s) override {
        return hipk::launch_pseudo_grad(pg, outer, local, count, lt, static_cast<hipStream_t>(s));
    }
    bool outer_sgd(float *outer, float *mom, const float *pg, void *local, size_t count, DType lt,
                   const kernels::OuterSgdParams &p, DevStream s) override {
        return hipk::launch_outer_sgd(outer, mom, pg, local, count, lt, p, static_cast<hipStream_t>(s));
    }

private:
    struct VmmMap {
        size_t size = 0;
        hipMemGenericAllocationHandle_t handle{};
        bool owns_handle = false;
        int device = 0;
    };
    std::mutex vmm_mtx_;
    std::map<void *, VmmMap> vmm_;
    std::map<void *, VmmMap> retained_; // freed exported allocations kept mapped for reuse
    size_t retained_bytes_ = 0;
    static size_t vmm_retain_cap() {
        static const size_t cap = [] {
            const char *v = std::getenv("PCCL_VMM_RETAIN_BYTES");
            return v ? static_cast<size_t>(std::strtoull(v, nullptr, 10)) : (size_t{16} << 30);
        }();
        return cap;
    }
    static hipMemAllocationProp vmm_prop(int device) {
        hipMemAllocationProp prop{};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = device;
        prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
        return prop;
    }
    // reserve + map + read/write access for every visible device that can reach `device` (peers on other GPUs of this
    // process may access it too)
    void *vmm_map(hipMemGenericAllocationHandle_t h, size_t size, int device, size_t gran) {
        void *p = nullptr;
        if (!HIP_OK(hipMemAddressReserve(&p, size, gran, nullptr, 0))) return nullptr;
        if (!HIP_OK(hipMemMap(p, size, 0, h, 0))) {
            (void)hipMemAddressFree(p, size);
            return nullptr;
        }
        std::vector<hipMemAccessDesc> acc;
        const int n = device_count();
        for (int d = 0; d < n; ++d) {
            if (d != device && !can_access_peer(d, device)) continue;
            hipMemAccessDesc a{};
            a.location.type = hipMemLocationTypeDevice;
            a.location.id = d;
            a.flags = hipMemAccessFlagsProtReadWrite;
            acc.push_back(a);
        }
        if (!HIP_OK(hipMemSetAccess(p, size, acc.data(), acc.size()))) {
            vmm_unmap_raw(p, size);
            return nullptr;
        }
        return p;
    }
    // Unmaps but never frees the address range. Measured on MI355X with both the ROCm 7.2 and PyTorch's bundled HIP
    // runtime (csrc/tools/vmm_churn_probe.hip, profiles/r2/ipc/vmm_churn.md): once a range is hipMemAddressFree'd
    // and handed out again by hipMemAddressReserve, kernels and copies on the new mapping read and write the wrong
    // pages (146 of 150 rounds corrupted; live allocations overwritten), and with the range kept reserved, 0 of 150.
    // A leaked range costs virtual address space only (the physical memory is released).
    static void vmm_unmap_raw(void *p, size_t size) { (void)hipMemUnmap(p, size); }

    struct Scratch {
        double *dev = nullptr;  // 2 x 1024 doubles: min/max partials, or 960 hash partials, or 4096 CRC partials
        double *host = nullptr; // pinned result words
        std::shared_ptr<std::mutex> mtx = std::make_shared<std::mutex>();
    };
    Scratch &scratch_for(DevStream s) {
        std::lock_guard l(scratch_mtx_);
        auto it = scratch_.find(s);
        if (it != scratch_.end()) return it->second;
        Scratch sc;
        (void)hipMalloc(&sc.dev, 2 * 1024 * sizeof(double));
        (void)hipHostMalloc(&sc.host, 16 * sizeof(double), hipHostMallocMapped);
        return scratch_[s] = sc;
    }

    int n_devices_ = 0;
    std::mutex peer_mtx_;
    std::set<std::pair<int, int>> peer_enabled_;
    std::mutex scratch_mtx_;
    std::map<DevStream, Scratch> scratch_;
    std::map<int, void *> crc_tables_; // per device, uploaded on first use
};

} // namespace
} // namespace pccl

extern "C" __attribute__((visibility("default"))) pccl::DeviceBackend *pccl_create_hip_backend() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return nullptr;
    }
    return new pccl::HipBackend();
}
