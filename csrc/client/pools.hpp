// Reusable buffer pools (pinned host / device / plain host) so collectives never allocate on the hot path.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../common/device_backend.hpp"
#include "../common/types.hpp"

namespace pccl::client {

// Staging memory of the collectives. Requests up to kSlabMaxRequest are carved out of kSlabBytes slabs (one runtime
// allocation per slab, first-fit with coalescing, 4 KiB granules); larger ones are whole runtime allocations kept in a
// best-fit cache. Pinned allocations are expensive (hipHostMalloc pins every page; milliseconds per call, serialised
// across processes by the driver), so a burst of concurrent small ops - e.g. 64 quantized ops in flight, each leasing
// ~8 staging buffers per peer - would otherwise pay hundreds of allocations on its first pass and churn the cache
// afterwards. A failed runtime allocation releases the pool's idle memory (cached buffers, empty slabs) and retries
// once before the lease reports failure.
class BufferPool {
public:
    enum class Kind { Host, Pinned, Device };
    explicit BufferPool(Kind k) : kind_(k) {}
    ~BufferPool();

    struct Slab;
    struct Buf {
        void *p = nullptr;
        size_t cap = 0;
        int device = -1;
        Slab *slab = nullptr; // carved out of this slab (nullptr: a whole runtime allocation)
    };

    Buf get(size_t n, int device = -1);
    void put(const Buf &b);

    // Bytes leased out right now, the most ever leased out at once (since the last reset_peak) and cached free bytes
    // (pcclxPoolStats: what a peer's staging actually holds, e.g. pinned memory per device-ring op).
    size_t in_use() const { return in_use_.load(std::memory_order_relaxed); }
    size_t peak() const { return peak_.load(std::memory_order_relaxed); }
    size_t cached();
    void reset_peak() { peak_.store(in_use_.load()); }
    // fresh allocations from the runtime (cache misses, slabs included) and the time they took (microseconds)
    uint64_t allocs() const { return allocs_.load(std::memory_order_relaxed); }
    uint64_t alloc_us() const { return alloc_us_.load(std::memory_order_relaxed); }

    // A ring step's staging lease is its chunk plus a few bytes of vector-phase slack (ring_device.cpp: chunk + 64):
    // the request limit and the slab leave room for that, so four leases of an exactly 32 MiB chunk (8 peers x 256 MiB
    // fp32, config 3's ops) still share one slab instead of each becoming a whole pinned allocation.
    static constexpr size_t kGranule = 4096;
    static constexpr size_t kSlabMaxRequest = (32u << 20) + 16 * kGranule;
    static constexpr size_t kSlabBytes = 4 * kSlabMaxRequest;

    struct Slab {
        uint8_t *base = nullptr;
        size_t size = 0;
        int device = -1;
        size_t used = 0;
        std::map<size_t, size_t> free; // offset -> length of free extents (coalesced)
    };

private:
    void note_lease(size_t cap);
    void *runtime_alloc(size_t n, int device);
    void runtime_free(void *p, int device);
    Buf carve_locked(size_t n, int device);
    void trim_idle_locked(bool everything);

    // Whole buffers stay cached up to kMaxFree buffers and PCCL_POOL_MAX_FREE_MIB (default 32 GiB) per pool (idle
    // slabs count against the same budget), oldest released first. The cap must cover a whole op's working set: the
    // device ring holds 9 staging buffers per peer (8 threaded peers: ~9 GiB of pinned memory with 128 MiB segment
    // chunks), and a pool that trims below that frees and re-allocates pinned memory on every op.
    static constexpr size_t kMaxFree = 256;
    std::atomic<size_t> in_use_{0}, peak_{0};
    std::atomic<uint64_t> allocs_{0}, alloc_us_{0};
    Kind kind_;
    std::mutex mtx_;
    std::vector<Buf> free_;
    size_t free_bytes_ = 0;
    std::vector<std::unique_ptr<Slab>> slabs_;
};

// RAII lease of a pooled buffer.
class Lease {
public:
    Lease() = default;
    Lease(BufferPool &pool, size_t n, int device = -1) : pool_(&pool), buf_(pool.get(n, device)) {}
    ~Lease() {
        if (pool_) pool_->put(buf_);
    }
    Lease(const Lease &) = delete;
    Lease &operator=(const Lease &) = delete;
    Lease(Lease &&o) noexcept : pool_(o.pool_), buf_(o.buf_) { o.pool_ = nullptr; }
    Lease &operator=(Lease &&o) noexcept {
        if (this != &o) {
            if (pool_) pool_->put(buf_);
            pool_ = o.pool_;
            buf_ = o.buf_;
            o.pool_ = nullptr;
        }
        return *this;
    }
    uint8_t *data() const { return static_cast<uint8_t *>(buf_.p); }
    bool ok() const { return buf_.p != nullptr; }

private:
    BufferPool *pool_ = nullptr;
    BufferPool::Buf buf_{};
};

// Reusable HIP streams / events per device: creating and destroying them per collective costs 10s-100s of us
// (hipStreamDestroy synchronises), which is visible on every op of the latency-bound paths.
class StreamPool {
public:
    DevStream get(int device) {
        {
            std::lock_guard l(mtx_);
            auto &v = free_[device];
            if (!v.empty()) {
                DevStream s = v.back();
                v.pop_back();
                return s;
            }
        }
        DeviceBackend *be = device_backend();
        if (!be) return nullptr;
        be->set_device(device);
        return be->create_stream();
    }
    void put(int device, DevStream s) {
        if (!s) return;
        std::lock_guard l(mtx_);
        free_[device].push_back(s);
    }

private:
    std::mutex mtx_;
    std::map<int, std::vector<DevStream>> free_;
};

// Events are bound to the device current at their creation, and recording one on another device's stream is an
// error: the pool keeps one free list per device and hands out only events of the device asked for (default: the
// calling thread's current device).
class EventPool {
public:
    DevEvent get(int device = -1) {
        DeviceBackend *be = device_backend();
        if (!be) return nullptr;
        if (device < 0) device = be->current_device();
        {
            std::lock_guard l(mtx_);
            auto &f = free_[device];
            if (!f.empty()) {
                DevEvent e = f.back();
                f.pop_back();
                return e;
            }
        }
        const int cur = be->current_device();
        if (cur != device) be->set_device(device);
        DevEvent e = be->create_event();
        if (cur != device) be->set_device(cur);
        if (e) {
            std::lock_guard l(mtx_);
            device_of_[e] = device;
        }
        return e;
    }
    void put(DevEvent e) {
        if (!e) return;
        std::lock_guard l(mtx_);
        auto it = device_of_.find(e);
        free_[it != device_of_.end() ? it->second : 0].push_back(e);
    }
    void forget(DevEvent e) { // a destroyed event (its handle may be reused by the runtime)
        std::lock_guard l(mtx_);
        device_of_.erase(e);
    }

private:
    std::mutex mtx_;
    std::map<int, std::vector<DevEvent>> free_;
    std::map<DevEvent, int> device_of_;
};

StreamPool &stream_pool();
EventPool &event_pool();

// RAII stream lease (the stream is synchronised by its user before it is returned)
class StreamLease {
public:
    explicit StreamLease(int device) : device_(device), s_(stream_pool().get(device)) {}
    ~StreamLease() { stream_pool().put(device_, s_); }
    StreamLease(const StreamLease &) = delete;
    StreamLease &operator=(const StreamLease &) = delete;
    DevStream get() const { return s_; }

private:
    int device_;
    DevStream s_;
};

BufferPool &host_pool();
BufferPool &pinned_pool();
BufferPool &device_pool();

} // namespace pccl::client
