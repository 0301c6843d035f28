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

class BufferPool {
public:
    enum class Kind { Host, Pinned, Device };
    explicit BufferPool(Kind k) : kind_(k) {}
    ~BufferPool() {
        for (auto &b : free_) release(b);
    }

    struct Buf {
        void *p = nullptr;
        size_t cap = 0;
        int device = -1;
    };

    Buf get(size_t n, int device = -1) {
        Buf b = get_raw(n, device);
        if (b.p) note_lease(b.cap);
        return b;
    }

    // Bytes leased out right now, the most ever leased out at once (since the last reset_peak) and cached free bytes
    // (pcclxPoolStats: what a peer's staging actually holds, e.g. pinned memory per device-ring op).
    size_t in_use() const { return in_use_.load(std::memory_order_relaxed); }
    size_t peak() const { return peak_.load(std::memory_order_relaxed); }
    size_t cached() {
        std::lock_guard l(mtx_);
        return free_bytes_;
    }
    void reset_peak() { peak_.store(in_use_.load()); }

private:
    void note_lease(size_t cap) {
        const size_t now = in_use_.fetch_add(cap) + cap;
        size_t pk = peak_.load(std::memory_order_relaxed);
        while (now > pk && !peak_.compare_exchange_weak(pk, now)) {
        }
    }
    Buf get_raw(size_t n, int device) {
        {
            std::lock_guard l(mtx_);
            size_t best = SIZE_MAX;
            size_t bi = 0;
            for (size_t i = 0; i < free_.size(); ++i)
                if (free_[i].cap >= n && free_[i].device == device && free_[i].cap < best) {
                    best = free_[i].cap;
                    bi = i;
                }
            if (best != SIZE_MAX) {
                Buf b = free_[bi];
                free_.erase(free_.begin() + static_cast<long>(bi));
                free_bytes_ -= b.cap;
                return b;
            }
        }
        Buf b;
        b.cap = n < 4096 ? 4096 : n;
        b.device = device;
        switch (kind_) {
            case Kind::Host: b.p = std::aligned_alloc(4096, (b.cap + 4095) / 4096 * 4096); break;
            case Kind::Pinned: b.p = device_backend() ? device_backend()->alloc_pinned(b.cap) : nullptr; break;
            case Kind::Device: b.p = device_backend() ? device_backend()->alloc_device(b.cap) : nullptr; break;
        }
        if (b.p == nullptr) b.cap = 0;
        return b;
    }

public:
    // Returned buffers stay cached up to kMaxFree buffers and PCCL_POOL_MAX_FREE_MIB (default 32 GiB) per pool,
    // oldest released first. The cap must cover a whole op's working set: the device ring holds 9 staging buffers
    // per peer (8 threaded peers x 1 GiB: 6 GiB of pinned memory), and a pool that trims below that frees and
    // re-allocates pinned memory on every op (hipHostFree / hipHostMalloc of 128 MiB cost milliseconds each).
    void put(const Buf &b) {
        if (b.p == nullptr) return;
        in_use_.fetch_sub(b.cap);
        static const size_t max_bytes = env_size("PCCL_POOL_MAX_FREE_MIB", 32u << 10) << 20;
        std::lock_guard l(mtx_);
        free_.push_back(b);
        free_bytes_ += b.cap;
        while (free_.size() > 1 && (free_.size() > kMaxFree || free_bytes_ > max_bytes)) {
            free_bytes_ -= free_.front().cap;
            release(free_.front());
            free_.erase(free_.begin());
        }
    }

private:
    void release(const Buf &b) {
        if (!b.p) return;
        switch (kind_) {
            case Kind::Host: std::free(b.p); break;
            case Kind::Pinned:
                if (device_backend()) device_backend()->free_pinned(b.p);
                break;
            case Kind::Device:
                if (device_backend()) {
                    const int cur = device_backend()->current_device();
                    if (b.device >= 0) device_backend()->set_device(b.device);
                    device_backend()->free_device(b.p);
                    if (cur >= 0) device_backend()->set_device(cur);
                }
                break;
        }
    }
    static constexpr size_t kMaxFree = 256;
    std::atomic<size_t> in_use_{0}, peak_{0};
    Kind kind_;
    std::mutex mtx_;
    std::vector<Buf> free_;
    size_t free_bytes_ = 0;
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

class EventPool {
public:
    DevEvent get() {
        {
            std::lock_guard l(mtx_);
            if (!free_.empty()) {
                DevEvent e = free_.back();
                free_.pop_back();
                return e;
            }
        }
        DeviceBackend *be = device_backend();
        return be ? be->create_event() : nullptr;
    }
    void put(DevEvent e) {
        if (!e) return;
        std::lock_guard l(mtx_);
        free_.push_back(e);
    }

private:
    std::mutex mtx_;
    std::vector<DevEvent> free_;
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
