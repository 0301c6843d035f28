// Staging buffer pools (pools.hpp): whole-buffer cache for large leases, slab sub-allocation for the rest.
#include "pools.hpp"

#include <algorithm>
#include <chrono>

namespace pccl::client {

namespace {
size_t round_up(size_t n, size_t g) { return (n + g - 1) / g * g; }
size_t max_free_bytes() {
    static const size_t v = env_size("PCCL_POOL_MAX_FREE_MIB", 32u << 10) << 20;
    return v;
}
} // namespace

BufferPool::~BufferPool() {
    for (auto &b : free_) runtime_free(b.p, b.device);
    for (auto &s : slabs_)
        if (s->used == 0) runtime_free(s->base, s->device); // (a lease still out at exit keeps its slab)
}

void BufferPool::note_lease(size_t cap) {
    const size_t now = in_use_.fetch_add(cap) + cap;
    size_t pk = peak_.load(std::memory_order_relaxed);
    while (now > pk && !peak_.compare_exchange_weak(pk, now)) {
    }
}

void *BufferPool::runtime_alloc(size_t n, int device) {
    const auto t0 = std::chrono::steady_clock::now();
    void *p = nullptr;
    DeviceBackend *be = device_backend();
    switch (kind_) {
        case Kind::Host: p = std::aligned_alloc(kGranule, round_up(n, kGranule)); break;
        case Kind::Pinned: p = be ? be->alloc_pinned(n) : nullptr; break;
        case Kind::Device:
            if (be) {
                const int cur = be->current_device();
                if (device >= 0 && device != cur) be->set_device(device);
                p = be->alloc_device(n);
                if (device >= 0 && device != cur && cur >= 0) be->set_device(cur);
            }
            break;
    }
    allocs_.fetch_add(1, std::memory_order_relaxed);
    alloc_us_.fetch_add(static_cast<uint64_t>(
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count()));
    return p;
}

void BufferPool::runtime_free(void *p, int device) {
    if (!p) return;
    DeviceBackend *be = device_backend();
    switch (kind_) {
        case Kind::Host: std::free(p); break;
        case Kind::Pinned:
            if (be) be->free_pinned(p);
            break;
        case Kind::Device:
            if (be) {
                const int cur = be->current_device();
                if (device >= 0) be->set_device(device);
                be->free_device(p);
                if (cur >= 0) be->set_device(cur);
            }
            break;
    }
}

size_t BufferPool::cached() {
    std::lock_guard l(mtx_);
    size_t idle = free_bytes_;
    for (auto &s : slabs_) idle += s->size - s->used;
    return idle;
}

// First fit over the slabs of `device` (lowest address extent that fits); nullptr buffer if none has room.
BufferPool::Buf BufferPool::carve_locked(size_t n, int device) {
    for (auto &s : slabs_) {
        if (s->device != device || s->size - s->used < n) continue;
        for (auto it = s->free.begin(); it != s->free.end(); ++it) {
            if (it->second < n) continue;
            const size_t off = it->first, len = it->second;
            s->free.erase(it);
            if (len > n) s->free.emplace(off + n, len - n);
            s->used += n;
            return Buf{s->base + off, n, device, s.get()};
        }
    }
    return Buf{};
}

// Releases idle memory: every cached whole buffer and every empty slab (`everything`), or what exceeds the cache
// budget: the oldest cached whole buffers (one is always kept), then empty slabs.
void BufferPool::trim_idle_locked(bool everything) {
    size_t idle_slabs = 0;
    for (auto &s : slabs_)
        if (s->used == 0) idle_slabs += s->size;
    const size_t budget = everything ? 0 : max_free_bytes();
    const size_t keep = everything ? 0 : 1;
    while (free_.size() > keep && (free_.size() > kMaxFree || free_bytes_ + idle_slabs > budget)) {
        free_bytes_ -= free_.front().cap;
        runtime_free(free_.front().p, free_.front().device);
        free_.erase(free_.begin());
    }
    for (size_t i = slabs_.size(); i-- > 0 && free_bytes_ + idle_slabs > budget;) {
        if (slabs_[i]->used != 0) continue;
        idle_slabs -= slabs_[i]->size;
        runtime_free(slabs_[i]->base, slabs_[i]->device);
        slabs_.erase(slabs_.begin() + static_cast<long>(i));
    }
}

// Runtime allocations happen outside the pool's lock (a 128 MiB hipHostMalloc takes tens of ms; other threads keep
// leasing and returning meanwhile); only a failed one trims the idle memory under the lock and retries.
BufferPool::Buf BufferPool::get(size_t n, int device) {
    n = round_up(std::max<size_t>(n, 1), kGranule);
    auto alloc_or_trim = [&](size_t bytes) {
        void *p = runtime_alloc(bytes, device);
        if (!p) {
            {
                std::lock_guard l(mtx_);
                trim_idle_locked(true);
            }
            p = runtime_alloc(bytes, device);
        }
        return p;
    };
    Buf b;
    if (n <= kSlabMaxRequest) {
        {
            std::lock_guard l(mtx_);
            b = carve_locked(n, device);
        }
        if (!b.p) {
            auto slab = std::make_unique<Slab>();
            slab->base = static_cast<uint8_t *>(alloc_or_trim(kSlabBytes));
            if (slab->base) {
                slab->size = kSlabBytes;
                slab->device = device;
                slab->free.emplace(0, kSlabBytes);
                std::lock_guard l(mtx_);
                slabs_.push_back(std::move(slab));
                b = carve_locked(n, device); // (another thread may have added a slab meanwhile: either fits)
            }
        }
    } else {
        {
            std::lock_guard l(mtx_);
            size_t best = SIZE_MAX, bi = 0;
            for (size_t i = 0; i < free_.size(); ++i)
                if (free_[i].cap >= n && free_[i].device == device && free_[i].cap < best) {
                    best = free_[i].cap;
                    bi = i;
                }
            if (best != SIZE_MAX) {
                b = free_[bi];
                free_.erase(free_.begin() + static_cast<long>(bi));
                free_bytes_ -= b.cap;
            }
        }
        if (!b.p) {
            b = Buf{alloc_or_trim(n), n, device, nullptr};
            if (!b.p) b = Buf{};
        }
    }
    if (b.p) note_lease(b.cap);
    return b;
}

void BufferPool::put(const Buf &b) {
    if (b.p == nullptr) return;
    in_use_.fetch_sub(b.cap);
    std::lock_guard l(mtx_);
    if (Slab *s = b.slab) {
        size_t off = static_cast<size_t>(static_cast<uint8_t *>(b.p) - s->base), len = b.cap;
        auto next = s->free.lower_bound(off);
        if (next != s->free.end() && off + len == next->first) { // merge with the following extent
            len += next->second;
            next = s->free.erase(next);
        }
        if (next != s->free.begin()) { // merge with the preceding extent
            auto prev = std::prev(next);
            if (prev->first + prev->second == off) {
                off = prev->first;
                len += prev->second;
                s->free.erase(prev);
            }
        }
        s->free.emplace(off, len);
        s->used -= b.cap;
        if (s->used == 0) trim_idle_locked(false);
        return;
    }
    free_.push_back(b);
    free_bytes_ += b.cap;
    trim_idle_locked(false);
}

BufferPool &host_pool() {
    static BufferPool p(BufferPool::Kind::Host);
    return p;
}
BufferPool &pinned_pool() {
    static BufferPool p(BufferPool::Kind::Pinned);
    return p;
}
BufferPool &device_pool() {
    static BufferPool p(BufferPool::Kind::Device);
    return p;
}

} // namespace pccl::client
