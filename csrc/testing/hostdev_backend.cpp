// Host-emulated device backend (libpccl_hostdev.so): the DeviceBackend interface on host memory, loaded instead of
// the HIP plugin with PCCL_HIP_PLUGIN=<path>/libpccl_hostdev.so. It exists for CPU-only testing of the library's
// device paths - the stream-ordered start path, the device ring pipeline, abort drains - under ThreadSanitizer, where
// neither a GPU nor the HIP runtime is available.
//
// Semantics follow a GPU's: every stream is a worker thread executing its queued work in order, asynchronously to
// the submitting thread; an event is complete once its stream reached it (a re-record makes it pending again);
// stream_wait_event makes a stream wait for an event of another stream; the null stream (nullptr) is one process-wide
// stream. Device memory is host memory: allocations of this backend are "device" pointers, and with
// PCCL_HOSTDEV_ALL_DEVICE=1 every pointer is (a test's own buffers then take the device paths). Copies and the
// reduce, quantize and de-quantize kernels run on the stream's thread with the host kernels (bit-identical to the HIP
// kernels). The xGMI / IPC and VMM entry points report failure, so the library uses the TCP rings.
//
// Extra entry points for tests (dlsym): pccl_hostdev_fill(stream, ptr, n_floats, value, delay_us) queues a "producer
// kernel" that sleeps delay_us, then writes `value` into n fp32 elements - input the stream-ordered ops must wait for;
// pccl_hostdev_create_stream() makes a stream.
#include <cstdlib>
#include <cstring>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>

#include "../common/device_backend.hpp"
#include "../kernels/host_kernels.hpp"

namespace {

using namespace pccl;

struct Event {
    std::mutex m;
    std::condition_variable cv;
    uint64_t recorded = 0; // generation of the latest record
    uint64_t reached = 0;  // generation its stream has reached
};

class Stream {
public:
    Stream() : th_([this] { loop(); }) {}
    ~Stream() {
        {
            std::lock_guard l(m_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void push(std::function<void()> fn) {
        {
            std::lock_guard l(m_);
            q_.push_back(std::move(fn));
            ++queued_;
        }
        cv_.notify_all();
    }
    void sync() {
        std::unique_lock l(m_);
        const uint64_t target = queued_;
        done_cv_.wait(l, [&] { return done_ >= target; });
    }

private:
    void loop() {
        std::unique_lock l(m_);
        while (true) {
            cv_.wait(l, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) return;
            auto fn = std::move(q_.front());
            q_.pop_front();
            l.unlock();
            fn();
            l.lock();
            ++done_;
            done_cv_.notify_all();
        }
    }
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::deque<std::function<void()>> q_;
    uint64_t queued_ = 0, done_ = 0;
    bool stop_ = false;
    std::thread th_;
};

class HostDevBackend final : public DeviceBackend {
public:
    HostDevBackend() : all_device_(std::getenv("PCCL_HOSTDEV_ALL_DEVICE") != nullptr) {}
    ~HostDevBackend() override { delete null_stream_.exchange(nullptr); }

    Stream *stream_of(DevStream s) {
        if (s) return static_cast<Stream *>(s);
        Stream *n = null_stream_.load();
        if (n) return n;
        auto *fresh = new Stream();
        if (null_stream_.compare_exchange_strong(n, fresh)) return fresh;
        delete fresh;
        return n;
    }

    int device_count() override { return 1; }
    bool pointer_info(const void *p, DevPtrInfo &out) override {
        out = DevPtrInfo{};
        if (p == nullptr) return true;
        if (all_device_ || owned(p)) {
            out.is_device = true;
            out.device = 0;
        }
        return true;
    }
    bool set_device(int dev) override { return dev == 0; }
    int current_device() override { return 0; }
    uint64_t device_uid(int) override { return 0x484f535444455631ull; } // "HOSTDEV1"
    int device_of_uid(uint64_t uid) override { return uid == device_uid(0) ? 0 : -1; }
    bool can_access_peer(int, int) override { return true; }
    bool enable_peer_access(int, int) override { return true; }

    void *alloc_device(size_t n) override {
        void *p = std::aligned_alloc(256, (std::max<size_t>(n, 1) + 255) / 256 * 256);
        if (p) {
            std::lock_guard l(alloc_m_);
            allocs_[reinterpret_cast<uintptr_t>(p)] = n;
        }
        return p;
    }
    void free_device(void *p) override {
        if (!p) return;
        {
            std::lock_guard l(alloc_m_);
            allocs_.erase(reinterpret_cast<uintptr_t>(p));
        }
        std::free(p);
    }
    void *alloc_pinned(size_t n) override { return std::aligned_alloc(4096, (std::max<size_t>(n, 1) + 4095) / 4096 * 4096); }
    void free_pinned(void *p) override { std::free(p); }
    bool ipc_export(void *, uint8_t *) override { return false; }
    void *ipc_open(const uint8_t *) override { return nullptr; }
    void ipc_close(void *) override {}
    void *vmm_alloc(size_t, int, int *, size_t *) override { return nullptr; }
    void vmm_free(void *) override {}
    void *vmm_import(int, size_t, int) override { return nullptr; }
    void vmm_unmap(void *) override {}
    bool address_range(const void *p, void **base, size_t *size) override {
        std::lock_guard l(alloc_m_);
        auto it = allocs_.upper_bound(reinterpret_cast<uintptr_t>(p));
        if (it == allocs_.begin()) return false;
        --it;
        if (reinterpret_cast<uintptr_t>(p) >= it->first + it->second) return false;
        *base = reinterpret_cast<void *>(it->first);
        *size = it->second;
        return true;
    }

    DevStream create_stream() override { return new Stream(); }
    void destroy_stream(DevStream s) override { delete static_cast<Stream *>(s); }
    bool stream_sync(DevStream s) override {
        stream_of(s)->sync();
        return true;
    }
    DevEvent create_event() override { return new Event(); }
    void destroy_event(DevEvent e) override { delete static_cast<Event *>(e); }
    bool event_record(DevEvent e, DevStream s) override {
        auto *ev = static_cast<Event *>(e);
        uint64_t gen;
        {
            std::lock_guard l(ev->m);
            gen = ++ev->recorded;
        }
        stream_of(s)->push([ev, gen] {
            {
                std::lock_guard l(ev->m);
                ev->reached = std::max(ev->reached, gen);
            }
            ev->cv.notify_all();
        });
        return true;
    }
    int event_query(DevEvent e) override {
        auto *ev = static_cast<Event *>(e);
        std::lock_guard l(ev->m);
        return ev->reached >= ev->recorded ? 1 : 0;
    }
    bool event_sync(DevEvent e) override {
        auto *ev = static_cast<Event *>(e);
        std::unique_lock l(ev->m);
        ev->cv.wait(l, [&] { return ev->reached >= ev->recorded; });
        return true;
    }
    bool stream_wait_event(DevStream s, DevEvent e) override {
        auto *ev = static_cast<Event *>(e);
        uint64_t gen;
        {
            std::lock_guard l(ev->m);
            gen = ev->recorded; // the record this wait refers to (a later re-record does not move it)
        }
        stream_of(s)->push([ev, gen] {
            std::unique_lock l(ev->m);
            ev->cv.wait(l, [&] { return ev->reached >= gen; });
        });
        return true;
    }
    bool memcpy_async(void *dst, const void *src, size_t n, DevStream s) override {
        stream_of(s)->push([dst, src, n] { std::memmove(dst, src, n); });
        return true;
    }
    bool memcpy_sync(void *dst, const void *src, size_t n) override {
        std::memmove(dst, src, n);
        return true;
    }
    bool copy_kernel(void *dst, const void *src, size_t n, int, DevStream s) override { return memcpy_async(dst, src, n, s); }
    bool device_sync() override {
        stream_of(nullptr)->sync();
        return true;
    }

    bool reduce(void *dst, const void *src, size_t count, DType t, ReduceOp op, DevStream s) override {
        stream_of(s)->push([=] { kernels::host_reduce(dst, src, count, t, op); });
        return true;
    }
    bool reduce_copy(void *dst, const void *src, void *out, size_t count, DType t, ReduceOp op, DevStream s) override {
        stream_of(s)->push([=] {
            kernels::host_reduce(dst, src, count, t, op);
            std::memcpy(out, dst, count * dtype_size(t));
        });
        return true;
    }
    bool finalize_avg(void *dst, size_t count, DType t, size_t world, DevStream s) override {
        stream_of(s)->push([=] { kernels::host_finalize_avg(dst, count, t, world); });
        return true;
    }
    // quantized paths: the host twins of the device kernels (bit-identical), run on the stream's thread
    bool dequant_reduce(void *dst, const void *src_q, size_t n, DType vt, DType qt, ReduceOp op,
                        const kernels::QuantParams &p, DevStream s) override {
        stream_of(s)->push([=] { kernels::host_dequant_reduce_params(dst, src_q, n, vt, qt, op, p); });
        return true;
    }
    // one (min, max) partial of the values stored (the device kernels emit one per workgroup)
    bool dequant_reduce_minmax(void *dst, const void *src_q, size_t n, DType vt, DType qt, ReduceOp op,
                               const kernels::QuantParams &p, double *partials, int max_blocks, int *blocks,
                               DevStream s) override {
        if (max_blocks < 1) return false;
        *blocks = 1;
        stream_of(s)->push([=] {
            kernels::host_dequant_reduce_params(dst, src_q, n, vt, qt, op, p);
            kernels::host_minmax(dst, n, vt, partials[0], partials[1]);
        });
        return true;
    }
    bool quantize(void *dst_q, const void *src, size_t n, DType vt, DType qt, const kernels::QuantParams &p,
                  DevStream s) override {
        stream_of(s)->push([=] { kernels::host_quantize_params(dst_q, src, n, vt, qt, p); });
        return true;
    }
    // own chunk := D(Q(x)) (what every other peer de-quantizes)
    bool quantize_setback(void *dst_q, void *src, size_t n, DType vt, DType qt, const kernels::QuantParams &p,
                          DevStream s) override {
        stream_of(s)->push([=] {
            kernels::host_quantize_params(dst_q, src, n, vt, qt, p);
            kernels::host_dequant_reduce_params(src, dst_q, n, vt, qt, ReduceOp::Set, p);
        });
        return true;
    }
    bool minmax(const void *src, size_t n, DType vt, double *out2, DevStream s) override {
        stream_of(s)->push([=] {
            kernels::host_minmax(src, n, vt, out2[0], out2[1]);
            if (n == 0) out2[0] = out2[1] = 0.0;
        });
        return true;
    }
    bool minmax_fold(const double *partials, int nparts, size_t n, double *out2, DevStream s) override {
        stream_of(s)->push([=] {
            double lo = __builtin_inf(), hi = -__builtin_inf();
            for (int i = 0; i < nparts; ++i) {
                lo = partials[2 * i] < lo ? partials[2 * i] : lo;
                hi = partials[2 * i + 1] > hi ? partials[2 * i + 1] : hi;
            }
            out2[0] = n ? lo : 0.0;
            out2[1] = n ? hi : 0.0;
        });
        return true;
    }
    bool multi_reduce(void *const *, int, const void *const *, int, size_t, DType, ReduceOp, DevStream, int,
                      bool) override {
        return false;
    }
    bool multi_gather(void *, const void *const *, const size_t *, const size_t *, int, int, DType, DevStream,
                      bool) override {
        return false;
    }
    uint32_t simplehash(const void *p, size_t n, DevStream s) override {
        stream_of(s)->sync();
        return kernels::simplehash_host(p, n);
    }
    bool simplehash_async(const void *p, size_t n, uint32_t *out, DevStream s) override {
        stream_of(s)->push([=] { *out = kernels::simplehash_host(p, n); });
        return true;
    }
    bool crc32c_tiles(const void *, size_t, const uint32_t *, const uint32_t *, uint32_t *, size_t, size_t &, size_t &,
                      DevStream) override {
        return false;
    }
    bool fill_test_pattern(void *, size_t, DevStream) override { return false; }
    bool pseudo_grad(float *, const float *, const void *, size_t, DType, DevStream) override { return false; }
    bool outer_sgd(float *, float *, const float *, void *, size_t, DType, const kernels::OuterSgdParams &,
                   DevStream) override {
        return false;
    }

    void fill(DevStream s, float *p, size_t n, float v, unsigned delay_us) {
        stream_of(s)->push([=] {
            if (delay_us) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
            for (size_t i = 0; i < n; ++i) p[i] = v;
        });
    }

private:
    bool owned(const void *p) {
        void *b;
        size_t n;
        return address_range(p, &b, &n);
    }
    const bool all_device_;
    std::atomic<Stream *> null_stream_{nullptr};
    std::mutex alloc_m_;
    std::map<uintptr_t, size_t> allocs_;
};

HostDevBackend *g_backend = nullptr;

} // namespace

extern "C" __attribute__((visibility("default"))) pccl::DeviceBackend *pccl_create_hip_backend() {
    static HostDevBackend *b = (g_backend = new HostDevBackend());
    return b;
}

// (the instance the library gets: a test may call these before the library first asked for its backend)
extern "C" __attribute__((visibility("default"))) void pccl_hostdev_fill(void *stream, float *p, size_t n, float v,
                                                                         unsigned delay_us) {
    pccl_create_hip_backend();
    g_backend->fill(stream, p, n, v, delay_us);
}

extern "C" __attribute__((visibility("default"))) void *pccl_hostdev_create_stream() {
    pccl_create_hip_backend();
    return g_backend->create_stream();
}
