// HIP implementation of pccl::DeviceBackend (built as libpccl_hip.so for gfx950, loaded by libpccl.so via dlopen).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "../common/device_backend.hpp"
#include "kernels.hpp"

namespace pccl {
namespace {

using namespace hipk;

#define HIP_OK(expr) (hipSuccess == (expr))

template<typename F>
bool launch_ok(F &&f) {
    f();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        std::fprintf(stderr, "[pccl_hip] kernel launch failed: %s\n", hipGetErrorString(e));
        return false;
    }
    return true;
}

// dtype dispatch -> element codec
template<typename F>
bool with_elem(DType t, F &&f) {
    switch (t) {
        case DType::F32: return f(EF32{});
        case DType::F64: return f(EF64{});
        case DType::BF16: return f(EBF16{});
        case DType::F16: return f(EF16{});
        case DType::U8: return f(EInt<uint8_t>{});
        case DType::I8: return f(EInt<int8_t>{});
        case DType::U16: return f(EInt<uint16_t>{});
        case DType::I16: return f(EInt<int16_t>{});
        case DType::U32: return f(EInt<uint32_t>{});
        case DType::I32: return f(EInt<int32_t>{});
        case DType::U64: return f(EInt<uint64_t>{});
        case DType::I64: return f(EInt<int64_t>{});
        default: return false;
    }
}

template<typename F>
bool with_float_elem(DType t, F &&f) {
    switch (t) {
        case DType::F32: return f(EF32{});
        case DType::F64: return f(EF64{});
        case DType::BF16: return f(EBF16{});
        case DType::F16: return f(EF16{});
        default: return false;
    }
}

template<typename F>
bool with_op(ReduceOp op, F &&f) {
    switch (op) {
        case ReduceOp::Set: return f(OpSet{});
        case ReduceOp::Sum:
        case ReduceOp::Avg: return f(OpSum{});
        case ReduceOp::Prod: return f(OpProd{});
        case ReduceOp::Max: return f(OpMax{});
        case ReduceOp::Min: return f(OpMin{});
    }
    return false;
}

template<typename F>
bool with_qint(DType q, F &&f) {
    switch (q) {
        case DType::U8: return f(uint8_t{});
        case DType::I8: return f(int8_t{});
        case DType::U16: return f(uint16_t{});
        case DType::I16: return f(int16_t{});
        case DType::U32: return f(uint32_t{});
        case DType::I32: return f(int32_t{});
        case DType::U64: return f(uint64_t{});
        case DType::I64: return f(int64_t{});
        default: return false;
    }
}

class HipBackend final : public DeviceBackend {
public:
    HipBackend() { hipGetDeviceCount(&n_devices_); }

    int device_count() override { return n_devices_; }

    bool pointer_info(const void *p, DevPtrInfo &out) override {
        out = DevPtrInfo{};
        if (p == nullptr || n_devices_ == 0) return true;
        hipPointerAttribute_t attr{};
        const hipError_t e = hipPointerGetAttributes(&attr, p);
        if (e != hipSuccess) {
            (void)hipGetLastError(); // unregistered host memory: clear sticky error
            return true;
        }
        if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) {
            out.is_device = true;
            out.device = attr.device;
        }
        return true;
    }

    bool set_device(int dev) override { return HIP_OK(hipSetDevice(dev)); }
    int current_device() override {
        int d = -1;
        hipGetDevice(&d);
        return d;
    }

    void *alloc_device(size_t n) override {
        void *p = nullptr;
        if (!HIP_OK(hipMalloc(&p, n ? n : 1))) return nullptr;
        return p;
    }
    void free_device(void *p) override {
        if (p) hipFree(p);
    }
    void *alloc_pinned(size_t n) override {
        void *p = nullptr;
        if (!HIP_OK(hipHostMalloc(&p, n ? n : 1, hipHostMallocPortable | hipHostMallocMapped))) return nullptr;
        return p;
    }
    void free_pinned(void *p) override {
        if (p) hipHostFree(p);
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
        if (mapped) hipIpcCloseMemHandle(mapped);
    }

    DevStream create_stream() override {
        hipStream_t s = nullptr;
        if (!HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking))) return nullptr;
        return s;
    }
    void destroy_stream(DevStream s) override {
        if (s) {
            std::lock_guard l(scratch_mtx_);
            auto it = scratch_.find(s);
            if (it != scratch_.end()) {
                hipFree(it->second.dev);
                hipHostFree(it->second.host);
                scratch_.erase(it);
            }
            hipStreamDestroy(static_cast<hipStream_t>(s));
        }
    }
    bool stream_sync(DevStream s) override { return HIP_OK(hipStreamSynchronize(static_cast<hipStream_t>(s))); }
    DevEvent create_event() override {
        hipEvent_t e = nullptr;
        if (!HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming))) return nullptr;
        return e;
    }
    void destroy_event(DevEvent e) override {
        if (e) hipEventDestroy(static_cast<hipEvent_t>(e));
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
    bool memcpy_async(void *dst, const void *src, size_t n, DevStream s) override {
        if (n == 0) return true;
        return HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDefault, static_cast<hipStream_t>(s)));
    }
    bool memcpy_sync(void *dst, const void *src, size_t n) override {
        if (n == 0) return true;
        return HIP_OK(hipMemcpy(dst, src, n, hipMemcpyDefault));
    }
    bool device_sync() override { return HIP_OK(hipDeviceSynchronize()); }

    // ------------------------------------------------------------------ ring-path kernels
    bool reduce(void *dst, const void *src, size_t count, DType t, ReduceOp op, DevStream s) override {
        if (count == 0) return true;
        auto st = static_cast<hipStream_t>(s);
        if (op == ReduceOp::Set) return memcpy_async(dst, src, count * dtype_size(t), s);
        return with_elem(t, [&](auto e) {
            using E = decltype(e);
            return with_op(op, [&](auto o) {
                using O = decltype(o);
                return launch_ok([&] {
                    k_reduce<E, O><<<grid_for(count), kBlock, 0, st>>>(static_cast<typename E::S *>(dst),
                                                                       static_cast<const typename E::S *>(src), count);
                });
            });
        });
    }

    bool dequant_reduce(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                        const kernels::QuantParams &p, DevStream s) override {
        if (count == 0) return true;
        auto st = static_cast<hipStream_t>(s);
        const int grid = grid_for(count);
        return with_float_elem(vtype, [&](auto e) {
            using E = decltype(e);
            using S = typename E::S;
            return with_op(op, [&](auto o) {
                using O = decltype(o);
                if (p.algo == QuantAlgo::MinMax && qtype == DType::F8E4M3)
                    return launch_ok([&] {
                        k_dq_fp8<E, O, true><<<grid, kBlock, 0, st>>>(static_cast<S *>(dst), static_cast<const uint8_t *>(src_q), count, p);
                    });
                if (p.algo == QuantAlgo::MinMax && qtype == DType::F8E5M2)
                    return launch_ok([&] {
                        k_dq_fp8<E, O, false><<<grid, kBlock, 0, st>>>(static_cast<S *>(dst), static_cast<const uint8_t *>(src_q), count, p);
                    });
                return with_qint(qtype, [&](auto qv) {
                    using Q = decltype(qv);
                    if (p.algo == QuantAlgo::MinMax)
                        return launch_ok([&] {
                            k_dq_minmax<E, O, Q><<<grid, kBlock, 0, st>>>(static_cast<S *>(dst), static_cast<const Q *>(src_q), count, p);
                        });
                    if constexpr (sizeof(Q) <= 4) {
                        if (p.algo == QuantAlgo::ZeroPointScale)
                            return launch_ok([&] {
                                k_dq_zps<E, O, Q><<<grid, kBlock, 0, st>>>(static_cast<S *>(dst), static_cast<const Q *>(src_q), count, p);
                            });
                    }
                    return false;
                });
            });
        });
    }

    bool quantize(void *dst_q, const void *src, size_t count, DType vtype, DType qtype, const kernels::QuantParams &p,
                  DevStream s) override {
        if (count == 0) return true;
        auto st = static_cast<hipStream_t>(s);
        const int grid = grid_for(count);
        return with_float_elem(vtype, [&](auto e) {
            using E = decltype(e);
            using S = typename E::S;
            if (p.algo == QuantAlgo::MinMax && qtype == DType::F8E4M3)
                return launch_ok([&] { k_q_fp8<E, true><<<grid, kBlock, 0, st>>>(static_cast<uint8_t *>(dst_q), static_cast<const S *>(src), count, p); });
            if (p.algo == QuantAlgo::MinMax && qtype == DType::F8E5M2)
                return launch_ok([&] { k_q_fp8<E, false><<<grid, kBlock, 0, st>>>(static_cast<uint8_t *>(dst_q), static_cast<const S *>(src), count, p); });
            return with_qint(qtype, [&](auto qv) {
                using Q = decltype(qv);
                if (p.algo == QuantAlgo::MinMax)
                    return launch_ok([&] { k_q_minmax<E, Q><<<grid, kBlock, 0, st>>>(static_cast<Q *>(dst_q), static_cast<const S *>(src), count, p); });
                if constexpr (sizeof(Q) <= 4) {
                    if (p.algo == QuantAlgo::ZeroPointScale)
                        return launch_ok([&] { k_q_zps<E, Q><<<grid, kBlock, 0, st>>>(static_cast<Q *>(dst_q), static_cast<const S *>(src), count, p); });
                }
                return false;
            });
        });
    }

    bool minmax(const void *src, size_t count, DType vtype, double *out2, DevStream s) override {
        auto st = static_cast<hipStream_t>(s);
        Scratch &sc = scratch_for(s);
        const int grid = std::min(grid_for(count), 1024);
        return with_float_elem(vtype, [&](auto e) {
            using E = decltype(e);
            return launch_ok([&] {
                k_minmax_partial<E><<<grid, kBlock, 0, st>>>(static_cast<const typename E::S *>(src), count, sc.dev);
                k_minmax_final<<<1, kBlock, 0, st>>>(sc.dev, grid, count, out2);
            });
        });
    }

    bool finalize_avg(void *dst, size_t count, DType t, size_t ws, DevStream s) override {
        if (count == 0) return true;
        auto st = static_cast<hipStream_t>(s);
        return with_elem(t, [&](auto e) {
            using E = decltype(e);
            return launch_ok([&] { k_avg<E><<<grid_for(count), kBlock, 0, st>>>(static_cast<typename E::S *>(dst), count, ws); });
        });
    }

    // ------------------------------------------------------------------ xGMI kernels
    bool multi_reduce(void *dst0, void *dst1, const void *const *srcs, int n, size_t count, DType t, ReduceOp op,
                      DevStream s) override {
        if (count == 0) return true;
        if (n < 1 || n > kMaxSrc) return false;
        auto st = static_cast<hipStream_t>(s);
        SrcList sl{};
        uintptr_t align_or = reinterpret_cast<uintptr_t>(dst0) | reinterpret_cast<uintptr_t>(dst1);
        for (int k = 0; k < n; ++k) {
            sl.p[k] = srcs[k];
            align_or |= reinterpret_cast<uintptr_t>(srcs[k]);
        }
        const bool avg = op == ReduceOp::Avg;
        return with_elem(t, [&](auto e) {
            using E = decltype(e);
            using S = typename E::S;
            constexpr size_t V = 16 / sizeof(S);
            const bool vec_ok = (align_or & 15) == 0;
            const size_t nvec = vec_ok ? count / V : 0;
            return with_op(op == ReduceOp::Set ? ReduceOp::Sum : op, [&](auto o) {
                using O = decltype(o);
                bool ok = true;
                if (nvec > 0) {
                    const int grid = grid_for(nvec, 2);
                    auto go = [&](auto maxn_tag) {
                        constexpr int M = decltype(maxn_tag)::value;
                        return launch_ok([&] {
                            if (avg)
                                k_multi_reduce_vec<E, O, true, M><<<grid, kBlock, 0, st>>>(static_cast<S *>(dst0), static_cast<S *>(dst1), sl, n, nvec);
                            else
                                k_multi_reduce_vec<E, O, false, M><<<grid, kBlock, 0, st>>>(static_cast<S *>(dst0), static_cast<S *>(dst1), sl, n, nvec);
                        });
                    };
                    if (n <= 2) ok = go(std::integral_constant<int, 2>{});
                    else if (n <= 4) ok = go(std::integral_constant<int, 4>{});
                    else if (n <= 8) ok = go(std::integral_constant<int, 8>{});
                    else ok = go(std::integral_constant<int, 16>{});
                }
                const size_t begin = nvec * V;
                if (ok && begin < count) {
                    ok = launch_ok([&] {
                        if (avg)
                            k_multi_reduce_scalar<E, O, true><<<grid_for(count - begin), kBlock, 0, st>>>(static_cast<S *>(dst0), static_cast<S *>(dst1), sl, n, count, begin);
                        else
                            k_multi_reduce_scalar<E, O, false><<<grid_for(count - begin), kBlock, 0, st>>>(static_cast<S *>(dst0), static_cast<S *>(dst1), sl, n, count, begin);
                    });
                }
                return ok;
            });
        });
    }

    bool multi_gather(void *dst, const void *const *srcs, const size_t *offsets, const size_t *counts, int n, int skip,
                      DType t, DevStream s) override {
        if (n < 1 || n > kMaxSrc) return false;
        GatherList g{};
        size_t maxb = 0;
        const size_t es = dtype_size(t);
        for (int k = 0; k < n; ++k) {
            g.src[k] = srcs[k];
            g.off[k] = offsets[k] * es;
            g.bytes[k] = counts[k] * es;
            if (k != skip) maxb = std::max(maxb, g.bytes[k]);
        }
        if (maxb == 0) return true;
        const int gx = std::max(1, std::min(grid_for(maxb / 16 + 1, 4), 1024 / std::max(1, n - 1)));
        auto st = static_cast<hipStream_t>(s);
        return launch_ok([&] { k_multi_gather<<<dim3(gx, n), kBlock, 0, st>>>(static_cast<uint8_t *>(dst), g, n, skip); });
    }

    uint32_t simplehash(const void *dev_ptr, size_t n_bytes, DevStream s) override {
        if (n_bytes == 0) return 0;
        auto st = static_cast<hipStream_t>(s);
        Scratch &sc = scratch_for(s);
        const size_t n_words = n_bytes / 4;
        const size_t n_vec = n_words / 4;
        size_t grid = (n_vec + 255) / 256;
        if (grid > 960) grid = 960;
        auto *partial = reinterpret_cast<uint32_t *>(sc.dev);
        auto *out = reinterpret_cast<uint32_t *>(sc.host);
        if (grid > 0) {
            const size_t vpb = (n_vec + grid - 1) / grid;
            k_hash_big<<<static_cast<int>(grid), kBlock, 0, st>>>(static_cast<const uint4 *>(dev_ptr), partial, n_vec, vpb);
        }
        k_hash_final<<<1, kBlock, 0, st>>>(partial, static_cast<int>(grid), static_cast<const uint8_t *>(dev_ptr), n_bytes, out);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
            std::fprintf(stderr, "[pccl_hip] simplehash failed\n");
            return 0;
        }
        return out[0];
    }

    bool fill_test_pattern(void *dev_ptr, size_t n_u64, DevStream s) override {
        return launch_ok([&] { k_test_pattern<<<8, 256, 0, static_cast<hipStream_t>(s)>>>(static_cast<uint64_t *>(dev_ptr), n_u64); });
    }

private:
    struct Scratch {
        double *dev = nullptr;   // 2 * 1024 doubles (min/max partials) / 960 hash partials
        double *host = nullptr;  // pinned, 16 doubles
    };
    Scratch &scratch_for(DevStream s) {
        std::lock_guard l(scratch_mtx_);
        auto it = scratch_.find(s);
        if (it != scratch_.end()) return it->second;
        Scratch sc;
        hipMalloc(&sc.dev, 2 * 1024 * sizeof(double));
        hipHostMalloc(&sc.host, 16 * sizeof(double), hipHostMallocMapped);
        return scratch_[s] = sc;
    }

    int n_devices_ = 0;
    std::mutex scratch_mtx_;
    std::map<DevStream, Scratch> scratch_;
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
