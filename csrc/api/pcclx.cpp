// [pccl-amd extension] Kernel-level entry points used by the test-suite and micro-benchmarks (not part of pccl.h).
// dtype arguments use the CCoIP wire encoding (pccl::DType), op uses pccl::ReduceOp, algo uses pccl::QuantAlgo.
#include <chrono>
#include <cstring>
#include <mutex>
#include <vector>

#include "../common/device_backend.hpp"
#include "../kernels/host_kernels.hpp"
#include "../kernels/optim_common.hpp"

using namespace pccl;

#define PCCLX_EXPORT extern "C" __attribute__((visibility("default")))

PCCLX_EXPORT int pcclxHipDeviceCount() {
    DeviceBackend *be = device_backend();
    return be ? be->device_count() : 0;
}

PCCLX_EXPORT uint32_t pcclxSimpleHash(const void *p, size_t n, int on_device) {
    if (!on_device) return kernels::simplehash_host(p, n);
    DeviceBackend *be = device_backend();
    if (!be) return 0;
    DevPtrInfo pi{};
    be->pointer_info(p, pi);
    if (pi.is_device) be->set_device(pi.device);
    return be->simplehash(p, n, nullptr);
}

// CRC-32C of host or device memory (device: HIP kernel, device_crc32c). force_sw selects the host table path.
PCCLX_EXPORT uint32_t pcclxCrc32c(const void *p, size_t n, int force_sw) {
    DeviceBackend *be = device_backend();
    DevPtrInfo pi{};
    if (be && n > 0) be->pointer_info(p, pi);
    if (pi.is_device) {
        be->set_device(pi.device);
        return device_crc32c(be, p, n, nullptr);
    }
    if (force_sw == 2 && kernels::crc32c_has_hw()) return kernels::crc32c_hw(p, n); // single-chain variant (tests)
    return force_sw ? kernels::crc32c_sw(p, n) : kernels::crc32c(p, n);
}

PCCLX_EXPORT int pcclxCrc32cHasHw() { return kernels::crc32c_has_hw() ? 1 : 0; }

PCCLX_EXPORT int pcclxFillTestPattern(void *dev, size_t n_u64) {
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    return be->fill_test_pattern(dev, n_u64, nullptr) && be->device_sync() ? 0 : -1;
}

PCCLX_EXPORT int pcclxReduce(void *dst, const void *src, size_t count, int dtype, int op, int on_device) {
    if (!on_device) return kernels::host_reduce(dst, src, count, static_cast<DType>(dtype), static_cast<ReduceOp>(op)) ? 0 : -1;
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    return be->reduce(dst, src, count, static_cast<DType>(dtype), static_cast<ReduceOp>(op), nullptr) && be->device_sync() ? 0 : -1;
}

PCCLX_EXPORT int pcclxFinalizeAvg(void *dst, size_t count, int dtype, size_t ws, int on_device) {
    if (!on_device) return kernels::host_finalize_avg(dst, count, static_cast<DType>(dtype), ws) ? 0 : -1;
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    return be->finalize_avg(dst, count, static_cast<DType>(dtype), ws, nullptr) && be->device_sync() ? 0 : -1;
}

// meta_out: {min, max, zero_point, scale}
PCCLX_EXPORT int pcclxQuantize(void *dst_q, const void *src, size_t count, int vtype, int qtype, int algo,
                               int on_device, double *meta_out) {
    const auto vt = static_cast<DType>(vtype), qt = static_cast<DType>(qtype);
    const auto al = static_cast<QuantAlgo>(algo);
    if (!kernels::quant_supported(vt, qt, al)) return -2;
    proto::QuantMeta m;
    if (!on_device) {
        m = kernels::host_quantize(dst_q, src, count, vt, qt, al);
    } else {
        DeviceBackend *be = device_backend();
        if (!be) return -1;
        // one process-wide pinned min/max slot: a hipHostMalloc/hipHostFree pair per call cost more than the kernels
        static std::mutex mm_mutex;
        static double *mm = nullptr;
        std::lock_guard<std::mutex> lk(mm_mutex);
        if (mm == nullptr && (mm = static_cast<double *>(be->alloc_pinned(16))) == nullptr) return -1;
        be->minmax(src, count, vt, mm, nullptr);
        if (!be->device_sync()) return -1;
        m = kernels::make_meta(al, vt, qt, mm[0], mm[1]);
        if (!be->quantize(dst_q, src, count, vt, qt, kernels::make_params(m, qt), nullptr) || !be->device_sync()) return -1;
    }
    if (meta_out) {
        meta_out[0] = m.min_value;
        meta_out[1] = m.max_value;
        meta_out[2] = static_cast<double>(m.zero_point);
        meta_out[3] = m.scale;
    }
    return 0;
}

// Device only: quantizes `src` (min / max from the data, like pcclxQuantize) and overwrites it with D(Q(src)) in the
// same kernel pass (the quantized device ring's owner parity step).
PCCLX_EXPORT int pcclxQuantizeSetback(void *dst_q, void *src, size_t count, int vtype, int qtype, int algo,
                                      double *meta_out) {
    const auto vt = static_cast<DType>(vtype), qt = static_cast<DType>(qtype);
    const auto al = static_cast<QuantAlgo>(algo);
    if (!kernels::quant_supported(vt, qt, al)) return -2;
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    double *mm = static_cast<double *>(be->alloc_pinned(16));
    if (!mm) return -1;
    be->minmax(src, count, vt, mm, nullptr);
    bool ok = be->device_sync();
    const proto::QuantMeta m = kernels::make_meta(al, vt, qt, mm[0], mm[1]);
    be->free_pinned(mm);
    ok = ok && be->quantize_setback(dst_q, src, count, vt, qt, kernels::make_params(m, qt), nullptr) &&
         be->device_sync();
    if (!ok) return -1;
    if (meta_out) {
        meta_out[0] = m.min_value;
        meta_out[1] = m.max_value;
        meta_out[2] = static_cast<double>(m.zero_point);
        meta_out[3] = m.scale;
    }
    return 0;
}

PCCLX_EXPORT int pcclxDequantReduce(void *dst, const void *src_q, size_t count, int vtype, int qtype, int algo, int op,
                                    const double *meta, int on_device) {
    proto::QuantMeta m;
    m.algo = static_cast<QuantAlgo>(algo);
    m.value_type = static_cast<DType>(vtype);
    m.min_value = meta[0];
    m.max_value = meta[1];
    m.zero_point = static_cast<int64_t>(meta[2]);
    m.scale = static_cast<float>(meta[3]);
    const auto vt = static_cast<DType>(vtype), qt = static_cast<DType>(qtype);
    if (!on_device) return kernels::host_dequant_reduce(dst, src_q, count, vt, qt, static_cast<ReduceOp>(op), m) ? 0 : -1;
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    return be->dequant_reduce(dst, src_q, count, vt, qt, static_cast<ReduceOp>(op), kernels::make_params(m, qt), nullptr) &&
                   be->device_sync()
               ? 0
               : -1;
}

// dequant_reduce on the device with the fused per-workgroup (min, max) of the stored results, split into `pieces`
// launches (as the ring's receive ranges are) and folded: minmax_out = {min, max} of dst after the reduce
PCCLX_EXPORT int pcclxDequantReduceMinmax(void *dst, const void *src_q, size_t count, int vtype, int qtype, int algo,
                                          int op, const double *meta, int pieces, double *minmax_out) {
    proto::QuantMeta m;
    m.algo = static_cast<QuantAlgo>(algo);
    m.value_type = static_cast<DType>(vtype);
    m.min_value = meta[0];
    m.max_value = meta[1];
    m.zero_point = static_cast<int64_t>(meta[2]);
    m.scale = static_cast<float>(meta[3]);
    const auto vt = static_cast<DType>(vtype), qt = static_cast<DType>(qtype);
    DeviceBackend *be = device_backend();
    if (!be || pieces < 1) return -1;
    constexpr int kSlots = 8192;
    double *partials = static_cast<double *>(be->alloc_device(kSlots * 2 * sizeof(double)));
    double *out = static_cast<double *>(be->alloc_pinned(16));
    bool ok = partials && out;
    int used = 0;
    const size_t es = dtype_size(vt), qs = dtype_size(qt);
    const auto params = kernels::make_params(m, qt);
    for (int k = 0; ok && k < pieces; ++k) {
        const size_t a = count * k / pieces, b = count * (k + 1) / pieces;
        int blocks = 0;
        ok = kSlots - used >= 1 &&
             be->dequant_reduce_minmax(static_cast<uint8_t *>(dst) + a * es, static_cast<const uint8_t *>(src_q) + a * qs,
                                       b - a, vt, qt, static_cast<ReduceOp>(op), params, partials + 2 * used,
                                       kSlots - used, &blocks, nullptr);
        used += blocks;
    }
    ok = ok && be->minmax_fold(partials, used, count, out, nullptr) && be->device_sync();
    if (ok) {
        minmax_out[0] = out[0];
        minmax_out[1] = out[1];
    }
    if (partials) be->free_device(partials);
    if (out) be->free_pinned(out);
    return ok ? 0 : -1;
}

PCCLX_EXPORT int pcclxMultiReduce(void *const *dsts, int ndst, const void *const *srcs, int n, size_t count, int dtype,
                                  int op) {
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    return be->multi_reduce(dsts, ndst, srcs, n, count, static_cast<DType>(dtype), static_cast<ReduceOp>(op), nullptr) &&
                   be->device_sync()
               ? 0
               : -1;
}

PCCLX_EXPORT int pcclxMultiGather(void *dst, const void *const *srcs, const size_t *offsets, const size_t *counts,
                                  int n, int skip, int dtype) {
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    return be->multi_gather(dst, srcs, offsets, counts, n, skip, static_cast<DType>(dtype), nullptr) && be->device_sync()
               ? 0
               : -1;
}

// Event-timed device kernel micro-benchmark: returns average microseconds per call of `which`
// (0 = reduce, 1 = simplehash, 2 = multi_reduce with `n` aliases of src, 3 = quantize u8 min-max, 4 = crc32c).
PCCLX_EXPORT double pcclxBenchKernel(int which, void *dst, const void *src, size_t count, int dtype, int n, int iters) {
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    DevStream st = be->create_stream();
    DevEvent e0 = be->create_event(), e1 = be->create_event();
    std::vector<const void *> srcs(static_cast<size_t>(n > 0 ? n : 1), src);
    kernels::QuantParams qp;
    proto::QuantMeta qm = kernels::make_meta(QuantAlgo::MinMax, static_cast<DType>(dtype), DType::U8, -1.0, 1.0);
    qp = kernels::make_params(qm, DType::U8);
    auto run = [&] {
        switch (which) {
            case 0: be->reduce(dst, src, count, static_cast<DType>(dtype), ReduceOp::Sum, st); break;
            case 1: be->simplehash(src, count * dtype_size(static_cast<DType>(dtype)), st); break;
            case 2: be->multi_reduce(&dst, 1, srcs.data(), n, count, static_cast<DType>(dtype), ReduceOp::Sum, st); break;
            case 3: be->quantize(dst, src, count, static_cast<DType>(dtype), DType::U8, qp, st); break;
            case 4: device_crc32c(be, src, count * dtype_size(static_cast<DType>(dtype)), st); break;
            default: break;
        }
    };
    run();
    be->stream_sync(st);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) run();
    be->stream_sync(st);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    be->destroy_event(e0);
    be->destroy_event(e1);
    be->destroy_stream(st);
    return us;
}

PCCLX_EXPORT int pcclxPseudoGrad(float *pg, const float *outer, const void *local, size_t count, int local_dtype,
                                 int on_device) {
    const auto lt = static_cast<DType>(local_dtype);
    if (!on_device) return kernels::host_pseudo_grad(pg, outer, local, count, lt) ? 0 : -1;
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    return be->pseudo_grad(pg, outer, local, count, lt, nullptr) && be->device_sync() ? 0 : -1;
}

PCCLX_EXPORT int pcclxOuterSgd(float *outer, float *mom, const float *pg, void *local, size_t count, int local_dtype,
                               float lr, float momentum, float dampening, float weight_decay, int nesterov, int first,
                               int on_device) {
    kernels::OuterSgdParams p;
    p.lr = lr;
    p.momentum = momentum;
    p.dampening = dampening;
    p.weight_decay = weight_decay;
    p.nesterov = nesterov;
    p.first = first;
    const auto lt = static_cast<DType>(local_dtype);
    if (!on_device) return kernels::host_outer_sgd(outer, mom, pg, local, count, lt, p) ? 0 : -1;
    DeviceBackend *be = device_backend();
    if (!be) return -1;
    return be->outer_sgd(outer, mom, pg, local, count, lt, p, nullptr) && be->device_sync() ? 0 : -1;
}
