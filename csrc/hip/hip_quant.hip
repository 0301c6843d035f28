// Quantize / fused dequantize+reduce / min-max kernels (launchers).
#include <algorithm>

#include "dispatch.hpp"
#include "launchers.hpp"

namespace pccl::hipk {

bool launch_dequant_reduce(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                           const kernels::QuantParams &p, hipStream_t st) {
    if (count == 0) return true;
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

bool launch_quantize(void *dst_q, const void *src, size_t count, DType vtype, DType qtype,
                     const kernels::QuantParams &p, hipStream_t st) {
    if (count == 0) return true;
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

bool launch_minmax(const void *src, size_t count, DType vtype, double *partial, double *out2, hipStream_t st) {
    const int grid = std::min(grid_for(count), 1024);
    return with_float_elem(vtype, [&](auto e) {
        using E = decltype(e);
        return launch_ok([&] {
            k_minmax_partial<E><<<grid, kBlock, 0, st>>>(static_cast<const typename E::S *>(src), count, partial);
            k_minmax_final<><<<1, kBlock, 0, st>>>(partial, grid, count, out2);
        });
    });
}

} // namespace pccl::hipk
