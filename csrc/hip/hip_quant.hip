// Quantize / fused dequantize+reduce / min-max kernels (launchers).
#include <algorithm>

#include "dispatch.hpp"
#include "launchers.hpp"

namespace pccl::hipk {

bool launch_dequant_reduce(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                           const kernels::QuantParams &p, hipStream_t st, double *mm, int mm_max_blocks,
                           int *mm_blocks) {
    if (mm_blocks) *mm_blocks = 0;
    if (count == 0) return true;
    // with `mm`, the grid is capped at mm_max_blocks workgroups (the tile loop strides over the rest), each writing
    // its (min, max) partial of the stored results to mm[2 * blockIdx.x ...]
    auto grid_of = [&](int g) {
        if (mm) g = std::max(1, std::min(g, mm_max_blocks));
        if (mm_blocks) *mm_blocks = mm ? g : 0;
        return g;
    };
    return with_float_elem(vtype, [&](auto e) {
        using E = decltype(e);
        using S = typename E::S;
        constexpr int V = vec_width<S>();
        return with_op(op, [&](auto o) {
            using O = decltype(o);
            if (p.algo == QuantAlgo::MinMax && (qtype == DType::F8E4M3 || qtype == DType::F8E5M2)) {
                const EwPlan pl = plan_ew<V>(count, {{dst, sizeof(S)}, {src_q, 1}});
                const int grid = grid_of(grid_ew(count, pl, V));
                auto *d = static_cast<S *>(dst);
                auto *q = static_cast<const uint8_t *>(src_q);
                return launch_ok([&] {
                    if (qtype == DType::F8E4M3) {
                        if (mm) k_dq_fp8<E, O, true, true><<<grid, kBlock, 0, st>>>(d, q, count, p, pl.head, pl.vec, mm);
                        else k_dq_fp8<E, O, true, false><<<grid, kBlock, 0, st>>>(d, q, count, p, pl.head, pl.vec, mm);
                    } else {
                        if (mm) k_dq_fp8<E, O, false, true><<<grid, kBlock, 0, st>>>(d, q, count, p, pl.head, pl.vec, mm);
                        else k_dq_fp8<E, O, false, false><<<grid, kBlock, 0, st>>>(d, q, count, p, pl.head, pl.vec, mm);
                    }
                });
            }
            return with_qint(qtype, [&](auto qv) {
                using Q = decltype(qv);
                const EwPlan pl = plan_ew<V>(count, {{dst, sizeof(S)}, {src_q, sizeof(Q)}});
                auto *d = static_cast<S *>(dst);
                auto *q = static_cast<const Q *>(src_q);
                if (p.algo == QuantAlgo::MinMax) {
                    const int grid = grid_of(grid_ew(count, pl, V));
                    return launch_ok([&] {
                        if (mm) k_dq_minmax<E, O, Q, true><<<grid, kBlock, 0, st>>>(d, q, count, p, pl.head, pl.vec, mm);
                        else k_dq_minmax<E, O, Q, false><<<grid, kBlock, 0, st>>>(d, q, count, p, pl.head, pl.vec, mm);
                    });
                }
                if (p.algo == QuantAlgo::ZeroPointScale) {
                    const int grid = grid_of(grid_for(count, pl.vec ? V : 1));
                    return launch_ok([&] {
                        if (mm) k_dq_zps<E, O, Q, true><<<grid, kBlock, 0, st>>>(d, q, count, p, pl.head, pl.vec, mm);
                        else k_dq_zps<E, O, Q, false><<<grid, kBlock, 0, st>>>(d, q, count, p, pl.head, pl.vec, mm);
                    });
                }
                return false;
            });
        });
    });
}

bool launch_quantize(void *dst_q, const void *src, size_t count, DType vtype, DType qtype,
                     const kernels::QuantParams &p, hipStream_t st, bool set_back) {
    if (count == 0) return true;
    return with_float_elem(vtype, [&](auto e) {
        using E = decltype(e);
        using S = typename E::S;
        constexpr int V = vec_width<S>();
        // (set_back: the kernels write D(Q(x)) back into src; otherwise src is only read)
        auto *s = static_cast<S *>(const_cast<void *>(src));
        auto go = [&](auto back_c) {
            constexpr bool B = decltype(back_c)::value;
            if (p.algo == QuantAlgo::MinMax && (qtype == DType::F8E4M3 || qtype == DType::F8E5M2)) {
                const EwPlan pl = plan_ew<V>(count, {{src, sizeof(S)}, {dst_q, 1}});
                const int grid = grid_ew(count, pl, V);
                auto *d = static_cast<uint8_t *>(dst_q);
                return launch_ok([&] {
                    if (qtype == DType::F8E4M3)
                        k_q_fp8<E, true, B><<<grid, kBlock, 0, st>>>(d, s, count, p, pl.head, pl.vec);
                    else
                        k_q_fp8<E, false, B><<<grid, kBlock, 0, st>>>(d, s, count, p, pl.head, pl.vec);
                });
            }
            return with_qint(qtype, [&](auto qv) {
                using Q = decltype(qv);
                const EwPlan pl = plan_ew<V>(count, {{src, sizeof(S)}, {dst_q, sizeof(Q)}});
                const int grid = grid_for(count, pl.vec ? V : 1);
                auto *d = static_cast<Q *>(dst_q);
                if (p.algo == QuantAlgo::MinMax)
                    return launch_ok([&] {
                        k_q_minmax<E, Q, B><<<grid_ew(count, pl, V), kBlock, 0, st>>>(d, s, count, p, pl.head, pl.vec);
                    });
                if (p.algo == QuantAlgo::ZeroPointScale)
                    return launch_ok([&] { k_q_zps<E, Q, B><<<grid, kBlock, 0, st>>>(d, s, count, p, pl.head, pl.vec); });
                return false;
            });
        };
        return set_back ? go(std::true_type{}) : go(std::false_type{});
    });
}

bool launch_minmax_fold(const double *partial, int nblocks, size_t count, double *out2, hipStream_t st) {
    return launch_ok([&] { k_minmax_final<><<<1, kBlock, 0, st>>>(partial, nblocks, count, out2); });
}

bool launch_minmax(const void *src, size_t count, DType vtype, double *partial, double *out2, hipStream_t st) {
    return with_float_elem(vtype, [&](auto e) {
        using E = decltype(e);
        using S = typename E::S;
        constexpr int V = vec_width<S>();
        const EwPlan pl = plan_ew<V>(count, {{src, sizeof(S)}});
        const int grid = std::min(grid_ew(count, pl, V), 1024); // <= 1024 partials (scratch size)
        return launch_ok([&] {
            k_minmax_partial<E><<<grid, kBlock, 0, st>>>(static_cast<const S *>(src), count, partial, pl.head, pl.vec);
            k_minmax_final<><<<1, kBlock, 0, st>>>(partial, grid, count, out2);
        });
    });
}

} // namespace pccl::hipk
