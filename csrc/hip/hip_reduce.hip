// Ring-path elementwise reduce + AVG finalization kernels (launchers).
#include <cstdlib>

#include "dispatch.hpp"
#include "launchers.hpp"

namespace pccl::hipk {

bool launch_reduce(void *dst, const void *src, size_t count, DType t, ReduceOp op, hipStream_t st) {
    if (count == 0) return true;
    if (op == ReduceOp::Set) return hipMemcpyAsync(dst, src, count * dtype_size(t), hipMemcpyDefault, st) == hipSuccess;
    return with_elem(t, [&](auto e) {
        using E = decltype(e);
        return with_op(op, [&](auto o) {
            using O = decltype(o);
            using S = typename E::S;
            constexpr int V = vec_width<S>();
            const EwPlan pl = plan_ew<V>(count, {{dst, sizeof(S)}, {src, sizeof(S)}});
            return launch_ok([&] {
                k_reduce<E, O><<<grid_ew(count, pl, V), kBlock, 0, st>>>(
                    static_cast<S *>(dst), static_cast<const S *>(src), count, pl.head, pl.vec);
            });
        });
    });
}

bool launch_reduce_copy(void *dst, const void *src, void *out, size_t count, DType t, ReduceOp op, hipStream_t st) {
    if (count == 0) return true;
    if (op == ReduceOp::Set) {
        return hipMemcpyAsync(dst, src, count * dtype_size(t), hipMemcpyDefault, st) == hipSuccess &&
               hipMemcpyAsync(out, src, count * dtype_size(t), hipMemcpyDefault, st) == hipSuccess;
    }
    return with_elem(t, [&](auto e) {
        using E = decltype(e);
        return with_op(op, [&](auto o) {
            using O = decltype(o);
            using S = typename E::S;
            constexpr int V = vec_width<S>();
            const EwPlan pl = plan_ew<V>(count, {{dst, sizeof(S)}, {src, sizeof(S)}, {out, sizeof(S)}});
            const int grid = grid_ew(count, pl, V);
            return launch_ok([&] {
                k_reduce_copy<E, O><<<grid, kBlock, 0, st>>>(
                    static_cast<S *>(dst), static_cast<const S *>(src), static_cast<S *>(out), count, pl.head, pl.vec);
            });
        });
    });
}

bool launch_copy_bytes(void *dst, const void *src, size_t n, int max_grid, hipStream_t st) {
    if (n == 0) return true;
    const EwPlan pl = plan_ew<16>(n, {{dst, 1}, {src, 1}});
    int grid = grid_ew(n, pl, 16);
    if (max_grid > 0) grid = std::min(grid, max_grid);
    return launch_ok([&] {
        k_copy_bytes<><<<grid, kBlock, 0, st>>>(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n,
                                              pl.head, pl.vec);
    });
}

bool launch_finalize_avg(void *dst, size_t count, DType t, size_t ws, hipStream_t st) {
    if (count == 0) return true;
    return with_elem(t, [&](auto e) {
        using E = decltype(e);
        using S = typename E::S;
        constexpr int V = vec_width<S>();
        const EwPlan pl = plan_ew<V>(count, {{dst, sizeof(S)}});
        return launch_ok([&] {
            k_avg<E><<<grid_ew(count, pl, V), kBlock, 0, st>>>(static_cast<S *>(dst), count, ws, pl.head, pl.vec);
        });
    });
}

} // namespace pccl::hipk
