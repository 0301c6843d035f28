// Ring-path elementwise reduce + AVG finalization kernels (launchers).
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
            return launch_ok([&] {
                k_reduce<E, O><<<grid_for(count), kBlock, 0, st>>>(static_cast<typename E::S *>(dst),
                                                                   static_cast<const typename E::S *>(src), count);
            });
        });
    });
}

bool launch_finalize_avg(void *dst, size_t count, DType t, size_t ws, hipStream_t st) {
    if (count == 0) return true;
    return with_elem(t, [&](auto e) {
        using E = decltype(e);
        return launch_ok([&] { k_avg<E><<<grid_for(count), kBlock, 0, st>>>(static_cast<typename E::S *>(dst), count, ws); });
    });
}

} // namespace pccl::hipk
