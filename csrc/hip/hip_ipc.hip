// Intra-node xGMI kernels: multi-source reduce (reduce-scatter) and multi-source gather (all-gather) launchers.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "dispatch.hpp"
#include "launchers.hpp"

namespace pccl::hipk {

bool launch_multi_reduce(void *const *dsts, int ndst, const void *const *srcs, int n, size_t count, DType t,
                         ReduceOp op, hipStream_t st, int max_grid_hint, bool release) {
    if (count == 0) return true;
    if (n < 1 || n > kMaxSrc || ndst < 1 || ndst > kMaxSrc) return false;
    SrcList sl{};
    DstList dl{};
    uintptr_t align_or = 0;
    for (int k = 0; k < n; ++k) {
        sl.p[k] = srcs[k];
        align_or |= reinterpret_cast<uintptr_t>(srcs[k]);
    }
    for (int k = 0; k < ndst; ++k) {
        if (!dsts[k]) return false;
        dl.p[k] = dsts[k];
        align_or |= reinterpret_cast<uintptr_t>(dsts[k]);
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
                // 512 workgroups (2 per CU) and 2 vectors per thread measured best on MI355X for one kernel per GPU
                // (profiles/r1_ipc_grid_sweep.md); concurrent peers on one GPU pass a smaller budget.
                // Single destination (two-shot / hierarchical host-local reduce) uses k_multi_reduce_tile (contiguous
                // tile per workgroup, non-temporal loads, 4 vectors per thread): 8 srcs -> 1 dst 5000 -> 5586 GB/s.
                // The multi-destination push keeps the strided kernel (2 -> 2: 5420 vs 5080 GB/s tiled);
                // profiles/r1_ipc_tiled.md.
                const bool tiled = ndst == 1;
                const int unroll = tiled ? 4 : 2;
                const int max_grid = max_grid_hint > 0 ? max_grid_hint : 512;
                const int grid = std::max(1, std::min(grid_for(nvec, unroll), max_grid));
                ok = launch_ok([&] {
                    auto go = [&](auto avg_c, auto u_c) {
                        if (tiled)
                            k_multi_reduce_tile<E, O, decltype(avg_c)::value, decltype(u_c)::value>
                                <<<grid, kBlock, 0, st>>>(dl, ndst, sl, n, nvec, release ? 1 : 0);
                        else
                            k_multi_reduce_vec<E, O, decltype(avg_c)::value, decltype(u_c)::value>
                                <<<grid, kBlock, 0, st>>>(dl, ndst, sl, n, nvec, release ? 1 : 0);
                    };
                    using T2 = std::integral_constant<int, 2>;
                    using T4 = std::integral_constant<int, 4>;
                    if constexpr (std::is_same_v<O, OpSum>) {
                        if (avg) {
                            if (unroll == 4) go(std::true_type{}, T4{});
                            else go(std::true_type{}, T2{});
                            return;
                        }
                    }
                    if (unroll == 4) go(std::false_type{}, T4{});
                    else go(std::false_type{}, T2{});
                });
            }
            const size_t begin = nvec * V;
            if (ok && begin < count) {
                const int grid = grid_for(count - begin);
                ok = launch_ok([&] {
                    if constexpr (std::is_same_v<O, OpSum>) {
                        if (avg) {
                            k_multi_reduce_scalar<E, O, true><<<grid, kBlock, 0, st>>>(dl, ndst, sl, n, count, begin, release ? 1 : 0);
                            return;
                        }
                    }
                    k_multi_reduce_scalar<E, O, false><<<grid, kBlock, 0, st>>>(dl, ndst, sl, n, count, begin, release ? 1 : 0);
                });
            }
            return ok;
        });
    });
}

bool launch_multi_gather(void *dst, const void *const *srcs, const size_t *offsets, const size_t *counts, int n,
                         int skip, DType t, hipStream_t st, bool release) {
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
    return launch_ok([&] { k_multi_gather<><<<dim3(gx, n), kBlock, 0, st>>>(static_cast<uint8_t *>(dst), g, n, skip,
                                                                         release ? 1 : 0); });
}

} // namespace pccl::hipk
