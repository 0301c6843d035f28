// Fused DiLoCo outer-step kernels (math in csrc/kernels/optim_common.hpp, shared with the host twin).
//
// Memory-bound elementwise work over the whole model: one pass reading outer/mom/pg (fp32) and writing
// outer/mom/local instead of the ~5 passes of the unfused torch update. 4 elements per thread per iteration with
// 16-byte fp32 vector accesses (local: 16 B for fp32, 8 B for 16-bit types); scalar tail for the remainder.
#include "dispatch.hpp"
#include "launchers.hpp"
#include "../kernels/optim_common.hpp"

namespace pccl::hipk {

template<typename E>
struct Local4; // 4 local elements as one vector access
template<>
struct Local4<EF32> {
    using V = float4;
};
template<>
struct Local4<EBF16> {
    using V = uint2;
};
template<>
struct Local4<EF16> {
    using V = uint2;
};

template<typename E>
__global__ __launch_bounds__(kBlock) void k_pseudo_grad(float *__restrict__ pg, const float *__restrict__ outer,
                                                        const typename E::S *__restrict__ local, size_t n4, size_t n) {
    using S = typename E::S;
    using V = typename Local4<E>::V;
    const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    const size_t tid = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
    for (size_t i = tid; i < n4; i += stride) {
        const float4 o = reinterpret_cast<const float4 *>(outer)[i];
        const V lv = reinterpret_cast<const V *>(local)[i];
        const S *l = reinterpret_cast<const S *>(&lv);
        float4 r;
        r.x = o.x - static_cast<float>(E::ld(l[0]));
        r.y = o.y - static_cast<float>(E::ld(l[1]));
        r.z = o.z - static_cast<float>(E::ld(l[2]));
        r.w = o.w - static_cast<float>(E::ld(l[3]));
        reinterpret_cast<float4 *>(pg)[i] = r;
    }
    for (size_t i = n4 * 4 + tid; i < n; i += stride) pg[i] = outer[i] - static_cast<float>(E::ld(local[i]));
}

template<typename E>
__global__ __launch_bounds__(kBlock) void k_outer_sgd(float *__restrict__ outer, float *__restrict__ mom,
                                                      const float *__restrict__ pg, typename E::S *__restrict__ local,
                                                      size_t n4, size_t n, OuterSgdParams p) {
    using S = typename E::S;
    using V = typename Local4<E>::V;
    const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    const size_t tid = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
    for (size_t i = tid; i < n4; i += stride) {
        float4 o = reinterpret_cast<const float4 *>(outer)[i];
        float4 m = p.first ? make_float4(0.f, 0.f, 0.f, 0.f) : reinterpret_cast<const float4 *>(mom)[i];
        const float4 g = reinterpret_cast<const float4 *>(pg)[i];
        outer_sgd_elem(o.x, m.x, g.x, p);
        outer_sgd_elem(o.y, m.y, g.y, p);
        outer_sgd_elem(o.z, m.z, g.z, p);
        outer_sgd_elem(o.w, m.w, g.w, p);
        reinterpret_cast<float4 *>(outer)[i] = o;
        reinterpret_cast<float4 *>(mom)[i] = m;
        V lv;
        S *l = reinterpret_cast<S *>(&lv);
        l[0] = E::st(o.x);
        l[1] = E::st(o.y);
        l[2] = E::st(o.z);
        l[3] = E::st(o.w);
        reinterpret_cast<V *>(local)[i] = lv;
    }
    for (size_t i = n4 * 4 + tid; i < n; i += stride) {
        float o = outer[i], m = p.first ? 0.f : mom[i];
        outer_sgd_elem(o, m, pg[i], p);
        outer[i] = o;
        mom[i] = m;
        local[i] = E::st(o);
    }
}

template<typename F>
static bool with_local(DType t, F &&f) {
    switch (t) {
        case DType::F32: return f(EF32{});
        case DType::BF16: return f(EBF16{});
        case DType::F16: return f(EF16{});
        default: return false;
    }
}

static bool aligned(const void *p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

bool launch_pseudo_grad(float *pg, const float *outer, const void *local, size_t count, DType lt, hipStream_t st) {
    if (count == 0) return true;
    return with_local(lt, [&](auto e) {
        using E = decltype(e);
        const bool vec = aligned(pg, 16) && aligned(outer, 16) && aligned(local, 4 * sizeof(typename E::S));
        const size_t n4 = vec ? count / 4 : 0;
        return launch_ok([&] {
            k_pseudo_grad<E><<<grid_for(n4 ? n4 : count), kBlock, 0, st>>>(
                pg, outer, static_cast<const typename E::S *>(local), n4, count);
        });
    });
}

bool launch_outer_sgd(float *outer, float *mom, const float *pg, void *local, size_t count, DType lt,
                      const OuterSgdParams &p, hipStream_t st) {
    if (count == 0) return true;
    return with_local(lt, [&](auto e) {
        using E = decltype(e);
        const bool vec = aligned(outer, 16) && aligned(mom, 16) && aligned(pg, 16) &&
                         aligned(local, 4 * sizeof(typename E::S));
        const size_t n4 = vec ? count / 4 : 0;
        return launch_ok([&] {
            k_outer_sgd<E><<<grid_for(n4 ? n4 : count), kBlock, 0, st>>>(
                outer, mom, pg, static_cast<typename E::S *>(local), n4, count, p);
        });
    });
}

} // namespace pccl::hipk
