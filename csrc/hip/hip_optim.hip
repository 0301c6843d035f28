// Fused DiLoCo outer-step kernels (math in csrc/kernels/optim_common.hpp, shared with the host twin).
//
// Memory-bound elementwise work over the whole model: one pass reading outer/mom/pg (fp32) and writing
// outer/mom/local instead of the ~5 passes of the unfused torch update. 4 elements per pack with 16-byte fp32 vector
// accesses (local: 16 B for fp32, 8 B for 16-bit types); scalar tail for the remainder.
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

__device__ __forceinline__ float4 ld4_nt(const float *p) {
    return __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const v4u32 *>(p)));
}
__device__ __forceinline__ void st4_nt(float *p, const float4 &v) {
    __builtin_nontemporal_store(__builtin_bit_cast(v4u32, v), reinterpret_cast<v4u32 *>(p));
}

// Both kernels run on the tiled ew_loop_ls (kernels.hpp): kEwUnroll independent 16-byte streaming loads per operand
// per thread, one tile per workgroup.
template<typename E>
__global__ __launch_bounds__(kBlock) void k_pseudo_grad(float *__restrict__ pg, const float *__restrict__ outer,
                                                        const typename E::S *__restrict__ local, size_t n, int vec) {
    using S = typename E::S;
    using V = typename Local4<E>::V;
    struct In {
        float4 o;
        V l;
    };
    ew_loop_ls<4, kEwUnroll>(
        n, 0, vec, [&](size_t i) { pg[i] = outer[i] - static_cast<float>(E::ld(local[i])); },
        [&](size_t b) { return In{ld4_nt(outer + b), *reinterpret_cast<const V *>(local + b)}; },
        [&](size_t b, const In &x) {
            const S *l = reinterpret_cast<const S *>(&x.l);
            float4 r;
            r.x = x.o.x - static_cast<float>(E::ld(l[0]));
            r.y = x.o.y - static_cast<float>(E::ld(l[1]));
            r.z = x.o.z - static_cast<float>(E::ld(l[2]));
            r.w = x.o.w - static_cast<float>(E::ld(l[3]));
            st4_nt(pg + b, r);
        });
}

template<typename E>
__global__ __launch_bounds__(kBlock) void k_outer_sgd(float *__restrict__ outer, float *__restrict__ mom,
                                                      const float *__restrict__ pg, typename E::S *__restrict__ local,
                                                      size_t n, int vec, OuterSgdParams p) {
    using S = typename E::S;
    using V = typename Local4<E>::V;
    struct In {
        float4 o, m, g;
    };
    ew_loop_ls<4, kEwUnroll>(
        n, 0, vec,
        [&](size_t i) {
            float o = outer[i], m = p.first ? 0.f : mom[i];
            outer_sgd_elem(o, m, pg[i], p);
            outer[i] = o;
            mom[i] = m;
            local[i] = E::st(o);
        },
        [&](size_t b) {
            return In{ld4_nt(outer + b), p.first ? make_float4(0.f, 0.f, 0.f, 0.f) : ld4_nt(mom + b), ld4_nt(pg + b)};
        },
        [&](size_t b, In x) {
            outer_sgd_elem(x.o.x, x.m.x, x.g.x, p);
            outer_sgd_elem(x.o.y, x.m.y, x.g.y, p);
            outer_sgd_elem(x.o.z, x.m.z, x.g.z, p);
            outer_sgd_elem(x.o.w, x.m.w, x.g.w, p);
            st4_nt(outer + b, x.o);
            st4_nt(mom + b, x.m);
            V lv;
            S *l = reinterpret_cast<S *>(&lv);
            l[0] = E::st(x.o.x);
            l[1] = E::st(x.o.y);
            l[2] = E::st(x.o.z);
            l[3] = E::st(x.o.w);
            *reinterpret_cast<V *>(local + b) = lv;
        });
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
        const EwPlan pl{0, vec && count >= 4 ? 1 : 0};
        return launch_ok([&] {
            k_pseudo_grad<E><<<grid_ew(count, pl, 4), kBlock, 0, st>>>(
                pg, outer, static_cast<const typename E::S *>(local), count, pl.vec);
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
        const EwPlan pl{0, vec && count >= 4 ? 1 : 0};
        return launch_ok([&] {
            k_outer_sgd<E><<<grid_ew(count, pl, 4), kBlock, 0, st>>>(
                outer, mom, pg, static_cast<typename E::S *>(local), count, pl.vec, p);
        });
    });
}

} // namespace pccl::hipk
