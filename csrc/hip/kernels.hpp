// HIP/CDNA4 kernels of pccl-amd. Header-only templates included by hip_backend.hip (single translation unit).
//
// Design notes (MI355X / gfx950):
//  * wave64, 256-thread workgroups (4 waves), grid-stride loops with the grid capped at 256 CUs x 8 WGs.
//  * Bit-exactness first: every arithmetic expression comes from csrc/common/numeric.hpp, csrc/kernels/elem.hpp and
//    csrc/kernels/quant_common.hpp, compiled with -ffp-contract=off exactly like the host SIMD loops, so a peer
//    reducing on the CPU and a peer reducing on an MI355X produce identical bytes.
//  * Ring/TCP-path kernels (reduce, dequant_reduce, quantize) read or write pinned host memory directly (zero-copy
//    over PCIe) — no staging H2D/D2H memcpy — and are bound by the network, so they use coalesced scalar element
//    access which works for the arbitrary (unaligned) chunk offsets of the ring.
//  * Intra-node xGMI kernels (multi_reduce / multi_gather) are bandwidth-critical: 16-byte vector loads
//    (global_load_dwordx4) from up to 16 IPC-mapped peer buffers per thread, two vectors in flight per source,
//    fp32 accumulation in fixed peer order, one rounding at the end.
//  * simplehash emulates the reference's 32-lane warp tree inside wave64 with __shfl_down(width=32).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <initializer_list>
#include <utility>

#include "../common/numeric.hpp"
#include "../common/types.hpp"
#include "../kernels/elem.hpp"
#include "../kernels/quant_common.hpp"

namespace pccl::hipk {

using namespace pccl::kernels;

constexpr int kBlock = 256;
constexpr int kMaxGrid = 2048;
constexpr int kMaxSrc = 16;

// streaming (non-temporal) 16-byte accesses: data that this GPU will not touch again soon (MI355X kbench: +5-20%
// over plain dwordx4 on HBM copies / reductions, csrc/tools/kbench.hip)
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load(const void *p) {
    const v4u32 v = __builtin_nontemporal_load(static_cast<const v4u32 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store(void *p, uint4 v) {
    const v4u32 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, static_cast<v4u32 *>(p));
}

inline int grid_for(size_t work_items, int per_thread = 1) {
    const size_t threads = (work_items + per_thread - 1) / per_thread;
    size_t g = (threads + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > static_cast<size_t>(kMaxGrid)) g = kMaxGrid;
    return static_cast<int>(g);
}

// ---------------------------------------------------------------- packed elementwise access
// Every elementwise kernel processes V = 16 / sizeof(S) elements per thread-iteration with 16-byte loads/stores of
// the value type (and V-element packs of the quantized type) when the operands can be aligned by peeling a scalar
// head; otherwise (ring chunks start at arbitrary element offsets) it falls back to a coalesced scalar loop. The
// per-element math is exactly the scalar math, so results stay bit-identical to the host twins.
template<typename T, int N>
struct alignas(sizeof(T) * N) Pack {
    T v[N];
};
template<typename S>
constexpr int vec_width() {
    return sizeof(S) >= 16 ? 1 : static_cast<int>(16 / sizeof(S));
}
template<typename T, int N>
__device__ __forceinline__ Pack<T, N> ldp(const T *p) {
    return *reinterpret_cast<const Pack<T, N> *>(p);
}
template<typename T, int N>
__device__ __forceinline__ void stp(T *p, const Pack<T, N> &v) {
    *reinterpret_cast<Pack<T, N> *>(p) = v;
}
// streaming variants of ldp/stp for 16-byte packs (HBM read-modify-write kernels: no reuse of either operand)
template<typename T, int N>
__device__ __forceinline__ Pack<T, N> ldp_nt(const T *p) {
    static_assert(sizeof(Pack<T, N>) == 16);
    return __builtin_bit_cast(Pack<T, N>, __builtin_nontemporal_load(reinterpret_cast<const v4u32 *>(p)));
}
template<typename T, int N>
__device__ __forceinline__ void stp_nt(T *p, const Pack<T, N> &v) {
    static_assert(sizeof(Pack<T, N>) == 16);
    __builtin_nontemporal_store(__builtin_bit_cast(v4u32, v), reinterpret_cast<v4u32 *>(p));
}

struct EwPlan {
    size_t head = 0; // scalar elements before the first aligned pack
    int vec = 0;
};
// operands: (pointer, element size); the first is the anchor whose 16-byte alignment fixes the head
template<int V>
inline EwPlan plan_ew(size_t n, std::initializer_list<std::pair<const void *, size_t>> ops) {
    EwPlan pl;
    const auto &a = *ops.begin();
    const size_t pack0 = static_cast<size_t>(V) * a.second;
    const size_t mis = reinterpret_cast<uintptr_t>(a.first) % pack0;
    size_t head = mis == 0 ? 0 : pack0 - mis;
    if (head % a.second != 0) return pl;
    head /= a.second;
    if (head >= n || (n - head) / V == 0) return pl;
    for (const auto &o : ops)
        if ((reinterpret_cast<uintptr_t>(o.first) + head * o.second) % (static_cast<size_t>(V) * o.second) != 0) return pl;
    pl.head = head;
    pl.vec = 1;
    return pl;
}

template<int V, typename Fs, typename Fv>
__device__ __forceinline__ void ew_loop(size_t n, size_t head, int vec, Fs &&scalar, Fv &&vector) {
    const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    const size_t tid = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (!vec) {
        for (size_t i = tid; i < n; i += stride) scalar(i);
        return;
    }
    for (size_t i = tid; i < head; i += stride) scalar(i);
    const size_t np = (n - head) / V;
    for (size_t k = tid; k < np; k += stride) vector(head + k * V);
    for (size_t i = head + np * V + tid; i < n; i += stride) scalar(i);
}

// Tiled variant for HBM-bound read-modify-write kernels (the torch-elementwise shape): a workgroup owns tiles of
// kBlock*U contiguous packs, each thread issues its U independent 16-byte loads (k, k+kBlock, ... — fully coalesced;
// all loads precede the stores in program order so they stay in flight together) before computing and storing, and
// the launcher sizes the grid to one tile per workgroup (grid_ew) instead of the 2048-workgroup grid-stride cap: a
// grid-stride loop with one pack in flight per thread leaves HBM3E under-subscribed (MI355X kbench: 5.0 vs 5.9 TB/s).
constexpr int kEwUnroll = 4;
template<int V, int U, typename Fs, typename Fl, typename Fst>
__device__ __forceinline__ void ew_loop_ls(size_t n, size_t head, int vec, Fs &&scalar, Fl &&vload, Fst &&vstore) {
    const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    const size_t tid = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (!vec) {
        for (size_t i = tid; i < n; i += stride) scalar(i);
        return;
    }
    for (size_t i = tid; i < head; i += stride) scalar(i);
    const size_t np = (n - head) / V;
    constexpr size_t T = static_cast<size_t>(kBlock) * U;
    const size_t ntiles = np / T;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t k = t * T + threadIdx.x;
        decltype(vload(size_t{0})) st[U];
#pragma unroll
        for (int u = 0; u < U; ++u) st[u] = vload(head + (k + static_cast<size_t>(u) * kBlock) * V);
#pragma unroll
        for (int u = 0; u < U; ++u) vstore(head + (k + static_cast<size_t>(u) * kBlock) * V, st[u]);
    }
    for (size_t k = ntiles * T + tid; k < np; k += stride) vstore(head + k * V, vload(head + k * V));
    for (size_t i = head + np * V + tid; i < n; i += stride) scalar(i);
}
// grid of an ew_loop_ls kernel: one workgroup per tile when vectorised, the grid-stride grid otherwise
inline int grid_ew(size_t n, const EwPlan &pl, int V) {
    if (!pl.vec) return grid_for(n, 1);
    const size_t tiles = ((n - pl.head) / V + static_cast<size_t>(kBlock) * kEwUnroll - 1) /
                         (static_cast<size_t>(kBlock) * kEwUnroll);
    return static_cast<int>(std::max<size_t>(1, std::min<size_t>(tiles, size_t{1} << 20)));
}


// ---------------------------------------------------------------- min / max helpers
// Comparisons run in the codec's compute type (exact for every value of the storage type); partials are doubles.
template<typename C>
__device__ __forceinline__ void wave_minmax(C &lo, C &hi) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const C l2 = __shfl_xor(lo, off, 64);
        const C h2 = __shfl_xor(hi, off, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
}

template<typename C>
__device__ __forceinline__ void block_minmax(C &lo, C &hi, C *s_lo, C *s_hi) {
    wave_minmax(lo, hi);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_lo[w] = lo;
        s_hi[w] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kBlock / 64; ++k) {
            lo = s_lo[k] < lo ? s_lo[k] : lo;
            hi = s_hi[k] > hi ? s_hi[k] : hi;
        }
    }
}

// Per-thread running (min, max) of the values a kernel stores, folded per workgroup into partial[2*blockIdx.x ...]
// at the end (the quantized ring's de-quantize-reduce kernels emit the min / max the next step's quantization needs,
// so no separate min / max pass over the chunk; folded by k_minmax_final). Off (no-op) when MM is false.
template<typename C, bool MM>
struct MinMaxAcc {
    C lo = static_cast<C>(__builtin_inf()), hi = static_cast<C>(-__builtin_inf());
    __device__ __forceinline__ void take(C v) {
        if constexpr (MM) {
            lo = v < lo ? v : lo;
            hi = v > hi ? v : hi;
        }
    }
    __device__ __forceinline__ void finish(double *partial) {
        if constexpr (MM) {
            __shared__ C s_lo[kBlock / 64], s_hi[kBlock / 64];
            block_minmax(lo, hi, s_lo, s_hi);
            if (threadIdx.x == 0) {
                partial[2 * blockIdx.x] = static_cast<double>(lo);
                partial[2 * blockIdx.x + 1] = static_cast<double>(hi);
            }
        }
    }
};

// ---------------------------------------------------------------- elementwise reduce (ring path)
template<typename E, typename Op>
__global__ __launch_bounds__(kBlock) void k_reduce(typename E::S *__restrict__ dst, const typename E::S *__restrict__ src,
                                                   size_t n, size_t head, int vec) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    struct DS {
        Pack<S, V> d, s;
    };
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec, [&](size_t i) { dst[i] = E::st(apply_op<Op, C>(E::ld(dst[i]), E::ld(src[i]))); },
        [&](size_t b) { return DS{ldp_nt<S, V>(dst + b), ldp_nt<S, V>(src + b)}; },
        [&](size_t b, DS x) {
#pragma unroll
            for (int e = 0; e < V; ++e) x.d.v[e] = E::st(apply_op<Op, C>(E::ld(x.d.v[e]), E::ld(x.s.v[e])));
            stp_nt<S, V>(dst + b, x.d);
        });
}

// Device-ring reduce-scatter step, fused with the next step's staging: dst op= src (both HBM) and the result is also
// streamed to `out` in pinned host memory (posted PCIe writes from the kernel), which is the next ring step's payload.
// A separate device->host copy would have to wait on this kernel on another stream - and ROCclr turns copies queued
// behind a cross-stream wait into blit kernels (measured: profiles/r2/ring_*.md) - so the producer writes it itself.
template<typename E, typename Op>
__global__ __launch_bounds__(kBlock) void k_reduce_copy(typename E::S *__restrict__ dst,
                                                        const typename E::S *__restrict__ src,
                                                        typename E::S *__restrict__ out, size_t n, size_t head,
                                                        int vec) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    struct DS {
        Pack<S, V> d, s;
    };
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec,
        [&](size_t i) {
            const S r = E::st(apply_op<Op, C>(E::ld(dst[i]), E::ld(src[i])));
            dst[i] = r;
            out[i] = r;
        },
        [&](size_t b) { return DS{ldp_nt<S, V>(dst + b), ldp_nt<S, V>(src + b)}; },
        [&](size_t b, DS x) {
#pragma unroll
            for (int e = 0; e < V; ++e) x.d.v[e] = E::st(apply_op<Op, C>(E::ld(x.d.v[e]), E::ld(x.s.v[e])));
            stp_nt<S, V>(dst + b, x.d);
            stp_nt<S, V>(out + b, x.d);
        });
}

// ---------------------------------------------------------------- fused dequant + reduce
// MM: also emit the workgroup's (min, max) of the stored results (MinMaxAcc) into `mm`
template<typename E, typename Op, typename Q, bool MM>
__global__ __launch_bounds__(kBlock) void k_dq_minmax(typename E::S *__restrict__ dst, const Q *__restrict__ src, size_t n,
                                                      QuantParams p, size_t head, int vec, double *__restrict__ mm) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    struct DQ {
        Pack<S, V> d;
        Pack<Q, V> q;
    };
    MinMaxAcc<C, MM> acc;
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec,
        [&](size_t i) {
            const C v = static_cast<C>(dq_minmax_int(static_cast<double>(src[i]), p));
            const S r = E::st(apply_op<Op, C>(E::ld(dst[i]), v));
            dst[i] = r;
            acc.take(E::ld(r));
        },
        [&](size_t b) { return DQ{ldp_nt<S, V>(dst + b), ldp<Q, V>(src + b)}; },
        [&](size_t b, DQ x) {
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const C v = static_cast<C>(dq_minmax_int(static_cast<double>(x.q.v[e]), p));
                x.d.v[e] = E::st(apply_op<Op, C>(E::ld(x.d.v[e]), v));
                acc.take(E::ld(x.d.v[e]));
            }
            stp_nt<S, V>(dst + b, x.d);
        });
    acc.finish(mm);
}

template<typename E, typename Op, bool E4M3, bool MM>
__global__ __launch_bounds__(kBlock) void k_dq_fp8(typename E::S *__restrict__ dst, const uint8_t *__restrict__ src, size_t n,
                                                   QuantParams p, size_t head, int vec, double *__restrict__ mm) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    auto deq = [&](uint8_t q) { return (E4M3 ? num::fp8e4m3_to_f32(q) : num::fp8e5m2_to_f32(q)) * p.f8_inv; };
    struct DQ {
        Pack<S, V> d;
        Pack<uint8_t, V> q;
    };
    MinMaxAcc<C, MM> acc;
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec,
        [&](size_t i) {
            const S r = E::st(apply_op<Op, C>(E::ld(dst[i]), static_cast<C>(deq(src[i]))));
            dst[i] = r;
            acc.take(E::ld(r));
        },
        [&](size_t b) { return DQ{ldp_nt<S, V>(dst + b), ldp<uint8_t, V>(src + b)}; },
        [&](size_t b, DQ x) {
#pragma unroll
            for (int e = 0; e < V; ++e) {
                x.d.v[e] = E::st(apply_op<Op, C>(E::ld(x.d.v[e]), static_cast<C>(deq(x.q.v[e]))));
                acc.take(E::ld(x.d.v[e]));
            }
            stp_nt<S, V>(dst + b, x.d);
        });
    acc.finish(mm);
}

template<typename E, typename Op, typename Q, bool MM>
__global__ __launch_bounds__(kBlock) void k_dq_zps(typename E::S *__restrict__ dst, const Q *__restrict__ src, size_t n,
                                                   QuantParams p, size_t head, int vec, double *__restrict__ mm) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    struct DQ {
        Pack<S, V> d;
        Pack<Q, V> q;
    };
    MinMaxAcc<C, MM> acc;
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec,
        [&](size_t i) {
            const S r = E::st(apply_op<Op, C>(E::ld(dst[i]), static_cast<C>(dq_zps_as<Q>(src[i], p))));
            dst[i] = r;
            acc.take(E::ld(r));
        },
        [&](size_t b) { return DQ{ldp_nt<S, V>(dst + b), ldp<Q, V>(src + b)}; },
        [&](size_t b, DQ x) {
#pragma unroll
            for (int e = 0; e < V; ++e) {
                x.d.v[e] = E::st(apply_op<Op, C>(E::ld(x.d.v[e]), static_cast<C>(dq_zps_as<Q>(x.q.v[e], p))));
                acc.take(E::ld(x.d.v[e]));
            }
            stp_nt<S, V>(dst + b, x.d);
        });
    acc.finish(mm);
}

// ---------------------------------------------------------------- quantize
template<typename Q>
__device__ __forceinline__ Q q_from_double(double q) {
    if constexpr (sizeof(Q) == 8 && !__is_signed(Q)) {
        return q >= 18446744073709551615.0 ? ~0ull : static_cast<uint64_t>(q);
    } else if constexpr (sizeof(Q) == 8) {
        return q >= 9223372036854775807.0 ? INT64_MAX : static_cast<int64_t>(q);
    } else if constexpr (__is_signed(Q)) { // integral and inside Q's range: the native 32-bit conversions are exact
        return static_cast<Q>(static_cast<int32_t>(q)); // (a 64-bit one is a ~6-instruction FP64 sequence)
    } else {
        return static_cast<Q>(static_cast<uint32_t>(q));
    }
}

// q_from_double(q_minmax_int(x, p)) without FP64 floor / add for wire types up to 32 bits: r is clamped to
// [0, range] first, where truncation (the native conversion) equals floor, and adding qlo as an integer is exact -
// the same integer for every input.
template<typename Q>
__device__ __forceinline__ Q q_minmax_as(double x, const QuantParams &p) {
    if constexpr (sizeof(Q) == 8) {
        return q_from_double<Q>(q_minmax_int(x, p));
    } else {
        double r = (x - p.min) * p.inv_dif * p.range + 0.5;
        r = r < 0.0 ? 0.0 : r;
        r = r > p.range ? p.range : r;
        return static_cast<Q>(static_cast<int64_t>(static_cast<uint32_t>(r)) + static_cast<int64_t>(p.qlo));
    }
}

// Quantize kernels. BACK: also overwrite the source with its de-quantized value, D(Q(x)), exactly as the
// de-quantize kernels with ReduceOp::Set compute it (the owner's copy of a quantized all-gather payload must equal what
// every other peer de-quantizes): one pass over the chunk instead of quantize + a de-quantize kernel that reads the
// quantized bytes back from pinned host memory.
template<typename E, typename Q, bool BACK>
__global__ __launch_bounds__(kBlock) void k_q_minmax(Q *__restrict__ dst, typename E::S *__restrict__ src, size_t n,
                                                     QuantParams p, size_t head, int vec) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    auto back = [&](Q q) { return E::st(static_cast<C>(dq_minmax_int(static_cast<double>(q), p))); };
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec,
        [&](size_t i) {
            const Q q = q_minmax_as<Q>(static_cast<double>(E::ld(src[i])), p);
            dst[i] = q;
            if constexpr (BACK) src[i] = back(q);
        },
        [&](size_t b) { return ldp_nt<S, V>(src + b); },
        [&](size_t b, const Pack<S, V> &s) {
            Pack<Q, V> q;
#pragma unroll
            for (int e = 0; e < V; ++e) q.v[e] = q_minmax_as<Q>(static_cast<double>(E::ld(s.v[e])), p);
            stp<Q, V>(dst + b, q);
            if constexpr (BACK) {
                Pack<S, V> d;
#pragma unroll
                for (int e = 0; e < V; ++e) d.v[e] = back(q.v[e]);
                stp_nt<S, V>(src + b, d);
            }
        });
}

template<typename E, bool E4M3, bool BACK>
__global__ __launch_bounds__(kBlock) void k_q_fp8(uint8_t *__restrict__ dst, typename E::S *__restrict__ src, size_t n,
                                                  QuantParams p, size_t head, int vec) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    auto qf = [&](S v) {
        const float x = static_cast<float>(E::ld(v)) * p.f8_scale;
        return E4M3 ? num::f32_to_fp8e4m3(x) : num::f32_to_fp8e5m2(x);
    };
    auto back = [&](uint8_t q) {
        return E::st(static_cast<C>((E4M3 ? num::fp8e4m3_to_f32(q) : num::fp8e5m2_to_f32(q)) * p.f8_inv));
    };
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec,
        [&](size_t i) {
            const uint8_t q = qf(src[i]);
            dst[i] = q;
            if constexpr (BACK) src[i] = back(q);
        },
        [&](size_t b) { return ldp_nt<S, V>(src + b); },
        [&](size_t b, const Pack<S, V> &s) {
            Pack<uint8_t, V> q;
#pragma unroll
            for (int e = 0; e < V; ++e) q.v[e] = qf(s.v[e]);
            stp<uint8_t, V>(dst + b, q);
            if constexpr (BACK) {
                Pack<S, V> d;
#pragma unroll
                for (int e = 0; e < V; ++e) d.v[e] = back(q.v[e]);
                stp_nt<S, V>(src + b, d);
            }
        });
}

template<typename E, typename Q, bool BACK>
__global__ __launch_bounds__(kBlock) void k_q_zps(Q *__restrict__ dst, typename E::S *__restrict__ src, size_t n,
                                                  QuantParams p, size_t head, int vec) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    auto back = [&](Q q) { return E::st(static_cast<C>(dq_zps_as<Q>(q, p))); };
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec,
        [&](size_t i) {
            const Q q = q_zps_as<Q>(static_cast<float>(E::ld(src[i])), p);
            dst[i] = q;
            if constexpr (BACK) src[i] = back(q);
        },
        [&](size_t b) { return ldp_nt<S, V>(src + b); },
        [&](size_t b, const Pack<S, V> &s) {
            Pack<Q, V> q;
#pragma unroll
            for (int e = 0; e < V; ++e) q.v[e] = q_zps_as<Q>(static_cast<float>(E::ld(s.v[e])), p);
            stp<Q, V>(dst + b, q);
            if constexpr (BACK) {
                Pack<S, V> d;
#pragma unroll
                for (int e = 0; e < V; ++e) d.v[e] = back(q.v[e]);
                stp_nt<S, V>(src + b, d);
            }
        });
}

// ---------------------------------------------------------------- min / max (two pass, exact)
// Pass 1: every workgroup reduces its tiles to a (min, max) partial. A single-launch variant (last workgroup folds
// the partials behind a device-scope ticket) measured slower on MI355X - each workgroup's agent-scope release is an
// L2 write-back (`buffer_wbl2`), 1024 of them cost more than the second launch (profiles/r2/kernels_polish.md).
template<typename E>
__global__ __launch_bounds__(kBlock) void k_minmax_partial(const typename E::S *__restrict__ src, size_t n,
                                                           double *__restrict__ partial, size_t head, int vec) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    __shared__ C s_lo[kBlock / 64], s_hi[kBlock / 64];
    C lo = static_cast<C>(__builtin_inf()), hi = static_cast<C>(-__builtin_inf());
    auto take = [&](C v) {
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    };
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec, [&](size_t i) { take(E::ld(src[i])); }, [&](size_t b) { return ldp_nt<S, V>(src + b); },
        [&](size_t, const Pack<S, V> &s) {
#pragma unroll
            for (int e = 0; e < V; ++e) take(E::ld(s.v[e]));
        });
    block_minmax(lo, hi, s_lo, s_hi);
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = static_cast<double>(lo);
        partial[2 * blockIdx.x + 1] = static_cast<double>(hi);
    }
}

// Pass 2 (one workgroup): fold the partials, write {min, max} to `out` (pinned host words)
template<int Unused = 0>
__global__ __launch_bounds__(kBlock) void k_minmax_final(const double *__restrict__ partial, int nblocks, size_t n,
                                                         double *__restrict__ out) {
    __shared__ double s_lo[kBlock / 64], s_hi[kBlock / 64];
    double lo = __builtin_inf(), hi = -__builtin_inf();
    // 8 independent 16-byte (min, max) loads in flight per thread and pass: the fused de-quantize kernels leave
    // thousands of partials per chunk, and a one-load-per-iteration loop waits out the memory latency each time
    // (rocprofv3: 150 us per fold of ~8k partials)
    constexpr int kIlp = 8;
    const double2 *pp = reinterpret_cast<const double2 *>(partial);
    for (int i0 = 0; i0 < nblocks; i0 += kBlock * kIlp) {
        double2 v[kIlp];
#pragma unroll
        for (int k = 0; k < kIlp; ++k) {
            const int i = i0 + k * kBlock + static_cast<int>(threadIdx.x);
            v[k] = i < nblocks ? pp[i] : make_double2(__builtin_inf(), -__builtin_inf());
        }
#pragma unroll
        for (int k = 0; k < kIlp; ++k) {
            lo = v[k].x < lo ? v[k].x : lo;
            hi = v[k].y > hi ? v[k].y : hi;
        }
    }
    block_minmax(lo, hi, s_lo, s_hi);
    if (threadIdx.x == 0) {
        out[0] = n ? lo : 0.0;
        out[1] = n ? hi : 0.0;
    }
}

// ---------------------------------------------------------------- AVG finalize
template<typename E>
__global__ __launch_bounds__(kBlock) void k_avg(typename E::S *__restrict__ dst, size_t n, size_t ws, size_t head, int vec) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = vec_width<S>();
    const C w = static_cast<C>(ws);
    ew_loop_ls<V, kEwUnroll>(
        n, head, vec, [&](size_t i) { dst[i] = E::st(static_cast<C>(E::ld(dst[i]) / w)); },
        [&](size_t b) { return ldp_nt<S, V>(dst + b); },
        [&](size_t b, Pack<S, V> d) {
#pragma unroll
            for (int e = 0; e < V; ++e) d.v[e] = E::st(static_cast<C>(E::ld(d.v[e]) / w));
            stp_nt<S, V>(dst + b, d);
        });
}

// ---------------------------------------------------------------- byte copy (device ring all-gather H2D)
// Plain copy of n bytes as 16-byte packs (scalar head / tail); the device ring's all-gather moves received chunks
// pinned -> HBM with it when it wants to choose the number of workgroups reading over PCIe (PCCL_RING_AG_COPY_GRID)
// instead of the runtime's blit kernel.
template<int Unused = 0> // a template: this header is included by several translation units
__global__ __launch_bounds__(kBlock) void k_copy_bytes(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                     size_t n, size_t head, int vec) {
    ew_loop_ls<16, kEwUnroll>(
        n, head, vec, [&](size_t i) { dst[i] = src[i]; }, [&](size_t b) { return ldp<uint8_t, 16>(src + b); },
        [&](size_t b, const Pack<uint8_t, 16> &v) { stp_nt<uint8_t, 16>(dst + b, v); });
}

// ---------------------------------------------------------------- xGMI multi-source reduce
struct SrcList {
    const void *p[kMaxSrc];
};

// One 16-byte vector holds VEC elements of storage type S.
template<typename E>
struct Vec {
    using S = typename E::S;
    static constexpr int N = 16 / sizeof(S);
};

// Destinations of a reduced shard: the owner's own output plus (one-shot push all-reduce) every peer's output.
struct DstList {
    void *p[kMaxSrc];
};

// Reads VEC-element vectors i and i+stride from every source (fixed peer order, fp32 accumulation, one rounding, so
// every peer gets bit-identical bytes) and stores the result to every destination. In the one-shot IPC all-reduce the
// destinations are the receive buffers of all peers (remote ones over xGMI: posted writes, so the outbound direction
// of the links carries the all-gather while the inbound direction carries the reduce-scatter reads).
// End of an xGMI kernel whose destinations include another GPU's HBM (IPC-mapped): one system-scope release per
// workgroup (after every wave's stores issued) makes them visible to a peer that observes this op's completion through
// the host-side barrier. Launched only when a destination is remote: per workgroup it costs ~5% of the kernel's
// bandwidth, per thread 15-35% (profiles/r2/kernels_fence.md); same-GPU destinations need no more than kernel end.
__device__ __forceinline__ void ipc_release_system() {
    __syncthreads();
    if (threadIdx.x == 0) __threadfence_system();
}

template<typename E, typename Op, bool AVG, int U = 2>
__global__ __launch_bounds__(kBlock) void k_multi_reduce_vec(DstList dsts, int ndst, SrcList srcs, int nsrc, size_t nvec,
                                                          int release) {
    // U vectors (i, i + stride, ...) per thread and iteration: U x nsrc 16-byte loads in flight
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = Vec<E>::N;
    const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    const size_t tid = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
    for (size_t i = tid; i < nvec; i += U * stride) {
        size_t idx[U];
        bool has[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + static_cast<size_t>(u) * stride;
            has[u] = j < nvec;
            idx[u] = has[u] ? j : i; // keep every load in bounds; results of the clamped ones are discarded
        }
        C acc[U][V];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint4 a = reinterpret_cast<const uint4 *>(srcs.p[0])[idx[u]];
            const S *s0 = reinterpret_cast<const S *>(&a);
#pragma unroll
            for (int e = 0; e < V; ++e) acc[u][e] = E::ld(s0[e]);
        }
        // sources are read in fixed peer order (bit-identical on every peer)
#pragma unroll 4
        for (int k = 1; k < nsrc; ++k) {
            uint4 a[U];
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = reinterpret_cast<const uint4 *>(srcs.p[k])[idx[u]];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const S *s1 = reinterpret_cast<const S *>(&a[u]);
#pragma unroll
                for (int e = 0; e < V; ++e) acc[u][e] = apply_op<Op, C>(acc[u][e], E::ld(s1[e]));
            }
        }
        uint4 out[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            S *o = reinterpret_cast<S *>(&out[u]);
#pragma unroll
            for (int e = 0; e < V; ++e) {
                if (AVG) acc[u][e] = static_cast<C>(acc[u][e] / static_cast<C>(nsrc));
                o[e] = E::st(acc[u][e]);
            }
        }
#pragma unroll 4
        for (int k = 0; k < ndst; ++k) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (has[u]) nt_store(static_cast<uint4 *>(dsts.p[k]) + idx[u], out[u]);
        }
    }
    if (release) ipc_release_system(); // uniform per launch
}

// Tiled variant of k_multi_reduce_vec: workgroup t owns the contiguous tile [t*kBlock*U, (t+1)*kBlock*U) of vectors
// (walking tiles blockIdx.x, blockIdx.x + gridDim.x, ...), every source read with non-temporal 16-byte loads so the
// streamed operands do not evict each other from L2; U x nsrc loads in flight per thread. Same fixed peer order and
// single rounding as k_multi_reduce_vec (bit-identical results).
template<typename E, typename Op, bool AVG, int U = 4>
__global__ __launch_bounds__(kBlock) void k_multi_reduce_tile(DstList dsts, int ndst, SrcList srcs, int nsrc, size_t nvec,
                                                           int release) {
    using S = typename E::S;
    using C = typename E::C;
    constexpr int V = Vec<E>::N;
    constexpr size_t T = static_cast<size_t>(kBlock) * U;
    const size_t ntiles = (nvec + T - 1) / T;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t base = t * T + threadIdx.x;
        size_t idx[U];
        bool has[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = base + static_cast<size_t>(u) * kBlock;
            has[u] = j < nvec;
            idx[u] = has[u] ? j : base; // base < nvec for every thread that has u = 0 work; clamped loads are discarded
        }
        if (!has[0]) continue;
        C acc[U][V];
        {
            uint4 a[U];
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = nt_load(static_cast<const uint4 *>(srcs.p[0]) + idx[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const S *s0 = reinterpret_cast<const S *>(&a[u]);
#pragma unroll
                for (int e = 0; e < V; ++e) acc[u][e] = E::ld(s0[e]);
            }
        }
#pragma unroll 4
        for (int k = 1; k < nsrc; ++k) {
            uint4 a[U];
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = nt_load(static_cast<const uint4 *>(srcs.p[k]) + idx[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const S *s1 = reinterpret_cast<const S *>(&a[u]);
#pragma unroll
                for (int e = 0; e < V; ++e) acc[u][e] = apply_op<Op, C>(acc[u][e], E::ld(s1[e]));
            }
        }
        uint4 out[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            S *o = reinterpret_cast<S *>(&out[u]);
#pragma unroll
            for (int e = 0; e < V; ++e) {
                if (AVG) acc[u][e] = static_cast<C>(acc[u][e] / static_cast<C>(nsrc));
                o[e] = E::st(acc[u][e]);
            }
        }
#pragma unroll 4
        for (int k = 0; k < ndst; ++k) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (has[u]) nt_store(static_cast<uint4 *>(dsts.p[k]) + idx[u], out[u]);
        }
    }
    if (release) ipc_release_system(); // uniform per launch
}

template<typename E, typename Op, bool AVG>
__global__ __launch_bounds__(kBlock) void k_multi_reduce_scalar(DstList dsts, int ndst, SrcList srcs, int nsrc, size_t n,
                                                                size_t begin, int release) {
    using S = typename E::S;
    using C = typename E::C;
    const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = begin + static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
        C acc = E::ld(static_cast<const S *>(srcs.p[0])[i]);
        for (int k = 1; k < nsrc; ++k) acc = apply_op<Op, C>(acc, E::ld(static_cast<const S *>(srcs.p[k])[i]));
        if (AVG) acc = static_cast<C>(acc / static_cast<C>(nsrc));
        const S v = E::st(acc);
        for (int k = 0; k < ndst; ++k) static_cast<S *>(dsts.p[k])[i] = v;
    }
    if (release) ipc_release_system(); // uniform per launch
}

// ---------------------------------------------------------------- xGMI multi-source gather (all-gather phase)
struct GatherList {
    const void *src[kMaxSrc];
    size_t off[kMaxSrc];   // destination byte offset of segment k
    size_t bytes[kMaxSrc]; // bytes of segment k
};

template<int Unused = 0>
__global__ __launch_bounds__(kBlock) void k_multi_gather(uint8_t *__restrict__ dst, GatherList g, int n, int skip,
                                                          int release) {
    // blockIdx.y selects the segment (every peer's segment streams concurrently over its own xGMI link); within a
    // segment each workgroup copies one contiguous chunk, 4 x 16 B per thread in flight, non-temporal both ways
    const int k = blockIdx.y;
    if (k >= n || k == skip) return;
    const uint8_t *src = static_cast<const uint8_t *>(g.src[k]);
    uint8_t *d = dst + g.off[k];
    const size_t bytes = g.bytes[k];
    const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d)) & 15) == 0;
    if (aligned) {
        const size_t nvec = bytes / 16;
        const size_t per = ((nvec + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
        const size_t lo = static_cast<size_t>(blockIdx.x) * per;
        const size_t hi = lo + per < nvec ? lo + per : nvec;
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(d);
        size_t i = lo + threadIdx.x;
        for (; i + 3 * kBlock < hi; i += 4 * kBlock) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = nt_load(s4 + i + u * kBlock);
#pragma unroll
            for (int u = 0; u < 4; ++u) nt_store(d4 + i + u * kBlock, v[u]);
        }
        for (; i < hi; i += kBlock) d4[i] = s4[i];
        const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
        for (size_t b = nvec * 16 + static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; b < bytes; b += stride)
            d[b] = src[b];
    } else {
        const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
        for (size_t b = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; b < bytes; b += stride) d[b] = src[b];
    }
    if (release) ipc_release_system(); // uniform per launch (the early return above is per workgroup)
}

// ---------------------------------------------------------------- simplehash
__device__ __forceinline__ uint32_t hcomb(uint32_t a, uint32_t b) {
    a ^= b + 0x9e3779b1u;
    a = (a << 7) | (a >> 25);
    return a * 0x85ebca6bu;
}

// 256-thread block reduction with the reference's exact 32-lane tree (8 groups of 32, then 8 partials + 24 zeros).
__device__ __forceinline__ uint32_t block_tree256(uint32_t v, uint32_t *lds8) {
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) v = hcomb(v, __shfl_down(v, off, 32));
    const int t = threadIdx.x;
    if ((t & 31) == 0) lds8[t >> 5] = v;
    __syncthreads();
    uint32_t r = 0;
    if (t < 32) {
        r = t < 8 ? lds8[t] : 0u;
#pragma unroll
        for (int off = 16; off > 0; off >>= 1) r = hcomb(r, __shfl_down(r, off, 32));
    }
    return r;
}

template<int Unused = 0>
__global__ __launch_bounds__(kBlock) void k_hash_big(const uint4 *__restrict__ d4, uint32_t *__restrict__ partial,
                                                     size_t n_vec, size_t vpb) {
    __shared__ uint32_t lds8[8];
    const size_t start = static_cast<size_t>(blockIdx.x) * vpb;
    size_t end = start + vpb;
    if (end > n_vec) end = n_vec;
    uint32_t h = 0;
    size_t i = start + threadIdx.x;
    // software pipeline: 8 independent 16-byte loads in flight ahead of the serial hash chain
    constexpr int D = 8;
    for (; i + (D - 1) * kBlock < end; i += D * kBlock) {
        uint4 v[D];
#pragma unroll
        for (int k = 0; k < D; ++k) v[k] = d4[i + k * kBlock];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            h = hcomb(h, v[k].x);
            h = hcomb(h, v[k].y);
            h = hcomb(h, v[k].z);
            h = hcomb(h, v[k].w);
        }
    }
    for (; i < end; i += kBlock) {
        const uint4 v = d4[i];
        h = hcomb(h, v.x);
        h = hcomb(h, v.y);
        h = hcomb(h, v.z);
        h = hcomb(h, v.w);
    }
    const uint32_t r = block_tree256(h, lds8);
    if (threadIdx.x == 0) partial[blockIdx.x] = r;
}

// final pass + tail words/bytes handled on device; writes the 32-bit hash to out[0]
template<int Unused = 0>
__global__ __launch_bounds__(kBlock) void k_hash_final(const uint32_t *__restrict__ partial, int nblocks,
                                                       const uint8_t *__restrict__ data, size_t n_bytes,
                                                       uint32_t *__restrict__ out) {
    __shared__ uint32_t lds8[8];
    uint32_t h = 0;
    for (int i = threadIdx.x; i < nblocks; i += kBlock) h = hcomb(h, partial[i]);
    uint32_t r = block_tree256(h, lds8);
    if (nblocks == 0) r = 0;
    if (threadIdx.x == 0) {
        const size_t n_words = n_bytes / 4;
        const size_t n_vec = n_words / 4;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(data);
        for (size_t k = n_vec * 4; k < n_words; ++k) r = hcomb(r, w[k]);
        const size_t tail = n_bytes % 4;
        if (tail) {
            uint32_t v = 0;
            for (size_t k = 0; k < tail; ++k) v |= static_cast<uint32_t>(data[n_words * 4 + k]) << (8 * k);
            r = hcomb(r, v);
        }
        out[0] = r;
    }
}

// ---------------------------------------------------------------- CRC-32C
// Split CRC (csrc/kernels/host_kernels.hpp): thread t of a workgroup owns the 64-byte chunk t of every 16 KiB tile of
// the workgroup's contiguous range (a wave reads 4 KiB contiguously). Per tile it computes the chunk's raw CRC with
// slicing-by-8 LDS tables and folds it into its accumulator, which is first moved 16 KiB further down the message
// (multiplication by the constant x^(8*16384) as 4 LDS table lookups). The 256 accumulators are then combined in an
// 8-level LDS tree (shift by 64 * 2^k bytes = one GF(2) multiply by a host-computed constant). The host folds the
// per-workgroup partials and the unaligned head / tail bytes, then applies the standard init / final inversion.
constexpr int kCrcChunk = 64;
constexpr int kCrcTile = kBlock * kCrcChunk; // 16 KiB
struct CrcTables {
    uint32_t slice[8][256]; // slice[k][b]: raw CRC of byte b followed by k zero bytes
    uint32_t tile[4][256];  // tile[k][b]: (b << 8k) * x^(8 * kCrcTile) mod P
};
struct CrcLevels {
    uint32_t m[8]; // x^(8 * kCrcChunk * 2^k) mod P
};

__device__ __forceinline__ uint32_t crc_gf_mul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        p ^= (0u - ((a >> i) & 1u)) & b;
        b = (b >> 1) ^ (0x82F63B78u & (0u - (b & 1u)));
    }
    return p;
}

template<int Unused = 0>
__global__ __launch_bounds__(kBlock) void k_crc32c(const uint8_t *__restrict__ data, size_t n_tiles,
                                                   size_t tiles_per_wg, const CrcTables *__restrict__ tabs,
                                                   CrcLevels lv, uint32_t *__restrict__ partial) {
    __shared__ uint32_t sl[8][256];
    __shared__ uint32_t st[4][256];
    __shared__ uint32_t red[kBlock];
    const int t = threadIdx.x;
    for (int i = t; i < 8 * 256; i += kBlock) (&sl[0][0])[i] = (&tabs->slice[0][0])[i];
    for (int i = t; i < 4 * 256; i += kBlock) (&st[0][0])[i] = (&tabs->tile[0][0])[i];
    __syncthreads();
    const size_t t0 = static_cast<size_t>(blockIdx.x) * tiles_per_wg;
    const size_t t1 = t0 + tiles_per_wg < n_tiles ? t0 + tiles_per_wg : n_tiles;
    uint32_t acc = 0;
    uint4 cur[4], nxt[4];
    auto load = [&](size_t tile, uint4 *v) {
        const uint4 *p = reinterpret_cast<const uint4 *>(data + tile * kCrcTile + static_cast<size_t>(t) * kCrcChunk);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = nt_load(p + k);
    };
    if (t0 < t1) load(t0, cur);
    for (size_t tile = t0; tile < t1; ++tile) {
        if (tile + 1 < t1) load(tile + 1, nxt); // next tile's loads in flight during this tile's table work
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t w[2] = {static_cast<uint64_t>(cur[k].x) | (static_cast<uint64_t>(cur[k].y) << 32),
                                   static_cast<uint64_t>(cur[k].z) | (static_cast<uint64_t>(cur[k].w) << 32)};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint64_t v = w[h] ^ c;
                c = sl[7][v & 0xff] ^ sl[6][(v >> 8) & 0xff] ^ sl[5][(v >> 16) & 0xff] ^ sl[4][(v >> 24) & 0xff] ^
                    sl[3][(v >> 32) & 0xff] ^ sl[2][(v >> 40) & 0xff] ^ sl[1][(v >> 48) & 0xff] ^ sl[0][v >> 56];
            }
        }
        acc = st[0][acc & 0xff] ^ st[1][(acc >> 8) & 0xff] ^ st[2][(acc >> 16) & 0xff] ^ st[3][acc >> 24];
        acc ^= c;
#pragma unroll
        for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
    }
    red[t] = acc;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int s = 1 << k;
        if ((t & (2 * s - 1)) == 0) red[t] = crc_gf_mul(red[t], lv.m[k]) ^ red[t + s];
        __syncthreads();
    }
    if (t == 0) partial[blockIdx.x] = red[0];
}

// reference test pattern (ccoip/tests/unit_tests/simple_hash/simplehash_cpu_test.cu:17-23), launched <<<8, 256>>>
template<int Unused = 0>
__global__ void k_test_pattern(uint64_t *data, size_t N) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nt = blockDim.x * gridDim.x;
    for (size_t i = tid; i < N; i += nt) data[i] = ((tid * nt) ^ (i & N)) * 0xaabaababab1ull;
}

} // namespace pccl::hipk
