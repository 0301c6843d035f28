#include <atomic>
#include <immintrin.h>
#include "host_kernels.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <limits>
#include <thread>
#include <vector>

#include "../common/log.hpp"
#include "elem.hpp"
#include "optim_common.hpp"

namespace pccl::kernels {

// ------------------------------------------------------------------------------------------------------------------
// reduce
// ------------------------------------------------------------------------------------------------------------------
template<typename E, typename Op>
static void reduce_loop(void *dst_v, const void *src_v, size_t n) {
    using S = typename E::S;
    using C = typename E::C;
    auto *__restrict dst = static_cast<S *>(dst_v);
    const auto *__restrict src = static_cast<const S *>(src_v);
    for (size_t i = 0; i < n; ++i) dst[i] = E::st(apply_op<Op, C>(E::ld(dst[i]), E::ld(src[i])));
}

template<typename E>
static bool reduce_op(void *dst, const void *src, size_t n, ReduceOp op) {
    switch (op) {
        case ReduceOp::Set: std::memmove(dst, src, n * sizeof(typename E::S)); return true;
        case ReduceOp::Sum:
        case ReduceOp::Avg: reduce_loop<E, OpSum>(dst, src, n); return true;
        case ReduceOp::Prod: reduce_loop<E, OpProd>(dst, src, n); return true;
        case ReduceOp::Max: reduce_loop<E, OpMax>(dst, src, n); return true;
        case ReduceOp::Min: reduce_loop<E, OpMin>(dst, src, n); return true;
    }
    return false;
}

bool host_reduce(void *dst, const void *src, size_t count, DType t, ReduceOp op) {
    // bf16 / fp32 sums take the AVX-512 body of host_reduce3 (element-wise: out may alias a)
    if ((op == ReduceOp::Sum || op == ReduceOp::Avg) && (t == DType::BF16 || t == DType::F32))
        return host_reduce3(dst, dst, src, count, t, op);
    switch (t) {
        case DType::F32: return reduce_op<EF32>(dst, src, count, op);
        case DType::F64: return reduce_op<EF64>(dst, src, count, op);
        case DType::BF16: return reduce_op<EBF16>(dst, src, count, op);
        case DType::F16: return reduce_op<EF16>(dst, src, count, op);
        case DType::U8: return reduce_op<EInt<uint8_t>>(dst, src, count, op);
        case DType::I8: return reduce_op<EInt<int8_t>>(dst, src, count, op);
        case DType::U16: return reduce_op<EInt<uint16_t>>(dst, src, count, op);
        case DType::I16: return reduce_op<EInt<int16_t>>(dst, src, count, op);
        case DType::U32: return reduce_op<EInt<uint32_t>>(dst, src, count, op);
        case DType::I32: return reduce_op<EInt<int32_t>>(dst, src, count, op);
        case DType::U64: return reduce_op<EInt<uint64_t>>(dst, src, count, op);
        case DType::I64: return reduce_op<EInt<int64_t>>(dst, src, count, op);
        default: break;
    }
    LOG(ERR) << "host_reduce: unsupported dtype " << dtype_name(t);
    return false;
}

template<typename E, typename Op>
static void reduce3_loop(void *out_v, const void *a_v, const void *b_v, size_t n) {
    using S = typename E::S;
    using C = typename E::C;
    auto *__restrict out = static_cast<S *>(out_v);
    const auto *__restrict a = static_cast<const S *>(a_v);
    const auto *__restrict b = static_cast<const S *>(b_v);
    for (size_t i = 0; i < n; ++i) out[i] = E::st(apply_op<Op, C>(E::ld(a[i]), E::ld(b[i])));
}

// bf16 sum, 16 lanes: widen to fp32 (<< 16), add, round to nearest even with NaN quieting exactly as
// num::f32_to_bf16, narrow. Returns the number of elements done (a multiple of 16).
__attribute__((target("avx512f,avx512bw"))) static size_t bf16_sum3_avx512(uint16_t *out, const uint16_t *a,
                                                                           const uint16_t *b, size_t n) {
    const __m512i abs_mask = _mm512_set1_epi32(0x7fffffff), inf = _mm512_set1_epi32(0x7f800000);
    const __m512i bias = _mm512_set1_epi32(0x7fff), one = _mm512_set1_epi32(1), quiet = _mm512_set1_epi32(0x40);
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const __m512i ai = _mm512_slli_epi32(_mm512_cvtepu16_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(a + i))), 16);
        const __m512i bi = _mm512_slli_epi32(_mm512_cvtepu16_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(b + i))), 16);
        const __m512i u = _mm512_castps_si512(_mm512_add_ps(_mm512_castsi512_ps(ai), _mm512_castsi512_ps(bi)));
        const __mmask16 nan = _mm512_cmpgt_epu32_mask(_mm512_and_si512(u, abs_mask), inf);
        const __m512i hi = _mm512_srli_epi32(u, 16);
        const __m512i rne = _mm512_srli_epi32(_mm512_add_epi32(u, _mm512_add_epi32(bias, _mm512_and_si512(hi, one))), 16);
        const __m512i r = _mm512_mask_blend_epi32(nan, rne, _mm512_or_si512(hi, quiet));
        _mm256_storeu_si256(reinterpret_cast<__m256i *>(out + i), _mm512_cvtepi32_epi16(r));
    }
    return i;
}

__attribute__((target("avx512f"))) static size_t f32_sum3_avx512(float *out, const float *a, const float *b, size_t n) {
    size_t i = 0;
    for (; i + 16 <= n; i += 16) _mm512_storeu_ps(out + i, _mm512_add_ps(_mm512_loadu_ps(a + i), _mm512_loadu_ps(b + i)));
    return i;
}

static bool cpu_has_avx512bw() {
    static const bool v = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
    return v;
}

template<typename E>
static bool reduce3_op(void *out, const void *a, const void *b, size_t n, ReduceOp op) {
    switch (op) {
        case ReduceOp::Set: std::memcpy(out, b, n * sizeof(typename E::S)); return true;
        case ReduceOp::Sum:
        case ReduceOp::Avg: reduce3_loop<E, OpSum>(out, a, b, n); return true;
        case ReduceOp::Prod: reduce3_loop<E, OpProd>(out, a, b, n); return true;
        case ReduceOp::Max: reduce3_loop<E, OpMax>(out, a, b, n); return true;
        case ReduceOp::Min: reduce3_loop<E, OpMin>(out, a, b, n); return true;
    }
    return false;
}

bool host_reduce3(void *out, const void *a, const void *b, size_t count, DType t, ReduceOp op) {
    const bool sum = op == ReduceOp::Sum || op == ReduceOp::Avg;
    size_t done = 0;
    if (sum && cpu_has_avx512bw()) {
        if (t == DType::BF16)
            done = bf16_sum3_avx512(static_cast<uint16_t *>(out), static_cast<const uint16_t *>(a),
                                    static_cast<const uint16_t *>(b), count);
        else if (t == DType::F32)
            done = f32_sum3_avx512(static_cast<float *>(out), static_cast<const float *>(a),
                                   static_cast<const float *>(b), count);
    }
    const size_t es = dtype_size(t);
    out = static_cast<uint8_t *>(out) + done * es;
    a = static_cast<const uint8_t *>(a) + done * es;
    b = static_cast<const uint8_t *>(b) + done * es;
    count -= done;
    switch (t) {
        case DType::F32: return reduce3_op<EF32>(out, a, b, count, op);
        case DType::F64: return reduce3_op<EF64>(out, a, b, count, op);
        case DType::BF16: return reduce3_op<EBF16>(out, a, b, count, op);
        case DType::F16: return reduce3_op<EF16>(out, a, b, count, op);
        case DType::U8: return reduce3_op<EInt<uint8_t>>(out, a, b, count, op);
        case DType::I8: return reduce3_op<EInt<int8_t>>(out, a, b, count, op);
        case DType::U16: return reduce3_op<EInt<uint16_t>>(out, a, b, count, op);
        case DType::I16: return reduce3_op<EInt<int16_t>>(out, a, b, count, op);
        case DType::U32: return reduce3_op<EInt<uint32_t>>(out, a, b, count, op);
        case DType::I32: return reduce3_op<EInt<int32_t>>(out, a, b, count, op);
        case DType::U64: return reduce3_op<EInt<uint64_t>>(out, a, b, count, op);
        case DType::I64: return reduce3_op<EInt<int64_t>>(out, a, b, count, op);
        default: break;
    }
    LOG(ERR) << "host_reduce3: unsupported dtype " << dtype_name(t);
    return false;
}

// ------------------------------------------------------------------------------------------------------------------
// min / max
// ------------------------------------------------------------------------------------------------------------------
template<typename E>
static void minmax_loop(const void *src_v, size_t n, double &mn, double &mx) {
    using S = typename E::S;
    const auto *src = static_cast<const S *>(src_v);
    double lo = std::numeric_limits<double>::infinity(), hi = -std::numeric_limits<double>::infinity();
    for (size_t i = 0; i < n; ++i) {
        const double v = static_cast<double>(E::ld(src[i]));
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    mn = n ? lo : 0.0;
    mx = n ? hi : 0.0;
}

void host_minmax(const void *src, size_t count, DType vtype, double &mn, double &mx) {
    switch (vtype) {
        case DType::F32: minmax_loop<EF32>(src, count, mn, mx); return;
        case DType::F64: minmax_loop<EF64>(src, count, mn, mx); return;
        case DType::BF16: minmax_loop<EBF16>(src, count, mn, mx); return;
        case DType::F16: minmax_loop<EF16>(src, count, mn, mx); return;
        default: mn = mx = 0; return;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// quantize / dequantize
// ------------------------------------------------------------------------------------------------------------------
template<typename E, typename Q>
static void quant_minmax_int(void *dst_v, const void *src_v, size_t n, const QuantParams &p) {
    const auto *src = static_cast<const typename E::S *>(src_v);
    auto *dst = static_cast<Q *>(dst_v);
    for (size_t i = 0; i < n; ++i) {
        const double q = q_minmax_int(static_cast<double>(E::ld(src[i])), p);
        if constexpr (std::is_same_v<Q, uint64_t>) {
            dst[i] = q >= 18446744073709551615.0 ? ~0ull : static_cast<uint64_t>(q);
        } else if constexpr (std::is_same_v<Q, int64_t>) {
            dst[i] = q >= 9223372036854775807.0 ? INT64_MAX : static_cast<int64_t>(q);
        } else {
            dst[i] = static_cast<Q>(static_cast<int64_t>(q));
        }
    }
}

template<typename E, bool E4M3>
static void quant_fp8(void *dst_v, const void *src_v, size_t n, const QuantParams &p) {
    const auto *src = static_cast<const typename E::S *>(src_v);
    auto *dst = static_cast<uint8_t *>(dst_v);
    for (size_t i = 0; i < n; ++i) {
        const float x = static_cast<float>(E::ld(src[i])) * p.f8_scale;
        dst[i] = E4M3 ? num::f32_to_fp8e4m3(x) : num::f32_to_fp8e5m2(x);
    }
}

template<typename E, typename Q>
static void quant_zps(void *dst_v, const void *src_v, size_t n, const QuantParams &p) {
    const auto *src = static_cast<const typename E::S *>(src_v);
    auto *dst = static_cast<Q *>(dst_v);
    for (size_t i = 0; i < n; ++i) dst[i] = q_zps_as<Q>(static_cast<float>(E::ld(src[i])), p);
}

template<typename E, typename Op, typename Q>
static void dq_minmax_int_loop(void *dst_v, const void *src_v, size_t n, const QuantParams &p) {
    using C = typename E::C;
    auto *dst = static_cast<typename E::S *>(dst_v);
    const auto *src = static_cast<const Q *>(src_v);
    for (size_t i = 0; i < n; ++i) {
        const C v = static_cast<C>(dq_minmax_int(static_cast<double>(src[i]), p));
        dst[i] = E::st(apply_op<Op, C>(E::ld(dst[i]), v));
    }
}

template<typename E, typename Op, bool E4M3>
static void dq_fp8_loop(void *dst_v, const void *src_v, size_t n, const QuantParams &p) {
    using C = typename E::C;
    auto *dst = static_cast<typename E::S *>(dst_v);
    const auto *src = static_cast<const uint8_t *>(src_v);
    for (size_t i = 0; i < n; ++i) {
        const float f = (E4M3 ? num::fp8e4m3_to_f32(src[i]) : num::fp8e5m2_to_f32(src[i])) * p.f8_inv;
        dst[i] = E::st(apply_op<Op, C>(E::ld(dst[i]), static_cast<C>(f)));
    }
}

template<typename E, typename Op, typename Q>
static void dq_zps_loop(void *dst_v, const void *src_v, size_t n, const QuantParams &p) {
    using C = typename E::C;
    auto *dst = static_cast<typename E::S *>(dst_v);
    const auto *src = static_cast<const Q *>(src_v);
    for (size_t i = 0; i < n; ++i) {
        const float f = dq_zps_as<Q>(src[i], p);
        dst[i] = E::st(apply_op<Op, C>(E::ld(dst[i]), static_cast<C>(f)));
    }
}

template<typename E>
static bool quantize_v(void *dst_q, const void *src, size_t n, DType qtype, const QuantParams &p) {
    if (p.algo == QuantAlgo::MinMax) {
        switch (qtype) {
            case DType::U8: quant_minmax_int<E, uint8_t>(dst_q, src, n, p); return true;
            case DType::I8: quant_minmax_int<E, int8_t>(dst_q, src, n, p); return true;
            case DType::U16: quant_minmax_int<E, uint16_t>(dst_q, src, n, p); return true;
            case DType::I16: quant_minmax_int<E, int16_t>(dst_q, src, n, p); return true;
            case DType::U32: quant_minmax_int<E, uint32_t>(dst_q, src, n, p); return true;
            case DType::I32: quant_minmax_int<E, int32_t>(dst_q, src, n, p); return true;
            case DType::U64: quant_minmax_int<E, uint64_t>(dst_q, src, n, p); return true;
            case DType::I64: quant_minmax_int<E, int64_t>(dst_q, src, n, p); return true;
            case DType::F8E4M3: quant_fp8<E, true>(dst_q, src, n, p); return true;
            case DType::F8E5M2: quant_fp8<E, false>(dst_q, src, n, p); return true;
            default: return false;
        }
    }
    if (p.algo == QuantAlgo::ZeroPointScale) {
        switch (qtype) {
            case DType::U8: quant_zps<E, uint8_t>(dst_q, src, n, p); return true;
            case DType::I8: quant_zps<E, int8_t>(dst_q, src, n, p); return true;
            case DType::U16: quant_zps<E, uint16_t>(dst_q, src, n, p); return true;
            case DType::I16: quant_zps<E, int16_t>(dst_q, src, n, p); return true;
            case DType::U32: quant_zps<E, uint32_t>(dst_q, src, n, p); return true;
            case DType::I32: quant_zps<E, int32_t>(dst_q, src, n, p); return true;
            case DType::U64: quant_zps<E, uint64_t>(dst_q, src, n, p); return true;
            case DType::I64: quant_zps<E, int64_t>(dst_q, src, n, p); return true;
            default: return false;
        }
    }
    return false;
}

bool host_quantize_params(void *dst_q, const void *src, size_t count, DType vtype, DType qtype, const QuantParams &p) {
    switch (vtype) {
        case DType::F32: return quantize_v<EF32>(dst_q, src, count, qtype, p);
        case DType::F64: return quantize_v<EF64>(dst_q, src, count, qtype, p);
        case DType::BF16: return quantize_v<EBF16>(dst_q, src, count, qtype, p);
        case DType::F16: return quantize_v<EF16>(dst_q, src, count, qtype, p);
        default: return false;
    }
}

proto::QuantMeta host_quantize(void *dst_q, const void *src, size_t count, DType vtype, DType qtype, QuantAlgo algo) {
    double mn = 0, mx = 0;
    host_minmax(src, count, vtype, mn, mx);
    proto::QuantMeta meta = make_meta(algo, vtype, qtype, mn, mx);
    const bool ok = host_quantize_params(dst_q, src, count, vtype, qtype, make_params(meta, qtype));
    if (!ok) {
        LOG(ERR) << "host_quantize: unsupported combination " << dtype_name(vtype) << " -> " << dtype_name(qtype);
    }
    return meta;
}

template<typename E, typename Op>
static bool dequant_v(void *dst, const void *src_q, size_t n, DType qtype, const QuantParams &p) {
    if (p.algo == QuantAlgo::MinMax) {
        switch (qtype) {
            case DType::U8: dq_minmax_int_loop<E, Op, uint8_t>(dst, src_q, n, p); return true;
            case DType::I8: dq_minmax_int_loop<E, Op, int8_t>(dst, src_q, n, p); return true;
            case DType::U16: dq_minmax_int_loop<E, Op, uint16_t>(dst, src_q, n, p); return true;
            case DType::I16: dq_minmax_int_loop<E, Op, int16_t>(dst, src_q, n, p); return true;
            case DType::U32: dq_minmax_int_loop<E, Op, uint32_t>(dst, src_q, n, p); return true;
            case DType::I32: dq_minmax_int_loop<E, Op, int32_t>(dst, src_q, n, p); return true;
            case DType::U64: dq_minmax_int_loop<E, Op, uint64_t>(dst, src_q, n, p); return true;
            case DType::I64: dq_minmax_int_loop<E, Op, int64_t>(dst, src_q, n, p); return true;
            case DType::F8E4M3: dq_fp8_loop<E, Op, true>(dst, src_q, n, p); return true;
            case DType::F8E5M2: dq_fp8_loop<E, Op, false>(dst, src_q, n, p); return true;
            default: return false;
        }
    }
    if (p.algo == QuantAlgo::ZeroPointScale) {
        switch (qtype) {
            case DType::U8: dq_zps_loop<E, Op, uint8_t>(dst, src_q, n, p); return true;
            case DType::I8: dq_zps_loop<E, Op, int8_t>(dst, src_q, n, p); return true;
            case DType::U16: dq_zps_loop<E, Op, uint16_t>(dst, src_q, n, p); return true;
            case DType::I16: dq_zps_loop<E, Op, int16_t>(dst, src_q, n, p); return true;
            case DType::U32: dq_zps_loop<E, Op, uint32_t>(dst, src_q, n, p); return true;
            case DType::I32: dq_zps_loop<E, Op, int32_t>(dst, src_q, n, p); return true;
            case DType::U64: dq_zps_loop<E, Op, uint64_t>(dst, src_q, n, p); return true;
            case DType::I64: dq_zps_loop<E, Op, int64_t>(dst, src_q, n, p); return true;
            default: return false;
        }
    }
    return false;
}

template<typename E>
static bool dequant_op(void *dst, const void *src_q, size_t n, DType qtype, ReduceOp op, const QuantParams &p) {
    switch (op) {
        case ReduceOp::Set: return dequant_v<E, OpSet>(dst, src_q, n, qtype, p);
        case ReduceOp::Sum:
        case ReduceOp::Avg: return dequant_v<E, OpSum>(dst, src_q, n, qtype, p);
        case ReduceOp::Prod: return dequant_v<E, OpProd>(dst, src_q, n, qtype, p);
        case ReduceOp::Max: return dequant_v<E, OpMax>(dst, src_q, n, qtype, p);
        case ReduceOp::Min: return dequant_v<E, OpMin>(dst, src_q, n, qtype, p);
    }
    return false;
}

bool host_dequant_reduce(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                         const proto::QuantMeta &meta) {
    return host_dequant_reduce_params(dst, src_q, count, vtype, qtype, op, make_params(meta, qtype));
}

bool host_dequant_reduce_params(void *dst, const void *src_q, size_t count, DType vtype, DType qtype, ReduceOp op,
                                const QuantParams &p) {
    switch (vtype) {
        case DType::F32: return dequant_op<EF32>(dst, src_q, count, qtype, op, p);
        case DType::F64: return dequant_op<EF64>(dst, src_q, count, qtype, op, p);
        case DType::BF16: return dequant_op<EBF16>(dst, src_q, count, qtype, op, p);
        case DType::F16: return dequant_op<EF16>(dst, src_q, count, qtype, op, p);
        default: return false;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// AVG finalization
// ------------------------------------------------------------------------------------------------------------------
template<typename E>
static void avg_loop(void *dst_v, size_t n, size_t ws) {
    using C = typename E::C;
    auto *dst = static_cast<typename E::S *>(dst_v);
    const C w = static_cast<C>(ws);
    for (size_t i = 0; i < n; ++i) dst[i] = E::st(static_cast<C>(E::ld(dst[i]) / w));
}

bool host_finalize_avg(void *dst, size_t count, DType t, size_t ws) {
    if (ws == 0) return false;
    switch (t) {
        case DType::F32: avg_loop<EF32>(dst, count, ws); return true;
        case DType::F64: avg_loop<EF64>(dst, count, ws); return true;
        case DType::BF16: avg_loop<EBF16>(dst, count, ws); return true;
        case DType::F16: avg_loop<EF16>(dst, count, ws); return true;
        case DType::U8: avg_loop<EInt<uint8_t>>(dst, count, ws); return true;
        case DType::I8: avg_loop<EInt<int8_t>>(dst, count, ws); return true;
        case DType::U16: avg_loop<EInt<uint16_t>>(dst, count, ws); return true;
        case DType::I16: avg_loop<EInt<int16_t>>(dst, count, ws); return true;
        case DType::U32: avg_loop<EInt<uint32_t>>(dst, count, ws); return true;
        case DType::I32: avg_loop<EInt<int32_t>>(dst, count, ws); return true;
        case DType::U64: avg_loop<EInt<uint64_t>>(dst, count, ws); return true;
        case DType::I64: avg_loop<EInt<int64_t>>(dst, count, ws); return true;
        default: return false;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// simplehash (host emulation of the 960 x 256 launch, 32-lane shuffle trees)
// ------------------------------------------------------------------------------------------------------------------
static inline uint32_t hc(uint32_t a, uint32_t b) {
    a ^= b + 0x9e3779b1u;
    a = (a << 7) | (a >> 25);
    return a * 0x85ebca6bu;
}

static uint32_t tree32(uint32_t *t) { // in-place 32-lane shuffle-down tree; returns lane 0
    for (int off = 16; off > 0; off >>= 1)
        for (int i = 0; i < off; ++i) t[i] = hc(t[i], t[i + off]);
    return t[0];
}

static uint32_t tree256(const uint32_t *acc) {
    uint32_t warps[32] = {0};
    uint32_t tmp[32];
    for (int w = 0; w < 8; ++w) {
        std::memcpy(tmp, acc + w * 32, sizeof(tmp));
        warps[w] = tree32(tmp);
    }
    return tree32(warps);
}

static uint32_t hash_block(const uint32_t *words, size_t n_vec, size_t vpb, size_t b) {
    const size_t start = b * vpb;
    const size_t end = std::min(start + vpb, n_vec);
    uint32_t acc[256] = {0};
    for (size_t i = start; i < end; i += 256) {
        const size_t m = std::min<size_t>(256, end - i);
        const uint32_t *v = words + i * 4;
        for (size_t t = 0; t < m; ++t) {
            uint32_t a = acc[t];
            a = hc(a, v[t * 4 + 0]);
            a = hc(a, v[t * 4 + 1]);
            a = hc(a, v[t * 4 + 2]);
            a = hc(a, v[t * 4 + 3]);
            acc[t] = a;
        }
    }
    return tree256(acc);
}

uint32_t simplehash_host(const void *data, size_t n_bytes) {
    if (n_bytes == 0) return 0;
    const auto *words = static_cast<const uint32_t *>(data);
    const size_t n_words = n_bytes / 4;
    const size_t n_vec = n_words / 4;
    size_t grid = (n_vec + 255) / 256;
    if (grid > 960) grid = 960;
    uint32_t h = 0;
    if (grid > 0) {
        const size_t vpb = (n_vec + grid - 1) / grid;
        std::vector<uint32_t> partial(grid);
        const size_t hw = std::max<size_t>(1, std::thread::hardware_concurrency() / 2);
        const size_t n_threads = n_bytes >= (32u << 20) ? std::min<size_t>(hw, grid) : 1;
        if (n_threads <= 1) {
            for (size_t b = 0; b < grid; ++b) partial[b] = hash_block(words, n_vec, vpb, b);
        } else {
            std::vector<std::thread> ts;
            for (size_t t = 0; t < n_threads; ++t)
                ts.emplace_back([&, t] {
                    for (size_t b = t; b < grid; b += n_threads) partial[b] = hash_block(words, n_vec, vpb, b);
                });
            for (auto &t : ts) t.join();
        }
        uint32_t fin[256] = {0};
        for (size_t b = 0; b < grid; ++b) fin[b % 256] = hc(fin[b % 256], partial[b]);
        h = tree256(fin);
    }
    for (size_t i = n_vec * 4; i < n_words; ++i) h = hc(h, words[i]);
    const size_t tail = n_bytes % 4;
    if (tail) {
        const auto *bytes = static_cast<const uint8_t *>(data) + n_words * 4;
        uint32_t v = 0;
        for (size_t i = 0; i < tail; ++i) v |= static_cast<uint32_t>(bytes[i]) << (8 * i);
        h = hc(h, v);
    }
    return h;
}

// ------------------------------------------------------------------------------------------------------------------
// CRC-32C
// ------------------------------------------------------------------------------------------------------------------
static uint32_t g_crc_table[8][256];
static uint32_t g_x2n[64]; // x^(2^k) mod P
static std::once_flag g_crc_once;
static bool g_spoof_no_hw = false;
static constexpr uint32_t kCrcPoly = 0x82F63B78u;

static void crc_init() {
    std::call_once(g_crc_once, [] {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : (c >> 1);
            g_crc_table[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int t = 1; t < 8; ++t)
                g_crc_table[t][i] = (g_crc_table[t - 1][i] >> 8) ^ g_crc_table[0][g_crc_table[t - 1][i] & 0xff];
        g_x2n[0] = 1u << 30; // x^1
        for (int k = 1; k < 64; ++k) g_x2n[k] = crc32c_gf_mul(g_x2n[k - 1], g_x2n[k - 1]);
    });
}

const uint32_t (*crc32c_tables())[256] {
    crc_init();
    return g_crc_table;
}

uint32_t crc32c_gf_mul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 31; i >= 0; --i) { // bit 31 of a is x^0
        p ^= (0u - ((a >> i) & 1u)) & b;
        b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
    }
    return p;
}

uint32_t crc32c_x8n(uint64_t n) {
    crc_init();
    uint32_t p = 1u << 31; // x^0
    for (int k = 3; n; n >>= 1, ++k) // x^(8n) = prod over set bits j of n of x^(2^(j+3))
        if (n & 1) p = crc32c_gf_mul(g_x2n[k & 63], p);
    return p;
}

uint32_t crc32c_raw_update(uint32_t c, const void *data, size_t n) {
    crc_init();
    const auto *p = static_cast<const uint8_t *>(data);
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        v ^= c;
        c = g_crc_table[7][v & 0xff] ^ g_crc_table[6][(v >> 8) & 0xff] ^ g_crc_table[5][(v >> 16) & 0xff] ^
            g_crc_table[4][(v >> 24) & 0xff] ^ g_crc_table[3][(v >> 32) & 0xff] ^ g_crc_table[2][(v >> 40) & 0xff] ^
            g_crc_table[1][(v >> 48) & 0xff] ^ g_crc_table[0][v >> 56];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ g_crc_table[0][(c ^ *p++) & 0xff];
    return c;
}

uint32_t crc32c_sw(const void *data, size_t n) {
    crc_init();
    const auto *p = static_cast<const uint8_t *>(data);
    uint32_t c = 0xffffffffu;
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        v ^= c;
        c = g_crc_table[7][v & 0xff] ^ g_crc_table[6][(v >> 8) & 0xff] ^ g_crc_table[5][(v >> 16) & 0xff] ^
            g_crc_table[4][(v >> 24) & 0xff] ^ g_crc_table[3][(v >> 32) & 0xff] ^ g_crc_table[2][(v >> 40) & 0xff] ^
            g_crc_table[1][(v >> 48) & 0xff] ^ g_crc_table[0][v >> 56];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ g_crc_table[0][(c ^ *p++) & 0xff];
    return ~c;
}

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const void *data, size_t n) {
    const auto *p = static_cast<const uint8_t *>(data);
    uint64_t c = 0xffffffffu;
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        c = __builtin_ia32_crc32di(c, v);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = static_cast<uint32_t>(c);
    while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
    return ~c32;
}

// Three interleaved crc32q chains (latency 3, throughput 1 per cycle: one chain leaves the unit 2/3 idle) over three
// consecutive lanes of each 3 x 8 KiB block, joined with the split algebra: state = shift(c0, 2L) ^ shift(c1, L) ^ c2.
// The two shifts are multiplications by constants, done with 4-entry byte tables (the reference uses PCLMUL for
// this step, crc32_amd64_sse42_pcmul.cpp).
namespace {
constexpr size_t kCrcLane = 8192;
struct ConstMul {
    uint32_t t[4][256];
    explicit ConstMul(uint32_t m) {
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 0; b < 256; ++b) t[k][b] = crc32c_gf_mul(m, b << (8 * k));
    }
    uint32_t operator()(uint32_t c) const {
        return t[0][c & 0xff] ^ t[1][(c >> 8) & 0xff] ^ t[2][(c >> 16) & 0xff] ^ t[3][c >> 24];
    }
};
} // namespace

__attribute__((target("sse4.2"))) uint32_t crc32c_hw3(const void *data, size_t n) {
    static const ConstMul by_lane(crc32c_x8n(kCrcLane)), by_2lanes(crc32c_x8n(2 * kCrcLane));
    const auto *p = static_cast<const uint8_t *>(data);
    uint64_t c0 = 0xffffffffu;
    while (n >= 3 * kCrcLane) {
        uint64_t c1 = 0, c2 = 0;
        for (size_t i = 0; i < kCrcLane; i += 8) {
            uint64_t a, b, d;
            std::memcpy(&a, p + i, 8);
            std::memcpy(&b, p + kCrcLane + i, 8);
            std::memcpy(&d, p + 2 * kCrcLane + i, 8);
            c0 = __builtin_ia32_crc32di(c0, a);
            c1 = __builtin_ia32_crc32di(c1, b);
            c2 = __builtin_ia32_crc32di(c2, d);
        }
        c0 = by_2lanes(static_cast<uint32_t>(c0)) ^ by_lane(static_cast<uint32_t>(c1)) ^ static_cast<uint32_t>(c2);
        p += 3 * kCrcLane;
        n -= 3 * kCrcLane;
    }
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        c0 = __builtin_ia32_crc32di(c0, v);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = static_cast<uint32_t>(c0);
    while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
    return ~c32;
}

// PCLMUL combine (reference crc32_amd64_sse42_pcmul.cpp): shifting a CRC by L bytes is a multiplication by a
// constant; one carry-less multiply of the 32-bit CRC by a 64-bit constant K followed by one crc32q of the product
// gives it. K is not hard-coded: g_K(c) = crc32q(0, clmul(c, K)) is linear in K and in c, so K is solved at first use
// from the 32 x 32 equations g_K(e_i) = shift(e_i, L) by Gaussian elimination over GF(2) (and checked).
namespace {
// fold with a 128-bit product: crc32q over the low qword, then xor in the high qword's contribution
__attribute__((target("sse4.2,pclmul"))) uint32_t clmul_apply(uint32_t c, uint64_t k) {
    const __m128i prod = _mm_clmulepi64_si128(_mm_cvtsi32_si128(static_cast<int>(c)), _mm_cvtsi64_si128(static_cast<long long>(k)), 0x00);
    const uint64_t lo = static_cast<uint64_t>(_mm_cvtsi128_si64(prod));
    const uint64_t hi = static_cast<uint64_t>(_mm_extract_epi64(prod, 1));
    return static_cast<uint32_t>(_mm_crc32_u64(0, lo)) ^ static_cast<uint32_t>(hi);
}

struct ClmulConst {
    uint64_t k = 0;
    bool ok = false;
};

// solves g_K = shift(., bytes) for K (64 unknown bits); needs pclmul + sse4.2 at run time
__attribute__((target("sse4.2,pclmul"))) ClmulConst solve_clmul_const(uint64_t bytes) {
    const uint32_t m = crc32c_x8n(bytes);
    // equations: for every input bit i (c = 1 << i) and output bit r: xor_j K_j * bit_r(g_{e_j}(e_i)) = bit_r(f(e_i))
    std::vector<std::pair<uint64_t, int>> rows; // (coefficients over the 64 K bits, rhs)
    for (int i = 0; i < 32; ++i) {
        uint32_t col[64];
        for (int j = 0; j < 64; ++j) col[j] = clmul_apply(1u << i, 1ull << j);
        const uint32_t want = crc32c_gf_mul(m, 1u << i);
        for (int r = 0; r < 32; ++r) {
            uint64_t coef = 0;
            for (int j = 0; j < 64; ++j) coef |= static_cast<uint64_t>((col[j] >> r) & 1u) << j;
            rows.emplace_back(coef, static_cast<int>((want >> r) & 1u));
        }
    }
    ClmulConst out;
    // Gauss-Jordan elimination
    size_t rank = 0;
    std::vector<int> pivot_col;
    for (int col = 0; col < 64 && rank < rows.size(); ++col) {
        size_t piv = rank;
        while (piv < rows.size() && !((rows[piv].first >> col) & 1)) ++piv;
        if (piv == rows.size()) continue;
        std::swap(rows[piv], rows[rank]);
        for (size_t r = 0; r < rows.size(); ++r)
            if (r != rank && ((rows[r].first >> col) & 1)) {
                rows[r].first ^= rows[rank].first;
                rows[r].second ^= rows[rank].second;
            }
        pivot_col.push_back(col);
        ++rank;
    }
    for (size_t r = rank; r < rows.size(); ++r)
        if (rows[r].second) return out; // inconsistent: no such K
    for (size_t r = 0; r < rank; ++r)
        if (rows[r].second) out.k |= 1ull << pivot_col[r];
    for (int i = 0; i < 32; ++i) // verify on the basis
        if (clmul_apply(1u << i, out.k) != crc32c_gf_mul(m, 1u << i)) return out;
    out.ok = true;
    return out;
}
} // namespace

static const ClmulConst &clmul_lane(int k) {
    static const ClmulConst by_lane = solve_clmul_const(kCrcLane), by_2lanes = solve_clmul_const(2 * kCrcLane);
    return k == 1 ? by_lane : by_2lanes;
}

bool crc32c_clmul_ready() {
    return __builtin_cpu_supports("sse4.2") && __builtin_cpu_supports("pclmul") && clmul_lane(1).ok && clmul_lane(2).ok;
}

__attribute__((target("sse4.2,pclmul"))) uint32_t crc32c_hw3_clmul(const void *data, size_t n) {
    const ClmulConst &by_lane = clmul_lane(1), &by_2lanes = clmul_lane(2);
    if (!by_lane.ok || !by_2lanes.ok) return crc32c_hw3(data, n);
    const auto *p = static_cast<const uint8_t *>(data);
    uint64_t c0 = 0xffffffffu;
    while (n >= 3 * kCrcLane) {
        uint64_t c1 = 0, c2 = 0;
        for (size_t i = 0; i < kCrcLane; i += 8) {
            uint64_t a, b, d;
            std::memcpy(&a, p + i, 8);
            std::memcpy(&b, p + kCrcLane + i, 8);
            std::memcpy(&d, p + 2 * kCrcLane + i, 8);
            c0 = _mm_crc32_u64(c0, a);
            c1 = _mm_crc32_u64(c1, b);
            c2 = _mm_crc32_u64(c2, d);
        }
        c0 = clmul_apply(static_cast<uint32_t>(c0), by_2lanes.k) ^ clmul_apply(static_cast<uint32_t>(c1), by_lane.k) ^
             static_cast<uint32_t>(c2);
        p += 3 * kCrcLane;
        n -= 3 * kCrcLane;
    }
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        c0 = _mm_crc32_u64(c0, v);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = static_cast<uint32_t>(c0);
    while (n--) c32 = _mm_crc32_u8(c32, *p++);
    return ~c32;
}

// Runtime dispatch with spoofable CPU features (reference crc32_cpu.cpp + crc32_cpu_test.cpp:139-185): tests force a
// lower tier to check every implementation on one machine.
static std::atomic<int> g_crc_tier_cap{3};

int crc32c_tier() {
    int t = 0;
    if (!g_spoof_no_hw && __builtin_cpu_supports("sse4.2")) t = __builtin_cpu_supports("pclmul") ? 2 : 1;
    return std::min(t, g_crc_tier_cap.load(std::memory_order_relaxed));
}

void crc32c_spoof_tier(int max_tier) { g_crc_tier_cap.store(max_tier < 0 ? 3 : max_tier, std::memory_order_relaxed); }

bool crc32c_has_hw() { return crc32c_tier() >= 1; }

void crc32c_spoof_no_hw(bool no_hw) { g_spoof_no_hw = no_hw; }

uint32_t crc32c(const void *data, size_t n) {
    switch (crc32c_tier()) {
        case 2: return crc32c_hw3_clmul(data, n);
        case 1: return crc32c_hw3(data, n);
        default: return crc32c_sw(data, n);
    }
}


// ------------------------------------------------------------------------------------------------------------------
// DiLoCo outer step (host twin of hip_optim.hip)
// ------------------------------------------------------------------------------------------------------------------
template<typename F>
static void host_parallel(size_t count, F &&body) {
    constexpr size_t kMinPerThread = 1 << 20;
    const size_t hw = std::max<size_t>(1, std::thread::hardware_concurrency());
    const size_t nt = std::min(hw, std::max<size_t>(1, count / kMinPerThread));
    if (nt <= 1) {
        body(size_t{0}, count);
        return;
    }
    std::vector<std::thread> ts;
    const size_t per = (count + nt - 1) / nt;
    for (size_t k = 0; k < nt; ++k) {
        const size_t lo = k * per, hi = std::min(count, lo + per);
        if (lo < hi) ts.emplace_back([&, lo, hi] { body(lo, hi); });
    }
    for (auto &th : ts) th.join();
}

template<typename E>
static void pg_loop(float *pg, const float *outer, const void *local, size_t count) {
    const auto *l = static_cast<const typename E::S *>(local);
    host_parallel(count, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) pg[i] = outer[i] - static_cast<float>(E::ld(l[i]));
    });
}

template<typename E>
static void sgd_loop(float *outer, float *mom, const float *pg, void *local, size_t count, const OuterSgdParams &p) {
    auto *l = static_cast<typename E::S *>(local);
    host_parallel(count, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            outer_sgd_elem(outer[i], mom[i], pg[i], p);
            l[i] = E::st(outer[i]);
        }
    });
}

bool host_pseudo_grad(float *pg, const float *outer, const void *local, size_t count, DType local_t) {
    switch (local_t) {
        case DType::F32: pg_loop<EF32>(pg, outer, local, count); return true;
        case DType::BF16: pg_loop<EBF16>(pg, outer, local, count); return true;
        case DType::F16: pg_loop<EF16>(pg, outer, local, count); return true;
        default: return false;
    }
}

bool host_outer_sgd(float *outer, float *mom, const float *pg, void *local, size_t count, DType local_t,
                    const OuterSgdParams &p) {
    switch (local_t) {
        case DType::F32: sgd_loop<EF32>(outer, mom, pg, local, count, p); return true;
        case DType::BF16: sgd_loop<EBF16>(outer, mom, pg, local, count, p); return true;
        case DType::F16: sgd_loop<EF16>(outer, mom, pg, local, count, p); return true;
        default: return false;
    }
}

} // namespace pccl::kernels
