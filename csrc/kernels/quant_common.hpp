// Quantization parameter math shared by the host kernels and the HIP kernels.
//
// Every peer must (de)quantize bit-identically, CPU or GPU. The scalar formulas below are the single definition; the
// host computes the per-chunk parameters (QuantParams) from the chunk statistics once, and both the SIMD host loops
// and the HIP kernels evaluate exactly these expressions (compiled with -ffp-contract=off on both sides).
//
// Algorithms (per ring-step chunk):
//  * MIN_MAX, integer wire type Q in [qlo, qhi]:  q = qlo + clamp(floor((x - min) * inv_dif * range + 0.5), 0, range)
//        dequant: x' = min + (q - qlo) * step          (step = dif / range; all in double)
//    Reference behaviour truncated instead of rounding — fixed here deliberately.
//  * MIN_MAX, fp8 wire type (e4m3 / e5m2): absmax scaling q = fp8(x * s), x' = float(q) * inv_s (float math),
//        s = FP8_MAX / max(|min|, |max|).
//  * ZERO_POINT_SCALE (integer wire types): scale = (max - min) / (qhi - qlo), zp = clamp(rint(qlo - min / scale)),
//        q = clamp(rint(x * inv_scale) + zp, qlo, qhi), x' = (q - zp) * scale (float math). The reference delegates
//        this to the absent piquant library; parity with piquant is unpinned. 64-bit wire types: the clamp and the
//        de-quantize difference run in double (their ranges fit neither int64 nor float), and zp (an int64 on the
//        wire, as in the reference's DeQuantizationMetaData) is additionally clamped to the int64 range.
// The 64-bit ranges end at the largest doubles below 2^64 / 2^63, so every clamped value converts without overflow.
#pragma once

#include <cmath>
#include <cstdint>

#include "../common/numeric.hpp"
#include "../common/types.hpp"
#include "../proto/packets.hpp"

namespace pccl::kernels {

struct QuantParams {
    QuantAlgo algo = QuantAlgo::None;
    DType qtype = DType::U8;
    // integer min-max
    double min = 0, inv_dif = 0, range = 0, step = 0, qlo = 0;
    // fp8
    float f8_scale = 1.0f, f8_inv = 1.0f;
    // zero-point-scale
    float zps_scale = 1.0f, zps_inv = 1.0f;
    int64_t zp = 0;
    int64_t ilo = 0, ihi = 0; // <= 32-bit wire types
    double dlo = 0, dhi = 0;  // 64-bit wire types
};

inline void int_range(DType q, double &lo, double &hi) {
    switch (q) {
        case DType::U8: lo = 0; hi = 255; break;
        case DType::I8: lo = -128; hi = 127; break;
        case DType::U16: lo = 0; hi = 65535; break;
        case DType::I16: lo = -32768; hi = 32767; break;
        case DType::U32: lo = 0; hi = 4294967295.0; break;
        case DType::I32: lo = -2147483648.0; hi = 2147483647.0; break;
        case DType::U64: lo = 0; hi = 18446744073709549568.0; break;                    // 2^64 - 2048
        case DType::I64: lo = -9223372036854775808.0; hi = 9223372036854774784.0; break; // 2^63 - 1024
        default: lo = 0; hi = 255; break;
    }
}

inline bool is_fp8(DType t) { return t == DType::F8E4M3 || t == DType::F8E5M2; }

inline bool quant_supported(DType vtype, DType qtype, QuantAlgo algo) {
    if (algo == QuantAlgo::None) return vtype == qtype;
    const bool vfloat = vtype == DType::F32 || vtype == DType::F64 || vtype == DType::BF16 || vtype == DType::F16;
    if (!vfloat) return false;
    if (algo == QuantAlgo::MinMax) return is_fp8(qtype) || (!dtype_is_float(qtype));
    if (algo == QuantAlgo::ZeroPointScale) return !dtype_is_float(qtype);
    return false;
}

// Build dequantization parameters from the wire metadata.
inline QuantParams make_params(const proto::QuantMeta &m, DType qtype) {
    QuantParams p;
    p.algo = m.algo;
    p.qtype = qtype;
    if (m.algo == QuantAlgo::MinMax) {
        if (is_fp8(qtype)) {
            const double amax = std::fmax(std::fabs(m.min_value), std::fabs(m.max_value));
            const double fmaxv = qtype == DType::F8E4M3 ? 448.0 : 57344.0;
            p.f8_scale = amax > 0 ? static_cast<float>(fmaxv / amax) : 1.0f;
            p.f8_inv = amax > 0 ? static_cast<float>(amax / fmaxv) : 1.0f;
        } else {
            double lo, hi;
            int_range(qtype, lo, hi);
            p.qlo = lo;
            p.range = hi - lo;
            p.min = m.min_value;
            const double dif = m.max_value - m.min_value;
            p.inv_dif = dif != 0.0 ? 1.0 / dif : 0.0;
            p.step = dif / p.range;
        }
    } else if (m.algo == QuantAlgo::ZeroPointScale) {
        double lo, hi;
        int_range(qtype, lo, hi);
        if (dtype_size(qtype) <= 4) {
            p.ilo = static_cast<int64_t>(lo);
            p.ihi = static_cast<int64_t>(hi);
        }
        p.dlo = lo;
        p.dhi = hi;
        p.zps_scale = m.scale;
        p.zps_inv = m.scale != 0.0f ? 1.0f / m.scale : 1.0f;
        p.zp = m.zero_point;
    }
    return p;
}

// Build metadata (what is sent on the wire) from chunk statistics.
inline proto::QuantMeta make_meta(QuantAlgo algo, DType vtype, DType qtype, double mn, double mx) {
    proto::QuantMeta m;
    m.algo = algo;
    m.value_type = vtype;
    m.min_value = mn;
    m.max_value = mx;
    if (algo == QuantAlgo::ZeroPointScale) {
        double lo, hi;
        int_range(qtype, lo, hi);
        float scale = static_cast<float>((mx - mn) / (hi - lo));
        if (!(scale > 0.0f) || !std::isfinite(scale)) scale = 1.0f;
        // uint64 wire type: the zero point travels as an int64; data reaching far below zero would need a larger
        // one, so the scale grows until it fits (the code then spans at least half of the uint64 range)
        constexpr double kZpMax = 9223372036854774784.0; // largest double below 2^63
        if (lo - mn / static_cast<double>(scale) > kZpMax)
            scale = static_cast<float>(-mn / kZpMax * (1.0 + 1.0 / (1 << 20)));
        double zp = std::nearbyint(lo - mn / static_cast<double>(scale));
        if (zp < lo) zp = lo;
        if (zp > hi) zp = hi;
        if (zp > kZpMax) zp = kZpMax;
        m.scale = scale;
        m.zero_point = static_cast<int64_t>(zp);
    }
    return m;
}

// ---- scalar element functions (identical expressions on host and device) ----
PCCL_HD double q_minmax_int(double x, const QuantParams &p) {
    double r = (x - p.min) * p.inv_dif * p.range + 0.5;
    r = r < 0.0 ? 0.0 : r;
    r = r > p.range ? p.range : r;
    r = __builtin_floor(r);
    return r + p.qlo;
}
PCCL_HD double dq_minmax_int(double q, const QuantParams &p) { return p.min + (q - p.qlo) * p.step; }

PCCL_HD int64_t q_zps(float x, const QuantParams &p) {
    float r = __builtin_rintf(x * p.zps_inv);
    // clamp in float domain first to avoid UB on conversion
    const float lo = static_cast<float>(p.ilo - p.zp), hi = static_cast<float>(p.ihi - p.zp);
    r = r < lo ? lo : r;
    r = r > hi ? hi : r;
    int64_t q = static_cast<int64_t>(r) + p.zp;
    q = q < p.ilo ? p.ilo : q;
    q = q > p.ihi ? p.ihi : q;
    return q;
}
PCCL_HD float dq_zps(int64_t q, const QuantParams &p) { return static_cast<float>(q - p.zp) * p.zps_scale; }

// wire element Q of zero-point-scale (64-bit types clamp and subtract in double)
template<typename Q>
PCCL_HD Q q_zps_as(float x, const QuantParams &p) {
    if constexpr (sizeof(Q) <= 2) { // same values as q_zps in 32-bit integers (|r|, |zp| < 2^17; no 64-bit emulation
        float r = __builtin_rintf(x * p.zps_inv); // on the GPU)
        const int32_t ilo = static_cast<int32_t>(p.ilo), ihi = static_cast<int32_t>(p.ihi);
        const int32_t zp = static_cast<int32_t>(p.zp);
        const float lo = static_cast<float>(ilo - zp), hi = static_cast<float>(ihi - zp);
        r = r < lo ? lo : r;
        r = r > hi ? hi : r;
        int32_t q = static_cast<int32_t>(r) + zp;
        q = q < ilo ? ilo : q;
        q = q > ihi ? ihi : q;
        return static_cast<Q>(q);
    } else if constexpr (sizeof(Q) <= 4) {
        return static_cast<Q>(q_zps(x, p));
    } else {
        double r = static_cast<double>(__builtin_rintf(x * p.zps_inv)) + static_cast<double>(p.zp);
        r = r < p.dlo ? p.dlo : r;
        r = r > p.dhi ? p.dhi : r;
        return static_cast<Q>(r);
    }
}
template<typename Q>
PCCL_HD float dq_zps_as(Q q, const QuantParams &p) {
    if constexpr (sizeof(Q) <= 2) return static_cast<float>(static_cast<int32_t>(q) - static_cast<int32_t>(p.zp)) * p.zps_scale;
    else if constexpr (sizeof(Q) <= 4) return dq_zps(static_cast<int64_t>(q), p);
    else return static_cast<float>(static_cast<double>(q) - static_cast<double>(p.zp)) * p.zps_scale;
}

} // namespace pccl::kernels
