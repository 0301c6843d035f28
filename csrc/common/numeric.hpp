// Bit-exact scalar numeric helpers shared by host (C++) and device (HIP) code.
//
// Every peer of a ring must produce bit-identical results whether it reduces on the CPU or on an MI355X, so the
// narrow-float conversions used by the reduce/quantize kernels are written once here with plain integer arithmetic
// (round-to-nearest-even, NaN preserving) and compiled into both the host kernels and the HIP kernels.
#pragma once

#include <cstdint>
#include <cstring>

#if defined(__HIPCC__) || defined(__HIP__)
#define PCCL_HD __host__ __device__ __forceinline__
#else
#define PCCL_HD inline __attribute__((always_inline))
#endif

namespace pccl::num {

PCCL_HD uint32_t f32_bits(float f) {
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
}
PCCL_HD float bits_f32(uint32_t u) {
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

// ---------------- bfloat16 ----------------
PCCL_HD float bf16_to_f32(uint16_t h) { return bits_f32(static_cast<uint32_t>(h) << 16); }

PCCL_HD uint16_t f32_to_bf16(float f) {
    const uint32_t u = f32_bits(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) { // NaN: keep sign, force quiet bit
        return static_cast<uint16_t>((u >> 16) | 0x0040u);
    }
    const uint32_t rounding_bias = 0x7fffu + ((u >> 16) & 1u);
    return static_cast<uint16_t>((u + rounding_bias) >> 16);
}

// ---------------- IEEE binary16 ----------------
PCCL_HD float f16_to_f32(uint16_t h) {
    const uint32_t sign = static_cast<uint32_t>(h & 0x8000u) << 16;
    const uint32_t exp = (h >> 10) & 0x1fu;
    uint32_t man = h & 0x3ffu;
    uint32_t out;
    if (exp == 0) {
        if (man == 0) {
            out = sign;
        } else { // subnormal: normalize
            int e = -1;
            do {
                ++e;
                man <<= 1;
            } while ((man & 0x400u) == 0);
            man &= 0x3ffu;
            out = sign | (static_cast<uint32_t>(127 - 15 - e) << 23) | (man << 13);
        }
    } else if (exp == 0x1f) {
        out = sign | 0x7f800000u | (man << 13) | (man ? 0x00400000u : 0u);
    } else {
        out = sign | ((exp + (127 - 15)) << 23) | (man << 13);
    }
    return bits_f32(out);
}

PCCL_HD uint16_t f32_to_f16(float f) {
    const uint32_t u = f32_bits(f);
    const uint32_t sign = (u >> 16) & 0x8000u;
    const uint32_t abs = u & 0x7fffffffu;
    if (abs > 0x7f800000u) return static_cast<uint16_t>(sign | 0x7e00u); // NaN
    if (abs >= 0x477ff000u) return static_cast<uint16_t>(sign | 0x7c00u); // overflow (>= 65520 rounds to inf)
    if (abs < 0x38800000u) { // result is subnormal or zero (|f| < 2^-14)
        if (abs < 0x33000000u) return static_cast<uint16_t>(sign); // < 2^-25 rounds to 0 (ties at 2^-25 -> 0, even)
        const uint32_t e = abs >> 23;             // biased f32 exponent
        const uint32_t man = (abs & 0x7fffffu) | 0x800000u;
        const uint32_t shift = 126u - e;         // value = man * 2^(e-150) = k * 2^-24  ->  k = man >> (126-e)
        const uint32_t kept = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u);
        const uint32_t half = 1u << (shift - 1u);
        uint32_t r = kept;
        if (rem > half || (rem == half && (kept & 1u))) r += 1u;
        return static_cast<uint16_t>(sign | r);
    }
    // normal range
    const uint32_t rebias = abs - ((127u - 15u) << 23);
    const uint32_t kept = rebias >> 13;
    const uint32_t rem = rebias & 0x1fffu;
    uint32_t r = kept;
    if (rem > 0x1000u || (rem == 0x1000u && (kept & 1u))) r += 1u;
    return static_cast<uint16_t>(sign | r);
}

// ---------------- OCP fp8 (e4m3fn: bias 7, no inf, NaN=0x7f; e5m2: bias 15, IEEE-like) ----------------
// Encoders saturate finite overflow to the max finite value (quantization use case, "satfinite").
PCCL_HD float fp8e4m3_to_f32(uint8_t v) {
    const uint32_t sign = static_cast<uint32_t>(v & 0x80u) << 24;
    const uint32_t exp = (v >> 3) & 0xfu;
    const uint32_t man = v & 0x7u;
    if (exp == 0xf && man == 0x7) return bits_f32(sign | 0x7fc00000u);
    if (exp == 0) {
        // subnormal: man * 2^-9
        const float mag = static_cast<float>(man) * 0.001953125f;
        return (v & 0x80u) ? -mag : mag;
    }
    return bits_f32(sign | ((exp + 120u) << 23) | (man << 20));
}

PCCL_HD uint8_t f32_to_fp8e4m3(float f) {
    const uint32_t u = f32_bits(f);
    const uint8_t sign = static_cast<uint8_t>((u >> 24) & 0x80u);
    const uint32_t abs = u & 0x7fffffffu;
    if (abs > 0x7f800000u) return static_cast<uint8_t>(sign | 0x7fu);
    if (abs >= 0x43e00000u) return static_cast<uint8_t>(sign | 0x7eu); // >= 448 saturate (also inf)
    if (abs < 0x3c800000u) {                                            // < 2^-6: subnormal region, step 2^-9
        const float a = bits_f32(abs) * 512.0f;                          // exact scaling
        uint32_t k = static_cast<uint32_t>(a);
        const float rem = a - static_cast<float>(k);
        if (rem > 0.5f || (rem == 0.5f && (k & 1u))) k += 1u;
        return static_cast<uint8_t>(sign | k); // k==8 becomes smallest normal (exp=1, man=0) naturally
    }
    const uint32_t rebias = abs - (120u << 23);
    const uint32_t kept = rebias >> 20;
    const uint32_t rem = rebias & 0xfffffu;
    uint32_t r = kept;
    if (rem > 0x80000u || (rem == 0x80000u && (kept & 1u))) r += 1u;
    if (r > 0x7eu) r = 0x7eu;
    return static_cast<uint8_t>(sign | r);
}

PCCL_HD float fp8e5m2_to_f32(uint8_t v) { return f16_to_f32(static_cast<uint16_t>(v) << 8); }

PCCL_HD uint8_t f32_to_fp8e5m2(float f) {
    const uint32_t u = f32_bits(f);
    const uint32_t abs = u & 0x7fffffffu;
    const uint8_t sign = static_cast<uint8_t>((u >> 24) & 0x80u);
    if (abs > 0x7f800000u) return static_cast<uint8_t>(sign | 0x7fu);
    if (abs >= 0x47600000u) return static_cast<uint8_t>(sign | 0x7bu); // >= 57344 saturate
    if (abs < 0x38800000u) { // < 2^-14: subnormal, step 2^-16
        const float a = bits_f32(abs) * 65536.0f;
        uint32_t k = static_cast<uint32_t>(a);
        const float rem = a - static_cast<float>(k);
        if (rem > 0.5f || (rem == 0.5f && (k & 1u))) k += 1u;
        return static_cast<uint8_t>(sign | k);
    }
    const uint32_t rebias = abs - (112u << 23);
    const uint32_t kept = rebias >> 21;
    const uint32_t rem = rebias & 0x1fffffu;
    uint32_t r = kept;
    if (rem > 0x100000u || (rem == 0x100000u && (kept & 1u))) r += 1u;
    if (r > 0x7bu) r = 0x7bu;
    return static_cast<uint8_t>(sign | r);
}

} // namespace pccl::num
