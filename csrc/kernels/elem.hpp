// Element codecs + reduce operators shared by host loops and HIP kernels (bit-exact between the two).
#pragma once

#include <cstdint>

#include "../common/numeric.hpp"

namespace pccl::kernels {

// Storage type S, compute type C, load/store conversions.
struct EF32 {
    using S = float;
    using C = float;
    static PCCL_HD C ld(S v) { return v; }
    static PCCL_HD S st(C v) { return v; }
};
struct EF64 {
    using S = double;
    using C = double;
    static PCCL_HD C ld(S v) { return v; }
    static PCCL_HD S st(C v) { return v; }
};
struct EBF16 {
    using S = uint16_t;
    using C = float;
    static PCCL_HD C ld(S v) { return num::bf16_to_f32(v); }
    static PCCL_HD S st(C v) { return num::f32_to_bf16(v); }
};
struct EF16 {
    using S = uint16_t;
    using C = float;
    static PCCL_HD C ld(S v) { return num::f16_to_f32(v); }
    static PCCL_HD S st(C v) { return num::f32_to_f16(v); }
};
template<typename T>
struct EInt {
    using S = T;
    using C = T;
    static PCCL_HD C ld(S v) { return v; }
    static PCCL_HD S st(C v) { return v; }
};

struct OpSet {
    template<typename C>
    static PCCL_HD C apply(C, C b) { return b; }
};
struct OpSum {
    template<typename C>
    static PCCL_HD C apply(C a, C b) { return a + b; }
};
struct OpProd {
    template<typename C>
    static PCCL_HD C apply(C a, C b) { return a * b; }
};
struct OpMax {
    template<typename C>
    static PCCL_HD C apply(C a, C b) { return a < b ? b : a; }
};
struct OpMin {
    template<typename C>
    static PCCL_HD C apply(C a, C b) { return b < a ? b : a; }
};

// Integer promotion-safe ops for narrow ints (int8/uint8/int16/uint16 arithmetic wraps in the storage type).
template<typename Op, typename C>
PCCL_HD C apply_op(C a, C b) {
    return static_cast<C>(Op::template apply<C>(a, b));
}

} // namespace pccl::kernels
