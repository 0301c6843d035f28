// dtype / op dispatch helpers shared by the HIP translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <type_traits>

#include "kernels.hpp"

namespace pccl::hipk {

template<typename F>
bool launch_ok(F &&f) {
    f();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        std::fprintf(stderr, "[pccl_hip] kernel launch failed: %s\n", hipGetErrorString(e));
        return false;
    }
    return true;
}

// dtype dispatch -> element codec
template<typename F>
bool with_elem(DType t, F &&f) {
    switch (t) {
        case DType::F32: return f(EF32{});
        case DType::F64: return f(EF64{});
        case DType::BF16: return f(EBF16{});
        case DType::F16: return f(EF16{});
        case DType::U8: return f(EInt<uint8_t>{});
        case DType::I8: return f(EInt<int8_t>{});
        case DType::U16: return f(EInt<uint16_t>{});
        case DType::I16: return f(EInt<int16_t>{});
        case DType::U32: return f(EInt<uint32_t>{});
        case DType::I32: return f(EInt<int32_t>{});
        case DType::U64: return f(EInt<uint64_t>{});
        case DType::I64: return f(EInt<int64_t>{});
        default: return false;
    }
}

template<typename F>
bool with_float_elem(DType t, F &&f) {
    switch (t) {
        case DType::F32: return f(EF32{});
        case DType::F64: return f(EF64{});
        case DType::BF16: return f(EBF16{});
        case DType::F16: return f(EF16{});
        default: return false;
    }
}

template<typename F>
bool with_op(ReduceOp op, F &&f) {
    switch (op) {
        case ReduceOp::Set: return f(OpSet{});
        case ReduceOp::Sum:
        case ReduceOp::Avg: return f(OpSum{});
        case ReduceOp::Prod: return f(OpProd{});
        case ReduceOp::Max: return f(OpMax{});
        case ReduceOp::Min: return f(OpMin{});
    }
    return false;
}

template<typename F>
bool with_qint(DType q, F &&f) {
    switch (q) {
        case DType::U8: return f(uint8_t{});
        case DType::I8: return f(int8_t{});
        case DType::U16: return f(uint16_t{});
        case DType::I16: return f(int16_t{});
        case DType::U32: return f(uint32_t{});
        case DType::I32: return f(int32_t{});
        case DType::U64: return f(uint64_t{});
        case DType::I64: return f(int64_t{});
        default: return false;
    }
}


} // namespace pccl::hipk
