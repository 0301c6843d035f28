// Core enums and small value types of the CCoIP protocol (wire values follow SURVEY Appendix A).
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>

#include "ccoip_inet.h"

namespace pccl {

// Wire data types (ccoip_data_type_t of the reference, ccoip_types.hpp:8-21) + fp8 extensions.
enum class DType : uint8_t {
    U8 = 0, I8 = 1, U16 = 2, U32 = 3, I16 = 4, I32 = 5, U64 = 6, I64 = 7,
    F16 = 8, BF16 = 9, F32 = 10, F64 = 11, F8E4M3 = 12, F8E5M2 = 13
};

inline size_t dtype_size(DType t) {
    switch (t) {
        case DType::U8: case DType::I8: case DType::F8E4M3: case DType::F8E5M2: return 1;
        case DType::U16: case DType::I16: case DType::F16: case DType::BF16: return 2;
        case DType::U32: case DType::I32: case DType::F32: return 4;
        case DType::U64: case DType::I64: case DType::F64: return 8;
    }
    return 0;
}

inline bool dtype_valid(uint8_t v) { return v <= static_cast<uint8_t>(DType::F8E5M2); }
inline bool dtype_is_float(DType t) {
    return t == DType::F16 || t == DType::BF16 || t == DType::F32 || t == DType::F64 || t == DType::F8E4M3 ||
           t == DType::F8E5M2;
}
inline bool dtype_is_unsigned_int(DType t) {
    return t == DType::U8 || t == DType::U16 || t == DType::U32 || t == DType::U64;
}
const char *dtype_name(DType t);

enum class ReduceOp : uint8_t { Set = 0, Sum = 1, Avg = 2, Prod = 3, Max = 4, Min = 5 };
enum class QuantAlgo : uint8_t { None = 0, MinMax = 1, ZeroPointScale = 2 };
enum class HashType : uint8_t { Simple = 0, Crc32 = 1 };
enum class SyncStrategy : uint8_t { EnforcePopular = 0, RxOnly = 1, TxOnly = 2 };
enum class DeviceType : uint8_t { Cpu = 0, Gpu = 1 };

// Which data path executed an all-reduce (exposed through PCCL_ATTRIBUTE_LAST_REDUCE_PATH).
enum class ReducePath : int { None = 0, HostRing = 1, DeviceRing = 2, DeviceIpc = 3, Hierarchical = 4 };

struct Uuid {
    std::array<uint8_t, 16> data{};
    bool operator==(const Uuid &o) const { return data == o.data; }
    bool operator!=(const Uuid &o) const { return data != o.data; }
    bool operator<(const Uuid &o) const { return data < o.data; }
    std::string str() const;
    static Uuid random();
};

struct UuidHash {
    size_t operator()(const Uuid &u) const noexcept {
        uint64_t a, b;
        __builtin_memcpy(&a, u.data.data(), 8);
        __builtin_memcpy(&b, u.data.data() + 8, 8);
        return std::hash<uint64_t>{}(a ^ (b * 0x9e3779b97f4a7c15ull));
    }
};

// Socket address helpers (ccoip_socket_address_t is the C-ABI type).
using SockAddr = ccoip_socket_address_t;
std::string sockaddr_str(const SockAddr &a);
bool sockaddr_equal(const SockAddr &a, const SockAddr &b);
bool sockaddr_is_loopback(const SockAddr &a);
bool sockaddr_is_zero(const SockAddr &a);
SockAddr make_sockaddr_v4(uint8_t a, uint8_t b, uint8_t c, uint8_t d, uint16_t port);

struct SockAddrKey { // hashable key for maps keyed by endpoint
    std::array<uint8_t, 16> ip{};
    uint16_t port = 0;
    bool v4 = true;
    bool operator==(const SockAddrKey &o) const { return ip == o.ip && port == o.port && v4 == o.v4; }
    static SockAddrKey of(const SockAddr &a);
};
struct SockAddrKeyHash {
    size_t operator()(const SockAddrKey &k) const noexcept {
        uint64_t a, b;
        __builtin_memcpy(&a, k.ip.data(), 8);
        __builtin_memcpy(&b, k.ip.data() + 8, 8);
        return std::hash<uint64_t>{}(a ^ (b << 1) ^ (static_cast<uint64_t>(k.port) << 48) ^ k.v4);
    }
};

// Environment knobs.
size_t env_size(const char *name, size_t dflt);
bool env_flag(const char *name, bool dflt);

// Fault injection for the crash tests: PCCL_FAULT_INJECT="<point>:<seq>[:<step>[:<phase>]]" makes this process
// SIGKILL itself when it reaches `point` in the op with master sequence number `seq` (and, if given, at ring step
// `step` (global step index 0 .. 2(W-1)-1, all-gather steps after the reduce-scatter's) in phase `phase`). Points:
// ipc_vote, ipc_kernel, ss_serve; ring (device ring; phases publish / rx / ahead / end), qring (quantized device
// ring; phases meta / rx / end) and hring (host ring; phases rx / end). Lets a test kill a peer at an exact protocol position, e.g. while its xGMI push kernel
// and its peers' kernels are running or while the next ring step's receive sinks are already posted.
void fault_point(const char *point, uint64_t seq, size_t step = SIZE_MAX, const char *phase = nullptr);
bool fault_injection_armed();
// PCCL_FAULT_STALL="<point>:<max_seq>:<ms>": ops with sequence number <= max_seq sleep `ms` at `point` (tests: a slow
// peer makes its partners' barriers time out, so ops abort while the ring membership stays the same)
void fault_stall(const char *point, uint64_t seq);
// PCCL_FAULT_DELAY="<tag>:<ms>[,*:<ms>]": an op with that tag (or any tag, "*") sleeps before it initiates
// (scheduler tests: a slow op among fast ones).
void fault_delay(uint64_t tag);
bool fault_delay_armed(); // PCCL_FAULT_DELAY is set (ops then initiate on their worker, after the delay)

// PCCL_DEBUG_BACKTRACE_SIGNAL=1 (debugging hangs and crashes on the GPU box, where debuggers may not attach): SIGUSR2
// prints the native backtrace of every thread of the process to stderr (each thread is signalled in turn), and a
// fatal signal (SIGSEGV / SIGBUS / SIGFPE / SIGILL) prints the faulting thread's before the previously installed
// handler (e.g. Python's faulthandler) runs.
void install_debug_backtrace_signal();

} // namespace pccl
