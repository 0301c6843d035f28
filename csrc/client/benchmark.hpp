// Point-to-point bandwidth benchmark used by topology optimization (reference: ccoip/src/cpp/benchmark_runner.cpp).
// The sender opens PCCL_NUM_BENCHMARK_CONNECTIONS (default 16) parallel TCP streams to the peer's benchmark port and
// streams 8 MiB buffers for PCCL_BENCHMARK_MILLIS (default 10000), the reference's defaults, reporting the summed
// goodput in Mbit/s.
#pragma once

#include "../common/types.hpp"

namespace pccl::client {

enum class BenchResult { Success = 0, Busy = 1, ConnectionFailure = 2, SendFailure = 3, OtherFailure = 4 };

BenchResult benchmark_send(const Uuid &self, const SockAddr &endpoint, double &mbps_out);
void benchmark_receive(int fd, const SockAddr &peer);

} // namespace pccl::client
