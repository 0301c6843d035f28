#include "benchmark.hpp"

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <random>
#include <sys/socket.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../common/log.hpp"
#include "../net/socket.hpp"

namespace pccl::client {

using namespace std::chrono;

BenchResult benchmark_send(const Uuid &self, const SockAddr &endpoint, double &mbps_out) {
    // reference defaults: 16 connections x 10 s of 8 MiB sends (benchmark_runner.cpp:11-13)
    const int n_conn = static_cast<int>(std::max<size_t>(1, env_size("PCCL_NUM_BENCHMARK_CONNECTIONS", 16)));
    const double seconds = static_cast<double>(env_size("PCCL_BENCHMARK_MILLIS", 10000)) / 1000.0;
    constexpr size_t kBuf = 8 << 20;
    std::vector<int> fds;
    for (int i = 0; i < n_conn; ++i) {
        const int fd = net::connect_tcp(endpoint, 3000);
        if (fd < 0) {
            for (int f : fds) ::close(f);
            return fds.empty() ? BenchResult::ConnectionFailure : BenchResult::SendFailure;
        }
        proto::C2BHello hello;
        hello.peer_uuid = self;
        timeval tv{5, 0};
        setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        // a target that stops reading (stopped, wedged) keeps the connection alive with a zero window: a send that
        // moves no byte for 2 s ends the probe instead of blocking until TCP_USER_TIMEOUT
        timeval stv{2, 0};
        setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &stv, sizeof(stv));
        if (!net::send_packet(fd, hello)) {
            ::close(fd);
            for (int f : fds) ::close(f);
            return BenchResult::SendFailure;
        }
        auto busy = net::recv_packet<proto::B2CBenchmarkServerIsBusy>(fd);
        if (!busy || busy->is_busy) {
            ::close(fd);
            for (int f : fds) ::close(f);
            return busy ? BenchResult::Busy : BenchResult::ConnectionFailure;
        }
        fds.push_back(fd);
    }
    std::vector<uint8_t> buf(kBuf);
    std::mt19937 gen(1234);
    for (auto &b : buf) b = static_cast<uint8_t>(gen());
    std::atomic<uint64_t> total{0};
    std::atomic<bool> failed{false};
    std::vector<std::thread> ts;
    const auto t0 = steady_clock::now();
    for (int fd : fds) {
        ts.emplace_back([&, fd] {
            while (duration<double>(steady_clock::now() - t0).count() < seconds) {
                const ssize_t k = ::send(fd, buf.data(), buf.size(), MSG_NOSIGNAL);
                if (k < 0) {
                    failed = true;
                    break;
                }
                total += static_cast<uint64_t>(k);
            }
        });
    }
    for (auto &t : ts) t.join();
    const double dt = duration<double>(steady_clock::now() - t0).count();
    for (int fd : fds) {
        ::shutdown(fd, SHUT_RDWR);
        ::close(fd);
    }
    if (failed && total == 0) return BenchResult::SendFailure;
    mbps_out = static_cast<double>(total.load()) * 8.0 / 1e6 / dt;
    return BenchResult::Success;
}

void benchmark_receive(int fd, const SockAddr &peer) {
    const double seconds = static_cast<double>(env_size("PCCL_BENCHMARK_MILLIS", 10000)) / 1000.0 + 8.0;
    std::vector<uint8_t> buf(1 << 20);
    const auto t0 = steady_clock::now();
    while (duration<double>(steady_clock::now() - t0).count() < seconds) {
        const int r = net::wait_readable(fd, 200);
        if (r < 0) break;
        if (r == 0) continue;
        const ssize_t k = ::recv(fd, buf.data(), buf.size(), 0);
        if (k <= 0) break;
    }
    ::shutdown(fd, SHUT_RDWR);
    ::close(fd);
    LOG(DEBUG) << "Benchmark receive from " << sockaddr_str(peer) << " finished";
}

} // namespace pccl::client
