// Plain multi-connection TCP stream for calibrating the WAN emulator (pccl_wan_relay): no framing, no library.
//   tcp_stream sink PORT                     accept connections on 127.0.0.1:PORT, drain them; print one JSON line per
//                                            second ({"t": s, "bytes": total received}) until every connection closed
//   tcp_stream send PORT CONNS SECONDS       CONNS connections to 127.0.0.1:PORT, each sending as fast as it can for
//                                            SECONDS (4 MiB sends from one buffer), then close; prints the bytes sent
// Sockets keep the kernel's buffer autotuning, like libpccl's data sockets to other hosts.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

int sink(uint16_t port) {
    const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons(port);
    if (::bind(ls, reinterpret_cast<sockaddr *>(&a), sizeof(a)) != 0 || ::listen(ls, 512) != 0) return 2;
    std::printf("{\"sink\": \"ready\"}\n");
    std::fflush(stdout);
    std::atomic<uint64_t> total{0};
    std::atomic<int> open{0}, seen{0};
    std::thread acceptor([&] {
        while (true) {
            const int c = ::accept(ls, nullptr, nullptr);
            if (c < 0) break;
            ++open;
            ++seen;
            std::thread([c, &total, &open] {
                std::vector<char> buf(4 << 20);
                while (true) {
                    const ssize_t k = ::recv(c, buf.data(), buf.size(), 0);
                    if (k <= 0) break;
                    total += static_cast<uint64_t>(k);
                }
                ::close(c);
                --open;
            }).detach();
        }
    });
    acceptor.detach();
    const auto t0 = Clock::now();
    while (true) {
        std::this_thread::sleep_for(std::chrono::milliseconds(250));
        const double t = std::chrono::duration<double>(Clock::now() - t0).count();
        std::printf("{\"t\": %.3f, \"bytes\": %llu, \"open\": %d}\n", t, static_cast<unsigned long long>(total.load()),
                    open.load());
        std::fflush(stdout);
        if (seen.load() > 0 && open.load() == 0) break;
    }
    return 0;
}

int send(uint16_t port, int conns, double seconds) {
    std::atomic<uint64_t> sent{0};
    std::vector<std::thread> th;
    const auto end = Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds));
    for (int i = 0; i < conns; ++i)
        th.emplace_back([&] {
            const int s = ::socket(AF_INET, SOCK_STREAM, 0);
            int one = 1;
            setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
            a.sin_port = htons(port);
            if (::connect(s, reinterpret_cast<sockaddr *>(&a), sizeof(a)) != 0) {
                ::close(s);
                return;
            }
            std::vector<char> buf(4 << 20, 'x');
            while (Clock::now() < end) {
                const ssize_t k = ::send(s, buf.data(), buf.size(), MSG_NOSIGNAL);
                if (k <= 0) break;
                sent += static_cast<uint64_t>(k);
            }
            ::shutdown(s, SHUT_WR);
            char c;
            while (::recv(s, &c, 1, 0) > 0) {
            }
            ::close(s);
        });
    for (auto &t : th) t.join();
    std::printf("{\"sent_bytes\": %llu}\n", static_cast<unsigned long long>(sent.load()));
    return 0;
}

} // namespace

int main(int argc, char **argv) {
    if (argc >= 3 && std::string(argv[1]) == "sink") return sink(static_cast<uint16_t>(std::atoi(argv[2])));
    if (argc >= 5 && std::string(argv[1]) == "send")
        return send(static_cast<uint16_t>(std::atoi(argv[2])), std::atoi(argv[3]), std::atof(argv[4]));
    std::fprintf(stderr, "usage: %s sink PORT | send PORT CONNS SECONDS\n", argv[0]);
    return 2;
}
