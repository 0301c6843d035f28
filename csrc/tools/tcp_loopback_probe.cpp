// Loopback TCP ceiling for the device ring: P "peers" in a ring (peer p sends to p+1 and receives from p-1), each
// link made of C parallel connections; every peer pushes `mib` MiB per link and drains what it receives, all at once
// (the shape of one ring step). Reports aggregate and per-peer send throughput.
//   tcp_loopback_probe [peers=2] [conns=8] [mib=512] [chunk_kib=4096] [sockbuf_kib=8192, 0 = kernel autotuning]
//                      [cold=0: 1 = send from / receive into whole per-connection buffers (DRAM, like the ring's
//                       staging buffers) instead of one cache-resident chunk]
// Also reports the process CPU time per moved GB (user + sys, RUSAGE_SELF).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static int listen_on(uint16_t &port) {
    int s = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = 0;
    if (bind(s, reinterpret_cast<sockaddr *>(&a), sizeof(a)) != 0 || listen(s, 256) != 0) std::exit(2);
    socklen_t l = sizeof(a);
    getsockname(s, reinterpret_cast<sockaddr *>(&a), &l);
    port = ntohs(a.sin_port);
    return s;
}

static int g_sockbuf = 8 << 20;
static void tune(int fd) {
    int one = 1, buf = g_sockbuf;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    if (buf > 0) {
        setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
        setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
    }
}

static double cpu_s() {
    rusage r{};
    getrusage(RUSAGE_SELF, &r);
    return r.ru_utime.tv_sec + r.ru_stime.tv_sec + 1e-6 * (r.ru_utime.tv_usec + r.ru_stime.tv_usec);
}

int main(int argc, char **argv) {
    const int P = argc > 1 ? std::atoi(argv[1]) : 2;
    const int C = argc > 2 ? std::atoi(argv[2]) : 8;
    const size_t bytes = (argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 512) << 20;
    const size_t chunk = (argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 4096) << 10;
    g_sockbuf = static_cast<int>((argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 8192) << 10);
    const bool cold = argc > 6 && std::atoi(argv[6]) != 0;
    std::vector<int> lfd(P);
    std::vector<uint16_t> port(P);
    for (int p = 0; p < P; ++p) lfd[p] = listen_on(port[p]);
    // tx[p][c]: peer p -> peer p+1, rx[p][c]: peer p <- peer p-1
    std::vector<std::vector<int>> tx(P, std::vector<int>(C)), rx(P, std::vector<int>(C));
    for (int p = 0; p < P; ++p) {
        const int q = (p + 1) % P;
        for (int c = 0; c < C; ++c) {
            int s = socket(AF_INET, SOCK_STREAM, 0);
            tune(s);
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
            a.sin_port = htons(port[q]);
            if (connect(s, reinterpret_cast<sockaddr *>(&a), sizeof(a)) != 0) return 3;
            tx[p][c] = s;
            int r = accept(lfd[q], nullptr, nullptr);
            tune(r);
            rx[q][c] = r;
        }
    }
    const size_t per_conn = bytes / C;
    std::atomic<int> go{0}, ready{0};
    std::vector<std::thread> th;
    for (int p = 0; p < P; ++p)
        for (int c = 0; c < C; ++c) {
            th.emplace_back([&, p, c] {
                std::vector<char> buf(cold ? per_conn : chunk, 1);
                ++ready;
                while (!go.load()) std::this_thread::yield();
                for (size_t off = 0; off < per_conn;) {
                    const ssize_t k = send(tx[p][c], buf.data() + (cold ? off : 0), std::min(chunk, per_conn - off), 0);
                    if (k <= 0) std::exit(4);
                    off += static_cast<size_t>(k);
                }
            });
            th.emplace_back([&, p, c] {
                std::vector<char> buf(cold ? per_conn : chunk, 2);
                ++ready;
                while (!go.load()) std::this_thread::yield();
                for (size_t off = 0; off < per_conn;) {
                    const ssize_t k = recv(rx[p][c], buf.data() + (cold ? off : 0), std::min(chunk, per_conn - off), 0);
                    if (k <= 0) std::exit(5);
                    off += static_cast<size_t>(k);
                }
            });
        }
    while (ready.load() < static_cast<int>(th.size())) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    const double c0 = cpu_s();
    const auto t0 = std::chrono::steady_clock::now();
    go = 1;
    for (auto &t : th) t.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double cpu = cpu_s() - c0;
    const double total = static_cast<double>(per_conn) * C * P;
    std::printf("{\"peers\": %d, \"conns_per_link\": %d, \"mib_per_peer\": %zu, \"chunk_kib\": %zu, "
                "\"sockbuf_kib\": %d, \"cold\": %d, \"sec\": %.4f, \"aggregate_GBps\": %.2f, "
                "\"per_peer_send_GBps\": %.2f, \"cpu_s\": %.3f, \"cores_busy\": %.2f, \"cpu_s_per_GB\": %.4f}\n",
                P, C, bytes >> 20, chunk >> 10, g_sockbuf >> 10, cold ? 1 : 0, s, total / s / 1e9, total / P / s / 1e9,
                cpu, cpu / s, cpu / (total / 1e9));
    return 0;
}
