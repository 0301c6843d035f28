// Userspace WAN emulator OUTSIDE libpccl (BASELINE config 3 without tc-netem, which needs root): a TCP relay that
// delays every byte by a fixed one-way latency and paces it through token buckets, per TCP connection (a window-
// limited long-fat-pipe flow) and per relayed link (the sending peer's NIC). Peers advertise a relay port as their
// P2P address (Communicator(..., advertised_p2p_port=...)); the relay forwards each accepted connection to the real
// listen port. Nothing inside the library is shaped, so the measurement is the library's behaviour over a link it
// cannot influence.
//
//   pccl_wan_relay --delay-ms 50 --flow-mbit 1000 --link-mbit 25000 --map 40001:48149 [--map 40002:48152 ...]
//                  [--blackhole-port 40001]
//
// Failure emulation: with --blackhole-port P, SIGUSR1 black-holes every connection of map P that exists at that
// moment - both directions stop forwarding while the sockets stay open (the relay reads until its window is full,
// then the sender's TCP sees a zero window), as a path that silently drops everything. Connections opened later
// (the ring re-established without the link) are forwarded normally.
//
// Model: one-way delay d in both directions; a connection's bytes leave the relay no earlier than arrival + d and no
// faster than flow_mbit (per direction); all bytes relayed towards one map target share link_mbit (in a ring, all
// of them come from the target's predecessor, so this is that peer's egress link). The relay reads at most
// 2 x d x flow_rate bytes ahead per direction (the bandwidth-delay product of the flow: the window a real WAN TCP
// connection would have in flight), so senders feel back-pressure as on a real long fat pipe.
//
// CPU: a real WAN path costs the hosts nothing, so the relay keeps its own share small. Chunks are recycled buffers
// (no allocation or zero-fill per chunk) and leave with MSG_ZEROCOPY sends: the kernel hands the relay's pages to
// the receiving peer, whose receive copy happens anyway, instead of copying them into socket buffers first
// (PCCL_RELAY_ZEROCOPY=0: plain sends). A chunk's buffer returns to the pool once the kernel reports its send complete.
// Collocated emulation, interleaved against the previous relay (profiles/r6/collocated_relay_ab/): warm repeats
// 0.60-0.76 s vs 0.83-1.03 s; the emulation's run-to-run spread on a 16-CPU share stays large.
#include <arpa/inet.h>
#include <linux/errqueue.h>
#include <malloc.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;
double now_s() { return std::chrono::duration<double>(Clock::now().time_since_epoch()).count(); }
void sleep_until_s(double t) {
    const double d = t - now_s();
    if (d > 0) std::this_thread::sleep_for(std::chrono::duration<double>(d));
}

struct Config {
    double delay_s = 0.05, flow_Bps = 125e6, link_Bps = 0;
};
Config g_cfg;
std::atomic<uint64_t> g_bytes{0};
volatile sig_atomic_t g_stop = 0;
uint16_t g_blackhole_port = 0;
std::atomic<int> g_blackhole_gen{0}; // bumped by SIGUSR1 (lock-free, async-signal-safe)

// shared egress link of one map target (all connections relayed towards it)
struct Link {
    std::mutex m;
    double next_free = 0;
    // reserves n bytes on the link no earlier than t; returns when they have left
    double reserve(size_t n, double t) {
        if (g_cfg.link_Bps <= 0) return t;
        std::lock_guard l(m);
        const double start = std::max(t, next_free);
        next_free = start + static_cast<double>(n) / g_cfg.link_Bps;
        return next_free;
    }
};

constexpr size_t kChunk = 256 << 10;

struct Chunk {
    double arrival = 0;
    std::unique_ptr<char[]> data;
    size_t n = 0;
};

// one direction of one connection: reader thread -> delay queue -> paced writer thread
class Pump {
public:
    Pump(int src, int dst, Link *link, bool blackholable = false)
        : src_(src), dst_(dst), link_(link), blackholable_(blackholable), born_gen_(g_blackhole_gen.load()) {
        window_ = std::max<size_t>(1 << 20, static_cast<size_t>(2 * g_cfg.delay_s * g_cfg.flow_Bps));
    }
    bool blackholed() const { return blackholable_ && g_blackhole_gen.load() > born_gen_; }
    void run() {
        std::thread r([this] { reader(); });
        writer();
        r.join();
    }

private:
    std::unique_ptr<char[]> take_buffer() {
        {
            std::lock_guard l(m_);
            if (!free_.empty()) {
                auto b = std::move(free_.back());
                free_.pop_back();
                return b;
            }
        }
        return std::unique_ptr<char[]>(new char[kChunk]); // (not zero-filled)
    }
    void reader() {
        while (true) {
            auto buf = take_buffer();
            const ssize_t k = ::recv(src_, buf.get(), kChunk, 0);
            if (k <= 0) break;
            std::unique_lock l(m_);
            cv_.wait(l, [&] { return queued_ < window_ || closed_; });
            if (closed_) break;
            queued_ += static_cast<size_t>(k);
            q_.push_back({now_s(), std::move(buf), static_cast<size_t>(k)});
            cv_.notify_all();
        }
        std::lock_guard l(m_);
        eof_ = true;
        cv_.notify_all();
    }
    // MSG_ZEROCOPY completions: the ids in [ee_info, ee_data] are done (in order on one socket); their buffers are
    // recycled. With `wait_ms` > 0, waits that long for completions to arrive.
    void reap(int wait_ms) {
        if (pending_.empty()) return;
        if (wait_ms > 0) {
            pollfd pfd{dst_, 0, 0}; // (POLLERR is always reported)
            ::poll(&pfd, 1, wait_ms);
        }
        while (true) {
            char ctrl[128];
            msghdr msg{};
            msg.msg_control = ctrl;
            msg.msg_controllen = sizeof(ctrl);
            if (::recvmsg(dst_, &msg, MSG_ERRQUEUE | MSG_DONTWAIT) < 0) break;
            for (cmsghdr *cm = CMSG_FIRSTHDR(&msg); cm; cm = CMSG_NXTHDR(&msg, cm)) {
                auto *se = reinterpret_cast<sock_extended_err *>(CMSG_DATA(cm));
                if (se->ee_errno != 0 || se->ee_origin != SO_EE_ORIGIN_ZEROCOPY) continue;
                if (static_cast<int32_t>(se->ee_data + 1 - done_to_) > 0) done_to_ = se->ee_data + 1;
            }
        }
        std::lock_guard l(m_);
        while (!pending_.empty() && static_cast<int32_t>(done_to_ - pending_.front().first) >= 0) {
            free_.push_back(std::move(pending_.front().second));
            pending_.pop_front();
        }
    }
    void writer() {
        int one = 1;
        const char *zenv = std::getenv("PCCL_RELAY_ZEROCOPY"); // 0: plain sends (A/B)
        const bool zc = !(zenv && std::strcmp(zenv, "0") == 0) &&
                        ::setsockopt(dst_, SOL_SOCKET, SO_ZEROCOPY, &one, sizeof(one)) == 0;
        double flow_next = 0;
        while (true) {
            Chunk c;
            {
                std::unique_lock l(m_);
                cv_.wait(l, [&] { return !q_.empty() || eof_; });
                if (q_.empty()) break;
                c = std::move(q_.front());
                q_.pop_front();
            }
            const size_t n = c.n;
            if (blackholed()) { // forwards nothing from now on; the sockets stay open (the reader fills its window)
                while (!g_stop) std::this_thread::sleep_for(std::chrono::milliseconds(50));
                break;
            }
            double t = std::max(c.arrival + g_cfg.delay_s, flow_next);
            flow_next = t + static_cast<double>(n) / g_cfg.flow_Bps;
            t = std::max(flow_next, link_ ? link_->reserve(n, t) : t);
            sleep_until_s(t);
            size_t off = 0;
            bool ok = true;
            while (off < n) {
                const ssize_t k = ::send(dst_, c.data.get() + off, n - off, MSG_NOSIGNAL | (zc ? MSG_ZEROCOPY : 0));
                if (k <= 0) {
                    ok = false;
                    break;
                }
                if (zc) ++next_id_;
                off += static_cast<size_t>(k);
            }
            g_bytes += off;
            {
                std::lock_guard l(m_);
                queued_ -= n;
                // the kernel may still read this buffer (zero-copy): it is recycled on its completion
                if (zc) pending_.emplace_back(next_id_, std::move(c.data));
                else free_.push_back(std::move(c.data));
                cv_.notify_all();
            }
            if (zc) reap(0);
            if (!ok) break;
        }
        // buffers the kernel may still read are not freed: wait for their completions, else leave them allocated
        for (int i = 0; i < 20 && !pending_.empty(); ++i) reap(100);
        for (auto &p : pending_) (void)p.second.release();
        {
            std::lock_guard l(m_);
            closed_ = true;
            cv_.notify_all();
        }
        ::shutdown(dst_, SHUT_WR);
        ::shutdown(src_, SHUT_RD);
    }
    int src_, dst_;
    Link *link_;
    const bool blackholable_;
    const int born_gen_;
    size_t window_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<Chunk> q_;
    std::vector<std::unique_ptr<char[]>> free_;
    std::deque<std::pair<uint32_t, std::unique_ptr<char[]>>> pending_; // (id after its last send, buffer)
    uint32_t next_id_ = 0, done_to_ = 0;
    size_t queued_ = 0;
    bool eof_ = false, closed_ = false;
};

void tune(int fd) {
    int one = 1, buf = 32 << 20;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

int listen_on(uint16_t port) {
    const int s = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons(port);
    if (::bind(s, reinterpret_cast<sockaddr *>(&a), sizeof(a)) != 0 || ::listen(s, 256) != 0) {
        std::fprintf(stderr, "wan_relay: cannot listen on %u\n", port);
        std::exit(2);
    }
    return s;
}

int connect_to(uint16_t port) {
    const int s = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons(port);
    for (int attempt = 0; attempt < 50; ++attempt) {
        if (::connect(s, reinterpret_cast<sockaddr *>(&a), sizeof(a)) == 0) return s;
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    ::close(s);
    return -1;
}

void serve(uint16_t listen_port, uint16_t target) {
    const int ls = listen_on(listen_port);
    auto *link = new Link(); // lives as long as the process
    while (true) {
        const int c = ::accept(ls, nullptr, nullptr);
        if (c < 0) continue;
        std::thread([c, target, link, listen_port] {
            const int t = connect_to(target);
            if (t < 0) {
                ::close(c);
                return;
            }
            tune(c);
            tune(t);
            const bool bh = listen_port == g_blackhole_port;
            Pump up(c, t, link, bh), down(t, c, nullptr, bh); // towards the target: the predecessor's egress link
            std::thread d([&] { down.run(); });
            up.run();
            d.join();
            ::close(c);
            ::close(t);
        }).detach();
    }
}

} // namespace

int main(int argc, char **argv) {
    std::vector<std::pair<uint16_t, uint16_t>> maps;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        const char *v = argv[i + 1];
        if (k == "--delay-ms") g_cfg.delay_s = std::atof(v) / 1e3;
        else if (k == "--flow-mbit") g_cfg.flow_Bps = std::atof(v) * 1e6 / 8;
        else if (k == "--link-mbit") g_cfg.link_Bps = std::atof(v) * 1e6 / 8;
        else if (k == "--blackhole-port") g_blackhole_port = static_cast<uint16_t>(std::atoi(v));
        else if (k == "--map") {
            unsigned a = 0, b = 0;
            if (std::sscanf(v, "%u:%u", &a, &b) != 2) return 2;
            maps.emplace_back(static_cast<uint16_t>(a), static_cast<uint16_t>(b));
        } else {
            std::fprintf(stderr, "usage: %s --delay-ms D --flow-mbit F --link-mbit L --map LISTEN:TARGET ... [--blackhole-port P]\n", argv[0]);
            return 2;
        }
    }
    if (maps.empty()) return 2;
    // chunk buffers from the heap, not one mmap (and its page faults) per buffer: the pools only grow
    mallopt(M_MMAP_THRESHOLD, 64 << 20);
    signal(SIGPIPE, SIG_IGN);
    signal(SIGTERM, [](int) { g_stop = 1; });
    signal(SIGUSR1, [](int) { g_blackhole_gen.fetch_add(1); });
    for (auto [l, t] : maps) std::thread(serve, l, t).detach();
    std::printf("{\"relay\": \"ready\", \"maps\": %zu}\n", maps.size());
    std::fflush(stdout);
    // until SIGTERM: relayed bytes once a second on stderr, the total as JSON on stdout at the end
    uint64_t last = 0;
    while (!g_stop) {
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        const uint64_t b = g_bytes.load();
        if (b - last > (1ull << 30)) {
            std::fprintf(stderr, "wan_relay: %.3f GB relayed\n", b / 1e9);
            last = b;
        }
    }
    std::printf("{\"relay\": \"done\", \"relayed_bytes\": %llu}\n", static_cast<unsigned long long>(g_bytes.load()));
    std::fflush(stdout);
    std::_Exit(0);
}
