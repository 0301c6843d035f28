// Transport test suite (reference tinysockets/tests: test_server_socket.cpp:19-1186, test_queued_socket.cpp:36-504,
// test_blocking_io_socket.cpp:36-240), rebuilt against this repo's components:
//   EventServer      - the master's epoll LTV server (reference ServerSocket)
//   MasterConnection - the client's predicate-receive master socket (reference QueuedSocket)
//   socket helpers   - blocking LTV / full send-recv / connect / listen (reference BlockingIOSocket)
//   MuxConn          - the multiplexed P2P data connection (reference MultiplexedIOSocket)
// Also run under the ASan/UBSan and TSan builds (tests/test_native.py).
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "harness.hpp"
#include "net/event_server.hpp"
#include "net/master_conn.hpp"
#include "net/mux.hpp"
#include "net/socket.hpp"
#include "proto/packets.hpp"

using namespace pccl;
using namespace std::chrono_literals;

namespace {

SockAddr any_v4(uint16_t port = 0) {
    SockAddr a{};
    a.inet.protocol = inetIPv4;
    a.port = port;
    return a;
}
SockAddr loop_v4(uint16_t port) { return make_sockaddr_v4(127, 0, 0, 1, port); }

template<typename F>
bool eventually(F &&f, std::chrono::milliseconds limit = 5000ms) {
    const auto t0 = std::chrono::steady_clock::now();
    while (!f()) {
        if (std::chrono::steady_clock::now() - t0 > limit) return false;
        std::this_thread::sleep_for(2ms);
    }
    return true;
}

// an EventServer that records every packet and echoes packets with id 100 back with id 101
struct EchoServer {
    net::EventServer srv{any_v4(), false};
    std::mutex m;
    std::vector<std::pair<uint16_t, std::vector<uint8_t>>> got;
    std::vector<SockAddr> joined;
    std::atomic<int> closed{0}, ticks{0};
    EchoServer() {
        srv.on_read([this](const SockAddr &a, uint16_t id, const uint8_t *p, size_t n) {
            {
                std::lock_guard l(m);
                got.emplace_back(id, std::vector<uint8_t>(p, p + n));
            }
            if (id == 100) srv.send_raw(a, 101, std::vector<uint8_t>(p, p + n));
        });
        srv.on_close([this](const SockAddr &) { closed++; });
        srv.on_join([this](const SockAddr &a) {
            std::lock_guard l(m);
            joined.push_back(a);
        });
        srv.on_tick([this] { ticks++; });
        EXPECT(srv.listen() && srv.run_async());
    }
    ~EchoServer() {
        srv.interrupt();
        srv.join();
    }
    size_t count() {
        std::lock_guard l(m);
        return got.size();
    }
    int connect() { return net::connect_tcp(loop_v4(srv.port()), 2000); }
};

std::vector<uint8_t> raw_ltv(uint64_t len_field, uint16_t id, size_t payload) {
    std::vector<uint8_t> b;
    for (int i = 7; i >= 0; --i) b.push_back(static_cast<uint8_t>(len_field >> (8 * i)));
    b.push_back(static_cast<uint8_t>(id >> 8));
    b.push_back(static_cast<uint8_t>(id));
    b.resize(b.size() + payload, 0xAB);
    return b;
}

} // namespace

// ================================================================ EventServer (reference ServerSocket)
TEST(es_bind_ephemeral_port) {
    net::EventServer s(any_v4(0), false);
    EXPECT(s.listen());
    EXPECT(s.port() > 0);
}

TEST(es_bump_port_when_taken) {
    uint16_t taken = 0;
    int fd = net::listen_tcp(inetIPv4, 0, false, taken);
    EXPECT(fd >= 0);
    net::EventServer bump(any_v4(taken), true);
    EXPECT(bump.listen() && bump.port() != taken);
    net::EventServer strict(any_v4(taken), false);
    EXPECT(!strict.listen());
    net::close_fd(fd);
}

TEST(es_interrupt_idle_server) {
    net::EventServer s(any_v4(), false);
    EXPECT(s.listen() && s.run_async());
    EXPECT(eventually([&] { return s.running(); }));
    const auto t0 = std::chrono::steady_clock::now();
    s.interrupt();
    s.join();
    EXPECT(std::chrono::steady_clock::now() - t0 < 5s);
    EXPECT(!s.running());
}

TEST(es_interrupt_with_connected_clients_closes_them) {
    auto *e = new EchoServer();
    int fds[4];
    for (int &fd : fds) fd = e->connect();
    EXPECT(eventually([&] { std::lock_guard l(e->m); return e->joined.size() == 4; }));
    const auto t0 = std::chrono::steady_clock::now();
    delete e; // interrupt + join: no close callbacks on interrupt, sockets closed
    EXPECT(std::chrono::steady_clock::now() - t0 < 5s);
    for (int fd : fds) {
        uint8_t b;
        EXPECT(!net::recv_all(fd, &b, 1)); // EOF
        ::close(fd);
    }
}

TEST(es_interrupt_while_client_streams) {
    auto *e = new EchoServer();
    const int fd = e->connect();
    std::atomic<bool> stop{false};
    std::thread t([&] {
        std::vector<uint8_t> p(1 << 20, 1);
        while (!stop && net::send_ltv(fd, 7, p.data(), p.size())) {
        }
    });
    EXPECT(eventually([&] { return e->count() > 3; }));
    const auto t0 = std::chrono::steady_clock::now();
    delete e;
    EXPECT(std::chrono::steady_clock::now() - t0 < 5s);
    stop = true;
    ::shutdown(fd, SHUT_RDWR);
    t.join();
    ::close(fd);
}

TEST(es_join_callback_reports_client_endpoint) {
    EchoServer e;
    const int fd = e.connect();
    EXPECT(eventually([&] { std::lock_guard l(e.m); return e.joined.size() == 1; }));
    sockaddr_storage ss{};
    socklen_t len = sizeof(ss);
    getsockname(fd, reinterpret_cast<sockaddr *>(&ss), &len);
    const SockAddr local = net::from_native(ss);
    {
        std::lock_guard l(e.m);
        EXPECT(e.joined[0].port == local.port);
    }
    ::close(fd);
}

TEST(es_several_packets_in_one_segment) {
    EchoServer e;
    const int fd = e.connect();
    std::vector<uint8_t> all;
    for (uint16_t id = 1; id <= 3; ++id) {
        auto b = raw_ltv(2 + id * 10, id, id * 10);
        all.insert(all.end(), b.begin(), b.end());
    }
    EXPECT(net::send_all(fd, all.data(), all.size()));
    EXPECT(eventually([&] { return e.count() == 3; }));
    std::lock_guard l(e.m);
    for (uint16_t id = 1; id <= 3; ++id) EXPECT(e.got[id - 1].first == id && e.got[id - 1].second.size() == id * 10u);
    ::close(fd);
}

TEST(es_packet_split_into_single_bytes) {
    EchoServer e;
    const int fd = e.connect();
    const auto b = raw_ltv(2 + 33, 9, 33);
    for (uint8_t c : b) {
        EXPECT(net::send_all(fd, &c, 1));
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    EXPECT(eventually([&] { return e.count() == 1; }));
    std::lock_guard l(e.m);
    EXPECT(e.got[0].first == 9 && e.got[0].second == std::vector<uint8_t>(33, 0xAB));
    ::close(fd);
}

TEST(es_empty_payload_packet) {
    EchoServer e;
    const int fd = e.connect();
    EXPECT(net::send_ltv(fd, 5, nullptr, 0));
    EXPECT(eventually([&] { return e.count() == 1; }));
    std::lock_guard l(e.m);
    EXPECT(e.got[0].first == 5 && e.got[0].second.empty());
    ::close(fd);
}

TEST(es_max_size_packet_accepted) { // 64 MiB payload: the reference cap
    EchoServer e;
    const int fd = e.connect();
    std::vector<uint8_t> p(net::kMaxControlPacket, 0x3C);
    std::thread t([&] { EXPECT(net::send_ltv(fd, 4, p.data(), p.size())); });
    EXPECT(eventually([&] { return e.count() == 1; }, 20000ms));
    t.join();
    std::lock_guard l(e.m);
    EXPECT(e.got.size() == 1 && e.got[0].second.size() == net::kMaxControlPacket && e.got[0].second.back() == 0x3C);
    EXPECT(e.closed.load() == 0);
    ::close(fd);
}

TEST(es_oversized_packet_closes_client_only) {
    EchoServer e;
    const int bad = e.connect(), good = e.connect();
    const auto b = raw_ltv(2 + net::kMaxControlPacket + 1, 3, 0); // header only: length over the cap
    EXPECT(net::send_all(bad, b.data(), b.size()));
    EXPECT(eventually([&] { return e.closed.load() == 1; }));
    uint8_t x;
    EXPECT(!net::recv_all(bad, &x, 1)); // server closed it
    std::vector<uint8_t> p(8, 1);
    EXPECT(net::send_ltv(good, 100, p.data(), p.size())); // the server keeps serving others
    auto r = net::recv_ltv(good);
    EXPECT(r && r->id == 101 && r->payload == p);
    ::close(bad);
    ::close(good);
}

TEST(es_malformed_length_closes_client) { // length field < 2 cannot hold the id
    EchoServer e;
    const int fd = e.connect();
    auto b = raw_ltv(1, 0, 0);
    EXPECT(net::send_all(fd, b.data(), b.size()));
    EXPECT(eventually([&] { return e.closed.load() == 1; }));
    EXPECT(e.count() == 0);
    ::close(fd);
}

TEST(es_many_concurrent_clients) {
    EchoServer e;
    constexpr int kClients = 32, kPackets = 50;
    std::atomic<int> ok{0};
    std::vector<std::thread> ts;
    for (int c = 0; c < kClients; ++c)
        ts.emplace_back([&, c] {
            const int fd = e.connect();
            bool good = fd >= 0;
            for (int k = 0; k < kPackets && good; ++k) {
                const uint32_t v = static_cast<uint32_t>(c * 1000 + k);
                good = net::send_ltv(fd, 100, reinterpret_cast<const uint8_t *>(&v), 4);
                auto r = net::recv_ltv(fd);
                uint32_t back = 0;
                if (r && r->payload.size() == 4) std::memcpy(&back, r->payload.data(), 4);
                good = good && r && r->id == 101 && back == v;
            }
            ok += good ? 1 : 0;
            ::close(fd);
        });
    for (auto &t : ts) t.join();
    EXPECT(ok.load() == kClients);
    EXPECT(e.count() == static_cast<size_t>(kClients * kPackets));
}

TEST(es_send_to_unknown_client_fails) {
    net::EventServer s(any_v4(), false);
    EXPECT(s.listen() && s.run_async());
    std::atomic<int> r{-1};
    s.post([&] { r = s.send_raw(loop_v4(1), 1, {}) ? 1 : 0; });
    EXPECT(eventually([&] { return r.load() != -1; }));
    EXPECT(r.load() == 0);
    s.interrupt();
    s.join();
}

TEST(es_close_from_handler_flushes_final_response) {
    net::EventServer s(any_v4(), false);
    std::atomic<int> closed{0};
    s.on_read([&](const SockAddr &a, uint16_t, const uint8_t *, size_t) {
        std::vector<uint8_t> bye(1 << 20, 0x77); // larger than one send: queued, then flushed by close_client
        s.send_raw(a, 9, bye);
        s.close_client(a);
    });
    s.on_close([&](const SockAddr &) { closed++; });
    EXPECT(s.listen() && s.run_async());
    const int fd = net::connect_tcp(loop_v4(s.port()), 2000);
    EXPECT(net::send_ltv(fd, 1, nullptr, 0));
    auto r = net::recv_ltv(fd);
    EXPECT(r && r->id == 9 && r->payload.size() == (1u << 20));
    uint8_t x;
    EXPECT(!net::recv_all(fd, &x, 1));
    EXPECT(eventually([&] { return closed.load() == 1; }));
    ::close(fd);
    s.interrupt();
    s.join();
}

TEST(es_tick_callback_runs_periodically) {
    EchoServer e;
    EXPECT(eventually([&] { return e.ticks.load() >= 2; }, 3000ms));
}

TEST(es_large_response_to_slow_reader) { // write queue + EPOLLOUT backpressure
    net::EventServer s(any_v4(), false);
    s.on_read([&](const SockAddr &a, uint16_t, const uint8_t *, size_t) {
        for (int k = 0; k < 8; ++k) s.send_raw(a, static_cast<uint16_t>(k), std::vector<uint8_t>(4 << 20, static_cast<uint8_t>(k)));
    });
    EXPECT(s.listen() && s.run_async());
    const int fd = net::connect_tcp(loop_v4(s.port()), 2000);
    EXPECT(net::send_ltv(fd, 1, nullptr, 0));
    std::this_thread::sleep_for(100ms); // the server's socket buffer fills up meanwhile
    for (int k = 0; k < 8; ++k) {
        auto r = net::recv_ltv(fd);
        EXPECT(r && r->id == k && r->payload.size() == (4u << 20) && r->payload[12345] == k);
    }
    ::close(fd);
    s.interrupt();
    s.join();
}

TEST(es_rebind_same_port_after_shutdown) {
    uint16_t port = 0;
    {
        net::EventServer a(any_v4(), false);
        EXPECT(a.listen() && a.run_async());
        port = a.port();
        const int fd = net::connect_tcp(loop_v4(port), 2000);
        EXPECT(fd >= 0);
        ::close(fd);
        a.interrupt();
        a.join();
    }
    net::EventServer b(any_v4(port), false);
    EXPECT(b.listen() && b.port() == port);
}

// ================================================================ MasterConnection (reference QueuedSocket)
namespace {
struct MasterSide {
    net::EventServer srv{any_v4(), false};
    std::mutex m;
    std::vector<SockAddr> clients;
    std::atomic<int> received{0};
    MasterSide() {
        srv.on_join([this](const SockAddr &a) {
            std::lock_guard l(m);
            clients.push_back(a);
        });
        srv.on_read([this](const SockAddr &, uint16_t, const uint8_t *, size_t) { received++; });
        EXPECT(srv.listen() && srv.run_async());
    }
    ~MasterSide() {
        srv.interrupt();
        srv.join();
    }
    template<typename P>
    void send_later(const P &p) { // to the first client, from the loop thread (EventServer::post keeps order)
        SockAddr to;
        {
            std::lock_guard l(m);
            to = clients.at(0);
        }
        srv.post([this, p, to] { srv.send_packet(to, p); });
    }
    bool wait_client() {
        return eventually([&] { std::lock_guard l(m); return !clients.empty(); });
    }
};
proto::M2CCollectiveCommsCommence commence(uint64_t tag, uint64_t seq) {
    proto::M2CCollectiveCommsCommence c;
    c.tag = tag;
    c.seq_nr = seq;
    return c;
}
} // namespace

TEST(mc_connect_fails_without_server) {
    uint16_t port = 0;
    int fd = net::listen_tcp(inetIPv4, 0, false, port);
    net::close_fd(fd); // the port is now closed
    net::MasterConnection c(loop_v4(port));
    EXPECT(!c.connect());
}

TEST(mc_receive_selects_packet_type) {
    MasterSide ms;
    net::MasterConnection c(loop_v4(ms.srv.port()));
    EXPECT(c.connect() && ms.wait_client());
    proto::M2CPeersPendingResponse pp;
    pp.peers_pending = true;
    ms.send_later(pp);
    ms.send_later(commence(5, 1));
    auto cm = c.receive<proto::M2CCollectiveCommsCommence>(nullptr, 3000ms); // skips the queued PeersPending
    EXPECT(cm && cm->tag == 5);
    auto p = c.receive<proto::M2CPeersPendingResponse>(nullptr, 3000ms);
    EXPECT(p && p->peers_pending);
    c.interrupt();
    c.join();
}

TEST(mc_predicate_picks_matching_packet) {
    MasterSide ms;
    net::MasterConnection c(loop_v4(ms.srv.port()));
    EXPECT(c.connect() && ms.wait_client());
    for (uint64_t t : {1, 2, 3}) ms.send_later(commence(t, t * 10));
    auto two = c.receive<proto::M2CCollectiveCommsCommence>([](const auto &x) { return x.tag == 2; }, 3000ms);
    EXPECT(two && two->seq_nr == 20);
    auto one = c.receive<proto::M2CCollectiveCommsCommence>([](const auto &x) { return x.tag == 1; }, 3000ms);
    auto three = c.receive<proto::M2CCollectiveCommsCommence>([](const auto &x) { return x.tag == 3; }, 3000ms);
    EXPECT(one && three && one->seq_nr == 10 && three->seq_nr == 30);
    c.interrupt();
    c.join();
}

TEST(mc_out_of_order_delivery_to_many_threads) {
    MasterSide ms;
    net::MasterConnection c(loop_v4(ms.srv.port()));
    EXPECT(c.connect() && ms.wait_client());
    constexpr int kThreads = 8;
    std::atomic<int> ok{0};
    std::vector<std::thread> ts;
    for (int k = 0; k < kThreads; ++k)
        ts.emplace_back([&, k] {
            auto p = c.receive<proto::M2CCollectiveCommsCommence>(
                [k](const auto &x) { return x.tag == static_cast<uint64_t>(k); }, 5000ms);
            ok += (p && p->seq_nr == static_cast<uint64_t>(100 + k)) ? 1 : 0;
        });
    std::this_thread::sleep_for(50ms);
    for (int k = kThreads - 1; k >= 0; --k) ms.send_later(commence(k, 100 + k)); // reverse order
    for (auto &t : ts) t.join();
    EXPECT(ok.load() == kThreads);
    c.interrupt();
    c.join();
}

TEST(mc_timeout_and_poll) {
    MasterSide ms;
    net::MasterConnection c(loop_v4(ms.srv.port()));
    EXPECT(c.connect());
    const auto t0 = std::chrono::steady_clock::now();
    EXPECT(!c.receive<proto::M2CCollectiveCommsAbort>(nullptr, 80ms));
    const auto dt = std::chrono::steady_clock::now() - t0;
    EXPECT(dt >= 70ms && dt < 5s);
    EXPECT(!c.receive<proto::M2CCollectiveCommsAbort>(nullptr, 0ms)); // poll
    c.interrupt();
    c.join();
}

// An op's abort polls only look (Client::abort_received): the packet stays queued for its completion protocol, however
// many threads of the op saw it first
TEST(mc_peek_leaves_packet_queued) {
    MasterSide ms;
    net::MasterConnection c(loop_v4(ms.srv.port()));
    EXPECT(c.connect() && ms.wait_client());
    auto is_abort_of = [](uint64_t tag) {
        return [tag](const proto::M2CCollectiveCommsAbort &a) { return a.tag == tag && a.aborted; };
    };
    EXPECT(!c.peek<proto::M2CCollectiveCommsAbort>(is_abort_of(7)));
    proto::M2CCollectiveCommsAbort ab;
    ab.tag = 7;
    ab.aborted = true;
    ms.send_later(ab);
    EXPECT(eventually([&] { return c.peek<proto::M2CCollectiveCommsAbort>(is_abort_of(7)); }));
    EXPECT(c.peek<proto::M2CCollectiveCommsAbort>(is_abort_of(7)));  // still there
    EXPECT(!c.peek<proto::M2CCollectiveCommsAbort>(is_abort_of(8))); // another op's tag
    auto a = c.receive<proto::M2CCollectiveCommsAbort>([](const auto &x) { return x.tag == 7; }, 0ms);
    EXPECT(a && a->aborted);
    EXPECT(!c.peek<proto::M2CCollectiveCommsAbort>(is_abort_of(7))); // taken by the receive
    c.interrupt();
    c.join();
}

TEST(mc_server_close_unblocks_receiver) {
    auto *ms = new MasterSide();
    net::MasterConnection c(loop_v4(ms->srv.port()));
    EXPECT(c.connect() && ms->wait_client());
    std::atomic<int> state{0};
    std::thread t([&] {
        auto p = c.receive<proto::M2CCollectiveCommsAbort>(); // waits forever unless the connection closes
        state = p ? 1 : 2;
    });
    std::this_thread::sleep_for(50ms);
    delete ms;
    t.join();
    EXPECT(state.load() == 2 && !c.is_open());
    c.interrupt();
    c.join();
}

TEST(mc_interrupt_unblocks_receiver) {
    MasterSide ms;
    net::MasterConnection c(loop_v4(ms.srv.port()));
    EXPECT(c.connect());
    std::atomic<bool> done{false};
    std::thread t([&] {
        c.receive<proto::M2CCollectiveCommsAbort>();
        done = true;
    });
    std::this_thread::sleep_for(50ms);
    c.interrupt();
    EXPECT(eventually([&] { return done.load(); }, 2000ms));
    t.join();
    c.join();
}

TEST(mc_concurrent_senders_keep_frames_intact) {
    MasterSide ms;
    net::MasterConnection c(loop_v4(ms.srv.port()));
    EXPECT(c.connect());
    std::vector<std::thread> ts;
    for (int k = 0; k < 8; ++k)
        ts.emplace_back([&, k] {
            for (int i = 0; i < 100; ++i) {
                proto::C2MCollectiveCommsInitiate p;
                p.tag = static_cast<uint64_t>(k * 1000 + i);
                p.count = 1;
                EXPECT(c.send(p));
            }
        });
    for (auto &t : ts) t.join();
    EXPECT(eventually([&] { return ms.received.load() == 800; }));
    c.interrupt();
    c.join();
}

// ================================================================ blocking socket helpers (reference BlockingIOSocket)
TEST(ltv_roundtrip_over_socketpair) {
    int sv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    std::vector<uint8_t> p = {1, 2, 3, 4, 5};
    EXPECT(net::send_ltv(sv[0], 0x1234, p.data(), p.size()));
    auto r = net::recv_ltv(sv[1]);
    EXPECT(r && r->id == 0x1234 && r->payload == p);
    ::close(sv[0]);
    ::close(sv[1]);
}

TEST(ltv_receive_rejects_length_over_cap) {
    int sv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    const auto b = raw_ltv(2 + 1000, 1, 0);
    EXPECT(net::send_all(sv[0], b.data(), b.size()));
    EXPECT(!net::recv_ltv(sv[1], 999).has_value());
    ::close(sv[0]);
    ::close(sv[1]);
}

TEST(recv_all_reports_eof_mid_message) {
    int sv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    uint8_t half[4] = {1, 2, 3, 4};
    EXPECT(net::send_all(sv[0], half, 4));
    ::close(sv[0]);
    uint8_t buf[8];
    EXPECT(!net::recv_all(sv[1], buf, 8));
    ::close(sv[1]);
}

TEST(send_all_large_buffer_with_concurrent_reader) {
    int sv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    std::vector<uint8_t> src(32 << 20), dst(32 << 20, 0);
    for (size_t i = 0; i < src.size(); ++i) src[i] = static_cast<uint8_t>(i * 131);
    std::thread r([&] { EXPECT(net::recv_all(sv[1], dst.data(), dst.size())); });
    EXPECT(net::send_all(sv[0], src.data(), src.size()));
    r.join();
    EXPECT(src == dst);
    ::close(sv[0]);
    ::close(sv[1]);
}

TEST(wait_readable_timeout_and_ready) {
    int sv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    EXPECT(net::wait_readable(sv[1], 30) == 0);
    uint8_t b = 1;
    EXPECT(net::send_all(sv[0], &b, 1));
    EXPECT(net::wait_readable(sv[1], 1000) == 1);
    ::close(sv[0]);
    ::close(sv[1]);
}

TEST(connect_to_closed_port_fails_fast) {
    uint16_t port = 0;
    int fd = net::listen_tcp(inetIPv4, 0, false, port);
    net::close_fd(fd);
    const auto t0 = std::chrono::steady_clock::now();
    EXPECT(net::connect_tcp(loop_v4(port), 2000) < 0);
    EXPECT(std::chrono::steady_clock::now() - t0 < 5s);
}

TEST(listen_bump_finds_next_free_port) {
    uint16_t a = 0, b = 0;
    int fa = net::listen_tcp(inetIPv4, 0, false, a);
    int fb = net::listen_tcp(inetIPv4, a, true, b);
    EXPECT(fa >= 0 && fb >= 0 && b != a);
    net::close_fd(fa);
    net::close_fd(fb);
}

// ================================================================ MuxConn (reference MultiplexedIOSocket)
namespace {
std::pair<net::MuxConn *, net::MuxConn *> mux_pair2() {
    int sv[2];
    socketpair(AF_UNIX, SOCK_STREAM, 0, sv);
    auto *tx = new net::MuxConn(sv[0], net::MuxConn::Mode::Tx, SockAddr{});
    auto *rx = new net::MuxConn(sv[1], net::MuxConn::Mode::Rx, SockAddr{});
    tx->start();
    rx->start();
    return {tx, rx};
}
} // namespace

TEST(mux_oversized_frame_closes_connection) { // reference pops and silently drops it (Appendix C #8)
    int sv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    auto *rx = new net::MuxConn(sv[1], net::MuxConn::Mode::Rx, SockAddr{});
    rx->start();
    uint8_t h[net::kMuxHeaderBytes];
    net::mux_frame_header(h, net::kMuxMaxFrame + 1, 1, 1);
    EXPECT(net::send_all(sv[0], h, sizeof(h)));
    EXPECT(eventually([&] { return !rx->is_open(); }, 3000ms));
    ::close(sv[0]);
    delete rx;
}

TEST(mux_frame_straddles_sinks_in_fifo_order) {
    // a frame larger than the oldest sink fills it and continues in the next sinks of the tag (posted before or after
    // it arrived); nothing is written past a sink (guard bytes stay untouched)
    auto [tx, rx] = mux_pair2();
    std::vector<uint8_t> big(250);
    for (size_t i = 0; i < big.size(); ++i) big[i] = static_cast<uint8_t>(i);
    std::vector<uint8_t> a(100 + 8, 0xee), b(100 + 8, 0xee), c(100 + 8, 0xee);
    auto sa = rx->post_sink(3, 1, a.data(), 100);
    EXPECT(tx->send_frame(3, 1, big.data(), big.size()));
    EXPECT(eventually([&] { return net::MuxConn::sink_progress(sa) == 100; }, 2000ms));
    auto sb = rx->post_sink(3, 1, b.data(), 100);
    auto sc = rx->post_sink(3, 1, c.data(), 100);
    EXPECT(eventually([&] { return net::MuxConn::sink_progress(sc) == 50; }, 2000ms));
    EXPECT(net::MuxConn::sink_progress(sb) == 100);
    EXPECT(std::equal(a.begin(), a.begin() + 100, big.begin()) && a[100] == 0xee);
    EXPECT(std::equal(b.begin(), b.begin() + 100, big.begin() + 100) && b[100] == 0xee);
    EXPECT(std::equal(c.begin(), c.begin() + 50, big.begin() + 200) && c[50] == 0xee);
    rx->remove_sink(3, sa);
    rx->remove_sink(3, sb);
    rx->remove_sink(3, sc);
    delete tx;
    delete rx;
}

TEST(mux_many_tags_from_many_senders) {
    auto [tx, rx] = mux_pair2();
    constexpr int kTags = 16, kFrames = 8, kLen = 4096;
    std::vector<std::vector<uint8_t>> dst(kTags, std::vector<uint8_t>(kFrames * kLen, 0));
    for (int t = 0; t < kTags; ++t) rx->post_sink(static_cast<uint64_t>(t), 9, dst[t].data(), dst[t].size());
    std::vector<std::thread> ss;
    for (int s = 0; s < 4; ++s)
        ss.emplace_back([&, s] {
            for (int t = s; t < kTags; t += 4)
                for (int f = 0; f < kFrames; ++f) {
                    std::vector<uint8_t> p(kLen, static_cast<uint8_t>(t * 16 + f));
                    tx->send_frame(static_cast<uint64_t>(t), 9, p.data(), p.size());
                }
        });
    for (auto &t : ss) t.join();
    for (int t = 0; t < kTags; ++t) {
        EXPECT(rx->wait_sink(static_cast<uint64_t>(t), dst[t].size(), 5s) == dst[t].size());
        for (int f = 0; f < kFrames; ++f) EXPECT(dst[t][static_cast<size_t>(f) * kLen] == static_cast<uint8_t>(t * 16 + f));
        rx->remove_sink(static_cast<uint64_t>(t));
    }
    delete tx;
    delete rx;
}

TEST(mux_send_jobs_run_in_fifo_order) {
    auto [tx, rx] = mux_pair2();
    std::mutex m;
    std::vector<int> order;
    std::atomic<int> done{0};
    for (int k = 0; k < 50; ++k)
        tx->post_send_job([&, k] {
            std::lock_guard l(m);
            order.push_back(k);
            done++;
        });
    EXPECT(eventually([&] { return done.load() == 50; }));
    for (int k = 0; k < 50; ++k) EXPECT(order[k] == k);
    delete tx;
    delete rx;
}

TEST(mux_send_on_closed_connection_fails) {
    auto [tx, rx] = mux_pair2();
    delete rx;
    std::vector<uint8_t> p(1 << 20, 1);
    bool failed = false;
    for (int k = 0; k < 64 && !failed; ++k) failed = !tx->send_frame(1, 1, p.data(), p.size());
    EXPECT(failed);
    delete tx;
}
