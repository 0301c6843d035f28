// Native unit tests of internal components (no gtest in the image: a tiny self-registering harness).
// Built as build/pccl_unit_tests, run by tests/test_native.py; also the target of the sanitizer build
// (cmake -DPCCL_SANITIZE=ON: ASan + UBSan on host code).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "common/numeric.hpp"
#include "kernels/host_kernels.hpp"
#include "master/topology.hpp"
#include "net/event_server.hpp"
#include "net/mux.hpp"
#include "net/socket.hpp"
#include "proto/packets.hpp"
#include "client/ipc.hpp"
#include "client/vmm_share.hpp"
#include "client/pools.hpp"

#include <signal.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <thread>

using namespace pccl;
using namespace std::chrono_literals;

#include "harness.hpp"

template<typename P>
static P roundtrip(const P &p) {
    auto bytes = proto::encode_with_id(p);
    EXPECT(bytes.size() >= 2);
    const uint16_t id = static_cast<uint16_t>((bytes[0] << 8) | bytes[1]);
    EXPECT(id == static_cast<uint16_t>(P::kId));
    auto back = proto::decode_payload<P>(bytes.data() + 2, bytes.size() - 2);
    EXPECT(back.has_value());
    // truncated payloads must be rejected, never over-read
    if (bytes.size() > 3) EXPECT(!proto::decode_payload<P>(bytes.data() + 2, bytes.size() - 3).has_value());
    return back ? *back : P{};
}

TEST(packet_collective_initiate) {
    proto::C2MCollectiveCommsInitiate p;
    p.tag = 0x0102030405060708ull;
    p.count = 12345;
    p.data_type = DType::BF16;
    p.op = ReduceOp::Max;
    auto q = roundtrip(p);
    EXPECT(q.tag == p.tag && q.count == p.count && q.data_type == p.data_type && q.op == p.op);
}

TEST(packet_sync_shared_state) {
    proto::C2MSyncSharedState p;
    p.revision = 77;
    p.strategy = SyncStrategy::TxOnly;
    for (int i = 0; i < 5; ++i) {
        proto::SharedStateHashEntry e;
        e.key = "layer." + std::to_string(i) + ".weight";
        e.hash = 1000u + i;
        e.hash_type = HashType::Simple;
        e.num_elements = 4096u * i;
        e.data_type = DType::F32;
        e.allow_content_inequality = i % 2;
        p.entries.push_back(e);
    }
    auto q = roundtrip(p);
    EXPECT(q.revision == 77 && q.strategy == SyncStrategy::TxOnly && q.entries == p.entries);
}

TEST(packet_complete) {
    proto::C2MCollectiveCommsComplete p;
    p.tag = 9;
    p.was_aborted = true;
    auto q = roundtrip(p);
    EXPECT(q.tag == 9 && q.was_aborted);
}

// Appended extension fields (host token, single_host, shared-state IPC) are optional on decode, so packets from a
// reference implementation (without them) still parse.
TEST(packet_extensions_backward_compatible) {
    proto::C2MRequestSessionRegistration r;
    r.peer_group = 3;
    r.p2p_port = 1;
    r.ss_port = 2;
    r.bm_port = 4;
    r.host_token = "boot-id|host";
    auto bytes = proto::encode_with_id(r);
    auto full = proto::decode_payload<proto::C2MRequestSessionRegistration>(bytes.data() + 2, bytes.size() - 2);
    EXPECT(full && full->host_token == "boot-id|host" && full->bm_port == 4);
    const size_t legacy = 2 + 4 + 1 + 6; // id + group + bool + 3 ports: the reference layout
    auto old = proto::decode_payload<proto::C2MRequestSessionRegistration>(bytes.data() + 2, legacy - 2);
    EXPECT(old && old->host_token.empty() && old->peer_group == 3 && old->bm_port == 4);

    proto::M2CP2PConnectionsEstablished e;
    e.success = true;
    e.ring_order = {Uuid::random(), Uuid::random()};
    e.single_host = true;
    bytes = proto::encode_with_id(e);
    auto fe = proto::decode_payload<proto::M2CP2PConnectionsEstablished>(bytes.data() + 2, bytes.size() - 2);
    EXPECT(fe && fe->single_host && fe->ring_order == e.ring_order);
    auto oe = proto::decode_payload<proto::M2CP2PConnectionsEstablished>(bytes.data() + 2, bytes.size() - 3);
    EXPECT(oe && !oe->single_host && oe->ring_order == e.ring_order);

    proto::S2CSharedStateIpcResponse s;
    s.revision = 9;
    s.pid = 1234;
    proto::SharedStateIpcEntry ie;
    ie.key = "w";
    ie.size_bytes = 4096;
    ie.mode = 1;
    ie.device = 2;
    ie.offset = 512;
    ie.raw_ptr = 0xdeadbeef;
    ie.handle[0] = 7;
    ie.handle[63] = 9;
    s.entries.push_back(ie);
    auto q = roundtrip(s);
    EXPECT(q.revision == 9 && q.pid == 1234 && q.entries.size() == 1 && q.entries[0].key == "w" &&
           q.entries[0].mode == 1 && q.entries[0].device == 2 && q.entries[0].offset == 512 &&
           q.entries[0].raw_ptr == 0xdeadbeef && q.entries[0].handle[0] == 7 && q.entries[0].handle[63] == 9);
    // mode 2 (VMM fd shares): segment size and the extra segment handles travel too; mode 0/1 entries carry none
    proto::SharedStateIpcEntry v = ie;
    v.key = "big";
    v.mode = 2;
    v.seg_bytes = 1 << 30;
    v.more_handles.resize(2);
    v.more_handles[0][5] = 11;
    v.more_handles[1][63] = 13;
    s.entries.push_back(v);
    proto::SharedStateIpcEntry plain;
    plain.key = "cpu";
    plain.size_bytes = 8;
    s.entries.push_back(plain);
    auto q2 = roundtrip(s);
    EXPECT(q2.entries.size() == 3 && q2.entries[1].mode == 2 && q2.entries[1].seg_bytes == (1u << 30) &&
           q2.entries[1].more_handles.size() == 2 && q2.entries[1].more_handles[0][5] == 11 &&
           q2.entries[1].more_handles[1][63] == 13 && q2.entries[0].more_handles.empty() &&
           q2.entries[2].key == "cpu" && q2.entries[2].mode == 0 && q2.entries[2].seg_bytes == 0);
    proto::C2SRequestSharedStateIpc rq;
    rq.keys = {"a", "b"};
    rq.host_token = "t";
    rq.pid = 5;
    auto rq2 = roundtrip(rq);
    EXPECT(rq2.keys == rq.keys && rq2.host_token == "t" && rq2.pid == 5);
}

// CRC-32C split algebra used by the HIP kernel: raw(A || B) = shift(raw(A), |B|) ^ raw(B)
TEST(host_reduce3_matches_scalar_bitwise) {
    // the 3-operand host reduce (AVX-512 path for bf16 / fp32 sums, also behind host_reduce) must equal the scalar
    // definition (fp32 add, round to nearest even) bit for bit, NaN / inf / denormal / rounding-tie inputs included,
    // at lengths that exercise the vector body and the tail
    std::mt19937_64 rng(11);
    for (size_t n : {size_t(1), size_t(15), size_t(16), size_t(17), size_t(1000), size_t(65537)}) {
        std::vector<uint16_t> a(n), b(n), want(n), got(n);
        for (size_t i = 0; i < n; ++i) {
            a[i] = static_cast<uint16_t>(rng());
            b[i] = static_cast<uint16_t>(rng());
        }
        if (n > 8) {
            a[0] = 0x7fc0; b[1] = 0xff81; a[2] = 0x7f80; b[2] = 0xff80; a[3] = 0x0001; b[3] = 0x0001;
            a[4] = 0x3f80; b[4] = 0x3380; // 1 + 2^-24-ish: a rounding tie
        }
        for (ReduceOp op : {ReduceOp::Sum, ReduceOp::Max}) {
            if (op == ReduceOp::Sum) {
                for (size_t i = 0; i < n; ++i)
                    want[i] = num::f32_to_bf16(num::bf16_to_f32(a[i]) + num::bf16_to_f32(b[i]));
            } else { // max: the scalar element op of host_reduce is the definition
                want = a;
                EXPECT(kernels::host_reduce(want.data(), b.data(), n, DType::BF16, op));
            }
            EXPECT(kernels::host_reduce3(got.data(), a.data(), b.data(), n, DType::BF16, op));
            for (size_t i = 0; i < n; ++i) {
                const bool both_nan = (want[i] & 0x7fff) > 0x7f80 && (got[i] & 0x7fff) > 0x7f80;
                // an op on two NaNs may return either (quieted) payload: x86 returns the first source operand's,
                // and which operand comes first is up to the compiler's / the intrinsics' operand order
                if (want[i] != got[i] && !both_nan) {
                    std::printf("    n %zu op %d i %zu a %04x b %04x want %04x got %04x\n", n, static_cast<int>(op), i, a[i], b[i], want[i], got[i]);
                    EXPECT(want[i] == got[i]);
                    break;
                }
            }
        }
        std::vector<float> fa(n), fb(n), fw(n), fg(n);
        for (size_t i = 0; i < n; ++i) {
            fa[i] = static_cast<float>(static_cast<int64_t>(rng() % 2000001) - 1000000) * 1e-3f;
            fb[i] = static_cast<float>(static_cast<int64_t>(rng() % 2000001) - 1000000) * 1e-5f;
        }
        for (size_t i = 0; i < n; ++i) fw[i] = fa[i] + fb[i];
        EXPECT(kernels::host_reduce3(fg.data(), fa.data(), fb.data(), n, DType::F32, ReduceOp::Sum));
        EXPECT(std::memcmp(fw.data(), fg.data(), n * 4) == 0);
    }
    // throughput of the bf16 path on this host (informational)
    const size_t n = 16u << 20;
    std::vector<uint16_t> a(n, 0x3f80), b(n, 0x4000), o(n);
    kernels::host_reduce3(o.data(), a.data(), b.data(), n, DType::BF16, ReduceOp::Sum);
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 4; ++r) kernels::host_reduce3(o.data(), a.data(), b.data(), n, DType::BF16, ReduceOp::Sum);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 4;
    std::printf("    host_reduce3 bf16 sum: %.1f GB/s of output (one thread)\n", n * 2 / s / 1e9);
    EXPECT(o[0] == 0x4040); // 1 + 2 = 3
}

TEST(crc32c_split_combine) {
    std::vector<uint8_t> m(100003);
    uint64_t x = 88172645463325252ull;
    for (auto &b : m) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        b = static_cast<uint8_t>(x);
    }
    const uint32_t ref = kernels::crc32c_sw(m.data(), m.size());
    EXPECT(kernels::crc32c_finish(kernels::crc32c_raw_update(0, m.data(), m.size()), m.size()) == ref);
    for (size_t cut : {size_t(0), size_t(1), size_t(7), size_t(4096), size_t(65536), m.size() - 3, m.size()}) {
        const uint32_t ra = kernels::crc32c_raw_update(0, m.data(), cut);
        const uint32_t rb = kernels::crc32c_raw_update(0, m.data() + cut, m.size() - cut);
        EXPECT(kernels::crc32c_finish(kernels::crc32c_shift(ra, m.size() - cut) ^ rb, m.size()) == ref);
        // continuing from a state equals the split form
        EXPECT(kernels::crc32c_raw_update(ra, m.data() + cut, m.size() - cut) ==
               (kernels::crc32c_shift(ra, m.size() - cut) ^ rb));
    }
    EXPECT(kernels::crc32c_gf_mul(1u << 31, 0x12345678u) == 0x12345678u); // 1 * b = b
}

static double brute_force_tour(const std::vector<std::vector<double>> &c) {
    const int n = static_cast<int>(c.size());
    std::vector<int> perm(n - 1);
    for (int i = 0; i < n - 1; ++i) perm[i] = i + 1;
    double best = 1e300;
    do {
        double cost = c[0][perm[0]];
        for (int i = 0; i + 1 < n - 1; ++i) cost += c[perm[i]][perm[i + 1]];
        cost += c[perm.back()][0];
        best = std::min(best, cost);
    } while (std::next_permutation(perm.begin(), perm.end()));
    return best;
}

TEST(atsp_exact_matches_brute_force) {
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> d(1.0, 100.0);
    for (int n = 3; n <= 8; ++n) {
        for (int rep = 0; rep < 5; ++rep) {
            std::vector<std::vector<double>> c(n, std::vector<double>(n, 0.0));
            for (int i = 0; i < n; ++i)
                for (int j = 0; j < n; ++j)
                    if (i != j) c[i][j] = d(rng);
            auto r = master::solve_atsp(c, 12, 1000, 4, 42);
            EXPECT(r.ok && r.optimal && static_cast<int>(r.tour.size()) == n);
            EXPECT(std::fabs(r.cost - brute_force_tour(c)) < 1e-6);
        }
    }
}

TEST(atsp_heuristic_within_2pct_of_exact) {
    // 50 random asymmetric instances, n = 12..16: the heuristic (exact search disabled) against Held-Karp
    std::mt19937_64 rng(2024);
    double worst = 0, sum = 0;
    int optimal_hits = 0;
    for (int inst = 0; inst < 50; ++inst) {
        const int n = 12 + inst % 5;
        std::uniform_real_distribution<double> d(1.0, 100.0);
        std::vector<std::vector<double>> c(n, std::vector<double>(n, 0));
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) c[i][j] = i == j ? -1 : d(rng);
        const auto exact = master::solve_atsp(c, 20, 1000, 1, 42);
        const auto heur = master::solve_atsp(c, 0, 1000, 4, 42);
        EXPECT(exact.ok && exact.optimal && heur.ok && !heur.optimal);
        const double gap = heur.cost / exact.cost - 1.0;
        EXPECT(gap >= -1e-9);
        worst = std::max(worst, gap);
        sum += gap;
        optimal_hits += gap < 1e-9;
    }
    std::printf("    atsp heuristic vs Held-Karp: mean gap %.3f %%, worst %.3f %%, optimal %d / 50\n", 100 * sum / 50,
                100 * worst, optimal_hits);
    EXPECT(worst <= 0.02);
}

TEST(atsp_64_nodes_within_budget) {
    std::mt19937_64 rng(5);
    std::uniform_real_distribution<double> d(1.0, 100.0);
    const int n = 64;
    std::vector<std::vector<double>> c(n, std::vector<double>(n, 0));
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) c[i][j] = i == j ? -1 : d(rng);
    const auto t0 = std::chrono::steady_clock::now();
    const auto r = master::solve_atsp(c, 8, 1000, 4, 42); // the reference's synchronous budget
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    EXPECT(r.ok && r.tour.size() == 64u && s < 1.5);
    std::vector<int> seen = r.tour;
    std::sort(seen.begin(), seen.end());
    for (int i = 0; i < n; ++i) EXPECT(seen[i] == i);
    // a greedy nearest-neighbour tour is a weak upper bound: the search must beat it
    std::vector<int> nn = {0};
    std::vector<bool> used(n, false);
    used[0] = true;
    for (int k = 1; k < n; ++k) {
        int b = -1;
        for (int j = 0; j < n; ++j)
            if (!used[j] && (b < 0 || c[nn.back()][j] < c[nn.back()][b])) b = j;
        used[b] = true;
        nn.push_back(b);
    }
    double nn_cost = 0;
    for (int i = 0; i < n; ++i) nn_cost += c[nn[i]][nn[(i + 1) % n]];
    std::printf("    atsp n=64: %.3f s, cost %.1f (nearest neighbour %.1f)\n", s, r.cost, nn_cost);
    EXPECT(r.cost < nn_cost);
    // cancellation returns promptly with a valid tour
    std::atomic<bool> cancel{true};
    const auto t1 = std::chrono::steady_clock::now();
    const auto rc = master::solve_atsp(c, 8, 30000, 16, 42, &cancel);
    EXPECT(rc.ok && std::chrono::steady_clock::now() - t1 < std::chrono::seconds(2));
}

TEST(optimizer_pool_bounds_threads_and_queue) {
    master::OptimizerPool pool(4, 64);
    std::atomic<int> ran{0};
    std::atomic<bool> release{false};
    int accepted = 0;
    for (uint64_t k = 0; k < 100; ++k) // 100 optimize rounds of 100 groups while the first ones block
        accepted += pool.submit(k, [&] {
            while (!release.load()) std::this_thread::sleep_for(1ms);
            ++ran;
        });
    EXPECT(pool.thread_count() <= 4);
    EXPECT(accepted <= 4 + 64 && accepted >= 64);
    EXPECT(!pool.submit(0, [] {})); // key 0 still queued / running
    release = true;
    for (int i = 0; i < 500 && ran.load() < accepted; ++i) std::this_thread::sleep_for(10ms);
    EXPECT(ran.load() == accepted);
    for (int i = 0; i < 100 && pool.pending() > 0; ++i) std::this_thread::sleep_for(5ms);
    for (int round = 0; round < 100; ++round) pool.submit(7, [&] { ++ran; }); // one group, 100 rounds
    EXPECT(pool.thread_count() <= 4);
    pool.stop();
}

TEST(atsp_heuristic_is_valid_tour) {
    const int n = 40;
    std::mt19937_64 rng(3);
    std::uniform_real_distribution<double> d(1.0, 100.0);
    std::vector<std::vector<double>> c(n, std::vector<double>(n, 0.0));
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
            if (i != j) c[i][j] = d(rng);
    auto r = master::solve_atsp(c, 12, 300, 4, 1);
    EXPECT(r.ok && static_cast<int>(r.tour.size()) == n);
    std::vector<int> seen(n, 0);
    for (int v : r.tour) seen[v]++;
    for (int s : seen) EXPECT(s == 1);
}

TEST(bandwidth_store_population) {
    master::BandwidthStore s;
    Uuid a = Uuid::random(), b = Uuid::random(), c = Uuid::random();
    s.register_peer(a);
    s.register_peer(b);
    s.register_peer(c);
    EXPECT(!s.fully_populated());
    EXPECT(s.missing_for(a).size() == 4);
    for (auto *x : {&a, &b, &c})
        for (auto *y : {&a, &b, &c})
            if (x != y) s.store(*x, *y, 1000.0);
    EXPECT(s.fully_populated());
    s.unregister_peer(c);
    EXPECT(s.fully_populated() && s.num_peers() == 2);
}

TEST(bf16_fp8_rne) {
    EXPECT(num::f32_to_bf16(1.0f) == 0x3f80);
    EXPECT(num::bf16_to_f32(num::f32_to_bf16(3.140625f)) == 3.140625f);
    // round-to-nearest-even at the tie
    EXPECT(num::f32_to_bf16(1.00390625f) == 0x3f80);
}

TEST(simplehash_host_small) {
    std::vector<uint8_t> one{0};
    const uint32_t h0 = kernels::simplehash_host(one.data(), 1);
    one[0] = 1;
    EXPECT(kernels::simplehash_host(one.data(), 1) != h0);
}

// ---------------------------------------------------------------- transport (reference tinysockets/tests)
TEST(listen_port_bumping) {
    uint16_t a = 0, b = 0;
    const int fa = net::listen_tcp(inetIPv4, 0, false, a);
    EXPECT(fa >= 0 && a != 0);
    const int fb = net::listen_tcp(inetIPv4, a, true, b); // taken -> bumped
    EXPECT(fb >= 0 && b > a);
    uint16_t c = 0;
    EXPECT(net::listen_tcp(inetIPv4, a, false, c) < 0); // taken, no bump -> fail
    ::close(fa);
    ::close(fb);
}

static std::pair<net::MuxConn *, net::MuxConn *> mux_pair() {
    int sv[2];
    EXPECT(::socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    auto *tx = new net::MuxConn(sv[0], net::MuxConn::Mode::Tx, SockAddr{});
    auto *rx = new net::MuxConn(sv[1], net::MuxConn::Mode::Rx, SockAddr{});
    tx->start();
    rx->start();
    return {tx, rx};
}

TEST(mux_sink_receives_frames_in_order) {
    auto [tx, rx] = mux_pair();
    std::vector<uint8_t> src(3 << 20), dst(3 << 20, 0);
    for (size_t i = 0; i < src.size(); ++i) src[i] = static_cast<uint8_t>(i * 7 + 3);
    rx->post_sink(5, 1, dst.data(), dst.size());
    std::thread s([&] {
        for (size_t off = 0; off < src.size(); off += 1 << 20) tx->send_frame(5, 1, src.data() + off, 1 << 20);
    });
    EXPECT(rx->wait_sink(5, dst.size(), 10s) == dst.size());
    s.join();
    EXPECT(src == dst);
    rx->remove_sink(5);
    delete tx;
    delete rx;
}

TEST(mux_early_frames_queue_until_sink_posted) {
    auto [tx, rx] = mux_pair();
    std::vector<uint8_t> a(1000, 1), b(500, 2), dst(1500, 0);
    tx->send_frame(9, 4, a.data(), a.size());
    tx->send_frame(9, 4, b.data(), b.size());
    std::this_thread::sleep_for(50ms); // both frames are queued by the RX thread before the sink exists
    rx->post_sink(9, 4, dst.data(), dst.size());
    EXPECT(rx->wait_sink(9, dst.size(), 5s) == dst.size());
    EXPECT(dst[0] == 1 && dst[999] == 1 && dst[1000] == 2 && dst[1499] == 2);
    rx->remove_sink(9);
    delete tx;
    delete rx;
}

TEST(mux_stale_ctr_frames_dropped_and_tags_independent) {
    auto [tx, rx] = mux_pair();
    std::vector<uint8_t> stale(64, 0xEE), good(64, 0x11), other(32, 0x22);
    tx->send_frame(1, 3, stale.data(), stale.size()); // aborted earlier op with the same tag
    tx->send_frame(2, 7, other.data(), other.size());  // another concurrent op
    tx->send_frame(1, 4, good.data(), good.size());
    std::this_thread::sleep_for(50ms);
    std::vector<uint8_t> dst(64, 0);
    rx->post_sink(1, 4, dst.data(), dst.size());
    EXPECT(rx->wait_sink(1, 64, 5s) == 64);
    EXPECT(dst == good);
    auto f = rx->recv_frame(2, 7, 1s);
    EXPECT(f.has_value() && *f == other);
    rx->remove_sink(1);
    delete tx;
    delete rx;
}

TEST(mux_sink_fifo_fills_oldest_sink_first) {
    // a ring op posts step g+1's sink while step g's still receives: frames fill the sinks in posting order
    auto [tx, rx] = mux_pair();
    std::vector<uint8_t> s1(3000), s2(2000), d1(3000, 0), d2(2000, 0);
    for (size_t i = 0; i < s1.size(); ++i) s1[i] = static_cast<uint8_t>(i * 3 + 1);
    for (size_t i = 0; i < s2.size(); ++i) s2[i] = static_cast<uint8_t>(i * 5 + 2);
    auto h1 = rx->post_sink(4, 2, d1.data(), d1.size());
    auto h2 = rx->post_sink(4, 2, d2.data(), d2.size());
    tx->send_frame(4, 2, s1.data(), 1000);
    tx->send_frame(4, 2, s1.data() + 1000, 2000);
    tx->send_frame(4, 2, s2.data(), 2000);
    EXPECT(rx->wait_sink(h1, d1.size(), 5s) == d1.size());
    EXPECT(rx->wait_sink(h2, d2.size(), 5s) == d2.size());
    EXPECT(d1 == s1 && d2 == s2);
    rx->remove_sink(4, h1);
    rx->remove_sink(4, h2);
    delete tx;
    delete rx;
}

TEST(mux_sink_fifo_late_second_sink_takes_queued_frames) {
    // frames of the next step arrive before its sink exists: queued, then copied in when it is posted
    auto [tx, rx] = mux_pair();
    std::vector<uint8_t> a(4096, 7), b(1024, 9), d1(4096, 0), d2(1024, 0);
    auto h1 = rx->post_sink(6, 1, d1.data(), d1.size());
    tx->send_frame(6, 1, a.data(), a.size());
    tx->send_frame(6, 1, b.data(), b.size());
    EXPECT(rx->wait_sink(h1, d1.size(), 5s) == d1.size());
    std::this_thread::sleep_for(50ms); // the second frame is queued (sink 1 full, no sink 2 yet)
    rx->remove_sink(6, h1);
    auto h2 = rx->post_sink(6, 1, d2.data(), d2.size());
    EXPECT(rx->wait_sink(h2, d2.size(), 5s) == d2.size());
    EXPECT(d1 == a && d2 == b);
    rx->remove_sink(6, h2);
    delete tx;
    delete rx;
}

TEST(vmm_share_serves_fds_by_random_id_only) {
    // the fd service is generic over fds: a pipe stands in for an exported VMM allocation
    int p[2];
    EXPECT(::pipe(p) == 0);
    auto &svc = client::VmmShare::instance();
    const uint64_t id = svc.publish(p[1]); // the service owns the write end now
    const uint64_t id2 = svc.publish(::dup(p[1]));
    EXPECT(id != 0 && id2 != 0 && id != id2);
    EXPECT(id2 != id + 1 && id != id2 + 1); // random capabilities, not a sequence
    const int got = client::VmmShare::fetch(::getpid(), svc.nonce(), id, 2000);
    EXPECT(got >= 0);
    if (got >= 0) {
        const char msg[] = "vmm";
        EXPECT(::write(got, msg, 3) == 3); // the duplicate refers to the published pipe
        char buf[4] = {};
        EXPECT(::read(p[0], buf, 3) == 3 && std::string(buf) == "vmm");
        ::close(got);
    }
    EXPECT(client::VmmShare::fetch(::getpid(), svc.nonce(), id ^ 0x5a5a5a5aULL, 2000) < 0); // unknown id
    EXPECT(client::VmmShare::fetch(::getpid(), svc.nonce() ^ 1, id, 500) < 0);             // wrong socket
    svc.retract(id);
    EXPECT(client::VmmShare::fetch(::getpid(), svc.nonce(), id, 2000) < 0); // retracted
    svc.retract(id2);
    ::close(p[0]);
}

TEST(ipc_zombie_leader_with_live_threads_is_not_quiesced) {
    // The case the IPC abort drain must not get wrong: the group leader of a peer is a zombie while other threads of
    // the process still run (they still hold the address space, so its GPU queues may still be live).
    int go[2];
    EXPECT(::pipe(go) == 0);
    const pid_t child = ::fork();
    if (child == 0) {
        for (int i = 0; i < 4; ++i)
            std::thread([] {
                while (true) std::this_thread::sleep_for(1ms);
            }).detach();
        if (::write(go[1], "r", 1) != 1) ::_exit(3);
        ::syscall(SYS_exit, 0); // only the leader thread exits
    }
    char c;
    EXPECT(::read(go[0], &c, 1) == 1);
    bool zombie_leader = false;
    for (int i = 0; i < 400 && !zombie_leader; ++i) { // leader turns zombie, its threads keep running
        zombie_leader = !client::ipc_pid_alive_for_test(child);
        if (!zombie_leader) std::this_thread::sleep_for(5ms);
    }
    EXPECT(zombie_leader);
    EXPECT(!client::ipc_pid_quiesced_for_test(child));
    ::kill(child, SIGKILL);
    bool quiet = false;
    for (int i = 0; i < 400 && !quiet; ++i) { // not reaped yet: quiesced once every thread is past do_exit
        quiet = client::ipc_pid_quiesced_for_test(child);
        if (!quiet) std::this_thread::sleep_for(5ms);
    }
    EXPECT(quiet);
    EXPECT(client::ipc_pid_alive_for_test(::getpid()) && !client::ipc_pid_quiesced_for_test(::getpid()));
    int st = 0;
    ::waitpid(child, &st, 0);
    EXPECT(client::ipc_pid_quiesced_for_test(child)); // reaped
    ::close(go[0]);
    ::close(go[1]);
}

TEST(mux_peer_close_is_detected) {
    auto [tx, rx] = mux_pair();
    std::vector<uint8_t> dst(128);
    rx->post_sink(1, 1, dst.data(), dst.size());
    delete tx; // closes the socket
    const auto t0 = std::chrono::steady_clock::now();
    rx->wait_sink(1, dst.size(), 5s);
    EXPECT(!rx->is_open());
    EXPECT(std::chrono::steady_clock::now() - t0 < 4s);
    rx->remove_sink(1);
    delete rx;
}

TEST(event_server_ltv_roundtrip_and_close_callbacks) {
    SockAddr any{};
    any.inet.protocol = inetIPv4;
    any.port = 0;
    net::EventServer srv(any, false);
    std::atomic<int> got{0}, closed{0};
    std::atomic<size_t> got_len{0};
    srv.on_read([&](const SockAddr &a, uint16_t id, const uint8_t *p, size_t n) {
        got_len = n;
        got += id == 42 ? 1 : 0;
        srv.send_raw(a, 43, std::vector<uint8_t>(p, p + n));
    });
    srv.on_close([&](const SockAddr &) { closed++; });
    EXPECT(srv.listen() && srv.run_async());
    SockAddr addr{};
    addr.inet.protocol = inetIPv4;
    addr.inet.ipv4.data[0] = 127;
    addr.inet.ipv4.data[3] = 1;
    addr.port = srv.port();
    const int fd = net::connect_tcp(addr, 2000);
    EXPECT(fd >= 0);
    std::vector<uint8_t> big(8 << 20, 0x5A); // large control packet
    EXPECT(net::send_ltv(fd, 42, big.data(), big.size()));
    auto back = net::recv_ltv(fd);
    EXPECT(back.has_value() && back->id == 43 && back->payload.size() == big.size());
    ::close(fd);
    for (int i = 0; i < 200 && closed.load() == 0; ++i) std::this_thread::sleep_for(10ms);
    EXPECT(got.load() == 1 && got_len.load() == big.size() && closed.load() == 1);
    srv.interrupt();
    srv.join();
}

// every CRC-32C implementation tier agrees with the table version (sizes around the 3 x 8 KiB block, odd offsets)
TEST(crc32c_tiers_agree) {
    std::vector<uint8_t> buf((1 << 20) + 64);
    std::mt19937 rng(7);
    for (auto &b : buf) b = static_cast<uint8_t>(rng());
    const int native = kernels::crc32c_tier();
    if (native >= 2) EXPECT(kernels::crc32c_clmul_ready()); // the solved fold constants were found and verified
    const size_t sizes[] = {0, 1, 7, 8, 9, 24575, 24576, 24577, 49152 + 13, 100000, 1 << 20};
    for (size_t n : sizes)
        for (size_t off : {0, 1, 3}) {
            const uint32_t want = kernels::crc32c_sw(buf.data() + off, n);
            EXPECT(kernels::crc32c_hw3(buf.data() + off, n) == want);
            EXPECT(kernels::crc32c_hw3_clmul(buf.data() + off, n) == want);
            for (int tier = 0; tier <= 2; ++tier) {
                kernels::crc32c_spoof_tier(tier);
                EXPECT(kernels::crc32c_tier() == std::min(tier, native));
                EXPECT(kernels::crc32c(buf.data() + off, n) == want);
            }
            kernels::crc32c_spoof_tier(-1);
        }
    EXPECT(kernels::crc32c("123456789", 9) == 0xE3069283u); // CRC-32C check value
    // throughput of each tier on this host (informational)
    std::vector<uint8_t> big(64 << 20, 0x5A);
    auto rate = [&](auto fn) {
        const auto t0 = std::chrono::steady_clock::now();
        volatile uint32_t sink = fn(big.data(), big.size());
        (void)sink;
        return big.size() / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 1e9;
    };
    std::printf("  crc32c GB/s: table %.2f, sse4.2 x3 %.2f, sse4.2 x3 + pclmul %.2f\n", rate(kernels::crc32c_sw),
                rate(kernels::crc32c_hw3), rate(kernels::crc32c_hw3_clmul));
}

// xGMI path on a multi-GPU node without the node: the workgroup budget and the peer-access precheck with fake GPU uids
TEST(ipc_preflight_and_remote_grid_decisions) {
    // fake GPU uids: which rings probe cross-GPU writes on their first op, and the push kernel's workgroup budget
    using client::ipc_needs_preflight;
    using client::ipc_push_grid;
    const std::vector<uint64_t> one_gpu(8, 7), eight = {1, 2, 3, 4, 5, 6, 7, 8}, pairs = {1, 1, 2, 2};
    EXPECT(!ipc_needs_preflight(one_gpu, false, 1 << 20));    // all peers on one GPU: nothing crosses xGMI
    EXPECT(ipc_needs_preflight(eight, false, 1 << 20));       // first op across GPUs
    EXPECT(!ipc_needs_preflight(eight, true, 1 << 20));       // once per arena
    EXPECT(!ipc_needs_preflight(eight, false, 8 * 256 - 2));  // too small for a slot per peer: a later op probes
    EXPECT(ipc_needs_preflight(pairs, false, 4 * 256));
    EXPECT(ipc_push_grid(eight, 0, 0) == 512);                // default: the local budget
    EXPECT(ipc_push_grid(eight, 3, 1024) == 1024);            // PCCL_IPC_REMOTE_GRID for remote destinations
    EXPECT(ipc_push_grid(one_gpu, 3, 1024) == 256);           // no remote destination: knob ignored
    EXPECT(ipc_push_grid(pairs, 1, 100000) == 4096);          // clamped
}

TEST(ipc_grid_budget_by_gpu_sharing) {
    using client::ipc_grid_budget;
    const std::vector<uint64_t> eight_gpus = {11, 12, 13, 14, 15, 16, 17, 18};
    for (size_t r = 0; r < 8; ++r) EXPECT(ipc_grid_budget(eight_gpus, r) == 512); // one peer per GPU: whole chip
    const std::vector<uint64_t> pairs = {1, 1, 2, 2};
    EXPECT(ipc_grid_budget(pairs, 0) == 256 && ipc_grid_budget(pairs, 3) == 256);
    const std::vector<uint64_t> one_gpu(8, 7);
    EXPECT(ipc_grid_budget(one_gpu, 5) == 256); // floor: fewer cannot saturate HBM
    const std::vector<uint64_t> mixed = {1, 2, 2, 2, 3};
    EXPECT(ipc_grid_budget(mixed, 0) == 512 && ipc_grid_budget(mixed, 1) == 256);
}

TEST(ipc_peer_access_precheck) {
    using client::ipc_unreachable_peer;
    const std::vector<uint64_t> uids = {100, 101, 102, 103};
    auto visible = [](uint64_t u) { return u >= 100 && u < 104 ? static_cast<int>(u - 100) : -1; };
    auto full_mesh = [](int, int) { return true; };
    EXPECT(ipc_unreachable_peer(uids, 0, 0, visible, full_mesh) == -1);
    auto no_2 = [](int d, int p) { return !(d == 0 && p == 2); }; // device 0 cannot map device 2
    EXPECT(ipc_unreachable_peer(uids, 0, 0, visible, no_2) == 2);
    EXPECT(ipc_unreachable_peer(uids, 1, 1, visible, no_2) == -1);
    auto invisible = [](uint64_t u) { return u == 100 ? 0 : -1; }; // other GPUs not visible: left to the IPC open
    EXPECT(ipc_unreachable_peer(uids, 0, 0, invisible, [](int, int) { return false; }) == -1);
    const std::vector<uint64_t> same = {5, 5, 5};
    EXPECT(ipc_unreachable_peer(same, 1, 0, visible, [](int, int) { return false; }) == -1);
}

TEST(pool_slabs_carve_coalesce_and_reuse) {
    using client::BufferPool;
    BufferPool pool(BufferPool::Kind::Host);
    // 64 small leases share slabs: 2 runtime allocations (128 MiB slabs) instead of 64
    std::vector<BufferPool::Buf> bufs;
    for (int i = 0; i < 64; ++i) bufs.push_back(pool.get(3u << 20));
    EXPECT(pool.allocs() == 2);
    EXPECT(pool.in_use() == 64u * (3u << 20));
    for (auto &b : bufs) {
        EXPECT(b.p != nullptr && b.slab != nullptr && reinterpret_cast<uintptr_t>(b.p) % BufferPool::kGranule == 0);
        std::memset(b.p, 0x5a, b.cap); // every lease is writable and disjoint from the others
    }
    for (size_t i = 0; i < bufs.size(); ++i)
        for (size_t j = i + 1; j < bufs.size(); ++j) {
            auto *a = static_cast<uint8_t *>(bufs[i].p), *b = static_cast<uint8_t *>(bufs[j].p);
            EXPECT(a + bufs[i].cap <= b || b + bufs[j].cap <= a);
        }
    // return every other lease, then the rest: extents coalesce back into whole slabs
    for (size_t i = 0; i < bufs.size(); i += 2) pool.put(bufs[i]);
    for (size_t i = 1; i < bufs.size(); i += 2) pool.put(bufs[i]);
    EXPECT(pool.in_use() == 0);
    // a lease as large as a whole slab fits again (the extents merged), without a new allocation
    auto big = pool.get(BufferPool::kSlabMaxRequest);
    auto again = pool.get(BufferPool::kSlabMaxRequest);
    EXPECT(big.p && again.p && pool.allocs() == 2);
    pool.put(big);
    pool.put(again);
    // large leases are whole allocations, cached best-fit
    auto huge = pool.get(BufferPool::kSlabMaxRequest + 1);
    EXPECT(huge.p != nullptr && huge.slab == nullptr && pool.allocs() == 3);
    pool.put(huge);
    auto huge2 = pool.get(BufferPool::kSlabMaxRequest + 4096);
    EXPECT(huge2.p == huge.p && pool.allocs() == 3);
    pool.put(huge2);
    EXPECT(pool.in_use() == 0 && pool.peak() >= 64u * (3u << 20));
    // four ring-step leases of an exactly 32 MiB chunk plus the 64-byte vector-phase slack (ring_device.cpp) share
    // one slab: config 3's fp32 ops (8 peers x 256 MiB) used to make each of them a whole pinned allocation
    BufferPool p4(BufferPool::Kind::Host);
    std::vector<BufferPool::Buf> step;
    for (int i = 0; i < 4; ++i) step.push_back(p4.get((32u << 20) + 64));
    EXPECT(p4.allocs() == 1);
    for (auto &b : step) EXPECT(b.p != nullptr && b.slab != nullptr);
    for (auto &b : step) p4.put(b);
}

TEST(pool_concurrent_leases_stay_disjoint) {
    using client::BufferPool;
    BufferPool pool(BufferPool::Kind::Host);
    std::atomic<int> bad{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 8; ++t)
        ths.emplace_back([&, t] {
            std::mt19937 rng(static_cast<unsigned>(t));
            std::vector<BufferPool::Buf> held;
            for (int i = 0; i < 400; ++i) {
                if (!held.empty() && (rng() % 3 == 0 || held.size() > 6)) {
                    const size_t k = rng() % held.size();
                    auto *p = static_cast<uint8_t *>(held[k].p);
                    for (size_t j = 0; j < held[k].cap; j += 4096)
                        if (p[j] != static_cast<uint8_t>(t)) ++bad; // nobody else wrote into my lease
                    pool.put(held[k]);
                    held.erase(held.begin() + static_cast<long>(k));
                } else {
                    const size_t n = (rng() % 2) ? (rng() % (8u << 20)) + 1 : (rng() % (48u << 20)) + 1;
                    auto b = pool.get(n);
                    if (!b.p || b.cap < n) {
                        ++bad;
                        continue;
                    }
                    std::memset(b.p, t, b.cap);
                    held.push_back(b);
                }
            }
            for (auto &b : held) pool.put(b);
        });
    for (auto &t : ths) t.join();
    EXPECT(bad.load() == 0);
    EXPECT(pool.in_use() == 0);
}

int main() {
    for (auto &[name, fn] : registry()) {
        const int before = g_failures;
        fn();
        std::printf("%-40s %s\n", name.c_str(), g_failures == before ? "ok" : "FAILED");
    }
    std::printf("%d failure(s)\n", g_failures);
    return g_failures == 0 ? 0 : 1;
}
