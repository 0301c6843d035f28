// Native unit tests of internal components (no gtest in the image: a tiny self-registering harness).
// Built as build/pccl_unit_tests, run by tests/test_native.py; also the target of the sanitizer build
// (cmake -DPCCL_SANITIZE=ON: ASan + UBSan on host code).
#include <cmath>
#include <cstdio>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "common/numeric.hpp"
#include "kernels/host_kernels.hpp"
#include "master/topology.hpp"
#include "proto/packets.hpp"

using namespace pccl;

static std::vector<std::pair<std::string, std::function<void()>>> &registry() {
    static std::vector<std::pair<std::string, std::function<void()>>> r;
    return r;
}
static int g_failures = 0;
#define TEST(name)                                                                                                   \
    static void name();                                                                                              \
    static const bool reg_##name = (registry().emplace_back(#name, name), true);                                     \
    static void name()
#define EXPECT(cond)                                                                                                 \
    do {                                                                                                             \
        if (!(cond)) {                                                                                               \
            std::fprintf(stderr, "  %s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #cond);                         \
            ++g_failures;                                                                                            \
        }                                                                                                            \
    } while (0)

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

int main() {
    for (auto &[name, fn] : registry()) {
        const int before = g_failures;
        fn();
        std::printf("%-40s %s\n", name.c_str(), g_failures == before ? "ok" : "FAILED");
    }
    std::printf("%d failure(s)\n", g_failures);
    return g_failures == 0 ? 0 : 1;
}
