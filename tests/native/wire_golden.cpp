// Golden wire-format tests: every CCoIP packet (29 ids), both framings, and the pccl-amd liveness
// extension (registration suffixes, heartbeat and op-stalled packets, as docs/WIRE_DIVERGENCES.md specifies them), against byte arrays
// written down from the reference's serialize() order (ccoip/src/cpp/ccoip_packets.cpp:6-625,
// tinysockets multiplexed_socket.cpp:406-411, queued_client_socket.cpp:299-305) - NOT produced by our encoder.
// Each case checks (1) our encoder emits exactly the golden bytes for a packet whose pccl-amd extension fields are
// at their defaults, and (2) our decoder parses the golden bytes (what a reference peer sends) back to the values.
// The few simple packets use literal byte arrays; the rest a minimal big-endian builder (`G`) that is independent of
// proto::WBuf. Intentional divergences (appended extensions, rounding) are listed in docs/WIRE_DIVERGENCES.md.
#include <cstring>
#include <vector>

#include "harness.hpp"
#include "net/mux.hpp"
#include "net/socket.hpp"
#include "proto/packets.hpp"

using namespace pccl;

namespace {

struct G {
    std::vector<uint8_t> b;
    explicit G(uint16_t id) { be(id, 2); }
    G &be(uint64_t v, int n) {
        for (int i = n - 1; i >= 0; --i) b.push_back(static_cast<uint8_t>(v >> (8 * i)));
        return *this;
    }
    G &u8(uint8_t v) { return be(v, 1); }
    G &u16(uint16_t v) { return be(v, 2); }
    G &u32(uint32_t v) { return be(v, 4); }
    G &u64(uint64_t v) { return be(v, 8); }
    G &boolean(bool v) { return u8(v ? 1 : 0); }
    G &raw(const void *p, size_t n) {
        const auto *c = static_cast<const uint8_t *>(p);
        b.insert(b.end(), c, c + n);
        return *this;
    }
    G &uuid(const Uuid &u) { return raw(u.data.data(), 16); }
    G &str(const std::string &s) { return u64(s.size()).raw(s.data(), s.size()); }
    G &v4(uint8_t a, uint8_t bb, uint8_t c, uint8_t d, uint16_t port) { return boolean(true).u8(a).u8(bb).u8(c).u8(d).u16(port); }
    G &f64(double d) {
        uint64_t u;
        std::memcpy(&u, &d, 8);
        return u64(u);
    }
};

Uuid uuid_of(uint8_t seed) {
    Uuid u;
    for (int i = 0; i < 16; ++i) u.data[i] = static_cast<uint8_t>(seed + i);
    return u;
}

template<typename P>
void check(const P &p, const std::vector<uint8_t> &golden, const char *name) {
    const auto ours = proto::encode_with_id(p);
    if (ours != golden) {
        std::fprintf(stderr, "  %s: encoded %zu bytes, golden %zu bytes\n", name, ours.size(), golden.size());
        for (size_t i = 0; i < std::max(ours.size(), golden.size()); ++i)
            if (i >= ours.size() || i >= golden.size() || ours[i] != golden[i]) {
                std::fprintf(stderr, "  first difference at byte %zu\n", i);
                break;
            }
    }
    EXPECT(ours == golden);
}

template<typename P>
std::optional<P> parse(const std::vector<uint8_t> &golden) {
    EXPECT(golden.size() >= 2 && ((golden[0] << 8) | golden[1]) == P::kId);
    return proto::decode_payload<P>(golden.data() + 2, golden.size() - 2);
}

SockAddr v4(uint8_t a, uint8_t b, uint8_t c, uint8_t d, uint16_t port) { return make_sockaddr_v4(a, b, c, d, port); }

} // namespace

// ---------------------------------------------------------------- literal byte arrays
TEST(golden_c2m_collective_initiate) { // id 10: u64 tag, u64 count, u8 dtype, u8 op
    const std::vector<uint8_t> g = {0x00, 0x0A, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 0x08,
                                    0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x11, 0x22, 0x09, 0x04};
    proto::C2MCollectiveCommsInitiate p;
    p.tag = 0x0102030405060708ull;
    p.count = 0x1122;
    p.data_type = DType::BF16; // ccoip_data_type_t BFloat16 = 9
    p.op = ReduceOp::Max;      // ccoip_reduce_op_t Max = 4
    check(p, g, "initiate");
    auto q = parse<proto::C2MCollectiveCommsInitiate>(g);
    EXPECT(q && q->tag == p.tag && q->count == 0x1122 && q->data_type == DType::BF16 && q->op == ReduceOp::Max &&
           q->flags == 0);
}

TEST(golden_c2m_collective_complete) { // id 11: u64 tag, bool was_aborted
    const std::vector<uint8_t> g = {0x00, 0x0B, 0, 0, 0, 0, 0, 0, 0, 0x2A, 0x01};
    proto::C2MCollectiveCommsComplete p;
    p.tag = 42;
    p.was_aborted = true;
    check(p, g, "c2m complete");
    auto q = parse<proto::C2MCollectiveCommsComplete>(g);
    EXPECT(q && q->tag == 42 && q->was_aborted);
}

TEST(golden_m2c_commence) { // id 9: u64 tag, u64 seq_nr
    const std::vector<uint8_t> g = {0x00, 0x09, 0, 0, 0, 0, 0, 0, 0, 0x07, 0, 0, 0, 0, 0, 0, 0x01, 0x00};
    proto::M2CCollectiveCommsCommence p;
    p.tag = 7;
    p.seq_nr = 256;
    check(p, g, "commence");
    auto q = parse<proto::M2CCollectiveCommsCommence>(g);
    EXPECT(q && q->tag == 7 && q->seq_nr == 256 && q->flags == 0);
}

TEST(golden_m2c_complete_and_abort) { // id 10: u64 tag; id 11: u64 tag, bool aborted
    const std::vector<uint8_t> gc = {0x00, 0x0A, 0, 0, 0, 0, 0, 0, 0x12, 0x34};
    proto::M2CCollectiveCommsComplete c;
    c.tag = 0x1234;
    check(c, gc, "m2c complete");
    const std::vector<uint8_t> ga = {0x00, 0x0B, 0, 0, 0, 0, 0, 0, 0, 0x05, 0x00};
    proto::M2CCollectiveCommsAbort a;
    a.tag = 5;
    a.aborted = false;
    check(a, ga, "abort");
    auto qa = parse<proto::M2CCollectiveCommsAbort>(ga);
    EXPECT(qa && qa->tag == 5 && !qa->aborted);
}

TEST(golden_c2m_session_registration_ports) { // id 1: u32 group, bool explicit=false, u16 p2p, u16 ss, u16 bm
    const std::vector<uint8_t> g = {0x00, 0x01, 0x00, 0x00, 0x00, 0x03, 0x00, 0xBC, 0x15, 0xBC, 0x16, 0xBC, 0x17};
    proto::C2MRequestSessionRegistration p;
    p.peer_group = 3;
    p.p2p_port = 48149;
    p.ss_port = 48150;
    p.bm_port = 48151;
    check(p, g, "registration");
    auto q = parse<proto::C2MRequestSessionRegistration>(g);
    EXPECT(q && q->peer_group == 3 && !q->use_explicit_addresses && q->p2p_port == 48149 && q->bm_port == 48151 &&
           q->host_token.empty());
}

TEST(golden_c2m_report_bandwidth) { // id 6: uuid to, f64 (bit pattern, big-endian)
    std::vector<uint8_t> g = {0x00, 0x06};
    const Uuid u = uuid_of(0x40);
    g.insert(g.end(), u.data.begin(), u.data.end());
    const uint8_t d[8] = {0x40, 0x8F, 0x40, 0x00, 0x00, 0x00, 0x00, 0x00}; // 1000.0
    g.insert(g.end(), d, d + 8);
    proto::C2MReportPeerBandwidth p;
    p.to_peer = u;
    p.bandwidth_mbps = 1000.0;
    check(p, g, "bandwidth");
    auto q = parse<proto::C2MReportPeerBandwidth>(g);
    EXPECT(q && q->to_peer == u && q->bandwidth_mbps == 1000.0);
}

TEST(golden_p2p_hello_and_ack) { // P2P id 1: uuid, u32 connection_nr; id 2: empty
    std::vector<uint8_t> g = {0x00, 0x01};
    const Uuid u = uuid_of(1);
    g.insert(g.end(), u.data.begin(), u.data.end());
    const uint8_t nr[4] = {0x00, 0x00, 0x00, 0x03};
    g.insert(g.end(), nr, nr + 4);
    proto::P2PHello h;
    h.peer_uuid = u;
    h.connection_nr = 3;
    check(h, g, "hello");
    auto q = parse<proto::P2PHello>(g);
    EXPECT(q && q->peer_uuid == u && q->connection_nr == 3);
    check(proto::P2PHelloAck{}, std::vector<uint8_t>{0x00, 0x02}, "hello ack");
}

TEST(golden_empty_packets) { // C2M 4, 5, 7, 9 and M2C 8: id only
    check(proto::C2MCheckPeersPending{}, {0x00, 0x04}, "check peers pending");
    check(proto::C2MOptimizeTopology{}, {0x00, 0x05}, "optimize topology");
    check(proto::C2MOptimizeTopologyWorkComplete{}, {0x00, 0x07}, "optimize work complete");
    check(proto::C2MDistSharedStateComplete{}, {0x00, 0x09}, "dist shared state complete");
    check(proto::M2CSyncSharedStateComplete{}, {0x00, 0x08}, "sync shared state complete");
}

TEST(golden_bool_packets) { // C2M 2, M2C 4, B2C 1: one bool
    proto::C2MRequestEstablishP2PConnections e;
    e.accept_new_peers = true;
    check(e, {0x00, 0x02, 0x01}, "request establish");
    proto::M2CPeersPendingResponse pp;
    pp.peers_pending = true;
    check(pp, {0x00, 0x04, 0x01}, "peers pending");
    proto::B2CBenchmarkServerIsBusy busy;
    busy.is_busy = true;
    check(busy, {0x00, 0x01, 0x01}, "benchmark busy");
    auto q = parse<proto::B2CBenchmarkServerIsBusy>({0x00, 0x01, 0x00});
    EXPECT(q && !q->is_busy);
}

TEST(golden_c2b_hello) { // C2B id 1: uuid
    std::vector<uint8_t> g = {0x00, 0x01};
    const Uuid u = uuid_of(0x90);
    g.insert(g.end(), u.data.begin(), u.data.end());
    proto::C2BHello p;
    p.peer_uuid = u;
    check(p, g, "c2b hello");
}

// ---------------------------------------------------------------- builder-based goldens
TEST(golden_c2m_session_registration_explicit) { // explicit=true: 3 x sockaddr (bool v4, 4 bytes, u16 port)
    const auto g = G(1).u32(9).boolean(true).v4(10, 0, 0, 1, 100).v4(10, 0, 0, 2, 200).v4(10, 0, 0, 3, 300).b;
    proto::C2MRequestSessionRegistration p;
    p.peer_group = 9;
    p.use_explicit_addresses = true;
    p.advertised_p2p = v4(10, 0, 0, 1, 100);
    p.advertised_ss = v4(10, 0, 0, 2, 200);
    p.advertised_bm = v4(10, 0, 0, 3, 300);
    check(p, g, "registration explicit");
    auto q = parse<proto::C2MRequestSessionRegistration>(g);
    EXPECT(q && q->use_explicit_addresses && q->ss_port == 200 && sockaddr_equal(q->advertised_bm, p.advertised_bm));
}

TEST(golden_c2m_p2p_established) { // id 3: bool success, u64 n, n x uuid
    const auto g = G(3).boolean(false).u64(2).uuid(uuid_of(1)).uuid(uuid_of(2)).b;
    proto::C2MP2PConnectionsEstablished p;
    p.success = false;
    p.failed_peers = {uuid_of(1), uuid_of(2)};
    check(p, g, "c2m established");
    auto q = parse<proto::C2MP2PConnectionsEstablished>(g);
    EXPECT(q && !q->success && q->failed_peers == p.failed_peers);
}

TEST(golden_c2m_sync_shared_state) { // id 8: u64 rev, u8 strategy, u64 n, n x {str, u64, u8, u64, u8, bool}
    const auto g = G(8).u64(17).u8(1).u64(2)
                       .str("w").u64(0xAABBCCDD).u8(0).u64(4096).u8(10).boolean(false)
                       .str("opt.m").u64(5).u8(1).u64(7).u8(9).boolean(true).b;
    proto::C2MSyncSharedState p;
    p.revision = 17;
    p.strategy = SyncStrategy::RxOnly;
    p.entries.push_back({"w", 0xAABBCCDD, HashType::Simple, 4096, DType::F32, false});
    p.entries.push_back({"opt.m", 5, HashType::Crc32, 7, DType::BF16, true});
    check(p, g, "c2m sync");
    auto q = parse<proto::C2MSyncSharedState>(g);
    EXPECT(q && q->revision == 17 && q->strategy == SyncStrategy::RxOnly && q->entries == p.entries);
}

TEST(golden_m2c_session_registration_response) { // M2C id 1: bool accepted, uuid
    const auto g = G(1).boolean(true).uuid(uuid_of(0x33)).b;
    proto::M2CSessionRegistrationResponse p;
    p.accepted = true;
    p.assigned_uuid = uuid_of(0x33);
    check(p, g, "registration response");
}

TEST(golden_m2c_p2p_connection_info) { // M2C id 2: bool unchanged, 4 x u64, [u64 n, n x {sockaddr, uuid}]
    const auto g = G(2).boolean(false).u64(3).u64(2).u64(2).u64(2).u64(2)
                       .v4(127, 0, 0, 1, 48149).uuid(uuid_of(1)).v4(127, 0, 0, 1, 48152).uuid(uuid_of(2)).b;
    proto::M2CP2PConnectionInfo p;
    p.global_world_size = 3;
    p.local_world_size = 2;
    p.num_distinct_peer_groups = 2;
    p.largest_peer_group_world_size = 2;
    p.all_peers = {{v4(127, 0, 0, 1, 48149), uuid_of(1)}, {v4(127, 0, 0, 1, 48152), uuid_of(2)}};
    check(p, g, "connection info");
    auto q = parse<proto::M2CP2PConnectionInfo>(g);
    EXPECT(q && !q->unchanged && q->all_peers.size() == 2 && q->all_peers[1].peer_uuid == uuid_of(2) &&
           q->all_peers[1].p2p_listen_addr.port == 48152 && q->extra_peers.empty());
    // unchanged: the peer list is omitted
    const auto gu = G(2).boolean(true).u64(3).u64(2).u64(2).u64(2).b;
    proto::M2CP2PConnectionInfo u = p;
    u.unchanged = true;
    check(u, gu, "connection info unchanged");
}

TEST(golden_m2c_p2p_established) { // M2C id 3: bool success, u64 n, n x uuid (ring order)
    const auto g = G(3).boolean(true).u64(3).uuid(uuid_of(3)).uuid(uuid_of(1)).uuid(uuid_of(2)).b;
    proto::M2CP2PConnectionsEstablished p;
    p.success = true;
    p.ring_order = {uuid_of(3), uuid_of(1), uuid_of(2)};
    check(p, g, "m2c established");
    auto q = parse<proto::M2CP2PConnectionsEstablished>(g);
    EXPECT(q && q->success && q->ring_order == p.ring_order && !q->has_host_info && !q->single_host);
}

TEST(golden_m2c_optimize_topology_response) { // M2C id 5: u64 n, n x {uuid from, uuid to, sockaddr}
    const auto g = G(5).u64(1).uuid(uuid_of(1)).uuid(uuid_of(2)).v4(192, 168, 1, 7, 48151).b;
    proto::M2COptimizeTopologyResponse p;
    p.requests.push_back({uuid_of(1), uuid_of(2), v4(192, 168, 1, 7, 48151)});
    check(p, g, "optimize response");
    auto q = parse<proto::M2COptimizeTopologyResponse>(g);
    EXPECT(q && q->requests.size() == 1 && q->requests[0].to_peer_endpoint.port == 48151);
}

TEST(golden_m2c_optimize_topology_complete) { // M2C id 6: bool success, u64 n, n x uuid
    const auto g = G(6).boolean(true).u64(2).uuid(uuid_of(2)).uuid(uuid_of(1)).b;
    proto::M2COptimizeTopologyComplete p;
    p.success = true;
    p.ring_order = {uuid_of(2), uuid_of(1)};
    check(p, g, "optimize complete");
}

TEST(golden_m2c_sync_shared_state) { // M2C id 7: bool, sockaddr, u64 n, n x str, n x u64, n x u8
    const auto g = G(7).boolean(true).v4(10, 1, 2, 3, 48150).u64(2).str("a").str("bb").u64(11).u64(22).u8(0).u8(1).b;
    proto::M2CSyncSharedState p;
    p.is_outdated = true;
    p.distributor = v4(10, 1, 2, 3, 48150);
    p.outdated_keys = {"a", "bb"};
    p.expected_hashes = {11, 22};
    p.expected_hash_types = {HashType::Simple, HashType::Crc32};
    check(p, g, "m2c sync");
    auto q = parse<proto::M2CSyncSharedState>(g);
    EXPECT(q && q->is_outdated && q->outdated_keys == p.outdated_keys && q->expected_hashes == p.expected_hashes &&
           q->expected_hash_types == p.expected_hash_types && q->fallback_distributors.empty());
}

TEST(golden_p2p_dequant_meta_minmax) { // P2P id 3: u64 tag, u8 MIN_MAX=0, u8 dtype, min, max (floats host-LE)
    const float mn = -1.5f, mx = 2.25f;
    const auto g = G(3).u64(77).u8(0).u8(10).raw(&mn, 4).raw(&mx, 4).b;
    proto::P2PDequantizationMeta p;
    p.tag = 77;
    p.meta.algo = QuantAlgo::MinMax;
    p.meta.value_type = DType::F32;
    p.meta.min_value = -1.5;
    p.meta.max_value = 2.25;
    check(p, g, "meta minmax f32");
    auto q = parse<proto::P2PDequantizationMeta>(g);
    EXPECT(q && q->meta.algo == QuantAlgo::MinMax && q->meta.min_value == -1.5 && q->meta.max_value == 2.25);
    // integer value types travel in network order (reference quantize.hpp:57-60)
    const auto gi = G(3).u64(1).u8(0).u8(5).u32(static_cast<uint32_t>(-3)).u32(300).b;
    proto::P2PDequantizationMeta pi;
    pi.tag = 1;
    pi.meta.algo = QuantAlgo::MinMax;
    pi.meta.value_type = DType::I32;
    pi.meta.min_value = -3;
    pi.meta.max_value = 300;
    check(pi, gi, "meta minmax i32");
}

TEST(golden_p2p_dequant_meta_zps) { // ZPS=1: u8 zp type (Int64=7), zp BE, u8 scale type (Float=10), scale LE
    const float scale = 0.125f;
    const auto g = G(3).u64(5).u8(1).u8(7).u64(static_cast<uint64_t>(-12)).u8(10).raw(&scale, 4).b;
    proto::P2PDequantizationMeta p;
    p.tag = 5;
    p.meta.algo = QuantAlgo::ZeroPointScale;
    p.meta.zero_point = -12;
    p.meta.scale = 0.125f;
    check(p, g, "meta zps");
    auto q = parse<proto::P2PDequantizationMeta>(g);
    EXPECT(q && q->meta.algo == QuantAlgo::ZeroPointScale && q->meta.zero_point == -12 && q->meta.scale == 0.125f);
}

TEST(golden_c2s_request_shared_state) { // C2S id 1: u64 n, n x str
    const auto g = G(1).u64(2).str("model.w").str("opt.v").b;
    proto::C2SRequestSharedState p;
    p.keys = {"model.w", "opt.v"};
    check(p, g, "c2s request");
}

TEST(golden_s2c_shared_state_response) { // S2C id 1: u8 status, u64 revision, u64 n, n x {str, u64 size}
    const auto g = G(1).u8(1).u64(9).u64(1).str("w").u64(4096).b;
    proto::S2CSharedStateResponse p;
    p.status = proto::SharedStateStatus::Success;
    p.revision = 9;
    p.entries.push_back({"w", 4096});
    check(p, g, "s2c response");
    auto q = parse<proto::S2CSharedStateResponse>(G(1).u8(4).u64(0).u64(0).b);
    EXPECT(q && q->status == proto::SharedStateStatus::UnknownKey && q->entries.empty());
}

// ---------------------------------------------------------------- framings
TEST(golden_ltv_header) { // u64 BE (payload + 2) | u16 BE id
    const auto h = net::ltv_header(10, 18);
    const std::vector<uint8_t> g = {0, 0, 0, 0, 0, 0, 0, 20, 0x00, 0x0A};
    EXPECT(h == g);
}

TEST(golden_mux_frame_header) { // u64 BE (payload + 16) | u64 BE tag | u64 BE stream_ctr
    uint8_t h[net::kMuxHeaderBytes];
    net::mux_frame_header(h, 0x100, 0x0A0B, 3);
    const uint8_t g[24] = {0, 0, 0, 0, 0, 0, 0x01, 0x10, 0, 0, 0, 0, 0, 0, 0x0A, 0x0B, 0, 0, 0, 0, 0, 0, 0, 0x03};
    EXPECT(std::memcmp(h, g, 24) == 0);
    uint64_t n = 0, tag = 0, ctr = 0;
    EXPECT(net::mux_parse_header(g, n, tag, ctr) && n == 0x100 && tag == 0x0A0B && ctr == 3);
    uint8_t bad[24] = {};
    bad[7] = 15; // length < 16
    EXPECT(!net::mux_parse_header(bad, n, tag, ctr));
    net::mux_frame_header(bad, net::kMuxMaxFrame + 1, 1, 1); // payload over the 1 GiB cap
    EXPECT(!net::mux_parse_header(bad, n, tag, ctr));
    net::mux_frame_header(bad, net::kMuxMaxFrame, 1, 1);
    EXPECT(net::mux_parse_header(bad, n, tag, ctr) && n == net::kMuxMaxFrame);
}

// appended pccl-amd extensions are only emitted when set, and their bytes FOLLOW the complete reference layout
TEST(golden_extensions_are_suffixes) {
    proto::M2CP2PConnectionsEstablished p;
    p.success = true;
    p.ring_order = {uuid_of(1)};
    p.has_host_info = true;
    p.single_host = true;
    p.host_of = {0};
    const auto base = G(3).boolean(true).u64(1).uuid(uuid_of(1)).b;
    const auto ours = proto::encode_with_id(p);
    EXPECT(ours.size() > base.size() && std::equal(base.begin(), base.end(), ours.begin()));
    proto::C2MCollectiveCommsInitiate i;
    i.tag = 1;
    i.flags = proto::kCollFlagHierarchical;
    const auto ib = proto::encode_with_id(i);
    EXPECT(ib.size() == 21 && ib.back() == proto::kCollFlagHierarchical);
}

// Liveness extension (pccl-amd only, docs/WIRE_DIVERGENCES.md): appended to the registration request after the
// xGMI byte, appended to the registration response only when the master runs it, and three packets of its own.
TEST(golden_liveness_registration_suffixes) {
    proto::C2MRequestSessionRegistration p;
    p.peer_group = 0;
    p.p2p_port = 1;
    p.ss_port = 2;
    p.bm_port = 3;
    p.host_token = "h";
    p.xgmi_capable = true;
    p.liveness = true;
    const auto g = G(1).u32(0).boolean(false).u16(1).u16(2).u16(3).str("h").boolean(true).u8(1).b;
    check(p, g, "registration + liveness");
    auto q = parse<proto::C2MRequestSessionRegistration>(g);
    EXPECT(q && q->liveness && q->xgmi_capable && q->host_token == "h");
    // without the liveness byte (an older pccl-amd peer): no liveness
    auto o = parse<proto::C2MRequestSessionRegistration>(G(1).u32(0).boolean(false).u16(1).u16(2).u16(3).str("h")
                                                             .boolean(true).b);
    EXPECT(o && !o->liveness);

    proto::M2CSessionRegistrationResponse r;
    r.accepted = true;
    r.assigned_uuid = uuid_of(0x40);
    r.heartbeat_ms = 400;
    r.peer_timeout_ms = 2000;
    r.op_stall_ms = 3000;
    const auto gr = G(1).boolean(true).uuid(uuid_of(0x40)).u32(400).u32(2000).u32(3000).b;
    check(r, gr, "registration response + liveness");
    auto rr = parse<proto::M2CSessionRegistrationResponse>(gr);
    EXPECT(rr && rr->heartbeat_ms == 400 && rr->peer_timeout_ms == 2000 && rr->op_stall_ms == 3000);
    // a reference master's response: no liveness parameters (everything off)
    auto rref = parse<proto::M2CSessionRegistrationResponse>(G(1).boolean(true).uuid(uuid_of(0x40)).b);
    EXPECT(rref && rref->heartbeat_ms == 0 && rref->peer_timeout_ms == 0 && rref->op_stall_ms == 0);
}

TEST(golden_liveness_packets) { // C2M 12 / M2C 12: id only; C2M 13: u64 tag, uuid, u8 kind, u32 step, u64 idle_ms
    check(proto::C2MHeartbeat{}, {0x00, 0x0C}, "C2MHeartbeat");
    check(proto::M2CHeartbeat{}, {0x00, 0x0C}, "M2CHeartbeat");
    proto::C2MOpStalled s;
    s.tag = 20;
    s.suspect = uuid_of(0x50);
    s.kind = proto::kStallTxBlocked;
    s.step = 3;
    s.idle_ms = 3011;
    const auto g = G(13).u64(20).uuid(uuid_of(0x50)).u8(1).u32(3).u64(3011).b;
    check(s, g, "C2MOpStalled");
    auto q = parse<proto::C2MOpStalled>(g);
    EXPECT(q && q->tag == 20 && q->suspect == uuid_of(0x50) && q->kind == proto::kStallTxBlocked && q->step == 3 &&
           q->idle_ms == 3011);
}
