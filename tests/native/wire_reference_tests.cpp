// Reference data-plane framing, byte for byte (reference ccoip/src/cpp/reduce.cpp:149-192,609-774): one quantized
// all-reduce of a 2-peer ring in which this test plays the reference peer at the socket level. The library peer must
//   * send each step's P2PDequantizationMeta packet on the op's data tag, on connection seq % pool (here: the only one),
//   * send no byte of the step's data before it has received the peer's packet,
//   * then send the step's quantized chunk as data frames on the same tag,
// and reduce / de-quantize exactly what the peer sent. Frames: u64 BE (payload + 16) | u64 BE tag | u64 BE stream_ctr
// (reference tinysockets multiplexed_socket.cpp:406-411); packet payload: u16 BE id | u64 BE tag | u8 0 (MIN_MAX) |
// u8 dtype | min | max (float: 4 bytes little-endian, reference DeQuantizationMetaData).
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "client/ring_common.hpp"
#include "harness.hpp"
#include "net/socket.hpp"

using namespace pccl;
using namespace pccl::client::ring;

namespace {

void put_be64(std::vector<uint8_t> &v, uint64_t x) {
    for (int i = 7; i >= 0; --i) v.push_back(static_cast<uint8_t>(x >> (8 * i)));
}

std::vector<uint8_t> frame(uint64_t tag, uint64_t seq, const std::vector<uint8_t> &payload) {
    std::vector<uint8_t> f;
    put_be64(f, payload.size() + 16);
    put_be64(f, tag);
    put_be64(f, seq);
    f.insert(f.end(), payload.begin(), payload.end());
    return f;
}

// the reference's P2PPacketDequantizationMeta (id 3) for a MIN_MAX float chunk
std::vector<uint8_t> meta_packet(uint64_t tag, float mn, float mx) {
    std::vector<uint8_t> p = {0x00, 0x03};
    put_be64(p, tag);
    p.push_back(0x00); // MIN_MAX
    p.push_back(10);   // ccoipFloat
    uint8_t b[4];
    std::memcpy(b, &mn, 4);
    p.insert(p.end(), b, b + 4);
    std::memcpy(b, &mx, 4);
    p.insert(p.end(), b, b + 4);
    return p;
}

bool readable_within(int fd, int ms) {
    pollfd p{fd, POLLIN, 0};
    return ::poll(&p, 1, ms) > 0;
}

std::vector<uint8_t> read_exact(int fd, size_t n) {
    std::vector<uint8_t> v(n);
    size_t got = 0;
    while (got < n) {
        if (!readable_within(fd, 5000)) break;
        const ssize_t r = ::recv(fd, v.data() + got, n - got, 0);
        if (r <= 0) break;
        got += static_cast<size_t>(r);
    }
    v.resize(got);
    return v;
}

} // namespace

TEST(reference_framed_quantized_ring_golden_bytes) {
    int txsv[2], rxsv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, txsv) == 0);
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, rxsv) == 0);
    auto tx = std::make_shared<net::MuxConn>(txsv[0], net::MuxConn::Mode::Tx, SockAddr{});
    auto rx = std::make_shared<net::MuxConn>(rxsv[1], net::MuxConn::Mode::Rx, SockAddr{});
    EXPECT(tx->start() && rx->start());
    const Conns txs{tx}, rxs{rx};
    const int ref_in = txsv[1], ref_out = rxsv[0]; // the emulated reference peer's ends

    // rank 0 of 2: chunk 0 = [0, 1, 2, 3] is its reduce-scatter payload, chunk 1 = [10] * 4 receives the peer's part
    std::vector<float> data = {0, 1, 2, 3, 10, 10, 10, 10};
    const uint64_t tag = 0x1234, seq = 7;
    const Shape shape = Shape::reference_framing();
    std::atomic<uint64_t> txc{0}, rxc{0};
    int rc = -1;
    std::thread lib([&] {
        HostRingArgs A{txs, rxs, 2, 0, tag, seq, shape, reinterpret_cast<uint8_t *>(data.data()), data.size(),
                       DType::F32, DType::U8, QuantAlgo::MinMax, ReduceOp::Sum, true, [] { return false; }, txc, rxc};
        rc = host_ring(A);
    });

    // reduce-scatter: the library's metadata packet on the data tag, then nothing until the peer's packet arrived
    const auto m0 = frame(tag, seq, meta_packet(tag, 0.f, 3.f));
    EXPECT(read_exact(ref_in, m0.size()) == m0);
    EXPECT(!readable_within(ref_in, 150));
    const auto pm0 = frame(tag, seq, meta_packet(tag, 20.f, 23.f));
    EXPECT(net::send_all(ref_out, pm0.data(), pm0.size()));
    const auto d0 = frame(tag, seq, {0x00, 0x55, 0xaa, 0xff}); // round((x - 0) / 3 * 255)
    EXPECT(read_exact(ref_in, d0.size()) == d0);
    const auto pd0 = frame(tag, seq, {0x00, 0xff, 0x00, 0xff}); // the peer's chunk 1: 20, 23, 20, 23
    EXPECT(net::send_all(ref_out, pd0.data(), pd0.size()));

    // all-gather: the library owns chunk 1 = [30, 33, 30, 33] (quantized once, its own copy := D(Q(x)))
    const auto m1 = frame(tag, seq, meta_packet(tag, 30.f, 33.f));
    EXPECT(read_exact(ref_in, m1.size()) == m1);
    EXPECT(!readable_within(ref_in, 150));
    const auto pm1 = frame(tag, seq, meta_packet(tag, 5.f, 8.f));
    EXPECT(net::send_all(ref_out, pm1.data(), pm1.size()));
    const auto d1 = frame(tag, seq, {0x00, 0xff, 0x00, 0xff});
    EXPECT(read_exact(ref_in, d1.size()) == d1);
    const auto pd1 = frame(tag, seq, {0x00, 0x55, 0xaa, 0xff}); // the peer's chunk 0: 5, 6, 7, 8
    EXPECT(net::send_all(ref_out, pd1.data(), pd1.size()));
    lib.join();

    EXPECT(rc == 0);
    const std::vector<float> want = {5, 6, 7, 8, 30, 33, 30, 33};
    EXPECT(data == want);
    // byte counters as the reference keeps them: a metadata packet counts its LTV header (u64 length + u16 id, 10)
    // plus serializedSize() = 8 + 1 + (4 + 4) + (4 + 4) = 25 for float min / max, 35 bytes (reduce.cpp:162-165,
    // 186-187, ccoip_packets.cpp:543-548), data its raw bytes: 2 x 35 + 2 x 4 each way
    EXPECT(txc.load() == 2 * 35 + 8 && rxc.load() == 2 * 35 + 8);
    EXPECT(!readable_within(ref_in, 50)); // nothing else on the wire
    tx->interrupt();
    rx->interrupt();
    ::close(ref_in);
    ::close(ref_out);
}

// The same op in the pccl-amd framing sends the metadata packet on the metadata tag (data tag | 1 << 63) and the data
// right behind it, without waiting for the peer's packet.
TEST(ext_framed_quantized_step_does_not_wait_for_peer_meta) {
    int txsv[2], rxsv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, txsv) == 0);
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, rxsv) == 0);
    auto tx = std::make_shared<net::MuxConn>(txsv[0], net::MuxConn::Mode::Tx, SockAddr{});
    auto rx = std::make_shared<net::MuxConn>(rxsv[1], net::MuxConn::Mode::Rx, SockAddr{});
    EXPECT(tx->start() && rx->start());
    const Conns txs{tx}, rxs{rx};
    std::vector<float> data = {0, 1, 2, 3, 10, 10, 10, 10};
    const uint64_t tag = 0x1234, seq = 7;
    proto::WireShape w;
    w.stripes = 1;
    w.quant_lanes = 1;
    const Shape shape = Shape::from_wire(w);
    std::atomic<uint64_t> txc{0}, rxc{0};
    std::atomic<bool> stop{false};
    std::thread lib([&] {
        HostRingArgs A{txs, rxs, 2, 0, tag, seq, shape, reinterpret_cast<uint8_t *>(data.data()), data.size(),
                       DType::F32, DType::U8, QuantAlgo::MinMax, ReduceOp::Sum, true,
                       [&] { return stop.load(); }, txc, rxc};
        host_ring(A);
    });
    const auto m0 = frame(tag ^ kMetaTagBit, seq, meta_packet(tag, 0.f, 3.f));
    EXPECT(read_exact(txsv[1], m0.size()) == m0);
    const auto d0 = frame(tag, seq, {0x00, 0x55, 0xaa, 0xff});
    EXPECT(read_exact(txsv[1], d0.size()) == d0); // no peer packet was sent
    stop = true; // abort the op (the test never answers)
    lib.join();
    tx->interrupt();
    rx->interrupt();
    ::close(txsv[1]);
    ::close(rxsv[0]);
}

TEST(stripe_conn_reference_framing_is_seq_mod_pool) {
    const Shape ref = Shape::reference_framing();
    for (uint64_t seq : {0ull, 1ull, 5ull, 31ull, 1000ull})
        for (size_t pool : {1ul, 4ul, 32ul}) EXPECT(stripe_conn(seq, 77, 0, pool, ref) == seq % pool);
    EXPECT(plan_stripes(size_t{1} << 30, 32, ref).off.size() == 1);
    EXPECT(quant_lane_bounds(size_t{1} << 30, 2, 1, ref).size() == 2);
}

TEST(stripe_conn_spreads_concurrent_ops_over_the_pool) {
    Shape sh;
    sh.stripes = 4;
    for (size_t pool : {2ul, 4ul, 8ul, 16ul, 32ul}) {
        // ops with one stripe per step (small steps): any `pool` consecutive ops use every connection once
        const Shape one = op_shape(sh, 1u << 20);
        EXPECT(op_stripes(one, pool) == 1);
        for (uint64_t first : {0ull, 7ull, 1000ull}) {
            std::vector<int> hits(pool, 0);
            for (uint64_t seq = first; seq < first + pool; ++seq) ++hits[stripe_conn(seq, 77, 0, pool, one)];
            for (size_t c = 0; c < pool; ++c) EXPECT(hits[c] == 1);
        }
        // wider ops take aligned groups of consecutive connections: pool / s consecutive ops tile the pool
        const Shape wide = op_shape(sh, 64u << 20);
        const size_t s = op_stripes(wide, pool);
        EXPECT(s == std::min<size_t>(4, pool));
        std::vector<int> hits(pool, 0);
        for (uint64_t seq = 5; seq < 5 + pool / s; ++seq)
            for (size_t k = 0; k < s; ++k) {
                const size_t c = stripe_conn(seq, 77, k, pool, wide);
                EXPECT(c == (stripe_conn(seq, 77, 0, pool, wide) + k) % pool && c % s == k);
                ++hits[c];
            }
        for (size_t c = 0; c < pool; ++c) EXPECT(hits[c] == 1);
    }
    // lanes of one quantized op take different groups
    const Shape wide = op_shape(sh, 64u << 20);
    EXPECT(stripe_conn(5, lane_tag(77, 0, 2), 0, 16, wide) != stripe_conn(5, lane_tag(77, 1, 2), 0, 16, wide));
}

TEST(stripe_count_matches_plan_and_pools_of_any_size) {
    Shape sh;
    sh.stripes = 4;
    sh.stripe_min = 1u << 20;
    for (size_t conns : {1ul, 2ul, 3ul, 4ul, 16ul})
        for (size_t bytes : {0ul, 1ul, 4096ul, (1ul << 20) - 1, 1ul << 20, (3ul << 20) + 7, 9000011ul * 2, 64ul << 20})
            EXPECT(stripe_count(bytes, conns, sh) == plan_stripes(bytes, conns, sh).off.size());
    // an op's group bounds the stripes of every step, also where rounding gives a larger step fewer stripes
    Shape s256 = sh;
    s256.stripe_min = 256u << 10;
    EXPECT(stripe_count((2u << 20) + 2048, 4, s256) == 3 && stripe_count(2u << 20, 4, s256) == 4);
    for (size_t conns : {1ul, 3ul, 4ul, 16ul})
        for (size_t maxb : {(2ul << 20) + 2048, (3ul << 20) + 4097, 9000011ul, 64ul << 20}) {
            const Shape op256 = op_shape(s256, maxb);
            for (size_t b = maxb > 600000 ? maxb - 600000 : 0; b <= maxb; b += 997)
                EXPECT(stripe_count(b, conns, s256) <= op_stripes(op256, conns));
        }
    // neighbours with pools of different sizes: both ends of a pool derive the same groups from the op's largest step
    const Shape op = op_shape(sh, 9000011ul * 2 / 3 + 2);
    for (size_t pool : {1ul, 2ul, 3ul})
        for (uint64_t seq : {0ull, 1ull, 2ull, 7ull})
            for (size_t k = 0; k < op_stripes(op, pool); ++k) EXPECT(stripe_conn(seq, 77, k, pool, op) < pool);
}

TEST(wire_shape_roundtrip_and_clamp) {
    proto::C2MCollectiveCommsInitiate a;
    a.tag = 5;
    a.count = 100;
    a.flags = proto::kCollFlagExtWire | proto::kCollFlagSmallPath;
    a.shape.stripes = 8;
    a.shape.quant_lanes = 3;
    a.shape.stripe_min_kib = 16384;
    auto bytes = proto::encode_with_id(a);
    auto b = proto::decode_payload<proto::C2MCollectiveCommsInitiate>(bytes.data() + 2, bytes.size() - 2);
    EXPECT(b && b->flags == a.flags && b->shape == a.shape);
    // a reference initiate (no extension bytes) decodes with no flags
    proto::C2MCollectiveCommsInitiate r;
    r.tag = 5;
    auto rb = proto::encode_with_id(r);
    EXPECT(rb.size() == 2 + 18);
    auto rd = proto::decode_payload<proto::C2MCollectiveCommsInitiate>(rb.data() + 2, rb.size() - 2);
    EXPECT(rd && rd->flags == 0);
    // the ext flag without its shape bytes (truncated) is dropped instead of misreading the packet
    std::vector<uint8_t> trunc(rb.begin(), rb.end());
    trunc.push_back(proto::kCollFlagExtWire);
    auto td = proto::decode_payload<proto::C2MCollectiveCommsInitiate>(trunc.data() + 2, trunc.size() - 2);
    EXPECT(td && td->flags == 0);
    const Shape s = Shape::from_wire(a.shape);
    EXPECT(!s.reference && s.stripes == 8 && s.quant_lanes == 3 && s.stripe_min == (size_t{16} << 20));
}

namespace {
// the reference's P2PPacketDequantizationMeta (id 3) for a ZERO_POINT_SCALE chunk: u8 1 | u8 zero point type (int64)
// | zero point big-endian (an integer: network order, reference quantize.hpp MakeZeroPointScale) | u8 scale type
// (float) | scale in host order (floats are not swapped)
std::vector<uint8_t> zps_packet(uint64_t tag, int64_t zp, float scale) {
    std::vector<uint8_t> p = {0x00, 0x03};
    put_be64(p, tag);
    p.push_back(0x01); // ZERO_POINT_SCALE
    p.push_back(7);    // ccoipInt64
    put_be64(p, static_cast<uint64_t>(zp));
    p.push_back(10); // ccoipFloat
    uint8_t b[4];
    std::memcpy(b, &scale, 4);
    p.insert(p.end(), b, b + 4);
    return p;
}
} // namespace

// A zero-point-scale (int8) quantized 2-peer ring in the reference framing, byte for byte: metadata packet on the
// data tag, the step's data only after the peer's packet, de-quantization of exactly what the peer sent.
TEST(reference_framed_zps_ring_golden_bytes) {
    int txsv[2], rxsv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, txsv) == 0);
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, rxsv) == 0);
    auto tx = std::make_shared<net::MuxConn>(txsv[0], net::MuxConn::Mode::Tx, SockAddr{});
    auto rx = std::make_shared<net::MuxConn>(rxsv[1], net::MuxConn::Mode::Rx, SockAddr{});
    EXPECT(tx->start() && rx->start());
    const Conns txs{tx}, rxs{rx};
    const int ref_in = txsv[1], ref_out = rxsv[0];
    // rank 0 of 2: chunk 0 = [-1, 0, 1, 2] is its reduce-scatter payload, chunk 1 = [10] * 4 receives the peer's
    std::vector<float> data = {-1, 0, 1, 2, 10, 10, 10, 10};
    const uint64_t tag = 0x77, seq = 3;
    std::atomic<uint64_t> txc{0}, rxc{0};
    int rc = -1;
    std::thread lib([&] {
        HostRingArgs A{txs, rxs, 2, 0, tag, seq, Shape::reference_framing(), reinterpret_cast<uint8_t *>(data.data()),
                       data.size(), DType::F32, DType::I8, QuantAlgo::ZeroPointScale, ReduceOp::Sum, true,
                       [] { return false; }, txc, rxc};
        rc = host_ring(A);
    });
    float s3;
    const uint8_t s3b[4] = {0xc1, 0xc0, 0x40, 0x3c}; // float(3 / 255)
    std::memcpy(&s3, s3b, 4);
    // reduce-scatter: scale (2 - -1) / 255, zero point rint(-128 + 1 / scale) = -43; q = rint(x / scale) - 43
    const auto m0 = frame(tag, seq, zps_packet(tag, -43, s3));
    EXPECT(read_exact(ref_in, m0.size()) == m0);
    EXPECT(!readable_within(ref_in, 150));
    const auto pm0 = frame(tag, seq, zps_packet(tag, 0, 0.5f));
    EXPECT(net::send_all(ref_out, pm0.data(), pm0.size()));
    const auto d0 = frame(tag, seq, {0x80, 0xd5, 0x2a, 0x7f}); // -128, -43, 42, 127
    EXPECT(read_exact(ref_in, d0.size()) == d0);
    const auto pd0 = frame(tag, seq, {0xec, 0xf2, 0xec, 0xf2}); // (-20, -14) x 0.5: the peer's -10, -7, -10, -7
    EXPECT(net::send_all(ref_out, pd0.data(), pd0.size()));
    // all-gather: the library owns chunk 1 = [0, 3, 0, 3]: scale 3 / 255, zero point -128, its copy := D(Q(x))
    const auto m1 = frame(tag, seq, zps_packet(tag, -128, s3));
    EXPECT(read_exact(ref_in, m1.size()) == m1);
    EXPECT(!readable_within(ref_in, 150));
    const auto pm1 = frame(tag, seq, zps_packet(tag, -100, 0.25f));
    EXPECT(net::send_all(ref_out, pm1.data(), pm1.size()));
    const auto d1 = frame(tag, seq, {0x80, 0x7f, 0x80, 0x7f});
    EXPECT(read_exact(ref_in, d1.size()) == d1);
    const auto pd1 = frame(tag, seq, {0xa0, 0xa4, 0xa8, 0xac}); // (q + 100) x 0.25: the peer's chunk 0 = 1, 2, 3, 4
    EXPECT(net::send_all(ref_out, pd1.data(), pd1.size()));
    lib.join();
    EXPECT(rc == 0);
    const std::vector<float> want = {1, 2, 3, 4, 0, 255 * s3, 0, 255 * s3};
    EXPECT(data == want);
    // a zero-point-scale packet counts 10 + serializedSize() = 10 + 8 + 1 + 4 + 4 (its min / max vectors are empty)
    EXPECT(txc.load() == 2 * 27 + 8 && rxc.load() == 2 * 27 + 8);
    EXPECT(!readable_within(ref_in, 50));
    tx->interrupt();
    rx->interrupt();
    ::close(ref_in);
    ::close(ref_out);
}

// An unquantized reference-framed ring step larger than the reference's 64 MiB frame (PCCL_MULTIPLEX_CHUNK_SIZE,
// reduce.cpp:20): rank 1 of a 3-peer ring, ring chunks of 64 MiB + 4 KiB. The emulated reference neighbours send each
// step as a 64 MiB frame plus a 4 KiB one on the op's data tag and stream counter (reference reduce.cpp:201-274); the
// library's frames carry the same tag / counter, every byte of every step is the ring algorithm's (reduce-scatter
// sends the own chunk, then the reduced one; all-gather forwards), and the byte counters hold the data bytes only.
TEST(reference_framed_plain_ring_frames_above_64mib) {
    int txsv[2], rxsv[2];
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, txsv) == 0);
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, rxsv) == 0);
    auto tx = std::make_shared<net::MuxConn>(txsv[0], net::MuxConn::Mode::Tx, SockAddr{});
    auto rx = std::make_shared<net::MuxConn>(rxsv[1], net::MuxConn::Mode::Rx, SockAddr{});
    EXPECT(tx->start() && rx->start());
    const Conns txs{tx}, rxs{rx};
    const int ref_in = txsv[1], ref_out = rxsv[0];
    constexpr size_t C = (size_t{16} << 20) + 1024; // floats per ring chunk: 64 MiB + 4 KiB
    std::vector<float> data(3 * C);
    for (size_t i = 0; i < data.size(); ++i) data[i] = static_cast<float>(i % 7);
    const std::vector<float> x = data;
    const uint64_t tag = 0xabc, seq = 41;
    std::atomic<uint64_t> txc{0}, rxc{0};
    int rc = -1;
    std::thread lib([&] {
        HostRingArgs A{txs, rxs, 3, 1, tag, seq, Shape::reference_framing(), reinterpret_cast<uint8_t *>(data.data()),
                       data.size(), DType::F32, DType::F32, QuantAlgo::None, ReduceOp::Sum, false,
                       [] { return false; }, txc, rxc};
        rc = host_ring(A);
    });
    // the previous peer's four steps (reduce-scatter 0, 1, all-gather 0, 1): constant chunks 1, 2, 3, 4
    std::thread prev([&] {
        std::vector<float> chunk(C);
        for (int g = 0; g < 4; ++g) {
            std::fill(chunk.begin(), chunk.end(), static_cast<float>(g + 1));
            const auto *b = reinterpret_cast<const uint8_t *>(chunk.data());
            for (size_t off = 0; off < C * 4;) {
                const size_t n = std::min<size_t>(size_t{64} << 20, C * 4 - off);
                uint8_t h[net::kMuxHeaderBytes];
                net::mux_frame_header(h, n, tag, seq);
                if (!net::send_all(ref_out, h, sizeof(h)) || !net::send_all(ref_out, b + off, n)) return;
                off += n;
            }
        }
    });
    // what the library must send per step, as a function of the element index inside the chunk
    auto expect_tx = [&](int g, size_t i) -> float {
        switch (g) {
            case 0: return x[C + i];         // its own chunk 1
            case 1: return x[i] + 1.0f;      // chunk 0 reduced with the peer's part
            case 2: return x[2 * C + i] + 2.0f; // chunk 2, fully reduced: it owns it
            default: return 3.0f;            // chunk 1 as received (forwarded)
        }
    };
    bool headers_ok = true, bytes_ok = true;
    size_t frames = 0;
    std::vector<uint8_t> buf;
    for (int g = 0; g < 4; ++g) {
        for (size_t got = 0; got < C * 4;) {
            const auto h = read_exact(ref_in, net::kMuxHeaderBytes);
            uint64_t n = 0, t = 0, c = 0;
            if (h.size() != net::kMuxHeaderBytes || !net::mux_parse_header(h.data(), n, t, c)) {
                headers_ok = false;
                break;
            }
            headers_ok = headers_ok && t == tag && c == seq && n > 0 && got + n <= C * 4 && n % 4 == 0;
            buf = read_exact(ref_in, n);
            if (buf.size() != n) {
                headers_ok = false;
                break;
            }
            const size_t e0 = got / 4;
            for (size_t k = 0; k < n / 4; ++k) {
                float v;
                std::memcpy(&v, buf.data() + 4 * k, 4);
                bytes_ok = bytes_ok && v == expect_tx(g, e0 + k);
            }
            got += n;
            ++frames;
        }
    }
    prev.join();
    lib.join();
    EXPECT(rc == 0 && headers_ok && bytes_ok && frames >= 8);
    bool result_ok = true;
    for (size_t i = 0; i < C; ++i)
        result_ok = result_ok && data[i] == 4.0f && data[C + i] == 3.0f && data[2 * C + i] == x[2 * C + i] + 2.0f;
    EXPECT(result_ok);
    EXPECT(txc.load() == 4 * C * 4 && rxc.load() == 4 * C * 4);
    EXPECT(!readable_within(ref_in, 50));
    tx->interrupt();
    rx->interrupt();
    ::close(ref_in);
    ::close(ref_out);
}
