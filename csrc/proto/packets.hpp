// CCoIP packet definitions. Wire layouts follow SURVEY Appendix A (reference ccoip/src/cpp/ccoip_packets.cpp);
// this is an independent implementation of the same byte format.
//
// Framing on control sockets (master, shared-state, benchmark, p2p hello): u64 length(payload+2) | u16 id | payload.
// Packets carried inside multiplexed P2P frames: u16 id | payload (no length; the frame carries it).
#pragma once

#include <array>
#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "../common/types.hpp"
#include "buffer.hpp"

namespace pccl::proto {

using PacketId = uint16_t;

// ---- client -> master ----
constexpr PacketId C2M_REQUEST_SESSION_REGISTRATION = 1;
constexpr PacketId C2M_REQUEST_ESTABLISH_P2P_CONNECTIONS = 2;
constexpr PacketId C2M_P2P_CONNECTIONS_ESTABLISHED = 3;
constexpr PacketId C2M_CHECK_PEERS_PENDING = 4;
constexpr PacketId C2M_OPTIMIZE_TOPOLOGY = 5;
constexpr PacketId C2M_REPORT_PEER_BANDWIDTH = 6;
constexpr PacketId C2M_OPTIMIZE_TOPOLOGY_WORK_COMPLETE = 7;
constexpr PacketId C2M_SYNC_SHARED_STATE = 8;
constexpr PacketId C2M_DIST_SHARED_STATE_COMPLETE = 9;
constexpr PacketId C2M_COLLECTIVE_COMMS_INITIATE = 10;
constexpr PacketId C2M_COLLECTIVE_COMMS_COMPLETE = 11;
// extensions (liveness, negotiated at registration: sent only to / by peers that announced it)
constexpr PacketId C2M_HEARTBEAT = 12;
constexpr PacketId C2M_OP_STALLED = 13;
// ---- master -> client ----
constexpr PacketId M2C_SESSION_REGISTRATION_RESPONSE = 1;
constexpr PacketId M2C_P2P_CONNECTION_INFO = 2;
constexpr PacketId M2C_P2P_CONNECTIONS_ESTABLISHED = 3;
constexpr PacketId M2C_PEERS_PENDING_RESPONSE = 4;
constexpr PacketId M2C_OPTIMIZE_TOPOLOGY_RESPONSE = 5;
constexpr PacketId M2C_OPTIMIZE_TOPOLOGY_COMPLETE = 6;
constexpr PacketId M2C_SYNC_SHARED_STATE = 7;
constexpr PacketId M2C_SYNC_SHARED_STATE_COMPLETE = 8;
constexpr PacketId M2C_COLLECTIVE_COMMS_COMMENCE = 9;
constexpr PacketId M2C_COLLECTIVE_COMMS_COMPLETE = 10;
constexpr PacketId M2C_COLLECTIVE_COMMS_ABORT = 11;
constexpr PacketId M2C_HEARTBEAT = 12; // extension (liveness)
// ---- peer <-> peer ----
constexpr PacketId P2P_HELLO = 1;
constexpr PacketId P2P_HELLO_ACK = 2;
constexpr PacketId P2P_DEQUANTIZATION_META = 3;
// ---- shared state client <-> server ----
constexpr PacketId C2S_REQUEST_SHARED_STATE = 1;
constexpr PacketId S2C_SHARED_STATE_RESPONSE = 1;
// extension (not in the reference protocol): same-host HBM hand-off over HIP IPC instead of a TCP byte stream
constexpr PacketId C2S_REQUEST_SHARED_STATE_IPC = 2;
constexpr PacketId S2C_SHARED_STATE_IPC_RESPONSE = 2;
constexpr PacketId C2S_SHARED_STATE_IPC_DONE = 3;
// ---- benchmark ----
constexpr PacketId C2B_HELLO = 1;
constexpr PacketId B2C_BENCHMARK_SERVER_IS_BUSY = 1;

struct Empty {
    void encode(WBuf &) const {}
    bool decode(RBuf &) { return true; }
};

struct C2MRequestSessionRegistration {
    static constexpr PacketId kId = C2M_REQUEST_SESSION_REGISTRATION;
    uint32_t peer_group = 0;
    bool use_explicit_addresses = false;
    SockAddr advertised_p2p{}, advertised_ss{}, advertised_bm{};
    uint16_t p2p_port = 0, ss_port = 0, bm_port = 0;
    // extension (appended, optional on decode): host identity (boot id + hostname) so the master can tell peers
    // that share a host -- and may use the xGMI IPC path -- even when the master is not on loopback
    std::string host_token;
    // extension after host_token (optional, default true): this peer can take the xGMI IPC path (a GPU backend and
    // no PCCL_DISABLE_IPC). Same-host pairs of which one cannot are benchmarked like remote pairs: their traffic
    // crosses loopback TCP, so a fixed xGMI-class cost would mislead the ring optimiser.
    bool xgmi_capable = true;
    // extension after xgmi_capable (optional, u8 version): the peer runs the liveness protocol - it sends
    // C2MHeartbeat at the interval the master answers with, reports stalled ops (C2MOpStalled) and watches the
    // master's M2CHeartbeat. A reference peer sends none of it and the master exempts it from the peer timeout.
    static constexpr uint8_t kLivenessVersion = 1;
    bool liveness = false;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct C2MRequestEstablishP2PConnections {
    static constexpr PacketId kId = C2M_REQUEST_ESTABLISH_P2P_CONNECTIONS;
    bool accept_new_peers = false;
    void encode(WBuf &w) const { w.boolean(accept_new_peers); }
    bool decode(RBuf &r) {
        accept_new_peers = r.boolean();
        return r.ok();
    }
};

struct C2MP2PConnectionsEstablished {
    static constexpr PacketId kId = C2M_P2P_CONNECTIONS_ESTABLISHED;
    bool success = false;
    std::vector<Uuid> failed_peers;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct C2MCheckPeersPending : Empty {
    static constexpr PacketId kId = C2M_CHECK_PEERS_PENDING;
};
struct C2MOptimizeTopology : Empty {
    static constexpr PacketId kId = C2M_OPTIMIZE_TOPOLOGY;
};
struct C2MOptimizeTopologyWorkComplete : Empty {
    static constexpr PacketId kId = C2M_OPTIMIZE_TOPOLOGY_WORK_COMPLETE;
};

struct C2MReportPeerBandwidth {
    static constexpr PacketId kId = C2M_REPORT_PEER_BANDWIDTH;
    Uuid to_peer;
    double bandwidth_mbps = 0;
    void encode(WBuf &w) const {
        w.uuid(to_peer);
        w.f64(bandwidth_mbps);
    }
    bool decode(RBuf &r) {
        to_peer = r.uuid();
        bandwidth_mbps = r.f64();
        return r.ok();
    }
};

struct SharedStateHashEntry {
    std::string key;
    uint64_t hash = 0;
    HashType hash_type = HashType::Simple;
    uint64_t num_elements = 0;
    DType data_type = DType::F32;
    bool allow_content_inequality = false;
    bool operator==(const SharedStateHashEntry &o) const {
        return key == o.key && hash == o.hash && hash_type == o.hash_type && num_elements == o.num_elements &&
               data_type == o.data_type && allow_content_inequality == o.allow_content_inequality;
    }
};

struct C2MSyncSharedState {
    static constexpr PacketId kId = C2M_SYNC_SHARED_STATE;
    uint64_t revision = 0;
    SyncStrategy strategy = SyncStrategy::EnforcePopular;
    std::vector<SharedStateHashEntry> entries;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct C2MDistSharedStateComplete : Empty {
    static constexpr PacketId kId = C2M_DIST_SHARED_STATE_COMPLETE;
};

// the peer can run this op hierarchically (device buffers, host-local IPC arena, inter-host ring connections)
constexpr uint8_t kCollFlagHierarchical = 1;
// this peer's PCCL_SMALL_ALLREDUCE_BYTES selects the all-gather small-message algorithm for this op; ANDed by the
// master like every capability bit, so a threshold that differs between peers cannot split the ring between the two
// algorithms (the op then uses the reduce-scatter ring everywhere)
constexpr uint8_t kCollFlagSmallPath = 2;
// the peer speaks the pccl-amd data-plane framing for this op: ring steps striped over several pooled connections,
// quantized ops split into lanes with their dequantization metadata on a separate tag (docs/WIRE_DIVERGENCES.md).
// Without it on every participant (a reference peer, or PCCL_WIRE=reference) the op runs the reference framing: one
// connection seq % pool per op, the metadata packet on the data tag before the step's data, one lane.
constexpr uint8_t kCollFlagExtWire = 4;

// Data-plane shape of one op (extension of the initiate / commence packets, present iff kCollFlagExtWire). Every peer
// proposes its own settings in its initiate; the master agrees on one shape per op (fewest stripes and lanes, largest
// stripe minimum, smallest segment) and every peer runs the commence's, so peers whose PCCL_RING_STRIPES /
// PCCL_STRIPE_MIN_BYTES / PCCL_QUANT_LANES / PCCL_SEGMENT_CHUNK_MIB differ still derive identical stripe plans,
// connections, lane tags and segments.
struct WireShape {
    uint8_t stripes = 4;            // PCCL_RING_STRIPES: striped connections per ring step (1..16)
    uint8_t quant_lanes = 2;        // PCCL_QUANT_LANES: lanes of a quantized op (1..4)
    uint16_t stripe_min_kib = 8192; // PCCL_STRIPE_MIN_BYTES / 1 KiB: smallest stripe (>= 256 KiB)
    uint16_t segment_chunk_mib = 128; // PCCL_SEGMENT_CHUNK_MIB: largest ring chunk of one segment (0: one segment)
    void encode(WBuf &w) const {
        w.u8(stripes);
        w.u8(quant_lanes);
        w.u16(stripe_min_kib);
        w.u16(segment_chunk_mib);
    }
    bool decode(RBuf &r) {
        if (!r.ok() || r.remaining() < 6) return false;
        stripes = r.u8();
        quant_lanes = r.u8();
        stripe_min_kib = r.u16();
        segment_chunk_mib = r.u16();
        stripes = stripes < 1 ? 1 : (stripes > 16 ? 16 : stripes);
        quant_lanes = quant_lanes < 1 ? 1 : (quant_lanes > 4 ? 4 : quant_lanes);
        if (stripe_min_kib < 256) stripe_min_kib = 256;
        return r.ok();
    }
    bool operator==(const WireShape &o) const {
        return stripes == o.stripes && quant_lanes == o.quant_lanes && stripe_min_kib == o.stripe_min_kib &&
               segment_chunk_mib == o.segment_chunk_mib;
    }
};

struct C2MCollectiveCommsInitiate {
    static constexpr PacketId kId = C2M_COLLECTIVE_COMMS_INITIATE;
    uint64_t tag = 0;
    uint64_t count = 0;
    DType data_type = DType::F32;
    ReduceOp op = ReduceOp::Sum;
    // extension (appended, optional): capability bits of this peer for this op (kCollFlagHierarchical)
    uint8_t flags = 0;
    // extension after flags, present iff flags has kCollFlagExtWire: the data-plane shape this peer proposes
    WireShape shape{};
    void encode(WBuf &w) const {
        w.u64(tag);
        w.u64(count);
        w.u8(static_cast<uint8_t>(data_type));
        w.u8(static_cast<uint8_t>(op));
        if (flags) w.u8(flags);
        if (flags & kCollFlagExtWire) shape.encode(w);
    }
    bool decode(RBuf &r) {
        tag = r.u64();
        count = r.u64();
        data_type = static_cast<DType>(r.u8());
        op = static_cast<ReduceOp>(r.u8());
        flags = r.ok() && r.remaining() > 0 ? r.u8() : 0;
        if ((flags & kCollFlagExtWire) && !shape.decode(r)) flags &= static_cast<uint8_t>(~kCollFlagExtWire);
        return r.ok();
    }
};


struct C2MCollectiveCommsComplete {
    static constexpr PacketId kId = C2M_COLLECTIVE_COMMS_COMPLETE;
    uint64_t tag = 0;
    bool was_aborted = false;
    void encode(WBuf &w) const {
        w.u64(tag);
        w.boolean(was_aborted);
    }
    bool decode(RBuf &r) {
        tag = r.u64();
        was_aborted = r.boolean();
        return r.ok();
    }
};

struct M2CSessionRegistrationResponse {
    static constexpr PacketId kId = M2C_SESSION_REGISTRATION_RESPONSE;
    bool accepted = false;
    Uuid assigned_uuid;
    // extension (appended only for a peer that announced liveness): the master's liveness parameters. The peer sends
    // C2MHeartbeat every heartbeat_ms and is dropped after peer_timeout_ms of silence; the master sends M2CHeartbeat
    // at the same interval, and a peer treats peer_timeout_ms without any packet from the master as a lost master.
    // op_stall_ms: an op's data path without progress for this long is reported (C2MOpStalled). 0 / absent: off.
    uint32_t heartbeat_ms = 0, peer_timeout_ms = 0, op_stall_ms = 0;
    void encode(WBuf &w) const {
        w.boolean(accepted);
        w.uuid(assigned_uuid);
        if (heartbeat_ms || peer_timeout_ms || op_stall_ms) {
            w.u32(heartbeat_ms);
            w.u32(peer_timeout_ms);
            w.u32(op_stall_ms);
        }
    }
    bool decode(RBuf &r) {
        accepted = r.boolean();
        assigned_uuid = r.uuid();
        if (r.ok() && r.remaining() >= 12) {
            heartbeat_ms = r.u32();
            peer_timeout_ms = r.u32();
            op_stall_ms = r.u32();
        }
        return r.ok();
    }
};

// Liveness extension packets (C2M_HEARTBEAT / M2C_HEARTBEAT carry nothing; any packet counts as a sign of life).
struct C2MHeartbeat : Empty {
    static constexpr PacketId kId = C2M_HEARTBEAT;
};
struct M2CHeartbeat : Empty {
    static constexpr PacketId kId = M2C_HEARTBEAT;
};

// A running op's data path made no progress (no byte received or sent on its connections) for op_stall_ms. The
// reporter names the peer its evidence points at: the next peer if its own send to it has been blocked (the next
// peer does not drain its socket), else the previous one (nothing arrives from it). `step` is the ring step the
// reporter waits in; in a ring stalled at one link the peers behind the broken link wait in later steps, so the
// report with the lowest step names the link. The master collects the reports of an op for a short window, kicks
// the peer the evidence names and aborts the op (docs/ARCHITECTURE.md, failure detection).
constexpr uint8_t kStallRxIdle = 0, kStallTxBlocked = 1;
struct C2MOpStalled {
    static constexpr PacketId kId = C2M_OP_STALLED;
    uint64_t tag = 0;
    Uuid suspect;
    uint8_t kind = kStallRxIdle;
    uint32_t step = 0;
    uint64_t idle_ms = 0;
    void encode(WBuf &w) const {
        w.u64(tag);
        w.uuid(suspect);
        w.u8(kind);
        w.u32(step);
        w.u64(idle_ms);
    }
    bool decode(RBuf &r) {
        tag = r.u64();
        suspect = r.uuid();
        kind = r.u8();
        step = r.u32();
        idle_ms = r.u64();
        return r.ok();
    }
};

struct PeerInfo {
    SockAddr p2p_listen_addr{};
    Uuid peer_uuid;
};

// Extension: inter-host ring partners of the hierarchical all-reduce (same local rank on the next / previous host).
struct ExtraPeer {
    PeerInfo peer;
    uint8_t role = 0; // kExtraTx: open a TX pool to it; kExtraRx: keep the RX pool it opens to us
};
constexpr uint8_t kExtraTx = 1, kExtraRx = 2;

struct M2CP2PConnectionInfo {
    static constexpr PacketId kId = M2C_P2P_CONNECTION_INFO;
    bool unchanged = false;
    uint64_t global_world_size = 0;
    uint64_t local_world_size = 0;
    uint64_t num_distinct_peer_groups = 0;
    uint64_t largest_peer_group_world_size = 0;
    std::vector<PeerInfo> all_peers;
    std::vector<ExtraPeer> extra_peers; // extension (appended, optional; sent even when `unchanged`)
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct M2CP2PConnectionsEstablished {
    static constexpr PacketId kId = M2C_P2P_CONNECTIONS_ESTABLISHED;
    bool success = false;
    std::vector<Uuid> ring_order;
    bool single_host = false; // extension (appended, optional): every ring member reported the same host token
    bool has_host_info = false; // the extension is present (decode) / to be sent (encode): single_host is authoritative
    std::vector<uint32_t> host_of; // extension (appended, optional): host index of every ring member (ring order)
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct M2CPeersPendingResponse {
    static constexpr PacketId kId = M2C_PEERS_PENDING_RESPONSE;
    bool peers_pending = false;
    void encode(WBuf &w) const { w.boolean(peers_pending); }
    bool decode(RBuf &r) {
        peers_pending = r.boolean();
        return r.ok();
    }
};

struct BenchmarkRequest {
    Uuid from_peer;
    Uuid to_peer;
    SockAddr to_peer_endpoint{};
};

struct M2COptimizeTopologyResponse {
    static constexpr PacketId kId = M2C_OPTIMIZE_TOPOLOGY_RESPONSE;
    std::vector<BenchmarkRequest> requests;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct M2COptimizeTopologyComplete {
    static constexpr PacketId kId = M2C_OPTIMIZE_TOPOLOGY_COMPLETE;
    bool success = false;
    std::vector<Uuid> ring_order;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct M2CSyncSharedState {
    static constexpr PacketId kId = M2C_SYNC_SHARED_STATE;
    bool is_outdated = false;
    SockAddr distributor{};
    std::vector<std::string> outdated_keys;
    std::vector<uint64_t> expected_hashes;
    std::vector<HashType> expected_hash_types;
    // [pccl-amd extension, appended] other peers holding the elected state: tried in order if the distributor
    // dies mid-transfer (absent in reference-encoded packets)
    std::vector<SockAddr> fallback_distributors;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct M2CSyncSharedStateComplete : Empty {
    static constexpr PacketId kId = M2C_SYNC_SHARED_STATE_COMPLETE;
};

struct M2CCollectiveCommsCommence {
    static constexpr PacketId kId = M2C_COLLECTIVE_COMMS_COMMENCE;
    uint64_t tag = 0;
    uint64_t seq_nr = 0;
    uint8_t flags = 0; // extension (appended, optional): AND of every participant's initiate flags
    WireShape shape{};  // extension after flags, present iff flags has kCollFlagExtWire: the op's agreed shape
    void encode(WBuf &w) const {
        w.u64(tag);
        w.u64(seq_nr);
        if (flags) w.u8(flags);
        if (flags & kCollFlagExtWire) shape.encode(w);
    }
    bool decode(RBuf &r) {
        tag = r.u64();
        seq_nr = r.u64();
        flags = r.ok() && r.remaining() > 0 ? r.u8() : 0;
        if ((flags & kCollFlagExtWire) && !shape.decode(r)) flags &= static_cast<uint8_t>(~kCollFlagExtWire);
        return r.ok();
    }
};

struct M2CCollectiveCommsComplete {
    static constexpr PacketId kId = M2C_COLLECTIVE_COMMS_COMPLETE;
    uint64_t tag = 0;
    void encode(WBuf &w) const { w.u64(tag); }
    bool decode(RBuf &r) {
        tag = r.u64();
        return r.ok();
    }
};

struct M2CCollectiveCommsAbort {
    static constexpr PacketId kId = M2C_COLLECTIVE_COMMS_ABORT;
    uint64_t tag = 0;
    bool aborted = false;
    void encode(WBuf &w) const {
        w.u64(tag);
        w.boolean(aborted);
    }
    bool decode(RBuf &r) {
        tag = r.u64();
        aborted = r.boolean();
        return r.ok();
    }
};

struct P2PHello {
    static constexpr PacketId kId = P2P_HELLO;
    Uuid peer_uuid;
    uint32_t connection_nr = 0;
    void encode(WBuf &w) const {
        w.uuid(peer_uuid);
        w.u32(connection_nr);
    }
    bool decode(RBuf &r) {
        peer_uuid = r.uuid();
        connection_nr = r.u32();
        return r.ok();
    }
};

struct P2PHelloAck : Empty {
    static constexpr PacketId kId = P2P_HELLO_ACK;
};

// De-quantization metadata exchanged per ring step (values kept as double/int64 in memory; encoded in the
// reference's byte layout: MIN_MAX -> u8 dtype + min bytes + max bytes (floats little-endian host order, ints
// big-endian), ZERO_POINT_SCALE -> u8 zp dtype + zp bytes + u8 scale dtype + scale bytes).
struct QuantMeta {
    QuantAlgo algo = QuantAlgo::None; // MinMax or ZeroPointScale
    DType value_type = DType::F32;    // dtype of min/max (== the unquantized data type)
    double min_value = 0, max_value = 0;
    int64_t zero_point = 0;
    float scale = 1.0f;
    bool operator==(const QuantMeta &o) const {
        return algo == o.algo && value_type == o.value_type && min_value == o.min_value &&
               max_value == o.max_value && zero_point == o.zero_point && scale == o.scale;
    }
};

struct P2PDequantizationMeta {
    static constexpr PacketId kId = P2P_DEQUANTIZATION_META;
    uint64_t tag = 0;
    QuantMeta meta;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct C2SRequestSharedState {
    static constexpr PacketId kId = C2S_REQUEST_SHARED_STATE;
    std::vector<std::string> keys;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

enum class SharedStateStatus : uint8_t { Success = 1, NotDistributed = 2, NotInMode = 3, UnknownKey = 4 };

struct SharedStateEntryInfo {
    std::string key;
    uint64_t size_bytes = 0;
};

struct S2CSharedStateResponse {
    static constexpr PacketId kId = S2C_SHARED_STATE_RESPONSE;
    SharedStateStatus status = SharedStateStatus::Success;
    uint64_t revision = 0;
    std::vector<SharedStateEntryInfo> entries;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

// Same-host request: like C2SRequestSharedState plus the requester's host identity (boot id + hostname) and pid.
// A distributor on the same host answers device-resident entries with HIP IPC handles (mode 1) that the requester
// maps and copies from over xGMI / HBM; everything else (mode 0) follows as raw bytes on the stream, in order.
struct C2SRequestSharedStateIpc {
    static constexpr PacketId kId = C2S_REQUEST_SHARED_STATE_IPC;
    std::vector<std::string> keys;
    std::string host_token;
    uint32_t pid = 0;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

struct SharedStateIpcEntry {
    std::string key;
    uint64_t size_bytes = 0;
    // 0: bytes follow on the stream, 1: hipIpc handle of the allocation (PCCL_IPC_MODE=fast), 2: VMM fd shares
    // (fault-safe: the importer keeps the pages alive if the distributor dies mid-copy) — `handle` is the first
    // segment, `more_handles` the rest; the entry's bytes are the segments back to back, `seg_bytes` each (the last
    // one shorter), starting at `offset` inside the first
    uint8_t mode = 0;
    int32_t device = -1;
    uint64_t offset = 0;   // byte offset of the entry inside the exported allocation
    uint64_t raw_ptr = 0;  // the distributor's pointer (usable directly when both peers share a process)
    uint8_t handle[64]{};  // hipIpcMemHandle_t of the allocation / VmmHandle of the first segment
    uint64_t seg_bytes = 0;                          // mode 2 only (encoded only then)
    std::vector<std::array<uint8_t, 64>> more_handles; // mode 2 only
};

struct S2CSharedStateIpcResponse {
    static constexpr PacketId kId = S2C_SHARED_STATE_IPC_RESPONSE;
    SharedStateStatus status = SharedStateStatus::Success;
    uint64_t revision = 0;
    uint32_t pid = 0;
    std::vector<SharedStateIpcEntry> entries;
    void encode(WBuf &w) const;
    bool decode(RBuf &r);
};

// Requester -> distributor after all IPC copies finished (the distributor keeps its exports alive until then).
struct C2SSharedStateIpcDone {
    static constexpr PacketId kId = C2S_SHARED_STATE_IPC_DONE;
    bool ok = true;
    void encode(WBuf &w) const { w.boolean(ok); }
    bool decode(RBuf &r) {
        ok = r.boolean();
        return r.ok();
    }
};

struct C2BHello {
    static constexpr PacketId kId = C2B_HELLO;
    Uuid peer_uuid;
    void encode(WBuf &w) const { w.uuid(peer_uuid); }
    bool decode(RBuf &r) {
        peer_uuid = r.uuid();
        return r.ok();
    }
};

struct B2CBenchmarkServerIsBusy {
    static constexpr PacketId kId = B2C_BENCHMARK_SERVER_IS_BUSY;
    bool is_busy = false;
    void encode(WBuf &w) const { w.boolean(is_busy); }
    bool decode(RBuf &r) {
        is_busy = r.boolean();
        return r.ok();
    }
};

// Serialize a packet as u16 id + payload (used inside multiplexed frames and after the LTV length prefix).
template<typename P>
std::vector<uint8_t> encode_with_id(const P &p) {
    WBuf w;
    w.u16(P::kId);
    p.encode(w);
    return std::move(w.data);
}

// Parse payload (after the id) into a packet; returns nullopt on malformed input.
template<typename P>
std::optional<P> decode_payload(const uint8_t *data, size_t n) {
    RBuf r(data, n);
    P p{};
    if (!p.decode(r) || !r.ok()) return std::nullopt;
    return p;
}

} // namespace pccl::proto
