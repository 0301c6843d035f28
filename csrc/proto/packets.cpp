#include "packets.hpp"

#include <cstring>

namespace pccl::proto {

void C2MRequestSessionRegistration::encode(WBuf &w) const {
    w.u32(peer_group);
    w.boolean(use_explicit_addresses);
    if (use_explicit_addresses) {
        w.sockaddr(advertised_p2p);
        w.sockaddr(advertised_ss);
        w.sockaddr(advertised_bm);
    } else {
        w.u16(p2p_port);
        w.u16(ss_port);
        w.u16(bm_port);
    }
    if (!host_token.empty()) {
        w.str(host_token);
        w.boolean(xgmi_capable);
        if (liveness) w.u8(kLivenessVersion);
    }
}

bool C2MRequestSessionRegistration::decode(RBuf &r) {
    peer_group = r.u32();
    use_explicit_addresses = r.boolean();
    if (use_explicit_addresses) {
        advertised_p2p = r.sockaddr();
        advertised_ss = r.sockaddr();
        advertised_bm = r.sockaddr();
        p2p_port = advertised_p2p.port;
        ss_port = advertised_ss.port;
        bm_port = advertised_bm.port;
    } else {
        p2p_port = r.u16();
        ss_port = r.u16();
        bm_port = r.u16();
    }
    if (r.ok() && r.remaining() > 0) host_token = r.str(); // absent when the peer is a reference implementation
    xgmi_capable = true;
    if (r.ok() && r.remaining() > 0) xgmi_capable = r.boolean();
    liveness = r.ok() && r.remaining() > 0 && r.u8() >= 1;
    return r.ok();
}

void C2MP2PConnectionsEstablished::encode(WBuf &w) const {
    w.boolean(success);
    w.u64(failed_peers.size());
    for (const auto &u : failed_peers) w.uuid(u);
}

bool C2MP2PConnectionsEstablished::decode(RBuf &r) {
    success = r.boolean();
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 16)) return false;
    failed_peers.resize(n);
    for (auto &u : failed_peers) u = r.uuid();
    return r.ok();
}

void C2MSyncSharedState::encode(WBuf &w) const {
    w.u64(revision);
    w.u8(static_cast<uint8_t>(strategy));
    w.u64(entries.size());
    for (const auto &e : entries) {
        w.str(e.key);
        w.u64(e.hash);
        w.u8(static_cast<uint8_t>(e.hash_type));
        w.u64(e.num_elements);
        w.u8(static_cast<uint8_t>(e.data_type));
        w.boolean(e.allow_content_inequality);
    }
}

bool C2MSyncSharedState::decode(RBuf &r) {
    revision = r.u64();
    strategy = static_cast<SyncStrategy>(r.u8());
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 27)) return false;
    entries.resize(n);
    for (auto &e : entries) {
        e.key = r.str();
        e.hash = r.u64();
        e.hash_type = static_cast<HashType>(r.u8());
        e.num_elements = r.u64();
        e.data_type = static_cast<DType>(r.u8());
        e.allow_content_inequality = r.boolean();
    }
    return r.ok() && static_cast<uint8_t>(strategy) <= 2;
}

void M2CP2PConnectionInfo::encode(WBuf &w) const {
    w.boolean(unchanged);
    w.u64(global_world_size);
    w.u64(local_world_size);
    w.u64(num_distinct_peer_groups);
    w.u64(largest_peer_group_world_size);
    if (!unchanged) {
        w.u64(all_peers.size());
        for (const auto &p : all_peers) {
            w.sockaddr(p.p2p_listen_addr);
            w.uuid(p.peer_uuid);
        }
    }
    if (!extra_peers.empty()) {
        w.u64(extra_peers.size());
        for (const auto &e : extra_peers) {
            w.sockaddr(e.peer.p2p_listen_addr);
            w.uuid(e.peer.peer_uuid);
            w.u8(e.role);
        }
    }
}

bool M2CP2PConnectionInfo::decode(RBuf &r) {
    unchanged = r.boolean();
    global_world_size = r.u64();
    local_world_size = r.u64();
    num_distinct_peer_groups = r.u64();
    largest_peer_group_world_size = r.u64();
    if (!unchanged) {
        const uint64_t n = r.u64();
        if (!r.plausible_count(n, 23)) return false;
        all_peers.resize(n);
        for (auto &p : all_peers) {
            p.p2p_listen_addr = r.sockaddr();
            p.peer_uuid = r.uuid();
        }
    }
    if (r.ok() && r.remaining() > 0) {
        const uint64_t m = r.u64();
        if (!r.plausible_count(m, 24)) return false;
        extra_peers.resize(m);
        for (auto &e : extra_peers) {
            e.peer.p2p_listen_addr = r.sockaddr();
            e.peer.peer_uuid = r.uuid();
            e.role = r.u8();
        }
    }
    return r.ok();
}

static void encode_uuid_list(WBuf &w, bool success, const std::vector<Uuid> &v) {
    w.boolean(success);
    w.u64(v.size());
    for (const auto &u : v) w.uuid(u);
}

static bool decode_uuid_list(RBuf &r, bool &success, std::vector<Uuid> &v) {
    success = r.boolean();
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 16)) return false;
    v.resize(n);
    for (auto &u : v) u = r.uuid();
    return r.ok();
}

void M2CP2PConnectionsEstablished::encode(WBuf &w) const {
    encode_uuid_list(w, success, ring_order);
    if (!has_host_info && !single_host && host_of.empty()) return; // reference layout
    w.boolean(single_host);
    if (!host_of.empty()) {
        w.u64(host_of.size());
        for (uint32_t h : host_of) w.u32(h);
    }
}
bool M2CP2PConnectionsEstablished::decode(RBuf &r) {
    if (!decode_uuid_list(r, success, ring_order)) return false;
    has_host_info = r.remaining() > 0;
    single_host = has_host_info && r.boolean();
    if (r.ok() && r.remaining() > 0) {
        const uint64_t n = r.u64();
        if (!r.plausible_count(n, 4)) return false;
        host_of.resize(n);
        for (auto &h : host_of) h = r.u32();
    }
    return r.ok();
}
void M2COptimizeTopologyComplete::encode(WBuf &w) const { encode_uuid_list(w, success, ring_order); }
bool M2COptimizeTopologyComplete::decode(RBuf &r) { return decode_uuid_list(r, success, ring_order); }

void M2COptimizeTopologyResponse::encode(WBuf &w) const {
    w.u64(requests.size());
    for (const auto &q : requests) {
        w.uuid(q.from_peer);
        w.uuid(q.to_peer);
        w.sockaddr(q.to_peer_endpoint);
    }
}

bool M2COptimizeTopologyResponse::decode(RBuf &r) {
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 39)) return false;
    requests.resize(n);
    for (auto &q : requests) {
        q.from_peer = r.uuid();
        q.to_peer = r.uuid();
        q.to_peer_endpoint = r.sockaddr();
    }
    return r.ok();
}

void M2CSyncSharedState::encode(WBuf &w) const {
    w.boolean(is_outdated);
    w.sockaddr(distributor);
    w.u64(outdated_keys.size());
    for (const auto &k : outdated_keys) w.str(k);
    for (size_t i = 0; i < outdated_keys.size(); ++i) w.u64(i < expected_hashes.size() ? expected_hashes[i] : 0);
    for (size_t i = 0; i < outdated_keys.size(); ++i)
        w.u8(static_cast<uint8_t>(i < expected_hash_types.size() ? expected_hash_types[i] : HashType::Simple));
    if (fallback_distributors.empty()) return; // reference layout
    w.u64(fallback_distributors.size());
    for (const auto &a : fallback_distributors) w.sockaddr(a);
}

bool M2CSyncSharedState::decode(RBuf &r) {
    is_outdated = r.boolean();
    distributor = r.sockaddr();
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 17)) return false;
    outdated_keys.resize(n);
    for (auto &k : outdated_keys) k = r.str();
    expected_hashes.resize(n);
    for (auto &h : expected_hashes) h = r.u64();
    expected_hash_types.resize(n);
    for (auto &t : expected_hash_types) t = static_cast<HashType>(r.u8());
    fallback_distributors.clear();
    if (r.ok() && r.remaining() >= 8) {
        const uint64_t m = r.u64();
        if (!r.plausible_count(m, 7)) return false;
        fallback_distributors.resize(m);
        for (auto &a : fallback_distributors) a = r.sockaddr();
    }
    return r.ok();
}

// ---- dequantization meta ----
static void put_value(WBuf &w, DType t, double v) {
    // floats in host (little-endian) byte order, integers in network order, as the reference does on x86
    switch (t) {
        case DType::F32: {
            const float f = static_cast<float>(v);
            w.bytes(&f, 4);
            break;
        }
        case DType::F64: w.bytes(&v, 8); break;
        case DType::F16: case DType::BF16: { // not used by the reference; 2-byte float of the value, LE
            const float f = static_cast<float>(v);
            uint32_t u;
            std::memcpy(&u, &f, 4);
            const uint16_t h = static_cast<uint16_t>(u >> 16);
            w.bytes(&h, 2);
            break;
        }
        default: { // integer types: big-endian, width of the type
            const size_t n = dtype_size(t);
            const auto iv = static_cast<int64_t>(v);
            for (int i = static_cast<int>(n) - 1; i >= 0; --i) w.u8(static_cast<uint8_t>(static_cast<uint64_t>(iv) >> (8 * i)));
        }
    }
}

static double get_value(RBuf &r, DType t) {
    switch (t) {
        case DType::F32: {
            float f = 0;
            r.bytes(&f, 4);
            return f;
        }
        case DType::F64: {
            double d = 0;
            r.bytes(&d, 8);
            return d;
        }
        case DType::F16: case DType::BF16: {
            uint16_t h = 0;
            r.bytes(&h, 2);
            const uint32_t u = static_cast<uint32_t>(h) << 16;
            float f;
            std::memcpy(&f, &u, 4);
            return f;
        }
        default: {
            const size_t n = dtype_size(t);
            uint64_t u = 0;
            for (size_t i = 0; i < n; ++i) u = (u << 8) | r.u8();
            return static_cast<double>(static_cast<int64_t>(u));
        }
    }
}

void P2PDequantizationMeta::encode(WBuf &w) const {
    w.u64(tag);
    if (meta.algo == QuantAlgo::ZeroPointScale) {
        w.u8(1); // ZERO_POINT_SCALE
        w.u8(static_cast<uint8_t>(DType::I64));
        w.i64(meta.zero_point);
        w.u8(static_cast<uint8_t>(DType::F32));
        w.bytes(&meta.scale, 4);
    } else {
        w.u8(0); // MIN_MAX
        w.u8(static_cast<uint8_t>(meta.value_type));
        put_value(w, meta.value_type, meta.min_value);
        put_value(w, meta.value_type, meta.max_value);
    }
}

bool P2PDequantizationMeta::decode(RBuf &r) {
    tag = r.u64();
    const uint8_t type = r.u8();
    if (type == 0) {
        meta.algo = QuantAlgo::MinMax;
        const uint8_t dt = r.u8();
        if (!dtype_valid(dt)) return false;
        meta.value_type = static_cast<DType>(dt);
        meta.min_value = get_value(r, meta.value_type);
        meta.max_value = get_value(r, meta.value_type);
    } else if (type == 1) {
        meta.algo = QuantAlgo::ZeroPointScale;
        const uint8_t zt = r.u8();
        if (!dtype_valid(zt)) return false;
        meta.zero_point = static_cast<int64_t>(get_value(r, static_cast<DType>(zt)));
        const uint8_t st = r.u8();
        if (!dtype_valid(st)) return false;
        meta.scale = static_cast<float>(get_value(r, static_cast<DType>(st)));
    } else {
        return false;
    }
    return r.ok();
}

void C2SRequestSharedState::encode(WBuf &w) const {
    w.u64(keys.size());
    for (const auto &k : keys) w.str(k);
}

bool C2SRequestSharedState::decode(RBuf &r) {
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 8)) return false;
    keys.resize(n);
    for (auto &k : keys) k = r.str();
    return r.ok();
}

void S2CSharedStateResponse::encode(WBuf &w) const {
    w.u8(static_cast<uint8_t>(status));
    w.u64(revision);
    w.u64(entries.size());
    for (const auto &e : entries) {
        w.str(e.key);
        w.u64(e.size_bytes);
    }
}

bool S2CSharedStateResponse::decode(RBuf &r) {
    status = static_cast<SharedStateStatus>(r.u8());
    revision = r.u64();
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 16)) return false;
    entries.resize(n);
    for (auto &e : entries) {
        e.key = r.str();
        e.size_bytes = r.u64();
    }
    return r.ok();
}

void C2SRequestSharedStateIpc::encode(WBuf &w) const {
    w.u64(keys.size());
    for (const auto &k : keys) w.str(k);
    w.str(host_token);
    w.u32(pid);
}

bool C2SRequestSharedStateIpc::decode(RBuf &r) {
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 8)) return false;
    keys.resize(n);
    for (auto &k : keys) k = r.str();
    host_token = r.str();
    pid = r.u32();
    return r.ok();
}

void S2CSharedStateIpcResponse::encode(WBuf &w) const {
    w.u8(static_cast<uint8_t>(status));
    w.u64(revision);
    w.u32(pid);
    w.u64(entries.size());
    for (const auto &e : entries) {
        w.str(e.key);
        w.u64(e.size_bytes);
        w.u8(e.mode);
        w.u32(static_cast<uint32_t>(e.device));
        w.u64(e.offset);
        w.u64(e.raw_ptr);
        w.bytes(e.handle, sizeof(e.handle));
        if (e.mode == 2) {
            w.u64(e.seg_bytes);
            w.u32(static_cast<uint32_t>(e.more_handles.size()));
            for (const auto &h : e.more_handles) w.bytes(h.data(), h.size());
        }
    }
}

bool S2CSharedStateIpcResponse::decode(RBuf &r) {
    status = static_cast<SharedStateStatus>(r.u8());
    revision = r.u64();
    pid = r.u32();
    const uint64_t n = r.u64();
    if (!r.plausible_count(n, 8 + 8 + 1 + 4 + 8 + 8 + 64)) return false;
    entries.resize(n);
    for (auto &e : entries) {
        e.key = r.str();
        e.size_bytes = r.u64();
        e.mode = r.u8();
        e.device = static_cast<int32_t>(r.u32());
        e.offset = r.u64();
        e.raw_ptr = r.u64();
        r.bytes(e.handle, sizeof(e.handle));
        if (e.mode == 2) {
            e.seg_bytes = r.u64();
            const uint32_t m = r.u32();
            if (!r.plausible_count(m, 64)) return false;
            e.more_handles.resize(m);
            for (auto &h : e.more_handles) r.bytes(h.data(), h.size());
        }
    }
    return r.ok();
}

} // namespace pccl::proto
