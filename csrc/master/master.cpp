#include "master.hpp"

#include <algorithm>
#include <functional>
#include <future>
#include <sstream>

#include "../common/log.hpp"

namespace pccl::master {

using namespace proto;

Master::Master(const SockAddr &listen_addr) : server_(listen_addr, false) {
    peer_timeout_ms_ = static_cast<uint32_t>(env_size("PCCL_PEER_TIMEOUT_MS", 10000));
    if (peer_timeout_ms_ > 0) {
        heartbeat_ms_ = static_cast<uint32_t>(std::max<size_t>(20, env_size("PCCL_HEARTBEAT_MS", peer_timeout_ms_ / 5)));
        op_stall_ms_ = static_cast<uint32_t>(env_size("PCCL_OP_STALL_MS", peer_timeout_ms_ + peer_timeout_ms_ / 2));
    } else {
        op_stall_ms_ = static_cast<uint32_t>(env_size("PCCL_OP_STALL_MS", 15000));
    }
    stall_window_ms_ = static_cast<uint32_t>(env_size("PCCL_STALL_WINDOW_MS", std::min<uint32_t>(1000, op_stall_ms_ / 4)));
    vote_timeout_ms_ = static_cast<uint32_t>(env_size("PCCL_VOTE_TIMEOUT_MS", 0));
    server_.on_read([this](const SockAddr &a, uint16_t id, const uint8_t *p, size_t n) { on_packet(a, id, p, n); });
    server_.on_close([this](const SockAddr &a) { on_disconnect(a); });
    server_.on_tick([this] { on_tick(); });
}

Master::~Master() {
    interrupt();
    join();
    stopping_ = true;
    optimizer_pool_.stop();
}

bool Master::launch() {
    if (running_) return false;
    if (!server_.listen()) return false;
    if (!server_.run_async()) return false;
    running_ = true;
    LOG(INFO) << "Master listening on port " << server_.port();
    return true;
}

bool Master::interrupt() {
    server_.interrupt();
    return true;
}

bool Master::join() {
    if (!running_) return false;
    server_.join();
    return true;
}

// ------------------------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------------------------
ClientInfo *Master::client_by_addr(const SockAddr &addr) {
    auto it = by_addr_.find(SockAddrKey::of(addr));
    if (it == by_addr_.end()) return nullptr;
    return client_by_uuid(it->second);
}

ClientInfo *Master::client_by_uuid(const Uuid &u) {
    auto it = clients_.find(u);
    return it == clients_.end() ? nullptr : &it->second;
}

void Master::kick(const SockAddr &addr) {
    LOG(WARN) << "Master: kicking client " << sockaddr_str(addr);
    server_.close_client(addr);
}

void Master::on_peer_accepted(ClientInfo &c) {
    groups_[c.group].bw.register_peer(c.uuid);
    LOG(DEBUG) << "Peer " << c.uuid.str() << " accepted into group " << c.group;
}

uint64_t Master::local_world_size(uint32_t group, bool include_registered) const {
    uint64_t n = 0;
    for (const auto &[_, c] : clients_)
        if (c.group == group && (include_registered || c.phase == Phase::Accepted)) ++n;
    return n;
}

uint64_t Master::num_groups(bool include_registered) const {
    std::set<uint32_t> g;
    for (const auto &[_, c] : clients_)
        if (include_registered || c.phase == Phase::Accepted) g.insert(c.group);
    return g.size();
}

uint64_t Master::largest_group(bool include_registered) const {
    std::map<uint32_t, uint64_t> sizes;
    for (const auto &[_, c] : clients_)
        if (include_registered || c.phase == Phase::Accepted) sizes[c.group]++;
    uint64_t m = 0;
    for (const auto &[_, s] : sizes) m = std::max(m, s);
    return m;
}

// The ring of a group: members are accepted peers plus newcomers currently connecting. Existing members keep their
// relative order (so optimized rings survive churn); new members are appended in UUID order.
std::vector<uint32_t> Master::host_layout(const std::vector<Uuid> &ring) {
    if (ring.size() < 4 || !env_flag("PCCL_HIERARCHICAL", true)) return {};
    std::vector<std::string> hosts;
    std::vector<uint32_t> host_of;
    std::vector<size_t> members;
    for (const auto &u : ring) {
        const ClientInfo *c = client_by_uuid(u);
        if (!c || c->host_token.empty()) return {};
        auto it = std::find(hosts.begin(), hosts.end(), c->host_token);
        if (it == hosts.end()) {
            hosts.push_back(c->host_token);
            members.push_back(0);
            it = hosts.end() - 1;
        }
        const auto h = static_cast<uint32_t>(it - hosts.begin());
        host_of.push_back(h);
        ++members[h];
    }
    if (hosts.size() < 2 || members[0] < 2) return {};
    for (size_t m : members)
        if (m != members[0]) return {};
    return host_of;
}

std::vector<Uuid> Master::ring_of(uint32_t group, bool /*include_registered*/) {
    auto &gs = groups_[group];
    std::set<Uuid> members;
    for (const auto &[u, c] : clients_)
        if (c.group == group && (c.phase == Phase::Accepted || c.state == State::ConnectingToPeers)) members.insert(u);
    std::vector<Uuid> ring;
    for (const auto &u : gs.ring)
        if (members.count(u)) ring.push_back(u);
    for (const auto &u : members)
        if (std::find(ring.begin(), ring.end(), u) == ring.end()) ring.push_back(u);
    if (ring != gs.ring) {
        gs.ring = ring;
        gs.ring_optimal = false;
    }
    return ring;
}

std::optional<std::vector<Uuid>> Master::reachable_ring(uint32_t group) {
    std::vector<Uuid> peers = ring_of(group, true);
    if (peers.empty()) return std::nullopt;
    if (peers.size() <= 1) return peers;
    auto reach = [&](const Uuid &a, const Uuid &b) {
        auto ia = unreachable_.find(a);
        auto ib = unreachable_.find(b);
        const bool ab = ia == unreachable_.end() || !ia->second.count(b);
        const bool ba = ib == unreachable_.end() || !ib->second.count(a);
        return ab && ba;
    };
    const size_t n = peers.size();
    std::vector<Uuid> path{peers[0]};
    std::vector<bool> used(n, false);
    used[0] = true;
    size_t budget = 2000000; // bounded backtracking
    std::function<bool()> bt = [&]() -> bool {
        if (budget-- == 0) return false;
        if (path.size() == n) return reach(path.back(), path.front());
        for (size_t j = 0; j < n; ++j) {
            if (used[j] || !reach(path.back(), peers[j])) continue;
            used[j] = true;
            path.push_back(peers[j]);
            if (bt()) return true;
            path.pop_back();
            used[j] = false;
        }
        return false;
    };
    if (bt()) return path;
    return std::nullopt;
}

void Master::apply_pending_rings() {
    std::lock_guard lock(pending_mtx_);
    for (auto &[group, pr] : pending_rings_) {
        auto &gs = groups_[group];
        // only apply if it is a permutation of the current ring membership
        std::vector<Uuid> cur = gs.ring, cand = pr.first;
        std::sort(cur.begin(), cur.end());
        std::sort(cand.begin(), cand.end());
        if (cur == cand) {
            gs.ring = pr.first;
            gs.ring_optimal = pr.second;
            LOG(INFO) << "Master: applied asynchronously optimized ring for group " << group;
        }
    }
    pending_rings_.clear();
}

void Master::send_connection_info(bool include_registered) {
    for (auto &[u, c] : clients_) {
        if (c.state != State::ConnectingToPeers) continue;
        M2CP2PConnectionInfo info;
        // peers still waiting for admission are not part of the run yet (the reference counts every registered
        // client here, which makes a lone peer with a pending newcomer believe it has company: ops then fail with
        // pcclTooFewPeers forever)
        info.global_world_size = 0;
        for (const auto &[_, o] : clients_)
            if (include_registered || o.phase == Phase::Accepted) ++info.global_world_size;
        info.local_world_size = local_world_size(c.group, include_registered);
        info.num_distinct_peer_groups = num_groups(include_registered);
        info.largest_peer_group_world_size = largest_group(include_registered);
        const auto ring = ring_of(c.group, include_registered);
        c.ring_members = ring;
        std::vector<Uuid> neighbors;
        if (ring.size() > 1) {
            const size_t pos = std::find(ring.begin(), ring.end(), u) - ring.begin();
            if (pos < ring.size()) {
                const Uuid prev = ring[(pos + ring.size() - 1) % ring.size()];
                const Uuid next = ring[(pos + 1) % ring.size()];
                neighbors.push_back(prev);
                if (next != prev) neighbors.push_back(next);
            }
        }
        // hierarchical layout: TX pool to the member with my local rank on the next host, RX pool from the previous
        const auto layout = host_layout(ring);
        const size_t me = std::find(ring.begin(), ring.end(), u) - ring.begin();
        if (!layout.empty() && me < ring.size()) {
            const uint32_t hosts = *std::max_element(layout.begin(), layout.end()) + 1;
            auto local_rank = [&](size_t k) {
                return static_cast<size_t>(std::count(layout.begin(), layout.begin() + static_cast<long>(k), layout[k]));
            };
            const size_t j = local_rank(me);
            for (size_t k = 0; k < ring.size(); ++k) {
                if (k == me || local_rank(k) != j) continue;
                // with two hosts the partner is both the next and the previous host
                const uint8_t role = (layout[k] == (layout[me] + 1) % hosts ? kExtraTx : 0) |
                                     (layout[k] == (layout[me] + hosts - 1) % hosts ? kExtraRx : 0);
                if (!role) continue;
                const ClientInfo *nc = client_by_uuid(ring[k]);
                if (nc) info.extra_peers.push_back(ExtraPeer{PeerInfo{nc->p2p, ring[k]}, role});
            }
        }
        auto &prev = prev_neighbors_[u];
        std::vector<Uuid> a = prev, b = neighbors;
        std::sort(a.begin(), a.end());
        std::sort(b.begin(), b.end());
        const bool changed = a != b;
        prev = neighbors;
        info.unchanged = !changed;
        if (changed)
            for (const auto &nu : neighbors) {
                const ClientInfo *nc = client_by_uuid(nu);
                if (nc) info.all_peers.push_back(PeerInfo{nc->p2p, nu});
            }
        server_.send_packet(c.addr, info);
    }
}

void Master::transition_to_establish(bool accept_new) {
    apply_pending_rings();
    for (auto &[_, c] : clients_) {
        if (!accept_new && c.phase != Phase::Accepted) continue;
        c.state = State::ConnectingToPeers;
    }
    peer_dropped_ = false;
    send_connection_info(accept_new);
}

// ------------------------------------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------------------------------------
template<typename P>
static std::optional<P> parse(const uint8_t *p, size_t n) {
    return decode_payload<P>(p, n);
}

void Master::on_packet(const SockAddr &addr, uint16_t id, const uint8_t *payload, size_t n) {
    auto bad = [&](const char *what) {
        LOG(ERR) << "Master: malformed " << what << " from " << sockaddr_str(addr);
        kick(addr);
    };
    if (ClientInfo *c = client_by_addr(addr)) c->last_seen = std::chrono::steady_clock::now(); // any packet is life
    switch (id) {
        case C2M_HEARTBEAT: return;
        case C2M_OP_STALLED: {
            auto p = parse<C2MOpStalled>(payload, n);
            if (!p) return bad("OpStalled");
            handle_op_stalled(addr, *p);
            return;
        }
        case C2M_REQUEST_SESSION_REGISTRATION: {
            auto p = parse<C2MRequestSessionRegistration>(payload, n);
            if (!p) return bad("RequestSessionRegistration");
            handle_join(addr, *p);
            return;
        }
        case C2M_REQUEST_ESTABLISH_P2P_CONNECTIONS: {
            auto p = parse<C2MRequestEstablishP2PConnections>(payload, n);
            if (!p) return bad("RequestEstablishP2PConnections");
            handle_request_establish(addr, p->accept_new_peers);
            return;
        }
        case C2M_P2P_CONNECTIONS_ESTABLISHED: {
            auto p = parse<C2MP2PConnectionsEstablished>(payload, n);
            if (!p) return bad("P2PConnectionsEstablished");
            handle_p2p_established(addr, *p);
            return;
        }
        case C2M_CHECK_PEERS_PENDING: handle_check_pending(addr); return;
        case C2M_OPTIMIZE_TOPOLOGY: handle_optimize(addr); return;
        case C2M_REPORT_PEER_BANDWIDTH: {
            auto p = parse<C2MReportPeerBandwidth>(payload, n);
            if (!p) return bad("ReportPeerBandwidth");
            handle_report_bw(addr, *p);
            return;
        }
        case C2M_OPTIMIZE_TOPOLOGY_WORK_COMPLETE: handle_optimize_work_complete(addr); return;
        case C2M_SYNC_SHARED_STATE: {
            auto p = parse<C2MSyncSharedState>(payload, n);
            if (!p) return bad("SyncSharedState");
            handle_sync_shared_state(addr, *p);
            return;
        }
        case C2M_DIST_SHARED_STATE_COMPLETE: handle_dist_complete(addr); return;
        case C2M_COLLECTIVE_COMMS_INITIATE: {
            auto p = parse<C2MCollectiveCommsInitiate>(payload, n);
            if (!p) return bad("CollectiveCommsInitiate");
            handle_coll_initiate(addr, *p);
            return;
        }
        case C2M_COLLECTIVE_COMMS_COMPLETE: {
            auto p = parse<C2MCollectiveCommsComplete>(payload, n);
            if (!p) return bad("CollectiveCommsComplete");
            handle_coll_complete(addr, *p);
            return;
        }
        default: LOG(ERR) << "Master: unknown packet id " << id; kick(addr);
    }
}

// ------------------------------------------------------------------------------------------------------------------
// join / establish
// ------------------------------------------------------------------------------------------------------------------
void Master::handle_join(const SockAddr &addr, const C2MRequestSessionRegistration &p) {
    M2CSessionRegistrationResponse resp;
    if (client_by_addr(addr) != nullptr) {
        LOG(WARN) << "Master: " << sockaddr_str(addr) << " already registered";
        kick(addr);
        return;
    }
    // Loopback exclusivity: a run is either entirely on 127.0.0.0/8 (single host) or entirely on routable addresses,
    // because loopback addresses cannot be handed to remote peers (reference ccoip_master_state.cpp:40-67).
    bool ok = true;
    if (!clients_.empty()) {
        bool all_local = true;
        for (const auto &[_, c] : clients_) all_local = all_local && sockaddr_is_loopback(c.addr);
        const bool local = sockaddr_is_loopback(addr);
        if (all_local != local) {
            LOG(WARN) << "Master: rejecting " << sockaddr_str(addr) << " (loopback/non-loopback mix)";
            ok = false;
        }
    }
    if (ok) {
        ClientInfo c;
        c.uuid = Uuid::random();
        c.addr = addr;
        c.group = p.peer_group;
        c.host_token = p.host_token;
        c.xgmi = p.xgmi_capable;
        c.liveness = p.liveness;
        c.last_seen = std::chrono::steady_clock::now();
        if (p.liveness) { // only a peer that announced the extension gets the appended fields
            resp.heartbeat_ms = heartbeat_ms_;
            resp.peer_timeout_ms = peer_timeout_ms_;
            resp.op_stall_ms = op_stall_ms_;
        }
        if (p.use_explicit_addresses) {
            c.p2p = p.advertised_p2p;
            c.ss = p.advertised_ss;
            c.bm = p.advertised_bm;
        } else {
            c.p2p = c.ss = c.bm = addr;
            c.p2p.port = p.p2p_port;
            c.ss.port = p.ss_port;
            c.bm.port = p.bm_port;
        }
        resp.accepted = true;
        resp.assigned_uuid = c.uuid;
        by_addr_[SockAddrKey::of(addr)] = c.uuid;
        clients_[c.uuid] = c;
        LOG(INFO) << "Master: registered " << sockaddr_str(addr) << " as " << c.uuid.str() << " (group " << c.group << ")";
    }
    server_.send_packet(addr, resp);
    if (!ok) return;
    if (clients_.size() == 1) {
        // The first peer is accepted immediately and establishes its (empty) ring alone.
        ClientInfo &c = clients_.begin()->second;
        c.phase = Phase::Accepted;
        on_peer_accepted(c);
        transition_to_establish(true);
    } else {
        check_establish_consensus();
    }
}

void Master::handle_request_establish(const SockAddr &addr, bool accept_new) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->phase != Phase::Accepted ||
        (c->state != State::Idle && c->state != State::ConnectingToPeersFailed)) {
        LOG(WARN) << "Master: illegal establish vote from " << sockaddr_str(addr);
        kick(addr);
        return;
    }
    c->state = accept_new ? State::VoteAcceptNewPeers : State::VoteNoNewPeersEstablishP2P;
    check_establish_consensus();
}

void Master::check_establish_consensus() {
    if (clients_.empty()) return;
    size_t accept_votes = 0, nonew_votes = 0, registered = 0, accepted = 0;
    for (const auto &[_, c] : clients_) {
        if (c.phase == Phase::Registered) {
            ++registered;
            continue;
        }
        ++accepted;
        if (c.state == State::VoteAcceptNewPeers) ++accept_votes;
        if (c.state == State::VoteNoNewPeersEstablishP2P) ++nonew_votes;
    }
    if (accepted == 0 || accept_votes + nonew_votes != accepted) return;
    // all accepted peers voted. Registered peers count as implicit "yes" for accepting new peers.
    const bool accept_new = nonew_votes == 0;
    LOG(DEBUG) << "Master: establish consensus (accept_new=" << accept_new << ")";
    transition_to_establish(accept_new);
}

void Master::handle_p2p_established(const SockAddr &addr, const C2MP2PConnectionsEstablished &p) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->state != State::ConnectingToPeers) {
        LOG(WARN) << "Master: unexpected P2PConnectionsEstablished from " << sockaddr_str(addr);
        kick(addr);
        return;
    }
    if (!p.success) {
        auto &un = unreachable_[c->uuid];
        for (const auto &f : p.failed_peers)
            if (client_by_uuid(f)) un.insert(f);
        if (un.size() + 1 >= clients_.size() && clients_.size() > 1) {
            LOG(WARN) << "Master: peer " << c->uuid.str() << " cannot reach any other peer; kicking";
            kick(addr);
            return;
        }
        auto ring = reachable_ring(c->group);
        if (!ring) {
            LOG(WARN) << "Master: no reachable ring exists with peer " << c->uuid.str() << "; kicking";
            kick(addr);
            return;
        }
        groups_[c->group].ring = *ring;
        groups_[c->group].ring_optimal = false;
        c->state = State::ConnectingToPeersFailed;
    } else {
        c->state = State::WaitingForOtherPeers;
    }
    check_p2p_established();
}

bool Master::check_p2p_established() {
    size_t voting = 0, connecting = 0;
    bool any_failed = false;
    for (const auto &[_, c] : clients_) {
        const bool v = c.state == State::WaitingForOtherPeers || c.state == State::ConnectingToPeersFailed;
        if (v) ++voting;
        if (v || c.state == State::ConnectingToPeers) ++connecting;
        if (c.state == State::ConnectingToPeersFailed) any_failed = true;
    }
    if (voting == 0 || voting != connecting) return false;
    const bool failure = any_failed || peer_dropped_;
    for (auto &[_, c] : clients_) {
        if (c.phase == Phase::Registered && c.state == State::Idle) continue; // did not make the cut
        if (failure) {
            if (c.state == State::WaitingForOtherPeers) c.state = State::ConnectingToPeersFailed;
        } else {
            if (c.state == State::WaitingForOtherPeers) c.state = State::Idle;
        }
        if (c.phase == Phase::Registered &&
            (c.state == State::Idle || c.state == State::ConnectingToPeersFailed)) {
            c.phase = Phase::Accepted;
            on_peer_accepted(c);
        }
    }
    for (auto &[u, c] : clients_) {
        if (c.phase == Phase::Registered && c.state == State::Idle) continue;
        if (c.state != State::Idle && c.state != State::ConnectingToPeersFailed) continue;
        M2CP2PConnectionsEstablished pkt;
        pkt.success = !failure;
        pkt.ring_order = ring_of(c.group, false);
        // every ring member on one host (same boot id + hostname): the peers may rendezvous for the xGMI IPC path
        // even if the master itself is remote
        pkt.has_host_info = true; // our clients read single_host / host_of (reference clients ignore trailing bytes)
        pkt.single_host = !pkt.ring_order.empty();
        for (const auto &ru : pkt.ring_order) {
            const ClientInfo *rc = client_by_uuid(ru);
            pkt.single_host = pkt.single_host && rc && !rc->host_token.empty() && rc->host_token == c.host_token;
        }
        pkt.host_of = host_layout(pkt.ring_order);
        server_.send_packet(c.addr, pkt);
    }
    if (failure) {
        // the next round must resend full neighbour lists (connections may be stale)
        prev_neighbors_.clear();
    }
    peer_dropped_ = false;
    return true;
}

// ------------------------------------------------------------------------------------------------------------------
// peers pending
// ------------------------------------------------------------------------------------------------------------------
void Master::handle_check_pending(const SockAddr &addr) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->phase != Phase::Accepted || c->voted_pending_query) {
        kick(addr);
        return;
    }
    c->voted_pending_query = true;
    check_pending_query_consensus();
}

void Master::check_pending_query_consensus() {
    bool any = false;
    for (const auto &[_, c] : clients_) {
        if (c.phase != Phase::Accepted) continue;
        any = true;
        if (!c.voted_pending_query) return;
    }
    if (!any) return;
    bool pending = false;
    for (const auto &[_, c] : clients_) pending = pending || c.phase == Phase::Registered;
    M2CPeersPendingResponse r;
    r.peers_pending = pending;
    for (auto &[_, c] : clients_) {
        if (c.phase != Phase::Accepted) continue;
        server_.send_packet(c.addr, r);
        c.voted_pending_query = false;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// topology optimization
// ------------------------------------------------------------------------------------------------------------------
void Master::handle_optimize(const SockAddr &addr) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->phase != Phase::Accepted ||
        (c->state != State::Idle && c->state != State::OptimizeTopologyFailed)) {
        kick(addr);
        return;
    }
    c->state = State::VoteOptimizeTopology;
    check_optimize_consensus();
}

double Master::same_host_mbps() { // ~xGMI link class; read per round (tests switch it)
    return static_cast<double>(env_size("PCCL_SAME_HOST_MBPS", 1000000));
}

void Master::check_optimize_consensus() {
    for (const auto &[_, c] : clients_)
        if (c.phase == Phase::Accepted && c.state != State::VoteOptimizeTopology) return;
    bool any = false;
    for (auto &[_, c] : clients_)
        if (c.phase == Phase::Accepted) {
            c.state = State::OptimizeTopology;
            any = true;
        }
    if (!any) return;
    // Each sender's probes in round-robin tournament order: the i-th peer (uuid order, per group) measures peer
    // i + 1, i + 2, ... in turn, so in every round each peer sends to one peer and receives from one, instead of all of
    // them queueing at the same first target (whose benchmark server takes one probe at a time).
    std::map<uint32_t, std::vector<Uuid>> members;
    for (const auto &[u, c] : clients_)
        if (c.phase == Phase::Accepted) members[c.group].push_back(u);
    auto index_in = [&](uint32_t group, const Uuid &u) -> size_t {
        const auto &m = members[group];
        return static_cast<size_t>(std::find(m.begin(), m.end(), u) - m.begin());
    };
    for (auto &[u, c] : clients_) {
        if (c.phase != Phase::Accepted) continue;
        M2COptimizeTopologyResponse resp;
        for (const auto &e : groups_[c.group].bw.missing_for(u)) {
            if (e.from != u) continue;
            auto un = unreachable_.find(e.from);
            if (un != unreachable_.end() && un->second.count(e.to)) continue;
            const ClientInfo *to = client_by_uuid(e.to);
            if (!to || to->phase != Phase::Accepted) continue;
            if (same_host_mbps() > 0 && !c.host_token.empty() && c.host_token == to->host_token && c.xgmi && to->xgmi) {
                // same host (boot id + hostname) and both peers can take the xGMI path: the pair never talks over
                // the NIC, so it is not benchmarked (reference benchmarks every pair for 10 s); a fixed, NIC-beating
                // cost makes the ATSP keep co-located peers adjacent (PCCL_SAME_HOST_MBPS, 0 = measure as usual).
                // Same-host pairs that use loopback TCP (PCCL_DISABLE_IPC, no GPU backend) are measured below.
                groups_[c.group].bw.store(u, e.to, same_host_mbps());
                continue;
            }
            resp.requests.push_back(BenchmarkRequest{u, e.to, to->bm});
        }
        const size_t n = std::max<size_t>(1, members[c.group].size()), me = index_in(c.group, u);
        std::stable_sort(resp.requests.begin(), resp.requests.end(), [&](const BenchmarkRequest &a, const BenchmarkRequest &b) {
            return (index_in(c.group, a.to_peer) + n - me) % n < (index_in(c.group, b.to_peer) + n - me) % n;
        });
        server_.send_packet(c.addr, resp);
    }
}

void Master::handle_report_bw(const SockAddr &addr, const C2MReportPeerBandwidth &p) {
    ClientInfo *c = client_by_addr(addr);
    if (!c) {
        kick(addr);
        return;
    }
    const ClientInfo *to = client_by_uuid(p.to_peer);
    if (!to || to->group != c->group) return;
    groups_[c->group].bw.store(c->uuid, p.to_peer, p.bandwidth_mbps);
}

void Master::handle_optimize_work_complete(const SockAddr &addr) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->phase != Phase::Accepted || c->state != State::OptimizeTopology) {
        kick(addr);
        return;
    }
    c->state = State::VoteCompleteTopologyOptimization;
    check_optimize_complete_consensus();
}

void Master::run_topology_optimization(uint32_t group) {
    auto &gs = groups_[group];
    std::vector<Uuid> ring = ring_of(group, false);
    if (ring.size() < 3) {
        gs.ring_optimal = true; // 1 or 2 peers: every ring is optimal
        return;
    }
    if (!gs.optimized_once) {
        bool optimal = false, improved = false;
        const auto t0 = std::chrono::steady_clock::now();
        if (optimize_ring(gs.bw, ring, false, optimal, improved)) {
            if (improved) {
                gs.ring = ring;
                topo_changes_.fetch_add(1);
            }
            gs.ring_optimal = optimal;
        }
        topo_last_us_.store(static_cast<uint64_t>(
            std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count()));
        topo_solves_.fetch_add(1);
        gs.optimized_once = true;
        return;
    }
    // moonshot: asynchronous wider search; result applied at the next establishment round
    // one moonshot per group at a time on the bounded pool (4 threads, 64 queued; reference master handler:13-14)
    BandwidthStore snapshot = gs.bw;
    const bool queued = optimizer_pool_.submit(group, [this, group, ring, snapshot]() mutable {
        if (stopping_) return;
        bool optimal = false, improved = false;
        if (optimize_ring(snapshot, ring, true, optimal, improved, &stopping_) && improved && !stopping_) {
            std::lock_guard lock(pending_mtx_);
            pending_rings_[group] = {ring, optimal};
            topo_changes_.fetch_add(1);
        }
        topo_moonshots_.fetch_add(1);
    });
    if (!queued) {
        LOG(DEBUG) << "moonshot topology optimization of group " << group << " already running / queue full";
    }
}

void Master::check_optimize_complete_consensus() {
    for (const auto &[_, c] : clients_)
        if (c.phase == Phase::Accepted && c.state != State::VoteCompleteTopologyOptimization) return;
    // Edges still unmeasured are considered unreachable so that later rounds do not retry timing-out benchmarks.
    for (const auto &[u, c] : clients_) {
        if (c.phase != Phase::Accepted) continue;
        for (const auto &e : groups_[c.group].bw.missing_for(u)) unreachable_[e.from].insert(e.to);
    }
    std::set<uint32_t> touched;
    for (auto &[_, c] : clients_)
        if (c.phase == Phase::Accepted) {
            c.state = State::Idle;
            touched.insert(c.group);
        }
    for (uint32_t g : touched)
        if (!groups_[g].ring_optimal) run_topology_optimization(g);
    for (auto &[_, c] : clients_) {
        if (c.phase != Phase::Accepted) continue;
        M2COptimizeTopologyComplete pkt;
        pkt.success = true;
        pkt.ring_order = ring_of(c.group, false);
        server_.send_packet(c.addr, pkt);
    }
}

// ------------------------------------------------------------------------------------------------------------------
// shared state
// ------------------------------------------------------------------------------------------------------------------
SSStatus Master::revision_status(ClientInfo &c, uint64_t revision) {
    auto &gs = groups_[c.group];
    SSStatus st = SSStatus::Match;
    if (gs.next_revision != 0) {
        if (revision < gs.next_revision) st = SSStatus::RevisionOutdated;
        else if (revision > gs.next_revision) st = SSStatus::RevisionIncrementViolation;
    } else if (revision > 0) {
        gs.next_revision = revision; // resume: adopt the first non-zero revision
        // Peers of this round that voted before with an older revision (e.g. a fresh peer at 0 ahead of a resuming
        // one) are outdated, not matching: they receive the state instead of competing for the election by
        // popularity (the reference keeps their early "match", so a 1:1 tie could hand the fresh state to the
        // resuming peer)
        for (auto &[u, prev] : gs.statuses) {
            const ClientInfo *o = client_by_uuid(u);
            if (o && o->state == State::VoteSyncSharedState && o->ss_revision < revision && prev == SSStatus::Match)
                prev = SSStatus::RevisionOutdated;
        }
    }
    gs.statuses[c.uuid] = st;
    c.ss_revision = revision;
    return st;
}

void Master::handle_sync_shared_state(const SockAddr &addr, const C2MSyncSharedState &p) {
    ClientInfo *c = client_by_addr(addr);
    if (!c) {
        kick(addr);
        return;
    }
    const SSStatus st = revision_status(*c, p.revision);
    if (st == SSStatus::RevisionIncrementViolation) {
        LOG(WARN) << "Master: revision increment violation by " << c->uuid.str() << " (revision " << p.revision << ")";
        kick(addr);
        return;
    }
    if (c->phase != Phase::Accepted || c->state != State::Idle) {
        LOG(WARN) << "Master: illegal shared state sync vote from " << sockaddr_str(addr);
        kick(addr);
        return;
    }
    auto &gs = groups_[c->group];
    c->state = State::VoteSyncSharedState;
    gs.strategies[c->uuid] = p.strategy;
    if (p.strategy != SyncStrategy::RxOnly) gs.candidates.emplace_back(c->uuid, p.entries);
    gs.entries.emplace_back(c->uuid, p.entries);
    const uint32_t group = c->group;
    if (!check_sync_consensus(group)) {
        // nothing can be distributed (e.g. every peer is RECEIVE_ONLY): the round cannot complete
        LOG(WARN) << "Master: shared state sync of group " << group << " cannot proceed; kicking the group";
        for (auto &[_, o] : clients_)
            if (o.group == group && o.phase == Phase::Accepted) kick(o.addr);
    }
}

bool Master::elect_mask(uint32_t group) {
    auto &gs = groups_[group];
    struct Cand {
        const std::vector<SharedStateHashEntry> *entries;
        size_t votes = 0;
        int priority = -1000;
        size_t first = 0;
    };
    std::vector<Cand> cands;
    // SEND_ONLY peers declare their state to be the correct one: if any voted, only they are electable (documented
    // semantics of PCCL_SHARED_STATE_SYNC_STRATEGY_SEND_ONLY; the reference elects purely by popularity).
    bool any_tx_only = false;
    for (const auto &[u, _] : gs.candidates) any_tx_only = any_tx_only || gs.strategies[u] == SyncStrategy::TxOnly;
    for (size_t i = 0; i < gs.candidates.size(); ++i) {
        const auto &[u, entries] = gs.candidates[i];
        if (any_tx_only && gs.strategies[u] != SyncStrategy::TxOnly) continue;
        int prio = -1;
        auto st = gs.statuses.find(u);
        if (st != gs.statuses.end()) prio = st->second == SSStatus::Match ? 1 : st->second == SSStatus::RevisionOutdated ? -2 : -1;
        auto it = std::find_if(cands.begin(), cands.end(), [&](const Cand &c) { return *c.entries == entries; });
        if (it == cands.end()) {
            cands.push_back(Cand{&entries, 0, prio, i});
            it = cands.end() - 1;
        }
        it->votes++;
        it->priority = std::max(it->priority, prio);
    }
    if (cands.empty()) return false;
    int best_prio = -1000;
    for (const auto &c : cands) best_prio = std::max(best_prio, c.priority);
    const Cand *win = nullptr;
    for (const auto &c : cands) {
        if (c.priority != best_prio) continue;
        if (!win || c.votes > win->votes) win = &c; // ties: earliest voter wins (deterministic)
    }
    gs.mask = *win->entries;
    return true;
}

void Master::compute_mismatches(uint32_t group) {
    auto &gs = groups_[group];
    gs.dirty_keys.clear();
    for (const auto &[u, entries] : gs.entries) {
        SSStatus &status = gs.statuses[u];
        if (status != SSStatus::Match && status != SSStatus::RevisionOutdated) continue;
        SSStatus st = SSStatus::Match;
        if (entries.size() != gs.mask.size()) st = SSStatus::KeySetMismatch;
        for (size_t i = 0; st != SSStatus::KeySetMismatch && i < gs.mask.size(); ++i) {
            const auto &m = gs.mask[i];
            const auto &e = entries[i];
            if (m.key != e.key || m.allow_content_inequality != e.allow_content_inequality ||
                m.data_type != e.data_type || m.hash_type != e.hash_type ||
                (m.num_elements != e.num_elements && m.num_elements != 0 && e.num_elements != 0)) {
                LOG(WARN) << "Master: shared state key set mismatch for " << u.str() << " at key " << m.key;
                st = SSStatus::KeySetMismatch;
                break;
            }
            if (m.hash != e.hash) {
                st = SSStatus::ContentHashMismatch;
                gs.hashes[m.key] = m.hash;
                gs.hash_types[m.key] = m.hash_type;
                gs.dirty_keys[u].push_back(m.key);
            }
        }
        if (status == SSStatus::Match || st == SSStatus::KeySetMismatch) status = st;
    }
}

bool Master::check_sync_consensus(uint32_t group) {
    bool any_voting = false;
    for (const auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        if (c.state == State::VoteSyncSharedState) any_voting = true;
        else return true; // not everyone voted yet (not an error)
    }
    if (!any_voting) return true;
    auto &gs = groups_[group];

    // Re-baseline if nobody holds the expected revision any more (all holders died).
    bool any_match = false;
    for (const auto &[u, st] : gs.statuses) any_match = any_match || st == SSStatus::Match;
    if (!any_match && !gs.statuses.empty()) {
        uint64_t maxrev = 0;
        for (const auto &[_, c] : clients_)
            if (c.group == group && c.phase == Phase::Accepted) maxrev = std::max(maxrev, c.ss_revision);
        LOG(WARN) << "Master: no peer of group " << group << " holds revision " << gs.next_revision
                  << "; re-baselining at " << maxrev;
        gs.next_revision = maxrev;
        for (auto &[u, st] : gs.statuses) {
            const ClientInfo *c = client_by_uuid(u);
            st = (c && c->ss_revision == maxrev) ? SSStatus::Match : SSStatus::RevisionOutdated;
        }
    }

    if (!elect_mask(group)) return false;
    compute_mismatches(group);
    for (auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        if (gs.statuses[c.uuid] == SSStatus::KeySetMismatch) {
            kick(c.addr);
            return true; // disconnect handling re-evaluates the round
        }
    }
    // transition: matching peers distribute, the rest request
    for (auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        c.state = gs.statuses[c.uuid] == SSStatus::Match ? State::DistributeSharedState : State::RequestSharedState;
    }
    gs.next_revision++;
    bool any_enforce = false, any_other = false;
    for (auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        const SyncStrategy s = gs.strategies[c.uuid];
        if (c.state == State::RequestSharedState && s == SyncStrategy::TxOnly) {
            LOG(WARN) << "Master: SEND_ONLY peer " << c.uuid.str() << " does not hold the popular state; kicking";
            kick(c.addr);
        }
        any_enforce = any_enforce || s == SyncStrategy::EnforcePopular;
        any_other = any_other || s != SyncStrategy::EnforcePopular;
    }
    if (any_enforce && any_other) {
        for (auto &[_, c] : clients_) {
            if (c.group != group || c.phase != Phase::Accepted) continue;
            if (gs.strategies[c.uuid] != SyncStrategy::EnforcePopular) {
                LOG(WARN) << "Master: mixed sync strategies; kicking non-ENFORCE_POPULAR peer " << c.uuid.str();
                kick(c.addr);
            }
        }
    }
    std::vector<const ClientInfo *> distributors;
    for (const auto &[_, c] : clients_)
        if (c.group == group && c.phase == Phase::Accepted && c.state == State::DistributeSharedState)
            distributors.push_back(&c);
    for (auto &[u, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        M2CSyncSharedState resp;
        resp.is_outdated = c.state == State::RequestSharedState;
        if (resp.is_outdated) {
            if (!distributors.empty()) {
                const size_t first = dist_rr_++ % distributors.size();
                resp.distributor = distributors[first]->ss;
                for (size_t k = 1; k < distributors.size(); ++k)
                    resp.fallback_distributors.push_back(distributors[(first + k) % distributors.size()]->ss);
            } else {
                LOG(ERR) << "Master: no shared state distributor for " << u.str();
            }
            resp.outdated_keys = gs.dirty_keys[u];
            for (const auto &k : resp.outdated_keys) {
                resp.expected_hashes.push_back(gs.hashes[k]);
                resp.expected_hash_types.push_back(gs.hash_types[k]);
            }
        }
        server_.send_packet(c.addr, resp);
    }
    return true;
}

void Master::handle_dist_complete(const SockAddr &addr) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->phase != Phase::Accepted ||
        (c->state != State::DistributeSharedState && c->state != State::RequestSharedState)) {
        kick(addr);
        return;
    }
    c->state = State::VoteCompleteSharedStateSync;
    check_sync_complete_consensus(c->group);
}

void Master::end_sync_phase(uint32_t group) {
    auto &gs = groups_[group];
    for (auto &[_, c] : clients_)
        if (c.group == group && c.phase == Phase::Accepted && c.state == State::VoteCompleteSharedStateSync)
            c.state = State::Idle;
    gs.candidates.clear();
    gs.entries.clear();
    gs.mask.clear();
    gs.statuses.clear();
    gs.hashes.clear();
    gs.hash_types.clear();
    gs.dirty_keys.clear();
    gs.strategies.clear();
}

void Master::check_sync_complete_consensus(uint32_t group) {
    bool any = false;
    for (const auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        if (c.state != State::VoteCompleteSharedStateSync) return;
        any = true;
    }
    if (!any) return;
    end_sync_phase(group);
    for (auto &[_, c] : clients_)
        if (c.group == group && c.phase == Phase::Accepted) server_.send_packet(c.addr, M2CSyncSharedStateComplete{});
}

// ------------------------------------------------------------------------------------------------------------------
// collectives
// ------------------------------------------------------------------------------------------------------------------
void Master::handle_coll_initiate(const SockAddr &addr, const C2MCollectiveCommsInitiate &p) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->phase != Phase::Accepted ||
        (c->state != State::Idle && c->state != State::CollectiveCommsRunning) || c->colls.count(p.tag)) {
        LOG(WARN) << "Master: illegal collective initiate (tag " << p.tag << ") from " << sockaddr_str(addr);
        kick(addr);
        return;
    }
    c->state = State::CollectiveCommsRunning;
    c->colls[p.tag] = CollState::VoteInitiate;
    c->coll_flags[p.tag] = p.flags;
    c->coll_shapes[p.tag] = p.shape;
    check_coll_initiate_consensus(c->group, p.tag);
}

void Master::check_coll_initiate_consensus(uint32_t group, uint64_t tag) {
    bool any = false;
    for (const auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        auto it = c.colls.find(tag);
        if (it == c.colls.end() || it->second != CollState::VoteInitiate) return;
        any = true;
    }
    if (!any) return;
    const uint64_t seq = next_seq_++;
    M2CCollectiveCommsCommence pkt;
    pkt.tag = tag;
    pkt.seq_nr = seq;
    pkt.flags = 0xff; // a capability holds for the op only if every participant announced it
    // one data-plane shape for every participant: fewest stripes and lanes, largest stripe minimum of the proposals
    pkt.shape.stripes = 16;
    pkt.shape.quant_lanes = 4;
    pkt.shape.stripe_min_kib = 256;
    pkt.shape.segment_chunk_mib = 0;
    bool seg_any = false;
    for (auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        auto f = c.coll_flags.find(tag);
        pkt.flags &= f == c.coll_flags.end() ? 0 : f->second;
        auto sh = c.coll_shapes.find(tag);
        if (sh == c.coll_shapes.end()) continue;
        pkt.shape.stripes = std::min(pkt.shape.stripes, sh->second.stripes);
        pkt.shape.quant_lanes = std::min(pkt.shape.quant_lanes, sh->second.quant_lanes);
        pkt.shape.stripe_min_kib = std::max(pkt.shape.stripe_min_kib, sh->second.stripe_min_kib);
        // smallest non-zero segment (0 = unsegmented only if every proposal says so)
        const uint16_t sg = sh->second.segment_chunk_mib;
        if (sg != 0 && (!seg_any || sg < pkt.shape.segment_chunk_mib)) {
            pkt.shape.segment_chunk_mib = sg;
            seg_any = true;
        }
    }
    bool stale = false;
    for (auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        c.colls[tag] = CollState::Perform;
        server_.send_packet(c.addr, pkt);
        for (const Uuid &m : c.ring_members)
            if (!clients_.count(m)) stale = true;
    }
    // A participant's ring still holds a peer that has left (dropped by the liveness protocol while the others were
    // between ops: no op of theirs was running to abort, and a stopped peer's connections stay open). The op would wait
    // on that peer until the stall watchdog fires; it is aborted right away instead, and the peers re-establish.
    if (stale) {
        LOG(WARN) << "Master: op tag " << tag << " commenced on a ring with a departed peer; aborting it";
        groups_[group].aborted[tag] = true;
        send_abort(group, tag, true);
    }
}

void Master::send_abort(uint32_t group, uint64_t tag, bool aborted) {
    M2CCollectiveCommsAbort pkt;
    pkt.tag = tag;
    pkt.aborted = aborted;
    for (auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted || c.state != State::CollectiveCommsRunning) continue;
        if (!c.colls.count(tag)) continue;
        server_.send_packet(c.addr, pkt);
    }
}

void Master::handle_coll_complete(const SockAddr &addr, const C2MCollectiveCommsComplete &p) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->phase != Phase::Accepted) {
        kick(addr);
        return;
    }
    auto it = c->colls.find(p.tag);
    if (it == c->colls.end() || it->second != CollState::Perform) {
        LOG(WARN) << "Master: illegal collective complete (tag " << p.tag << ") from " << sockaddr_str(addr);
        kick(addr);
        return;
    }
    it->second = CollState::VoteComplete;
    const uint32_t group = c->group;
    if (p.was_aborted) {
        auto &ab = groups_[group].aborted[p.tag];
        if (!ab) {
            ab = true;
            send_abort(group, p.tag, true); // first abort report: tell everyone (exactly one abort packet each)
        }
    }
    check_coll_complete_consensus(group, p.tag);
}

void Master::check_coll_complete_consensus(uint32_t group, uint64_t tag) {
    bool any = false;
    for (const auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        auto it = c.colls.find(tag);
        if (it == c.colls.end() || it->second != CollState::VoteComplete) return;
        any = true;
    }
    if (!any) return;
    auto &gs = groups_[group];
    if (!gs.aborted[tag]) send_abort(group, tag, false);
    gs.aborted.erase(tag);
    M2CCollectiveCommsComplete pkt;
    pkt.tag = tag;
    for (auto &[_, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        c.colls.erase(tag);
        c.coll_flags.erase(tag);
        c.coll_shapes.erase(tag);
        if (c.colls.empty()) c.state = State::Idle;
        server_.send_packet(c.addr, pkt);
    }
}

// ------------------------------------------------------------------------------------------------------------------
// disconnect
// ------------------------------------------------------------------------------------------------------------------
void Master::on_disconnect(const SockAddr &addr) {
    auto ait = by_addr_.find(SockAddrKey::of(addr));
    if (ait == by_addr_.end()) return;
    const Uuid u = ait->second;
    by_addr_.erase(ait);
    auto cit = clients_.find(u);
    if (cit == clients_.end()) return;
    const ClientInfo info = cit->second;
    clients_.erase(cit);
    auto &gs = groups_[info.group];
    if (info.phase == Phase::Accepted) gs.bw.unregister_peer(u);
    gs.candidates.erase(std::remove_if(gs.candidates.begin(), gs.candidates.end(), [&](auto &e) { return e.first == u; }),
                        gs.candidates.end());
    gs.entries.erase(std::remove_if(gs.entries.begin(), gs.entries.end(), [&](auto &e) { return e.first == u; }),
                     gs.entries.end());
    gs.statuses.erase(u);
    gs.strategies.erase(u);
    gs.dirty_keys.erase(u);
    unreachable_.erase(u);
    for (auto &[_, s] : unreachable_) s.erase(u);
    prev_neighbors_.erase(u);
    LOG(INFO) << "Master: peer " << u.str() << " (" << sockaddr_str(addr) << ") left; " << clients_.size() << " remain";

    check_establish_consensus();
    peer_dropped_ = true; // an establishment round in flight must fail and be retried with fresh neighbour lists
    check_p2p_established();
    check_pending_query_consensus();
    if (!check_sync_consensus(info.group)) {
        for (auto &[_, o] : clients_)
            if (o.group == info.group && o.phase == Phase::Accepted) kick(o.addr);
    }
    check_sync_complete_consensus(info.group);
    check_optimize_consensus();
    check_optimize_complete_consensus();

    std::set<uint64_t> tags;
    for (const auto &[_, c] : clients_)
        if (c.group == info.group)
            for (const auto &[t, _s] : c.colls) tags.insert(t);
    for (uint64_t tag : tags) {
        // a running op lost a participant: abort it (once) before completing any consensus
        bool running = false;
        for (const auto &[_, c] : clients_) {
            if (c.group != info.group) continue;
            auto it = c.colls.find(tag);
            if (it != c.colls.end() && it->second == CollState::Perform) running = true;
        }
        if (running && info.colls.count(tag)) {
            auto &ab = gs.aborted[tag];
            if (!ab) {
                ab = true;
                send_abort(info.group, tag, true);
            }
        }
        check_coll_initiate_consensus(info.group, tag);
        check_coll_complete_consensus(info.group, tag);
    }
    maybe_bootstrap_orphans();
}

// PCCL_MASTER_DUMP_SEC=N: log the full consensus state every N seconds (diagnosing stuck runs)
void Master::on_tick() {
    check_liveness(std::chrono::steady_clock::now());
    static const size_t every = env_size("PCCL_MASTER_DUMP_SEC", 0);
    if (every == 0) return;
    const auto now = std::chrono::steady_clock::now();
    if (now - last_dump_ < std::chrono::seconds(every)) return;
    last_dump_ = now;
    LOG(WARN) << "Master state:\n" << dump_state();
}

// ------------------------------------------------------------------------------------------------------------------
// liveness: heartbeats, stalled ops, vote timeouts
//
// The reference detects failures only by TCP close / RST and SO_KEEPALIVE (tinysockets multiplexed_socket.cpp:29-49,
// server_socket.cpp). Neither fires for a peer that stops without closing its sockets (SIGSTOP, a wedged driver
// call, a swapped-out host, a black-holed path): its kernel keeps ACKing, and keepalive never probes while data is
// outstanding. Such a peer used to hang its whole group forever. Three bounded detectors act through the existing
// disconnect path (unregister, abort the running tags, re-form the ring):
//  * heartbeats: a liveness peer silent for PCCL_PEER_TIMEOUT_MS is dropped (the master sends M2CHeartbeat too, so
//    peers detect a lost master);
//  * stalled ops: peers report an op whose TCP data path made no progress (C2MOpStalled); the master collects the
//    reports of the op for PCCL_STALL_WINDOW_MS, or until every performing participant reported, and drops the
//    peer the evidence names;
//  * vote timeout (PCCL_VOTE_TIMEOUT_MS, off by default: a slow peer cannot be told from a hung one): an idle peer
//    that has not joined a consensus every other waiter of its group has waited in for that long is dropped.
// ------------------------------------------------------------------------------------------------------------------
void Master::check_liveness(std::chrono::steady_clock::time_point now) {
    using std::chrono::milliseconds;
    if (peer_timeout_ms_ > 0) {
        if (now - last_heartbeat_ >= milliseconds(heartbeat_ms_)) {
            last_heartbeat_ = now;
            for (const auto &[_, c] : clients_)
                if (c.liveness) server_.send_packet(c.addr, M2CHeartbeat{});
        }
        std::vector<SockAddr> silent;
        for (const auto &[u, c] : clients_)
            if (c.liveness && now - c.last_seen > milliseconds(peer_timeout_ms_)) silent.push_back(c.addr);
        for (const auto &a : silent) {
            const ClientInfo *c = client_by_addr(a);
            LOG(WARN) << "Master: peer " << (c ? c->uuid.str() : std::string("?")) << " (" << sockaddr_str(a)
                      << ") silent for more than " << peer_timeout_ms_ << " ms; dropping it";
            live_silent_++;
            kick(a);
        }
    }
    std::vector<std::pair<uint32_t, uint64_t>> keys;
    for (const auto &[k, _] : stalls_) keys.push_back(k);
    for (const auto &k : keys) decide_stall(k.first, k.second, now);
    if (vote_timeout_ms_ > 0) check_vote_timeouts(now);
}

void Master::handle_op_stalled(const SockAddr &addr, const C2MOpStalled &p) {
    ClientInfo *c = client_by_addr(addr);
    if (!c || c->phase != Phase::Accepted) return;
    live_reports_++;
    auto it = c->colls.find(p.tag);
    if (it == c->colls.end() || it->second != CollState::Perform) return; // the op ended meanwhile
    auto &v = stalls_[{c->group, p.tag}];
    for (const auto &r : v)
        if (r.reporter == c->uuid) return;
    LOG(WARN) << "Master: op tag " << p.tag << " stalled at " << c->uuid.str() << " (step " << p.step << ", "
              << (p.kind == kStallTxBlocked ? "send blocked to " : "nothing from ") << p.suspect.str() << ", "
              << p.idle_ms << " ms)";
    v.push_back(StallReport{c->uuid, p, std::chrono::steady_clock::now()});
    decide_stall(c->group, p.tag, std::chrono::steady_clock::now());
}

bool Master::decide_stall(uint32_t group, uint64_t tag, std::chrono::steady_clock::time_point now) {
    const auto key = std::make_pair(group, tag);
    auto sit = stalls_.find(key);
    if (sit == stalls_.end()) return false;
    auto &v = sit->second;
    size_t performing = 0, reported = 0;
    for (const auto &[u, c] : clients_) {
        if (c.group != group || c.phase != Phase::Accepted) continue;
        auto it = c.colls.find(tag);
        if (it == c.colls.end() || it->second != CollState::Perform) continue;
        ++performing;
        for (const auto &r : v)
            if (r.reporter == u) ++reported;
    }
    if (performing == 0 || v.empty()) { // the op ended (aborted / completed) or its reporters left
        stalls_.erase(sit);
        return false;
    }
    if (reported < performing && now - v.front().at < std::chrono::milliseconds(stall_window_ms_)) return false;
    // A blocked send is direct evidence against its receiver. Otherwise the ring stalled at one link: the peers
    // behind it wait in later ring steps (each can finish the step it already has data for), so the report with the
    // lowest step names the link's sender; ties go to the longest idle time.
    const StallReport *best = nullptr;
    for (const auto &r : v) {
        const auto &a = r.report;
        if (!best) {
            best = &r;
            continue;
        }
        const auto &b = best->report;
        const bool a_tx = a.kind == kStallTxBlocked, b_tx = b.kind == kStallTxBlocked;
        if (a_tx != b_tx) {
            if (a_tx) best = &r;
            continue;
        }
        if (a.step != b.step ? a.step < b.step : a.idle_ms > b.idle_ms) best = &r;
    }
    const Uuid suspect = best->report.suspect;
    stalls_.erase(sit);
    ClientInfo *s = client_by_uuid(suspect);
    live_stalled_++;
    if (s && s->group == group) {
        LOG(WARN) << "Master: op tag " << tag << " of group " << group << " stalled (" << reported << " of "
                  << performing << " participants reported); dropping peer " << suspect.str();
        kick(s->addr); // the disconnect path aborts the op for everyone
    } else {
        LOG(WARN) << "Master: op tag " << tag << " stalled; the suspect already left: aborting the op";
        auto &ab = groups_[group].aborted[tag];
        if (!ab) {
            ab = true;
            send_abort(group, tag, true);
        }
    }
    return true;
}

bool Master::is_waiting(const ClientInfo &c) {
    switch (c.state) {
        case State::VoteAcceptNewPeers:
        case State::VoteNoNewPeersEstablishP2P:
        case State::WaitingForOtherPeers:
        case State::VoteOptimizeTopology:
        case State::VoteCompleteTopologyOptimization:
        case State::VoteSyncSharedState:
        case State::VoteCompleteSharedStateSync: return true;
        default: break;
    }
    if (c.voted_pending_query) return true;
    for (const auto &[_, cs] : c.colls)
        if (cs == CollState::VoteInitiate || cs == CollState::VoteComplete) return true;
    return false;
}

// in application code: nothing pending at the master (a peer in a data phase - connecting, benchmarking, moving
// shared state, running an op - is watched by the other detectors)
bool Master::is_lagging(const ClientInfo &c) {
    return c.phase == Phase::Accepted && c.state == State::Idle && c.colls.empty() && !c.voted_pending_query;
}

void Master::check_vote_timeouts(std::chrono::steady_clock::time_point now) {
    std::map<uint32_t, std::chrono::steady_clock::time_point> oldest;
    for (auto &[_, c] : clients_) {
        if (c.phase != Phase::Accepted) continue;
        const bool w = is_waiting(c);
        if (w && !c.waiting) c.waiting_since = now;
        c.waiting = w;
        if (w) {
            auto it = oldest.find(c.group);
            if (it == oldest.end() || c.waiting_since < it->second) oldest[c.group] = c.waiting_since;
        }
    }
    std::vector<SockAddr> late;
    for (const auto &[u, c] : clients_) {
        auto it = oldest.find(c.group);
        if (it == oldest.end() || now - it->second < std::chrono::milliseconds(vote_timeout_ms_)) continue;
        if (is_lagging(c)) late.push_back(c.addr);
    }
    for (const auto &a : late) {
        const ClientInfo *c = client_by_addr(a);
        LOG(WARN) << "Master: peer " << (c ? c->uuid.str() : std::string("?")) << " did not vote within "
                  << vote_timeout_ms_ << " ms while its group waited; dropping it";
        live_vote_++;
        kick(a);
    }
}

std::string Master::bandwidth_table() {
    auto done = std::make_shared<std::promise<std::string>>();
    auto fut = done->get_future();
    server_.post([this, done] {
        std::string out;
        for (const auto &[g, gs] : groups_) {
            std::istringstream in(gs.bw.dump());
            for (std::string ln; std::getline(in, ln);) out += std::to_string(g) + " " + ln + "\n";
        }
        done->set_value(out);
    });
    if (fut.wait_for(std::chrono::seconds(10)) != std::future_status::ready) return {};
    return fut.get();
}

std::string Master::dump_state() const {
    static const char *phases[] = {"registered", "accepted"};
    static const char *states[] = {"idle", "vote_accept_new", "vote_no_new", "connecting", "connecting_failed",
                                   "waiting_for_others", "vote_optimize", "optimize", "optimize_failed",
                                   "vote_optimize_complete", "vote_sync_ss", "distribute_ss", "request_ss",
                                   "vote_ss_complete", "collectives_running"};
    static const char *colls[] = {"vote_initiate", "perform", "vote_complete"};
    std::string s;
    for (const auto &[u, c] : clients_) {
        s += "  " + u.str().substr(0, 8) + " " + sockaddr_str(c.addr) + " group " + std::to_string(c.group) + " " +
             phases[static_cast<int>(c.phase)] + " " + states[static_cast<int>(c.state)] +
             (c.voted_pending_query ? " (voted pending query)" : "");
        for (const auto &[tag, cs] : c.colls) s += " tag" + std::to_string(tag) + ":" + colls[static_cast<int>(cs)];
        s += "\n";
    }
    return s;
}

// Newcomers are admitted by a vote of the accepted peers. If every accepted peer left while newcomers were waiting,
// nobody would ever vote: bootstrap them like the very first peer of a run.
void Master::maybe_bootstrap_orphans() {
    bool any_accepted = false, any_waiting = false, any_connecting = false;
    for (const auto &[_, c] : clients_) {
        any_accepted = any_accepted || c.phase == Phase::Accepted;
        any_waiting = any_waiting || (c.phase == Phase::Registered && c.state == State::Idle);
        any_connecting = any_connecting || c.state == State::ConnectingToPeers || c.state == State::WaitingForOtherPeers;
    }
    if (any_accepted || !any_waiting || any_connecting) return;
    LOG(INFO) << "Master: no accepted peers left; admitting the waiting newcomers";
    for (auto &[_, c] : clients_) {
        if (c.phase == Phase::Registered && c.state == State::Idle) {
            c.phase = Phase::Accepted;
            on_peer_accepted(c);
            break;
        }
    }
    transition_to_establish(true);
}

} // namespace pccl::master
