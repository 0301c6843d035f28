#include "client.hpp"

#include <algorithm>
#include <chrono>
#include <csignal>
#include <cstring>
#include <list>
#include <sstream>
#include <sys/socket.h>
#include <unistd.h>

#include "../common/log.hpp"
#include "../net/socket.hpp"
#include "benchmark.hpp"
#include "ipc.hpp"

namespace pccl::client {

using namespace proto;
using namespace std::chrono_literals;

namespace {
// PCCL_WIRE: "reference" makes this peer speak exactly the reference protocol (interop testing, mixed deployments);
// unset / "ext" (default) the pccl-amd extensions, negotiated per op with the other participants
bool wire_reference_env() {
    const char *e = std::getenv("PCCL_WIRE");
    if (!e || !*e || std::strcmp(e, "ext") == 0) return false;
    if (std::strcmp(e, "reference") == 0) return true;
    LOG(WARN) << "PCCL_WIRE=" << e << " unknown (reference | ext): using ext";
    return false;
}
} // namespace

Client::Client(const ClientConfig &cfg) : cfg_(cfg), wire_reference_(wire_reference_env()), master_(cfg.master) {
    std::signal(SIGPIPE, SIG_IGN);
}

Client::~Client() {
    interrupt();
    join();
}

// ------------------------------------------------------------------------------------------------------------------
// listeners
// ------------------------------------------------------------------------------------------------------------------
bool Client::start_listeners() {
    const auto proto = cfg_.master.inet.protocol;
    p2p_listener_ = std::make_unique<net::Listener>(proto, cfg_.p2p_port);
    ss_listener_ = std::make_unique<net::Listener>(proto, cfg_.ss_port);
    bm_listener_ = std::make_unique<net::Listener>(proto, cfg_.bm_port);
    if (!p2p_listener_->listen() || !ss_listener_->listen() || !bm_listener_->listen()) {
        LOG(ERR) << "Failed to bind peer listeners";
        return false;
    }
    p2p_listener_->run_async([this](int fd, const SockAddr &a) { on_p2p_accept(fd, a); });
    ss_listener_->run_async([this](int fd, const SockAddr &a) { on_ss_accept(fd, a); });
    bm_listener_->run_async([this](int fd, const SockAddr &a) { on_bm_accept(fd, a); });
    LOG(INFO) << "Peer listening: p2p " << p2p_listener_->port() << ", shared state " << ss_listener_->port()
              << ", benchmark " << bm_listener_->port();
    return true;
}

void Client::on_p2p_accept(int fd, const SockAddr &peer) {
    timeval tv{10, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    auto hello = net::recv_packet<P2PHello>(fd);
    if (!hello) {
        LOG(WARN) << "P2P: no hello from " << sockaddr_str(peer);
        ::close(fd);
        return;
    }
    timeval none{0, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
    auto conn = std::make_shared<net::MuxConn>(fd, net::MuxConn::Mode::Rx, peer);
    conn->start();
    {
        std::lock_guard lock(p2p_mtx_);
        auto &pool = rx_[hello->peer_uuid];
        if (pool.size() <= hello->connection_nr) pool.resize(hello->connection_nr + 1);
        if (pool[hello->connection_nr]) pool[hello->connection_nr]->interrupt();
        pool[hello->connection_nr] = conn;
    }
    // ack only after the RX side is registered: an op may use it as soon as the connector reports success
    if (!net::send_packet(fd, P2PHelloAck{})) {
        LOG(WARN) << "P2P: failed to ack " << sockaddr_str(peer);
        conn->interrupt();
        return;
    }
    LOG(DEBUG) << "P2P RX connection #" << hello->connection_nr << " from " << hello->peer_uuid.str();
}

void Client::on_bm_accept(int fd, const SockAddr &peer) {
    timeval tv{10, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    auto hello = net::recv_packet<C2BHello>(fd);
    if (!hello) {
        ::close(fd);
        return;
    }
    std::lock_guard lock(bm_mtx_);
    // one benchmarked peer at a time (its parallel connections are all admitted)
    if (bm_running_.load() > 0 && bm_peer_ && *bm_peer_ != hello->peer_uuid) {
        net::send_packet(fd, B2CBenchmarkServerIsBusy{true});
        ::close(fd);
        return;
    }
    for (auto it = bm_threads_.begin(); bm_running_.load() == 0 && it != bm_threads_.end();) {
        if (it->joinable()) it->join();
        it = bm_threads_.erase(it);
    }
    net::send_packet(fd, B2CBenchmarkServerIsBusy{false});
    bm_peer_ = hello->peer_uuid;
    bm_running_++;
    bm_threads_.emplace_back([this, fd, peer] {
        benchmark_receive(fd, peer);
        bm_running_--;
    });
}

void Client::on_ss_accept(int fd, const SockAddr &peer) {
    std::lock_guard lock(ss_mtx_);
    ss_threads_.emplace_back([this, fd, peer] { serve_shared_state(fd, peer); });
}

// ------------------------------------------------------------------------------------------------------------------
// connect / establish
// ------------------------------------------------------------------------------------------------------------------
bool Client::connect() {
    if (accepted_) {
        LOG(WARN) << "connect() called twice";
        return false;
    }
    if (!start_listeners()) return false;
    if (!master_.connect()) return false;

    C2MRequestSessionRegistration reg;
    reg.peer_group = cfg_.peer_group;
    if (!wire_reference_) reg.host_token = net::host_token(); // (no token: the reference's registration bytes)
    // PCCL_XGMI_CAPABLE=0/1 overrides the advertised capability (tests on GPU-less hosts)
    reg.xgmi_capable = std::getenv("PCCL_XGMI_CAPABLE") ? env_flag("PCCL_XGMI_CAPABLE", true)
                                                       : !env_flag("PCCL_DISABLE_IPC", false) && device_backend_available();
    reg.liveness = !wire_reference_; // (encoded only with the host token: a reference peer's bytes stay unchanged)
    reg.use_explicit_addresses = cfg_.explicit_addresses;
    if (cfg_.explicit_addresses) {
        reg.advertised_p2p = cfg_.adv_p2p;
        reg.advertised_ss = cfg_.adv_ss;
        reg.advertised_bm = cfg_.adv_bm;
    } else {
        reg.p2p_port = p2p_listener_->port();
        reg.ss_port = ss_listener_->port();
        reg.bm_port = bm_listener_->port();
    }
    if (!master_.send(reg)) return false;
    // a live master answers at once; one that accepted the connection but does not run (stopped, wedged) must not
    // hang connect() (the liveness thread watches the master only from the response on)
    auto resp = master_.receive<M2CSessionRegistrationResponse>(
        nullptr, std::chrono::milliseconds(env_size("PCCL_REGISTRATION_TIMEOUT_MS", 30000)));
    if (!resp) {
        LOG(ERR) << "No registration response from master";
        return false;
    }
    if (!resp->accepted) {
        LOG(ERR) << "Master rejected registration";
        return false;
    }
    uuid_ = resp->assigned_uuid;
    LOG(INFO) << "Registered with master as " << uuid_.str();
    // liveness parameters: the master's (it runs the protocol), else only the local op watchdog (a reference
    // master: a stalled op fails here instead of being reported). PCCL_OP_STALL_MS overrides the stall timeout.
    master_liveness_ = !wire_reference_ && (resp->heartbeat_ms || resp->peer_timeout_ms || resp->op_stall_ms);
    hb_ms_ = master_liveness_ ? resp->heartbeat_ms : 0;
    peer_timeout_ms_ = master_liveness_ ? resp->peer_timeout_ms : 0;
    stall_ms_ = master_liveness_ ? resp->op_stall_ms : 15000;
    if (std::getenv("PCCL_OP_STALL_MS")) stall_ms_ = static_cast<uint32_t>(env_size("PCCL_OP_STALL_MS", stall_ms_));
    if (hb_ms_ || peer_timeout_ms_ || stall_ms_) liveness_thread_ = std::thread([this] { liveness_loop(); });
    const EstablishResult r = establish();
    if (r == EstablishResult::Failed) return false;
    accepted_ = true;
    if (r == EstablishResult::Retry) {
        // we were accepted even though the round failed: retry like every other peer
        if (!request_and_establish(true)) return false;
        return true;
    }
    conn_revision_++;
    return true;
}

bool Client::connect_pool(const PeerInfo &peer, std::vector<std::shared_ptr<net::MuxConn>> &pool) {
    pool.clear();
    for (uint32_t nr = 0; nr < cfg_.pool_size; ++nr) {
        const int fd = net::connect_tcp(peer.p2p_listen_addr, 5000);
        if (fd < 0) {
            LOG(WARN) << "P2P connect to " << sockaddr_str(peer.p2p_listen_addr) << " failed";
            for (auto &c : pool) c->interrupt();
            pool.clear();
            return false;
        }
        P2PHello hello;
        hello.peer_uuid = uuid_;
        hello.connection_nr = nr;
        timeval tv{10, 0};
        setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        if (!net::send_packet(fd, hello) || !net::recv_packet<P2PHelloAck>(fd)) {
            LOG(WARN) << "P2P handshake with " << peer.peer_uuid.str() << " failed";
            ::close(fd);
            for (auto &c : pool) c->interrupt();
            pool.clear();
            return false;
        }
        timeval none{0, 0};
        setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
        auto conn = std::make_shared<net::MuxConn>(fd, net::MuxConn::Mode::Tx, peer.p2p_listen_addr);
        conn->start();
        pool.push_back(std::move(conn));
    }
    return true;
}

Client::EstablishResult Client::establish() {
    auto info = master_.receive<M2CP2PConnectionInfo>();
    if (!info) {
        LOG(ERR) << "Failed to receive P2P connection info";
        return EstablishResult::Failed;
    }
    global_ws_ = info->global_world_size;
    local_ws_ = info->local_world_size;
    n_groups_ = info->num_distinct_peer_groups;
    largest_group_ = info->largest_peer_group_world_size;

    std::vector<PeerInfo> neighbors, tx_targets;
    std::vector<ExtraPeer> extras;
    {
        std::lock_guard lock(p2p_mtx_);
        if (!info->unchanged) neighbors_ = info->all_peers;
        extras_ = info->extra_peers;
        neighbors = neighbors_;
        extras = extras_;
    }
    tx_targets = neighbors;
    std::vector<PeerInfo> extra_tx; // inter-host ring partners: connection failures only disable the hierarchy
    for (const auto &e : extras) {
        const bool dup = std::any_of(neighbors.begin(), neighbors.end(),
                                     [&](const PeerInfo &p) { return p.peer_uuid == e.peer.peer_uuid; });
        if ((e.role & kExtraTx) && !dup) extra_tx.push_back(e.peer);
    }
    bool ok = true;
    std::vector<Uuid> failed;
    for (const auto &n : extra_tx) {
        bool healthy = false;
        {
            std::lock_guard lock(p2p_mtx_);
            auto it = tx_.find(n.peer_uuid);
            if (it != tx_.end() && it->second.size() == cfg_.pool_size)
                healthy = std::all_of(it->second.begin(), it->second.end(), [](auto &c) { return c && c->is_open(); });
        }
        if (healthy) continue;
        std::vector<std::shared_ptr<net::MuxConn>> pool;
        if (!connect_pool(n, pool)) {
            LOG(WARN) << "P2P: inter-host ring partner " << n.peer_uuid.str() << " unreachable (hierarchy disabled)";
            continue;
        }
        std::lock_guard lock(p2p_mtx_);
        auto &slot = tx_[n.peer_uuid];
        for (auto &c : slot)
            if (c) c->interrupt();
        slot = std::move(pool);
    }
    for (const auto &n : neighbors) {
        bool healthy = false;
        {
            std::lock_guard lock(p2p_mtx_);
            auto it = tx_.find(n.peer_uuid);
            if (it != tx_.end() && it->second.size() == cfg_.pool_size)
                healthy = std::all_of(it->second.begin(), it->second.end(), [](auto &c) { return c && c->is_open(); });
        }
        if (healthy) continue;
        std::vector<std::shared_ptr<net::MuxConn>> pool;
        if (!connect_pool(n, pool)) {
            ok = false;
            failed.push_back(n.peer_uuid);
            break;
        }
        std::lock_guard lock(p2p_mtx_);
        auto &slot = tx_[n.peer_uuid];
        for (auto &c : slot)
            if (c) c->interrupt();
        slot = std::move(pool);
    }
    {
        // drop TX pools to non-neighbours and RX pools from non-neighbours / dead RX connections
        std::lock_guard lock(p2p_mtx_);
        auto is_nb = [&](const Uuid &u) {
            return std::any_of(neighbors.begin(), neighbors.end(), [&](const PeerInfo &p) { return p.peer_uuid == u; });
        };
        auto is_extra = [&](const Uuid &u, uint8_t role) {
            return std::any_of(extras.begin(), extras.end(),
                               [&](const ExtraPeer &e) { return e.peer.peer_uuid == u && (e.role & role); });
        };
        for (auto it = tx_.begin(); it != tx_.end();) {
            if (!is_nb(it->first) && !is_extra(it->first, kExtraTx)) {
                for (auto &c : it->second)
                    if (c) c->interrupt();
                it = tx_.erase(it);
            } else {
                ++it;
            }
        }
        for (auto it = rx_.begin(); it != rx_.end();) {
            if (!is_nb(it->first) && !is_extra(it->first, kExtraRx)) {
                for (auto &c : it->second)
                    if (c) c->interrupt();
                it = rx_.erase(it);
            } else {
                ++it;
            }
        }
    }
    C2MP2PConnectionsEstablished est;
    est.success = ok;
    est.failed_peers = failed;
    if (!master_.send(est)) return EstablishResult::Failed;
    auto resp = master_.receive<M2CP2PConnectionsEstablished>();
    if (!resp) {
        LOG(ERR) << "Failed to receive P2P established response";
        return EstablishResult::Failed;
    }
    if (!resp->success) {
        LOG(INFO) << "P2P establishment round failed (peer churn); retrying";
        return EstablishResult::Retry;
    }
    std::shared_ptr<IpcArena> old_arena;
    {
        std::lock_guard lock(p2p_mtx_);
        ring_ = resp->ring_order;
        old_arena = arena_;
    }
    // Intra-node fast path: every peer of a loopback run lives on this host (the master enforces loopback
    // exclusivity), or the master reports that every ring member registered with this host's identity; the ring can
    // then rendezvous in shared memory and exchange device buffers over xGMI.
    std::shared_ptr<IpcArena> arena;
    // (a master that predates the host extension: a loopback master implies one host)
    const bool one_host = resp->has_host_info ? resp->single_host : sockaddr_is_loopback(cfg_.master);
    if (resp->ring_order.size() >= 2 && one_host && !env_flag("PCCL_DISABLE_IPC", false) &&
        device_backend_available()) {
        if (old_arena && old_arena->matches(resp->ring_order)) {
            arena = old_arena;
        } else {
            arena = IpcArena::create(*this, resp->ring_order, cfg_.master.port, cfg_.peer_group);
        }
    }
    // Hierarchical layout across hosts: IPC arena over my host's members + the inter-host ring of my local rank
    std::shared_ptr<HierState> hier;
    const auto &host_of = resp->host_of;
    if (host_of.size() == resp->ring_order.size() && host_of.size() >= 4 && !env_flag("PCCL_DISABLE_IPC", false) &&
        env_flag("PCCL_HIERARCHICAL", true) && device_backend_available()) {
        const auto &ring = resp->ring_order;
        const size_t me = static_cast<size_t>(std::find(ring.begin(), ring.end(), uuid_) - ring.begin());
        if (me < ring.size()) {
            auto h = std::make_shared<HierState>();
            h->hosts = *std::max_element(host_of.begin(), host_of.end()) + 1;
            h->host = host_of[me];
            std::vector<Uuid> local;
            for (size_t k = 0; k < ring.size(); ++k) {
                if (host_of[k] != h->host) continue;
                if (k == me) h->local_rank = local.size();
                local.push_back(ring[k]);
            }
            h->local = local.size();
            std::vector<std::vector<Uuid>> per_host(h->hosts);
            for (size_t k = 0; k < ring.size(); ++k) per_host[host_of[k]].push_back(ring[k]);
            bool valid = h->local >= 2 && h->hosts >= 2;
            for (const auto &ph : per_host) valid = valid && ph.size() == h->local;
            if (valid) {
                for (const auto &ph : per_host) h->host_ring.push_back(ph[h->local_rank]);
                std::shared_ptr<HierState> prev;
                {
                    std::lock_guard lock(p2p_mtx_);
                    prev = hier_;
                }
                if (prev && prev->arena && prev->arena->matches(local)) {
                    h->arena = prev->arena;
                } else {
                    h->arena = IpcArena::create(*this, local, cfg_.master.port, cfg_.peer_group);
                }
                if (h->arena) hier = h;
            }
        }
    }
    {
        std::lock_guard lock(p2p_mtx_);
        arena_ = arena;
        hier_ = hier;
    }
    return EstablishResult::Success;
}

bool Client::request_and_establish(bool accept_new) {
    std::lock_guard lock(establish_mtx_);
    return request_and_establish_locked(accept_new);
}

bool Client::request_and_establish_locked(bool accept_new) {
    if (!accepted_) return false;
    if (!master_.is_open()) {
        LOG(ERR) << "Master connection closed (kicked?)";
        return false;
    }
    EstablishResult r;
    do {
        C2MRequestEstablishP2PConnections pkt;
        pkt.accept_new_peers = accept_new;
        if (!master_.send(pkt)) return false;
        r = establish();
    } while (r == EstablishResult::Retry);
    if (r == EstablishResult::Failed) return false;
    conn_revision_++;
    return true;
}

bool Client::update_topology() {
    if (any_collective_running()) return false;
    return request_and_establish(true);
}

bool Client::are_peers_pending(bool &pending) {
    if (!accepted_ || !master_.is_open()) return false;
    if (!master_.send(C2MCheckPeersPending{})) return false;
    auto r = master_.receive<M2CPeersPendingResponse>();
    if (!r) return false;
    pending = r->peers_pending;
    return true;
}

int Client::ring_rank() {
    std::lock_guard lock(p2p_mtx_);
    for (size_t i = 0; i < ring_.size(); ++i)
        if (ring_[i] == uuid_) return static_cast<int>(i);
    return -1;
}

std::optional<Client::RingView> Client::ring_view(uint64_t seq) {
    std::lock_guard lock(p2p_mtx_);
    RingView rv;
    rv.ring = ring_;
    auto it = std::find(ring_.begin(), ring_.end(), uuid_);
    if (it == ring_.end()) return std::nullopt;
    rv.rank = static_cast<size_t>(it - ring_.begin());
    rv.arena = arena_;
    if (ring_.size() < 2) return rv;
    const Uuid next = ring_[(rv.rank + 1) % ring_.size()];
    const Uuid prev = ring_[(rv.rank + ring_.size() - 1) % ring_.size()];
    auto t = tx_.find(next);
    auto r = rx_.find(prev);
    if (t == tx_.end() || r == rx_.end() || t->second.empty() || r->second.empty()) return std::nullopt;
    rv.tx = t->second;
    rv.rx = r->second;
    if (hier_) {
        const auto &hr = hier_->host_ring;
        const Uuid hnext = hr[(hier_->host + 1) % hr.size()];
        const Uuid hprev = hr[(hier_->host + hr.size() - 1) % hr.size()];
        auto ht = tx_.find(hnext);
        auto hrx = rx_.find(hprev);
        if (ht != tx_.end() && hrx != rx_.end() && !ht->second.empty() && !hrx->second.empty()) {
            rv.hier = hier_;
            rv.htx = ht->second;
            rv.hrx = hrx->second;
        }
    }
    (void)seq;
    return rv;
}

// ------------------------------------------------------------------------------------------------------------------
// topology optimization (bandwidth benchmarks + ATSP on the master)
// ------------------------------------------------------------------------------------------------------------------
bool Client::optimize_topology() {
    if (!accepted_ || !master_.is_open()) return false;
    bool complete = false;
    do {
        if (!master_.send(C2MOptimizeTopology{})) return false;
        auto resp = master_.receive<M2COptimizeTopologyResponse>();
        if (!resp) return false;
        // The master orders the probes as a round-robin schedule (every peer sends to one peer and receives from one
        // per round): probe them in that order. A target still serving the previous round's sender (one probe holds
        // it for PCCL_BENCHMARK_MILLIS) is retried with a back-off from 20 ms up to 1/8 of a probe, and moved behind
        // the other targets once it has refused for half a probe's length, so a busy server sees a few connection
        // attempts per probe instead of fifty per second.
        std::list<BenchmarkRequest> todo(resp->requests.begin(), resp->requests.end());
        std::map<Uuid, int> refusals;
        std::map<Uuid, std::chrono::steady_clock::time_point> busy_since;
        const auto probe = std::chrono::milliseconds(env_size("PCCL_BENCHMARK_MILLIS", 10000));
        auto delay = std::chrono::milliseconds(20);
        while (!todo.empty()) {
            auto it = todo.begin();
            double mbps = 0;
            const BenchResult r = benchmark_send(uuid_, it->to_peer_endpoint, mbps);
            if (r == BenchResult::Success) {
                delay = std::chrono::milliseconds(20);
                busy_since.erase(it->to_peer);
                C2MReportPeerBandwidth rep;
                rep.to_peer = it->to_peer;
                rep.bandwidth_mbps = mbps;
                if (!master_.send(rep)) return false;
                LOG(INFO) << "Bandwidth to " << it->to_peer.str() << ": " << mbps << " Mbit/s";
                todo.erase(it);
            } else if (r == BenchResult::Busy || r == BenchResult::SendFailure) {
                const auto now = std::chrono::steady_clock::now();
                auto since = busy_since.emplace(it->to_peer, now).first;
                ++refusals[it->to_peer];
                if (now - since->second >= probe / 2 && todo.size() > 1) {
                    busy_since.erase(since);
                    todo.splice(todo.end(), todo, it);
                    delay = std::chrono::milliseconds(20);
                    continue;
                }
                std::this_thread::sleep_for(delay);
                delay = std::min<std::chrono::milliseconds>(delay * 2, std::max<std::chrono::milliseconds>(20ms, probe / 8));
            } else {
                LOG(WARN) << "Benchmark to " << sockaddr_str(it->to_peer_endpoint) << " failed; skipping";
                todo.erase(it);
            }
        }
        if (!master_.send(C2MOptimizeTopologyWorkComplete{})) return false;
        auto done = master_.receive<M2COptimizeTopologyComplete>();
        if (!done) return false;
        complete = done->success;
    } while (!complete);
    // rewire to the (possibly) new ring order
    return request_and_establish(false);
}

// ------------------------------------------------------------------------------------------------------------------
// liveness: heartbeats, master silence, op stall watchdog
// ------------------------------------------------------------------------------------------------------------------
void Client::watch_op(const std::shared_ptr<OpState> &op, const RingView &rv) {
    if (stall_ms_ == 0 || rv.ring.size() < 2) return;
    Watched w;
    w.op = op;
    w.rx = rv.rx;
    w.tx = rv.tx;
    w.prev = rv.ring[(rv.rank + rv.ring.size() - 1) % rv.ring.size()];
    w.next = rv.ring[(rv.rank + 1) % rv.ring.size()];
    w.progress = std::chrono::steady_clock::now();
    for (const auto &c : w.rx) w.bytes += c ? c->rx_bytes_total() : 0;
    for (const auto &c : w.tx) w.bytes += c ? c->tx_bytes_total() : 0;
    std::lock_guard l(live_mtx_);
    watched_[op.get()] = std::move(w);
}

void Client::unwatch_op(const OpState *op) {
    std::lock_guard l(live_mtx_);
    watched_.erase(op);
}

void Client::liveness_loop() {
    name_thread("pccl-liveness");
    using clock = std::chrono::steady_clock;
    const auto hb = std::chrono::milliseconds(hb_ms_), stall = std::chrono::milliseconds(stall_ms_);
    auto next_hb = clock::now();
    std::unique_lock l(live_mtx_);
    while (!live_stop_) {
        live_cv_.wait_for(l, std::chrono::milliseconds(50));
        if (live_stop_) break;
        const auto now = clock::now();
        if (hb_ms_ > 0 && now >= next_hb && master_.is_open()) {
            l.unlock();
            if (master_.send(C2MHeartbeat{})) heartbeats_++;
            l.lock();
            next_hb = now + hb;
        }
        // PCCL_CLIENT_DUMP_SEC=N: log this peer's consensus-relevant state every N seconds (diagnosing stuck runs;
        // the master's counterpart is PCCL_MASTER_DUMP_SEC)
        static const size_t dump_every = env_size("PCCL_CLIENT_DUMP_SEC", 0);
        if (dump_every && now - last_dump_ >= std::chrono::seconds(dump_every)) {
            last_dump_ = now;
            l.unlock();
            std::ostringstream os;
            os << "Client " << uuid_.str() << ": revision " << conn_revision_.load() << " pending-reestablish "
               << static_cast<int64_t>(reestablish_pending_.load()) << " ops";
            {
                std::lock_guard ol(ops_mtx_);
                for (const auto &[t, op] : ops_)
                    os << " " << t << (op->done.load() ? (op->success ? ":ok" : ":failed") : ":running")
                       << (op->joined.load() ? "/joined" : "") << "@" << op->revision_at_start;
            }
            LOG(WARN) << os.str();
            l.lock();
        }
        // a master that has been silent for twice the peer timeout (it sends M2CHeartbeat every heartbeat interval)
        // is lost: closing the connection fails every wait on it instead of hanging the application
        if (peer_timeout_ms_ > 0 && master_.is_open()) {
            const auto silent = std::chrono::nanoseconds(
                std::chrono::duration_cast<std::chrono::nanoseconds>(now.time_since_epoch()).count() -
                master_.last_rx_ns());
            if (silent > 2 * std::chrono::milliseconds(peer_timeout_ms_)) {
                LOG(ERR) << "Master silent for " << std::chrono::duration_cast<std::chrono::milliseconds>(silent).count()
                         << " ms: treating it as lost";
                master_lost_++;
                l.unlock();
                master_.interrupt();
                l.lock();
            }
        }
        if (stall_ms_ == 0) continue;
        for (auto &[_, w] : watched_) {
            uint64_t bytes = 0;
            for (const auto &c : w.rx) bytes += c ? c->rx_bytes_total() : 0;
            for (const auto &c : w.tx) bytes += c ? c->tx_bytes_total() : 0;
            if (bytes != w.bytes) {
                w.bytes = bytes;
                w.progress = now;
                continue;
            }
            const auto idle = now - w.progress;
            if (!w.reported && idle >= stall) {
                // the evidence: a send to the next peer blocked for half the timeout means it does not drain its
                // socket; otherwise nothing arrives from the previous peer
                std::chrono::nanoseconds blocked{0};
                for (const auto &c : w.tx)
                    if (c) blocked = std::max(blocked, c->send_blocked_for());
                C2MOpStalled rep;
                rep.tag = w.op->req.tag;
                rep.kind = blocked >= stall / 2 ? kStallTxBlocked : kStallRxIdle;
                rep.suspect = rep.kind == kStallTxBlocked ? w.next : w.prev;
                rep.step = w.op->watch.step.load(std::memory_order_relaxed);
                rep.idle_ms = static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::milliseconds>(idle).count());
                LOG(WARN) << "all-reduce tag " << rep.tag << ": no progress for " << rep.idle_ms << " ms in ring step "
                          << rep.step << " (" << (rep.kind == kStallTxBlocked ? "send to " : "nothing from ")
                          << rep.suspect.str() << ")";
                w.reported = true;
                w.reported_at = now;
                if (master_liveness_ && master_.is_open()) {
                    l.unlock();
                    const bool sent = master_.send(rep);
                    l.lock();
                    if (sent) stall_reports_++;
                    break; // watched_ may have changed while unlocked: rescan at the next tick
                }
                w.op->watch.failed.store(true, std::memory_order_release);
                stall_fails_++;
            } else if (w.reported && now - w.reported_at >= stall && !w.op->watch.failed.load()) {
                // the master did not resolve the stall (no abort): fail the op here
                LOG(WARN) << "all-reduce tag " << w.op->req.tag << ": stall unresolved by the master; failing the op";
                w.op->watch.failed.store(true, std::memory_order_release);
                stall_fails_++;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------------------------
// lifecycle
// ------------------------------------------------------------------------------------------------------------------
bool Client::any_collective_running() {
    std::lock_guard lock(ops_mtx_);
    for (auto &[_, op] : ops_)
        if (!op->joined.load()) return true; // started and not yet awaited (reference semantics)
    return false;
}

bool Client::interrupt() {
    if (interrupted_.exchange(true)) return true;
    {
        std::lock_guard l(live_mtx_);
        live_stop_ = true;
    }
    live_cv_.notify_all();
    master_.interrupt();
    {
        std::lock_guard lock(p2p_mtx_);
        for (auto &[_, pool] : tx_)
            for (auto &c : pool)
                if (c) c->interrupt();
        for (auto &[_, pool] : rx_)
            for (auto &c : pool)
                if (c) c->interrupt();
    }
    if (p2p_listener_) p2p_listener_->interrupt();
    if (ss_listener_) ss_listener_->interrupt();
    if (bm_listener_) bm_listener_->interrupt();
    return true;
}

bool Client::join() {
    std::vector<std::shared_ptr<OpState>> ops;
    {
        std::lock_guard lock(ops_mtx_);
        for (auto &[_, op] : ops_) ops.push_back(op);
    }
    for (auto &op : ops) op->wait();
    if (liveness_thread_.joinable()) liveness_thread_.join();
    if (p2p_listener_) p2p_listener_->join();
    if (ss_listener_) ss_listener_->join();
    if (bm_listener_) bm_listener_->join();
    master_.join();
    {
        std::lock_guard lock(p2p_mtx_);
        tx_.clear();
        rx_.clear();
        arena_.reset();
    }
    std::vector<std::thread> ss, bm;
    {
        std::lock_guard lock(ss_mtx_);
        ss.swap(ss_threads_);
    }
    for (auto &t : ss)
        if (t.joinable()) t.join();
    {
        std::lock_guard lock(bm_mtx_);
        bm.swap(bm_threads_);
    }
    for (auto &t : bm)
        if (t.joinable()) t.join();
    return true;
}

} // namespace pccl::client
