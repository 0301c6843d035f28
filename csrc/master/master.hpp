// Master coordinator: authoritative per-peer state machine + micro-consensus for every phase change
// (reference behaviour: ccoip/src/cpp/ccoip_master_state.cpp and ccoip_master_handler.cpp).
//
// All state lives on the EventServer loop thread; the only other thread is the asynchronous "moonshot" ATSP
// search, which hands its result back through `pending_rings_` and is applied at the start of the next P2P
// establishment round (never in the middle of one).
//
// Deliberate divergences from the reference:
//  * reachable-ring search uses mutual *reachability* as adjacency (reference used the unreachable set, #5)
//  * topology task result is applied when it improved the tour (reference returned early on improvement, #4) and
//    M2COptimizeTopologyComplete carries the ring order
//  * revision-legality check of an unknown client cannot dereference an end iterator (#6)
//  * a peer group whose latest-revision holders all died re-baselines instead of failing with "no distributor"
//  * a mixed round of accept-new / no-new establish votes proceeds as "no new peers" instead of deadlocking
//  * ring order survives membership changes (members keep their relative order, new peers are appended) instead of
//    falling back to UUID order, so an optimized ring is not thrown away on every join/leave
#pragma once

#include <array>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "../common/types.hpp"
#include "../net/event_server.hpp"
#include "../proto/packets.hpp"
#include "topology.hpp"

namespace pccl::master {

enum class Phase { Registered, Accepted };

enum class State {
    Idle,
    VoteAcceptNewPeers,
    VoteNoNewPeersEstablishP2P,
    ConnectingToPeers,
    ConnectingToPeersFailed,
    WaitingForOtherPeers,
    VoteOptimizeTopology,
    OptimizeTopology,
    OptimizeTopologyFailed,
    VoteCompleteTopologyOptimization,
    VoteSyncSharedState,
    DistributeSharedState,
    RequestSharedState,
    VoteCompleteSharedStateSync,
    CollectiveCommsRunning
};

enum class CollState { VoteInitiate, Perform, VoteComplete };

enum class SSStatus { Match, KeySetMismatch, ContentHashMismatch, RevisionOutdated, RevisionIncrementViolation };

struct ClientInfo {
    Uuid uuid;
    SockAddr addr{};
    Phase phase = Phase::Registered;
    State state = State::Idle;
    bool voted_pending_query = false;
    std::map<uint64_t, CollState> colls;
    // the ring members of this peer's last P2P establishment: an op whose participants' rings still hold a peer that
    // has left cannot complete (a stopped peer's connections stay open, so nothing on the data plane fails)
    std::vector<Uuid> ring_members;
    std::map<uint64_t, uint8_t> coll_flags; // initiate capability bits per running tag
    std::map<uint64_t, proto::WireShape> coll_shapes; // proposed data-plane shape per running tag (kCollFlagExtWire)
    uint32_t group = 0;
    SockAddr p2p{}, ss{}, bm{};
    uint64_t ss_revision = 0; // revision announced in the current shared-state round
    std::string host_token;   // registration extension; empty for reference clients
    bool xgmi = true;         // registration extension: may take the xGMI IPC path
    // liveness extension (registration): the peer sends heartbeats; silent for PCCL_PEER_TIMEOUT_MS -> dropped.
    // Reference peers (liveness = false) are exempt, as the reference master has no timeout at all.
    bool liveness = false;
    std::chrono::steady_clock::time_point last_seen{};
    // vote timeout bookkeeping (PCCL_VOTE_TIMEOUT_MS): since when the peer waits in a consensus
    bool waiting = false;
    std::chrono::steady_clock::time_point waiting_since{};
};

// One C2MOpStalled report of a running op (collected per group and tag, decided by decide_stall)
struct StallReport {
    Uuid reporter;
    proto::C2MOpStalled report;
    std::chrono::steady_clock::time_point at;
};

struct GroupState {
    std::vector<Uuid> ring;
    bool ring_optimal = false;
    bool optimized_once = false;
    BandwidthStore bw;
    uint64_t next_revision = 0;
    // shared-state round
    std::vector<std::pair<Uuid, std::vector<proto::SharedStateHashEntry>>> candidates, entries;
    std::vector<proto::SharedStateHashEntry> mask;
    std::map<Uuid, SSStatus> statuses;
    std::map<std::string, uint64_t> hashes;
    std::map<std::string, HashType> hash_types;
    std::map<Uuid, std::vector<std::string>> dirty_keys;
    std::map<Uuid, SyncStrategy> strategies;
    std::map<uint64_t, bool> aborted; // per tag
};

class Master {
public:
    explicit Master(const SockAddr &listen_addr);
    ~Master();

    bool launch();    // listen + start loop thread (non-blocking)
    bool interrupt(); // stop loop
    bool join();      // wait for loop thread
    uint16_t port() const { return server_.port(); }

private:
    // dispatch
    void on_packet(const SockAddr &addr, uint16_t id, const uint8_t *payload, size_t n);
    void on_disconnect(const SockAddr &addr);
    void maybe_bootstrap_orphans();
    void on_tick();
    std::chrono::steady_clock::time_point last_dump_{};

public:
    std::string dump_state() const;
    // "<group> <from uuid> <to uuid> <Mbit/s>" per measured (or same-host constant) edge of every group's bandwidth
    // store; runs on the loop thread (must not be called from it)
    std::string bandwidth_table();

private:
    void kick(const SockAddr &addr);

    // handlers
    void handle_join(const SockAddr &addr, const proto::C2MRequestSessionRegistration &p);
    void handle_request_establish(const SockAddr &addr, bool accept_new);
    void handle_p2p_established(const SockAddr &addr, const proto::C2MP2PConnectionsEstablished &p);
    void handle_check_pending(const SockAddr &addr);
    void handle_optimize(const SockAddr &addr);
    void handle_report_bw(const SockAddr &addr, const proto::C2MReportPeerBandwidth &p);
    void handle_optimize_work_complete(const SockAddr &addr);
    void handle_sync_shared_state(const SockAddr &addr, const proto::C2MSyncSharedState &p);
    void handle_dist_complete(const SockAddr &addr);
    void handle_coll_initiate(const SockAddr &addr, const proto::C2MCollectiveCommsInitiate &p);
    void handle_coll_complete(const SockAddr &addr, const proto::C2MCollectiveCommsComplete &p);
    void handle_op_stalled(const SockAddr &addr, const proto::C2MOpStalled &p);

    // liveness (on the loop thread; docs/ARCHITECTURE.md "Failure detection")
    void check_liveness(std::chrono::steady_clock::time_point now);
    // decides a stalled op once every performing participant reported or the decision window passed: kicks the peer
    // the reports name (which aborts the op through the disconnect path); returns true if it decided
    bool decide_stall(uint32_t group, uint64_t tag, std::chrono::steady_clock::time_point now);
    void check_vote_timeouts(std::chrono::steady_clock::time_point now);
    static bool is_waiting(const ClientInfo &c);
    static bool is_lagging(const ClientInfo &c);

    // consensus checks
    void check_establish_consensus();
    bool check_p2p_established();
    void check_pending_query_consensus();
    void check_optimize_consensus();
    static double same_host_mbps();
    void check_optimize_complete_consensus();
    bool check_sync_consensus(uint32_t group);
    void check_sync_complete_consensus(uint32_t group);
    void check_coll_initiate_consensus(uint32_t group, uint64_t tag);
    void check_coll_complete_consensus(uint32_t group, uint64_t tag);
    void send_abort(uint32_t group, uint64_t tag, bool aborted);

    // helpers
    ClientInfo *client_by_addr(const SockAddr &addr);
    ClientInfo *client_by_uuid(const Uuid &u);
    void on_peer_accepted(ClientInfo &c);
    std::vector<Uuid> ring_of(uint32_t group, bool include_registered);
    // Host index of every ring member (hosts numbered by first appearance) if the ring qualifies for the hierarchical
    // all-reduce: >= 2 hosts, every host with the same number (>= 2) of members, every member with a host token.
    std::vector<uint32_t> host_layout(const std::vector<Uuid> &ring);
    std::optional<std::vector<Uuid>> reachable_ring(uint32_t group);
    uint64_t local_world_size(uint32_t group, bool include_registered) const;
    uint64_t num_groups(bool include_registered) const;
    uint64_t largest_group(bool include_registered) const;
    void send_connection_info(bool include_registered);
    void transition_to_establish(bool accept_new);
    void apply_pending_rings();
    void run_topology_optimization(uint32_t group);
    SSStatus revision_status(ClientInfo &c, uint64_t revision);
    bool elect_mask(uint32_t group);
    void compute_mismatches(uint32_t group);
    void end_sync_phase(uint32_t group);

    net::EventServer server_;
    std::map<Uuid, ClientInfo> clients_;
    std::unordered_map<SockAddrKey, Uuid, SockAddrKeyHash> by_addr_;
    std::map<uint32_t, GroupState> groups_;
    uint64_t dist_rr_ = 0; // round-robin cursor over shared-state distributors
    std::map<Uuid, std::set<Uuid>> unreachable_;
    std::map<Uuid, std::vector<Uuid>> prev_neighbors_;
    uint64_t next_seq_ = 0;
    bool peer_dropped_ = false;
    bool running_ = false;

    // liveness parameters (PCCL_PEER_TIMEOUT_MS default 10 s, 0 = off; PCCL_HEARTBEAT_MS default timeout / 5;
    // PCCL_OP_STALL_MS default 1.5 x timeout; PCCL_STALL_WINDOW_MS default min(1 s, stall / 4); PCCL_VOTE_TIMEOUT_MS
    // default 0 = off)
    uint32_t peer_timeout_ms_ = 0, heartbeat_ms_ = 0, op_stall_ms_ = 0, stall_window_ms_ = 0, vote_timeout_ms_ = 0;
    std::chrono::steady_clock::time_point last_heartbeat_{};
    std::map<std::pair<uint32_t, uint64_t>, std::vector<StallReport>> stalls_;

    // async moonshot optimization
    std::mutex pending_mtx_;
    std::map<uint32_t, std::pair<std::vector<Uuid>, bool>> pending_rings_;
    std::atomic<bool> stopping_{false};
    OptimizerPool optimizer_pool_{4, 64}; // declared last: stopped (joined) before the state its tasks touch

public:
    size_t optimizer_thread_count() { return optimizer_pool_.thread_count(); }
    // topology optimization counters (pcclxMasterTopologyStats): [0] synchronous ATSP solves, [1] microseconds of the
    // last one, [2] rings changed by a solve (synchronous or moonshot), [3] moonshot solves finished
    std::array<uint64_t, 4> topology_stats() const {
        return {topo_solves_.load(), topo_last_us_.load(), topo_changes_.load(), topo_moonshots_.load()};
    }
    // liveness counters (pcclxMasterLivenessStats): [0] peers dropped for silence, [1] peers dropped on stall
    // reports, [2] peers dropped for not voting (PCCL_VOTE_TIMEOUT_MS), [3] stall reports received
    std::array<uint64_t, 4> liveness_stats() const {
        return {live_silent_.load(), live_stalled_.load(), live_vote_.load(), live_reports_.load()};
    }

private:
    std::atomic<uint64_t> topo_solves_{0}, topo_last_us_{0}, topo_changes_{0}, topo_moonshots_{0};
    std::atomic<uint64_t> live_silent_{0}, live_stalled_{0}, live_vote_{0}, live_reports_{0};
};

} // namespace pccl::master
