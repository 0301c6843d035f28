// Peer (client) protocol engine: connection management, phase votes, collectives and shared state
// (reference behaviour: ccoip/src/cpp/ccoip_client_handler.cpp, ccoip_client_state.cpp, reduce.cpp).
#pragma once

#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "../common/device_backend.hpp"
#include "../common/spin.hpp"
#include "../common/types.hpp"
#include "../net/listener.hpp"
#include "../net/master_conn.hpp"
#include "../net/mux.hpp"
#include "ring_common.hpp"

namespace pccl::client {

struct ClientConfig {
    SockAddr master{};
    uint32_t peer_group = 0;
    uint32_t pool_size = 1;
    uint16_t p2p_port = 48149, ss_port = 48150, bm_port = 48151;
    bool explicit_addresses = false;
    SockAddr adv_p2p{}, adv_ss{}, adv_bm{};
};

struct SSEntry {
    std::string key;
    DType dtype = DType::F32;
    DeviceType device = DeviceType::Cpu;
    void *data = nullptr;
    size_t count = 0;
    size_t bytes = 0;
    bool allow_content_inequality = false;
};

struct SharedState {
    uint64_t revision = 0;
    SyncStrategy strategy = SyncStrategy::EnforcePopular;
    std::vector<SSEntry> entries;
};

struct SSInfo {
    uint64_t tx_bytes = 0;
    uint64_t rx_bytes = 0;
};

struct ReduceInfo {
    uint32_t world_size = 0;
    uint64_t tx_bytes = 0;
    uint64_t rx_bytes = 0;
};

struct ReduceRequest {
    const void *src = nullptr;
    void *dst = nullptr;
    size_t count = 0;
    DType dtype = DType::F32;
    DType qtype = DType::F32;
    QuantAlgo qalgo = QuantAlgo::None;
    ReduceOp op = ReduceOp::Sum;
    uint64_t tag = 0;
    bool scratch = false; // internal: dst is library scratch, no abort backup needed (hierarchical inner ring)
    // stream-ordered ops (pcclxAllReduce*OnStream): an event recorded on `ready_stream` on the submitting thread,
    // right after the initiate packet went out (its host cost overlaps the master round trip); the op waits for it
    // before its data path reads `src`, then returns it to the event pool
    bool stream_ordered = false;
    DevStream ready_stream = nullptr;
    DevEvent ready = nullptr;
};

class IpcArena; // intra-node shared-memory + IPC rendezvous (ipc.cpp)

// Reusable collective worker threads (the reference runs ops on a pithreadpool of PCCL_MAX_CONCURRENT_COLLECTIVE_OPS
// workers, ccoip_client_state.hpp:17-25,98). Grows whenever every worker is busy, so an op never queues behind
// another one (a queued op could deadlock against peers that already run it); idle workers are reused, which keeps
// thread creation off the latency-critical path of back-to-back ops.
class OpWorkers {
public:
    OpWorkers() = default;
    OpWorkers(const OpWorkers &) = delete;
    OpWorkers &operator=(const OpWorkers &) = delete;
    ~OpWorkers();
    void submit(std::function<void()> fn);
    size_t thread_count();
    static size_t max_workers();

private:
    void loop();
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    std::vector<std::thread> threads_;
    size_t idle_ = 0;
    bool stop_ = false;
};

class Client {
public:
    explicit Client(const ClientConfig &cfg);
    ~Client();

    bool connect();
    bool interrupt();
    bool join();

    bool update_topology();                         // accept new peers + (re)establish ring
    bool request_and_establish(bool accept_new);
    bool are_peers_pending(bool &pending);
    bool optimize_topology();
    bool sync_shared_state(SharedState &ss, SSInfo &info);

    // inline_run: execute on the calling thread (blocking pcclAllReduce), else on a collective worker
    bool all_reduce_async(const ReduceRequest &req, bool inline_run = false);
    bool join_async_reduce(uint64_t tag);           // true on success
    bool get_reduce_info(uint64_t tag, ReduceInfo &out);
    bool any_collective_running();
    // Blocks until one of the given async ops (tags) has completed (or `timeout` passed); returns its tag, or
    // nullopt on timeout / if none of the tags is known. Used by the sliding-window retry scheduler.
    std::optional<uint64_t> wait_any(const std::vector<uint64_t> &tags, std::chrono::milliseconds timeout);

    size_t global_world_size() const { return global_ws_.load(); }
    size_t local_world_size() const { return local_ws_.load(); }
    size_t num_distinct_groups() const { return n_groups_.load(); }
    size_t largest_group_size() const { return largest_group_.load(); }
    uint64_t connection_revision() const { return conn_revision_.load(); }
    int ring_rank();
    int last_reduce_path() const { return last_path_.load(); }
    int last_reduce_framing() const { return last_framing_.load(); }
    size_t collective_worker_threads() { return workers_.thread_count(); }
    const Uuid &uuid() const { return uuid_; }
    bool master_connected() const { return master_.is_open(); }
    // liveness counters (pcclxLivenessStats): [0] stall reports sent, [1] ops failed by the local watchdog,
    // [2] master declared lost (silent for 2 x the peer timeout), [3] heartbeats sent
    std::array<uint64_t, 4> liveness_stats() const {
        return {stall_reports_.load(), stall_fails_.load(), master_lost_.load(), heartbeats_.load()};
    }

private:
    friend class IpcArena;
    enum class EstablishResult { Success, Retry, Failed };

    // Hierarchical layout (master's host_of extension): hosts x local ranks. The host-local peers share an IPC arena;
    // the peers with my local rank on every host form the inter-host ring (extra TX / RX pools).
    struct HierState {
        size_t hosts = 0, local = 0;   // H, L
        size_t host = 0, local_rank = 0;
        std::vector<Uuid> host_ring;   // the member with my local rank on host 0 .. H-1
        std::shared_ptr<IpcArena> arena; // over my host's members, in ring order
    };
    struct RingView { // immutable snapshot used by an op thread
        std::vector<Uuid> ring;
        size_t rank = 0;
        std::vector<std::shared_ptr<net::MuxConn>> tx; // pool to next
        std::vector<std::shared_ptr<net::MuxConn>> rx; // pool from prev
        std::shared_ptr<IpcArena> arena;
        std::shared_ptr<HierState> hier;                    // null unless the layout qualifies
        std::vector<std::shared_ptr<net::MuxConn>> htx, hrx; // inter-host ring pools (to next / from previous host)
    };

    struct OpState {
        ReduceRequest req;
        std::mutex m;
        std::condition_variable cv;
        std::atomic<bool> done{false};
        // awaited by the application; until then the op counts as running (reference ccoip_client_state.cpp:
        // a tag stays in running_collective_coms_ops_tags until joinAsyncCollectiveOp)
        std::atomic<bool> joined{false};
        void wait() {
            // short ops finish within tens of us of the wait: spin briefly before paying a futex wake-up
            if (spin_until([this] { return done.load(std::memory_order_acquire); })) return;
            std::unique_lock l(m);
            cv.wait(l, [this] { return done.load(); });
        }
        void finish() {
            {
                std::lock_guard l(m);
                done.store(true);
            }
            cv.notify_all();
        }
        bool success = false;
        bool info_taken = false;
        uint64_t revision_at_start = 0;
        std::atomic<uint64_t> tx{0}, rx{0};
        uint32_t world = 0;
        bool small_path = false; // every peer agreed on the small-message algorithm (kCollFlagSmallPath)
        ring::Shape shape;       // the op's agreed data-plane framing (commence: kCollFlagExtWire + WireShape)
        // Set by a data path that finished its part of an in-place op: holds the input's backup until the master's
        // verdict. run_op calls it once with restore = true if the op failed anyway (a peer was lost after this
        // peer's part was done), so a retry reduces the caller's input, not the result.
        std::function<void(bool restore)> settle;
        // initiate_op's results: the ring snapshot, where the buffers live, whether the master got the initiate
        // (async ops are initiated on the submitting thread, so a worker's wake-up overlaps the master round trip)
        bool initiated = false, init_sent = false, device = false;
        std::optional<RingView> rv;
        DevPtrInfo si{}, di{};
        ring::OpWatch watch; // progress of the op's TCP data path (the liveness thread's stall watchdog)
    };

    // Liveness (negotiated at registration, proto::C2MRequestSessionRegistration::liveness; docs/ARCHITECTURE.md):
    // a thread that sends the master heartbeats, declares a silent master lost, and watches the TCP data paths of
    // running ops - an op whose connections moved no byte for the stall timeout is reported to the master
    // (C2MOpStalled), which kicks the peer the evidence names and aborts the op; if the master cannot (a reference
    // master) or does not resolve it within another timeout, the op fails locally (OpWatch::failed).
    struct Watched {
        std::shared_ptr<OpState> op;
        ring::Conns rx, tx;
        Uuid prev, next;
        uint64_t bytes = 0;
        std::chrono::steady_clock::time_point progress, reported_at;
        bool reported = false;
    };
    void liveness_loop();
    void watch_op(const std::shared_ptr<OpState> &op, const RingView &rv);
    void unwatch_op(const OpState *op);

    // connection management
    bool start_listeners();
    void on_p2p_accept(int fd, const SockAddr &peer);
    void on_ss_accept(int fd, const SockAddr &peer);
    void on_bm_accept(int fd, const SockAddr &peer);
    EstablishResult establish();
    bool request_and_establish_locked(bool accept_new);
    bool connect_pool(const proto::PeerInfo &peer, std::vector<std::shared_ptr<net::MuxConn>> &pool);
    std::optional<RingView> ring_view(uint64_t seq);

    // collectives
    void initiate_op(OpState &op);
    // on_caller: running on the submitting thread (blocking call), which then also records the readiness event
    void run_op(const std::shared_ptr<OpState> &op, bool on_caller);
    void arm_ready(OpState &op);
    // returns {success, abort_received}
    std::pair<bool, bool> ring_reduce_host(OpState &op, const RingView &rv, uint64_t seq);
    std::pair<bool, bool> ring_reduce_device(OpState &op, const RingView &rv, uint64_t seq, int device);
    std::pair<bool, bool> ring_reduce_device_quant(OpState &op, const RingView &rv, uint64_t seq, int device);
    std::pair<bool, bool> device_quant_reference_framing(OpState &op, const RingView &rv, uint64_t seq, int device);
    std::pair<bool, bool> ipc_reduce(OpState &op, const RingView &rv, uint64_t seq, int device);
    // An xGMI op above the arena's staged size (kIpcMaxOpBytes) as consecutive sub-ops; `use_ring` is set when the
    // first sub-op's vote chose the TCP ring (the whole op then takes it)
    std::pair<bool, bool> ipc_reduce_segmented(OpState &op, const RingView &rv, uint64_t seq, int device,
                                               bool &use_ring);
    std::pair<bool, bool> hier_reduce(OpState &op, const RingView &rv, uint64_t seq, int device);
    // Whether the master's abort of the running op `tag` has arrived. It only looks: the packet is consumed by the
    // op's completion protocol (run_op), so a poll from any thread of the op can never take it from that wait.
    bool abort_received(uint64_t tag);

    // shared state
    void serve_shared_state(int fd, SockAddr peer);
    bool hash_entry(const SSEntry &e, uint64_t &hash, HashType &type);
    // Hashes many entries: device simplehashes are queued on one pooled stream per GPU (results into pinned words,
    // one sync per GPU at the end) while host entries hash on the CPU meanwhile.
    bool hash_entries(const std::vector<const SSEntry *> &entries, std::vector<uint64_t> &hashes, HashType &type);

    ClientConfig cfg_;
    // PCCL_WIRE=reference: register and run every op exactly as a reference peer would (no host token, so no IPC /
    // hierarchical paths; initiate packets without capability flags, so every op of the ring uses the reference
    // framing; no shared-state IPC hand-off)
    const bool wire_reference_;
    net::MasterConnection master_;
    std::unique_ptr<net::Listener> p2p_listener_, ss_listener_, bm_listener_;
    Uuid uuid_;
    std::atomic<bool> accepted_{false};
    std::atomic<bool> interrupted_{false};

    std::mutex p2p_mtx_;
    std::map<Uuid, std::vector<std::shared_ptr<net::MuxConn>>> tx_;
    std::map<Uuid, std::vector<std::shared_ptr<net::MuxConn>>> rx_;
    std::vector<proto::PeerInfo> neighbors_;
    std::vector<proto::ExtraPeer> extras_;
    std::vector<Uuid> ring_;
    std::shared_ptr<IpcArena> arena_;
    std::shared_ptr<HierState> hier_;
    std::mutex establish_mtx_; // serializes concurrent re-establishment attempts
    // a failed op was joined while other ops were still running (no establishment vote possible then): the connection
    // revision it failed on, or UINT64_MAX; the next join with nothing running performs the round (guarded by
    // establish_mtx_)
    std::atomic<uint64_t> reestablish_pending_{UINT64_MAX};

    std::atomic<uint64_t> conn_revision_{0};
    std::atomic<size_t> global_ws_{0}, local_ws_{0}, n_groups_{0}, largest_group_{0};
    std::atomic<int> last_path_{0};
    std::atomic<int> last_framing_{0}; // PCCL_ATTRIBUTE_LAST_REDUCE_FRAMING

    std::mutex ops_mtx_;
    std::mutex done_mtx_;           // signalled whenever an op finishes (wait_any)
    std::condition_variable done_cv_;
    std::map<uint64_t, std::shared_ptr<OpState>> ops_;
    OpWorkers workers_;

    // shared-state distribution (server side)
    std::mutex ss_mtx_;
    SharedState *serving_ = nullptr;
    int ss_active_serves_ = 0;       // serve threads still reading serving_'s memory (guarded by ss_mtx_)
    std::condition_variable ss_cv_;  // signalled when a serve ends
    std::atomic<uint64_t> ss_tx_bytes_{0};
    std::vector<std::thread> ss_threads_;

    // liveness (see Watched)
    uint32_t hb_ms_ = 0, peer_timeout_ms_ = 0, stall_ms_ = 0;
    bool master_liveness_ = false; // the master runs the protocol (its registration response carried the parameters)
    std::mutex live_mtx_;
    std::condition_variable live_cv_;
    bool live_stop_ = false;
    std::chrono::steady_clock::time_point last_dump_{}; // PCCL_CLIENT_DUMP_SEC (liveness thread only)
    std::map<const OpState *, Watched> watched_;
    std::thread liveness_thread_;
    std::atomic<uint64_t> stall_reports_{0}, stall_fails_{0}, master_lost_{0}, heartbeats_{0};

    // benchmark server
    std::mutex bm_mtx_;
    std::optional<Uuid> bm_peer_;
    std::atomic<int> bm_running_{0};
    std::vector<std::thread> bm_threads_;
};

} // namespace pccl::client
