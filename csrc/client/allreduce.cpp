// All-reduce: op orchestration (master consensus) + pipelined ring reduce-scatter/all-gather over multiplexed TCP.
//
// Algorithm (reference ccoip/src/cpp/reduce.cpp:528-784): chunk r = [r*base + min(r, rem), ...), ws-1 reduce-scatter
// steps sending chunk (rank - step) and accumulating chunk (rank - step - 1), then ws-1 all-gather steps forwarding the
// owned chunk. With quantization the owner quantizes its finished chunk once, overwrites its own copy with
// D(Q(x)) (so every peer ends bit-identical), and received quantized chunks are forwarded verbatim.
//
// Two implementations of the same wire protocol:
//  * host ring: buffers in host memory; frames are received straight into the destination (all-gather) or a pooled
//    receive buffer (reduce-scatter); arrived elements are reduced while the rest of the chunk is still in flight.
//  * device ring: buffers in HBM. The chunk to send is copied to pinned host memory in pieces on a HIP stream and
//    each piece is sent as soon as its event completes; received bytes land in pinned memory and HIP kernels reduce /
//    de-quantize them straight from pinned memory into HBM (zero-copy over PCIe), overlapped with the socket.
#include <algorithm>
#include <atomic>
#include <array>
#include <map>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <chrono>
#include <cstring>
#include <string>

#include "../common/log.hpp"
#include "../common/spin.hpp"
#include "../kernels/host_kernels.hpp"
#include "client.hpp"
#include "../common/trace.hpp"
#include "ipc.hpp"
#include "pools.hpp"

namespace pccl::client {

using namespace proto;
using namespace std::chrono_literals;

StreamPool &stream_pool() {
    static auto *p = new StreamPool(); // never destroyed: streams may outlive static destruction order
    return *p;
}
EventPool &event_pool() {
    static auto *p = new EventPool();
    return *p;
}

BufferPool &host_pool() {
    static BufferPool p(BufferPool::Kind::Host);
    return p;
}
BufferPool &pinned_pool() {
    static BufferPool p(BufferPool::Kind::Pinned);
    return p;
}
BufferPool &device_pool() {
    static BufferPool p(BufferPool::Kind::Device);
    return p;
}

// quantized device ring: min / max of a step's payload folded from the previous step's fused partials (pcclxQuantStats)
static std::atomic<uint64_t> g_quant_minmax_folds{0}, g_quant_minmax_passes{0};

static std::vector<std::pair<size_t, size_t>> chunk_bounds(size_t total, size_t ws) {
    std::vector<std::pair<size_t, size_t>> b(ws);
    const size_t base = total / ws, rem = total % ws;
    size_t cur = 0;
    for (size_t r = 0; r < ws; ++r) {
        const size_t n = base + (r < rem ? 1 : 0);
        b[r] = {cur, cur + n};
        cur += n;
    }
    return b;
}

namespace {
bool use_small_path(size_t bytes, size_t ws);
} // namespace

bool Client::abort_received(uint64_t tag) {
    auto p = master_.receive<M2CCollectiveCommsAbort>([tag](const M2CCollectiveCommsAbort &a) { return a.tag == tag; },
                                                       0ms);
    return p.has_value();
}

// ------------------------------------------------------------------------------------------------------------------
// op orchestration
// ------------------------------------------------------------------------------------------------------------------
OpWorkers::~OpWorkers() {
    {
        std::lock_guard l(m_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : threads_)
        if (t.joinable()) t.join();
}

// Bounded like the reference's collective thread pool (PCCL_MAX_CONCURRENT_COLLECTIVE_OPS, default 16; reference
// ccoip_client_state.hpp:17-25): a new worker starts only while fewer than the bound exist; otherwise the op waits
// in the FIFO queue. Ops start in submission order, so peers that issue the same tag sequence dequeue it in the same
// order (a worker blocked in the commence of tag X never starves the peers' tag X).
size_t OpWorkers::max_workers() {
    static const size_t v = std::max<size_t>(1, env_size("PCCL_MAX_CONCURRENT_COLLECTIVE_OPS", 16));
    return v;
}

void OpWorkers::submit(std::function<void()> fn) {
    std::lock_guard l(m_);
    q_.push_back(std::move(fn));
    if (q_.size() > idle_ && threads_.size() < max_workers()) {
        threads_.emplace_back([this] {
            name_thread("pccl-op");
            loop();
        });
    } else {
        cv_.notify_one();
    }
}

size_t OpWorkers::thread_count() {
    std::lock_guard l(m_);
    return threads_.size();
}

void OpWorkers::loop() {
    std::unique_lock l(m_);
    while (true) {
        ++idle_;
        cv_.wait(l, [this] { return stop_ || !q_.empty(); });
        --idle_;
        if (q_.empty()) return; // stop requested and nothing left to run
        auto fn = std::move(q_.front());
        q_.pop_front();
        l.unlock();
        fn();
        l.lock();
    }
}

bool Client::all_reduce_async(const ReduceRequest &req, bool inline_run) {
    if (!accepted_) return false;
    std::shared_ptr<OpState> op;
    {
        std::lock_guard lock(ops_mtx_);
        auto it = ops_.find(req.tag);
        if (it != ops_.end()) {
            if (!it->second->joined.load()) return false; // tag in use until its op has been awaited
            ops_.erase(it);
        }
        op = std::make_shared<OpState>();
        op->req = req;
        op->revision_at_start = conn_revision_.load();
        ops_[req.tag] = op;
    }
    if (inline_run) {
        run_op(op);
    } else {
        if (!fault_delay_armed()) initiate_op(*op);
        workers_.submit([this, op] { run_op(op); });
    }
    return true;
}

// Snapshot of the ring, the buffers' location and the initiate packet. The ring cannot change while the op is
// registered (re-establishment waits for running ops), so the view taken here is the one the op executes on.
void Client::initiate_op(OpState &op) {
    op.initiated = true;
    op.rv = ring_view(0);
    if (DeviceBackend *be = device_backend()) {
        be->pointer_info(op.req.src, op.si);
        be->pointer_info(op.req.dst, op.di);
    }
    // an empty op moves no data: the host ring runs its protocol without touching either buffer
    op.device = op.req.count > 0 && op.si.is_device && op.di.is_device && op.si.device == op.di.device;
    C2MCollectiveCommsInitiate init;
    init.tag = op.req.tag;
    init.count = op.req.count;
    init.data_type = op.req.dtype;
    init.op = op.req.op;
    const auto &rv = op.rv;
    if (rv && rv->hier && op.device) init.flags |= kCollFlagHierarchical;
    if (rv && rv->ring.size() >= 2 && use_small_path(op.req.count * dtype_size(op.req.dtype), rv->ring.size()) &&
        (op.req.qalgo == QuantAlgo::None || op.req.qtype == op.req.dtype))
        init.flags |= kCollFlagSmallPath;
    op.init_sent = master_.send(init);
}

void Client::run_op(const std::shared_ptr<OpState> &op) {
    const uint64_t tag = op->req.tag;
    low_timer_slack();
    if (!op->initiated) {
        fault_delay(tag);
        initiate_op(*op);
    }
    OpTrace trace;
    current_trace() = trace_ops_enabled() ? &trace : nullptr;
    char range_name[96];
    std::snprintf(range_name, sizeof(range_name), "pccl all_reduce tag %llu bytes %zu",
                  static_cast<unsigned long long>(tag), op->req.count * dtype_size(op->req.dtype));
    RoctxRange range(range_name);
    bool success = false, abort_seen = false;
    uint64_t seq = 0;
    bool commenced = false;
    uint8_t agreed = 0;
    const auto &rv = op->rv;
    const DevPtrInfo &si = op->si, &di = op->di;
    const bool device = op->device;
    if (op->init_sent) {
        auto c = master_.receive<M2CCollectiveCommsCommence>(
            [tag](const M2CCollectiveCommsCommence &p) { return p.tag == tag; });
        if (c) {
            seq = c->seq_nr;
            agreed = c->flags;
            op->small_path = (agreed & kCollFlagSmallPath) != 0;
            commenced = true;
            trace_mark("commence");
        }
    }
    if (commenced) {
        if (rv && rv->ring.size() >= 2) {
            op->world = static_cast<uint32_t>(rv->ring.size());
            std::pair<bool, bool> r{false, false};
            bool done = false;
            if ((agreed & kCollFlagHierarchical) && rv->hier) {
                // every participant announced the capability (master AND): IPC inside hosts, TCP ring across them
                r = hier_reduce(*op, *rv, seq, di.device);
                done = true;
                if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::Hierarchical);
            } else if (rv->arena) {
                // every peer of an intra-node ring votes; the xGMI path runs only if all buffers are on GPUs
                const int decision = rv->arena->vote(*this, *op, seq, device, device ? di.device : -1);
                trace_mark("vote");
                if (decision == IpcArena::kUseIpc) {
                    r = ipc_reduce(*op, *rv, seq, di.device);
                    done = true;
                    if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::DeviceIpc);
                } else if (decision == IpcArena::kAborted || decision == IpcArena::kAbortedByMaster) {
                    r = {false, decision == IpcArena::kAbortedByMaster || abort_received(tag)};
                    done = true;
                }
            }
            if (!done) {
                if (device) {
                    r = ring_reduce_device(*op, *rv, seq, di.device);
                    if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::DeviceRing);
                } else if ((!si.is_device && !di.is_device) || op->req.count == 0) {
                    r = ring_reduce_host(*op, *rv, seq);
                    if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::HostRing);
                } else {
                    LOG(ERR) << "all-reduce: send and receive buffers must both be host or both be on one GPU";
                    r = {false, false};
                }
            }
            success = r.first && !r.second;
            abort_seen = r.second;
            if (success) fault_point("op_end", seq); // this peer's part is done, the master has no verdict yet
        } else {
            LOG(WARN) << "all-reduce tag " << tag << ": no usable ring (peers lost)";
        }
    }
    // completion protocol: exactly one Abort(tag) packet per op, then Complete(tag)
    bool ok = false;
    if (commenced) {
        C2MCollectiveCommsComplete comp;
        comp.tag = tag;
        comp.was_aborted = !success;
        if (master_.send(comp)) {
            bool aborted = abort_seen;
            bool got_abort = abort_seen;
            if (!got_abort) {
                auto a = master_.receive<M2CCollectiveCommsAbort>(
                    [tag](const M2CCollectiveCommsAbort &p) { return p.tag == tag; });
                if (a) {
                    got_abort = true;
                    aborted = a->aborted;
                }
            }
            auto c = master_.receive<M2CCollectiveCommsComplete>(
                [tag](const M2CCollectiveCommsComplete &p) { return p.tag == tag; });
            ok = got_abort && c.has_value() && !aborted && success;
        }
    }
    if (!ok) {
        LOG(WARN) << "all-reduce tag " << tag << " failed/aborted";
    }
    if (op->settle) {
        op->settle(!ok);
        op->settle = nullptr;
    }
    if (current_trace()) {
        trace.mark("complete");
        static const char *names[] = {"none", "host_ring", "device_ring", "ipc", "hier", "?", "?", "?"};
        std::fprintf(stderr, "[pccl-trace] tag %llu seq %llu bytes %zu world %u path %s %s%s\n",
                     static_cast<unsigned long long>(tag), static_cast<unsigned long long>(seq),
                     op->req.count * dtype_size(op->req.dtype), op->world, names[last_path_.load() & 7],
                     ok ? "ok" : "FAILED", trace.str().c_str());
        current_trace() = nullptr;
    }
    op->success = ok;
    op->rv.reset(); // the snapshot's connections must not outlive the op (a re-established ring closes them)
    op->finish();
    {
        std::lock_guard l(done_mtx_);
    }
    done_cv_.notify_all();
}

std::optional<uint64_t> Client::wait_any(const std::vector<uint64_t> &tags, std::chrono::milliseconds timeout) {
    std::vector<std::shared_ptr<OpState>> ops;
    {
        std::lock_guard lock(ops_mtx_);
        for (uint64_t t : tags) {
            auto it = ops_.find(t);
            ops.push_back(it == ops_.end() ? nullptr : it->second);
        }
    }
    const auto deadline = std::chrono::steady_clock::now() + timeout;
    std::unique_lock l(done_mtx_);
    while (true) {
        bool any_known = false;
        for (size_t i = 0; i < ops.size(); ++i) {
            if (!ops[i]) continue;
            any_known = true;
            if (ops[i]->done.load()) return tags[i];
        }
        if (!any_known) return std::nullopt;
        if (done_cv_.wait_until(l, deadline) == std::cv_status::timeout) return std::nullopt;
    }
}

bool Client::join_async_reduce(uint64_t tag) {
    std::shared_ptr<OpState> op;
    {
        std::lock_guard lock(ops_mtx_);
        auto it = ops_.find(tag);
        if (it == ops_.end()) return false;
        op = it->second;
    }
    op->wait();
    op->joined.store(true);
    if (!op->success) {
        // Re-establish the ring once per connection revision: every peer sees the same failures, so every peer
        // performs exactly one establishment round (several concurrent failed ops must not cascade into more).
        // Ops still in flight keep this peer in the master's COLLECTIVE_COMMUNICATIONS_RUNNING state, where an
        // establish vote is illegal; the last failed op to be joined performs the round instead.
        std::lock_guard lock(establish_mtx_);
        if (conn_revision_.load() == op->revision_at_start && !interrupted_ && !any_collective_running()) {
            if (!request_and_establish_locked(false)) {
                LOG(ERR) << "Failed to re-establish P2P connections after abort";
            }
        }
        return false;
    }
    return true;
}

bool Client::get_reduce_info(uint64_t tag, ReduceInfo &out) {
    std::lock_guard lock(ops_mtx_);
    auto it = ops_.find(tag);
    if (it == ops_.end() || it->second->info_taken) return false;
    out.world_size = it->second->world;
    out.tx_bytes = it->second->tx.load();
    out.rx_bytes = it->second->rx.load();
    it->second->info_taken = true;
    if (it->second->done.load()) ops_.erase(it);
    return true;
}

// ------------------------------------------------------------------------------------------------------------------
// shared step machinery
// ------------------------------------------------------------------------------------------------------------------
namespace {

// Quantized ring protocol. The buffer is split into lanes (quant_lane_bounds), each a complete ring all-reduce over
// a contiguous part with its own data tag (lane_tag) and its own metadata tag (meta_tag). Per ring step a peer sends
// the step's dequantization metadata packet on the metadata tag (on connection seq % pool) and the quantized payload
// striped on the data tag. Keeping the packets off the data tag lets a peer post every receive sink of a step (and
// the next step's) before the packet arrives: the reference sends the packet on the data tag and waits for the peer's
// before any data moves (reference reduce.cpp:154-192), one extra latency per ring step. Host and device rings speak
// the same protocol, so CPU and GPU peers mix in one quantized ring.
constexpr uint64_t kMetaTagBit = 1ull << 63;
inline uint64_t lane_tag(uint64_t tag, size_t lane, size_t lanes) {
    return tag ^ (static_cast<uint64_t>(lane) << 60) ^ (static_cast<uint64_t>(lanes - 1) << 58);
}
inline uint64_t meta_tag(uint64_t data_tag) { return data_tag ^ kMetaTagBit; }

// Lane split of a quantized all-reduce of `count` elements (wire element size `qs`) over `ws` peers: element offsets
// lo[0] = 0 < lo[1] < ... < lo[nl] = count. A quantized reduce-scatter step must receive and reduce its whole chunk
// before the next step's min / max, and so its metadata and payload, exist: a single ring leaves its links idle for
// a step's fill and drain at every step, and further lanes fill each other's gaps. Depends only on values every peer
// shares (element count, ring size, wire type, PCCL_QUANT_LANES, which must match on all peers).
std::vector<size_t> quant_lane_bounds(size_t count, size_t ws, size_t qs) {
    constexpr size_t kMinLaneChunk = 8u << 20; // wire bytes per ring chunk and lane
    const size_t max_lanes = std::max<size_t>(1, std::min<size_t>(4, env_size("PCCL_QUANT_LANES", 2)));
    const size_t nl = std::min(max_lanes, std::max<size_t>(1, count / std::max<size_t>(1, ws) * qs / kMinLaneChunk));
    std::vector<size_t> lo(nl + 1, 0);
    for (size_t k = 1; k < nl; ++k) lo[k] = count / nl * k / 4096 * 4096;
    lo[nl] = count;
    return lo;
}

// finer per-step marks for PCCL_TRACE_OPS (global step g < 32): `kind` q = payload metadata known and its quantize
// kernels queued, f = first received piece consumed
void step_sub_mark(char kind, size_t g) {
    if (g >= 32 || !current_trace()) return;
    static const auto names = [] {
        auto *v = new std::vector<std::string>();
        for (char k : {'q', 'f'})
            for (int i = 0; i < 32; ++i) v->push_back(std::string(1, k) + std::to_string(i));
        return v;
    }();
    trace_mark((*names)[(kind == 'q' ? 0 : 32) + g].c_str());
}

// Abort state of one op shared by all of its threads: the master's abort packet for a tag is consumed by the first
// poll that sees it (Client::abort_received), so that poll records it here for every other thread of the op.
class OpAbort {
public:
    explicit OpAbort(std::function<bool()> poll) : poll_(std::move(poll)) {}
    bool operator()() {
        if (seen_.load(std::memory_order_acquire)) return true;
        std::lock_guard l(m_);
        if (seen_.load(std::memory_order_acquire)) return true;
        if (!poll_()) return false;
        seen_.store(true, std::memory_order_release);
        return true;
    }

private:
    std::function<bool()> poll_;
    std::mutex m_;
    std::atomic<bool> seen_{false};
};

// the connections a quantized step's metadata packet travels on, and its tag
struct StepIo {
    net::MuxConn *tx;
    net::MuxConn *rx;
    uint64_t tag; // metadata tag
    uint64_t seq;
};

constexpr size_t kMetaFrameOverhead = 24;

// Returns 0 ok, 1 io failure.
int send_meta(const StepIo &io, const QuantMeta &mine, std::atomic<uint64_t> &tx) {
    P2PDequantizationMeta pkt;
    pkt.tag = io.tag ^ kMetaTagBit; // the lane's data tag
    pkt.meta = mine;
    auto bytes = encode_with_id(pkt);
    if (!io.tx->send_frame(io.tag, io.seq, bytes.data(), bytes.size())) return 1;
    tx += bytes.size() + kMetaFrameOverhead;
    return 0;
}

// Waits for the peer's metadata of the next step (the packets of a lane arrive in step order). Returns 0 ok, 1 io
// failure, 2 abort.
int recv_meta(const StepIo &io, QuantMeta &theirs, std::atomic<uint64_t> &rx, const std::function<bool()> &aborted,
              const std::function<bool()> &failed = {}) {
    while (true) {
        auto m = io.rx->recv_packet<P2PDequantizationMeta>(io.tag, io.seq, 20ms);
        if (m) {
            theirs = m->meta;
            rx += encode_with_id(*m).size() + kMetaFrameOverhead;
            return 0;
        }
        if (!io.rx->is_open() || (failed && failed())) return 1;
        if (aborted()) return 2;
    }
}

// Striping: a large ring-step payload is split into up to PCCL_RING_STRIPES contiguous stripes, each sent on its own
// pooled TCP connection by its own thread (one loopback/WAN TCP stream tops out well below the NIC / memory
// bandwidth). Stripe boundaries depend only on (bytes, connection count, alignment), so sender and receiver derive
// the same plan: the sender's pool to `next` is exactly the receiver's RX pool from `prev`.
struct StripePlan {
    std::vector<size_t> off, len;
};

// (read per step: cheap next to a ring step, and lets tests / tuning change them at runtime)
size_t ring_stripes() { return std::max<size_t>(1, std::min<size_t>(16, env_size("PCCL_RING_STRIPES", 4))); }
size_t stripe_min_bytes() { return std::max<size_t>(1 << 20, env_size("PCCL_STRIPE_MIN_BYTES", 8u << 20)); }
constexpr size_t kStripeAlign = 1 << 20; // multiple of every element size and of the device staging piece

// Connection of stripe k of op `seq` (data tag `tag`) in a pool of `pool`: consecutive ops, and the lanes of one
// quantized op (lane_tag: lane in bits 60-61, lane count - 1 in bits 58-59), start PCCL_RING_STRIPES connections
// apart, so concurrent ops spread over the whole pool instead of piling onto its first connections (a long-fat-pipe
// link is filled by many concurrent ops, reference src/pccl.cpp:345-523). Sender and receiver derive the same index.
size_t stripe_conn(uint64_t seq, uint64_t tag, size_t k, size_t pool) {
    const uint64_t lanes = ((tag >> 58) & 3) + 1, lane = (tag >> 60) & 3;
    const uint64_t base = (seq * lanes + lane) * ring_stripes();
    return static_cast<size_t>((base + k) % pool);
}

StripePlan plan_stripes(size_t bytes, size_t conns) {
    StripePlan s;
    size_t p = std::min({ring_stripes(), std::max<size_t>(1, conns), std::max<size_t>(1, bytes / stripe_min_bytes())});
    const size_t per = (bytes / p + kStripeAlign - 1) / kStripeAlign * kStripeAlign;
    size_t off = 0;
    for (size_t k = 0; k < p && (off < bytes || k == 0); ++k) {
        const size_t n = (k + 1 == p) ? bytes - off : std::min(per, bytes - off);
        s.off.push_back(off);
        s.len.push_back(n);
        off += n;
    }
    return s;
}

// One full-duplex ring step over the striped connections. `tx_ready(end)` blocks until payload bytes [0, end) of the
// calling stripe may be sent; `consume(a, b)` processes received elements [a, b) (called from this thread only, any
// order across stripes, in order within a stripe, in batches of at least `gran` bytes unless a stripe ends).
// `before_rx` (optional) runs after the senders started and the receive sinks are posted, before anything is consumed
// (the quantized steps receive the peer's metadata there). Returns 0 ok, 1 io failure, 2 abort.
// Stripes are sent by each connection's persistent sender thread (MuxConn::post_send_job); steps of at most
// kInlineSendBytes are sent on the calling thread after the sinks are posted.
constexpr size_t kInlineSendBytes = 256 << 10;

struct CountDown {
    std::mutex m;
    std::condition_variable cv;
    size_t n = 0;
    void done() {
        std::lock_guard l(m);
        if (--n == 0) cv.notify_all();
    }
    void wait() {
        std::unique_lock l(m);
        cv.wait(l, [&] { return n == 0; });
    }
};

int striped_step(const std::vector<std::shared_ptr<net::MuxConn>> &txs,
                 const std::vector<std::shared_ptr<net::MuxConn>> &rxs, uint64_t tag, uint64_t seq,
                 const uint8_t *payload, size_t tx_bytes, const std::function<bool(size_t)> &tx_ready, uint8_t *sink,
                 size_t rx_bytes, size_t elem, size_t frame, const std::function<void(size_t, size_t)> &consume,
                 const std::function<bool()> &aborted, std::atomic<uint64_t> &tx_ctr, std::atomic<uint64_t> &rx_ctr,
                 const std::function<int()> &before_rx = {}, size_t gran = 0) {
    const StripePlan tp = plan_stripes(tx_bytes, txs.size());
    const StripePlan rp = plan_stripes(rx_bytes, rxs.size());
    auto rx_conn = [&](size_t k) { return rxs[stripe_conn(seq, tag, k, rxs.size())].get(); };
    auto tx_conn = [&](size_t k) { return txs[stripe_conn(seq, tag, k, txs.size())].get(); };
    bool sinks_posted = false;
    auto remove_sinks = [&] {
        if (!sinks_posted) return;
        for (size_t k = 0; k < rp.off.size(); ++k) rx_conn(k)->remove_sink(tag);
    };

    std::atomic<int> send_rc{0};
    auto send_stripe = [&](size_t k) {
        net::MuxConn *c = tx_conn(k);
        const size_t base = tp.off[k], len = tp.len[k];
        for (size_t sent = 0; sent < len && send_rc.load(std::memory_order_relaxed) == 0;) {
            const size_t n = std::min(frame, len - sent);
            if (!tx_ready(base + sent + n) || !c->send_frame(tag, seq, payload + base + sent, n)) {
                send_rc.store(1);
                return;
            }
            sent += n;
            tx_ctr += n;
        }
    };
    const bool inline_send = tx_bytes <= kInlineSendBytes;
    CountDown senders;
    if (!inline_send) {
        for (size_t k = 0; k < tp.off.size(); ++k)
            if (tp.len[k] > 0) ++senders.n;
        for (size_t k = 0; k < tp.off.size(); ++k)
            if (tp.len[k] > 0)
                tx_conn(k)->post_send_job([&, k] {
                    send_stripe(k);
                    senders.done();
                });
    }
    // (a quantized step's metadata packet travels on its own tag: no sink of this step can swallow it)
    for (size_t k = 0; k < rp.off.size(); ++k) rx_conn(k)->post_sink(tag, seq, sink + rp.off[k], rp.len[k]);
    sinks_posted = true;
    if (before_rx) {
        if (const int brc = before_rx()) {
            send_rc.store(brc);
            senders.wait();
            remove_sinks();
            return brc;
        }
    }
    if (inline_send)
        for (size_t k = 0; k < tp.off.size(); ++k)
            if (tp.len[k] > 0) send_stripe(k);

    const size_t gran_el = std::max<size_t>(1, gran / elem);
    std::vector<size_t> done(rp.off.size(), 0); // elements consumed per stripe
    size_t remaining = rp.off.size();
    for (size_t k = 0; k < rp.off.size(); ++k)
        if (rp.len[k] == 0) --remaining;
    int rc = 0;
    size_t idle = 0, rr = 0;
    while (remaining > 0) {
        bool progress = false;
        for (size_t k = 0; k < rp.off.size(); ++k) {
            const size_t want = rp.len[k] / elem;
            if (done[k] >= want) continue;
            const size_t have = rx_conn(k)->sink_progress(tag) / elem;
            if (have > done[k] && (have - done[k] >= gran_el || have >= want)) {
                const size_t e0 = rp.off[k] / elem;
                consume(e0 + done[k], e0 + have);
                done[k] = have;
                progress = true;
                if (done[k] >= want) --remaining;
            }
        }
        if (remaining == 0 || progress) {
            idle = 0;
            continue;
        }
        // block on one unfinished stripe (round robin) until its next batch is complete or a short timeout
        size_t k = rr++ % rp.off.size();
        while (done[k] >= rp.len[k] / elem) k = rr++ % rp.off.size();
        net::MuxConn *c = rx_conn(k);
        c->wait_sink(tag, std::min(rp.len[k], (done[k] + gran_el) * elem), 5ms);
        if (!c->is_open() || send_rc.load() != 0) {
            rc = 1;
            break;
        }
        if (++idle % 8 == 0 && aborted()) {
            rc = 2;
            break;
        }
    }
    if (rc != 0) {
        send_rc.store(rc);
        // senders stuck in send() on a dead peer return once the connection is torn down
        senders.wait();
        remove_sinks();
        return rc;
    }
    senders.wait();
    remove_sinks();
    if (send_rc.load() != 0) return 1;
    rx_ctr += rx_bytes;
    return 0;
}

// Small all-reduces: the whole vector travels W-1 ring hops (all-gather) and every peer reduces the W vectors locally
// in ring-index order, instead of 2(W-1) hops of 1/W pieces. Such ops are bound by per-hop latency (socket wake-ups,
// and on the device ring per-step staging copies), not bytes, so this halves their critical path; every peer reduces
// the same vectors in the same order, so results stay bit-identical across peers. Taken when the vector is at most
// PCCL_SMALL_ALLREDUCE_BYTES (default 1 MiB; must match on every peer) and the all-gather sends at most 8x that
// (W-1 copies). Measured on MI355X, 8 peers, TCP device ring (profiles/r2/small_messages/): 64 KiB 1770 -> 547 us,
// 256 KiB 2822 -> 921 us, 1 MiB 2968 -> 2496 us, 4 MiB 4182 -> 10277 us (hence the cap).
// Returns 0 ok, 1 io failure, 2 abort; `dst` is written only after every hop succeeded.
bool use_small_path(size_t bytes, size_t ws) {
    const size_t lim = env_size("PCCL_SMALL_ALLREDUCE_BYTES", 1u << 20);
    return bytes <= lim && bytes * (ws - 1) <= 8 * lim;
}

int small_allgather_reduce(const std::vector<std::shared_ptr<net::MuxConn>> &txs,
                           const std::vector<std::shared_ptr<net::MuxConn>> &rxs, uint64_t tag, uint64_t seq,
                           const void *src, void *dst, size_t count, DType dt, ReduceOp op, size_t ws, size_t rank,
                           const std::function<bool()> &aborted, std::atomic<uint64_t> &tx_ctr,
                           std::atomic<uint64_t> &rx_ctr) {
    const size_t es = dtype_size(dt), bytes = count * es;
    Lease all(host_pool(), std::max<size_t>(ws * bytes, 64));
    if (!all.ok()) return 1;
    uint8_t *v = all.data();
    std::memcpy(v + rank * bytes, src, bytes);
    for (size_t step = 0; step + 1 < ws; ++step) {
        const size_t send_idx = (rank + ws - step) % ws, recv_idx = (rank + ws - step - 1) % ws;
        const int rc = striped_step(txs, rxs, tag, seq, v + send_idx * bytes, bytes, [](size_t) { return true; },
                                    v + recv_idx * bytes, bytes, es, std::max<size_t>(bytes, 1),
                                    [](size_t, size_t) {}, aborted, tx_ctr, rx_ctr);
        if (rc) return rc;
    }
    std::memcpy(dst, v, bytes);
    for (size_t k = 1; k < ws; ++k)
        if (!kernels::host_reduce(dst, v + k * bytes, count, dt, op)) return 1;
    if (op == ReduceOp::Avg) kernels::host_finalize_avg(dst, count, dt, ws);
    return 0;
}

} // namespace

// ------------------------------------------------------------------------------------------------------------------
// host ring
// ------------------------------------------------------------------------------------------------------------------
namespace {

// One ring all-reduce over host memory of `count` elements at `dst` (already holding the input) on data tag `tag`:
// the plain host ring, or one lane of a quantized ring (`quant`; metadata on meta_tag(tag)). Returns 0 ok, 1 io
// failure, 2 abort.
int host_ring(const std::vector<std::shared_ptr<net::MuxConn>> &txs, const std::vector<std::shared_ptr<net::MuxConn>> &rxs,
              size_t ws, size_t rank, uint64_t tag, uint64_t seq, uint8_t *dst, size_t count, const ReduceRequest &q,
              bool quant, const std::function<bool()> &aborted, std::atomic<uint64_t> &tx_ctr,
              std::atomic<uint64_t> &rx_ctr) {
    const size_t es = dtype_size(q.dtype);
    const size_t qs = quant ? dtype_size(q.qtype) : es;
    const size_t chunk = net::multiplex_chunk_size();
    StepIo io{txs[stripe_conn(seq, tag, 0, txs.size())].get(), rxs[stripe_conn(seq, tag, 0, rxs.size())].get(),
              meta_tag(tag), seq};

    const auto bounds = chunk_bounds(count, ws);
    size_t max_chunk = 0;
    for (auto &b : bounds) max_chunk = std::max(max_chunk, b.second - b.first);
    Lease rbuf(host_pool(), max_chunk * qs + 64);
    Lease qbuf;
    if (quant) qbuf = Lease(host_pool(), max_chunk * qs + 64);
    if (!rbuf.ok() || (quant && !qbuf.ok())) return 1;

    // One full-duplex (striped) step g (global: reduce-scatter 0 .. ws-2, then all-gather): sends `payload`,
    // receives `rx_bytes` into `sink`, calling `consume(from, to)` for newly complete received elements. Returns 0 ok,
    // 1 io failure, 2 abort. Fault points (tests): hring:<seq>:<g>:rx after the first consume, :end after the step.
    auto run_step = [&](size_t g, const uint8_t *payload, size_t tx_bytes, uint8_t *sink, size_t rx_bytes,
                        const std::function<void(size_t, size_t)> &consume,
                        const std::function<int()> &before_rx = {}) -> int {
        bool first = true;
        const int rc = striped_step(txs, rxs, tag, seq, payload, tx_bytes, [](size_t) { return true; }, sink, rx_bytes,
                                    qs, chunk, [&](size_t a, size_t b) {
                                        consume(a, b);
                                        if (first) {
                                            first = false;
                                            fault_point("hring", seq, g, "rx");
                                        }
                                    }, aborted, tx_ctr, rx_ctr, before_rx);
        if (rc == 0) fault_point("hring", seq, g, "end");
        return rc;
    };
    auto await_meta = [&](QuantMeta &theirs) { return [&, pt = &theirs] { return recv_meta(io, *pt, rx_ctr, aborted); }; };

    // ---- reduce-scatter
    for (size_t step = 0; step + 1 < ws; ++step) {
        const size_t tx_idx = (rank + ws - step) % ws, rx_idx = (rank + ws - step - 1) % ws;
        const auto [ts, te] = bounds[tx_idx];
        const auto [rs, re] = bounds[rx_idx];
        const uint8_t *payload = dst + ts * es;
        QuantMeta mine, theirs;
        if (quant) {
            if (te > ts) mine = kernels::host_quantize(qbuf.data(), dst + ts * es, te - ts, q.dtype, q.qtype, q.qalgo);
            else mine = kernels::make_meta(q.qalgo, q.dtype, q.qtype, 0, 0);
            payload = qbuf.data();
            if (int rc = send_meta(io, mine, tx_ctr)) return rc;
        }
        uint8_t *rx_region = dst + rs * es;
        const int rc = run_step(step, payload, (te - ts) * qs, rbuf.data(), (re - rs) * qs, [&](size_t a, size_t b) {
            if (quant)
                kernels::host_dequant_reduce(rx_region + a * es, rbuf.data() + a * qs, b - a, q.dtype, q.qtype, q.op, theirs);
            else
                kernels::host_reduce(rx_region + a * es, rbuf.data() + a * es, b - a, q.dtype, q.op);
        }, quant ? std::function<int()>(await_meta(theirs)) : std::function<int()>());
        if (rc) return rc;
    }

    trace_mark("reduce_scatter");
    // ---- all-gather
    Lease ag[2];
    if (quant) {
        ag[0] = Lease(host_pool(), max_chunk * qs + 64);
        ag[1] = Lease(host_pool(), max_chunk * qs + 64);
        if (!ag[0].ok() || !ag[1].ok()) return 1;
    }
    QuantMeta prev_meta;
    size_t cur = (rank + 1) % ws;
    for (size_t step = 0; step + 1 < ws; ++step) {
        const size_t inc = (cur + ws - 1) % ws;
        const auto [ts, te] = bounds[cur];
        const auto [rs, re] = bounds[inc];
        uint8_t *rx_region = dst + rs * es;
        int rc;
        if (quant) {
            QuantMeta mine, theirs;
            const uint8_t *payload;
            if (step == 0) {
                if (te > ts) {
                    mine = kernels::host_quantize(qbuf.data(), dst + ts * es, te - ts, q.dtype, q.qtype, q.qalgo);
                    // parity: our own copy becomes exactly what the other peers will de-quantize
                    kernels::host_dequant_reduce(dst + ts * es, qbuf.data(), te - ts, q.dtype, q.qtype, ReduceOp::Set, mine);
                } else {
                    mine = kernels::make_meta(q.qalgo, q.dtype, q.qtype, 0, 0);
                }
                payload = qbuf.data();
            } else {
                mine = prev_meta;
                payload = ag[(step - 1) % 2].data();
            }
            if (int m = send_meta(io, mine, tx_ctr)) return m;
            uint8_t *sink = ag[step % 2].data();
            rc = run_step(ws - 1 + step, payload, (te - ts) * qs, sink, (re - rs) * qs, [&](size_t a, size_t b) {
                kernels::host_dequant_reduce(rx_region + a * es, sink + a * qs, b - a, q.dtype, q.qtype, ReduceOp::Set, theirs);
            }, await_meta(theirs));
            prev_meta = theirs;
        } else {
            rc = run_step(ws - 1 + step, dst + ts * es, (te - ts) * es, rx_region, (re - rs) * es, [](size_t, size_t) {});
        }
        if (rc) return rc;
        cur = inc;
    }
    return 0;
}

// Runs fn(lane, lo, hi) for every lane of `lo` (lane 0 on the calling thread); returns the worst lane result
// (abort 2 outranks io failure 1).
int run_lanes(const std::vector<size_t> &lo, const std::function<int(size_t, size_t, size_t)> &fn) {
    const size_t nl = lo.size() - 1;
    std::vector<int> rc(nl, 0);
    std::vector<std::thread> th;
    for (size_t k = 1; k < nl; ++k) th.emplace_back([&, k] {
        name_thread("pccl-ring-lane");
        rc[k] = fn(k, lo[k], lo[k + 1]);
    });
    rc[0] = fn(0, lo[0], lo[1]);
    for (auto &t : th) t.join();
    return *std::max_element(rc.begin(), rc.end());
}

} // namespace

std::pair<bool, bool> Client::ring_reduce_host(OpState &op, const RingView &rv, uint64_t seq) {
    const ReduceRequest &q = op.req;
    const size_t ws = rv.ring.size(), rank = rv.rank;
    const size_t es = dtype_size(q.dtype);
    const bool quant = q.qalgo != QuantAlgo::None && q.qtype != q.dtype;
    auto *dst = static_cast<uint8_t *>(q.dst);
    const size_t bytes = q.count * es;
    OpAbort aborted([this, t = q.tag] { return abort_received(t); });
    auto abort_fn = [&] { return aborted(); };

    // in place: a backup of the input, restored if the ring fails or the master aborts the op afterwards (settle)
    Lease backup;
    if (q.src == q.dst && !q.scratch && bytes) {
        backup = Lease(host_pool(), bytes);
        if (!backup.ok()) return {false, false};
        std::memcpy(backup.data(), q.src, bytes);
    }
    auto keep_backup = [&] {
        if (!backup.ok()) return;
        op.settle = [b = std::make_shared<Lease>(std::move(backup)), dst, bytes](bool restore) {
            if (restore) std::memcpy(dst, b->data(), bytes);
        };
    };
    if (!quant && op.small_path) { // writes dst only once every contribution arrived
        const int rc = small_allgather_reduce(rv.tx, rv.rx, q.tag, seq, q.src, dst, q.count, q.dtype, q.op, ws, rank,
                                              abort_fn, op.tx, op.rx);
        trace_mark("allgather_reduce");
        if (rc == 0) keep_backup();
        return {rc == 0, rc == 2};
    }
    if (q.src != q.dst && bytes) std::memcpy(dst, q.src, bytes);
    const std::vector<size_t> lo = quant ? quant_lane_bounds(q.count, ws, dtype_size(q.qtype))
                                         : std::vector<size_t>{0, q.count};
    const int rc = run_lanes(lo, [&](size_t k, size_t a, size_t b) {
        return host_ring(rv.tx, rv.rx, ws, rank, lane_tag(q.tag, k, lo.size() - 1), seq, dst + a * es, b - a, q, quant,
                         abort_fn, op.tx, op.rx);
    });
    if (rc) {
        if (backup.ok()) std::memcpy(dst, backup.data(), bytes); // every lane returned: nothing writes dst
        return {rc == 2, rc == 2};
    }
    if (q.op == ReduceOp::Avg) kernels::host_finalize_avg(dst, q.count, q.dtype, ws);
    keep_backup();
    return {true, false};
}

// ------------------------------------------------------------------------------------------------------------------
// device ring (HBM buffers, pinned staging, HIP kernels)
// ------------------------------------------------------------------------------------------------------------------
//
// PCIe is the device ring's second bottleneck after the network (8 peers on one GPU share one x16 link). Measured on
// MI355X (profiles/r2/pcie_probe.md): one copy-engine queue per direction reaches ~55 GB/s one way and ~94 GB/s full
// duplex with >= 4 MiB copies, while 4-8 queues per direction fall to ~60 GB/s duplex, kernels reading pinned host
// memory run at <= 57 GB/s and drop to ~60 GB/s duplex next to copy traffic, and a copy issued behind a kernel on
// the same stream becomes a blit kernel. Hence:
//   * every staging copy of the process goes to ONE host->device and ONE device->host stream per GPU (shared by all
//     ops and all peers of the process); nothing is queued behind a cross-stream wait there, so ROCclr keeps them on
//     the copy engines;
//   * reduce-scatter: received bytes are copied into HBM staging by the copy engine and reduced HBM->HBM on the op's
//     stream (cross-stream event wait, no host round trip) by k_reduce_copy, which also streams the result into
//     pinned memory as the NEXT step's payload: a ring step's sends start the moment the previous step's last piece
//     lands, and the only device->host copies left are the step-0 pieces of the input;
//   * all-gather: received chunks go to HBM as copies on the op's stream (blit kernels reading pinned memory, one per
//     peer in parallel, next to the shared copy-engine queue that carries the reduce-scatter's bytes): interleaved
//     A/B, 8 peers x 1 GiB: 347 vs 376 ms and 337 vs 342 ms (profiles/r3/h2d_modes/).
// PCIe bytes per peer and 1 GiB: D2H 1 GiB (step-0 payload + reduced pieces), H2D 1.75 GiB (received pieces).
// Round 3 measured the alternatives (several H2D queues, per-op queues, a process-wide reduce stream, CPU-reduced
// parts, kernels reading received bytes from pinned memory, lanes, a step-synchronous schedule): none was faster, so
// none is kept (profiles/r3/{ring_ab,h2d_modes,shared_reduce,host_reduce,grid_caps}/).

namespace {

struct PcieQueues {
    DevStream h2d = nullptr; // received pieces -> HBM staging
    DevStream d2h = nullptr; // step-0 payload pieces -> pinned
};

// process-wide copy queues of `device` (never destroyed: they may outlive static destruction order)
PcieQueues shared_pcie_queues(DeviceBackend *be, int device) {
    static std::mutex m;
    static auto *q = new std::map<int, PcieQueues>();
    std::lock_guard l(m);
    PcieQueues &e = (*q)[device];
    if (!e.h2d) {
        const int cur = be->current_device();
        be->set_device(device);
        e.h2d = be->create_stream();
        e.d2h = be->create_stream();
        if (cur >= 0) be->set_device(cur);
    }
    return e;
}

// per-step phase marks for PCCL_TRACE_OPS (first 16 steps of each phase)
void step_mark(bool reduce_scatter, size_t step) {
    static const char *rs[] = {"rs0", "rs1", "rs2", "rs3", "rs4", "rs5", "rs6", "rs7",
                               "rs8", "rs9", "rs10", "rs11", "rs12", "rs13", "rs14", "rs15"};
    static const char *ag[] = {"ag0", "ag1", "ag2", "ag3", "ag4", "ag5", "ag6", "ag7",
                               "ag8", "ag9", "ag10", "ag11", "ag12", "ag13", "ag14", "ag15"};
    if (step < 16) trace_mark(reduce_scatter ? rs[step] : ag[step]);
}

// Waits until every piece of work queued on `s` so far has completed, sleeping between polls (hipStreamSynchronize
// busy-waits: with 16 quantized lanes syncing once per ring step that took the process's CPU share from the socket
// copies)
bool stream_wait_polling(DeviceBackend *be, DevStream s) {
    DevEvent e = event_pool().get();
    const bool ok = be->event_record(e, s) && event_wait_polling(be, e);
    event_pool().put(e);
    return ok;
}

// payload bytes [a, b) of a pinned staging buffer become valid once `e` has completed (nullptr: already valid)
struct Staged {
    size_t a, b;
    DevEvent e;
};

// Readiness of one ring step's payload, shared between the op thread that produces it (staging copies, the fused
// reduce, received bytes) and the connections' sender threads that send it while it is still being produced
// (send-ahead). A range is readable once its event (nullptr: none) has completed. Ranges arrive in any order across
// the producer's stripes, and the sender's stripe plan need not match the producer's (neighbours may run different
// connection pool sizes), so a wait covers the whole byte range it sends.
struct ReadyRanges {
    std::mutex m;
    std::condition_variable cv; // signalled by add(): a waiting sender wakes when its range may be complete
    std::vector<Staged> v;
    void clear() {
        std::lock_guard l(m);
        v.clear();
    }
    void add(size_t a, size_t b, DevEvent e) {
        {
            std::lock_guard l(m);
            v.push_back({a, b, e});
        }
        cv.notify_all();
    }
    // blocks until every byte of [begin, end) is readable; false if `cancel` became non-zero first
    bool wait(size_t begin, size_t end, DeviceBackend *be, const std::atomic<int> &cancel) {
        if (end <= begin) return true;
        std::vector<std::pair<size_t, size_t>> iv;
        std::vector<DevEvent> evs;
        while (true) {
            bool covered = false;
            {
                std::unique_lock l(m);
                iv.clear();
                evs.clear();
                for (const auto &r : v)
                    if (r.b > begin && r.a < end) {
                        iv.emplace_back(r.a, r.b);
                        if (r.e) evs.push_back(r.e);
                    }
                std::sort(iv.begin(), iv.end());
                size_t cur = begin;
                for (const auto &[a, b] : iv) {
                    if (a > cur) break;
                    cur = std::max(cur, b);
                }
                covered = cur >= end;
                if (!covered) {
                    if (cancel.load(std::memory_order_relaxed) != 0) return false;
                    cv.wait_for(l, std::chrono::milliseconds(1)); // (cancel is polled, not signalled)
                    continue;
                }
            }
            for (DevEvent e : evs)
                if (!event_wait_polling(be, e)) return false;
            return true;
        }
    }
};

// The send side of one pipelined ring op: one thread per stripe for the whole op (not per step), each sending its
// stripe of every step in order over connection stripe_conn(seq, tag, k). The op thread publishes step g (payload, bytes,
// readiness) as soon as step g may start sending — with send-ahead while step g-1 still receives — and a stripe thread
// streams each piece once it is readable. Per-op threads instead of the connections' shared sender threads: a stripe
// thread may wait on its op's network progress (the previous peer's data), which must never hold up another op's
// sends queued on the same connection (two peers with concurrent ops could otherwise wait on each other).
class OpSenders {
public:
    struct Step {
        const uint8_t *payload = nullptr;
        size_t bytes = 0;
        ReadyRanges *ready = nullptr;
    };
    OpSenders(const std::vector<std::shared_ptr<net::MuxConn>> &txs, uint64_t tag, uint64_t seq, size_t frame,
              size_t nsteps, size_t max_stripes, DeviceBackend *be, std::atomic<uint64_t> &tx_ctr)
        : txs_(txs), tag_(tag), seq_(seq), frame_(frame), be_(be), tx_ctr_(tx_ctr), steps_(nsteps),
          done_(nsteps) {
        for (size_t k = 0; k < max_stripes; ++k) th_.emplace_back([this, k] {
            name_thread("pccl-stripe-tx");
            run(k);
        });
    }
    ~OpSenders() {
        cancel();
        for (auto &t : th_) t.join();
    }
    // step g may be sent from now on (steps are published in order)
    void publish(size_t g, const Step &st) {
        const StripePlan tp = plan_stripes(st.bytes, txs_.size());
        size_t n = 0;
        for (size_t k = 0; k < tp.off.size(); ++k)
            if (tp.len[k] > 0) ++n;
        {
            std::lock_guard l(m_);
            steps_[g] = st;
            done_[g] = n;
            published_ = g + 1;
        }
        cv_.notify_all();
    }
    bool published(size_t g) {
        std::lock_guard l(m_);
        return published_ > g;
    }
    // every stripe of step g has been sent (non-blocking)
    bool sent(size_t g) {
        std::lock_guard l(m_);
        return published_ > g && done_[g] == 0;
    }
    // blocks until every stripe of step g is sent; false on failure / cancel
    bool wait(size_t g) {
        std::unique_lock l(m_);
        cv_.wait(l, [&] { return rc_.load() != 0 || (published_ > g && done_[g] == 0); });
        return rc_.load() == 0;
    }
    // blocks until every stripe of every step is sent (a stripe with no bytes in the last step may still be sending
    // an earlier one); false on failure / cancel
    bool wait_all() {
        std::unique_lock l(m_);
        cv_.wait(l, [&] {
            if (rc_.load() != 0) return true;
            if (published_ < steps_.size()) return false;
            for (size_t d : done_)
                if (d != 0) return false;
            return true;
        });
        return rc_.load() == 0;
    }
    void cancel() {
        rc_.store(1);
        std::lock_guard l(m_);
        cv_.notify_all();
    }
    bool failed() const { return rc_.load() != 0; }

private:
    void run(size_t k) {
        for (size_t g = 0; g < steps_.size(); ++g) {
            Step st;
            {
                std::unique_lock l(m_);
                cv_.wait(l, [&] { return rc_.load() != 0 || published_ > g; });
                if (rc_.load() != 0) return;
                st = steps_[g];
            }
            const StripePlan tp = plan_stripes(st.bytes, txs_.size());
            if (k >= tp.off.size() || tp.len[k] == 0) continue;
            net::MuxConn *c = txs_[stripe_conn(seq_, tag_, k, txs_.size())].get();
            const size_t base = tp.off[k], len = tp.len[k];
            for (size_t sent = 0; sent < len;) {
                const size_t n = std::min(frame_, len - sent);
                if (!st.ready->wait(base + sent, base + sent + n, be_, rc_)) {
                    cancel();
                    return;
                }
                RoctxIoRange io("send");
                if (!c->send_frame(tag_, seq_, st.payload + base + sent, n)) {
                    cancel();
                    return;
                }
                sent += n;
                tx_ctr_ += n;
            }
            {
                std::lock_guard l(m_);
                --done_[g];
            }
            cv_.notify_all();
        }
    }
    const std::vector<std::shared_ptr<net::MuxConn>> &txs_;
    const uint64_t tag_, seq_;
    const size_t frame_;
    DeviceBackend *be_;
    std::atomic<uint64_t> &tx_ctr_;
    std::mutex m_;
    std::condition_variable cv_;
    std::vector<Step> steps_;
    std::vector<size_t> done_;
    size_t published_ = 0;
    std::atomic<int> rc_{0};
    std::vector<std::thread> th_;
};

// The receive side of one pipelined ring op: per step one sink per stripe on the connections from the previous peer.
// Sinks of a tag form a FIFO on each connection, so step g+1's sinks may be posted while step g still receives (the
// previous peer streams both steps back to back on every connection). Sinks never outlive the op: the destructor
// removes every posted one (declare a RingRx after the buffers its sinks point into).
class RingRx {
public:
    RingRx(const std::vector<std::shared_ptr<net::MuxConn>> &rxs, uint64_t tag, uint64_t seq, size_t nsteps)
        : rxs_(rxs), tag_(tag), seq_(seq), steps_(nsteps) {}
    ~RingRx() {
        for (size_t g = 0; g < steps_.size(); ++g) unpost(g);
    }
    RingRx(const RingRx &) = delete;
    RingRx &operator=(const RingRx &) = delete;

    bool posted(size_t g) const { return steps_[g].posted; }
    // step g receives `bytes` into `buf`
    void post(size_t g, uint8_t *buf, size_t bytes) {
        Step &r = steps_[g];
        r.rp = plan_stripes(bytes, rxs_.size());
        r.sinks.assign(r.rp.off.size(), nullptr);
        r.done.assign(r.rp.off.size(), 0);
        r.remaining = 0;
        for (size_t k = 0; k < r.rp.off.size(); ++k) {
            if (r.rp.len[k] == 0) continue;
            r.sinks[k] = conn(k)->post_sink(tag_, seq_, buf + r.rp.off[k], r.rp.len[k]);
            ++r.remaining;
        }
        r.posted = true;
    }
    void unpost(size_t g) {
        Step &r = steps_[g];
        if (!r.posted) return;
        for (size_t k = 0; k < r.sinks.size(); ++k)
            if (r.sinks[k]) conn(k)->remove_sink(tag_, r.sinks[k]);
        r.sinks.clear();
        r.posted = false;
    }
    // Receives step g: consume(a, b) for newly arrived bytes [a, b) of the step (multiples of `unit`, at least `gran`
    // bytes per call unless a stripe ends; in order within a stripe, any order across stripes). `between` runs after
    // every scan of the stripes (the caller posts the next step's sinks there). Returns 0 ok, 1 io failure (a
    // connection closed or `failed()`), 2 abort.
    int receive(size_t g, size_t unit, size_t gran, const std::function<void(size_t, size_t)> &consume,
                const std::function<void()> &between, const std::function<bool()> &failed,
                const std::function<bool()> &aborted) {
        Step &r = steps_[g];
        const size_t gb = std::max(unit, gran / unit * unit);
        size_t idle = 0, rr = 0;
        while (r.remaining > 0) {
            bool progress = false;
            for (size_t k = 0; k < r.sinks.size(); ++k) {
                if (!r.sinks[k]) continue;
                const size_t want = r.rp.len[k];
                if (r.done[k] >= want) continue;
                const size_t have = net::MuxConn::sink_progress(r.sinks[k]) / unit * unit;
                if (have > r.done[k] && (have - r.done[k] >= gb || have >= want)) {
                    consume(r.rp.off[k] + r.done[k], r.rp.off[k] + have);
                    r.done[k] = have;
                    progress = true;
                    if (have >= want) --r.remaining;
                }
            }
            if (between) between();
            if (r.remaining == 0 || progress) {
                idle = 0;
                continue;
            }
            // block on one unfinished stripe (round robin) until its next batch is complete or a short timeout
            size_t k = rr++ % r.sinks.size();
            while (!r.sinks[k] || r.done[k] >= r.rp.len[k]) k = rr++ % r.sinks.size();
            net::MuxConn *c = conn(k);
            c->wait_sink(r.sinks[k], std::min(r.rp.len[k], r.done[k] + gb), 5ms);
            if (!c->is_open() || (failed && failed())) return 1;
            if (++idle % 8 == 0 && aborted()) return 2;
        }
        return 0;
    }

private:
    struct Step {
        StripePlan rp;
        std::vector<net::MuxConn::SinkRef> sinks;
        std::vector<size_t> done; // bytes consumed per stripe
        size_t remaining = 0;     // stripes not yet fully consumed
        bool posted = false;
    };
    net::MuxConn *conn(size_t k) const { return rxs_[stripe_conn(seq_, tag_, k, rxs_.size())].get(); }
    const std::vector<std::shared_ptr<net::MuxConn>> &rxs_;
    const uint64_t tag_, seq_;
    std::vector<Step> steps_;
};

// chunk index a peer sends / receives at global ring step g (reduce-scatter steps 0 .. ws-2, then all-gather)
size_t ring_chunk_tx(size_t g, size_t rank, size_t ws) {
    return g + 1 < ws ? (rank + ws - g) % ws : (rank + 1 + ws - (g - (ws - 1)) % ws) % ws;
}
size_t ring_chunk_rx(size_t g, size_t rank, size_t ws) { return (ring_chunk_tx(g, rank, ws) + ws - 1) % ws; }

// inputs of one device-ring op
struct DevRing {
    const std::vector<std::shared_ptr<net::MuxConn>> &txs, &rxs; // the ring's connections to next / from prev
    size_t ws, rank;
    uint64_t tag, seq;
    DeviceBackend *be;
    PcieQueues pq;
    DevStream st;       // the op's stream (input copy / backup before any of the ring's work)
    const uint8_t *src; // step-0 payload source: the caller's input (ready at call time, never written by the op
                        // before its step-0 copies completed)
    uint8_t *dst;       // the output, holding the input once `st` reaches the ring's first kernel
    size_t count, es, piece;
    DType dtype;
    ReduceOp rop;
    int device;
    std::function<bool()> aborted;
    std::atomic<uint64_t> &tx, &rx;
};

// The device ring as one pipeline over all 2(W-1) steps: step g+1's payload is produced (reduced into pinned
// memory) and sent while step g still receives, and step g+1's sinks are posted as soon as their staging buffer is
// free. Returns 0 ok, 1 io failure, 2 abort; on return no GPU work or socket write of the op touches any of its
// buffers any more (the caller may restore the input).
int device_ring_pipeline(DevRing &R) {
    DeviceBackend *be = R.be;
    const PcieQueues pq = R.pq;
    DevStream st = R.st;
    const size_t ws = R.ws, rank = R.rank, es = R.es, piece = R.piece;
    const uint64_t seq = R.seq;

    std::vector<DevEvent> owned; // events of this op (back to the pool once everything they guard has completed)
    DevEvent last_d2h = nullptr;
    auto record = [&](DevStream s) {
        DevEvent e = event_pool().get();
        owned.push_back(e);
        be->event_record(e, s);
        return e;
    };
    const auto bounds = chunk_bounds(R.count, ws);
    size_t max_chunk = 0;
    for (auto &b : bounds) max_chunk = std::max(max_chunk, b.second - b.first);
    const size_t stage_bytes = max_chunk * es + 64;
    // Staging rings of kNb buffers: step g receives into rxbuf[g % kNb] (HBM twin rxdev[g % kNb] for the reduce) and
    // its reduce writes the next payload into txbuf[(g + 1) % kNb]. Three deep, because step g+1's sinks are posted
    // while step g still receives and step g+1's sends run while step g's do: a buffer is refilled only after the
    // step two back finished with it.
    constexpr size_t kNb = 3;
    Lease txl[kNb], rxl[kNb], dvl[kNb];
    uint8_t *txbuf[kNb], *rxbuf[kNb], *rxdev[kNb];
    for (size_t i = 0; i < kNb; ++i) {
        txl[i] = Lease(pinned_pool(), stage_bytes);
        rxl[i] = Lease(pinned_pool(), stage_bytes);
        dvl[i] = Lease(device_pool(), stage_bytes, R.device);
        if (!txl[i].ok() || !rxl[i].ok() || !dvl[i].ok()) return 1;
        txbuf[i] = txl[i].data();
        rxbuf[i] = rxl[i].data();
        rxdev[i] = dvl[i].data();
    }
    // declared after every staging lease: destroyed first, so nothing of this op still reads or writes them when
    // they go back to the pools (also on the early returns below). The op stream waited for every H2D copy it
    // issued; the step-0 device->host copies are not behind it.
    struct Drain {
        DeviceBackend *be;
        DevStream st;
        DevEvent *d2h;
        std::vector<DevEvent> *ev;
        ~Drain() {
            if (*d2h) event_wait_polling(be, *d2h);
            stream_wait_polling(be, st);
            for (auto e : *ev) event_pool().put(e);
        }
    } drain{be, st, &last_d2h, &owned};

    ReadyRanges txready[kNb];        // payload ranges of txbuf[i] (relative to txbuf[i] + txshift[i])
    ReadyRanges rxready[kNb];        // received ranges of rxbuf[i] (the next all-gather step forwards them)
    size_t txshift[kNb] = {0, 0, 0}; // payload of txbuf[i] starts at this offset (16-byte phase of its HBM source)
    DevEvent buf_free[kNb] = {nullptr, nullptr, nullptr}; // last GPU work reading rxbuf[i] / rxdev[i]

    const size_t nsteps = 2 * (ws - 1);
    auto is_rs = [&](size_t g) { return g + 1 < ws; };
    auto chunk_tx = [&](size_t g) { return ring_chunk_tx(g, rank, ws); };
    auto chunk_rx = [&](size_t g) { return ring_chunk_rx(g, rank, ws); };
    auto region_of = [&](size_t g) { return R.dst + bounds[chunk_rx(g)].first * es; };

    size_t max_stripes = 1;
    for (size_t g = 0; g < nsteps; ++g) {
        const auto [ts, te] = bounds[chunk_tx(g)];
        max_stripes = std::max(max_stripes, plan_stripes((te - ts) * es, R.txs.size()).off.size());
    }
    // declared after the buffers and ready lists it reads: destroyed (cancelled + joined) before them
    OpSenders senders(R.txs, R.tag, seq, piece, nsteps, max_stripes, be, R.tx);
    auto publish = [&](size_t g) {
        if (senders.published(g)) return;
        const auto [ts, te] = bounds[chunk_tx(g)];
        const bool staged = g < ws; // reduce-scatter steps and all-gather step 0 send txbuf payloads
        OpSenders::Step stp;
        stp.payload = staged ? txbuf[g % kNb] + txshift[g % kNb] : rxbuf[(g - 1) % kNb];
        stp.bytes = (te - ts) * es;
        stp.ready = staged ? &txready[g % kNb] : &rxready[(g - 1) % kNb];
        senders.publish(g, stp);
    };

    RingRx rx(R.rxs, R.tag, seq, nsteps); // after the buffers its sinks point into
    // rxbuf[g % kNb] may take step g's bytes once the step that used it before (g - kNb) is finished with it: its
    // GPU work completed and (all-gather) the step after it has forwarded its bytes
    auto can_post = [&](size_t g) {
        if (g < kNb) return true;
        const size_t b = g % kNb, prev = g - kNb;
        if (buf_free[b] && be->event_query(buf_free[b]) == 0) return false;
        if (!is_rs(prev) && prev + 1 < nsteps && !senders.sent(prev + 1)) return false;
        return true;
    };
    auto post = [&](size_t g) {
        const size_t b = g % kNb;
        buf_free[b] = nullptr;
        if (!is_rs(g)) rxready[b].clear();
        const auto [c0, c1] = bounds[chunk_rx(g)];
        rx.post(g, rxbuf[b], (c1 - c0) * es);
    };
    auto fail = [&](int code) {
        senders.cancel();
        return code;
    };

    for (size_t g = 0; g < nsteps; ++g) {
        const size_t b = g % kNb, nb = (g + 1) % kNb;
        const bool rs = is_rs(g);
        // 1. step g's sinks (normally posted during step g-1)
        while (!rx.posted(g)) {
            if (can_post(g)) {
                post(g);
                break;
            }
            if (senders.failed()) return fail(1);
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        // 2. this step's reduce writes txbuf[nb], last read by step g-2's sends
        uint8_t *region = region_of(g);
        const size_t shift = reinterpret_cast<uintptr_t>(region) % 16;
        if (rs) {
            if (g >= 2 && !senders.wait(g - 2)) return fail(1);
            txready[nb].clear();
            txshift[nb] = shift;
        }
        // 3. own input chunk -> pinned, in pieces (from src: ready at call time)
        if (g == 0) {
            const auto [ts, te] = bounds[chunk_tx(0)];
            txready[0].clear();
            txshift[0] = 0;
            for (size_t off = 0; off < (te - ts) * es; off += piece) {
                const size_t n = std::min(piece, (te - ts) * es - off);
                be->memcpy_async(txbuf[0] + off, R.src + ts * es + off, n, pq.d2h);
                last_d2h = record(pq.d2h);
                txready[0].add(off, off + n, last_d2h);
            }
        }
        publish(g);
        if (g + 1 < nsteps) publish(g + 1); // its payload fills while this step runs
        fault_point("ring", seq, g, "publish");
        // 4. receive + consume step g
        DevEvent step_last = nullptr;
        std::function<void(size_t, size_t)> consume;
        if (rs) {
            // HBM staging and the next payload share the 16-byte phase of `region`: the fused kernel stays vectorised
            uint8_t *stage = rxdev[b] + shift, *out = txbuf[nb] + shift, *sink = rxbuf[b];
            consume = [&, stage, out, sink, region, nb](size_t a, size_t e) {
                be->memcpy_async(stage + a, sink + a, e - a, pq.h2d);
                DevEvent ce = record(pq.h2d);
                be->stream_wait_event(st, ce);
                be->reduce_copy(region + a, stage + a, out + a, (e - a) / es, R.dtype, R.rop, st);
                step_last = record(st);
                txready[nb].add(a, e, step_last);
            };
        } else {
            uint8_t *sink = rxbuf[b];
            consume = [&, sink, region, b](size_t a, size_t e) {
                be->memcpy_async(region + a, sink + a, e - a, st);
                step_last = record(st);
                rxready[b].add(a, e, nullptr); // in host memory: forwardable at once
            };
        }
        bool first = true;
        const int rc = rx.receive(
            g, es, piece,
            [&](size_t a, size_t e) {
                consume(a, e);
                if (first) {
                    first = false;
                    fault_point("ring", seq, g, "rx"); // kernels / copies of this step in flight
                }
            },
            [&] { // post the next step's sinks as soon as its buffer is free (its sender may already be streaming)
                if (g + 1 < nsteps && !rx.posted(g + 1) && can_post(g + 1)) {
                    post(g + 1);
                    fault_point("ring", seq, g, "ahead");
                }
            },
            [&] { return senders.failed(); }, R.aborted);
        buf_free[b] = step_last;
        if (rc) return fail(rc);
        R.rx += (bounds[chunk_rx(g)].second - bounds[chunk_rx(g)].first) * es;
        rx.unpost(g);
        step_mark(rs, rs ? g : g - (ws - 1));
        if (g + 2 == ws) trace_mark("reduce_scatter");
        fault_point("ring", seq, g, "end");
    }
    if (!senders.wait_all()) return fail(1);
    return 0; // complete once its last received bytes landed in HBM (the Drain waits for them)
}

// An in-place device op finished its part: keep the input's backup (HBM or pinned) until the master's verdict and
// copy it back into dst if the op failed anyway (OpState::settle).
void settle_device_backup(std::function<void(bool)> &settle, DeviceBackend *be, int device, Lease &&backup,
                          void *dst, size_t bytes) {
    settle = [be, device, b = std::make_shared<Lease>(std::move(backup)), dst, bytes](bool restore) {
        if (!restore) return;
        be->set_device(device);
        StreamLease s(device);
        if (!s.get() || !be->memcpy_async(dst, b->data(), bytes, s.get()) || !be->stream_sync(s.get())) {
            LOG(ERR) << "all-reduce: could not restore the in-place input after a late abort";
        }
    };
}

} // namespace

std::pair<bool, bool> Client::ring_reduce_device(OpState &op, const RingView &rv, uint64_t seq, int device) {
    const ReduceRequest &q = op.req;
    if (q.qalgo != QuantAlgo::None && q.qtype != q.dtype) return ring_reduce_device_quant(op, rv, seq, device);
    DeviceBackend *be = device_backend();
    const size_t ws = rv.ring.size(), rank = rv.rank;
    const size_t es = dtype_size(q.dtype);
    auto *dst = static_cast<uint8_t *>(q.dst);
    const size_t bytes = q.count * es;
    // Copy / reduce / frame granularity. >= 4 MiB keeps the copy engines near their peak (1 MiB copies: ~37 GB/s);
    // with the send-ahead pipeline the step fill no longer scales with the piece, and 32 MiB measured fastest at
    // 8 peers x 1 GiB on one MI355X (8 MiB 391-409 ms, 16 MiB 345-421, 32 MiB 331-346 in most runs;
    // profiles/r3/ring_ab/): fewer copies, kernels, events and socket wake-ups per byte.
    const size_t piece = std::max<size_t>(1 << 20, env_size("PCCL_DEVICE_PIECE_BYTES", 32u << 20)) / es * es;

    be->set_device(device);
    StreamLease stream(device);
    DevStream st = stream.get();
    if (!st) return {false, false};
    if (op.small_path) { // latency-bound (agreed by every peer): one D2H, host all-gather + reduce, one H2D
        Lease hin(pinned_pool(), std::max<size_t>(bytes, 64)), hout(pinned_pool(), std::max<size_t>(bytes, 64));
        if (!hin.ok() || !hout.ok()) return {false, false};
        if (!be->memcpy_async(hin.data(), q.src, bytes, st) || !be->stream_sync(st)) return {false, false};
        const int rc = small_allgather_reduce(rv.tx, rv.rx, q.tag, seq, hin.data(), hout.data(), q.count, q.dtype,
                                              q.op, ws, rank, [&] { return abort_received(q.tag); }, op.tx, op.rx);
        if (rc) return {false, rc == 2};
        if (!be->memcpy_async(dst, hout.data(), bytes, st) || !be->stream_sync(st)) return {false, false};
        trace_mark("allgather_reduce");
        if (q.src == q.dst && !q.scratch) settle_device_backup(op.settle, be, device, std::move(hin), dst, bytes);
        return {true, false};
    }
    const PcieQueues pq = shared_pcie_queues(be, device);
    if (!pq.h2d || !pq.d2h) return {false, false};

    // the caller's input -> dst (out of place) or a backup of it (in place, restored on abort), on the op stream
    Lease backup;
    const bool keep_backup = q.src == q.dst && !q.scratch;
    if (keep_backup) {
        backup = Lease(device_pool(), bytes, device);
        if (!backup.ok()) return {false, false};
        be->memcpy_async(backup.data(), q.src, bytes, st);
    } else if (q.src != q.dst) {
        be->memcpy_async(dst, q.src, bytes, st);
    }
    OpAbort aborted([this, t = q.tag] { return abort_received(t); });
    DevRing R{rv.tx, rv.rx, ws, rank, q.tag, seq, be, pq, st, static_cast<const uint8_t *>(q.src), dst, q.count, es,
              piece, q.dtype, q.op, device, [&] { return aborted(); }, op.tx, op.rx};
    const int rc = device_ring_pipeline(R);
    if (rc != 0) {
        // the pipeline drained every copy and kernel of the op and no sink of it is posted any more: restore
        be->stream_sync(st);
        if (keep_backup) {
            be->memcpy_async(dst, backup.data(), bytes, st);
            be->stream_sync(st);
        }
        return {rc == 2, rc == 2};
    }
    if (q.op == ReduceOp::Avg) be->finalize_avg(dst, q.count, q.dtype, ws, st);
    if (!stream_wait_polling(be, st)) return {false, false};
    if (keep_backup) settle_device_backup(op.settle, be, device, std::move(backup), dst, bytes);
    return {true, false};
}

// Quantized device ring (protocol: quant_lane_bounds / meta_tag). Each lane is one pipeline over its 2(W-1) steps on
// its own thread and stream, built like the plain device ring (OpSenders, RingRx, sinks posted a step early):
//   * reduce-scatter step g: the payload is the chunk step g-1 reduced, so its min / max (folded from the partials
//     that step's de-quantize-reduce kernels emitted, one host round trip for the metadata packet) exists only once
//     step g-1 has received everything; the quantize kernels then write it into pinned memory piece by piece (two
//     payload buffers: step g quantizes while step g-1's sends drain) and each piece leaves once its kernel is done;
//     received pieces go to HBM on the shared copy-engine queue and de-quantize-reduce there;
//   * all-gather: the owner quantizes its finished chunk once and overwrites its own copy with D(Q(x)) (every peer
//     ends bit-identical); received quantized chunks are forwarded cut-through (the next step's metadata and sends
//     start when this step's metadata arrives; every piece leaves as it lands) and de-quantized by kernels reading
//     pinned memory.
// The per-step serialisation of the reduce-scatter is inherent to the protocol; lanes overlap it (one lane's fill and
// drain runs while another lane's data moves).
namespace {

// Start order of the lanes of one quantized op: lane k+1 starts once lane k's first payload is quantized. The lanes
// then run half a phase apart: one lane's reduce-scatter step quantizes (device->host writes) while the other's data
// arrives (host->device copies), instead of every lane of every peer quantizing at once and then receiving at once.
struct LaneGate {
    std::mutex m;
    std::condition_variable cv;
    bool open = false;
    void signal() {
        {
            std::lock_guard l(m);
            open = true;
        }
        cv.notify_all();
    }
    // false if `stop` became true first
    bool wait(const std::atomic<bool> &stop) {
        std::unique_lock l(m);
        while (!open) {
            if (stop.load()) return false;
            cv.wait_for(l, std::chrono::milliseconds(1));
        }
        return true;
    }
};

struct QLane {
    const std::vector<std::shared_ptr<net::MuxConn>> *txs, *rxs;
    size_t ws, rank;
    uint64_t tag, seq; // the lane's data tag (metadata on meta_tag(tag))
    DeviceBackend *be;
    DevStream st;   // the lane's stream (its copies, kernels and events)
    DevEvent ready; // the op's input copy / backup into dst (recorded on the op stream)
    uint8_t *dst;   // the lane's elements (hold the input once `ready` completed)
    size_t count, es, qs, piece_el;
    DType dtype, qtype;
    QuantAlgo qalgo;
    ReduceOp rop;
    int device;
    std::function<bool()> aborted;
    std::atomic<uint64_t> *tx, *rx;
    std::atomic<bool> *op_failed; // set by a lane that failed: its sibling lanes stop too
    LaneGate *wait_gate, *open_gate; // start after / open when the first payload is quantized (nullptr: none)
};

// Returns 0 ok, 1 io failure, 2 abort; on return no GPU work or socket write of the lane touches its buffers.
int device_quant_lane(QLane &L) {
    DeviceBackend *be = L.be;
    DevStream st = L.st;
    const size_t ws = L.ws, rank = L.rank, es = L.es, qs = L.qs, piece_el = L.piece_el;
    const uint64_t seq = L.seq;
    struct GateOpener { // the next lane never waits for a lane that ended (any exit)
        LaneGate *g;
        ~GateOpener() {
            if (g) g->signal();
        }
    } gate_opener{L.open_gate};
    if (L.wait_gate && !L.wait_gate->wait(*L.op_failed)) return 1;
    be->stream_wait_event(st, L.ready);

    std::vector<DevEvent> owned;
    auto record = [&](DevStream s) {
        DevEvent e = event_pool().get();
        owned.push_back(e);
        be->event_record(e, s);
        return e;
    };
    const auto bounds = chunk_bounds(L.count, ws);
    size_t max_chunk = 0;
    for (auto &b : bounds) max_chunk = std::max(max_chunk, b.second - b.first);
    const size_t qbytes = max_chunk * qs + 64;
    constexpr size_t kNb = 3;
    // The reduce-scatter's de-quantize-reduce kernels emit per-workgroup (min, max) partials of the values they store
    // into `mm_partials`: the chunk a step receives is the chunk the next step quantizes (and the last step's is the
    // all-gather's first payload), so its min / max is one fold of those partials instead of a second pass. A step
    // whose launches do not fit the partials buffer falls back to a separate min / max pass.
    constexpr int kMmSlots = 65536, kMmMinRoom = 64; // 1 MiB of partials: ~1 GiB bf16 chunks
    Lease txl[2], rxl[kNb], dvl[kNb], mml, mmp;
    uint8_t *txq[2], *rxbuf[kNb], *rxdev[kNb];
    for (size_t i = 0; i < kNb; ++i) {
        if (i < 2) {
            txl[i] = Lease(pinned_pool(), qbytes);
            if (!txl[i].ok()) return 1;
            txq[i] = txl[i].data();
        }
        rxl[i] = Lease(pinned_pool(), qbytes);
        dvl[i] = Lease(device_pool(), qbytes, L.device);
        if (!rxl[i].ok() || !dvl[i].ok()) return 1;
        rxbuf[i] = rxl[i].data();
        rxdev[i] = dvl[i].data();
    }
    mml = Lease(pinned_pool(), 64);
    mmp = Lease(device_pool(), kMmSlots * 2 * sizeof(double), L.device);
    if (!mml.ok()) return 1;
    auto *minmax_out = reinterpret_cast<double *>(mml.data());
    auto *mm_partials = mmp.ok() ? reinterpret_cast<double *>(mmp.data()) : nullptr;
    // declared after every lease: the lane's stream drains (every copy it waited for included) before they go back
    struct Drain {
        DeviceBackend *be;
        DevStream st;
        std::vector<DevEvent> *ev;
        ~Drain() {
            stream_wait_polling(be, st);
            for (auto e : *ev) event_pool().put(e);
        }
    } drain{be, st, &owned};

    ReadyRanges txready[2], rxready[kNb];
    DevEvent buf_free[kNb] = {nullptr, nullptr, nullptr}; // last GPU work reading rxbuf[i] / rxdev[i]
    const size_t nsteps = 2 * (ws - 1);
    auto is_rs = [&](size_t g) { return g + 1 < ws; };
    auto chunk_tx = [&](size_t g) { return ring_chunk_tx(g, rank, ws); };
    auto chunk_rx = [&](size_t g) { return ring_chunk_rx(g, rank, ws); };
    auto nel = [&](size_t c) { return bounds[c].second - bounds[c].first; };

    size_t max_stripes = 1;
    for (size_t g = 0; g < nsteps; ++g)
        max_stripes = std::max(max_stripes, plan_stripes(nel(chunk_tx(g)) * qs, L.txs->size()).off.size());
    OpSenders senders(*L.txs, L.tag, seq, piece_el * qs, nsteps, max_stripes, be, *L.tx);
    RingRx rx(*L.rxs, L.tag, seq, nsteps);
    const StepIo io{(*L.txs)[stripe_conn(seq, L.tag, 0, L.txs->size())].get(),
                    (*L.rxs)[stripe_conn(seq, L.tag, 0, L.rxs->size())].get(), meta_tag(L.tag), seq};

    auto can_post = [&](size_t g) {
        if (g < kNb) return true;
        const size_t b = g % kNb, prev = g - kNb;
        if (buf_free[b] && be->event_query(buf_free[b]) == 0) return false;
        if (!is_rs(prev) && prev + 1 < nsteps && !senders.sent(prev + 1)) return false;
        return true;
    };
    auto post = [&](size_t g) {
        const size_t b = g % kNb;
        buf_free[b] = nullptr;
        if (!is_rs(g)) rxready[b].clear();
        rx.post(g, rxbuf[b], nel(chunk_rx(g)) * qs);
    };
    auto fail = [&](int code) {
        senders.cancel();
        L.op_failed->store(true);
        return code;
    };
    auto failed = [&] { return senders.failed() || L.op_failed->load(); };

    int mm_used = 0;
    bool mm_complete = false; // the partials cover every element of the chunk consumed by the last step
    // metadata of `n` elements at device `src` (min / max folded from the previous step's partials when `fused` and
    // they are complete, else a separate pass; one host round trip)
    auto make_step_meta = [&](const uint8_t *src, size_t n, bool fused) -> QuantMeta {
        const bool fold = fused && mm_complete && mm_partials;
        const int folded = mm_used;
        mm_used = 0;
        mm_complete = mm_partials != nullptr; // the next step's consumes start collecting afresh
        if (n == 0) return kernels::make_meta(L.qalgo, L.dtype, L.qtype, 0, 0);
        if (fold) {
            g_quant_minmax_folds.fetch_add(1, std::memory_order_relaxed);
            be->minmax_fold(mm_partials, folded, n, minmax_out, st);
        } else {
            g_quant_minmax_passes.fetch_add(1, std::memory_order_relaxed);
            be->minmax(src, n, L.dtype, minmax_out, st);
        }
        stream_wait_polling(be, st);
        return kernels::make_meta(L.qalgo, L.dtype, L.qtype, minmax_out[0], minmax_out[1]);
    };
    auto dequant_consume = [&](uint8_t *dst_el, const uint8_t *src_q, size_t n, const kernels::QuantParams &params) {
        int blocks = 0;
        if (mm_complete && mm_partials && kMmSlots - mm_used >= kMmMinRoom &&
            be->dequant_reduce_minmax(dst_el, src_q, n, L.dtype, L.qtype, L.rop, params, mm_partials + 2 * mm_used,
                                      kMmSlots - mm_used, &blocks, st)) {
            mm_used += blocks;
            return;
        }
        mm_complete = false;
        be->dequant_reduce(dst_el, src_q, n, L.dtype, L.qtype, L.rop, params, st);
    };
    auto publish = [&](size_t g, const uint8_t *payload, ReadyRanges *ready) {
        OpSenders::Step stp;
        stp.payload = payload;
        stp.bytes = nel(chunk_tx(g)) * qs;
        stp.ready = ready;
        senders.publish(g, stp);
    };

    DevEvent first_payload = nullptr; // last quantize kernel of step 0
    bool gate_opened = L.open_gate == nullptr;
    auto maybe_open_gate = [&] {
        if (gate_opened || (first_payload && be->event_query(first_payload) == 0)) return;
        L.open_gate->signal();
        gate_opened = true;
    };
    QuantMeta theirs;
    // Where received pieces go to HBM. Large steps (>= 4 MiB of quantized bytes per lane and step): on the lane's own
    // stream, in both phases - in the process-wide queue a step's last pieces wait behind every other peer's copies
    // before the next min / max exists (8 peers x 1 GiB bf16, interleaved: 188.1 vs 197.9 ms, profiles/r4/b23/;
    // all-gather 186.5 vs 190.4 ms, b25/). Small steps (many concurrent ops, e.g. config 3 over the WAN emulator with
    // ~1 MiB steps): the shared queue in the reduce-scatter, kernels reading pinned memory in the all-gather, as
    // per-lane copies there measured 1.34-1.38 vs 1.09-1.16 s per 2 GiB (b29/). The plain ring keeps the shared queue
    // at every size (332.9 vs 365.3 ms, b23/).
    const bool lane_copies = max_chunk * qs >= (size_t{4} << 20);
    const PcieQueues pq = lane_copies ? PcieQueues{} : shared_pcie_queues(be, L.device);
    if (!lane_copies && !pq.h2d) return fail(1);
    for (size_t g = 0; g < nsteps; ++g) {
        const size_t b = g % kNb;
        const bool rs = is_rs(g);
        while (!rx.posted(g)) {
            if (can_post(g)) {
                post(g);
                break;
            }
            if (failed()) return fail(1);
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        if (g < ws) { // own payload: reduce-scatter steps and the all-gather's first step
            const size_t slot = g % 2, c = chunk_tx(g);
            uint8_t *src = L.dst + bounds[c].first * es;
            const size_t n = nel(c);
            if (g >= 2 && !senders.wait(g - 2)) return fail(1); // txq[slot] was step g-2's payload
            const QuantMeta mine = make_step_meta(src, n, g > 0);
            const auto params = kernels::make_params(mine, L.qtype);
            txready[slot].clear();
            for (size_t off = 0; off < n; off += piece_el) {
                const size_t k = std::min(piece_el, n - off);
                if (g + 1 == ws) // the all-gather's payload; parity: own chunk := D(Q(x)), what the others de-quantize
                    be->quantize_setback(txq[slot] + off * qs, src + off * es, k, L.dtype, L.qtype, params, st);
                else
                    be->quantize(txq[slot] + off * qs, src + off * es, k, L.dtype, L.qtype, params, st);
                DevEvent e = record(st);
                txready[slot].add(off * qs, (off + k) * qs, e);
                if (g == 0) first_payload = e;
            }
            if (int m = send_meta(io, mine, *L.tx)) return fail(m);
            publish(g, txq[slot], &txready[slot]);
            step_sub_mark('q', g);
        } // else: forwarded chunk, published with its metadata when step g-1's metadata arrived
        fault_point("qring", seq, g, "meta");
        if (int m = recv_meta(io, theirs, *L.rx, L.aborted, failed)) return fail(m);
        const auto params = kernels::make_params(theirs, L.qtype);
        if (!rs && g + 1 < nsteps) { // cut-through all-gather: the next step forwards this chunk as it lands
            if (int m = send_meta(io, theirs, *L.tx)) return fail(m);
            publish(g + 1, rxbuf[b], &rxready[b]);
        }
        uint8_t *region = L.dst + bounds[chunk_rx(g)].first * es;
        DevEvent step_last = nullptr;
        bool first = true;
        const int rc = rx.receive(
            g, qs, piece_el * qs,
            [&](size_t a, size_t e) {
                const size_t n = (e - a) / qs;
                if (rs) { // host -> HBM, then de-quantize-reduce HBM -> HBM (staged beats kernels reading pinned
                          // memory: 218.5 vs 223.7 ms, profiles/r4/b9/q_rs.jsonl)
                    if (lane_copies) {
                        be->memcpy_async(rxdev[b] + a, rxbuf[b] + a, e - a, st);
                    } else {
                        be->memcpy_async(rxdev[b] + a, rxbuf[b] + a, e - a, pq.h2d);
                        be->stream_wait_event(st, record(pq.h2d));
                    }
                    dequant_consume(region + a / qs * es, rxdev[b] + a, n, params);
                } else if (lane_copies) { // forwardable at once (from pinned memory); host -> HBM on the lane's stream,
                                          // de-quantized from HBM
                    rxready[b].add(a, e, nullptr);
                    be->memcpy_async(rxdev[b] + a, rxbuf[b] + a, e - a, st);
                    be->dequant_reduce(region + a / qs * es, rxdev[b] + a, n, L.dtype, L.qtype, ReduceOp::Set, params,
                                       st);
                } else { // forwardable at once; de-quantized straight from pinned memory
                    rxready[b].add(a, e, nullptr);
                    be->dequant_reduce(region + a / qs * es, rxbuf[b] + a, n, L.dtype, L.qtype, ReduceOp::Set, params,
                                       st);
                }
                step_last = record(st);
                if (first) {
                    first = false;
                    step_sub_mark('f', g);
                    fault_point("qring", seq, g, "rx");
                }
            },
            [&] {
                maybe_open_gate();
                if (g + 1 < nsteps && !rx.posted(g + 1) && can_post(g + 1)) post(g + 1);
            },
            failed, L.aborted);
        buf_free[b] = step_last;
        if (rc) return fail(rc);
        *L.rx += nel(chunk_rx(g)) * qs;
        rx.unpost(g);
        step_mark(rs, rs ? g : g - (ws - 1));
        fault_point("qring", seq, g, "end");
    }
    if (!senders.wait_all()) return fail(1);
    return 0;
}

} // namespace

std::pair<bool, bool> Client::ring_reduce_device_quant(OpState &op, const RingView &rv, uint64_t seq, int device) {
    DeviceBackend *be = device_backend();
    const ReduceRequest &q = op.req;
    const size_t ws = rv.ring.size();
    const size_t es = dtype_size(q.dtype), qs = dtype_size(q.qtype);
    auto *dst = static_cast<uint8_t *>(q.dst);
    const size_t bytes = q.count * es;
    // value bytes per quantize / de-quantize piece (and frame): PCCL_QUANT_PIECE_BYTES, default 32 MiB (interleaved
    // A/B, uint8, 8 peers x 1 GiB on one MI355X: 8 MiB 223 ms, 16 MiB 210, 32 MiB 201-206, 64 MiB 204-208;
    // profiles/r4/ab2/): fewer kernels, copies, events and frames per byte
    const size_t piece = std::max<size_t>(1 << 20, env_size("PCCL_QUANT_PIECE_BYTES", 32u << 20)) / es * es;

    be->set_device(device);
    StreamLease stream(device);
    DevStream st = stream.get();
    if (!st) return {false, false};

    Lease backup;
    const bool keep_backup = q.src == q.dst && !q.scratch;
    if (keep_backup) {
        backup = Lease(device_pool(), bytes, device);
        if (!backup.ok()) return {false, false};
        be->memcpy_async(backup.data(), q.src, bytes, st);
    } else if (q.src != q.dst) {
        be->memcpy_async(dst, q.src, bytes, st);
    }
    DevEvent ready = event_pool().get();
    struct EvBack { // the op stream drains before the event returns to the pool (every exit)
        DeviceBackend *be;
        DevStream st;
        DevEvent e;
        ~EvBack() {
            stream_wait_polling(be, st);
            event_pool().put(e);
        }
    } ev_back{be, st, ready};
    be->event_record(ready, st);

    const std::vector<size_t> lo = quant_lane_bounds(q.count, ws, qs);
    const size_t nl = lo.size() - 1;
    std::vector<std::unique_ptr<StreamLease>> lane_streams;
    for (size_t k = 0; k < nl; ++k) {
        lane_streams.push_back(std::make_unique<StreamLease>(device));
        if (!lane_streams.back()->get()) return {false, false};
    }
    OpAbort aborted([this, t = q.tag] { return abort_received(t); });
    std::atomic<bool> op_failed{false};
    std::vector<LaneGate> gates(nl);
    const int rc = run_lanes(lo, [&](size_t k, size_t a, size_t b) {
        QLane L{&rv.tx, &rv.rx, ws, rv.rank, lane_tag(q.tag, k, nl), seq, be, lane_streams[k]->get(), ready,
                dst + a * es, b - a, es, qs, piece / es, q.dtype, q.qtype, q.qalgo, q.op, device,
                [&] { return aborted(); }, &op.tx, &op.rx, &op_failed, k > 0 ? &gates[k - 1] : nullptr,
                k + 1 < nl ? &gates[k] : nullptr};
        return device_quant_lane(L);
    });
    if (rc != 0) {
        be->stream_sync(st); // every lane drained its own stream before returning
        if (keep_backup) {
            be->memcpy_async(dst, backup.data(), bytes, st);
            be->stream_sync(st);
        }
        return {rc == 2, rc == 2};
    }
    // the lanes' streams are drained (each lane's Drain): the result is complete in HBM
    if (q.op == ReduceOp::Avg) be->finalize_avg(dst, q.count, q.dtype, ws, st);
    if (!stream_wait_polling(be, st)) return {false, false};
    if (keep_backup) settle_device_backup(op.settle, be, device, std::move(backup), dst, bytes);
    return {true, false};
}

} // namespace pccl::client

// [0] quantized-ring payloads whose min / max came from the fused de-quantize partials, [1] separate min / max passes
extern "C" __attribute__((visibility("default"))) void pcclxQuantStats(uint64_t *out2) {
    out2[0] = pccl::client::g_quant_minmax_folds.load(std::memory_order_relaxed);
    out2[1] = pccl::client::g_quant_minmax_passes.load(std::memory_order_relaxed);
}
