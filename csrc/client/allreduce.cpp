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
        workers_.submit([this, op] { run_op(op); });
    }
    return true;
}

void Client::run_op(const std::shared_ptr<OpState> &op) {
    const uint64_t tag = op->req.tag;
    low_timer_slack();
    fault_delay(tag);
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
    // the ring cannot change while this op runs (re-establishment waits for running ops), so the view taken here
    // is the one the op executes on
    auto rv = ring_view(0);
    DevPtrInfo si{}, di{};
    DeviceBackend *be = device_backend();
    if (be) {
        be->pointer_info(op->req.src, si);
        be->pointer_info(op->req.dst, di);
    }
    const bool device = si.is_device && di.is_device && si.device == di.device;
    {
        C2MCollectiveCommsInitiate init;
        init.tag = tag;
        init.count = op->req.count;
        init.data_type = op->req.dtype;
        init.op = op->req.op;
        if (rv && rv->hier && device) init.flags |= kCollFlagHierarchical;
        if (rv && rv->ring.size() >= 2 && use_small_path(op->req.count * dtype_size(op->req.dtype), rv->ring.size()) &&
            (op->req.qalgo == QuantAlgo::None || op->req.qtype == op->req.dtype))
            init.flags |= kCollFlagSmallPath;
        if (master_.send(init)) {
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
                } else if (!si.is_device && !di.is_device) {
                    r = ring_reduce_host(*op, *rv, seq);
                    if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::HostRing);
                } else {
                    LOG(ERR) << "all-reduce: send and receive buffers must both be host or both be on one GPU";
                    r = {false, false};
                }
            }
            success = r.first && !r.second;
            abort_seen = r.second;
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

struct StepIo {
    net::MuxConn *tx;
    net::MuxConn *rx;
    uint64_t tag;
    uint64_t seq;
};

constexpr size_t kMetaFrameOverhead = 24;

// Dequantization metadata of one quantized step (reference reduce.cpp:154-192 sends its own and then waits for the
// peer's before any data moves, which costs one extra network latency per ring step). Here the sender sends its meta
// and immediately its data; the receiver waits for the peer's meta before posting its data sink (data frames that
// arrive first are queued by the connection), so meta and data share one latency. Returns 0 ok, 1 io failure.
int send_meta(const StepIo &io, const QuantMeta &mine, std::atomic<uint64_t> &tx) {
    P2PDequantizationMeta pkt;
    pkt.tag = io.tag;
    pkt.meta = mine;
    auto bytes = encode_with_id(pkt);
    if (!io.tx->send_frame(io.tag, io.seq, bytes.data(), bytes.size())) return 1;
    tx += bytes.size() + kMetaFrameOverhead;
    return 0;
}

// Waits for the peer's metadata of this step. Returns 0 ok, 1 io failure, 2 abort.
int recv_meta(const StepIo &io, QuantMeta &theirs, std::atomic<uint64_t> &rx, const std::function<bool()> &aborted) {
    while (true) {
        auto m = io.rx->recv_packet<P2PDequantizationMeta>(io.tag, io.seq, 20ms);
        if (m) {
            theirs = m->meta;
            rx += encode_with_id(*m).size() + kMetaFrameOverhead;
            return 0;
        }
        if (!io.rx->is_open()) return 1;
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
// `before_rx` (optional) runs after the senders started and before the receive sinks are posted (the quantized steps
// receive the peer's metadata there). Returns 0 ok, 1 io failure, 2 abort.
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
                 const std::function<int()> &before_rx = {}, size_t gran = 0, size_t early_from = SIZE_MAX) {
    const StripePlan tp = plan_stripes(tx_bytes, txs.size());
    const StripePlan rp = plan_stripes(rx_bytes, rxs.size());
    auto rx_conn = [&](size_t k) { return rxs[(seq + k) % rxs.size()].get(); };
    auto tx_conn = [&](size_t k) { return txs[(seq + k) % txs.size()].get(); };
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
    // stripes >= early_from may take their sinks before before_rx runs: their connections carry only this op's data
    // frames (the metadata packet travels on stripe 0's connection, where a sink posted too early would swallow it)
    const size_t nst = rp.off.size();
    const size_t early = before_rx ? std::min(std::max<size_t>(early_from, 1), nst) : nst; // [early, nst) go first
    for (size_t k = early; k < nst; ++k) rx_conn(k)->post_sink(tag, seq, sink + rp.off[k], rp.len[k]);
    sinks_posted = early < nst;
    if (before_rx) {
        if (const int brc = before_rx()) {
            send_rc.store(brc);
            senders.wait();
            remove_sinks();
            return brc;
        }
    }
    for (size_t k = 0; k < early; ++k) rx_conn(k)->post_sink(tag, seq, sink + rp.off[k], rp.len[k]);
    sinks_posted = true;
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
std::pair<bool, bool> Client::ring_reduce_host(OpState &op, const RingView &rv, uint64_t seq) {
    const ReduceRequest &q = op.req;
    const size_t ws = rv.ring.size(), rank = rv.rank;
    const size_t es = dtype_size(q.dtype);
    const bool quant = q.qalgo != QuantAlgo::None && q.qtype != q.dtype;
    const size_t qs = quant ? dtype_size(q.qtype) : es;
    auto *dst = static_cast<uint8_t *>(q.dst);
    const size_t bytes = q.count * es;
    const size_t chunk = net::multiplex_chunk_size();

    StepIo io{rv.tx[seq % rv.tx.size()].get(), rv.rx[seq % rv.rx.size()].get(), q.tag, seq};
    auto aborted = [&] { return abort_received(q.tag); };

    if (!quant && op.small_path) {
        const int rc = small_allgather_reduce(rv.tx, rv.rx, q.tag, seq, q.src, dst, q.count, q.dtype, q.op, ws, rank,
                                              aborted, op.tx, op.rx);
        trace_mark("allgather_reduce");
        return {rc == 0, rc == 2};
    }

    Lease backup;
    if (q.src == q.dst) {
        backup = Lease(host_pool(), bytes);
        std::memcpy(backup.data(), q.src, bytes);
    } else {
        std::memcpy(dst, q.src, bytes);
    }
    auto restore = [&] {
        if (q.src == q.dst) std::memcpy(dst, backup.data(), bytes);
    };

    const auto bounds = chunk_bounds(q.count, ws);
    size_t max_chunk = 0;
    for (auto &b : bounds) max_chunk = std::max(max_chunk, b.second - b.first);
    Lease rbuf(host_pool(), max_chunk * qs + 64);
    Lease qbuf;
    if (quant) qbuf = Lease(host_pool(), max_chunk * qs + 64);

    // One full-duplex (striped) step: sends `payload`, receives `rx_bytes` into `sink`, calling `consume(from, to)`
    // for newly complete received elements. Returns 0 ok, 1 io failure, 2 abort.
    auto run_step = [&](const uint8_t *payload, size_t tx_bytes, uint8_t *sink, size_t rx_bytes,
                        const std::function<void(size_t, size_t)> &consume,
                        const std::function<int()> &before_rx = {}) -> int {
        return striped_step(rv.tx, rv.rx, q.tag, seq, payload, tx_bytes, [](size_t) { return true; }, sink, rx_bytes,
                            qs, chunk, consume, aborted, op.tx, op.rx, before_rx);
    };
    auto await_meta = [&](QuantMeta &theirs) { return [&, pt = &theirs] { return recv_meta(io, *pt, op.rx, aborted); }; };
    auto fail = [&](int code) -> std::pair<bool, bool> {
        restore();
        return {code == 2, code == 2};
    };

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
            if (int rc = send_meta(io, mine, op.tx)) return fail(rc);
        }
        uint8_t *rx_region = dst + rs * es;
        const int rc = run_step(payload, (te - ts) * qs, rbuf.data(), (re - rs) * qs, [&](size_t a, size_t b) {
            if (quant)
                kernels::host_dequant_reduce(rx_region + a * es, rbuf.data() + a * qs, b - a, q.dtype, q.qtype, q.op, theirs);
            else
                kernels::host_reduce(rx_region + a * es, rbuf.data() + a * es, b - a, q.dtype, q.op);
        }, quant ? std::function<int()>(await_meta(theirs)) : std::function<int()>());
        if (rc) return fail(rc);
    }

    trace_mark("reduce_scatter");
    // ---- all-gather
    Lease ag[2];
    if (quant) {
        ag[0] = Lease(host_pool(), max_chunk * qs + 64);
        ag[1] = Lease(host_pool(), max_chunk * qs + 64);
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
            if (int m = send_meta(io, mine, op.tx)) return fail(m);
            uint8_t *sink = ag[step % 2].data();
            rc = run_step(payload, (te - ts) * qs, sink, (re - rs) * qs, [&](size_t a, size_t b) {
                kernels::host_dequant_reduce(rx_region + a * es, sink + a * qs, b - a, q.dtype, q.qtype, ReduceOp::Set, theirs);
            }, await_meta(theirs));
            prev_meta = theirs;
        } else {
            rc = run_step(dst + ts * es, (te - ts) * es, rx_region, (re - rs) * es, [](size_t, size_t) {});
        }
        if (rc) return fail(rc);
        cur = inc;
    }
    if (q.op == ReduceOp::Avg) kernels::host_finalize_avg(dst, q.count, q.dtype, ws);
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
//   * received bytes are copied into HBM staging by the copy engine and reduced HBM->HBM on the op's compute stream
//     (cross-stream event wait, no host round trip) by k_reduce_copy, which also streams the result into pinned
//     memory as the NEXT step's payload: a ring step's sends start the moment the previous step's last piece lands,
//     and the only device->host copies left are the step-0 pieces of the input.
// PCIe bytes per peer and 1 GiB: D2H 1 GiB (step-0 payload + reduced pieces), H2D 1.75 GiB (received pieces).

namespace {

struct PcieQueues {
    static constexpr size_t kMaxH2d = 4;
    std::array<DevStream, kMaxH2d> h2d{}; // received pieces -> HBM, round robin over nh2d queues
    size_t nh2d = 1;
    DevStream d2h = nullptr;
    // one compute stream for the fused reduce-scatter kernels of every device-ring op of the process on this GPU
    // (PCCL_RING_SHARED_REDUCE), with the lock that keeps each (H2D copy, reduce) pair in the same order on both queues
    DevStream red = nullptr;
    std::mutex *red_mtx = nullptr;
};

// process-wide copy queues of `device` (never destroyed: they may outlive static destruction order)
PcieQueues shared_pcie_queues(DeviceBackend *be, int device) {
    static std::mutex m;
    static auto *q = new std::map<int, PcieQueues>();
    std::lock_guard l(m);
    PcieQueues &e = (*q)[device];
    if (!e.h2d[0]) {
        const int cur = be->current_device();
        be->set_device(device);
        // PCCL_H2D_QUEUES (1..4, default 1): one host->device stream runs ~46 GB/s on MI355X, several together
        // ~57 GB/s one way (profiles/r2/sysprobe.json)
        e.nh2d = std::max<size_t>(1, std::min(PcieQueues::kMaxH2d, env_size("PCCL_H2D_QUEUES", 1)));
        for (size_t k = 0; k < e.nh2d; ++k) e.h2d[k] = be->create_stream();
        e.d2h = be->create_stream();
        e.red_mtx = new std::mutex();
        if (cur >= 0) be->set_device(cur);
    }
    if (!e.red && env_size("PCCL_RING_SHARED_REDUCE", 0) != 0) { // only when asked for: streams share HW queues
        const int cur = be->current_device();
        be->set_device(device);
        e.red = be->create_stream();
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
    std::vector<Staged> v;
    void clear() {
        std::lock_guard l(m);
        v.clear();
    }
    void add(size_t a, size_t b, DevEvent e) {
        std::lock_guard l(m);
        v.push_back({a, b, e});
    }
    // blocks until every byte of [begin, end) is readable; false if `cancel` became non-zero first
    bool wait(size_t begin, size_t end, DeviceBackend *be, const std::atomic<int> &cancel) {
        if (end <= begin) return true;
        unsigned us = 2;
        std::vector<std::pair<size_t, size_t>> iv;
        std::vector<DevEvent> evs;
        while (true) {
            bool covered = false;
            {
                std::lock_guard l(m);
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
            }
            if (covered) {
                for (DevEvent e : evs)
                    if (!event_wait_polling(be, e)) return false;
                return true;
            }
            if (cancel.load(std::memory_order_relaxed) != 0) return false;
            std::this_thread::sleep_for(std::chrono::microseconds(us));
            us = std::min(us * 2, 200u);
        }
    }
};

// The send side of one device-ring op: one thread per stripe for the whole op (not per step), each sending its
// stripe of every step in order over connection (seq + k) % pool. The op thread publishes step g (payload, bytes,
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
    void cancel() {
        rc_.store(1);
        std::lock_guard l(m_);
        cv_.notify_all();
    }
    bool failed() const { return rc_.load() != 0; }
    const std::atomic<int> &rc() const { return rc_; }

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
            net::MuxConn *c = txs_[(seq_ + k) % txs_.size()].get();
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

} // namespace

namespace {

// Start signal between the lanes of one device-ring op (lane k+1 starts once lane k reached its all-gather).
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
};

// One lane of the device ring: a complete pipelined ring all-reduce of `n` elements at `region` (HBM, already holding
// the input) whose step-0 payload is staged from `src`, on its own compute stream, tag and staging rings.
struct Lane {
    // inputs
    const std::vector<std::shared_ptr<net::MuxConn>> *txs, *rxs; // the ring's connections to next / from prev
    size_t ws, rank;                                              // ring size, my position
    uint64_t tag, seq;
    DeviceBackend *be;
    PcieQueues pq;
    DevStream st;       // this lane's compute stream (waits for `ready` first)
    DevEvent ready;     // the op-level input copy / backup (recorded on the op stream), or nullptr
    const uint8_t *src; // step-0 source of this lane's elements
    uint8_t *dst;       // this lane's elements in the op's destination
    size_t count, es, piece;
    DType dtype;
    ReduceOp rop;
    int device;
    bool ahead, step0_on_op_stream;
    double host_frac = 0; // share of every intermediate reduce-scatter chunk reduced by the CPU (see run_lane)
    bool ag_on_lane_stream = false; // all-gather bytes -> HBM by blit kernels on the lane stream, not the H2D queue
    int rs_h2d = 0; // reduce-scatter received bytes: 0 copy engine -> HBM staging, 1 blit copy on the lane stream,
                    // 2 none (the fused reduce reads them from pinned memory)
    bool shared_reduce = false; // reduce-scatter kernels on the process-wide stream pq.red (see ring_reduce_device)
    int ag_copy_grid = 0; // > 0: all-gather copies as our copy kernel with this many workgroups (PCCL_RING_AG_COPY_GRID)
    bool shared_ag = false; // with shared_reduce: the all-gather copies on the shared stream too (PCCL_RING_SHARED_AG)
    LaneGate *wait_gate = nullptr, *open_gate = nullptr; // start after / signal when reaching the all-gather
    std::function<bool()> aborted;
    std::atomic<uint64_t> *tx, *rx;
    bool main_lane = false; // trace marks and fault points
    // output
    int rc = 0; // 0 ok, 1 io failure, 2 abort
};

void run_lane(Lane &L) {
    const auto &txs = *L.txs;
    const auto &rxs = *L.rxs;
    DeviceBackend *be = L.be;
    const PcieQueues pq = L.pq;
    DevStream st = L.st;
    const size_t ws = L.ws, rank = L.rank, es = L.es, piece = L.piece;
    const uint64_t tag = L.tag, seq = L.seq;
    auto fail = [&](int code) {
        L.rc = code;
        if (L.open_gate) L.open_gate->signal(); // never leave a waiting lane behind
    };
    if (L.wait_gate) {
        std::unique_lock l(L.wait_gate->m);
        L.wait_gate->cv.wait(l, [&] { return L.wait_gate->open; });
    }
    if (L.ready) be->stream_wait_event(st, L.ready);
    const bool shared_red = L.shared_reduce && pq.red && pq.red_mtx;
    DevStream rst = shared_red ? pq.red : st; // stream of this lane's reduce-scatter kernels
    if (shared_red && L.ready) {
        std::lock_guard l(*pq.red_mtx);
        be->stream_wait_event(rst, L.ready); // the op's input copy into dst precedes the reduces into it
    }

    // events of this lane (returned to the pool once everything they guard has completed)
    std::vector<DevEvent> owned;
    DevEvent last_d2h = nullptr;
    DevEvent lane_last_red = nullptr; // last reduce-scatter kernel of this lane (on rst)
    std::array<DevEvent, PcieQueues::kMaxH2d> last_h2d{}; // last copy issued on each H2D queue
    size_t h2d_rr = 0;
    auto record = [&](DevStream s) {
        DevEvent e = event_pool().get();
        owned.push_back(e);
        be->event_record(e, s);
        return e;
    };
    const auto bounds = chunk_bounds(L.count, ws);
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
        dvl[i] = Lease(device_pool(), stage_bytes, L.device);
        if (!txl[i].ok() || !rxl[i].ok() || !dvl[i].ok()) return fail(1);
        txbuf[i] = txl[i].data();
        rxbuf[i] = rxl[i].data();
        rxdev[i] = dvl[i].data();
    }
    // own input staged for the host-reduced part of a step (PCCL_RING_HOST_REDUCE, see host_elems below)
    Lease locl[2];
    uint8_t *locbuf[2] = {nullptr, nullptr};
    if (L.host_frac > 0 && ws >= 3) {
        for (int i = 0; i < 2; ++i) {
            locl[i] = Lease(pinned_pool(), stage_bytes);
            if (!locl[i].ok()) return fail(1);
            locbuf[i] = locl[i].data();
        }
    }
    // declared after every staging lease: destroyed first, so nothing of this lane still reads or writes them when
    // they go back to the pools (also on the early returns below)
    struct Drain {
        DeviceBackend *be;
        DevStream st;
        std::array<DevEvent, PcieQueues::kMaxH2d> *h2d;
        DevEvent *d2h, *red;
        std::vector<DevEvent> *ev;
        ~Drain() {
            for (DevEvent e : *h2d)
                if (e) be->event_sync(e);
            if (*d2h) be->event_sync(*d2h);
            if (*red) be->event_sync(*red);
            be->stream_sync(st);
            for (auto e : *ev) event_pool().put(e);
        }
    } drain{be, st, &last_h2d, &last_d2h, &lane_last_red, &owned};

    ReadyRanges txready[kNb];     // payload ranges of txbuf[i] (relative to txbuf[i] + txshift[i])
    ReadyRanges rxready[kNb];     // received ranges of rxbuf[i] (the next all-gather step forwards them)
    size_t txshift[kNb] = {0, 0, 0}; // payload of txbuf[i] starts at this offset (16-byte phase of its HBM source)
    // last H2D copies (one per queue) reading rxbuf[i] / writing rxdev[i]
    std::array<DevEvent, PcieQueues::kMaxH2d> h2d_done[kNb] = {};
    DevEvent red_done[kNb] = {nullptr, nullptr, nullptr}; // last reduce kernel reading rxdev[i]

    const size_t nsteps = 2 * (ws - 1);
    auto is_rs = [&](size_t g) { return g + 1 < ws; };
    auto chunk_tx = [&](size_t g) { // chunk index this peer sends at global step g
        return g + 1 < ws ? (rank + ws - g) % ws : (rank + 1 + ws - (g - (ws - 1)) % ws) % ws;
    };
    auto chunk_rx = [&](size_t g) { return (chunk_tx(g) + ws - 1) % ws; };
    auto region_of = [&](size_t g) { return L.dst + bounds[chunk_rx(g)].first * es; };
    // PCIe-balanced reduce placement (PCCL_RING_HOST_REDUCE = f): of every intermediate reduce-scatter chunk (steps
    // whose result is only forwarded), the first f of the elements are reduced by the CPU from the received bytes and
    // the peer's own input staged device -> host one step ahead, straight into the next payload. Those bytes then
    // never cross PCIe host -> device, the link direction that bounds the device ring (every received byte otherwise
    // goes up for the GPU reduce), while the device -> host volume is unchanged (the input piece instead of the
    // reduced piece). The last reduce-scatter step (the owner's final chunk) always reduces on the GPU.
    const bool host_red = L.host_frac > 0 && ws >= 3;
    auto host_elems = [&](size_t g) -> size_t {
        if (!host_red || g + 2 >= ws) return 0;
        const auto [c0, c1] = bounds[chunk_rx(g)];
        return static_cast<size_t>(static_cast<double>(c1 - c0) * std::min(1.0, L.host_frac)) / 64 * 64;
    };
    DevEvent loc_ready[2] = {nullptr, nullptr};
    auto stage_local = [&](size_t g) { // own input of step g's host part -> pinned (read once by step g's reduce)
        const size_t hb = g < 2 * (ws - 1) ? host_elems(g) : 0;
        if (hb == 0) return;
        be->memcpy_async(locbuf[g % 2], L.src + bounds[chunk_rx(g)].first * es, hb * es, pq.d2h);
        loc_ready[g % 2] = last_d2h = record(pq.d2h);
    };

    size_t max_stripes = 1;
    for (size_t g = 0; g < nsteps; ++g) {
        const auto [ts, te] = bounds[chunk_tx(g)];
        max_stripes = std::max(max_stripes, plan_stripes((te - ts) * es, txs.size()).off.size());
    }
    // declared after the buffers and ready lists it reads: destroyed (cancelled + joined) before them
    OpSenders senders(txs, tag, seq, piece, nsteps, max_stripes, be, *L.tx);
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
    auto fail_all = [&](int code) {
        senders.cancel();
        fail(code);
    };

    // ---- receive side: one set of sinks per step, posted up to one step early
    struct StepRx {
        StripePlan rp;
        std::vector<net::MuxConn::SinkRef> sinks;
        std::vector<size_t> done; // elements consumed per stripe
        size_t remaining = 0;
        bool posted = false;
    };
    std::vector<StepRx> srx(nsteps);
    auto rx_conn = [&](size_t k) { return rxs[(seq + k) % rxs.size()].get(); };
    // rxbuf[g % kNb] may take step g's bytes once the step that used it before (g - kNb) is finished with it: its H2D
    // copies and reduce kernels completed and (all-gather) the step after it has forwarded its bytes
    auto can_post = [&](size_t g) {
        if (g < kNb) return true;
        const size_t b = g % kNb, prev = g - kNb;
        for (DevEvent e : h2d_done[b])
            if (e && be->event_query(e) == 0) return false;
        if (red_done[b] && be->event_query(red_done[b]) == 0) return false;
        if (!is_rs(prev) && prev + 1 < nsteps && !senders.sent(prev + 1)) return false;
        return true;
    };
    // zero-copy reduce-scatter reads the received bytes in place: they share the 16-byte phase of the HBM chunk they
    // are reduced into, so the fused kernel stays vectorised
    auto sink_shift = [&](size_t g) -> size_t {
        return L.rs_h2d == 2 && is_rs(g) ? reinterpret_cast<uintptr_t>(region_of(g)) % 16 : 0;
    };
    auto post = [&](size_t g) {
        StepRx &r = srx[g];
        const size_t b = g % kNb;
        h2d_done[b] = {};
        red_done[b] = nullptr;
        if (!is_rs(g)) rxready[b].clear();
        const auto [rs0, re0] = bounds[chunk_rx(g)];
        r.rp = plan_stripes((re0 - rs0) * es, rxs.size());
        r.sinks.resize(r.rp.off.size());
        r.done.assign(r.rp.off.size(), 0);
        r.remaining = 0;
        for (size_t k = 0; k < r.rp.off.size(); ++k) {
            if (r.rp.len[k] == 0) continue;
            r.sinks[k] = rx_conn(k)->post_sink(tag, seq, rxbuf[b] + sink_shift(g) + r.rp.off[k], r.rp.len[k]);
            ++r.remaining;
        }
        r.posted = true;
    };
    auto unpost = [&](size_t g) {
        StepRx &r = srx[g];
        if (!r.posted) return;
        for (size_t k = 0; k < r.sinks.size(); ++k)
            if (r.sinks[k]) rx_conn(k)->remove_sink(tag, r.sinks[k]);
        r.sinks.clear();
        r.posted = false;
    };
    struct Unposter { // sinks must never outlive their buffers (also on failure)
        std::function<void()> fn;
        ~Unposter() { fn(); }
    } unposter{[&] {
        for (size_t g = 0; g < nsteps; ++g) unpost(g);
    }};

    for (size_t g = 0; g < nsteps; ++g) {
        const size_t b = g % kNb, nb = (g + 1) % kNb;
        const bool rs = is_rs(g);
        if (!L.ahead && g > 0 && !senders.wait(g - 1)) return fail_all(1);
        // 1. step g's sinks (normally posted during step g-1)
        while (!srx[g].posted) {
            if (can_post(g)) {
                post(g);
                break;
            }
            if (senders.failed()) return fail_all(1);
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        // 2. this step's reduce writes txbuf[nb], last read by step g-2's sends
        uint8_t *region = region_of(g);
        const size_t shift = reinterpret_cast<uintptr_t>(region) % 16;
        if (rs) {
            if (g >= 2 && !senders.wait(g - 2)) return fail_all(1);
            txready[nb].clear();
            txshift[nb] = shift;
        }
        // own input of the host-reduced part of steps g (first step only) and g+1, one step ahead
        if (host_red) {
            if (g == 0) stage_local(0);
            stage_local(g + 1);
        }
        // 3. own input chunk -> pinned, in pieces (from src: ready at call time, never written here)
        if (g == 0) {
            const auto [ts, te] = bounds[chunk_tx(0)];
            txready[0].clear();
            txshift[0] = 0;
            DevStream q0 = L.step0_on_op_stream ? st : pq.d2h;
            for (size_t off = 0; off < (te - ts) * es; off += piece) {
                const size_t n = std::min(piece, (te - ts) * es - off);
                be->memcpy_async(txbuf[0] + off, L.src + ts * es + off, n, q0);
                DevEvent e = record(q0);
                if (!L.step0_on_op_stream) last_d2h = e;
                txready[0].add(off, off + n, e);
            }
        }
        publish(g);
        if (L.ahead && g + 1 < nsteps) publish(g + 1); // its payload fills while this step runs
        if (g + 1 == ws - 1 && L.open_gate) L.open_gate->signal(); // next step is this lane's all-gather
        // 4. receive + consume step g
        StepRx &r = srx[g];
        uint8_t *sink = rxbuf[b] + sink_shift(g);
        DevEvent last_red = nullptr;
        std::array<DevEvent, PcieQueues::kMaxH2d> step_h2d{}; // this step's last copy per queue
        auto h2d_queue = [&] { return h2d_rr++ % pq.nh2d; };
        std::function<void(size_t, size_t)> consume;
        // the all-gather overwrites regions this lane's reduce-scatter kernels wrote: with those on the shared stream,
        // the lane stream (which takes the all-gather copies) waits for the last of them first
        if (!rs && g + 1 == ws && shared_red && lane_last_red) be->stream_wait_event(st, lane_last_red);
        if (rs) {
            // HBM staging and the next payload share the 16-byte phase of `region`: the fused kernel stays vectorised
            uint8_t *stage = rxdev[b] + shift, *out = txbuf[nb] + shift;
            const size_t hb = host_elems(g);
            bool loc_waited = false;
            consume = [&, stage, out, sink, region, nb, hb, g](size_t a, size_t e) {
                if (a < hb) { // CPU part: out = op(own input, received), straight into the next payload
                    const size_t he = std::min(e, hb);
                    if (!loc_waited) {
                        event_wait_polling(be, loc_ready[g % 2]);
                        loc_waited = true;
                    }
                    kernels::host_reduce3(out + a * es, locbuf[g % 2] + a * es, sink + a * es, he - a, L.dtype,
                                          L.rop);
                    txready[nb].add(a * es, he * es, nullptr);
                    a = he;
                    if (a >= e) return;
                }
                const size_t off = a * es, n = (e - a) * es;
                if (shared_red) { // copy engine -> HBM staging, then the reduce on the process-wide stream
                    std::lock_guard l(*pq.red_mtx);
                    const size_t qi = h2d_queue();
                    be->memcpy_async(stage + off, sink + off, n, pq.h2d[qi]);
                    DevEvent ce = record(pq.h2d[qi]);
                    last_h2d[qi] = step_h2d[qi] = ce;
                    be->stream_wait_event(rst, ce);
                    be->reduce_copy(region + off, stage + off, out + off, e - a, L.dtype, L.rop, rst);
                    lane_last_red = last_red = record(rst);
                    txready[nb].add(off, off + n, last_red);
                    return;
                }
                if (L.rs_h2d == 2) { // the kernel reads the received piece straight from pinned memory
                    be->reduce_copy(region + off, sink + off, out + off, e - a, L.dtype, L.rop, st);
                } else {
                    if (L.rs_h2d == 1) {
                        be->memcpy_async(stage + off, sink + off, n, st);
                    } else {
                        const size_t qi = h2d_queue();
                        be->memcpy_async(stage + off, sink + off, n, pq.h2d[qi]);
                        DevEvent ce = record(pq.h2d[qi]);
                        last_h2d[qi] = step_h2d[qi] = ce;
                        be->stream_wait_event(st, ce);
                    }
                    be->reduce_copy(region + off, stage + off, out + off, e - a, L.dtype, L.rop, st);
                }
                last_red = record(st);
                txready[nb].add(off, off + n, last_red);
            };
        } else {
            consume = [&, sink, region, b](size_t a, size_t e) {
                if (shared_red && L.shared_ag) { // our copy kernel on the process-wide stream, after the reduces
                    std::lock_guard l(*pq.red_mtx);
                    be->copy_kernel(region + a * es, sink + a * es, (e - a) * es, L.ag_copy_grid, rst);
                    lane_last_red = last_h2d[0] = step_h2d[0] = record(rst);
                    rxready[b].add(a * es, e * es, nullptr);
                    return;
                }
                if (L.ag_on_lane_stream) { // blit kernel reading pinned memory, on this lane's stream
                    if (L.ag_copy_grid > 0)
                        be->copy_kernel(region + a * es, sink + a * es, (e - a) * es, L.ag_copy_grid, st);
                    else
                        be->memcpy_async(region + a * es, sink + a * es, (e - a) * es, st);
                    last_h2d[0] = step_h2d[0] = record(st);
                    rxready[b].add(a * es, e * es, nullptr);
                    return;
                }
                const size_t qi = h2d_queue();
                be->memcpy_async(region + a * es, sink + a * es, (e - a) * es, pq.h2d[qi]);
                last_h2d[qi] = step_h2d[qi] = record(pq.h2d[qi]);
                rxready[b].add(a * es, e * es, nullptr); // in host memory: forwardable at once
            };
        }
        const size_t gran_el = std::max<size_t>(1, piece / es);
        int rc = 0;
        size_t idle = 0, rr = 0;
        while (r.remaining > 0) {
            bool progress = false;
            for (size_t k = 0; k < r.sinks.size(); ++k) {
                if (!r.sinks[k]) continue;
                const size_t want = r.rp.len[k] / es;
                if (r.done[k] >= want) continue;
                const size_t have = net::MuxConn::sink_progress(r.sinks[k]) / es;
                if (have > r.done[k] && (have - r.done[k] >= gran_el || have >= want)) {
                    const size_t e0 = r.rp.off[k] / es;
                    consume(e0 + r.done[k], e0 + have);
                    r.done[k] = have;
                    progress = true;
                    if (r.done[k] >= want) --r.remaining;
                }
            }
            // post the next step's sinks as soon as its buffer is free (its sender may already be streaming)
            if (L.ahead && g + 1 < nsteps && !srx[g + 1].posted && can_post(g + 1)) post(g + 1);
            if (r.remaining == 0 || progress) {
                idle = 0;
                continue;
            }
            size_t k = rr++ % r.sinks.size();
            while (!r.sinks[k] || r.done[k] >= r.rp.len[k] / es) k = rr++ % r.sinks.size();
            net::MuxConn *c = rx_conn(k);
            c->wait_sink(r.sinks[k], std::min(r.rp.len[k], (r.done[k] + gran_el) * es), 5ms);
            if (!c->is_open() || senders.failed()) {
                rc = 1;
                break;
            }
            if (++idle % 8 == 0 && L.aborted()) {
                rc = 2;
                break;
            }
        }
        h2d_done[b] = step_h2d;
        red_done[b] = last_red;
        if (rc) return fail_all(rc);
        *L.rx += (bounds[chunk_rx(g)].second - bounds[chunk_rx(g)].first) * es;
        unpost(g);
        if (!L.ahead && !senders.wait(g)) return fail_all(1); // classic schedule: a step ends when its sends are done
        if (L.main_lane) {
            step_mark(rs, rs ? g : g - (ws - 1));
            if (g == 0) fault_point("ring_step", seq);
            if (g + 2 == ws) trace_mark("reduce_scatter");
        }
    }
    if (!senders.wait(nsteps - 1)) return fail_all(1);
    if (L.open_gate) L.open_gate->signal();
    // the lane is complete once its last received bytes landed in HBM (the Drain waits for them)
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
        return {true, false};
    }
    PcieQueues pq;
    StreamLease own_h2d(device), own_d2h(device);
    if (env_size("PCCL_SHARED_COPY_QUEUES", 1) != 0) {
        pq = shared_pcie_queues(be, device);
    } else { // A/B switch: per-op copy streams
        pq.h2d[0] = own_h2d.get();
        pq.nh2d = 1;
        pq.d2h = own_d2h.get();
    }
    if (!pq.h2d[0] || !pq.d2h) return {false, false};

    // the caller's input -> dst (out of place) or a backup of it (in place, restored on abort), on the op stream
    Lease backup;
    if (q.src == q.dst && !q.scratch) {
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
            be->stream_sync(st);
            event_pool().put(e);
        }
    } ev_back{be, st, ready};
    be->event_record(ready, st);

    // Lanes: the buffer is split into PCCL_RING_LANES contiguous parts, each a complete ring all-reduce with its own
    // tag (the op's tag with the lane number in bits 60-63), stream and staging rings; lane k+1 starts when lane k
    // reaches its all-gather. The all-gather moves bytes host -> device only while a reduce-scatter moves them both
    // ways, so overlapping lane k's all-gather with lane k+1's reduce-scatter keeps both PCIe directions busy.
    const size_t lanes_req = std::max<size_t>(1, std::min<size_t>(4, env_size("PCCL_RING_LANES", 1)));
    const size_t align_el = std::max<size_t>(1, 4096 / es);
    size_t nl = lanes_req;
    while (nl > 1 && q.count / nl < ws * piece / es) --nl; // every lane keeps >= one piece per chunk
    std::vector<size_t> lo(nl + 1, 0);
    for (size_t k = 1; k < nl; ++k) lo[k] = std::min(q.count, (q.count * k / nl) / align_el * align_el);
    lo[nl] = q.count;
    std::vector<LaneGate> gates(nl);
    std::vector<std::unique_ptr<StreamLease>> lane_streams;
    std::vector<Lane> lanes(nl);
    for (size_t k = 0; k < nl; ++k) {
        lane_streams.push_back(std::make_unique<StreamLease>(device));
        if (!lane_streams.back()->get()) return {false, false};
        Lane &L = lanes[k];
        L.txs = &rv.tx;
        L.rxs = &rv.rx;
        L.ws = ws;
        L.rank = rank;
        L.tag = q.tag ^ (static_cast<uint64_t>(k) << 60);
        L.seq = seq;
        L.be = be;
        L.pq = pq;
        L.st = lane_streams.back()->get();
        L.ready = ready;
        L.src = static_cast<const uint8_t *>(q.src) + lo[k] * es;
        L.dst = dst + lo[k] * es;
        L.count = lo[k + 1] - lo[k];
        L.es = es;
        L.piece = piece;
        L.dtype = q.dtype;
        L.rop = q.op;
        L.device = device;
        L.ahead = env_size("PCCL_RING_SEND_AHEAD", 1) != 0;
        // step-0 payload (own input chunk -> pinned): on the process-wide D2H copy queue (default; FIFO across the
        // peers of this process) or on the lane's stream (PCCL_RING_STEP0_OP_STREAM=1: blit kernels, per-peer copies
        // run concurrently). 8 peers x 1 GiB, 32 MiB pieces, 3 runs each: queue 358 / 337 / 341 ms, op stream 331 /
        // 429 / 388 ms (profiles/r3/ring_ab/summary.txt).
        L.step0_on_op_stream = env_size("PCCL_RING_STEP0_OP_STREAM", 0) != 0;
        // (the CPU produces the same bits as the kernel, so peers may differ in this setting)
        const char *hr = std::getenv("PCCL_RING_HOST_REDUCE");
        L.host_frac = hr ? std::max(0.0, std::min(1.0, std::atof(hr))) : 0.0;
        // the all-gather's received chunks go to HBM as copies on the lane stream (ROCclr blit kernels reading pinned
        // memory, one per peer in parallel) instead of the shared copy-engine queue, which one stream drives at
        // ~47 GB/s: interleaved A/B, 8 peers x 1 GiB, median of 6-8 windows: 347 vs 376 ms and 337 vs 342 ms on two
        // boxes (profiles/r3/h2d_modes/). The reduce-scatter keeps the copy engine (blit: 366 ms, zero-copy reduce
        // from pinned: 347 ms, copy engine: 337 ms). PCCL_RING_AG_KERNEL_COPY=0 / PCCL_RING_RS_H2D=1|2 for A/B.
        L.ag_on_lane_stream = env_size("PCCL_RING_AG_KERNEL_COPY", 1) != 0;
        L.rs_h2d = static_cast<int>(std::min<size_t>(2, env_size("PCCL_RING_RS_H2D", 0)));
        // PCCL_RING_SHARED_REDUCE=1: the fused reduce-scatter kernels of all device-ring ops of this process on one
        // stream per GPU (the kernels' pinned writes are the device->host traffic of the ring: one writer at a time
        // instead of one per peer). Copy-engine reduce-scatter H2D with the all-gather on the lane stream only.
        L.shared_reduce = env_size("PCCL_RING_SHARED_REDUCE", 0) != 0 && L.rs_h2d == 0 && L.host_frac == 0 &&
                          L.ag_on_lane_stream;
        L.ag_copy_grid = static_cast<int>(std::min<size_t>(4096, env_size("PCCL_RING_AG_COPY_GRID", 0)));
        L.shared_ag = L.shared_reduce && env_size("PCCL_RING_SHARED_AG", 0) != 0;
        L.wait_gate = k > 0 ? &gates[k - 1] : nullptr;
        L.open_gate = k + 1 < nl ? &gates[k] : nullptr;
        L.aborted = [this, t = q.tag] { return abort_received(t); };
        L.tx = &op.tx;
        L.rx = &op.rx;
        L.main_lane = k == 0;
    }
    if (nl == 1) {
        run_lane(lanes[0]);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 1; k < nl; ++k) th.emplace_back([&, k] {
            name_thread("pccl-ring-lane");
            run_lane(lanes[k]);
        });
        run_lane(lanes[0]);
        for (auto &t : th) t.join();
    }
    int rc = 0;
    for (const auto &L : lanes) rc = std::max(rc, L.rc); // abort (2) outranks an io failure (1)
    if (rc != 0) {
        be->stream_sync(st);
        if (q.src == q.dst && !q.scratch) { // every lane drained: restore the caller's buffer
            be->memcpy_async(dst, backup.data(), bytes, st);
            be->stream_sync(st);
        }
        return {rc == 2, rc == 2};
    }
    if (q.op == ReduceOp::Avg) be->finalize_avg(dst, q.count, q.dtype, ws, st);
    if (!be->stream_sync(st)) return {false, false};
    return {true, false};
}

// Quantized device ring: per ring step the owner reduces min/max of its outgoing chunk on the GPU (the metadata
// packet needs them on the host), then quantizes the chunk piece by piece straight into pinned memory; each piece
// is sent as soon as its quantize kernel has finished. The receiver de-quantizes + reduces from pinned memory (the
// wire bytes are 2-4x smaller than the values, so PCIe is not the bound here; the network is).
std::pair<bool, bool> Client::ring_reduce_device_quant(OpState &op, const RingView &rv, uint64_t seq, int device) {
    DeviceBackend *be = device_backend();
    const ReduceRequest &q = op.req;
    const size_t ws = rv.ring.size(), rank = rv.rank;
    const size_t es = dtype_size(q.dtype);
    const size_t qs = dtype_size(q.qtype);
    auto *dst = static_cast<uint8_t *>(q.dst);
    const size_t bytes = q.count * es;
    // value bytes per quantize / de-quantize piece: PCCL_QUANT_PIECE_BYTES, else PCCL_DEVICE_PIECE_BYTES, else 8 MiB
    const size_t piece = std::max<size_t>(1 << 20, env_size("PCCL_QUANT_PIECE_BYTES",
                                                            env_size("PCCL_DEVICE_PIECE_BYTES", 8u << 20))) / es * es;
    const size_t piece_el = piece / es; // quantized pieces hold the same elements

    be->set_device(device);
    StreamLease stream(device);
    DevStream st = stream.get();
    if (!st) return {false, false};

    StepIo io{rv.tx[seq % rv.tx.size()].get(), rv.rx[seq % rv.rx.size()].get(), q.tag, seq};
    auto aborted = [&] { return abort_received(q.tag); };

    Lease backup;
    if (q.src == q.dst && !q.scratch) {
        backup = Lease(device_pool(), bytes, device);
        if (!backup.ok()) return {false, false};
        be->memcpy_async(backup.data(), q.src, bytes, st);
    } else if (q.src != q.dst) {
        be->memcpy_async(dst, q.src, bytes, st);
    }
    auto restore = [&] {
        be->stream_sync(st);
        if (q.src == q.dst && !q.scratch) {
            be->memcpy_async(dst, backup.data(), bytes, st);
            be->stream_sync(st);
        }
    };

    const auto bounds = chunk_bounds(q.count, ws);
    size_t max_chunk = 0;
    for (auto &b : bounds) max_chunk = std::max(max_chunk, b.second - b.first);
    const size_t stage_bytes = max_chunk * qs + 64;
    Lease txbuf(pinned_pool(), stage_bytes), rxa(pinned_pool(), stage_bytes), rxb(pinned_pool(), stage_bytes);
    Lease mm(pinned_pool(), 64);
    if (!txbuf.ok() || !rxa.ok() || !rxb.ok() || !mm.ok()) return {false, false};
    uint8_t *rxbuf[2] = {rxa.data(), rxb.data()};
    auto *minmax_out = reinterpret_cast<double *>(mm.data());

    std::vector<DevEvent> events;
    auto ev = [&](size_t i) {
        while (events.size() <= i) events.push_back(event_pool().get());
        return events[i];
    };
    // Received quantized pieces are copied to HBM on the process's shared copy-engine queue and the de-quantize kernels
    // read them there (PCCL_QUANT_RX_STAGE=0: the kernels read pinned memory over PCIe themselves), like the
    // unquantized ring. Interleaved A/B, uint8, 8 peers x 1 GiB: 249 vs 256 ms and 245 vs 244 ms on two boxes
    // (profiles/r3/quant_fused/ab_rx_stage*.jsonl): the same PCIe bytes either way.
    const bool rx_stage = env_size("PCCL_QUANT_RX_STAGE", 1) != 0;
    Lease dva, dvb;
    uint8_t *rxdev[2] = {nullptr, nullptr};
    PcieQueues pq;
    if (rx_stage) {
        dva = Lease(device_pool(), stage_bytes, device);
        dvb = Lease(device_pool(), stage_bytes, device);
        pq = shared_pcie_queues(be, device);
        if (!dva.ok() || !dvb.ok() || !pq.h2d[0]) return {false, false};
        rxdev[0] = dva.data();
        rxdev[1] = dvb.data();
    }
    std::vector<DevEvent> copy_events; // the staging copies (each waited for by the op stream before its kernel)
    struct EvGuard { // drains the op's stream before its events / staging buffers are recycled
        DeviceBackend *be;
        DevStream s;
        std::vector<DevEvent> *e, *c;
        ~EvGuard() {
            be->stream_sync(s);
            for (auto x : *e) event_pool().put(x);
            for (auto x : *c) event_pool().put(x);
        }
    } eg{be, st, &events, &copy_events};
    // where the kernels read received quantized elements [a, b) of `sink` (after queueing their copy when staging)
    auto rx_src = [&](uint8_t *sink, size_t a, size_t b) -> const uint8_t * {
        if (!rx_stage) return sink + a * qs;
        uint8_t *d = rxdev[sink == rxbuf[0] ? 0 : 1] + a * qs;
        be->memcpy_async(d, sink + a * qs, (b - a) * qs, pq.h2d[0]);
        DevEvent e = event_pool().get();
        copy_events.push_back(e);
        be->event_record(e, pq.h2d[0]);
        be->stream_wait_event(st, e);
        return d;
    };

    // The reduce-scatter's de-quantize-reduce kernels emit per-workgroup (min, max) partials of the values they store
    // (dequant_reduce_minmax) into `mmp`: the chunk a step receives is the chunk the next step quantizes (and the last
    // step's is the all-gather's first payload), so its min / max is one fold of those partials instead of a second
    // pass over the chunk. PCCL_QUANT_FUSED_MINMAX=0 turns it off; a step whose launches do not fit the partials
    // buffer falls back to the separate min / max pass.
    const bool fuse_mm = env_size("PCCL_QUANT_FUSED_MINMAX", 1) != 0;
    constexpr int kMmSlots = 65536, kMmMinRoom = 64; // 1 MiB of partials: ~1 GiB bf16 chunks
    Lease mmp;
    if (fuse_mm) mmp = Lease(device_pool(), kMmSlots * 2 * sizeof(double), device);
    auto *mm_partials = mmp.ok() ? reinterpret_cast<double *>(mmp.data()) : nullptr;
    int mm_used = 0;
    bool mm_complete = false; // the partials cover every element of the chunk consumed by the last step
    auto dequant_consume = [&](uint8_t *dst_el, const uint8_t *src_q, size_t n, ReduceOp rop,
                               const kernels::QuantParams &params) {
        int blocks = 0;
        if (mm_complete && mm_partials && kMmSlots - mm_used >= kMmMinRoom &&
            be->dequant_reduce_minmax(dst_el, src_q, n, q.dtype, q.qtype, rop, params, mm_partials + 2 * mm_used,
                                      kMmSlots - mm_used, &blocks, st)) {
            mm_used += blocks;
            return;
        }
        mm_complete = false;
        be->dequant_reduce(dst_el, src_q, n, q.dtype, q.qtype, rop, params, st);
    };

    // min/max of `n` elements at device `src` (one host round trip: the meta packet carries them) - folded from the
    // previous step's partials when `fused` and they are complete - then the quantize kernels of every piece into
    // pinned txbuf, each followed by an event that releases the piece to the senders
    auto quantize_to_pinned = [&](const uint8_t *src, size_t n, bool fused) -> QuantMeta {
        const bool fold = fused && mm_complete && mm_partials;
        const int folded = mm_used;
        mm_used = 0;
        mm_complete = mm_partials != nullptr; // the next step's consumes start collecting afresh
        if (n == 0) return kernels::make_meta(q.qalgo, q.dtype, q.qtype, 0, 0);
        if (fold) {
            g_quant_minmax_folds.fetch_add(1, std::memory_order_relaxed);
            be->minmax_fold(mm_partials, folded, n, minmax_out, st);
        } else {
            g_quant_minmax_passes.fetch_add(1, std::memory_order_relaxed);
            be->minmax(src, n, q.dtype, minmax_out, st);
        }
        be->stream_sync(st);
        QuantMeta m = kernels::make_meta(q.qalgo, q.dtype, q.qtype, minmax_out[0], minmax_out[1]);
        const auto params = kernels::make_params(m, q.qtype);
        size_t k = 0;
        for (size_t off = 0; off < n; off += piece_el, ++k) {
            be->quantize(txbuf.data() + off * qs, src + off * es, std::min(piece_el, n - off), q.dtype, q.qtype, params,
                         st);
            be->event_record(ev(k), st);
        }
        return m;
    };
    auto quant_ready = [&](size_t end) { return end == 0 || event_wait_polling(be, ev((end - 1) / (piece_el * qs))); };
    auto always_ready = [](size_t) { return true; };

    // No stream synchronisation per step: the reduce-scatter's next quantization reads its min / max after the
    // previous step's de-quantize kernels in stream order (quantize_to_pinned syncs once for the meta packet), and an
    // all-gather step's received bytes are de-quantized asynchronously while the next step forwards them. A pinned
    // sink is refilled two steps later, so step s waits only for the kernels that read its sink at step s-2.
    DevEvent sink_read[2] = {nullptr, nullptr};
    struct SinkEvents { // back to the pool once the op's stream is drained
        DeviceBackend *be;
        DevStream s;
        DevEvent e[2];
        ~SinkEvents() {
            be->stream_sync(s);
            for (auto x : e) event_pool().put(x);
        }
    } sink_events{be, st, {event_pool().get(), event_pool().get()}};
    // PCCL_QUANT_EARLY_SINKS=1: the data stripes other than stripe 0 (whose connection carries the metadata packet)
    // take their receive sinks before the step waits for the peer's metadata (see striped_step). Interleaved A/B,
    // uint8, 8 peers x 1 GiB: 234.3 vs 233.1 ms (profiles/r3/quant_fused/ab_early_sinks.jsonl), so off by default.
    const bool early_sinks = env_size("PCCL_QUANT_EARLY_SINKS", 0) != 0;
    auto run_step = [&](const uint8_t *payload, size_t tx_bytes, const std::function<bool(size_t)> &tx_ready,
                        uint8_t *sink, size_t rx_bytes, const std::function<void(size_t, size_t)> &consume,
                        const std::function<int()> &before_rx) -> int {
        const int b = sink == rxbuf[0] ? 0 : 1;
        if (sink_read[b]) event_wait_polling(be, sink_read[b]);
        const int rc = striped_step(rv.tx, rv.rx, q.tag, seq, payload, tx_bytes, tx_ready, sink, rx_bytes, qs,
                                    piece_el * qs, consume, aborted, op.tx, op.rx, before_rx, piece_el * qs,
                                    early_sinks ? 1 : SIZE_MAX);
        if (rc == 0) {
            sink_read[b] = sink_events.e[b]; // waited for above before it is recorded again
            be->event_record(sink_read[b], st);
        }
        return rc;
    };
    auto fail = [&](int code) -> std::pair<bool, bool> {
        restore();
        return {code == 2, code == 2};
    };
    auto meta_then = [&](QuantMeta &theirs, kernels::QuantParams &params) {
        return [&, pt = &theirs, pp = &params] {
            const int m = recv_meta(io, *pt, op.rx, aborted);
            if (m == 0) *pp = kernels::make_params(*pt, q.qtype);
            return m;
        };
    };

    // ---- reduce-scatter
    for (size_t step = 0; step + 1 < ws; ++step) {
        const size_t tx_idx = (rank + ws - step) % ws, rx_idx = (rank + ws - step - 1) % ws;
        const auto [ts, te] = bounds[tx_idx];
        const auto [rs, re] = bounds[rx_idx];
        uint8_t *rx_region = dst + rs * es;
        uint8_t *sink = rxbuf[step % 2];
        QuantMeta theirs;
        kernels::QuantParams params{};
        // step > 0: this chunk was produced by the previous step's de-quantize-reduce (fused min / max partials)
        const QuantMeta mine = quantize_to_pinned(dst + ts * es, te - ts, step > 0);
        if (int m = send_meta(io, mine, op.tx)) return fail(m);
        const int rc = run_step(txbuf.data(), (te - ts) * qs, quant_ready, sink, (re - rs) * qs, [&](size_t a, size_t b) {
            dequant_consume(rx_region + a * es, rx_src(sink, a, b), b - a, q.op, params);
        }, meta_then(theirs, params));
        if (rc) return fail(rc);
        step_mark(true, step);
    }

    trace_mark("reduce_scatter");
    // ---- all-gather: the owner quantizes its finished chunk once and overwrites its own copy with D(Q(x)) (every
    // peer ends bit-identical); received quantized chunks are forwarded verbatim
    QuantMeta prev_meta;
    size_t cur = (rank + 1) % ws;
    for (size_t step = 0; step + 1 < ws; ++step) {
        const size_t inc = (cur + ws - 1) % ws;
        const auto [ts, te] = bounds[cur];
        const auto [rs, re] = bounds[inc];
        uint8_t *rx_region = dst + rs * es;
        uint8_t *sink = rxbuf[step % 2];
        const uint8_t *payload;
        QuantMeta mine, theirs;
        std::function<bool(size_t)> ready = always_ready;
        if (step == 0) {
            mine = quantize_to_pinned(dst + ts * es, te - ts, true); // the reduce-scatter's last received chunk
            if (te > ts) // parity: own chunk := D(Q(x))
                be->dequant_reduce(dst + ts * es, txbuf.data(), te - ts, q.dtype, q.qtype, ReduceOp::Set,
                                   kernels::make_params(mine, q.qtype), st);
            payload = txbuf.data();
            ready = quant_ready;
        } else {
            mine = prev_meta;
            payload = rxbuf[(step - 1) % 2];
        }
        if (int m = send_meta(io, mine, op.tx)) return fail(m);
        kernels::QuantParams params{};
        const int rc = run_step(payload, (te - ts) * qs, ready, sink, (re - rs) * qs, [&](size_t a, size_t b) {
            be->dequant_reduce(rx_region + a * es, rx_src(sink, a, b), b - a, q.dtype, q.qtype, ReduceOp::Set, params,
                               st);
        }, meta_then(theirs, params));
        prev_meta = theirs;
        if (rc) return fail(rc);
        step_mark(false, step);
        cur = inc;
    }
    if (q.op == ReduceOp::Avg) be->finalize_avg(dst, q.count, q.dtype, ws, st);
    if (!be->stream_sync(st)) return {false, false};
    return {true, false};
}

} // namespace pccl::client

// [0] quantized-ring payloads whose min / max came from the fused de-quantize partials, [1] separate min / max passes
extern "C" __attribute__((visibility("default"))) void pcclxQuantStats(uint64_t *out2) {
    out2[0] = pccl::client::g_quant_minmax_folds.load(std::memory_order_relaxed);
    out2[1] = pccl::client::g_quant_minmax_passes.load(std::memory_order_relaxed);
}
