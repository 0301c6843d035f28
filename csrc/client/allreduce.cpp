// All-reduce op orchestration: initiate -> master consensus (commence, agreed capability flags and data-plane shape)
// -> the data path -> completion protocol (exactly one abort verdict per op) -> settle (reference
// ccoip/src/cpp/ccoip_client_handler.cpp:1187-1396, ccoip_client_state.cpp:184-243). The data paths live in
// ring_host.cpp (host ring), ring_device.cpp / ring_device_quant.cpp (HBM pipelines) and ipc.cpp (xGMI / IPC,
// hierarchical); their shared machinery in ring_common.{hpp,cpp}.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

#include "../common/log.hpp"
#include "../common/spin.hpp"
#include "../common/trace.hpp"
#include "client.hpp"
#include "ipc.hpp"
#include "pools.hpp"
#include "ring_common.hpp"

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


bool Client::abort_received(uint64_t tag) {
    return master_.peek<M2CCollectiveCommsAbort>(
        [tag](const M2CCollectiveCommsAbort &a) { return a.tag == tag && a.aborted; });
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
        run_op(op, true);
    } else {
        if (!fault_delay_armed()) initiate_op(*op);
        arm_ready(*op);
        workers_.submit([this, op] { run_op(op, false); });
    }
    return true;
}

// A stream-ordered op's readiness event, on the submitting thread (before the call returns: it marks the work queued
// on the caller's stream up to this call). If it cannot be recorded the stream is synchronised instead.
void Client::arm_ready(OpState &op) {
    if (!op.req.stream_ordered || op.req.ready) return;
    op.req.stream_ordered = false;
    DeviceBackend *be = device_backend();
    // (an event of the buffers' device: the caller's stream is that device's, whatever the thread's current device)
    DevEvent e = be ? event_pool().get(op.si.is_device ? op.si.device : -1) : nullptr;
    if (e && be->event_record(e, op.req.ready_stream)) {
        op.req.ready = e;
        return;
    }
    event_pool().put(e);
    if (be) be->stream_sync(op.req.ready_stream);
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
    if (rv && rv->ring.size() >= 2 && ring::use_small_path(op.req.count * dtype_size(op.req.dtype), rv->ring.size()) &&
        (op.req.qalgo == QuantAlgo::None || op.req.qtype == op.req.dtype))
        init.flags |= kCollFlagSmallPath;
    if (wire_reference_) {
        init.flags = 0; // PCCL_WIRE=reference: the reference's initiate packet, byte for byte
    } else {
        init.flags |= kCollFlagExtWire; // pccl-amd framing, with this peer's proposed shape
        init.shape = ring::local_wire_shape();
    }
    op.init_sent = master_.send(init);
}

void Client::run_op(const std::shared_ptr<OpState> &op, bool on_caller) {
    const uint64_t tag = op->req.tag;
    low_timer_slack();
    if (!op->initiated) {
        fault_delay(tag);
        initiate_op(*op);
    }
    if (on_caller) arm_ready(*op); // (async ops armed it on the submitting thread before the hand-off)
    OpTrace trace;
    current_trace() = trace_ops_enabled() ? &trace : nullptr;
    char range_name[96];
    std::snprintf(range_name, sizeof(range_name), "pccl all_reduce tag %llu bytes %zu",
                  static_cast<unsigned long long>(tag), op->req.count * dtype_size(op->req.dtype));
    RoctxRange range(range_name);
    bool success = false;
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
            // every participant speaks the extended framing: the master's agreed shape; else the reference framing
            op->shape = (agreed & kCollFlagExtWire) ? ring::Shape::from_wire(c->shape) : ring::Shape::reference_framing();
            commenced = true;
            trace_mark("commence");
        }
    }
    if (op->req.ready) { // stream-ordered op: its input's producers (overlapped with the master round trip)
        if (commenced) {
            // usually complete by now or within microseconds (an idle stream's marker): spin briefly before the
            // sleeping poll, whose 2-100 us back-off would round a short wait up
            DeviceBackend *be = device_backend();
            if (!spin_until([&] { return be->event_query(op->req.ready) != 0; })) event_wait_polling(be, op->req.ready);
            trace_mark("input_ready");
        }
        // a pooled event is never pending: one still in flight (an op that did not commence) is released instead
        DeviceBackend *be = device_backend();
        if (commenced || be->event_query(op->req.ready) != 0) {
            event_pool().put(op->req.ready);
        } else {
            be->destroy_event(op->req.ready);
            event_pool().forget(op->req.ready);
        }
        op->req.ready = nullptr;
    }
    if (commenced) {
        if (rv && rv->ring.size() >= 2) {
            op->world = static_cast<uint32_t>(rv->ring.size());
            std::pair<bool, bool> r{false, false};
            bool done = false, tcp_ring = false;
            if ((agreed & kCollFlagHierarchical) && rv->hier) {
                // every participant announced the capability (master AND): IPC inside hosts, TCP ring across them
                r = hier_reduce(*op, *rv, seq, di.device);
                done = true;
                if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::Hierarchical);
            } else if (rv->arena && device && op->req.count * dtype_size(op->req.dtype) > kIpcMaxOpBytes) {
                // above one arena op's staged size: consecutive xGMI sub-ops (every peer derives the same split)
                bool use_ring = false;
                r = ipc_reduce_segmented(*op, *rv, seq, di.device, use_ring);
                done = !use_ring;
                if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::DeviceIpc);
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
                // the TCP rings run under the stall watchdog (liveness_loop); xGMI barriers watch peers themselves
                ring::current_watch() = &op->watch;
                watch_op(op, *rv);
                if (device) {
                    r = ring_reduce_device(*op, *rv, seq, di.device);
                    if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::DeviceRing);
                    tcp_ring = true;
                } else if ((!si.is_device && !di.is_device) || op->req.count == 0) {
                    r = ring_reduce_host(*op, *rv, seq);
                    if (r.first && !r.second) last_path_ = static_cast<int>(ReducePath::HostRing);
                    tcp_ring = true;
                } else {
                    LOG(ERR) << "all-reduce: send and receive buffers must both be host or both be on one GPU";
                    r = {false, false};
                }
                unwatch_op(op.get());
                ring::current_watch() = nullptr;
            }
            success = r.first && !r.second;
            if (success) last_framing_ = !tcp_ring ? 0 : (op->shape.reference ? 2 : 1);
            if (success) fault_point("op_end", seq); // this peer's part is done, the master has no verdict yet
        } else {
            LOG(WARN) << "all-reduce tag " << tag << ": no usable ring (peers lost)";
        }
    }
    // completion protocol: exactly one Abort(tag) packet per op, then Complete(tag). The op's polls only peek at the
    // abort (abort_received), so it is taken here whether or not they saw it: a poll that took it while the op went
    // on to finish (a step's last sends completing after the poll) left this wait with nothing to receive.
    bool ok = false;
    if (commenced) {
        C2MCollectiveCommsComplete comp;
        comp.tag = tag;
        comp.was_aborted = !success;
        if (master_.send(comp)) {
            auto a = master_.receive<M2CCollectiveCommsAbort>(
                [tag](const M2CCollectiveCommsAbort &p) { return p.tag == tag; });
            auto c = master_.receive<M2CCollectiveCommsComplete>(
                [tag](const M2CCollectiveCommsComplete &p) { return p.tag == tag; });
            ok = a.has_value() && c.has_value() && !a->aborted && success;
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
        // t0: the op thread's start on the host-wide monotonic clock (us), so traces of several processes line up
        const auto t0_us = std::chrono::duration_cast<std::chrono::microseconds>(trace.t0.time_since_epoch()).count();
        std::fprintf(stderr, "[pccl-trace] tag %llu seq %llu bytes %zu world %u t0 %lld path %s %s%s\n",
                     static_cast<unsigned long long>(tag), static_cast<unsigned long long>(seq),
                     op->req.count * dtype_size(op->req.dtype), op->world, static_cast<long long>(t0_us),
                     names[last_path_.load() & 7], ok ? "ok" : "FAILED", trace.str().c_str());
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
    // Re-establish the ring once per connection revision after a failed op: every peer sees the same failures, so
    // every peer performs exactly one establishment round (several concurrent failed ops must not cascade into more;
    // reference ccoip_client_handler.cpp:1349-1367). Ops still in flight keep this peer in the master's
    // COLLECTIVE_COMMUNICATIONS_RUNNING state, where an establish vote is illegal: the round is then left pending and
    // performed by the next join with nothing running - whether that op failed or succeeded, so a peer whose last
    // joined op succeeded still joins the round its peers are waiting in.
    if (op->success && reestablish_pending_.load() == UINT64_MAX) return true; // (the common path takes no lock)
    std::lock_guard lock(establish_mtx_);
    if (!op->success && conn_revision_.load() == op->revision_at_start) reestablish_pending_ = op->revision_at_start;
    if (reestablish_pending_.load() != UINT64_MAX && !interrupted_ && !any_collective_running()) {
        const bool due = reestablish_pending_.load() == conn_revision_.load();
        reestablish_pending_ = UINT64_MAX;
        if (due && !request_and_establish_locked(false)) {
            LOG(ERR) << "Failed to re-establish P2P connections after abort";
        }
    }
    return op->success;
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

} // namespace pccl::client

// Staging pools of this process: [0..2] pinned host (in use, peak in use, cached free), [3..5] HBM, [6..8] plain host
// bytes; [9..11] fresh runtime allocations of the pinned / HBM / host pool and [12..14] the microseconds they took.
// Returns how many counters exist (writes at most n). `reset` restarts the peaks at the current use.
extern "C" __attribute__((visibility("default"))) size_t pcclxPoolStats(uint64_t *out, size_t n, int reset) {
    using namespace pccl::client;
    BufferPool *pools[3] = {&pinned_pool(), &device_pool(), &host_pool()};
    constexpr size_t kN = 15;
    uint64_t v[kN];
    for (int k = 0; k < 3; ++k) {
        v[3 * k] = pools[k]->in_use();
        v[3 * k + 1] = pools[k]->peak();
        v[3 * k + 2] = pools[k]->cached();
        v[9 + k] = pools[k]->allocs();
        v[12 + k] = pools[k]->alloc_us();
        if (reset) pools[k]->reset_peak();
    }
    for (size_t i = 0; i < n && i < kN; ++i) out[i] = v[i];
    return kN;
}

// Fills the staging pools ahead of the first ops: leases `pinned_count` pinned buffers of `pinned_bytes` and
// `device_count` HBM buffers of `device_bytes` on `device` at once and hands them back to the pools, which keep them
// cached (PCCL_POOL_MAX_FREE_MIB). An application can run it next to connect(), whose admission wait it overlaps
// (RCCL allocates its buffers at communicator init; these pools otherwise fill on the first op). With HBM buffers it
// also warms the device side a first op would set up (copy queues, a stream, the kernels' code object). 0 on success.
extern "C" __attribute__((visibility("default"))) int pcclxPoolReserve(uint64_t pinned_bytes, uint32_t pinned_count,
                                                                      uint64_t device_bytes, uint32_t device_count,
                                                                      int device) {
    using namespace pccl::client;
    std::vector<Lease> held;
    held.reserve(pinned_count + device_count);
    for (uint32_t i = 0; i < pinned_count && pinned_bytes > 0; ++i) {
        held.emplace_back(pinned_pool(), pinned_bytes);
        if (!held.back().ok()) return 1;
    }
    for (uint32_t i = 0; i < device_count && device_bytes > 0; ++i) {
        if (device < 0 || pccl::device_backend() == nullptr) return 2;
        held.emplace_back(device_pool(), device_bytes, device);
        if (!held.back().ok()) return 1;
    }
    if (device_count > 0 && device_bytes > 0) {
        // the rest of a fresh process's first device op: the process-wide copy queues (created on first use), a
        // pooled stream and the kernels' code object (loaded at the first launch)
        pccl::DeviceBackend *be = pccl::device_backend();
        const int cur = be->current_device(); // (the caller's thread keeps its current device)
        be->set_device(device);
        bool ok = false;
        {
            const ring::PcieQueues pq = ring::shared_pcie_queues(be, device);
            StreamLease st(device);
            Lease h(pinned_pool(), 4096), d(device_pool(), 4096, device);
            ok = h.ok() && d.ok() && pq.h2d && pq.d2h && st.get() &&
                 be->memcpy_async(d.data(), h.data(), 4096, pq.h2d) && be->stream_sync(pq.h2d) &&
                 be->reduce_copy(d.data(), d.data(), h.data(), 16, pccl::DType::F32, pccl::ReduceOp::Sum,
                                 st.get()) &&
                 be->stream_sync(st.get()) && be->memcpy_async(h.data(), d.data(), 4096, pq.d2h) &&
                 be->stream_sync(pq.d2h);
        }
        if (cur >= 0) be->set_device(cur);
        if (!ok) return 1;
    }
    return 0;
}
