// Shared machinery of the ring all-reduce data paths (host ring, device ring, quantized device ring): chunking, the
// agreed data-plane shape and framing (striping over pooled connections, quantized metadata, reference framing), the
// per-op send threads (OpSenders), the posted receive sinks (RingRx), payload readiness (ReadyRanges) and the
// staging-slot discipline of a pipelined op (StepSlots).
//
// Algorithm (reference ccoip/src/cpp/reduce.cpp:528-784): chunk r = [r*base + min(r, rem), ...), ws-1 reduce-scatter
// steps sending chunk (rank - step) and accumulating chunk (rank - step - 1), then ws-1 all-gather steps forwarding the
// owned chunk. With quantization the owner quantizes its finished chunk once, overwrites its own copy with D(Q(x)) (so
// every peer ends bit-identical), and received quantized chunks are forwarded verbatim.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../common/device_backend.hpp"
#include "../common/trace.hpp"
#include "../net/mux.hpp"
#include "../proto/packets.hpp"
#include "pools.hpp"

namespace pccl::client::ring {

using Conns = std::vector<std::shared_ptr<net::MuxConn>>;

// element range [first, second) of chunk r of `total` elements over `ws` peers (remainder to the low ranks)
std::vector<std::pair<size_t, size_t>> chunk_bounds(size_t total, size_t ws);

// chunk index a peer sends / receives at global ring step g (reduce-scatter steps 0 .. ws-2, then all-gather)
inline size_t chunk_tx(size_t g, size_t rank, size_t ws) {
    return g + 1 < ws ? (rank + ws - g) % ws : (rank + 1 + ws - (g - (ws - 1)) % ws) % ws;
}
inline size_t chunk_rx(size_t g, size_t rank, size_t ws) { return (chunk_tx(g, rank, ws) + ws - 1) % ws; }

// ------------------------------------------------------------------------------------------------------------------
// the op's data-plane shape (agreed per op through the master: proto::WireShape, kCollFlagExtWire)
// ------------------------------------------------------------------------------------------------------------------
struct Shape {
    // reference framing (a participant without the extension, or PCCL_WIRE=reference): every step of the op on
    // connection seq % pool, no striping, one quantized lane, the dequantization packet on the data tag before the
    // step's data (reference reduce.cpp:149-192)
    bool reference = false;
    size_t stripes = 4;             // striped connections per step
    size_t stripe_min = 8u << 20;   // smallest stripe (bytes)
    size_t quant_lanes = 2;         // lanes of a quantized op
    size_t segment_chunk = 128u << 20; // largest ring chunk of one segment, value bytes (0: the op is one segment)
    // bytes of the op's largest ring step (op_shape; 0: not derived, stripe_conn assumes `stripes`): every peer
    // derives it from the op's agreed values; with the size of a connection pool it gives the op's stripe count on
    // that pool (stripe_count), the same at both of its ends even when neighbours' pools differ in size
    size_t op_max_step = 0;
    static Shape from_wire(const proto::WireShape &w);
    static Shape reference_framing();
};
// this peer's proposal for its ops (PCCL_RING_STRIPES, PCCL_STRIPE_MIN_BYTES, PCCL_QUANT_LANES)
proto::WireShape local_wire_shape();

// Quantized ring: the buffer is split into lanes (quant_lane_bounds), each a complete ring all-reduce over a
// contiguous part with its own data tag (lane_tag) and its own metadata tag (meta_tag). Per ring step a peer sends
// the step's dequantization metadata packet on the metadata tag and the quantized payload striped on the data tag.
// Keeping the packets off the data tag lets a peer post every receive sink of a step (and the next step's) before the
// packet arrives: the reference sends the packet on the data tag and waits for the peer's before any data moves
// (reference reduce.cpp:154-192), one extra latency per ring step; the reference framing (Shape::reference) does
// exactly that. Host and device rings speak the same protocol, so CPU and GPU peers mix in one quantized ring.
constexpr uint64_t kMetaTagBit = 1ull << 63;
inline uint64_t lane_tag(uint64_t tag, size_t lane, size_t lanes) {
    return tag ^ (static_cast<uint64_t>(lane) << 60) ^ (static_cast<uint64_t>(lanes - 1) << 58);
}
// Lane split of a quantized all-reduce of `count` elements (wire element size `qs`) over `ws` peers: element offsets
// lo[0] = 0 < lo[1] < ... < lo[nl] = count, from values every peer shares (count, ring size, wire type, agreed shape).
std::vector<size_t> quant_lane_bounds(size_t count, size_t ws, size_t qs, const Shape &shape);

// Segments: an op (or a quantized lane) of `count` elements of `es` value bytes is run as consecutive ring
// all-reduces over contiguous element ranges, each small enough that one ring chunk holds at most
// shape.segment_chunk bytes, so every per-step staging buffer (pinned TX / RX, HBM) is bounded by the segment instead
// of growing with the tensor. The pipelined device rings run the segments as one pipeline (the next segment's first
// payload is staged while the current one's last step still receives). Offsets lo[0] = 0 < ... < lo[S] = count,
// multiples of 4096 elements, from values every peer shares; one segment in the reference framing.
std::vector<size_t> segment_bounds(size_t count, size_t es, size_t ws, const Shape &shape);

// Striping: a large ring-step payload is split into up to `stripes` contiguous stripes, each sent on its own pooled
// TCP connection (one loopback / WAN TCP stream tops out well below the NIC / memory bandwidth). Stripe boundaries
// depend only on (bytes, connection count, agreed shape), so sender and receiver derive the same plan: the sender's
// pool to `next` is exactly the receiver's RX pool from `prev`.
struct StripePlan {
    std::vector<size_t> off, len;
};
constexpr size_t kStripeAlign = 256 << 10; // multiple of every element size (and 16-byte vector phase)
StripePlan plan_stripes(size_t bytes, size_t conns, const Shape &shape);
// Connection of stripe k of op `seq` (data tag `tag`) in a pool of `pool`. Pccl-amd framing: consecutive ops, and the
// lanes of one quantized op (lane_tag: lane in bits 60-61, lane count - 1 in bits 58-59), take consecutive groups of
// op_stripes(shape, pool) connections, so concurrent ops spread over the whole pool (a long-fat pipe is filled by many concurrent
// ops, reference src/pccl.cpp:345-523). Reference framing: seq % pool (reference reduce.cpp:149-151).
size_t stripe_conn(uint64_t seq, uint64_t tag, size_t k, size_t pool, const Shape &shape);
// `shape` for one op (or quantized lane) whose largest ring step carries `max_step_bytes` over `conns` connections
Shape op_shape(const Shape &shape, size_t max_step_bytes);
// stripes plan_stripes(bytes, conns, shape) makes (without building the plan)
size_t stripe_count(size_t bytes, size_t conns, const Shape &shape);
// upper bound of the stripes of every step of the op on a pool of `conns` connections (the size of its connection
// group and the number of its sender threads; shape.stripes if op_max_step is unset)
size_t op_stripes(const Shape &shape, size_t conns);

// Progress watch of the op whose data path runs on this thread (Client::run_op installs it; run_lanes hands it to
// its lane threads). The data paths publish the ring step they wait in; the client's liveness thread sets `failed`
// when the op made no progress for PCCL_OP_STALL_MS and the master did not resolve the stall (or cannot: a reference
// master), and every receive loop then returns an io failure.
struct OpWatch {
    std::atomic<uint32_t> step{0};
    std::atomic<bool> failed{false};
};
OpWatch *&current_watch();
inline void watch_step(size_t g) {
    if (OpWatch *w = current_watch()) w->step.store(static_cast<uint32_t>(g), std::memory_order_relaxed);
}
inline bool watch_failed() {
    const OpWatch *w = current_watch();
    return w != nullptr && w->failed.load(std::memory_order_acquire);
}

// Abort state of one op shared by all of its threads: the first poll that sees the master's abort packet
// (Client::abort_received, which leaves it queued for run_op's completion protocol) records it here, so the other
// threads of the op stop scanning the master queue.
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

// Where a quantized step's metadata packet travels: connections (the op's first stripe connection), tag (meta_tag of
// the lane's data tag, or the data tag itself in the reference framing) and the packet's own tag field.
struct StepIo {
    net::MuxConn *tx;
    net::MuxConn *rx;
    uint64_t tag;     // frame tag of the metadata packets
    uint64_t seq;
    uint64_t pkt_tag; // P2PDequantizationMeta::tag (the lane's data tag)
};
StepIo step_io(const Conns &txs, const Conns &rxs, uint64_t data_tag, uint64_t seq, const Shape &shape);
// tx / rx byte accounting of a metadata packet, exactly as the reference counts it (reduce.cpp:162-165,186-189): its
// LTV header (u64 length + u16 id = 10 bytes) plus P2PPacketDequantizationMeta::serializedSize() = tag 8 + meta type 1
// + 4 + |min value| + 4 + |max value| (ccoip_packets.cpp:543-548; both value vectors are empty for zero-point-scale):
// 35 bytes for a float min-max packet, 27 for zero-point-scale, whatever the encoded size. Frame preambles are not
// counted (reduce.cpp:212).
inline size_t meta_accounting_bytes(const proto::QuantMeta &m) {
    return 10 + 8 + 1 + 4 + 4 + (m.algo == QuantAlgo::MinMax ? 2 * dtype_size(m.value_type) : 0);
}
// Returns 0 ok, 1 io failure.
int send_meta(const StepIo &io, const proto::QuantMeta &mine, std::atomic<uint64_t> &tx);
// Waits for the peer's metadata of the next step (the packets of a lane arrive in step order). Returns 0 ok, 1 io
// failure, 2 abort.
int recv_meta(const StepIo &io, proto::QuantMeta &theirs, std::atomic<uint64_t> &rx, const std::function<bool()> &aborted,
              const std::function<bool()> &failed = {});

// One full-duplex ring step over the striped connections. `tx_ready(end)` blocks until payload bytes [0, end) of the
// calling stripe may be sent; `consume(a, b)` processes received elements [a, b) (called from this thread only, any
// order across stripes, in order within a stripe, in batches of at least `gran` bytes unless a stripe ends).
// `before_rx` (optional) runs after the senders started and the receive sinks are posted, before anything is consumed.
// Returns 0 ok, 1 io failure, 2 abort. Stripes are sent by each connection's persistent sender thread
// (MuxConn::post_send_job); steps of at most kInlineSendBytes are sent on the calling thread after the sinks are posted.
constexpr size_t kInlineSendBytes = 256 << 10;
int striped_step(const Conns &txs, const Conns &rxs, uint64_t tag, uint64_t seq, const Shape &shape,
                 const uint8_t *payload, size_t tx_bytes, const std::function<bool(size_t)> &tx_ready, uint8_t *sink,
                 size_t rx_bytes, size_t elem, size_t frame, const std::function<void(size_t, size_t)> &consume,
                 const std::function<bool()> &aborted, std::atomic<uint64_t> &tx_ctr, std::atomic<uint64_t> &rx_ctr,
                 const std::function<int()> &before_rx = {}, size_t gran = 0);

// Small all-reduces (agreed per op, kCollFlagSmallPath): the whole vector travels W-1 ring hops (all-gather) and every
// peer reduces the W vectors locally in ring-index order. Returns 0 ok, 1 io failure, 2 abort; `dst` is written only
// after every hop succeeded.
bool use_small_path(size_t bytes, size_t ws);
int small_allgather_reduce(const Conns &txs, const Conns &rxs, uint64_t tag, uint64_t seq, const Shape &shape,
                           const void *src, void *dst, size_t count, DType dt, ReduceOp op, size_t ws, size_t rank,
                           const std::function<bool()> &aborted, std::atomic<uint64_t> &tx_ctr,
                           std::atomic<uint64_t> &rx_ctr);

// Runs fn(lane, lo, hi) for every lane of `lo` (lane 0 on the calling thread); returns the worst lane result (abort 2
// outranks io failure 1).
int run_lanes(const std::vector<size_t> &lo, const std::function<int(size_t, size_t, size_t)> &fn);

// One ring all-reduce over host memory of `count` elements at `dst` (already holding the input) on data tag `tag`:
// the plain host ring, or one lane of a quantized ring (`quant`). Returns 0 ok, 1 io failure, 2 abort.
struct HostRingArgs {
    const Conns &txs, &rxs;
    size_t ws, rank;
    uint64_t tag, seq;
    const Shape &shape;
    uint8_t *dst;
    size_t count;
    DType dtype, qtype;
    QuantAlgo qalgo;
    ReduceOp op;
    bool quant;
    std::function<bool()> aborted;
    std::atomic<uint64_t> &tx, &rx;
};
int host_ring(const HostRingArgs &A);
// The whole host-memory all-reduce of `count` elements at `dst` (holding the input): lanes of the quantized ring or
// the plain ring, then the AVG finalisation. Returns 0 ok, 1 io failure, 2 abort.
int host_allreduce(const Conns &txs, const Conns &rxs, size_t ws, size_t rank, uint64_t tag, uint64_t seq,
                   const Shape &shape, uint8_t *dst, size_t count, DType dtype, DType qtype, QuantAlgo qalgo,
                   ReduceOp op, const std::function<bool()> &aborted, std::atomic<uint64_t> &tx,
                   std::atomic<uint64_t> &rx);

// ------------------------------------------------------------------------------------------------------------------
// device pipelines
// ------------------------------------------------------------------------------------------------------------------
struct PcieQueues {
    DevStream h2d = nullptr; // received pieces -> HBM staging
    DevStream d2h = nullptr; // step-0 payload pieces -> pinned
};
// process-wide copy queues of `device` (never destroyed: they may outlive static destruction order)
PcieQueues shared_pcie_queues(DeviceBackend *be, int device);

// Host <-> device bytes the device rings move across the GPU's PCIe link (copies between pinned staging and HBM, and
// kernels that read / write pinned memory), per process: what a multi-GPU run's per-GPU link carries per op
// (pcclxPcieStats). Counted where the work is queued.
void pcie_note(size_t h2d, size_t d2h);
void pcie_read(uint64_t &h2d, uint64_t &d2h);

// per-step phase marks for PCCL_TRACE_OPS (first 16 steps of each phase)
void step_mark(bool reduce_scatter, size_t step);
// finer per-step marks (global step g < 32): `kind` q = payload metadata known and its quantize kernels queued,
// f = first received piece consumed
void step_sub_mark(char kind, size_t g);

// Waits until every piece of work queued on `s` so far has completed, sleeping between polls (hipStreamSynchronize
// busy-waits: with many lanes syncing once per ring step that took the process's CPU share from the socket copies)
bool stream_wait_polling(DeviceBackend *be, DevStream s);

// payload bytes [a, b) of a pinned staging buffer become valid once `e` has completed (nullptr: already valid)
struct Staged {
    size_t a, b;
    DevEvent e;
};

// Readiness of one ring step's payload, shared between the op thread that produces it (staging copies, the fused
// reduce, received bytes) and the connections' sender threads that send it while it is still being produced
// (send-ahead). A range is readable once its event (nullptr: none) has completed. Ranges arrive in any order across
// the producer's stripes, and the sender's stripe plan need not match the producer's, so a wait covers the whole byte
// range it sends.
class ReadyRanges {
public:
    void clear();
    void add(size_t a, size_t b, DevEvent e);
    // blocks until every byte of [begin, end) is readable; false if `cancel` became non-zero first
    bool wait(size_t begin, size_t end, DeviceBackend *be, const std::atomic<int> &cancel);

private:
    std::mutex m_;
    std::condition_variable cv_; // signalled by add(): a waiting sender wakes when its range may be complete
    std::vector<Staged> v_;
};

// The send side of one pipelined ring op: one thread per stripe for the whole op (not per step), each sending its
// stripe of every step in order over connection stripe_conn(seq, tag, k). The op thread publishes step g (payload,
// bytes, readiness) as soon as step g may start sending - with send-ahead while step g-1 still receives - and a stripe
// thread streams each piece once it is readable. Per-op threads instead of the connections' shared sender threads: a
// stripe thread may wait on its op's network progress (the previous peer's data), which must never hold up another
// op's sends queued on the same connection (two peers with concurrent ops could otherwise wait on each other).
class OpSenders {
public:
    struct Step {
        const uint8_t *payload = nullptr;
        size_t bytes = 0;
        ReadyRanges *ready = nullptr;
    };
    OpSenders(const Conns &txs, uint64_t tag, uint64_t seq, const Shape &shape, size_t frame, size_t nsteps,
              size_t max_stripes, DeviceBackend *be, std::atomic<uint64_t> &tx_ctr);
    ~OpSenders();
    OpSenders(const OpSenders &) = delete;
    OpSenders &operator=(const OpSenders &) = delete;
    // step g may be sent from now on (steps are published in order)
    void publish(size_t g, const Step &st);
    bool published(size_t g);
    // every stripe of step g has been sent (non-blocking)
    bool sent(size_t g);
    // blocks until every stripe of step g is sent; false on failure / cancel
    bool wait(size_t g);
    // blocks until every stripe of every step is sent; false on failure / cancel
    bool wait_all();
    void cancel();
    bool failed() const { return rc_.load() != 0; }
    // the op's abort poll: wait / wait_all also end (false) once it reports the master's abort or the op's watchdog
    // failed it (a stripe blocked on a peer that stopped reading would otherwise never let them return). The caller
    // must then report the op as aborted if the poll saw the abort (it consumed the master's only abort packet).
    void set_abort(std::function<bool()> abort) { abort_ = std::move(abort); }

private:
    void run(size_t k);
    bool should_stop();
    std::function<bool()> abort_;
    const Conns &txs_;
    const uint64_t tag_, seq_;
    const Shape shape_;
    const size_t frame_;
    DeviceBackend *be_;
    std::atomic<uint64_t> &tx_ctr_;
    std::mutex m_;
    std::condition_variable cv_;
    std::vector<Step> steps_;
    std::vector<size_t> done_;
    size_t published_ = 0;
    size_t running_ = 0; // stripe threads that have not returned yet (guarded by m_)
    std::atomic<int> rc_{0};
    std::vector<std::thread> th_;
};

// The receive side of one pipelined ring op: per step one sink per stripe on the connections from the previous peer.
// Sinks of a tag form a FIFO on each connection, so step g+1's sinks may be posted while step g still receives (the
// previous peer streams both steps back to back on every connection). Sinks never outlive the op: the destructor
// removes every posted one (declare a RingRx after the buffers its sinks point into).
class RingRx {
public:
    RingRx(const Conns &rxs, uint64_t tag, uint64_t seq, const Shape &shape, size_t nsteps)
        : rxs_(rxs), tag_(tag), seq_(seq), shape_(shape), steps_(nsteps) {}
    ~RingRx() {
        for (size_t g = 0; g < steps_.size(); ++g) unpost(g);
    }
    RingRx(const RingRx &) = delete;
    RingRx &operator=(const RingRx &) = delete;

    bool posted(size_t g) const { return steps_[g].posted; }
    // step g receives `bytes` into `buf`
    void post(size_t g, uint8_t *buf, size_t bytes);
    void unpost(size_t g);
    // Receives step g: consume(a, b) for newly arrived bytes [a, b) of the step (multiples of `unit`, at least `gran`
    // bytes per call unless a stripe ends; in order within a stripe, any order across stripes). `between` runs after
    // every scan of the stripes (the caller posts the next step's sinks there). Returns 0 ok, 1 io failure (a
    // connection closed or `failed()`), 2 abort.
    int receive(size_t g, size_t unit, size_t gran, const std::function<void(size_t, size_t)> &consume,
                const std::function<void()> &between, const std::function<bool()> &failed,
                const std::function<bool()> &aborted);

private:
    struct Step {
        StripePlan rp;
        std::vector<net::MuxConn::SinkRef> sinks;
        std::vector<size_t> done; // bytes consumed per stripe
        size_t remaining = 0;     // stripes not yet fully consumed
        bool posted = false;
    };
    net::MuxConn *conn(size_t k) const { return rxs_[stripe_conn(seq_, tag_, k, rxs_.size(), shape_)].get(); }
    const Conns &rxs_;
    const uint64_t tag_, seq_;
    const Shape shape_;
    std::vector<Step> steps_;
};

// The receive staging of a pipelined device op: step g receives into slot g % slots (a pinned buffer, with an HBM
// twin where the path stages through HBM). A slot takes a new step's bytes once the step that used it before
// (g - slots) is finished with it: its GPU work completed (`free_after`) and, in the all-gather, the step after it
// has forwarded its bytes. At least three slots, because step g+1's sinks are posted while step g still receives and
// step g+1's sends run while step g's do; more let a step's sinks be posted while older forwarded bytes still wait
// for a congested downstream link (the quantized ring's small WAN steps).
// Steps are numbered across the op's segments (global step G = segment * 2(ws-1) + ring step).
class StepSlots {
public:
    static constexpr size_t kDefaultSlots = 3, kMaxSlots = 8;
    StepSlots(DeviceBackend *be, RingRx &rx, OpSenders &senders, size_t ws, size_t nsteps, uint8_t *const *bufs,
              size_t slots, std::function<size_t(size_t)> rx_bytes)
        : be_(be), rx_(rx), senders_(senders), ws_(ws), nps_(2 * (ws - 1)), nsteps_(nsteps),
          n_(std::max<size_t>(kDefaultSlots, std::min(slots, kMaxSlots))), rx_bytes_(std::move(rx_bytes)) {
        for (size_t i = 0; i < n_; ++i) buf_[i] = bufs[i];
    }
    size_t slots() const { return n_; }
    uint8_t *buf(size_t g) const { return buf_[g % n_]; }
    ReadyRanges &ready(size_t g) { return ready_[g % n_]; } // received ranges (the all-gather forwards them)
    bool can_post(size_t g) const;
    void post(size_t g);
    // posts step g's sinks (normally already posted during step g-1), waiting for its slot; false if `failed`, the
    // op's watchdog failed it, or `aborted` (the master's abort poll) reports
    bool ensure_posted(size_t g, const std::function<bool()> &failed, const std::function<bool()> &aborted = {});
    // posts step g's sinks if not yet posted and its slot is free (non-blocking; from the receive loop)
    bool try_post(size_t g);
    // the last GPU work reading step g's slot
    void free_after(size_t g, DevEvent e) { free_[g % n_] = e; }

private:
    bool is_rs(size_t g) const { return g % nps_ + 1 < ws_; }
    // step g's received bytes are forwarded by step g+1 (an all-gather step that is not its segment's last)
    bool forwarded(size_t g) const { return !is_rs(g) && g % nps_ + 1 < nps_; }
    DeviceBackend *be_;
    RingRx &rx_;
    OpSenders &senders_;
    size_t ws_, nps_, nsteps_, n_;
    std::function<size_t(size_t)> rx_bytes_;
    uint8_t *buf_[kMaxSlots] = {};
    ReadyRanges ready_[kMaxSlots];
    DevEvent free_[kMaxSlots] = {};
};

// An in-place device op finished its part: keep the input's backup (HBM or pinned) until the master's verdict and
// copy it back into dst if the op failed anyway (OpState::settle).
void settle_device_backup(std::function<void(bool)> &settle, DeviceBackend *be, int device, Lease &&backup,
                          void *dst, size_t bytes);

} // namespace pccl::client::ring
