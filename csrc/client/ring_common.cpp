// Shared machinery of the ring all-reduce data paths (see ring_common.hpp).
#include "ring_common.hpp"

#include <cstring>
#include <map>

#include "../common/log.hpp"
#include "../common/spin.hpp"
#include "../kernels/host_kernels.hpp"

namespace pccl::client::ring {

using namespace std::chrono_literals;

namespace {
std::atomic<uint64_t> g_pcie_h2d{0}, g_pcie_d2h{0};
}
OpWatch *&current_watch() {
    thread_local OpWatch *w = nullptr;
    return w;
}
void pcie_note(size_t h2d, size_t d2h) {
    if (h2d) g_pcie_h2d.fetch_add(h2d, std::memory_order_relaxed);
    if (d2h) g_pcie_d2h.fetch_add(d2h, std::memory_order_relaxed);
}
void pcie_read(uint64_t &h2d, uint64_t &d2h) {
    h2d = g_pcie_h2d.load(std::memory_order_relaxed);
    d2h = g_pcie_d2h.load(std::memory_order_relaxed);
}

std::vector<std::pair<size_t, size_t>> chunk_bounds(size_t total, size_t ws) {
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

// ------------------------------------------------------------------------------------------------------------------
// shape
// ------------------------------------------------------------------------------------------------------------------
Shape Shape::from_wire(const proto::WireShape &w) {
    Shape s;
    s.stripes = std::max<size_t>(1, std::min<size_t>(16, w.stripes));
    s.quant_lanes = std::max<size_t>(1, std::min<size_t>(4, w.quant_lanes));
    s.stripe_min = std::max<size_t>(256, w.stripe_min_kib) << 10;
    s.segment_chunk = static_cast<size_t>(w.segment_chunk_mib) << 20;
    return s;
}

Shape Shape::reference_framing() {
    Shape s;
    s.reference = true;
    s.stripes = 1;
    s.quant_lanes = 1;
    s.segment_chunk = 0;
    return s;
}

proto::WireShape local_wire_shape() {
    proto::WireShape w;
    w.stripes = static_cast<uint8_t>(std::max<size_t>(1, std::min<size_t>(16, env_size("PCCL_RING_STRIPES", 4))));
    w.quant_lanes = static_cast<uint8_t>(std::max<size_t>(1, std::min<size_t>(4, env_size("PCCL_QUANT_LANES", 2))));
    const size_t min_bytes = std::max<size_t>(256 << 10, env_size("PCCL_STRIPE_MIN_BYTES", 8u << 20));
    w.stripe_min_kib = static_cast<uint16_t>(std::min<size_t>(65535, min_bytes >> 10));
    w.segment_chunk_mib = static_cast<uint16_t>(std::min<size_t>(65535, env_size("PCCL_SEGMENT_CHUNK_MIB", 128)));
    return w;
}

std::vector<size_t> segment_bounds(size_t count, size_t es, size_t ws, const Shape &shape) {
    constexpr size_t kAlign = 4096; // elements
    size_t nseg = 1;
    if (!shape.reference && shape.segment_chunk > 0 && count > 0) {
        const size_t per_seg = std::max(kAlign * ws, shape.segment_chunk / std::max<size_t>(1, es) * ws);
        nseg = (count + per_seg - 1) / per_seg;
    }
    std::vector<size_t> lo(nseg + 1, 0);
    for (size_t k = 1; k < nseg; ++k) lo[k] = count / nseg * k / kAlign * kAlign;
    lo[nseg] = count;
    return lo;
}

// A quantized reduce-scatter step must receive and reduce its whole chunk before the next step's min / max, and so its
// metadata and payload, exist: a single ring leaves its links idle for a step's fill and drain at every step, and
// further lanes fill each other's gaps.
std::vector<size_t> quant_lane_bounds(size_t count, size_t ws, size_t qs, const Shape &shape) {
    constexpr size_t kMinLaneChunk = 8u << 20; // wire bytes per ring chunk and lane
    const size_t max_lanes = shape.reference ? 1 : shape.quant_lanes;
    const size_t nl = std::min(max_lanes, std::max<size_t>(1, count / std::max<size_t>(1, ws) * qs / kMinLaneChunk));
    std::vector<size_t> lo(nl + 1, 0);
    for (size_t k = 1; k < nl; ++k) lo[k] = count / nl * k / 4096 * 4096;
    lo[nl] = count;
    return lo;
}

StripePlan plan_stripes(size_t bytes, size_t conns, const Shape &shape) {
    StripePlan s;
    const size_t p = shape.reference ? 1
                                     : std::min({shape.stripes, std::max<size_t>(1, conns),
                                                 std::max<size_t>(1, bytes / shape.stripe_min)});
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

// Op o (= seq * lanes + lane) uses connections o*s .. o*s + s-1 (mod pool), s = the op's stripe count on this pool
// (op_stripes: the most stripes any of its steps uses; shape.stripes if unset): concurrent ops tile the pool in groups that every one
// of their steps uses in the same order. Ops whose steps need fewer stripes than shape.stripes (64 concurrent 32 MiB
// ops have 1 MiB steps, one stripe each) then still spread over the whole pool: starting them shape.stripes apart
// left 12 of 16 WAN flows idle (64 uint8 ops: 2.0 s per 2 GiB vs 1.07 s with 32 ops). Starts that overlap other
// ops' groups partially measured slower than aligned groups at 16 / 32 ops (1.55-1.64 vs 1.22-1.25 s, 1.40-1.64 vs
// 1.07 s; profiles/r5/b5/): an op's step waits for its slowest stripe, and partly shared connections desynchronise them.
size_t stripe_conn(uint64_t seq, uint64_t tag, size_t k, size_t pool, const Shape &shape) {
    if (shape.reference) return static_cast<size_t>((seq + k) % pool);
    const uint64_t lanes = ((tag >> 58) & 3) + 1, lane = (tag >> 60) & 3;
    const uint64_t s = op_stripes(shape, pool);
    return static_cast<size_t>(((seq * lanes + lane) * s + k) % pool);
}

Shape op_shape(const Shape &shape, size_t max_step_bytes) {
    Shape s = shape;
    s.op_max_step = std::max<size_t>(1, max_step_bytes);
    return s;
}

size_t stripe_count(size_t bytes, size_t conns, const Shape &shape) {
    if (shape.reference) return 1;
    const size_t p = std::min({shape.stripes, std::max<size_t>(1, conns), std::max<size_t>(1, bytes / shape.stripe_min)});
    const size_t per = (bytes / p + kStripeAlign - 1) / kStripeAlign * kStripeAlign;
    // stripes of `per` bytes until the bytes run out (the last one takes the rest); at least one
    return per == 0 ? 1 : std::max<size_t>(1, std::min(p, (bytes + per - 1) / per));
}

// The stripe-count bound min(stripes, conns, bytes / stripe_min) of the op's largest step: it grows with the step
// size, so it bounds the stripes of every step of the op (the stripe count itself does not: rounding stripes up to
// kStripeAlign can give a slightly larger step fewer stripes: with 256 KiB stripes over 4 connections, 2 MiB + 2 KiB
// go in 3 stripes of <= 768 KiB, 2 MiB in 4)
size_t op_stripes(const Shape &shape, size_t conns) {
    if (!shape.op_max_step) return shape.stripes;
    if (shape.reference) return 1;
    return std::min({shape.stripes, std::max<size_t>(1, conns), std::max<size_t>(1, shape.op_max_step / shape.stripe_min)});
}

// ------------------------------------------------------------------------------------------------------------------
// quantization metadata
// ------------------------------------------------------------------------------------------------------------------
StepIo step_io(const Conns &txs, const Conns &rxs, uint64_t data_tag, uint64_t seq, const Shape &shape) {
    return StepIo{txs[stripe_conn(seq, data_tag, 0, txs.size(), shape)].get(),
                  rxs[stripe_conn(seq, data_tag, 0, rxs.size(), shape)].get(),
                  shape.reference ? data_tag : data_tag ^ kMetaTagBit, seq, data_tag};
}

int send_meta(const StepIo &io, const proto::QuantMeta &mine, std::atomic<uint64_t> &tx) {
    proto::P2PDequantizationMeta pkt;
    pkt.tag = io.pkt_tag;
    pkt.meta = mine;
    auto bytes = proto::encode_with_id(pkt);
    if (!io.tx->send_frame(io.tag, io.seq, bytes.data(), bytes.size())) return 1;
    tx += meta_accounting_bytes(mine);
    return 0;
}

int recv_meta(const StepIo &io, proto::QuantMeta &theirs, std::atomic<uint64_t> &rx,
              const std::function<bool()> &aborted, const std::function<bool()> &failed) {
    while (true) {
        auto m = io.rx->recv_packet<proto::P2PDequantizationMeta>(io.tag, io.seq, 20ms);
        if (m) {
            theirs = m->meta;
            rx += meta_accounting_bytes(m->meta);
            return 0;
        }
        if (!io.rx->is_open() || (failed && failed()) || watch_failed()) return 1;
        if (aborted()) return 2;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// one striped step (host memory)
// ------------------------------------------------------------------------------------------------------------------
namespace {
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
    // false once `stop` reports (polled every 20 ms) before every sender finished
    bool wait_until_done(const std::function<bool()> &stop) {
        std::unique_lock l(m);
        while (!cv.wait_for(l, std::chrono::milliseconds(20), [&] { return n == 0; })) {
            l.unlock();
            const bool s = stop();
            l.lock();
            if (s && n != 0) return false;
        }
        return true;
    }
    // the senders of a failed step: a sender blocked in sendmsg on a peer that stopped reading is interrupted
    void wait_failed(const Conns &txs) {
        std::unique_lock l(m);
        while (!cv.wait_for(l, std::chrono::milliseconds(100), [&] { return n == 0; })) {
            l.unlock();
            net::interrupt_blocked_senders(txs, net::sink_drain_grace());
            l.lock();
        }
    }
};
} // namespace

int striped_step(const Conns &txs, const Conns &rxs, uint64_t tag, uint64_t seq, const Shape &shape,
                 const uint8_t *payload, size_t tx_bytes, const std::function<bool(size_t)> &tx_ready, uint8_t *sink,
                 size_t rx_bytes, size_t elem, size_t frame, const std::function<void(size_t, size_t)> &consume,
                 const std::function<bool()> &aborted, std::atomic<uint64_t> &tx_ctr, std::atomic<uint64_t> &rx_ctr,
                 const std::function<int()> &before_rx, size_t gran) {
    const StripePlan tp = plan_stripes(tx_bytes, txs.size(), shape);
    const StripePlan rp = plan_stripes(rx_bytes, rxs.size(), shape);
    auto rx_conn = [&](size_t k) { return rxs[stripe_conn(seq, tag, k, rxs.size(), shape)].get(); };
    auto tx_conn = [&](size_t k) { return txs[stripe_conn(seq, tag, k, txs.size(), shape)].get(); };
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
    // (a quantized step's metadata packet travels on its own tag, or - reference framing - was received before the
    // step: no sink of this step can swallow it)
    for (size_t k = 0; k < rp.off.size(); ++k) rx_conn(k)->post_sink(tag, seq, sink + rp.off[k], rp.len[k]);
    sinks_posted = true;
    // small steps leave before the peer's metadata is awaited (a step never waits one extra network latency)
    if (inline_send)
        for (size_t k = 0; k < tp.off.size(); ++k)
            if (tp.len[k] > 0) send_stripe(k);
    if (before_rx) {
        if (const int brc = before_rx()) {
            send_rc.store(brc);
            senders.wait_failed(txs);
            remove_sinks();
            return brc;
        }
    }

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
        if (!c->is_open() || send_rc.load() != 0 || watch_failed()) {
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
        // senders stuck in send() on a peer that stopped reading are interrupted (wait_failed)
        senders.wait_failed(txs);
        remove_sinks();
        return rc;
    }
    // every byte arrived; this step's own sends may still be blocked on a next peer that stopped reading: the wait
    // ends on the op's abort / watchdog verdict as well
    if (!senders.wait_until_done([&] { return watch_failed() || aborted(); })) {
        send_rc.store(1);
        senders.wait_failed(txs);
        remove_sinks();
        return aborted() ? 2 : 1;
    }
    remove_sinks();
    if (send_rc.load() != 0) return 1;
    rx_ctr += rx_bytes;
    return 0;
}

// Small all-reduces: the whole vector travels W-1 ring hops (all-gather) and every peer reduces the W vectors locally
// in ring-index order, instead of 2(W-1) hops of 1/W pieces. Such ops are bound by per-hop latency (socket wake-ups,
// and on the device ring per-step staging copies), not bytes, so this halves their critical path; every peer reduces
// the same vectors in the same order, so results stay bit-identical across peers. Taken when the vector is at most
// PCCL_SMALL_ALLREDUCE_BYTES (default 1 MiB; a peer with another threshold simply does not announce the capability
// for an op: kCollFlagSmallPath) and the all-gather sends at most 8x that (W-1 copies). Measured on MI355X, 8 peers,
// TCP device ring (profiles/r2/small_messages/): 64 KiB 1770 -> 547 us, 256 KiB 2822 -> 921 us, 1 MiB 2968 ->
// 2496 us, 4 MiB 4182 -> 10277 us (hence the cap).
bool use_small_path(size_t bytes, size_t ws) {
    const size_t lim = env_size("PCCL_SMALL_ALLREDUCE_BYTES", 1u << 20);
    return bytes <= lim && bytes * (ws - 1) <= 8 * lim;
}

int small_allgather_reduce(const Conns &txs, const Conns &rxs, uint64_t tag, uint64_t seq, const Shape &agreed,
                           const void *src, void *dst, size_t count, DType dt, ReduceOp op, size_t ws, size_t rank,
                           const std::function<bool()> &aborted, std::atomic<uint64_t> &tx_ctr,
                           std::atomic<uint64_t> &rx_ctr) {
    const size_t es = dtype_size(dt), bytes = count * es;
    const Shape shape = op_shape(agreed, bytes);
    Lease all(host_pool(), std::max<size_t>(ws * bytes, 64));
    if (!all.ok()) return 1;
    uint8_t *v = all.data();
    std::memcpy(v + rank * bytes, src, bytes);
    for (size_t step = 0; step + 1 < ws; ++step) {
        watch_step(step);
        const size_t send_idx = (rank + ws - step) % ws, recv_idx = (rank + ws - step - 1) % ws;
        const int rc = striped_step(txs, rxs, tag, seq, shape, v + send_idx * bytes, bytes, [](size_t) { return true; },
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

int run_lanes(const std::vector<size_t> &lo, const std::function<int(size_t, size_t, size_t)> &fn) {
    const size_t nl = lo.size() - 1;
    std::vector<int> rc(nl, 0);
    std::vector<std::thread> th;
    OpWatch *watch = current_watch();
    for (size_t k = 1; k < nl; ++k) th.emplace_back([&, k, watch] {
        name_thread("pccl-ring-lane");
        current_watch() = watch;
        rc[k] = fn(k, lo[k], lo[k + 1]);
    });
    rc[0] = fn(0, lo[0], lo[1]);
    for (auto &t : th) t.join();
    return *std::max_element(rc.begin(), rc.end());
}

// ------------------------------------------------------------------------------------------------------------------
// device pipeline helpers
// ------------------------------------------------------------------------------------------------------------------
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

void step_mark(bool reduce_scatter, size_t step) {
    static const char *rs[] = {"rs0", "rs1", "rs2", "rs3", "rs4", "rs5", "rs6", "rs7",
                               "rs8", "rs9", "rs10", "rs11", "rs12", "rs13", "rs14", "rs15"};
    static const char *ag[] = {"ag0", "ag1", "ag2", "ag3", "ag4", "ag5", "ag6", "ag7",
                               "ag8", "ag9", "ag10", "ag11", "ag12", "ag13", "ag14", "ag15"};
    if (step < 16) trace_mark(reduce_scatter ? rs[step] : ag[step]);
}

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

bool stream_wait_polling(DeviceBackend *be, DevStream s) {
    DevEvent e = event_pool().get();
    const bool ok = be->event_record(e, s) && event_wait_polling(be, e);
    event_pool().put(e);
    return ok;
}

void ReadyRanges::clear() {
    std::lock_guard l(m_);
    v_.clear();
}

void ReadyRanges::add(size_t a, size_t b, DevEvent e) {
    {
        std::lock_guard l(m_);
        v_.push_back({a, b, e});
    }
    cv_.notify_all();
}

bool ReadyRanges::wait(size_t begin, size_t end, DeviceBackend *be, const std::atomic<int> &cancel) {
    if (end <= begin) return true;
    std::vector<std::pair<size_t, size_t>> iv;
    std::vector<DevEvent> evs;
    while (true) {
        {
            std::unique_lock l(m_);
            iv.clear();
            evs.clear();
            for (const auto &r : v_)
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
            if (cur < end) {
                if (cancel.load(std::memory_order_relaxed) != 0) return false;
                cv_.wait_for(l, std::chrono::milliseconds(1)); // (cancel is polled, not signalled)
                continue;
            }
        }
        for (DevEvent e : evs)
            if (!event_wait_polling(be, e)) return false;
        return true;
    }
}

OpSenders::OpSenders(const Conns &txs, uint64_t tag, uint64_t seq, const Shape &shape, size_t frame, size_t nsteps,
                     size_t max_stripes, DeviceBackend *be, std::atomic<uint64_t> &tx_ctr)
    : txs_(txs), tag_(tag), seq_(seq), shape_(shape), frame_(frame), be_(be), tx_ctr_(tx_ctr), steps_(nsteps),
      done_(nsteps) {
    running_ = max_stripes;
    for (size_t k = 0; k < max_stripes; ++k) th_.emplace_back([this, k] {
        name_thread("pccl-stripe-tx");
        run(k);
        {
            std::lock_guard l(m_);
            --running_;
        }
        cv_.notify_all();
    });
}

OpSenders::~OpSenders() {
    cancel();
    // A stripe thread still blocked in sendmsg (its peer stopped reading: stopped, wedged, black-holed) would never
    // return: interrupt such connections after a grace period instead of waiting for TCP to give up.
    {
        std::unique_lock l(m_);
        while (!cv_.wait_for(l, std::chrono::milliseconds(100), [&] { return running_ == 0; })) {
            l.unlock();
            net::interrupt_blocked_senders(txs_, net::sink_drain_grace());
            l.lock();
        }
    }
    for (auto &t : th_) t.join();
}

void OpSenders::publish(size_t g, const Step &st) {
    const StripePlan tp = plan_stripes(st.bytes, txs_.size(), shape_);
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

bool OpSenders::published(size_t g) {
    std::lock_guard l(m_);
    return published_ > g;
}

bool OpSenders::sent(size_t g) {
    std::lock_guard l(m_);
    return published_ > g && done_[g] == 0;
}

bool OpSenders::should_stop() {
    return watch_failed() || (abort_ && abort_());
}

// The op thread waits here for its own sends; a stripe blocked on a peer that stopped reading never finishes its
// step, so the wait also ends on the op's abort / watchdog verdict (polled between short sleeps)
bool OpSenders::wait(size_t g) {
    std::unique_lock l(m_);
    for (size_t polls = 1; !(rc_.load() != 0 || (published_ > g && done_[g] == 0)); ++polls) {
        if (cv_.wait_for(l, std::chrono::milliseconds(5)) == std::cv_status::timeout && polls % 4 == 0) {
            l.unlock();
            const bool stop = should_stop();
            l.lock();
            if (stop) {
                rc_.store(1);
                cv_.notify_all();
            }
        }
    }
    return rc_.load() == 0;
}

// (a stripe with no bytes in the last step may still be sending an earlier one)
bool OpSenders::wait_all() {
    auto all_sent = [&] {
        if (published_ < steps_.size()) return false;
        for (size_t d : done_)
            if (d != 0) return false;
        return true;
    };
    std::unique_lock l(m_);
    for (size_t polls = 1; !(rc_.load() != 0 || all_sent()); ++polls) {
        if (cv_.wait_for(l, std::chrono::milliseconds(5)) == std::cv_status::timeout && polls % 4 == 0) {
            l.unlock();
            const bool stop = should_stop();
            l.lock();
            if (stop) {
                rc_.store(1);
                cv_.notify_all();
            }
        }
    }
    return rc_.load() == 0;
}

void OpSenders::cancel() {
    rc_.store(1);
    std::lock_guard l(m_);
    cv_.notify_all();
}

void OpSenders::run(size_t k) {
    for (size_t g = 0; g < steps_.size(); ++g) {
        Step st;
        {
            std::unique_lock l(m_);
            cv_.wait(l, [&] { return rc_.load() != 0 || published_ > g; });
            if (rc_.load() != 0) return;
            st = steps_[g];
        }
        const StripePlan tp = plan_stripes(st.bytes, txs_.size(), shape_);
        if (k >= tp.off.size() || tp.len[k] == 0) continue;
        net::MuxConn *c = txs_[stripe_conn(seq_, tag_, k, txs_.size(), shape_)].get();
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

void RingRx::post(size_t g, uint8_t *buf, size_t bytes) {
    Step &r = steps_[g];
    r.rp = plan_stripes(bytes, rxs_.size(), shape_);
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

void RingRx::unpost(size_t g) {
    Step &r = steps_[g];
    if (!r.posted) return;
    for (size_t k = 0; k < r.sinks.size(); ++k)
        if (r.sinks[k]) conn(k)->remove_sink(tag_, r.sinks[k]);
    r.sinks.clear();
    r.posted = false;
}

int RingRx::receive(size_t g, size_t unit, size_t gran, const std::function<void(size_t, size_t)> &consume,
                    const std::function<void()> &between, const std::function<bool()> &failed,
                    const std::function<bool()> &aborted) {
    Step &r = steps_[g];
    const size_t gb = std::max(unit, gran / unit * unit);
    size_t idle = 0, rr = 0;
    watch_step(g);
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
        if (!c->is_open() || (failed && failed()) || watch_failed()) return 1;
        if (++idle % 8 == 0 && aborted()) return 2;
    }
    return 0;
}

bool StepSlots::can_post(size_t g) const {
    if (g < n_) return true;
    const size_t b = g % n_, prev = g - n_;
    if (free_[b] && be_->event_query(free_[b]) == 0) return false;
    // an all-gather step's bytes are forwarded by the next step's sends (straight from the pinned slot)
    if (forwarded(prev) && !senders_.sent(prev + 1)) return false;
    return true;
}

void StepSlots::post(size_t g) {
    const size_t b = g % n_;
    free_[b] = nullptr;
    if (!is_rs(g)) ready_[b].clear();
    rx_.post(g, buf_[b], rx_bytes_(g));
}

bool StepSlots::ensure_posted(size_t g, const std::function<bool()> &failed, const std::function<bool()> &aborted) {
    for (size_t polls = 1; !rx_.posted(g); ++polls) {
        if (can_post(g)) {
            post(g);
            break;
        }
        // (the slot may wait on forwarded bytes whose sender is blocked on a peer that stopped reading: the wait
        // also ends on the op's watchdog verdict or the master's abort, polled every ~20 ms)
        if (failed() || watch_failed()) return false;
        if (aborted && polls % 1000 == 0 && aborted()) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    return true;
}

bool StepSlots::try_post(size_t g) {
    if (g >= nsteps_ || rx_.posted(g) || !can_post(g)) return false;
    post(g);
    return true;
}

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

} // namespace pccl::client::ring

// Host <-> device staging bytes of the device rings in this process: [0] host->device, [1] device->host (pcie_note).
// Returns how many counters exist (writes at most n).
extern "C" __attribute__((visibility("default"))) size_t pcclxPcieStats(uint64_t *out, size_t n) {
    uint64_t v[2];
    pccl::client::ring::pcie_read(v[0], v[1]);
    for (size_t i = 0; i < n && i < 2; ++i) out[i] = v[i];
    return 2;
}
