// Quantized device ring (protocol: ring_common.hpp, quant_lane_bounds / lane_tag). Each lane is one pipeline over its
// 2(W-1) steps on its own thread and stream, built like the plain device ring (OpSenders, RingRx, sinks posted a step
// early):
//   * reduce-scatter step g: the payload is the chunk step g-1 reduced, so its min / max (folded from the partials
//     that step's de-quantize-reduce kernels emitted, one host round trip for the metadata packet) exists only once
//     step g-1 has received everything; the quantize kernels then write it into pinned memory piece by piece (two
//     payload buffers: step g quantizes while step g-1's sends drain) and each piece leaves once its kernel is done;
//     received pieces go to HBM and de-quantize-reduce there;
//   * all-gather: the owner quantizes its finished chunk once and overwrites its own copy with D(Q(x)) (every peer
//     ends bit-identical); received quantized chunks are forwarded cut-through (the next step's metadata and sends
//     start when this step's metadata arrives; every piece leaves as it lands) and de-quantized.
// The per-step serialisation of the reduce-scatter is inherent to the protocol; lanes overlap it (one lane's fill and
// drain runs while another lane's data moves). Reference (host memory, one lane): ccoip/src/cpp/reduce.cpp:609-774.
// In the reference framing (a reference peer in the ring, or PCCL_WIRE=reference) the op runs the host ring's
// step-synchronous protocol on a pinned bounce buffer instead (device_quant_reference_framing).
#include <cstring>

#include "../common/log.hpp"
#include "../kernels/host_kernels.hpp"
#include "client.hpp"
#include "ring_common.hpp"

namespace pccl::client {

// quantized device ring: min / max of a step's payload folded from the previous step's fused partials (pcclxQuantStats)
static std::atomic<uint64_t> g_quant_minmax_folds{0}, g_quant_minmax_passes{0};

namespace {

using namespace ring;
using proto::QuantMeta;

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
    const Conns *txs, *rxs;
    size_t ws, rank;
    uint64_t tag, seq; // the lane's data tag (metadata on its meta tag)
    const Shape *shape;
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
    const Shape &agreed = *L.shape;
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
    // the lane's segments (global step G = segment * nps + ring step); staging is sized by the largest segment chunk
    const std::vector<size_t> seg = segment_bounds(L.count, es, ws, agreed);
    const size_t nseg = seg.size() - 1, nps = 2 * (ws - 1);
    std::vector<std::vector<std::pair<size_t, size_t>>> sbounds(nseg);
    size_t max_chunk = 0;
    for (size_t k = 0; k < nseg; ++k) {
        sbounds[k] = chunk_bounds(seg[k + 1] - seg[k], ws);
        for (auto &b : sbounds[k]) max_chunk = std::max(max_chunk, b.second - b.first);
    }
    // element range (lane-relative) a global step sends / receives
    auto tx_range = [&](size_t G) {
        const auto c = sbounds[G / nps][chunk_tx(G % nps, rank, ws)];
        return std::pair<size_t, size_t>{seg[G / nps] + c.first, seg[G / nps] + c.second};
    };
    auto rx_range = [&](size_t G) {
        const auto c = sbounds[G / nps][chunk_rx(G % nps, rank, ws)];
        return std::pair<size_t, size_t>{seg[G / nps] + c.first, seg[G / nps] + c.second};
    };
    auto ntx = [&](size_t G) { return tx_range(G).second - tx_range(G).first; };
    auto nrx = [&](size_t G) { return rx_range(G).second - rx_range(G).first; };
    const size_t qbytes = max_chunk * qs + 64;
    const Shape shape = op_shape(agreed, max_chunk * qs); // the lane's connection groups
    // receive slots (3, 6 and 8 slots for the small steps of 32 / 64 concurrent WAN ops measured the same:
    // profiles/r5/b10/)
    constexpr size_t kNb = StepSlots::kDefaultSlots;
    // The reduce-scatter's de-quantize-reduce kernels emit per-workgroup (min, max) partials of the values they store
    // into `mm_partials`: the chunk a step receives is the chunk the next step quantizes (and the last step's is the
    // all-gather's first payload), so its min / max is one fold of those partials instead of a second pass. A step
    // whose launches do not fit the partials buffer falls back to a separate min / max pass.
    constexpr int kMmSlots = 65536, kMmMinRoom = 64; // 1 MiB of partials: ~1 GiB bf16 chunks
    Lease txl[2], rxl[StepSlots::kMaxSlots], dvl[StepSlots::kMaxSlots], mml, mmp;
    uint8_t *txq[2], *rxbuf[StepSlots::kMaxSlots], *rxdev[StepSlots::kMaxSlots];
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

    ReadyRanges txready[2];
    const size_t nsteps = nseg * nps;
    auto is_rs = [&](size_t G) { return G % nps + 1 < ws; };

    OpSenders senders(*L.txs, L.tag, seq, shape, piece_el * qs, nsteps, op_stripes(shape, L.txs->size()), be, *L.tx);
    RingRx rx(*L.rxs, L.tag, seq, shape, nsteps);
    StepSlots slots(be, rx, senders, ws, nsteps, rxbuf, kNb, [&](size_t G) { return nrx(G) * qs; });
    const StepIo io = step_io(*L.txs, *L.rxs, L.tag, seq, shape);

    senders.set_abort(L.aborted);
    auto fail = [&](int code) {
        senders.cancel();
        L.op_failed->store(true);
        // a send wait that ended on the master's abort consumed its packet: report the abort
        return code == 1 && L.aborted() ? 2 : code;
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
        stp.bytes = ntx(g) * qs;
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
    for (size_t G = 0; G < nsteps; ++G) {
        const size_t g = G % nps, b = G % kNb;
        const bool rs = is_rs(G);
        if (!slots.ensure_posted(G, failed, L.aborted)) return fail(1);
        if (g < ws) { // own payload: reduce-scatter steps and the all-gather's first step
            const size_t slot = G % 2;
            const auto [c0, c1] = tx_range(G);
            uint8_t *src = L.dst + c0 * es;
            const size_t n = c1 - c0;
            if (G >= 2 && !senders.wait(G - 2)) return fail(1); // txq[slot] was step G-2's payload
            // min / max folded from the previous step's partials, except for a segment's first payload
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
                pcie_note(0, k * qs);
                txready[slot].add(off * qs, (off + k) * qs, e);
                if (G == 0) first_payload = e;
            }
            if (int m = send_meta(io, mine, *L.tx)) return fail(m);
            publish(G, txq[slot], &txready[slot]);
            step_sub_mark('q', G);
        } // else: forwarded chunk, published with its metadata when step G-1's metadata arrived
        fault_point("qring", seq, g, "meta");
        if (int m = recv_meta(io, theirs, *L.rx, L.aborted, failed)) return fail(m);
        const auto params = kernels::make_params(theirs, L.qtype);
        if (!rs && g + 1 < nps) { // cut-through all-gather: the next step forwards this chunk as it lands
            if (int m = send_meta(io, theirs, *L.tx)) return fail(m);
            publish(G + 1, slots.buf(G), &slots.ready(G));
        }
        uint8_t *region = L.dst + rx_range(G).first * es;
        uint8_t *sink = slots.buf(G);
        ReadyRanges *fwd = &slots.ready(G);
        DevEvent step_last = nullptr;
        bool first = true;
        const int rc = rx.receive(
            G, qs, piece_el * qs,
            [&](size_t a, size_t e) {
                const size_t n = (e - a) / qs;
                pcie_note(e - a, 0); // every received byte crosses once (a copy to HBM or a kernel reading it)
                if (rs) { // host -> HBM, then de-quantize-reduce HBM -> HBM (staged beats kernels reading pinned
                          // memory: 218.5 vs 223.7 ms, profiles/r4/b9/q_rs.jsonl; small steps of 64 concurrent WAN
                          // ops: the same either way, 1.98-1.99 vs 1.98-2.07 s, profiles/r5/b3/)
                    if (lane_copies) {
                        be->memcpy_async(rxdev[b] + a, sink + a, e - a, st);
                    } else {
                        be->memcpy_async(rxdev[b] + a, sink + a, e - a, pq.h2d);
                        be->stream_wait_event(st, record(pq.h2d));
                    }
                    dequant_consume(region + a / qs * es, rxdev[b] + a, n, params);
                } else if (lane_copies) { // forwardable at once (from pinned memory); host -> HBM on the lane's stream,
                                          // de-quantized from HBM
                    fwd->add(a, e, nullptr);
                    be->memcpy_async(rxdev[b] + a, sink + a, e - a, st);
                    be->dequant_reduce(region + a / qs * es, rxdev[b] + a, n, L.dtype, L.qtype, ReduceOp::Set, params,
                                       st);
                } else { // forwardable at once; de-quantized straight from pinned memory
                    fwd->add(a, e, nullptr);
                    be->dequant_reduce(region + a / qs * es, sink + a, n, L.dtype, L.qtype, ReduceOp::Set, params, st);
                }
                step_last = record(st);
                if (first) {
                    first = false;
                    step_sub_mark('f', G);
                    fault_point("qring", seq, g, "rx");
                }
            },
            [&] {
                maybe_open_gate();
                slots.try_post(G + 1);
            },
            failed, L.aborted);
        slots.free_after(G, step_last);
        if (rc) return fail(rc);
        *L.rx += nrx(G) * qs;
        rx.unpost(G);
        step_mark(rs, rs ? g : g - (ws - 1));
        fault_point("qring", seq, g, "end");
    }
    if (!senders.wait_all()) return fail(1);
    return 0;
}

} // namespace

// Reference framing (kCollFlagExtWire not agreed): the quantized op's steps are synchronous with the peer's metadata
// (reference reduce.cpp:154-192), so the pipelined lanes above do not apply. The buffer goes to pinned host memory,
// runs the host ring's quantized protocol there (the host quantize / de-quantize kernels are the device kernels'
// bit-exact twins, tests/test_gpu_kernels.py) and the result comes back in one copy. `dst` is written only on success.
std::pair<bool, bool> Client::device_quant_reference_framing(OpState &op, const RingView &rv, uint64_t seq,
                                                             int device) {
    DeviceBackend *be = device_backend();
    const ReduceRequest &q = op.req;
    const size_t es = dtype_size(q.dtype), bytes = q.count * es;
    be->set_device(device);
    StreamLease stream(device);
    DevStream st = stream.get();
    Lease hbuf(pinned_pool(), std::max<size_t>(bytes, 64));
    if (!st || !hbuf.ok()) return {false, false};
    if (!be->memcpy_async(hbuf.data(), q.src, bytes, st) || !be->stream_sync(st)) return {false, false};
    pcie_note(0, bytes);
    Lease backup; // in place: the input, restored if the master aborts the op after this peer's part (settle)
    const bool keep_backup = q.src == q.dst && !q.scratch;
    if (keep_backup) {
        backup = Lease(pinned_pool(), std::max<size_t>(bytes, 64));
        if (!backup.ok()) return {false, false};
        std::memcpy(backup.data(), hbuf.data(), bytes);
    }
    OpAbort aborted([this, t = q.tag] { return abort_received(t); });
    const int rc = host_allreduce(rv.tx, rv.rx, rv.ring.size(), rv.rank, q.tag, seq, op.shape, hbuf.data(), q.count,
                                  q.dtype, q.qtype, q.qalgo, q.op, [&] { return aborted(); }, op.tx, op.rx);
    if (rc) return {rc == 2, rc == 2};
    if (!be->memcpy_async(q.dst, hbuf.data(), bytes, st) || !be->stream_sync(st)) return {false, false};
    pcie_note(bytes, 0);
    if (keep_backup) settle_device_backup(op.settle, be, device, std::move(backup), q.dst, bytes);
    return {true, false};
}

std::pair<bool, bool> Client::ring_reduce_device_quant(OpState &op, const RingView &rv, uint64_t seq, int device) {
    if (op.shape.reference) return device_quant_reference_framing(op, rv, seq, device);
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

    const std::vector<size_t> lo = quant_lane_bounds(q.count, ws, qs, op.shape);
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
        QLane L{&rv.tx, &rv.rx, ws, rv.rank, lane_tag(q.tag, k, nl), seq, &op.shape, be, lane_streams[k]->get(), ready,
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
