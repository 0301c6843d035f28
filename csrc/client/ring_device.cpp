// Device ring: buffers in HBM. Ring-step payloads are staged to pinned host memory (step 0 by copy-engine copies,
// later steps by the fused reduce kernel that writes the next payload while it reduces), sent over the striped
// connections as soon as each piece is ready, and received bytes are copied into HBM staging and reduced HBM -> HBM
// (reference ccoip/src/cpp/reduce.cpp:528-784 on host memory; SURVEY §2.1 N8 "HIP device pipeline").
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
#include <cstring>

#include "../common/log.hpp"
#include "client.hpp"
#include "ring_common.hpp"

namespace pccl::client {

namespace {

using namespace ring;

// inputs of one device-ring op
struct DevRing {
    const Conns &txs, &rxs; // the ring's connections to next / from prev
    size_t ws, rank;
    uint64_t tag, seq;
    const Shape &shape;
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

// The device ring as one pipeline over all 2(W-1) steps of every segment (ring_common.hpp segment_bounds): step G+1's
// payload is produced (reduced into pinned memory, or - a segment's first step - staged from the input) and sent
// while step G still receives, and step G+1's sinks are posted as soon as their staging buffer is free. Staging is
// sized by the largest segment chunk, not by the tensor. Returns 0 ok, 1 io failure, 2 abort; on return no GPU work
// or socket write of the op touches any of its buffers any more (the caller may restore the input).
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
    // segments (global step G = segment * nps + ring step) and their chunks, as absolute element ranges
    const std::vector<size_t> seg = segment_bounds(R.count, es, ws, R.shape);
    const size_t nseg = seg.size() - 1, nps = 2 * (ws - 1), nsteps = nseg * nps;
    std::vector<std::vector<std::pair<size_t, size_t>>> sbounds(nseg);
    size_t max_chunk = 0;
    for (size_t k = 0; k < nseg; ++k) {
        sbounds[k] = chunk_bounds(seg[k + 1] - seg[k], ws);
        for (auto &b : sbounds[k]) max_chunk = std::max(max_chunk, b.second - b.first);
    }
    auto lstep = [&](size_t G) { return G % nps; };
    auto is_rs = [&](size_t G) { return lstep(G) + 1 < ws; };
    auto tx_range = [&](size_t G) {
        const auto c = sbounds[G / nps][chunk_tx(lstep(G), rank, ws)];
        return std::pair<size_t, size_t>{seg[G / nps] + c.first, seg[G / nps] + c.second};
    };
    auto rx_range = [&](size_t G) {
        const auto c = sbounds[G / nps][chunk_rx(lstep(G), rank, ws)];
        return std::pair<size_t, size_t>{seg[G / nps] + c.first, seg[G / nps] + c.second};
    };
    auto rx_bytes = [&](size_t G) {
        const auto [a, b] = rx_range(G);
        return (b - a) * es;
    };
    const size_t stage_bytes = max_chunk * es + 64;
    // Staging rings of kNb buffers: step G receives into rxbuf[G % kNb] (HBM twin rxdev[G % kNb] for the reduce) and
    // its reduce writes the next payload into txbuf[(G + 1) % kNb]: a buffer is refilled only after the step two back
    // finished with it (StepSlots).
    constexpr size_t kNb = StepSlots::kDefaultSlots;
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
    size_t txshift[kNb] = {0, 0, 0}; // payload of txbuf[i] starts at this offset (16-byte phase of its HBM source)
    auto region_of = [&](size_t G) { return R.dst + rx_range(G).first * es; };

    // every chunk of the op is sent by this peer at some step: the largest one sets the op's stripe count
    const Shape shape = op_shape(R.shape, max_chunk * es);
    // declared after the buffers and ready lists it reads: destroyed (cancelled + joined) before them
    OpSenders senders(R.txs, R.tag, seq, shape, piece, nsteps, op_stripes(shape, R.txs.size()), be, R.tx);
    RingRx rx(R.rxs, R.tag, seq, shape, nsteps); // after the buffers its sinks point into
    StepSlots slots(be, rx, senders, ws, nsteps, rxbuf, kNb, rx_bytes);
    senders.set_abort(R.aborted);
    auto fail = [&](int code) {
        senders.cancel();
        // a send wait that ended on the master's abort consumed its packet: report the abort (run_op must not wait
        // for a second one)
        return code == 1 && R.aborted() ? 2 : code;
    };
    // a segment's first payload: its own input chunk -> pinned, in pieces (from src: ready at call time, never
    // written by the op). Its slot was last read by the sends of step G - kNb.
    std::vector<bool> staged0(nsteps, false);
    auto stage_first = [&](size_t G) -> bool {
        if (staged0[G]) return true;
        if (G >= kNb && !senders.wait(G - kNb)) return false;
        const size_t b = G % kNb;
        const auto [ts, te] = tx_range(G);
        txready[b].clear();
        txshift[b] = 0;
        for (size_t off = 0; off < (te - ts) * es; off += piece) {
            const size_t n = std::min(piece, (te - ts) * es - off);
            be->memcpy_async(txbuf[b] + off, R.src + ts * es + off, n, pq.d2h);
            pcie_note(0, n);
            last_d2h = record(pq.d2h);
            txready[b].add(off, off + n, last_d2h);
        }
        staged0[G] = true;
        return true;
    };
    auto publish = [&](size_t G) {
        if (senders.published(G)) return true;
        if (lstep(G) == 0 && !stage_first(G)) return false;
        const auto [ts, te] = tx_range(G);
        const bool staged = lstep(G) < ws; // reduce-scatter steps and all-gather step 0 send txbuf payloads
        OpSenders::Step stp;
        stp.payload = staged ? txbuf[G % kNb] + txshift[G % kNb] : slots.buf(G - 1);
        stp.bytes = (te - ts) * es;
        stp.ready = staged ? &txready[G % kNb] : &slots.ready(G - 1);
        senders.publish(G, stp);
        return true;
    };

    for (size_t G = 0; G < nsteps; ++G) {
        const size_t g = lstep(G), b = G % kNb, nb = (G + 1) % kNb;
        const bool rs = is_rs(G);
        // 1. step G's sinks (normally posted during step G-1)
        if (!slots.ensure_posted(G, [&] { return senders.failed(); }, R.aborted)) return fail(1);
        // 2. this step's reduce writes txbuf[nb], last read by step G-2's sends
        uint8_t *region = region_of(G);
        const size_t shift = reinterpret_cast<uintptr_t>(region) % 16;
        if (rs) {
            if (G >= 2 && !senders.wait(G - 2)) return fail(1);
            txready[nb].clear();
            txshift[nb] = shift;
        }
        // 3. this step's and (send-ahead) the next step's payloads may leave as they become ready; a segment's first
        //    payload is staged from the input here
        if (!publish(G)) return fail(1);
        if (G + 1 < nsteps && !publish(G + 1)) return fail(1); // its payload fills while this step runs
        fault_point("ring", seq, g, "publish");
        // 4. receive + consume step G
        DevEvent step_last = nullptr;
        std::function<void(size_t, size_t)> consume;
        if (rs) {
            // HBM staging and the next payload share the 16-byte phase of `region`: the fused kernel stays vectorised
            uint8_t *stage = rxdev[b] + shift, *out = txbuf[nb] + shift, *sink = slots.buf(G);
            consume = [&, stage, out, sink, region, nb](size_t a, size_t e) {
                be->memcpy_async(stage + a, sink + a, e - a, pq.h2d);
                DevEvent ce = record(pq.h2d);
                be->stream_wait_event(st, ce);
                be->reduce_copy(region + a, stage + a, out + a, (e - a) / es, R.dtype, R.rop, st);
                pcie_note(e - a, e - a); // received bytes in, the next payload out
                step_last = record(st);
                txready[nb].add(a, e, step_last);
            };
        } else {
            uint8_t *sink = slots.buf(G);
            ReadyRanges *fwd = &slots.ready(G);
            consume = [&, sink, region, fwd](size_t a, size_t e) {
                be->memcpy_async(region + a, sink + a, e - a, st);
                pcie_note(e - a, 0);
                step_last = record(st);
                fwd->add(a, e, nullptr); // in host memory: forwardable at once
            };
        }
        bool first = true;
        const int rc = rx.receive(
            G, es, piece,
            [&](size_t a, size_t e) {
                consume(a, e);
                if (first) {
                    first = false;
                    fault_point("ring", seq, g, "rx"); // kernels / copies of this step in flight
                }
            },
            [&] { // post the next step's sinks as soon as its buffer is free (its sender may already be streaming)
                if (slots.try_post(G + 1)) fault_point("ring", seq, g, "ahead");
            },
            [&] { return senders.failed(); }, R.aborted);
        slots.free_after(G, step_last);
        if (rc) return fail(rc);
        R.rx += rx_bytes(G);
        rx.unpost(G);
        step_mark(rs, rs ? g : g - (ws - 1));
        if (g + 2 == ws) trace_mark("reduce_scatter");
        fault_point("ring", seq, g, "end");
    }
    if (!senders.wait_all()) return fail(1);
    return 0; // complete once its last received bytes landed in HBM (the Drain waits for them)
}

// The device ring in the reference framing (a participant without the pccl-amd extension, Shape::reference): every
// ring step carries its whole chunk on one connection (reference reduce.cpp:149-151, 528-784), so the op cannot be
// split into segments as device_ring_pipeline does, and that pipeline's per-step staging (3 slots x pinned TX, pinned
// RX and HBM, each a whole chunk) would grow with the tensor: 2 peers x 16 GiB bf16 leased 48 GiB of pinned memory.
// Here a step is moved in pieces of PCCL_REF_PIECE_BYTES (64 MiB, the reference's frame size) through fixed rings of
// pinned and HBM slots: received pieces land in posted piece sinks (the tag's byte stream fills them in order, a
// sender's frames may straddle them), are copied to HBM and reduced into the output in place (reduce-scatter) or
// copied there (all-gather); a sender thread stages each piece of the next step's payload from HBM into pinned memory
// (device->host copy once the piece it depends on was reduced) and sends it. The wire is byte-identical to the
// unsegmented pipeline's; staging is 3 + 3 pinned and 3 HBM slots of one piece, whatever the tensor. Costs one extra
// device->host copy per reduce-scatter byte (the pipeline streams the next payload out of the reduce kernel).
int device_ring_reference_pieces(DevRing &R) {
    DeviceBackend *be = R.be;
    const PcieQueues pq = R.pq;
    DevStream st = R.st;
    const size_t ws = R.ws, rank = R.rank, es = R.es, nsteps = 2 * (ws - 1);
    const uint64_t seq = R.seq;
    const size_t P = std::max<size_t>(1 << 20, env_size("PCCL_REF_PIECE_BYTES", 64u << 20)) / es * es;
    const auto bounds = chunk_bounds(R.count, ws);
    net::MuxConn *txc = R.txs[stripe_conn(seq, R.tag, 0, R.txs.size(), R.shape)].get();
    net::MuxConn *rxc = R.rxs[stripe_conn(seq, R.tag, 0, R.rxs.size(), R.shape)].get();

    std::mutex ev_m;
    std::condition_variable ev_cv;
    std::vector<DevEvent> owned;
    auto record = [&](DevStream s) {
        DevEvent e = event_pool().get();
        be->event_record(e, s);
        std::lock_guard l(ev_m);
        owned.push_back(e);
        return e;
    };
    // one unit per (step, piece) in wire order; done[u]: the event after the unit's consume (its bytes in HBM)
    struct Unit {
        size_t g, off, n; // step, byte offset in the step's chunk, bytes
    };
    std::vector<Unit> units;
    std::vector<std::vector<size_t>> unit_of(nsteps); // unit index of (step, piece)
    for (size_t g = 0; g < nsteps; ++g) {
        const auto [rs, re] = bounds[chunk_rx(g, rank, ws)];
        for (size_t off = 0; off < (re - rs) * es; off += P) {
            unit_of[g].push_back(units.size());
            units.push_back(Unit{g, off, std::min(P, (re - rs) * es - off)});
        }
    }
    std::vector<DevEvent> done(units.size(), nullptr);
    constexpr size_t K = 3;
    Lease rxl[K], stl[K], txl[2];
    for (size_t i = 0; i < K; ++i) {
        rxl[i] = Lease(pinned_pool(), P);
        stl[i] = Lease(device_pool(), P, R.device);
        if (!rxl[i].ok() || !stl[i].ok()) return 1;
    }
    for (auto &t : txl) {
        t = Lease(pinned_pool(), P);
        if (!t.ok()) return 1;
    }
    const DevEvent input_ready = record(st); // dst holds the input once the op stream gets here
    std::atomic<int> cancel{0}, send_rc{0};
    std::atomic<bool> sender_done{false};

    // ---- sender: step g's payload is chunk_tx(g) of dst, which step g-1 received (g = 0: the own input chunk)
    std::thread sender([&] {
        name_thread("pccl-ref-tx");
        struct Done {
            std::atomic<bool> &f;
            ~Done() { f.store(true); }
        } mark{sender_done};
        struct Staged {
            size_t slot = 0, n = 0;
            DevEvent copied = nullptr;
        };
        std::vector<std::pair<size_t, size_t>> plan; // (step, byte offset) of every piece sent, in order
        for (size_t g = 0; g < nsteps; ++g) {
            const auto [ts, te] = bounds[chunk_tx(g, rank, ws)];
            for (size_t off = 0; off < (te - ts) * es; off += P) plan.emplace_back(g, off);
        }
        auto stage = [&](size_t k) -> Staged {
            const auto [g, off] = plan[k];
            const auto [ts, te] = bounds[chunk_tx(g, rank, ws)];
            DevEvent dep = input_ready;
            if (g > 0) { // the piece of step g-1 that received these bytes (same chunk, same offsets)
                const size_t u = unit_of[g - 1][off / P];
                std::unique_lock l(ev_m);
                ev_cv.wait(l, [&] { return done[u] != nullptr || cancel.load() != 0; });
                if (cancel.load() != 0) return {};
                dep = done[u];
            }
            if (!event_wait_polling(be, dep)) return {};
            Staged s{k % 2, std::min(P, (te - ts) * es - off), nullptr};
            be->memcpy_async(txl[s.slot].data(), R.dst + ts * es + off, s.n, pq.d2h);
            pcie_note(0, s.n);
            s.copied = record(pq.d2h);
            return s;
        };
        Staged cur = plan.empty() ? Staged{} : stage(0);
        for (size_t k = 0; k < plan.size(); ++k) {
            if (!cur.copied) {
                send_rc.store(1);
                return;
            }
            const Staged next = k + 1 < plan.size() ? stage(k + 1) : Staged{}; // its copy overlaps this send
            if (!event_wait_polling(be, cur.copied) || cancel.load() != 0 ||
                !txc->send_frame(R.tag, seq, txl[cur.slot].data(), cur.n)) {
                send_rc.store(1);
                return;
            }
            R.tx += cur.n;
            cur = next;
        }
    });
    auto stop_sender = [&] {
        cancel.store(1);
        {
            std::lock_guard l(ev_m);
        }
        ev_cv.notify_all();
        // a send blocked on a peer that stopped reading is interrupted after a grace period, not waited for
        const auto t0 = std::chrono::steady_clock::now();
        while (!sender_done.load()) {
            if (std::chrono::steady_clock::now() - t0 > net::sink_drain_grace())
                net::interrupt_blocked_senders(R.txs, std::chrono::nanoseconds(1));
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        sender.join();
    };

    // ---- receiver (this thread): unit u lands in rx slot u % K, whose previous unit's consume must be complete
    std::vector<net::MuxConn::SinkRef> sinks(units.size());
    size_t posted = 0;
    // sinks of the next units (at most K ahead of the one consumed, u): unit v reuses slot v % K once unit v - K's
    // copy / reduce out of it completed
    auto post_ready = [&](size_t u) {
        while (posted < units.size() && posted < u + K) {
            if (posted >= K && be->event_query(done[posted - K]) == 0) return;
            sinks[posted] = rxc->post_sink(R.tag, seq, rxl[posted % K].data(), units[posted].n);
            ++posted;
        }
    };
    int rc = 0;
    for (size_t u = 0; u < units.size() && rc == 0; ++u) {
        const Unit &un = units[u];
        watch_step(un.g);
        size_t idle = 0;
        while (true) {
            post_ready(u);
            if (u < posted && net::MuxConn::sink_progress(sinks[u]) >= un.n) break;
            if (u < posted) rxc->wait_sink(sinks[u], un.n, std::chrono::milliseconds(5));
            else std::this_thread::sleep_for(std::chrono::microseconds(50));
            if (!rxc->is_open() || send_rc.load() != 0 || watch_failed()) {
                rc = 1;
                break;
            }
            if (++idle % 8 == 0 && R.aborted()) {
                rc = 2;
                break;
            }
        }
        if (rc) break;
        const size_t s = u % K;
        const auto [rs0, re0] = bounds[chunk_rx(un.g, rank, ws)];
        uint8_t *region = R.dst + rs0 * es + un.off;
        DevEvent e;
        if (un.g + 1 < ws) { // reduce-scatter: pinned -> HBM stage (copy engine), reduce into the output in place
            be->memcpy_async(stl[s].data(), rxl[s].data(), un.n, pq.h2d);
            be->stream_wait_event(st, record(pq.h2d));
            be->reduce(region, stl[s].data(), un.n / es, R.dtype, R.rop, st);
            e = record(st);
        } else { // all-gather: the owner's reduced bytes straight into the output
            be->memcpy_async(region, rxl[s].data(), un.n, st);
            e = record(st);
        }
        pcie_note(un.n, 0);
        rxc->remove_sink(R.tag, sinks[u]);
        sinks[u] = nullptr;
        {
            std::lock_guard l(ev_m);
            done[u] = e;
        }
        ev_cv.notify_all();
        R.rx += un.n;
        if (u + 1 == units.size() || units[u + 1].g != un.g) {
            const size_t g = un.g;
            step_mark(g + 1 < ws, g + 1 < ws ? g : g - (ws - 1));
            if (g + 2 == ws) trace_mark("reduce_scatter");
        }
    }
    // every piece arrived; the last step's sends may still be in flight (ended by the op's abort / watchdog too)
    for (size_t polls = 1; rc == 0 && !sender_done.load(); ++polls) {
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        if (polls % 25 == 0 && (watch_failed() || R.aborted())) rc = R.aborted() ? 2 : 1;
    }
    if (rc != 0) stop_sender();
    else sender.join();
    if (rc == 0 && send_rc.load() != 0) rc = R.aborted() ? 2 : 1;
    for (auto &sk : sinks)
        if (sk) rxc->remove_sink(R.tag, sk);
    // nothing of the op may still read or write its buffers when they go back to the pools
    stream_wait_polling(be, pq.h2d);
    stream_wait_polling(be, pq.d2h);
    stream_wait_polling(be, st);
    for (auto e : owned) event_pool().put(e);
    return rc;
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
    // profiles/r3/ring_ab/): fewer copies, kernels, events and socket wake-ups per byte. (A sender choice: frames of
    // any size up to 1 GiB are accepted, also by the reference.)
    const size_t piece = std::max<size_t>(1 << 20, env_size("PCCL_DEVICE_PIECE_BYTES", 32u << 20)) / es * es;

    be->set_device(device);
    StreamLease stream(device);
    DevStream st = stream.get();
    if (!st) return {false, false};
    if (op.small_path) { // latency-bound (agreed by every peer): one D2H, host all-gather + reduce, one H2D
        Lease hin(pinned_pool(), std::max<size_t>(bytes, 64)), hout(pinned_pool(), std::max<size_t>(bytes, 64));
        if (!hin.ok() || !hout.ok()) return {false, false};
        if (!be->memcpy_async(hin.data(), q.src, bytes, st) || !be->stream_sync(st)) return {false, false};
        pcie_note(0, bytes);
        const int rc = small_allgather_reduce(rv.tx, rv.rx, q.tag, seq, op.shape, hin.data(), hout.data(), q.count,
                                              q.dtype, q.op, ws, rank, [&] { return abort_received(q.tag); }, op.tx,
                                              op.rx);
        if (rc) return {false, rc == 2};
        if (!be->memcpy_async(dst, hout.data(), bytes, st) || !be->stream_sync(st)) return {false, false};
        pcie_note(bytes, 0);
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
    DevRing R{rv.tx, rv.rx, ws, rank, q.tag, seq, op.shape, be, pq, st, static_cast<const uint8_t *>(q.src), dst,
              q.count, es, piece, q.dtype, q.op, device, [&] { return aborted(); }, op.tx, op.rx};
    // reference framing cannot be segmented: ring chunks above the segment bound move in pieces instead
    const size_t ref_bound = std::max<size_t>(1, env_size("PCCL_SEGMENT_CHUNK_MIB", 128)) << 20;
    const int rc = op.shape.reference && (q.count + ws - 1) / ws * es > ref_bound ? device_ring_reference_pieces(R)
                                                                                 : device_ring_pipeline(R);
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

} // namespace pccl::client
