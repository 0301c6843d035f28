// Host ring: buffers in host memory; frames are received straight into the destination (all-gather) or a pooled
// receive buffer (reduce-scatter); arrived elements are reduced while the rest of the chunk is still in flight
// (reference ccoip/src/cpp/reduce.cpp:116-438,528-784).
#include <cstring>

#include "../common/log.hpp"
#include "../kernels/host_kernels.hpp"
#include "client.hpp"
#include "ring_common.hpp"

namespace pccl::client {

using namespace proto;

namespace ring {

int host_ring(const HostRingArgs &A) {
    const size_t ws = A.ws, rank = A.rank;
    const size_t es = dtype_size(A.dtype);
    const size_t qs = A.quant ? dtype_size(A.qtype) : es;
    const size_t chunk = net::multiplex_chunk_size();
    const StepIo io = step_io(A.txs, A.rxs, A.tag, A.seq, A.shape);
    uint8_t *const dst = A.dst;

    const auto bounds = chunk_bounds(A.count, ws);
    size_t max_chunk = 0;
    for (auto &b : bounds) max_chunk = std::max(max_chunk, b.second - b.first);
    Lease rbuf(host_pool(), max_chunk * qs + 64);
    Lease qbuf;
    if (A.quant) qbuf = Lease(host_pool(), max_chunk * qs + 64);
    if (!rbuf.ok() || (A.quant && !qbuf.ok())) return 1;

    // One full-duplex (striped) step g (global: reduce-scatter 0 .. ws-2, then all-gather): sends `payload`,
    // receives `rx_bytes` into `sink`, calling `consume(from, to)` for newly complete received elements. Returns 0 ok,
    // 1 io failure, 2 abort. Fault points (tests): hring:<seq>:<g>:rx after the first consume, :end after the step.
    auto run_step = [&](size_t g, const uint8_t *payload, size_t tx_bytes, uint8_t *sink, size_t rx_bytes,
                        const std::function<void(size_t, size_t)> &consume,
                        const std::function<int()> &before_rx = {}) -> int {
        bool first = true;
        watch_step(g);
        const int rc = striped_step(A.txs, A.rxs, A.tag, A.seq, A.shape, payload, tx_bytes, [](size_t) { return true; },
                                    sink, rx_bytes, qs, chunk, [&](size_t a, size_t b) {
                                        consume(a, b);
                                        if (first) {
                                            first = false;
                                            fault_point("hring", A.seq, g, "rx");
                                        }
                                    }, A.aborted, A.tx, A.rx, before_rx);
        if (rc == 0) fault_point("hring", A.seq, g, "end");
        return rc;
    };
    // A quantized step exchanges the dequantization metadata: pccl-amd framing sends ours on the metadata tag and
    // receives the peer's once the step's sinks are posted (the packet cannot land in them); the reference framing
    // sends ours and waits for the peer's on the data tag before any sink of the step exists (reference
    // reduce.cpp:154-192: a sink would swallow the packet). Returns the before_rx hook for striped_step, or an error.
    auto exchange_meta = [&](const QuantMeta &mine, QuantMeta &theirs, std::function<int()> &before_rx) -> int {
        if (int rc = send_meta(io, mine, A.tx)) return rc;
        if (A.shape.reference) return recv_meta(io, theirs, A.rx, A.aborted);
        before_rx = [&, pt = &theirs] { return recv_meta(io, *pt, A.rx, A.aborted); };
        return 0;
    };

    // ---- reduce-scatter
    for (size_t step = 0; step + 1 < ws; ++step) {
        const size_t tx_idx = (rank + ws - step) % ws, rx_idx = (rank + ws - step - 1) % ws;
        const auto [ts, te] = bounds[tx_idx];
        const auto [rs, re] = bounds[rx_idx];
        const uint8_t *payload = dst + ts * es;
        QuantMeta mine, theirs;
        std::function<int()> before_rx;
        if (A.quant) {
            if (te > ts) mine = kernels::host_quantize(qbuf.data(), dst + ts * es, te - ts, A.dtype, A.qtype, A.qalgo);
            else mine = kernels::make_meta(A.qalgo, A.dtype, A.qtype, 0, 0);
            payload = qbuf.data();
            if (int rc = exchange_meta(mine, theirs, before_rx)) return rc;
        }
        uint8_t *rx_region = dst + rs * es;
        const int rc = run_step(step, payload, (te - ts) * qs, rbuf.data(), (re - rs) * qs, [&](size_t a, size_t b) {
            if (A.quant)
                kernels::host_dequant_reduce(rx_region + a * es, rbuf.data() + a * qs, b - a, A.dtype, A.qtype, A.op,
                                             theirs);
            else
                kernels::host_reduce(rx_region + a * es, rbuf.data() + a * es, b - a, A.dtype, A.op);
        }, before_rx);
        if (rc) return rc;
    }

    trace_mark("reduce_scatter");
    // ---- all-gather
    Lease ag[2];
    if (A.quant) {
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
        if (A.quant) {
            QuantMeta mine, theirs;
            const uint8_t *payload;
            if (step == 0) {
                if (te > ts) {
                    mine = kernels::host_quantize(qbuf.data(), dst + ts * es, te - ts, A.dtype, A.qtype, A.qalgo);
                    // parity: our own copy becomes exactly what the other peers will de-quantize
                    kernels::host_dequant_reduce(dst + ts * es, qbuf.data(), te - ts, A.dtype, A.qtype, ReduceOp::Set,
                                                 mine);
                } else {
                    mine = kernels::make_meta(A.qalgo, A.dtype, A.qtype, 0, 0);
                }
                payload = qbuf.data();
            } else {
                mine = prev_meta;
                payload = ag[(step - 1) % 2].data();
            }
            std::function<int()> before_rx;
            if (int m = exchange_meta(mine, theirs, before_rx)) return m;
            uint8_t *sink = ag[step % 2].data();
            rc = run_step(ws - 1 + step, payload, (te - ts) * qs, sink, (re - rs) * qs, [&](size_t a, size_t b) {
                kernels::host_dequant_reduce(rx_region + a * es, sink + a * qs, b - a, A.dtype, A.qtype, ReduceOp::Set,
                                             theirs);
            }, before_rx);
            prev_meta = theirs;
        } else {
            rc = run_step(ws - 1 + step, dst + ts * es, (te - ts) * es, rx_region, (re - rs) * es, [](size_t, size_t) {});
        }
        if (rc) return rc;
        cur = inc;
    }
    return 0;
}

int host_allreduce(const Conns &txs, const Conns &rxs, size_t ws, size_t rank, uint64_t tag, uint64_t seq,
                   const Shape &shape, uint8_t *dst, size_t count, DType dtype, DType qtype, QuantAlgo qalgo,
                   ReduceOp op, const std::function<bool()> &aborted, std::atomic<uint64_t> &tx,
                   std::atomic<uint64_t> &rx) {
    const size_t es = dtype_size(dtype);
    const bool quant = qalgo != QuantAlgo::None && qtype != dtype;
    const std::vector<size_t> lo = quant ? quant_lane_bounds(count, ws, dtype_size(qtype), shape)
                                         : std::vector<size_t>{0, count};
    const int rc = run_lanes(lo, [&](size_t k, size_t a, size_t b) {
        // the lane's segments one after the other (the device rings pipeline them; the wire is the same)
        const std::vector<size_t> seg = segment_bounds(b - a, es, ws, shape);
        size_t max_chunk = 0; // elements of the lane's largest ring chunk: its stripe count (as the device rings)
        for (size_t s = 0; s + 1 < seg.size(); ++s) max_chunk = std::max(max_chunk, (seg[s + 1] - seg[s] + ws - 1) / ws);
        const Shape lane_shape = op_shape(shape, max_chunk * (quant ? dtype_size(qtype) : es));
        for (size_t s = 0; s + 1 < seg.size(); ++s) {
            HostRingArgs A{txs, rxs, ws, rank, lane_tag(tag, k, lo.size() - 1), seq, lane_shape,
                           dst + (a + seg[s]) * es, seg[s + 1] - seg[s], dtype, qtype, qalgo, op, quant, aborted, tx,
                           rx};
            if (const int r = host_ring(A)) return r;
        }
        return 0;
    });
    if (rc == 0 && op == ReduceOp::Avg) kernels::host_finalize_avg(dst, count, dtype, ws);
    return rc;
}

} // namespace ring

std::pair<bool, bool> Client::ring_reduce_host(OpState &op, const RingView &rv, uint64_t seq) {
    const ReduceRequest &q = op.req;
    const size_t ws = rv.ring.size(), rank = rv.rank;
    const size_t es = dtype_size(q.dtype);
    const bool quant = q.qalgo != QuantAlgo::None && q.qtype != q.dtype;
    auto *dst = static_cast<uint8_t *>(q.dst);
    const size_t bytes = q.count * es;
    ring::OpAbort aborted([this, t = q.tag] { return abort_received(t); });
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
        const int rc = ring::small_allgather_reduce(rv.tx, rv.rx, q.tag, seq, op.shape, q.src, dst, q.count, q.dtype,
                                                    q.op, ws, rank, abort_fn, op.tx, op.rx);
        trace_mark("allgather_reduce");
        if (rc == 0) keep_backup();
        return {rc == 0, rc == 2};
    }
    if (q.src != q.dst && bytes) std::memcpy(dst, q.src, bytes);
    const int rc = ring::host_allreduce(rv.tx, rv.rx, ws, rank, q.tag, seq, op.shape, dst, q.count, q.dtype, q.qtype,
                                        q.qalgo, q.op, abort_fn, op.tx, op.rx);
    if (rc) {
        if (backup.ok()) std::memcpy(dst, backup.data(), bytes); // every lane returned: nothing writes dst
        return {rc == 2, rc == 2};
    }
    keep_backup();
    return {true, false};
}

} // namespace pccl::client
