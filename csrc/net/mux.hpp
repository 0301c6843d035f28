// Multiplexed P2P data connection (one TCP stream carrying frames of many concurrent collectives).
//
// Frame format (reference tinysockets multiplexed socket): u64 BE length(= payload + 16) | u64 BE tag |
// u64 BE stream_ctr | payload. A collective op is identified by its tag; stream_ctr is the master-assigned sequence
// number so that frames of an aborted earlier op with the same tag are discarded.
//
// Design (differs from the reference's TX-thread + SPSC-queue design):
//   * TX: the sending op thread writes whole frames directly with sendmsg under a per-connection mutex; no copy,
//     no extra thread hop.
//   * RX: one thread per connection reads frame headers; if the owning op has posted a *sink* (destination memory —
//     user host memory or a pinned staging buffer for the HIP path) the payload is received straight into it
//     (zero copy) in pieces, publishing progress after every piece so the consumer can pipeline reduction/H2D behind
//     the socket. Frames without a matching sink (early arrivals, packet frames) are queued per tag.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../common/types.hpp"
#include "../proto/packets.hpp"

namespace pccl::net {

class MuxConn {
public:
    enum class Mode { Tx, Rx };
    MuxConn(int fd, Mode mode, const SockAddr &peer_addr);
    ~MuxConn();

    bool start();
    void interrupt();
    void join();
    bool is_open() const { return open_.load(std::memory_order_acquire); }
    const SockAddr &peer_addr() const { return peer_addr_; }

    // ---- TX side ----
    bool send_frame(uint64_t tag, uint64_t ctr, const void *data, size_t n);
    // Runs `job` on this connection's persistent sender thread (started on first use, FIFO). Ring steps post one
    // job per stripe instead of starting a thread per stripe per step. A job must not wait on another job of the
    // same connection; it may block on the socket or on device events (both finish on their own).
    void post_send_job(std::function<void()> job);
    template<typename P>
    bool send_packet(uint64_t tag, uint64_t ctr, const P &p) {
        auto bytes = proto::encode_with_id(p);
        return send_frame(tag, ctr, bytes.data(), bytes.size());
    }

    // ---- RX side ----
    // Next queued frame for (tag, ctr); frames for the tag with an older ctr are dropped. Waits up to `timeout`.
    std::optional<std::vector<uint8_t>> recv_frame(uint64_t tag, uint64_t ctr, std::chrono::milliseconds timeout);
    template<typename P>
    std::optional<P> recv_packet(uint64_t tag, uint64_t ctr, std::chrono::milliseconds timeout) {
        auto f = recv_frame(tag, ctr, timeout);
        if (!f || f->size() < 2) return std::nullopt;
        const uint16_t id = static_cast<uint16_t>(((*f)[0] << 8) | (*f)[1]);
        if (id != P::kId) return std::nullopt;
        return proto::decode_payload<P>(f->data() + 2, f->size() - 2);
    }

    // Posts a sink of exactly `n` bytes at `dst` for (tag, ctr). Already-queued matching frames are copied in.
    // Sinks of one tag form a FIFO over the tag's byte stream: bytes fill the oldest sink that still has room (a
    // frame may straddle sinks, so sink sizes need not match the sender's frames), so a ring op can post the next
    // step's sinks while the current step is still receiving (the sender streams both steps back to back on this
    // connection) and early frames land in place instead of being queued and copied once more.
    struct Sink {
        uint64_t ctr = 0;
        uint8_t *dst = nullptr;
        size_t capacity = 0;
        std::atomic<size_t> received{0};
        // the waiter's threshold (wait_sink): the RX thread wakes it only once `received` reaches it (one wake-up
        // per awaited batch instead of one per recv() call)
        std::atomic<size_t> wake_at{SIZE_MAX};
        bool busy = false; // RX thread is writing into dst
    };
    using SinkRef = std::shared_ptr<Sink>;
    SinkRef post_sink(uint64_t tag, uint64_t ctr, uint8_t *dst, size_t n);
    // Bytes delivered into the sink so far (acquire).
    static size_t sink_progress(const SinkRef &s) { return s ? s->received.load(std::memory_order_acquire) : 0; }
    // Waits until progress >= want, the connection closed, or timeout. Returns current progress.
    size_t wait_sink(const SinkRef &s, size_t want, std::chrono::milliseconds timeout);
    // Removes the sink; waits for an in-flight write into it to finish (interrupts the connection if it hangs).
    void remove_sink(uint64_t tag, const SinkRef &s);
    // Tag-keyed forms acting on the oldest sink of the tag (single-sink users)
    size_t sink_progress(uint64_t tag);
    size_t wait_sink(uint64_t tag, size_t want, std::chrono::milliseconds timeout);
    void remove_sink(uint64_t tag);

    uint64_t rx_bytes_total() const { return rx_total_.load(std::memory_order_relaxed); }
    uint64_t tx_bytes_total() const { return tx_total_.load(std::memory_order_relaxed); }
    // How long the frame being sent right now has been inside send_frame (0: no send in progress). A send that does
    // not finish means the peer does not drain its socket (stopped, wedged, or a black-holed path): the op watchdog
    // names it, and aborting ops interrupt such a connection instead of joining a sender blocked in sendmsg.
    std::chrono::nanoseconds send_blocked_for() const;

private:
    struct Frame {
        uint64_t ctr;
        std::vector<uint8_t> data;
        size_t off = 0; // bytes already copied into sinks (a frame may straddle sinks)
    };
    void rx_loop();
    bool read_into(uint8_t *dst, size_t n, Sink *progress_sink);

    int fd_;
    Mode mode_;
    SockAddr peer_addr_;
    std::atomic<bool> open_{false};
    std::atomic<bool> stop_{false};
    std::thread rx_thread_;
    std::mutex tx_mtx_;
    void tx_job_loop();
    std::mutex job_mtx_;
    std::condition_variable job_cv_;
    std::deque<std::function<void()>> jobs_;
    std::thread tx_job_thread_;
    bool jobs_stop_ = false;
    double sim_next_free_ = 0; // WAN emulation: time (s, steady clock) at which this flow's link is free again
    double sim_last_send_ = -1e9;
    const bool zerocopy_;     // bulk frames as MSG_ZEROCOPY (enabled and SO_ZEROCOPY set on this socket)
    uint32_t zc_next_id_ = 0; // MSG_ZEROCOPY notification counter of this socket (guarded by tx_mtx_)

    std::mutex mtx_;
    std::condition_variable cv_;
    // oldest sink of (`tag`, `ctr`) that is not full (the next bytes of the tag's stream go there; a frame may
    // straddle sinks); nullptr if none or it is being written. Caller holds mtx_.
    Sink *sink_for_locked(uint64_t tag, uint64_t ctr);
    void drain_queued_locked(uint64_t tag, uint64_t ctr);
    std::unordered_map<uint64_t, std::deque<SinkRef>> sinks_;
    std::unordered_map<uint64_t, std::deque<Frame>> queued_;
    std::atomic<uint64_t> rx_total_{0};
    std::atomic<uint64_t> tx_total_{0};
    std::atomic<int64_t> send_since_ns_{0}; // steady-clock ns at which the current send_frame started (0: none)
};

// Interrupts (shuts down) every connection of `conns` whose current send has been blocked for at least `min_blocked`:
// the sender thread returns from sendmsg with an error. Used on failed ops, whose senders must not stay blocked on a
// peer that stopped reading (the ring is re-established after a failed op anyway). Returns how many it interrupted.
size_t interrupt_blocked_senders(const std::vector<std::shared_ptr<MuxConn>> &conns, std::chrono::nanoseconds min_blocked);
// PCCL_SINK_DRAIN_MS (default 1000): how long removing a receive sink waits for a frame that is still being written
// into it (the sender of a failed op is mid-frame) before it interrupts the connection.
std::chrono::milliseconds sink_drain_grace();

size_t multiplex_chunk_size();

// 24-byte multiplexed frame header (reference tinysockets multiplexed_socket.cpp:406-411):
// u64 BE (payload + 16) | u64 BE tag | u64 BE stream_ctr.
constexpr size_t kMuxHeaderBytes = 24;
constexpr uint64_t kMuxMaxFrame = 1ull << 30; // largest accepted payload (1 GiB)
void mux_frame_header(uint8_t out[kMuxHeaderBytes], uint64_t payload, uint64_t tag, uint64_t ctr);
// false if the length field is malformed (< 16) or the payload exceeds kMuxMaxFrame
bool mux_parse_header(const uint8_t in[kMuxHeaderBytes], uint64_t &payload, uint64_t &tag, uint64_t &ctr);

// Built-in WAN emulation for tests and benchmarks without root / tc-netem (reference BASELINE config "int8-quantized
// all-reduce over tc-netem 50 ms simulated WAN"): PCCL_SIM_WAN="<one-way latency ms>:<per-flow Mbit/s>[:<link Mbit/s>]"
// shapes every P2P data connection: each frame is serialised at the flow rate (and the shared link rate), and a burst
// that starts after an idle gap pays the latency once (pipelined frames overlap it, as on a real long-fat pipe).
struct WanSim {
    bool enabled = false;
    double latency_s = 0, flow_bps = 0, link_bps = 0;
};
const WanSim &wan_sim();

} // namespace pccl::net
