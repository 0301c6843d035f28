// Client-side connection to the master: a blocking TCP socket with a dedicated RX thread that parses LTV packets
// into a queue. Consumers wait for a packet by id (+ optional predicate), so concurrent collective worker threads
// never steal each other's Commence/Abort/Complete packets (same contract as the reference QueuedSocket,
// tinysockets/src/queued_client_socket.cpp:332-424).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <optional>
#include <thread>
#include <vector>

#include "../common/types.hpp"
#include "../proto/packets.hpp"

namespace pccl::net {

class MasterConnection {
public:
    explicit MasterConnection(const SockAddr &master);
    ~MasterConnection();

    bool connect();
    void interrupt();
    void join();
    bool is_open() const { return open_.load(); }
    // steady-clock ns of the last packet received from the master (any packet, M2CHeartbeat included; 0: none yet)
    int64_t last_rx_ns() const { return last_rx_ns_.load(std::memory_order_relaxed); }

    template<typename P>
    bool send(const P &p) {
        proto::WBuf w;
        p.encode(w);
        return send_raw(P::kId, w.data);
    }

    // Blocks until a packet of type P (matching pred) arrives; nullopt if the connection closed or timeout elapsed.
    // timeout < 0 waits forever; timeout == 0 polls without blocking.
    template<typename P>
    std::optional<P> receive(std::function<bool(const P &)> pred = nullptr,
                             std::chrono::milliseconds timeout = std::chrono::milliseconds(-1)) {
        std::optional<P> result;
        auto match = [&](uint16_t id, const std::vector<uint8_t> &payload) -> bool {
            if (id != P::kId) return false;
            auto p = proto::decode_payload<P>(payload.data(), payload.size());
            if (!p) return false;
            if (pred && !pred(*p)) return false;
            result = std::move(p);
            return true;
        };
        if (!take(match, timeout)) return std::nullopt;
        return result;
    }

    // Whether a packet of type P (matching pred) is queued; it stays queued (its owner still receives it).
    template<typename P>
    bool peek(const std::function<bool(const P &)> &pred) {
        return contains([&](uint16_t id, const std::vector<uint8_t> &payload) {
            if (id != P::kId) return false;
            auto p = proto::decode_payload<P>(payload.data(), payload.size());
            return p && pred(*p);
        });
    }

private:
    bool send_raw(uint16_t id, const std::vector<uint8_t> &payload);
    bool contains(const std::function<bool(uint16_t, const std::vector<uint8_t> &)> &match);
    bool take(const std::function<bool(uint16_t, const std::vector<uint8_t> &)> &match,
              std::chrono::milliseconds timeout);
    void rx_loop();

    SockAddr master_;
    int fd_ = -1;
    std::thread rx_thread_;
    std::atomic<bool> open_{false};
    std::atomic<bool> interrupted_{false};
    std::mutex send_mtx_;
    std::mutex q_mtx_;
    std::condition_variable q_cv_;
    struct Item {
        uint16_t id;
        std::vector<uint8_t> payload;
    };
    std::deque<Item> queue_;
    std::atomic<uint64_t> gen_{0}; // bumped per queued packet (spinning waiters watch it without the lock)
    // steady-clock ns until which the RX thread polls the socket instead of sleeping in recv(): set by every send
    // (a request to the master is usually answered within tens of us, and waking a thread parked on an idle core
    // costs about as much: 200 us)
    std::atomic<int64_t> rx_hot_until_{0};
    std::atomic<int64_t> last_rx_ns_{0};
};

} // namespace pccl::net
