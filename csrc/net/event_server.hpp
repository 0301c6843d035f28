// Single-threaded epoll TCP server with LTV packet framing. Used by the master coordinator: every packet handler,
// state mutation and send runs on the loop thread (the reference's libuv ServerSocket plays this role,
// tinysockets/src/server_socket.cpp). Clients are identified by the remote endpoint of their connection.
#pragma once

#include <atomic>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../common/types.hpp"
#include "../proto/packets.hpp"

namespace pccl::net {

class EventServer {
public:
    using ReadCb = std::function<void(const SockAddr &client, uint16_t id, const uint8_t *payload, size_t n)>;
    using CloseCb = std::function<void(const SockAddr &client)>;
    using JoinCb = std::function<void(const SockAddr &client)>;

    EventServer(const SockAddr &listen_addr, bool bump_port);
    ~EventServer();

    void on_read(ReadCb cb) { read_cb_ = std::move(cb); }
    void on_close(CloseCb cb) { close_cb_ = std::move(cb); }
    // called on the loop thread after every wake-up (at least every 500 ms)
    void on_tick(std::function<void()> cb) { tick_cb_ = std::move(cb); }
    void on_join(JoinCb cb) { join_cb_ = std::move(cb); }

    bool listen();
    uint16_t port() const { return port_; }
    bool run_async();
    void interrupt();
    void join();
    bool running() const { return running_.load(); }
    std::thread::id loop_thread_id() const { return loop_tid_.load(std::memory_order_acquire); }

    // Loop-thread only.
    bool send_raw(const SockAddr &client, uint16_t id, std::vector<uint8_t> payload);
    template<typename P>
    bool send_packet(const SockAddr &client, const P &p) {
        proto::WBuf w;
        p.encode(w);
        return send_raw(client, P::kId, std::move(w.data));
    }
    bool close_client(const SockAddr &client); // deferred: close callback fires after the current handler
    // Any thread: runs `fn` on the loop thread soon (after the current batch of events).
    void post(std::function<void()> fn);

private:
    struct Client {
        int fd = -1;
        SockAddr addr{};
        std::vector<uint8_t> rbuf;
        size_t rpos = 0;
        std::deque<std::vector<uint8_t>> wq;
        size_t woff = 0;
        bool want_out = false;
        bool closing = false;
        bool dirty = false; // queued bytes not yet handed to the socket (flushed at the end of the batch)
    };

    void loop();
    void accept_all();
    void handle_readable(Client &c);
    void flush(Client &c);
    void process_pending_closes();
    void update_events(Client &c);
    void flush_dirty();

    SockAddr listen_addr_;
    bool bump_;
    int listen_fd_ = -1;
    int epoll_fd_ = -1;
    int event_fd_ = -1;
    uint16_t port_ = 0;
    std::thread thread_;
    std::atomic<std::thread::id> loop_tid_{};
    std::atomic<bool> running_{false};
    std::atomic<bool> stop_{false};
    std::unordered_map<int, std::unique_ptr<Client>> clients_by_fd_;
    std::unordered_map<SockAddrKey, int, SockAddrKeyHash> fd_by_addr_;
    std::vector<int> pending_close_;
    // Sends issued while handling one batch of events are coalesced per client and flushed once at the end of the
    // batch: a consensus that answers every peer (Abort + Complete to 8 peers) costs one send() per peer, not two.
    bool corked_ = false;
    std::vector<int> dirty_;
    std::mutex posted_mtx_;
    std::vector<std::function<void()>> posted_;
    ReadCb read_cb_;
    CloseCb close_cb_;
    std::function<void()> tick_cb_;
    JoinCb join_cb_;
};

} // namespace pccl::net
