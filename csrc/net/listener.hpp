// Accept-thread TCP listener (P2P, shared-state and benchmark servers of a peer).
#pragma once

#include <atomic>
#include <functional>
#include <thread>

#include "../common/types.hpp"

namespace pccl::net {

class Listener {
public:
    using AcceptCb = std::function<void(int fd, const SockAddr &peer)>;
    Listener(ccoip_inet_protocol_t proto, uint16_t port);
    ~Listener();
    bool listen(); // bumps to the next free port
    uint16_t port() const { return port_; }
    bool run_async(AcceptCb cb);
    void interrupt();
    void join();

private:
    ccoip_inet_protocol_t proto_;
    uint16_t requested_port_;
    uint16_t port_ = 0;
    int fd_ = -1;
    int wake_fd_ = -1;
    std::atomic<bool> stop_{false};
    std::thread thread_;
};

} // namespace pccl::net
