#include "listener.hpp"

#include <cerrno>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include "../common/log.hpp"
#include "socket.hpp"

namespace pccl::net {

Listener::Listener(ccoip_inet_protocol_t proto, uint16_t port) : proto_(proto), requested_port_(port) {}

Listener::~Listener() {
    interrupt();
    join();
    if (fd_ >= 0) ::close(fd_);
    if (wake_fd_ >= 0) ::close(wake_fd_);
}

bool Listener::listen() {
    fd_ = listen_tcp(proto_, requested_port_, true, port_);
    if (fd_ < 0) return false;
    wake_fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    return true;
}

bool Listener::run_async(AcceptCb cb) {
    if (fd_ < 0) return false;
    thread_ = std::thread([this, cb = std::move(cb)] {
        while (!stop_) {
            pollfd p[2] = {{fd_, POLLIN, 0}, {wake_fd_, POLLIN, 0}};
            const int rc = ::poll(p, 2, 1000);
            if (rc < 0 && errno != EINTR) break;
            if (stop_) break;
            if (rc <= 0 || !(p[0].revents & POLLIN)) continue;
            sockaddr_storage ss{};
            socklen_t len = sizeof(ss);
            const int cfd = ::accept4(fd_, reinterpret_cast<sockaddr *>(&ss), &len, SOCK_CLOEXEC);
            if (cfd < 0) continue;
            tune_socket(cfd, true);
            cb(cfd, from_native(ss));
        }
    });
    return true;
}

void Listener::interrupt() {
    stop_ = true;
    if (wake_fd_ >= 0) {
        const uint64_t one = 1;
        [[maybe_unused]] auto r = ::write(wake_fd_, &one, 8);
    }
}

void Listener::join() {
    if (thread_.joinable()) thread_.join();
}

} // namespace pccl::net
