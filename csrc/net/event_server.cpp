#include "event_server.hpp"

#include <chrono>

#include <cerrno>
#include <csignal>
#include <cstring>
#include <fcntl.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include "../common/log.hpp"
#include "socket.hpp"

namespace pccl::net {

EventServer::EventServer(const SockAddr &listen_addr, bool bump_port) : listen_addr_(listen_addr), bump_(bump_port) {}

EventServer::~EventServer() {
    interrupt();
    join();
    for (auto &[fd, c] : clients_by_fd_) ::close(fd);
    if (listen_fd_ >= 0) ::close(listen_fd_);
    if (epoll_fd_ >= 0) ::close(epoll_fd_);
    if (event_fd_ >= 0) ::close(event_fd_);
}

bool EventServer::listen() {
    std::signal(SIGPIPE, SIG_IGN);
    listen_fd_ = listen_tcp(listen_addr_.inet.protocol, listen_addr_.port, bump_, port_);
    if (listen_fd_ < 0) {
        LOG(ERR) << "EventServer: failed to listen on port " << listen_addr_.port;
        return false;
    }
    fcntl(listen_fd_, F_SETFL, fcntl(listen_fd_, F_GETFL, 0) | O_NONBLOCK);
    epoll_fd_ = epoll_create1(EPOLL_CLOEXEC);
    event_fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = listen_fd_;
    epoll_ctl(epoll_fd_, EPOLL_CTL_ADD, listen_fd_, &ev);
    ev.data.fd = event_fd_;
    epoll_ctl(epoll_fd_, EPOLL_CTL_ADD, event_fd_, &ev);
    return true;
}

bool EventServer::run_async() {
    if (listen_fd_ < 0 || running_) return false;
    running_ = true;
    thread_ = std::thread([this] { loop(); });
    loop_tid_.store(thread_.get_id(), std::memory_order_release);
    return true;
}

void EventServer::interrupt() {
    stop_ = true;
    if (event_fd_ >= 0) {
        const uint64_t one = 1;
        [[maybe_unused]] auto r = ::write(event_fd_, &one, 8);
    }
}

void EventServer::post(std::function<void()> fn) {
    {
        std::lock_guard l(posted_mtx_);
        posted_.push_back(std::move(fn));
    }
    if (event_fd_ >= 0) {
        const uint64_t one = 1;
        [[maybe_unused]] auto r = ::write(event_fd_, &one, 8);
    }
}

void EventServer::join() {
    if (thread_.joinable() && std::this_thread::get_id() != thread_.get_id()) thread_.join();
}

void EventServer::loop() {
    loop_tid_.store(std::this_thread::get_id(), std::memory_order_release);
    std::vector<epoll_event> events(256);
    // After a batch of events, poll without blocking for a short while before sleeping in epoll_wait: the peers'
    // packets of one consensus (8 collective initiates, 8 completes) arrive spread over tens of microseconds, and a
    // sleeping loop thread pays a scheduler wake-up (10-30 us on a loaded host) for each. 100 us bounds the spin.
    constexpr long spin_us = 100;
    auto last_event = std::chrono::steady_clock::now() - std::chrono::hours(1);
    while (!stop_) {
        const bool spinning = spin_us > 0 && std::chrono::steady_clock::now() - last_event < std::chrono::microseconds(spin_us);
        const int n = epoll_wait(epoll_fd_, events.data(), static_cast<int>(events.size()), spinning ? 0 : 500);
        if (n > 0) last_event = std::chrono::steady_clock::now();
        if (n == 0 && spinning) {
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
            continue;
        }
        if (n < 0) {
            if (errno == EINTR) continue;
            break;
        }
        corked_ = true;
        for (int i = 0; i < n && !stop_; ++i) {
            const int fd = events[i].data.fd;
            if (fd == listen_fd_) {
                accept_all();
                continue;
            }
            if (fd == event_fd_) {
                uint64_t v;
                [[maybe_unused]] auto r = ::read(event_fd_, &v, 8);
                continue;
            }
            auto it = clients_by_fd_.find(fd);
            if (it == clients_by_fd_.end()) continue;
            Client &c = *it->second;
            if (c.closing) continue;
            if (events[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) handle_readable(c);
            if (!c.closing && (events[i].events & EPOLLOUT)) flush(c);
        }
        flush_dirty();
        process_pending_closes();
        std::vector<std::function<void()>> posted;
        {
            std::lock_guard l(posted_mtx_);
            posted.swap(posted_);
        }
        for (auto &f : posted)
            if (!stop_) f();
        flush_dirty();
        if (!posted.empty()) process_pending_closes();
        if (tick_cb_ && !stop_) tick_cb_();
        flush_dirty();
        corked_ = false;
    }
    // shutdown: close all clients (no callbacks on interrupt)
    for (auto &[fd, c] : clients_by_fd_) ::close(fd);
    clients_by_fd_.clear();
    fd_by_addr_.clear();
    running_ = false;
}

void EventServer::accept_all() {
    while (true) {
        sockaddr_storage ss{};
        socklen_t len = sizeof(ss);
        const int fd = ::accept4(listen_fd_, reinterpret_cast<sockaddr *>(&ss), &len, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (fd < 0) return;
        tune_socket(fd, false);
        auto c = std::make_unique<Client>();
        c->fd = fd;
        c->addr = from_native(ss);
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.fd = fd;
        epoll_ctl(epoll_fd_, EPOLL_CTL_ADD, fd, &ev);
        fd_by_addr_[SockAddrKey::of(c->addr)] = fd;
        const SockAddr addr = c->addr;
        clients_by_fd_[fd] = std::move(c);
        LOG(DEBUG) << "EventServer: accepted " << sockaddr_str(addr);
        if (join_cb_) join_cb_(addr);
    }
}

void EventServer::handle_readable(Client &c) {
    uint8_t tmp[65536];
    bool closed = false;
    // at most 1 MiB per readiness event: a client that streams faster than we drain would otherwise keep every recv()
    // full, so the loop never reached the dispatch below (rbuf grew without bound and no packet was handled; seen in
    // transport_tests es_interrupt_while_client_streams). epoll is level-triggered: the rest is read next round.
    for (int rounds = 0; rounds < 16; ++rounds) {
        const ssize_t k = ::recv(c.fd, tmp, sizeof(tmp), 0);
        if (k > 0) {
            c.rbuf.insert(c.rbuf.end(), tmp, tmp + k);
            if (static_cast<size_t>(k) < sizeof(tmp)) break;
            continue;
        }
        if (k == 0) {
            closed = true;
            break;
        }
        if (errno == EINTR) continue;
        if (errno != EAGAIN && errno != EWOULDBLOCK) closed = true;
        break;
    }
    // dispatch complete frames
    while (!c.closing) {
        const size_t avail = c.rbuf.size() - c.rpos;
        if (avail < 10) break;
        const uint8_t *h = c.rbuf.data() + c.rpos;
        uint64_t len = 0;
        for (int i = 0; i < 8; ++i) len = (len << 8) | h[i];
        if (len < 2 || len - 2 > kMaxControlPacket) {
            LOG(WARN) << "EventServer: malformed frame from " << sockaddr_str(c.addr) << "; closing";
            close_client(c.addr);
            break;
        }
        if (avail < 8 + len) break;
        const uint16_t id = static_cast<uint16_t>((h[8] << 8) | h[9]);
        const SockAddr addr = c.addr;
        const size_t payload_off = c.rpos + 10;
        c.rpos += 8 + len;
        // copy payload out: the callback may send/close and we must not hold references into rbuf
        std::vector<uint8_t> payload(c.rbuf.begin() + static_cast<long>(payload_off),
                                     c.rbuf.begin() + static_cast<long>(payload_off + len - 2));
        if (read_cb_) read_cb_(addr, id, payload.data(), payload.size());
    }
    if (c.rpos > 0 && c.rpos == c.rbuf.size()) {
        c.rbuf.clear();
        c.rpos = 0;
    } else if (c.rpos > (1 << 20)) {
        c.rbuf.erase(c.rbuf.begin(), c.rbuf.begin() + static_cast<long>(c.rpos));
        c.rpos = 0;
    }
    if (closed && !c.closing) close_client(c.addr);
}

bool EventServer::send_raw(const SockAddr &client, uint16_t id, std::vector<uint8_t> payload) {
    auto it = fd_by_addr_.find(SockAddrKey::of(client));
    if (it == fd_by_addr_.end()) return false;
    Client &c = *clients_by_fd_.at(it->second);
    if (c.closing) return false;
    auto h = ltv_header(id, payload.size());
    if (corked_ && !c.wq.empty()) { // append to the pending buffer: one send() for the batch
        auto &back = c.wq.back();
        back.insert(back.end(), h.begin(), h.end());
        back.insert(back.end(), payload.begin(), payload.end());
    } else {
        h.insert(h.end(), payload.begin(), payload.end());
        c.wq.push_back(std::move(h));
    }
    if (!corked_) {
        flush(c);
    } else if (!c.dirty) {
        c.dirty = true;
        dirty_.push_back(c.fd);
    }
    return true;
}

void EventServer::flush_dirty() {
    for (int fd : dirty_) {
        auto it = clients_by_fd_.find(fd);
        if (it == clients_by_fd_.end()) continue;
        Client &c = *it->second;
        c.dirty = false;
        if (!c.closing) flush(c);
    }
    dirty_.clear();
}

void EventServer::flush(Client &c) {
    while (!c.wq.empty()) {
        auto &front = c.wq.front();
        const ssize_t k = ::send(c.fd, front.data() + c.woff, front.size() - c.woff, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            close_client(c.addr);
            return;
        }
        c.woff += static_cast<size_t>(k);
        if (c.woff == front.size()) {
            c.wq.pop_front();
            c.woff = 0;
        }
    }
    const bool want = !c.wq.empty();
    if (want != c.want_out) {
        c.want_out = want;
        update_events(c);
    }
}

void EventServer::update_events(Client &c) {
    epoll_event ev{};
    ev.events = EPOLLIN | (c.want_out ? static_cast<uint32_t>(EPOLLOUT) : 0u);
    ev.data.fd = c.fd;
    epoll_ctl(epoll_fd_, EPOLL_CTL_MOD, c.fd, &ev);
}

bool EventServer::close_client(const SockAddr &client) {
    auto it = fd_by_addr_.find(SockAddrKey::of(client));
    if (it == fd_by_addr_.end()) return false;
    Client &c = *clients_by_fd_.at(it->second);
    if (c.closing) return true;
    c.closing = true;
    // best effort: push out anything queued (e.g. a final response) before closing
    if (!c.wq.empty()) {
        const int flags = fcntl(c.fd, F_GETFL, 0);
        fcntl(c.fd, F_SETFL, flags & ~O_NONBLOCK);
        timeval tv{0, 200000};
        setsockopt(c.fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
        for (auto &buf : c.wq) {
            if (!send_all(c.fd, buf.data() + c.woff, buf.size() - c.woff)) break;
            c.woff = 0;
        }
        c.wq.clear();
    }
    ::shutdown(c.fd, SHUT_RDWR);
    pending_close_.push_back(c.fd);
    return true;
}

void EventServer::process_pending_closes() {
    while (!pending_close_.empty()) {
        const int fd = pending_close_.back();
        pending_close_.pop_back();
        auto it = clients_by_fd_.find(fd);
        if (it == clients_by_fd_.end()) continue;
        const SockAddr addr = it->second->addr;
        epoll_ctl(epoll_fd_, EPOLL_CTL_DEL, fd, nullptr);
        ::close(fd);
        fd_by_addr_.erase(SockAddrKey::of(addr));
        clients_by_fd_.erase(it);
        LOG(DEBUG) << "EventServer: client " << sockaddr_str(addr) << " closed";
        if (close_cb_) close_cb_(addr);
    }
}

} // namespace pccl::net
