#include "master_conn.hpp"

#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include "../common/log.hpp"
#include "../common/spin.hpp"
#include "socket.hpp"

namespace pccl::net {

namespace {
int64_t steady_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
constexpr int64_t rx_spin_ns() { return 200 * 1000; }
} // namespace

MasterConnection::MasterConnection(const SockAddr &master) : master_(master) {}

MasterConnection::~MasterConnection() {
    interrupt();
    join();
}

bool MasterConnection::connect() {
    fd_ = connect_tcp(master_, 5000);
    if (fd_ < 0) {
        LOG(ERR) << "Failed to connect to master " << sockaddr_str(master_);
        return false;
    }
    timeval tv{10, 0}; // bounded sends (reference: SO_SNDTIMEO 10 s)
    setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    open_ = true;
    last_rx_ns_.store(steady_ns(), std::memory_order_relaxed);
    rx_thread_ = std::thread([this] {
        name_thread("pccl-master-rx");
        rx_loop();
    });
    return true;
}

void MasterConnection::interrupt() {
    interrupted_ = true;
    if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
    open_ = false;
    q_cv_.notify_all();
}

void MasterConnection::join() {
    if (rx_thread_.joinable()) rx_thread_.join();
    if (fd_ >= 0) {
        ::close(fd_);
        fd_ = -1;
    }
}

bool MasterConnection::send_raw(uint16_t id, const std::vector<uint8_t> &payload) {
    if (!open_) return false;
    if (const int64_t w = rx_spin_ns(); w > 0) rx_hot_until_.store(steady_ns() + w, std::memory_order_relaxed);
    std::lock_guard lock(send_mtx_);
    if (!send_ltv(fd_, id, payload.data(), payload.size())) {
        LOG(WARN) << "Failed to send packet " << id << " to master";
        return false;
    }
    return true;
}

void MasterConnection::rx_loop() {
    while (!interrupted_) {
        // shortly after a request: poll the socket (non-blocking) until the reply is readable or the window closes
        while (!interrupted_ && steady_ns() < rx_hot_until_.load(std::memory_order_relaxed)) {
            pollfd pfd{fd_, POLLIN, 0};
            if (::poll(&pfd, 1, 0) != 0) break;
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
        }
        auto pkt = recv_ltv(fd_);
        if (!pkt) break;
        last_rx_ns_.store(steady_ns(), std::memory_order_relaxed);
        if (pkt->id == proto::M2C_HEARTBEAT) continue; // a sign of life only (liveness extension): never queued
        {
            std::lock_guard lock(q_mtx_);
            queue_.push_back(Item{pkt->id, std::move(pkt->payload)});
            gen_.fetch_add(1, std::memory_order_release);
        }
        q_cv_.notify_all();
    }
    open_ = false;
    q_cv_.notify_all();
    LOG(DEBUG) << "Master connection RX loop ended";
}

bool MasterConnection::contains(const std::function<bool(uint16_t, const std::vector<uint8_t> &)> &match) {
    std::lock_guard lock(q_mtx_);
    for (const auto &it : queue_)
        if (match(it.id, it.payload)) return true;
    return false;
}

bool MasterConnection::take(const std::function<bool(uint16_t, const std::vector<uint8_t> &)> &match,
                            std::chrono::milliseconds timeout) {
    std::unique_lock lock(q_mtx_);
    const auto deadline = std::chrono::steady_clock::now() + timeout;
    bool spun = false;
    while (true) {
        for (auto it = queue_.begin(); it != queue_.end(); ++it) {
            if (match(it->id, it->payload)) {
                queue_.erase(it);
                return true;
            }
        }
        if (!open_) return false;
        if (timeout.count() == 0) return false;
        if (!spun) { // gen_ only changes under q_mtx_, so re-checking it after relocking cannot miss a notify
            spun = true;
            const uint64_t g = gen_.load(std::memory_order_acquire);
            lock.unlock();
            spin_until([&] { return gen_.load(std::memory_order_acquire) != g || !open_; });
            lock.lock();
            if (gen_.load(std::memory_order_acquire) != g || !open_) continue;
        }
        if (timeout.count() < 0) {
            q_cv_.wait(lock);
        } else if (q_cv_.wait_until(lock, deadline) == std::cv_status::timeout) {
            // one final scan happens on next loop iteration only if time remains
            for (auto it = queue_.begin(); it != queue_.end(); ++it) {
                if (match(it->id, it->payload)) {
                    queue_.erase(it);
                    return true;
                }
            }
            return false;
        }
    }
}

} // namespace pccl::net
