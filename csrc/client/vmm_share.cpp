#include "vmm_share.hpp"

#include <poll.h>
#include <sys/random.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <fcntl.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <chrono>
#include <map>
#include <mutex>
#include <random>
#include <thread>

#include "../common/log.hpp"

namespace pccl::client {

namespace {
std::mutex g_mtx;
std::map<uint64_t, int> g_fds; // id -> exported fd

// 64 random bits from the kernel CSPRNG (ids are the capability that grants access to an allocation)
uint64_t random_u64() {
    uint64_t v = 0;
    if (::getrandom(&v, sizeof(v), 0) == static_cast<ssize_t>(sizeof(v))) return v;
    std::random_device rd;
    return (static_cast<uint64_t>(rd()) << 32) ^ rd();
}

socklen_t socket_name(sockaddr_un &a, int pid, uint64_t nonce) {
    a = sockaddr_un{};
    a.sun_family = AF_UNIX;
    // abstract namespace: sun_path[0] == 0, no file to clean up, gone with the process
    const int n = std::snprintf(a.sun_path + 1, sizeof(a.sun_path) - 1, "pccl-vmm-%d-%016llx", pid,
                                static_cast<unsigned long long>(nonce));
    return static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + n);
}
} // namespace

VmmShare &VmmShare::instance() {
    static auto *s = new VmmShare(); // never destroyed: the service lives as long as the process
    return *s;
}

VmmShare::VmmShare() { nonce_ = random_u64() ^ static_cast<uint64_t>(::getpid()); }

bool VmmShare::start() {
    if (started_) return listen_fd_ >= 0;
    started_ = true;
    listen_fd_ = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_un a;
    const socklen_t len = socket_name(a, ::getpid(), nonce_);
    if (listen_fd_ < 0 || ::bind(listen_fd_, reinterpret_cast<sockaddr *>(&a), len) != 0 || ::listen(listen_fd_, 64) != 0) {
        LOG(ERR) << "VMM share: cannot listen on the fd socket";
        if (listen_fd_ >= 0) ::close(listen_fd_);
        listen_fd_ = -1;
        return false;
    }
    std::thread([this] { serve(); }).detach();
    return true;
}

// Access control: the socket name (pid + nonce) is visible to every process of the network namespace
// (/proc/net/unix), so it is no secret. A caller gets an fd only if (1) it runs under this process's uid
// (SO_PEERCRED) and (2) it names a live allocation id; ids are 64 random bits that travel only inside the handles
// exchanged between the peers of a ring, never in the socket name.
void VmmShare::serve() {
    const uid_t me = ::geteuid();
    while (true) {
        const int c = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
        if (c < 0) {
            if (errno != EINTR && errno != ECONNABORTED) // EMFILE / ENFILE / ENOBUFS / ENOMEM: back off, do not spin
                std::this_thread::sleep_for(std::chrono::milliseconds(10));
            continue;
        }
        ucred cred{};
        socklen_t cl = sizeof(cred);
        if (::getsockopt(c, SOL_SOCKET, SO_PEERCRED, &cred, &cl) != 0 || cred.uid != me) {
            LOG(WARN) << "VMM share: refused a request from uid " << cred.uid << " (pid " << cred.pid << ")";
            ::close(c);
            continue;
        }
        uint64_t id = 0;
        timeval tv{2, 0};
        ::setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        ::setsockopt(c, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
        if (::recv(c, &id, sizeof(id), MSG_WAITALL) == static_cast<ssize_t>(sizeof(id))) {
            int fd = -1;
            {
                // a private duplicate, taken under the lock: a concurrent retract() closes the registered fd, never
                // the one being sent (its number could otherwise be reused by an unrelated file in between)
                std::lock_guard l(g_mtx);
                auto it = g_fds.find(id);
                if (it != g_fds.end()) fd = ::fcntl(it->second, F_DUPFD_CLOEXEC, 0);
            }
            char status = fd >= 0 ? 1 : 0;
            iovec iov{&status, 1};
            char ctrl[CMSG_SPACE(sizeof(int))] = {};
            msghdr m{};
            m.msg_iov = &iov;
            m.msg_iovlen = 1;
            if (fd >= 0) {
                m.msg_control = ctrl;
                m.msg_controllen = sizeof(ctrl);
                cmsghdr *cm = CMSG_FIRSTHDR(&m);
                cm->cmsg_level = SOL_SOCKET;
                cm->cmsg_type = SCM_RIGHTS;
                cm->cmsg_len = CMSG_LEN(sizeof(int));
                std::memcpy(CMSG_DATA(cm), &fd, sizeof(int));
            }
            (void)::sendmsg(c, &m, MSG_NOSIGNAL);
            if (fd >= 0) ::close(fd);
        }
        ::close(c);
    }
}

uint64_t VmmShare::publish(int fd) {
    std::lock_guard l(g_mtx);
    if (!start()) return 0;
    uint64_t id = 0;
    while (id == 0 || g_fds.count(id)) id = random_u64();
    g_fds[id] = fd;
    return id;
}

void VmmShare::retract(uint64_t id) {
    std::lock_guard l(g_mtx);
    auto it = g_fds.find(id);
    if (it == g_fds.end()) return;
    ::close(it->second);
    g_fds.erase(it);
}

int VmmShare::fetch(int pid, uint64_t nonce, uint64_t id, int timeout_ms) {
    const int s = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (s < 0) return -1;
    sockaddr_un a;
    const socklen_t len = socket_name(a, pid, nonce);
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    ::setsockopt(s, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    ::setsockopt(s, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    int fd = -1;
    if (::connect(s, reinterpret_cast<sockaddr *>(&a), len) == 0 &&
        ::send(s, &id, sizeof(id), MSG_NOSIGNAL) == static_cast<ssize_t>(sizeof(id))) {
        char status = 0;
        iovec iov{&status, 1};
        char ctrl[CMSG_SPACE(sizeof(int))] = {};
        msghdr m{};
        m.msg_iov = &iov;
        m.msg_iovlen = 1;
        m.msg_control = ctrl;
        m.msg_controllen = sizeof(ctrl);
        if (::recvmsg(s, &m, MSG_CMSG_CLOEXEC) > 0 && status == 1) {
            cmsghdr *cm = CMSG_FIRSTHDR(&m);
            if (cm && cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) std::memcpy(&fd, CMSG_DATA(cm), sizeof(int));
        }
    }
    ::close(s);
    return fd;
}

} // namespace pccl::client
