#include "socket.hpp"

#include <arpa/inet.h>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <ifaddrs.h>
#include <linux/errqueue.h>
#include <fstream>
#include <mutex>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/uio.h>
#include <unistd.h>

#include "../common/log.hpp"

namespace pccl::net {

bool to_native(const SockAddr &a, sockaddr_storage &ss, socklen_t &len) {
    std::memset(&ss, 0, sizeof(ss));
    if (a.inet.protocol == inetIPv4) {
        auto *s4 = reinterpret_cast<sockaddr_in *>(&ss);
        s4->sin_family = AF_INET;
        s4->sin_port = htons(a.port);
        std::memcpy(&s4->sin_addr, a.inet.ipv4.data, 4);
        len = sizeof(sockaddr_in);
        return true;
    }
    auto *s6 = reinterpret_cast<sockaddr_in6 *>(&ss);
    s6->sin6_family = AF_INET6;
    s6->sin6_port = htons(a.port);
    std::memcpy(&s6->sin6_addr, a.inet.ipv6.data, 16);
    len = sizeof(sockaddr_in6);
    return true;
}

SockAddr from_native(const sockaddr_storage &ss) {
    SockAddr a{};
    if (ss.ss_family == AF_INET) {
        const auto *s4 = reinterpret_cast<const sockaddr_in *>(&ss);
        a.inet.protocol = inetIPv4;
        std::memcpy(a.inet.ipv4.data, &s4->sin_addr, 4);
        a.port = ntohs(s4->sin_port);
    } else if (ss.ss_family == AF_INET6) {
        const auto *s6 = reinterpret_cast<const sockaddr_in6 *>(&ss);
        // map v4-mapped v6 addresses back to v4
        const uint8_t *b = reinterpret_cast<const uint8_t *>(&s6->sin6_addr);
        static const uint8_t prefix[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};
        if (std::memcmp(b, prefix, 12) == 0) {
            a.inet.protocol = inetIPv4;
            std::memcpy(a.inet.ipv4.data, b + 12, 4);
        } else {
            a.inet.protocol = inetIPv6;
            std::memcpy(a.inet.ipv6.data, b, 16);
        }
        a.port = ntohs(s6->sin6_port);
    }
    return a;
}

// the connected peer is this host (loopback or one of its own addresses)
static bool peer_is_local(int fd) {
    sockaddr_storage ss{};
    socklen_t len = sizeof(ss);
    if (::getpeername(fd, reinterpret_cast<sockaddr *>(&ss), &len) != 0) return false;
    return is_local_address(from_native(ss));
}

void tune_socket(int fd, bool bulk) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof(one));
    int idle = 30, intvl = 5, cnt = 4;
    setsockopt(fd, IPPROTO_TCP, TCP_KEEPIDLE, &idle, sizeof(idle));
    setsockopt(fd, IPPROTO_TCP, TCP_KEEPINTVL, &intvl, sizeof(intvl));
    setsockopt(fd, IPPROTO_TCP, TCP_KEEPCNT, &cnt, sizeof(cnt));
    // Keepalive never fires while sent data is unacknowledged (retransmission governs, ~15 min) nor for a stopped
    // peer (its kernel still ACKs, with a zero window once its buffer is full). TCP_USER_TIMEOUT bounds both: data
    // unacknowledged, or unsent behind a zero window, for this long closes the connection (PCCL_TCP_USER_TIMEOUT_MS,
    // default 30 s, 0 = the kernel's default). The liveness protocol usually acts first (PCCL_PEER_TIMEOUT_MS).
    static const unsigned uto = static_cast<unsigned>(env_size("PCCL_TCP_USER_TIMEOUT_MS", 30000));
    if (uto > 0) setsockopt(fd, IPPROTO_TCP, TCP_USER_TIMEOUT, &uto, sizeof(uto));
    if (bulk) {
        // Same-host data sockets get fixed 8 MiB buffers and MSG_ZEROCOPY sends (loopback: the receiver copies at
        // memory speed, and zero-copy saves the sender's copy, profiles/r3/zerocopy/). A socket to another host keeps
        // the kernel's buffer autotuning, which grows the window to the path's bandwidth-delay product (a fixed
        // 8 MiB caps a 100 ms-RTT connection at ~0.7 Gbit/s), and plain sends: a MSG_ZEROCOPY frame completes only
        // once the peer acknowledged it, which turns every frame into one round trip on a long path (reference
        // tinysockets/src/multiplexed_socket.cpp:19-61 leaves autotuning on as well).
        if (peer_is_local(fd)) {
            int sz = 8 << 20;
            setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
            setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
            setsockopt(fd, SOL_SOCKET, SO_ZEROCOPY, &one, sizeof(one)); // best effort (socket_zerocopy_on)
        }
        // like the reference's data sockets (tinysockets/src/multiplexed_socket.cpp:51-59): immediate ACKs, and busy
        // polling of the device queue on NICs that support it (best effort: a value above net.core.busy_poll needs
        // CAP_NET_ADMIN, and loopback has no NAPI queue to poll)
        setsockopt(fd, IPPROTO_TCP, TCP_QUICKACK, &one, sizeof(one));
        int busy = 50;
        setsockopt(fd, SOL_SOCKET, SO_BUSY_POLL, &busy, sizeof(busy));
    }
}

bool socket_zerocopy_on(int fd) {
    int v = 0;
    socklen_t l = sizeof(v);
    return ::getsockopt(fd, SOL_SOCKET, SO_ZEROCOPY, &v, &l) == 0 && v != 0;
}


int connect_tcp(const SockAddr &addr, int timeout_ms) {
    sockaddr_storage ss{};
    socklen_t len{};
    to_native(addr, ss, len);
    const int fd = ::socket(ss.ss_family, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    if (fd < 0) return -1;
    int rc = ::connect(fd, reinterpret_cast<sockaddr *>(&ss), len);
    if (rc != 0 && errno != EINPROGRESS) {
        ::close(fd);
        return -1;
    }
    if (rc != 0) {
        pollfd p{fd, POLLOUT, 0};
        rc = ::poll(&p, 1, timeout_ms);
        int err = 0;
        socklen_t el = sizeof(err);
        if (rc <= 0 || getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el) != 0 || err != 0) {
            ::close(fd);
            return -1;
        }
    }
    // back to blocking
    const int flags = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, flags & ~O_NONBLOCK);
    tune_socket(fd, true);
    return fd;
}

int listen_tcp(ccoip_inet_protocol_t proto, uint16_t port, bool bump, uint16_t &bound_port, int backlog) {
    for (int attempt = 0; attempt < 2048; ++attempt) {
        const uint16_t try_port = static_cast<uint16_t>(port == 0 ? 0 : port + attempt);
        const int fam = proto == inetIPv4 ? AF_INET : AF_INET6;
        const int fd = ::socket(fam, SOCK_STREAM | SOCK_CLOEXEC, 0);
        if (fd < 0) return -1;
        int one = 1;
        setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        sockaddr_storage ss{};
        socklen_t len;
        if (fam == AF_INET) {
            auto *s4 = reinterpret_cast<sockaddr_in *>(&ss);
            s4->sin_family = AF_INET;
            s4->sin_addr.s_addr = htonl(INADDR_ANY);
            s4->sin_port = htons(try_port);
            len = sizeof(sockaddr_in);
        } else {
            auto *s6 = reinterpret_cast<sockaddr_in6 *>(&ss);
            s6->sin6_family = AF_INET6;
            s6->sin6_addr = in6addr_any;
            s6->sin6_port = htons(try_port);
            int off = 0;
            setsockopt(fd, IPPROTO_IPV6, IPV6_V6ONLY, &off, sizeof(off));
            len = sizeof(sockaddr_in6);
        }
        if (::bind(fd, reinterpret_cast<sockaddr *>(&ss), len) == 0 && ::listen(fd, backlog) == 0) {
            sockaddr_storage got{};
            socklen_t gl = sizeof(got);
            getsockname(fd, reinterpret_cast<sockaddr *>(&got), &gl);
            bound_port = from_native(got).port;
            return fd;
        }
        ::close(fd);
        if (!bump || port == 0) return -1;
    }
    return -1;
}

bool send_all(int fd, const void *data, size_t n) {
    const auto *p = static_cast<const uint8_t *>(data);
    while (n > 0) {
        const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += k;
        n -= static_cast<size_t>(k);
    }
    return true;
}

bool sendv_all(int fd, iovec *iov, int iovcnt) {
    while (iovcnt > 0) {
        msghdr msg{};
        msg.msg_iov = iov;
        msg.msg_iovlen = static_cast<size_t>(iovcnt);
        ssize_t k = ::sendmsg(fd, &msg, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        while (k > 0 && iovcnt > 0) {
            if (static_cast<size_t>(k) >= iov->iov_len) {
                k -= static_cast<ssize_t>(iov->iov_len);
                ++iov;
                --iovcnt;
            } else {
                iov->iov_base = static_cast<uint8_t *>(iov->iov_base) + k;
                iov->iov_len -= static_cast<size_t>(k);
                k = 0;
            }
        }
        while (iovcnt > 0 && iov->iov_len == 0) {
            ++iov;
            --iovcnt;
        }
    }
    return true;
}

// MSG_ZEROCOPY send (same-host sockets, socket_zerocopy_on): the kernel pins the
// user pages instead of copying them into socket buffers and reports completion on the socket's error queue; the call returns once every
// byte it sent is released, so the caller may reuse the buffer as after a plain send. On loopback the kernel copies
// the pages anyway when it delivers them to the receiving socket ("deferred copy", reported as
// SO_EE_CODE_ZEROCOPY_COPIED), so only a real NIC saves the copy. Returns false on error.
bool sendv_all_zerocopy(int fd, iovec *iov, int iovcnt, uint32_t &next_id) {
    uint32_t first = next_id;
    bool sent_any = false;
    while (iovcnt > 0) {
        msghdr msg{};
        msg.msg_iov = iov;
        msg.msg_iovlen = static_cast<size_t>(iovcnt);
        ssize_t k = ::sendmsg(fd, &msg, MSG_NOSIGNAL | MSG_ZEROCOPY);
        if (k < 0) {
            if (errno == EINTR) continue;
            if (errno == ENOBUFS) { // optmem exhausted by pinned pages in flight: fall back for this piece
                k = ::sendmsg(fd, &msg, MSG_NOSIGNAL);
                if (k < 0) return false;
            } else {
                return false;
            }
        } else {
            ++next_id; // every successful MSG_ZEROCOPY call takes one notification id
            sent_any = true;
        }
        while (k > 0 && iovcnt > 0) {
            if (static_cast<size_t>(k) >= iov->iov_len) {
                k -= static_cast<ssize_t>(iov->iov_len);
                ++iov;
                --iovcnt;
            } else {
                iov->iov_base = static_cast<uint8_t *>(iov->iov_base) + k;
                iov->iov_len -= static_cast<size_t>(k);
                k = 0;
            }
        }
        while (iovcnt > 0 && iov->iov_len == 0) {
            ++iov;
            --iovcnt;
        }
    }
    if (!sent_any) return true;
    // wait for the notifications of ids [first, next_id)
    uint32_t done_to = first; // completed below this id
    int idle_polls = 0;
    while (static_cast<int32_t>(next_id - done_to) > 0) {
        pollfd pfd{fd, 0, 0}; // POLLERR is always reported
        const int pr = ::poll(&pfd, 1, 1000);
        if (pr < 0 && errno != EINTR) return false;
        if (pr == 0 && ++idle_polls >= 30) { // no completion for 30 s: the peer stopped reading
            LOG(WARN) << "MSG_ZEROCOPY: no send completion for 30 s; closing the connection";
            return false;
        }
        // the socket was shut down (an aborted op interrupts a sender blocked on a peer that stopped reading) or
        // failed: completions may never come, and poll would report the hang-up at once, forever
        const bool hup = pr > 0 && (pfd.revents & (POLLHUP | POLLNVAL)) != 0;
        while (true) {
            char ctrl[128];
            msghdr msg{};
            msg.msg_control = ctrl;
            msg.msg_controllen = sizeof(ctrl);
            if (::recvmsg(fd, &msg, MSG_ERRQUEUE | MSG_DONTWAIT) < 0) {
                if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
                return false;
            }
            for (cmsghdr *cm = CMSG_FIRSTHDR(&msg); cm; cm = CMSG_NXTHDR(&msg, cm)) {
                if (!((cm->cmsg_level == SOL_IP && cm->cmsg_type == IP_RECVERR) ||
                      (cm->cmsg_level == SOL_IPV6 && cm->cmsg_type == IPV6_RECVERR)))
                    continue;
                sock_extended_err se{};
                std::memcpy(&se, CMSG_DATA(cm), sizeof(se));
                if (se.ee_origin != SO_EE_ORIGIN_ZEROCOPY) continue;
                // [ee_info, ee_data] completed; notifications arrive in order on one socket
                if (static_cast<int32_t>(se.ee_data + 1 - done_to) > 0) done_to = se.ee_data + 1;
            }
        }
        if (hup && static_cast<int32_t>(next_id - done_to) > 0) return false;
    }
    return true;
}

bool recv_all(int fd, void *data, size_t n) {
    auto *p = static_cast<uint8_t *>(data);
    while (n > 0) {
        const ssize_t k = ::recv(fd, p, n, 0);
        if (k < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (k == 0) return false;
        p += k;
        n -= static_cast<size_t>(k);
    }
    return true;
}

int wait_readable(int fd, int timeout_ms) {
    pollfd p{fd, POLLIN, 0};
    const int rc = ::poll(&p, 1, timeout_ms);
    if (rc < 0) return errno == EINTR ? 0 : -1;
    if (rc == 0) return 0;
    if (p.revents & POLLIN) return 1;
    return -1;
}

std::vector<uint8_t> ltv_header(uint16_t id, size_t payload_len) {
    std::vector<uint8_t> h(10);
    const uint64_t len = payload_len + 2;
    for (int i = 0; i < 8; ++i) h[i] = static_cast<uint8_t>(len >> (8 * (7 - i)));
    h[8] = static_cast<uint8_t>(id >> 8);
    h[9] = static_cast<uint8_t>(id);
    return h;
}

bool send_ltv(int fd, uint16_t id, const uint8_t *payload, size_t n) {
    auto h = ltv_header(id, n);
    iovec iov[2] = {{h.data(), h.size()}, {const_cast<uint8_t *>(payload), n}};
    return sendv_all(fd, iov, n ? 2 : 1);
}

std::optional<LtvPacket> recv_ltv(int fd, size_t max_len) {
    uint8_t h[10];
    if (!recv_all(fd, h, 10)) return std::nullopt;
    uint64_t len = 0;
    for (int i = 0; i < 8; ++i) len = (len << 8) | h[i];
    if (len < 2 || len - 2 > max_len) return std::nullopt;
    LtvPacket p;
    p.id = static_cast<uint16_t>((h[8] << 8) | h[9]);
    p.payload.resize(len - 2);
    if (len > 2 && !recv_all(fd, p.payload.data(), len - 2)) return std::nullopt;
    return p;
}

void close_fd(int &fd) {
    if (fd >= 0) {
        ::shutdown(fd, SHUT_RDWR);
        ::close(fd);
        fd = -1;
    }
}

bool is_connected(int fd) {
    if (fd < 0) return false;
    char c;
    const ssize_t k = ::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
    if (k == 0) return false;
    if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) return false;
    return true;
}

bool is_local_address(const SockAddr &a) {
    if (sockaddr_is_loopback(a)) return true;
    ifaddrs *ifs = nullptr;
    if (getifaddrs(&ifs) != 0) return false;
    bool found = false;
    for (ifaddrs *it = ifs; it && !found; it = it->ifa_next) {
        if (!it->ifa_addr) continue;
        if (it->ifa_addr->sa_family == AF_INET && a.inet.protocol == inetIPv4) {
            const auto *s4 = reinterpret_cast<const sockaddr_in *>(it->ifa_addr);
            found = std::memcmp(&s4->sin_addr, a.inet.ipv4.data, 4) == 0;
        } else if (it->ifa_addr->sa_family == AF_INET6 && a.inet.protocol == inetIPv6) {
            const auto *s6 = reinterpret_cast<const sockaddr_in6 *>(it->ifa_addr);
            found = std::memcmp(&s6->sin6_addr, a.inet.ipv6.data, 16) == 0;
        }
    }
    freeifaddrs(ifs);
    return found;
}

const std::string &host_token() {
    static std::once_flag once;
    static std::string token;
    std::call_once(once, [] {
        if (const char *o = std::getenv("PCCL_HOST_TOKEN"); o && *o) { // tests: simulate several hosts on one box
            token = o;
            return;
        }
        std::ifstream f("/proc/sys/kernel/random/boot_id");
        std::getline(f, token);
        char host[256] = {};
        gethostname(host, sizeof(host) - 1);
        token += "|";
        token += host;
    });
    return token;
}

} // namespace pccl::net
