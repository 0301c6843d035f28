// Thin POSIX TCP helpers + LTV (length | id | payload) framing used by every control-plane socket.
#pragma once

#include <sys/socket.h>

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "../common/types.hpp"
#include "../proto/packets.hpp"

namespace pccl::net {

constexpr size_t kMaxControlPacket = 64ull << 20; // 64 MiB cap for LTV packets (reference cap)

bool to_native(const SockAddr &a, sockaddr_storage &ss, socklen_t &len);
SockAddr from_native(const sockaddr_storage &ss);

// Tunes a connected data socket: TCP_NODELAY, keepalive (idle 30 s), large buffers, SIGPIPE-free sends.
void tune_socket(int fd, bool bulk);

// Blocking connect with timeout. Returns fd or -1.
int connect_tcp(const SockAddr &addr, int timeout_ms = 5000);

// Binds+listens on 0.0.0.0 / [::] at `port` (0 = ephemeral). If `bump`, tries successive ports until one binds.
// Returns fd or -1; `bound_port` receives the actual port.
int listen_tcp(ccoip_inet_protocol_t proto, uint16_t port, bool bump, uint16_t &bound_port, int backlog = 1024);

// Full send / receive. Return false on error or EOF. recv_all honours an optional abort flag polled every 100 ms.
bool send_all(int fd, const void *data, size_t n);
bool sendv_all(int fd, struct iovec *iov, int iovcnt);
// MSG_ZEROCOPY variant (same-host sockets); `next_id` = the socket's notification counter (starts at 0)
bool sendv_all_zerocopy(int fd, iovec *iov, int iovcnt, uint32_t &next_id);
bool socket_zerocopy_on(int fd); // SO_ZEROCOPY is set (else MSG_ZEROCOPY would be ignored: no completions)
bool recv_all(int fd, void *data, size_t n);

// Waits until `fd` is readable. Returns 1 readable, 0 timeout, -1 error/hup.
int wait_readable(int fd, int timeout_ms);

// LTV framing: u64 BE length (= payload + 2) | u16 BE id | payload
bool send_ltv(int fd, uint16_t id, const uint8_t *payload, size_t n);
std::vector<uint8_t> ltv_header(uint16_t id, size_t payload_len);
struct LtvPacket {
    uint16_t id = 0;
    std::vector<uint8_t> payload;
};
std::optional<LtvPacket> recv_ltv(int fd, size_t max_len = kMaxControlPacket);

template<typename P>
bool send_packet(int fd, const P &p) {
    proto::WBuf w;
    p.encode(w);
    return send_ltv(fd, P::kId, w.data.data(), w.data.size());
}

template<typename P>
std::optional<P> recv_packet(int fd) {
    auto pkt = recv_ltv(fd);
    if (!pkt || pkt->id != P::kId) return std::nullopt;
    return proto::decode_payload<P>(pkt->payload.data(), pkt->payload.size());
}

void close_fd(int &fd);
// True if `a` is a loopback address or one of this host's interface addresses.
bool is_local_address(const SockAddr &a);
// Identifies this host (kernel boot id + hostname): equal tokens mean two processes can share HIP IPC handles.
// PCCL_HOST_TOKEN overrides it (tests simulate several hosts on one machine).
const std::string &host_token();
bool is_connected(int fd); // MSG_PEEK probe (non-blocking)

} // namespace pccl::net

