// Shared-state synchronization (reference: ccoip_client_handler.cpp:344-638, 1022-1164).
//
// Every peer hashes its entries (HIP simplehash kernel for HBM tensors, bit-identical to the host emulation), the
// master elects the most popular content, and outdated peers pull the dirty entries from a distributor over a
// one-off TCP connection. HBM tensors are streamed through a double-buffered pinned staging ring
// (D2H of piece k+1 overlaps the send of piece k on the distributor; receive of piece k+1 overlaps the H2D of piece k
// on the receiver) instead of the reference's whole-tensor malloc + blocking cuMemcpy.
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>

#include "../common/log.hpp"
#include "../kernels/host_kernels.hpp"
#include "../net/socket.hpp"
#include "client.hpp"
#include "pools.hpp"

namespace pccl::client {

using namespace proto;

static constexpr size_t kStagePiece = 32ull << 20;

bool Client::hash_entry(const SSEntry &e, uint64_t &hash, HashType &type) {
    type = HashType::Simple;
    if (e.bytes == 0) {
        hash = 0;
        return true;
    }
    DeviceBackend *be = device_backend();
    DevPtrInfo pi{};
    if (be) be->pointer_info(e.data, pi);
    if (pi.is_device) {
        be->set_device(pi.device);
        if (reinterpret_cast<uintptr_t>(e.data) % 16 != 0) {
            Lease tmp(device_pool(), e.bytes, pi.device);
            be->memcpy_sync(tmp.data(), e.data, e.bytes);
            hash = be->simplehash(tmp.data(), e.bytes, nullptr);
        } else {
            hash = be->simplehash(e.data, e.bytes, nullptr);
        }
        return true;
    }
    if (e.device == DeviceType::Gpu) {
        LOG(ERR) << "Shared state entry '" << e.key << "' declared as GPU tensor but pointer is not device memory";
        return false;
    }
    if (reinterpret_cast<uintptr_t>(e.data) % 16 != 0) {
        Lease tmp(host_pool(), e.bytes);
        std::memcpy(tmp.data(), e.data, e.bytes);
        hash = kernels::simplehash_host(tmp.data(), e.bytes);
    } else {
        hash = kernels::simplehash_host(e.data, e.bytes);
    }
    return true;
}

static bool verify_hash(Client *, const SSEntry &e, uint64_t expected, HashType type, uint64_t actual_simple) {
    if (type == HashType::Simple) return actual_simple == expected;
    // CRC32 (accepted for compatibility; never produced by this implementation)
    std::vector<uint8_t> host(e.bytes);
    DeviceBackend *be = device_backend();
    DevPtrInfo pi{};
    if (be) be->pointer_info(e.data, pi);
    if (pi.is_device) be->memcpy_sync(host.data(), e.data, e.bytes);
    else std::memcpy(host.data(), e.data, e.bytes);
    return kernels::crc32c(host.data(), host.size()) == expected;
}

bool Client::sync_shared_state(SharedState &ss, SSInfo &info) {
    info = SSInfo{};
    if (!accepted_ || !master_.is_open()) return false;
    if (any_collective_running()) return false;

    C2MSyncSharedState vote;
    vote.revision = ss.revision;
    vote.strategy = ss.strategy;
    for (const auto &e : ss.entries) {
        SharedStateHashEntry he;
        he.key = e.key;
        he.data_type = e.dtype;
        he.num_elements = e.count;
        he.allow_content_inequality = e.allow_content_inequality;
        if (!e.allow_content_inequality) {
            if (!hash_entry(e, he.hash, he.hash_type)) return false;
        }
        vote.entries.push_back(he);
    }

    struct PhaseGuard {
        Client *c;
        PhaseGuard(Client *cl, SharedState *s) : c(cl) {
            std::lock_guard l(c->ss_mtx_);
            c->serving_ = s;
        }
        ~PhaseGuard() {
            std::lock_guard l(c->ss_mtx_);
            c->serving_ = nullptr;
        }
    } guard(this, &ss); // serve requests from the moment we vote (peers may be faster than our master packet)

    if (!master_.send(vote)) return false;
    auto resp = master_.receive<M2CSyncSharedState>();
    if (!resp) {
        LOG(ERR) << "Shared state sync: no response from master (kicked?)";
        return false;
    }
    // Fetches the outdated entries from one distributor; false if it failed or died mid-transfer (partially written
    // entries are overwritten by the next attempt, and every entry is hash-verified at the end).
    auto fetch_from = [&](const SockAddr &distributor) -> bool {
        const int fd = net::connect_tcp(distributor, 10000);
        if (fd < 0) {
            LOG(WARN) << "Shared state sync: cannot reach distributor " << sockaddr_str(distributor);
            return false;
        }
        struct FdGuard {
            int fd;
            ~FdGuard() { ::close(fd); }
        } fdg{fd};
        C2SRequestSharedState req;
        req.keys = resp->outdated_keys;
        if (!net::send_packet(fd, req)) return false;
        auto sresp = net::recv_packet<S2CSharedStateResponse>(fd);
        if (!sresp || sresp->status != SharedStateStatus::Success) {
            LOG(WARN) << "Shared state sync: distributor refused (status "
                     << (sresp ? static_cast<int>(sresp->status) : -1) << ")";
            return false;
        }
        ss.revision = sresp->revision;
        std::map<std::string, SSEntry *> by_key;
        for (auto &e : ss.entries) by_key[e.key] = &e;
        if (sresp->entries.size() != resp->outdated_keys.size()) return false;
        DeviceBackend *be = device_backend();
        for (size_t i = 0; i < sresp->entries.size(); ++i) {
            const auto &se = sresp->entries[i];
            auto it = by_key.find(se.key);
            if (it == by_key.end() || se.key != resp->outdated_keys[i]) {
                LOG(ERR) << "Shared state sync: unexpected key " << se.key;
                return false;
            }
            SSEntry &dst = *it->second;
            if (se.size_bytes != dst.bytes) {
                LOG(ERR) << "Shared state sync: size mismatch for " << se.key;
                return false;
            }
            DevPtrInfo pi{};
            if (be) be->pointer_info(dst.data, pi);
            if (pi.is_device) {
                be->set_device(pi.device);
                StreamLease stream(pi.device);
                DevStream st = stream.get();
                Lease a(pinned_pool(), kStagePiece), b(pinned_pool(), kStagePiece);
                uint8_t *stage[2] = {a.data(), b.data()};
                DevEvent evs[2] = {event_pool().get(), event_pool().get()};
                bool ok = a.ok() && b.ok();
                size_t off = 0, k = 0;
                while (ok && off < dst.bytes) {
                    const size_t n = std::min(kStagePiece, dst.bytes - off);
                    if (k >= 2) be->event_sync(evs[k % 2]); // previous H2D from this staging buffer done
                    ok = net::recv_all(fd, stage[k % 2], n);
                    if (!ok) break;
                    be->memcpy_async(static_cast<uint8_t *>(dst.data) + off, stage[k % 2], n, st);
                    be->event_record(evs[k % 2], st);
                    off += n;
                    ++k;
                }
                be->stream_sync(st);
                event_pool().put(evs[0]);
                event_pool().put(evs[1]);
                if (!ok) {
                    LOG(ERR) << "Shared state sync: transfer of " << se.key << " failed";
                    return false;
                }
            } else {
                if (!net::recv_all(fd, dst.data, dst.bytes)) {
                    LOG(ERR) << "Shared state sync: transfer of " << se.key << " failed";
                    return false;
                }
            }
            info.rx_bytes += dst.bytes;
            if (!dst.allow_content_inequality && i < resp->expected_hashes.size()) {
                uint64_t h = 0;
                HashType t;
                if (!hash_entry(dst, h, t)) return false;
                if (!verify_hash(this, dst, resp->expected_hashes[i], resp->expected_hash_types[i], h)) {
                    LOG(ERR) << "Shared state sync: distributor sent corrupt content for " << se.key;
                    return false;
                }
            }
        }
        return true;
    };
    bool fetched = !resp->is_outdated;
    if (resp->is_outdated) {
        std::vector<SockAddr> sources;
        if (!sockaddr_is_zero(resp->distributor)) sources.push_back(resp->distributor);
        for (const auto &f : resp->fallback_distributors) sources.push_back(f);
        if (sources.empty()) LOG(ERR) << "Shared state sync: master assigned no distributor";
        for (const auto &src : sources) {
            info.rx_bytes = 0;
            if ((fetched = fetch_from(src))) break;
            LOG(WARN) << "Shared state sync: distributor " << sockaddr_str(src) << " failed; trying the next one";
        }
    }
    // complete the round even if nothing could be fetched: the other peers must not wait for us forever
    if (!master_.send(C2MDistSharedStateComplete{})) return false;
    if (!master_.receive<M2CSyncSharedStateComplete>()) {
        LOG(ERR) << "Shared state sync: no completion from master";
        return false;
    }
    if (!fetched) {
        LOG(ERR) << "Shared state sync: no distributor could deliver the shared state";
        return false;
    }
    info.tx_bytes = ss_tx_bytes_.exchange(0);
    return true;
}

void Client::serve_shared_state(int fd, SockAddr peer) {
    struct FdGuard {
        int fd;
        ~FdGuard() {
            ::shutdown(fd, SHUT_RDWR);
            ::close(fd);
        }
    } g{fd};
    timeval tv{30, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    auto req = net::recv_packet<C2SRequestSharedState>(fd);
    if (!req) return;
    S2CSharedStateResponse resp;
    std::vector<SSEntry> to_send;
    {
        std::lock_guard l(ss_mtx_);
        if (serving_ == nullptr) {
            resp.status = SharedStateStatus::NotDistributed;
        } else {
            resp.status = SharedStateStatus::Success;
            resp.revision = serving_->revision;
            for (const auto &k : req->keys) {
                auto it = std::find_if(serving_->entries.begin(), serving_->entries.end(),
                                       [&](const SSEntry &e) { return e.key == k; });
                if (it == serving_->entries.end()) {
                    resp.status = SharedStateStatus::UnknownKey;
                    resp.entries.clear();
                    to_send.clear();
                    break;
                }
                resp.entries.push_back(SharedStateEntryInfo{k, it->bytes});
                to_send.push_back(*it);
            }
        }
    }
    if (!net::send_packet(fd, resp)) return;
    DeviceBackend *be = device_backend();
    for (const auto &e : to_send) {
        DevPtrInfo pi{};
        if (be) be->pointer_info(e.data, pi);
        if (pi.is_device) {
            be->set_device(pi.device);
            StreamLease stream(pi.device);
            DevStream st = stream.get();
            Lease a(pinned_pool(), kStagePiece), b(pinned_pool(), kStagePiece);
            uint8_t *stage[2] = {a.data(), b.data()};
            DevEvent evs[2] = {event_pool().get(), event_pool().get()};
            bool ok = a.ok() && b.ok();
            const size_t npieces = (e.bytes + kStagePiece - 1) / kStagePiece;
            auto issue = [&](size_t k) {
                const size_t off = k * kStagePiece;
                const size_t n = std::min(kStagePiece, e.bytes - off);
                be->memcpy_async(stage[k % 2], static_cast<const uint8_t *>(e.data) + off, n, st);
                be->event_record(evs[k % 2], st);
            };
            if (ok && npieces > 0) issue(0);
            for (size_t k = 0; ok && k < npieces; ++k) {
                be->event_sync(evs[k % 2]);
                if (k + 1 < npieces) issue(k + 1); // overlap next D2H with this send
                const size_t off = k * kStagePiece;
                const size_t n = std::min(kStagePiece, e.bytes - off);
                ok = net::send_all(fd, stage[k % 2], n);
                if (ok) ss_tx_bytes_ += n;
            }
            be->stream_sync(st);
            event_pool().put(evs[0]);
            event_pool().put(evs[1]);
            if (!ok) {
                LOG(WARN) << "Shared state: streaming " << e.key << " to " << sockaddr_str(peer) << " failed";
                return;
            }
        } else {
            if (!net::send_all(fd, e.data, e.bytes)) {
                LOG(WARN) << "Shared state: streaming " << e.key << " to " << sockaddr_str(peer) << " failed";
                return;
            }
            ss_tx_bytes_ += e.bytes;
        }
    }
}

} // namespace pccl::client
