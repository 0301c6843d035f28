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
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>

#include "../common/log.hpp"
#include "../common/trace.hpp"
#include "../kernels/host_kernels.hpp"
#include "../net/socket.hpp"
#include "client.hpp"
#include "ipc.hpp"
#include "pools.hpp"
#include "shareable.hpp"
#include "vmm_share.hpp"

namespace pccl::client {

using namespace proto;

static constexpr size_t kStagePiece = 32ull << 20;

// PCCL_SHARED_STATE_HASH=crc32c makes this peer announce CRC-32C content hashes (HIP kernel for HBM tensors, SSE4.2
// on the host) instead of simplehash. Every peer of a group must use the same setting: the master compares values.
static HashType announced_hash_type() {
    static const HashType t = [] {
        const char *v = std::getenv("PCCL_SHARED_STATE_HASH");
        return v && (std::strcmp(v, "crc32c") == 0 || std::strcmp(v, "crc32") == 0) ? HashType::Crc32 : HashType::Simple;
    }();
    return t;
}

bool Client::hash_entries(const std::vector<const SSEntry *> &entries, std::vector<uint64_t> &hashes, HashType &type) {
    type = announced_hash_type();
    hashes.assign(entries.size(), 0);
    DeviceBackend *be = device_backend();
    if (type != HashType::Simple || !be) {
        for (size_t i = 0; i < entries.size(); ++i)
            if (!hash_entry(*entries[i], hashes[i], type)) return false;
        return true;
    }
    struct DevBatch {
        std::unique_ptr<StreamLease> stream;
        std::vector<size_t> idx;
    };
    std::map<int, DevBatch> batches;
    std::vector<size_t> host_idx;
    std::vector<DevPtrInfo> info(entries.size());
    for (size_t i = 0; i < entries.size(); ++i) {
        be->pointer_info(entries[i]->data, info[i]);
        if (entries[i]->bytes > 0 && info[i].is_device) batches[info[i].device].idx.push_back(i);
        else host_idx.push_back(i);
    }
    Lease words(pinned_pool(), std::max<size_t>(entries.size(), 1) * sizeof(uint32_t));
    auto *out = reinterpret_cast<uint32_t *>(words.data());
    std::vector<Lease> temps; // 16-byte aligned copies of misaligned tensors (alive until the sync)
    bool ok = out != nullptr;
    for (auto &[dev, b] : batches) {
        if (!ok) break;
        be->set_device(dev);
        b.stream = std::make_unique<StreamLease>(dev);
        const DevStream st = b.stream->get();
        for (size_t i : b.idx) {
            const SSEntry &e = *entries[i];
            const void *p = e.data;
            if (reinterpret_cast<uintptr_t>(p) % 16 != 0) {
                temps.emplace_back(device_pool(), e.bytes, dev);
                be->memcpy_async(temps.back().data(), p, e.bytes, st);
                p = temps.back().data();
            }
            ok = ok && be->simplehash_async(p, e.bytes, out + i, st);
        }
    }
    for (size_t i : host_idx) // CPU entries hash while the GPUs work
        ok = ok && hash_entry(*entries[i], hashes[i], type);
    for (auto &[dev, b] : batches) {
        if (!b.stream) continue;
        be->set_device(dev);
        ok = be->stream_sync(b.stream->get()) && ok;
        for (size_t i : b.idx) hashes[i] = out[i];
    }
    return ok;
}

bool Client::hash_entry(const SSEntry &e, uint64_t &hash, HashType &type) {
    type = announced_hash_type();
    if (e.bytes == 0) {
        hash = 0;
        return true;
    }
    DeviceBackend *be = device_backend();
    DevPtrInfo pi{};
    if (be) be->pointer_info(e.data, pi);
    if (type == HashType::Crc32) {
        if (pi.is_device) {
            be->set_device(pi.device);
            StreamLease stream(pi.device);
            bool ok = true;
            hash = device_crc32c(be, e.data, e.bytes, stream.get(), &ok);
            return ok;
        }
        if (e.device == DeviceType::Gpu) {
            LOG(ERR) << "Shared state entry '" << e.key << "' declared as GPU tensor but pointer is not device memory";
            return false;
        }
        hash = kernels::crc32c(e.data, e.bytes);
        return true;
    }
    if (pi.is_device) {
        // a pooled non-blocking stream (never the null stream: that would serialise against every stream of the
        // application); the Python layer / caller has already synchronised the tensor's producer
        be->set_device(pi.device);
        StreamLease stream(pi.device);
        if (reinterpret_cast<uintptr_t>(e.data) % 16 != 0) {
            Lease tmp(device_pool(), e.bytes, pi.device);
            be->memcpy_async(tmp.data(), e.data, e.bytes, stream.get());
            hash = be->simplehash(tmp.data(), e.bytes, stream.get());
        } else {
            hash = be->simplehash(e.data, e.bytes, stream.get());
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

// `actual` was computed with announced_hash_type(); recompute if the distributor's entry uses the other type
static bool verify_hash(Client *, const SSEntry &e, uint64_t expected, HashType type, uint64_t actual,
                        HashType actual_type) {
    if (type == actual_type) return actual == expected;
    DeviceBackend *be = device_backend();
    DevPtrInfo pi{};
    if (be && e.bytes > 0) be->pointer_info(e.data, pi);
    if (type == HashType::Crc32) {
        if (pi.is_device) {
            be->set_device(pi.device);
            bool ok = true;
            const uint32_t c = device_crc32c(be, e.data, e.bytes, nullptr, &ok);
            return ok && c == expected;
        }
        return kernels::crc32c(e.data, e.bytes) == expected;
    }
    if (pi.is_device) {
        be->set_device(pi.device);
        if (reinterpret_cast<uintptr_t>(e.data) % 16 != 0) {
            Lease tmp(device_pool(), e.bytes, pi.device);
            be->memcpy_sync(tmp.data(), e.data, e.bytes);
            return be->simplehash(tmp.data(), e.bytes, nullptr) == expected;
        }
        return be->simplehash(e.data, e.bytes, nullptr) == expected;
    }
    Lease tmp(host_pool(), e.bytes);
    std::memcpy(tmp.data(), e.data, e.bytes);
    return kernels::simplehash_host(tmp.data(), e.bytes) == expected;
}

bool Client::sync_shared_state(SharedState &ss, SSInfo &info) {
    RoctxRange range("pccl sync_shared_state");
    info = SSInfo{};
    if (!accepted_ || !master_.is_open()) return false;
    if (any_collective_running()) return false;

    C2MSyncSharedState vote;
    vote.revision = ss.revision;
    vote.strategy = ss.strategy;
    std::vector<const SSEntry *> to_hash;
    for (const auto &e : ss.entries)
        if (!e.allow_content_inequality) to_hash.push_back(&e);
    std::vector<uint64_t> hashes;
    HashType htype = HashType::Simple;
    if (!hash_entries(to_hash, hashes, htype)) return false;
    size_t hi = 0;
    for (const auto &e : ss.entries) {
        SharedStateHashEntry he;
        he.key = e.key;
        he.data_type = e.dtype;
        he.num_elements = e.count;
        he.allow_content_inequality = e.allow_content_inequality;
        if (!e.allow_content_inequality) {
            he.hash = hashes[hi++];
            he.hash_type = htype;
        }
        vote.entries.push_back(he);
    }

    struct PhaseGuard {
        Client *c;
        PhaseGuard(Client *cl, SharedState *s) : c(cl) {
            std::lock_guard l(c->ss_mtx_);
            c->serving_ = s;
        }
        bool released = false;
        ~PhaseGuard() { release(); }
        void release() {
            if (released) return;
            released = true;
            std::unique_lock l(c->ss_mtx_);
            c->serving_ = nullptr;
            // a requester reports completion once it holds the bytes, possibly before our sender thread returned
            // from its last send: wait for the serves so the caller may modify its tensors and tx_bytes is final
            if (!c->ss_cv_.wait_for(l, std::chrono::seconds(30), [&] { return c->ss_active_serves_ == 0; })) {
                LOG(WARN) << "Shared state sync: a serve to a peer is still running after 30 s";
            }
        }
    } guard(this, &ss); // serve requests from the moment we vote (peers may be faster than our master packet)

    if (!master_.send(vote)) return false;
    auto resp = master_.receive<M2CSyncSharedState>();
    if (!resp) {
        LOG(ERR) << "Shared state sync: no response from master (kicked?)";
        return false;
    }
    std::map<std::string, SSEntry *> by_key;
    for (auto &e : ss.entries) by_key[e.key] = &e;
    DeviceBackend *be = device_backend();

    // receives one entry streamed as raw bytes (HBM destinations through a double-buffered pinned staging ring)
    auto recv_stream_entry = [&](int fd, SSEntry &dst) -> bool {
        DevPtrInfo pi{};
        if (be) be->pointer_info(dst.data, pi);
        if (!pi.is_device) return net::recv_all(fd, dst.data, dst.bytes);
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
        return ok;
    };
    auto lookup = [&](size_t i, const std::string &key, uint64_t size) -> SSEntry * {
        auto it = by_key.find(key);
        if (it == by_key.end() || i >= resp->outdated_keys.size() || key != resp->outdated_keys[i]) {
            LOG(ERR) << "Shared state sync: unexpected key " << key;
            return nullptr;
        }
        if (size != it->second->bytes) {
            LOG(ERR) << "Shared state sync: size mismatch for " << key;
            return nullptr;
        }
        return it->second;
    };
    auto verify = [&](size_t i, SSEntry &dst) -> bool {
        if (dst.allow_content_inequality || i >= resp->expected_hashes.size()) return true;
        uint64_t h = 0;
        HashType t;
        if (!hash_entry(dst, h, t)) return false;
        if (!verify_hash(this, dst, resp->expected_hashes[i], resp->expected_hash_types[i], h, t)) {
            LOG(ERR) << "Shared state sync: distributor sent corrupt content for " << dst.key;
            return false;
        }
        return true;
    };
    struct FdGuard {
        int fd;
        ~FdGuard() { ::close(fd); }
    };

    // Same-host distributor: HBM entries are handed over as HIP IPC handles and copied device-to-device (over xGMI
    // between GPUs) instead of D2H -> TCP -> H2D. `fallback` is set if the distributor does not speak the extension.
    // A distributor that stops without closing its socket (SIGSTOP, a wedged host) keeps the connection alive: its
    // kernel still ACKs, so neither keepalive nor TCP_USER_TIMEOUT ends a receive from it. A fetch receive that gets
    // no byte for the op-stall timeout (PCCL_OP_STALL_MS) fails instead, and the next distributor is tried.
    auto stall_guard = [this](int fd) {
        if (stall_ms_ == 0) return;
        timeval tv{static_cast<time_t>(stall_ms_ / 1000), static_cast<suseconds_t>(stall_ms_ % 1000) * 1000};
        setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    };
    auto fetch_ipc = [&](const SockAddr &distributor, bool &fallback) -> bool {
        fallback = false;
        const int fd = net::connect_tcp(distributor, 10000);
        if (fd < 0) return false;
        FdGuard fdg{fd};
        stall_guard(fd);
        C2SRequestSharedStateIpc req;
        req.keys = resp->outdated_keys;
        req.host_token = net::host_token();
        req.pid = static_cast<uint32_t>(getpid());
        if (!net::send_packet(fd, req)) return false;
        auto pkt = net::recv_ltv(fd);
        if (!pkt || pkt->id != S2CSharedStateIpcResponse::kId) {
            fallback = true;
            return false;
        }
        auto sresp = decode_payload<S2CSharedStateIpcResponse>(pkt->payload.data(), pkt->payload.size());
        if (!sresp || sresp->status != SharedStateStatus::Success ||
            sresp->entries.size() != resp->outdated_keys.size()) {
            LOG(WARN) << "Shared state sync: distributor refused the IPC request";
            return false;
        }
        ss.revision = sresp->revision;
        bool ok = true;
        const bool same_process = sresp->pid == static_cast<uint32_t>(getpid());
        // phase 1: map the source of every handed-over entry (VMM imports hold their own reference to the pages, so
        // from here on the distributor may die without invalidating them)
        struct Mapped {
            void *ptr;
            bool vmm;
            int device;
        };
        std::vector<Mapped> mapped;
        struct Unmap { // every exit path releases the mappings
            DeviceBackend *be;
            std::vector<Mapped> &m;
            ~Unmap() {
                for (const auto &x : m) {
                    be->set_device(x.device);
                    if (x.vmm) be->vmm_unmap(x.ptr);
                    else be->ipc_close(x.ptr);
                }
            }
        } unmap{be, mapped};
        std::map<std::pair<std::array<uint8_t, 64>, int>, void *> imported; // (handle, device) -> mapping
        std::vector<std::vector<const uint8_t *>> srcs(sresp->entries.size());
        std::vector<int> devs(sresp->entries.size(), 0);
        for (size_t i = 0; ok && i < sresp->entries.size(); ++i) {
            const auto &se = sresp->entries[i];
            if (se.mode == 0) continue;
            SSEntry *dst = lookup(i, se.key, se.size_bytes);
            if (!dst) {
                ok = false;
                break;
            }
            if (!be) {
                LOG(ERR) << "Shared state sync: IPC entry " << se.key << " but no HIP backend";
                ok = false;
                break;
            }
            DevPtrInfo pi{};
            be->pointer_info(dst->data, pi);
            const int dev = devs[i] = pi.is_device ? pi.device : std::max(0, se.device);
            be->set_device(dev);
            if (same_process) {
                srcs[i].push_back(reinterpret_cast<const uint8_t *>(se.raw_ptr)); // plain pointer
            } else if (se.mode == 1) {
                void *m = be->ipc_open(se.handle);
                if (m) {
                    mapped.push_back({m, false, dev});
                    srcs[i].push_back(static_cast<const uint8_t *>(m) + se.offset);
                }
            } else {
                std::vector<const uint8_t *> hs{se.handle};
                for (const auto &h : se.more_handles) hs.push_back(h.data());
                for (size_t j = 0; j < hs.size(); ++j) {
                    // packed entries share segments: import each one once per fetch (an import reserves VA space
                    // for the whole allocation, and VMM ranges are never freed, hip_backend.hip)
                    std::array<uint8_t, 64> hk;
                    std::memcpy(hk.data(), hs[j], hk.size());
                    void *m = nullptr;
                    auto hit = imported.find({hk, dev});
                    if (hit != imported.end()) {
                        m = hit->second;
                    } else {
                        VmmHandle vh;
                        int vfd = -1;
                        if (VmmHandle::decode(hs[j], vh) && (vfd = VmmShare::fetch(vh.pid, vh.nonce, vh.id)) >= 0) {
                            m = be->vmm_import(vfd, vh.size, dev);
                            ::close(vfd);
                        }
                        if (m) {
                            mapped.push_back({m, true, dev});
                            imported[{hk, dev}] = m;
                        }
                    }
                    if (!m) {
                        srcs[i].clear();
                        break;
                    }
                    srcs[i].push_back(static_cast<const uint8_t *>(m) + (j == 0 ? se.offset : 0));
                }
            }
            if (srcs[i].empty()) {
                LOG(ERR) << "Shared state sync: cannot map the distributor's copy of " << se.key;
                ok = false;
            }
        }
        if (const size_t ms = env_size("PCCL_SS_COPY_DELAY_MS", 0)) // tests: let the distributor die in between
            std::this_thread::sleep_for(std::chrono::milliseconds(ms));
        // phase 2: copy / receive every entry in order, hash-verify it
        for (size_t i = 0; ok && i < sresp->entries.size(); ++i) {
            const auto &se = sresp->entries[i];
            SSEntry *dst = lookup(i, se.key, se.size_bytes);
            if (!dst) {
                ok = false;
                break;
            }
            if (se.mode != 0) {
                be->set_device(devs[i]);
                const size_t nseg = se.seg_bytes ? (dst->bytes + se.seg_bytes - 1) / se.seg_bytes : 0;
                if (se.mode == 1 || same_process) {
                    ok = be->memcpy_sync(dst->data, srcs[i][0], dst->bytes);
                } else if (nseg == 0 || nseg > srcs[i].size()) {
                    LOG(ERR) << "Shared state sync: malformed segment list for " << se.key;
                    ok = false;
                } else { // VMM imports: copy kernel (no copy-engine path for imported VMM memory)
                    StreamLease stream(devs[i]);
                    ok = stream.get() != nullptr;
                    for (size_t j = 0, off = 0; ok && off < dst->bytes; ++j, off += se.seg_bytes) {
                        const size_t n = std::min<size_t>(se.seg_bytes, dst->bytes - off);
                        const void *src = srcs[i][j];
                        const size_t zero = 0;
                        ok = be->multi_gather(static_cast<uint8_t *>(dst->data) + off, &src, &zero, &n, 1, -1, DType::U8,
                                              stream.get());
                    }
                    ok = ok && be->stream_sync(stream.get());
                }
                if (!ok) {
                    LOG(ERR) << "Shared state sync: IPC copy of " << se.key << " failed";
                }
            } else {
                ok = recv_stream_entry(fd, *dst);
                if (!ok) {
                    LOG(ERR) << "Shared state sync: transfer of " << se.key << " failed";
                }
            }
            if (ok) {
                info.rx_bytes += dst->bytes;
                ok = verify(i, *dst);
            }
        }
        net::send_packet(fd, C2SSharedStateIpcDone{ok});
        return ok;
    };

    // Fetches the outdated entries from one distributor; false if it failed or died mid-transfer (partially written
    // entries are overwritten by the next attempt, and every entry is hash-verified at the end).
    auto fetch_from = [&](const SockAddr &distributor) -> bool {
        // PCCL_SS_IPC_PROTOCOL=1 forces the extension even without a GPU (tests: every entry is then streamed)
        const bool try_ipc = (be || env_flag("PCCL_SS_IPC_PROTOCOL", false)) && !env_flag("PCCL_SS_NO_IPC", false) &&
                             !wire_reference_;
        if (try_ipc && net::is_local_address(distributor)) {
            bool fallback = false;
            if (fetch_ipc(distributor, fallback)) return true;
            if (!fallback) return false;
            info.rx_bytes = 0;
        }
        // The outdated keys are requested over up to PCCL_SS_STREAMS (default 4) connections at once, each an ordinary
        // request for a subset of the keys (balanced by size), so a reference distributor serves them as well; one
        // TCP stream carries ~9 GB/s over loopback and far less over a long path, where parallel streams add up.
        const size_t nkeys = resp->outdated_keys.size();
        const size_t streams = wire_reference_ ? 1 : std::max<size_t>(1, std::min(env_size("PCCL_SS_STREAMS", 4), nkeys));
        std::vector<std::vector<size_t>> bins(streams);
        {
            std::vector<size_t> order(nkeys);
            for (size_t i = 0; i < nkeys; ++i) order[i] = i;
            auto bytes_of = [&](size_t i) -> uint64_t {
                auto it = by_key.find(resp->outdated_keys[i]);
                return it == by_key.end() ? 0 : it->second->bytes;
            };
            std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return bytes_of(a) > bytes_of(b); });
            std::vector<uint64_t> load(streams, 0);
            for (size_t i : order) {
                const size_t k = static_cast<size_t>(std::min_element(load.begin(), load.end()) - load.begin());
                bins[k].push_back(i);
                load[k] += bytes_of(i);
            }
            for (auto &b : bins) std::sort(b.begin(), b.end());
        }
        std::atomic<uint64_t> rx{0}, revision{0};
        // the first stream that fails ends the others at once (shut down their sockets): the next distributor is
        // tried as soon as one stream of this one failed, not after every other stream's own timeouts
        std::mutex fds_m;
        std::vector<int> fds;
        std::atomic<bool> failed{false};
        auto fail_all = [&] {
            failed.store(true);
            std::lock_guard l(fds_m);
            for (int f : fds) ::shutdown(f, SHUT_RDWR);
        };
        // one connection: the keys of `idx` (indices into the master's outdated-key list), received in that order
        // (no key at all: the request still runs, its response carries the revision)
        auto fetch_keys = [&](const std::vector<size_t> &idx) -> bool {
            if (failed.load()) return false;
            const int fd = net::connect_tcp(distributor, 10000);
            if (fd < 0) {
                LOG(WARN) << "Shared state sync: cannot reach distributor " << sockaddr_str(distributor);
                return false;
            }
            FdGuard fdg{fd};
            stall_guard(fd);
            {
                std::lock_guard l(fds_m);
                if (failed.load()) return false;
                fds.push_back(fd);
            }
            struct Unlist {
                std::mutex &m;
                std::vector<int> &v;
                int fd;
                ~Unlist() {
                    std::lock_guard l(m);
                    v.erase(std::remove(v.begin(), v.end(), fd), v.end());
                }
            } unlist{fds_m, fds, fd};
            C2SRequestSharedState req;
            for (size_t i : idx) req.keys.push_back(resp->outdated_keys[i]);
            if (!net::send_packet(fd, req)) return false;
            auto sresp = net::recv_packet<S2CSharedStateResponse>(fd);
            if (!sresp || sresp->status != SharedStateStatus::Success) {
                LOG(WARN) << "Shared state sync: distributor refused (status "
                          << (sresp ? static_cast<int>(sresp->status) : -1) << ")";
                return false;
            }
            revision.store(sresp->revision);
            if (sresp->entries.size() != idx.size()) return false;
            for (size_t j = 0; j < idx.size(); ++j) {
                const auto &se = sresp->entries[j];
                SSEntry *dst = lookup(idx[j], se.key, se.size_bytes);
                if (!dst) return false;
                if (!recv_stream_entry(fd, *dst)) {
                    LOG(ERR) << "Shared state sync: transfer of " << se.key << " failed";
                    return false;
                }
                rx += dst->bytes;
            }
            return true;
        };
        std::vector<char> ok(streams, 0);
        std::vector<std::thread> ts;
        auto run = [&](size_t k) {
            ok[k] = fetch_keys(bins[k]);
            if (!ok[k]) fail_all();
        };
        for (size_t k = 1; k < streams; ++k) ts.emplace_back(run, k);
        run(0);
        for (auto &t : ts) t.join();
        info.rx_bytes += rx.load();
        if (std::find(ok.begin(), ok.end(), 0) != ok.end()) return false;
        ss.revision = revision.load();
        // hashes verified once every stream is done (one thread: the hash kernels share their scratch)
        for (size_t i = 0; i < nkeys; ++i) {
            auto it = by_key.find(resp->outdated_keys[i]);
            if (it == by_key.end() || !verify(i, *it->second)) return false;
        }
        return true;
    };
    bool fetched = !resp->is_outdated;
    if (resp->is_outdated) {
        std::vector<SockAddr> sources;
        if (!sockaddr_is_zero(resp->distributor)) sources.push_back(resp->distributor);
        for (const auto &f : resp->fallback_distributors) sources.push_back(f);
        if (sources.empty()) {
            LOG(ERR) << "Shared state sync: master assigned no distributor";
        }
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
    guard.release();
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
    auto pkt = net::recv_ltv(fd);
    if (!pkt) return;
    std::vector<std::string> keys;
    bool ipc_request = false, same_host = false;
    uint32_t ipc_pid = 0;
    if (pkt->id == C2SRequestSharedState::kId) {
        auto req = decode_payload<C2SRequestSharedState>(pkt->payload.data(), pkt->payload.size());
        if (!req) return;
        keys = std::move(req->keys);
    } else if (pkt->id == C2SRequestSharedStateIpc::kId && !wire_reference_) { // (a reference peer: unknown packet)
        auto req = decode_payload<C2SRequestSharedStateIpc>(pkt->payload.data(), pkt->payload.size());
        if (!req) return;
        keys = std::move(req->keys);
        ipc_request = true;
        same_host = req->host_token == net::host_token();
        ipc_pid = req->pid;
    } else {
        return;
    }
    SharedStateStatus status = SharedStateStatus::Success;
    uint64_t revision = 0;
    std::vector<SSEntry> to_send;
    // the sync that owns serving_ waits for this serve (its tensors stay untouched and its tx count is final)
    bool counted = false;
    struct ServeGuard {
        Client *c;
        bool &counted;
        ~ServeGuard() {
            if (!counted) return;
            std::lock_guard l(c->ss_mtx_);
            --c->ss_active_serves_;
            c->ss_cv_.notify_all();
        }
    } serve_guard{this, counted};
    {
        std::lock_guard l(ss_mtx_);
        if (serving_ == nullptr) {
            status = SharedStateStatus::NotDistributed;
        } else {
            ++ss_active_serves_;
            counted = true;
            revision = serving_->revision;
            for (const auto &k : keys) {
                auto it = std::find_if(serving_->entries.begin(), serving_->entries.end(),
                                       [&](const SSEntry &e) { return e.key == k; });
                if (it == serving_->entries.end()) {
                    status = SharedStateStatus::UnknownKey;
                    to_send.clear();
                    break;
                }
                to_send.push_back(*it);
            }
        }
    }
    DeviceBackend *be = device_backend();
    auto stream_entry = [&](const SSEntry &e) -> bool {
        DevPtrInfo pi{};
        if (be) be->pointer_info(e.data, pi);
        if (!pi.is_device) return net::send_all(fd, e.data, e.bytes);
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
        }
        be->stream_sync(st);
        event_pool().put(evs[0]);
        event_pool().put(evs[1]);
        return ok;
    };

    if (!ipc_request) {
        S2CSharedStateResponse resp;
        resp.status = status;
        resp.revision = revision;
        for (const auto &e : to_send) resp.entries.push_back(SharedStateEntryInfo{e.key, e.bytes});
        if (!net::send_packet(fd, resp)) return;
        fault_point("ss_serve", revision); // tests: fail after the response, before the entries
        for (const auto &e : to_send) {
            if (!stream_entry(e)) {
                LOG(WARN) << "Shared state: streaming " << e.key << " to " << sockaddr_str(peer) << " failed";
                return;
            }
            ss_tx_bytes_ += e.bytes;
        }
        return;
    }

    // IPC request: hand HBM entries over (same host only), stream the rest, keep what was handed over valid until
    // the requester reports that its copies are done. Fault-safe (PCCL_IPC_MODE=safe, default): only VMM fd shares
    // cross the process boundary — the entry's own allocation if it lies in shareable memory, else a staged copy in
    // kIpcSegBytes VMM segments — so a distributor that dies mid-copy leaves valid memory behind. "fast": hipIpc
    // export of the entry's allocation (no staging copy, but the requester's copy faults if we die under it).
    S2CSharedStateIpcResponse resp;
    resp.status = status;
    resp.revision = revision;
    resp.pid = static_cast<uint32_t>(getpid());
    uint64_t ipc_bytes = 0;
    std::vector<void *> staged; // VMM staging segments of this request
    struct StagedGuard {
        std::vector<void *> &v;
        ~StagedGuard() {
            for (void *p : v) shareable::free(p);
        }
    } staged_guard{staged};
    const bool same_process = ipc_pid == static_cast<uint32_t>(getpid());
    // Staging (safe mode, entries not in shareable memory): entries up to kPackMax are packed back to back into
    // shared VMM segments (one allocation / fd / import per segment instead of per tensor: a model's state has
    // hundreds of small tensors); larger ones get their own kIpcSegBytes segments. Copies run on one stream per
    // device and are synchronised once, before the response goes out.
    constexpr size_t kPackMax = 64u << 20, kPackAlign = 256;
    struct PackSeg {
        uint8_t *seg = nullptr;
        size_t cap = 0, used = 0;
        std::array<uint8_t, 64> h{};
    };
    std::map<int, PackSeg> pack;           // open pack segment per device
    std::map<int, size_t> small_left;      // bytes of small staged entries still to place, per device
    std::map<int, std::unique_ptr<StreamLease>> streams;
    auto stream_for = [&](int dev) -> DevStream {
        auto &sl = streams[dev];
        if (!sl) sl = std::make_unique<StreamLease>(dev);
        return sl->get();
    };
    auto new_seg = [&](size_t n, int dev, std::array<uint8_t, 64> &h) -> uint8_t * {
        void *seg = shareable::alloc(n, dev);
        shareable::Share sh;
        if (!seg || !shareable::lookup(seg, n, sh)) {
            if (seg) shareable::free(seg);
            return nullptr;
        }
        staged.push_back(seg);
        h.fill(0);
        std::memcpy(h.data(), &sh.handle, sizeof(sh.handle));
        return static_cast<uint8_t *>(seg);
    };
    auto copy_into = [&](uint8_t *dst, const uint8_t *src, size_t n, int dev) {
        const void *s = src;
        const size_t zero = 0;
        const DevStream st = stream_for(dev);
        return st && be->multi_gather(dst, &s, &zero, &n, 1, -1, DType::U8, st);
    };
    auto stage = [&](const SSEntry &e, SharedStateIpcEntry &ie, int dev) -> bool {
        const auto *src = static_cast<const uint8_t *>(e.data);
        if (e.bytes <= kPackMax) {
            PackSeg &p = pack[dev];
            size_t off = (p.used + kPackAlign - 1) / kPackAlign * kPackAlign;
            if (!p.seg || off + e.bytes > p.cap) {
                p = PackSeg{};
                p.cap = std::max(e.bytes, std::min(small_left[dev], kIpcSegBytes));
                if (!(p.seg = new_seg(p.cap, dev, p.h))) return false;
                off = 0;
            }
            if (!copy_into(p.seg + off, src, e.bytes, dev)) return false;
            p.used = off + e.bytes;
            small_left[dev] -= std::min(small_left[dev], (e.bytes + kPackAlign - 1) / kPackAlign * kPackAlign);
            ie.mode = 2;
            std::memcpy(ie.handle, p.h.data(), p.h.size());
            ie.offset = off;
            ie.seg_bytes = e.bytes;
            return true;
        }
        std::vector<std::array<uint8_t, 64>> hs;
        for (size_t off = 0; off < e.bytes; off += kIpcSegBytes) {
            const size_t n = std::min(kIpcSegBytes, e.bytes - off);
            std::array<uint8_t, 64> h{};
            uint8_t *seg = new_seg(n, dev, h);
            if (!seg || !copy_into(seg, src + off, n, dev)) return false;
            hs.push_back(h);
        }
        ie.mode = 2;
        std::memcpy(ie.handle, hs[0].data(), hs[0].size());
        ie.more_handles.assign(hs.begin() + 1, hs.end());
        ie.seg_bytes = kIpcSegBytes;
        ie.offset = 0;
        return true;
    };
    if (!same_process && ipc_safe_mode() && be && same_host) // pass 1: how much will be packed, per device
        for (const auto &e : to_send) {
            DevPtrInfo pi{};
            shareable::Share sh;
            if (e.bytes == 0 || e.bytes > kPackMax) continue;
            be->pointer_info(e.data, pi);
            if (pi.is_device && !(shareable::lookup(e.data, e.bytes, sh) && sh.size <= kIpcMaxExport))
                small_left[pi.device] += (e.bytes + kPackAlign - 1) / kPackAlign * kPackAlign;
        }
    for (const auto &e : to_send) {
        SharedStateIpcEntry ie;
        ie.key = e.key;
        ie.size_bytes = e.bytes;
        DevPtrInfo pi{};
        if (be && same_host && e.bytes > 0) be->pointer_info(e.data, pi);
        if (!pi.is_device) {
            resp.entries.push_back(ie);
            continue;
        }
        be->set_device(pi.device);
        shareable::Share sh;
        void *base = nullptr;
        size_t size = 0;
        if (same_process) {
            ie.mode = 1; // the requester reads through raw_ptr
        } else if (shareable::lookup(e.data, e.bytes, sh) && sh.size <= kIpcMaxExport) {
            ie.mode = 2; // zero-copy and fault-safe: the tensor itself is fd-shareable
            std::memcpy(ie.handle, &sh.handle, sizeof(sh.handle));
            ie.offset = sh.offset;
            ie.seg_bytes = e.bytes;
        } else if (ipc_safe_mode()) {
            if (!stage(e, ie, pi.device)) {
                LOG(WARN) << "Shared state: staging " << e.key << " for the IPC hand-off failed; streaming it";
            }
        } else if (be->address_range(e.data, &base, &size) && base && be->ipc_export(base, ie.handle)) {
            ie.mode = 1;
            ie.offset = static_cast<uint64_t>(static_cast<const uint8_t *>(e.data) - static_cast<uint8_t *>(base));
        }
        if (ie.mode != 0) {
            ie.device = pi.device;
            ie.raw_ptr = reinterpret_cast<uint64_t>(e.data);
            ipc_bytes += e.bytes;
        }
        resp.entries.push_back(ie);
    }
    for (auto &[dev, sl] : streams) { // staged copies complete before anyone is told where they are
        be->set_device(dev);
        if (!sl->get() || !be->stream_sync(sl->get())) {
            LOG(ERR) << "Shared state: staging copies for the IPC hand-off failed";
            resp.status = SharedStateStatus::NotDistributed;
            resp.entries.clear();
            break;
        }
    }
    if (!net::send_packet(fd, resp)) return;
    fault_point("ss_serve", revision); // tests: die while the requester maps / copies what was handed over
    for (size_t i = 0; i < to_send.size(); ++i) {
        if (resp.entries[i].mode != 0) continue;
        if (!stream_entry(to_send[i])) {
            LOG(WARN) << "Shared state: streaming " << to_send[i].key << " to " << sockaddr_str(peer) << " failed";
            return;
        }
        ss_tx_bytes_ += to_send[i].bytes;
    }
    if (status != SharedStateStatus::Success) return;
    timeval tv_done{600, 0}; // the requester copies (and re-hashes) every entry before it answers
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv_done, sizeof(tv_done));
    auto done = net::recv_packet<C2SSharedStateIpcDone>(fd);
    if (done && done->ok) ss_tx_bytes_ += ipc_bytes;
}

} // namespace pccl::client
