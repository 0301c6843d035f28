#include "ipc.hpp"

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <thread>
#include <tuple>

#include "../common/log.hpp"
#include "client.hpp"
#include "pools.hpp"
#include "../common/trace.hpp"

namespace pccl::client {

using namespace std::chrono;

namespace {
constexpr uint64_t kMagic = 0x5043434c49504331ull; // "PCCLIPC1"
constexpr uint32_t kClosed = 0x80000000u;
constexpr uint32_t kSlots = 256;
constexpr uint32_t kMaxWorld = 16;

constexpr uint32_t PH_VOTED = 1, PH_REDUCED = 3, PH_GATHERED = 4, PH_RELEASED = 5, PH_ABORTED = 0xEE;

uint64_t fnv1a(const void *p, size_t n, uint64_t h = 1469598103934665603ull) {
    const auto *b = static_cast<const uint8_t *>(p);
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

inline void cpu_relax() { __builtin_ia32_pause(); }
} // namespace

struct alignas(64) PeerSlotShm {
    std::atomic<uint32_t> present;
    int32_t pid;
    uint32_t can_ipc;
    uint8_t uuid[16];
};

// Per (op slot, peer) record. Every peer publishes where its op *input* (read by the reduce-scatter) and *output*
// (written by its own reduce, read by the all-gather) live:
//   zero-copy (out-of-place device buffers): input = the caller's send buffer, output = the caller's receive buffer
//   staged (in-place or export failure):     input / output = the two halves of a pooled, exported comm buffer
// Peers may mix the two modes. *_raw are usable directly by peers in the same process (threaded peers).
struct alignas(64) OpPeerShm {
    std::atomic<uint64_t> phase; // (seq + 1) << 8 | phase
    uint32_t vote;
    int32_t device;
    uint64_t bytes;
    uint32_t dtype;
    uint32_t op;
    uint32_t zero_copy; // bit 0: input is the caller's send buffer, bit 1: output is the caller's receive buffer
    uint32_t pad;
    uint64_t gpu_uid;   // physical GPU of this op's buffers (peers sharing a GPU split its CUs)
    uint64_t in_raw, out_raw;
    uint64_t in_off, out_off;
    uint8_t in_handle[kIpcHandleBytes];
    uint8_t out_handle[kIpcHandleBytes];
};

struct ArenaShm {
    std::atomic<uint64_t> magic;
    std::atomic<uint32_t> join;
    std::atomic<uint32_t> unlinked;
    uint32_t world;
    uint32_t pad[11];
    PeerSlotShm *peers() { return reinterpret_cast<PeerSlotShm *>(reinterpret_cast<uint8_t *>(this) + 64); }
    OpPeerShm *op(uint32_t slot, uint32_t peer) {
        auto *base = reinterpret_cast<uint8_t *>(this) + 64 + sizeof(PeerSlotShm) * kMaxWorld;
        return reinterpret_cast<OpPeerShm *>(base) + slot * kMaxWorld + peer;
    }
    static size_t bytes() { return 64 + sizeof(PeerSlotShm) * kMaxWorld + sizeof(OpPeerShm) * kSlots * kMaxWorld; }
};

struct OpCtx {
    void *comm = nullptr;          // pooled comm buffer (input half | output half) if either side is staged
    bool in_staged = false;        // peers read my input from the comm buffer's input half (copied in before the vote)
    bool out_staged = false;       // peers write / gather my output into the comm buffer's output half (copied out)
    uint8_t *my_out = nullptr;     // my output: the caller's receive buffer or the comm output half
    std::vector<const uint8_t *> peer_in;
    std::vector<uint8_t *> peer_out;
    size_t bytes = 0;
};

// per-process bookkeeping
static std::mutex g_ctx_mtx;
static std::map<std::pair<const IpcArena *, uint64_t>, OpCtx> g_ctx;
static std::mutex g_attempt_mtx;
static std::map<uint64_t, int> g_attempts;

std::shared_ptr<IpcArena> IpcArena::create(Client &c, const std::vector<Uuid> &ring, uint16_t master_port,
                                           uint32_t group) {
    const size_t W = ring.size();
    if (W < 2 || W > kMaxWorld) return nullptr;
    auto it = std::find(ring.begin(), ring.end(), c.uuid());
    if (it == ring.end()) return nullptr;
    const size_t rank = static_cast<size_t>(it - ring.begin());

    uint64_t h = fnv1a(&group, sizeof(group));
    h = fnv1a(&master_port, sizeof(master_port), h);
    for (const auto &u : ring) h = fnv1a(u.data.data(), 16, h);
    int attempt;
    {
        std::lock_guard l(g_attempt_mtx);
        // counted per (ring, peer) so that threaded peers sharing a process agree on the attempt number
        attempt = g_attempts[fnv1a(c.uuid().data.data(), 16, h)]++;
    }
    char nbuf[96];
    std::snprintf(nbuf, sizeof(nbuf), "/pccl_arena_%016llx_%d", static_cast<unsigned long long>(h), attempt);
    const std::string name(nbuf);
    const size_t bytes = ArenaShm::bytes();
    const int timeout_ms = static_cast<int>(env_size("PCCL_IPC_RENDEZVOUS_MS", 15000));
    const auto t0 = steady_clock::now();
    auto elapsed_ms = [&] { return duration_cast<milliseconds>(steady_clock::now() - t0).count(); };

    int fd = -1;
    if (rank == 0) {
        shm_unlink(name.c_str());
        fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
            LOG(WARN) << "IPC arena: cannot create " << name << ": " << std::strerror(errno);
            if (fd >= 0) close(fd);
            return nullptr;
        }
    } else {
        while (true) {
            fd = shm_open(name.c_str(), O_RDWR, 0600);
            if (fd >= 0) {
                struct stat st{};
                if (fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) >= bytes) break;
                close(fd);
                fd = -1;
            }
            if (elapsed_ms() > timeout_ms) {
                LOG(WARN) << "IPC arena: rendezvous " << name << " timed out (peers not on this host?)";
                return nullptr;
            }
            std::this_thread::sleep_for(milliseconds(1));
        }
    }
    void *mem = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (mem == MAP_FAILED) return nullptr;
    auto *shm = static_cast<ArenaShm *>(mem);
    if (rank == 0) {
        shm->world = static_cast<uint32_t>(W);
        shm->magic.store(kMagic, std::memory_order_release);
    } else {
        while (shm->magic.load(std::memory_order_acquire) != kMagic) {
            if (elapsed_ms() > timeout_ms) {
                munmap(mem, bytes);
                return nullptr;
            }
            std::this_thread::sleep_for(milliseconds(1));
        }
    }
    PeerSlotShm &me = shm->peers()[rank];
    me.pid = static_cast<int32_t>(getpid());
    me.can_ipc = device_backend_available() ? 1 : 0;
    std::memcpy(me.uuid, c.uuid().data.data(), 16);
    me.present.store(1, std::memory_order_release);
    // join unless the rendezvous was closed by a peer that gave up
    uint32_t v = shm->join.load();
    bool joined = false;
    while (!(v & kClosed)) {
        if (shm->join.compare_exchange_weak(v, v + 1)) {
            joined = true;
            break;
        }
    }
    bool ok = false;
    if (joined) {
        while (true) {
            v = shm->join.load(std::memory_order_acquire);
            if ((v & ~kClosed) == W) {
                ok = true;
                break;
            }
            if (v & kClosed) break;
            if (elapsed_ms() > timeout_ms) {
                uint32_t expect = v;
                if (shm->join.compare_exchange_strong(expect, v | kClosed)) break;
                continue; // the last peer joined concurrently: re-read
            }
            std::this_thread::sleep_for(milliseconds(1));
        }
    }
    if (ok) {
        if (shm->unlinked.fetch_add(1) + 1 == W) shm_unlink(name.c_str());
        for (size_t k = 0; k < W; ++k)
            if (!shm->peers()[k].can_ipc) ok = false; // consistent: every peer reads the same slots
    } else {
        shm_unlink(name.c_str());
    }
    if (!ok) {
        munmap(mem, bytes);
        LOG(INFO) << "IPC arena not used for this ring";
        return nullptr;
    }
    auto arena = std::shared_ptr<IpcArena>(new IpcArena());
    arena->ring_ = ring;
    arena->rank_ = rank;
    arena->name_ = name;
    arena->shm_ = shm;
    arena->shm_bytes_ = bytes;
    for (size_t k = 0; k < W; ++k) arena->pids_.push_back(shm->peers()[k].pid);
    LOG(INFO) << "IPC arena established (" << W << " peers on this host, rank " << rank << ")";
    return arena;
}

IpcArena::~IpcArena() {
    DeviceBackend *be = device_backend();
    if (be) {
        const int cur = be->current_device();
        for (auto &[key, p] : mappings_) {
            be->set_device(std::get<2>(key));
            be->ipc_close(p);
        }
        for (auto &b : bufs_) {
            be->set_device(b->device);
            be->free_device(b->ptr);
        }
        if (cur >= 0) be->set_device(cur);
    }
    if (shm_) munmap(shm_, shm_bytes_);
}

IpcArena::CommBuf *IpcArena::acquire_buffer(size_t bytes, int device) {
    std::lock_guard l(mtx_);
    CommBuf *best = nullptr;
    for (auto &b : bufs_)
        if (!b->busy && b->device == device && b->cap >= bytes && (!best || b->cap < best->cap)) best = b.get();
    if (best) {
        best->busy = true;
        return best;
    }
    DeviceBackend *be = device_backend();
    auto b = std::make_unique<CommBuf>();
    b->cap = std::max<size_t>(bytes, 1 << 20);
    b->device = device;
    be->set_device(device);
    b->ptr = be->alloc_device(b->cap);
    if (!b->ptr || !be->ipc_export(b->ptr, b->handle)) {
        if (b->ptr) be->free_device(b->ptr);
        LOG(ERR) << "IPC arena: failed to allocate/export " << b->cap << " bytes";
        return nullptr;
    }
    b->id = next_buf_id_++;
    b->busy = true;
    bufs_.push_back(std::move(b));
    return bufs_.back().get();
}

void IpcArena::release_buffer(CommBuf *b) {
    if (!b) return;
    std::lock_guard l(mtx_);
    b->busy = false;
}

void *IpcArena::peer_mapping(int peer, const uint8_t *handle, int my_device) {
    std::lock_guard l(mtx_);
    std::array<uint8_t, kIpcHandleBytes> hb;
    std::memcpy(hb.data(), handle, kIpcHandleBytes);
    const auto key = std::make_tuple(peer, hb, my_device);
    auto it = mappings_.find(key);
    if (it != mappings_.end()) {
        auto pos = std::find(mapping_lru_.begin(), mapping_lru_.end(), key); // touch (most recently used last)
        if (pos != mapping_lru_.end() && pos + 1 != mapping_lru_.end()) {
            mapping_lru_.erase(pos);
            mapping_lru_.push_back(key);
        }
        return it->second;
    }
    DeviceBackend *be = device_backend();
    be->set_device(my_device);
    void *p = be->ipc_open(handle);
    if (!p) return nullptr;
    mappings_[key] = p;
    mapping_lru_.push_back(key);
    // bound the number of open mappings (user allocations come and go); never evict entries of in-flight ops:
    // those were (re)inserted at the back by this call or by the vote of the op that uses them
    constexpr size_t kMaxMappings = 256;
    while (mapping_lru_.size() > kMaxMappings) {
        auto old = mapping_lru_.front();
        mapping_lru_.erase(mapping_lru_.begin());
        auto mit = mappings_.find(old);
        if (mit != mappings_.end()) {
            be->set_device(std::get<2>(old));
            be->ipc_close(mit->second);
            mappings_.erase(mit);
        }
    }
    be->set_device(my_device);
    return p;
}

bool IpcArena::export_user(void *p, int device, uint8_t handle[kIpcHandleBytes], uint64_t &offset) {
    DeviceBackend *be = device_backend();
    void *base = nullptr;
    size_t size = 0;
    if (!be->address_range(p, &base, &size) || base == nullptr) return false;
    be->set_device(device);
    if (!be->ipc_export(base, handle)) return false; // e.g. VMM / expandable-segment memory: use the staged mode
    offset = static_cast<uint64_t>(static_cast<uint8_t *>(p) - static_cast<uint8_t *>(base));
    return true;
}

void IpcArena::set_phase(uint64_t seq, uint32_t phase) {
    shm_->op(static_cast<uint32_t>(seq % kSlots), static_cast<uint32_t>(rank_))
        ->phase.store(((seq + 1) << 8) | phase, std::memory_order_release);
}

// A crashed peer stays a zombie until its parent reaps it, and kill(pid, 0) succeeds on zombies: also check the
// process state in /proc so that survivors abort promptly instead of waiting for the barrier timeout.
static bool pid_alive(int pid) {
    if (kill(pid, 0) != 0 && errno != EPERM) return false;
    char path[64];
    std::snprintf(path, sizeof(path), "/proc/%d/stat", pid);
    FILE *f = std::fopen(path, "r");
    if (!f) return true; // no procfs view of it (other namespace): trust kill()
    char buf[512];
    const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char *rp = std::strrchr(buf, ')'); // "pid (comm) state ..."; comm may contain spaces or parentheses
    if (!rp || rp[1] == 0 || rp[2] == 0) return true;
    const char state = rp[2];
    return state != 'Z' && state != 'X' && state != 'x';
}

int IpcArena::barrier(Client &c, uint64_t tag, uint64_t seq, uint32_t phase) {
    const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
    const auto t0 = steady_clock::now();
    const auto timeout = milliseconds(env_size("PCCL_IPC_TIMEOUT_MS", 60000));
    auto last_check = t0;
    uint64_t spins = 0;
    for (size_t k = 0; k < ring_.size(); ++k) {
        if (k == rank_) continue;
        OpPeerShm *p = shm_->op(slot, static_cast<uint32_t>(k));
        while (true) {
            const uint64_t v = p->phase.load(std::memory_order_acquire);
            const uint64_t vs = v >> 8;
            const uint32_t vp = static_cast<uint32_t>(v & 0xff);
            if (vs == seq + 1) {
                if (vp == PH_ABORTED) {
                    LOG(WARN) << "IPC: peer " << k << " aborted op seq " << seq << " (phase " << phase << ")";
                    return 1;
                }
                if (vp >= phase) break;
            } else if (vs > seq + 1) {
                LOG(WARN) << "IPC: peer " << k << " is ahead (seq " << vs - 1 << " > " << seq << ")";
                return 1;
            }
            if (++spins < 4096) {
                cpu_relax();
                continue;
            }
            std::this_thread::sleep_for(microseconds(spins < 20000 ? 5 : 50));
            const auto now = steady_clock::now();
            if (now - last_check > milliseconds(10)) {
                last_check = now;
                if (c.abort_received(tag)) return 2;
                if (!pid_alive(pids_[k])) {
                    LOG(WARN) << "IPC: peer process " << pids_[k] << " died";
                    return 1;
                }
                if (!c.master_.is_open()) return 1;
                if (now - t0 > timeout) {
                    LOG(WARN) << "IPC: barrier timeout (seq " << seq << ", phase " << phase << ")";
                    return 1;
                }
            }
        }
    }
    return 0;
}

bool IpcArena::wait_slot_free(Client &c, uint64_t seq) {
    const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
    const auto t0 = steady_clock::now();
    for (size_t k = 0; k < ring_.size(); ++k) {
        OpPeerShm *p = shm_->op(slot, static_cast<uint32_t>(k));
        while (true) {
            const uint64_t v = p->phase.load(std::memory_order_acquire);
            const uint32_t vp = static_cast<uint32_t>(v & 0xff);
            if (v == 0 || (v >> 8) >= seq + 1 || vp == PH_RELEASED || vp == PH_ABORTED) break;
            std::this_thread::sleep_for(microseconds(20));
            if (steady_clock::now() - t0 > seconds(30) || !pid_alive(pids_[k]) || !c.master_.is_open()) return false;
        }
    }
    return true;
}

bool IpcArena::push_algorithm() {
    static const bool two_shot = [] {
        const char *v = std::getenv("PCCL_IPC_ALGO");
        return v && std::strcmp(v, "two_shot") == 0;
    }();
    return !two_shot;
}

void IpcArena::drain_peers(Client &c, uint64_t seq) {
    // Used before restoring an in-place buffer after an abort: in the push algorithm peers write into my receive
    // buffer, so wait until every live peer that may have passed the vote barrier is past its kernel. A peer that has
    // not voted for `seq` yet will see my ABORTED phase in its vote barrier and never launch.
    (void)c;
    const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
    const auto t0 = steady_clock::now();
    const auto timeout = milliseconds(env_size("PCCL_IPC_TIMEOUT_MS", 60000));
    for (size_t k = 0; k < ring_.size(); ++k) {
        if (k == rank_) continue;
        const OpPeerShm *p = shm_->op(slot, static_cast<uint32_t>(k));
        while (true) {
            const uint64_t v = p->phase.load(std::memory_order_acquire);
            const uint64_t vs = v >> 8;
            const uint32_t vp = static_cast<uint32_t>(v & 0xff);
            if (vs != seq + 1 || vp == PH_GATHERED || vp == PH_RELEASED || vp == PH_ABORTED) break;
            if (!pid_alive(pids_[k])) break;
            if (steady_clock::now() - t0 > timeout) {
                LOG(WARN) << "IPC: peer " << k << " did not finish op seq " << seq << " before the restore";
                break;
            }
            std::this_thread::sleep_for(microseconds(20));
        }
    }
}

int IpcArena::vote_impl(Client &c, uint64_t tag, uint64_t seq, bool device_ok, int device, size_t bytes, DType dtype,
                        ReduceOp op, const void *src, void *dst) {
    if (!wait_slot_free(c, seq)) {
        LOG(WARN) << "IPC: slot of op seq " << seq << " not released by a peer";
        return kAborted;
    }
    OpPeerShm *mine = shm_->op(static_cast<uint32_t>(seq % kSlots), static_cast<uint32_t>(rank_));
    DeviceBackend *be = device_backend();
    CommBuf *buf = nullptr;
    bool in_direct = false, out_direct = false;
    if (map_failed_.load(std::memory_order_relaxed)) device_ok = false; // vote for the TCP ring from now on
    if (device_ok) {
        // Direct (zero-copy) access to the caller's buffers where HIP IPC can export them. An in-place op always
        // stages its input: peers read the staged copy while results land in the caller's buffer, and the copy is
        // the abort backup (reference reduce.cpp:551-580 keeps a backup for src == dst too).
        const bool allow_direct = !env_flag("PCCL_IPC_NO_ZERO_COPY", false);
        if (allow_direct && src != dst) in_direct = export_user(const_cast<void *>(src), device, mine->in_handle, mine->in_off);
        if (allow_direct) out_direct = export_user(dst, device, mine->out_handle, mine->out_off);
        if (in_direct) mine->in_raw = reinterpret_cast<uint64_t>(src);
        if (out_direct) mine->out_raw = reinterpret_cast<uint64_t>(dst);
        if (!in_direct || !out_direct) {
            buf = acquire_buffer(2 * bytes, device);
            if (!buf) {
                device_ok = false;
            } else {
                if (!in_direct) {
                    std::memcpy(mine->in_handle, buf->handle, kIpcHandleBytes);
                    mine->in_off = 0;
                    mine->in_raw = reinterpret_cast<uint64_t>(buf->ptr);
                    // copy-in before the vote: a passed vote barrier means every peer's input is readable
                    StreamLease stream(device);
                    if (!stream.get() || !be->memcpy_async(buf->ptr, src, bytes, stream.get()) ||
                        !be->stream_sync(stream.get())) {
                        LOG(ERR) << "IPC: copy-in of " << bytes << " bytes failed";
                        device_ok = false;
                    }
                    trace_mark("copy_in");
                }
                if (!out_direct) {
                    std::memcpy(mine->out_handle, buf->handle, kIpcHandleBytes);
                    mine->out_off = bytes;
                    mine->out_raw = reinterpret_cast<uint64_t>(static_cast<uint8_t *>(buf->ptr) + bytes);
                }
            }
        }
    }
    mine->gpu_uid = device_ok ? be->device_uid(device) : 0;
    mine->vote = device_ok ? 1 : 0;
    mine->zero_copy = (in_direct ? 1u : 0u) | (out_direct ? 2u : 0u);
    mine->device = device;
    mine->bytes = bytes;
    mine->dtype = static_cast<uint32_t>(dtype);
    mine->op = static_cast<uint32_t>(op);
    set_phase(seq, PH_VOTED);
    const int rc = barrier(c, tag, seq, PH_VOTED);
    if (rc != 0) {
        LOG(WARN) << "IPC: vote barrier failed (rc " << rc << ")";
        set_phase(seq, PH_ABORTED);
        if (device_ok && buf && !in_direct && src == dst && out_direct) {
            // peers that passed the barrier before my abort may be pushing into the caller's buffer: let them
            // finish, then restore it from the staged copy
            drain_peers(c, seq);
            be->memcpy_sync(dst, buf->ptr, bytes);
        }
        release_buffer(buf);
        return rc == 2 ? kAbortedByMaster : kAborted;
    }
    bool all = true;
    const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
    for (size_t k = 0; k < ring_.size(); ++k) {
        const OpPeerShm *p = shm_->op(slot, static_cast<uint32_t>(k));
        all = all && p->vote == 1 && p->bytes == bytes && p->dtype == static_cast<uint32_t>(dtype) &&
              p->op == static_cast<uint32_t>(op);
    }
    if (!all) {
        set_phase(seq, PH_RELEASED);
        release_buffer(buf);
        return kUseRing;
    }
    OpCtx ctx;
    ctx.bytes = bytes;
    ctx.comm = buf ? buf->ptr : nullptr;
    ctx.in_staged = !in_direct;
    ctx.out_staged = !out_direct;
    ctx.my_out = out_direct ? static_cast<uint8_t *>(dst) : static_cast<uint8_t *>(buf->ptr) + bytes;
    ctx.peer_in.resize(ring_.size());
    ctx.peer_out.resize(ring_.size());
    for (size_t k = 0; k < ring_.size(); ++k) {
        const OpPeerShm *p = shm_->op(slot, static_cast<uint32_t>(k));
        if (k == rank_ || pids_[k] == pids_[rank_]) { // same process (threaded peers): raw pointers are usable
            ctx.peer_in[k] = reinterpret_cast<const uint8_t *>(p->in_raw);
            ctx.peer_out[k] = reinterpret_cast<uint8_t *>(p->out_raw);
            continue;
        }
        auto *in_base = static_cast<const uint8_t *>(peer_mapping(static_cast<int>(k), p->in_handle, device));
        auto *out_base = static_cast<uint8_t *>(peer_mapping(static_cast<int>(k), p->out_handle, device));
        if (!in_base || !out_base) {
            // e.g. no peer access between these GPUs: this op aborts (every peer sees ABORTED), and this peer
            // votes against the xGMI path from now on, so the ring falls back to TCP instead of failing every op
            LOG(ERR) << "IPC: cannot map the buffers of peer " << k << "; using the TCP ring for later ops";
            map_failed_.store(true, std::memory_order_relaxed);
            set_phase(seq, PH_ABORTED);
            if (buf && !in_direct && src == dst && out_direct) {
                drain_peers(c, seq);
                be->memcpy_sync(dst, buf->ptr, bytes);
            }
            release_buffer(buf);
            return kAborted;
        }
        ctx.peer_in[k] = in_base + p->in_off;
        ctx.peer_out[k] = out_base + p->out_off;
    }
    {
        std::lock_guard l(g_ctx_mtx);
        g_ctx[{this, seq}] = std::move(ctx);
    }
    return kUseIpc;
}

std::pair<bool, bool> IpcArena::run(Client &c, uint64_t tag, uint64_t seq, const void *src, void *dst, size_t count,
                                    DType dtype, ReduceOp op, int device, std::atomic<uint64_t> &tx,
                                    std::atomic<uint64_t> &rx, const InterHost *inter, size_t world) {
    OpCtx ctx;
    {
        std::lock_guard l(g_ctx_mtx);
        auto it = g_ctx.find({this, seq});
        if (it == g_ctx.end()) {
            LOG(ERR) << "IPC: no context for op seq " << seq;
            return {false, false};
        }
        ctx = std::move(it->second);
        g_ctx.erase(it);
    }
    CommBuf *mybuf = nullptr;
    if (ctx.comm) {
        std::lock_guard l(mtx_);
        for (auto &b : bufs_)
            if (b->ptr == ctx.comm) mybuf = b.get();
    }
    DeviceBackend *be = device_backend();
    be->set_device(device);
    StreamLease stream(device);
    DevStream st = stream.get();
    const size_t W = ring_.size();
    const size_t es = dtype_size(dtype);
    const size_t bytes = ctx.bytes;
    uint8_t *my_out = ctx.my_out;
    const bool push = inter != nullptr || push_algorithm();

    auto finish = [&](int rc) -> std::pair<bool, bool> {
        if (rc != 0) {
            be->stream_sync(st); // my kernels are done: no further writes from this peer
            set_phase(seq, PH_ABORTED);
            if (src == dst && ctx.in_staged && ctx.comm) {
                // restore the caller's buffer from the staged original once no peer can still write into it
                if (push && !ctx.out_staged) drain_peers(c, seq);
                be->memcpy_async(dst, ctx.comm, bytes, st);
                be->stream_sync(st);
            }
        } else {
            set_phase(seq, PH_RELEASED);
        }
        release_buffer(mybuf);
        return {rc == 0, rc == 2};
    };
    if (!st) {
        LOG(ERR) << "IPC: no stream on device " << device;
        return finish(1);
    }

    // shard bounds: 256-byte aligned so every peer's shard is 16-byte-vector aligned
    const size_t align_el = std::max<size_t>(1, 256 / es);
    const size_t per = ((count + W - 1) / W + align_el - 1) / align_el * align_el;
    std::vector<size_t> lo(W), n(W);
    for (size_t k = 0; k < W; ++k) {
        lo[k] = std::min(k * per, count);
        n[k] = std::min(lo[k] + per, count) - lo[k];
    }
    std::vector<const void *> srcs(W);
    for (size_t k = 0; k < W; ++k) srcs[k] = ctx.peer_in[k] + lo[rank_] * es;
    // workgroup budget: 512 per GPU (2 per CU, the measured optimum for these streaming kernels), split between the
    // peers whose kernels run concurrently on this GPU, but not below 256 per kernel (fewer cannot saturate HBM)
    int sharing = 0;
    {
        const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
        const uint64_t me = shm_->op(slot, static_cast<uint32_t>(rank_))->gpu_uid;
        for (size_t k = 0; k < W; ++k) sharing += shm_->op(slot, static_cast<uint32_t>(k))->gpu_uid == me ? 1 : 0;
    }
    const int grid = std::max(256, 512 / std::max(1, sharing));

    if (inter) {
        // hierarchical: host-local reduce of my shard into scratch, inter-host ring on the scratch, local push
        Lease part(device_pool(), std::max<size_t>(n[rank_] * es, 256), device);
        if (!part.ok()) return finish(1);
        void *p = part.data();
        const ReduceOp local_op = op == ReduceOp::Avg ? ReduceOp::Sum : op;
        if (!be->multi_reduce(&p, 1, srcs.data(), static_cast<int>(W), n[rank_], dtype, local_op, st, grid) ||
            !be->stream_sync(st)) {
            LOG(ERR) << "IPC: host-local reduce failed";
            return finish(1);
        }
        trace_mark("local_reduce");
        if (int rc = (*inter)(p, n[rank_])) return finish(rc);
        trace_mark("inter_host");
        if (op == ReduceOp::Avg && n[rank_] > 0) be->finalize_avg(p, n[rank_], dtype, world, st);
        std::vector<void *> dsts(W);
        for (size_t k = 0; k < W; ++k) dsts[k] = ctx.peer_out[k] + lo[rank_] * es;
        const void *one = p;
        if (!be->multi_reduce(dsts.data(), static_cast<int>(W), &one, 1, n[rank_], dtype, ReduceOp::Sum, st, grid) ||
            !be->stream_sync(st)) {
            LOG(ERR) << "IPC: host-local broadcast failed";
            return finish(1);
        }
        trace_mark("local_bcast");
    } else if (push) {
        // one-shot: read shard `rank` of every peer's input (inbound xGMI), reduce in fixed peer order and write the
        // result into every peer's output (outbound xGMI, posted writes) — reduce-scatter and all-gather overlap in
        // one kernel and one barrier; every peer receives the owner's bytes, so results are bit-identical
        std::vector<void *> dsts(W);
        for (size_t k = 0; k < W; ++k) dsts[k] = ctx.peer_out[k] + lo[rank_] * es;
        if (!be->multi_reduce(dsts.data(), static_cast<int>(W), srcs.data(), static_cast<int>(W), n[rank_], dtype, op,
                              st, grid) ||
            !be->stream_sync(st)) {
            LOG(ERR) << "IPC: multi-source reduce + broadcast failed";
            return finish(1);
        }
        trace_mark("reduce_bcast");
    } else {
        // two-shot: reduce-scatter into my output, barrier, then pull every other shard (reads only)
        void *d0 = my_out + lo[rank_] * es;
        if (!be->multi_reduce(&d0, 1, srcs.data(), static_cast<int>(W), n[rank_], dtype, op, st, grid) ||
            !be->stream_sync(st)) {
            LOG(ERR) << "IPC: multi-source reduce failed";
            return finish(1);
        }
        trace_mark("reduce");
        set_phase(seq, PH_REDUCED);
        if (int rc = barrier(c, tag, seq, PH_REDUCED)) return finish(rc);
        trace_mark("reduced_barrier");
        std::vector<const void *> gsrc(W);
        for (size_t k = 0; k < W; ++k) gsrc[k] = ctx.peer_out[k] + lo[k] * es;
        if (!be->multi_gather(my_out, gsrc.data(), lo.data(), n.data(), static_cast<int>(W), static_cast<int>(rank_),
                              dtype, st) ||
            !be->stream_sync(st)) {
            LOG(ERR) << "IPC: gather failed";
            return finish(1);
        }
        trace_mark("gather");
    }
    set_phase(seq, PH_GATHERED);
    if (int rc = barrier(c, tag, seq, PH_GATHERED)) return finish(rc);
    trace_mark("gathered_barrier");
    if (ctx.out_staged) { // the caller's receive buffer could not be exported: copy the assembled result out
        if (!be->memcpy_async(dst, my_out, bytes, st) || !be->stream_sync(st)) {
            LOG(ERR) << "IPC: copy-out failed";
            return finish(1);
        }
    }

    const uint64_t moved = static_cast<uint64_t>(bytes) * (W - 1) / W;
    tx += 2 * moved;
    rx += 2 * moved;
    return finish(0);
}

std::pair<bool, bool> Client::ipc_reduce(OpState &op, const RingView &rv, uint64_t seq, int device) {
    return rv.arena->run(*this, op.req.tag, seq, op.req.src, op.req.dst, op.req.count, op.req.dtype, op.req.op, device,
                         op.tx, op.rx);
}

// Hierarchical all-reduce (ring spans several hosts with L peers each): reduce-scatter inside each host over xGMI,
// one TCP device ring per local rank across hosts on the 1/L shard, all-gather inside the host over xGMI. Every byte
// crosses the network once per host instead of once per GPU.
std::pair<bool, bool> Client::hier_reduce(OpState &op, const RingView &rv, uint64_t seq, int device) {
    const HierState &h = *rv.hier;
    const int decision = h.arena->vote(*this, op, seq, true, device);
    if (decision != IpcArena::kUseIpc) {
        // every participant announced the capability, so a local refusal means inconsistent buffers: fail the op
        LOG(ERR) << "hierarchical all-reduce: host-local vote failed (decision " << decision << ")";
        return {false, decision == IpcArena::kAbortedByMaster || abort_received(op.req.tag)};
    }
    RingView sub;
    sub.ring = h.host_ring;
    sub.rank = h.host;
    sub.tx = rv.htx;
    sub.rx = rv.hrx;
    IpcArena::InterHost inter = [&](void *part, size_t count) -> int {
        OpState inner;
        inner.req = op.req;
        inner.req.src = part;
        inner.req.dst = part;
        inner.req.count = count;
        inner.req.scratch = true;
        if (inner.req.op == ReduceOp::Avg) inner.req.op = ReduceOp::Sum; // divided by the whole world afterwards
        const auto r = ring_reduce_device(inner, sub, seq, device);
        op.tx += inner.tx.load();
        op.rx += inner.rx.load();
        return r.first && !r.second ? 0 : (r.second ? 2 : 1);
    };
    return h.arena->run(*this, op.req.tag, seq, op.req.src, op.req.dst, op.req.count, op.req.dtype, op.req.op, device,
                        op.tx, op.rx, &inter, rv.ring.size());
}

} // namespace pccl::client
