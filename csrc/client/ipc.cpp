#include "ipc.hpp"

#include <dirent.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <climits>
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
#include <mutex>
#include <thread>
#include <tuple>

#include "../common/log.hpp"
#include "client.hpp"
#include "pools.hpp"
#include "shareable.hpp"
#include "vmm_share.hpp"
#include "../common/trace.hpp"

namespace pccl::client {

using namespace std::chrono;

namespace {
constexpr uint64_t kMagic = 0x5043434c49504331ull; // "PCCLIPC1"
constexpr uint32_t kClosed = 0x80000000u;
constexpr uint32_t kSlots = 128; // ops in flight per ring (slot = seq % kSlots)
constexpr uint32_t kMaxWorld = 16;

constexpr uint32_t PH_VOTED = 1, PH_PROBED = 2, PH_REDUCED = 3, PH_GATHERED = 4, PH_RELEASED = 5, PH_ABORTED = 0xEE;

uint64_t fnv1a(const void *p, size_t n, uint64_t h = 1469598103934665603ull) {
    const auto *b = static_cast<const uint8_t *>(p);
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

inline void cpu_relax() { __builtin_ia32_pause(); }

// Futex on the low 32 bits of a shared 64-bit phase word (little endian: they change with every phase store).
// Shared (not FUTEX_PRIVATE): the word lives in a shm segment mapped by several processes.
int futex_wait32(std::atomic<uint64_t> *word, uint32_t expect, long timeout_us) {
    timespec ts{timeout_us / 1000000, (timeout_us % 1000000) * 1000};
    return static_cast<int>(::syscall(SYS_futex, reinterpret_cast<uint32_t *>(word), FUTEX_WAIT, expect, &ts,
                                      nullptr, 0));
}
void futex_wake_all(std::atomic<uint64_t> *word) {
    ::syscall(SYS_futex, reinterpret_cast<uint32_t *>(word), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}
} // namespace

struct alignas(64) PeerSlotShm {
    std::atomic<uint32_t> present;
    int32_t pid;
    uint32_t can_ipc;
    uint8_t uuid[16];
};

// Per (op slot, peer) record. Every peer publishes where its op *input* (read by the reduce-scatter) and *output*
// (written by its own reduce, read by the all-gather) live:
//   zero-copy (out-of-place device buffers in allocations of <= kIpcMaxExport bytes): the caller's send / receive
//     buffer, one exported allocation + offset (n_segs = 1)
//   staged (in-place, large allocations, export failure): a pooled comm buffer of n_segs kIpcSegBytes segments
// Peers may mix the two modes. *_raw are usable directly by peers in the same process (threaded peers).
struct alignas(64) OpPeerShm {
    std::atomic<uint64_t> phase; // (seq + 1) << 8 | phase
    uint32_t vote;
    int32_t device;
    uint64_t bytes;
    uint32_t dtype;
    uint32_t op;
    uint32_t zero_copy; // bit 0: input is the caller's send buffer, bit 1: output is the caller's receive buffer
    uint32_t algo;      // 0 push, 1 two-shot (PCCL_IPC_ALGO at the vote; every peer must vote the same)
    uint64_t gpu_uid;   // physical GPU of this op's buffers (peers sharing a GPU split its CUs)
    uint32_t in_segs, out_segs;
    uint64_t in_off, out_off; // offset into the (single) exported allocation
    uint64_t in_raw[kIpcMaxSegs], out_raw[kIpcMaxSegs];
    uint8_t in_handle[kIpcMaxSegs][kIpcHandleBytes];
    uint8_t out_handle[kIpcMaxSegs][kIpcHandleBytes];
};

struct ArenaShm {
    std::atomic<uint64_t> magic;
    std::atomic<uint32_t> join;
    std::atomic<uint32_t> unlinked;
    uint32_t world;
    // threads of any ring member sleeping in futex_wait_phase on a phase word: set_phase wakes only when non-zero
    std::atomic<uint32_t> sleepers;
    uint32_t pad[10];
    PeerSlotShm *peers() { return reinterpret_cast<PeerSlotShm *>(reinterpret_cast<uint8_t *>(this) + 64); }
    OpPeerShm *op(uint32_t slot, uint32_t peer) {
        auto *base = reinterpret_cast<uint8_t *>(this) + 64 + sizeof(PeerSlotShm) * kMaxWorld;
        return reinterpret_cast<OpPeerShm *>(base) + slot * kMaxWorld + peer;
    }
    static size_t bytes() { return 64 + sizeof(PeerSlotShm) * kMaxWorld + sizeof(OpPeerShm) * kSlots * kMaxWorld; }
};

// One peer's input or output as seen from this process: one contiguous mapping (offset applied) or the segments of
// a staged comm buffer. Kernels only ever touch [x, y) ranges that do not cross a multiple of kIpcSegBytes.
struct PeerView {
    std::vector<uint8_t *> seg;
    uint8_t *at(size_t x) const { return seg.size() == 1 ? seg[0] + x : seg[x / kIpcSegBytes] + x % kIpcSegBytes; }
};

struct OpCtx {
    void *in_buf = nullptr, *out_buf = nullptr; // my staged comm buffers (IpcArena::CommBuf *), if any
    bool in_staged = false;  // peers read my input from my staged input buffer (copied in before the vote)
    bool out_staged = false; // peers write / gather my output into my staged output buffer (copied out)
    std::vector<PeerView> in, out;
    std::vector<IpcArena::MapKey> pins; // mappings this op holds
    size_t bytes = 0;
};

// per-process counters of how op buffers were handed to the peers (pcclxIpcStats): [0] direct inputs, [1] direct
// outputs, [2] staged inputs, [3] staged outputs
// [0..3] direct_in, direct_out, staged_in, staged_out; [4] comm buffers quarantined after an abort; [5] drains that
// waited for a dead peer's threads to finish tearing down its address space; [6] / [7] cross-GPU pre-flight probes
// failed / passed; [8] quarantined buffers reclaimed (no peer can still touch them); [9] quarantined VMM buffers
// freed beyond the quarantine cap
static std::atomic<uint64_t> g_buf_stats[10];

// per-process bookkeeping
static std::mutex g_ctx_mtx;
static std::map<std::pair<const IpcArena *, uint64_t>, OpCtx> g_ctx;
static std::mutex g_attempt_mtx;
static std::map<uint64_t, int> g_attempts;

int ipc_grid_budget(const std::vector<uint64_t> &gpu_uids, size_t rank) {
    int sharing = 0;
    for (uint64_t u : gpu_uids) sharing += u == gpu_uids[rank] ? 1 : 0;
    return std::max(256, 512 / std::max(1, sharing));
}

bool ipc_needs_preflight(const std::vector<uint64_t> &gpu_uids, bool done, size_t bytes) {
    // PCCL_IPC_PREFLIGHT: 0 off, 1 (default) rings spanning several GPUs, 2 every ring (rehearsal on one GPU)
    static const size_t mode = env_size("PCCL_IPC_PREFLIGHT", 1);
    if (done || mode == 0 || bytes < gpu_uids.size() * 256) return false;
    if (mode >= 2) return true;
    for (uint64_t u : gpu_uids)
        if (u != gpu_uids[0]) return true;
    return false;
}

int ipc_push_grid(const std::vector<uint64_t> &gpu_uids, size_t rank, int remote_grid) {
    const int base = ipc_grid_budget(gpu_uids, rank);
    if (remote_grid <= 0) return base;
    for (uint64_t u : gpu_uids)
        if (u != gpu_uids[rank]) return std::min(remote_grid, 4096);
    return base;
}

int ipc_unreachable_peer(const std::vector<uint64_t> &gpu_uids, size_t rank, int my_device,
                         const std::function<int(uint64_t)> &device_of_uid,
                         const std::function<bool(int, int)> &can_access_peer) {
    for (size_t k = 0; k < gpu_uids.size(); ++k) {
        if (k == rank || gpu_uids[k] == gpu_uids[rank]) continue;
        const int d = device_of_uid(gpu_uids[k]);
        if (d >= 0 && !can_access_peer(my_device, d)) return static_cast<int>(k);
    }
    return -1;
}

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

bool ipc_safe_mode() {
    static const bool safe = [] {
        const char *v = std::getenv("PCCL_IPC_MODE");
        return !(v && std::strcmp(v, "fast") == 0);
    }();
    return safe;
}

bool IpcArena::safe_mode() { return ipc_safe_mode(); }

void IpcArena::release_mapping(const MapKey &key, Mapping &m) {
    DeviceBackend *be = device_backend();
    be->set_device(std::get<2>(key));
    if (m.vmm) be->vmm_unmap(m.ptr);
    else be->ipc_close(m.ptr);
}

IpcArena::~IpcArena() {
    DeviceBackend *be = device_backend();
    if (be) {
        const int cur = be->current_device();
        for (auto &[key, m] : mappings_) release_mapping(key, m);
        for (auto &b : bufs_) {
            be->set_device(b->device);
            for (size_t k = 0; k < b->segs.size(); ++k) {
                if (b->share_ids[k]) {
                    VmmShare::instance().retract(b->share_ids[k]);
                    be->vmm_free(b->segs[k]);
                } else {
                    be->free_device(b->segs[k]);
                }
            }
        }
        if (cur >= 0) be->set_device(cur);
    }
    if (shm_) munmap(shm_, shm_bytes_);
}

static bool pid_alive(int pid);
static bool pid_quiesced(int pid);

IpcArena::CommBuf *IpcArena::acquire_buffer(size_t bytes, int device) {
    std::lock_guard l(mtx_);
    reclaim_quarantined_locked();
    CommBuf *best = nullptr;
    for (auto &b : bufs_)
        if (!b->busy && b->device == device && b->cap >= bytes && (!best || b->cap < best->cap)) best = b.get();
    if (best) {
        best->busy = true;
        return best;
    }
    if (bytes > kIpcSegBytes * kIpcMaxSegs) return nullptr;
    DeviceBackend *be = device_backend();
    auto b = std::make_unique<CommBuf>();
    b->device = device;
    be->set_device(device);
    const size_t nseg = bytes <= kIpcSegBytes ? 1 : (bytes + kIpcSegBytes - 1) / kIpcSegBytes;
    const size_t seg_cap = nseg == 1 ? std::max<size_t>(bytes, 1 << 20) : kIpcSegBytes;
    const bool vmm = safe_mode();
    auto undo = [&] {
        for (size_t k = 0; k < b->segs.size(); ++k) {
            if (b->share_ids[k]) {
                VmmShare::instance().retract(b->share_ids[k]);
                be->vmm_free(b->segs[k]);
            } else {
                be->free_device(b->segs[k]);
            }
        }
    };
    for (size_t k = 0; k < nseg; ++k) {
        std::array<uint8_t, kIpcHandleBytes> h{};
        void *p = nullptr;
        uint64_t id = 0;
        if (vmm) { // fault-safe: VMM allocation shared as an fd (importers hold their own reference)
            int fd = -1;
            size_t alloc = 0;
            p = be->vmm_alloc(seg_cap, device, &fd, &alloc);
            if (p) {
                id = VmmShare::instance().publish(fd);
                if (id == 0) {
                    ::close(fd);
                    be->vmm_free(p);
                    p = nullptr;
                }
            }
            if (p) {
                VmmHandle vh;
                vh.pid = static_cast<int32_t>(getpid());
                vh.nonce = VmmShare::instance().nonce();
                vh.id = id;
                vh.size = alloc;
                std::memcpy(h.data(), &vh, sizeof(vh));
            }
        } else {
            p = be->alloc_device(seg_cap);
            if (p && !be->ipc_export(p, h.data())) {
                be->free_device(p);
                p = nullptr;
            }
        }
        if (!p) {
            undo();
            LOG(ERR) << "IPC arena: failed to allocate/export a " << seg_cap << "-byte comm buffer segment"
                     << (vmm ? " (VMM)" : "");
            return nullptr;
        }
        b->segs.push_back(p);
        b->handles.push_back(h);
        b->share_ids.push_back(id);
    }
    b->cap = nseg * seg_cap;
    b->busy = true;
    bufs_.push_back(std::move(b));
    return bufs_.back().get();
}

void IpcArena::release_buffer(CommBuf *b) {
    if (!b) return;
    std::lock_guard l(mtx_);
    if (!b->quarantined) b->busy = false;
}

void IpcArena::quarantine_buffer(CommBuf *b, uint64_t seq) {
    if (!b) return;
    std::lock_guard l(mtx_);
    if (!b->quarantined) ++g_buf_stats[4];
    b->quarantined = true;
    b->qseq = seq;
    b->busy = true;
}

bool IpcArena::op_quiet(uint64_t seq) const {
    const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
    for (size_t k = 0; k < ring_.size(); ++k) {
        if (k == rank_) continue;
        if (!pid_alive(pids_[k])) {
            if (!pid_quiesced(pids_[k])) return false;
            continue;
        }
        const uint64_t v = shm_->op(slot, static_cast<uint32_t>(k))->phase.load(std::memory_order_acquire);
        const uint64_t vs = v >> 8;
        const uint32_t vp = static_cast<uint32_t>(v & 0xff);
        if (vs == seq + 1 && vp != PH_GATHERED && vp != PH_RELEASED && vp != PH_ABORTED) return false;
    }
    return true;
}

// Every peer that may still be inside op `seq` (see op_quiet) is another process: such a peer reaches my segments
// only through its own VMM import, which keeps the pages alive after I free my mapping. A peer thread of this process
// writes through raw pointers into my mapping (no import), so a buffer it may still touch is never freed.
bool IpcArena::unquiet_peers_remote(uint64_t seq) const {
    const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
    const int self = static_cast<int>(::getpid());
    for (size_t k = 0; k < ring_.size(); ++k) {
        if (k == rank_) continue;
        if (!pid_alive(pids_[k])) {
            if (!pid_quiesced(pids_[k]) && pids_[k] == self) return false;
            continue;
        }
        const uint64_t v = shm_->op(slot, static_cast<uint32_t>(k))->phase.load(std::memory_order_acquire);
        const uint32_t vp = static_cast<uint32_t>(v & 0xff);
        const bool quiet = (v >> 8) != seq + 1 || vp == PH_GATHERED || vp == PH_RELEASED || vp == PH_ABORTED;
        if (!quiet && pids_[k] == self) return false;
    }
    return true;
}

void IpcArena::reclaim_quarantined_locked() {
    constexpr size_t kQuarantineCapBytes = size_t{8} << 30;
    size_t held = 0;
    for (auto &b : bufs_) {
        if (!b->quarantined) continue;
        if (op_quiet(b->qseq)) {
            b->quarantined = false;
            b->busy = false;
            ++g_buf_stats[8];
        } else {
            held += b->cap;
        }
    }
    if (held <= kQuarantineCapBytes) return;
    DeviceBackend *be = device_backend();
    const int cur = be->current_device();
    for (auto it = bufs_.begin(); it != bufs_.end() && held > kQuarantineCapBytes;) {
        CommBuf *b = it->get();
        const bool vmm = std::all_of(b->share_ids.begin(), b->share_ids.end(), [](uint64_t id) { return id != 0; });
        if (!b->quarantined || !vmm || !unquiet_peers_remote(b->qseq)) {
            ++it;
            continue;
        }
        be->set_device(b->device);
        for (size_t k = 0; k < b->segs.size(); ++k) {
            VmmShare::instance().retract(b->share_ids[k]);
            be->vmm_free(b->segs[k]);
        }
        held -= b->cap;
        ++g_buf_stats[9];
        it = bufs_.erase(it);
    }
    if (cur >= 0) be->set_device(cur);
}

void *IpcArena::pin_mapping(int peer, const uint8_t *handle, int my_device, MapKey &key) {
    std::lock_guard l(mtx_);
    std::array<uint8_t, kIpcHandleBytes> hb;
    std::memcpy(hb.data(), handle, kIpcHandleBytes);
    key = std::make_tuple(peer, hb, my_device);
    auto it = mappings_.find(key);
    if (it != mappings_.end()) {
        ++it->second.refs;
        it->second.used = ++map_clock_;
        return it->second.ptr;
    }
    DeviceBackend *be = device_backend();
    be->set_device(my_device);
    void *p = nullptr;
    VmmHandle vh;
    const bool vmm = VmmHandle::decode(handle, vh);
    if (vmm) {
        const int fd = VmmShare::fetch(vh.pid, vh.nonce, vh.id);
        if (fd < 0) return nullptr;
        p = be->vmm_import(fd, vh.size, my_device);
        ::close(fd);
    } else {
        p = be->ipc_open(handle);
    }
    if (!p) return nullptr;
    mappings_[key] = Mapping{p, vmm, 1, ++map_clock_};
    // bound the number of open mappings (user allocations come and go): close the least recently used ones that no
    // op holds (an op's kernels may be reading / writing through every mapping it pinned)
    constexpr size_t kMaxMappings = 256;
    while (mappings_.size() > kMaxMappings) {
        auto victim = mappings_.end();
        for (auto m = mappings_.begin(); m != mappings_.end(); ++m)
            if (m->second.refs == 0 && (victim == mappings_.end() || m->second.used < victim->second.used)) victim = m;
        if (victim == mappings_.end()) break; // everything is pinned by in-flight ops
        release_mapping(victim->first, victim->second);
        mappings_.erase(victim);
    }
    be->set_device(my_device);
    return p;
}

void IpcArena::unpin_mappings(const std::vector<MapKey> &keys) {
    std::lock_guard l(mtx_);
    for (const auto &k : keys) {
        auto it = mappings_.find(k);
        if (it != mappings_.end() && it->second.refs > 0) --it->second.refs;
    }
}

bool IpcArena::export_user(void *p, int device, uint8_t handle[kIpcHandleBytes], uint64_t &offset) {
    DeviceBackend *be = device_backend();
    void *base = nullptr;
    size_t size = 0;
    if (!be->address_range(p, &base, &size) || base == nullptr) return false;
    if (size > kIpcMaxExport) return false; // see kIpcMaxExport: staged instead
    be->set_device(device);
    if (!be->ipc_export(base, handle)) return false; // e.g. VMM / expandable-segment memory: use the staged mode
    offset = static_cast<uint64_t>(static_cast<uint8_t *>(p) - static_cast<uint8_t *>(base));
    return true;
}

void IpcArena::set_phase(uint64_t seq, uint32_t phase) {
    OpPeerShm *p = shm_->op(static_cast<uint32_t>(seq % kSlots), static_cast<uint32_t>(rank_));
    p->phase.store(((seq + 1) << 8) | phase, std::memory_order_seq_cst);
    // a waiter registers in `sleepers` before it checks the word inside FUTEX_WAIT, and the store above precedes
    // this load: either it sees the new value and does not sleep, or this wake reaches it
    if (shm_->sleepers.load(std::memory_order_seq_cst) != 0) futex_wake_all(&p->phase);
}

// Sleeps until the phase word changes from `seen` (or `timeout_us` passed), instead of a fixed sleep.
void IpcArena::wait_phase_change(std::atomic<uint64_t> *word, uint64_t seen, long timeout_us) {
    shm_->sleepers.fetch_add(1, std::memory_order_seq_cst);
    if (word->load(std::memory_order_seq_cst) == seen)
        futex_wait32(word, static_cast<uint32_t>(seen & 0xffffffffu), timeout_us);
    shm_->sleepers.fetch_sub(1, std::memory_order_seq_cst);
}

// One-character state of /proc/<pid>/task/<tid>/stat (or /proc/<pid>/stat with tid < 0); 0 if unreadable.
static char proc_state(int pid, int tid) {
    char path[96];
    if (tid < 0) std::snprintf(path, sizeof(path), "/proc/%d/stat", pid);
    else std::snprintf(path, sizeof(path), "/proc/%d/task/%d/stat", pid, tid);
    FILE *f = std::fopen(path, "r");
    if (!f) return 0;
    char buf[512];
    const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char *rp = std::strrchr(buf, ')'); // "pid (comm) state ..."; comm may contain spaces or parentheses
    if (!rp || rp[1] == 0 || rp[2] == 0) return 0;
    return rp[2];
}

// A crashed peer stays a zombie until its parent reaps it, and kill(pid, 0) succeeds on zombies: also check the
// process state in /proc so that survivors abort promptly instead of waiting for the barrier timeout. "Not alive"
// only means the peer will make no more protocol progress - NOT that its GPU work has stopped (see pid_quiesced).
static bool pid_alive(int pid) {
    if (kill(pid, 0) != 0 && errno != EPERM) return false;
    const char state = proc_state(pid, -1);
    if (state == 0) return true; // no procfs view of it (other namespace): trust kill()
    return state != 'Z' && state != 'X' && state != 'x';
}

// Whether a dead peer can no longer touch GPU memory. Its kernels and copy queues live until its address space is
// torn down: KFD evicts the process's queues from the mm teardown (exit_mmap of the last thread holding the mm).
// A SIGKILLed multi-threaded process shows its group leader as a zombie while other threads are still running
// do_exit, so a zombie leader alone proves nothing. Every thread runs exit_mm (which drops the mm and, for the last
// user, tears it down synchronously) before it turns zombie or is released, hence: quiesced once the process is
// gone, or once every thread listed under /proc/<pid>/task is a zombie / dead.
static bool pid_quiesced(int pid) {
    if (kill(pid, 0) != 0 && errno == ESRCH) return true; // reaped: nothing of it is left
    char path[64];
    std::snprintf(path, sizeof(path), "/proc/%d/task", pid);
    DIR *d = ::opendir(path);
    if (!d) return errno == ENOENT; // gone between the calls; no procfs view (other namespace): not provable
    bool quiet = true;
    while (dirent *e = ::readdir(d)) {
        if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
        const char st = proc_state(pid, std::atoi(e->d_name));
        if (st != 0 && st != 'Z' && st != 'X' && st != 'x') {
            quiet = false;
            break;
        }
    }
    ::closedir(d);
    return quiet;
}

bool ipc_pid_quiesced_for_test(int pid) { return pid_quiesced(pid); }
bool ipc_pid_alive_for_test(int pid) { return pid_alive(pid); }

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
            // spun for a while: sleep until the peer's phase word changes (futex; woken by its set_phase), at most
            // 2 ms so the liveness / abort checks below keep running
            wait_phase_change(&p->phase, v, 2000);
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
            wait_phase_change(&p->phase, v, 2000);
            if (steady_clock::now() - t0 > seconds(30) || !pid_alive(pids_[k]) || !c.master_.is_open()) return false;
        }
    }
    return true;
}

bool IpcArena::all_local_peers() const {
    return std::all_of(pids_.begin(), pids_.end(), [&](int p) { return p == pids_[rank_]; });
}

bool IpcArena::push_algorithm() { // read per op (the bench switches it between phases; the vote checks agreement)
    const char *v = std::getenv("PCCL_IPC_ALGO");
    return !(v && std::strcmp(v, "two_shot") == 0);
}

void IpcArena::drain_peers(Client &c, uint64_t seq) {
    // Used before restoring an in-place buffer after an abort: in the push algorithm peers write into my receive
    // buffer, so wait until every live peer that may have passed the vote barrier is past its kernel. A peer that has
    // not voted for `seq` yet will see my ABORTED phase in its vote barrier and never launch.
    (void)c;
    const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
    const auto t0 = steady_clock::now();
    const auto timeout = milliseconds(env_size("PCCL_IPC_TIMEOUT_MS", 60000));
    bool waited_zombie = false;
    for (size_t k = 0; k < ring_.size(); ++k) {
        if (k == rank_) continue;
        const OpPeerShm *p = shm_->op(slot, static_cast<uint32_t>(k));
        while (true) {
            const uint64_t v = p->phase.load(std::memory_order_acquire);
            const uint64_t vs = v >> 8;
            const uint32_t vp = static_cast<uint32_t>(v & 0xff);
            if (vs != seq + 1 || vp == PH_GATHERED || vp == PH_RELEASED || vp == PH_ABORTED) break;
            // a dead peer may still have kernels in flight until its address space is gone (pid_quiesced)
            if (!pid_alive(pids_[k])) {
                if (pid_quiesced(pids_[k])) break;
                if (!waited_zombie) ++g_buf_stats[5];
                waited_zombie = true;
            }
            if (steady_clock::now() - t0 > timeout) {
                LOG(WARN) << "IPC: peer " << k << " did not finish op seq " << seq << " before the restore";
                break;
            }
            std::this_thread::sleep_for(microseconds(20));
        }
    }
}

namespace {
// staged comm buffer segments <-> a contiguous device buffer (copies on `st`, not synchronised), as a kernel:
// same-device kernel -> kernel ordering on one stream, no copy-engine path for VMM memory.
bool copy_staged(DeviceBackend *be, const std::vector<void *> &segs, uint8_t *user, size_t bytes, bool to_user,
                 DevStream st) {
    for (size_t k = 0, off = 0; off < bytes; ++k, off += kIpcSegBytes) {
        const size_t n = std::min(kIpcSegBytes, bytes - off);
        uint8_t *seg = static_cast<uint8_t *>(segs[k]);
        void *d = to_user ? static_cast<void *>(user + off) : static_cast<void *>(seg);
        const void *s = to_user ? static_cast<const void *>(seg) : static_cast<const void *>(user + off);
        const size_t zero = 0;
        if (!be->multi_gather(d, &s, &zero, &n, 1, -1, DType::U8, st)) return false;
    }
    return true;
}
} // namespace

int IpcArena::vote_impl(Client &c, uint64_t tag, uint64_t seq, bool device_ok, int device, size_t bytes, DType dtype,
                        ReduceOp op, const void *src, void *dst) {
    if (!wait_slot_free(c, seq)) {
        LOG(WARN) << "IPC: slot of op seq " << seq << " not released by a peer";
        return kAborted;
    }
    const uint32_t slot = static_cast<uint32_t>(seq % kSlots);
    OpPeerShm *mine = shm_->op(slot, static_cast<uint32_t>(rank_));
    DeviceBackend *be = device_backend();
    CommBuf *inb = nullptr, *outb = nullptr;
    bool in_direct = false, out_direct = false;
    if (map_failed_.load(std::memory_order_relaxed)) device_ok = false; // vote for the TCP ring from now on
    if (bytes > kIpcSegBytes * kIpcMaxSegs) device_ok = false;          // beyond the staged segments: TCP ring
    auto publish = [](const CommBuf *b, uint32_t &nsegs, uint64_t &off, uint64_t *raw,
                      uint8_t (*handles)[kIpcHandleBytes]) {
        nsegs = static_cast<uint32_t>(b->segs.size());
        off = 0;
        for (size_t k = 0; k < b->segs.size(); ++k) {
            raw[k] = reinterpret_cast<uint64_t>(b->segs[k]);
            std::memcpy(handles[k], b->handles[k].data(), kIpcHandleBytes);
        }
    };
    if (device_ok) {
        // Direct (zero-copy) access to the caller's buffers where that is fault-safe or opted into:
        //   * every ring member is a thread of this process: raw pointers (no process can die alone);
        //   * the buffer lies in shareable memory (shareable.hpp, VMM + fd): peers import it like a staged buffer;
        //   * PCCL_IPC_MODE=fast: hipIpc export of the caller's allocation.
        // An in-place op always stages its input: peers read the staged copy while results land in the caller's
        // buffer, and the copy is the abort backup (reference reduce.cpp:551-580 keeps a backup for src == dst too).
        const bool allow_direct = !env_flag("PCCL_IPC_NO_ZERO_COPY", false);
        const bool all_local = all_local_peers();
        auto direct = [&](const void *p, uint8_t *handle, uint64_t &off) {
            if (!allow_direct) return false;
            if (all_local) {
                std::memset(handle, 0, kIpcHandleBytes);
                off = 0;
                return true;
            }
            shareable::Share s;
            if (shareable::lookup(p, bytes, s) && s.device == device && s.size <= kIpcMaxExport) {
                std::memset(handle, 0, kIpcHandleBytes);
                std::memcpy(handle, &s.handle, sizeof(s.handle));
                off = s.offset;
                return true;
            }
            return !safe_mode() && export_user(const_cast<void *>(p), device, handle, off);
        };
        if (src != dst) in_direct = direct(src, mine->in_handle[0], mine->in_off);
        out_direct = direct(dst, mine->out_handle[0], mine->out_off);
        if (in_direct) {
            mine->in_segs = 1;
            mine->in_raw[0] = reinterpret_cast<uint64_t>(src);
        }
        if (out_direct) {
            mine->out_segs = 1;
            mine->out_raw[0] = reinterpret_cast<uint64_t>(dst);
        }
        if (!in_direct) {
            inb = acquire_buffer(bytes, device);
            if (!inb) {
                device_ok = false;
            } else {
                publish(inb, mine->in_segs, mine->in_off, mine->in_raw, mine->in_handle);
                // copy-in before the vote: a passed vote barrier means every peer's input is readable
                StreamLease stream(device);
                if (!stream.get() ||
                    !copy_staged(be, inb->segs, static_cast<uint8_t *>(const_cast<void *>(src)), bytes, false,
                                 stream.get()) ||
                    !be->stream_sync(stream.get())) {
                    LOG(ERR) << "IPC: copy-in of " << bytes << " bytes failed";
                    device_ok = false;
                }
                trace_mark("copy_in");
            }
        }
        if (device_ok && !out_direct) {
            outb = acquire_buffer(bytes, device);
            if (!outb) device_ok = false;
            else publish(outb, mine->out_segs, mine->out_off, mine->out_raw, mine->out_handle);
        }
    }
    mine->gpu_uid = device_ok ? be->device_uid(device) : 0;
    mine->vote = device_ok ? 1 : 0;
    mine->zero_copy = (in_direct ? 1u : 0u) | (out_direct ? 2u : 0u);
    mine->algo = push_algorithm() ? 0u : 1u;
    mine->device = device;
    mine->bytes = bytes;
    mine->dtype = static_cast<uint32_t>(dtype);
    mine->op = static_cast<uint32_t>(op);
    fault_stall("ipc_vote", seq);
    set_phase(seq, PH_VOTED);
    fault_point("ipc_vote", seq);

    std::vector<MapKey> pins;
    // abort after my vote was published: peers that passed the barrier may be reading my input / pushing into my
    // output; once none can, restore an in-place caller buffer from the staged original and recycle everything
    auto abort_voted = [&](int code) {
        set_phase(seq, PH_ABORTED);
        drain_peers(c, seq);
        if (device_ok && inb && src == dst && out_direct) {
            StreamLease stream(device);
            if (stream.get() && copy_staged(be, inb->segs, static_cast<uint8_t *>(dst), bytes, true, stream.get()))
                be->stream_sync(stream.get());
        }
        unpin_mappings(pins);
        quarantine_buffer(inb, seq);
        quarantine_buffer(outb, seq);
        return code;
    };
    const int rc = barrier(c, tag, seq, PH_VOTED);
    if (rc != 0) {
        LOG(WARN) << "IPC: vote barrier failed (rc " << rc << ")";
        return abort_voted(rc == 2 ? kAbortedByMaster : kAborted);
    }
    bool all = true;
    for (size_t k = 0; k < ring_.size(); ++k) {
        const OpPeerShm *p = shm_->op(slot, static_cast<uint32_t>(k));
        all = all && p->vote == 1 && p->bytes == bytes && p->dtype == static_cast<uint32_t>(dtype) &&
              p->op == static_cast<uint32_t>(op) && p->algo == mine->algo && p->in_segs >= 1 &&
              p->in_segs <= kIpcMaxSegs &&
              p->out_segs >= 1 && p->out_segs <= kIpcMaxSegs;
    }
    if (!all) {
        set_phase(seq, PH_RELEASED);
        release_buffer(inb);
        release_buffer(outb);
        return kUseRing;
    }
    {
        std::vector<uint64_t> uids(ring_.size());
        for (size_t k = 0; k < ring_.size(); ++k) uids[k] = shm_->op(slot, static_cast<uint32_t>(k))->gpu_uid;
        const int bad = ipc_unreachable_peer(
            uids, rank_, device, [be](uint64_t u) { return be->device_of_uid(u); },
            [be](int d, int p) { return be->can_access_peer(d, p); });
        if (bad >= 0) {
            LOG(ERR) << "IPC: GPU of peer " << bad << " is not peer-accessible from device " << device
                     << "; using the TCP ring for later ops";
            map_failed_.store(true, std::memory_order_relaxed);
            return abort_voted(kAborted);
        }
        // peers in this process are reached through raw pointers (possibly plain hipMalloc memory of another GPU):
        // my kernels need peer access to their devices
        for (size_t k = 0; k < ring_.size(); ++k) {
            if (k == rank_ || pids_[k] != pids_[rank_] || uids[k] == uids[rank_]) continue;
            const int pd = be->device_of_uid(uids[k]);
            if (pd < 0 || !be->enable_peer_access(device, pd)) {
                LOG(ERR) << "IPC: cannot enable peer access from device " << device << " to the GPU of peer " << k
                         << "; using the TCP ring for later ops";
                map_failed_.store(true, std::memory_order_relaxed);
                return abort_voted(kAborted);
            }
        }
    }
    OpCtx ctx;
    ctx.bytes = bytes;
    ctx.in_buf = inb;
    ctx.out_buf = outb;
    ctx.in_staged = !in_direct;
    ctx.out_staged = !out_direct;
    ctx.in.resize(ring_.size());
    ctx.out.resize(ring_.size());
    for (size_t k = 0; k < ring_.size(); ++k) {
        const OpPeerShm *p = shm_->op(slot, static_cast<uint32_t>(k));
        const bool local = k == rank_ || pids_[k] == pids_[rank_]; // same process (threaded peers): raw pointers
        auto view = [&](uint32_t nsegs, uint64_t off, const uint64_t *raw, const uint8_t (*handles)[kIpcHandleBytes],
                        PeerView &v) {
            for (uint32_t j = 0; j < nsegs; ++j) {
                if (local) {
                    v.seg.push_back(reinterpret_cast<uint8_t *>(raw[j]));
                    continue;
                }
                MapKey key;
                auto *base = static_cast<uint8_t *>(pin_mapping(static_cast<int>(k), handles[j], device, key));
                if (!base) return false;
                pins.push_back(key);
                v.seg.push_back(base + (nsegs == 1 ? off : 0));
            }
            return true;
        };
        if (!view(p->in_segs, p->in_off, p->in_raw, p->in_handle, ctx.in[k]) ||
            !view(p->out_segs, p->out_off, p->out_raw, p->out_handle, ctx.out[k])) {
            // e.g. no peer access between these GPUs: this op aborts (every peer sees ABORTED), and this peer
            // votes against the xGMI path from now on, so the ring falls back to TCP instead of failing every op
            LOG(ERR) << "IPC: cannot map the buffers of peer " << k << "; using the TCP ring for later ops";
            map_failed_.store(true, std::memory_order_relaxed);
            return abort_voted(kAborted);
        }
        if (PCCL_LOG_ENABLED(DEBUG)) {
            LOG(DEBUG) << "IPC seq " << seq << " peer " << k << " pid " << pids_[k] << " in "
                       << static_cast<const void *>(ctx.in[k].seg[0]) << " (" << ctx.in[k].seg.size() << " segs) out "
                       << static_cast<const void *>(ctx.out[k].seg[0]) << " (" << ctx.out[k].seg.size()
                       << " segs) bytes " << bytes;
        }
    }
    ctx.pins = std::move(pins);
    ++g_buf_stats[in_direct ? 0 : 2];
    ++g_buf_stats[out_direct ? 1 : 3];
    // ordinary (non-shareable) tensors between processes: both directions staged, two extra full copies per op
    // (8 peers x 1 GiB: 12.7 vs 3.7 ms with shareable buffers, docs/PERFORMANCE.md); say so once per process
    if (!in_direct && !out_direct && src != dst && !all_local_peers()) {
        static std::once_flag warned;
        std::call_once(warned, [&] {
            LOG(WARN) << "IPC: all-reduce of " << bytes << " bytes between processes stages both input and output "
                      << "(the tensors are not in shareable memory); allocate them inside pccl_amd.memory."
                      << "shareable_memory() for zero-copy xGMI ops";
        });
    }
    {
        std::lock_guard l(g_ctx_mtx);
        g_ctx[{this, seq}] = std::move(ctx);
    }
    return kUseIpc;
}

bool IpcArena::preflight(Client &c, uint64_t tag, uint64_t seq, OpCtx &ctx, int device, DevStream st) {
    DeviceBackend *be = device_backend();
    const size_t W = ring_.size();
    constexpr size_t kSlot = 256;
    std::vector<uint32_t> pat(kSlot / 4);
    auto pattern = [&](size_t from) {
        for (size_t i = 0; i < pat.size(); ++i)
            pat[i] = 0x9e3779b9u * static_cast<uint32_t>(seq + 1) ^ static_cast<uint32_t>(from << 16 | i);
    };
    Lease src(device_pool(), kSlot, device);
    if (!src.ok()) return false;
    pattern(rank_);
    bool ok = be->memcpy_async(src.data(), pat.data(), kSlot, st) && be->stream_sync(st);
    for (size_t k = 0; k < W && ok; ++k) {
        if (k == rank_) continue;
        const void *s = src.data();
        const size_t zero = 0, n = kSlot;
        ok = be->multi_gather(ctx.out[k].at(rank_ * kSlot), &s, &zero, &n, 1, -1, DType::U8, st, true);
    }
    ok = ok && be->stream_sync(st);
    if (!ok) return false;
    set_phase(seq, PH_PROBED);
    if (barrier(c, tag, seq, PH_PROBED) != 0) return false;
    std::vector<uint32_t> got(W * kSlot / 4);
    if (!be->memcpy_async(got.data(), ctx.out[rank_].at(0), W * kSlot, st) || !be->stream_sync(st)) return false;
    for (size_t k = 0; k < W; ++k) {
        if (k == rank_) continue;
        pattern(k);
        if (std::memcmp(got.data() + k * kSlot / 4, pat.data(), kSlot) != 0) {
            LOG(ERR) << "IPC pre-flight: the probe of peer " << k << " did not arrive in my output buffer";
            return false;
        }
    }
    return true;
}

std::pair<bool, bool> IpcArena::run(Client &c, uint64_t tag, uint64_t seq, const void *src, void *dst, size_t count,
                                    DType dtype, ReduceOp op, int device, std::atomic<uint64_t> &tx,
                                    std::atomic<uint64_t> &rx, const InterHost *inter, size_t world,
                                    std::function<void(bool)> *settle) {
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
    auto *inb = static_cast<CommBuf *>(ctx.in_buf);
    auto *outb = static_cast<CommBuf *>(ctx.out_buf);
    DeviceBackend *be = device_backend();
    be->set_device(device);
    StreamLease stream(device);
    DevStream st = stream.get();
    const size_t W = ring_.size();
    const size_t es = dtype_size(dtype);
    const size_t bytes = ctx.bytes;
    const bool push = inter != nullptr || shm_->op(static_cast<uint32_t>(seq % kSlots), static_cast<uint32_t>(rank_))->algo == 0;

    auto finish = [&](int rc) -> std::pair<bool, bool> {
        if (rc != 0) {
            if (st) be->stream_sync(st); // my kernels are done: no further accesses from this peer
            set_phase(seq, PH_ABORTED);
            // peers may still be running kernels that read my input / write my output for this op: nothing is
            // restored, recycled or handed back to the caller before every live peer is past them
            drain_peers(c, seq);
            if (src == dst && ctx.in_staged && inb && st) { // restore the caller's buffer from the staged original
                copy_staged(be, inb->segs, static_cast<uint8_t *>(dst), bytes, true, st);
                be->stream_sync(st);
            }
        } else {
            set_phase(seq, PH_RELEASED);
        }
        unpin_mappings(ctx.pins);
        if (rc != 0) { // peers may have written into them for this op: never reissued (drain_peers is bounded)
            quarantine_buffer(inb, seq);
            quarantine_buffer(outb, seq);
        } else if (settle && src == dst && ctx.in_staged && inb) {
            // in place: the staged original stays until the master's verdict (restored if the op fails anyway)
            release_buffer(outb);
            *settle = [this, be, device, inb, dst, bytes](bool restore) {
                if (restore) {
                    be->set_device(device);
                    StreamLease s(device);
                    if (!s.get() || !copy_staged(be, inb->segs, static_cast<uint8_t *>(dst), bytes, true, s.get()) ||
                        !be->stream_sync(s.get())) {
                        LOG(ERR) << "IPC: could not restore the in-place input after a late abort";
                    }
                }
                release_buffer(inb);
            };
        } else {
            release_buffer(inb);
            release_buffer(outb);
        }
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
    // kernels run per piece of a byte range that does not cross a staged segment boundary (same for every peer)
    auto for_pieces = [&](size_t a_el, size_t n_el, const std::function<bool(size_t, size_t)> &fn) {
        for (size_t a = a_el * es, b = (a_el + n_el) * es; a < b;) {
            const size_t e = std::min(b, (a / kIpcSegBytes + 1) * kIpcSegBytes);
            if (!fn(a, e)) return false;
            a = e;
        }
        return true;
    };
    std::vector<const void *> srcs(W);
    std::vector<void *> dsts(W);
    // workgroup budget: 512 per GPU (2 per CU, the measured optimum for these streaming kernels), split between the
    // peers whose kernels run concurrently on this GPU, but not below 256 per kernel (fewer cannot saturate HBM)
    std::vector<uint64_t> uids(W);
    for (size_t k = 0; k < W; ++k) uids[k] = shm_->op(static_cast<uint32_t>(seq % kSlots), static_cast<uint32_t>(k))->gpu_uid;
    const int remote_grid = static_cast<int>(env_size("PCCL_IPC_REMOTE_GRID", 0)); // per op: bench phases switch it
    const int grid = ipc_push_grid(uids, rank_, remote_grid);
    // system-scope release at kernel end when a destination lives on another GPU, or is a staged buffer that the
    // copy-out reads with a copy engine: without it whole 4 KiB workgroup tiles of the result were still zero in the
    // copy (measured: test_device_ipc_modes, 6144 stale floats in 6 tiles of a 12 MB op)
    bool remote = false;
    for (size_t k = 0; k < W; ++k) {
        const OpPeerShm *p = shm_->op(static_cast<uint32_t>(seq % kSlots), static_cast<uint32_t>(k));
        remote = remote || uids[k] != uids[rank_] || !(p->zero_copy & 2u);
    }

    // Pre-flight on the first cross-GPU op of this arena: every peer writes a 256-byte pattern into slot `rank` of
    // every other peer's output through the same mappings the push kernels use (system-scope release), then reads
    // its own slots back. A write that did not land (wrong access flags on an imported allocation, a broken peer
    // mapping) fails this op and makes this peer vote for the TCP ring from now on, instead of every later op
    // producing wrong results; the kernels below overwrite the slots.
    if (ipc_needs_preflight(uids, preflight_done_, bytes)) {
        preflight_done_ = true;
        if (!preflight(c, tag, seq, ctx, device, st)) {
            ++g_buf_stats[6];
            map_failed_.store(true, std::memory_order_relaxed);
            LOG(ERR) << "IPC: cross-GPU pre-flight failed on device " << device << "; using the TCP ring for later ops";
            return finish(1);
        }
        ++g_buf_stats[7];
        trace_mark("preflight");
    }

    if (inter) {
        // hierarchical: host-local reduce of my shard into scratch, inter-host ring on the scratch, local push
        Lease part(device_pool(), std::max<size_t>(n[rank_] * es, 256), device);
        if (!part.ok()) return finish(1);
        uint8_t *pbase = part.data();
        const size_t b0 = lo[rank_] * es;
        const ReduceOp local_op = op == ReduceOp::Avg ? ReduceOp::Sum : op;
        const bool reduced = for_pieces(lo[rank_], n[rank_], [&](size_t a, size_t b) {
            for (size_t k = 0; k < W; ++k) srcs[k] = ctx.in[k].at(a);
            void *p = pbase + (a - b0);
            return be->multi_reduce(&p, 1, srcs.data(), static_cast<int>(W), (b - a) / es, dtype, local_op, st, grid);
        });
        if (!reduced || !be->stream_sync(st)) {
            LOG(ERR) << "IPC: host-local reduce failed";
            return finish(1);
        }
        trace_mark("local_reduce");
        if (int rc = (*inter)(pbase, n[rank_])) return finish(rc);
        trace_mark("inter_host");
        if (op == ReduceOp::Avg && n[rank_] > 0) be->finalize_avg(pbase, n[rank_], dtype, world, st);
        const bool bcast = for_pieces(lo[rank_], n[rank_], [&](size_t a, size_t b) {
            for (size_t k = 0; k < W; ++k) dsts[k] = ctx.out[k].at(a);
            const void *one = pbase + (a - b0);
            return be->multi_reduce(dsts.data(), static_cast<int>(W), &one, 1, (b - a) / es, dtype, ReduceOp::Sum, st,
                                    grid, remote);
        });
        if (!bcast || !be->stream_sync(st)) {
            LOG(ERR) << "IPC: host-local broadcast failed";
            return finish(1);
        }
        trace_mark("local_bcast");
    } else if (push) {
        // one-shot: read shard `rank` of every peer's input (inbound xGMI), reduce in fixed peer order and write the
        // result into every peer's output (outbound xGMI, posted writes) — reduce-scatter and all-gather overlap in
        // one kernel and one barrier; every peer receives the owner's bytes, so results are bit-identical
        const bool launched = for_pieces(lo[rank_], n[rank_], [&](size_t a, size_t b) {
            for (size_t k = 0; k < W; ++k) {
                srcs[k] = ctx.in[k].at(a);
                dsts[k] = ctx.out[k].at(a);
            }
            return be->multi_reduce(dsts.data(), static_cast<int>(W), srcs.data(), static_cast<int>(W), (b - a) / es,
                                    dtype, op, st, grid, remote);
        });
        fault_point("ipc_kernel", seq); // the kernels of every peer are in flight here
        if (!launched || !be->stream_sync(st)) {
            LOG(ERR) << "IPC: multi-source reduce + broadcast failed";
            return finish(1);
        }
        trace_mark("reduce_bcast");
    } else {
        // two-shot: reduce-scatter into my output, barrier, then pull every other shard (reads only)
        const bool reduced = for_pieces(lo[rank_], n[rank_], [&](size_t a, size_t b) {
            for (size_t k = 0; k < W; ++k) srcs[k] = ctx.in[k].at(a);
            void *d0 = ctx.out[rank_].at(a);
            return be->multi_reduce(&d0, 1, srcs.data(), static_cast<int>(W), (b - a) / es, dtype, op, st, grid,
                                    remote);
        });
        if (!reduced || !be->stream_sync(st)) {
            LOG(ERR) << "IPC: multi-source reduce failed";
            return finish(1);
        }
        trace_mark("reduce");
        set_phase(seq, PH_REDUCED);
        if (int rc = barrier(c, tag, seq, PH_REDUCED)) return finish(rc);
        trace_mark("reduced_barrier");
        bool gathered = true;
        for (size_t k = 0; k < W && gathered; ++k) {
            if (k == rank_) continue;
            gathered = for_pieces(lo[k], n[k], [&](size_t a, size_t b) {
                const void *s = ctx.out[k].at(a);
                const size_t off = 0, cnt = (b - a) / es;
                return be->multi_gather(ctx.out[rank_].at(a), &s, &off, &cnt, 1, -1, dtype, st, ctx.out_staged);
            });
        }
        if (!gathered || !be->stream_sync(st)) {
            LOG(ERR) << "IPC: gather failed";
            return finish(1);
        }
        trace_mark("gather");
    }
    set_phase(seq, PH_GATHERED);
    if (int rc = barrier(c, tag, seq, PH_GATHERED)) return finish(rc);
    trace_mark("gathered_barrier");
    if (ctx.out_staged) { // the caller's receive buffer could not be exported: copy the assembled result out
        if (!copy_staged(be, outb->segs, static_cast<uint8_t *>(dst), bytes, true, st) || !be->stream_sync(st)) {
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
                         op.tx, op.rx, nullptr, 0, &op.settle);
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
        inner.shape = op.shape;
        if (inner.req.op == ReduceOp::Avg) inner.req.op = ReduceOp::Sum; // divided by the whole world afterwards
        const auto r = ring_reduce_device(inner, sub, seq, device);
        op.tx += inner.tx.load();
        op.rx += inner.rx.load();
        return r.first && !r.second ? 0 : (r.second ? 2 : 1);
    };
    return h.arena->run(*this, op.req.tag, seq, op.req.src, op.req.dst, op.req.count, op.req.dtype, op.req.op, device,
                        op.tx, op.rx, &inter, rv.ring.size(), &op.settle);
}

} // namespace pccl::client

extern "C" __attribute__((visibility("default"))) void pcclxIpcStats(uint64_t *out4) {
    for (int k = 0; k < 4; ++k) out4[k] = pccl::client::g_buf_stats[k].load(std::memory_order_relaxed);
}

// All counters (see g_buf_stats); returns how many exist (writes at most n).
extern "C" __attribute__((visibility("default"))) size_t pcclxIpcStatsEx(uint64_t *out, size_t n) {
    constexpr size_t kN = sizeof(pccl::client::g_buf_stats) / sizeof(pccl::client::g_buf_stats[0]);
    for (size_t k = 0; k < n && k < kN; ++k) out[k] = pccl::client::g_buf_stats[k].load(std::memory_order_relaxed);
    return kN;
}
