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
#include "ipc_shm.hpp"

namespace pccl::client {

using namespace std::chrono;
using namespace ipc_detail;

namespace ipc_detail {
std::atomic<uint64_t> g_buf_stats[10];
std::mutex g_ctx_mtx;
std::map<std::pair<const IpcArena *, uint64_t>, OpCtx> g_ctx;
} // namespace ipc_detail

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
    arena->push_algo_ = push_algorithm_env();
    arena->remote_grid_ = static_cast<int>(env_size("PCCL_IPC_REMOTE_GRID", 0));
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
bool ipc_detail::pid_alive(int pid) {
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
bool ipc_detail::pid_quiesced(int pid) {
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

bool ipc_detail::pid_stopped(int pid) {
    char path[64];
    std::snprintf(path, sizeof(path), "/proc/%d/task", pid);
    DIR *d = ::opendir(path);
    if (!d) return false;
    bool stopped = true, any = false;
    while (dirent *e = ::readdir(d)) {
        if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
        const char st = proc_state(pid, std::atoi(e->d_name));
        if (st == 0 || st == 'Z' || st == 'X' || st == 'x') continue;
        any = true;
        if (st != 'T' && st != 't') {
            stopped = false;
            break;
        }
    }
    ::closedir(d);
    return stopped && any;
}

bool ipc_pid_quiesced_for_test(int pid) { return pid_quiesced(pid); }
bool ipc_pid_stopped_for_test(int pid) { return pid_stopped(pid); }
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

bool IpcArena::push_algorithm_env() {
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
            } else if (p->launch.load(std::memory_order_acquire) != seq + 1 && pid_stopped(pids_[k])) {
                // stopped before its pre-launch check: on resume it sees the abort and never launches (run)
                LOG(WARN) << "IPC: peer " << k << " (pid " << pids_[k] << ") is stopped outside its launch window of "
                          << "op seq " << seq << "; not waiting for it";
                break;
            }
            if (steady_clock::now() - t0 > timeout) {
                LOG(WARN) << "IPC: peer " << k << " did not finish op seq " << seq << " before the restore";
                break;
            }
            std::this_thread::sleep_for(microseconds(20));
        }
    }
}


} // namespace pccl::client
