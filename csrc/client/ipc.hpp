// Intra-node xGMI fast path.
//
// When every peer of a ring runs on this host (loopback run), the peers rendezvous in a POSIX shared-memory arena
// and exchange HIP IPC handles of their op buffers. An all-reduce whose buffers are on GPUs at every peer then runs
// as a direct-access collective instead of a TCP ring. Each peer publishes an *input* (the caller's send buffer, or a
// staged copy for in-place ops) and an *output* (the caller's receive buffer, or a staged comm buffer if it cannot be
// exported). Peer r owns shard r:
//   push (default, "one-shot"): one kernel reads shard r of every peer's input over xGMI (inbound), reduces in fixed
//     peer order with fp32 accumulation and writes the result into every peer's output (outbound, posted writes).
//     Reduce-scatter and all-gather overlap in one pass and use both directions of every link; one barrier.
//   two_shot (PCCL_IPC_ALGO=two_shot): reduce shard r into my output, barrier, then pull every other peer's shard.
// Either way every peer holds the owner's bytes for every shard (bit-identical results), all W-1 links of the fully
// connected MI355X node are used concurrently, and an op needs 1-2 kernel launches instead of 2(W-1) ring steps.
//
// Synchronization is a per-op barrier in shared memory keyed by the master-assigned sequence number (so concurrent
// ops with different tags proceed independently). Every wait is bounded and also watches the master's abort packet
// and the liveness of the peer processes, so a peer dying mid-collective aborts the op on all survivors
// (fault tolerance is preserved); a vote at the start of each op lets all peers agree on the data path.
//
// Exported allocations are at most kIpcMaxExport bytes: PyTorch's bundled ROCm 7.0 HIP runtime (the one every
// Python peer process runs on) never returns from hipIpcOpenMemHandle for an allocation of >= 2 GiB (ROCm 7.2 does;
// profiles/r2/ipc/). Staged comm buffers are therefore built from kIpcSegBytes segments, each exported separately,
// and kernels run in pieces that never cross a segment boundary (boundaries are multiples of kIpcSegBytes in op
// byte space, the same for every peer). User buffers in larger allocations are staged.
//
// Buffer lifetime under faults (PCCL_IPC_MODE, default "safe"): every exported buffer is a VMM allocation
// (hipMemCreate) shared as a POSIX fd (vmm_share.hpp); an importer maps it into its own address space and holds its own
// reference to the physical memory, so a peer SIGKILLed while the others' kernels read its input / write its output
// leaves valid memory behind (profiles/r2/ipc/vmm_exporter_death_probe.log). hipIpc handles of the caller's buffers
// are faster (no copy-in / copy-out) but a dead exporter's memory can vanish under a running kernel (GPU memory fault
// in the 8-peer kill + rejoin benchmark, profiles/r2/ipc/): "fast" opts into them. A mapping is pinned
// (reference-counted) by every op that uses it and is only closed when unpinned; after an abort a peer waits until
// every live peer is past its kernels for that op before it restores / releases buffers or returns.
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../common/device_backend.hpp"
#include "../common/types.hpp"

namespace pccl::client {

constexpr size_t kIpcSegBytes = size_t{1} << 30;                 // staged comm buffer segment
constexpr size_t kIpcMaxExport = (size_t{2} << 30) - (size_t{2} << 20); // largest user allocation exported as is
constexpr uint32_t kIpcMaxSegs = 16;                              // staged segments of one arena op
// Largest xGMI op handled in one arena op (16 GiB); larger ones run as consecutive sub-ops of at most this size
// (Client::ipc_reduce_segmented), sub-op i under arena sequence number seq + (i << kIpcSubSeqShift) in the op's slot
constexpr size_t kIpcMaxOpBytes = kIpcSegBytes * kIpcMaxSegs;
constexpr unsigned kIpcSubSeqShift = 40;

class Client;
struct ArenaShm;

// PCCL_IPC_MODE: "safe" (default) — buffers cross processes only as VMM allocations shared as fds (the importer keeps
// the pages alive if the exporter dies); "fast" — hipIpc exports of plain allocations are allowed too. Shared by the
// all-reduce arena and the same-host shared-state hand-off.
bool ipc_safe_mode();

// Workgroup budget of one xGMI kernel: 512 per GPU (2 per CU, the measured optimum for these streaming kernels,
// profiles/r1_ipc_grid_sweep.md) split between the ring members whose kernels run on the same physical GPU (same
// uid), but not below 256 per kernel (fewer cannot saturate HBM).
int ipc_grid_budget(const std::vector<uint64_t> &gpu_uids, size_t rank);

// Peer-access precheck of an IPC op: every ring member's GPU that is visible here (uid -> local ordinal) must be
// mappable from `my_device`; members on GPUs this process cannot see are left to hipIpcOpenMemHandle (its failure
// also falls back to the TCP ring). Returns the first member that fails, or -1.
int ipc_unreachable_peer(const std::vector<uint64_t> &gpu_uids, size_t rank, int my_device,
                         const std::function<int(uint64_t)> &device_of_uid,
                         const std::function<bool(int, int)> &can_access_peer);

// peer-process liveness as the IPC path sees it (exposed for the unit tests): alive = can still make protocol
// progress; quiesced = can no longer touch GPU memory (every thread past its address-space teardown)
bool ipc_pid_alive_for_test(int pid);
// Whether an op on this ring runs the cross-GPU pre-flight write probe (first op of an arena whose peers span more
// than one GPU and that is large enough to hold one 256-byte probe slot per peer); identical on every peer.
bool ipc_needs_preflight(const std::vector<uint64_t> &gpu_uids, bool done, size_t bytes);
// Workgroup budget of this peer's push kernel: ipc_grid_budget, or `remote_grid` (> 0, PCCL_IPC_REMOTE_GRID) when a
// destination lives on another GPU (remote xGMI writes and reads have more latency to cover).
int ipc_push_grid(const std::vector<uint64_t> &gpu_uids, size_t rank, int remote_grid);
bool ipc_pid_quiesced_for_test(int pid);
bool ipc_pid_stopped_for_test(int pid);

struct OpCtx; // per-op mapping context (ipc_shm.hpp)

class IpcArena {
public:
    // kAbortedByMaster: the vote barrier consumed the master's abort packet for this op (exactly one is sent per op,
    // so the caller must not wait for it again)
    static constexpr int kUseIpc = 1, kUseRing = 0, kAborted = -1, kAbortedByMaster = -2;
    using MapKey = std::tuple<int, std::array<uint8_t, kIpcHandleBytes>, int>; // (peer, handle, my device)
    std::atomic<bool> map_failed_{false}; // a peer's IPC handle could not be opened: stop voting for xGMI
    bool preflight_done_ = false;         // the cross-GPU write probe ran on this arena (first eligible op)

    static std::shared_ptr<IpcArena> create(Client &c, const std::vector<Uuid> &ring, uint16_t master_port,
                                            uint32_t group);
    ~IpcArena();

    bool matches(const std::vector<Uuid> &ring) const { return ring == ring_; }
    size_t world() const { return ring_.size(); }
    size_t rank() const { return rank_; }

    template<typename Op>
    int vote(Client &c, Op &op, uint64_t seq, bool device_ok, int device);

    // Inter-host stage of the hierarchical all-reduce: all-reduces (SUM / MIN / MAX / PROD, never AVG) `count`
    // elements of device scratch in place across hosts. Returns 0 ok, 1 failure, 2 master abort.
    using InterHost = std::function<int(void *part, size_t count)>;

    // Runs the IPC all-reduce for a voted op. Returns {success, aborted}.
    // With `inter` (hierarchical mode, this arena spans one host): reduce my local shard into scratch, all-reduce it
    // across hosts with `inter`, divide by `world` for AVG, then push it into every local peer's output.
    std::pair<bool, bool> run(Client &c, uint64_t tag, uint64_t seq, const void *src, void *dst, size_t count,
                              DType dtype, ReduceOp op, int device, std::atomic<uint64_t> &tx,
                              std::atomic<uint64_t> &rx, const InterHost *inter = nullptr, size_t world = 0,
                              std::function<void(bool)> *settle = nullptr);

    // internal (exposed for the vote template)
    int vote_impl(Client &c, uint64_t tag, uint64_t seq, bool device_ok, int device, size_t bytes, DType dtype,
                  ReduceOp op, const void *src, void *dst);

private:
    IpcArena() = default;
    // a staged comm buffer: `segs` allocations of kIpcSegBytes (one smaller allocation for small buffers)
    struct CommBuf {
        std::vector<void *> segs;
        std::vector<std::array<uint8_t, kIpcHandleBytes>> handles;
        std::vector<uint64_t> share_ids; // VMM mode: ids of the fds published with VmmShare (0 = hipIpc export)
        size_t cap = 0;
        int device = -1;
        bool busy = false;
        bool quarantined = false; // used by aborted op `qseq`: not handed out again until reclaimed
        uint64_t qseq = 0;
    };
    CommBuf *acquire_buffer(size_t bytes, int device);
    void release_buffer(CommBuf *b);
    // After an abort: the buffer stays busy, so a late write of a peer that the abort drain could not prove finished
    // lands in memory no later op uses. acquire_buffer reclaims it once no ring member can still touch it for that op
    // (op_quiet), and frees quarantined VMM buffers beyond kQuarantineCapBytes (a VMM importer holds its own
    // reference to the pages, so a late write lands in memory nobody reads).
    void quarantine_buffer(CommBuf *b, uint64_t seq);
    void reclaim_quarantined_locked();
    // every other ring member is provably past op `seq`: its phase word shows a later op in that slot, or the op at
    // PH_GATHERED / PH_RELEASED / PH_ABORTED, or no vote for it yet (it then sees my PH_ABORTED and never launches);
    // a dead member's threads have all left its address space (pid_quiesced)
    bool unquiet_peers_remote(uint64_t seq) const;
    bool op_quiet(uint64_t seq) const;
    struct Mapping {
        void *ptr = nullptr;
        bool vmm = false;  // imported VMM allocation (unmap) vs hipIpc mapping (close)
        int refs = 0;      // ops that hold this mapping (never closed while > 0)
        uint64_t used = 0; // LRU stamp
    };
    // opens (or reuses) peer `peer`'s allocation `handle` on `my_device` and pins it; nullptr on failure
    void *pin_mapping(int peer, const uint8_t *handle, int my_device, MapKey &key);
    void unpin_mappings(const std::vector<MapKey> &keys);
    // exports the allocation holding a user device buffer (zero-copy path); cached per allocation base
    bool export_user(void *p, int device, uint8_t handle[kIpcHandleBytes], uint64_t &offset);
    // waits until every peer reached `phase` for `seq`; 0 ok, 1 failure (peer dead/aborted/timeout), 2 master abort
    int barrier(Client &c, uint64_t tag, uint64_t seq, uint32_t phase);
    void wait_phase_change(std::atomic<uint64_t> *word, uint64_t seen, long timeout_us);
    bool all_local_peers() const; // every ring member is a thread of this process
    // cross-GPU write probe of one op (see run()); true if every peer's probe arrived in my output
    bool preflight(Client &c, uint64_t tag, uint64_t seq, OpCtx &ctx, int device, DevStream st);
    void set_phase(uint64_t seq, uint32_t phase);
    bool wait_slot_free(Client &c, uint64_t seq);
    // waits until no live peer can still write into my receive buffer for `seq` (push algorithm, abort path)
    void drain_peers(Client &c, uint64_t seq);
    // PCCL_IPC_ALGO: "push" (default, one-shot reduce + broadcast) or "two_shot" (reduce-scatter, then gather) and
    // PCCL_IPC_REMOTE_GRID, read once when the arena is created (a ring establishment), never on op threads: a
    // process that switches them (the bench's per-phase variants) does so between establishments, and the vote still
    // checks that every peer runs the same algorithm
    bool push_algo_ = true;
    int remote_grid_ = 0;
    static bool push_algorithm_env();
    // PCCL_IPC_MODE: "safe" (default: VMM-shared staging buffers only) or "fast" (hipIpc, zero-copy user buffers)
    static bool safe_mode();
    void release_mapping(const MapKey &key, Mapping &m);

    std::vector<Uuid> ring_;
    size_t rank_ = 0;
    std::string name_;
    ArenaShm *shm_ = nullptr;
    size_t shm_bytes_ = 0;
    std::vector<int> pids_;

    std::mutex mtx_;
    std::vector<std::unique_ptr<CommBuf>> bufs_;
    uint64_t next_buf_id_ = 1;
    // (peer, handle bytes, my device) -> mapped allocation base; handles identify allocations uniquely (a freed and
    // re-allocated block at the same address gets a new handle), so stale entries are merely unused
    std::map<MapKey, Mapping> mappings_;
    uint64_t map_clock_ = 0;
};

template<typename Op>
int IpcArena::vote(Client &c, Op &op, uint64_t seq, bool device_ok, int device) {
    return vote_impl(c, op.req.tag, seq, device_ok, device, op.req.count * dtype_size(op.req.dtype), op.req.dtype,
                     op.req.op, op.req.src, op.req.dst);
}

} // namespace pccl::client
