// Private to the xGMI/IPC arena sources (ipc.cpp: arena lifecycle, comm buffers, mappings, phase barriers;
// ipc_op.cpp: the per-op vote, pre-flight and reduce): the shared-memory layout of an arena and per-process state.
#pragma once

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <climits>
#include <cstdint>
#include <map>
#include <mutex>
#include <vector>

#include "ipc.hpp"

namespace pccl::client::ipc_detail {
constexpr uint64_t kMagic = 0x5043434c49504332ull; // "PCCLIPC2" (layout version)
constexpr uint32_t kClosed = 0x80000000u;
constexpr uint32_t kSlots = 128; // ops in flight per ring (slot = seq % kSlots)
constexpr uint32_t kMaxWorld = 16;

constexpr uint32_t PH_VOTED = 1, PH_PROBED = 2, PH_REDUCED = 3, PH_GATHERED = 4, PH_RELEASED = 5, PH_ABORTED = 0xEE;

inline uint64_t fnv1a(const void *p, size_t n, uint64_t h = 1469598103934665603ull) {
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
inline int futex_wait32(std::atomic<uint64_t> *word, uint32_t expect, long timeout_us) {
    timespec ts{timeout_us / 1000000, (timeout_us % 1000000) * 1000};
    return static_cast<int>(::syscall(SYS_futex, reinterpret_cast<uint32_t *>(word), FUTEX_WAIT, expect, &ts,
                                      nullptr, 0));
}
inline void futex_wake_all(std::atomic<uint64_t> *word) {
    ::syscall(SYS_futex, reinterpret_cast<uint32_t *>(word), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}
} // namespace pccl::client::ipc_detail

namespace pccl::client {

using namespace ipc_detail;

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
    // seq + 1 from the moment this peer re-checked the op's aborts before its first kernel that touches other peers'
    // buffers until those kernels completed (IpcArena::run); 0 otherwise. A peer stopped (SIGSTOP) outside that
    // window will re-check on resume and never launch, so survivors need not wait for it (drain_peers).
    std::atomic<uint64_t> launch;
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

} // namespace pccl::client

namespace pccl::client::ipc_detail {

// per-process counters of how op buffers were handed to the peers (pcclxIpcStats): [0] direct inputs, [1] direct
// outputs, [2] staged inputs, [3] staged outputs
// [0..3] direct_in, direct_out, staged_in, staged_out; [4] comm buffers quarantined after an abort; [5] drains that
// waited for a dead peer's threads to finish tearing down its address space; [6] / [7] cross-GPU pre-flight probes
// failed / passed; [8] quarantined buffers reclaimed (no peer can still touch them); [9] quarantined VMM buffers
// freed beyond the quarantine cap
extern std::atomic<uint64_t> g_buf_stats[10];

// per-process bookkeeping
extern std::mutex g_ctx_mtx;
extern std::map<std::pair<const IpcArena *, uint64_t>, OpCtx> g_ctx;

bool pid_alive(int pid);
bool pid_quiesced(int pid);
// every thread of the process is stopped (job control / ptrace stop) or gone: it runs no code until resumed
bool pid_stopped(int pid);

} // namespace pccl::client::ipc_detail
