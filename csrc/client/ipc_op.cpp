// xGMI/IPC all-reduce of one op: the vote (every ring member agrees on the path, algorithm and buffers), the cross-GPU
// pre-flight, the push / two-shot kernels over the peers' mapped buffers, and the hierarchical (IPC inside hosts,
// TCP ring across them) variant. Arena lifecycle, comm buffers and barriers: ipc.cpp.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>

#include "../common/log.hpp"
#include "../common/trace.hpp"
#include "client.hpp"
#include "ipc_shm.hpp"
#include "pools.hpp"
#include "shareable.hpp"
#include "vmm_share.hpp"

namespace pccl::client {

using namespace std::chrono;
using namespace ipc_detail;

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
    mine->algo = push_algo_ ? 0u : 1u;
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
    OpPeerShm *mine = shm_->op(static_cast<uint32_t>(seq % kSlots), static_cast<uint32_t>(rank_));
    const bool push = inter != nullptr || mine->algo == 0;

    auto finish = [&](int rc) -> std::pair<bool, bool> {
        if (rc != 0) {
            if (st) be->stream_sync(st); // my kernels are done: no further accesses from this peer
            mine->launch.store(0, std::memory_order_release);
            set_phase(seq, PH_ABORTED);
            // peers may still be running kernels that read my input / write my output for this op: nothing is
            // restored, recycled or handed back to the caller before every live peer is past them
            drain_peers(c, seq);
            if (src == dst && ctx.in_staged && inb && st) { // restore the caller's buffer from the staged original
                copy_staged(be, inb->segs, static_cast<uint8_t *>(dst), bytes, true, st);
                be->stream_sync(st);
            }
        } else {
            mine->launch.store(0, std::memory_order_release);
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
    // Last check before the first kernel that touches other peers' buffers: a peer that was stopped (SIGSTOP, a
    // wedged call) after the vote barrier and resumed after the others gave up on the op - the master dropped it,
    // or a peer aborted - must not write into buffers they restored or reused. The launch window is published so
    // that survivors waiting for a stopped peer know whether it could still launch (drain_peers).
    mine->launch.store(seq + 1, std::memory_order_seq_cst);
    if (!c.master_.is_open()) return finish(1);
    for (size_t k = 0; k < W; ++k) {
        const uint64_t v = shm_->op(static_cast<uint32_t>(seq % kSlots), static_cast<uint32_t>(k))->phase.load();
        if ((v >> 8) > seq + 1 || ((v >> 8) == seq + 1 && (v & 0xff) == PH_ABORTED)) return finish(1);
    }
    if (c.abort_received(tag)) return finish(2);

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
    const int grid = ipc_push_grid(uids, rank_, remote_grid_);
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

// xGMI ops above kIpcMaxOpBytes (one arena op publishes at most kIpcMaxSegs staged 1 GiB segments per buffer): the
// op runs as consecutive sub-ops over element ranges of at most that size, each a complete arena op (vote, kernels,
// barriers) under its own sequence number seq + (i << kIpcSubSeqShift) in the op's slot - every peer derives the same
// split from the op's count, and a sub-op reuses the slot only after every peer released the previous one
// (wait_slot_free), so phase words stay ordered. MI355X holds 288 GB of HBM: such tensors used to drop to the TCP ring
// (~100x slower on one node). In place, each finished sub-op keeps its input backup until the master's verdict, and a
// sub-op that fails restores the ranges of the ones before it.
std::pair<bool, bool> Client::ipc_reduce_segmented(OpState &op, const RingView &rv, uint64_t seq, int device,
                                                   bool &use_ring) {
    use_ring = false;
    const size_t es = dtype_size(op.req.dtype);
    const size_t per = kIpcMaxOpBytes / es / 4096 * 4096; // elements per sub-op
    const size_t nsub = (op.req.count + per - 1) / per;
    std::vector<std::function<void(bool)>> settles;
    auto restore_done = [&] {
        for (auto &s : settles)
            if (s) s(true);
        settles.clear();
    };
    for (size_t i = 0; i < nsub; ++i) {
        const size_t lo = i * per, n = std::min(per, op.req.count - lo);
        OpState sub;
        sub.req = op.req;
        sub.req.src = static_cast<const uint8_t *>(op.req.src) + lo * es;
        sub.req.dst = static_cast<uint8_t *>(op.req.dst) + lo * es;
        sub.req.count = n;
        const uint64_t aseq = seq + (static_cast<uint64_t>(i) << kIpcSubSeqShift);
        const int decision = rv.arena->vote(*this, sub, aseq, true, device);
        if (decision == IpcArena::kUseRing && i == 0) {
            use_ring = true;
            return {false, false};
        }
        if (decision != IpcArena::kUseIpc) {
            LOG(WARN) << "IPC: sub-op " << i << " of " << nsub << " of op seq " << seq << " not run (decision "
                      << decision << ")";
            restore_done();
            return {false, decision == IpcArena::kAbortedByMaster || abort_received(op.req.tag)};
        }
        const auto r = rv.arena->run(*this, op.req.tag, aseq, sub.req.src, sub.req.dst, n, op.req.dtype, op.req.op,
                                     device, op.tx, op.rx, nullptr, 0, &sub.settle);
        if (!r.first || r.second) {
            restore_done();
            return r;
        }
        settles.push_back(std::move(sub.settle));
    }
    op.settle = [settles = std::move(settles)](bool restore) mutable {
        for (auto &s : settles)
            if (s) s(restore);
    };
    return {true, false};
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
    for (int k = 0; k < 4; ++k) out4[k] = pccl::client::ipc_detail::g_buf_stats[k].load(std::memory_order_relaxed);
}

// All counters (see g_buf_stats); returns how many exist (writes at most n).
extern "C" __attribute__((visibility("default"))) size_t pcclxIpcStatsEx(uint64_t *out, size_t n) {
    constexpr size_t kN = sizeof(pccl::client::ipc_detail::g_buf_stats) / sizeof(pccl::client::ipc_detail::g_buf_stats[0]);
    for (size_t k = 0; k < n && k < kN; ++k) out[k] = pccl::client::ipc_detail::g_buf_stats[k].load(std::memory_order_relaxed);
    return kN;
}

