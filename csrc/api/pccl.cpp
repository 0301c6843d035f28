// Public C API (include/pccl.h). Same validation / result semantics as the reference src/pccl.cpp, implemented over
// pccl::client::Client and pccl::master::Master.
#include <cstddef>
#include "pccl.h"

#include <atomic>
#include <chrono>
#include <deque>
#include <cstring>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <vector>

#include "../client/client.hpp"
#include "../client/pools.hpp"
#include "../common/device_backend.hpp"
#include "../common/log.hpp"
#include "../master/master.hpp"

struct pcclComm_t {
    pcclCommCreateParams_t params{};
    std::unique_ptr<pccl::client::Client> client;
    // Control-plane calls (connect, topology update / optimisation, shared-state sync) drive one master dialogue at
    // a time. The reference asserts they stay on the creating thread (THREAD_GUARD); here a second concurrent call
    // is refused with pcclInvalidUsage instead of interleaving two dialogues.
    mutable std::mutex control;
};

#define PCCL_CONTROL_GUARD(comm)                                                                                       \
    std::unique_lock<std::mutex> control_guard((comm)->control, std::try_to_lock);                                     \
    if (!control_guard.owns_lock()) {                                                                                  \
        LOG(ERR) << __func__ << ": another control-plane call of this communicator is running on another thread";     \
        return pcclInvalidUsage;                                                                                       \
    }

struct pcclMasterInstanceState_t {
    std::unique_ptr<pccl::master::Master> master;
};

static std::atomic<bool> g_initialized{false};

#define PCCL_CHECK_INIT()                                                                                              \
    if (!g_initialized.load()) return pcclNotInitialized
#define PCCL_REQUIRE(cond, err)                                                                                        \
    if (!(cond)) return (err)

static std::optional<pccl::DType> to_dtype(pcclDataType_t t) {
    using pccl::DType;
    switch (t) {
        case pcclUint8: return DType::U8;
        case pcclInt8: return DType::I8;
        case pcclInt16: return DType::I16;
        case pcclUint16: return DType::U16;
        case pcclUint32: return DType::U32;
        case pcclInt32: return DType::I32;
        case pcclUint64: return DType::U64;
        case pcclInt64: return DType::I64;
        case pcclFloat16: return DType::F16;
        case pcclBFloat16: return DType::BF16;
        case pcclFloat: return DType::F32;
        case pcclDouble: return DType::F64;
        case pcclFloat8E4M3: return DType::F8E4M3;
        case pcclFloat8E5M2: return DType::F8E5M2;
    }
    return std::nullopt;
}

static std::optional<pccl::ReduceOp> to_op(pcclRedOp_t op) {
    switch (op) {
        case pcclSum: return pccl::ReduceOp::Sum;
        case pcclAvg: return pccl::ReduceOp::Avg;
        case pcclProd: return pccl::ReduceOp::Prod;
        case pcclMax: return pccl::ReduceOp::Max;
        case pcclMin: return pccl::ReduceOp::Min;
    }
    return std::nullopt;
}

static std::optional<pccl::QuantAlgo> to_qalgo(pcclQuantizationAlgorithm_t a) {
    switch (a) {
        case pcclQuantNone: return pccl::QuantAlgo::None;
        case pcclQuantMinMax: return pccl::QuantAlgo::MinMax;
        case pcclQuantZeroPointScale: return pccl::QuantAlgo::ZeroPointScale;
    }
    return std::nullopt;
}

extern "C" {

pcclResult_t pcclInit(void) {
    pccl::install_debug_backtrace_signal();
    g_initialized.store(true);
    return pcclSuccess;
}

size_t pcclDataTypeSize(pcclDataType_t datatype) {
    auto t = to_dtype(datatype);
    return t ? pccl::dtype_size(*t) : 0;
}

pcclResult_t pcclCreateCommunicator(const pcclCommCreateParams_t *params, pcclComm_t **comm_out) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(params != nullptr && comm_out != nullptr, pcclInvalidArgument);
    auto *c = new pcclComm_t();
    c->params = *params;
    *comm_out = c;
    return pcclSuccess;
}

pcclResult_t pcclGetAttribute(const pcclComm_t *comm, pcclAttribute_t attribute, int *out) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(comm != nullptr && out != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(comm->client != nullptr, pcclInvalidUsage);
    auto &c = *comm->client;
    switch (attribute) {
        case PCCL_ATTRIBUTE_GLOBAL_WORLD_SIZE: *out = static_cast<int>(c.global_world_size()); break;
        case PCCL_ATTRIBUTE_PEER_GROUP_WORLD_SIZE: *out = static_cast<int>(c.local_world_size()); break;
        case PCCL_ATTRIBUTE_NUM_DISTINCT_PEER_GROUPS: *out = static_cast<int>(c.num_distinct_groups()); break;
        case PCCL_ATTRIBUTE_LARGEST_PEER_GROUP_WORLD_SIZE: *out = static_cast<int>(c.largest_group_size()); break;
        case PCCL_ATTRIBUTE_CONNECTION_REVISION: *out = static_cast<int>(c.connection_revision()); break;
        case PCCL_ATTRIBUTE_RING_RANK: *out = c.ring_rank(); break;
        case PCCL_ATTRIBUTE_LAST_REDUCE_PATH: *out = c.last_reduce_path(); break;
        case PCCL_ATTRIBUTE_COLLECTIVE_WORKER_THREADS: *out = static_cast<int>(c.collective_worker_threads()); break;
        case PCCL_ATTRIBUTE_LAST_REDUCE_FRAMING: *out = c.last_reduce_framing(); break;
        case PCCL_ATTRIBUTE_MASTER_CONNECTED: *out = c.master_connected() ? 1 : 0; break;
        default: return pcclInvalidArgument;
    }
    return pcclSuccess;
}

pcclResult_t pcclDestroyCommunicator(pcclComm_t *comm) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(comm != nullptr, pcclInvalidArgument);
    if (comm->client) {
        comm->client->interrupt();
        comm->client->join();
    }
    delete comm;
    return pcclSuccess;
}

pcclResult_t pcclConnect(pcclComm_t *comm) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(comm != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(comm->client == nullptr, pcclInvalidUsage);
    PCCL_CONTROL_GUARD(comm);
    const auto &p = comm->params;
    pccl::client::ClientConfig cfg;
    cfg.master = p.master_address;
    cfg.peer_group = p.peer_group;
    cfg.pool_size = std::max(1u, p.p2p_connection_pool_size);
    cfg.p2p_port = p.internal_p2p_listen_port;
    cfg.ss_port = p.internal_shared_state_listen_port;
    cfg.bm_port = p.internal_benchmark_listen_port;
    cfg.explicit_addresses = p.use_explicit_p2p_addresses;
    cfg.adv_p2p = p.advertised_p2p_address;
    cfg.adv_ss = p.advertised_shared_state_address;
    cfg.adv_bm = p.advertised_benchmark_address;
    comm->client = std::make_unique<pccl::client::Client>(cfg);
    if (!comm->client->connect()) {
        comm->client->interrupt();
        comm->client->join();
        comm->client.reset();
        return pcclMasterConnectionFailed;
    }
    return pcclSuccess;
}

pcclResult_t pcclUpdateTopology(pcclComm_t *comm) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(comm != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(comm->client != nullptr, pcclInvalidUsage);
    PCCL_CONTROL_GUARD(comm);
    if (comm->client->any_collective_running()) return pcclPendingAsyncOps;
    if (!comm->client->update_topology()) return pcclUpdateTopologyFailed;
    return pcclSuccess;
}

pcclResult_t pcclArePeersPending(const pcclComm_t *comm, bool *pending_out) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(comm != nullptr && pending_out != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(comm->client != nullptr, pcclInvalidUsage);
    bool pending = false;
    if (!comm->client->are_peers_pending(pending)) return pcclInvalidUsage;
    *pending_out = pending;
    return pcclSuccess;
}

pcclResult_t pcclOptimizeTopology(const pcclComm_t *comm) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(comm != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(comm->client != nullptr, pcclInvalidUsage);
    PCCL_CONTROL_GUARD(comm);
    if (comm->client->global_world_size() <= 1) return pcclInvalidUsage;
    if (comm->client->any_collective_running()) return pcclPendingAsyncOps;
    if (!comm->client->optimize_topology()) return pcclTopologyOptimizationFailed;
    return pcclSuccess;
}

// Validates and starts one all-reduce. `inline_run` executes the op on the calling thread (blocking pcclAllReduce:
// no hand-off to a worker thread on the latency-critical path); otherwise a collective worker thread runs it.
// `stream` (optional, device buffers): the op's input is ready once the work queued on it so far has completed.
static pcclResult_t start_all_reduce(const void *sendbuff, void *recvbuff, const pcclReduceDescriptor_t *descriptor,
                                     const pcclComm_t *comm, pcclAsyncReduceOp_t *handle_out, bool inline_run,
                                     void *const *stream = nullptr) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(comm != nullptr && descriptor != nullptr && handle_out != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(comm->client != nullptr, pcclInvalidUsage);
    // a zero-length op is legal (every peer still runs the protocol; empty tensors have null data pointers)
    PCCL_REQUIRE((sendbuff != nullptr && recvbuff != nullptr) || descriptor->count == 0, pcclInvalidArgument);
    auto dt = to_dtype(descriptor->src_descriptor.datatype);
    auto op = to_op(descriptor->op);
    auto qa = to_qalgo(descriptor->quantization_options.algorithm);
    PCCL_REQUIRE(dt && op && qa, pcclInvalidArgument);
    auto qt = *qa == pccl::QuantAlgo::None ? dt : to_dtype(descriptor->quantization_options.quantized_datatype);
    PCCL_REQUIRE(qt.has_value(), pcclInvalidArgument);
    // fp8 / float data types can only be the *wire* type of a quantized op, and reductions of fp8 data are undefined
    PCCL_REQUIRE(*dt != pccl::DType::F8E4M3 && *dt != pccl::DType::F8E5M2, pcclInvalidArgument);
    if (*qa != pccl::QuantAlgo::None && *qt != *dt && !pccl::kernels::quant_supported(*dt, *qt, *qa))
        return pcclInvalidArgument;
    if (comm->client->local_world_size() < 2) return pcclTooFewPeers;
    pccl::client::ReduceRequest req;
    req.src = sendbuff;
    req.dst = recvbuff;
    req.count = descriptor->count;
    req.dtype = *dt;
    req.qtype = *qt;
    req.qalgo = *qt == *dt ? pccl::QuantAlgo::None : *qa;
    req.op = *op;
    req.tag = descriptor->tag;
    pccl::DeviceBackend *be = pccl::device_backend();
    if (stream != nullptr && be != nullptr && descriptor->count > 0) {
        pccl::DevPtrInfo pi{};
        // an event on the caller's stream marks the input's producers; the op waits for it, the caller does not. The
        // client records it on this thread right after the op's initiate packet went out (Client::arm_ready).
        // (Skipping it for an idle stream, checked with hipStreamQuery, saved ~20 us per small op but was followed
        // by a SIGSEGV inside that call on a peer thread once in three GPU suites, profiles/r5/full2/: not kept.)
        if (be->pointer_info(sendbuff, pi) && pi.is_device) {
            req.stream_ordered = true;
            req.ready_stream = static_cast<pccl::DevStream>(*stream);
        }
    }
    if (!comm->client->all_reduce_async(req, inline_run)) return pcclInvalidArgument;
    handle_out->comm = const_cast<pcclComm_t *>(comm);
    handle_out->tag = descriptor->tag;
    return pcclSuccess;
}

pcclResult_t pcclAllReduceAsync(const void *sendbuff, void *recvbuff, const pcclReduceDescriptor_t *descriptor,
                                const pcclComm_t *comm, pcclAsyncReduceOp_t *handle_out) {
    return start_all_reduce(sendbuff, recvbuff, descriptor, comm, handle_out, false);
}

pcclResult_t pcclAwaitAsyncReduce(const pcclAsyncReduceOp_t *handle, pcclReduceInfo_t *info_out) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(handle != nullptr && handle->comm != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(handle->comm->client != nullptr, pcclInvalidUsage);
    auto &c = *handle->comm->client;
    const bool ok = c.join_async_reduce(handle->tag);
    pccl::client::ReduceInfo info;
    const bool have_info = c.get_reduce_info(handle->tag, info);
    if (!ok) return pcclRankConnectionLost;
    if (info_out != nullptr) {
        if (!have_info) return pcclInvalidUsage;
        info_out->local_world_size = info.world_size;
        info_out->tx_bytes = info.tx_bytes;
        info_out->rx_bytes = info.rx_bytes;
    }
    return pcclSuccess;
}

pcclResult_t pcclAllReduce(const void *sendbuff, void *recvbuff, const pcclReduceDescriptor_t *descriptor,
                           const pcclComm_t *comm, pcclReduceInfo_t *info_out) {
    pcclAsyncReduceOp_t h{};
    const pcclResult_t r = start_all_reduce(sendbuff, recvbuff, descriptor, comm, &h, true);
    if (r != pcclSuccess) return r;
    return pcclAwaitAsyncReduce(&h, info_out);
}

pcclResult_t pcclxAllReduceAsyncOnStream(const void *sendbuff, void *recvbuff, const pcclReduceDescriptor_t *descriptor,
                                        const pcclComm_t *comm, void *hip_stream, pcclAsyncReduceOp_t *handle_out) {
    return start_all_reduce(sendbuff, recvbuff, descriptor, comm, handle_out, false, &hip_stream);
}

pcclResult_t pcclxAllReduceOnStream(const void *sendbuff, void *recvbuff, const pcclReduceDescriptor_t *descriptor,
                                   const pcclComm_t *comm, void *hip_stream, pcclReduceInfo_t *info_out) {
    pcclAsyncReduceOp_t h{};
    const pcclResult_t r = start_all_reduce(sendbuff, recvbuff, descriptor, comm, &h, true, &hip_stream);
    if (r != pcclSuccess) return r;
    return pcclAwaitAsyncReduce(&h, info_out);
}

pcclResult_t pcclAllReduceMultipleWithRetry(const pcclReduceOpDescriptor_t *descriptors, size_t count,
                                            const pcclComm_t *comm, pcclReduceInfo_t *info_out, int max_in_flight) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(descriptors != nullptr && count > 0 && comm != nullptr && max_in_flight > 0, pcclInvalidArgument);
    PCCL_REQUIRE(comm->client != nullptr, pcclInvalidUsage);
    auto &c = *comm->client;
    if (c.local_world_size() < 2) return pcclTooFewPeers;

    // Sliding window (reference src/pccl.cpp:345-523): keep up to max_in_flight ops running, launch the next pending
    // op (in index order, so every peer issues the same tag sequence) as soon as ANY in-flight op completes (the
    // reference awaits the oldest one, so one slow op holds back every launch behind it);
    // on a failure drain every in-flight op (their successes count), then relaunch everything still pending on the
    // re-formed ring.
    uint64_t total_tx = 0, total_rx = 0;
    std::vector<bool> completed(count, false);
    size_t n_completed = 0;
    std::deque<size_t> pending, in_flight;
    for (size_t i = 0; i < count; ++i) pending.push_back(i);
    auto handle_of = [&](size_t i) {
        return pcclAsyncReduceOp_t{const_cast<pcclComm_t *>(comm), descriptors[i].descriptor.tag};
    };
    auto await_one = [&](size_t i) {
        pcclAsyncReduceOp_t h = handle_of(i);
        pcclReduceInfo_t info{};
        if (pcclAwaitAsyncReduce(&h, &info) != pcclSuccess) return false;
        completed[i] = true;
        ++n_completed;
        total_tx += info.tx_bytes;
        total_rx += info.rx_bytes;
        return true;
    };
    while (n_completed < count && c.local_world_size() >= 2) {
        while (in_flight.size() < static_cast<size_t>(max_in_flight) && !pending.empty()) {
            const size_t i = pending.front();
            const auto &d = descriptors[i];
            pcclAsyncReduceOp_t h{};
            const pcclResult_t r = pcclAllReduceAsync(d.sendbuf, d.recvbuf, &d.descriptor, comm, &h);
            if (r == pcclTooFewPeers) break;
            if (r != pcclSuccess) {
                for (size_t j : in_flight) await_one(j);
                return r;
            }
            pending.pop_front();
            in_flight.push_back(i);
        }
        if (in_flight.empty()) break;
        // the first in-flight op to complete (not the oldest: a slow op must not stall the launches behind it)
        std::vector<uint64_t> tags;
        for (size_t j : in_flight) tags.push_back(descriptors[j].descriptor.tag);
        std::optional<uint64_t> done;
        while (!(done = c.wait_any(tags, std::chrono::milliseconds(1000))) && c.local_world_size() >= 2) {
        }
        auto pos = in_flight.begin();
        if (done)
            while (pos != in_flight.end() && descriptors[*pos].descriptor.tag != *done) ++pos;
        if (pos == in_flight.end()) pos = in_flight.begin();
        const size_t i = *pos;
        in_flight.erase(pos);
        if (await_one(i)) continue;
        LOG(WARN) << "pcclAllReduceMultipleWithRetry: all-reduce tag " << descriptors[i].descriptor.tag
                  << " failed; draining " << in_flight.size() << " in-flight ops and retrying";
        for (size_t j : in_flight) await_one(j);
        in_flight.clear();
        pending.clear();
        for (size_t j = 0; j < count; ++j)
            if (!completed[j]) pending.push_back(j);
    }
    if (info_out != nullptr) {
        info_out->local_world_size = static_cast<uint32_t>(c.local_world_size());
        info_out->tx_bytes = total_tx;
        info_out->rx_bytes = total_rx;
    }
    return n_completed == count ? pcclSuccess : pcclTooFewPeers;
}

pcclResult_t pcclSynchronizeSharedState(const pcclComm_t *comm, pcclSharedState_t *shared_state,
                                        pcclSharedStateSyncStrategy_t strategy,
                                        pcclSharedStateSyncInfo_t *sync_info_out) {
    PCCL_CHECK_INIT();
    PCCL_REQUIRE(comm != nullptr && shared_state != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(comm->client != nullptr, pcclInvalidUsage);
    PCCL_CONTROL_GUARD(comm);
    if (comm->client->any_collective_running()) return pcclPendingAsyncOps;
    pccl::client::SharedState ss;
    switch (strategy) {
        case PCCL_SHARED_STATE_SYNC_STRATEGY_ENFORCE_POPULAR: ss.strategy = pccl::SyncStrategy::EnforcePopular; break;
        case PCCL_SHARED_STATE_SYNC_STRATEGY_RECEIVE_ONLY: ss.strategy = pccl::SyncStrategy::RxOnly; break;
        case PCCL_SHARED_STATE_SYNC_STRATEGY_SEND_ONLY: ss.strategy = pccl::SyncStrategy::TxOnly; break;
        default: return pcclInvalidArgument;
    }
    ss.revision = shared_state->revision;
    std::set<std::string> keys;
    for (size_t i = 0; i < shared_state->count; ++i) {
        const pcclTensorInfo_t &t = shared_state->infos[i];
        PCCL_REQUIRE(t.name != nullptr && (t.data != nullptr || t.count == 0), pcclInvalidArgument);
        auto dt = to_dtype(t.datatype);
        PCCL_REQUIRE(dt.has_value(), pcclInvalidArgument);
        PCCL_REQUIRE(t.device_type == pcclDeviceCpu || t.device_type == pcclDeviceHip, pcclInvalidArgument);
        if (t.device_type == pcclDeviceHip && !pccl::device_backend_available()) {
            LOG(WARN) << "GPU shared state entry '" << t.name << "' but the HIP backend is unavailable";
            return pcclInvalidArgument;
        }
        PCCL_REQUIRE(keys.insert(t.name).second, pcclInvalidArgument); // duplicate keys
        pccl::client::SSEntry e;
        e.key = t.name;
        e.dtype = *dt;
        e.device = t.device_type == pcclDeviceCpu ? pccl::DeviceType::Cpu : pccl::DeviceType::Gpu;
        e.data = t.data;
        e.count = t.count;
        e.bytes = t.count * pccl::dtype_size(*dt);
        e.allow_content_inequality = t.allow_content_inequality;
        ss.entries.push_back(e);
    }
    pccl::client::SSInfo info;
    if (!comm->client->sync_shared_state(ss, info)) return pcclInvalidUsage;
    shared_state->revision = ss.revision;
    if (sync_info_out != nullptr) {
        sync_info_out->tx_bytes = info.tx_bytes;
        sync_info_out->rx_bytes = info.rx_bytes;
    }
    return pcclSuccess;
}

pcclResult_t pcclCreateMaster(ccoip_socket_address_t listen_address, pcclMasterInstance_t **out) {
    PCCL_REQUIRE(out != nullptr, pcclInvalidArgument);
    auto *m = new pcclMasterInstanceState_t();
    m->master = std::make_unique<pccl::master::Master>(listen_address);
    *out = m;
    return pcclSuccess;
}

// Extension: the master's bandwidth stores as text ("<group> <from> -> <to>: <Mbit/s> Mbit/s" per line). Writes at
// most cap bytes (NUL-terminated when cap > 0); returns the full length.
extern "C" __attribute__((visibility("default"))) size_t pcclxMasterBandwidthTable(pcclMasterInstance_t *m, char *buf,
                                                                                  size_t cap) {
    if (m == nullptr || m->master == nullptr) return 0;
    const std::string t = m->master->bandwidth_table();
    if (cap > 0) {
        const size_t n = std::min(cap - 1, t.size());
        std::memcpy(buf, t.data(), n);
        buf[n] = 0;
    }
    return t.size();
}

// topology optimization counters of the master (pccl::master::Master::topology_stats); returns how many it wrote
extern "C" __attribute__((visibility("default"))) size_t pcclxMasterTopologyStats(pcclMasterInstance_t *m,
                                                                                  uint64_t *out, size_t n) {
    if (m == nullptr || m->master == nullptr || out == nullptr) return 0;
    const auto s = m->master->topology_stats();
    const size_t k = std::min(n, s.size());
    for (size_t i = 0; i < k; ++i) out[i] = s[i];
    return k;
}

// liveness counters of the master (pccl::master::Master::liveness_stats); returns how many it wrote
extern "C" __attribute__((visibility("default"))) size_t pcclxMasterLivenessStats(pcclMasterInstance_t *m,
                                                                                  uint64_t *out, size_t n) {
    if (m == nullptr || m->master == nullptr || out == nullptr) return 0;
    const auto s = m->master->liveness_stats();
    const size_t k = std::min(n, s.size());
    for (size_t i = 0; i < k; ++i) out[i] = s[i];
    return k;
}

// liveness counters of a peer (pccl::client::Client::liveness_stats); returns how many it wrote
extern "C" __attribute__((visibility("default"))) size_t pcclxLivenessStats(const pcclComm_t *comm, uint64_t *out,
                                                                            size_t n) {
    if (comm == nullptr || comm->client == nullptr || out == nullptr) return 0;
    const auto s = comm->client->liveness_stats();
    const size_t k = std::min(n, s.size());
    for (size_t i = 0; i < k; ++i) out[i] = s[i];
    return k;
}

pcclResult_t pcclRunMaster(pcclMasterInstance_t *m) {
    PCCL_REQUIRE(m != nullptr && m->master != nullptr, pcclInvalidArgument);
    if (!m->master->launch()) return pcclInvalidUsage;
    return pcclSuccess;
}

pcclResult_t pcclInterruptMaster(pcclMasterInstance_t *m) {
    PCCL_REQUIRE(m != nullptr && m->master != nullptr, pcclInvalidArgument);
    if (!m->master->interrupt()) return pcclInvalidUsage;
    return pcclSuccess;
}

pcclResult_t pcclMasterAwaitTermination(pcclMasterInstance_t *m) {
    PCCL_REQUIRE(m != nullptr && m->master != nullptr, pcclInvalidArgument);
    if (!m->master->join()) return pcclInvalidUsage;
    return pcclSuccess;
}

pcclResult_t pcclDestroyMaster(pcclMasterInstance_t *m) {
    PCCL_REQUIRE(m != nullptr, pcclInvalidArgument);
    m->master.reset();
    delete m;
    return pcclSuccess;
}

pcclResult_t pcclGetBuildInfo(pcclBuildInfo_t *info) {
    PCCL_REQUIRE(info != nullptr, pcclInvalidArgument);
    pccl::DeviceBackend *be = pccl::device_backend();
    info->has_cuda_support = be != nullptr; // reference layout: exactly one bool is written
    return pcclSuccess;
}

pcclResult_t pcclGetBuildInfoEx(pcclBuildInfoEx_t *info) {
    PCCL_REQUIRE(info != nullptr, pcclInvalidArgument);
    PCCL_REQUIRE(info->struct_size >= offsetof(pcclBuildInfoEx_t, hip_device_count) + sizeof(int),
                 pcclInvalidArgument);
    pccl::DeviceBackend *be = pccl::device_backend();
    info->has_cuda_support = be != nullptr;
    info->has_hip_support = be != nullptr;
    info->hip_device_count = be ? be->device_count() : 0;
    return pcclSuccess;
}

} // extern "C"
