/*
 * pccl.h — public C99 API of pccl-amd, an MI355X-native fault-tolerant collective communications library.
 *
 * ABI-compatible with the reference PCCL C API (include/pccl.h of jundi69/pccl): every enum value, struct layout and
 * function signature of the reference is preserved so that existing C/C++ programs compile and link unchanged.
 * Extensions (all additive) are marked "[pccl-amd extension]":
 *   - HIP device memory is a first-class operand everywhere (pcclDeviceHip == pcclDeviceCuda == 1). All-reduce
 *     buffers may live in HBM; same-host peers exchange data over xGMI through IPC-mapped buffers, remote peers
 *     through pinned-host staging over TCP with reduction/quantization done by CDNA4 HIP kernels.
 *   - fp16/bf16 reduction and OCP fp8 (e4m3 / e5m2) as quantized wire types.
 *   - extra communicator attributes (connection revision, ring rank, data path of the last all-reduce).
 *   - pcclGetBuildInfoEx reports HIP support and the visible HIP device count (pcclBuildInfo_t itself keeps the
 *     reference's one-field layout: a caller built against the reference header allocates exactly that).
 */
#ifndef PCCL_AMD_PCCL_H
#define PCCL_AMD_PCCL_H

#include "ccoip_inet.h"

#ifdef __cplusplus
#include <cstddef>
#else
#include <stddef.h>
#include <stdbool.h>
#endif

#define PCCL_EXPORT __attribute__((visibility("default")))

#ifdef __cplusplus
extern "C" {
#endif

typedef enum pcclResult_t {
    pcclSuccess = 0,
    pcclNotInitialized = 1,
    pcclInternalError = 2,
    pcclInvalidArgument = 3,
    pcclInvalidUsage = 4,
    pcclTooFewPeers = 5,
    pcclMasterConnectionFailed = 6,
    pcclRankConnectionFailed = 7,
    pcclRankConnectionLost = 8,
    pcclNoSharedStateAvailable = 9,
    pcclPendingAsyncOps = 10,
    pcclUpdateTopologyFailed = 11,
    pcclTopologyOptimizationFailed = 12
} pcclResult_t;

typedef enum pcclDataType_t {
    pcclUint8 = 0,
    pcclInt8 = 1,
    pcclInt16 = 2,
    pcclUint16 = 3,
    pcclUint32 = 4,
    pcclInt32 = 5,
    pcclUint64 = 6,
    pcclInt64 = 7,
    pcclFloat16 = 8,
    pcclBFloat16 = 9,
    pcclFloat = 10,
    pcclDouble = 11,
    pcclFloat8E4M3 = 12, /* [pccl-amd extension] OCP fp8 e4m3fn (gfx950 native format) */
    pcclFloat8E5M2 = 13  /* [pccl-amd extension] OCP fp8 e5m2 */
} pcclDataType_t;

typedef enum pcclDeviceType_t {
    pcclDeviceCpu = 0,
    pcclDeviceCuda = 1, /* kept for source compatibility; means "GPU device memory" */
    pcclDeviceHip = 1   /* [pccl-amd extension] preferred spelling on ROCm */
} pcclDeviceType_t;

typedef enum pcclRedOp_t {
    pcclSum,
    pcclAvg,
    pcclProd,
    pcclMax,
    pcclMin
} pcclRedOp_t;

typedef enum pcclAttribute_t {
    /** Total number of peers part of the run */
    PCCL_ATTRIBUTE_GLOBAL_WORLD_SIZE = 1,
    /** Number of peers in the peer group that this peer is part of */
    PCCL_ATTRIBUTE_PEER_GROUP_WORLD_SIZE = 2,
    /** Number of distinct peer groups in the run */
    PCCL_ATTRIBUTE_NUM_DISTINCT_PEER_GROUPS = 3,
    /** Number of peers in the largest peer group */
    PCCL_ATTRIBUTE_LARGEST_PEER_GROUP_WORLD_SIZE = 4,
    /** [pccl-amd extension] number of successful p2p (re-)establishments so far */
    PCCL_ATTRIBUTE_CONNECTION_REVISION = 64,
    /** [pccl-amd extension] position of this peer in the current ring order (-1 if unknown) */
    PCCL_ATTRIBUTE_RING_RANK = 65,
    /** [pccl-amd extension] data path of the last completed all-reduce: 0 none, 1 host ring/TCP,
     *  2 device ring/TCP via pinned staging, 3 device xGMI/IPC (same host), 4 hierarchical (xGMI/IPC inside each
     *  host + one TCP ring per local rank across hosts) */
    PCCL_ATTRIBUTE_LAST_REDUCE_PATH = 66,
    /** [pccl-amd extension] worker threads of the async collective pool so far (bounded by
     *  PCCL_MAX_CONCURRENT_COLLECTIVE_OPS, default 16) */
    PCCL_ATTRIBUTE_COLLECTIVE_WORKER_THREADS = 67,
    /** [pccl-amd extension] wire framing of the last completed all-reduce: 0 none (no TCP data ring, e.g. xGMI/IPC),
     *  1 pccl-amd framing (agreed per op by every participant: striped connections, quantized lanes and metadata tag),
     *  2 reference framing (a participant without the extension, or PCCL_WIRE=reference) */
    PCCL_ATTRIBUTE_LAST_REDUCE_FRAMING = 68,
    /** [pccl-amd extension] 1 while the connection to the master is open; 0 once it is gone (the master dropped this
     *  peer - e.g. after it was stopped longer than PCCL_PEER_TIMEOUT_MS - or the master was lost). A peer at 0 can
     *  only destroy the communicator and join again as a new peer. */
    PCCL_ATTRIBUTE_MASTER_CONNECTED = 69
} pcclAttribute_t;

typedef enum pcclSharedStateSyncStrategy_t {
    /** Transmit and receive as necessary so that every peer ends with the most popular shared state.
     *  If one peer uses this strategy, all peers of the sync must use it. */
    PCCL_SHARED_STATE_SYNC_STRATEGY_ENFORCE_POPULAR = 0,
    /** Only receive. This peer's content never takes part in the popularity election. */
    PCCL_SHARED_STATE_SYNC_STRATEGY_RECEIVE_ONLY = 1,
    /** Only send. This peer's content must be the elected content; otherwise the master kicks the peer. */
    PCCL_SHARED_STATE_SYNC_STRATEGY_SEND_ONLY = 2,
} pcclSharedStateSyncStrategy_t;

typedef struct {
    ccoip_socket_address_t master_address;
    uint32_t peer_group;
    uint32_t p2p_connection_pool_size;

    /** If true, the advertised_* addresses below are what the master hands out to other peers. */
    bool use_explicit_p2p_addresses;
    ccoip_socket_address_t advertised_p2p_address;
    ccoip_socket_address_t advertised_shared_state_address;
    ccoip_socket_address_t advertised_benchmark_address;

    /** Ports this peer listens on (0.0.0.0 / [::]). Listeners bump to the next free port when taken. */
    uint16_t internal_p2p_listen_port;          /* default 48149 */
    uint16_t internal_shared_state_listen_port; /* default 48150 */
    uint16_t internal_benchmark_listen_port;    /* default 48151 */
} pcclCommCreateParams_t;

typedef struct pcclComm_t pcclComm_t;

typedef struct pcclRankInfo_t pcclRankInfo_t;

typedef struct pcclReduceInfo_t {
    /** World size used by the operation (number of participating peers if it completed). */
    uint32_t local_world_size;
    uint64_t tx_bytes;
    uint64_t rx_bytes;
} pcclReduceInfo_t;

typedef enum pcclDistributionHint_t {
    pcclDistributionNone = 0,
    pcclDistributionNormal = 1,
    pcclDistributionUniform = 2
} pcclDistributionHint_t;

typedef struct pcclReduceOperandDescriptor_t {
    pcclDataType_t datatype;
    pcclDistributionHint_t distribution_hint;
} pcclReduceOperandDescriptor_t;

typedef enum pcclQuantizationAlgorithm_t {
    pcclQuantNone = 0,
    pcclQuantMinMax = 1,
    pcclQuantZeroPointScale = 2
} pcclQuantizationAlgorithm_t;

typedef struct pcclQuantizationOptions_t {
    pcclDataType_t quantized_datatype;
    pcclQuantizationAlgorithm_t algorithm;
} pcclQuantizationOptions_t;

typedef struct pcclReduceDescriptor_t {
    size_t count;
    pcclRedOp_t op;
    uint64_t tag;
    pcclReduceOperandDescriptor_t src_descriptor;
    pcclQuantizationOptions_t quantization_options;
} pcclReduceDescriptor_t;

typedef struct pcclReduceSingleDescriptor_t {
    void *sendbuf;
    void *recvbuf;
    pcclReduceDescriptor_t descriptor;
} pcclReduceOpDescriptor_t;

typedef struct pcclAsyncReduceOp_t {
    pcclComm_t *comm;
    uint64_t tag;
} pcclAsyncReduceOp_t;

typedef struct pcclRankUuid_t {
    uint8_t data[16];
} pcclRankUuid_t;

typedef struct pcclTensorInfo_t {
    const char *name;
    void *data;
    size_t count;
    pcclDataType_t datatype;
    pcclDeviceType_t device_type;
    bool allow_content_inequality;
} pcclTensorInfo_t;

typedef struct pcclSharedState_t {
    uint64_t revision;
    size_t count;
    pcclTensorInfo_t *infos;
} pcclSharedState_t;

typedef struct pcclSharedStateSyncInfo_t {
    uint64_t tx_bytes;
    uint64_t rx_bytes;
} pcclSharedStateSyncInfo_t;

typedef struct pcclMasterInstanceState_t pcclMasterInstance_t;

typedef struct pcclBuildInfo_t {
    /** True if this build can operate on GPU device memory (name kept from the reference ABI). */
    bool has_cuda_support;
} pcclBuildInfo_t;

/** [pccl-amd extension] Extended build information (pcclGetBuildInfoEx). `struct_size` must be set by the caller to
 *  sizeof(pcclBuildInfoEx_t); fields beyond it are not written, so the struct can grow without breaking callers. */
typedef struct pcclBuildInfoEx_t {
    size_t struct_size;
    /** True if this build can operate on GPU device memory. */
    bool has_cuda_support;
    /** True if the HIP (ROCm) backend is compiled in and loadable. */
    bool has_hip_support;
    /** Number of HIP devices visible (0 if none / HIP unavailable). */
    int hip_device_count;
} pcclBuildInfoEx_t;

#define PCCL_NULLABLE /* nothing */

/** Initializes the library. Must be called before any other function (idempotent). */
PCCL_EXPORT pcclResult_t pcclInit(void);

/** Creates a communicator (no network activity until pcclConnect). */
PCCL_EXPORT pcclResult_t pcclCreateCommunicator(const pcclCommCreateParams_t *params, pcclComm_t **comm_out);

/** Reads a communicator attribute (see pcclAttribute_t). */
PCCL_EXPORT pcclResult_t pcclGetAttribute(const pcclComm_t *communicator, pcclAttribute_t attribute,
                                          int *p_attribute_out);

/** Destroys a communicator; blocks until its threads have exited. */
PCCL_EXPORT pcclResult_t pcclDestroyCommunicator(pcclComm_t *communicator);

/** Connects to the master and blocks until this peer has been accepted into the run. */
PCCL_EXPORT pcclResult_t pcclConnect(pcclComm_t *communicator);

/** Jointly (all peers) accepts pending peers and (re-)establishes ring connections. */
PCCL_EXPORT pcclResult_t pcclUpdateTopology(pcclComm_t *communicator);

/** Jointly (all peers) asks the master whether peers are waiting to be accepted. */
PCCL_EXPORT pcclResult_t pcclArePeersPending(const pcclComm_t *communicator, bool *pending_out);

/** Jointly measures pairwise bandwidth and re-orders the ring with an asymmetric TSP solver. */
PCCL_EXPORT pcclResult_t pcclOptimizeTopology(const pcclComm_t *communicator);

/** Blocking all-reduce. sendbuff/recvbuff may be host memory or HIP device memory (may alias). */
PCCL_EXPORT pcclResult_t pcclAllReduce(const void *sendbuff, void *recvbuff,
                                       const pcclReduceDescriptor_t *descriptor,
                                       const pcclComm_t *communicator,
                                       pcclReduceInfo_t *PCCL_NULLABLE reduce_info_out);

/** Asynchronous all-reduce; complete it with pcclAwaitAsyncReduce. Tags of in-flight ops must be distinct. */
PCCL_EXPORT pcclResult_t pcclAllReduceAsync(const void *sendbuff, void *recvbuff,
                                            const pcclReduceDescriptor_t *descriptor,
                                            const pcclComm_t *communicator,
                                            pcclAsyncReduceOp_t *reduce_handle_out);

/** Runs several all-reduces with at most max_in_flight outstanding; failed ones are retried on the re-formed ring
 *  until all succeed or the peer group shrinks to one peer (pcclTooFewPeers). */
PCCL_EXPORT pcclResult_t pcclAllReduceMultipleWithRetry(const pcclReduceOpDescriptor_t *descriptors,
                                                        size_t count,
                                                        const pcclComm_t *communicator,
                                                        pcclReduceInfo_t *PCCL_NULLABLE reduce_info_out,
                                                        int max_in_flight);

/** Waits for an async all-reduce. Returns pcclRankConnectionLost if it was aborted (peer loss); the ring is then
 *  re-established once so that a retry can run. */
PCCL_EXPORT pcclResult_t pcclAwaitAsyncReduce(const pcclAsyncReduceOp_t *reduce_handle,
                                              pcclReduceInfo_t *PCCL_NULLABLE reduce_info_out);

/** Jointly synchronizes the shared state (hash-popularity election, outdated peers pull from a distributor). */
PCCL_EXPORT pcclResult_t pcclSynchronizeSharedState(const pcclComm_t *communicator,
                                                    pcclSharedState_t *shared_state,
                                                    pcclSharedStateSyncStrategy_t strategy,
                                                    pcclSharedStateSyncInfo_t *PCCL_NULLABLE sync_info_out);

/** Creates a master (coordinator) instance listening on listen_address. */
PCCL_EXPORT pcclResult_t pcclCreateMaster(ccoip_socket_address_t listen_address,
                                          pcclMasterInstance_t **p_master_handle_out);

/** Starts the master's event loop thread (non-blocking). */
PCCL_EXPORT pcclResult_t pcclRunMaster(pcclMasterInstance_t *master_instance);

/** Asks the master's event loop to stop. */
PCCL_EXPORT pcclResult_t pcclInterruptMaster(pcclMasterInstance_t *master_instance);

/** Blocks until the master's event loop thread has exited. */
PCCL_EXPORT pcclResult_t pcclMasterAwaitTermination(pcclMasterInstance_t *master_instance);

/** Frees a master instance (after pcclMasterAwaitTermination). */
PCCL_EXPORT pcclResult_t pcclDestroyMaster(pcclMasterInstance_t *master_instance);

/** Reports build / backend information (reference layout: one bool). */
PCCL_EXPORT pcclResult_t pcclGetBuildInfo(pcclBuildInfo_t *info);

/** [pccl-amd extension] Extended build information; info->struct_size must be initialised by the caller. */
PCCL_EXPORT pcclResult_t pcclGetBuildInfoEx(pcclBuildInfoEx_t *info);

/** [pccl-amd extension] Size in bytes of a pcclDataType_t (0 for unknown). Fixes reference bug returning 0 for
 *  fp16/bf16/int16. */
PCCL_EXPORT size_t pcclDataTypeSize(pcclDataType_t datatype);

/** [pccl-amd extension] Stream-ordered all-reduce of HIP device buffers. The op reads its input after the work
 *  queued on `hip_stream` (a hipStream_t, NULL = the null stream) before this call - an event recorded on it, waited
 *  for by the op itself, so the caller's thread never synchronises the stream - and runs on a collective worker;
 *  await it with pcclAwaitAsyncReduce, which returns once the op's last device write has completed (the result is
 *  then visible to every stream). Host buffers: `hip_stream` is ignored (same as pcclAllReduceAsync). */
PCCL_EXPORT pcclResult_t pcclxAllReduceAsyncOnStream(const void *sendbuff, void *recvbuff,
                                                     const pcclReduceDescriptor_t *descriptor,
                                                     const pcclComm_t *communicator, void *hip_stream,
                                                     pcclAsyncReduceOp_t *reduce_handle_out);

/** [pccl-amd extension] Blocking form of pcclxAllReduceAsyncOnStream: the op runs on the calling thread, which
 *  waits only for the input's producers on `hip_stream` (not for the whole stream) after the master's commence. */
PCCL_EXPORT pcclResult_t pcclxAllReduceOnStream(const void *sendbuff, void *recvbuff,
                                                const pcclReduceDescriptor_t *descriptor,
                                                const pcclComm_t *communicator, void *hip_stream,
                                                pcclReduceInfo_t *reduce_info_out);

#ifdef __cplusplus
}
#endif

#endif /* PCCL_AMD_PCCL_H */
