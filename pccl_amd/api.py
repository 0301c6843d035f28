"""User-facing Python API of pccl-amd.

Mirrors the reference Python API (python/framework/pccl/_pccl.py: Communicator, MasterNode, SharedState, TensorInfo,
ReduceOp, ... ) so existing scripts run unchanged, with one capability the reference lacks: tensors may live on the
GPU (``device.type == 'cuda'`` on ROCm) for all-reduce *and* shared state. Device all-reduces run on HBM through the
HIP backend (xGMI between peers on one host, pinned-memory staging over TCP otherwise).
"""
from __future__ import annotations

import ctypes
import functools
import importlib
import logging
import time
from enum import Enum
from ipaddress import IPv4Address, IPv6Address, ip_address
from typing import Dict, List, Optional, Tuple, Union

from . import _native
from ._native import C

logger = logging.getLogger("pccl_amd")


class _ModuleDummy:
    def __init__(self, name: str):
        self.name = name

    def __getattr__(self, item):
        raise RuntimeError(f"Module {self.name} is not available; install it to interoperate with pccl-amd.")


def _optional(name: str):
    """The module if importable, else a dummy (reference: numpy-only and torch-only installs both work)."""
    try:
        return importlib.import_module(name)
    except ImportError:
        return _ModuleDummy(name)


torch = _optional("torch")
np = _optional("numpy")


class Result(Enum):
    SUCCESS = 0
    NOT_INITIALIZED = 1
    INTERNAL_ERROR = 2
    INVALID_ARGUMENT = 3
    INVALID_USAGE = 4
    TOO_FEW_PEERS = 5
    MASTER_CONNECTION_FAILED = 6
    RANK_CONNECTION_FAILED = 7
    RANK_CONNECTION_LOST = 8
    NO_SHARED_STATE_AVAILABLE = 9
    PENDING_ASYNC_OPS = 10
    UPDATE_TOPOLOGY_FAILED = 11
    TOPOLOGY_OPTIMIZATION_FAILED = 12


class PCCLError(Exception):
    def __init__(self, result: Result, func_name: str):
        super().__init__(f"{func_name} failed with error: {result.name}")
        self.result = result

    @staticmethod
    def check(result: int, func_name: str):
        if result != Result.SUCCESS.value:
            raise PCCLError(Result(result), func_name)


PCCLError.check(C.pcclInit(), "pcclInit")


def build_info() -> Dict[str, object]:
    bi = _native.BuildInfoExC()
    bi.struct_size = ctypes.sizeof(bi)
    PCCLError.check(C.pcclGetBuildInfoEx(ctypes.byref(bi)), "pcclGetBuildInfoEx")
    return {"has_cuda_support": bool(bi.has_cuda_support), "has_hip_support": bool(bi.has_hip_support),
            "hip_device_count": int(bi.hip_device_count)}


class ReduceOp(Enum):
    SUM = 0
    AVG = 1
    PROD = 2
    MAX = 3
    MIN = 4


class Attribute(Enum):
    GLOBAL_WORLD_SIZE = 1
    LOCAL_WORLD_SIZE = 2
    PEER_GROUP_WORLD_SIZE = 2
    NUM_DISTINCT_PEER_GROUPS = 3
    LARGEST_PEER_GROUP_WORLD_SIZE = 4
    CONNECTION_REVISION = 64
    RING_RANK = 65
    LAST_REDUCE_PATH = 66
    COLLECTIVE_WORKER_THREADS = 67
    LAST_REDUCE_FRAMING = 68
    MASTER_CONNECTED = 69


class ReducePath(Enum):
    NONE = 0
    HOST_RING = 1
    DEVICE_RING = 2
    DEVICE_IPC = 3
    HIERARCHICAL = 4


class SharedStateSyncStrategy(Enum):
    ENFORCE_POPULAR = 0
    RECEIVE_ONLY = 1
    SEND_ONLY = 2


class DataType(Enum):
    UINT8 = 0
    INT8 = 1
    INT16 = 2
    UINT16 = 3
    UINT32 = 4
    INT32 = 5
    UINT64 = 6
    INT64 = 7
    FLOAT16 = 8
    BFLOAT16 = 9
    FLOAT = 10
    DOUBLE = 11
    FLOAT8_E4M3 = 12
    FLOAT8_E5M2 = 13

    def size(self) -> int:
        return int(C.pcclDataTypeSize(self.value))

    def to_torch_dtype(self):
        m = _torch_map()
        inv = {v: k for k, v in m.items()}
        if self not in inv:
            raise ValueError(f"Unsupported DataType: {self}")
        return inv[self]

    @classmethod
    def from_torch_dtype(cls, dtype) -> "DataType":
        m = _torch_map()
        if dtype not in m:
            raise ValueError(f"Unsupported dtype: {dtype}")
        return m[dtype]

    def to_numpy_dtype(self):
        m = {DataType.UINT8: np.uint8, DataType.INT8: np.int8, DataType.INT16: np.int16, DataType.UINT16: np.uint16,
             DataType.UINT32: np.uint32, DataType.INT32: np.int32, DataType.UINT64: np.uint64,
             DataType.INT64: np.int64, DataType.FLOAT16: np.float16, DataType.FLOAT: np.float32,
             DataType.DOUBLE: np.float64}
        if self not in m:
            raise ValueError(f"Unsupported DataType for numpy: {self}")
        return np.dtype(m[self])

    @classmethod
    def from_numpy_dtype(cls, dtype) -> "DataType":
        dt = dtype if isinstance(dtype, np.dtype) else np.dtype(dtype)
        m = _numpy_map()
        if dt not in m:
            raise ValueError(f"Unsupported dtype: {dtype}")
        return m[dt]


@functools.lru_cache(maxsize=None)
def _numpy_map():
    return {np.dtype(np.uint8): DataType.UINT8, np.dtype(np.int8): DataType.INT8, np.dtype(np.int16): DataType.INT16,
            np.dtype(np.uint16): DataType.UINT16, np.dtype(np.uint32): DataType.UINT32,
            np.dtype(np.int32): DataType.INT32, np.dtype(np.uint64): DataType.UINT64,
            np.dtype(np.int64): DataType.INT64, np.dtype(np.float16): DataType.FLOAT16,
            np.dtype(np.float32): DataType.FLOAT, np.dtype(np.float64): DataType.DOUBLE}


@functools.lru_cache(maxsize=None)
def _torch_map():
    m = {torch.uint8: DataType.UINT8, torch.int8: DataType.INT8, torch.int16: DataType.INT16,
         torch.int32: DataType.INT32, torch.int64: DataType.INT64, torch.float16: DataType.FLOAT16,
         torch.bfloat16: DataType.BFLOAT16, torch.float32: DataType.FLOAT, torch.float64: DataType.DOUBLE}
    for name, dt in (("uint16", DataType.UINT16), ("uint32", DataType.UINT32), ("uint64", DataType.UINT64),
                     ("float8_e4m3fn", DataType.FLOAT8_E4M3), ("float8_e5m2", DataType.FLOAT8_E5M2)):
        if hasattr(torch, name):
            m[getattr(torch, name)] = dt
    return m


class DeviceType(Enum):
    CPU = 0
    CUDA = 1
    HIP = 1

    @classmethod
    def from_torch_device_type(cls, device_type: str) -> "DeviceType":
        return {"cpu": cls.CPU, "cuda": cls.CUDA}.get(device_type)


class DistributionHint(Enum):
    NONE = 0
    NORMAL = 1
    UNIFORM = 2


class QuantizationAlgorithm(Enum):
    NONE = 0
    MIN_MAX = 1
    ZERO_POINT_SCALE = 2


class ReduceOperandDescriptor:
    def __init__(self, datatype: DataType, distribution_hint: DistributionHint = DistributionHint.NONE):
        self.datatype = datatype
        self.distribution_hint = distribution_hint


class QuantizationOptions:
    def __init__(self, quantized_datatype: DataType = DataType.UINT8,
                 algorithm: QuantizationAlgorithm = QuantizationAlgorithm.MIN_MAX):
        self.quantized_datatype = quantized_datatype
        self.algorithm = algorithm


class ReduceDescriptor:
    def __init__(self, count: int, op: ReduceOp, tag: int, operand_descriptor: ReduceOperandDescriptor,
                 quantization_options: QuantizationOptions):
        self.count = count
        self.op = op
        self.tag = tag
        self.operand_descriptor = operand_descriptor
        self.quantization_options = quantization_options

    def fill(self, c: _native.ReduceDescriptorC):
        c.count = self.count
        c.op = self.op.value
        c.tag = self.tag
        c.src_descriptor.datatype = self.operand_descriptor.datatype.value
        c.src_descriptor.distribution_hint = self.operand_descriptor.distribution_hint.value
        c.quantization_options.quantized_datatype = self.quantization_options.quantized_datatype.value
        c.quantization_options.algorithm = self.quantization_options.algorithm.value
        return c

    def to_c(self) -> _native.ReduceDescriptorC:
        return self.fill(_native.ReduceDescriptorC())


def _sync_device(t) -> None:
    """Makes the tensor's producer kernels visible to the library's own HIP streams."""
    if t.device.type == "cuda":
        torch.cuda.current_stream(t.device).synchronize()


def _hip_stream(t, stream):
    """The hipStream_t (int) a stream-ordered op of GPU tensor ``t`` waits on: ``stream`` (a torch.cuda.Stream) or the
    device's current stream; None for host tensors / non-torch buffers (they take the plain entry points)."""
    if isinstance(torch, _ModuleDummy) or not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        return None
    return (stream if stream is not None else torch.cuda.current_stream(t.device)).cuda_stream


def _check_pair_torch(send, recv):
    assert send.is_contiguous(), "Input tensor must be contiguous"
    assert recv.is_contiguous(), "Output tensor must be contiguous"
    assert send.device == recv.device, "Input and output tensors must be on the same device"
    assert send.dtype == recv.dtype, "Input and output tensors must have the same dtype"
    assert send.numel() == recv.numel(), "Input and output tensors must have the same number of elements"
    assert send.device.type in ("cpu", "cuda"), f"Unsupported device {send.device}"


def _check_pair_numpy(send, recv):
    assert send.flags.c_contiguous, "Input array must be contiguous"
    assert recv.flags.c_contiguous, "Output array must be contiguous"
    assert send.dtype == recv.dtype, "Input and output arrays must have the same dtype"
    assert send.size == recv.size, "Input and output arrays must have the same number of elements"


class ReduceOpDescriptor:
    def __init__(self, sendbuf_ptr: int, recvbuf_ptr: int, reduce_descriptor: ReduceDescriptor):
        self.sendbuf_ptr = sendbuf_ptr
        self.recvbuf_ptr = recvbuf_ptr
        self.reduce_descriptor = reduce_descriptor
        self._keepalive = None

    @staticmethod
    def from_torch(send, recv, reduce_descriptor: ReduceDescriptor) -> "ReduceOpDescriptor":
        _check_pair_torch(send, recv)
        _sync_device(send)
        d = ReduceOpDescriptor(send.data_ptr(), recv.data_ptr(), reduce_descriptor)
        d._keepalive = (send, recv)
        return d

    @staticmethod
    def from_numpy(send, recv, reduce_descriptor: ReduceDescriptor) -> "ReduceOpDescriptor":
        _check_pair_numpy(send, recv)
        d = ReduceOpDescriptor(send.ctypes.data, recv.ctypes.data, reduce_descriptor)
        d._keepalive = (send, recv)
        return d

    def fill(self, c: _native.ReduceOpDescriptorC):
        c.sendbuf = self.sendbuf_ptr
        c.recvbuf = self.recvbuf_ptr
        self.reduce_descriptor.fill(c.descriptor)

    to_c_inpl = fill  # reference name (python/framework/pccl/_pccl.py:319)

    def to_c(self) -> _native.ReduceOpDescriptorC:
        c = _native.ReduceOpDescriptorC()
        self.fill(c)
        return c


class TensorInfo:
    def __init__(self, name: str, data_ptr: int, *, numel: int, dtype: DataType, device_type: DeviceType,
                 allow_content_inequality: bool):
        if data_ptr == 0:
            raise ValueError("Invalid data pointer: nullptr")
        self.name = name
        self.data_ptr = data_ptr
        self.numel = numel
        self.dtype = dtype
        self.device_type = device_type
        self.allow_content_inequality = allow_content_inequality
        self._keepalive = None

    @classmethod
    def from_torch(cls, tensor, name: str, *, allow_content_inequality: bool = False) -> "TensorInfo":
        try:
            from torch.distributed.tensor import DTensor
            assert not isinstance(tensor, DTensor), "Input tensor must not be a distributed tensor (use .to_local())"
        except ImportError:
            pass
        assert tensor.is_contiguous(), "Input tensor must be contiguous"
        info = cls(name, tensor.data_ptr(), numel=tensor.numel(), dtype=DataType.from_torch_dtype(tensor.dtype),
                   device_type=DeviceType.from_torch_device_type(tensor.device.type),
                   allow_content_inequality=allow_content_inequality)
        info._keepalive = tensor
        return info

    @classmethod
    def from_numpy(cls, array, name: str, *, allow_content_inequality: bool = False) -> "TensorInfo":
        assert array.flags["C_CONTIGUOUS"], "Input array must be contiguous"
        info = cls(name, array.ctypes.data, numel=array.size, dtype=DataType.from_numpy_dtype(array.dtype),
                   device_type=DeviceType.CPU, allow_content_inequality=allow_content_inequality)
        info._keepalive = array
        return info


class SharedState:
    def __init__(self, tensor_infos: List[TensorInfo]):
        assert tensor_infos, "At least one tensor info must be provided"
        self._tensor_infos = list(tensor_infos)
        self._infos = (_native.TensorInfoC * len(tensor_infos))()
        self._names = []
        for i, info in enumerate(tensor_infos):
            name = ctypes.c_char_p(info.name.encode("utf-8"))
            self._names.append(name)
            self._infos[i].name = name.value
            self._infos[i].data = info.data_ptr
            self._infos[i].count = info.numel
            self._infos[i].datatype = info.dtype.value
            self._infos[i].device_type = info.device_type.value
            self._infos[i].allow_content_inequality = info.allow_content_inequality
        self._state = _native.SharedStateC(0, len(tensor_infos), self._infos)

    @property
    def revision(self) -> int:
        return int(self._state.revision)

    @revision.setter
    def revision(self, value: int):
        self._state.revision = value

    def push_revision(self):
        self._state.revision += 1

    def _sync_devices(self):
        for info in self._tensor_infos:
            if info.device_type == DeviceType.CUDA and info._keepalive is not None:
                _sync_device(info._keepalive)


class SharedStateSyncInfo:
    def __init__(self, tx_bytes: int, rx_bytes: int):
        self.tx_bytes = tx_bytes
        self.rx_bytes = rx_bytes


class ReduceInfo:
    def __init__(self, local_world_size: int, tx_bytes: int, rx_bytes: int):
        self.local_world_size = local_world_size
        self.tx_bytes = tx_bytes
        self.rx_bytes = rx_bytes


class AsyncReduceHandle:
    def __init__(self, handle: _native.AsyncReduceOpC, keepalive=None):
        self._handle = handle
        self._info: Optional[Tuple[bool, int, ReduceInfo]] = None
        self._keepalive = keepalive

    def wait(self) -> Tuple[bool, int, ReduceInfo]:
        """Blocks until the async all-reduce completes; returns (success, status, info)."""
        if self._info is not None:
            return self._info
        info = _native.ReduceInfoC()
        status = C.pcclAwaitAsyncReduce(ctypes.byref(self._handle), ctypes.byref(info))
        self._info = (status == 0, status, ReduceInfo(info.local_world_size, info.tx_bytes, info.rx_bytes))
        self._keepalive = None
        return self._info


def _socket_address(ip: Union[IPv4Address, IPv6Address], port: int) -> _native.SocketAddress:
    a = _native.SocketAddress()
    if isinstance(ip, IPv4Address):
        a.inet.protocol = 0
        for i, b in enumerate(ip.packed):
            a.inet.ipv4.data[i] = b
    elif isinstance(ip, IPv6Address):
        a.inet.protocol = 1
        for i, b in enumerate(ip.packed):
            a.inet.ipv6.data[i] = b
    else:
        raise ValueError(f"Unsupported IP address type: {type(ip)}")
    a.port = port & 0xFFFF
    return a


def _parse_host_port(address: str) -> Tuple[Union[IPv4Address, IPv6Address], int]:
    assert ":" in address, f"Invalid address: {address}, expected ip:port"
    host, port = address.rsplit(":", 1)
    host = host.strip("[]")
    return ip_address(host), int(port)


class Communicator:
    """A peer of a PCCL run. ``address`` is the master's ``ip:port``."""

    def __init__(self, address: str, peer_group: int = 0, p2p_connection_pool_size: int = 0,
                 public_advertise_ip: Optional[str] = None, p2p_listen_port: int = 48149,
                 shared_state_listen_port: int = 48150, benchmark_listen_port: int = 48151,
                 advertised_p2p_port: Optional[int] = None, advertised_shared_state_port: Optional[int] = None):
        """``advertised_p2p_port`` / ``advertised_shared_state_port``: the port announced to the other peers when it
        differs from the listen port (behind NAT / port forwarding, or a relay such as ``pccl_wan_relay``); implies
        advertising ``public_advertise_ip`` (default 127.0.0.1)."""
        ip, port = _parse_host_port(address)
        params = _native.CommCreateParams()
        params.master_address = _socket_address(ip, port)
        params.peer_group = peer_group
        params.p2p_connection_pool_size = p2p_connection_pool_size
        params.internal_p2p_listen_port = p2p_listen_port
        params.internal_shared_state_listen_port = shared_state_listen_port
        params.internal_benchmark_listen_port = benchmark_listen_port
        if (advertised_p2p_port is not None or advertised_shared_state_port is not None) and not public_advertise_ip:
            public_advertise_ip = "127.0.0.1"
        if public_advertise_ip:
            adv = ip_address(public_advertise_ip)
            params.use_explicit_p2p_addresses = True
            params.advertised_p2p_address = _socket_address(adv, advertised_p2p_port or p2p_listen_port)
            params.advertised_shared_state_address = _socket_address(adv, advertised_shared_state_port or
                                                                     shared_state_listen_port)
            params.advertised_benchmark_address = _socket_address(adv, benchmark_listen_port)
        self._comm = ctypes.c_void_p()
        PCCLError.check(C.pcclCreateCommunicator(ctypes.byref(params), ctypes.byref(self._comm)),
                        "pcclCreateCommunicator")

    def __del__(self):
        self.destroy()

    def destroy(self):
        comm = getattr(self, "_comm", None)
        if comm is not None and comm.value:
            C.pcclDestroyCommunicator(comm)
            self._comm = ctypes.c_void_p()

    def liveness_stats(self):
        """This peer's liveness counters: stalled-op reports sent to the master, ops failed by the local stall
        watchdog, master declared lost (silent for 2 x PCCL_PEER_TIMEOUT_MS), heartbeats sent."""
        out = (ctypes.c_uint64 * 4)()
        C.pcclxLivenessStats(self._comm, out, 4)
        return {"stall_reports": int(out[0]), "stall_fails": int(out[1]), "master_lost": int(out[2]),
                "heartbeats": int(out[3])}

    def get_attribute(self, attribute: Attribute) -> int:
        v = ctypes.c_int()
        PCCLError.check(C.pcclGetAttribute(self._comm, attribute.value, ctypes.byref(v)), "pcclGetAttribute")
        return v.value

    def connect(self, n_attempts: int = 5):
        for attempt in range(1, n_attempts + 1):
            try:
                PCCLError.check(C.pcclConnect(self._comm), "pcclConnect")
                logger.info("Connected to the master node")
                return
            except PCCLError as e:
                logger.warning("Failed to connect (attempt %d/%d): %s", attempt, n_attempts, e)
                time.sleep(1)
        raise Exception("Failed to connect to the master node")

    def update_topology(self):
        PCCLError.check(C.pcclUpdateTopology(self._comm), "pcclUpdateTopology")

    def are_peers_pending(self) -> bool:
        b = ctypes.c_bool()
        PCCLError.check(C.pcclArePeersPending(self._comm, ctypes.byref(b)), "pcclArePeersPending")
        return bool(b.value)

    def optimize_topology(self):
        PCCLError.check(C.pcclOptimizeTopology(self._comm), "pcclOptimizeTopology")

    def sync_shared_state(self, shared_state: SharedState,
                          strategy: SharedStateSyncStrategy = SharedStateSyncStrategy.ENFORCE_POPULAR
                          ) -> SharedStateSyncInfo:
        shared_state._sync_devices()
        info = _native.SharedStateSyncInfoC()
        PCCLError.check(C.pcclSynchronizeSharedState(self._comm, ctypes.byref(shared_state._state), strategy.value,
                                                     ctypes.byref(info)), "pcclSynchronizeSharedState")
        return SharedStateSyncInfo(info.tx_bytes, info.rx_bytes)

    # --- all-reduce -------------------------------------------------------------------------------------------
    def _descriptor(self, send, recv, op, tag, operand_descriptor, quantization_options, sync=True):
        if not isinstance(torch, _ModuleDummy) and isinstance(send, torch.Tensor) and isinstance(recv, torch.Tensor):
            _check_pair_torch(send, recv)
            if sync:
                _sync_device(send)
            dtype = DataType.from_torch_dtype(send.dtype)
            sptr, rptr, n = send.data_ptr(), recv.data_ptr(), recv.numel()
        elif not isinstance(np, _ModuleDummy) and isinstance(send, np.ndarray) and isinstance(recv, np.ndarray):
            _check_pair_numpy(send, recv)
            dtype = DataType.from_numpy_dtype(send.dtype)
            sptr, rptr, n = send.ctypes.data, recv.ctypes.data, recv.size
        else:
            raise ValueError(f"Unsupported input types: {type(send)}, {type(recv)}; "
                             "send and recv must both be torch.Tensor or both np.ndarray")
        # filled directly (the per-op Python cost matters next to a ~50-100 us small all-reduce)
        desc = _native.ReduceDescriptorC()
        desc.count = n
        desc.op = op.value
        desc.tag = tag
        if operand_descriptor is None:
            desc.src_descriptor.datatype = dtype.value
        else:
            desc.src_descriptor.datatype = operand_descriptor.datatype.value
            desc.src_descriptor.distribution_hint = operand_descriptor.distribution_hint.value
        if quantization_options is None:
            desc.quantization_options.quantized_datatype = dtype.value
        else:
            desc.quantization_options.quantized_datatype = quantization_options.quantized_datatype.value
            desc.quantization_options.algorithm = quantization_options.algorithm.value
        return sptr, rptr, desc

    def all_reduce(self, send, recv, *, op: ReduceOp, tag: int = 0,
                   operand_descriptor: Optional[ReduceOperandDescriptor] = None,
                   quantization_options: Optional[QuantizationOptions] = None, stream=None) -> ReduceInfo:
        """Blocking all-reduce. GPU tensors are stream-ordered: the op reads ``send`` after the work queued on
        ``stream`` (default: the current stream) before this call, without the caller synchronising that stream; the
        result is complete on return."""
        hs = _hip_stream(send, stream)
        sptr, rptr, desc = self._descriptor(send, recv, op, tag, operand_descriptor, quantization_options,
                                            sync=hs is None)
        info = _native.ReduceInfoC()
        if hs is None:
            PCCLError.check(C.pcclAllReduce(sptr, rptr, ctypes.byref(desc), self._comm, ctypes.byref(info)),
                            "pcclAllReduce")
        else:
            PCCLError.check(C.pcclxAllReduceOnStream(sptr, rptr, ctypes.byref(desc), self._comm, hs,
                                                     ctypes.byref(info)), "pcclxAllReduceOnStream")
        return ReduceInfo(info.local_world_size, info.tx_bytes, info.rx_bytes)

    def all_reduce_async(self, send, recv, *, op: ReduceOp, tag: int = 0,
                         operand_descriptor: Optional[ReduceOperandDescriptor] = None,
                         quantization_options: Optional[QuantizationOptions] = None, stream=None) -> AsyncReduceHandle:
        """Asynchronous all-reduce; ``handle.wait()`` awaits it. GPU tensors are stream-ordered (see all_reduce): this
        call returns at once, even while ``send``'s producers are still queued on ``stream``."""
        hs = _hip_stream(send, stream)
        sptr, rptr, desc = self._descriptor(send, recv, op, tag, operand_descriptor, quantization_options,
                                            sync=hs is None)
        handle = _native.AsyncReduceOpC()
        if hs is None:
            PCCLError.check(C.pcclAllReduceAsync(sptr, rptr, ctypes.byref(desc), self._comm, ctypes.byref(handle)),
                            "pcclAllReduceAsync")
        else:
            PCCLError.check(C.pcclxAllReduceAsyncOnStream(sptr, rptr, ctypes.byref(desc), self._comm, hs,
                                                          ctypes.byref(handle)), "pcclxAllReduceAsyncOnStream")
        return AsyncReduceHandle(handle, keepalive=(send, recv))

    def _all_reduce_async_ready(self, send, recv, *, op: ReduceOp, tag: int,
                                operand_descriptor: Optional[ReduceOperandDescriptor] = None,
                                quantization_options: Optional[QuantizationOptions] = None) -> AsyncReduceHandle:
        """all_reduce_async for device tensors whose producers the caller already waited for (e.g. on an event):
        skips the current-stream synchronisation, so a comm thread does not wait for unrelated queued kernels."""
        sptr, rptr, desc = self._descriptor(send, recv, op, tag, operand_descriptor, quantization_options, sync=False)
        handle = _native.AsyncReduceOpC()
        PCCLError.check(C.pcclAllReduceAsync(sptr, rptr, ctypes.byref(desc), self._comm, ctypes.byref(handle)),
                        "pcclAllReduceAsync")
        return AsyncReduceHandle(handle, keepalive=(send, recv))

    def all_reduce_multiple_with_retry(self, descriptors: List[ReduceOpDescriptor], *,
                                       max_in_flight: int = 4) -> ReduceInfo:
        arr = (_native.ReduceOpDescriptorC * len(descriptors))()
        for i, d in enumerate(descriptors):
            d.fill(arr[i])
        info = _native.ReduceInfoC()
        PCCLError.check(C.pcclAllReduceMultipleWithRetry(arr, len(descriptors), self._comm, ctypes.byref(info),
                                                         max_in_flight), "pcclAllReduceMultipleWithRetry")
        return ReduceInfo(info.local_world_size, info.tx_bytes, info.rx_bytes)


class MasterNode:
    """The coordinator. ``listen_address`` is ``ip:port`` (use 0.0.0.0 to listen on all interfaces)."""

    def __init__(self, listen_address: str):
        ip, port = _parse_host_port(listen_address)
        self._master = ctypes.c_void_p()
        PCCLError.check(C.pcclCreateMaster(_socket_address(ip, port), ctypes.byref(self._master)), "pcclCreateMaster")
        self._running = False

    def run(self):
        PCCLError.check(C.pcclRunMaster(self._master), "pcclRunMaster")
        self._running = True

    def interrupt(self):
        PCCLError.check(C.pcclInterruptMaster(self._master), "pcclInterruptMaster")

    def bandwidth_table(self):
        """The master's measured link bandwidths: [(peer group, from uuid, to uuid, Mbit/s)] (every entry of every
        group's bandwidth store, including the fixed cost of same-host xGMI pairs)."""
        n = int(C.pcclxMasterBandwidthTable(self._master, None, 0))
        buf = ctypes.create_string_buffer(n + 1)
        C.pcclxMasterBandwidthTable(self._master, buf, n + 1)
        out = []
        for ln in buf.value.decode().splitlines():
            g, frm, _, to, mbps, _unit = ln.replace(":", "").split()
            out.append((int(g), frm, to, float(mbps)))
        return out

    def topology_stats(self):
        """The master's topology-optimization counters: synchronous ATSP solves, the last one's duration (us), rings
        a solve changed (synchronous or moonshot) and finished moonshot solves."""
        out = (ctypes.c_uint64 * 4)()
        C.pcclxMasterTopologyStats(self._master, out, 4)
        return {"solves": int(out[0]), "last_solve_us": int(out[1]), "ring_changes": int(out[2]),
                "moonshot_solves": int(out[3])}

    def liveness_stats(self):
        """The master's liveness counters: peers dropped for silence (no heartbeat for PCCL_PEER_TIMEOUT_MS), peers
        dropped on stalled-op reports, peers dropped for not voting (PCCL_VOTE_TIMEOUT_MS), stall reports received."""
        out = (ctypes.c_uint64 * 4)()
        C.pcclxMasterLivenessStats(self._master, out, 4)
        return {"dropped_silent": int(out[0]), "dropped_stalled": int(out[1]), "dropped_vote_timeout": int(out[2]),
                "stall_reports": int(out[3])}

    def await_termination(self):
        if self._running:
            C.pcclMasterAwaitTermination(self._master)
            self._running = False

    def __del__(self):
        m = getattr(self, "_master", None)
        if m is not None and m.value:
            if getattr(self, "_running", False):
                C.pcclInterruptMaster(m)
                C.pcclMasterAwaitTermination(m)
            C.pcclDestroyMaster(m)
            self._master = ctypes.c_void_p()
