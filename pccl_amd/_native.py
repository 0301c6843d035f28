"""ctypes bindings of libpccl.so (replaces the reference's cffi loader, python/framework/pccl/_loader.py).

The library is loaded from ``pccl_amd/lib``. If PyTorch is installed it is imported *first* so that its bundled HIP
runtime (SONAME libamdhip64.so.7) is the one the HIP plugin binds to — one HIP runtime per process.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_bool, c_char_p, c_double, c_float, c_int, c_size_t, c_uint8, c_uint16, c_uint32,
                    c_uint64, c_void_p)

try:  # share torch's HIP runtime with the plugin
    import torch  # noqa: F401
except ImportError:
    pass

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = ""  # the libpccl.so this process loaded (torch's pluggable allocator dlopens the same file)


class IPv4(Structure):
    _fields_ = [("data", c_uint8 * 4)]


class IPv6(Structure):
    _fields_ = [("data", c_uint8 * 16)]


class InetAddress(Structure):
    _fields_ = [("protocol", c_int), ("ipv4", IPv4), ("ipv6", IPv6)]


class SocketAddress(Structure):
    _fields_ = [("inet", InetAddress), ("port", c_uint16)]


class CommCreateParams(Structure):
    _fields_ = [
        ("master_address", SocketAddress),
        ("peer_group", c_uint32),
        ("p2p_connection_pool_size", c_uint32),
        ("use_explicit_p2p_addresses", c_bool),
        ("advertised_p2p_address", SocketAddress),
        ("advertised_shared_state_address", SocketAddress),
        ("advertised_benchmark_address", SocketAddress),
        ("internal_p2p_listen_port", c_uint16),
        ("internal_shared_state_listen_port", c_uint16),
        ("internal_benchmark_listen_port", c_uint16),
    ]


class ReduceOperandDescriptorC(Structure):
    _fields_ = [("datatype", c_int), ("distribution_hint", c_int)]


class QuantizationOptionsC(Structure):
    _fields_ = [("quantized_datatype", c_int), ("algorithm", c_int)]


class ReduceDescriptorC(Structure):
    _fields_ = [
        ("count", c_size_t),
        ("op", c_int),
        ("tag", c_uint64),
        ("src_descriptor", ReduceOperandDescriptorC),
        ("quantization_options", QuantizationOptionsC),
    ]


class ReduceOpDescriptorC(Structure):
    _fields_ = [("sendbuf", c_void_p), ("recvbuf", c_void_p), ("descriptor", ReduceDescriptorC)]


class AsyncReduceOpC(Structure):
    _fields_ = [("comm", c_void_p), ("tag", c_uint64)]


class ReduceInfoC(Structure):
    _fields_ = [("local_world_size", c_uint32), ("tx_bytes", c_uint64), ("rx_bytes", c_uint64)]


class TensorInfoC(Structure):
    _fields_ = [
        ("name", c_char_p),
        ("data", c_void_p),
        ("count", c_size_t),
        ("datatype", c_int),
        ("device_type", c_int),
        ("allow_content_inequality", c_bool),
    ]


class SharedStateC(Structure):
    _fields_ = [("revision", c_uint64), ("count", c_size_t), ("infos", POINTER(TensorInfoC))]


class SharedStateSyncInfoC(Structure):
    _fields_ = [("tx_bytes", c_uint64), ("rx_bytes", c_uint64)]


class BuildInfoC(Structure):
    _fields_ = [("has_cuda_support", c_bool)]  # reference layout (one bool)


class BuildInfoExC(Structure):
    _fields_ = [("struct_size", c_size_t), ("has_cuda_support", c_bool), ("has_hip_support", c_bool),
                ("hip_device_count", c_int)]


def _load() -> ctypes.CDLL:
    path = os.environ.get("PCCL_LIBRARY", os.path.join(LIB_DIR, "libpccl.so"))
    if not os.path.exists(path):
        raise ImportError(
            f"libpccl.so not found at {path}; build it first: python -c 'import __graft_entry__ as g; g.build()' "
            f"(or cmake -S . -B build -G Ninja && ninja -C build)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    global LIB_PATH
    LIB_PATH = path
    p = POINTER
    sig = {
        "pcclInit": ([], c_int),
        "pcclCreateCommunicator": ([p(CommCreateParams), p(c_void_p)], c_int),
        "pcclGetAttribute": ([c_void_p, c_int, p(c_int)], c_int),
        "pcclDestroyCommunicator": ([c_void_p], c_int),
        "pcclConnect": ([c_void_p], c_int),
        "pcclUpdateTopology": ([c_void_p], c_int),
        "pcclArePeersPending": ([c_void_p, p(c_bool)], c_int),
        "pcclOptimizeTopology": ([c_void_p], c_int),
        "pcclAllReduce": ([c_void_p, c_void_p, p(ReduceDescriptorC), c_void_p, p(ReduceInfoC)], c_int),
        "pcclAllReduceAsync": ([c_void_p, c_void_p, p(ReduceDescriptorC), c_void_p, p(AsyncReduceOpC)], c_int),
        "pcclxAllReduceOnStream": ([c_void_p, c_void_p, p(ReduceDescriptorC), c_void_p, c_void_p, p(ReduceInfoC)],
                                   c_int),
        "pcclxAllReduceAsyncOnStream": ([c_void_p, c_void_p, p(ReduceDescriptorC), c_void_p, c_void_p,
                                        p(AsyncReduceOpC)], c_int),
        "pcclAllReduceMultipleWithRetry": ([p(ReduceOpDescriptorC), c_size_t, c_void_p, p(ReduceInfoC), c_int], c_int),
        "pcclAwaitAsyncReduce": ([p(AsyncReduceOpC), p(ReduceInfoC)], c_int),
        "pcclSynchronizeSharedState": ([c_void_p, p(SharedStateC), c_int, p(SharedStateSyncInfoC)], c_int),
        "pcclCreateMaster": ([SocketAddress, p(c_void_p)], c_int),
        "pcclRunMaster": ([c_void_p], c_int),
        "pcclInterruptMaster": ([c_void_p], c_int),
        "pcclMasterAwaitTermination": ([c_void_p], c_int),
        "pcclDestroyMaster": ([c_void_p], c_int),
        "pcclGetBuildInfo": ([p(BuildInfoC)], c_int),
        "pcclGetBuildInfoEx": ([p(BuildInfoExC)], c_int),
        "pcclDataTypeSize": ([c_int], c_size_t),
        # kernel-level extension API (tests / micro-benchmarks)
        "pcclxHipDeviceCount": ([], c_int),
        "pcclxSimpleHash": ([c_void_p, c_size_t, c_int], c_uint32),
        "pcclxCrc32c": ([c_void_p, c_size_t, c_int], c_uint32),
        "pcclxCrc32cHasHw": ([], c_int),
        "pcclxFillTestPattern": ([c_void_p, c_size_t], c_int),
        "pcclxReduce": ([c_void_p, c_void_p, c_size_t, c_int, c_int, c_int], c_int),
        "pcclxFinalizeAvg": ([c_void_p, c_size_t, c_int, c_size_t, c_int], c_int),
        "pcclxQuantize": ([c_void_p, c_void_p, c_size_t, c_int, c_int, c_int, c_int, p(c_double)], c_int),
        "pcclxQuantizeSetback": ([c_void_p, c_void_p, c_size_t, c_int, c_int, c_int, p(c_double)], c_int),
        "pcclxDequantReduce": ([c_void_p, c_void_p, c_size_t, c_int, c_int, c_int, c_int, p(c_double), c_int], c_int),
        "pcclxDequantReduceMinmax": ([c_void_p, c_void_p, c_size_t, c_int, c_int, c_int, c_int, p(c_double), c_int,
                                      p(c_double)], c_int),
        "pcclxQuantStats": ([p(c_uint64)], None),
        "pcclxMultiReduce": ([p(c_void_p), c_int, p(c_void_p), c_int, c_size_t, c_int, c_int], c_int),
        "pcclxMultiGather": ([c_void_p, p(c_void_p), p(c_size_t), p(c_size_t), c_int, c_int, c_int], c_int),
        "pcclxBenchKernel": ([c_int, c_void_p, c_void_p, c_size_t, c_int, c_int, c_int], c_double),
        "pcclxPseudoGrad": ([c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int], c_int),
        "pcclxOuterSgd": ([c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_float, c_float, c_float, c_float,
                           c_int, c_int, c_int], c_int),
        # shareable (VMM + fd) device memory and xGMI/IPC buffer-mode counters (pccl_amd.memory)
        "pcclxShareableQuery": ([c_void_p, c_size_t, p(c_uint64), p(c_size_t)], c_int),
        "pcclxShareableLiveBytes": ([], c_size_t),
        "pcclxIpcStats": ([p(c_uint64)], None),
        "pcclxIpcStatsEx": ([p(c_uint64), c_size_t], c_size_t),
        "pcclxPoolStats": ([p(c_uint64), c_size_t, c_int], c_size_t),
        "pcclxPoolReserve": ([c_uint64, c_uint32, c_uint64, c_uint32, c_int], c_int),
        "pcclxPcieStats": ([p(c_uint64), c_size_t], c_size_t),
        "pcclxMasterBandwidthTable": ([c_void_p, c_char_p, c_size_t], c_size_t),
        "pcclxMasterTopologyStats": ([c_void_p, p(c_uint64), c_size_t], c_size_t),
        "pcclxMasterLivenessStats": ([c_void_p, p(c_uint64), c_size_t], c_size_t),
        "pcclxLivenessStats": ([c_void_p, p(c_uint64), c_size_t], c_size_t),
    }
    for name, (argtypes, restype) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    return lib


C = _load()
