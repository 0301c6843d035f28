"""pccl-amd: MI355X-native fault-tolerant collective communications (PCCL-compatible API).

Layers:
  * ``pccl_amd.api``       Communicator / MasterNode / SharedState — the PCCL API (host + GPU tensors)
  * ``pccl_amd.ops``       direct access to the HIP/CDNA4 kernels (reduce, quantize, hash, xGMI reduce/gather)
  * ``pccl_amd.parallel``  training integrations: PCCL DDP gradient sync, DiLoCo (sync / async), hybrid RCCL x PCCL
  * ``pccl_amd.models``    reference workloads (nanoGPT, MNIST MLP) used by examples and the end-to-end tests
  * ``pccl_amd.memory``    fd-shareable device memory (zero-copy, fault-safe xGMI all-reduce buffers)
  * ``pccl_amd.utils``     profiler, launch helpers
"""
from .api import (AsyncReduceHandle, Attribute, Communicator, DataType, DeviceType, DistributionHint, MasterNode,
                  PCCLError, QuantizationAlgorithm, QuantizationOptions, ReduceDescriptor, ReduceInfo, ReduceOp,
                  ReduceOpDescriptor, ReduceOperandDescriptor, ReducePath, Result, SharedState,
                  SharedStateSyncInfo, SharedStateSyncStrategy, TensorInfo, build_info)
from . import memory
from .memory import shareable_memory, shareable_pool

__version__ = "0.1.0"


class cuda:  # reference exposes pccl.cuda.is_available()
    @staticmethod
    def is_available() -> bool:
        return bool(build_info()["has_hip_support"])


hip = cuda

__all__ = [
    "AsyncReduceHandle", "Attribute", "Communicator", "DataType", "DeviceType", "DistributionHint", "MasterNode",
    "PCCLError", "QuantizationAlgorithm", "QuantizationOptions", "ReduceDescriptor", "ReduceInfo", "ReduceOp",
    "ReduceOpDescriptor", "ReduceOperandDescriptor", "ReducePath", "Result", "SharedState", "SharedStateSyncInfo",
    "SharedStateSyncStrategy", "TensorInfo", "build_info", "cuda", "hip", "memory", "shareable_memory", "shareable_pool",
]
