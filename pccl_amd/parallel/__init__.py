"""Training integrations on top of the PCCL communicator.

* :mod:`.elastic` — multi-tensor all-reduce with retry, topology-update gate, shared state for model + optimizer
* :mod:`.ddp`     — device-resident gradient buckets + all-reduce (DDP over PCCL)
* :mod:`.diloco`  — DiLoCo outer optimisation (sync and 1-step-delayed async) with fused HIP outer-step kernel
* :mod:`.hybrid`  — RCCL (torch.distributed) inside a node x PCCL across nodes / peer groups per shard
"""
from .ddp import DataParallel, GradBuckets
from .elastic import (RetryResult, all_reduce_multiple_with_retry, init_optimizer_state, maybe_update_topology,
                      shared_state_for, state_tensors, world_size)

__all__ = ["DataParallel", "GradBuckets", "RetryResult", "all_reduce_multiple_with_retry", "init_optimizer_state",
           "maybe_update_topology", "shared_state_for", "state_tensors", "world_size"]
