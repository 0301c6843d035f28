"""Hierarchical data parallelism: RCCL inside a node (torch.distributed, backend "nccl" = RCCL over xGMI) x PCCL
across nodes, one PCCL peer group per local rank (HSDP-style "peer group per shard").

Reference: python/examples/nanogptddp/train_pccl.py:162-177,306-319 runs torch DDP inside the node and additionally
has *every* rank all-reduce the full (already identical) gradient over PCCL in peer group 0, and
sync_diloco_fsdp.py:188-208 puts FSDP shard i of every node into PCCL peer group i. Bandwidth-optimal hierarchy used
here instead, per flat gradient buffer of size S on a node with L GPUs:

  1. intra-node reduce-scatter (RCCL, xGMI)           -> local rank l owns shard l (S/L) summed over the node
  2. inter-node all-reduce of shard l over PCCL, in peer group l (fault tolerant, elastic across nodes)
  3. intra-node all-gather (RCCL, xGMI)                -> every GPU holds the global average

so each GPU sends only S/L over the WAN/TCP and the L peer groups run their rings concurrently.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..api import Communicator, QuantizationOptions, ReduceOp
from .ddp import GradBuckets
from .elastic import RetryResult, all_reduce_multiple_with_retry


def local_peer_group() -> int:
    """The PCCL peer group of this process in the hierarchical layout (= LOCAL_RANK)."""
    import os
    return int(os.environ.get("LOCAL_RANK", "0"))


class HierarchicalGradSync:
    def __init__(self, model: torch.nn.Module, comm: Optional[Communicator], *, group=None,
                 bucket_bytes: int = 1 << 30, max_in_flight: int = 8, tag_base: int = 3 << 20,
                 quantization: Optional[QuantizationOptions] = None):
        self.comm = comm
        self.group = group
        self.L = dist.get_world_size(group) if dist.is_initialized() else 1
        self.l = dist.get_rank(group) if dist.is_initialized() else 0
        self.bucket_bytes = bucket_bytes
        self.max_in_flight = max_in_flight
        self.tag_base = tag_base
        self.quantization = quantization
        self.buckets = GradBuckets(list(model.parameters()))
        # padded flat buffers so that every buffer splits into L equal shards
        self.padded = {}
        for key, buf in self.buckets.flat.items():
            n = buf.numel()
            pad = (-n) % self.L
            self.padded[key] = (n, pad)

    def sync_gradients(self) -> Optional[RetryResult]:
        self.buckets.rebind()
        shards = []
        scratch = []
        for key, buf in self.buckets.flat.items():
            n, pad = self.padded[key]
            full = buf if pad == 0 else torch.cat([buf, buf.new_zeros(pad)])
            if self.L > 1:
                shard = full.new_empty(full.numel() // self.L)
                dist.reduce_scatter_tensor(shard, full, op=dist.ReduceOp.SUM, group=self.group)
                shard.div_(self.L)
            else:
                shard = full
            shards.append(shard)
            scratch.append((buf, full, shard, n))
        res = None
        if self.comm is not None:
            per = max(1, self.bucket_bytes // shards[0].element_size()) if shards else 1
            pieces = [s[i:i + per] for s in shards for i in range(0, s.numel(), per)]
            res = all_reduce_multiple_with_retry(self.comm, pieces, ReduceOp.AVG, max_in_flight=self.max_in_flight,
                                                 tag_base=self.tag_base, quantization=self.quantization)
        for buf, full, shard, n in scratch:
            if self.L > 1:
                dist.all_gather_into_tensor(full, shard, group=self.group)
            if full.data_ptr() != buf.data_ptr():
                buf.copy_(full[:n])
        return res
