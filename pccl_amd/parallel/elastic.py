"""Elastic-run building blocks shared by the DDP and DiLoCo integrations.

* :func:`all_reduce_multiple_with_retry` — concurrent all-reduces (one tag per tensor, at most ``max_in_flight``
  outstanding) that survive peers dropping out: a failed op makes every peer drain its in-flight ops, the library
  re-establishes the ring, and the failed/undone tensors are reduced again by the survivors
  (reference python/tests/end_to_end/mnist_ddp/mnist_peer.py:111-215 and src/pccl.cpp:345-523).
* :func:`maybe_update_topology` — the per-step "admit pending peers" vote in the shape the reference's training loops
  use (mnist_peer.py:263-273: every iteration but a freshly accepted peer's first one).
* :func:`shared_state_for` / :func:`init_optimizer_state` — model + optimizer state as a PCCL shared state
  (mnist_peer.py:225-256, train_pccl.py:330-352).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence

import torch

from ..api import (Attribute, Communicator, DataType, DistributionHint, PCCLError, QuantizationAlgorithm,
                   QuantizationOptions, ReduceOp, ReduceOperandDescriptor, Result, SharedState, TensorInfo)


@dataclass
class RetryResult:
    ok: bool              # False: the world shrank to a single peer before everything was reduced
    tx_bytes: int
    rx_bytes: int
    retries: int
    world_size: int


def world_size(comm: Communicator) -> int:
    return comm.get_attribute(Attribute.GLOBAL_WORLD_SIZE)


def all_reduce_multiple_with_retry(comm: Communicator, tensors: Sequence[torch.Tensor], op: ReduceOp = ReduceOp.AVG,
                                   *, max_in_flight: int = 8, tag_base: int = 0,
                                   quantization: Optional[QuantizationOptions] = None,
                                   outputs: Optional[Sequence[torch.Tensor]] = None) -> RetryResult:
    """All-reduces every tensor (in place unless ``outputs`` is given); retries on peer churn.

    Each tensor gets tag ``tag_base + i``. Returns ok=False if this peer ended up alone.
    """
    outs = list(outputs) if outputs is not None else list(tensors)
    n = len(tensors)
    done = [False] * n
    handles: List[Optional[object]] = [None] * n
    tx = rx = retries = 0
    ws = world_size(comm)

    def launch(i: int):
        t = tensors[i]
        desc = ReduceOperandDescriptor(DataType.from_torch_dtype(t.dtype), DistributionHint.NONE)
        q = quantization or QuantizationOptions(DataType.from_torch_dtype(t.dtype), QuantizationAlgorithm.NONE)
        return comm.all_reduce_async(t, outs[i], op=op, tag=tag_base + i, operand_descriptor=desc,
                                     quantization_options=q)

    too_few = False
    while ws > 1 and not all(done) and not too_few:
        failed = False
        in_flight: List[int] = []
        pending = [i for i in range(n) if not done[i]]
        cursor = 0
        while (cursor < len(pending) or in_flight) and not failed:
            while cursor < len(pending) and len(in_flight) < max_in_flight:
                i = pending[cursor]
                try:
                    handles[i] = launch(i)
                except PCCLError as e:
                    if e.result == Result.TOO_FEW_PEERS:  # alone (the ring shrank to this peer)
                        failed = too_few = True
                        break
                    raise
                in_flight.append(i)
                cursor += 1
            if not in_flight:
                break
            i = in_flight.pop(0)
            ok, _, info = handles[i].wait()
            handles[i] = None
            if ok:
                done[i] = True
                tx += info.tx_bytes
                rx += info.rx_bytes
            else:
                failed = True
        if failed:
            # drain everything still in flight before the retry (an op may also have succeeded)
            for j in in_flight:
                ok, _, info = handles[j].wait()
                handles[j] = None
                if ok:
                    done[j] = True
                    tx += info.tx_bytes
                    rx += info.rx_bytes
            retries += 1
        ws = world_size(comm)
    return RetryResult(all(done) and not too_few, tx, rx, retries, ws)


def maybe_update_topology(comm: Communicator, iteration: int, *, retries: int = 10) -> bool:
    """Admits pending peers (collective vote). Skipped on a peer's first iteration. Returns True if a vote ran."""
    if iteration <= 0:
        return False
    if not comm.are_peers_pending():
        return False
    for attempt in range(retries):
        try:
            comm.update_topology()
            return True
        except PCCLError:
            time.sleep(0.05 * (attempt + 1))
    raise RuntimeError("update_topology kept failing")


def init_optimizer_state(optimizer: torch.optim.Optimizer) -> None:
    """Materialises lazily created optimizer state (Adam moments, step) with a zero-gradient step."""
    saved = {}
    for group in optimizer.param_groups:
        for p in group["params"]:
            saved[p] = p.detach().clone()
            if p.grad is None:
                p.grad = torch.zeros_like(p)
    lrs = [g["lr"] for g in optimizer.param_groups]
    for g in optimizer.param_groups:
        g["lr"] = 0.0
    optimizer.step()
    for g, lr in zip(optimizer.param_groups, lrs):
        g["lr"] = lr
    with torch.no_grad():
        for p, v in saved.items():
            p.copy_(v)  # weight decay with lr 0 is a no-op, but be exact anyway
    optimizer.zero_grad(set_to_none=False)


def state_tensors(model: torch.nn.Module, optimizer: Optional[torch.optim.Optimizer] = None,
                  extra: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
    """name -> tensor of everything that must be identical on every peer (params, optimizer state, extras)."""
    out: Dict[str, torch.Tensor] = {}
    for name, p in model.named_parameters():
        out[name] = p.data
        if optimizer is not None:
            for k, v in optimizer.state.get(p, {}).items():
                if isinstance(v, torch.Tensor):
                    if not v.is_contiguous():
                        raise ValueError(f"optimizer state {name}.{k} is not contiguous")
                    out[f"{name}.{k}"] = v
    for name, b in model.named_buffers():
        if b.is_floating_point() or b.dtype in (torch.int64, torch.int32):
            out[f"buffer.{name}"] = b
    if extra:
        out.update(extra)
    return out


def shared_state_for(model: torch.nn.Module, optimizer: Optional[torch.optim.Optimizer] = None,
                     extra: Optional[Dict[str, torch.Tensor]] = None,
                     allow_content_inequality: Iterable[str] = ()) -> SharedState:
    allow = set(allow_content_inequality)
    infos = [TensorInfo.from_torch(t, name, allow_content_inequality=name in allow)
             for name, t in state_tensors(model, optimizer, extra).items()]
    return SharedState(infos)
