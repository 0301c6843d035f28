"""DiLoCo (local SGD with an outer optimizer on averaged pseudo-gradients) over PCCL — sync and 1-step-delayed async.

Reference: python/examples/nanogpt_diloco/sync_diloco.py (outer SGD on CPU copies of the parameters, AVG all-reduce
of ``outer - local`` via all_reduce_multiple_with_retry) and async_diloco.py:386-621 (the reduce of step t overlaps
the inner steps of t+1; newcomers are inserted into the pipeline by a second SEND_ONLY / RECEIVE_ONLY shared-state
sync). docs/md/07-DiLoCo*.

MI355X-first differences:
  * the outer state lives in HBM next to the model (288 GB leaves room for fp32 outer params + momentum of even
    very large models), so the pseudo-gradient reduce takes the device path (xGMI IPC intra-node);
  * the local parameters of each (device, dtype) group are views into one flat buffer, so the pseudo-gradient and the
    outer step are single fused HIP kernels over the whole model (``pcclxPseudoGrad`` / ``pcclxOuterSgd``) instead of
    ~5 torch passes per parameter;
  * optional quantized pseudo-gradients (uint8 min-max or fp8) on the wire.
"""
from __future__ import annotations

import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch

from ..api import Communicator, QuantizationOptions, ReduceOp, SharedState, SharedStateSyncStrategy, TensorInfo
from ..memory import maybe_shareable
from ..ops import kernels as K
from .elastic import RetryResult, all_reduce_multiple_with_retry


class FlatParams:
    """Re-homes a module's parameters into one contiguous buffer per (device, dtype); ``p.data`` become views."""

    def __init__(self, model: torch.nn.Module):
        groups: "OrderedDict[Tuple[torch.device, torch.dtype], List[torch.nn.Parameter]]" = OrderedDict()
        for p in model.parameters():
            groups.setdefault((p.device, p.dtype), []).append(p)
        self.flat: Dict[Tuple[torch.device, torch.dtype], torch.Tensor] = {}
        for key, ps in groups.items():
            buf = torch.empty(sum(p.numel() for p in ps), device=key[0], dtype=key[1])
            off = 0
            for p in ps:
                n = p.numel()
                buf[off:off + n].copy_(p.data.reshape(-1))
                p.data = buf[off:off + n].view_as(p)
                off += n
            self.flat[key] = buf

    def buffers(self) -> List[torch.Tensor]:
        return list(self.flat.values())


class DiLoCo:
    """Synchronous DiLoCo: call :meth:`outer_step` every ``inner_steps`` local optimizer steps.

    Outer optimizer = SGD with optional (Nesterov) momentum, exactly torch.optim.SGD's rule; defaults follow the
    reference example (lr 0.7, no momentum). All outer tensors are fp32.
    """

    def __init__(self, model: torch.nn.Module, comm: Communicator, *, outer_lr: float = 0.7,
                 outer_momentum: float = 0.0, nesterov: bool = False, weight_decay: float = 0.0,
                 quantization: Optional[QuantizationOptions] = None, bucket_bytes: int = 1 << 30,
                 max_in_flight: int = 8, tag_base: int = 2 << 20, tensors: Optional[List[torch.Tensor]] = None):
        """``tensors``: explicit local parameter tensors (e.g. FSDP2 shards, ``p.to_local()``) instead of flattening
        ``model``'s parameters; each must be contiguous and stay the live storage of its parameter."""
        self.model = model
        self.comm = comm
        self.lr, self.momentum, self.nesterov, self.wd = outer_lr, outer_momentum, nesterov, weight_decay
        self.quantization = quantization
        self.bucket_bytes = bucket_bytes
        self.max_in_flight = max_in_flight
        self.tag_base = tag_base
        if tensors is None:
            self.params = FlatParams(model)
            self.local = self.params.buffers()
        else:
            assert all(t.is_contiguous() for t in tensors), "DiLoCo local tensors must be contiguous"
            self.params = None
            self.local = [t.view(-1) for t in tensors]
        self.outer = [b.detach().float().clone() for b in self.local]
        self.mom = [torch.zeros_like(o) for o in self.outer]
        self.pg = [self._comm_buffer_like(o) for o in self.outer]
        self.outer_steps = torch.zeros(1, dtype=torch.int64)  # shared: decides the momentum bootstrap on every peer

    @staticmethod
    def _comm_buffer_like(t: torch.Tensor) -> torch.Tensor:
        """All-reduced buffers live in fd-shareable memory on HIP devices (zero-copy on the xGMI path)."""
        with maybe_shareable(t.device):
            return torch.empty_like(t)

    # --- shared state ------------------------------------------------------------------------------------------
    def state_tensors(self) -> Dict[str, torch.Tensor]:
        out: Dict[str, torch.Tensor] = {}
        for i, (o, m) in enumerate(zip(self.outer, self.mom)):
            out[f"diloco.outer.{i}"] = o
            if self.momentum:
                out[f"diloco.momentum.{i}"] = m
        out["diloco.outer_steps"] = self.outer_steps
        return out

    def shared_state(self, inner_optimizer: Optional[torch.optim.Optimizer] = None,
                     extra: Optional[Dict[str, torch.Tensor]] = None) -> SharedState:
        tensors = self.state_tensors()
        if inner_optimizer is not None:
            for gi, g in enumerate(inner_optimizer.param_groups):
                for pi, p in enumerate(g["params"]):
                    for k, v in inner_optimizer.state.get(p, {}).items():
                        if isinstance(v, torch.Tensor):
                            tensors[f"inner.{gi}.{pi}.{k}"] = v
        if extra:
            tensors.update(extra)
        return SharedState([TensorInfo.from_torch(t, n) for n, t in tensors.items()])

    def load_outer_into_model(self) -> None:
        """local := outer (after a shared-state sync delivered new outer params)."""
        with torch.no_grad():
            for loc, o in zip(self.local, self.outer):
                loc.copy_(o)

    # --- outer step --------------------------------------------------------------------------------------------
    def _slices(self) -> List[torch.Tensor]:
        per = max(1, self.bucket_bytes // 4)
        return [pg[i:i + per] for pg in self.pg for i in range(0, pg.numel(), per)]

    def compute_pseudo_grads(self) -> None:
        for pg, o, loc in zip(self.pg, self.outer, self.local):
            K.pseudo_grad(pg, o, loc)

    def apply_outer(self, pgs: Optional[List[torch.Tensor]] = None) -> None:
        first = int(self.outer_steps.item()) == 0
        for o, m, g, loc in zip(self.outer, self.mom, pgs or self.pg, self.local):
            K.outer_sgd(o, m, g, loc, lr=self.lr, momentum=self.momentum, nesterov=self.nesterov,
                        weight_decay=self.wd, first=first and self.momentum != 0.0)
        self.outer_steps += 1

    def reduce(self, pgs: Optional[List[torch.Tensor]] = None) -> RetryResult:
        slices = self._slices() if pgs is None else [
            g[i:i + max(1, self.bucket_bytes // 4)] for g in pgs for i in range(0, g.numel(), max(1, self.bucket_bytes // 4))]
        return all_reduce_multiple_with_retry(self.comm, slices, ReduceOp.AVG, max_in_flight=self.max_in_flight,
                                              tag_base=self.tag_base, quantization=self.quantization)

    def outer_step(self) -> RetryResult:
        """pseudo-grad -> AVG all-reduce (retry on churn) -> fused outer SGD + copy-back."""
        self.compute_pseudo_grads()
        res = self.reduce()
        self.apply_outer()
        return res


class AsyncDiLoCo(DiLoCo):
    """1-step-delayed DiLoCo: the all-reduce of round t runs in the background during the inner steps of t+1.

    Call :meth:`outer_step` after each round of inner steps. Round t's averaged pseudo-gradient is applied at the end
    of round t+1 (to the outer params it was computed against); the first round only launches its reduce and resets
    the local model to the outer params (reference async_diloco.py:524-621).

    Pipeline insertion of new peers (reference async_diloco.py:556-590): after a topology update that admitted a
    peer mid-run, pre-existing peers call :meth:`outer_step` with ``topology_updated=True`` which re-syncs the shared
    state with SEND_ONLY after applying the update; the newcomer's first outer step syncs with RECEIVE_ONLY.
    """

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self.pg_next = [self._comm_buffer_like(o) for o in self.outer]
        self._thread: Optional[threading.Thread] = None
        self._result: Optional[RetryResult] = None
        self._error: Optional[BaseException] = None

    def wait(self) -> Optional[RetryResult]:
        if self._thread is None:
            return None
        self._thread.join()
        self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise e
        return self._result

    def _launch(self) -> None:
        pgs = self.pg
        # the torch stream must have produced the pseudo-gradients before another thread reduces them
        if pgs and pgs[0].is_cuda:
            torch.cuda.current_stream(pgs[0].device).synchronize()

        def run():
            try:
                self._result = self.reduce(pgs)
            except BaseException as e:  # noqa: BLE001 - re-raised in wait()
                self._error = e

        self._thread = threading.Thread(target=run, name="pccl-diloco-reduce", daemon=True)
        self._thread.start()

    def outer_step(self, *, topology_updated: bool = False, joined_mid_run: bool = False,
                   shared_state: Optional[SharedState] = None) -> Optional[RetryResult]:
        prev = self.wait()
        had_prev = prev is not None
        # pseudo-gradient of this round against the (still unchanged) outer params -> pg_next
        for pg, o, loc in zip(self.pg_next, self.outer, self.local):
            K.pseudo_grad(pg, o, loc)
        if had_prev:
            self.apply_outer(self.pg)  # round t-1's averaged pseudo-gradient; also local := outer
            if topology_updated and shared_state is not None:
                self.comm.sync_shared_state(shared_state, SharedStateSyncStrategy.SEND_ONLY)
                shared_state.revision += 1
        else:
            if joined_mid_run and shared_state is not None:
                self.comm.sync_shared_state(shared_state, SharedStateSyncStrategy.RECEIVE_ONLY)
                shared_state.revision += 1
            self.load_outer_into_model()
        self.pg, self.pg_next = self.pg_next, self.pg
        self._launch()
        return prev

    def close(self) -> None:
        self.wait()
