"""Data-parallel gradient synchronisation over PCCL, device resident.

The reference trainers flatten gradients, move them to the CPU and all-reduce one host buffer
(python/examples/nanogptddp/train_pccl.py:471-531, mnist_peer.py:326-347). Here gradients stay in HBM: every
parameter's ``.grad`` is a view into one flat buffer per (device, dtype), so a backward pass writes straight into the
communication buffer and the all-reduce runs on the device path (xGMI IPC between local peers, pinned-staged TCP ring
otherwise) with no gather/scatter copies. Large buckets (default 1 GiB) suit 288 GB of HBM and keep per-op protocol
overhead negligible; they are reduced concurrently (one tag each) with retry on peer churn.

``overlap=True`` starts each bucket's all-reduce during the backward pass, as soon as every gradient in it has been
accumulated (post-accumulate-grad hooks). The launch is stream-ordered (pcclxAllReduceAsyncOnStream): the op waits
for an event recorded on the stream that queued the gradient kernels, so no thread synchronises that stream and the
autograd thread returns at once. Gradients arrive roughly in reverse parameter order, so buckets are cut from the end
of the flat buffer; with buckets smaller than the model, the reduction of late layers runs while the early layers are
still back-propagating. ``sync_gradients`` launches buckets whose hooks did not all fire (unused parameters), waits
for every op and re-reduces failed buckets through the retry path (the library restores an aborted in-place buffer,
and the master's per-tag abort decision is the same on every peer, so all peers retry the same buckets).
"""
from __future__ import annotations

import contextlib
import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch

from ..api import (Communicator, DataType, DistributionHint, PCCLError, QuantizationAlgorithm, QuantizationOptions,
                   ReduceOp, ReduceOperandDescriptor)
from ..memory import maybe_shareable
from .elastic import RetryResult, all_reduce_multiple_with_retry, world_size


class GradBuckets:
    """Flat gradient storage: one contiguous buffer per (device, dtype); ``param.grad`` are views into it."""

    def __init__(self, params: List[torch.nn.Parameter]):
        self.params = [p for p in params if p.requires_grad]
        groups: "OrderedDict[Tuple[torch.device, torch.dtype], List[torch.nn.Parameter]]" = OrderedDict()
        for p in self.params:
            groups.setdefault((p.device, p.dtype), []).append(p)
        self.flat: Dict[Tuple[torch.device, torch.dtype], torch.Tensor] = {}
        self.views: Dict[torch.nn.Parameter, torch.Tensor] = {}
        for key, ps in groups.items():
            total = sum(p.numel() for p in ps)
            with maybe_shareable(key[0]):  # fd-shareable: the xGMI path reduces it without a staged copy-out
                buf = torch.zeros(total, device=key[0], dtype=key[1])
            off = 0
            for p in ps:
                v = buf[off:off + p.numel()].view_as(p)
                if p.grad is not None:
                    v.copy_(p.grad)
                p.grad = v
                self.views[p] = v
                off += p.numel()
            self.flat[key] = buf

    def rebind(self) -> None:
        """Re-attach views if the user replaced/cleared ``.grad`` (e.g. ``zero_grad(set_to_none=True)``)."""
        for p, v in self.views.items():
            g = p.grad
            if g is None:
                v.zero_()
                p.grad = v
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
                p.grad = v

    def zero_(self) -> None:
        for buf in self.flat.values():
            buf.zero_()

    def slices(self, bucket_bytes: int) -> List[torch.Tensor]:
        out = []
        for buf in self.flat.values():
            per = max(1, bucket_bytes // buf.element_size())
            out.extend(buf[i:i + per] for i in range(0, buf.numel(), per))
        return out


class DataParallel:
    """Gradient all-reduce for a model replicated across PCCL peers.

    usage::

        dp = DataParallel(model, comm)             # overlap=True: buckets are reduced during backward
        loss.backward()
        res = dp.sync_gradients()        # AVG over the current world; retries on churn
        optimizer.step()
    """

    def __init__(self, model: torch.nn.Module, comm: Communicator, *, bucket_bytes: Optional[int] = None,
                 op: ReduceOp = ReduceOp.AVG, max_in_flight: int = 8, tag_base: int = 1 << 20,
                 quantization: Optional[QuantizationOptions] = None, overlap: bool = False):
        self.model = model
        self.comm = comm
        # overlap needs several buckets per model to have anything to overlap with
        self.bucket_bytes = bucket_bytes or ((128 << 20) if overlap else (1 << 30))
        self.op = op
        self.max_in_flight = max_in_flight
        self.tag_base = tag_base
        self.quantization = quantization
        self.buckets = GradBuckets(list(model.parameters()))
        self.overlap = overlap
        self._sync_enabled = True
        self._hooks = []
        if overlap:
            self._setup_overlap()

    # -- synchronous path ------------------------------------------------------------------------------------------
    def sync_gradients(self) -> RetryResult:
        if self.overlap:
            return self._finish_overlapped()
        self.buckets.rebind()
        slices = self.buckets.slices(self.bucket_bytes)
        return all_reduce_multiple_with_retry(self.comm, slices, self.op, max_in_flight=self.max_in_flight,
                                              tag_base=self.tag_base, quantization=self.quantization)

    def zero_grad(self) -> None:
        self.buckets.zero_()

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation: backward passes inside do not start all-reduces (overlap mode)."""
        prev, self._sync_enabled = self._sync_enabled, False
        try:
            yield
        finally:
            self._sync_enabled = prev

    # -- overlapped path -------------------------------------------------------------------------------------------
    def _setup_overlap(self) -> None:
        # buckets cut from the END of each flat buffer (reverse parameter order = backward order)
        self._bucket_views: List[torch.Tensor] = []
        members: List[List[torch.nn.Parameter]] = []
        for (dev, dt), buf in self.buckets.flat.items():
            per = max(1, self.bucket_bytes // buf.element_size())
            ps = [p for p in self.buckets.params if (p.device, p.dtype) == (dev, dt)]
            spans, off = [], 0
            for p in ps:
                spans.append((off, off + p.numel(), p))
                off += p.numel()
            end = buf.numel()
            while end > 0:
                start = max(0, end - per)
                self._bucket_views.append(buf[start:end])
                members.append([p for a, b, p in spans if a < end and b > start])
                end = start
        self._bucket_of: Dict[torch.nn.Parameter, List[int]] = {}
        for i, ps in enumerate(members):
            for p in ps:
                self._bucket_of.setdefault(p, []).append(i)
        self._need = [len(ps) for ps in members]
        self._pending = list(self._need)
        self._launched = [False] * len(self._bucket_views)
        self._handles: List[Optional[object]] = [None] * len(self._bucket_views)
        self._errors: List[BaseException] = []
        self._lock = threading.Lock()
        for p in self._bucket_of:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        v = self.buckets.views.get(p)
        if v is not None and (p.grad is None or p.grad.data_ptr() != v.data_ptr()):
            # .grad was reset to None (zero_grad(set_to_none=True)): autograd allocated a fresh tensor
            if p.grad is not None:
                v.copy_(p.grad)
            p.grad = v
        if not self._sync_enabled:
            return
        ready = []
        with self._lock:
            for i in self._bucket_of.get(p, ()):
                self._pending[i] -= 1
                if self._pending[i] == 0 and not self._launched[i]:
                    self._launched[i] = True
                    ready.append(i)
        for i in ready:
            self._start(i)

    def _start(self, i: int) -> None:
        """Launches bucket i's all-reduce from the hook: stream-ordered on the stream the gradient kernels were queued
        on (pcclxAllReduceAsyncOnStream), so neither the autograd thread nor any other thread synchronises it - the op
        waits for those kernels itself."""
        t = self._bucket_views[i]
        dt = DataType.from_torch_dtype(t.dtype)
        q = self.quantization or QuantizationOptions(dt, QuantizationAlgorithm.NONE)
        try:
            self._handles[i] = self.comm.all_reduce_async(
                t, t, op=self.op, tag=self.tag_base + i,
                operand_descriptor=ReduceOperandDescriptor(dt, DistributionHint.NONE), quantization_options=q,
                stream=torch.cuda.current_stream(t.device) if t.is_cuda else None)
        except BaseException as e:  # surfaced by sync_gradients
            self._errors.append(e)
            self._handles[i] = None

    def _finish_overlapped(self) -> RetryResult:
        # buckets whose hooks did not all fire (unused parameters, or no_sync ended mid-step) start now; unused
        # parameters get zero gradients like on the synchronous path
        self.buckets.rebind()
        with self._lock:
            rest = [i for i, l in enumerate(self._launched) if not l]
            for i in rest:
                self._launched[i] = True
        for i in rest:
            self._start(i)
        tx = rx = 0
        failed = []
        for i, h in enumerate(self._handles):
            if h is None:
                failed.append(i)
                continue
            ok, _, info = h.wait()
            if ok:
                tx += info.tx_bytes
                rx += info.rx_bytes
            else:
                failed.append(i)
        self._handles = [None] * len(self._bucket_views)
        with self._lock:
            self._pending = list(self._need)
            self._launched = [False] * len(self._bucket_views)
        errors, self._errors = self._errors, []
        for e in errors:
            if not isinstance(e, PCCLError):
                raise e
        retries = 0
        if failed:
            # same buckets on every peer (per-tag abort consensus); aborted in-place buffers were restored
            res = all_reduce_multiple_with_retry(self.comm, [self._bucket_views[i] for i in failed], self.op,
                                                 max_in_flight=self.max_in_flight, tag_base=self.tag_base,
                                                 quantization=self.quantization)
            return RetryResult(res.ok, tx + res.tx_bytes, rx + res.rx_bytes, res.retries + 1, res.world_size)
        return RetryResult(True, tx, rx, retries, world_size(self.comm))

    def close(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
