"""Lightweight nested-session profiler for training loops.

Same role as the reference's python/examples/nanogptddp/profiler.py (nested ``session(name)`` context managers, a
text report, a timeline export) without matplotlib: the timeline is written as a Chrome/Perfetto trace JSON, and
every session is also emitted as a roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm) so it lines up with the
kernels in ``rocprofv3 --marker-trace`` output.
"""
from __future__ import annotations

import json
import os
import time
from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional


def _roctx():
    try:
        import torch
        if torch.cuda.is_available() and os.environ.get("PCCL_PROFILER_ROCTX", "1") == "1":
            return torch.cuda.nvtx
    except Exception:  # noqa: BLE001
        pass
    return None


@dataclass
class Session:
    name: str
    start: float
    end: float = 0.0
    children: List["Session"] = field(default_factory=list)

    @property
    def seconds(self) -> float:
        return self.end - self.start


class Profiler:
    def __init__(self, sync_cuda: bool = False):
        self.root = Session("root", time.perf_counter())
        self._stack = [self.root]
        self._sync = sync_cuda
        self._tx = _roctx()

    @contextmanager
    def session(self, name: str) -> Iterator[Session]:
        s = Session(name, time.perf_counter())
        self._stack[-1].children.append(s)
        self._stack.append(s)
        if self._tx:
            self._tx.range_push(name)
        try:
            yield s
        finally:
            if self._sync:
                import torch
                torch.cuda.synchronize()
            if self._tx:
                self._tx.range_pop()
            s.end = time.perf_counter()
            self._stack.pop()

    def totals(self) -> Dict[str, float]:
        out: Dict[str, float] = {}

        def walk(s: Session, prefix: str):
            for c in s.children:
                key = f"{prefix}{c.name}"
                out[key] = out.get(key, 0.0) + c.seconds
                walk(c, key + "/")

        walk(self.root, "")
        return out

    def report(self) -> str:
        self.root.end = time.perf_counter()
        lines = []

        def walk(s: Session, depth: int):
            for c in s.children:
                pct = 100.0 * c.seconds / max(1e-12, self.root.seconds)
                lines.append(f"{'  ' * depth}{c.name:<{40 - 2 * depth}} {c.seconds * 1e3:10.3f} ms {pct:6.1f}%")
                walk(c, depth + 1)

        walk(self.root, 0)
        return "\n".join(lines)

    def chrome_trace(self, path: str, pid: int = 0, tid: int = 0) -> None:
        events = []

        def walk(s: Session):
            for c in s.children:
                events.append({"name": c.name, "ph": "X", "ts": (c.start - self.root.start) * 1e6,
                               "dur": c.seconds * 1e6, "pid": pid, "tid": tid})
                walk(c)

        walk(self.root)
        with open(path, "w") as f:
            json.dump({"traceEvents": events}, f)


class ProfilerCollection:
    """Accumulates per-step profilers (e.g. one per training iteration) and reports averages."""

    def __init__(self):
        self.profilers: List[Profiler] = []

    def add(self, p: Profiler) -> None:
        self.profilers.append(p)

    def averages(self) -> Dict[str, float]:
        acc: Dict[str, float] = {}
        for p in self.profilers:
            for k, v in p.totals().items():
                acc[k] = acc.get(k, 0.0) + v
        n = max(1, len(self.profilers))
        return {k: v / n for k, v in acc.items()}

    def chrome_trace(self, path: str) -> None:
        events = []
        t0: Optional[float] = self.profilers[0].root.start if self.profilers else None
        for p in self.profilers:
            def walk(s: Session):
                for c in s.children:
                    events.append({"name": c.name, "ph": "X", "ts": (c.start - t0) * 1e6, "dur": c.seconds * 1e6,
                                   "pid": 0, "tid": 0})
                    walk(c)
            walk(p.root)
        with open(path, "w") as f:
            json.dump({"traceEvents": events}, f)
