"""Per-op latency of the Python API with one process per peer, the deployment shape (one process per GPU).

    python benchmarks/py_latency.py [--peers 8] [--iters 200] [--sizes 65536,1048576,16777216] [--device cuda:0]

bench.py's ``extra.latency_1MiB_ipc_python_threads_us`` runs its 8 peers as threads of ONE Python process, where every
op's Python work (argument checks, descriptor, stream sync, ctypes call) of all 8 peers is serialised by the GIL. Here
every peer is its own process, as under torchrun, so the number is what a DDP bucket of that size costs from Python.
With every peer on one GPU the buffers are fd-shareable and the ops run the xGMI/IPC path; ``--device cpu`` measures
the host ring.

Per size: the median / p90 of the per-op wall time maximum over the peers (ops are matched by index: every peer runs
the same sequence). Call variants on the same buffers, interleaved op by op (a machine-wide slow phase hits every
variant alike):
  * ``all_reduce``: the public blocking call - stream-ordered (pcclxAllReduceOnStream: the op waits for an event
    recorded on the current stream; no stream synchronisation) and run on the calling thread;
  * ``async``: the public ``all_reduce_async(...).wait()`` - stream-ordered, run on a collective worker thread;
  * ``ready``: ``_all_reduce_async_ready(...).wait()`` - no readiness handling at all (producers already waited for),
    worker thread: the floor of the two above;
  * ``sync_inline`` / ``sync_worker``: the round-4 behaviour - ``current_stream().synchronize()`` on the caller, then
    the op inline (pcclAllReduce) / on a worker; with ``ready`` and ``ready_inline`` (no sync, inline) this is the
    {host stream sync, none} x {inline, worker} matrix that isolates what the round-4 blocking call paid.
Prints one JSON object.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def peer(a):
    import contextlib

    import torch

    import ctypes

    import pccl_amd as pccl
    from pccl_amd import _native
    from pccl_amd._native import C
    from pccl_amd.utils import wait_for_world
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = pccl.Communicator(a.master, 0)
    comm.connect(n_attempts=60)
    wait_for_world(comm, a.peers, timeout=120)
    out = {}
    tag = 0
    for b in [int(s) for s in a.sizes.split(",")]:
        n = b // 2
        with pccl.memory.maybe_shareable(dev) if dev.type == "cuda" else contextlib.nullcontext():
            x = torch.full((n,), float(a.rank + 1), device=dev, dtype=torch.bfloat16)
            y = torch.empty_like(x)
        variants = a.variants.split(",")
        res = {v: [] for v in variants}
        if dev.type == "cuda" and a.caller_stream == "side":
            torch.cuda.set_stream(torch.cuda.Stream(dev))
        cur = torch.cuda.current_stream(dev) if dev.type == "cuda" else None

        def run(variant):
            nonlocal tag
            if variant == "all_reduce":
                comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=tag)
            elif variant == "async":
                ok, _, _ = comm.all_reduce_async(x, y, op=pccl.ReduceOp.SUM, tag=tag).wait()
                assert ok
            elif variant in ("ready", "sync_worker"):
                if variant == "sync_worker" and cur is not None:
                    cur.synchronize()
                ok, _, _ = comm._all_reduce_async_ready(x, y, op=pccl.ReduceOp.SUM, tag=tag).wait()
                assert ok
            elif variant in ("ready_inline", "sync_inline"):
                if variant == "sync_inline" and cur is not None:
                    cur.synchronize()
                sptr, rptr, desc = comm._descriptor(x, y, pccl.ReduceOp.SUM, tag, None, None, sync=False)
                info = _native.ReduceInfoC()
                pccl.PCCLError.check(C.pcclAllReduce(sptr, rptr, ctypes.byref(desc), comm._comm, ctypes.byref(info)),
                                     "pcclAllReduce")
            else:
                raise ValueError(variant)
            tag += 1

        for i in range(a.iters + a.warmup):
            for variant in variants:
                t0 = time.perf_counter()
                run(variant)
                if i >= a.warmup:
                    res[variant].append(time.perf_counter() - t0)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        want = a.peers * (a.peers + 1) / 2
        assert float(y.min()) == float(y.max()) == want, (float(y.min()), float(y.max()), want)
        res["path"] = comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)
        out[b] = res
    print(json.dumps(out), flush=True)
    comm.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--sizes", default="65536,1048576,16777216")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--variants", default="all_reduce,async,ready",
                    help="comma list of all_reduce, async, ready, ready_inline, sync_inline, sync_worker")
    ap.add_argument("--trace-dir", default="", help="PCCL_TRACE_OPS=1 in every peer, its stderr to <dir>/peer<r>.err")
    ap.add_argument("--caller-stream", default="default", choices=["default", "side"],
                    help="the stream the peers' calls are ordered on: torch's default (null) stream or a created one")
    ap.add_argument("--peer", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--master", default="")
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args()
    if a.peer:
        peer(a)
        return
    import pccl_amd as pccl
    from pccl_amd.utils import DIAG_SIGNALS, communicate_all, free_port
    port = free_port()
    env = dict(os.environ)
    if a.device.startswith("cuda"):  # several processes on one GPU: 2 hardware queues each (README), so the peers'
        env.setdefault("GPU_MAX_HW_QUEUES", "2")  # queues fit the GPU's slots without time-slicing
    errs = []
    if a.trace_dir:
        os.makedirs(a.trace_dir, exist_ok=True)
        env["PCCL_TRACE_OPS"] = "1"
        errs = [open(os.path.join(a.trace_dir, f"peer{r}.err"), "w") for r in range(a.peers)]
    master = pccl.MasterNode(f"0.0.0.0:{port}")
    master.run()
    try:
        procs = [subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--peer", "--master",
                                   f"127.0.0.1:{port}", "--rank", str(r), "--peers", str(a.peers), "--iters",
                                   str(a.iters), "--warmup", str(a.warmup), "--sizes", a.sizes, "--device", a.device,
                                   "--variants", a.variants, "--caller-stream", a.caller_stream],
                                  stdout=subprocess.PIPE, stderr=errs[r] if errs else subprocess.PIPE, text=True,
                                  env=env)
                 for r in range(a.peers)]
        outs = communicate_all(procs, 600, DIAG_SIGNALS)
    finally:
        master.interrupt()
        master.await_termination()
    res = []
    for p, (o, e) in zip(procs, outs):
        if p.returncode != 0:
            raise SystemExit(f"peer failed rc={p.returncode}: {(e or '')[-3000:]}")
        res.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    names = {0: "none", 1: "host_ring", 2: "device_ring", 3: "ipc", 4: "hier"}
    summary = {"peers": a.peers, "device": a.device, "iters": a.iters, "processes": "one per peer", "sizes": {}}
    for b in res[0]:
        row = {"path": names.get(res[0][b]["path"], "?")}
        for v in a.variants.split(","):
            per_op = [max(r[b][v][i] for r in res) for i in range(a.iters)]
            q = statistics.quantiles(per_op, n=10)
            row[v] = {"median_us": round(statistics.median(per_op) * 1e6, 1), "p90_us": round(q[-1] * 1e6, 1),
                      "min_us": round(min(per_op) * 1e6, 1),
                      "rank0_median_us": round(statistics.median(res[0][b][v]) * 1e6, 1)}
        summary["sizes"][f"{int(b) >> 10}KiB"] = row
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
