"""BASELINE config 1: 2-peer fp32 all-reduce on localhost CPU (the reference's basic_reduce_test path, no GPU).

    python benchmarks/basic_reduce.py [--peers 2] [--iters 500] [--device cpu|cuda:0]

Two measurements, each with peer processes and an in-process master on 127.0.0.1:
  * latency: pcclAllReduce(SUM) of 4 fp32 elements, median / p99 over --iters ops (the smallest possible op: master
    consensus + one ring exchange);
  * throughput: the reference harness tests/basic_reduce_test/main.cpp:46-164 — 32 tensors x 16 Mi fp32 with
    pcclAllReduceMultipleWithRetry (max_in_flight 32, connection pool 32), reported in the reference's own metric
    MB/s of (rx_bytes + tx_bytes) / wall time per peer (main.cpp:141-143).
The reference publishes no number for either. --device cuda:0 runs the same ops on HBM tensors (all
peers on one GPU: the xGMI IPC path) to show the per-op latency of the device path.
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
    import torch

    import pccl_amd as pccl
    from pccl_amd.utils import wait_for_world
    comm = pccl.Communicator(a.master, 0, p2p_connection_pool_size=a.pool)
    comm.connect(n_attempts=60)
    wait_for_world(comm, a.peers, timeout=120)
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    x = torch.full((4,), float(a.rank + 1), device=dev)
    y = torch.empty(4, device=dev)
    lat = []
    for i in range(a.iters + 20):
        t0 = time.perf_counter()
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=i)
        if i >= 20:
            lat.append(time.perf_counter() - t0)
    expect = sum(range(1, a.peers + 1))
    assert torch.all(y == expect), y
    # reference harness: 32 x 16 Mi fp32, max_in_flight 32
    n = a.numel
    bufs = [torch.full((n,), float(a.rank + 1), device=dev) for _ in range(a.tensors)]
    outs = [torch.empty(n, device=dev) for _ in range(a.tensors)]
    descs = [pccl.ReduceOpDescriptor.from_torch(
        bufs[i], outs[i], pccl.ReduceDescriptor(n, pccl.ReduceOp.SUM, 1000 + i,
                                                pccl.ReduceOperandDescriptor(pccl.DataType.FLOAT),
                                                pccl.QuantizationOptions(pccl.DataType.FLOAT,
                                                                         pccl.QuantizationAlgorithm.NONE)))
        for i in range(a.tensors)]
    comm.all_reduce_multiple_with_retry(descs, max_in_flight=a.tensors)  # warm-up
    for i, d in enumerate(descs):
        d.reduce_descriptor.tag = 5000 + i
    t0 = time.perf_counter()
    info = comm.all_reduce_multiple_with_retry(descs, max_in_flight=a.tensors)
    dt = time.perf_counter() - t0
    assert all(torch.all(o == expect) for o in outs)
    print(json.dumps({"rank": a.rank, "lat": lat, "mt_seconds": dt, "tx": info.tx_bytes, "rx": info.rx_bytes,
                      "path": comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)}),
          flush=True)
    comm.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=2)
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--tensors", type=int, default=32)
    ap.add_argument("--numel", type=int, default=16 << 20)
    ap.add_argument("--pool", type=int, default=32)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--master", default=None)
    a = ap.parse_args()
    if a.rank is not None:
        return peer(a)
    from pccl_amd.utils import local_master, spawn_python
    args = ["--peers", str(a.peers), "--iters", str(a.iters), "--tensors", str(a.tensors), "--numel", str(a.numel),
            "--pool", str(a.pool), "--device", a.device]
    with local_master() as addr:
        ps = [spawn_python([os.path.abspath(__file__), "--rank", str(r), "--master", addr, *args],
                           env={"PCCL_DISABLE_HIP": "1"} if a.device == "cpu" else {}, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True) for r in range(a.peers)]
        outs = [p.communicate(timeout=900) for p in ps]
    res = []
    for p, (o, e) in zip(ps, outs):
        if p.returncode != 0:
            raise RuntimeError(e[-3000:])
        res.append(json.loads([x for x in o.splitlines() if x.startswith("{")][-1]))
    lat = sorted(res[0]["lat"])
    mt = max(r["mt_seconds"] for r in res)
    per_peer_MBps = [(r["tx"] + r["rx"]) / r["mt_seconds"] / 1e6 for r in res]
    print(json.dumps({
        "metric": f"basic_reduce ({a.device}, localhost)", "device": a.device,
        "config": f"{a.peers}-peer fp32 4-elem all-reduce on localhost "
                  + ("CPU (basic_reduce_test path, no GPU)" if a.device == "cpu" else f"{a.device} (xGMI IPC path)"),
        "peers": a.peers, "reduce_path": res[0].get("path"),
        "latency_us": {"median": round(statistics.median(lat) * 1e6, 1),
                       "p99": round(lat[int(0.99 * (len(lat) - 1))] * 1e6, 1), "min": round(lat[0] * 1e6, 1)},
        "multi_tensor": {"tensors": a.tensors, "numel": a.numel, "max_in_flight": a.tensors, "pool": a.pool,
                         "seconds": round(mt, 4), "ref_metric_MBps_per_peer": [round(v, 1) for v in per_peer_MBps],
                         "busbw_GBps": round(a.tensors * a.numel * 4 / mt * 2 * (a.peers - 1) / a.peers / 1e9, 3)}}),
        flush=True)


if __name__ == "__main__":
    main()
