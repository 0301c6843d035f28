"""Flagship benchmark: ring all-reduce of a 1 GiB bf16 HIP device buffer per peer (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mib 1024]

N == 1 : two peers (threads of this process) share cuda:0 — an all-reduce needs >= 2 peers.
N  > 1 : launched by torch.distributed.run, one peer per GPU (LOCAL_RANK); rank 0 also hosts the CCoIP master.
         torch.distributed (gloo) is used only for the bench's own barriers / max-over-ranks and to share the port.

Each timed step is one pcclAllReduce(SUM) of the whole buffer on every peer. Peers on one host rendezvous in shared
memory and reduce over xGMI (DEVICE_IPC path); the ring over loopback TCP is the fallback (PCCL_DISABLE_IPC=1).

Reported: ``value`` = whole-job aggregate bus bandwidth = n_peers x busBW, with the nccl-tests convention
busBW = (bytes / t) x 2 (n - 1) / n. ``extra`` carries per-peer busBW/algBW and the reference's own metric,
(rx_bytes + tx_bytes) / t per peer (reference tests/basic_reduce_test/main.cpp:141-143).
vs_baseline = value / 5.625 GB/s (the reference's best published all-reduce throughput, 45 Gbit/s,
docs/md/01_Introduction.md:8).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_GBPS = 45e9 / 8 / 1e9  # 45 Gbit/s


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mib", type=int, default=1024, help="buffer size per peer in MiB (flagship: 1024)")
    ap.add_argument("--peers-per-gpu", type=int, default=0, help="N==1 only: peers sharing cuda:0 (default 2)")
    ap.add_argument("--path", default="auto", choices=["auto", "ring"],
                    help="auto: xGMI IPC between same-host peers; ring: force the pipelined TCP ring")
    ap.add_argument("--pool", type=int, default=4, help="P2P connections per neighbour (ring stripes)")
    ap.add_argument("--rejoin", type=int, default=1, help="N==1: also measure peer-rejoin latency after the timed steps")
    return ap.parse_args()


def _peer_loop(comm, x, y, steps, warmup, sync_all, torch, pccl):
    """Runs warmup + timed steps; sync_all() is the cross-peer barrier. Returns (seconds, tx, rx, path)."""
    for s in range(warmup):
        for attempt in range(3):  # an aborted warmup op (e.g. the xGMI path fell back to TCP) is retried by all peers
            try:
                comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=s)
                break
            except pccl.PCCLError:
                if attempt == 2:
                    raise
    torch.cuda.synchronize()
    sync_all()
    t0 = time.perf_counter()
    tx = rx = 0
    for s in range(steps):
        info = comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=warmup + s)
        tx += info.tx_bytes
        rx += info.rx_bytes
    torch.cuda.synchronize()
    sync_all()
    dt = time.perf_counter() - t0
    return dt, tx, rx, comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)


def _report(n_gpus, n_peers, steps, warmup, nbytes, dt, tx, rx, path, parallelism, rejoin_s=None):
    import pccl_amd as pccl
    t = dt / steps
    alg = nbytes / t / 1e9
    bus = alg * 2 * (n_peers - 1) / n_peers
    value = bus * n_peers
    line = {
        "metric": "all-reduce bus BW (GB/s) vs tensor bytes, 2/4/8 peers; peer-rejoin latency",
        "value": round(value, 3), "unit": "GB/s", "n_gpus": n_gpus, "steps": steps, "warmup": warmup,
        "ms_per_step": round(t * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": round(value / BASELINE_GBPS, 3), "dtype": "bf16",
        "data": "synthetic (torch.randn bf16 on device)",
        "config": {"model": "8-peer ring all-reduce, 1 GiB bf16 HIP device buffer per MI355X, loopback TCP",
                   "global_batch": n_peers, "seq_len": nbytes // 2, "parallelism": parallelism,
                   "tensor_bytes": nbytes, "n_peers": n_peers},
        "extra": {"bus_bw_per_peer_GBps": round(bus, 3), "alg_bw_GBps": round(alg, 3),
                  "ref_metric_rx_plus_tx_per_peer_GBps": round((tx + rx) / steps / t / 1e9, 3),
                  "reduce_path": pccl.ReducePath(path).name,
                  "peer_rejoin_latency_ms": round(rejoin_s * 1e3, 1) if rejoin_s else None,
                  "baseline_note": "vs_baseline divides the aggregate value by the reference's 45 Gbit/s "
                                   "per-run WAN figure (no like-for-like MI355X number is published)"},
    }
    print(json.dumps(line), flush=True)


def _rejoin_latency(comm, rank, addr, dev, bar, torch, pccl, pool):
    """After the timed steps: a new peer connects mid-run; returns seconds from its connect() call until its first
    all-reduce completed (admission vote + P2P establishment + IPC rendezvous + first op). Untimed for the metric."""
    small = torch.ones(1 << 16, device=dev, dtype=torch.bfloat16)
    out = {}
    joiner = None
    bar.wait()
    if rank == 0:
        def join():
            c = pccl.Communicator(addr, 0, p2p_connection_pool_size=pool)
            t0 = time.perf_counter()
            c.connect(n_attempts=30)
            y = torch.empty_like(small)
            c.all_reduce(small, y, op=pccl.ReduceOp.SUM, tag=77)
            torch.cuda.synchronize()
            out["s"] = time.perf_counter() - t0
            out["c"] = c
        joiner = threading.Thread(target=join, daemon=True)
        joiner.start()
    deadline = time.time() + 120
    while time.time() < deadline:
        if comm.are_peers_pending():
            comm.update_topology()
            y = torch.empty_like(small)
            comm.all_reduce(small, y, op=pccl.ReduceOp.SUM, tag=77)
            break
        time.sleep(0.001)
    if joiner is not None:
        joiner.join(timeout=120)
        out["c"].destroy()
    bar.wait()
    return out.get("s")


def bench_single_gpu(a):
    import torch

    import pccl_amd as pccl
    from pccl_amd.utils import local_master, run_threaded_peers
    n_peers = a.peers_per_gpu or 2
    nbytes = a.mib << 20
    n = nbytes // 2
    dev = torch.device("cuda:0")
    bar = threading.Barrier(n_peers)

    with local_master() as addr:
        def fn(rank, comm):
            torch.cuda.set_device(dev)
            g = torch.Generator(device=dev).manual_seed(rank)
            x = torch.randn(n, device=dev, dtype=torch.bfloat16, generator=g)
            y = torch.empty_like(x)
            r = _peer_loop(comm, x, y, a.steps, a.warmup, bar.wait, torch, pccl)
            rejoin = _rejoin_latency(comm, rank, addr, dev, bar, torch, pccl, a.pool) if a.rejoin else None
            return (*r, rejoin)

        res = run_threaded_peers(n_peers, fn, address=addr, timeout=1800,
                                 comm_kwargs={"p2p_connection_pool_size": a.pool})
    dt = max(r[0] for r in res)
    _report(1, n_peers, a.steps, a.warmup, nbytes, dt, res[0][1], res[0][2], res[0][3], f"{n_peers} peers on 1 GPU",
            rejoin_s=res[0][4])


def bench_multi_gpu(a):
    import torch
    import torch.distributed as dist

    import pccl_amd as pccl
    from pccl_amd.utils import free_port, wait_for_world
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    # rehearsal on a 1-GPU box: PCCL_BENCH_SAME_GPU=1 puts every rank on cuda:0 (the real run uses one GPU per rank)
    if os.environ.get("PCCL_BENCH_SAME_GPU") == "1":
        local_rank = 0
    dist.init_process_group("gloo")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    master = None
    port = [free_port() if rank == 0 else 0]
    if rank == 0:
        master = pccl.MasterNode(f"127.0.0.1:{port[0]}")
        master.run()
    dist.broadcast_object_list(port, src=0)
    comm = pccl.Communicator(f"127.0.0.1:{port[0]}", 0, p2p_connection_pool_size=a.pool)
    comm.connect(n_attempts=30)
    wait_for_world(comm, world, timeout=300)
    nbytes = a.mib << 20
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(nbytes // 2, device=dev, dtype=torch.bfloat16, generator=g)
    y = torch.empty_like(x)
    dt, tx, rx, path = _peer_loop(comm, x, y, a.steps, a.warmup, dist.barrier, torch, pccl)
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        _report(world, world, a.steps, a.warmup, nbytes, float(t.item()), tx, rx, path, f"dp{world} (1 peer/GPU)")
    dist.barrier()
    comm.destroy()
    if master is not None:
        master.interrupt()
        master.await_termination()
    dist.destroy_process_group()


def main():
    a = _args()
    if a.path == "ring":
        os.environ["PCCL_DISABLE_IPC"] = "1"
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        bench_multi_gpu(a)
    else:
        bench_single_gpu(a)


if __name__ == "__main__":
    main()
