"""Hierarchical vs flat all-reduce when a peer group spans several hosts.

    python benchmarks/hierarchical.py [--hosts 2] [--per-host 2] [--mib 256] [--steps 10] [--device cuda:0]
                                      [--wan 1:10000:25000]

Hosts are simulated on one machine (PCCL_HOST_TOKEN per process; every process uses the same GPU), so the
"network" is loopback TCP and the "xGMI" hops are same-GPU IPC copies. Two runs of the same op loop:
  * hierarchical (default): reduce inside each host over IPC, one TCP device ring per local rank across hosts on a
    1/L shard, broadcast inside the host -- every byte crosses the network once per host;
  * flat (PCCL_HIERARCHICAL=0): one TCP device ring over all H*L peers -- every byte crosses the network per GPU.
Reported: median ms per op, and the TCP bytes each peer sends per op in each mode (2(n-1)/n of its ring's buffer).
--wan shapes every TCP flow (PCCL_SIM_WAN: latency, per-flow and per-peer link rate) like a data-center network.
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
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    world = a.hosts * a.per_host
    comm = pccl.Communicator(a.master, 0, p2p_connection_pool_size=a.pool)
    comm.connect(n_attempts=60)
    wait_for_world(comm, world, timeout=300)
    n = (a.mib << 20) // 2
    x = torch.full((n,), float(a.rank + 1), dtype=torch.bfloat16, device=dev)
    y = torch.empty_like(x)
    times = []
    for s in range(a.steps + 2):
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=s)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        if s >= 2:
            times.append(time.perf_counter() - t0)
    ok = bool(torch.all(y == float(world * (world + 1) // 2)))
    print(json.dumps({"rank": a.rank, "times": times, "exact": ok,
                      "path": comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)}), flush=True)
    comm.destroy()


def run(a, hierarchical: bool):
    from pccl_amd.utils import local_master, spawn_python
    world = a.hosts * a.per_host
    args = ["--hosts", str(a.hosts), "--per-host", str(a.per_host), "--mib", str(a.mib), "--steps", str(a.steps),
            "--device", a.device, "--pool", str(a.pool)]
    with local_master() as addr:
        ps = [spawn_python([os.path.abspath(__file__), "--rank", str(r), "--master", addr, *args],
                           env={"PCCL_HOST_TOKEN": f"simhost{r // a.per_host}",
                                "PCCL_HIERARCHICAL": "1" if hierarchical else "0",
                                **({"PCCL_SIM_WAN": a.wan} if a.wan else {})},
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
        outs = [p.communicate(timeout=900) for p in ps]
    res = []
    for p, (o, e) in zip(ps, outs):
        if p.returncode != 0:
            raise RuntimeError(e[-3000:])
        res.append(json.loads([x for x in o.splitlines() if x.startswith("{")][-1]))
    per_op = [max(r["times"][i] for r in res) for i in range(a.steps)]
    return {"ms_per_op": round(1e3 * statistics.median(per_op), 3), "exact": all(r["exact"] for r in res),
            "path": res[0]["path"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hosts", type=int, default=2)
    ap.add_argument("--per-host", type=int, default=2)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--wan", default="", help="PCCL_SIM_WAN for the TCP links, e.g. 1:10000:25000 (ms:Mbit:Mbit)")
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--master", default=None)
    a = ap.parse_args()
    if a.rank is not None:
        return peer(a)
    world = a.hosts * a.per_host
    nbytes = a.mib << 20
    hier = run(a, True)
    flat = run(a, False)
    print(json.dumps({
        "metric": "hierarchical vs flat all-reduce (simulated hosts on one machine)", "hosts": a.hosts,
        "per_host": a.per_host, "mib_per_peer": a.mib, "dtype": "bf16", "wan_emulation": a.wan or None,
        "hierarchical": {**hier, "tcp_bytes_sent_per_peer": round(nbytes / a.per_host * 2 * (a.hosts - 1) / a.hosts)},
        "flat": {**flat, "tcp_bytes_sent_per_peer": round(nbytes * 2 * (world - 1) / world)},
        "speedup": round(flat["ms_per_op"] / hier["ms_per_op"], 2)}), flush=True)


if __name__ == "__main__":
    main()
