"""Diagnostic: xGMI/IPC all-reduce time at 1 GiB bf16 per peer (threaded peers on cuda:0, shareable buffers, as in
bench.py's IPC phases) for 2 and 8 peers; prints one JSON line per peer count."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", default="2,8")
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--ops", type=int, default=20)
    a = ap.parse_args()
    import argparse as _ap

    import torch

    import bench
    import pccl_amd as pccl
    for p in (int(x) for x in a.peers.split(",")):
        ba = _ap.Namespace(gpus=1, steps=a.ops, warmup=3, peers=p, mib=a.mib, pool=0, windows=1, quick=True,
                           no_ipc_extra=True, no_peer_curve=True, no_quant_extra=True, extras_child="")
        job = bench.Job(ba)
        r = bench.measure(job, ipc=True, nbytes=a.mib << 20, steps=a.ops, warmup=3)
        print(json.dumps({"peers": p, "ms_per_op": round(r["t"] * 1e3, 4),
                          "path": pccl.ReducePath(r["path"]).name,
                          "spin_us": os.environ.get("PCCL_MASTER_RX_SPIN_US", "default")}), flush=True)
        torch.cuda.synchronize()
        time.sleep(0.5)


if __name__ == "__main__":
    main()
