"""xGMI/IPC path only: ms per 1 GiB bf16 all-reduce for 8 and 2 threaded peers on cuda:0 (bench.py's measure()),
under whatever PCCL_IPC_* tuning variables the caller set. One JSON line on stdout."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--peers", type=int, nargs="+", default=[8, 2])
    a = ap.parse_args()
    ns = argparse.Namespace(gpus=1, steps=a.steps, warmup=3, peers=max(a.peers), mib=a.mib, pool=2, quick=True,
                            no_ipc_extra=False, no_peer_curve=True, extras_child="")
    job = bench.Job(ns)
    out = {k: os.environ[k] for k in os.environ if k.startswith("PCCL_IPC_")}
    for p in a.peers:
        r = bench.measure(job, ipc=True, nbytes=a.mib << 20, steps=a.steps, warmup=3, peers=p, check=True)
        out[f"{p}_peers_ms"] = round(r["t"] * 1e3, 4)
        out[f"{p}_peers_exact"] = r.get("ok")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
