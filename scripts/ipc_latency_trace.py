"""Per-phase latency of small all-reduces on the xGMI/IPC path (threaded peers on one device), with PCCL_TRACE_OPS=1
phase marks: prints the median time of every phase mark over the timed ops and the median op time.

    python scripts/ipc_latency_trace.py [--peers 8] [--kib 1024] [--iters 200]
"""
import argparse
import json
import os
import re
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--kib", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    # the library prints the trace lines on stderr (fd 2): capture them in a file
    log = tempfile.NamedTemporaryFile(mode="w+", suffix=".trace", delete=False)
    os.environ["PCCL_TRACE_OPS"] = "1"
    saved = os.dup(2)
    os.dup2(log.fileno(), 2)
    import torch

    import pccl_amd as pccl
    from pccl_amd.utils import local_master, run_threaded_peers
    dev = torch.device(a.device)
    n = a.kib * 256

    def fn(rank, comm):
        x = torch.ones(n, device=dev)
        y = torch.empty_like(x)
        ts = []
        for _ in range(a.iters):
            t0 = time.perf_counter()
            comm.all_reduce(x, y, op=pccl.ReduceOp.SUM, tag=0)
            ts.append(time.perf_counter() - t0)
        return ts, comm.get_attribute(pccl.Attribute.LAST_REDUCE_PATH)

    with local_master() as addr:
        res = run_threaded_peers(a.peers, fn, address=addr, timeout=300)
    os.dup2(saved, 2)
    log.seek(0)
    marks = {}
    warm = a.iters // 4
    for ln in log:
        m = re.match(r"\[pccl-trace\] tag \d+ seq (\d+) .* ok (.*)", ln)
        if not m or int(m.group(1)) < warm:
            continue
        for k, us in re.findall(r"(\w+) (\d+)us", m.group(2)):
            marks.setdefault(k, []).append(int(us))
    ts = sorted(t for r in res for t in r[0][warm:])
    print(json.dumps({"peers": a.peers, "kib": a.kib, "path": pccl.ReducePath(res[0][1]).name,
                      "ipc_mode": os.environ.get("PCCL_IPC_MODE", "safe"),
                      "median_op_us": round(1e6 * ts[len(ts) // 2], 1), "p90_op_us": round(1e6 * ts[int(len(ts) * .9)], 1),
                      "median_mark_us": {k: statistics.median(v) for k, v in marks.items()}}), flush=True)


if __name__ == "__main__":
    main()
