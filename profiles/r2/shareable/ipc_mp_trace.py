"""Per-phase trace of xGMI/IPC all-reduces between separate peer PROCESSES on one GPU (shareable buffers):
median time of each phase mark per process count, to separate kernel time from control / barrier time.

    python profiles/r2/shareable/ipc_mp_trace.py [--procs 2 4 8] [--n 536870912] [--steps 30]
"""
import argparse
import json
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--n", type=int, default=1 << 29)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    from pccl_amd.utils import local_master, spawn_python
    worker = os.path.join(ROOT, "tests", "workers", "allreduce_peer.py")
    for w in a.procs:
        with local_master() as addr:
            ps = [spawn_python([worker, addr, str(w), str(r), "--n", str(a.n), "--dtype", "bf16", "--device", "cuda:0",
                                "--steps", str(a.steps), "--reuse", "--shareable", "--check-every", "1000"],
                               env={"PCCL_TRACE_OPS": "1"}, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                  for r in range(w)]
            outs = [p.communicate(timeout=300) for p in ps]
        marks, secs = {}, []
        for p, (o, e) in zip(ps, outs):
            if p.returncode != 0:
                print(json.dumps({"procs": w, "error": e[-1500:]}), flush=True)
                break
            for ln in e.splitlines():
                m = re.match(r"\[pccl-trace\] tag (\d+) seq \d+ .* ok (.*)", ln)
                if m and int(m.group(1)) >= 5:
                    for k, us in re.findall(r"(\w+) (\d+)us", m.group(2)):
                        marks.setdefault(k, []).append(int(us))
            secs += [json.loads(x)["sec"] for x in o.splitlines() if x.startswith("{")][5:]
        print(json.dumps({"procs": w, "n": a.n, "median_op_ms": round(1e3 * statistics.median(secs), 3) if secs else None,
                          "median_mark_us": {k: statistics.median(v) for k, v in marks.items()}}), flush=True)


if __name__ == "__main__":
    main()
