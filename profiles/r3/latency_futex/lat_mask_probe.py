"""Diagnostic: latency phases of bench.py under different CPU masks, interleaved over repetitions:
full (the process's mask), node0 (CPUs of NUMA node 0), ccd0 (the first L3 domain). Measures the native 8-peer
xGMI 1 MiB latency (pccl_latency) and BASELINE config 1 with threaded Python peers (bench.latency_cpu)."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from pccl_amd.utils import free_port  # noqa: E402


def cpulist(spec):
    out = set()
    for part in spec.strip().split(","):
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


full = os.sched_getaffinity(0)
masks = {"full": full}
try:
    with open("/sys/devices/system/node/node0/cpulist") as f:
        masks["node0"] = cpulist(f.read()) & full
    with open(f"/sys/devices/system/cpu/cpu{min(full)}/cache/index3/shared_cpu_list") as f:
        masks["ccd0"] = cpulist(f.read()) & full
except OSError:
    pass
ba = argparse.Namespace(gpus=1, steps=1, warmup=0, peers=2, mib=1, pool=0, windows=1, quick=True, no_ipc_extra=True,
                        no_peer_curve=True, no_quant_extra=True, extras_child="")
job = bench.Job(ba)
exe = os.path.join(ROOT, "pccl_amd", "lib", "pccl_latency")
for rep in range(int(os.environ.get("REPS", "3"))):
    for name, m in masks.items():
        os.sched_setaffinity(0, m)
        env = dict(os.environ)
        env.pop("PCCL_DISABLE_IPC", None)  # latency_cpu's phases set it in this process
        r = subprocess.run([exe, str(free_port()), "8", str(1 << 20), "400", "50"], capture_output=True, text=True,
                           timeout=120, env=env)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        nat = json.loads(line[-1]) if line else {"error": r.stderr[-200:]}
        cfg1 = bench.latency_cpu(job)
        os.sched_setaffinity(0, full)
        print(json.dumps({"mask": name, "cpus": len(m), "rep": rep, "ipc8_1MiB_median_us": nat.get("median_us"),
                          "ipc8_p90_us": nat.get("p90_us"), "cfg1": cfg1}), flush=True)
