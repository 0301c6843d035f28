"""Diagnostic: xGMI/IPC 8-peer 1 MiB latency (pccl_latency) with the process's full CPU mask vs the bench's
3-CPUs-per-L3 spread (bench.py _cpu_spread), interleaved."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pccl_amd.utils import free_port  # noqa: E402

full = sorted(os.sched_getaffinity(0))
domains = {}
for c in full:
    try:
        with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
            domains.setdefault(f.read().strip(), []).append(c)
    except OSError:
        pass
spread = sorted(c for cpus in domains.values() for c in cpus[:3])
exe = os.path.join(ROOT, "pccl_amd", "lib", "pccl_latency")
for rep in range(2):
    for name, mask in (("full", full), ("spread3", spread)):
        r = subprocess.run([exe, str(free_port()), "8", str(1 << 20), "400", "50"], capture_output=True, text=True,
                           timeout=120, preexec_fn=lambda m=mask: os.sched_setaffinity(0, m))
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        print(json.dumps({"mask": name, "cpus": len(mask), "rep": rep, "rc": r.returncode,
                          "res": json.loads(line[-1]) if line else r.stderr[-300:]}), flush=True)
