"""Repeats benchmarks/py_latency.py (8 peer processes on cuda:0, 1 MiB) and records, per repetition, the cgroup's CPU
throttling and the CPUs the run used, to see what separates the ~125-190 us runs from the ~550 us ones
(profiles/r4/b13, b14).

    python profiles/scripts_archive/lat_mode_probe.py [--reps 6] [--peers 8]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cpu_stat():
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for ln in f:
                k, v = ln.split()
                out[k] = int(v)
    except OSError:
        pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--peers", type=int, default=8)
    a = ap.parse_args()
    for rep in range(a.reps):
        s0, t0 = cpu_stat(), time.time()
        r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "py_latency.py"), "--peers", str(a.peers),
                            "--iters", "300", "--sizes", str(1 << 20)], capture_output=True, text=True, timeout=240)
        s1, t1 = cpu_stat(), time.time()
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        row = json.loads(line[-1])["sizes"]["1024KiB"] if r.returncode == 0 and line else {"error": r.stderr[-500:]}
        d = {k: s1.get(k, 0) - s0.get(k, 0) for k in ("usage_usec", "nr_throttled", "throttled_usec", "nr_periods")}
        print(json.dumps({"rep": rep, "wall_s": round(t1 - t0, 2), "cores_busy": round(d["usage_usec"] / 1e6 / (t1 - t0), 2),
                          "nr_throttled": d["nr_throttled"], "throttled_ms": round(d["throttled_usec"] / 1e3, 1),
                          "blocking_median_us": row.get("all_reduce", {}).get("median_us"),
                          "ready_median_us": row.get("ready", {}).get("median_us"),
                          "cpus_allowed": len(os.sched_getaffinity(0))}), flush=True)


if __name__ == "__main__":
    main()
