"""Calibration of the WAN emulator (pccl_wan_relay): plain TCP streams (pccl_tcp_stream, no library) through one
relayed link, at several connection counts. Reports the delivered rate in the steady state (after the first RTT and
the window fill) against the configured per-flow and per-link rates, and the relay process's CPU use, so a library
measurement through the relay can be read against what the emulator itself can carry.

    python scripts/wan_relay_calibrate.py [--delay-ms 50] [--flow-mbit 1000] [--link-mbit 25000]
                                          [--conns 8,16,32,64] [--seconds 8]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "pccl_amd", "lib")


def _cpu_s(pid):
    with open(f"/proc/{pid}/stat") as f:
        st = f.read()
    fields = st[st.rindex(")") + 2:].split()
    tick = os.sysconf("SC_CLK_TCK")
    return (int(fields[11]) + int(fields[12])) / tick


def run(a, conns):
    from pccl_amd.utils import free_ports
    sink_port, relay_port = free_ports(2)
    sink = subprocess.Popen([os.path.join(LIB, "pccl_tcp_stream"), "sink", str(sink_port)], stdout=subprocess.PIPE,
                            text=True)
    sink.stdout.readline()
    relay = subprocess.Popen([os.path.join(LIB, "pccl_wan_relay"), "--delay-ms", str(a.delay_ms), "--flow-mbit",
                              str(a.flow_mbit), "--link-mbit", str(a.link_mbit), "--map", f"{relay_port}:{sink_port}"],
                             stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    relay.stdout.readline()
    sender = subprocess.Popen([os.path.join(LIB, "pccl_tcp_stream"), "send", str(relay_port), str(conns),
                               str(a.seconds)], stdout=subprocess.PIPE, text=True)
    samples = []
    cpu = []
    t_start = time.time()
    for line in sink.stdout:
        r = json.loads(line)
        samples.append((r["t"], r["bytes"]))
        cpu.append((time.time() - t_start, _cpu_s(relay.pid)))
        if time.time() - t_start > a.seconds + 30:
            break
    sender.wait(timeout=60)
    sink.wait(timeout=60)
    relay.terminate()
    relay.wait(timeout=10)
    # steady state: from 2 RTT + 1 s after the first byte arrived to the sender's end
    first = next((t for t, b in samples if b > 0), samples[0][0])
    lo, hi = first + 4 * a.delay_ms / 1e3 + 1.0, first + a.seconds - 0.5
    win = [(t, b) for t, b in samples if lo <= t <= hi]
    rate = (win[-1][1] - win[0][1]) / (win[-1][0] - win[0][0]) if len(win) >= 2 else 0.0
    cwin = [(t, c) for t, c in cpu if lo <= t <= hi]
    cores = (cwin[-1][1] - cwin[0][1]) / (cwin[-1][0] - cwin[0][0]) if len(cwin) >= 2 else None
    expect = min(conns * a.flow_mbit, a.link_mbit) if a.link_mbit > 0 else conns * a.flow_mbit
    return {"conns": conns, "delivered_Gbit": round(rate * 8 / 1e9, 2), "configured_Gbit": round(expect / 1e3, 2),
            "efficiency": round(rate * 8 / 1e6 / expect, 3) if expect else None,
            "relay_cpu_cores": round(cores, 2) if cores is not None else None,
            "relay_cpu_cores_per_10Gbit": round(cores / (rate * 8 / 1e10), 2) if cores and rate else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--delay-ms", type=float, default=50)
    ap.add_argument("--flow-mbit", type=float, default=1000)
    ap.add_argument("--link-mbit", type=float, default=25000)
    ap.add_argument("--conns", default="8,16,32,64")
    ap.add_argument("--seconds", type=float, default=8)
    a = ap.parse_args()
    for c in [int(x) for x in a.conns.split(",")]:
        r = run(a, c)
        r.update({"delay_ms": a.delay_ms, "flow_mbit": a.flow_mbit, "link_mbit": a.link_mbit})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
