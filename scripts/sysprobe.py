"""Host-side transport probe for the device TCP ring's bounds on one MI355X box.

Measures (1) pinned-host <-> HBM copy bandwidth per direction and full duplex (the PCIe hop every TCP ring byte takes
twice), with 1 and 8 concurrent streams, and (2) loopback TCP throughput with k parallel streams (the socket hop).

    python scripts/sysprobe.py [--tcp-streams 1,2,4,8,16] [--mib 256]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import threading
import time


def pcie(mib: int):
    import torch
    dev = torch.device("cuda:0")
    n = mib << 20
    out = {}
    for nstreams in (1, 8):
        hs = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(nstreams)]
        ds = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(nstreams)]
        hs2 = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(nstreams)]
        ds2 = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(nstreams)]
        streams = [torch.cuda.Stream() for _ in range(2 * nstreams)]

        def run(kind, reps=5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                for i in range(nstreams):
                    if kind in ("d2h", "duplex"):
                        with torch.cuda.stream(streams[i]):
                            hs[i].copy_(ds[i], non_blocking=True)
                    if kind in ("h2d", "duplex"):
                        with torch.cuda.stream(streams[nstreams + i]):
                            ds2[i].copy_(hs2[i], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            nbytes = reps * nstreams * n * (2 if kind == "duplex" else 1)
            return round(nbytes / dt / 1e9, 2)

        run("d2h", 1)
        out[f"streams{nstreams}"] = {k: run(k) for k in ("d2h", "h2d", "duplex")}
    return out


def tcp(streams: int, mib: int, secs: float = 2.0):
    """k loopback TCP streams, each sending mib-MiB buffers for ~secs; returns aggregate GB/s."""
    srv = socket.socket()
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind(("127.0.0.1", 0))
    srv.listen(64)
    port = srv.getsockname()[1]
    buf = bytearray(mib << 20)
    total = [0] * streams
    stop = threading.Event()

    def rx(conn, i):
        mv = memoryview(bytearray(mib << 20))
        while True:
            k = conn.recv_into(mv)
            if k == 0:
                break
            total[i] += k

    def tx(i):
        c = socket.create_connection(("127.0.0.1", port))
        c.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
        mv = memoryview(buf)
        while not stop.is_set():
            c.sendall(mv)
        c.close()

    rxs = []
    txs = [threading.Thread(target=tx, args=(i,)) for i in range(streams)]
    for t in txs:
        t.start()
    for i in range(streams):
        conn, _ = srv.accept()
        conn.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
        t = threading.Thread(target=rx, args=(conn, i))
        t.start()
        rxs.append(t)
    time.sleep(0.3)
    b0 = sum(total)
    t0 = time.perf_counter()
    time.sleep(secs)
    b1 = sum(total)
    dt = time.perf_counter() - t0
    stop.set()
    for t in txs + rxs:
        t.join()
    srv.close()
    return round((b1 - b0) / dt / 1e9, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tcp-streams", default="1,2,4,8,16")
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--no-gpu", action="store_true")
    a = ap.parse_args()
    res = {"cpus_affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    res["cpu_model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    if not a.no_gpu:
        res["pcie_GBps"] = pcie(a.mib)
    res["loopback_tcp_GBps"] = {k: tcp(int(k), 8) for k in a.tcp_streams.split(",")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
