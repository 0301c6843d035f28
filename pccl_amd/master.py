"""``python -m pccl_amd.master [--host 0.0.0.0] [--port 48148]`` — runs a CCoIP master until SIGINT/SIGTERM
(reference python/framework/pccl/master.py and ccoip_master/src/main.cpp)."""
from __future__ import annotations

import argparse
import signal
import threading


def main(argv=None) -> None:
    from .api import MasterNode
    ap = argparse.ArgumentParser(description="PCCL master node")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=48148)
    a = ap.parse_args(argv)
    master = MasterNode(f"{a.host}:{a.port}")
    master.run()
    print(f"pccl master listening on {a.host}:{a.port}", flush=True)
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stop.set())
    while not stop.wait(0.2):
        pass
    master.interrupt()
    master.await_termination()


if __name__ == "__main__":
    main()
